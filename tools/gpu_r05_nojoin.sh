# round 5: what the level-0 join costs (diagnostic build without it)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_basefv.so gpurun_exp/libbos_nojoin0.so 3 > gpurun_out/r05_ab_nojoin0.txt 2>&1
