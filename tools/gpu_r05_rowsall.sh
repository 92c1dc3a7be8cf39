# round 5: all row columns read at once
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_basefv.so gpurun_exp/libbos_rowsall.so 3 > gpurun_out/r05_ab_rowsall.txt 2>&1 &&
timeout -k 10 120 python tools/pivot_cycles.py gpurun_exp/libbos_rowsallcyc.so > gpurun_out/r05_pivcyc_rowsall.txt 2>&1
