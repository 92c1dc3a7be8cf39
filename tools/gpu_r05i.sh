# round 5: cache policy of the folded landmarks' L columns
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/gn_ab.py gpurun_exp/libbos_prod.so gpurun_exp/libbos_foldc.so gpurun_exp/libbos_foldlc.so 3 > gpurun_out/r05_ab_foldl.txt 2>&1
