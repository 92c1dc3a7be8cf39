# round 5: two children waited for together in the factor flow
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_rowsraw.so gpurun_exp/libbos_sweep2.so 3 > gpurun_out/r05_ab_sweep2.txt 2>&1 &&
timeout -k 10 120 python tools/pivot_cycles.py gpurun_exp/libbos_pivcyc.so > gpurun_out/r05_pivcyc_sweep2.txt 2>&1
