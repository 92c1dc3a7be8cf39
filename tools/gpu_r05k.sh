# round 5: the trailing update's pairs read eight at a time
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_prod.so gpurun_exp/libbos_pairs8.so 3 > gpurun_out/r05_ab_pairs8.txt 2>&1 &&
timeout -k 10 120 python tools/pivot_cycles.py gpurun_exp/libbos_pivcyc.so > gpurun_out/r05_pivcyc_pairs8.txt 2>&1
