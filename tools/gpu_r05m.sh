# round 5: rows taken as read (no zero selects above the diagonal)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_pairs8.so gpurun_exp/libbos_rowsraw.so 3 > gpurun_out/r05_ab_rowsraw.txt 2>&1 &&
timeout -k 10 120 python tools/pivot_cycles.py gpurun_exp/libbos_pivcyc.so > gpurun_out/r05_pivcyc_rowsraw.txt 2>&1
