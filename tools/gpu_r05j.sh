# round 5: plain loads for every L read; two-pivot step broadcast forms
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./gpurun_exp/pivot_probe2 > gpurun_out/r05_pivot_probe2b.txt 2>&1 &&
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_prod.so gpurun_exp/libbos_ldplain.so 3 > gpurun_out/r05_ab_ldplain.txt 2>&1
