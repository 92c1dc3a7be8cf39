# round 5: batched steps as the J+H launch plus the step's tail graph
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_basefv.so gpurun_exp/libbos_batchsplit.so 3 > gpurun_out/r05_ab_batchsplit.txt 2>&1
