# round 5: separator balance of the Schur ordering's nested dissection
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/gn_ab.py gpurun_exp/libbos_basefv.so gpurun_exp/libbos_nd45.so gpurun_exp/libbos_nd48.so gpurun_exp/libbos_nd50.so 2 > gpurun_out/r05_ab_nd_balance.txt 2>&1
