# round 5: flow geometry, second sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python tools/gn_ab.py gpurun_exp/libbos_basefv.so gpurun_exp/libbos_fw5.so gpurun_exp/libbos_fw7.so gpurun_exp/libbos_sw128.so gpurun_exp/libbos_fwide1024.so 3 > gpurun_out/r05_ab_geometry2.txt 2>&1
