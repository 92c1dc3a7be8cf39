# round 5: backward flow polls with the sweep; flow and fold geometry re-swept
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/gn_ab.py gpurun_exp/libbos_rowsraw.so gpurun_exp/libbos_bwdnoprobe.so gpurun_exp/libbos_fw8.so gpurun_exp/libbos_bw8.so gpurun_exp/libbos_fl8.so gpurun_exp/libbos_fl2.so 3 > gpurun_out/r05_ab_geometry.txt 2>&1
