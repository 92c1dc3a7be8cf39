# round 5: register triangle in the backward flow; grouped reads in the single-pivot tail
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/gn_ab.py gpurun_exp/libbos_pairs8.so gpurun_exp/libbos_bwdreg.so gpurun_exp/libbos_tail8.so gpurun_exp/libbos_bwdtail.so 3 > gpurun_out/r05_ab_bwdreg_tail8.txt 2>&1
