# blocked panel + MFMA Schur variant: pivot cycles of both builds, A/B against the product build,
# then the variant's parity (the product library replaced by it in this box's copy only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python tools/pivot_cycles.py gpurun_exp/libbos_pivcyc.so > gpurun_out/r05_pivcyc.txt 2>&1 &&
timeout -k 10 150 python tools/pivot_cycles.py gpurun_exp/libbos_blkcyc.so > gpurun_out/r05_pivcyc_blocked.txt 2>&1 &&
timeout -k 10 600 python tools/gn_ab.py gpurun_exp/libbos_base.so gpurun_exp/libbos_blocked.so gpurun_exp/libbos_ntl.so 3 > gpurun_out/r05_ab_blocked.txt 2>&1 &&
cp gpurun_exp/libbos_blocked.so prb-project-bearing-only-slam_amd/lib/libbos.so &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sharding.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "not p2p and not two_processes" > gpurun_out/r05_blocked_parity.log 2>&1
