# round 5: the pivot loop in isolation, the short-chain pivot step A/B against the broadcast form, its cycle stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./gpurun_exp/pivot_probe > gpurun_out/r05_pivot_probe.txt 2>&1 &&
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_probe.so gpurun_exp/libbos_fastpiv.so 3 > gpurun_out/r05_ab_fastpiv.txt 2>&1 &&
timeout -k 10 120 python tools/pivot_cycles.py gpurun_exp/libbos_pivcycfast.so > gpurun_out/r05_pivcyc_fast.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_c3_gn.py > gpurun_out/r05_gpu_suite_fastpiv.log 2>&1
