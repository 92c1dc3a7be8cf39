# round 5: the GPU suite and the C3 accuracy tests on this build, the unscaled-pivot A/B, the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./gpurun_exp/lat_probe > gpurun_out/r05_lat_probe.txt 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_c3_gn.py > gpurun_out/r05_gpu_suite.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests/test_gpu_c3_gn.py -m gpu -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_c3_gn.log 2>&1 &&
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_probe.so gpurun_exp/libbos_unscaled.so 3 > gpurun_out/r05_ab_unscaled.txt 2>&1
