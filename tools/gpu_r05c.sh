# round 5: A/B of the previous product (base), this build (new) and this build with cached L
# panels, per-phase cycles of this build, then the GPU suite without the C3 GN tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/gn_ab.py gpurun_exp/libbos_base.so gpurun_exp/libbos_new.so gpurun_exp/libbos_tag.so gpurun_exp/libbos_cachedl.so 3 > gpurun_out/r05_ab_new.txt 2>&1 &&
timeout -k 10 150 python tools/pivot_cycles.py gpurun_exp/libbos_pivcyc.so > gpurun_out/r05_pivcyc_new.txt 2>&1 &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_c3_gn.py > gpurun_out/r05_gpu_suite.log 2>&1
