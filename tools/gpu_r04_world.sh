# Round 4: the parallax world on the GPU — C3 GN parity (50 fp32 iterations, lpp 1 and 2; 200-iteration
# pivot check; fp64 20 iterations), then the default bench line without CPU baselines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_c3_gn.py -x -v -s --timeout 700 --timeout-method thread -p no:cacheprovider > gpurun_out/w_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/w_pytest.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/w_bench.json 2> gpurun_out/w_bench.err || exit 1
