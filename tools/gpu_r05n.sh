# round 5: GPU suite, smoke and the bench line on the current build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05n_smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r05n_gpu_suite.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r05n_bench.json 2> gpurun_out/r05n_bench.err
