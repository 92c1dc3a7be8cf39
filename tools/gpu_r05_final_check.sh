# round 5: the round-end checks on the final tree (smoke, GPU suite, default bench line)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z_smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r05z_gpu_suite.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r05z_bench.json 2> gpurun_out/r05z_bench.err
