# round 5 final measurements (C), on the final build: smoke, GPU suite, bench lines, the profile set, rehearsals
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05c_smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r05c_gpu_suite.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r05c_bench_fp32.json 2> gpurun_out/r05c_bench_fp32.err &&
timeout -k 10 400 python bench.py --precision fp64 --no-cpu-baseline > gpurun_out/r05c_bench_fp64.json 2> gpurun_out/r05c_bench_fp64.err &&
bash tools/gpu_profile.sh r05 > gpurun_out/r05c_profile.log 2>&1
