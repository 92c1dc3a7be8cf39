set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/jh_timeline.py fp32 cold > gpurun_out/tl_cold.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_cases.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/q_pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --gn-steps 10 --no-cpu-baseline --no-gn-other --tri-steps 0 > gpurun_out/q_fp32.json 2> gpurun_out/q_fp32.err || exit 1
