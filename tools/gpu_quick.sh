set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > gpurun_out/q_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/q_pytest.log; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --gn-steps 50 --no-cpu-baseline > gpurun_out/q_fp32.json 2> gpurun_out/q_fp32.err || exit 1
