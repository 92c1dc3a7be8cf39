# Round 4: smoke, the full GPU test suite, the default bench line without a profiler.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1 || { echo "smoke failed" >> gpurun_out/f_smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/f_bench.json 2> gpurun_out/f_bench.err || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/f_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/f_pytest.log; exit 1; }
