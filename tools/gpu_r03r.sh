# final-build check: GPU tests, smoke, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || exit 1
