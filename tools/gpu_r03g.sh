# wave-end J+H timing check (bench vs rocprofv3), solver experiments: level-0 fold stamps; GN rate
# with and without the side stream; GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --replay-steps 0 --cold-steps 0 --no-cpu-baseline --no-gn-other --tri-steps 0 > $O/bench_instep.json 2> $O/bench_instep.err || exit 1
BOS_LIB=gpurun_exp/libbos_foldst.so timeout -k 10 180 python3 -u tools/fold_stamps.py > $O/fold_stamps.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/gn_rate_check.py prb-project-bearing-only-slam_amd/lib/libbos.so gpurun_exp/libbos_noside.so prb-project-bearing-only-slam_amd/lib/libbos.so gpurun_exp/libbos_noside.so > $O/gn_side.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || exit 1
