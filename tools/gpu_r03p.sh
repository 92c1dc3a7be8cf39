# one-workgroup top launches vs the flows taking the top (BOS_MF_TOP=0): GN rate + checksums, solver
# stamps, step timeline; GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
L=prb-project-bearing-only-slam_amd/lib/libbos.so
timeout -k 10 120 python3 -u tools/gn_rate_check.py --child $L > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 500 python3 -u tools/gn_rate_check.py $L gpurun_exp/libbos_notop.so $L gpurun_exp/libbos_notop.so > $O/gn.txt 2>&1 || exit 1
timeout -k 10 180 python3 -u tools/solver_stamps.py > $O/solver_stamps.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/gn_rate_check.py --child $L > $O/prof.txt 2>&1 || exit 1
python3 tools/step_timeline.py $O/tr > $O/timeline.txt || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || exit 1
