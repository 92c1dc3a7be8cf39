# Round-3 first GPU pass: solver variant A/B (committed solver / branch-free loads / + formal agent
# acquire), GPU tests (new partition / scenario / deeper C3 parity tests first), bench at N = 1, the
# no-launcher two-rank bench rehearsal (gloo, both ranks on GPU 0), J+H timelines, lanes-per-pose
# sweep. Each step has its own time limit; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 300 python -u tools/gn_ab.py gpurun_exp/libbos_base.so gpurun_exp/libbos_bf.so gpurun_exp/libbos_acq.so 3 > $O/ab_solver.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_partitions.py tests/test_gpu_scenarios.py tests/test_gpu_c3_gn.py -x -v -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest_new.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || exit 1
timeout -k 10 400 python bench.py --gpus 2 --exchange gloo --same-device --steps 20 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || exit 1
timeout -k 10 120 python -u tools/jh_timeline.py fp32 cold > $O/tl_cold.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/jh_timeline.py fp32 > $O/tl_warm.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/jh_lpp_sweep.py fp32 > $O/lpp.log 2>&1 || exit 1
