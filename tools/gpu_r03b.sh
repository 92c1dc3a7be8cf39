# Round-3 GPU pass b: J+H variant timing (pair loop / ILP lanes), then the GPU tests, bench (N = 1 and
# the no-launcher two-rank gloo rehearsal), J+H timelines, lanes-per-pose sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
for rep in 1 2; do
  for v in pairs ilp12 ilp12w5 ilp10; do
    timeout -k 10 120 python -u tools/jh_variant_timing.py gpurun_exp/libbos_$v.so fp32 >> $O/jh_variants.log 2>&1 || exit 1
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_scenarios.py tests/test_gpu_c3_gn.py tests/test_partitions.py -x -v -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest_new.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || exit 1
timeout -k 10 400 python bench.py --gpus 2 --exchange gloo --same-device --steps 20 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || exit 1
timeout -k 10 120 python -u tools/jh_timeline.py fp32 cold > $O/tl_cold.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/jh_timeline.py fp32 > $O/tl_warm.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/jh_lpp_sweep.py fp32 > $O/lpp.log 2>&1 || exit 1
