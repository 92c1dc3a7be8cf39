# Round 4: sharded-path tests, kernel timelines of the one-rank sharded step (RCCL, direct exchange),
# flow-start A/B, shard timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sharding.py tests/test_partitions.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/s_pytest.log; exit 1; }
for m in rccl p2p; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sr_$m -- python3 tools/shard_step_trace.py $m 20 > gpurun_out/sr_$m.log 2>&1 || { echo "trace $m failed" >> gpurun_out/sr_$m.log; exit 1; }
  python3 tools/step_timeline.py gpurun_out/sr_$m > gpurun_out/sl_$m.txt 2>&1 || exit 1
done
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_base.so gpurun_exp/libbos_wide4096.so 2 > gpurun_out/s_ab.txt 2>&1 || exit 1
timeout -k 10 400 python tools/shard_timeline.py 1 2 4 8 > gpurun_out/s_shard.txt 2>&1 || exit 1
