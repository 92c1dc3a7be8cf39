# Round 4: kernel timelines of one synchronous GN step — one-rank sharded path (RCCL, direct
# exchange) and the plain one-GPU step (tools/shard_step_trace.py, tools/step_timeline.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in rccl p2p plain; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$m -- python3 tools/shard_step_trace.py $m 20 > gpurun_out/tr_$m.log 2>&1 || { echo "trace $m failed" >> gpurun_out/tr_$m.log; exit 1; }
  python3 tools/step_timeline.py gpurun_out/tr_$m > gpurun_out/tl_$m.txt 2>&1 || exit 1
done
