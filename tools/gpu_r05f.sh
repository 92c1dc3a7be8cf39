# round 5: per-rank timelines of the subtree partition (device stamps and kernel traces), the 4-rank rehearsal
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python tools/shard_timeline.py 1 2 4 8 > gpurun_out/r05_shard_timeline.txt 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace -o run --output-format csv -d gpurun_out/r05_tr8 -- python3 tools/shard_step_trace.py ranks 8 4 > gpurun_out/r05_tr8.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace -o run --output-format csv -d gpurun_out/r05_tr2 -- python3 tools/shard_step_trace.py ranks 2 4 > gpurun_out/r05_tr2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace -o run --output-format csv -d gpurun_out/r05_tr1 -- python3 tools/shard_step_trace.py plain 20 > gpurun_out/r05_tr1.log 2>&1 &&
timeout -k 10 400 python bench.py --gpus 4 --same-device --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05_bench_p2p4.json 2> gpurun_out/r05_bench_p2p4.err
rc=$?
python tools/burst_timeline.py gpurun_out/r05_tr8 8 > gpurun_out/r05_rank_timeline_w8.txt 2>&1
python tools/burst_timeline.py gpurun_out/r05_tr2 2 > gpurun_out/r05_rank_timeline_w2.txt 2>&1
python tools/step_timeline.py gpurun_out/r05_tr1 > gpurun_out/r05_gn_step_timeline.txt 2>&1
exit $rc
