# round 5: two-pivot step anatomy; per-rank kernel traces; backward per-level threshold at W = 8
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./gpurun_exp/pivot_probe2 > gpurun_out/r05_pivot_probe2.txt 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace -o run --output-format csv -d gpurun_out/r05_tr8 -- python3 tools/shard_step_trace.py ranks 8 4 > gpurun_out/r05_tr8.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace -o run --output-format csv -d gpurun_out/r05_tr1 -- python3 tools/shard_step_trace.py plain 20 > gpurun_out/r05_tr1.log 2>&1 &&
BOS_LIB=gpurun_exp/libbos_sw1024.so timeout -k 10 200 python tools/shard_timeline.py 8 > gpurun_out/r05_shard8_sw1024.txt 2>&1 &&
BOS_LIB=gpurun_exp/libbos_sw2048.so timeout -k 10 200 python tools/shard_timeline.py 8 > gpurun_out/r05_shard8_sw2048.txt 2>&1 &&
timeout -k 10 200 python tools/shard_timeline.py 8 > gpurun_out/r05_shard8_base.txt 2>&1
rc=$?
python tools/burst_timeline.py gpurun_out/r05_tr8 8 0 > gpurun_out/r05_rank_timeline_w8.txt 2>&1
python tools/step_timeline.py gpurun_out/r05_tr1 > gpurun_out/r05_gn_step_timeline.txt 2>&1
rm -rf gpurun_out/r05_tr8 gpurun_out/r05_tr1
exit $rc
