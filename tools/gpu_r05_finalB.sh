# round 5 final measurements (B): sharded-path tests on the gathering push, per-rank timelines, rehearsals
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_sharding.py tests/test_partitions.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05g_shard_tests.log 2>&1 &&
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r05g_bench_fp32.json 2> gpurun_out/r05g_bench_fp32.err &&
timeout -k 10 500 python tools/shard_timeline.py 1 2 4 8 > gpurun_out/r05g_shard_timeline.txt 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace -o run --output-format csv -d gpurun_out/r05g_tr8 -- python3 tools/shard_step_trace.py ranks 8 4 > gpurun_out/r05g_tr8.log 2>&1 &&
timeout -k 10 400 python bench.py --gpus 4 --same-device --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05g_bench_p2p4.json 2> gpurun_out/r05g_bench_p2p4.err &&
timeout -k 10 400 python bench.py --gpus 2 --same-device --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05g_bench_p2p2.json 2> gpurun_out/r05g_bench_p2p2.err
rc=$?
python tools/burst_timeline.py gpurun_out/r05g_tr8 8 0 > gpurun_out/r05g_rank_timeline_w8.txt 2>&1
rm -rf gpurun_out/r05g_tr8
exit $rc
