# round 5: the 8-rank sharded path rehearsed on one GPU, launched as the driver launches the scaling bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 8 --same-device --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05h_bench_p2p8.json 2> gpurun_out/r05h_bench_p2p8.err
# the same with two hardware queues per process (8 x 2 on the one GPU instead of 8 x 4)
[ $? -eq 0 ] && GPU_MAX_HW_QUEUES=2 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 8 --same-device --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05h_bench_p2p8_q2.json 2> gpurun_out/r05h_bench_p2p8_q2.err
