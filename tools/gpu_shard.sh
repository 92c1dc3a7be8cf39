set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python tools/shard_timeline.py > gpurun_out/shard_tl.txt 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 5 --gn-steps 5 --exchange gloo --same-device --no-cpu-baseline > gpurun_out/b2.json 2> gpurun_out/b2.err || exit 1
