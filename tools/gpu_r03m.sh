# 8-rank rehearsal of bench.py --gpus 8 on one GPU (gloo exchanges, every rank on GPU 0), both partitions
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 8 --exchange gloo --same-device --steps 10 --warmup 2 --no-cpu-baseline --tri-steps 0 --no-gn-other > $O/bench_n8_gloo.json 2> $O/bench_n8_gloo.err || exit 1
