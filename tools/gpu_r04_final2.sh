# Round 4: the default bench line without a profiler (the profiled build), then a two-rank
# direct-exchange rehearsal of bench.py --gpus 2 on the one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/g_bench.json 2> gpurun_out/g_bench.err || exit 1
timeout -k 10 400 python bench.py --gpus 2 --same-device --steps 20 --warmup 3 --no-cpu-baseline --no-gn-other --tri-steps 0 --replay-steps 0 --cold-steps 0 --no-partition-other > gpurun_out/g_bench2.json 2> gpurun_out/g_bench2.err || exit 1
