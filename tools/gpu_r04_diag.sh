# Round 4 diagnostics: per-front solver stamps, one GN step's kernel timeline (rocprofv3 kernel
# trace of the timed steps), per-rank shard timeline (W = 1 through the one-graph RCCL path, 2/4/8
# through the phase API with device stamps).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python tools/solver_stamps.py > gpurun_out/d_stamps.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/d_trace -o run --output-format csv -- \
  python3 bench.py --replay-steps 0 --cold-steps 0 --no-cpu-baseline --no-gn-other --tri-steps 0 > gpurun_out/d_bench_traced.json 2> gpurun_out/d_bench_traced.err || exit 1
python3 tools/step_timeline.py gpurun_out/d_trace > gpurun_out/d_timeline.txt 2>&1 || exit 1
timeout -k 10 400 python tools/shard_timeline.py 1 2 4 8 > gpurun_out/d_shard.txt 2>&1 || exit 1
