# GPU-box steps of the round's measurements (run through gpurun from the repo root), one per call:
#   bash tools/gpu_run.sh ab LIB_A LIB_B [...]   A/B of library builds (tools/gn_ab.py, 3 rounds)
#   bash tools/gpu_run.sh stamps                 per-front solver phases (tools/solver_stamps.py)
#   bash tools/gpu_run.sh trace MODE [LIB]       kernel timeline of one synchronous step, MODE plain |
#                                                rccl | p2p (tools/shard_step_trace.py + step_timeline.py)
#   bash tools/gpu_run.sh shard                  per-rank timeline of W = 1, 2, 4, 8 shards (shard_timeline.py)
#   bash tools/gpu_run.sh tests [PYTEST_ARGS]    smoke, then the GPU tests (all by default)
#   bash tools/gpu_run.sh bench                  the default bench line, no profiler
#   bash tools/gpu_run.sh rehearse               bench.py --gpus 2 with both ranks on the one GPU
#   bash tools/gpu_run.sh probes                 RCCL latency, any-order launches, v_rsq_f64 accuracy
# Library variants are built on the CPU side first (tools/build_rev_variant.sh, or a copy of
# lib/libbos.so) into gpurun_exp/. Outputs land in gpurun_out/<step>*. The profile set is
# tools/gpu_profile.sh; smoke + tests + profile set tools/gpu_round.sh.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
step=$1
shift
case $step in
  ab)
    timeout -k 10 480 python tools/gn_ab.py "$@" 3 > gpurun_out/ab.txt 2>&1 ;;
  stamps)
    timeout -k 10 120 python tools/solver_stamps.py > gpurun_out/stamps.txt 2>&1 ;;
  trace)
    mode=$1
    lib=${2:-prb-project-bearing-only-slam_amd/lib/libbos.so}
    BOS_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$mode -- \
      python3 tools/shard_step_trace.py $mode 20 > gpurun_out/trace_$mode.log 2>&1 &&
      python3 tools/step_timeline.py gpurun_out/trace_$mode > gpurun_out/timeline_$mode.txt 2>&1 ;;
  shard)
    timeout -k 10 400 python tools/shard_timeline.py 1 2 4 8 > gpurun_out/shard.txt 2>&1 ;;
  tests)
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
      timeout -k 10 800 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 400 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 ;;
  bench)
    timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err ;;
  rehearse)
    timeout -k 10 400 python bench.py --gpus 2 --same-device --steps 20 --warmup 3 --no-cpu-baseline --no-gn-other \
      --tri-steps 0 --replay-steps 0 --cold-steps 0 --no-partition-other > gpurun_out/bench2.json 2> gpurun_out/bench2.err ;;
  probes)
    timeout -k 10 60 ./tools/rccl_latency > gpurun_out/rccl_latency.txt 2>&1 &&
      timeout -k 10 60 ./tools/anyorder_probe > gpurun_out/anyorder.txt 2>&1 &&
      timeout -k 10 60 ./tools/rsq_probe > gpurun_out/rsq.txt 2>&1 ;;
  *)
    echo "unknown step $step" >&2
    exit 2 ;;
esac
