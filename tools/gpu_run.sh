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
#   bash tools/gpu_run.sh final TAG              the driver's order (smoke, GPU suite, bench fp32 + fp64), then
#                                                the profile set (tools/gpu_profile.sh TAG)
#   bash tools/gpu_run.sh c2                     bench.py --config c2 (config 2, fp64, one GPU, vs the CPU backend)
#   bash tools/gpu_run.sh c2trace [LIB]          kernel timeline of one config-2 GN step (tools/c2_steps.py + c2_timeline.py)
#   bash tools/gpu_run.sh ladder                 the N > 1 exchange ladder on the one GPU: two ranks with the default
#                                                p2p, two with --exchange rccl (RCCL refuses ranks sharing a device:
#                                                falls back to the gloo host exchange)
#   bash tools/gpu_run.sh p2p8                   eight ranks on the one GPU, launched as the driver's scaling bench is
#   bash tools/gpu_run.sh l2hit                  J+H L2 hit rate in the step and back to back (TCC_HIT / TCC_MISS)
#   bash tools/gpu_run.sh cycles LIB [--rows]    pivot-loop cycle stamps of a diagnostic build (tools/pivot_cycles.py)
#   bash tools/gpu_run.sh leaf SIZES...          Schur leaf-size sweep (tools/leaf_sweep.py)
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
    timeout -k 10 120 python tools/solver_stamps.py "$@" > gpurun_out/stamps${1:+_$1}.txt 2>&1 ;;
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
  final)
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 &&
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/final_gpu_suite.log 2>&1 &&
      timeout -k 10 400 python bench.py > gpurun_out/final_bench_fp32.json 2> gpurun_out/final_bench_fp32.err &&
      timeout -k 10 400 python bench.py --precision fp64 --no-cpu-baseline > gpurun_out/final_bench_fp64.json \
        2> gpurun_out/final_bench_fp64.err &&
      bash tools/gpu_profile.sh $1 > gpurun_out/final_profile.log 2>&1 ;;
  c2)
    timeout -k 10 300 python bench.py --config c2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err ;;
  c2trace)
    lib=${1:-prb-project-bearing-only-slam_amd/lib/libbos.so}
    BOS_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c2 -- \
      python3 tools/c2_steps.py 20 > gpurun_out/trace_c2.log 2>&1 &&
      python3 tools/c2_timeline.py gpurun_out/trace_c2 > gpurun_out/c2_timeline.txt 2>&1 ;;
  ladder)
    FLAGS="--same-device --steps 20 --warmup 3 --no-cpu-baseline --no-gn-other --tri-steps 0 --replay-steps 20 --cold-steps 0"
    timeout -k 10 400 python bench.py --gpus 2 $FLAGS > gpurun_out/ladder_p2p.json 2> gpurun_out/ladder_p2p.err &&
      timeout -k 10 400 python bench.py --gpus 2 --exchange rccl $FLAGS > gpurun_out/ladder_rccl.json \
        2> gpurun_out/ladder_rccl.err ;;
  p2p8)
    timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 8 --same-device --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/p2p8.json 2> gpurun_out/p2p8.err ;;
  l2hit)
    INSTEP="--replay-steps 0 --cold-steps 0 --no-cpu-baseline --no-gn-other --tri-steps 0"
    WARM="--steps 0 --warmup 0 --replay-steps 20 --cold-steps 0 --no-cpu-baseline --no-gn-other --tri-steps 0"
    timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex linearize -d gpurun_out/tcc_instep \
      -o run --output-format csv -- python3 bench.py $INSTEP > gpurun_out/tcc_instep.json 2> gpurun_out/tcc_instep.err &&
      timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex linearize \
        -d gpurun_out/tcc_warm -o run --output-format csv -- python3 bench.py $WARM > gpurun_out/tcc_warm.json \
        2> gpurun_out/tcc_warm.err &&
      python3 tools/tcc_hit_summary.py gpurun_out/tcc_instep gpurun_out/tcc_warm > gpurun_out/l2hit.txt 2>&1
    rc=$?
    rm -rf gpurun_out/tcc_instep gpurun_out/tcc_warm
    exit $rc ;;
  cycles)
    timeout -k 10 120 python tools/pivot_cycles.py "$@" > gpurun_out/cycles.txt 2>&1 ;;
  leaf)
    timeout -k 10 600 python tools/leaf_sweep.py "$@" > gpurun_out/leaf_sweep.txt 2>&1 ;;
  *)
    echo "unknown step $step" >&2
    exit 2 ;;
esac
