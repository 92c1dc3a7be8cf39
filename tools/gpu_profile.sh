# Profiles of the J+H kernel on config 3 (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats of a bench run (per-kernel durations)
#   2. PMC passes, one counter group each (no tracing domains together with --pmc):
#      FETCH_SIZE | WRITE_SIZE | SQ occupancy/issue | SQ LDS/VMEM
# Usage: bash tools/gpu_profile.sh TAG   (outputs under gpurun_out/prof_TAG_*)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
for PREC in fp32 fp64; do
  B="python3 bench.py --steps 50 --warmup 5 --gn-steps 3 --no-cpu-baseline --precision $PREC"
  O=gpurun_out/prof_${TAG}_${PREC}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O.trace.out 2>&1 || exit 1
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex linearize -d $O/fetch -o run --output-format csv -- $B > $O.fetch.out 2>&1 || exit 1
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex linearize -d $O/write -o run --output-format csv -- $B > $O.write.out 2>&1 || exit 1
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex linearize -d $O/sq -o run --output-format csv -- $B > $O.sq.out 2>&1 || exit 1
done
