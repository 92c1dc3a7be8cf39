# Profiles of the J+H kernel on config 3, run on the GPU box from the repo root:
#   1. rocprofv3 --kernel-trace --stats of the default bench command (fp32) and of the fp64 bench
#   2. PMC passes, one counter group each (never together with tracing domains):
#      L2<->fabric read requests by size | write requests by size | SQ wave/issue counters
# Usage: bash tools/gpu_profile.sh TAG      (outputs under gpurun_out/prof_TAG_*)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
for PREC in fp32 fp64; do
  O=gpurun_out/prof_${TAG}_${PREC}
  mkdir -p $O
  if [ $PREC = fp32 ]; then B="python3 bench.py"; else B="python3 bench.py --precision fp64"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/bench.json 2> $O/trace.err || exit 1
  P="python3 bench.py --steps 20 --warmup 2 --gn-steps 0 --no-cpu-baseline --precision $PREC"
  timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-include-regex linearize -d $O/rd -o run --output-format csv -- $P > $O/rd.out 2>&1 || exit 1
  timeout -k 10 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-include-regex linearize -d $O/wr -o run --output-format csv -- $P > $O/wr.out 2>&1 || exit 1
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex linearize -d $O/sq -o run --output-format csv -- $P > $O/sq.out 2>&1 || exit 1
done
