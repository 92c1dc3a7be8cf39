# Profile set for the committed numbers ($1 = tag, e.g. r03), fp32 and fp64 J+H builds:
#   * rocprofv3 --kernel-trace --stats of bench.py with only the timed GN steps (no warm replay, no
#     cold builds): its linearize_kernel average is the in-step J+H, the line's roofline.kernel_ms
#   * three separate --pmc passes on those in-step J+H launches (read requests by size | writes |
#     SQ), and the same on back-to-back builds (warm replay, --steps 0)
#   * the full default bench line (fp32) under --kernel-trace --stats
# Results land in gpurun_out/prof_<tag>/; tools/collect_profiles.py copies the summaries.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03}
O=gpurun_out/prof_$TAG
mkdir -p $O
INSTEP="--replay-steps 0 --cold-steps 0 --no-cpu-baseline --no-gn-other --tri-steps 0"
for P in fp32 fp64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_${P}_instep -o run --output-format csv -- \
    python3 bench.py $INSTEP --precision $P > $O/bench_${P}_instep.json 2> $O/bench_${P}_instep.err || exit 1
  for MODE in instep warm; do
    if [ $MODE = instep ]; then ARGS="$INSTEP"; else ARGS="--steps 0 --warmup 0 --replay-steps 20 --cold-steps 0 --no-cpu-baseline --no-gn-other --tri-steps 0"; fi
    i=0
    for C in "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" \
             "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
      timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex linearize -d $O/pmc_${P}_${MODE}_$i -o run --output-format csv -- \
        python3 bench.py $ARGS --precision $P > $O/pmc_${P}_${MODE}_$i.json 2> $O/pmc_${P}_${MODE}_$i.err || exit 1
      i=$((i+1))
    done
    ALGO=$(python3 -c "
import sys; sys.path.insert(0, 'prb-project-bearing-only-slam_amd'); import bos
P = bos.synthetic(100000, 200000, 10, seed=0xB05EED01 + 3)
print((36 if '$P' == 'fp32' else 64) * len(P.b_z) + (80 if '$P' == 'fp32' else 152) * len(P.o_z) + (60 if '$P' == 'fp32' else 120) * P.NP + (32 if '$P' == 'fp32' else 64) * P.NL)")
    python3 tools/pmc_summary.py $O/pmc_linearize_${P}_${MODE}.json $ALGO \
      "config 3 synthetic, 100k poses / 200k landmarks / 1M bearings, J+H build $P, $MODE" \
      $O/pmc_${P}_${MODE}_0 $O/pmc_${P}_${MODE}_1 $O/pmc_${P}_${MODE}_2 || exit 1
  done
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace_fp32_default -o run --output-format csv -- \
  python3 bench.py > $O/bench_fp32_default.json 2> $O/bench_fp32_default.err || exit 1
python3 tools/step_timeline.py $O/trace_fp32_default > $O/gn_step_timeline.txt || exit 1
timeout -k 10 180 python3 tools/solver_stamps.py > $O/solver_stamps.txt 2> $O/solver_stamps.err || exit 1
