# Profile set for the committed numbers ($1 = tag, e.g. r02): for fp32 and fp64 J+H builds
#   * three separate --pmc passes on the J+H kernel (read requests by size | writes | SQ), once on
#     back-to-back builds (warm) and once on builds from cold caches (512 MiB read before each)
#   * rocprofv3 --kernel-trace --stats of the bench command (bench JSON + kernel stats), and of a
#     cold-only bench run (its linearize_kernel average is the bench line's roofline.kernel_ms)
# Results land in gpurun_out/prof_<tag>/; tools/collect_profiles.py copies the summaries.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
O=gpurun_out/prof_$TAG
mkdir -p $O
for P in fp32 fp64; do
  CPU=""
  [ $P = fp64 ] && CPU="--no-cpu-baseline"
  for MODE in warm cold; do
    if [ $MODE = warm ]; then
      ARGS="--steps 20 --warmup 2 --cold-steps 0"; SUF=""
    else
      ARGS="--steps 1 --warmup 0 --cold-steps 30"; SUF="_cold"
    fi
    i=0
    for C in "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" \
             "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
      timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex linearize -d $O/pmc_${P}${SUF}_$i -o run --output-format csv -- \
        python3 bench.py $ARGS --gn-steps 0 --tri-steps 0 --no-cpu-baseline --precision $P > $O/pmc_${P}${SUF}_$i.json 2> $O/pmc_${P}${SUF}_$i.err || exit 1
      i=$((i+1))
    done
    ALGO=$(python3 -c "import json; print(json.loads([l for l in open('$O/pmc_${P}${SUF}_0.json').read().splitlines() if l.startswith('{')][-1])['roofline']['algorithmic_bytes_per_launch'])")
    python3 tools/pmc_summary.py $O/pmc_linearize_${P}${SUF}.json $ALGO \
      "config 3 synthetic, 100k poses / 200k landmarks / 1M bearings, J+H build $P, $MODE caches" \
      $O/pmc_${P}${SUF}_0 $O/pmc_${P}${SUF}_1 $O/pmc_${P}${SUF}_2 || exit 1
    cp $O/pmc_linearize_${P}${SUF}.json profiles/${TAG}_pmc_linearize_${P}${SUF}.json || exit 1
  done
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_${P}_cold -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --cold-steps 50 --gn-steps 0 --tri-steps 0 --no-cpu-baseline --precision $P \
    > $O/bench_${P}_cold.json 2> $O/bench_${P}_cold.err || exit 1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace_$P -o run --output-format csv -- \
    python3 bench.py --steps 200 --warmup 20 --precision $P $CPU > $O/bench_$P.json 2> $O/bench_$P.err || exit 1
done
