# round 5: L2 hit rate of the J+H in the GN step and back to back (one --pmc pass each)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
INSTEP="--replay-steps 0 --cold-steps 0 --no-cpu-baseline --no-gn-other --tri-steps 0"
WARM="--steps 0 --warmup 0 --replay-steps 20 --cold-steps 0 --no-cpu-baseline --no-gn-other --tri-steps 0"
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex linearize -d gpurun_out/tcc_instep -o run --output-format csv -- python3 bench.py $INSTEP > gpurun_out/tcc_instep.json 2> gpurun_out/tcc_instep.err &&
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex linearize -d gpurun_out/tcc_warm -o run --output-format csv -- python3 bench.py $WARM > gpurun_out/tcc_warm.json 2> gpurun_out/tcc_warm.err
rc=$?
python3 tools/tcc_hit_summary.py gpurun_out/tcc_instep gpurun_out/tcc_warm > gpurun_out/r05_tcc_hit.txt 2>&1
rm -rf gpurun_out/tcc_instep gpurun_out/tcc_warm
exit $rc
