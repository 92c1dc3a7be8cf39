# J+H kernel time vs lanes per pose (BOS_LANES_PER_POSE), fp32 and fp64; optional parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-x}
if [ "${2:-}" = parity ]; then
  timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu --timeout 400 -p no:cacheprovider > gpurun_out/parity_$TAG.log 2>&1 || { echo "pytest failed" >> gpurun_out/parity_$TAG.log; exit 1; }
fi
for PREC in fp32 fp64; do
  for L in 1; do
    BOS_LANES_PER_POSE=$L timeout -k 10 200 python bench.py --steps 200 --warmup 20 --gn-steps 0 --no-cpu-baseline --precision $PREC > gpurun_out/lpp_${TAG}_${PREC}_$L.json 2>/dev/null || exit 1
  done
done
