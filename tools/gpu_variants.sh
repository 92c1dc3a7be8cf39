# J+H kernel time under environment variants: $1 precision, $2.. "VAR=value[,VAR=value]" items ("-" = none)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PREC=$1; shift
i=0
for v in "$@"; do
  E=""
  [ "$v" != "-" ] && E=$(echo $v | tr ',' ' ')
  env $E timeout -k 10 200 python3 bench.py --steps 300 --warmup 30 --gn-steps 0 --no-cpu-baseline --precision $PREC > gpurun_out/v_${PREC}_$i.json 2> gpurun_out/v_${PREC}_$i.err || exit 1
  python3 -c "import json; b=json.loads(open('gpurun_out/v_${PREC}_$i.json').read().splitlines()[-1]); print('$PREC', '$v', round(b['roofline']['kernel_ms']*1e3,2), 'us', round(b['roofline']['frac'],3))" >> gpurun_out/variants.txt
  i=$((i+1))
done
