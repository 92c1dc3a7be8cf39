# GN iterations/s of config 3 under environment variants ($1.. "VAR=value[,VAR=value]" or "-")
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for v in "$@"; do
  E=""
  [ "$v" != "-" ] && E=$(echo $v | tr ',' ' ')
  env $E timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --gn-steps 30 --no-cpu-baseline --no-gn-other --tri-steps 0 > gpurun_out/eb_$i.json 2> gpurun_out/eb_$i.err || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/eb_$i.json')); print('$v', round(d['gn_iters_per_s'],1), {k: round(x*1e3,1) for k,x in d['gn_phase_ms'].items()})" >> gpurun_out/env_bench.txt || exit 1
  i=$((i+1))
done
