# Solver kernel times of the last GN step under environment variants ($1.. "VAR=value[,VAR=value]" or "-")
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for v in "$@"; do
  E=""
  [ "$v" != "-" ] && E=$(echo $v | tr ',' ' ')
  env $E timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/mfv_$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --gn-steps 5 --no-cpu-baseline --no-gn-other > gpurun_out/mfv_$i.json 2> gpurun_out/mfv_$i.err || exit 1
  echo "== $v" >> gpurun_out/mf_variants.txt
  python3 tools/trace_levels.py gpurun_out/mfv_$i >> gpurun_out/mf_variants.txt || exit 1
  i=$((i+1))
done
