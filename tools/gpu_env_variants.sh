# GN timing (kernel trace) of one solver under several environment settings: $1 solver, $2.. "VAR=value" items
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SOLVER=$1; shift
i=0
for v in "$@"; do
  env $v timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/var_$i -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --gn-steps 10 --no-cpu-baseline --solver $SOLVER > gpurun_out/var_$i.json 2> gpurun_out/var_$i.err || exit 1
  i=$((i+1))
done
