# Schur path: parity suite, then GN timing of both multifrontal orderings on config 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-schur}
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu --timeout 400 -p no:cacheprovider > gpurun_out/gn_$TAG.log 2>&1 || { echo "pytest failed" >> gpurun_out/gn_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gn_$TAG -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --gn-steps 10 --no-cpu-baseline --solver schur > gpurun_out/gn_$TAG.json 2> gpurun_out/gn_$TAG.err || exit 1
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --gn-steps 10 --no-cpu-baseline > gpurun_out/gn_${TAG}_sn.json 2> gpurun_out/gn_${TAG}_sn.err
