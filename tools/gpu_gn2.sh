# GN timing of two env variants (after the parity suite): $1 tag, $2 env assignment for variant B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu --timeout 400 -p no:cacheprovider > gpurun_out/gn_$1.log 2>&1 || { echo "pytest failed" >> gpurun_out/gn_$1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gn_$1 -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --gn-steps 10 --no-cpu-baseline > gpurun_out/gn_$1.json 2> gpurun_out/gn_$1.err || exit 1
env $2 timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --gn-steps 10 --no-cpu-baseline > gpurun_out/gn_$1_b.json 2> gpurun_out/gn_$1_b.err
