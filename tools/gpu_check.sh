set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu --timeout 400 -p no:cacheprovider > gpurun_out/t8.log 2>&1 || { echo "pytest failed" >> gpurun_out/t8.log; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --gn-steps 3 --no-cpu-baseline > gpurun_out/bench8_fp32.json 2> gpurun_out/bench8_fp32.err
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --gn-steps 0 --precision fp64 --no-cpu-baseline > gpurun_out/bench8_fp64.json 2> gpurun_out/bench8_fp64.err
