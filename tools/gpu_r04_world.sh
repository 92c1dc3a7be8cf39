# Round 4: the parallax world on the GPU — C3 GN parity (50 fp32 iterations, lpp 1 and 2; 200-iteration
# pivot check; fp64 20 iterations), the multi-rank tests (one-graph sharded step), the default bench
# line without CPU baselines, and the per-rank shard timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_sharding.py tests/test_partitions.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w_shard.log 2>&1 || { echo "shard tests failed" >> gpurun_out/w_shard.log; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/w_bench.json 2> gpurun_out/w_bench.err || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_c3_gn.py -x -v -s --timeout 650 --timeout-method thread -p no:cacheprovider > gpurun_out/w_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/w_pytest.log; exit 1; }
