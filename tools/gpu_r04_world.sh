# Round 4: A/B of the pose-group fold against the committed build, the multi-rank tests (one-graph
# sharded step), the default bench line without CPU baselines, the C3 GN parity tests on the
# parallax world (50 fp32 iterations, lpp 1 and 2; 200-iteration pivot check; fp64 20 iterations).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/gn_ab.py gpurun_exp/libbos_r4base.so gpurun_exp/libbos_fold3.so gpurun_exp/libbos_fold3om.so 2 > gpurun_out/w_ab.txt 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest tests/test_sharding.py tests/test_partitions.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w_shard.log 2>&1 || { echo "shard tests failed" >> gpurun_out/w_shard.log; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/w_bench.json 2> gpurun_out/w_bench.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3_gn.py -x -v -s --timeout 550 --timeout-method thread -p no:cacheprovider > gpurun_out/w_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/w_pytest.log; exit 1; }
