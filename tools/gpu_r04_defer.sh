# Round 4: deferred side-stream join A/B (tools/gn_ab.py), step timeline, solver tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/gn_ab.py gpurun_exp/libbos_chain.so gpurun_exp/libbos_defer.so 3 > gpurun_out/d_ab.txt 2>&1 || exit 1
BOS_LIB=gpurun_exp/libbos_defer.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dtr -- python3 tools/shard_step_trace.py plain 20 > gpurun_out/dtr.log 2>&1 || { echo "trace failed" >> gpurun_out/dtr.log; exit 1; }
python3 tools/step_timeline.py gpurun_out/dtr > gpurun_out/d_timeline.txt 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3_gn.py tests/test_sharding.py tests/test_partitions.py -m gpu -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/d_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/d_pytest.log; exit 1; }
