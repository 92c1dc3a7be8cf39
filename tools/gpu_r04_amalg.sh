# Round 4: top amalgamation A/B (tools/gn_ab.py), solver stamps, shard timeline, solver/sharding tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/gn_ab.py gpurun_exp/libbos_chain.so gpurun_exp/libbos_amalg.so 3 > gpurun_out/a_ab.txt 2>&1 || exit 1
timeout -k 10 120 python tools/solver_stamps.py > gpurun_out/a_stamps.txt 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3_gn.py tests/test_sharding.py tests/test_partitions.py -m gpu -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/a_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/a_pytest.log; exit 1; }
timeout -k 10 300 python tools/shard_timeline.py 1 2 4 8 > gpurun_out/a_shard.txt 2>&1 || exit 1
