# Round 4: odometry-chain J+H A/B (tools/gn_ab.py), J+H parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/gn_ab.py gpurun_exp/libbos_base.so gpurun_exp/libbos_nochain.so gpurun_exp/libbos_chain.so 3 > gpurun_out/c_ab.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3_gn.py tests/test_partitions.py -m gpu -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/c_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/c_pytest.log; exit 1; }
