# Round 4: fold W W^T block-skip A/B (tools/gn_ab.py; libbos_nomfma.so is a diagnostic build without
# the MFMA products, wrong results, timing bound only), solver stamps, solver parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/gn_ab.py gpurun_exp/libbos_chain.so gpurun_exp/libbos_mfskip.so gpurun_exp/libbos_nomfma.so 3 > gpurun_out/m_ab.txt 2>&1 || exit 1
timeout -k 10 120 python tools/solver_stamps.py > gpurun_out/m_stamps.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3_gn.py -m gpu -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/m_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/m_pytest.log; exit 1; }
