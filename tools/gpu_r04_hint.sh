# Round 4: fold-hint A/B (tools/gn_ab.py), solver stamps, solver parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_base.so gpurun_exp/libbos_hint.so 3 > gpurun_out/h_ab.txt 2>&1 || exit 1
timeout -k 10 120 python tools/solver_stamps.py > gpurun_out/h_stamps.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3_gn.py -m gpu -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/h_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/h_pytest.log; exit 1; }
