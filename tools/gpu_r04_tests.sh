# Round 4: RCCL small-collective latency, then the full GPU test suite and smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/rccl_latency > gpurun_out/t_rccl.txt 2>&1 || { echo "rccl_latency failed" >> gpurun_out/t_rccl.txt; exit 1; }
timeout -k 10 60 ./tools/anyorder_probe > gpurun_out/t_anyorder.txt 2>&1 || { echo "anyorder_probe failed" >> gpurun_out/t_anyorder.txt; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t_smoke.log 2>&1 || { echo "smoke failed" >> gpurun_out/t_smoke.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread -p no:cacheprovider > gpurun_out/t_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/t_pytest.log; exit 1; }
