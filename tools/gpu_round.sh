# Round check: smoke, GPU parity suite, then the profile set ($1 = tag)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed" >> gpurun_out/smoke.log; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed" >> gpurun_out/pytest_gpu.log; exit 1; }
bash tools/gpu_profile.sh ${1:-r02}
