# smoke + full profile set for the committed numbers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed" >> gpurun_out/smoke.log; exit 1; }
bash tools/gpu_profile.sh ${1:-r01}
