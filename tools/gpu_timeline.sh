set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/jh_timeline.py fp32 > gpurun_out/timeline_fp32.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/jh_timeline.py fp64 > gpurun_out/timeline_fp64.txt 2>&1 || exit 1
