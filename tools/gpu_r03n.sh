# J+H per-wave timeline (cold and warm); front size distribution
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 200 python3 -u tools/front_sizes.py > $O/front_sizes.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/jh_timeline.py fp32 cold > $O/jh_timeline_cold.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/jh_timeline.py fp32 > $O/jh_timeline_warm.txt 2>&1 || exit 1
