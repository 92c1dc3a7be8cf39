# front size distribution (fixed bins); default bench line of the final build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 200 python3 -u tools/front_sizes.py > $O/front_sizes.txt 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || exit 1
