# class-40 launch (16 < m <= 40 at 4 waves per SIMD) on the main or the side stream vs the product
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
L=prb-project-bearing-only-slam_amd/lib/libbos.so
timeout -k 10 700 python3 -u tools/gn_rate_check.py $L gpurun_exp/libbos_c40main.so gpurun_exp/libbos_c40side.so $L gpurun_exp/libbos_c40main.so gpurun_exp/libbos_c40side.so > $O/gn.txt 2>&1 || exit 1
for v in c40main c40side; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr_$v -o run --output-format csv -- python3 tools/gn_rate_check.py --child gpurun_exp/libbos_$v.so > $O/prof_$v.txt 2>&1 || exit 1
  python3 tools/step_timeline.py $O/tr_$v > $O/timeline_$v.txt || exit 1
done
