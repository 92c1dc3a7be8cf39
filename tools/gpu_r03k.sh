# fork/join event fence scope: GN rate (state checksums) and one GN step's kernel timeline per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
L=prb-project-bearing-only-slam_amd/lib/libbos.so
timeout -k 10 600 python3 -u tools/gn_rate_check.py $L gpurun_exp/libbos_evdsf.so gpurun_exp/libbos_evdev.so $L gpurun_exp/libbos_evdsf.so gpurun_exp/libbos_evdev.so > $O/gn.txt 2>&1 || exit 1
for v in prod evdsf evdev; do
  lib=$L; [ $v != prod ] && lib=gpurun_exp/libbos_$v.so
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr_$v -o run --output-format csv -- python3 tools/gn_rate_check.py --child $lib > $O/prof_$v.txt 2>&1 || exit 1
  python3 tools/step_timeline.py $O/tr_$v > $O/timeline_$v.txt || exit 1
done
