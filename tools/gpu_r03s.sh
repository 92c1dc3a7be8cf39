# lane headers (one dependent load fewer per J+H lane) vs the previous build: GN rate + checksums,
# in-step J+H kernel durations, cold J+H timeline; GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
L=prb-project-bearing-only-slam_amd/lib/libbos.so
E=gpurun_exp
timeout -k 10 120 python3 -u tools/gn_rate_check.py --child $L > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u tools/gn_rate_check.py $L $E/libbos_prev.so $L $E/libbos_prev.so $L $E/libbos_prev.so > $O/gn.txt 2>&1 || exit 1
for v in prod prev; do
  lib=$L; [ $v != prod ] && lib=$E/libbos_$v.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr_$v -o run --output-format csv -- python3 tools/gn_rate_check.py --child $lib > $O/prof_$v.txt 2>&1 || exit 1
done
timeout -k 10 200 python3 -u tools/jh_timeline.py fp32 cold > $O/jh_timeline_cold.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || exit 1
