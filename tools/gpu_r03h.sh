# J+H store cache policy: in-step kernel durations (rocprofv3) and GN rate per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
L=prb-project-bearing-only-slam_amd/lib/libbos.so
for v in prod sc1 sc1nt nt0; do
  lib=$L; [ $v != prod ] && lib=gpurun_exp/libbos_$v.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr_$v -o run --output-format csv -- python3 tools/gn_rate_check.py --child $lib > $O/prof_$v.txt 2>&1 || exit 1
done
timeout -k 10 500 python3 -u tools/gn_rate_check.py $L gpurun_exp/libbos_sc1.so gpurun_exp/libbos_sc1nt.so gpurun_exp/libbos_nt0.so $L gpurun_exp/libbos_sc1.so > $O/gn.txt 2>&1 || exit 1
