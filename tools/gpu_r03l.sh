# J+H workgroup size 128/256/512/1024: in-step J+H (device stamps), GN rate, rocprofv3 kernel durations
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
L=prb-project-bearing-only-slam_amd/lib/libbos.so
timeout -k 10 700 python3 -u tools/gn_rate_check.py $L gpurun_exp/libbos_jhb128.so gpurun_exp/libbos_jhb512.so gpurun_exp/libbos_jhb1024.so $L gpurun_exp/libbos_jhb512.so gpurun_exp/libbos_jhb1024.so > $O/gn.txt 2>&1 || exit 1
for v in prod jhb128 jhb512 jhb1024; do
  lib=$L; [ $v != prod ] && lib=gpurun_exp/libbos_$v.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr_$v -o run --output-format csv -- python3 tools/gn_rate_check.py --child $lib > $O/prof_$v.txt 2>&1 || exit 1
done
