# backward launches split by LDS need (BOS_MF_BWD_SPLIT bytes) vs one launch per level
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
L=prb-project-bearing-only-slam_amd/lib/libbos.so
E=gpurun_exp
timeout -k 10 900 python3 -u tools/gn_rate_check.py $L $E/libbos_bs6.so $E/libbos_bs8.so $E/libbos_bs10.so $E/libbos_bs12.so $L $E/libbos_bs6.so $E/libbos_bs8.so $E/libbos_bs10.so $E/libbos_bs12.so > $O/gn.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/gn_rate_check.py --child $E/libbos_bs8.so > $O/prof.txt 2>&1 || exit 1
python3 tools/step_timeline.py $O/tr > $O/timeline_bs8.txt || exit 1
