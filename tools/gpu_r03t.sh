set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=prb-project-bearing-only-slam_amd/lib/libbos.so
E=gpurun_exp
timeout -k 10 600 python3 -u tools/gn_rate_check.py $L $E/libbos_nohdr.so $E/libbos_prev.so > gpurun_out/hdr_ab.txt 2>&1 || exit 1
