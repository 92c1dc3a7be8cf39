set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 300 python -u tools/jh_diag_timing.py gpurun_exp/libbos_pairs.so gpurun_exp/libbos_ilp12.so gpurun_exp/libbos_nocomp.so gpurun_exp/libbos_nogath.so gpurun_exp/libbos_ilp10.so > $O/jh_diag.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/gn_rate_check.py gpurun_exp/libbos_pairs.so gpurun_exp/libbos_ilp12.so > $O/gnrate.log 2>&1 || exit 1
