# fold: product (fp32 source, uniform stores, no loop-top wait) vs the fp64 copy (nof32) vs deep
# (values two chunks ahead); fold stamps; GN rate with state checksums; GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
L=prb-project-bearing-only-slam_amd/lib/libbos.so
timeout -k 10 500 python3 -u tools/gn_rate_check.py $L gpurun_exp/libbos_nof32.so gpurun_exp/libbos_deep.so $L gpurun_exp/libbos_nof32.so gpurun_exp/libbos_deep.so > $O/gn.txt 2>&1 || exit 1
BOS_LIB=gpurun_exp/libbos_foldst.so timeout -k 10 180 python3 -u tools/fold_stamps.py > $O/fold_stamps_prod.txt 2>&1 || exit 1
BOS_LIB=gpurun_exp/libbos_deepst.so timeout -k 10 180 python3 -u tools/fold_stamps.py > $O/fold_stamps_deep.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || exit 1
