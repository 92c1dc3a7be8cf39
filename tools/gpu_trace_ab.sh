set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
for v in pairs ilp12; do
  BOS_LIB=gpurun_exp/libbos_$v.so timeout -k 10 120 rocprofv3 --runtime-trace --kernel-trace -d gpurun_out/tr/$v -o run --output-format csv -- python3 tools/sync_step_trace.py > gpurun_out/tr/$v.log 2>&1 || exit 1
  python3 tools/sync_step_trace.py gpurun_out/tr/$v >> gpurun_out/tr/$v.txt 2>&1 || exit 1
done
