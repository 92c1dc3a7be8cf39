# Round 4 diagnostics: kernel timelines of one synchronous step with the level-0 side stream as
# shipped (chain), without it (diagA: class 64 after class 48 on one stream) and forked before the
# rhs gather (diagB: stale inputs, timing only); gn_ab timing of the three.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in chain diagA diagB; do
  BOS_LIB=gpurun_exp/libbos_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fk_$v -- python3 tools/shard_step_trace.py plain 20 > gpurun_out/fk_$v.log 2>&1 || { echo "trace $v failed" >> gpurun_out/fk_$v.log; exit 1; }
  python3 tools/step_timeline.py gpurun_out/fk_$v > gpurun_out/fkl_$v.txt 2>&1 || exit 1
done
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_chain.so gpurun_exp/libbos_diagA.so gpurun_exp/libbos_diagB.so 2 > gpurun_out/fk_ab.txt 2>&1 || exit 1
