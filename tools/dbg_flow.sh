cd $GRAFT_REPO_ROOT
for dbg in 8 9 6 7; do
  echo "== C2 BOS_MF_FLOW=1 DBG=$dbg" >> gpurun_out/dbg_flow.log
  BOS_MF_FLOW=1 BOS_MF_FLOW_DBG=$dbg timeout -k 5 25 python tools/debug_flow.py >> gpurun_out/dbg_flow.log 2>&1 || { echo "rc=$?" >> gpurun_out/dbg_flow.log; }
done
