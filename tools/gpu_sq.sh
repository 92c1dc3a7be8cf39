# SQ counter passes on the J+H kernel ($1 precision, $2 tag); env of the caller applies
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
         "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex linearize -d gpurun_out/sq_$2_$i -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 2 --gn-steps 0 --no-cpu-baseline --precision $1 > gpurun_out/sq_$2_$i.out 2>&1 || exit 1
  i=$((i+1))
done
