# SQ counter passes on the multifrontal solver kernels during GN steps ($1 tag); env of the caller applies
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR"; do
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex mf_ -d gpurun_out/sqmf_$1_$i -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --gn-steps 3 --no-cpu-baseline --no-gn-other --tri-steps 0 > gpurun_out/sqmf_$1_$i.out 2>&1 || exit 1
  i=$((i+1))
done
