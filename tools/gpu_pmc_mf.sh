# HBM traffic and SQ counters of the multifrontal solver kernels during GN steps ($1 tag); env of the caller applies
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for C in "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY"; do
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex mf_ -d gpurun_out/pmcmf_$1_$i -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --gn-steps 3 --no-cpu-baseline --no-gn-other --tri-steps 0 > gpurun_out/pmcmf_$1_$i.out 2>&1 || exit 1
  i=$((i+1))
done
