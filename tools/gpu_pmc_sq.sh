# SQ/TCC counters for the J+H kernel (one counter group per pass; no tracing domains with --pmc)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PREC=${1:-fp32}
B="python3 bench.py --steps 20 --warmup 2 --gn-steps 0 --no-cpu-baseline --precision $PREC"
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex linearize -d gpurun_out/sq1_$PREC -o run --output-format csv -- $B > gpurun_out/sq1_$PREC.out 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex linearize -d gpurun_out/sq2_$PREC -o run --output-format csv -- $B > gpurun_out/sq2_$PREC.out 2>&1
