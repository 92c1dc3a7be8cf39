# Request-size-resolved L2<->fabric traffic of the J+H kernel (calibrates FETCH_SIZE/WRITE_SIZE
# for this kernel's access widths). Usage: bash tools/gpu_pmc_bytes.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
for PREC in fp32 fp64; do
  B="python3 bench.py --steps 20 --warmup 2 --gn-steps 0 --no-cpu-baseline --precision $PREC"
  O=gpurun_out/bytes_${TAG}_${PREC}
  timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-include-regex linearize -d $O/rd -o run --output-format csv -- $B > $O.rd.out 2>&1 || exit 1
  timeout -k 10 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --kernel-include-regex linearize -d $O/wr -o run --output-format csv -- $B > $O.wr.out 2>&1 || exit 1
done
