# A/B of libbos.so build variants (tools/build_full_variant.sh) with tools/jh_variant_timing.py, in
# alternating processes, two rounds; results appended to gpurun_out/$1.txt.
# Usage: tools/gpu_ab_jh.sh <out-name> variant1 variant2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/$1.txt
shift
for r in 1 2; do
  for v in "$@"; do
    timeout -k 10 120 python tools/jh_variant_timing.py gpurun_exp/libbos_$v.so >> $OUT 2>&1 || exit 1
  done
done
