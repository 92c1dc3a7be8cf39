# HBM read/write bytes of the J+H kernel under environment variants ($1 precision, $2.. "VAR=value" or "-")
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PREC=$1; shift
i=0
for v in "$@"; do
  E=""
  [ "$v" != "-" ] && E=$(echo $v | tr ',' ' ')
  env $E timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-include-regex linearize -d gpurun_out/jht_r_$i -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 2 --gn-steps 0 --no-cpu-baseline --precision $PREC > gpurun_out/jht_r_$i.out 2>&1 || exit 1
  env $E timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-include-regex linearize -d gpurun_out/jht_w_$i -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 2 --gn-steps 0 --no-cpu-baseline --precision $PREC > gpurun_out/jht_w_$i.out 2>&1 || exit 1
  python3 - "$v" $i >> gpurun_out/jh_traffic.txt <<'PY' || exit 1
import csv, glob, sys, statistics
v, i = sys.argv[1], sys.argv[2]
def load(d):
    per = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            per.setdefault(r["Dispatch_Id"], {}).setdefault(r["Counter_Name"], 0.0)
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return list(per.values())
rd = statistics.median(32 * p.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * p.get("TCC_EA0_RDREQ_64B_sum", 0) + 128 * p.get("TCC_EA0_RDREQ_128B_sum", 0) for p in load(f"gpurun_out/jht_r_{i}"))
wr = statistics.median(64 * p.get("TCC_EA0_WRREQ_64B_sum", 0) + 32 * (p.get("TCC_EA0_WRREQ_sum", 0) - p.get("TCC_EA0_WRREQ_64B_sum", 0)) for p in load(f"gpurun_out/jht_w_{i}"))
print(v, "read MB", round(rd / 1e6, 2), "write MB", round(wr / 1e6, 2))
PY
  i=$((i+1))
done
