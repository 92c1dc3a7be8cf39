#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes of the J+H kernel into profiles/<tag>_pmc_linearize_<prec>.json.

Each pass is a directory written by ``rocprofv3 --pmc ... -d DIR -o run --output-format csv``
(tools/gpu_profile.sh). HBM bytes follow MI355X_MICROARCH.md §HBM: the L2<->fabric request
counters resolved by request size (TCC_EA0_RDREQ_{32B,64B,128B}, TCC_EA0_WRREQ{,_64B}), bytes =
sum(size x count) -- this sidesteps FETCH_SIZE's 64-B tally of 128-B requests on gfx950.

    python tools/pmc_summary.py OUT.json ALGO_BYTES WORKLOAD DIR_READ DIR_WRITE DIR_SQ
"""
import csv
import glob
import hashlib
import json
import os
import statistics
import sys

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "prb-project-bearing-only-slam_amd",
                   "lib", "libbos.so")


def lib_sha256(path=LIB):
    """Hash of the libbos.so the profiled runs loaded (bench.py reports a profile's traffic only for
    the same build)."""
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def load(d, regex="linearize"):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}   # dispatch -> {counter: value}
    meta = {}
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if regex not in r["Kernel_Name"]:
                    continue
                key = (fn, r["Dispatch_Id"])
                per.setdefault(key, {})
                per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                meta = {"kernel": r["Kernel_Name"], "vgpr": int(float(r.get("VGPR_Count", 0) or 0)),
                        "sgpr": int(float(r.get("SGPR_Count", 0) or 0)),
                        "lds_bytes": int(float(r.get("LDS_Block_Size", 0) or 0)),
                        "grid": int(float(r.get("Grid_Size", 0) or 0))}
    return list(per.values()), meta


def median_of(rows):
    keys = sorted({k for r in rows for k in r})
    return {k: statistics.median([r[k] for r in rows if k in r]) for k in keys}


def main():
    out, algo, workload, d_rd, d_wr, d_sq = sys.argv[1:7]
    algo = float(algo)
    rd, meta = load(d_rd)
    wr, _ = load(d_wr)
    sq, _ = load(d_sq)
    r = median_of(rd)
    w = median_of(wr)
    read_bytes = 32 * r.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * r.get("TCC_EA0_RDREQ_64B_sum", 0) \
        + 128 * r.get("TCC_EA0_RDREQ_128B_sum", 0)
    w64 = w.get("TCC_EA0_WRREQ_64B_sum", 0)
    write_bytes = 64 * w64 + 32 * (w.get("TCC_EA0_WRREQ_sum", 0) - w64)
    res = dict(meta)
    res.update({
        "workload": workload,
        "launches": len(rd),
        "read_requests": r,
        "write_requests": w,
        "read_bytes": read_bytes,
        "write_bytes": write_bytes,
        "hbm_bytes_per_launch": read_bytes + write_bytes,
        "sq_median": median_of(sq),
        "method": "rocprofv3 --pmc, separate passes (read requests by size | write requests by size | SQ), "
                  "--kernel-include-regex linearize; bytes = sum(request size x count), median over launches; "
                  "SQ cycle counters in quad-cycles summed over waves",
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": (read_bytes + write_bytes) / algo,
        "libbos_sha256": lib_sha256(),
    })
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("hbm_bytes_per_launch", "traffic_over_algorithmic", "launches")}))


if __name__ == "__main__":
    main()
