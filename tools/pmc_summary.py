"""Summarise the rocprofv3 outputs of tools/gpu_profile.sh into profiles/<tag>_*.{json,csv}.

HBM traffic per launch of the J+H kernel = FETCH_SIZE x 2 + WRITE_SIZE (kB -> bytes): on gfx950
FETCH_SIZE counts half of a wide read (MI355X_MICROARCH.md, HBM/rocprofv3 section)."""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    per = {}
    kern = None
    for r in csv.DictReader(open(path)):
        if "linearize" not in r["Kernel_Name"]:
            continue
        kern = r["Kernel_Name"]
        d = per.setdefault(r["Dispatch_Id"], {"vgpr": r["VGPR_Count"], "sgpr": r["SGPR_Count"],
                                              "lds": r["LDS_Block_Size"], "grid": r["Grid_Size"]})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return kern, list(per.values())


def main(tag, algo_bytes_fp32=None, algo_bytes_fp64=None):
    out = os.path.join(ROOT, "profiles")
    for prec in ("fp32", "fp64"):
        base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{prec}")
        kern, fetch = counters(glob.glob(base + "/fetch/**/run_counter_collection.csv", recursive=True)[0])
        _, write = counters(glob.glob(base + "/write/**/run_counter_collection.csv", recursive=True)[0])
        _, sq = counters(glob.glob(base + "/sq/**/run_counter_collection.csv", recursive=True)[0])
        f = statistics.median(d["FETCH_SIZE"] for d in fetch)
        w = statistics.median(d["WRITE_SIZE"] for d in write)
        sqm = {k: statistics.median(d[k] for d in sq) for k in sq[0] if k.startswith("SQ_")}
        hbm = f * 1024 * 2 + w * 1024
        res = {"kernel": kern, "workload": f"config 3 synthetic, 100k/200k/1M, J+H build {prec}",
               "launches": len(fetch), "FETCH_SIZE_kB_median": f, "WRITE_SIZE_kB_median": w,
               "fetch_bytes_corrected": f * 1024 * 2, "write_bytes": w * 1024, "hbm_bytes_per_launch": hbm,
               "sq_median": sqm, "vgpr": fetch[0]["vgpr"], "sgpr": fetch[0]["sgpr"], "lds_bytes": fetch[0]["lds"],
               "grid": fetch[0]["grid"],
               "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_* in separate passes, --kernel-include-regex "
                         "linearize; FETCH_SIZE and WRITE_SIZE are kB; FETCH doubled per MI355X_MICROARCH.md "
                         "(gfx950 counts half of a wide read); SQ_*CYCLES in quad-cycles summed over waves"}
        algo = algo_bytes_fp32 if prec == "fp32" else algo_bytes_fp64
        if algo:
            res["algorithmic_bytes_per_launch"] = algo
            res["traffic_over_algorithmic"] = hbm / algo
        json.dump(res, open(os.path.join(out, f"{tag}_pmc_linearize_{prec}.json"), "w"), indent=1)
        stats = glob.glob(base + "/trace/**/run_kernel_stats.csv", recursive=True)
        if stats:
            shutil.copy(stats[0], os.path.join(out, f"{tag}_kernel_stats_{prec}.csv"))
        print(prec, f"HBM {hbm / 1e6:.1f} MB/launch", {k: round(v) for k, v in sqm.items()})


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:]))
