"""Summarise the rocprofv3 outputs of tools/gpu_profile.sh into profiles/<tag>_*.

HBM traffic per launch of the J+H kernel comes from the L2's memory-side request counters split
by request size (TCC_EA0_RDREQ_{32B,64B,128B}, TCC_EA0_WRREQ{,_64B}; writes that are not 64 B are
32 B): bytes = sum(size x requests). This resolves the access-width ambiguity of FETCH_SIZE on
gfx950 (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for 16 B/lane streaming reads).
Usage: python tools/pmc_summary.py TAG"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(pattern):
    path = glob.glob(pattern, recursive=True)[0]
    per, meta = {}, {}
    for r in csv.DictReader(open(path)):
        if "linearize" not in r["Kernel_Name"]:
            continue
        meta = {"kernel": r["Kernel_Name"], "vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                "lds_bytes": int(r["LDS_Block_Size"]), "grid": int(r["Grid_Size"])}
        d = per.setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    med = {k: statistics.median(d[k] for d in per.values()) for k in next(iter(per.values()))}
    return meta, med, len(per)


def main(tag):
    out = os.path.join(ROOT, "profiles")
    for prec in ("fp32", "fp64"):
        base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{prec}")
        meta, rd, n = counters(base + "/rd/**/run_counter_collection.csv")
        _, wr, _ = counters(base + "/wr/**/run_counter_collection.csv")
        _, sq, _ = counters(base + "/sq/**/run_counter_collection.csv")
        rbytes = 32 * rd["TCC_EA0_RDREQ_32B_sum"] + 64 * rd["TCC_EA0_RDREQ_64B_sum"] + 128 * rd["TCC_EA0_RDREQ_128B_sum"]
        wbytes = 64 * wr["TCC_EA0_WRREQ_64B_sum"] + 32 * (wr["TCC_EA0_WRREQ_sum"] - wr["TCC_EA0_WRREQ_64B_sum"])
        bench = None
        bj = os.path.join(base, "bench.json")
        if os.path.exists(bj):
            lines = [ln for ln in open(bj).read().splitlines() if ln.startswith("{")]
            bench = json.loads(lines[-1]) if lines else None
        res = dict(meta)
        res.update({"workload": f"config 3 synthetic, 100k poses / 200k landmarks / 1M bearings, J+H build {prec}",
                    "launches": n, "read_requests": rd, "write_requests": wr, "read_bytes": rbytes,
                    "write_bytes": wbytes, "hbm_bytes_per_launch": rbytes + wbytes, "sq_median": sq,
                    "method": "rocprofv3 --pmc, separate passes (read requests by size | write requests by size | "
                              "SQ), --kernel-include-regex linearize; bytes = sum(request size x count); SQ cycle "
                              "counters in quad-cycles summed over waves"})
        if bench:
            algo = bench["roofline"]["algorithmic_bytes_per_launch"]
            res["algorithmic_bytes_per_launch"] = algo
            res["traffic_over_algorithmic"] = (rbytes + wbytes) / algo
            json.dump(bench, open(os.path.join(out, f"{tag}_bench_{prec}.json"), "w"), indent=1)
        json.dump(res, open(os.path.join(out, f"{tag}_pmc_linearize_{prec}.json"), "w"), indent=1)
        stats = glob.glob(base + "/trace/**/run_kernel_stats.csv", recursive=True)
        if stats:
            shutil.copy(stats[0], os.path.join(out, f"{tag}_kernel_stats_{prec}.csv"))
        print(prec, f"read {rbytes / 1e6:.1f} MB write {wbytes / 1e6:.1f} MB per launch",
              f"x{res.get('traffic_over_algorithmic', 0):.2f} algorithmic")


if __name__ == "__main__":
    main(sys.argv[1])
