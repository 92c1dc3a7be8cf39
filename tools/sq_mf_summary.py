#!/usr/bin/env python3
"""Per-kernel mean of SQ counters from tools/gpu_sq_mf.sh passes (diagnostics).
usage: sq_mf_summary.py gpurun_out/sqmf_<tag>_0 gpurun_out/sqmf_<tag>_1 ..."""
import csv
import glob
import re
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("bos::dev::(anonymous namespace)::", "").replace("void ", ""))
            key = (name, r.get("Grid_Size", ""))
            tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[key][r["Counter_Name"]] += 1
for key in sorted(tot):
    vals = {c: tot[key][c] / cnt[key][c] for c in tot[key]}
    print(key[0], "grid", key[1])
    print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))
