import csv, glob, re, sys
from collections import defaultdict
tot = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(lambda: defaultdict(int))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("bos::dev::(anonymous namespace)::", "").replace("void ", ""))
            key = (name, r.get("Grid_Size", ""))
            tot[key][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[key][r["Counter_Name"]] += 1
for key in sorted(tot):
    v = {c: tot[key][c] / cnt[key][c] for c in tot[key]}
    rd = 32 * v.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * v.get("TCC_EA0_RDREQ_64B_sum", 0) + 128 * v.get("TCC_EA0_RDREQ_128B_sum", 0)
    wr = 64 * v.get("TCC_EA0_WRREQ_64B_sum", 0) + 32 * (v.get("TCC_EA0_WRREQ_sum", 0) - v.get("TCC_EA0_WRREQ_64B_sum", 0))
    print(f"{key[0]:28s} grid {key[1]:>8s} read {rd/1e6:8.1f} MB write {wr/1e6:8.1f} MB")
