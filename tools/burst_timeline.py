"""Per-rank kernel timelines of the sharded GN step from a rocprofv3 kernel trace of
`tools/shard_step_trace.py ranks W` (diagnostics): the ranks' phases run one after another with host
exchanges between them, so the trace splits into bursts at idle gaps > 40 us; the last iteration's
3 W bursts are phase 0 of ranks 0..W-1, phase 1 of ranks 0..W-1, phase 2 of ranks 0..W-1. Prints
every rank's three bursts (kernel start / end relative to the burst's first kernel) for the ranks
named (default: all). Usage: python tools/burst_timeline.py <rocprofv3 dir> W [ranks...]"""
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
W = int(sys.argv[2])
want = [int(a) for a in sys.argv[3:]] or list(range(W))
r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
bursts, cur, last_end = [], [], None
for x in r:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    if last_end is not None and s - last_end > 40000:
        bursts.append(cur)
        cur = []
    cur.append(x)
    last_end = e if last_end is None else max(last_end, e)
bursts.append(cur)
it = bursts[-3 * W:]


def name(x):
    n = x["Kernel_Name"].replace("(anonymous namespace)::", "").replace("bos::dev::", "").replace("void ", "")
    return n[:n.index("(")] if "(" in n else n


for rk in want:
    tot = 0.0
    for ph in range(3):
        b = it[ph * W + rk]
        t0 = int(b[0]["Start_Timestamp"])
        span = (max(int(x["End_Timestamp"]) for x in b) - t0) / 1e3
        tot += span
        print(f"rank {rk} phase {ph}: {len(b)} launches, span {span:.1f} us")
        for x in b:
            s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
            print(f"  {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {name(x)[:56]:56s} grid {x['Grid_Size_X']:>8s} "
                  f"stream {x['Stream_Id']}")
    print(f"rank {rk}: phases total {tot:.1f} us")
