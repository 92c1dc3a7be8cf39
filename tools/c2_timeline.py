"""One GN step's kernel timeline from a rocprofv3 kernel trace directory (diagnostics): the kernels
between the last two J+H launches that are followed by the solver's rhs gather (a GN step, not a
back-to-back J+H replay); WHICH = last (default) or the index of the step among the traced ones.
Usage: python tools/c2_timeline.py TRACE_DIR [WHICH]"""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "linearize_kernel" in r["Kernel_Name"] and i + 1 < len(rows)
       and "gather" in rows[i + 1]["Kernel_Name"]]
w = sys.argv[2] if len(sys.argv) > 2 else "last"
i0, i1 = (idx[-2], idx[-1]) if w == "last" else (idx[int(w)], idx[int(w) + 1])
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    nm = r["Kernel_Name"].replace("bos::dev::(anonymous namespace)::", "").replace("void ", "")[:40]
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} {nm:40s} grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):>6} "
          f"lds {r['LDS_Block_Size']:>6} vgpr {r['VGPR_Count']:>4} stream {r['Stream_Id']}")
