"""Kernel timeline of one GN step from a rocprofv3 kernel trace (diagnostics): the last Schur-ordering
step (between two box-plus launches, with the folded landmarks' backward launch) (graph replays do not report the stats launch). Usage: python tools/step_timeline.py <rocprofv3 output dir>"""
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if "boxplus_kernel" in x["Kernel_Name"]]
# the last step of the default (Schur) solver: its steps run the folded landmarks' backward launch
# (the bench times the nested-dissection ordering after it)
pairs = [(p, q) for p, q in zip(idx, idx[1:]) if any("mf_backward_fold" in x["Kernel_Name"] for x in r[p:q])]
a, b = pairs[-1] if pairs else (idx[-2], idx[-1])
t0 = int(r[a]["End_Timestamp"])
busy = 0.0
for x in r[a + 1:b + 1]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    busy += (e - s) / 1e3
    name = x["Kernel_Name"].replace("(anonymous namespace)::", "").replace("bos::dev::", "").replace("void ", "")
    name = name[:name.index("(")] if "(" in name else name
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {name[:60]:60s} grid {x['Grid_Size_X']:>8s} "
          f"vgpr {x['VGPR_Count']:>3s} agpr {x.get('Accum_VGPR_Count', ''):>3s} lds {x['LDS_Block_Size']:>6s} stream {x['Stream_Id']}")
print(f"step span {(int(r[b]['End_Timestamp']) - t0) / 1e3:.1f} us (from the previous step's end), kernel busy {busy:.1f} us")
