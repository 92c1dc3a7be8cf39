"""Per-level solver kernel durations of the last GN step in a rocprofv3 kernel trace."""
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(path)))
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
names = ["mf_factor_flow", "mf_backward_flow", "mf_factor_reg", "mf_factor_wave", "mf_factor_level", "mf_forward_wave", "mf_forward_level", "mf_backward_wave", "mf_backward_fold",
         "mf_backward_level", "linearize_kernel", "gather_f64", "to_f64", "boxplus", "reduce_stats"]
# the last GN step: from the last linearize launch followed by a factor launch
idx = [i for i, r in enumerate(rows) if "linearize_kernel" in r["Kernel_Name"]]
start = idx[-1]
step = rows[start:]
for n in names:
    d = [dur(r) for r in step if n + "(" in r["Kernel_Name"] or n + "<" in r["Kernel_Name"]]
    if d:
        print(f"{n:20s} launches {len(d):3d} total {sum(d):8.1f} us  first: {[round(x, 1) for x in d[:8]]}")
t0 = int(step[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in step)
busy = sum(dur(r) for r in step)
print(f"step span {(t1 - t0) / 1e3:.1f} us, kernel busy {busy:.1f} us, launches {len(step)}")
