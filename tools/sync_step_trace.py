"""Host/device timing of synchronous GN steps (diagnostics): run under
rocprofv3 --runtime-trace --kernel-trace; prints, per step, the time from hipGraphLaunch's call to
the step's first kernel start and from its last kernel end to the return of the host wait.
Usage: rocprofv3 --runtime-trace --kernel-trace -d DIR -o run --output-format csv -- python3 tools/sync_step_trace.py
       python3 tools/sync_step_trace.py DIR"""
import csv
import glob
import os
import sys

if len(sys.argv) > 1:
    d = sys.argv[1]
    kt = sorted(csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])),
                key=lambda x: int(x["Start_Timestamp"]))
    ht = sorted(csv.DictReader(open(glob.glob(d + "/**/*hip_api_trace.csv", recursive=True)[0])),
                key=lambda x: int(x["Start_Timestamp"]))
    launches = [h for h in ht if h["Function"] == "hipGraphLaunch"]
    syncs = [h for h in ht if h["Function"] in ("hipStreamSynchronize", "hipEventSynchronize")]
    firsts = [k for k in kt if "linearize_kernel" in k["Kernel_Name"]]
    lasts = [k for k in kt if "reduce_stats" in k["Kernel_Name"]]
    rows = []
    for L in launches[-15:]:
        t0 = int(L["Start_Timestamp"])
        f = next((k for k in firsts if int(k["Start_Timestamp"]) >= t0), None)
        z = next((k for k in lasts if f and int(k["Start_Timestamp"]) >= int(f["Start_Timestamp"])), None)
        w = next((h for h in syncs if z and int(h["End_Timestamp"]) >= int(z["End_Timestamp"])), None)
        if not (f and z and w):
            continue
        rows.append(((int(L["End_Timestamp"]) - t0) / 1e3, (int(f["Start_Timestamp"]) - t0) / 1e3,
                     (int(z["End_Timestamp"]) - int(f["Start_Timestamp"])) / 1e3,
                     (int(w["End_Timestamp"]) - int(z["End_Timestamp"])) / 1e3))
    for r in rows:
        print("launch call %6.1f us  launch->first kernel %6.1f us  device %6.1f us  last kernel->wait return %6.1f us" % r)
    sys.exit(0)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import bos  # noqa: E402

if os.environ.get("BOS_LIB"):   # a library variant (experiments)
    bos.LIB_PATH = os.path.abspath(os.environ["BOS_LIB"])
    bos.ALLOW_MISSING_SYMBOLS = True

P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
S = bos.Solver(P, precision=bos.BOS_FP32, device=0)
for _ in range(30):
    S.step()
