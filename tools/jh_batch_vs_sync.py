"""In-step J+H (linearize_kernel start to the next kernel's start) of synchronous bos_step calls (J+H
launched directly, the rest of the step a graph) against bos_step_n batches (every step of a batch
but its last is one graph). Run under rocprofv3 --kernel-trace, then pass the trace directory:
    rocprofv3 --kernel-trace -d gpurun_out/tr_sync -o run --output-format csv -- python3 tools/jh_batch_vs_sync.py sync
    rocprofv3 --kernel-trace -d gpurun_out/tr_batch -o run --output-format csv -- python3 tools/jh_batch_vs_sync.py batch
    python3 tools/jh_batch_vs_sync.py report gpurun_out/tr_sync gpurun_out/tr_batch
Config 3, fp32. Diagnostics only."""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import numpy as np  # noqa: E402

if sys.argv[1] == "report":
    for d in sys.argv[2:]:
        f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
        rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))))
        gaps, durs, tails = [], [], []
        for i, (s, e, n) in enumerate(rows[:-1]):
            if "linearize_kernel" in n and "gather" in rows[i + 1][2]:
                gaps.append((rows[i + 1][0] - s) / 1e3)
                durs.append((e - s) / 1e3)
                tails.append((rows[i + 1][0] - e) / 1e3)
        print(f"{d}: {len(gaps)} J+H launches followed by the gather: start to next start median {np.median(gaps):6.2f} us, "
              f"kernel duration {np.median(durs):6.2f} us, end to next start {np.median(tails):6.2f} us")
    sys.exit(0)

import bos  # noqa: E402

P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
S = bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, device=0)
init = S.get_state()
for rep in range(3):
    S.set_state(*init)
    if sys.argv[1] == "sync":
        for _ in range(40):
            S.step()
    else:
        S.step_n(40)
print("done", flush=True)
