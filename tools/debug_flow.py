"""Debug helper: one GN step on C2 with timing and solver_info (stall counter = info >> 20)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import bos  # noqa: E402

P = bos.synthetic(1000, 2000, 20)
info = bos.plan_inspect(P)
print("plan", {k: info[k] for k in ("n", "mf_supernodes", "mf_levels", "mf_max_front")}, flush=True)
S = bos.Solver(P)
t = time.time()
st = S.step()
print("step", time.time() - t, "s", st, flush=True)
