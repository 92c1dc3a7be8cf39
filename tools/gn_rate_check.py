"""GN iterations/s of a libbos.so build three ways (diagnostics): bos_time_steps (synchronous
bos_step in a C loop), synchronous steps from Python (wall), one bos_step_n batch (wall); each from
the initial guess, 50 iterations. Usage: python tools/gn_rate_check.py <lib.so> [more libs]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import numpy as np  # noqa: E402
import bos  # noqa: E402

if sys.argv[1] != "--child":
    import subprocess
    for lib in sys.argv[1:]:
        subprocess.run([sys.executable, os.path.abspath(__file__), "--child", lib], check=True, timeout=120)
    sys.exit(0)
bos.LIB_PATH = os.path.abspath(sys.argv[2])
bos.ALLOW_MISSING_SYMBOLS = True
P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
S = bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, device=0)
init = S.get_state()
S.step()
out = []
for rep in range(3):
    S.set_state(*init)
    c = 1e3 / S.time_steps(50)
    S.set_state(*init)
    t0 = time.perf_counter()
    st = [S.step() for _ in range(50)]
    py = 50 / (time.perf_counter() - t0)
    S.set_state(*init)
    t0 = time.perf_counter()
    S.step_n(50)
    bt = 50 / (time.perf_counter() - t0)
    ph = {k: round(float(np.median([g[k] for g in st])) * 1e3, 2) for k in ("t_linearize_ms", "t_solve_ms", "t_update_ms")}
    bad = [i for i, g in enumerate(st) if g["solver_info"] != 0]
    ph["first_nonpd_iter"] = bad[0] + 1 if bad else None
    ph["chi2_50"] = float(st[-1]["chi2"])
    out.append(f"c-loop {c:7.1f}  python {py:7.1f}  batched {bt:7.1f} it/s  phases(us) {ph}")
import hashlib  # noqa: E402
pose, lm = S.get_state()   # after the last 50-iteration batch from the initial guess
out.append("state sha1 " + hashlib.sha1(pose.tobytes() + lm.tobytes()).hexdigest()[:16])
print(os.path.basename(sys.argv[2]), *out, sep="\n  ", flush=True)
