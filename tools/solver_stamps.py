"""Per-level phase times of the multifrontal solve of one config-3 GN step (diagnostics,
bos_debug_solver_stamps): every front of the per-level launches and of the dataflow launches.
Factor phases: fold, assemble, wait for children (flow), extend-add, pivots, [writes, publish (flow)];
backward: stage, wait for parent (flow), solve, [publish (flow)]. Times in us (100 MHz clock), start
and end relative to the first front of the factorization / backward substitution.
Usage: python tools/solver_stamps.py [c2]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import numpy as np  # noqa: E402
import bos  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] == "c2":   # config 2 (fp64), the GPU parity tests' world
    P = bos.synthetic(1000, 2000, 20)
    S = bos.Solver(P, precision=bos.BOS_FP64, device=0, solver=bos.BOS_SOLVER_SCHUR)
else:
    P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
    S = bos.Solver(P, precision=bos.BOS_FP32, device=0)
nsuper = bos.plan_inspect(P, solver=bos.BOS_SOLVER_SCHUR)["mf_supernodes"]
for _ in range(3):
    S.step()
st, meta = S.debug_solver_stamps(nsuper)
st = st.astype(np.int64)
lev = meta[:, 0]
for name, A, labels in (("factor", st[0], ["fold", "assemble", "wait", "extend", "pivots", "write", "publish"]),
                        ("backward", st[1], ["stage", "wait", "solve", "publish"])):
    ok = A[:, 0] > 0
    end = A.max(axis=1)
    t0 = A[ok, 0].min()
    print(f"{name}: fronts {ok.sum()}, span {(end[ok].max() - t0) / 100:.1f} us")
    print(f"{'lvl':>3} {'fronts':>6} {'k':>4} {'r':>4} {'start':>7} {'end':>7} {'lat':>6} " + " ".join(f"{x:>8}" for x in labels))
    big = meta[:, 1] + meta[:, 2] > 64   # fronts of the blocked workgroup kernel (marked "b")
    for l in sorted(set(lev[ok])):
        for kind in ((False, True) if (ok & (lev == l) & big).any() else (None,)):
            sel = ok & (lev == l) & (True if kind is None else (big == kind))
            if not sel.any():
                continue
            B = A[sel][:, :len(labels) + 1].astype(float)
            B[B == 0] = np.nan
            d = np.diff(B, axis=1) / 100.0
            med = np.nanmedian(d, axis=0)
            tag = "b" if kind else " "
            print(f"{l:2d}{tag} {sel.sum():6d} {np.median(meta[sel, 1]):4.0f} {np.median(meta[sel, 2]):4.0f} "
                  f"{(A[sel, 0].min() - t0) / 100:7.1f} {(end[sel].max() - t0) / 100:7.1f} "
                  f"{np.median(end[sel] - A[sel, 0]) / 100:6.2f} " + " ".join(f"{v:8.2f}" for v in med))
