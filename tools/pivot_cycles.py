"""Core-clock cycles of the multifrontal pivot loop per tree level (diagnostics; a library built
with -DBOS_MF_PIVOT_CYCLES, tools/build_full_variant.sh): one config-3 GN step with
bos_debug_solver_stamps, whose backward half then holds s_memtime stamps of every front's pivot loop
([0] start, [1..6] after two-pivot step i, [7] end). Prints per level the median k, cycles of the
whole loop, cycles per two-pivot step (first step and the rest), and the core clock measured
against the factor stamps' realtime clock (loop start .. end).
Usage: python tools/pivot_cycles.py gpurun_exp/libbos_pivcyc.so"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import numpy as np  # noqa: E402
import bos  # noqa: E402

if len(sys.argv) > 1:
    bos.LIB_PATH = os.path.abspath(sys.argv[1])
    bos.ALLOW_MISSING_SYMBOLS = True
P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
S = bos.Solver(P, precision=bos.BOS_FP32, device=0, solver=bos.BOS_SOLVER_SCHUR)
nsuper = bos.plan_inspect(P, solver=bos.BOS_SOLVER_SCHUR)["mf_supernodes"]
for _ in range(3):
    S.step()
st, meta = S.debug_solver_stamps(nsuper)
F = st[0].astype(np.int64)   # realtime (100 MHz): [4] pivots start .. [5] pivots end
C = st[1].astype(np.int64)   # core cycles
lev = meta[:, 0]
ok = (C[:, 0] > 0) & (C[:, 7] > 0) & (F[:, 4] > 0) & (F[:, 5] > 0)
print(f"fronts with cycle stamps: {ok.sum()} of {nsuper}")
print(f"{'lvl':>3} {'fronts':>6} {'k':>4} {'m':>4} {'loop cyc':>9} {'step1':>7} {'step2+':>7} {'cyc/pivot':>9} "
      f"{'loop us':>8} {'GHz':>6}")
for l in sorted(set(lev[ok])):
    sel = ok & (lev == l)
    k = meta[sel, 1]
    m = meta[sel, 1] + meta[sel, 2]
    loop = C[sel, 7] - C[sel, 0]
    s1 = C[sel, 1] - C[sel, 0]
    steps = []
    for i in range(1, 6):
        good = C[sel, i + 1] > 0
        steps.extend((C[sel, i + 1] - C[sel, i])[good & (k >= 2 * (i + 1))])
    us = (F[sel, 5] - F[sel, 4]) / 100.0
    ghz = np.median(loop / np.maximum(us * 1e3, 1e-9))
    print(f"{l:3d} {sel.sum():6d} {np.median(k):4.0f} {np.median(m):4.0f} {np.median(loop):9.0f} {np.median(s1):7.0f} "
          f"{np.median(steps) if steps else float('nan'):7.0f} {np.median(loop / np.maximum(k, 1)):9.0f} "
          f"{np.median(us):8.2f} {ghz:6.2f}")
