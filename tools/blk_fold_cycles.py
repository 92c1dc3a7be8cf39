"""Wave 0's core cycles per fold-chunk phase in the blocked kernel (diagnostics; a library built with
-DBOS_MF_PIVOT_CYCLES -DBOS_MF_BLK_FOLD_CYCLES): config 2, per level's blocked fronts with folds, the
median per front of: chunks, cycles per chunk in wave 0's record work (head), the wait at the first
barrier, the all-wave work (u-vector and W W^T tiles, wave 0's share), the wait at the second barrier.
Usage: python tools/blk_fold_cycles.py LIB.so"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import numpy as np  # noqa: E402
import bos  # noqa: E402

bos.LIB_PATH = os.path.abspath(sys.argv[1])
bos.ALLOW_MISSING_SYMBOLS = True
P = bos.synthetic(1000, 2000, 20)
S = bos.Solver(P, precision=bos.BOS_FP64, device=0, solver=bos.BOS_SOLVER_SCHUR)
nsuper = bos.plan_inspect(P, solver=bos.BOS_SOLVER_SCHUR)["mf_supernodes"]
for _ in range(3):
    S.step()
st, meta = S.debug_solver_stamps(nsuper)
C = st[1].astype(np.int64)
lev = meta[:, 0]
big = meta[:, 1] + meta[:, 2] > 64
ok = big & (C[:, 4] > 0)
print(f"{'lvl':>3} {'fronts':>6} {'chunks':>6} {'head':>7} {'bar1':>7} {'work':>7} {'bar2':>7}  (cycles per chunk, medians)")
for l in sorted(set(lev[ok])):
    sel = ok & (lev == l)
    c = C[sel].astype(float)
    n = c[:, 4]
    print(f"{l:3d} {sel.sum():6d} {np.median(n):6.0f} " + " ".join(f"{np.median(c[:, i] / n):7.0f}" for i in range(4)))
