"""Core-clock cycles of the multifrontal front phases per tree level (diagnostics; a library built
with -DBOS_MF_PIVOT_CYCLES, tools/build_full_variant.sh): one config-3 GN step with
bos_debug_solver_stamps, whose backward half then holds s_memtime stamps of every front: [1]
children ready, [2] their update matrices loaded (coherent loads), [3] extend-added, [0] pivot loop
start (rows in registers), [4..6] after two-pivot steps 1-3, [7] pivot loop end. Prints per level the
median k and m, cycles of: child value loads, LDS extend-add, row loads, the whole pivot loop, one
two-pivot step; and the core clock (GHz) from the factor stamps' realtime clock over the pivot loop.
Usage: python tools/pivot_cycles.py gpurun_exp/libbos_pivcyc.so [--rows]
--rows: a build with -DBOS_MF_ROWS_STAMPS, whose stamps [5] / [6] mark the row loads' start and the
end of their first group of 8: prints the row loads split as (extend end -> start), first group,
the rest (up to the pivot loop)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import numpy as np  # noqa: E402
import bos  # noqa: E402

ROWS = "--rows" in sys.argv
args = [a for a in sys.argv[1:] if a != "--rows"]
if args:
    bos.LIB_PATH = os.path.abspath(args[0])
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
print(f"{'lvl':>3} {'fronts':>6} {'k':>4} {'m':>4} {'Uload':>7} {'extend':>7} {'rows':>6} {'loop':>7} {'step':>6} "
      f"{'cyc/piv':>7} {'loop us':>8} {'GHz':>5}")


def med(x):
    x = x[np.isfinite(x)]
    return float(np.median(x)) if len(x) else float("nan")


if ROWS:
    print(f"{'lvl':>3} {'fronts':>6} {'k':>4} {'m':>4} {'pre':>6} {'group0':>7} {'rest':>6} {'rows':>6}")
    for l in sorted(set(lev[ok])):
        sel = ok & (lev == l)
        c = C[sel].astype(float)
        k = meta[sel, 1].astype(float)
        m = k + meta[sel, 2]
        print(f"{l:3d} {sel.sum():6d} {np.median(k):4.0f} {np.median(m):4.0f} {med(c[:, 5] - c[:, 3]):6.0f} "
              f"{med(c[:, 6] - c[:, 5]):7.0f} {med(c[:, 0] - c[:, 6]):6.0f} {med(c[:, 0] - c[:, 3]):6.0f}")
    sys.exit(0)
for l in sorted(set(lev[ok])):
    sel = ok & (lev == l)
    k = meta[sel, 1].astype(float)
    m = k + meta[sel, 2]
    c = C[sel].astype(float)
    c[c == 0] = np.nan
    uload, ext, rows = c[:, 2] - c[:, 1], c[:, 3] - c[:, 2], c[:, 0] - c[:, 3]
    loop = c[:, 7] - c[:, 0]
    step = np.concatenate([c[:, 4] - c[:, 0], c[:, 5] - c[:, 4], c[:, 6] - c[:, 5]])
    us = (F[sel, 5] - F[sel, 4]) / 100.0
    ghz = med(loop / np.maximum(us * 1e3, 1e-9))
    print(f"{l:3d} {sel.sum():6d} {np.median(k):4.0f} {np.median(m):4.0f} {med(uload):7.0f} {med(ext):7.0f} "
          f"{med(rows):6.0f} {med(loop):7.0f} {med(step):6.0f} {med(loop / np.maximum(k, 1)):7.0f} "
          f"{np.median(us):8.2f} {ghz:5.2f}")
