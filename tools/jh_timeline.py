#!/usr/bin/env python3
"""Per-wave timeline of the J+H kernel (config 3): where the waves of one launch spend their time.
Diagnostics only (bos_debug_linearize_timeline). Usage: python tools/jh_timeline.py [fp32|fp64] [cold]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import bos  # noqa: E402

prec = bos.BOS_FP32 if (len(sys.argv) < 2 or sys.argv[1] == "fp32") else bos.BOS_FP64
P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
S = bos.Solver(P, precision=prec, device=0)
for _ in range(30):
    S.linearize_async()
S.synchronize()
cold = len(sys.argv) > 2 and sys.argv[2] == "cold"
runs = [S.debug_timeline(flush_caches=cold) for _ in range(5)]
print("caches:", "cold (1 GiB read before each launch)" if cold else "warm (back to back)")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", f"timeline_{sys.argv[1] if len(sys.argv) > 1 else 'fp32'}.npy"), np.stack(runs))
T = runs[-1].astype(np.int64)
T = T[T[:, 3] > 0]
t0 = T[:, 3].min()
us = lambda x: x / 100.0  # 100 MHz ticks -> us
print(f"waves {len(T)}  kernel span (first start -> last end) {us(T[:, 6].max() - t0):.2f} us")
for kind, name in ((0, "pose"), (1, "landmark")):
    K = T[T[:, 2] == kind]
    if not len(K):
        continue
    start = us(K[:, 3] - t0)
    pro = us(K[:, 4] - K[:, 3])
    loop = us(K[:, 5] - K[:, 4])
    tail = us(K[:, 6] - K[:, 5])
    end = us(K[:, 6] - t0)
    q = lambda a: " ".join(f"{v:6.2f}" for v in np.percentile(a, [0, 10, 50, 90, 100]))
    print(f"{name:9s} n={len(K)}  (percentiles 0/10/50/90/100, us)")
    print(f"   start     {q(start)}")
    print(f"   prologue  {q(pro)}")
    print(f"   loop      {q(loop)}")
    print(f"   tail      {q(tail)}")
    print(f"   end       {q(end)}")
# resident waves over time
ev = np.concatenate([np.stack([T[:, 3], np.ones(len(T))], 1), np.stack([T[:, 6], -np.ones(len(T))], 1)])
ev = ev[np.argsort(ev[:, 0], kind="stable")]
occ = np.cumsum(ev[:, 1])
print("max resident waves", int(occ.max()))
for f in (0.1, 0.25, 0.5, 0.75, 0.9):
    t = t0 + f * (T[:, 6].max() - t0)
    print(f"  at {f:4.2f} of span: {int(((T[:, 3] <= t) & (T[:, 6] > t)).sum())} waves resident")
xcc = (T[:, 7] >> 32) & 0xF
print("waves per xcc", np.bincount(xcc.astype(int), minlength=8).tolist())
print("last end per xcc (us)", [round(us(T[xcc == x, 6].max() - t0), 2) for x in range(8) if (xcc == x).any()])
# per-CU load: HW_ID (gfx9 layout) cu_id [11:8], sh_id [12], se_id [15:13]; the CU key adds the xcc
hw = T[:, 7] & 0xFFFFFFFF
cu_key = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
keys, inv = np.unique(cu_key, return_inverse=True)
npose = np.bincount(inv, weights=(T[:, 2] == 0), minlength=len(keys))
nlm = np.bincount(inv, weights=(T[:, 2] == 1), minlength=len(keys))
last = np.zeros(len(keys))
np.maximum.at(last, inv, us(T[:, 6] - t0))
print(f"CUs seen {len(keys)}; waves per CU: pose {np.percentile(npose, [0, 50, 100]).tolist()}, "
      f"landmark {np.percentile(nlm, [0, 50, 100]).tolist()}")
for p in sorted(set(npose.astype(int).tolist())):
    sel = npose == p
    print(f"  CUs with {p:2d} pose waves: {int(sel.sum()):3d}  landmark waves median {np.median(nlm[sel]):5.1f}  "
          f"last end median {np.median(last[sel]):6.2f} max {last[sel].max():6.2f} us")
