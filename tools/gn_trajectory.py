"""chi^2, max |dx| and solver word over many GN iterations of the bench world (diagnostics).
Usage: python tools/gn_trajectory.py [iterations] [fp32|fp64]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import bos  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 250
prec = bos.BOS_FP64 if len(sys.argv) > 2 and sys.argv[2] == "fp64" else bos.BOS_FP32
P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
S = bos.Solver(P, precision=prec, device=0)
for i in range(n):
    st = S.step()
    if i < 5 or i % 10 == 0 or st["solver_info"] != 0:
        print(f"{i:4d} chi2 {st['chi2']:.6e} robust {st['n_robust']:7d} max|dx| {st['max_abs_dx']:.3e} info {st['solver_info']}",
              flush=True)
