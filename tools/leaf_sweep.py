"""Schur ordering leaf size vs GN time on config 3 (experiments; bos_options.schur_leaf).
Usage: python tools/leaf_sweep.py 10 8 12 ..."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import numpy as np  # noqa: E402
import bos  # noqa: E402

P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
for leaf in [int(a) for a in sys.argv[1:]]:
    t0 = time.perf_counter()
    info = bos.plan_inspect(P, solver=bos.BOS_SOLVER_SCHUR, schur_leaf=leaf)
    S = bos.Solver(P, precision=bos.BOS_FP32, device=0, solver=bos.BOS_SOLVER_SCHUR, schur_leaf=leaf)
    tc = time.perf_counter() - t0
    S.step()
    st = [S.step() for _ in range(10)]
    sol = np.median([x["t_solve_ms"] for x in st]) * 1e3
    t0 = time.perf_counter()
    S.step_n(20)
    it = 20 / (time.perf_counter() - t0)
    print(f"leaf {leaf}: levels {info['mf_levels']} max front {info['mf_max_front']} upper {info['mf_max_front_upper']} "
          f"fits {info['mf_fits']} balance {info['mf_balance_pct']} flops {info['mf_flops']:.3g} nnzL {info['nnz_factor']} "
          f"create+plan {tc:.1f} s  solve {sol:.1f} us  GN batched {it:.0f} it/s chi2 {st[-1]['chi2']:.8e}", flush=True)
    S.close()
