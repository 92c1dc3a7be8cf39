"""GN rate of the config-3 Schur plan with forced 40-pose leaves (fronts > 64 rows: workgroup path)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "prb-project-bearing-only-slam_amd"))
import bos
P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
for leaf in (0, 40):
    t = time.perf_counter()
    info = bos.plan_inspect(P, 0, 1, solver=bos.BOS_SOLVER_SCHUR, schur_leaf=leaf)
    S = bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, schur_leaf=leaf)
    tc = time.perf_counter() - t
    st = S.step()
    init = S.get_state()
    S.set_state(*init)
    ms = S.time_steps(20)
    print(f"leaf {leaf or 'default'}: max front {info['mf_max_front']}, fits {info['mf_fits']}, create {tc:.1f} s, "
          f"solver_info {st['solver_info']}, GN {1e3 / ms:.0f} it/s ({ms:.3f} ms/step)", flush=True)
    S.close()
