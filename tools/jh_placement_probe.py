"""In-step J+H of several solver handles of the bench's config-3 world created one after another in
ONE process (each with its own device allocations, all kept alive): whether the spread of the
in-step J+H between processes (bench lines, gn_ab.py) also shows between allocations of one process.
Per handle: median device-stamped J+H and solve over 50 synchronous GN steps from the initial guess,
twice; with warm_steps > 0 the second time follows that many more untimed steps (clock ramp check).

    python tools/jh_placement_probe.py [handles] [warm_steps]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "prb-project-bearing-only-slam_amd"))
import bos  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
    keep = []
    for i in range(n):
        S = bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, device=0)
        keep.append(S)
        init = S.get_state()
        S.step()
        res = []
        for rnd in range(2):   # the same handle twice: the spread within one set of allocations
            if rnd == 1 and warm > 0:
                S.set_state(*init)
                S.step_n(warm)
            S.set_state(*init)
            st = [S.step() for _ in range(50)]
            res.append((np.median([g["t_linearize_ms"] for g in st]) * 1e3,
                        np.median([g["t_solve_ms"] for g in st]) * 1e3))
        print(f"handle {i}: J+H {res[0][0]:.2f} / {res[1][0]:.2f} us  solve {res[0][1]:.1f} / {res[1][1]:.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
