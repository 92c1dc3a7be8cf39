"""A/B timing of libbos.so build variants on the bench's config-3 world (fp32 J+H, fp64 Schur
solve; experiments). Each variant runs in its own process, alternating A B A B ...; per run: the
median device-stamped phases of 50 synchronous steps, synchronous GN it/s (bos_time_steps, best of
3 x 50), batched GN it/s (bos_step_n of 50, best of 3) and a checksum of the state after 50 iterations (equal for variants that compute the same).

    python tools/gn_ab.py <libA.so> <libB.so> [<libC.so> ...] [rounds]

A variant may carry environment settings for its process: <lib.so>@NAME=VALUE[@NAME=VALUE...].
BOS_AB_CONFIG=c2 in the environment: config 2 (fp64 J+H and solve) instead.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, label):
    sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
    import numpy as np
    import bos
    bos.LIB_PATH = os.path.abspath(lib)
    bos.ALLOW_MISSING_SYMBOLS = True
    if os.environ.get("BOS_AB_CONFIG") == "c2":   # config 2 (fp64), bench.py --config c2's world
        P = bos.synthetic(1000, 2000, 20)
        S = bos.Solver(P, precision=bos.BOS_FP64, solver=bos.BOS_SOLVER_SCHUR, device=0)
    else:
        P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
        S = bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, device=0)
    init = S.get_state()
    S.step()
    S.set_state(*init)
    st = [S.step() for _ in range(50)]
    assert all(g["solver_info"] == 0 for g in st)
    ph = {k: float(np.median([g[k] for g in st])) * 1e3 for k in ("t_linearize_ms", "t_solve_ms", "t_update_ms")}
    pose, lm = S.get_state()
    ck = float(np.abs(pose).sum() + np.abs(lm).sum())
    best = 0.0
    for _ in range(3):
        S.set_state(*init)
        best = max(best, 1e3 / S.time_steps(50))
    import time
    batched = 0.0
    for _ in range(3):   # bos_step_n batches of 50 (the host ahead of the device)
        S.set_state(*init)
        S.synchronize()
        t0 = time.perf_counter()
        S.step_n(50)
        S.synchronize()
        batched = max(batched, 50 / (time.perf_counter() - t0))
    info = bos.plan_inspect(P, solver=bos.BOS_SOLVER_SCHUR)
    plan = f"levels {info['mf_levels']} balance {info['mf_balance_pct']} fits {info['mf_fits']}"
    print(f"{label}: J+H {ph['t_linearize_ms']:.2f} us  solve {ph['t_solve_ms']:.1f} us  "
          f"update {ph['t_update_ms']:.1f} us  GN {best:.0f} it/s  batched {batched:.0f} it/s  state {ck!r}  {plan}",
          flush=True)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
        return
    libs = [a for a in sys.argv[1:] if a.split("@")[0].endswith(".so")]
    rest = [a for a in sys.argv[1:] if a not in libs]
    rounds = int(rest[0]) if rest else 2
    for _ in range(rounds):
        for spec in libs:
            lib, *env = spec.split("@")
            label = os.path.basename(spec)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", lib, label], timeout=120,
                               env=dict(os.environ, **dict(e.split("=", 1) for e in env)))
            if r.returncode != 0:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
