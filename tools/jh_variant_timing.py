"""J+H kernel timing of a libbos.so build variant on config 3 (experiments): warm (back to back) and
cold (1 GiB read before each) event times, cold wave span, and the in-step J+H phase of a GN step.
Usage: python tools/jh_variant_timing.py <path/to/libbos.so> [fp32|fp64]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import numpy as np  # noqa: E402
import bos  # noqa: E402

bos.LIB_PATH = os.path.abspath(sys.argv[1])
bos.ALLOW_MISSING_SYMBOLS = True
prec = bos.BOS_FP64 if len(sys.argv) > 2 and sys.argv[2] == "fp64" else bos.BOS_FP32
P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
S = bos.Solver(P, precision=prec, device=0, lanes_per_pose=int(os.environ.get("BOS_LPP", "0")))
print("created", flush=True)
S.time_linearize(20)
print("warmed", flush=True)
warm = S.time_linearize(100)
print("warm timed", flush=True)
cold = S.time_linearize(20, flush_caches=True)
print("cold timed", flush=True)
spans = []
for _ in range(3):
    T = S.debug_timeline(flush_caches=True).astype(np.int64)
    T = T[T[:, 3] > 0]
    spans.append((T[:, 6].max() - T[:, 3].min()) / 100.0)
print("timelines", flush=True)
init = S.get_state()
S.step()
S.set_state(*init)
st = [S.step() for _ in range(10)]
print("steps", flush=True)
lin = np.median([x["t_linearize_ms"] for x in st]) * 1e3
sol = np.median([x["t_solve_ms"] for x in st]) * 1e3
upd = np.median([x["t_update_ms"] for x in st]) * 1e3
import time  # noqa: E402
pose, lm = S.get_state()
S.set_state(*init)
gn = 1e3 / S.time_steps(50)   # iterations 1..50 from the initial guess, as bench.py
print(f"  chi2 after 10 steps {st[-1]['chi2']:.10e}  state sum {pose.sum():.12e} {lm.sum():.12e}")
print(f"{sys.argv[1]}: warm {warm * 1e3:6.2f} us  cold {cold * 1e3:6.2f} us  cold span {np.median(spans):6.2f} us  "
      f"in-step J+H {lin:6.2f} us  solve {sol:6.1f} us  update {upd:5.1f} us  GN {gn:7.1f} it/s", flush=True)
