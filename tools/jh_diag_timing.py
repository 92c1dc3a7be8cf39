"""J+H build time only (warm back to back, cold after a 512 MiB scrub; HIP events) of libbos.so
builds, each in its own process (experiments; the diagnostic builds compute wrong values, so no GN
step runs). Usage: python tools/jh_diag_timing.py <lib.so> [more libs]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if sys.argv[1] != "--child":
    for lib in sys.argv[1:]:
        subprocess.run([sys.executable, os.path.abspath(__file__), "--child", lib], check=True, timeout=120)
    sys.exit(0)
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import bos  # noqa: E402

bos.LIB_PATH = os.path.abspath(sys.argv[2])
P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
S = bos.Solver(P, precision=bos.BOS_FP32, device=0)
S.time_linearize(20)
w = [S.time_linearize(200) * 1e3 for _ in range(3)]
c = [S.time_linearize(30, flush_caches=True) * 1e3 for _ in range(3)]
print(f"{os.path.basename(sys.argv[2]):22s} warm {min(w):6.2f} us  cold {min(c):6.2f} us", flush=True)
