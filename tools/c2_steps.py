"""Config-2 GN steps for a kernel trace (diagnostics): rocprofv3 --kernel-trace -- python3 tools/c2_steps.py [N]
then tools/c2_timeline.py on the trace directory."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import bos  # noqa: E402

if os.environ.get("BOS_LIB"):   # a library build variant (diagnostics)
    bos.LIB_PATH = os.path.abspath(os.environ["BOS_LIB"])

P = bos.synthetic(1000, 2000, 20)
S = bos.Solver(P, precision=bos.BOS_FP64, device=0, solver=bos.BOS_SOLVER_SCHUR)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    st = S.step()
print("chi2", st["chi2"], "solve_ms", st["t_solve_ms"])
S.close()
