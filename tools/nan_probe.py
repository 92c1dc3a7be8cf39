"""Diagnostics: C1 (the reference dataset) and config 2 with each solver ordering, per library build:
non-finite entries and a state checksum after 5 GN iterations. Usage: python tools/nan_probe.py LIB.so..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import numpy as np  # noqa: E402
import bos  # noqa: E402

import subprocess  # noqa: E402

for spec in sys.argv[1:]:   # LIB.so[@NAME=VALUE...]: environment settings for that process
    lib, *env = spec.split("@")
    code = f"""
import os, sys, numpy as np
sys.path.insert(0, {os.path.join(ROOT, 'prb-project-bearing-only-slam_amd')!r})
import bos
bos.LIB_PATH = {os.path.abspath(lib)!r}
bos.ALLOW_MISSING_SYMBOLS = True
C1 = bos.load_g2o({os.path.join(ROOT, 'tests', 'golden', 'data', 'slam2D_bearing_only_initial_guess.g2o')!r})
C2 = bos.synthetic(1000, 2000, 20)
for name, P in (("c1", C1), ("c2", C2)):
  for prec in (bos.BOS_FP32, bos.BOS_FP64):
    for sv in (bos.BOS_SOLVER_SUPERNODAL, bos.BOS_SOLVER_SCHUR, bos.BOS_SOLVER_DENSE_CHOL):
        if name == "c2" and sv == bos.BOS_SOLVER_DENSE_CHOL: continue
        if os.environ.get("BOS_PROBE_QUICK") and (prec == bos.BOS_FP32 or sv == bos.BOS_SOLVER_DENSE_CHOL): continue
        S = bos.Solver(P, solver=sv, precision=prec)
        st = S.step_n(5)
        p, l = S.get_state()
        print({os.path.basename(lib)!r}, name, "fp32" if prec == bos.BOS_FP32 else "fp64", sv, "nonfinite", int((~np.isfinite(p)).sum() + (~np.isfinite(l)).sum()),
              "sum", float(np.nansum(np.abs(p)) + np.nansum(np.abs(l))), "info", st.get("solver_info"), flush=True)
        S.close()
"""
    subprocess.run([sys.executable, "-c", code.replace(repr(os.path.basename(lib)), repr(os.path.basename(spec)))],
                   timeout=120, env=dict(os.environ, **dict(e.split("=", 1) for e in env)))
