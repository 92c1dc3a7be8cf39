"""J+H parity check of a libbos.so build (experiments): mini, C1 and C2 (fp64 and fp32) against the
oracle, then one C3 fp32 build checked for finite values and one GN step; prints as it goes.
Usage: python tools/jh_check.py [path/to/libbos.so]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "prb-project-bearing-only-slam_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import bos  # noqa: E402

if len(sys.argv) > 1:
    bos.LIB_PATH = os.path.abspath(sys.argv[1])
    bos.ALLOW_MISSING_SYMBOLS = True
import oracle as O  # noqa: E402
from helpers import gpu_lower, oracle_lower_nf, rel_err, to_oracle  # noqa: E402

DATA = os.path.join(ROOT, "tests", "golden", "data")
for name, P in (("mini", bos.load_g2o(os.path.join(DATA, "mini_initial_guess.g2o"))),
                ("c1", bos.load_g2o(os.path.join(DATA, "slam2D_bearing_only_initial_guess.g2o"))),
                ("c2", bos.synthetic(1000, 2000, 20))):
    for prec in (bos.BOS_FP64, bos.BOS_FP32):
        Q = to_oracle(P)
        S = bos.Solver(P, precision=prec)
        st = S.linearize()
        rows, cols, vals, b = S.export_system()
        lin = O.linearize(Q, precision=32 if prec == bos.BOS_FP32 else 64)
        eh = rel_err(gpu_lower(rows, cols, vals, P.N), oracle_lower_nf(Q, lin))
        keep = np.ones(P.N, dtype=bool)
        keep[3 * P.fixed:3 * P.fixed + 3] = False
        eb = float(np.abs(b - lin.b)[keep].max() / max(np.abs(lin.b[keep]).max(), 1e-300))
        print(f"{name} fp{prec}: H rel err {eh:.3g}  b rel err {eb:.3g}  chi2 {st['chi2']:.9g} vs {lin.chi2:.9g}", flush=True)
        S.close()
P = bos.synthetic(100000, 200000, 10, seed=0xB05EED01 + 3)
S = bos.Solver(P, precision=bos.BOS_FP32)
st = S.linearize()
rows, cols, vals, b = S.export_system()
print(f"c3 fp32: chi2 {st['chi2']:.9g} finite H {np.isfinite(vals).all()} b {np.isfinite(b).all()} max|H| {np.abs(vals).max():.3g}",
      flush=True)
st = S.step()
print("c3 step:", st, flush=True)
