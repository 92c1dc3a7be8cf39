"""Compare the J+H output (exported H lower triangle and b after one linearize, config 3, fp32) of two
libbos.so builds (diagnostics). Usage: python tools/jh_export_diff.py <libA.so> <libB.so>"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if sys.argv[1] == "--child":
    sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
    import numpy as np
    import bos
    bos.LIB_PATH = os.path.abspath(sys.argv[2])
    bos.ALLOW_MISSING_SYMBOLS = True
    P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
    S = bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, device=0)
    st = S.linearize()
    rows, cols, vals, b = S.export_system()
    np.savez(sys.argv[3], rows=rows, cols=cols, vals=vals, b=b, chi2=np.array([st["chi2"]]))
    sys.exit(0)
import numpy as np  # noqa: E402
out = []
for i, lib in enumerate(sys.argv[1:3]):
    f = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"jh_export_{i}.npz")
    subprocess.run([sys.executable, os.path.abspath(__file__), "--child", lib, f], check=True, timeout=300)
    out.append(np.load(f))
a, c = out
print("chi2", float(a["chi2"][0]), float(c["chi2"][0]))
same_pat = np.array_equal(a["rows"], c["rows"]) and np.array_equal(a["cols"], c["cols"])
print("pattern equal", same_pat)
dv = np.flatnonzero(a["vals"] != c["vals"])
db = np.flatnonzero(a["b"] != c["b"])
print("H values differing", dv.size, "of", a["vals"].size, "; b entries differing", db.size, "of", a["b"].size)
for q in dv[:12]:
    print("  H", int(a["rows"][q]), int(a["cols"][q]), a["vals"][q], c["vals"][q])
for q in db[:12]:
    print("  b", int(q), a["b"][q], c["b"][q])
# which poses differ: by their odometry entry count and bearing count
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import bos  # noqa: E402
P = bos.synthetic(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)
nodo = np.bincount(np.concatenate([P.o_src, P.o_dst]), minlength=P.NP)
nb = np.bincount(P.b_pose, minlength=P.NP)
bad = np.zeros(P.NP, bool)
dp = db[db < 3 * P.NP] // 3
bad[dp] = True
print("poses differing", bad.sum(), "landmark b entries differing", int((db >= 3 * P.NP).sum()))
for k in sorted(set(nodo)):
    sel = nodo == k
    print(f"  odometry entries {k}: poses {sel.sum()}, differing {int((bad & sel).sum())}")
for k in sorted(set(nb))[:12]:
    sel = nb == k
    print(f"  bearings {k}: poses {sel.sum()}, differing {int((bad & sel).sum())}")
# the pose stix vs ids: are differing poses those whose first odometry entry is the destination side?
first_is_dst = np.zeros(P.NP, bool)
print("fixed pose", P.fixed)
