"""Generate golden vectors for the bearing-only SLAM GN path.

This is an INDEPENDENT, fully vectorised NumPy/SciPy restatement of the reference
(torchipeppo/prb-project-bearing-only-slam) written separately from the C++ oracle
(oracle/bos_oracle.cpp), so that the two cross-check each other. It restates:

* utils/g2o_utils.cpp:10-146            g2o parsing (bearing info column ignored, omega = 1)
* slam/triangulation.cpp:5-74           landmark initial guess, ascending-id landmark order;
                                        1-observation landmarks get the column-pivoted basic solution
* slam/solver_jacobians.cpp:9-168,301-333   errors, analytic Jacobians, angle normalisation
* slam/solver.cpp:27-125                robust kernel (scales e only), H/b accumulation,
                                        damping on all N, fixed-pose elimination, sparse solve
* framework/state.cpp:69-80             left-multiplicative SE(2) box-plus

Outputs tests/golden/<name>.npz (fp64). Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

HERE = os.path.dirname(os.path.abspath(__file__))
PI = np.pi


def wrap(a):
    """normalized_angle: [-pi, pi) (slam/solver_jacobians.cpp:325-333)."""
    a = np.asarray(a, dtype=np.float64)
    a = a - 2 * PI * np.floor((a + PI) / (2 * PI))
    return np.where(a >= PI, a - 2 * PI, a)


def smallest(a):
    """Rotation2D::smallestAngle: fmod 2pi then one correction into [-pi, pi]."""
    t = np.fmod(np.asarray(a, dtype=np.float64), 2 * PI)
    return np.where(t > PI, t - 2 * PI, np.where(t < -PI, t + 2 * PI, t))


def parse(path):
    poses, bear, odo, fix = [], [], [], -1
    for line in open(path):
        t = line.split()
        if not t:
            continue
        if t[0] == "VERTEX_SE2":
            poses.append((int(t[1]), float(t[2]), float(t[3]), float(t[4])))
        elif t[0] == "FIX":
            fix = int(t[1])
        elif t[0] == "EDGE_BEARING_SE2_XY":
            bear.append((int(t[1]), int(t[2]), float(t[3])))
        elif t[0] == "EDGE_SE2":
            u = [float(v) for v in t[6:12]]
            odo.append((int(t[1]), int(t[2]), float(t[3]), float(t[4]), float(t[5]),
                        [[u[0], u[1], u[2]], [u[1], u[3], u[4]], [u[2], u[4], u[5]]]))
    return poses, bear, odo, fix


def setup(path):
    poses, bear, odo, fix = parse(path)
    pid = {p[0]: i for i, p in enumerate(poses)}
    X = np.array([[p[1], p[2], p[3]] for p in poses])
    X[:, 2] = wrap(smallest(X[:, 2]))
    bp = np.array([pid[b[0]] for b in bear])
    blid = np.array([b[1] for b in bear])
    bz = smallest(np.array([b[2] for b in bear]))
    lm_ids = np.unique(blid)                           # std::map => ascending ids
    lid = {int(l): i for i, l in enumerate(lm_ids)}
    bl = np.array([lid[int(l)] for l in blid])
    # triangulation (slam/triangulation.cpp:21-62)
    L = np.zeros((len(lm_ids), 2))
    for j in range(len(lm_ids)):
        ks = np.nonzero(bl == j)[0]
        th = X[bp[ks], 2] + bz[ks]
        s, c = np.sin(th), np.cos(th)
        A = np.stack([s, -c], axis=1)
        r = s * X[bp[ks], 0] - c * X[bp[ks], 1]
        if len(ks) == 1:                                # basic solution, pivot = larger |A0j|
            piv = 0 if abs(A[0, 0]) >= abs(A[0, 1]) else 1
            L[j, piv] = r[0] / A[0, piv]
        else:
            L[j] = np.linalg.lstsq(A, r, rcond=None)[0]
    osrc = np.array([pid[o[0]] for o in odo], dtype=np.int64)
    odst = np.array([pid[o[1]] for o in odo], dtype=np.int64)
    oz = np.array([[o[2], o[3], o[4]] for o in odo]).reshape(-1, 3)
    oom = np.array([o[5] for o in odo]).reshape(-1, 3, 3)
    fixed = pid[fix if fix >= 0 else poses[0][0]]
    return dict(X=X, L=L, bp=bp, bl=bl, bz=bz, osrc=osrc, odst=odst, oz=oz, oom=oom, fixed=fixed,
                lm_ids=lm_ids, pose_ids=np.array([p[0] for p in poses]))


def linearize(S, X, L, k=1.0, lam=0.01):
    NP, NL = len(X), len(L)
    N = 3 * NP + 2 * NL
    bp, bl = S["bp"], S["bl"]
    c, s = np.cos(X[bp, 2]), np.sin(X[bp, 2])
    tx, ty = X[bp, 0], X[bp, 1]
    lx, ly = L[bl, 0], L[bl, 1]
    dx, dy = lx - tx, ly - ty
    gx, gy = c * dx + s * dy, -s * dx + c * dy          # g = R^T (l - t)
    e = wrap(np.arctan2(gy, gx) - S["bz"])
    f = 1.0 / (gx * gx + gy * gy)
    a0, a1 = -gy * f, gx * f
    Jl = np.stack([a0 * c - a1 * s, a0 * s + a1 * c], 1)
    Jth = a0 * (c * ly - s * lx) + a1 * (-s * ly - c * lx)
    Jb = np.concatenate([-Jl, Jth[:, None], Jl], 1)         # [Mb, 5]
    rho = e * e
    chi2 = rho.sum()
    eb = np.where(rho > k, e * np.sqrt(k / np.maximum(rho, 1e-300)), e)
    nrob = int((rho > k).sum())
    colb = np.concatenate([3 * bp[:, None] + np.arange(3), 3 * NP + 2 * bl[:, None] + np.arange(2)], 1)
    rows = [np.repeat(colb, 5, axis=1).ravel()]
    cols = [np.tile(colb, (1, 5)).ravel()]
    vals = [(Jb[:, :, None] * Jb[:, None, :]).ravel()]
    bvec = np.zeros(N)
    np.add.at(bvec, colb.ravel(), (Jb * eb[:, None]).ravel())
    # odometry
    si, di = S["osrc"], S["odst"]
    if len(si):
        cs, ss = np.cos(X[si, 2]), np.sin(X[si, 2])
        txd, tyd = X[di, 0] - X[si, 0], X[di, 1] - X[si, 1]
        pred = np.stack([cs * txd + ss * tyd, -ss * txd + cs * tyd, wrap(X[di, 2] - X[si, 2])], 1)
        eo = pred - S["oz"]
        eo[:, 2] = wrap(eo[:, 2])
        xd, yd = X[di, 0], X[di, 1]
        M = len(si)
        J = np.zeros((M, 3, 6))
        J[:, 0, 0], J[:, 0, 1] = -cs, -ss
        J[:, 1, 0], J[:, 1, 1] = ss, -cs
        J[:, 0, 2], J[:, 1, 2] = -ss * xd + cs * yd, -cs * xd - ss * yd
        J[:, 2, 2] = -1
        J[:, 0, 3], J[:, 0, 4] = cs, ss
        J[:, 1, 3], J[:, 1, 4] = -ss, cs
        J[:, 0, 5], J[:, 1, 5] = ss * xd - cs * yd, ss * yd + cs * xd
        J[:, 2, 5] = 1
        Om = S["oom"]
        rho_o = np.einsum("mi,mij,mj->m", eo, Om, eo)
        chi2 += rho_o.sum()
        nrob += int((rho_o > k).sum())
        sc = np.where(rho_o > k, np.sqrt(k / np.maximum(rho_o, 1e-300)), 1.0)
        eo = eo * sc[:, None]
        Hh = np.einsum("mri,mrs,msj->mij", J, Om, J)
        bb = np.einsum("mri,mrs,ms->mi", J, Om, eo)
        colo = np.concatenate([3 * si[:, None] + np.arange(3), 3 * di[:, None] + np.arange(3)], 1)
        rows.append(np.repeat(colo, 6, axis=1).ravel())
        cols.append(np.tile(colo, (1, 6)).ravel())
        vals.append(Hh.ravel())
        np.add.at(bvec, colo.ravel(), bb.ravel())
    rows.append(np.arange(N)); cols.append(np.arange(N)); vals.append(np.full(N, lam))
    H = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(N, N)).tocsr()
    return H, bvec, chi2, nrob


def step(S, X, L):
    H, b, chi2, nrob = linearize(S, X, L)
    NP = len(X)
    N = H.shape[0]
    keep = np.setdiff1d(np.arange(N), 3 * S["fixed"] + np.arange(3))
    dx = np.zeros(N)
    dx[keep] = spla.spsolve(H[keep][:, keep].tocsc(), -b[keep])
    d = dx[:3 * NP].reshape(-1, 3)
    c, s = np.cos(d[:, 2]), np.sin(d[:, 2])
    Xn = np.stack([c * X[:, 0] - s * X[:, 1] + d[:, 0], s * X[:, 0] + c * X[:, 1] + d[:, 1],
                   wrap(X[:, 2] + d[:, 2])], 1)
    Ln = L + dx[3 * NP:].reshape(-1, 2)
    return Xn, Ln, H, b, chi2, nrob, dx


def golden(name, path, iters=50):
    S = setup(path)
    X, L = S["X"].copy(), S["L"].copy()
    rng = np.random.default_rng(1234)
    out = dict(pose_ids=S["pose_ids"], lm_ids=S["lm_ids"], fixed=S["fixed"], X0=X.copy(), L0=L.copy())
    chis, nrobs = [], []
    for it in range(iters):
        Xn, Ln, H, b, chi2, nrob, dx = step(S, X, L)
        if it == 0:
            N = H.shape[0]
            V = rng.standard_normal((N, 3))
            out.update(H_diag=H.diagonal(), H_nnz=H.nnz, H_fro=np.sqrt((H.data ** 2).sum()), H_V=V,
                       H_HV=H @ V, b0=b, dx0=dx)
        chis.append(chi2)
        nrobs.append(nrob)
        X, L = Xn, Ln
        if it + 1 in (1, 5, 20, 50):
            out[f"X{it + 1}"] = X.copy()
            out[f"L{it + 1}"] = L.copy()
    out["chi2"] = np.array(chis)
    out["n_robust"] = np.array(nrobs)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, "N", 3 * len(X) + 2 * len(L), "chi2[0]", chis[0], "chi2[-1]", chis[-1])


def kats():
    """predict_bearing known answers (tests/solver_stuff.cpp:25-38)."""
    cases = [((0, 0, 0), (1, 0), 0.0), ((0, 0, 0), (0, 1), PI / 2), ((0, 0, 0), (-1, 0), PI),
             ((0, 0, 0), (0, -1), -PI / 2), ((0, 0, 0), (1, 1), PI / 4),
             ((0, 0, PI / 2), (1, 1), -PI / 4), ((0, 0, PI), (1, 0), PI)]
    return cases


if __name__ == "__main__":
    data = os.path.join(HERE, "data")
    golden("mini", os.path.join(data, "mini_initial_guess.g2o"))
    golden("c1", os.path.join(data, "slam2D_bearing_only_initial_guess.g2o"))
    sys.exit(0)
