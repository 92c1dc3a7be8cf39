"""Shared helpers for the parity tests: convert between the product's problem (bos.Problem)
and the oracle's (oracle.Problem), and bring both H's into one comparable form."""
import contextlib
import itertools

import numpy as np
import scipy.sparse as sp

import bos
import oracle as O


def to_oracle(P: "bos.Problem") -> "O.Problem":
    """Same arrays, same initial state: parity tests start the oracle and the HIP path from
    identical inputs (the product's own triangulation is checked separately)."""
    return O.Problem(pose_ids=P.pose_ids, lm_ids=P.lm_ids, pose_xyt=P.pose_xyt.copy(), lm_xy=P.lm_xy.copy(),
                     b_pose=P.b_pose.copy(), b_lm=P.b_lm.copy(), b_z=P.b_z.copy(),
                     b_omega=None if P.b_omega is None else P.b_omega.copy(), o_src=P.o_src.copy(),
                     o_dst=P.o_dst.copy(), o_z=P.o_z.copy(), o_omega=P.o_omega.copy(), fixed=P.fixed)


def oracle_lower_nf(Q: "O.Problem", lin) -> sp.csr_matrix:
    """Lower triangle of H with the fixed pose's rows/cols removed (kept in N numbering)."""
    H = O.assemble_H(Q, lin).tocoo()
    keep = np.ones(Q.N, dtype=bool)
    keep[3 * Q.fixed:3 * Q.fixed + 3] = False
    m = (H.row >= H.col) & keep[H.row] & keep[H.col]
    return sp.coo_matrix((H.data[m], (H.row[m], H.col[m])), shape=H.shape).tocsr()


def gpu_lower(rows, cols, vals, N) -> sp.csr_matrix:
    return sp.coo_matrix((vals, (rows.astype(np.int64), cols.astype(np.int64))), shape=(N, N)).tocsr()


def rel_err(a: sp.spmatrix, b: sp.spmatrix) -> float:
    d = (a - b).tocoo()
    scale = max(abs(a).max(), abs(b).max(), 1e-300)
    return (np.abs(d.data).max() if d.nnz else 0.0) / scale


def state_rel_err(pa, la, pb, lb, floor=1e-9):
    """max |a - b| / max(|b|, floor) over poses (x, y, wrapped theta) and landmarks."""
    dp = pa - pb
    dp[:, 2] = (dp[:, 2] + np.pi) % (2 * np.pi) - np.pi
    e1 = np.abs(dp) / np.maximum(np.abs(pb), floor)
    e2 = np.abs(la - lb) / np.maximum(np.abs(lb), floor) if len(lb) else np.zeros(1)
    return max(e1.max(), e2.max())


def close_state(pa, la, pb, lb, rtol=1e-6, atol=1e-9):
    dp = pa - pb
    dp[:, 2] = (dp[:, 2] + np.pi) % (2 * np.pi) - np.pi
    ok_p = np.all(np.abs(dp) <= rtol * np.abs(pb) + atol)
    ok_l = np.all(np.abs(la - lb) <= rtol * np.abs(lb) + atol)
    return ok_p and ok_l, float(np.abs(dp).max()), float(np.abs(la - lb).max() if len(lb) else 0.0)


def knife_edge_bearings(P, tol=1e-9):
    """Bearings whose error (the oracle's literal evaluation, at P's state) lies on the +-pi wrap:
    their sign is decided by the last ulp of atan2 and g (the reference dataset's single-observation
    landmarks after triangulation)."""
    with O.literal():
        e = O.bearing_errors(P)
    return np.nonzero(np.abs(e) >= np.pi - tol)[0], e


def wrap_signs_from_gpu(P, b_gpu, kt=1.0):
    """The sign the GPU path gave each knife-edge bearing's error, read off its exported b (fp64,
    P's state): flipping bearing k's error changes b by -2 J_k^T w e_k (robust-scaled e_k) on its
    pose's and landmark's dofs; the combination of flips that reproduces the GPU's b (to 1e-9 of
    max |b|) gives the signs. None when P has no such bearing. The oracle then evaluates every
    bearing literally (Eigen's product sums, libm atan2: no code shared with the product) and only
    takes these signs from the GPU (bos_oracle.cpp knife_edge)."""
    ks, e = knife_edge_bearings(P)
    if len(ks) == 0:
        return None
    # The only bearings whose sign may be taken from the GPU are the sole observations of their
    # landmark (triangulated onto their own ray); on the reference dataset exactly
    # the three on landmarks 69, 112 and 114 (the set cannot grow silently). Their sign
    # is parity-unpinned.
    counts = np.bincount(P.b_lm, minlength=P.NL)
    assert np.all(counts[P.b_lm[ks]] == 1), [int(k) for k in ks if counts[P.b_lm[k]] != 1]
    if getattr(P, "lm_ids", None) is not None and P.NP == 301 and P.NL == 141:
        assert sorted(int(P.lm_ids[P.b_lm[k]]) for k in ks) == [69, 112, 114], ks
    Q = to_oracle(P)
    with O.literal():
        lin = O.linearize(Q, kernel_threshold=kt)
        contrib = []
        for k in ks:
            ek, J = O.bearing_error_and_jacobian(P.pose_xyt[P.b_pose[k]], P.lm_xy[P.b_lm[k]], P.b_z[k])
            w = 1.0 if P.b_omega is None else float(P.b_omega[k])
            rho = ek * w * ek
            es = ek * np.sqrt(kt / rho) if rho > kt else ek
            d = np.zeros(P.N)
            d[3 * P.b_pose[k]:3 * P.b_pose[k] + 3] = J[:3] * w * es
            d[3 * P.NP + 2 * P.b_lm[k]:3 * P.NP + 2 * P.b_lm[k] + 2] = J[3:] * w * es
            contrib.append(d)
    keep = np.ones(P.N, dtype=bool)
    keep[3 * P.fixed:3 * P.fixed + 3] = False
    best, best_flip = None, None
    for flips in itertools.product((False, True), repeat=len(ks)):
        alt = lin.b - sum(2 * c for c, f in zip(contrib, flips) if f)
        err = np.abs(b_gpu - alt)[keep].max()
        if best is None or err < best:
            best, best_flip = err, flips
    assert best <= 1e-9 * np.abs(lin.b[keep]).max(), f"no sign combination of the knife-edge bearings reproduces b ({best})"
    signs = np.zeros(len(P.b_z), dtype=np.int8)
    for k, f in zip(ks, best_flip):
        signs[k] = -int(np.sign(e[k])) if f else int(np.sign(e[k]))
    return signs


@contextlib.contextmanager
def literal_oracle(P, b_gpu=None, kt=1.0):
    """The oracle in its literal form for the block, with the knife-edge bearings' signs taken from
    the GPU path's b at P's initial state (b_gpu, or one fp64 GPU linearization made here)."""
    if b_gpu is None and len(knife_edge_bearings(P)[0]):
        S = bos.Solver(P, kernel_threshold=kt)
        S.linearize()
        b_gpu = S.export_system()[3]
        S.close()
    signs = None if b_gpu is None else wrap_signs_from_gpu(P, b_gpu, kt)
    with O.literal(wrap_signs=signs):
        yield signs


def lin_parity(P, precision=bos.BOS_FP64, kt=1.0, damping=0.01, tol=1e-12, p999=None, btol=None, **solver_kw):
    """H, b, chi^2 of one GPU J+H build against the oracle's literal evaluation (knife-edge
    bearings' signs from the GPU's fp64 b, literal_oracle)."""
    Q = to_oracle(P)
    S = bos.Solver(P, precision=precision, kernel_threshold=kt, damping=damping, **solver_kw)
    st = S.linearize()
    rows, cols, vals, b = S.export_system()
    b64 = b
    if precision != bos.BOS_FP64 and len(knife_edge_bearings(P)[0]):
        S64 = bos.Solver(P, kernel_threshold=kt, damping=damping, **solver_kw)
        S64.linearize()
        b64 = S64.export_system()[3]
        S64.close()
    with literal_oracle(P, b64, kt):
        lin = O.linearize(Q, kernel_threshold=kt, damping=damping, precision=32 if precision == bos.BOS_FP32 else 64)
    Hg = gpu_lower(rows, cols, vals, P.N)
    Ho = oracle_lower_nf(Q, lin)
    eh = rel_err(Hg, Ho)
    # b of the fixed pose is discarded by the reference (solver.cpp:73) and not produced here
    keep = np.ones(P.N, dtype=bool)
    keep[3 * P.fixed:3 * P.fixed + 3] = False
    assert np.all(b[~keep] == 0.0)
    eb = np.abs(b - lin.b)[keep].max() / max(np.abs(lin.b[keep]).max(), 1e-300)
    assert eh <= tol, f"H rel err {eh}"
    assert eb <= (10 * tol if btol is None else btol), f"b rel err {eb}"
    if p999 is not None:
        # scale-invariant per-entry error |dH_ij| / sqrt(H_ii H_jj) (bounded by 1 for SPD H)
        d = (Hg - Ho).tocoo()
        dg = np.abs(Ho.diagonal())
        per = np.abs(d.data) / np.sqrt(np.maximum(dg[d.row] * dg[d.col], 1e-300))
        assert np.quantile(per, 0.999) <= p999, np.quantile(per, 0.999)
    if precision == bos.BOS_FP64:
        assert abs(st["chi2"] - lin.chi2) <= 1e-9 * max(lin.chi2, 1.0)
        assert st["n_robust"] == lin.n_robust
    else:
        assert abs(st["chi2"] - lin.chi2) <= 1e-3 * max(lin.chi2, 1.0)
    S.close()
    return eh, eb
