"""ORACLE — TEST INFRASTRUCTURE ONLY.

Python side of the CPU restatement of the reference's Gauss-Newton solver
(torchipeppo/prb-project-bearing-only-slam). Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg import this module, as the checker or as the timed
CPU baseline. The product (``libbos.so``) never imports, links or calls it.

Pieces and the reference code each one restates:

* :func:`parse_g2o` — ``utils/g2o_utils.cpp:10-146`` (tokens VERTEX_SE2, VERTEX_XY, FIX,
  EDGE_SE2 with the 6 upper-triangular information values, EDGE_BEARING_SE2_XY with its
  information column ignored and omega = 1, ``bound += 3``).
* :func:`build_problem` — ``executables/bearing_only_slam.cpp:62-71``: default fixed pose
  (``framework/state.cpp:65-67``), ``triangulate_landmarks`` (``slam/triangulation.cpp:65-74``,
  landmarks appended in ascending id order), stix resolution (``framework/state.cpp:58-63``).
* :func:`linearize` — ``slam/solver.cpp:28-69`` through ``bos_oracle.cpp`` (C++).
* :func:`step` — ``slam/solver.cpp:71-96``: gauge fix by dropping the fixed pose's 3 rows
  and columns (``:99-125``), sparse SPD solve of ``H_nf dx = -b_nf`` (the reference uses
  Eigen ``SimplicialLDLT``; here SciPy's sparse direct solver — the solve is not pinned by any
  reference test), re-insertion of the zero fixed-pose delta and the
  left-multiplicative box-plus (``framework/state.cpp:69-80``).

Parity pinning: see DESIGN.md §Oracle (reference KATs + README convergence claim +
independent NumPy restatement ``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

CV_PI = 3.1415926535897932384626433832795


def build(force: bool = False) -> str:
    """Compile the C++ oracle (gcc only; no GPU)."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-C", _HERE, "-s"] + (["-B"] if force else []))
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        fp = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int32)
        L.oracle_version.restype = ctypes.c_int
        L.oracle_set_literal.restype = None
        L.oracle_set_literal.argtypes = [ctypes.c_int]
        L.oracle_get_literal.restype = ctypes.c_int
        L.oracle_bearing_errors.restype = None
        L.oracle_bearing_errors.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 6
        L.oracle_set_wrap_signs.restype = None
        L.oracle_set_wrap_signs.argtypes = [ctypes.c_int, ctypes.c_void_p]
        L.oracle_normalized_angle_f64.restype = ctypes.c_double
        L.oracle_normalized_angle_f64.argtypes = [ctypes.c_double]
        L.oracle_normalized_angle_f32.restype = ctypes.c_float
        L.oracle_normalized_angle_f32.argtypes = [ctypes.c_float]
        L.oracle_smallest_angle_f64.restype = ctypes.c_double
        L.oracle_smallest_angle_f64.argtypes = [ctypes.c_double]
        L.oracle_smallest_angle_f32.restype = ctypes.c_float
        L.oracle_smallest_angle_f32.argtypes = [ctypes.c_float]
        L.oracle_atan2_f64.restype = ctypes.c_double
        L.oracle_atan2_f64.argtypes = [ctypes.c_double, ctypes.c_double]
        L.oracle_atan2_f32.restype = ctypes.c_float
        L.oracle_atan2_f32.argtypes = [ctypes.c_float, ctypes.c_float]
        L.oracle_predict_bearing_f64.restype = ctypes.c_double
        L.oracle_predict_bearing_f64.argtypes = [dp, ctypes.c_double, ctypes.c_double]
        L.oracle_predict_bearing_f32.restype = ctypes.c_float
        L.oracle_predict_bearing_f32.argtypes = [fp, ctypes.c_float, ctypes.c_float]
        L.oracle_predict_odometry_f64.restype = None
        L.oracle_predict_odometry_f64.argtypes = [dp, dp, dp]
        L.oracle_bearing_ej_f64.restype = ctypes.c_double
        L.oracle_bearing_ej_f64.argtypes = [dp, dp, ctypes.c_double, dp]
        L.oracle_bearing_ej_f32.restype = ctypes.c_float
        L.oracle_bearing_ej_f32.argtypes = [fp, fp, ctypes.c_float, fp]
        L.oracle_odometry_ej_f64.restype = None
        L.oracle_odometry_ej_f64.argtypes = [dp, dp, dp, dp, dp]
        L.oracle_odometry_ej_f32.restype = None
        L.oracle_odometry_ej_f32.argtypes = [fp, fp, fp, fp, fp]
        L.oracle_linearize.restype = ctypes.c_int
        L.oracle_linearize.argtypes = [ctypes.c_int] * 5 + [dp, dp, ip, ip, dp, dp, ip, ip, dp, dp,
                                                            ctypes.c_double, ctypes.c_double,
                                                            dp, dp, dp, dp, dp, dp,
                                                            ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.oracle_linearize_owner.restype = ctypes.c_int
        L.oracle_linearize_owner.argtypes = [ctypes.c_int] * 5 + [dp, dp, ip, ip, dp, dp, ip, ip, dp, dp,
                                                                  ip, ip, ip, ip, ip, ip,
                                                                  ctypes.c_double, ctypes.c_double,
                                                                  dp, dp, dp, dp, dp, dp,
                                                                  ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.oracle_apply_boxplus.restype = None
        L.oracle_apply_boxplus.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, dp, dp, dp]
        L.oracle_triangulate.restype = ctypes.c_int
        L.oracle_triangulate.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ip, ip, dp,
                                         ctypes.c_int, ip, dp]
        assert L.oracle_version() == 5
        _lib = L
    return _lib


def _p(a: np.ndarray, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def _pd(a):
    return None if a is None else _p(a, ctypes.c_double)


def _pi(a):
    return _p(a, ctypes.c_int32)


# ----------------------------------------------------------------------------------- angles
def set_literal(on: bool) -> None:
    """Bearing prediction evaluated as the reference writes it (Eigen's ``pose.inverse() * lm`` as
    plain product sums, libm atan2; shares no code with the product) instead of the GPU kernels'
    rounding sequence and portable atan2 (bos_oracle.cpp bearing_g). Use for worlds without
    bearings on the +-pi wrap (the synthetic ones)."""
    lib().oracle_set_literal(1 if on else 0)


_wrap_signs_keep = None


def set_wrap_signs(signs) -> None:
    """Knife-edge bearings (bos_oracle.cpp knife_edge): ``signs[k]`` in {-1, 0, +1} fixes the sign
    of bearing k's error when it lies on the +-pi wrap (within 1e-9 of pi in fp64); None clears."""
    global _wrap_signs_keep
    if signs is None:
        _wrap_signs_keep = None
        lib().oracle_set_wrap_signs(0, None)
        return
    _wrap_signs_keep = np.ascontiguousarray(signs, dtype=np.int8)
    lib().oracle_set_wrap_signs(len(_wrap_signs_keep), _wrap_signs_keep.ctypes.data)


class literal:
    """``with O.literal(wrap_signs=None): ...`` — set_literal(True) and the knife-edge bearings'
    signs (set_wrap_signs; None = none) for the block, both restored after (blocks nest)."""

    def __init__(self, wrap_signs=None):
        self._signs = wrap_signs

    def __enter__(self):
        self._was = lib().oracle_get_literal()
        self._was_signs = _wrap_signs_keep
        set_literal(True)
        set_wrap_signs(self._signs)
        return self

    def __exit__(self, *exc):
        set_literal(bool(self._was))
        set_wrap_signs(self._was_signs)
        return False


def normalized_angle(a: float, precision: int = 64) -> float:
    """``Solver::normalized_angle`` (slam/solver_jacobians.cpp:325-333)."""
    if precision == 32:
        return lib().oracle_normalized_angle_f32(a)
    return lib().oracle_normalized_angle_f64(a)


def smallest_angle(a: float, precision: int = 64) -> float:
    """``Rotation2D::smallestAngle`` (used at slam/solver_jacobians.cpp:18)."""
    if precision == 32:
        return lib().oracle_smallest_angle_f32(a)
    return lib().oracle_smallest_angle_f64(a)


def atan2(y: float, x: float, precision: int = 64) -> float:
    """The portable atan2 shared by the oracle and the GPU path (det_atan2.hpp)."""
    L = lib()
    return L.oracle_atan2_f64(y, x) if precision == 64 else L.oracle_atan2_f32(y, x)


def predict_bearing(pose, lm, precision: int = 64) -> float:
    """``Solver::predict_bearing`` (slam/solver_jacobians.cpp:301-305)."""
    if precision == 32:
        p = np.asarray(pose, dtype=np.float32)
        return lib().oracle_predict_bearing_f32(_p(p, ctypes.c_float), float(lm[0]), float(lm[1]))
    p = np.ascontiguousarray(pose, dtype=np.float64)
    return lib().oracle_predict_bearing_f64(_pd(p), float(lm[0]), float(lm[1]))


def predict_odometry(src, dst) -> np.ndarray:
    """``Solver::predict_odometry`` (slam/solver_jacobians.cpp:307-323)."""
    s = np.ascontiguousarray(src, dtype=np.float64)
    d = np.ascontiguousarray(dst, dtype=np.float64)
    out = np.zeros(3)
    lib().oracle_predict_odometry_f64(_pd(s), _pd(d), _pd(out))
    return out


def bearing_error_and_jacobian(pose, lm, z, precision: int = 64):
    """Bearing ``error_and_jacobian`` (slam/solver_jacobians.cpp:9-95): (e, J[5])."""
    if precision == 32:
        p = np.asarray(pose, dtype=np.float32)
        l = np.asarray(lm, dtype=np.float32)
        J = np.zeros(5, dtype=np.float32)
        e = lib().oracle_bearing_ej_f32(_p(p, ctypes.c_float), _p(l, ctypes.c_float), float(z),
                                         _p(J, ctypes.c_float))
        return e, J
    p = np.ascontiguousarray(pose, dtype=np.float64)
    l = np.ascontiguousarray(lm, dtype=np.float64)
    J = np.zeros(5)
    e = lib().oracle_bearing_ej_f64(_pd(p), _pd(l), float(z), _pd(J))
    return e, J


def bearing_errors(P: "Problem", pose_xyt=None, lm_xy=None) -> np.ndarray:
    """e_k of every bearing at a state (fp64, the current evaluation form, no knife-edge override)."""
    pose = np.ascontiguousarray(P.pose_xyt if pose_xyt is None else pose_xyt, dtype=np.float64)
    lm = np.ascontiguousarray(P.lm_xy if lm_xy is None else lm_xy, dtype=np.float64)
    bp = np.ascontiguousarray(P.b_pose, dtype=np.int32)
    bl = np.ascontiguousarray(P.b_lm, dtype=np.int32)
    bz = np.ascontiguousarray(P.b_z, dtype=np.float64)
    e = np.zeros(len(bz))
    lib().oracle_bearing_errors(len(bz), pose.ctypes.data, lm.ctypes.data, bp.ctypes.data, bl.ctypes.data,
                                bz.ctypes.data, e.ctypes.data)
    return e


def odometry_error_and_jacobian(src, dst, z, precision: int = 64):
    """Odometry ``error_and_jacobian`` (slam/solver_jacobians.cpp:97-168): (e[3], J[3x6])."""
    if precision == 32:
        s = np.asarray(src, dtype=np.float32)
        d = np.asarray(dst, dtype=np.float32)
        zz = np.asarray(z, dtype=np.float32)
        e = np.zeros(3, dtype=np.float32)
        J = np.zeros(18, dtype=np.float32)
        f = ctypes.c_float
        lib().oracle_odometry_ej_f32(_p(s, f), _p(d, f), _p(zz, f), _p(e, f), _p(J, f))
        return e, J.reshape(3, 6)
    s = np.ascontiguousarray(src, dtype=np.float64)
    d = np.ascontiguousarray(dst, dtype=np.float64)
    zz = np.ascontiguousarray(z, dtype=np.float64)
    e = np.zeros(3)
    J = np.zeros(18)
    lib().oracle_odometry_ej_f64(_pd(s), _pd(d), _pd(zz), _pd(e), _pd(J))
    return e, J.reshape(3, 6)


# ----------------------------------------------------------------------------------- g2o
@dataclass
class G2O:
    pose_ids: list = field(default_factory=list)
    pose_xyt: list = field(default_factory=list)
    lm_vertex_ids: list = field(default_factory=list)
    lm_vertex_xy: list = field(default_factory=list)
    fixed_pose_id: int = -1
    bearing_pose_id: list = field(default_factory=list)
    bearing_lm_id: list = field(default_factory=list)
    bearing_raw: list = field(default_factory=list)
    odom_src_id: list = field(default_factory=list)
    odom_dst_id: list = field(default_factory=list)
    odom_z: list = field(default_factory=list)
    odom_omega: list = field(default_factory=list)
    bound: float = 0.0
    unrecognized: list = field(default_factory=list)


def parse_g2o(path: str) -> G2O:
    """Restates ``parse_g2o`` (utils/g2o_utils.cpp:10-146)."""
    g = G2O()
    bound = 0.0
    with open(path) as f:
        for line in f:
            tok = line.split()
            if not tok:
                continue                                       # :113-116
            t = tok[0]
            if t == "VERTEX_SE2":                              # :19-37
                i, x, y, th = int(tok[1]), float(tok[2]), float(tok[3]), float(tok[4])
                bound = max(bound, abs(x), abs(y))
                g.pose_ids.append(i)
                g.pose_xyt.append((x, y, th))
            elif t == "VERTEX_XY":                             # :40-56
                i, x, y = int(tok[1]), float(tok[2]), float(tok[3])
                bound = max(bound, abs(x), abs(y))
                g.lm_vertex_ids.append(i)
                g.lm_vertex_xy.append((x, y))
            elif t == "FIX":                                   # :59-65 (last one wins)
                g.fixed_pose_id = int(tok[1])
            elif t == "EDGE_SE2":                              # :68-98
                s, d = int(tok[1]), int(tok[2])
                x, y, th = float(tok[3]), float(tok[4]), float(tok[5])
                u = [float(v) for v in tok[6:12]]
                om = [[u[0], u[1], u[2]], [u[1], u[3], u[4]], [u[2], u[4], u[5]]]
                g.odom_src_id.append(s)
                g.odom_dst_id.append(d)
                g.odom_z.append((x, y, th))
                g.odom_omega.append(om)
            elif t == "EDGE_BEARING_SE2_XY":                   # :101-110 (info column ignored)
                g.bearing_pose_id.append(int(tok[1]))
                g.bearing_lm_id.append(int(tok[2]))
                g.bearing_raw.append(float(tok[3]))
            else:
                g.unrecognized.append(t)                       # :118-120
    g.bound = bound + 3.0                                      # :124
    return g


@dataclass
class Problem:
    """SoA problem in stix order — the layout ``bos_create`` consumes (include/bos.h)."""
    pose_ids: np.ndarray
    lm_ids: np.ndarray
    pose_xyt: np.ndarray          # [NP,3] float64
    lm_xy: np.ndarray             # [NL,2]
    b_pose: np.ndarray            # [Mb] int32 pose stix
    b_lm: np.ndarray              # [Mb] int32 lm stix
    b_z: np.ndarray               # [Mb] smallestAngle(bearing)
    b_omega: Optional[np.ndarray]
    o_src: np.ndarray             # [Mo] int32
    o_dst: np.ndarray
    o_z: np.ndarray               # [Mo,3]
    o_omega: np.ndarray           # [Mo,3,3]
    fixed: int                    # fixed pose stix

    @property
    def NP(self):
        return len(self.pose_xyt)

    @property
    def NL(self):
        return len(self.lm_xy)

    @property
    def N(self):
        return 3 * self.NP + 2 * self.NL

    def copy_state(self):
        return self.pose_xyt.copy(), self.lm_xy.copy()


def triangulate(pose_xyt, b_pose, b_lmid, b_z, precision: int = 64):
    """``triangulate_landmarks`` (slam/triangulation.cpp:65-74) via the C++ oracle."""
    pose_xyt = np.ascontiguousarray(pose_xyt, dtype=np.float64)
    b_pose = np.ascontiguousarray(b_pose, dtype=np.int32)
    b_lmid = np.ascontiguousarray(b_lmid, dtype=np.int32)
    b_z = np.ascontiguousarray(b_z, dtype=np.float64)
    nmax = len(np.unique(b_lmid)) if len(b_lmid) else 0
    ids = np.zeros(max(nmax, 1), dtype=np.int32)
    xy = np.zeros((max(nmax, 1), 2))
    n = lib().oracle_triangulate(precision, len(pose_xyt), _pd(pose_xyt), len(b_pose), _pi(b_pose),
                                 _pi(b_lmid), _pd(b_z), nmax, _pi(ids), _pd(xy))
    if n < 0:
        raise ValueError(f"oracle_triangulate failed: {n}")
    return ids[:n].copy(), xy[:n].copy()


def build_problem(g: G2O, precision: int = 64) -> Problem:
    """Everything ``main`` does before constructing the Solver
    (executables/bearing_only_slam.cpp:62-71)."""
    if g.lm_vertex_ids:
        raise ValueError("initial-guess inputs must not contain VERTEX_XY (SURVEY.md §3.1)")
    pose_ids = np.asarray(g.pose_ids, dtype=np.int64)
    pid2stix = {int(i): k for k, i in enumerate(g.pose_ids)}  # later duplicate wins (state.cpp:23)
    raw = np.asarray(g.pose_xyt, dtype=np.float64).reshape(-1, 3)
    pose_xyt = raw.copy()
    # theta kept wrapped: the reference stores R (Isometry2f) and reads its angle with t2v
    pose_xyt[:, 2] = [normalized_angle(smallest_angle(t)) for t in raw[:, 2]]
    fixed_id = g.fixed_pose_id if g.fixed_pose_id >= 0 else int(g.pose_ids[0])
    b_pose = np.asarray([pid2stix[i] for i in g.bearing_pose_id], dtype=np.int32)
    b_lmid = np.asarray(g.bearing_lm_id, dtype=np.int32)
    b_z = np.asarray([smallest_angle(a) for a in g.bearing_raw], dtype=np.float64)
    lm_ids, lm_xy = triangulate(pose_xyt, b_pose, b_lmid, b_z, precision)
    lid2stix = {int(i): k for k, i in enumerate(lm_ids)}
    b_lm = np.asarray([lid2stix[i] for i in g.bearing_lm_id], dtype=np.int32)
    o_src = np.asarray([pid2stix[i] for i in g.odom_src_id], dtype=np.int32)
    o_dst = np.asarray([pid2stix[i] for i in g.odom_dst_id], dtype=np.int32)
    o_z = np.asarray(g.odom_z, dtype=np.float64).reshape(-1, 3)
    o_om = np.asarray(g.odom_omega, dtype=np.float64).reshape(-1, 3, 3)
    return Problem(pose_ids, lm_ids, pose_xyt, lm_xy, b_pose, b_lm, b_z, None, o_src, o_dst, o_z,
                   o_om, pid2stix[fixed_id])


# ----------------------------------------------------------------------------------- GN
@dataclass
class Linearization:
    pose_diag: np.ndarray   # [NP,3,3]
    lm_diag: np.ndarray     # [NL,2,2]
    hpl: np.ndarray         # [Mb,3,2]
    hoff: np.ndarray        # [Mo,3,3] (src rows, dst cols)
    b: np.ndarray           # [N]
    chi2: float
    n_robust: int


def owner_index(P: Problem):
    """Bearings grouped by pose and by landmark, odometry entries grouped by pose (CSR), for
    linearize(..., owner=True). Built once per problem and cached on it."""
    idx = getattr(P, "_owner_index", None)
    if idx is not None:
        return idx
    NP, NL = P.NP, P.NL
    bp = np.asarray(P.b_pose, dtype=np.int64)
    bl = np.asarray(P.b_lm, dtype=np.int64)
    pb_obs = np.argsort(bp, kind="stable").astype(np.int32)
    lb_obs = np.argsort(bl, kind="stable").astype(np.int32)
    pb_ptr = np.concatenate([[0], np.cumsum(np.bincount(bp, minlength=NP))]).astype(np.int32)
    lb_ptr = np.concatenate([[0], np.cumsum(np.bincount(bl, minlength=NL))]).astype(np.int32)
    Mo = len(P.o_z)
    ends = np.concatenate([np.asarray(P.o_src, dtype=np.int64), np.asarray(P.o_dst, dtype=np.int64)])
    ent = np.concatenate([2 * np.arange(Mo), 2 * np.arange(Mo) + 1]).astype(np.int32)
    order = np.argsort(ends, kind="stable")
    po_ent = ent[order].astype(np.int32)
    po_ptr = np.concatenate([[0], np.cumsum(np.bincount(ends, minlength=NP))]).astype(np.int32)
    idx = (pb_ptr, pb_obs, lb_ptr, lb_obs, po_ptr, po_ent)
    P._owner_index = idx
    return idx


def linearize(P: Problem, pose_xyt=None, lm_xy=None, kernel_threshold=1.0, damping=0.01,
              precision: int = 64, threads: int = 1, owner: bool = False) -> Linearization:
    """One J+H build. owner=False: the reference's accumulation order (bearings in file order,
    then odometry; per-thread partials when threads > 1). owner=True: the owner-computes parallel
    form (no per-thread copies; the CPU baseline of bench.py)."""
    pose_xyt = np.ascontiguousarray(P.pose_xyt if pose_xyt is None else pose_xyt, dtype=np.float64)
    lm_xy = np.ascontiguousarray(P.lm_xy if lm_xy is None else lm_xy, dtype=np.float64)
    NP, NL, Mb, Mo = P.NP, P.NL, len(P.b_z), len(P.o_z)
    pd = np.zeros((max(NP, 1), 3, 3))
    ld = np.zeros((max(NL, 1), 2, 2))
    hpl = np.zeros((max(Mb, 1), 3, 2))
    hoff = np.zeros((max(Mo, 1), 3, 3))
    b = np.zeros(max(P.N, 1))
    chi2 = ctypes.c_double(0)
    nrob = ctypes.c_int(0)
    bom = None if P.b_omega is None else np.ascontiguousarray(P.b_omega, dtype=np.float64)
    o_z = np.ascontiguousarray(P.o_z, dtype=np.float64)
    o_om = np.ascontiguousarray(P.o_omega, dtype=np.float64)
    if owner:
        pb_ptr, pb_obs, lb_ptr, lb_obs, po_ptr, po_ent = owner_index(P)
        rc = lib().oracle_linearize_owner(precision, NP, NL, Mb, Mo, _pd(pose_xyt), _pd(lm_xy), _pi(P.b_pose),
                                          _pi(P.b_lm), _pd(np.ascontiguousarray(P.b_z)), _pd(bom), _pi(P.o_src),
                                          _pi(P.o_dst), _pd(o_z), _pd(o_om), _pi(pb_ptr), _pi(pb_obs), _pi(lb_ptr),
                                          _pi(lb_obs), _pi(po_ptr), _pi(po_ent), float(kernel_threshold),
                                          float(damping), _pd(pd), _pd(ld), _pd(hpl), _pd(hoff), _pd(b),
                                          ctypes.byref(chi2), ctypes.byref(nrob), int(threads))
        if rc != 0:
            raise RuntimeError(f"oracle_linearize_owner failed: {rc}")
        return Linearization(pd[:NP], ld[:NL], hpl[:Mb], hoff[:Mo], b[:P.N], chi2.value, nrob.value)
    rc = lib().oracle_linearize(precision, NP, NL, Mb, Mo, _pd(pose_xyt), _pd(lm_xy), _pi(P.b_pose),
                                _pi(P.b_lm), _pd(np.ascontiguousarray(P.b_z)), _pd(bom), _pi(P.o_src),
                                _pi(P.o_dst), _pd(o_z), _pd(o_om), float(kernel_threshold),
                                float(damping), _pd(pd), _pd(ld), _pd(hpl), _pd(hoff), _pd(b),
                                ctypes.byref(chi2), ctypes.byref(nrob), int(threads))
    if rc != 0:
        raise RuntimeError(f"oracle_linearize failed: {rc}")
    return Linearization(pd[:NP], ld[:NL], hpl[:Mb], hoff[:Mo], b[:P.N], chi2.value, nrob.value)


def _h_pattern(P: Problem):
    """(rows, cols) of every H contribution in assemble_H's order: pose diagonal, landmark
    diagonal, pose-landmark blocks and their transposes, odometry off-diagonal blocks and theirs."""
    NP = P.NP
    rows, cols = [], []
    pi = 3 * np.arange(NP)
    li = 3 * NP + 2 * np.arange(P.NL)
    for i in range(3):
        for j in range(3):
            rows.append(pi + i); cols.append(pi + j)
    for i in range(2):
        for j in range(2):
            rows.append(li + i); cols.append(li + j)
    bp = 3 * P.b_pose.astype(np.int64)
    bl = 3 * NP + 2 * P.b_lm.astype(np.int64)
    for i in range(3):
        for j in range(2):
            rows += [bp + i, bl + j]; cols += [bl + j, bp + i]
    os_ = 3 * P.o_src.astype(np.int64)
    od = 3 * P.o_dst.astype(np.int64)
    for i in range(3):
        for j in range(3):
            rows += [os_ + i, od + j]; cols += [od + j, os_ + i]
    return np.concatenate(rows), np.concatenate(cols)


def _h_values(lin: Linearization):
    vals = []
    for i in range(3):
        for j in range(3):
            vals.append(lin.pose_diag[:, i, j])
    for i in range(2):
        for j in range(2):
            vals.append(lin.lm_diag[:, i, j])
    for i in range(3):
        for j in range(2):
            vals += [lin.hpl[:, i, j]] * 2
    for i in range(3):
        for j in range(3):
            vals += [lin.hoff[:, i, j]] * 2
    return np.concatenate(vals)


def assemble_H(P: Problem, lin: Linearization):
    """Full symmetric N x N H (scipy CSR, reference dof order: poses 3*stix, landmarks
    3*NP + 2*stix — slam/solver_jacobians.cpp:70-71)."""
    import scipy.sparse as sp
    r, c = _h_pattern(P)
    return sp.coo_matrix((_h_values(lin), (r, c)), shape=(P.N, P.N)).tocsr()


def reduced_system(P: Problem, H, b):
    """``(P H P^T).topLeftCorner(N-3)`` / ``(P b).head(N-3)`` (slam/solver.cpp:71-73):
    drop the fixed pose's 3 rows/cols, keep the order of everything else."""
    keep = np.ones(P.N, dtype=bool)
    keep[3 * P.fixed:3 * P.fixed + 3] = False
    idx = np.nonzero(keep)[0]
    return H[idx][:, idx], b[idx], idx


def reduced_system_csc(P: Problem, lin: Linearization):
    """reduced_system(P, assemble_H(P, lin), lin.b) with H_nf as CSC, through a scatter map built
    once per problem (the pattern is static, slam/solver.hpp:71-82): the same matrix, its
    duplicates summed in another order (fp64 rounding)."""
    import scipy.sparse as sp
    cache = getattr(P, "_hnf_map", None)
    keep = np.ones(P.N, dtype=bool)
    keep[3 * P.fixed:3 * P.fixed + 3] = False
    idx = np.nonzero(keep)[0]
    n = len(idx)
    if cache is None:
        r, c = _h_pattern(P)
        new = np.full(P.N, -1, dtype=np.int64)
        new[idx] = np.arange(n)
        rr, cc = new[r], new[c]
        sel = (rr >= 0) & (cc >= 0)
        uk, inv = np.unique(cc[sel] * n + rr[sel], return_inverse=True)
        indptr = np.concatenate([[0], np.cumsum(np.bincount(uk // n, minlength=n))])
        cache = (sel, inv, (uk % n).astype(np.int32), indptr.astype(np.int64), len(uk))
        P._hnf_map = cache
    sel, inv, indices, indptr, nnz = cache
    data = np.bincount(inv, weights=_h_values(lin)[sel], minlength=nnz)
    return sp.csc_matrix((data, indices, indptr), shape=(n, n)), lin.b[idx], idx


def solve_dx(P: Problem, H, b) -> np.ndarray:
    """Solve ``H_nf dx_nf = -b_nf`` and re-insert the fixed pose as zero delta
    (slam/solver.cpp:75-94)."""
    import scipy.sparse.linalg as spla
    Hnf, bnf, idx = reduced_system(P, H, b)
    dxnf = spla.spsolve(Hnf.tocsc(), -bnf)
    dx = np.zeros(P.N)
    dx[idx] = dxnf
    return dx


def apply_boxplus(P: Problem, pose_xyt, lm_xy, dx, precision: int = 64):
    """``State::apply_boxplus`` (framework/state.cpp:69-80), in place."""
    dx = np.ascontiguousarray(dx, dtype=np.float64)
    lib().oracle_apply_boxplus(precision, P.NP, P.NL, _pd(pose_xyt), _pd(lm_xy), _pd(dx))


def step(P: Problem, pose_xyt, lm_xy, kernel_threshold=1.0, damping=0.01, precision: int = 64,
         threads: int = 1):
    """One ``Solver::step`` (slam/solver.cpp:27-97) in place; returns (chi2, n_robust, dx)."""
    lin = linearize(P, pose_xyt, lm_xy, kernel_threshold, damping, precision, threads)
    H = assemble_H(P, lin)
    dx = solve_dx(P, H, lin.b)
    apply_boxplus(P, pose_xyt, lm_xy, dx, precision)
    return lin.chi2, lin.n_robust, dx


def run(P: Problem, iters: int, kernel_threshold=1.0, damping=0.01, precision: int = 64, threads: int = 1):
    """``iters`` GN steps from the problem's initial state; returns (pose_xyt, lm_xy, chi2s)."""
    pose_xyt, lm_xy = P.copy_state()
    chi = []
    for _ in range(iters):
        c, _, _ = step(P, pose_xyt, lm_xy, kernel_threshold, damping, precision, threads)
        chi.append(c)
    return pose_xyt, lm_xy, chi


def load(path: str, precision: int = 64) -> Problem:
    return build_problem(parse_g2o(path), precision)
