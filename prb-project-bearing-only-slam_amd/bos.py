"""ctypes binding of libbos.so (include/bos.h, include/bos_host.h).

Python mirror of the reference's host interface for the GN path
(torchipeppo/prb-project-bearing-only-slam):

* :func:`load_g2o`  — ``parse_g2o`` + default fixed pose + ``triangulate_landmarks``
  (utils/g2o_utils.cpp:10-146, executables/bearing_only_slam.cpp:62-71,
  slam/triangulation.cpp:65-74), implemented in C++ inside libbos.so.
* :class:`Solver`   — ``proj02::Solver`` (slam/solver.hpp:21-92): ``step()``,
  ``set_kernel_threshold``, ``set_damping_factor``, ``state``.

There is no CPU fallback: constructing a :class:`Solver` without a visible HIP device raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libbos.so")
# diagnostics tools that load an older build (tools/gn_ab.py) set this: its missing entry points
# are then left unbound instead of failing the load
ALLOW_MISSING_SYMBOLS = False

BOS_OK = 0
BOS_FP64 = 64
BOS_FP32 = 32
BOS_SOLVER_SUPERNODAL = 0
BOS_SOLVER_DENSE_CHOL = 1
BOS_SOLVER_ROCSOLVER_RF = 2
BOS_SOLVER_SCHUR = 3
BOS_SOLVER_SPARSE_CHOL = BOS_SOLVER_SCHUR
BOS_PARTITION_SUBTREE = 0
BOS_PARTITION_OBSERVATIONS = 1
ABI_VERSION = 3

# every symbol declared in include/bos.h and include/bos_host.h
EXPORTED_SYMBOLS = [
    "bos_default_options", "bos_last_error", "bos_abi_version", "bos_device_count", "bos_device_peer_access",
    "bos_nccl_unique_id",
    "bos_create", "bos_destroy", "bos_set_kernel_threshold", "bos_set_damping_factor", "bos_step", "bos_step_n",
    "bos_linearize", "bos_linearize_async", "bos_synchronize", "bos_system_info_get", "bos_export_system",
    "bos_get_state", "bos_set_state", "bos_get_last_dx",
    "bos_dataset_load_g2o", "bos_dataset_synthetic", "bos_dataset_problem", "bos_dataset_pose_ids",
    "bos_dataset_landmark_ids", "bos_dataset_fixed_pose_id", "bos_dataset_bound", "bos_dataset_ground_truth",
    "bos_dataset_write_g2o", "bos_dataset_free", "bos_plan_inspect", "bos_plan_mf_selftest",
    "bos_debug_linearize_timeline", "bos_triangulate", "bos_triangulate_async", "bos_plan_shard_selftest",
    "bos_plan_node_owner", "bos_step_phase", "bos_exchange_size", "bos_exchange_download", "bos_exchange_upload",
    "bos_node_owner",
    "bos_debug_set_g2o_parser", "bos_debug_inject_stall", "bos_debug_set_step_graph", "bos_debug_solver_stamps",
    "bos_time_linearize", "bos_time_triangulate", "bos_time_steps", "bos_cpu_gn_create", "bos_cpu_gn_step", "bos_cpu_gn_get_state",
    "bos_cpu_gn_destroy", "bos_normalized_angle_f64", "bos_normalized_angle_f32", "bos_exchange_p2p_handle",
    "bos_exchange_p2p_connect", "bos_time_facade_steps", "bos_debug_facade_selftest", "bos_set_exchange_timeout",
    "bos_last_step_stamps",
]

P2P_HANDLE_BYTES = 64   # include/bos.h BOS_P2P_HANDLE_BYTES

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


class BosError(RuntimeError):
    pass


class bos_problem(ctypes.Structure):
    _fields_ = [("num_poses", ctypes.c_int32), ("num_landmarks", ctypes.c_int32),
                ("num_bearings", ctypes.c_int32), ("num_odometry", ctypes.c_int32),
                ("pose_xyt", _dp), ("landmark_xy", _dp), ("bearing_pose", _ip), ("bearing_landmark", _ip),
                ("bearing_z", _dp), ("bearing_omega", _dp), ("odom_src", _ip), ("odom_dst", _ip),
                ("odom_z", _dp), ("odom_omega", _dp), ("fixed_pose", ctypes.c_int32)]


class bos_options(ctypes.Structure):
    _fields_ = [("precision", ctypes.c_int32), ("solver", ctypes.c_int32), ("device", ctypes.c_int32),
                ("rank", ctypes.c_int32), ("world_size", ctypes.c_int32), ("nccl_unique_id", ctypes.c_void_p),
                ("kernel_threshold", ctypes.c_double), ("damping", ctypes.c_double), ("stream", ctypes.c_void_p),
                ("partition", ctypes.c_int32), ("lanes_per_pose", ctypes.c_int32), ("schur_leaf", ctypes.c_int32)]


class bos_step_stats(ctypes.Structure):
    _fields_ = [("chi2", ctypes.c_double), ("n_robust", ctypes.c_int32), ("solver_info", ctypes.c_int32),
                ("max_abs_dx", ctypes.c_double), ("t_linearize_ms", ctypes.c_double),
                ("t_exchange_ms", ctypes.c_double), ("t_solve_ms", ctypes.c_double), ("t_update_ms", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class bos_system_info(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("nnz_lower", ctypes.c_int64), ("nnz_factor", ctypes.c_int64),
                ("algorithmic_bytes", ctypes.c_int64), ("num_block_values", ctypes.c_int64),
                ("lanes_per_pose", ctypes.c_int32), ("pose_lane_groups", ctypes.c_int32),
                ("landmark_lanes", ctypes.c_int32), ("own_fronts", ctypes.c_int32), ("top_fronts", ctypes.c_int32),
                ("comm_ranks", ctypes.c_int32), ("partition", ctypes.c_int32),
                ("pl_factored", ctypes.c_int32), ("fold_fp32", ctypes.c_int32), ("layout_bytes", ctypes.c_int64)]


class bos_plan_info(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("nnz_lower", ctypes.c_int64), ("nnz_factor", ctypes.c_int64),
                ("num_block_values", ctypes.c_int64), ("lanes_per_pose", ctypes.c_int64),
                ("flops_temporal", ctypes.c_double), ("flops_nested_dissection", ctypes.c_double),
                ("ordering", ctypes.c_char * 32), ("mf_supernodes", ctypes.c_int64),
                ("mf_levels", ctypes.c_int64), ("mf_max_front", ctypes.c_int64), ("mf_flops", ctypes.c_double),
                ("mf_update_bytes", ctypes.c_int64), ("mf_fits", ctypes.c_int64),
                ("mf_max_front_upper", ctypes.c_int64), ("mf_balance_pct", ctypes.c_int64),
                ("shard_own_fronts", ctypes.c_int64), ("shard_top_fronts", ctypes.c_int64),
                ("shard_roots", ctypes.c_int64), ("shard_ex1_doubles", ctypes.c_int64),
                ("shard_ex2_doubles", ctypes.c_int64), ("shard_pose_lanes", ctypes.c_int64),
                ("shard_own_pose_lanes", ctypes.c_int64), ("shard_lm_lanes", ctypes.c_int64),
                ("shard_update_nodes", ctypes.c_int64), ("mf_fold_fp32", ctypes.c_int64),
                ("lm_lanes_consecutive", ctypes.c_int64), ("pose_odometry_chain", ctypes.c_int64)]


_lib = None


def lib():
    """Load libbos.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BosError(f"{LIB_PATH} not built: run `make -C {_HERE}` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    sig = {
        "bos_default_options": (None, [ctypes.POINTER(bos_options)]),
        "bos_last_error": (ctypes.c_char_p, []),
        "bos_abi_version": (ctypes.c_int, []),
        "bos_device_count": (ctypes.c_int, []),
        "bos_device_peer_access": (ctypes.c_int, [ctypes.c_int32, _ip, _ip]),
        "bos_nccl_unique_id": (ctypes.c_int, [vp, ctypes.c_int64]),
        "bos_create": (ctypes.c_int, [ctypes.POINTER(bos_problem), ctypes.POINTER(bos_options), ctypes.POINTER(vp)]),
        "bos_destroy": (ctypes.c_int, [vp]),
        "bos_set_kernel_threshold": (ctypes.c_int, [vp, ctypes.c_double]),
        "bos_set_damping_factor": (ctypes.c_int, [vp, ctypes.c_double]),
        "bos_step": (ctypes.c_int, [vp, ctypes.POINTER(bos_step_stats)]),
        "bos_step_n": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(bos_step_stats)]),
        "bos_linearize": (ctypes.c_int, [vp, ctypes.POINTER(bos_step_stats)]),
        "bos_linearize_async": (ctypes.c_int, [vp]),
        "bos_synchronize": (ctypes.c_int, [vp]),
        "bos_triangulate": (ctypes.c_int, [vp]),
        "bos_triangulate_async": (ctypes.c_int, [vp]),
        "bos_debug_linearize_timeline": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64),
                                                        ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]),
        "bos_system_info_get": (ctypes.c_int, [vp, ctypes.POINTER(bos_system_info)]),
        "bos_export_system": (ctypes.c_int, [vp, ctypes.c_int64, _ip, _ip, _dp, _dp]),
        "bos_get_state": (ctypes.c_int, [vp, _dp, _dp]),
        "bos_set_state": (ctypes.c_int, [vp, _dp, _dp]),
        "bos_get_last_dx": (ctypes.c_int, [vp, _dp]),
        "bos_dataset_load_g2o": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]),
        "bos_dataset_synthetic": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64,
                                                 ctypes.POINTER(vp)]),
        "bos_dataset_problem": (ctypes.c_int, [vp, ctypes.POINTER(bos_problem)]),
        "bos_dataset_pose_ids": (_ip, [vp]),
        "bos_dataset_landmark_ids": (_ip, [vp]),
        "bos_dataset_fixed_pose_id": (ctypes.c_int32, [vp]),
        "bos_dataset_bound": (ctypes.c_float, [vp]),
        "bos_dataset_ground_truth": (ctypes.c_int, [vp, ctypes.POINTER(_dp), ctypes.POINTER(_dp)]),
        "bos_dataset_write_g2o": (ctypes.c_int, [vp, ctypes.c_char_p, _dp, _dp, ctypes.c_int]),
        "bos_dataset_free": (None, [vp]),
        "bos_plan_inspect": (ctypes.c_int, [ctypes.POINTER(bos_problem), ctypes.POINTER(bos_options), ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int64, _ip, _ip, ctypes.POINTER(ctypes.c_uint8),
                                            ctypes.POINTER(ctypes.c_uint8), _ip, ctypes.POINTER(bos_plan_info)]),
        "bos_plan_mf_selftest": (ctypes.c_int, [ctypes.POINTER(bos_problem), ctypes.POINTER(bos_options), _dp, _dp, _dp]),
        "bos_plan_shard_selftest": (ctypes.c_int, [ctypes.POINTER(bos_problem), ctypes.POINTER(bos_options), ctypes.c_int32,
                                                   _dp, _dp, _dp]),
        "bos_plan_node_owner": (ctypes.c_int, [ctypes.POINTER(bos_problem), ctypes.POINTER(bos_options), ctypes.c_int32, _ip]),
        "bos_step_phase": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.POINTER(bos_step_stats)]),
        "bos_exchange_size": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]),
        "bos_exchange_download": (ctypes.c_int, [vp, ctypes.c_int32, _dp]),
        "bos_exchange_upload": (ctypes.c_int, [vp, ctypes.c_int32, _dp]),
        "bos_node_owner": (ctypes.c_int, [vp, _ip]),
        "bos_debug_set_g2o_parser": (None, [ctypes.c_int32]),
        "bos_debug_inject_stall": (ctypes.c_int, [vp]),
        "bos_debug_set_step_graph": (ctypes.c_int, [vp, ctypes.c_int32]),
        "bos_debug_solver_stamps": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64),
                                                   ctypes.POINTER(ctypes.c_int32)]),
        "bos_time_linearize": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, _dp]),
        "bos_time_triangulate": (ctypes.c_int, [vp, ctypes.c_int32, _dp]),
        "bos_time_steps": (ctypes.c_int, [vp, ctypes.c_int32, _dp]),
        "bos_cpu_gn_create": (ctypes.c_int, [ctypes.POINTER(bos_problem), ctypes.c_int32, ctypes.c_int32,
                                             ctypes.POINTER(vp)]),
        "bos_cpu_gn_step": (ctypes.c_int, [vp, _dp]),
        "bos_cpu_gn_get_state": (ctypes.c_int, [vp, _dp, _dp]),
        "bos_cpu_gn_destroy": (None, [vp]),
        "bos_exchange_p2p_handle": (ctypes.c_int, [vp, ctypes.c_void_p]),
        "bos_exchange_p2p_connect": (ctypes.c_int, [vp, ctypes.c_void_p]),
        "bos_set_exchange_timeout": (ctypes.c_int, [vp, ctypes.c_double]),
        "bos_last_step_stamps": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64)]),
        "bos_normalized_angle_f64": (ctypes.c_double, [ctypes.c_double]),
        "bos_normalized_angle_f32": (ctypes.c_float, [ctypes.c_float]),
        "bos_time_facade_steps": (ctypes.c_int, [ctypes.POINTER(bos_problem), ctypes.POINTER(bos_options), ctypes.c_int32,
                                                 _dp, _dp, _dp, ctypes.POINTER(ctypes.c_int64)]),
        "bos_debug_facade_selftest": (ctypes.c_int, [ctypes.POINTER(bos_problem), ctypes.POINTER(bos_options),
                                                     ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]),
    }
    for name, (res, args) in sig.items():
        if ALLOW_MISSING_SYMBOLS and not hasattr(L, name):   # A/B tools loading an older build
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc: int, what: str):
    if rc != BOS_OK:
        raise BosError(f"{what} failed ({rc}): {lib().bos_last_error().decode()}")


def _ptr(a, ct):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ct))


def device_count() -> int:
    return lib().bos_device_count()


def device_peer_access(capacity: int = 64) -> list:
    """Peer-access matrix of the visible devices (hipDeviceCanAccessPeer; 1 on the diagonal)."""
    out = np.zeros(capacity * capacity, dtype=np.int32)
    n = np.zeros(1, dtype=np.int32)
    _check(lib().bos_device_peer_access(capacity, _ptr(out, ctypes.c_int32), _ptr(n, ctypes.c_int32)),
           "bos_device_peer_access")
    k = int(n[0])
    return out[:k * k].reshape(k, k).tolist()


class Problem:
    """SoA problem in stix order (include/bos.h bos_problem). Owns its numpy arrays."""

    def __init__(self, pose_xyt, lm_xy, b_pose, b_lm, b_z, o_src, o_dst, o_z, o_omega, fixed, b_omega=None,
                 pose_ids=None, lm_ids=None):
        self.pose_xyt = np.ascontiguousarray(pose_xyt, dtype=np.float64).reshape(-1, 3)
        self.lm_xy = np.ascontiguousarray(lm_xy, dtype=np.float64).reshape(-1, 2)
        self.b_pose = np.ascontiguousarray(b_pose, dtype=np.int32)
        self.b_lm = np.ascontiguousarray(b_lm, dtype=np.int32)
        self.b_z = np.ascontiguousarray(b_z, dtype=np.float64)
        self.b_omega = None if b_omega is None else np.ascontiguousarray(b_omega, dtype=np.float64)
        self.o_src = np.ascontiguousarray(o_src, dtype=np.int32)
        self.o_dst = np.ascontiguousarray(o_dst, dtype=np.int32)
        self.o_z = np.ascontiguousarray(o_z, dtype=np.float64).reshape(-1, 3)
        self.o_omega = np.ascontiguousarray(o_omega, dtype=np.float64).reshape(-1, 3, 3)
        self.fixed = int(fixed)
        self.pose_ids = pose_ids
        self.lm_ids = lm_ids

    @property
    def NP(self):
        return len(self.pose_xyt)

    @property
    def NL(self):
        return len(self.lm_xy)

    @property
    def N(self):
        return 3 * self.NP + 2 * self.NL

    def c_struct(self) -> bos_problem:
        p = bos_problem()
        p.num_poses, p.num_landmarks = self.NP, self.NL
        p.num_bearings, p.num_odometry = len(self.b_z), len(self.o_z)
        p.pose_xyt = _ptr(self.pose_xyt, ctypes.c_double)
        p.landmark_xy = _ptr(self.lm_xy, ctypes.c_double) if self.NL else None
        p.bearing_pose = _ptr(self.b_pose, ctypes.c_int32)
        p.bearing_landmark = _ptr(self.b_lm, ctypes.c_int32)
        p.bearing_z = _ptr(self.b_z, ctypes.c_double)
        p.bearing_omega = _ptr(self.b_omega, ctypes.c_double)
        p.odom_src = _ptr(self.o_src, ctypes.c_int32)
        p.odom_dst = _ptr(self.o_dst, ctypes.c_int32)
        p.odom_z = _ptr(self.o_z, ctypes.c_double)
        p.odom_omega = _ptr(self.o_omega, ctypes.c_double)
        p.fixed_pose = self.fixed
        return p


def _problem_from_dataset(h) -> Problem:
    L = lib()
    v = bos_problem()
    _check(L.bos_dataset_problem(h, ctypes.byref(v)), "bos_dataset_problem")
    NP, NL, Mb, Mo = v.num_poses, v.num_landmarks, v.num_bearings, v.num_odometry

    def arr(p, n, dt):
        if n == 0 or not p:
            return np.zeros(0, dtype=dt)
        return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True)

    pose_ids = arr(L.bos_dataset_pose_ids(h), NP, np.int32)
    lm_ids = arr(L.bos_dataset_landmark_ids(h), NL, np.int32)
    return Problem(arr(v.pose_xyt, 3 * NP, np.float64), arr(v.landmark_xy, 2 * NL, np.float64),
                   arr(v.bearing_pose, Mb, np.int32), arr(v.bearing_landmark, Mb, np.int32),
                   arr(v.bearing_z, Mb, np.float64), arr(v.odom_src, Mo, np.int32), arr(v.odom_dst, Mo, np.int32),
                   arr(v.odom_z, 3 * Mo, np.float64), arr(v.odom_omega, 9 * Mo, np.float64), v.fixed_pose,
                   pose_ids=pose_ids, lm_ids=lm_ids)


def load_g2o(path: str, triangulate: bool = True, verbose: bool = False) -> Problem:
    """parse_g2o + default FIX + triangulate_landmarks, in libbos.so's C++ host code."""
    L = lib()
    h = ctypes.c_void_p()
    _check(L.bos_dataset_load_g2o(path.encode(), int(triangulate), int(verbose), ctypes.byref(h)), "load_g2o")
    try:
        P = _problem_from_dataset(h)
        P.fixed_pose_id = L.bos_dataset_fixed_pose_id(h)
        P.bound = L.bos_dataset_bound(h)
    finally:
        L.bos_dataset_free(h)
    return P


def synthetic(num_poses: int, num_landmarks: int, bearings_per_pose: int, seed: int = 0xB05EED01) -> Problem:
    """Deterministic synthetic world; P.gt_pose_xyt / P.gt_lm_xy hold ground truth."""
    L = lib()
    h = ctypes.c_void_p()
    _check(L.bos_dataset_synthetic(num_poses, num_landmarks, bearings_per_pose, seed, ctypes.byref(h)), "synthetic")
    try:
        P = _problem_from_dataset(h)
        gp, gl = _dp(), _dp()
        _check(L.bos_dataset_ground_truth(h, ctypes.byref(gp), ctypes.byref(gl)), "ground_truth")
        P.gt_pose_xyt = np.ctypeslib.as_array(gp, shape=(3 * P.NP,)).reshape(-1, 3).copy()
        P.gt_lm_xy = np.ctypeslib.as_array(gl, shape=(2 * P.NL,)).reshape(-1, 2).copy()
        P.fixed_pose_id = L.bos_dataset_fixed_pose_id(h)
    finally:
        L.bos_dataset_free(h)
    return P


def write_g2o(P: Problem, path: str, pose_xyt=None, lm_xy=None, with_landmarks=True, source: Optional[str] = None):
    """Write a problem (and optionally a state) as g2o via the C++ writer."""
    L = lib()
    h = ctypes.c_void_p()
    if source is None:
        raise BosError("write_g2o needs the source g2o path (or use bearing_only_slam --dump)")
    _check(L.bos_dataset_load_g2o(source.encode(), 1, 0, ctypes.byref(h)), "load_g2o")
    try:
        pp = None if pose_xyt is None else np.ascontiguousarray(pose_xyt, dtype=np.float64)
        ll = None if lm_xy is None else np.ascontiguousarray(lm_xy, dtype=np.float64)
        _check(L.bos_dataset_write_g2o(h, path.encode(), _ptr(pp, ctypes.c_double), _ptr(ll, ctypes.c_double),
                                       int(with_landmarks)), "write_g2o")
    finally:
        L.bos_dataset_free(h)


def time_facade_steps(P: Problem, n: int, opts=None) -> dict:
    """n x proj02::Solver::step() through the C++ façade, then one read of solver.state
    (bos_time_facade_steps; the reference's loop, executables/bearing_only_slam.cpp:93-99)."""
    ms, rd, capi, bad = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    pb = P.c_struct()
    _check(lib().bos_time_facade_steps(ctypes.byref(pb), None if opts is None else ctypes.byref(opts), n,
                                       ctypes.byref(ms), ctypes.byref(rd), ctypes.byref(capi), ctypes.byref(bad)),
           "bos_time_facade_steps")
    return {"ms_per_step": ms.value, "ms_state_read": rd.value, "ms_per_step_capi": capi.value,
            "state_mismatches": bad.value}


def facade_selftest(P: Problem, n: int, opts=None) -> int:
    """Doubles of the façade's solver.state that differ from the device state (bos_debug_facade_selftest)."""
    bad = ctypes.c_int64()
    pb = P.c_struct()
    _check(lib().bos_debug_facade_selftest(ctypes.byref(pb), None if opts is None else ctypes.byref(opts), n,
                                           ctypes.byref(bad)), "bos_debug_facade_selftest")
    return bad.value


def options(solver: int = BOS_SOLVER_SUPERNODAL, partition: int = BOS_PARTITION_SUBTREE, lanes_per_pose: int = 0,
            schur_leaf: int = 0, precision: int = BOS_FP64) -> bos_options:
    """bos_options with the planning fields set (bos_default_options for the rest)."""
    o = bos_options()
    lib().bos_default_options(ctypes.byref(o))
    o.solver, o.partition, o.lanes_per_pose, o.schur_leaf, o.precision = solver, partition, lanes_per_pose, schur_leaf, precision
    return o


def plan_inspect(P: Problem, rank: int = 0, world: int = 1, entries: bool = False,
                 solver: int = BOS_SOLVER_SUPERNODAL, partition: int = BOS_PARTITION_SUBTREE, lanes_per_pose: int = 0,
                 schur_leaf: int = 0):
    """Host-only plan build (ordering, CSR layout, shard ownership) — no GPU needed."""
    L = lib()
    cs = P.c_struct()
    info = bos_plan_info()
    opt = options(solver, partition, lanes_per_pose, schur_leaf)
    _check(L.bos_plan_inspect(ctypes.byref(cs), ctypes.byref(opt), rank, world, 0, None, None, None, None, None,
                              ctypes.byref(info)), "plan_inspect")
    out = {"n": info.n, "nnz_lower": info.nnz_lower, "nnz_factor": info.nnz_factor,
           "num_block_values": info.num_block_values, "lanes_per_pose": info.lanes_per_pose,
           "flops_temporal": info.flops_temporal, "flops_nested_dissection": info.flops_nested_dissection,
           "ordering": info.ordering.decode(), "mf_supernodes": info.mf_supernodes,
           "mf_levels": info.mf_levels, "mf_max_front": info.mf_max_front, "mf_flops": info.mf_flops,
           "mf_update_bytes": info.mf_update_bytes, "mf_fits": bool(info.mf_fits),
           "mf_max_front_upper": info.mf_max_front_upper, "mf_balance_pct": info.mf_balance_pct,
           "mf_fold_fp32": bool(info.mf_fold_fp32), "lm_lanes_consecutive": info.lm_lanes_consecutive,
           "pose_odometry_chain": info.pose_odometry_chain}
    out.update({k: getattr(info, k) for k, _ in bos_plan_info._fields_ if k.startswith("shard_")})
    if entries:
        nnz = info.nnz_lower
        rows = np.zeros(nnz, dtype=np.int32)
        cols = np.zeros(nnz, dtype=np.int32)
        owned = np.zeros(nnz, dtype=np.uint8)
        b_owned = np.zeros(P.N, dtype=np.uint8)
        perm = np.zeros(P.N, dtype=np.int32)
        _check(L.bos_plan_inspect(ctypes.byref(cs), ctypes.byref(opt), rank, world, nnz, _ptr(rows, ctypes.c_int32),
                                  _ptr(cols, ctypes.c_int32), _ptr(owned, ctypes.c_uint8),
                                  _ptr(b_owned, ctypes.c_uint8), _ptr(perm, ctypes.c_int32), None), "plan_inspect")
        out.update(rows=rows, cols=cols, owned=owned.astype(bool), b_owned=b_owned.astype(bool), perm_to_ref=perm)
    return out


def plan_mf_selftest(P: Problem, vals, rhs, solver: int = BOS_SOLVER_SUPERNODAL, schur_leaf: int = 0):
    """Host re-run of the GPU multifrontal algorithm on the plan's tree (test hook)."""
    cs = P.c_struct()
    v = np.ascontiguousarray(vals, dtype=np.float64)
    b = np.ascontiguousarray(rhs, dtype=np.float64)
    x = np.zeros_like(b)
    opt = options(solver, schur_leaf=schur_leaf)
    _check(lib().bos_plan_mf_selftest(ctypes.byref(cs), ctypes.byref(opt), _ptr(v, ctypes.c_double),
                                      _ptr(b, ctypes.c_double), _ptr(x, ctypes.c_double)), "plan_mf_selftest")
    return x


def plan_shard_selftest(P: Problem, world: int, vals, rhs, solver: int = BOS_SOLVER_SCHUR):
    """Host simulation of the sharded solve over `world` ranks, exchanges included (test hook):
    raises unless the merged solution equals the one-rank solution bit for bit and every rank's J+H
    reads only nodes its box-plus keeps current; returns x (permuted order)."""
    cs = P.c_struct()
    v = np.ascontiguousarray(vals, dtype=np.float64)
    b = np.ascontiguousarray(rhs, dtype=np.float64)
    x = np.zeros_like(b)
    opt = options(solver)
    _check(lib().bos_plan_shard_selftest(ctypes.byref(cs), ctypes.byref(opt), world, _ptr(v, ctypes.c_double),
                                         _ptr(b, ctypes.c_double), _ptr(x, ctypes.c_double)), "plan_shard_selftest")
    return x


def plan_node_owner(P: Problem, world: int, solver: int = BOS_SOLVER_SCHUR) -> np.ndarray:
    """Owner rank of every node (poses, then landmarks) of a `world`-rank shard; -1 top, -2 fixed pose."""
    cs = P.c_struct()
    o = np.zeros(P.NP + P.NL, dtype=np.int32)
    opt = options(solver)
    _check(lib().bos_plan_node_owner(ctypes.byref(cs), ctypes.byref(opt), world, _ptr(o, ctypes.c_int32)),
           "plan_node_owner")
    return o


class CpuGN:
    """The CPU baseline of bench.py (include/bos_host.h bos_cpu_gn_*): the same GN iteration on the
    host's cores with the build's own host multifrontal Cholesky. Not a fallback of Solver."""

    def __init__(self, P: Problem, threads: int, solver: int = BOS_SOLVER_SCHUR):
        self.P = P
        self._h = ctypes.c_void_p()
        cs = P.c_struct()
        _check(lib().bos_cpu_gn_create(ctypes.byref(cs), solver, threads, ctypes.byref(self._h)), "bos_cpu_gn_create")

    def step(self) -> float:
        c = ctypes.c_double(0)
        _check(lib().bos_cpu_gn_step(self._h, ctypes.byref(c)), "bos_cpu_gn_step")
        return c.value

    def get_state(self):
        pose = np.zeros((self.P.NP, 3))
        lm = np.zeros((self.P.NL, 2))
        _check(lib().bos_cpu_gn_get_state(self._h, _ptr(pose, ctypes.c_double), _ptr(lm, ctypes.c_double)),
               "bos_cpu_gn_get_state")
        return pose, lm

    def close(self):
        if self._h:
            lib().bos_cpu_gn_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def nccl_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(lib().bos_nccl_unique_id(buf, 128), "bos_nccl_unique_id")
    return buf.raw


class Solver:
    """``proj02::Solver`` over the HIP path. ``state`` is downloaded after every ``step()``."""

    def __init__(self, P: Problem, precision: int = BOS_FP64, solver: int = BOS_SOLVER_SPARSE_CHOL,
                 device: int = -1, kernel_threshold: float = 1.0, damping: float = 0.01, stream: int = 0,
                 rank: int = 0, world_size: int = 1, nccl_id: Optional[bytes] = None, triangulate: bool = False,
                 partition: int = BOS_PARTITION_SUBTREE, lanes_per_pose: int = 0, schur_leaf: int = 0):
        """triangulate=True: ignore P.lm_xy and triangulate the landmarks on the device from the
        initial poses (bos_problem.landmark_xy = NULL). partition / lanes_per_pose / schur_leaf: the
        bos_options fields of the same names."""
        L = lib()
        self.P = P
        self.partition = partition
        opt = bos_options()
        L.bos_default_options(ctypes.byref(opt))
        opt.precision, opt.solver, opt.device = precision, solver, device
        opt.kernel_threshold, opt.damping = kernel_threshold, damping
        opt.stream = stream or None
        opt.rank, opt.world_size = rank, world_size
        opt.partition, opt.lanes_per_pose, opt.schur_leaf = partition, lanes_per_pose, schur_leaf
        self._nid = None
        if nccl_id is not None:
            self._nid = ctypes.create_string_buffer(nccl_id, len(nccl_id))
            opt.nccl_unique_id = ctypes.cast(self._nid, ctypes.c_void_p)
        self._h = ctypes.c_void_p()
        cs = P.c_struct()
        if triangulate:
            cs.landmark_xy = None
        _check(L.bos_create(ctypes.byref(cs), ctypes.byref(opt), ctypes.byref(self._h)), "bos_create")
        self.last_stats = None

    def close(self):
        if self._h:
            lib().bos_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_kernel_threshold(self, kt: float):
        _check(lib().bos_set_kernel_threshold(self._h, kt), "set_kernel_threshold")

    def set_damping_factor(self, df: float):
        _check(lib().bos_set_damping_factor(self._h, df), "set_damping_factor")

    def step(self) -> dict:
        st = bos_step_stats()
        _check(lib().bos_step(self._h, ctypes.byref(st)), "bos_step")
        self.last_stats = st.as_dict()
        return self.last_stats

    def step_n(self, n: int) -> dict:
        st = bos_step_stats()
        _check(lib().bos_step_n(self._h, n, ctypes.byref(st)), "bos_step_n")
        self.last_stats = st.as_dict()
        return self.last_stats

    def linearize(self) -> dict:
        st = bos_step_stats()
        _check(lib().bos_linearize(self._h, ctypes.byref(st)), "bos_linearize")
        return st.as_dict()

    def linearize_async(self):
        _check(lib().bos_linearize_async(self._h), "bos_linearize_async")

    def debug_timeline(self, flush_caches: bool = False) -> np.ndarray:
        """One J+H launch with per-wave stamps (diagnostics): rows of [block, wave, kind, t_start,
        t_loop, t_loop_end, t_end, hw_id | xcc << 32], times in 100 MHz ticks; flush_caches: the
        launch reads its inputs from HBM (1 GiB read before it)."""
        n = ctypes.c_int64(0)
        _check(lib().bos_debug_linearize_timeline(self._h, 0, None, ctypes.byref(n), 0), "timeline")
        out = np.zeros((n.value, 8), dtype=np.uint64)
        _check(lib().bos_debug_linearize_timeline(self._h, n.value, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                                  ctypes.byref(n), int(flush_caches)), "timeline")
        return out

    # ---- sharded (multi-GPU) step, external exchange: see include/bos.h
    def step_phase(self, phase: int):
        """One phase of an external-exchange step; returns the step's stats from its last phase
        (2 for the subtree partition, 1 for the observations partition), else None."""
        st = bos_step_stats()
        _check(lib().bos_step_phase(self._h, phase, ctypes.byref(st)), f"bos_step_phase({phase})")
        if phase == (1 if self.partition == BOS_PARTITION_OBSERVATIONS else 2):
            self.last_stats = st.as_dict()
            return self.last_stats
        return None

    def exchange_size(self, which: int) -> int:
        n = ctypes.c_int64(0)
        _check(lib().bos_exchange_size(self._h, which, ctypes.byref(n)), "bos_exchange_size")
        return n.value

    def exchange_download(self, which: int) -> np.ndarray:
        out = np.zeros(self.exchange_size(which))
        _check(lib().bos_exchange_download(self._h, which, _ptr(out, ctypes.c_double)), "bos_exchange_download")
        return out

    def exchange_upload(self, which: int, all_ranks: np.ndarray):
        """Subtree partition: every rank's buffer concatenated in rank order (all-gather);
        observations partition: the element-wise sum over the ranks (all-reduce)."""
        a = np.ascontiguousarray(all_ranks, dtype=np.float64)
        _check(lib().bos_exchange_upload(self._h, which, _ptr(a, ctypes.c_double)), "bos_exchange_upload")

    def p2p_handle(self) -> bytes:
        """This rank's direct-exchange mailbox handle (bos_exchange_p2p_handle)."""
        buf = ctypes.create_string_buffer(P2P_HANDLE_BYTES)
        _check(lib().bos_exchange_p2p_handle(self._h, buf), "bos_exchange_p2p_handle")
        return buf.raw

    def p2p_connect(self, handles) -> None:
        """Every rank's handle in rank order (bos_exchange_p2p_connect): bos_step then exchanges
        directly between the ranks' mailboxes."""
        blob = b"".join(handles)
        buf = ctypes.create_string_buffer(blob, len(blob))
        _check(lib().bos_exchange_p2p_connect(self._h, buf), "bos_exchange_p2p_connect")

    def last_step_stamps(self) -> np.ndarray:
        """Phase stamps of the last step (bos_last_step_stamps; 100 MHz realtime ticks)."""
        st = np.zeros(8, dtype=np.uint64)
        _check(lib().bos_last_step_stamps(self._h, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))),
               "bos_last_step_stamps")
        return st

    def set_exchange_timeout(self, seconds: float) -> None:
        """Bound of the direct exchange's device-side flag waits (bos_set_exchange_timeout, 2 s default)."""
        _check(lib().bos_set_exchange_timeout(self._h, float(seconds)), "bos_set_exchange_timeout")

    def node_owner(self) -> np.ndarray:
        o = np.zeros(self.P.NP + self.P.NL, dtype=np.int32)
        _check(lib().bos_node_owner(self._h, _ptr(o, ctypes.c_int32)), "bos_node_owner")
        return o

    def debug_inject_stall(self):
        """Test hook: the next step's factor dataflow launch skips its first front (a stalled
        dependency); that step must fail with BOS_ERR_SOLVER and leave the state unchanged."""
        _check(lib().bos_debug_inject_stall(self._h), "bos_debug_inject_stall")

    def debug_solver_stamps(self, nsuper: int):
        """Diagnostics: one GN step with per-front stamps of the dataflow launches (bos_host.h)."""
        st = np.zeros((2, nsuper, 8), dtype=np.uint64)
        meta = np.zeros((nsuper, 4), dtype=np.int32)
        _check(lib().bos_debug_solver_stamps(self._h, st.size, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                             meta.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))), "solver stamps")
        return st, meta

    def debug_set_step_graph(self, enable: bool):
        """Test hook: GN steps as individual launches (False) or the captured graph (True, default)."""
        _check(lib().bos_debug_set_step_graph(self._h, int(enable)), "bos_debug_set_step_graph")

    def time_linearize(self, n: int, flush_caches: bool = False) -> float:
        """ms per J+H build (HIP events on the handle's stream, see bos_time_linearize)."""
        ms = ctypes.c_double(0)
        _check(lib().bos_time_linearize(self._h, n, int(flush_caches), ctypes.byref(ms)), "bos_time_linearize")
        return ms.value

    def time_steps(self, n: int) -> float:
        """ms per synchronous GN iteration over n bos_step calls made from C (bos_time_steps)."""
        ms = ctypes.c_double(0)
        _check(lib().bos_time_steps(self._h, n, ctypes.byref(ms)), "bos_time_steps")
        return ms.value

    def time_triangulate(self, n: int) -> float:
        ms = ctypes.c_double(0)
        _check(lib().bos_time_triangulate(self._h, n, ctypes.byref(ms)), "bos_time_triangulate")
        return ms.value

    def triangulate(self):
        """triangulate_landmarks on the device from the current poses (slam/triangulation.cpp:65-74)."""
        _check(lib().bos_triangulate(self._h), "bos_triangulate")

    def triangulate_async(self):
        _check(lib().bos_triangulate_async(self._h), "bos_triangulate_async")

    def synchronize(self):
        _check(lib().bos_synchronize(self._h), "bos_synchronize")

    def system_info(self) -> dict:
        info = bos_system_info()
        _check(lib().bos_system_info_get(self._h, ctypes.byref(info)), "system_info")
        return {k: getattr(info, k) for k, _ in info._fields_}

    def export_system(self):
        """(rows, cols, vals, b): lower triangle of H_nf in reference dof numbering + full b."""
        info = self.system_info()
        nnz = info["nnz_lower"]
        rows = np.zeros(nnz, dtype=np.int32)
        cols = np.zeros(nnz, dtype=np.int32)
        vals = np.zeros(nnz)
        b = np.zeros(self.P.N)
        _check(lib().bos_export_system(self._h, nnz, _ptr(rows, ctypes.c_int32), _ptr(cols, ctypes.c_int32),
                                       _ptr(vals, ctypes.c_double), _ptr(b, ctypes.c_double)), "export_system")
        return rows, cols, vals, b

    def get_state(self):
        pose = np.zeros((self.P.NP, 3))
        lm = np.zeros((self.P.NL, 2))
        _check(lib().bos_get_state(self._h, _ptr(pose, ctypes.c_double), _ptr(lm, ctypes.c_double)), "get_state")
        return pose, lm

    def set_state(self, pose_xyt, lm_xy):
        pose = np.ascontiguousarray(pose_xyt, dtype=np.float64)
        lm = np.ascontiguousarray(lm_xy, dtype=np.float64)
        _check(lib().bos_set_state(self._h, _ptr(pose, ctypes.c_double), _ptr(lm, ctypes.c_double)), "set_state")

    def last_dx(self):
        dx = np.zeros(self.P.N)
        _check(lib().bos_get_last_dx(self._h, _ptr(dx, ctypes.c_double)), "get_last_dx")
        return dx

    @property
    def state(self):
        return self.get_state()
