"""Edge cases of the HIP J+H build and GN step against the CPU oracle, on variants of the
reference dataset (C1) and small synthetic worlds. Each case exercises a kernel path the
headline configs do not: duplicate (pose, landmark) observations (summed into one block, the
run-continuation flag), duplicate odometry pairs, poses with more than two odometry entries (loop
closures), odometry edges in both directions between the same poses (one shared pose-pose block
stored by the lower pose), odometry self-loops (zero Jacobian in the reference: chi^2 only),
bearing weights (HAS_W), poses without bearings and landmarks without observations (empty lanes),
two lanes per pose (dense poses), odd list lengths (the pair loop's tail). Every GN step must
report solver_info == 0.

Tolerances as tests/test_gpu_parity.py: fp64 H within 1e-12 of max |H| (b 1e-11), fp32 within 2e-4;
state after 3 GN steps within rtol 1e-6 / atol 1e-9 of the oracle's."""
import numpy as np
import pytest

import bos
import oracle as O
from conftest import C1
from helpers import close_state, lin_parity, literal_oracle, to_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c1():
    return bos.load_g2o(C1)


def _variant(P, **kw):
    a = dict(pose_xyt=P.pose_xyt, lm_xy=P.lm_xy, b_pose=P.b_pose, b_lm=P.b_lm, b_z=P.b_z, o_src=P.o_src,
             o_dst=P.o_dst, o_z=P.o_z, o_omega=P.o_omega, fixed=P.fixed, b_omega=P.b_omega,
             pose_ids=P.pose_ids, lm_ids=P.lm_ids)
    a.update(kw)
    return bos.Problem(**a)


def _dup_bearings(P, n=200, seed=1):
    rng = np.random.default_rng(seed)
    k = rng.choice(len(P.b_z), n, replace=False)
    return _variant(P, b_pose=np.concatenate([P.b_pose, P.b_pose[k]]), b_lm=np.concatenate([P.b_lm, P.b_lm[k]]),
                    b_z=np.concatenate([P.b_z, P.b_z[k] + rng.normal(0, 0.01, n)]))


def _dup_odometry(P, n=20, seed=2):
    rng = np.random.default_rng(seed)
    k = rng.choice(len(P.o_z), n, replace=False)
    return _variant(P, o_src=np.concatenate([P.o_src, P.o_src[k]]), o_dst=np.concatenate([P.o_dst, P.o_dst[k]]),
                    o_z=np.concatenate([P.o_z, P.o_z[k] + rng.normal(0, 0.02, (n, 3))]),
                    o_omega=np.concatenate([P.o_omega, P.o_omega[k]]))


def _loop_closures(P, n=30, gap=50, seed=3):
    """Edges (i, i + gap) measured from the current estimate plus noise: those poses get 3-4 entries."""
    rng = np.random.default_rng(seed)
    src = rng.choice(P.NP - gap, n, replace=False).astype(np.int32)
    dst = (src + gap).astype(np.int32)
    Q = to_oracle(P)
    z = np.zeros((n, 3))
    for i, (s, d) in enumerate(zip(src, dst)):
        z[i] = O.predict_odometry(Q.pose_xyt[s], Q.pose_xyt[d]) + rng.normal(0, 0.05, 3)
    return _variant(P, o_src=np.concatenate([P.o_src, src]), o_dst=np.concatenate([P.o_dst, dst]),
                    o_z=np.concatenate([P.o_z, z]), o_omega=np.concatenate([P.o_omega, P.o_omega[:n]]))


def _reversed_edges(P, n=25, seed=6):
    """Edges (d, s) added next to existing (s, d): g2o files hold such reversed loop closures, and
    the reference sums both into H(s, d) / H(d, s) (slam/solver.cpp:48-62)."""
    rng = np.random.default_rng(seed)
    k = rng.choice(len(P.o_z), n, replace=False)
    Q = to_oracle(P)
    src, dst = P.o_dst[k].astype(np.int32), P.o_src[k].astype(np.int32)
    z = np.array([O.predict_odometry(Q.pose_xyt[s], Q.pose_xyt[d]) for s, d in zip(src, dst)]) + rng.normal(0, 0.03, (n, 3))
    return _variant(P, o_src=np.concatenate([P.o_src, src]), o_dst=np.concatenate([P.o_dst, dst]),
                    o_z=np.concatenate([P.o_z, z]), o_omega=np.concatenate([P.o_omega, P.o_omega[k]]))


def _self_loops(P, n=7, seed=7):
    """Odometry edges (i, i): their Jacobian is zero in the reference (the two 3x3 blocks land on
    the same columns and cancel exactly), so they add chi^2 (and may trip the robust count) only."""
    rng = np.random.default_rng(seed)
    p = rng.choice(P.NP, n, replace=False).astype(np.int32)
    z = rng.normal(0, 0.05, (n, 3))
    z[0] = (2.0, -1.0, 0.5)   # rho far above the kernel threshold
    return _variant(P, o_src=np.concatenate([P.o_src, p]), o_dst=np.concatenate([P.o_dst, p]),
                    o_z=np.concatenate([P.o_z, z]), o_omega=np.concatenate([P.o_omega, P.o_omega[:n]]))


def _weights(P, seed=4):
    rng = np.random.default_rng(seed)
    return _variant(P, b_omega=rng.uniform(0.5, 2.0, len(P.b_z)))


def _poses_without_bearings(P, n=20, seed=5):
    """All bearings of n poses dropped: empty pose lanes, and landmarks seen only by those poses
    keep no observation at all (empty landmark lanes; damping keeps H positive definite)."""
    rng = np.random.default_rng(seed)
    cand = np.setdiff1d(np.arange(P.NP), [P.fixed])
    drop = rng.choice(cand, n, replace=False)
    keep = ~np.isin(P.b_pose, drop)
    return _variant(P, b_pose=P.b_pose[keep], b_lm=P.b_lm[keep], b_z=P.b_z[keep])


CASES = {
    "dup_bearings": _dup_bearings,
    "dup_odometry": _dup_odometry,
    "loop_closures": _loop_closures,
    "weights": _weights,
    "poses_without_bearings": _poses_without_bearings,
    "reversed_edges": _reversed_edges,
    "self_loops": _self_loops,
    "everything": lambda P: _self_loops(_reversed_edges(_weights(_loop_closures(_dup_odometry(_dup_bearings(
        _poses_without_bearings(P))))))),
}


def _steps_match(P, precision=bos.BOS_FP64, n=3, rtol=1e-6):
    Q = to_oracle(P)
    S = bos.Solver(P, precision=precision)
    chis = []
    for _ in range(n):
        st = S.step()
        assert st["solver_info"] == 0
        chis.append(st["chi2"])
    pg, lg = S.get_state()
    S.close()
    po, lo = Q.copy_state()
    with literal_oracle(P):
        for i in range(n):
            c, _, _ = O.step(Q, po, lo)
            assert abs(chis[i] - c) <= 1e-9 * max(c, 1.0), (i, chis[i], c)
    return close_state(pg, lg, po, lo, rtol=rtol)


@pytest.mark.parametrize("case", sorted(CASES))
def test_edge_case_linearize_fp64(c1, case):
    lin_parity(CASES[case](c1))


@pytest.mark.parametrize("case", ["dup_bearings", "everything"])
def test_edge_case_linearize_fp32(c1, case):
    lin_parity(CASES[case](c1), precision=bos.BOS_FP32, tol=2e-4, btol=2e-3)


@pytest.mark.parametrize("case", sorted(CASES))
def test_edge_case_steps(c1, case):
    ok, dp, dl = _steps_match(CASES[case](c1))
    assert ok, (dp, dl)


def test_two_lanes_per_pose():
    """Poses with >= 32 bearings on average run two lanes per pose (lane-group butterfly)."""
    P = bos.synthetic(300, 3000, 40, seed=11)
    assert bos.plan_inspect(P, 0, 1)["lanes_per_pose"] == 2
    lin_parity(P)
    ok, dp, dl = _steps_match(P)
    assert ok, (dp, dl)


def test_odd_list_lengths():
    """Every pose with an odd number of bearings: the pair loop's last item runs alone and its
    block goes to the lane's padding slot."""
    P = bos.synthetic(400, 1200, 9, seed=12)
    assert np.all(np.bincount(P.b_pose, minlength=P.NP) % 2 == 1)
    lin_parity(P)
