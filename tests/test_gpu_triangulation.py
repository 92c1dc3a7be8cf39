"""Landmark triangulation on the device (bos_triangulate; reference slam/triangulation.cpp:21-74)
against the CPU oracle's restatement (oracle.triangulate: column-pivoted Householder QR as Eigen's
colPivHouseholderQr, the basic solution for rank-1 systems) and the host loader's triangulation.

Tolerance: max |xy_gpu - xy_ref| <= 1e-9 * max(1, |xy_ref|) per landmark. The device evaluates the
same operation sequence as the host code (host/triangulation.cpp) without FP contraction; the
device and glibc sin/cos differ in the last ulp, and single-observation landmarks (basic solution,
rank 1) are the ill-conditioned ones."""
import numpy as np
import pytest

import bos
import oracle as O
from conftest import C1

pytestmark = pytest.mark.gpu


def _oracle_tri(P, pose_xyt):
    ids, xy = O.triangulate(pose_xyt, P.b_pose, np.arange(P.NL, dtype=np.int32)[P.b_lm], P.b_z)
    assert np.array_equal(ids, np.arange(P.NL))
    return xy


def _close(a, b, tol=1e-9):
    err = np.abs(a - b) / np.maximum(1.0, np.abs(b))
    return float(err.max())


def test_triangulate_at_create_c1():
    P = bos.load_g2o(C1)                      # the host loader triangulates (host/triangulation.cpp)
    S = bos.Solver(P, triangulate=True)       # landmark_xy = NULL: triangulated on the device
    pg, lg = S.get_state()
    assert _close(lg, P.lm_xy) <= 1e-9
    assert _close(lg, _oracle_tri(P, P.pose_xyt)) <= 1e-9
    # same GN iteration as from the host-triangulated landmarks
    S0 = bos.Solver(P)
    a, b = S.step(), S0.step()
    assert abs(a["chi2"] - b["chi2"]) <= 1e-9 * b["chi2"]
    S.close()
    S0.close()


def test_single_observation_landmarks_basic_solution():
    P = bos.load_g2o(C1)
    counts = np.bincount(P.b_lm, minlength=P.NL)
    assert (counts == 1).sum() >= 1
    S = bos.Solver(P, triangulate=True)
    _, lg = S.get_state()
    one = counts == 1
    assert _close(lg[one], P.lm_xy[one]) <= 1e-9
    # basic solution: one component exactly zero
    assert np.all(np.min(np.abs(lg[one]), axis=1) == 0.0)
    S.close()


@pytest.mark.parametrize("precision", [bos.BOS_FP64, bos.BOS_FP32])
def test_retriangulate_after_steps(precision):
    P = bos.load_g2o(C1)
    S = bos.Solver(P, precision=precision)
    for _ in range(10):
        S.step()
    pg, _ = S.get_state()
    S.triangulate()
    pg2, lg = S.get_state()
    assert np.array_equal(pg, pg2)            # poses untouched
    assert _close(lg, _oracle_tri(P, pg)) <= 1e-9
    S.step()                                  # the caches were refreshed: the next iteration runs
    S.close()


@pytest.mark.parametrize("size", [(1000, 2000, 20), (100000, 200000, 10)])
def test_triangulate_synthetic(size):
    P = bos.synthetic(*size, seed=0xB05EED01 + (2 if size[0] == 1000 else 3))
    S = bos.Solver(P, precision=bos.BOS_FP32, triangulate=True)
    _, lg = S.get_state()
    ref = _oracle_tri(P, P.pose_xyt)
    assert _close(lg, ref) <= 1e-9, _close(lg, ref)
    S.close()
