"""GN steps on a Schur plan that no separator balance fits to the wave kernels (fronts with more
than 64 rows: the workgroup factorization / forward / backward launches, mf_factor_level and
friends, instead of the register kernels), against the oracle's GN iterations
(/root/reference/slam/solver.cpp:27-97). The plan is forced with 40-pose Schur leaves
(bos_options.schur_leaf, a planning option: it changes the ordering, never the arithmetic of a
front), as in tests/test_host.py::test_schur_plan_fallback_keeps_a_valid_plan."""
import pytest

import bos
import oracle as O
from conftest import C1
from helpers import close_state, literal_oracle, to_oracle

pytestmark = pytest.mark.gpu


def _solver_with_leaf(P, leaf):
    info = bos.plan_inspect(P, 0, 1, solver=bos.BOS_SOLVER_SCHUR, schur_leaf=leaf)
    S = bos.Solver(P, solver=bos.BOS_SOLVER_SCHUR, schur_leaf=leaf)
    return S, info


@pytest.mark.parametrize("which,iters", [("c1", 50), ("c2", 10)])
def test_schur_plan_with_large_fronts_matches_oracle(which, iters):
    P = bos.load_g2o(C1) if which == "c1" else bos.synthetic(1000, 2000, 20)
    S, info = _solver_with_leaf(P, 40)
    assert info["mf_max_front"] > 64   # the workgroup path is exercised
    for _ in range(iters):
        assert S.step()["solver_info"] == 0
    pg, lg = S.get_state()
    with literal_oracle(P):
        po, lo, _ = O.run(to_oracle(P), iters)
    ok, ep, el = close_state(pg, lg, po, lo)
    assert ok, (ep, el)
