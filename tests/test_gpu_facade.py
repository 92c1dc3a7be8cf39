"""The C++ façade proj02::Solver (csrc/host/solver.hpp) as the reference's executable uses its
class (executables/bearing_only_slam.cpp:71,93-99,108: construct, step() in a loop, read
solver.state to draw it; slam/solver.hpp:26,36).

The façade leaves the state on the device after step() and downloads it on the first read of
solver.state (fp64, bit for bit bos_get_state); a write to solver.state between steps is uploaded
before the next step, as the reference's step() reads its member state. Tested through
bos_debug_facade_selftest (csrc/host/facade_capi.cpp): the façade stepping beside a plain C ABI
handle, reads every 7 steps and one write halfway; every double of solver.state must equal the
device state bit for bit. The rate: bos_time_facade_steps, the façade's loop against bos_step in a
C loop on the same handle (bench.py reports both at config 3)."""
import pytest

import bos
from conftest import C1

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2():
    return bos.synthetic(1000, 2000, 20)


@pytest.mark.parametrize("precision", [bos.BOS_FP64, bos.BOS_FP32])
def test_facade_state_is_the_device_state_bit_for_bit(c2, precision):
    bad = bos.facade_selftest(c2, 50, bos.options(solver=bos.BOS_SOLVER_SCHUR, precision=precision))
    assert bad == 0


def test_facade_state_reference_dataset():
    P = bos.load_g2o(C1)
    assert bos.facade_selftest(P, 50, bos.options(solver=bos.BOS_SOLVER_SCHUR)) == 0


def test_facade_loop_costs_what_bos_step_costs(c2):
    """No per-step state transfer: 50 façade steps take at most 15 % (+ 10 us) longer per step than
    bos_step in a C loop on the same handle, and the one read of solver.state afterwards returns the
    device state (no mismatching double)."""
    f = bos.time_facade_steps(c2, 50, bos.options(solver=bos.BOS_SOLVER_SCHUR, precision=bos.BOS_FP32))
    print(f)
    assert f["state_mismatches"] == 0
    assert f["ms_per_step"] <= 1.15 * f["ms_per_step_capi"] + 0.010, f
