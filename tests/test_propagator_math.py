"""The Magnus scheme of the LZ propagator against the reference's closed form
in the single-crossing limit, on CPU (numpy restatement tests/lz_ref.py)."""
import math

import pytest

from lz_ref import propagate


@pytest.mark.parametrize("m,dp", [(0.1, 1.0), (0.2, 0.5), (0.01, 0.1)])
def test_single_crossing_reduces_to_closed_form(m, dp):
    v_w = 0.3
    delta = m * m / (2 * v_w * dp)
    P_cf = 1.0 - math.exp(-2.0 * math.pi * delta)     # fpy:183-184
    P = propagate([m], [dp], [0.0], v_w, 20, 400)
    assert abs(P - P_cf) / P_cf < 1e-4                # finite window W = 20 xi_LZ, S = 400


def test_window_convergence_order():
    m, dp, v_w = 0.1, 1.0, 0.3
    P_cf = 1.0 - math.exp(-2.0 * math.pi * m * m / (2 * v_w * dp))
    e20 = abs(propagate([m], [dp], [0.0], v_w, 20, 400) - P_cf)
    e40 = abs(propagate([m], [dp], [0.0], v_w, 40, 1600) - P_cf)
    assert e40 < e20 / 4                               # adiabatic-basis window error ~ W^-3


def test_norm_and_trivial_limits():
    # no coupling -> no conversion; huge coupling -> adiabatic following (P -> 1)
    assert propagate([0.0], [1.0], [0.0], 0.3, 10.0, 200) < 1e-24
    assert propagate([1.0], [0.1], [0.0], 0.3, 40, 16000) > 1 - 1e-6
