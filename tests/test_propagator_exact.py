"""The LZ propagator's scheme (numpy restatement tests/lz_ref.py, the kernel's exact step
sequence) against the EXACT finite-window solution of the same model: cell-by-cell Weber
(parabolic-cylinder) functions, tests/weber_ref.py, committed as tests/golden/golden_weber.json
by tests/golden/make_golden_weber.py.

Stated accuracy of the kernel's scheme (eighth-order Magnus on each cell's core at 6 steps per
radian of adiabatic phase, superadiabatic following of order 10 outside it, exact adiabatic cells
for delta > 16) at K = 20 LZ lengths: |P - P_exact| <= 1e-10 at the C5 default S = 64 (measured
3.4e-11) and step-converged (S = 16000; measured 4.2e-11, the following error).  The Magnus
error falls as S^-8 (brute force, whole cells).  The exact
single-crossing P at K = 20 (dressed window edges) is within 5e-9 relative of eq.(9)
(measured 1.95e-9).
"""
import json
import os

import pytest

from lz_ref import propagate
from weber_ref import propagate_exact

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden_weber.json")))
V_W = GOLD["v_w"]


def _cases(kind):
    return [c for c in GOLD["cases"] if c["kind"] == kind]


def test_fixture_rederives():
    for c in (_cases("single")[7], _cases("multi")[1], _cases("multi")[3], _cases("c5")[4]):
        P = propagate_exact(c["m"], c["d"], c["x"], V_W, c["K"])
        assert abs(P - c["P"]) <= 1e-14, (c, P)


def test_exact_reduces_to_closed_form():
    """Single crossing, K = 20: the exact P of the dressed-edge window is eq.(9) (fpy:183-184)
    to 5e-9 relative over the C2 (m_mix, |Delta'|) ranges (delta 1.7e-7 .. 1.7e3)."""
    import math
    for c in _cases("single"):
        delta = c["m"][0] ** 2 / (2 * V_W * c["d"][0])
        P9 = -math.expm1(-2.0 * math.pi * delta)
        assert abs(c["P"] - P9) <= 5e-9 * P9, (delta, c["P"], P9)


@pytest.mark.parametrize("i", range(3))
def test_brute_force_magnus_matches_exact(i):
    c = _cases("multi")[i]
    P = propagate(c["m"], c["d"], c["x"], V_W, c["K"], 6000, hybrid=False)
    assert abs(P - c["P"]) <= 1e-10, (c, P)


def test_hybrid_at_production_settings():
    from conftest import pkg
    assert pkg("sweep").CrossingSpec().steps == 64          # the C5 default
    for S in (64, 16000):
        for c in GOLD["cases"]:
            P = propagate(c["m"], c["d"], c["x"], V_W, c["K"], S)
            assert abs(P - c["P"]) <= 1e-10, (S, c, P)


def test_hybrid_step_converged_with_adiabatic_cell():
    c = _cases("multi")[3]         # delta = 0.6 then an exact adiabatic cell (delta = 24)
    P = propagate(c["m"], c["d"], c["x"], V_W, c["K"], 16000)
    assert abs(P - c["P"]) <= 1e-11, (c, P)


def test_magnus_eighth_order():
    c = _cases("c5")[5]            # (m_mix, |Delta'|) = (1, 10): 8 crossings, delta ~ 0.17
    e1 = abs(propagate(c["m"], c["d"], c["x"], V_W, c["K"], 600, hybrid=False) - c["P"])
    e2 = abs(propagate(c["m"], c["d"], c["x"], V_W, c["K"], 1200, hybrid=False) - c["P"])
    assert 150.0 < e1 / e2 < 600.0, (e1, e2)    # 2^8 = 256 (measured 297)
