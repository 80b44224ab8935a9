"""The Magnus scheme of the LZ propagator against the reference's closed form
in the single-crossing limit, on CPU (numpy restatement tests/lz_ref.py).  With the
second-order dressed edge states the finite window costs ~2e-9 relative at K = 20 LZ lengths
(falling as ~K^-7), inside north_star's 1e-8 on P_LZ."""
import math

import pytest

from lz_ref import propagate


@pytest.mark.parametrize("m,dp", [(0.1, 1.0), (0.2, 0.5), (0.01, 0.1)])
def test_single_crossing_reduces_to_closed_form(m, dp):
    v_w = 0.3
    delta = m * m / (2 * v_w * dp)
    P_cf = 1.0 - math.exp(-2.0 * math.pi * delta)     # fpy:183-184
    P = propagate([m], [dp], [0.0], v_w, 20, 2000)
    assert abs(P - P_cf) / P_cf < 5e-9                # window K = 20 LZ lengths (dressed edges), S = 16000


def test_window_convergence_order():
    m, dp, v_w = 0.1, 1.0, 0.3
    P_cf = 1.0 - math.exp(-2.0 * math.pi * m * m / (2 * v_w * dp))
    # whole-window Magnus (hybrid=False), so only the window's own error is left
    e20 = abs(propagate([m], [dp], [0.0], v_w, 20, 2000, hybrid=False) - P_cf)
    e40 = abs(propagate([m], [dp], [0.0], v_w, 40, 16000, hybrid=False) - P_cf)
    assert e40 < e20 / 50                              # dressed-edge window error ~ K^-7 (measured 125x)
    assert e20 < 5e-9 * P_cf
    # the kernel's scheme (core + superadiabatic following) leaves the window error as it is
    assert abs(propagate([m], [dp], [0.0], v_w, 20, 1) - P_cf) < 5e-9 * P_cf


def test_norm_and_trivial_limits():
    # no coupling -> no conversion; huge coupling -> adiabatic following (P -> 1)
    assert propagate([0.0], [1.0], [0.0], 0.3, 10.0, 200) < 1e-24
    assert propagate([1.0], [0.1], [0.0], 0.3, 40, 16000) > 1 - 1e-6


def test_adiabatic_cell_matches_brute_force_magnus():
    """Two crossings: the first (delta = 0.6) splits the state, the second (delta = 23) is
    adiabatic and only adds the WKB + Stokes phase, which the final interference exposes.
    The hybrid's exact adiabatic cell must agree with brute-force Magnus (step-converged)."""
    m = [0.3, 1.2]
    d = [0.25, 0.1]
    x = [0.0, 200.0]      # cell edge |D| = 14 m; dressed-basis edge error ~ eps (alpha/E^2)^2 ~ 1e-11
    K, v_w = 20.0, 0.3
    hyb = propagate(m, d, x, v_w, K, 16000)
    bf1 = propagate(m, d, x, v_w, K, 40000, hybrid=False)
    bf2 = propagate(m, d, x, v_w, K, 80000, hybrid=False)
    assert abs(bf1 - bf2) < 1e-8                        # brute force converged
    # the second cell's phase decides the interference: P moves 0.015 -> 0.032 for x_2 180 -> 201
    hyb_far = propagate(m, d, [0.0, 201.0], v_w, K, 2000)
    assert abs(hyb_far - hyb) > 0.01
    # measured 1.8e-11 (the plain adiabatic basis at the edges cost 6e-6)
    assert abs(hyb - bf2) < 1e-9, (hyb, bf2)


def test_stokes_phase_series_vs_mpmath():
    import mpmath as mp
    from lz_ref import stokes_phase
    for dl in (16.0, 20.0, 50.0, 400.0):
        d = mp.mpf(dl)
        exact = mp.pi / 4 + d * (mp.log(d) - 1) + mp.arg(mp.gamma(1 - 1j * d))
        exact = float((exact + mp.pi) % (2 * mp.pi) - mp.pi)
        assert abs(stokes_phase(dl) - exact) < 1e-11, (dl, stokes_phase(dl), exact)
