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


def test_magnus_vector_polynomials_in_D():
    """Round 4 (lzq_propagator.hip, LZQ_PROP_POLY): the kernel evaluates the eighth-order Magnus
    vector as per-cell polynomials in the step's midpoint D = D0 + i dD; the expansion in
    E^2 = D^2 + m^2 is an identity of the header's per-step expressions (checked in exact
    rational arithmetic), and D0 + i dD is the midpoint slope (cl + (i + 1/2) h - xc)."""
    from fractions import Fraction as Fr
    import random
    rng = random.Random(7)
    for _ in range(50):
        slope = Fr(rng.choice([-1, 1])) * Fr(rng.randint(1, 1000), 97)
        v_w, m = Fr(rng.randint(1, 95), 100), Fr(rng.randint(1, 500), 113)
        dt, cl, xc, h = Fr(rng.randint(1, 90), 1000), Fr(rng.randint(-500, 0), 37), Fr(rng.randint(-50, 50), 41), \
            Fr(rng.randint(1, 100), 997)
        ddot = slope * v_w
        dd2, m2 = ddot * ddot, m * m
        dt2 = dt * dt
        dt4 = dt2 * dt2
        ax, bx = 1 - dd2 * dt4 / 60, dd2 * dt4 * dt2 / 1890
        cxm, cy, ey1, ey2 = dt * m, ddot * m * dt * dt2, dt2 / 90, dt4 / 7560
        cz = dt * (1 - bx * m2)
        D0, dD = slope * ((cl - xc) + h / 2), slope * h
        kx0, kx2 = cxm * (ax - bx * 4 * m2), -3 * cxm * bx
        ky0 = cy * (ey2 * (8 * m2 * m2 - 9 * dd2) + ey1 * m2 + Fr(1, 6))
        ky2, ky4 = cy * (16 * ey2 * m2 + ey1), 8 * cy * ey2
        for i in (0, 1, 7, 63):
            D = slope * (cl + (i + Fr(1, 2)) * h - xc)
            assert D0 + i * dD == D
            D2, E2 = D * D, D * D + m2
            assert kx0 + kx2 * D2 == cxm * (ax - bx * (3 * D2 + 4 * m2))
            assert ky0 + (ky2 + ky4 * D2) * D2 == cy * (ey2 * (8 * E2 * E2 - 9 * dd2) + ey1 * E2 + Fr(1, 6))


def test_profile_magnus_alphas_in_step_index():
    """Round 4 (lzq_profile.hip axis_poly): the Blanes-Casas-Ros alphas of a cubic, written in
    u = s / h (st + 1/2, exact), have the coefficients dk[m] c_m (alpha1), dk[1] (c1 + 0.15 h^2 c3),
    2 dk[2] c2, 3 dk[3] c3 (alpha2) and dk[2] c2, 3 dk[3] c3 (alpha3), dk[m] = dt h^m; checked
    against the Gauss-node definitions in exact arithmetic (sqrt(15) enters squared only)."""
    from fractions import Fraction as Fr
    import random
    rng = random.Random(11)
    for _ in range(30):
        c = [Fr(rng.randint(-99, 99), rng.randint(1, 50)) for _ in range(4)]
        h, dt = Fr(rng.randint(1, 60), 100), Fr(rng.randint(1, 60), 77)
        P = lambda s: ((c[3] * s + c[2]) * s + c[1]) * s + c[0]   # noqa: E731
        dk = [dt * h ** m for m in range(4)]
        e = [dk[m] * c[m] for m in range(4)]
        f = [dk[1] * (Fr(15, 100) * h * h * c[3] + c[1]), 2 * dk[2] * c[2], 3 * dk[3] * c[3]]
        g = [dk[2] * c[2], 3 * dk[3] * c[3]]
        for st in (0, 1, 5, 1000):
            u = st + Fr(1, 2)
            s = u * h
            d2 = Fr(15, 100) * h * h                                # delta^2, delta = sqrt(15)/10 h
            # P(s + d) - P(s - d) = 2 d (P'(s) + d^2 c3) and P(s + d) - 2 P(s) + P(s - d) = 2 d^2 (c2 + 3 c3 s)
            a1 = dt * P(s)
            a2 = dt * h * ((3 * c[3] * s + 2 * c[2]) * s + c[1] + d2 * c[3])  # sqrt15/3 dt (P+ - P-)
            a3 = Fr(10, 3) * dt * 2 * d2 * (c[2] + 3 * c[3] * s)             # 10/3 dt (P+ - 2P + P-)
            assert ((e[3] * u + e[2]) * u + e[1]) * u + e[0] == a1
            assert (f[2] * u + f[1]) * u + f[0] == a2
            assert g[1] * u + g[0] == a3
