"""Independent numpy restatement of the coherent two-level LZ propagation of
csrc/lzq_propagator.hip (TEST INFRASTRUCTURE).

The reference has no propagator, so parity is UNPINNED beyond the single-
crossing limit, which must reproduce the reference's closed form P = 1 - exp(-2 pi delta)
(fpy:183-184, PAPER eqs.(8)-(9)).  This module restates the same model with
the same fourth-order Magnus scheme, step by step, so the GPU kernel can be checked against
it to rounding, and the scheme itself against the closed form.
"""
import math

import numpy as np

S3 = math.sqrt(3.0) / 6.0


def chi_like(d, m):
    th = 0.5 * math.atan2(m, d)
    c, s = math.cos(th), math.sin(th)
    return (c, s) if abs(c) >= abs(s) else (-s, c)


DELTA_ADIABATIC = 16.0
STEPS_PER_RADIAN = 1.0


def wkb_G(x, m):
    return 0.5 * (x * math.sqrt(x * x + m * m) + (m * m * math.asinh(x / m) if m > 0 else 0.0))


def stokes_phase(delta):
    """pi/4 + delta (ln delta - 1) + arg Gamma(1 - i delta), large-delta (Stirling) series."""
    i1 = 1.0 / delta
    i2 = i1 * i1
    return i1 * (1.0 / 12.0 + i2 * (1.0 / 360.0 + i2 * (1.0 / 1260.0 + i2 * (1.0 / 1680.0))))


def adiabatic_cell(p, m, a, slope, xc, left, right, v_w):
    tl = 0.5 * math.atan2(m, slope * (left - xc))
    tr = 0.5 * math.atan2(m, slope * (right - xc))
    bp = math.cos(tl) * p[0] + math.sin(tl) * p[1]
    bm = -math.sin(tl) * p[0] + math.cos(tl) * p[1]
    Phi = (wkb_G(a * (right - xc), m) - wkb_G(a * (left - xc), m)) / (a * v_w)
    ph = Phi + stokes_phase(m * m / (2.0 * v_w * a))
    bp *= complex(math.cos(ph), -math.sin(ph))
    bm *= complex(math.cos(ph), math.sin(ph))
    return np.array([math.cos(tr) * bp - math.sin(tr) * bm, math.sin(tr) * bp + math.cos(tr) * bm])


def propagate(m_mix, dprime, xi, v_w, K, S, hybrid=True):
    """K = outer half-window in LZ lengths of the first / last crossing.  hybrid=True is the
    kernel's scheme (Magnus with max(S, phase) steps, exact adiabatic cells for delta > 16);
    hybrid=False is plain Magnus with S uniform steps in every cell (brute force)."""
    N = len(m_mix)
    left = xi[0] - K * xi_lz(m_mix[0], dprime[0], v_w)
    u0, u1 = chi_like(abs(dprime[0]) * (left - xi[0]), m_mix[0])
    p = np.array([u0 + 0j, u1 + 0j])
    sgn = 1.0
    right = left
    for c in range(N):
        ac = abs(dprime[c])
        if c + 1 < N:
            an = abs(dprime[c + 1])
            right = (ac * xi[c] + an * xi[c + 1]) / (ac + an)
        else:
            right = xi[c] + K * xi_lz(m_mix[c], dprime[c], v_w)
        slope = sgn * ac
        delta = m_mix[c] ** 2 / (2.0 * v_w * ac)
        if hybrid and delta > DELTA_ADIABATIC:
            p = adiabatic_cell(p, m_mix[c], ac, slope, xi[c], left, right, v_w)
            left = right
            sgn = -sgn
            continue
        Phi = (wkb_G(ac * (right - xi[c]), m_mix[c]) - wkb_G(ac * (left - xi[c]), m_mix[c])) / (ac * v_w)
        Sc = int(max(S, math.ceil(Phi * STEPS_PER_RADIAN))) if hybrid else S
        h = (right - left) / Sc
        dt = h / v_w
        nx = dt * m_mix[c]
        for i in range(Sc):
            xm = left + (i + 0.5) * h
            D1 = slope * ((xm - S3 * h) - xi[c])
            D2 = slope * ((xm + S3 * h) - xi[c])
            ny = S3 * dt * m_mix[c] * (D2 - D1) * dt
            nz = 0.5 * dt * (D1 + D2)
            nn = math.sqrt(nx * nx + ny * ny + nz * nz)
            sn, cs = math.sin(nn), math.cos(nn)
            sc = sn / nn if nn > 0 else 1.0
            sx, sy, sz = sc * nx, sc * ny, sc * nz
            U = np.array([[cs - 1j * sz, -sy - 1j * sx], [sy - 1j * sx, cs + 1j * sz]])
            p = U @ p
        left = right
        sgn = -sgn
    u0, u1 = chi_like(-sgn * abs(dprime[-1]) * (right - xi[-1]), m_mix[-1])
    a = u0 * p[0] + u1 * p[1]
    return 1.0 - abs(a) ** 2 / np.vdot(p, p).real


def xi_lz(m_mix, dprime, v_w):
    """LZ length scale in xi: sqrt(v_w/|Delta'|) * max(1, sqrt(delta)) (as the kernel's lz_length)."""
    a = abs(dprime)
    delta = m_mix * m_mix / (2.0 * v_w * a)
    return math.sqrt(v_w / a) * max(1.0, math.sqrt(delta))
