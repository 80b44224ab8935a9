"""Independent numpy restatement of the coherent two-level LZ propagation of
csrc/lzq_propagator.hip (TEST INFRASTRUCTURE).

The reference has no propagator, so parity is UNPINNED beyond the single-
crossing limit, which must reproduce the reference's closed form P = 1 - exp(-2 pi delta)
(fpy:183-184, PAPER eqs.(8)-(9)).  This module restates the same model with
the same eighth-order Magnus scheme, step by step, so the GPU kernel can be checked against
it to rounding, and the scheme itself against the closed form.  Start state and final
projection are the second-order dressed (superadiabatic) chi-like states of the outer cells.
"""
import math

import numpy as np



def chi_like(d, m):
    th = 0.5 * math.atan2(m, d)
    c, s = math.cos(th), math.sin(th)
    return (c, s) if abs(c) >= abs(s) else (-s, c)


def dressed_basis(d, ddot, m):
    """Second-order superadiabatic ("dressed") states of H = d sz + m sx with d' = ddot (d linear
    in t), as the kernel's dressed_basis: returns (plus, minus), orthonormal complex 2-vectors.
    With theta = atan2(m, d)/2, |+> = (cos, sin), |-> = (-sin, cos), E = sqrt(d^2 + m^2),
    eps = theta'/(2E) = -m ddot/(4E^3) and eps' = 3 m ddot^2 d/(4E^5):
        |+~> ~ |+> + beta |->,   beta  = -i eps - eps'/(2E)
        |-~> ~ |-> + gamma |+>,  gamma = -i eps + eps'/(2E) = -conj(beta)
    (adiabatic elimination of the non-adiabatic coupling to second order: a state prepared in
    |+~> stays in it up to O(eps / (alpha tau^2)^2), so the window edges are K^-7 accurate)."""
    th = 0.5 * math.atan2(m, d)
    c, s = math.cos(th), math.sin(th)
    E = math.hypot(d, m)
    eps = -m * ddot / (4.0 * E ** 3)
    epsd = 3.0 * m * ddot * ddot * d / (4.0 * E ** 5)
    beta = complex(-epsd / (2.0 * E), -eps)
    nrm = 1.0 / math.sqrt(1.0 + abs(beta) ** 2)
    plus = np.array([c - s * beta, s + c * beta]) * nrm
    minus = np.array([-s - c * beta.conjugate(), c - s * beta.conjugate()]) * nrm
    return plus, minus


def chi_like_dressed(d, ddot, m):
    """The dressed state that is chi-like (|<chi|.>| >= 1/sqrt2): kernel's start / projection."""
    plus, minus = dressed_basis(d, ddot, m)
    return plus if abs(plus[0]) >= abs(plus[1]) else minus


def tail_T(x0, m):
    """int_{|x0|}^inf dx / (x^2 + m^2)^{5/2} (second-order dressed-energy tail, adiabatic cells)."""
    x0 = abs(x0)
    u = (m / x0) ** 2 if x0 > 0 else math.inf
    if u < 1e-3:   # series in u = m^2/x0^2: (1/4 - 5u/12 + 35u^2/64 - 21u^3/32) / x0^4
        return (0.25 - u * (5.0 / 12.0 - u * (35.0 / 64.0 - u * (21.0 / 32.0)))) / x0 ** 4
    E = math.hypot(x0, m)
    return (2.0 - x0 * (2.0 * x0 * x0 + 3.0 * m * m) / E ** 3) / (3.0 * m ** 4)


DELTA_ADIABATIC = 16.0
STEPS_PER_RADIAN = 3.0
CORE_EPS = 1e-5   # Magnus core of a cell: where the adiabaticity eps = m|alpha|/(4E^3) exceeds this


def core_halfwidth(m, a, v_w, K):
    """Half-width (in xi) of the cell's Magnus core.  delta <= 1: 2K LZ lengths (the
    transition builds up over the whole crossing region, so the dressed following error is set
    by the distance in LZ lengths: ~1e-12 at 2K = 40, 2e-11 at K = 20).  delta > 1: out to
    |D| where eps = m|alpha|/(4E^3) falls to CORE_EPS (beyond it the dressed basis follows the
    state to ~eps^2), at least one and at most 2K LZ lengths.  Cells narrower than the core
    (C5's are +-20 LZ lengths) are stepped end to end as before."""
    L = xi_lz(m, a, v_w)
    if m * m <= 2.0 * v_w * a:     # delta <= 1
        return 2.0 * K * L
    Ec = (m * a * v_w / (4.0 * CORE_EPS)) ** (1.0 / 3.0)
    Dc = math.sqrt(max(Ec * Ec - m * m, 0.0))
    return min(2.0 * K * L, max(L, Dc / a))


def far_segment(p, m, a, slope, xc, xa, xb, v_w):
    """Dressed-basis following from xa to xb on one side of crossing xc (no stepping): the
    dressed amplitudes pick up exp(-+ i (Phi + (m^2 |alpha|/8) |int dD/E^5|)) over the segment
    (the second-order dressed energy; the same terms as adiabatic_cell's tails)."""
    Da, Db = slope * (xa - xc), slope * (xb - xc)
    ddot = slope * v_w
    lp, lm = dressed_basis(Da, ddot, m)
    rp, rm = dressed_basis(Db, ddot, m)
    bp, bm = np.vdot(lp, p), np.vdot(lm, p)
    Phi = (wkb_G(a * (xb - xc), m) - wkb_G(a * (xa - xc), m)) / (a * v_w)
    corr = m * m * a * v_w / 8.0 * abs(tail_T(Da, m) - tail_T(Db, m))
    ph = Phi + corr
    bp *= complex(math.cos(ph), -math.sin(ph))
    bm *= complex(math.cos(ph), math.sin(ph))
    return bp * rp + bm * rm


def wkb_G(x, m):
    return 0.5 * (x * math.sqrt(x * x + m * m) + (m * m * math.asinh(x / m) if m > 0 else 0.0))


def stokes_phase(delta):
    """pi/4 + delta (ln delta - 1) + arg Gamma(1 - i delta), large-delta (Stirling) series."""
    i1 = 1.0 / delta
    i2 = i1 * i1
    return i1 * (1.0 / 12.0 + i2 * (1.0 / 360.0 + i2 * (1.0 / 1260.0 + i2 * (1.0 / 1680.0))))


def adiabatic_cell(p, m, a, slope, xc, left, right, v_w):
    """Exact adiabatic following in the dressed basis of the cell: phase = WKB Phi + Stokes phase
    (the whole line's dressed-energy correction) minus the part of that correction, (m^2 alpha/8)
    int dx/E^5, that lies outside the cell."""
    DL, DR = slope * (left - xc), slope * (right - xc)
    ddot = slope * v_w
    lp, lm = dressed_basis(DL, ddot, m)
    rp, rm = dressed_basis(DR, ddot, m)
    bp, bm = np.vdot(lp, p), np.vdot(lm, p)
    Phi = (wkb_G(a * (right - xc), m) - wkb_G(a * (left - xc), m)) / (a * v_w)
    tails = m * m * a * v_w / 8.0 * (tail_T(DL, m) + tail_T(DR, m))
    ph = Phi + stokes_phase(m * m / (2.0 * v_w * a)) - tails
    bp *= complex(math.cos(ph), -math.sin(ph))
    bm *= complex(math.cos(ph), math.sin(ph))
    return bp * rp + bm * rm


def propagate(m_mix, dprime, xi, v_w, K, S, hybrid=True):
    """K = outer half-window in LZ lengths of the first / last crossing.  hybrid=True is the
    kernel's scheme (Magnus with max(S, phase) steps, exact adiabatic cells for delta > 16);
    hybrid=False is plain Magnus with S uniform steps in every cell (brute force)."""
    N = len(m_mix)
    left = xi[0] - K * xi_lz(m_mix[0], dprime[0], v_w)
    a0 = abs(dprime[0])
    p = chi_like_dressed(a0 * (left - xi[0]), a0 * v_w, m_mix[0])
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
        cell_right = right
        if hybrid:   # Magnus only on the cell's core; dressed following outside it
            W = core_halfwidth(m_mix[c], ac, v_w, K)
            cl, cr = max(left, xi[c] - W), min(right, xi[c] + W)
            if left < cl:
                p = far_segment(p, m_mix[c], ac, slope, xi[c], left, cl, v_w)
            left, right = cl, cr
        Phi = (wkb_G(ac * (right - xi[c]), m_mix[c]) - wkb_G(ac * (left - xi[c]), m_mix[c])) / (ac * v_w)
        Sc = int(max(S, math.ceil(Phi * STEPS_PER_RADIAN))) if hybrid else S
        h = (right - left) / Sc
        dt = h / v_w
        mc = m_mix[c]
        # eighth-order Magnus vector of the linear-in-t Hamiltonian (kernel header), same
        # operation order as the kernel
        ddot = slope * v_w
        dd2, m2 = ddot * ddot, mc * mc
        dt2 = dt * dt
        dt4 = dt2 * dt2
        ax = 1.0 - dd2 * dt4 * (1.0 / 60.0)
        bx = dd2 * dt4 * dt2 * (1.0 / 1890.0)
        cxm, m2x4 = dt * mc, 4.0 * m2
        cy, ey1, ey2 = ddot * mc * dt * dt2, dt2 * (1.0 / 90.0), dt4 * (1.0 / 7560.0)
        dd2x9 = 9.0 * dd2
        cz = dt * (1.0 - bx * m2)
        for i in range(Sc):
            xm = left + (i + 0.5) * h
            D = slope * (xm - xi[c])
            D2 = D * D
            E2 = D2 + m2
            nx = cxm * (ax - bx * (3.0 * D2 + m2x4))
            ny = cy * ((1.0 / 6.0) + ey1 * E2 + ey2 * (8.0 * E2 * E2 - dd2x9))
            nz = cz * D
            nn = math.sqrt(nx * nx + ny * ny + nz * nz)
            sn, cs = math.sin(nn), math.cos(nn)
            sc = sn / nn if nn > 0 else 1.0
            sx, sy, sz = sc * nx, sc * ny, sc * nz
            U = np.array([[cs - 1j * sz, -sy - 1j * sx], [sy - 1j * sx, cs + 1j * sz]])
            p = U @ p
        if right < cell_right:
            p = far_segment(p, m_mix[c], ac, slope, xi[c], right, cell_right, v_w)
        left = right = cell_right
        sgn = -sgn
    slope = -sgn * abs(dprime[-1])
    u = chi_like_dressed(slope * (right - xi[-1]), slope * v_w, m_mix[-1])
    a = np.vdot(u, p)
    return 1.0 - abs(a) ** 2 / np.vdot(p, p).real


def xi_lz(m_mix, dprime, v_w):
    """LZ length scale in xi: sqrt(v_w/|Delta'|) * max(1, sqrt(delta)) (as the kernel's lz_length)."""
    a = abs(dprime)
    delta = m_mix * m_mix / (2.0 * v_w * a)
    return math.sqrt(v_w / a) * max(1.0, math.sqrt(delta))
