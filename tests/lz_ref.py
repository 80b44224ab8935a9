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
STEPS_PER_RADIAN = 6.0   # Magnus steps per radian of adiabatic phase in a cell's core
SA_LEVELS = 10           # superadiabatic frame order outside the core (rotations V_0 .. V_9)
SA_TOL = 1e-11           # core edge: next rotation angle |theta_10| ~ SA_C m / E^21 <= SA_TOL
SA_C = 3.2e5             # fitted: |theta_10| <= 3.2e5 m / E^21 (alpha = 1 units), conservative for m > 1
SA_M_FLOOR = 0.05        # core width floor: relative P error <= ~1e-10 for small couplings
SA_FAR_LEVELS = 6        # order of the frame at a follow stretch's outer end when
SA_FAR_C = 80.0          #   |theta_6| ~ SA_FAR_C max(mh, floor) / E^13 <= SA_TOL / 10
GL4_X = (-0.8611363115940526, -0.3399810435848563, 0.3399810435848563, 0.8611363115940526)
GL4_W = (0.3478548451374538, 0.6521451548625461, 0.6521451548625461, 0.3478548451374538)


def sa_levels(Dh, s, mh, N):
    """Superadiabatic frames of H = Dh sz + mh sx (alpha = 1 units: dDh/dtau = s = +-1) at one
    instant, by Taylor jets of length N in tau.  Level j: H_j = e_j sz + g_j sigma_(x if j even
    else y); the rotation V_j (about y for even j, about x for odd j) by theta_j = atan2(g_j, e_j)/2
    diagonalises it, and the frame after it has e_{j+1} = sqrt(e_j^2 + g_j^2), coupling
    g_{j+1} = -theta_j' (j even) or +theta_j' (j odd).  Returns [(cos theta_j, sin theta_j)],
    the values e_1 .. e_N and g_0 .. g_{N-1}."""
    e = [Dh, s] + [0.0] * (N - 2) if N >= 2 else [Dh]
    g = [mh] + [0.0] * (N - 1)
    cs, ev, gv = [], [], []
    for j in range(N):
        n = N - j
        q = [sum(e[i] * e[l - i] + g[i] * g[l - i] for i in range(l + 1)) for l in range(n)]
        r = [math.sqrt(q[0])]
        for l in range(1, max(n - 1, 1)):
            r.append((q[l] - sum(r[i] * r[l - i] for i in range(1, l))) / (2.0 * r[0]))
        c2, s2 = e[0] / r[0], g[0] / r[0]
        if e[0] >= 0.0:
            c = math.sqrt(0.5 * (1.0 + c2))
            sn = s2 / (2.0 * c)
        else:
            sn = math.sqrt(0.5 * (1.0 - c2))
            c = s2 / (2.0 * sn)
        cs.append((c, sn))
        ev.append(r[0])
        gv.append(g[0])
        if n == 1:
            break
        # theta_j' = (e g' - g e') / (2 q)
        num = [sum(e[i] * (l - i + 1) * g[l - i + 1] - g[i] * (l - i + 1) * e[l - i + 1] for i in range(l + 1))
               for l in range(n - 1)]
        w = []
        for l in range(n - 1):
            w.append((num[l] - sum(w[i] * q[l - i] for i in range(l))) / q[0])
        f = -0.5 if j % 2 == 0 else 0.5
        g = [f * x for x in w]
        e = r[:n - 1]
    return cs, ev, gv


def sa_to_frame(p, cs):
    """phi = V_{N-1}^+ ... V_0^+ p (diabatic -> frame N)."""
    a, b = complex(p[0]), complex(p[1])
    for j, (c, sn) in enumerate(cs):
        if j % 2 == 0:
            a, b = c * a + sn * b, c * b - sn * a
        else:
            a, b = c * a - 1j * sn * b, c * b - 1j * sn * a
    return a, b


def sa_from_frame(a, b, cs):
    """p = V_0 ... V_{N-1} (a, b) (frame N -> diabatic)."""
    for j in range(len(cs) - 1, -1, -1):
        c, sn = cs[j]
        if j % 2 == 0:
            a, b = c * a - sn * b, c * b + sn * a
        else:
            a, b = c * a + 1j * sn * b, c * b + 1j * sn * a
    return np.array([a, b])


def sa_core_tau(mh):
    """Core half-width in tau = sqrt(alpha) (xi - xi_c)/v_w: out to E = sqrt(tau^2 + mh^2) where
    the first neglected rotation, |theta_10| ~ SA_C mh / E^21, falls to SA_TOL, with mh floored at
    SA_M_FLOOR (for small mh, P ~ pi mh^2 and the relative error ~ 1/E^21); at least 1."""
    Ec = (SA_C * max(mh, SA_M_FLOOR) / SA_TOL) ** (1.0 / (2 * SA_LEVELS + 1))
    return math.sqrt(max(Ec * Ec - mh * mh, 1.0))


def sa_phase(ta, tb, mh):
    """int_ta^tb e_4 dtau on one side of the crossing (|ta|, |tb| >= 1): the WKB phase G, the
    leading dressed-energy term mh^2/(8E^5) in closed form (tail_T), and the rest,
    e_4 - E - mh^2/(8E^5) = O(E^-9), by 4-point Gauss-Legendre in u = 1/|tau|."""
    base = wkb_G(tb, mh) - wkb_G(ta, mh)
    lead = mh * mh * 0.125 * abs(tail_T(ta, mh) - tail_T(tb, mh))
    u1, u2 = 1.0 / abs(ta), 1.0 / abs(tb)
    ulo, uhi = min(u1, u2), max(u1, u2)
    half, mid = 0.5 * (uhi - ulo), 0.5 * (uhi + ulo)
    acc = 0.0
    for x, w in zip(GL4_X, GL4_W):
        u = mid + half * x
        _, ev, gv = sa_levels(1.0 / u, 1.0, mh, 4)
        E = ev[0]
        d1 = gv[1] * gv[1] / (E + ev[1])
        d2 = gv[2] * gv[2] / (ev[1] + ev[2])
        d3 = gv[3] * gv[3] / (ev[2] + ev[3])
        E5 = E * E * E * E * E
        f = d3 + d2 - mh * mh * d1 / (8.0 * E5 * (E + ev[1]))
        acc += w * f / (u * u)
    return base + lead + half * acc


def sa_follow(p, mh, s, ta, tb):
    """Superadiabatic following from tau = ta to tb (ta < tb, same side of the crossing): p to
    the frame of order SA_LEVELS at ta, the frame amplitudes pick up exp(-+ i int e dtau), back
    to the diabatic basis at tb.  Error ~ the first neglected rotation angle at the inner end."""
    tf = max(abs(ta), abs(tb))
    Ef2 = tf * tf + mh * mh
    Ef12 = (Ef2 * Ef2) * (Ef2 * Ef2) * (Ef2 * Ef2)
    far6 = SA_FAR_C * max(mh, SA_M_FLOOR) <= 0.1 * SA_TOL * Ef12 * math.sqrt(Ef2)
    ca, _, _ = sa_levels(s * ta, s, mh, SA_FAR_LEVELS if far6 and abs(ta) == tf else SA_LEVELS)
    cb, _, _ = sa_levels(s * tb, s, mh, SA_FAR_LEVELS if far6 and abs(tb) == tf else SA_LEVELS)
    a, b = sa_to_frame(p, ca)
    ph = sa_phase(ta, tb, mh)
    a *= complex(math.cos(ph), -math.sin(ph))
    b *= complex(math.cos(ph), math.sin(ph))
    return sa_from_frame(a, b, cb)


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
        if hybrid:   # Magnus only on the cell's core; superadiabatic following outside it
            sa = math.sqrt(ac * v_w)
            mh = m_mix[c] / sa
            tc = sa_core_tau(mh)
            sgn_s = 1.0 if slope > 0 else -1.0
            tl, tr = sa * (left - xi[c]) / v_w, sa * (right - xi[c]) / v_w
            if tl < -tc:
                p = sa_follow(p, mh, sgn_s, tl, -tc)
                left = xi[c] - tc * v_w / sa
            if tr > tc:
                right = xi[c] + tc * v_w / sa
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
        if hybrid and right < cell_right:
            p = sa_follow(p, mh, sgn_s, tc, sa * (cell_right - xi[c]) / v_w)
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
