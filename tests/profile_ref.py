"""Independent numpy restatement of the bounce-profile LZ path (TEST INFRASTRUCTURE):
PAPER p.3 eqs.(5)-(9) on a profile of two background fields phi(xi), Phi(xi), as
csrc/lzq_profile.hip computes it.

The upstream `transport_from_profile` module the reference's hook imports (fpy:173) is absent,
so parity is UNPINNED against it; this restatement pins the kernels to the paper's equations:

  xi = r - R_0                                    (PAPER p.3 §3.1, wall coordinate)
  phi, Phi: not-a-knot cubic splines of the samples (scipy CubicSpline, as fpy:212 builds its
            A/V spline) -- "interpolated as smooth functions"
  Delta(xi)  = y_B phi(xi) - y_chi Phi(xi)        eq.(5); crossings xi*: Delta(xi*) = 0
  Delta'*    = y_B phi'(xi*) - y_chi Phi'(xi*)    eq.(6)
  m_mix(xi)  = lambda_tr_eff phi(xi)              eq.(7)
  delta_LZ   = m_mix(xi*)^2 / (2 v_w |Delta'*|)   eq.(8), F(k) = 1
  P          = 1 - exp(-2 pi delta_LZ)            eq.(9) (fpy:183-184)

and, beyond the minimal estimator, the time-ordered propagation of
i dpsi/dt = H psi, H = Delta(xi) sigma_z + m_mix(xi) sigma_x, xi = v_w t, through the whole
profile (several crossings interfere): sixth-order Magnus (three Gauss-Legendre nodes, the
Blanes-Casas-Ros commutator form) on uniform steps per knot interval, started in and projected
on the chi-like second-order dressed (superadiabatic) state at the profile's two ends.
"""
import math
from fractions import Fraction

import numpy as np

SQ15 = math.sqrt(15.0)
GL3 = (0.5 - SQ15 / 10.0, 0.5, 0.5 + SQ15 / 10.0)


# ---- splines ----------------------------------------------------------------------------
def spline_coefs(x, y):
    """Not-a-knot cubic spline (scipy CubicSpline default) as ascending local coefficients
    [n-1][4]: y(x) = c0 + c1 t + c2 t^2 + c3 t^3, t = x - x_j on [x_j, x_{j+1}]."""
    from scipy.interpolate import CubicSpline
    cs = CubicSpline(np.asarray(x, float), np.asarray(y, float))
    return np.ascontiguousarray(cs.c[::-1].T)


def pp_eval(c, t, der=0):
    c0, c1, c2, c3 = c
    if der == 0:
        return c0 + t * (c1 + t * (c2 + t * c3))
    if der == 1:
        return c1 + t * (2.0 * c2 + t * 3.0 * c3)
    if der == 2:
        return 2.0 * c2 + 6.0 * c3 * t
    return 6.0 * c3


def locate(knots, x):
    j = int(np.searchsorted(knots, x, side="right")) - 1
    return min(max(j, 0), len(knots) - 2)


def dm_coefs(cphi, cPhi, yB, ychi, lam):
    """Per-interval coefficients of Delta (eq.5) and m_mix (eq.7)."""
    cD = yB * np.asarray(cphi) - ychi * np.asarray(cPhi)
    cM = lam * np.asarray(cphi)
    return cD, cM


# ---- crossings (eqs.(5)-(8)) --------------------------------------------------------------
def _root(c, a, b):
    """The root of the cubic c on [a, b] where it changes sign (monotone there): safeguarded
    Newton, to full precision."""
    fa = pp_eval(c, a)
    lo, hi = a, b
    x = a - fa * (b - a) / (pp_eval(c, b) - fa)
    for _ in range(100):
        f = pp_eval(c, x)
        if f == 0.0:
            return x
        if (f < 0) == (fa < 0):
            lo = x
        else:
            hi = x
        d = pp_eval(c, x, 1)
        xn = x - f / d if d != 0 else 0.5 * (lo + hi)
        if not (lo < xn < hi):
            xn = 0.5 * (lo + hi)
        if xn == x or hi - lo <= 4e-16 * max(abs(lo), abs(hi), 1e-300):
            return xn
        x = xn
    return x


def crossings(knots, cphi, cPhi, yB, ychi, lam, v_w):
    """[(xi*, Delta'*, m_mix*, delta_LZ)] for every sign change of Delta over the profile.  Each
    knot interval's cubic is cut at its stationary points into monotone pieces; a piece whose
    end values have opposite signs holds one root (safeguarded Newton); a zero exactly on a
    piece boundary is a crossing when the last nonzero value before it and the first after it
    differ in sign (taken where the zero was met)."""
    cD, cM = dm_coefs(cphi, cPhi, yB, ychi, lam)
    out = []
    last = 0.0            # sign of the last nonzero boundary value
    pend = None           # (j, t) of a boundary zero awaiting the next sign

    def emit(j, t):
        dp = pp_eval(cD[j], t, 1)
        m = pp_eval(cM[j], t)
        out.append((knots[j] + t, dp, m, m * m / (2.0 * max(v_w, 1e-12) * abs(dp))))

    def boundary(v, j, t, last, pend, emit):
        if v == 0.0:
            return last, (pend if pend is not None or last == 0.0 else (j, t))
        sg = 1.0 if v > 0.0 else -1.0
        if pend is not None and sg != last:
            emit(*pend)
        return sg, None

    for j in range(len(knots) - 1):
        L = knots[j + 1] - knots[j]
        c = cD[j]
        cuts = [0.0]
        A, B, C = 3.0 * c[3], 2.0 * c[2], c[1]
        if A != 0.0:
            disc = B * B - 4 * A * C
            if disc > 0:
                s = math.sqrt(disc)
                q = -0.5 * (B + math.copysign(s, B))
                r1, r2 = sorted((q / A, C / q))
                cuts += [r for r in (r1, r2) if 0.0 < r < L]
        elif B != 0.0:
            r = -C / B
            if 0.0 < r < L:
                cuts.append(r)
        cuts.append(L)
        for a, b in zip(cuts[:-1], cuts[1:]):
            fa, fb = pp_eval(c, a), pp_eval(c, b)
            last, pend = boundary(fa, j, a, last, pend, emit)
            if fa * fb < 0.0:
                emit(j, _root(c, a, b))
            last, pend = boundary(fb, j, b, last, pend, emit)
    return out


# ---- dressed edges -------------------------------------------------------------------------
def dressed_chi_like(D, Dd, Ddd, m, md, mdd):
    """The chi-like second-order dressed state of H = D sz + m sx with time derivatives
    (Dd, Ddd), (md, mdd): theta = atan2(m, D)/2, eps = theta'/(2E), beta = -i eps - eps'/(2E)
    (lz_ref.dressed_basis with m(t) varying)."""
    E2 = D * D + m * m
    E = math.sqrt(E2)
    th = 0.5 * math.atan2(m, D)
    c, s = math.cos(th), math.sin(th)
    w = md * D - m * Dd
    thd = w / (2.0 * E2)
    Ed = (D * Dd + m * md) / E
    thdd = (mdd * D - m * Ddd) / (2.0 * E2) - w * Ed / (E2 * E)
    eps = thd / (2.0 * E)
    epsd = thdd / (2.0 * E) - thd * Ed / (2.0 * E2)
    beta = complex(-epsd / (2.0 * E), -eps)
    nrm = 1.0 / math.sqrt(1.0 + abs(beta) ** 2)
    plus = np.array([c - s * beta, s + c * beta]) * nrm
    minus = np.array([-s - c * beta.conjugate(), c - s * beta.conjugate()]) * nrm
    return plus if abs(plus[0]) >= abs(plus[1]) else minus


def _edge(cD, cM, t, v_w):
    return dressed_chi_like(pp_eval(cD, t), v_w * pp_eval(cD, t, 1), v_w * v_w * pp_eval(cD, t, 2),
                            pp_eval(cM, t), v_w * pp_eval(cM, t, 1), v_w * v_w * pp_eval(cM, t, 2))


# ---- propagation ---------------------------------------------------------------------------
STEPS_PER_RADIAN = 4.0
MIN_STEPS = 1
HDOT_RATE = 4.0   # the crossing region's rate: HDOT_RATE / (LZ time), LZ time = |dH/dt|^-1/2


def fma(a, b, c):
    """a * b + c with one rounding (exact rational arithmetic, then Python's correctly rounded
    conversion): the restatement of the kernels' fused multiply-adds."""
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def _samples(c, L):
    """The shape's samples at t_q = (q/4) L, q = 0..4 (profile_samples_kernel), as the products the
    rule's quadratic forms take: (phi^2, phi Phi, Phi^2, phi'^2, phi' Phi', Phi'^2)."""
    cphi, cPhi = c
    out = []
    for q in range(5):
        t = (0.25 * q) * L
        a, b = pp_eval(cphi, t), pp_eval(cPhi, t)
        da, db = pp_eval(cphi, t, 1), pp_eval(cPhi, t, 1)
        out.append((a * a, a * b, b * b, da * da, da * db, db * db))
    return out


def interval_steps(knots, cphi, cPhi, j, yB, ychi, lam, v_w, spr=STEPS_PER_RADIAN, n_min=MIN_STEPS):
    """Uniform Magnus steps on knot interval j: spr x the interval's largest local rate
    omega = max(E, HDOT_RATE sqrt(v_w |dH/dt|)) x its duration (L / v_w), at least n_min.  The rate
    is sampled at t_q = (q/4) L, q = 0..3, from the interval's own cubic and at its end from the
    next interval's q = 0 sample (the last interval: its own q = 4).  E^2 = D^2 + m^2 with
    Delta = y_B phi - y_chi Phi, m = lambda phi (eqs.(5),(7)) is the quadratic form
    A phi^2 + B phi Phi + C Phi^2, A = y_B^2 + lambda^2, B = -2 y_B y_chi, C = y_chi^2, over the
    shape's (coupling-independent, precomputed) sample products; |dH/dt|^2 the same in phi', Phi'.
    The kernel's operations: the maxima e2, h2 over the samples, then
    W2 = max(e2, HDOT_RATE^2 (v_w sqrt(h2))), S = ceil((spr (L (1 / v_w))) sqrt(W2))."""
    L = knots[j + 1] - knots[j]
    own = _samples((cphi[j], cPhi[j]), L)
    nI = len(knots) - 1
    end = _samples((cphi[j + 1], cPhi[j + 1]), knots[j + 2] - knots[j + 1])[0] if j + 1 < nI else own[4]
    A, B, C = fma(yB, yB, lam * lam), (-2.0 * yB) * ychi, ychi * ychi
    e2 = h2 = 0.0
    for aa, ab, bb, dada, dadb, dbdb in own[:4] + [end]:
        e2 = max(e2, fma(A, aa, fma(B, ab, C * bb)))
        h2 = max(h2, fma(A, dada, fma(B, dadb, C * dbdb)))
    W2 = max(e2, (HDOT_RATE * HDOT_RATE) * (v_w * math.sqrt(h2)))
    return max(n_min, int(math.ceil((spr * (L * (1.0 / v_w))) * math.sqrt(W2))))


def magnus6_vector(a1, a2, a3, dt):
    """Omega = -i n.sigma of one step from H = x sigma_x + z sigma_z at the three GL nodes
    (a_k = (x_k, z_k)); the Lie bracket of -i a.sigma and -i b.sigma is -i (2 a x b).sigma."""
    x1, z1 = dt * a2[0], dt * a2[1]                           # alpha1
    k2 = SQ15 / 3.0 * dt
    x2, z2 = k2 * (a3[0] - a1[0]), k2 * (a3[1] - a1[1])       # alpha2
    k3 = 10.0 / 3.0 * dt
    x3, z3 = k3 * (a3[0] - 2.0 * a2[0] + a1[0]), k3 * (a3[1] - 2.0 * a2[1] + a1[1])  # alpha3
    c = 2.0 * (z1 * x2 - x1 * z2)                             # C1 = [alpha1, alpha2] (y only)
    C2 = (z1 * c / 30.0, -(z1 * x3 - x1 * z3) / 15.0, -x1 * c / 30.0)  # -[alpha1, 2 alpha3 + C1]/60
    Lv = (-20.0 * x1 - x3, c, -20.0 * z1 - z3)                # -20 alpha1 - alpha3 + C1
    R = (x2 + C2[0], C2[1], z2 + C2[2])                       # alpha2 + C2
    cr = (Lv[1] * R[2] - Lv[2] * R[1], Lv[2] * R[0] - Lv[0] * R[2], Lv[0] * R[1] - Lv[1] * R[0])
    nx = x1 + x3 / 12.0 + cr[0] / 120.0
    ny = cr[1] / 120.0
    nz = z1 + z3 / 12.0 + cr[2] / 120.0
    return nx, ny, nz


def su2(nx, ny, nz):
    nn = math.sqrt(nx * nx + ny * ny + nz * nz)
    cs = math.cos(nn)
    sc = math.sin(nn) / nn if nn > 0 else 1.0
    sx, sy, sz = sc * nx, sc * ny, sc * nz
    return np.array([[cs - 1j * sz, -sy - 1j * sx], [sy - 1j * sx, cs + 1j * sz]])


def propagate_profile(knots, cphi, cPhi, yB, ychi, lam, v_w, spr=STEPS_PER_RADIAN, n_min=MIN_STEPS,
                      cD=None, cM=None):
    """Coherent conversion probability through the whole profile [x_0, x_{n-1}].  (cD, cM):
    Delta and m_mix rows given directly = phi := m, Phi := Delta with y_B = 0, y_chi = -1,
    lambda = 1 (exact)."""
    if cD is not None:
        cphi, cPhi, yB, ychi, lam = np.asarray(cM), np.asarray(cD), 0.0, -1.0, 1.0
    cD, cM = dm_coefs(cphi, cPhi, yB, ychi, lam)
    nI = len(knots) - 1
    p = _edge(cD[0], cM[0], 0.0, v_w)
    for j in range(nI):
        L = knots[j + 1] - knots[j]
        S = interval_steps(knots, cphi, cPhi, j, yB, ychi, lam, v_w, spr, n_min)
        h = L / S
        dt = h / v_w
        for i in range(S):
            a = [(pp_eval(cM[j], (i + g) * h), pp_eval(cD[j], (i + g) * h)) for g in GL3]
            p = su2(*magnus6_vector(a[0], a[1], a[2], dt)) @ p
    u = _edge(cD[-1], cM[-1], knots[-1] - knots[-2], v_w)
    amp = np.vdot(u, p)
    return 1.0 - abs(amp) ** 2 / np.vdot(p, p).real


# ---- the piecewise-linear cell model of lzq_lz_propagate as a profile ---------------------
def linear_cells_profile(m_mix, dprime, xi, v_w, K):
    """Knots and (Delta, m) coefficients of lzq_lz_propagate's model (tests/lz_ref.py):
    cell edges = window edges and turning points, Delta linear with alternating slope,
    m constant per cell.  Returned as (knots, cD, cM)."""
    from lz_ref import xi_lz
    N = len(m_mix)
    edges = [xi[0] - K * xi_lz(m_mix[0], dprime[0], v_w)]
    for c in range(N - 1):
        a, b = abs(dprime[c]), abs(dprime[c + 1])
        edges.append((a * xi[c] + b * xi[c + 1]) / (a + b))
    edges.append(xi[-1] + K * xi_lz(m_mix[-1], dprime[-1], v_w))
    cD, cM = [], []
    sgn = 1.0
    for c in range(N):
        s = sgn * abs(dprime[c])
        cD.append([s * (edges[c] - xi[c]), s, 0.0, 0.0])
        cM.append([m_mix[c], 0.0, 0.0, 0.0])
        sgn = -sgn
    return np.array(edges), np.array(cD), np.array(cM)
