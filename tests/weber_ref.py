"""Exact finite-time solution of the piecewise-linear LZ model of csrc/lzq_propagator.hip via
Weber (parabolic-cylinder) functions, in mpmath (TEST INFRASTRUCTURE; SURVEY §8f(2)
"validation ... against the exact finite-time Weber-function solution").

Model: i dpsi/dt = H psi, t = xi / v_w, H = Delta(xi) sigma_z + m_c sigma_x with
Delta = s_c |Delta'_c| (xi - xi_c) on cell c.  On one cell, with tau = t - t_c and
alpha = s_c |Delta'_c| v_w, the lower component obeys

    c2'' + (alpha^2 tau^2 + m^2 - i alpha) c2 = 0,

which z = sqrt(2 alpha) e^{i pi/4} tau turns into Weber's equation
y'' + (nu + 1/2 - z^2/4) y = 0 with nu = -1 - i m^2/(2 alpha).  D_nu(z) and D_nu(-z) are
independent for non-integer nu, and c1 = (i c2' + alpha tau c2) / m.  Each cell is solved
exactly in closed form (no time stepping), so this pins the kernel's Magnus / adiabatic-cell
scheme and its window edges without sharing any of its numerics.  Cell edges, start state and
final projection (the second-order dressed chi-like states of the outer cells) are the
kernel's (tests/lz_ref.py); inside the window the solution is exact.
"""
import math

import mpmath as mp

from lz_ref import chi_like_dressed, xi_lz


def _cell(psi, m, alpha, tau0, tau1):
    """Exact propagation of psi = (c1, c2) from tau0 to tau1 under H = alpha tau sz + m sx."""
    c1, c2 = psi
    if m == 0:
        ph = alpha * (tau1 * tau1 - tau0 * tau0) / 2
        return (c1 * mp.expj(-ph), c2 * mp.expj(ph))
    k = mp.sqrt(2 * alpha) * mp.expj(mp.pi / 4)          # dz/dtau
    nu = -1 - 1j * (m * m) / (2 * alpha)

    def basis(tau):
        z = k * tau
        y1, y1n = mp.pcfd(nu, z), mp.pcfd(nu + 1, z)
        y2, y2n = mp.pcfd(nu, -z), mp.pcfd(nu + 1, -z)
        # D'_nu(z) = z/2 D_nu(z) - D_{nu+1}(z)
        d1 = k * (z / 2 * y1 - y1n)
        d2 = -k * (-z / 2 * y2 - y2n)
        return y1, d1, y2, d2

    y1, d1, y2, d2 = basis(tau0)
    c2p = -1j * (m * c1 - alpha * tau0 * c2)                  # i c2' = m c1 - alpha tau c2
    det = y1 * d2 - y2 * d1
    A = (c2 * d2 - y2 * c2p) / det
    B = (y1 * c2p - c2 * d1) / det
    y1, d1, y2, d2 = basis(tau1)
    c2n = A * y1 + B * y2
    c2pn = A * d1 + B * d2
    c1n = (1j * c2pn + alpha * tau1 * c2n) / m
    return (c1n, c2n)


def propagate_exact(m_mix, dprime, xi, v_w, K, dps=40):
    """P of tests/lz_ref.propagate (same windows, start state and projection), exact."""
    with mp.workdps(dps):
        N = len(m_mix)
        left = xi[0] - K * xi_lz(m_mix[0], dprime[0], v_w)
        a0 = abs(dprime[0])
        u = chi_like_dressed(a0 * (left - xi[0]), a0 * v_w, m_mix[0])
        psi = (mp.mpc(u[0]), mp.mpc(u[1]))
        sgn = 1.0
        right = left
        for c in range(N):
            ac = abs(dprime[c])
            if c + 1 < N:
                an = abs(dprime[c + 1])
                right = (ac * xi[c] + an * xi[c + 1]) / (ac + an)
            else:
                right = xi[c] + K * xi_lz(m_mix[c], dprime[c], v_w)
            alpha = mp.mpf(sgn * ac * v_w)
            t0 = (mp.mpf(left) - xi[c]) / v_w
            t1 = (mp.mpf(right) - xi[c]) / v_w
            psi = _cell(psi, mp.mpf(m_mix[c]), alpha, t0, t1)
            left = right
            sgn = -sgn
        slope = -sgn * abs(dprime[-1])
        u = chi_like_dressed(slope * (right - xi[-1]), slope * v_w, m_mix[-1])
        a = mp.conj(mp.mpc(u[0])) * psi[0] + mp.conj(mp.mpc(u[1])) * psi[1]
        nrm = abs(psi[0]) ** 2 + abs(psi[1]) ** 2
        return float(1 - abs(a) ** 2 / nrm)


if __name__ == "__main__":
    import time
    from lz_ref import propagate
    for m, d, K in [(0.1, 1.0, 6.0), (0.3, 0.5, 12.0), (0.01, 0.1, 12.0)]:
        t = time.time()
        pe = propagate_exact([m], [d], [0.0], 0.3, K)
        te = time.time() - t
        pm = propagate([m], [d], [0.0], 0.3, K, 4000, hybrid=False)
        delta = m * m / (2 * 0.3 * d)
        print(m, d, K, pe, pm, abs(pe - pm), 1 - math.exp(-2 * math.pi * delta), f"{te:.2f}s")
