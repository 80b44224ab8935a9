#!/usr/bin/env python3
"""Coefficients of the table-driven exponential (csrc/lzq_exp2.h, table variant):

    2^(r/N) - 1 ~= r*(B1 + r*(B2 + ... + r*B_deg)),   r in [-1/2, 1/2],   N = 2^bits,

fitted as a weighted discrete minimax (Lawson iteration, mpmath at 60 digits) of the
ABSOLUTE error of q (the kernel forms T*(1+q) with one fma, so |dq| is the relative error of
the result), then rounded to double.  Prints C hex-floats plus the fitted error and the
worst error of the double-precision evaluation against mpmath.

    python tools/exp2_tab_poly.py BITS DEG
    python tools/exp2_tab_poly.py --sq [A]     (completed-square form, 13 bits)

--sq fits the completed-square form of LZQ_SQFORM, 2^(r/N) ~= C*((r + A)^2 + beta) with A a
fixed INTEGER (default 11819): a minimax of the RELATIVE error over (C, C*D), D = A^2 + beta,
which is linear in those two unknowns (a linear program), and prints kSqC / kSqBeta.
"""
import sys

import mpmath as mp
import numpy as np

mp.mp.dps = 60


def fit(bits, deg, npts=300, iters=80):
    N = mp.mpf(2) ** bits
    xs = [mp.mpf(0.5) * mp.cos(mp.pi * (i + mp.mpf(0.5)) / npts) for i in range(npts)]
    f = [(mp.power(2, x / N) - 1) for x in xs]
    A = [[x ** (j + 1) for j in range(deg)] for x in xs]
    lw = [mp.mpf(1)] * npts
    for _ in range(iters):
        M = mp.matrix(deg, deg)
        v = mp.matrix(deg, 1)
        for i in range(npts):
            for a in range(deg):
                v[a] += lw[i] * A[i][a] * f[i]
                for c in range(deg):
                    M[a, c] += lw[i] * A[i][a] * A[i][c]
        B = mp.lu_solve(M, v)
        err = [abs(sum(B[j] * A[i][j] for j in range(deg)) - f[i]) for i in range(npts)]
        tot = sum(lw[i] * err[i] for i in range(npts))
        lw = [lw[i] * err[i] / tot for i in range(npts)]
    return [B[j] for j in range(deg)], max(err)


def evaluate(Bd, r):
    def fma(a, b, c):
        return float(mp.mpf(a) * mp.mpf(b) + mp.mpf(c))
    acc = Bd[-1]
    for c in reversed(Bd[:-1]):
        acc = fma(r, acc, c)
    return float(mp.mpf(r) * mp.mpf(acc))  # q = r * (...), one rounding


def fit_sq(A, bits=13, npts=4001):
    """Minimax by linear programming (scipy HiGHS) on a uniform grid of [-1/2, 1/2]: the
    relative error is linear in (C, C*D); solved as corrections to Taylor's (C, C*D) scaled by
    1e-14 so the LP sees O(1) numbers (the header's kSqC / kSqBeta come from this)."""
    from scipy.optimize import linprog
    mp.mp.dps = 40
    N = mp.mpf(2) ** bits
    h = mp.log(2) / N
    A = mp.mpf(A)
    xs = [mp.mpf(-0.5) + mp.mpf(i) / (npts - 1) for i in range(npts)]
    fs = [mp.power(2, x / N) for x in xs]
    x10 = h / (2 * A)
    a1 = np.array([float(x10 * (x * x + 2 * A * x) / fv) for x, fv in zip(xs, fs)])
    a2 = np.array([float(1 / fv) for fv in fs])
    e0 = np.array([float(x10 * (x * x + 2 * A * x) / fv + 1 / fv - 1) for x, fv in zip(xs, fs)])
    S = 1e-14
    one = np.ones_like(a1)
    res = linprog([0, 0, 1], A_ub=np.vstack([np.c_[a1, a2, -one], np.c_[-a1, -a2, -one]]),
                  b_ub=np.r_[-e0 / S, e0 / S], bounds=[(None, None)] * 3, method="highs")
    d1, d2, t = res.x
    C = x10 * (1 + mp.mpf(d1) * S)
    beta = (1 + mp.mpf(d2) * S) / C - A * A
    return C, beta, t * S


def main_sq(A):
    C, beta, e = fit_sq(A)
    print(f"A = {A}: minimax relative error ~ {mp.nstr(e, 5)}")
    print(f"  kSqC    = {mp.nstr(C, 20)}L")
    print(f"  kSqBeta = {mp.nstr(beta, 20)}")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--sq":
        return main_sq(int(sys.argv[2]) if len(sys.argv) > 2 else 11819)
    bits = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    deg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    B, e = fit(bits, deg)
    Bd = [float(b) for b in B]
    print(f"bits {bits} deg {deg}: minimax |dq| ~ {mp.nstr(e, 5)} = {float(e) / 2**-53:.3f} half-ulps of 1")
    for j, c in enumerate(Bd):
        print(f"  B{j + 1} = {c.hex()}  ({c!r})")
    rng = np.random.default_rng(0)
    N = mp.mpf(2) ** bits
    worst = 0.0
    for r in np.concatenate([rng.uniform(-0.5, 0.5, 4000), [-0.5, 0.5, 0.0]]):
        q = evaluate(Bd, float(r))
        worst = max(worst, abs(float(mp.mpf(q) - (mp.power(2, mp.mpf(float(r)) / N) - 1))))
    print(f"  double evaluation worst |dq| {worst:.3e} = {worst / 2**-53:.3f} half-ulps of 1")


if __name__ == "__main__":
    main()
