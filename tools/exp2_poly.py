#!/usr/bin/env python3
"""Derive the FP64 polynomial p(r) ~= 2**r on r in [-1/2, 1/2] used by the quadrature
kernel's exp (csrc/lzq_exp2.h).  p(r) = 1 + r*q(r); q is fitted to (2**r - 1)/r with a
weighted discrete Remez (Lawson) iteration in mpmath at 60 digits, then rounded to double.
Prints the coefficients as C hex-floats and the measured error of the double-precision
Horner evaluation (with fma) against mpmath on 2e4 random points.

    python tools/exp2_poly.py [degree]
"""
import sys
import mpmath as mp
import numpy as np

mp.mp.dps = 60
DEG = int(sys.argv[1]) if len(sys.argv) > 1 else 11   # degree of p; q has degree DEG-1
LN2 = mp.log(2)


def g(r):
    return (mp.power(2, r) - 1) / r if r != 0 else LN2


def fit(deg_q, npts=400, iters=60):
    # Chebyshev-distributed sample points on [-1/2, 1/2] (avoid r = 0 exactly)
    xs = [mp.mpf(0.5) * mp.cos(mp.pi * (i + mp.mpf(0.5)) / npts) for i in range(npts)]
    w = [abs(x) / mp.power(2, x) for x in xs]          # relative-error weight of p
    lw = [mp.mpf(1)] * npts                            # Lawson weights
    A = [[x ** j for j in range(deg_q + 1)] for x in xs]
    b = [g(x) for x in xs]
    for _ in range(iters):
        # weighted least squares: minimise sum lw * (w*(Aq - b))^2
        M = mp.matrix(deg_q + 1, deg_q + 1)
        v = mp.matrix(deg_q + 1, 1)
        for i in range(npts):
            s = lw[i] * w[i] ** 2
            for a in range(deg_q + 1):
                v[a] += s * A[i][a] * b[i]
                for c in range(deg_q + 1):
                    M[a, c] += s * A[i][a] * A[i][c]
        q = mp.lu_solve(M, v)
        err = [abs(w[i] * (sum(q[j] * A[i][j] for j in range(deg_q + 1)) - b[i])) for i in range(npts)]
        tot = sum(lw[i] * err[i] for i in range(npts))
        lw = [lw[i] * err[i] / tot for i in range(npts)]
    return [q[j] for j in range(deg_q + 1)], max(err)


def main():
    q, e = fit(DEG - 1)
    qd = [float(c) for c in q]
    print(f"degree {DEG}: mp minimax rel err ~ {mp.nstr(e, 5)}")
    for j, c in enumerate(qd):
        print(f"  a{j + 1} = {c.hex()}  ({c!r})")
    rng = np.random.default_rng(0)
    rs = np.concatenate([rng.uniform(-0.5, 0.5, 20000), [-0.5, 0.5, 0.0, 1e-300, -1e-17]])
    worst = 0.0

    def fma(a, b, c):  # correctly rounded fused multiply-add via 60-digit mpmath
        return float(mp.mpf(a) * mp.mpf(b) + mp.mpf(c))
    for r in rs:
        r = float(r)
        acc = qd[-1]
        for c in reversed(qd[:-1]):
            acc = fma(acc, r, c)
        p = fma(r, acc, 1.0)
        exact = mp.power(2, mp.mpf(float(r)))
        rel = abs((mp.mpf(p) - exact) / exact)
        worst = max(worst, float(rel))
    print(f"  double-Horner worst rel err {worst:.3e} = {worst / 2**-53:.2f} half-ulps")


if __name__ == "__main__":
    main()
