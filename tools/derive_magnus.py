#!/usr/bin/env python3
"""Symbolic derivation of the Magnus vector used by csrc/lzq_propagator.hip.

H(t) = m sx + (D + Dd t) sz on a step t in [-h/2, h/2] (D at the midpoint, Dd = dD/dt).  The
Dyson series of U is built to h^8, then the SU(2) logarithm U = exp(-i n.sigma) is taken as a
series: sin|n| n_hat = i tr(U sigma)/2 and |n|/sin|n| = asin(sqrt x)/sqrt x with x = sin^2|n|.
Prints the coefficients of n_x, n_y, n_z by power of h (odd powers only: the step is
time-symmetric).  Takes ~1 minute.
"""
import sympy as sp

ORDER = 9  # keep h^0 .. h^8


def main():
    m, D, Dd, h, t, tp = sp.symbols("m D Dd h t tp", real=True)
    I = sp.I
    sx = sp.Matrix([[0, 1], [1, 0]])
    sy = sp.Matrix([[0, -I], [I, 0]])
    sz = sp.Matrix([[1, 0], [0, -1]])
    E2 = sp.eye(2)

    def trunc_poly(e):
        p = sp.Poly(sp.expand(e), h)
        return sum(c * h ** k[0] for k, c in zip(p.monoms(), p.coeffs()) if k[0] < ORDER)

    def H(tt):  # time in units of the step: s = h * tt
        return m * sx + (D + Dd * h * tt) * sz

    # U(tt) = 1 + h int_{-1/2}^{tt} (-i H) U, iterated to order h^8
    U = E2
    for _ in range(ORDER):
        integrand = (-I * H(tp) * U.subs(t, tp)) * h
        Un = E2 + integrand.applyfunc(lambda e: sp.integrate(sp.expand(e), (tp, -sp.Rational(1, 2), t)))
        U = Un.applyfunc(trunc_poly)
    U1 = U.subs(t, sp.Rational(1, 2)).applyfunc(sp.expand)
    v = [sp.expand(I * (U1 * s).trace() / 2) for s in (sx, sy, sz)]  # sin|n| n_hat
    x = trunc_poly(sum(vi * vi for vi in v))                            # sin^2|n|
    X = sp.symbols("X")
    f = sp.series(sp.asin(sp.sqrt(X)) / sp.sqrt(X), X, 0, 5).removeO()
    fx = trunc_poly(f.subs(X, x))
    for k, vk in zip("xyz", v):
        p = sp.Poly(trunc_poly(sp.expand(vk * fx)), h)
        print("n_" + k)
        for (deg,), c in sorted(zip(p.monoms(), p.coeffs())):
            print("  h^%d:" % deg, sp.factor(c))


if __name__ == "__main__":
    main()
