"""The inner-loop exponential lzq::exp2_nonpos (csrc/lzq_exp2.h), compiled for the HOST
with g++ and checked against mpmath.  Its device form uses only correctly-rounded IEEE
operations (v_mul/v_fma/v_rndne/v_ldexp_f64) plus the saturating v_cvt_i32_f64 that the
host build emulates, so this pins the arithmetic the GPU executes."""
import ctypes
import os
import subprocess
import tempfile

import mpmath as mp

mp.mp.dps = 40
import numpy as np
import pytest

from conftest import ROOT, PKG_NAME

SRC = r'''
#include <math.h>
#include "lzq_exp2.h"
extern "C" void ev(const double* c2, const double* g, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = lzq::exp2_nonpos(c2[i], g[i]);
}
extern "C" void pv(const double* r, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = lzq::exp2_poly(r[i]);
}
static double tab[lzq::kTabN];
extern "C" void evt(const double* c2, const double* g, long n, double* out) {
  for (int j = 0; j < lzq::kTabN; ++j) tab[j] = (double)exp2l((long double)j / (long double)lzq::kTabN);
  for (long i = 0; i < n; ++i) out[i] = lzq::exp2_nonpos_tab(c2[i] * lzq::kTabN, g[i], tab);
}
'''


@pytest.fixture(scope="module")
def lib():
    d = tempfile.mkdtemp()
    src = os.path.join(d, "t.cpp")
    with open(src, "w") as f:
        f.write(SRC)
    so = os.path.join(d, "t.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                    "-I", os.path.join(ROOT, PKG_NAME, "csrc"), src, "-o", so], check=True)
    L = ctypes.CDLL(so)
    for fn in (L.ev, L.pv, L.evt):
        fn.restype = None
    return L


def run(L, c2, g, fn="ev"):
    c2 = np.ascontiguousarray(c2, float)
    g = np.ascontiguousarray(g, float)
    out = np.empty_like(c2)
    P = ctypes.POINTER(ctypes.c_double)
    getattr(L, fn)(c2.ctypes.data_as(P), g.ctypes.data_as(P), c2.size, out.ctypes.data_as(P))
    return out


def test_poly_accuracy(lib):
    rng = np.random.default_rng(3)
    r = np.concatenate([rng.uniform(-0.5, 0.5, 3000), [-0.5, 0.5, 0.0]])
    out = np.empty_like(r)
    P = ctypes.POINTER(ctypes.c_double)
    lib.pv(r.ctypes.data_as(P), r.size, out.ctypes.data_as(P))
    worst = max(abs(float((mp.mpf(o) - mp.power(2, mp.mpf(x))) / mp.power(2, mp.mpf(x)))) for o, x in zip(out, r))
    assert worst < 1.5e-16, worst  # <= 0.7 ulp


@pytest.mark.parametrize("fn", ["ev", "evt"])
def test_exp2_nonpos_range(lib, fn):
    rng = np.random.default_rng(4)
    u = -np.concatenate([10 ** rng.uniform(-20, 3.1, 20000), [0.0, 1e-300, 0.5, 1.5, 1021.5, 1022.0, 1074.0, 1074.5,
                                                            1075.0, 1080.0, 2 ** 31 + 0.5, 1e15, 1e22]])
    g = rng.uniform(0.1, 8.0, u.size)
    c2 = u / g
    got = run(lib, c2, g, fn)
    exact = np.exp2(c2 * g)  # libm exp2 of the rounded product (<= 0.5 ulp + product rounding)
    # tolerance: 1 ulp of the polynomial + |u| ulps from rounding the product inside exp2(c2*g)
    # (relative), plus 2 subnormal ulps of absolute slack for gradual underflow
    u_abs = np.abs(c2 * g)
    tol = exact * (2.5e-16 + u_abs * 2.3e-16) + 2 * 5e-324
    assert np.all(np.abs(got - exact) <= tol), (np.abs(got - exact) / tol).max()
    assert np.all(got[c2 * g <= -1076.0] == 0.0)
    assert np.all(got >= 0.0) and np.all(np.isfinite(got))


@pytest.mark.parametrize("fn", ["ev", "evt"])
def test_exp2_nonpos_zero_gamma(lib, fn):
    # gamma4(z_0) = 0 and c2 from y = 50 (|c2| ~ 4e21): 2^(c2*0) = 1
    assert run(lib, [-4.1e21, -1.0], [0.0, 0.0], fn).tolist() == [1.0, 1.0]


def test_table_variant_matches_mpmath(lib):
    rng = np.random.default_rng(5)
    u = -np.concatenate([rng.uniform(0, 60, 3000), 10 ** rng.uniform(-15, 0, 1000)])
    g = np.ones_like(u)
    got = run(lib, u, g, "evt")
    worst = max(abs(float((mp.mpf(o) - mp.power(2, mp.mpf(x))) / mp.power(2, mp.mpf(x)))) for o, x in zip(got, u))
    assert worst < 2.25e-16, worst  # <= 1 ulp (T[j] and the final fma each round once; measured 0.89)
