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
#include <string.h>
#include "lzq_exp2.h"
extern "C" void ev(const double* c2, const double* g, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = lzq::exp2_nonpos(c2[i], g[i]);
}
extern "C" void pv(const double* r, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = lzq::exp2_poly(r[i]);
}
static double tab[lzq::kTabN];
extern "C" void evt(const double* c2, const double* g, long n, double* out) {
  for (int j = 0; j < lzq::kTabN; ++j) {
    uint64_t b = lzq::tab_entry_bits(lzq::tab_exact(j), j);
    memcpy(&tab[j], &b, 8);
  }
  // the kernel multiplies the 2^512-scaled value by omega' = omega * 2^-512 in one fma; here
  // omega = 1, i.e. one rounding of v * 2^-512 (exact unless the result is subnormal)
  for (long i = 0; i < n; ++i)
    out[i] = ldexp(lzq::exp2_tab_scaled(c2[i] * lzq::kTabN, g[i], tab), -lzq::kOmegaBias);
}
'''


def _build(defines=()):
    d = tempfile.mkdtemp()
    src = os.path.join(d, "t.cpp")
    with open(src, "w") as f:
        f.write(SRC)
    so = os.path.join(d, "t.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                    *[f"-D{k}={v}" for k, v in defines],
                    "-I", os.path.join(ROOT, PKG_NAME, "csrc"), src, "-o", so], check=True)
    L = ctypes.CDLL(so)
    for fn in (L.ev, L.pv, L.evt):
        fn.restype = None
    return L


@pytest.fixture(scope="module")
def lib():
    return _build()


# (table bits, polynomial degree) -> minimax |dq| of tools/exp2_tab_poly.py (Taylor for (8, 4))
# (13, 2) is the completed-square form C*((r + A)^2 + beta) with integer A (LZQ_SQFORM, the
# default: one VALU fewer per node); (13, 2, 0) the plain r*(B1 + r*B2) form it replaced.
DEFAULT_TAB = (13, 2)  # LZQ_TABBITS / LZQ_POLYDEG defaults in lzq_exp2.h
TAB_VARIANTS = {(8, 4): 1.9e-17, (10, 3): 9.4e-17, (12, 2): 2.53e-14, (12, 3): 3.7e-19, (13, 2): 1.73e-14,
                (13, 2, 0): 3.16e-15, (14, 2): 3.95e-16, (14, 3): 1.5e-21}


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
    poly = TAB_VARIANTS[DEFAULT_TAB] if fn == "evt" else 0.0  # default table variant's |dq|
    tol = exact * (2.5e-16 + poly + u_abs * 2.3e-16) + 2 * 5e-324
    assert np.all(np.abs(got - exact) <= tol), (np.abs(got - exact) / tol).max()
    assert np.all(got[c2 * g <= -1076.0] == 0.0)
    assert np.all(got >= 0.0) and np.all(np.isfinite(got))


@pytest.mark.parametrize("fn", ["ev", "evt"])
def test_exp2_nonpos_zero_gamma(lib, fn):
    # gamma4(z_0) = 0 and c2 from y = 50 (|c2| ~ 4e21): 2^(c2*0) = 1 (exactly for the
    # r*(B1 + r*B2) forms; within the minimax bound for the completed-square table form)
    got = run(lib, [-4.1e21, -1.0], [0.0, 0.0], fn)
    tol = TAB_VARIANTS[DEFAULT_TAB] + 2.3e-16 if fn == "evt" else 0.0
    assert np.all(np.abs(got - 1.0) <= tol), got


@pytest.mark.parametrize("variant", sorted(TAB_VARIANTS))
def test_table_variant_matches_mpmath(variant):
    bits, deg = variant[:2]
    sq = variant[2] if len(variant) > 2 else 1
    L = _build([("LZQ_TABBITS", bits), ("LZQ_POLYDEG", deg), ("LZQ_SQFORM", sq)])
    rng = np.random.default_rng(5)
    u = -np.concatenate([rng.uniform(0, 60, 3000), 10 ** rng.uniform(-15, 0, 1000)])
    g = np.ones_like(u)
    got = run(L, u, g, "evt")
    worst = max(abs(float((mp.mpf(o) - mp.power(2, mp.mpf(x))) / mp.power(2, mp.mpf(x)))) for o, x in zip(got, u))
    # polynomial error + rounding of T[j] (1/2 ulp) + the final fma (1/2 ulp) + q's own rounding
    assert worst < TAB_VARIANTS[variant] + 2.3e-16, worst
