"""Pin the CPU oracle (oracle/lzq_oracle.c) against the reference's own outputs.

tests/golden/*.json were produced by tests/golden/make_golden.py running
/root/reference/first_principles_yields.py itself (545 main() runs, A/V at 84 y-values for
4 kernels, the plug-in closed form at 25 lambdas).  The oracle restates the reference with
libm exp/pow instead of numpy's AVX-512 ones, so agreement is ~1e-13, not bitwise.
"""
import numpy as np
import pytest

from conftest import BASE_CFG, full_cfg, golden, rel_err
from oracle import oracle as O

TOL_POINTS = 1e-12   # measured worst 1.2e-13
TOL_AOV = 1e-11      # measured worst 5.3e-13 (tiny A/V values)


def test_numpy_primitives_bit_exact():
    rng = np.random.default_rng(7)
    for n in (1, 5, 8, 9, 100, 128, 129, 1199, 7999, 8192, 8193, 20000):
        a = rng.uniform(0, 1, n) * np.exp(rng.uniform(-30, 0, n))
        assert O.pairwise_sum(a) == np.add.reduce(a), n
    for a, b, n in ((0.0, 30.0, 1200), (-48.0, 50.0, 8000), (-80.0, 11.7, 8000), (-3.3, 1.7, 2000)):
        assert np.array_equal(O.linspace(a, b, n), np.linspace(a, b, n))


def test_golden_points():
    d = golden("golden_points.json")["points"]
    assert not any("error" in r for r in d)
    tab = O.points_batch([full_cfg(r["config"]) for r in d], nthreads=8)
    worst = 0.0
    for row, r in zip(tab, d):
        o = dict(zip(O.YIELD_FIELDS, row))
        for k, v in r["final"].items():
            worst = max(worst, rel_err(o[k], v))
        assert o["P_used"] == r["P_used"]
    assert worst < TOL_POINTS, worst


def test_c1_published_numbers():
    o = O.point_yields(full_cfg(BASE_CFG))
    assert rel_err(o["Y_B"], 8.720885362714675e-11) < 1e-13
    assert rel_err(o["DM_over_B"], 5.688926334903014) < 1e-13
    assert f"{o['Y_B']:.10e}" == "8.7208853627e-11"       # PAPER p.6 eq.(19)
    assert f"{o['DM_over_B']:.10f}" == "5.6889263349"     # PAPER p.6 eq.(21)


def test_golden_aov():
    for case in golden("golden_aov.json"):
        kw = case["kernel"]
        for y, ref in zip(case["y"], case["aov"]):
            got = O.aov(kw["I_p"], kw["beta_over_H"], kw["T_p"], kw["v_w"], kw["g_star"], y)
            assert rel_err(got, ref) < TOL_AOV, (kw, y, got, ref)


def test_golden_lz_closed_form_bit_exact():
    d = golden("golden_lz.json")
    for lam_s, P in zip(d["lambda"], d["P"]):
        assert O.p_closed_form(float(lam_s)) == P, lam_s


def test_batch_matches_single():
    d = golden("golden_points.json")["points"][:24]
    cfgs = [full_cfg(r["config"]) for r in d]
    tab = O.points_batch(cfgs, nthreads=4)
    for row, c in zip(tab, cfgs):
        o = O.point_yields(c)
        assert list(row) == [o[k] for k in O.YIELD_FIELDS]


def test_regime_auto_is_an_error():
    with pytest.raises(UnboundLocalError):
        O.point_yields(full_cfg({**BASE_CFG, "regime": "auto"}))


def test_oracle_under_asan_ubsan():
    """The CPU restatement built with -fsanitize=address,undefined (oracle/asan_driver.c,
    `make -C oracle asan-check`): quadrature, closed form, ODE paths run clean."""
    import os
    import subprocess
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    subprocess.run(["make", "-s", "-C", here, "asan-check"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(here, "_build", "asan_driver")], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, (r.stdout, r.stderr[-3000:])
    assert "ok (0 failures)" in r.stdout
