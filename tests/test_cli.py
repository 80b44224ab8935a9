"""Driver behaviour that needs no GPU, against the reference's own recorded CLI output
(tests/golden/golden_cli.json): missing --config, --write-template bytes, regime 'auto',
unknown keys, the config schema and the plug-in hook's module order."""
import contextlib
import io
import json
import os
import sys
import types

import pytest

from conftest import golden, pkg


def cli_case(name):
    return next(c for c in golden("golden_cli.json") if c["name"] == name)


def run_cli(argv, cwd):
    old = os.getcwd()
    buf = io.StringIO()
    try:
        os.chdir(cwd)
        with contextlib.redirect_stdout(buf):
            pkg("cli").main(argv)
    finally:
        os.chdir(old)
    return buf.getvalue()


def test_no_config(tmp_path):
    assert run_cli([], tmp_path) == cli_case("no_config")["stdout"]


def test_write_template_bytes(tmp_path):
    c = cli_case("write_template")
    out = run_cli(["--write-template", "--config", "tmpl.json"], tmp_path)
    assert out == c["stdout"]
    assert (tmp_path / "tmpl.json").read_text() == c["template_text"]


def test_regime_auto_raises_like_reference(tmp_path):
    c = cli_case("regime_auto")
    (tmp_path / "auto.json").write_text(c["config_text"])
    with pytest.raises(UnboundLocalError) as ei:
        run_cli(["--config", "auto.json"], tmp_path)
    assert str(ei.value) in c["stderr_last_line"]


def test_unknown_key_typeerror(tmp_path):
    (tmp_path / "bad.json").write_text(json.dumps({"not_a_field": 1}))
    with pytest.raises(TypeError):
        pkg("config").load_config(str(tmp_path / "bad.json"))


def test_ode_fallback_configs_need_the_gpu(tmp_path):
    """ODE configs (fpy:385-410) go to the GPU like the fast path: no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present (covered by tests/test_gpu_cli.py)")
    (tmp_path / "ode.json").write_text(json.dumps({"P_chi_to_B": 0.1, "Gamma_wash_over_H": 1e-3}))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        run_cli(["--config", "ode.json"], tmp_path)


def test_config_schema_order_matches_reference_dump():
    """yields_out.json 'inputs' = cfg.__dict__ + P_used in dataclass order (fpy:424)."""
    ref = json.loads(cli_case("equal_mass")["yields_out_json"])
    cfgm = pkg("config")
    path = os.path.join(os.path.dirname(__file__), "_tmp_cfg.json")
    try:
        with open(path, "w") as f:
            f.write(cli_case("equal_mass")["config_text"])
        cfg = cfgm.load_config(path)
    finally:
        os.remove(path)
    ours = {**cfg.__dict__, "P_used": cfg.P_chi_to_B}
    assert list(ours) == list(ref["inputs"]) and ours == ref["inputs"]


def test_plugin_hook_order_and_swallowing(monkeypatch):
    lz = pkg("lz")
    a = types.ModuleType("extended_LZ_lambda")
    a.compute_prob_from_profile = lambda path, v_w: 1.7       # clamped to 1.0
    b = types.ModuleType("transport_from_profile")
    b.compute_prob_from_profile = lambda path, v_w: 0.25
    monkeypatch.setitem(sys.modules, "extended_LZ_lambda", a)
    monkeypatch.setitem(sys.modules, "transport_from_profile", b)
    assert lz.try_compute_P_from_profile("x.csv", 0.3) == 1.0    # earlier module wins
    a.compute_prob_from_profile = lambda path, v_w: 1 / 0         # raises -> None
    assert lz.try_compute_P_from_profile("x.csv", 0.3) is None
    monkeypatch.delitem(sys.modules, "extended_LZ_lambda")
    monkeypatch.setitem(sys.modules, "extended_LZ_lambda", None)  # import fails -> skipped
    assert lz.try_compute_P_from_profile("x.csv", 0.3) == 0.25


def test_maybe_P_messages(capsys):
    lz = pkg("lz")
    cfg = pkg("config").Config(P_chi_to_B=0.2)
    assert lz.maybe_P(cfg, None) == 0.2
    assert lz.maybe_P(cfg, "missing.csv") == 0.2
    assert capsys.readouterr().out == "[warn] Could not compute P from profile automatically; falling back to config.\n"
    with pytest.raises(RuntimeError, match="P_chi_to_B is not set"):
        lz.maybe_P(pkg("config").Config(), None)


def test_incoherent_composition():
    lz = pkg("lz")
    assert lz.p_incoherent([0.3]) == pytest.approx(0.3)
    assert lz.p_incoherent([0.5, 0.2, 0.9]) == pytest.approx(0.5)
    assert lz.p_incoherent([1.0, 1.0]) == pytest.approx(0.0)


def test_plugin_profile_formats(tmp_path):
    """plugins/transport_from_profile.py parses its documented CSV formats (host logic; the
    splines, crossings and propagation are tests/test_gpu_plugin.py)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "tfp_cpu", os.path.join(os.path.dirname(os.path.dirname(__file__)), "plugins", "transport_from_profile.py"))
    tfp = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tfp)
    (tmp_path / "a.csv").write_text("# window_lz = 30\n# v_w = 0.3\nxi,m_mix,dprime\n0,0.1,-1.0\n50,0.2,2.0\n")
    xs, ms, ds, o = tfp.read_profile(str(tmp_path / "a.csv"))
    assert xs == [0.0, 50.0] and ms == [0.1, 0.2] and ds == [1.0, 2.0]
    assert o["window_lz"] == 30.0 and o["v_w"] == 0.3 and o["steps"] == 1000.0
    # the sampled formats' crossings come from the GPU splines (tests/test_gpu_plugin.py); their
    # header / size / option errors are caught on the host
    (tmp_path / "p.csv").write_text("xi,phi,Phi\n0,1,0\n1,1,1\n2,1,2\n3,1,3\n")
    with pytest.raises(ValueError, match="y_B"):
        tfp.read_profile(str(tmp_path / "p.csv"))
    (tmp_path / "e.csv").write_text("# estimator = bogus\nxi,m_mix,dprime\n0,0.1,1\n")
    with pytest.raises(ValueError, match="estimator"):
        tfp.read_profile(str(tmp_path / "e.csv"))
    for bad in ("xi,foo\n1,2\n", "xi,m_mix,dprime\n", "xi,m_mix,dprime\n1,0.1,1\n0,0.1,1\n",
                "xi,Delta,m_mix\n0,1,0.1\n1,2,0.1\n"):
        (tmp_path / "bad.csv").write_text(bad)
        with pytest.raises(ValueError):
            tfp.read_profile(str(tmp_path / "bad.csv"))


def test_hook_does_not_mask_library_failures(monkeypatch, tmp_path):
    """lz.py: a plug-in's own exception is swallowed (fpy:186-187), but a failure of lzq's
    closed form (the HIP library) propagates instead of a silent fallback to the config P."""
    lz = pkg("lz")
    stub = types.ModuleType("lambda_local_LZ_from_profile")
    stub.compute_lambda_eff_from_profile = lambda path: 0.01
    monkeypatch.setitem(sys.modules, "lambda_local_LZ_from_profile", stub)

    def broken(lam):
        raise pkg("_native").LzqError(-2, "simulated HIP failure")
    monkeypatch.setattr(lz, "p_closed_form", broken)
    with pytest.raises(RuntimeError, match="simulated HIP failure"):
        lz.try_compute_P_from_profile("x.csv", 0.3)
    stub.compute_lambda_eff_from_profile = lambda path: 1 / 0
    assert lz.try_compute_P_from_profile("x.csv", 0.3) is None


def test_boltzmann_scalar_wrappers():
    """BoltzmannSystem.H / .s (fpy:203-204) exist with the reference's formulas (fpy:84-88)."""
    import math
    B = pkg("boltzmann")
    cfg = pkg("config").Config(P_chi_to_B=0.1)
    bs = B.BoltzmannSystem.__new__(B.BoltzmannSystem)   # no GPU: only the scalar wrappers
    bs.cfg = cfg
    assert bs.H(100.0) == 1.66 * math.sqrt(cfg.g_star) * 100.0 * 100.0 / 1.220890e19
    assert bs.s(100.0) == (2.0 * math.pi ** 2 / 45.0) * cfg.g_star_s * 100.0 ** 3
