"""The drop-in CLI on the GPU vs the reference's recorded output (golden_cli.json): stdout
byte-identical; yields_out.json identical in structure and inputs, finals within 1e-11."""
import json

import pytest

from conftest import golden, rel_err
from test_cli import run_cli

pytestmark = pytest.mark.gpu
CASES = [c for c in golden("golden_cli.json") if c["yields_out_json"] is not None or c["name"] == "profile_fallback"]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"] + "".join(c["flags"]))
def test_cli_matches_reference(case, tmp_path, gpu_engine):
    if case["config_text"] is not None:
        (tmp_path / "cfg.json").write_text(case["config_text"])
        argv = ["--config", "cfg.json"] + case["flags"]
    else:  # the shipped config (run.txt) with extra flags
        (tmp_path / "cfg.json").write_text(next(c for c in golden("golden_cli.json")
                                                if c["name"] == "equal_mass")["config_text"])
        argv = ["--config", "cfg.json"] + case["flags"]
    out = run_cli(argv, tmp_path)
    assert out == case["stdout"]
    if case["yields_out_json"] is None:
        return
    ref = json.loads(case["yields_out_json"])
    ours = json.loads((tmp_path / "yields_out.json").read_text())
    assert ours["inputs"] == ref["inputs"]
    assert list(ours["final"]) == list(ref["final"])
    for k, v in ref["final"].items():
        assert rel_err(ours["final"][k], v) < 1e-11, (k, ours["final"][k], v)


@pytest.mark.parametrize("case", golden("golden_cli_ode.json"), ids=lambda c: c["name"])
def test_cli_ode_path_matches_reference(case, tmp_path, gpu_engine):
    """sigma_v / Gamma_wash / depletion configs: the CLI takes the GPU ODE fallback (fpy:385-410);
    stdout byte-identical, finals within 1e-10 of the reference's Radau."""
    (tmp_path / "cfg.json").write_text(case["config_text"])
    assert run_cli(["--config", "cfg.json"], tmp_path) == case["stdout"]
    ref = json.loads(case["yields_out_json"])
    ours = json.loads((tmp_path / "yields_out.json").read_text())
    assert ours["inputs"] == ref["inputs"]
    for k, v in ref["final"].items():
        assert rel_err(ours["final"][k], v) < 1e-10, (k, ours["final"][k], v)
