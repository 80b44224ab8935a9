#!/usr/bin/env python3
"""Golden fixtures for the LZ plug-in path of the reference CLI (fpy:170-187, 317-328):
`--maybe-compute-P-from-profile` with stub plug-in modules on PYTHONPATH, run through the
REFERENCE itself (build container only; the reference never travels to the GPU box).

Each case records the stub module (our own few lines, not reference code), the reference's
stdout bytes and yields_out.json; tests/test_gpu_cli.py re-creates the same stub for lzq's
driver and compares bytes.  -> tests/golden/golden_cli_profile.json

    python tests/golden/make_golden_profile.py
"""
import json
import os
import subprocess
import sys
import tempfile

REF_DIR = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

CASES = [
    # (name, module name, module source)
    ("prob_stub", "transport_from_profile",
     "def compute_prob_from_profile(path, v_w):\n    return 0.2113 + 0.0 * v_w\n"),
    ("prob_clamped", "transport_from_profile",
     "def compute_prob_from_profile(path, v_w):\n    return 1.7\n"),
    ("lambda_stub", "extended_LZ_lambda",
     "def compute_lambda_eff_from_profile(path):\n    return 0.025726891712928787\n"),
    ("lambda_wins_order", "extended_LZ_lambda+transport_from_profile",
     "def compute_lambda_eff_from_profile(path):\n    return 0.5\n"
     "###\n"
     "def compute_prob_from_profile(path, v_w):\n    return 0.9\n"),
    ("plugin_raises", "transport_from_profile",
     "def compute_prob_from_profile(path, v_w):\n    raise ValueError('bad profile')\n"),
]


def main():
    cases = []
    for name, mods, src in CASES:
        with tempfile.TemporaryDirectory() as d:
            plug = os.path.join(d, "plug")
            os.makedirs(plug)
            for mod, body in zip(mods.split("+"), src.split("###\n")):
                with open(os.path.join(plug, mod + ".py"), "w") as f:
                    f.write(body)
            with open(os.path.join(d, "bounce.csv"), "w") as f:
                f.write("xi,m_mix,dprime\n0.0,0.1,1.0\n")
            env = dict(os.environ, PYTHONPATH=plug, PYTHONDONTWRITEBYTECODE="1")
            r = subprocess.run([sys.executable, "-B", os.path.join(REF_DIR, "first_principles_yields.py"),
                                "--config", os.path.join(REF_DIR, "yields_config_equal_mass.json"),
                                "--maybe-compute-P-from-profile", "bounce.csv"],
                               cwd=d, env=env, capture_output=True, text=True)
            assert r.returncode == 0, r.stderr
            with open(os.path.join(d, "yields_out.json")) as f:
                yo = f.read()
        cases.append({"name": name, "modules": mods.split("+"), "module_sources": src.split("###\n"),
                      "flags": ["--maybe-compute-P-from-profile", "bounce.csv"],
                      "config": "yields_config_equal_mass.json", "stdout": r.stdout, "yields_out_json": yo})
    with open(os.path.join(HERE, "golden_cli_profile.json"), "w") as f:
        json.dump(cases, f, indent=1)
    for c in cases:
        print(c["name"], c["stdout"].splitlines()[0])


if __name__ == "__main__":
    main()
