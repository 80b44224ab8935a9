"""transport_from_profile -- the LZ plug-in module the reference's hook looks for
(fpy:170-187 imports `lambda_local_LZ_from_profile`, `extended_LZ_lambda`,
`transport_from_profile` in that order; PAPER p.5 §6.1 and App. A name this one).

Put this directory on sys.path (PYTHONPATH=plugins) and run the reference, or lzq's own
driver, with `--maybe-compute-P-from-profile profile.csv`: the hook calls
compute_prob_from_profile(csv, v_w), which returns the coherent conversion probability of
the profile's crossings from the MI355X propagator (lzq_lz_propagate, via lzq_binding).

The upstream modules are absent from the reference, so their CSV format is unknown; this
module reads two documented formats (comma separated, one header row, '#' lines are comments;
`# key = value` comment lines set options):

  crossing list   header  xi,m_mix,dprime          one row per avoided crossing: position xi_c
                                                   (increasing), coupling m_mix(xi_c) and slope
                                                   |Delta'(xi_c)| (sign ignored; slopes alternate)
  bounce profile  header  xi,Delta,m_mix           samples of the detuning Delta(xi) and the
                                                   coupling m_mix(xi) along the wall coordinate
                                                   (PAPER p.3 eqs.(5)-(7)); crossings are the sign
                                                   changes of Delta (linear interpolation), with
                                                   |Delta'| the secant slope of the bracketing
                                                   samples and m_mix interpolated at xi_c

  options: window_lz (default 20: outer half-window in LZ lengths), steps (default 1000:
  Magnus steps per crossing, the floor), v_w (only for compute_lambda_eff_from_profile,
  whose signature has no v_w).

For one crossing the propagator reproduces the closed form 1 - exp(-2 pi delta),
delta = m_mix^2 / (2 v_w |Delta'|) (PAPER eqs.(8)-(9), fpy:183-184), to <= 1e-8 relative.
"""
from __future__ import annotations

import math
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:   # lzq_binding lives next to this module
    sys.path.insert(0, _HERE)
import lzq_binding  # noqa: E402

DEFAULTS = {"window_lz": 20.0, "steps": 1000.0}


def read_profile(path: str):
    """-> (xi, m_mix, dprime) crossing lists and the `# key = value` options."""
    opts = dict(DEFAULTS)
    header, rows = None, []
    with open(path) as f:
        for raw in f:
            line = raw.strip()
            if not line:
                continue
            if line.startswith("#"):
                body = line.lstrip("#").strip()
                if "=" in body:
                    k, v = (s.strip() for s in body.split("=", 1))
                    try:
                        opts[k] = float(v)
                    except ValueError:
                        pass
                continue
            cells = [c.strip() for c in line.split(",")]
            if header is None:
                header = [c.lower() for c in cells]
                continue
            rows.append([float(c) for c in cells])
    if header is None or not rows:
        raise ValueError(f"{path}: no header / no data rows")
    col = {h: i for i, h in enumerate(header)}
    if {"xi", "m_mix", "dprime"} <= set(col):
        xs = [r[col["xi"]] for r in rows]
        ms = [r[col["m_mix"]] for r in rows]
        ds = [abs(r[col["dprime"]]) for r in rows]
    elif {"xi", "delta", "m_mix"} <= set(col):
        xs, ms, ds = crossings_from_samples([r[col["xi"]] for r in rows], [r[col["delta"]] for r in rows],
                                            [r[col["m_mix"]] for r in rows])
    else:
        raise ValueError(f"{path}: header must be 'xi,m_mix,dprime' or 'xi,Delta,m_mix', got {header}")
    if not xs:
        raise ValueError(f"{path}: no avoided crossing (Delta never changes sign)")
    if any(b <= a for a, b in zip(xs, xs[1:])):
        raise ValueError(f"{path}: crossings must have increasing xi")
    if any(not (d > 0) for d in ds):
        raise ValueError(f"{path}: |Delta'| must be > 0 at every crossing")
    return xs, ms, ds, opts


def crossings_from_samples(xi, Delta, m_mix):
    """Zero crossings of a sampled Delta(xi): (xi_c, m_mix(xi_c), |Delta'(xi_c)|)."""
    if any(b <= a for a, b in zip(xi, xi[1:])):
        raise ValueError("profile xi must be strictly increasing")
    xs, ms, ds = [], [], []
    n = len(xi)
    for i in range(n - 1):
        a, b = Delta[i], Delta[i + 1]
        if a == 0.0 and 0 < i and Delta[i - 1] * b < 0:          # a sample exactly on the crossing
            xs.append(xi[i])
            ms.append(m_mix[i])
            ds.append(abs((b - Delta[i - 1]) / (xi[i + 1] - xi[i - 1])))
        elif a * b < 0:
            t = a / (a - b)
            xs.append(xi[i] + t * (xi[i + 1] - xi[i]))
            ms.append(m_mix[i] + t * (m_mix[i + 1] - m_mix[i]))
            ds.append(abs((b - a) / (xi[i + 1] - xi[i])))
    return xs, ms, ds


def compute_prob_from_profile(profile_csv_path: str, v_w: float) -> float:
    """The hook's first choice (fpy:178-180): coherent P through all crossings (GPU)."""
    xs, ms, ds, o = read_profile(profile_csv_path)
    return lzq_binding.lz_propagate(ms, ds, xs, float(v_w), o["window_lz"], int(o["steps"]))


def compute_lambda_eff_from_profile(profile_csv_path: str) -> float:
    """lambda_eff with 1 - exp(-2 pi lambda_eff) = P (fpy:181-184).  One crossing: delta of
    PAPER eq.(8) exactly; several: -ln(1 - P_coherent)/(2 pi).  Needs `# v_w = ...`."""
    xs, ms, ds, o = read_profile(profile_csv_path)
    if "v_w" not in o:
        raise ValueError(f"{profile_csv_path}: compute_lambda_eff_from_profile needs a '# v_w = ...' line")
    v_w = o["v_w"]
    if len(xs) == 1:
        return ms[0] * ms[0] / (2.0 * max(v_w, 1e-12) * ds[0])
    P = lzq_binding.lz_propagate(ms, ds, xs, v_w, o["window_lz"], int(o["steps"]))
    return -math.log1p(-P) / (2.0 * math.pi) if P < 1.0 else math.inf
