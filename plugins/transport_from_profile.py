"""transport_from_profile -- the LZ plug-in module the reference's hook looks for
(fpy:170-187 imports `lambda_local_LZ_from_profile`, `extended_LZ_lambda`,
`transport_from_profile` in that order; PAPER p.5 §6.1 and App. A name this one: "computes
P_chi->B from a bounce profile CSV using the minimal LZ estimator").

Put this directory on sys.path (PYTHONPATH=plugins) and run the reference, or lzq's own
driver, with `--maybe-compute-P-from-profile profile.csv`: the hook calls
compute_prob_from_profile(csv, v_w).  Every number is computed on the MI355X through the C ABI
(lzq_binding, no torch).  The upstream module is absent from the reference, so its CSV format is
unknown and parity against it is UNPINNED; this module implements the paper's definition
(PAPER p.3 §3, eqs.(5)-(9)) and reads three documented formats (comma separated, one header
row, '#' lines are comments, `# key = value` comment lines set options):

  bounce profile  header  xi,phi,Phi  (or r,phi,Phi with `# R0 = ...`: xi = r - R0, §3.1)
                  the bounce solution's background fields phi(xi), Phi(xi) (case matters:
                  phi and Phi are different columns), "interpolated as smooth functions":
                  not-a-knot cubic splines (scipy CubicSpline's interpolant, as fpy:212).
                  Options y_B, y_chi, lambda_tr_eff (required):
                    Delta(xi) = y_B phi - y_chi Phi            eq.(5), crossings Delta(xi*) = 0
                    Delta'*   = y_B phi'(xi*) - y_chi Phi'(xi*) eq.(6)
                    m_mix(xi) = lambda_tr_eff phi(xi)          eq.(7)
                    delta_LZ  = m_mix(xi*)^2 / (2 v_w |Delta'*|) eq.(8), F(k) = 1
  sampled levels  header  xi,Delta,m_mix: Delta(xi) and m_mix(xi) sampled directly (the same
                  splines, with phi = m_mix, Phi = -Delta, y_B = 0, y_chi = 1, lambda = 1)
  crossing list   header  xi,m_mix,dprime: one row per crossing (xi increasing, |Delta'|)

  estimator (option):
    auto      (default) one crossing: the minimal estimator, P = 1 - exp(-2 pi delta_LZ)
              (eq.(9), fpy:183-184); several: `propagate` for profiles, `linear` for lists
    minimal   eq.(9) of the single crossing (an error if there are several)
    propagate the time-ordered propagation through the whole profile, i dpsi/dt = H psi,
              H = Delta(xi) sz + m_mix(xi) sx, xi = v_w t (lzq_lz_propagate_profile): the
              crossings' energy dependence and their interference are kept
    linear    each crossing linearised (Delta' and m_mix at xi*), coherent through the
              piecewise-linear model (lzq_lz_propagate); window_lz (20), steps (1000)
  steps_per_radian (4), min_steps (1): the profile propagator's step control.
  v_w: only for compute_lambda_eff_from_profile, whose signature has no v_w.

Command line (PAPER App. A): python transport_from_profile.py --params transport_params.json
with {"profile_csv": ..., "v_w": ..., and any option above}; prints the crossings and P.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:   # lzq_binding lives next to this module
    sys.path.insert(0, _HERE)
import lzq_binding  # noqa: E402

DEFAULTS = {"window_lz": 20.0, "steps": 1000.0, "steps_per_radian": 4.0, "min_steps": 1.0, "estimator": "auto",
            "R0": 0.0}
ESTIMATORS = ("auto", "minimal", "propagate", "linear")


def _opt_value(v: str):
    try:
        return float(v)
    except ValueError:
        return v


def read_csv(path: str):
    """-> (header cells as written, float rows, options)."""
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
                    opts[k] = _opt_value(v)
                continue
            cells = [c.strip() for c in line.split(",")]
            if header is None:
                header = cells
                continue
            rows.append([float(c) for c in cells])
    if header is None or not rows:
        raise ValueError(f"{path}: no header / no data rows")
    return header, rows, opts


class Profile:
    """A parsed profile CSV: either fields (knots + phi, Phi + couplings) or a crossing list."""

    def __init__(self, path: str, overrides: dict | None = None):
        header, rows, opts = read_csv(path)
        opts.update(overrides or {})
        self.path, self.opts = path, opts
        if opts["estimator"] not in ESTIMATORS:
            raise ValueError(f"{path}: estimator must be one of {ESTIMATORS}")
        col = {h: i for i, h in enumerate(header)}
        low = {h.lower(): i for i, h in enumerate(header)}
        self.fields = None
        if "phi" in col and "Phi" in col and ("xi" in low or "r" in low):
            pos = [r[low["xi"]] for r in rows] if "xi" in low else [r[low["r"]] - float(opts["R0"]) for r in rows]
            for k in ("y_B", "y_chi", "lambda_tr_eff"):
                if not isinstance(opts.get(k), float):
                    raise ValueError(f"{path}: a phi/Phi profile needs a '# {k} = ...' line (PAPER eqs.(5),(7))")
            self.fields = (pos, [r[col["phi"]] for r in rows], [r[col["Phi"]] for r in rows],
                           opts["y_B"], opts["y_chi"], opts["lambda_tr_eff"])
        elif {"xi", "delta", "m_mix"} <= set(low):
            self.fields = ([r[low["xi"]] for r in rows], [r[low["m_mix"]] for r in rows],
                           [-r[low["delta"]] for r in rows], 0.0, 1.0, 1.0)
        elif {"xi", "m_mix", "dprime"} <= set(low):
            self.xs = [r[low["xi"]] for r in rows]
            self.ms = [r[low["m_mix"]] for r in rows]
            self.ds = [abs(r[low["dprime"]]) for r in rows]
            if any(b <= a for a, b in zip(self.xs, self.xs[1:])):
                raise ValueError(f"{path}: crossings must have increasing xi")
        else:
            raise ValueError(f"{path}: header must be 'xi,phi,Phi', 'r,phi,Phi', 'xi,Delta,m_mix' or "
                             f"'xi,m_mix,dprime', got {header}")
        if self.fields is not None and len(self.fields[0]) < 4:
            raise ValueError(f"{path}: a sampled profile needs at least 4 rows")

    def crossings(self, v_w: float):
        """[(xi*, |Delta'*|, m_mix(xi*), delta_LZ)] (eqs.(5)-(8))."""
        if self.fields is None:
            return [(x, d, m, m * m / (2.0 * max(v_w, 1e-12) * d)) for x, m, d in zip(self.xs, self.ms, self.ds)]
        return [(x, abs(d), m, l) for x, d, m, l in lzq_binding.profile_crossings(*self.fields, v_w)]

    def probability(self, v_w: float) -> float:
        est = self.opts["estimator"]
        cr = self.crossings(v_w)
        if not cr:
            raise ValueError(f"{self.path}: no avoided crossing (Delta never changes sign)")
        if est == "auto":
            est = "minimal" if len(cr) == 1 else ("linear" if self.fields is None else "propagate")
        if est == "minimal":
            if len(cr) != 1:
                raise ValueError(f"{self.path}: the minimal estimator takes one crossing, found {len(cr)}")
            return lzq_binding.p_closed_form([cr[0][3]])[0]                 # eq.(9), fpy:183-184
        if est == "propagate":
            if self.fields is None:
                raise ValueError(f"{self.path}: estimator 'propagate' needs a sampled profile")
            return lzq_binding.lz_propagate_profile(*self.fields, v_w, self.opts["steps_per_radian"],
                                                    int(self.opts["min_steps"]))
        xs, ds, ms = [c[0] for c in cr], [c[1] for c in cr], [c[2] for c in cr]
        if any(not (d > 0) for d in ds):
            raise ValueError(f"{self.path}: |Delta'| must be > 0 at every crossing")
        return lzq_binding.lz_propagate(ms, ds, xs, float(v_w), self.opts["window_lz"], int(self.opts["steps"]))


def read_profile(path: str, v_w: float = 1.0):
    """-> (xi*, m_mix*, |Delta'*|) crossing lists and the options (the crossing geometry does not
    depend on v_w; only delta_LZ does)."""
    p = Profile(path)
    cr = p.crossings(v_w)
    return [c[0] for c in cr], [c[2] for c in cr], [c[1] for c in cr], p.opts


def compute_prob_from_profile(profile_csv_path: str, v_w: float) -> float:
    """The hook's first choice (fpy:178-180): P_chi->B of the profile (estimator above)."""
    return Profile(profile_csv_path).probability(float(v_w))


def compute_lambda_eff_from_profile(profile_csv_path: str) -> float:
    """lambda_eff with 1 - exp(-2 pi lambda_eff) = P (fpy:181-184).  One crossing: delta_LZ of
    PAPER eq.(8) exactly; several: -ln(1 - P)/(2 pi) of the estimator's P.  Needs `# v_w = ...`."""
    p = Profile(profile_csv_path)
    if not isinstance(p.opts.get("v_w"), float):
        raise ValueError(f"{profile_csv_path}: compute_lambda_eff_from_profile needs a '# v_w = ...' line")
    v_w = p.opts["v_w"]
    cr = p.crossings(v_w)
    if len(cr) == 1 and p.opts["estimator"] in ("auto", "minimal"):
        return cr[0][3]
    P = p.probability(v_w)
    return -math.log1p(-P) / (2.0 * math.pi) if P < 1.0 else math.inf


def main(argv=None) -> int:
    """python transport_from_profile.py --params transport_params.json (PAPER App. A)."""
    ap = argparse.ArgumentParser(description="P_chi->B from a bounce-profile CSV (PAPER eqs.(5)-(9)) on the MI355X")
    ap.add_argument("--params", required=True, help="JSON: profile_csv, v_w, and optional CSV options")
    ap.add_argument("--out", default=None, help="also write the result as JSON here")
    a = ap.parse_args(argv)
    with open(a.params) as f:
        prm = json.load(f)
    csv = prm.pop("profile_csv")
    if not os.path.isabs(csv):
        csv = os.path.join(os.path.dirname(os.path.abspath(a.params)), csv)
    v_w = float(prm.pop("v_w"))
    p = Profile(csv, {k: (float(v) if isinstance(v, (int, float)) else v) for k, v in prm.items()})
    cr = p.crossings(v_w)
    P = p.probability(v_w)
    for i, (x, d, m, l) in enumerate(cr):
        print(f"crossing {i}: xi* = {x:.10g}  |Delta'*| = {d:.10g}  m_mix = {m:.10g}  delta_LZ = {l:.10g}")
    print(f"P_chi_to_B = {P!r}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"P_chi_to_B": P, "v_w": v_w, "estimator": p.opts["estimator"],
                       "crossings": [dict(zip(("xi", "dprime_abs", "m_mix", "delta_LZ"), c)) for c in cr]}, f,
                      indent=2)
    return 0


if __name__ == "__main__":
    sys.exit(main())
