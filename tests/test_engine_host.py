"""Host-side logic of engine.py that needs no GPU: the ODE launch order (wave_order), which
puts points with equal stage keys next to each other so that whole wavefronts qualify for the
integrator's cooperative mode."""
import numpy as np
import torch

from conftest import BASE_CFG, full_cfg, pkg


def _recs(cfgs):
    cfgm = pkg("config")
    return (np.concatenate([cfgm.to_point(c) for c in cfgs]), np.concatenate([cfgm.to_ode_params(c) for c in cfgs]))


def _order(p, o):
    """engine.wave_order on CPU byte tensors of the records, as a numpy permutation (or None)."""
    tp = torch.from_numpy(np.ascontiguousarray(p).view(np.uint8).copy())
    to = torch.from_numpy(np.ascontiguousarray(o).view(np.uint8).copy())
    r = pkg("engine").wave_order(tp, to, p.size)
    return None if r is None else r.numpy()


def _cfgs(m_values, reps, rng):
    out = []
    for m in m_values:
        for _ in range(reps):
            c = full_cfg(BASE_CFG)
            c.update(m_chi_GeV=float(m), P_chi_to_B=float(rng.uniform(0.1, 1.0)),
                     sigma_v_chi_GeV_m2=float(rng.choice([0.0, 1e-16])), Gamma_wash_over_H=1.0)
            out.append(c)
    return out


def test_wave_order_groups_interleaved_points():
    rng = np.random.default_rng(3)
    grouped = _cfgs([0.95, 40.0, 300.0], 100, rng)
    p, o = _recs(grouped)
    assert _order(p, o) is None                      # already contiguous
    perm = rng.permutation(len(grouped))
    order = _order(p[perm], o[perm])
    assert order is not None and sorted(order.tolist()) == list(range(len(grouped)))
    m = p[perm]["m_chi_GeV"][order]
    assert int(np.count_nonzero(m[1:] != m[:-1])) == 2  # three contiguous groups
    # stable within a group: the original relative order is kept
    for val in (0.95, 40.0, 300.0):
        idx = order[m == val]
        assert np.all(np.diff(idx) > 0)


def test_wave_order_no_repeats_or_small():
    rng = np.random.default_rng(4)
    distinct = _cfgs(np.linspace(1.0, 2.0, 200), 1, rng)
    p, o = _recs(distinct)
    assert _order(p, o) is None                      # nothing to group
    small = _cfgs([0.95, 40.0], 20, rng)
    p, o = _recs(small)
    assert _order(p[::-1], o[::-1]) is None          # <= 64 points: one wavefront anyway
    # the deplete flag is part of the key (it selects the Y_chi-only stage function)
    cfgs = _cfgs([0.95], 200, rng)
    for i, c in enumerate(cfgs):
        c["deplete_DM_from_source"] = bool(i % 2)
    p, o = _recs(cfgs)
    order = _order(p, o)
    d = o["deplete_DM_from_source"][order]
    assert int(np.count_nonzero(d[1:] != d[:-1])) == 1
