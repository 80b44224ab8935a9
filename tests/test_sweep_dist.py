"""Sweep driver host logic on CPU: sharding, gloo all-gather at world_size 2, 3, 4 and 8 (even and
uneven shards, the gather's chunked rounds), chunk
checkpoints and resume, spec decoding.  The per-point compute is replaced by a
deterministic function of the global flat index, so any sharding / ordering / gather bug
shows up as a wrong row (the GPU compute itself is covered by tests/test_gpu_*.py)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import pkg


def fake_compute(start, n, out):
    idx = torch.arange(start, start + n, dtype=torch.float64)
    out.copy_(torch.stack([idx * k + 0.25 for k in range(1, 7)], dim=1))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, chunk, out_dir, res_path, rows_per_round=1 << 18):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sw = pkg("sweep")
    s, e = sw.shard_range(total, rank, world)
    local = sw.run_local(fake_compute, s, e, lambda n: torch.empty((n, 6), dtype=torch.float64), chunk, out_dir)
    table = sw.gather_table(local, total, rank, world, rows_per_round=rows_per_round)
    # every rank holds the whole table
    np.save(res_path + f".{rank}.npy", table.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total,chunk,rounds", [
    (2, 1001, 97, 1 << 18), (3, 20, 4, 1 << 18), (3, 2, 1, 1 << 18),      # total < world: empty shards
    (4, 100_003, 8192, 7_000),         # uneven (25001 / 25000 rows), several gather rounds
    (8, 100_003, 4096, 1 << 18),       # uneven at the C4 world size
    (8, 80_000, 4096, 1 << 18)])       # equal shards (C4's case): one direct all_gather_into_tensor
def test_gloo_gather_matches_single_rank(world, total, chunk, rounds):
    sw = pkg("sweep")
    ref = torch.empty((total, 6), dtype=torch.float64)
    fake_compute(0, total, ref)
    with tempfile.TemporaryDirectory() as d:
        res = os.path.join(d, "res")
        mp.spawn(_worker, args=(world, free_port(), total, chunk, d, res, rounds), nprocs=world, join=True)
        for r in range(world):
            assert np.array_equal(np.load(res + f".{r}.npy"), ref.numpy()), r
        # every chunk of every shard was checkpointed
        files = sorted(f for f in os.listdir(d) if f.startswith("shard_"))
        covered = sum(int(f.split("_")[2].split(".")[0]) for f in files)
        assert covered == total
        # resume: nothing is recomputed
        def boom(*a):
            raise AssertionError("recomputed a checkpointed chunk")
        for r in range(world):
            s, e = sw.shard_range(total, r, world)
            loc = sw.run_local(boom, s, e, lambda n: torch.empty((n, 6), dtype=torch.float64), chunk, d,
                               resume=True)
            assert np.array_equal(loc.numpy(), ref.numpy()[s:e])


def test_shard_ranges_partition():
    sw = pkg("sweep")
    for total in (1, 7, 10**6, 10**8 + 3):
        for world in (1, 2, 3, 4, 8):
            r = [sw.shard_range(total, k, world) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == total
            assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))
            sizes = [b - a for a, b in r]
            assert max(sizes) - min(sizes) <= 1


def test_builtin_specs_match_survey_grids():
    specs = pkg("sweep").builtin_specs()
    assert specs["C2"].total == 10**6 and specs["C3"].total == 10**7 and specs["C4"].total == 10**8
    c2 = specs["C2"]
    p = c2.point_params(1234)
    assert p["m_mix"] == np.logspace(-3, 0, 1000)[1] and p["dprime"] == np.logspace(-3, 1, 1000)[234]


def test_spec_json_roundtrip():
    sw = pkg("sweep")
    spec = sw.spec_from_json({"name": "t", "base": {"I_p": 0.5},
                              "axes": [{"field": "m_chi_GeV", "logspace": [0, 1, 3]},
                                       {"field": "delta_LZ", "values": [1e-3, 1e-2]}]})
    assert spec.total == 6 and spec.base["I_p"] == 0.5
    again = sw.spec_from_json(spec.to_json())
    assert again.total == 6 and np.array_equal(again.axes[0][1], spec.axes[0][1])
    with pytest.raises(ValueError):
        sw.spec_from_json({"axes": [{"field": "nope", "values": [1]}]})
    # ode_max_steps: 0 and null both mean "no cap" (as --ode-max-steps 0 does), < 0 is refused
    ax = [{"field": "I_p", "values": [0.3]}]
    for ms, want in ((0, None), (None, None), (5000, 5000)):
        assert sw.spec_from_json({"axes": ax, "ode_max_steps": ms}).ode_max_steps == want, ms
    assert sw.spec_from_json({"axes": ax}).ode_max_steps == sw.ODE_MAX_STEPS
    with pytest.raises(ValueError):
        sw.spec_from_json({"axes": ax, "ode_max_steps": -1})


def test_summary_fixed_order():
    sw = pkg("sweep")
    spec = sw.builtin_specs()["C2"]
    t = np.random.default_rng(0).uniform(0, 10, (1000, 6))
    s1 = sw.summarize(t, spec)
    s2 = sw.summarize(t.copy(), spec)
    assert s1 == s2 and set(s1["final"]) == set(pkg("_native").YIELD_FIELDS)


def test_out_dir_manifest_and_foreign_resume(tmp_path):
    """--out is created if missing; shard names carry the sweep's key; --resume into a
    directory written by another sweep definition refuses instead of mixing tables."""
    sw = pkg("sweep")
    specs = sw.builtin_specs()
    out = tmp_path / "new" / "dir"
    k2 = sw.prepare_out_dir(str(out), specs["C2"], resume=False)
    assert (out / "manifest.json").exists() and len(k2) == 16
    assert sw.prepare_out_dir(str(out), specs["C2"], resume=True) == k2   # same sweep: fine
    with pytest.raises(RuntimeError, match="another sweep"):
        sw.prepare_out_dir(str(out), specs["C3"], resume=True)
    # the key depends on everything a shard's rows depend on
    c2b = sw.SweepSpec("C2", dict(specs["C2"].base, I_p=0.5), specs["C2"].axes)
    assert sw.spec_key(c2b) != k2 and sw.spec_key(specs["C5"]) != k2
    assert sw.spec_key(sw.SweepSpec("C2", specs["C2"].base, specs["C2"].axes, notes="x")) == k2
    # shards of one key are invisible to a run with another key
    loc = sw.run_local(fake_compute, 0, 10, lambda n: torch.empty((n, 6), dtype=torch.float64), 4, str(out), key=k2)
    names = sorted(os.listdir(out))
    assert all(n.startswith(f"shard_{k2}_") for n in names if n.startswith("shard_"))

    def boom(*a):
        raise AssertionError("recomputed")
    again = sw.run_local(boom, 0, 10, lambda n: torch.empty((n, 6), dtype=torch.float64), 4, str(out),
                         resume=True, key=k2)
    assert torch.equal(again, loc)
    seen = []
    sw.run_local(lambda s, n, o: (seen.append(s), fake_compute(s, n, o)), 0, 10,
                 lambda n: torch.empty((n, 6), dtype=torch.float64), 4, str(out), resume=True, key="other")
    assert seen == [0, 4, 8]


def test_spec_ode_method_roundtrip():
    sw = pkg("sweep")
    d = {"name": "w", "ode_method": "quadrature",
         "axes": [{"field": "Gamma_wash_over_H", "values": [0.5, 1.0]}]}
    spec = sw.spec_from_json(d)
    assert spec.ode_method == "quadrature" and sw.is_ode_spec(spec)
    again = sw.spec_from_json(spec.to_json())
    assert again.ode_method == "quadrature"
    assert sw.spec_key(again) != sw.spec_key(sw.spec_from_json({**d, "ode_method": "radau"}))
    with pytest.raises(ValueError):
        sw.spec_from_json({**d, "ode_method": "rk4"})


def test_profile_spec_json_and_axis_mapping():
    """A profile sweep (P from a bounce profile, PAPER eqs.(5)-(9)): JSON round trip, coupling axes
    ride on P_chi_to_B for the grid kernel (overridden per point), and their names are rejected
    without a 'profile' section."""
    sw = pkg("sweep")
    d = {"name": "prof", "profile": {"estimator": "propagate", "y_chi": 1.2},
         "axes": [{"field": "y_B", "linspace": [0.5, 2.0, 4]}, {"field": "v_w", "values": [0.2, 0.4]}]}
    spec = sw.spec_from_json(d)
    assert spec.profile.estimator == "propagate" and spec.profile.y_chi == 1.2 and spec.total == 8
    again = sw.spec_from_json(spec.to_json())
    assert again.profile == spec.profile and sw.spec_key(again) == sw.spec_key(spec)
    assert [n for n, _ in sw.grid_axes_for_kernel(spec)] == ["P_chi_to_B", "v_w"]
    assert sw.spec_key(sw.spec_from_json({**d, "profile": {"estimator": "minimal"}})) != sw.spec_key(spec)
    with pytest.raises(ValueError):
        sw.spec_from_json({"axes": [{"field": "y_B", "values": [1.0]}]})
    with pytest.raises(ValueError):
        sw.spec_from_json({**d, "profile": {"estimator": "nope"}})
    p1 = sw.builtin_specs()["P1"]
    assert p1.total == 10**6 and p1.profile is not None
    x, a, b = p1.profile.arrays()
    assert x.shape == a.shape == b.shape and np.all(np.diff(x) > 0)


def test_resumed_ode_status_counts_every_chunk():
    """ODE status counts (summary.json ode_status) after --resume: each checkpointed chunk carries
    its counts in a .status.npy record, so a resumed run reports the same totals as an
    uninterrupted one, not only the chunks it computed itself."""
    sw = pkg("sweep")

    def make():
        counts = np.zeros(8, dtype=np.int64)

        def comp(start, n, out):
            fake_compute(start, n, out)
            chunk = np.zeros(8, dtype=np.int64)
            chunk[0], chunk[3] = n - (start % 3), start % 3     # "ok" and "too_many_steps" per chunk
            counts[:] += chunk
            comp.last_chunk = chunk
        comp.ode_status = counts
        comp.last_chunk = np.zeros(8, dtype=np.int64)
        return comp

    mk = lambda n: torch.empty((n, 6), dtype=torch.float64)
    with tempfile.TemporaryDirectory() as d:
        full = make()
        os.makedirs(os.path.join(d, "a"))
        ref = sw.run_local(full, 0, 1000, mk, 64, os.path.join(d, "a"))
        # an interrupted run: the first 5 chunks only, then a resume over the whole range
        os.makedirs(os.path.join(d, "b"))
        sw.run_local(make(), 0, 320, mk, 64, os.path.join(d, "b"))
        res = make()
        tab = sw.run_local(res, 0, 1000, mk, 64, os.path.join(d, "b"), resume=True)
        assert np.array_equal(tab.numpy(), ref.numpy())
        assert np.array_equal(res.ode_status, full.ode_status) and full.ode_status[3] > 0
        # a checkpoint without its status record is refused, never silently under-counted
        st = [f for f in os.listdir(os.path.join(d, "b")) if f.endswith(".status.npy")]
        os.remove(os.path.join(d, "b", st[0]))
        with pytest.raises(RuntimeError, match="status"):
            sw.run_local(make(), 0, 1000, mk, 64, os.path.join(d, "b"), resume=True)
