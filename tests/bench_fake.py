"""A CPU stand-in for the HIP engine behind bench.py (tests/test_bench_roofline.py only): the
dense sweep writes the C oracle's rows of the C2 grid, the secondary modes (truncation, z-sum
reuse) write NaN rows, so the evidence checks pass only if they look at the dense timed table.

    python tests/bench_fake.py <bench args>                          # one process
    python -m torch.distributed.run --nproc-per-node 2 ... tests/bench_fake.py <bench args>
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class FakeEngine:
    # the stand-in claims one device per rank, so bench.py's duplicate-device check applies to it
    # as to RCCL ranks; FAKE_DUP_DEVICE=1 makes every rank report device 0
    exclusive_devices = True

    def __init__(self, bad_dense_row: int | None = None):
        self.device = torch.device("cpu")
        self.truncate = False
        self.bad = bad_dense_row
        self._cache = {}

    def device_identity(self, rank: int, local: int) -> dict:
        dev = 0 if os.environ.get("FAKE_DUP_DEVICE") else local
        return {"device_index": dev, "pci_bus_id": f"0000:{0x11 + dev:02x}:00", "uuid": f"fake-gpu-{dev}"}

    def tune_truncate(self, on: bool) -> bool:
        prev, self.truncate = self.truncate, bool(on)
        return prev

    def sweep(self, base, axes, start, count, out=None, reuse=False, **kw):
        import bench
        from oracle import oracle as O
        if reuse or self.truncate:
            out.fill_(float("nan"))
            return out
        key = (start, count)
        if key not in self._cache:
            rows = O.points_batch([bench.grid_config(axes, start + i, O) for i in range(count)])
            if self.bad is not None:
                rows[self.bad, 0] *= 1.0 + 1e-6
            self._cache[key] = torch.from_numpy(rows)
        out.copy_(self._cache[key])
        return out


if __name__ == "__main__":
    import bench
    bad = os.environ.get("FAKE_BAD_ROW")
    sys.exit(bench.main(sys.argv[1:], engine=FakeEngine(None if bad is None else int(bad))))
