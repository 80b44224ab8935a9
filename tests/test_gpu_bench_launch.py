"""bench.py --gpus N on a box with fewer GPUs: the self-launched ranks refuse
to run RCCL ranks without their GPUs, the command exits non-zero and no line -- in particular no
n_gpus = 1 line -- is printed.  Needs the GPU box (one MI355X); the ranks exit before any HIP
initialisation."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_gpus_beyond_the_node_exit_nonzero():
    n = torch.cuda.device_count()
    if n >= 2:
        pytest.skip("this check is for a box with fewer GPUs than --gpus")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode != 0, r.stderr[-2000:]
    assert not lines, lines
    assert "needs 2 GPUs" in r.stderr, r.stderr[-2000:]
