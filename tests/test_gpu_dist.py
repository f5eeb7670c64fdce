"""Multi-rank round pipeline on real HIP kernels: two ranks share the box's one GPU
(``DBA_SHARE_GPU=1``) with gloo collectives standing in for RCCL (which refuses two ranks on
one device).  Exercises LPT placement, early local tests on the owner rank, image-sharded
global tests, the snapshot all-gather and the counter all-reduce exactly as the 8-GPU run
does, and checks the world-2 metrics against a world-1 run of the same rounds (exactly)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT
from dba_mod_amd.tools.dist_check import free_port

pytestmark = pytest.mark.gpu

ARGS = ["--config", os.path.join(ROOT, "configs", "mnist_params.yaml"), "--pretrain-rounds", "3", "--steps", "2",
        "--warmup", "1", "--set", "synthetic_train_size=6000", "synthetic_test_size=1000", "eval_batch_size=500"]


def _bench(cmd, extra_env):
    env = dict(os.environ, PYTHONPATH=ROOT, **extra_env)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_two_ranks_share_one_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    one = _bench([sys.executable, "bench.py", *ARGS], {})
    two = _bench([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                  "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", *ARGS],
                 {"DBA_SHARE_GPU": "1", "DBA_DIST_BACKEND": "gloo"})
    assert one["ops_backend"] == two["ops_backend"] == "hip"
    assert two["n_gpus"] == 2 and len(two["rounds"]) == 2
    # fp32 (default) kernels are deterministic and their split factors depend on the
    # per-replica geometry only, so placing the round's clients on two ranks (5 + 5 instead
    # of 10 per launch) changes no bits: the world-2 round metrics equal world 1's exactly
    assert one["dtype"] == two["dtype"] == "fp32"
    for (e1, a1, s1), (e2, a2, s2) in zip(one["rounds"], two["rounds"]):
        assert (e1, a1, s1) == (e2, a2, s2)
