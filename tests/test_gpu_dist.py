"""Multi-rank round pipeline on real HIP kernels: two ranks share the box's one GPU
(``DBA_SHARE_GPU=1``) with gloo collectives standing in for RCCL (which refuses two ranks on
one device).  Exercises LPT placement, early local tests on the owner rank, image-sharded
global tests with owner broadcasts of the sharded clients' snapshots, the reduction-based
aggregations (fp64 FedAvg delta all-reduce, distributed Weiszfeld, FoolsGold feature +
weighted-sum all-reduces) and the counter all-reduce exactly as the 8-GPU run does, and checks
the world-2 run against a world-1 run of the same rounds: FedAvg's global model BITWISE (its
hash) and every round's metrics; RFA / FoolsGold add fp64 rank partial sums in a world-dependent
order (tests/test_distributed.py) and round once to fp32, so their models agree to within an
occasional last-bit difference.  Also the launch forms the round driver uses for the scaling bench:
``python bench.py --gpus N`` (self-spawn) and a --gpus / WORLD_SIZE mismatch."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT
from dba_mod_amd.tools.dist_check import free_port

pytestmark = pytest.mark.gpu

MNIST = ["--config", os.path.join(ROOT, "configs", "mnist_params.yaml"), "--pretrain-rounds", "3", "--steps", "2",
         "--warmup", "1", "--set", "synthetic_train_size=6000", "synthetic_test_size=1000", "eval_batch_size=500"]
# the flagship CIFAR ResNet-18 path (fused training BN, split-K, solo tail), small synthetic sets;
# rounds 202 (benign) and 203 (attacker 17, model replacement)
CIFAR = ["--config", os.path.join(ROOT, "configs", "cifar_params.yaml"), "--pretrain-rounds", "1", "--steps", "2",
         "--warmup", "1", "--start-epoch", "201", "--set", "synthetic_train_size=8000", "synthetic_test_size=1000",
         "eval_batch_size=500"]
SHARED = {"DBA_SHARE_GPU": "1", "DBA_DIST_BACKEND": "gloo"}


def _bench(cmd, extra_env, expect_ok=True):
    env = dict(os.environ, PYTHONPATH=ROOT, **extra_env)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    if not expect_ok:
        return r
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _torchrun(n, args):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(n), *args]


def _same(one, two):
    assert one["ops_backend"] == two["ops_backend"] == "hip"
    assert two["world"] == 2 and two["n_gpus"] == 2 and len(two["rounds"]) == len(one["rounds"])
    # fp32 kernels are deterministic and every summation-order decision follows the per-replica
    # geometry (split-K, fused BN groups), so placing the round's clients on two ranks changes
    # no bit: the world-2 global model and round metrics equal world 1's exactly
    assert one["dtype"] == two["dtype"] == "fp32"
    assert one["rounds"] == two["rounds"]
    assert one["state_sha"] == two["state_sha"]


def test_two_ranks_share_one_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    one = _bench([sys.executable, "bench.py", *MNIST], {})
    two = _bench(_torchrun(2, MNIST), SHARED)
    _same(one, two)


@pytest.mark.parametrize("agg,extra", [("mean", []), ("geom_median", ["rfa_mode=distributed"]), ("foolsgold", [])])
def test_cifar_world2(tmp_path, agg, extra):
    """The flagship CIFAR ResNet-18 rounds (fused training BN, attacker 17's model replacement)
    at world 2 (gloo on the shared GPU) vs world 1: bitwise for every aggregation — FedAvg's
    fp64 delta sums, and the distributed RFA / FoolsGold weighted sums through the exact
    fixed-point limb all-reduce (fl/aggregate.py fixed_exponent)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    args = CIFAR + extra + ["--aggregation", agg]
    one = _bench([sys.executable, "bench.py", *args, "--dump-state", str(tmp_path / "w1.pt")], {})
    two = _bench(_torchrun(2, args) + ["--dump-state", str(tmp_path / "w2.pt")], SHARED)
    _same(one, two)
    assert two["world"] == 2 and one["dtype"] == two["dtype"] == "fp32"
    s1 = torch.load(tmp_path / "w1.pt", weights_only=True)
    s2 = torch.load(tmp_path / "w2.pt", weights_only=True)
    assert torch.equal(s1, s2)


def test_self_spawn_bench_world2():
    """``python bench.py --gpus 2`` (no launcher: the driver's scaling form) spawns two ranks,
    exits 0, reports world 2 and the same rounds as world 1."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    one = _bench([sys.executable, "bench.py", *MNIST], {})
    two = _bench([sys.executable, "bench.py", "--gpus", "2", *MNIST], SHARED)
    _same(one, two)


def test_gpus_world_size_mismatch_fails():
    """Launched with WORLD_SIZE 2 but --gpus 1: every rank refuses (non-zero exit, no JSON)."""
    cmd = _torchrun(2, MNIST)
    cmd[cmd.index("--gpus") + 1] = "1"
    r = _bench(cmd, SHARED, expect_ok=False)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
