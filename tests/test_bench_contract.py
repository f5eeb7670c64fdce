"""The driver's bench.py contract, rehearsed on CPU: one JSON line from rank 0 with the
required keys, K timed steps, and the multi-rank launch the driver uses
(``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1``),
here with the gloo backend and world sizes 2 and 8."""
import json
import os
import subprocess
import sys

from conftest import ROOT
from dba_mod_amd.tools.dist_check import free_port

SMALL = ["--cpu", "--config", os.path.join(ROOT, "configs", "mnist_params.yaml"), "--pretrain-rounds", "1",
         "--steps", "2", "--warmup", "1", "--set", "synthetic_train_size=3000", "synthetic_test_size=400",
         "eval_batch_size=200"]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(cmd, timeout=600):
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]       # exactly one JSON line (rank 0)
    return json.loads(lines[0])


def _check(out, n):
    assert KEYS <= set(out), KEYS - set(out)
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == 1
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["higher_is_better"] is True
    assert out["config"]["parallelism"] == f"client-dp{n}"
    assert len(out["rounds"]) == 2


def test_bench_world1_cpu():
    _check(_run([sys.executable, "bench.py", *SMALL]), 1)


def test_bench_torchrun_world2_cpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", *SMALL]
    _check(_run(cmd), 2)


def test_bench_torchrun_world8_cpu():
    """The driver's N=8 launch shape, rehearsed with 8 gloo ranks on the CPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "8", *SMALL]
    _check(_run(cmd, timeout=900), 8)
