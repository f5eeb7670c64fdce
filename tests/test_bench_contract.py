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
    # per-round pacing: one positive interval per timed round, summing to the timed window
    rm = out["round_ms"]
    assert len(rm) == 2 and all(v > 0 for v in rm)
    assert sum(rm) <= out["ms_per_step"] * 2 * 1.05


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


def test_bench_self_spawn_world4_cpu():
    """``python bench.py --cpu --gpus 4`` with NO launcher: the parent spawns 4 fresh ranks
    (gloo), relays rank 0's line, and the result equals the world-1 run round for round."""
    out = _run([sys.executable, "bench.py", "--gpus", "4", *SMALL], timeout=900)
    _check(out, 4)
    assert out["world"] == 4 and out["dist_backend"] == "gloo" and out["emulated"] is False
    assert out["collective_selfcheck_ok"] is True and out["rccl_ok"] is None
    assert len(out["devices"]) == 4
    assert out["comm_bytes_per_round"].get("all_reduce", 0) > 0
    one = _run([sys.executable, "bench.py", *SMALL])
    assert one["world"] == 1 and one["dist_backend"] == "none" and one["comm_bytes_per_round"] == {}
    assert out["rounds"] == one["rounds"]


def test_bench_launcher_world_mismatch_fails():
    """Under a launcher, --gpus must equal WORLD_SIZE (no silent one-GPU run)."""
    env = dict(os.environ, PYTHONPATH=ROOT, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", *SMALL], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_bench_emulated_rank_cpu():
    """--emulate-rank R --emulate-world N: one process runs rank R's share; collectives are
    counted no-ops (the bytes of the real N-rank run are still reported)."""
    out = _run([sys.executable, "bench.py", "--emulate-rank", "1", "--emulate-world", "4", *SMALL])
    assert out["emulated"] is True and out["world"] == 4 and out["n_gpus"] == 1
    assert out["dist_backend"] == "emulated"
    assert out["config"]["parallelism"] == "emulated rank 1 of client-dp4"
    assert out["comm_bytes_per_round"].get("all_reduce", 0) > 0
