"""Multi-process rehearsal of the distributed round (gloo on CPU), and an RCCL self-check.

* :func:`run_world` (tests/test_distributed.py) spawns ``world`` ranks over 127.0.0.1 and runs
  FL rounds; each rank saves its global model, metrics and per-round collective bytes.
* ``python -m torch.distributed.run --nproc-per-node N -m dba_mod_amd.tools.dist_check --rccl``
  on a multi-GPU node: initialises RCCL (backend "nccl" on ROCm), checks an
  ``all_gather_into_tensor`` and a padded / split ``all_reduce`` against their closed forms,
  and times a FedAvg-sized (CIFAR S fp64) all-reduce.  Prints one line per rank.
"""
from __future__ import annotations

import os
import socket
from typing import Any, Dict, List

import torch
import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank: int, world: int, port: int, outdir: str, cfg: str, over: Dict[str, Any], rounds: List[int]) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from .. import config as C
    from ..fl.server import Server
    from ..parallel.dist import init_distributed, shutdown
    dctx = init_distributed(prefer_gpu=False)
    try:
        params = C.load_params(cfg, dict(over))
        s = Server(params, dctx, write_outputs=(rank == 0), folder=os.path.join(outdir, "run") if rank == 0 else None)
        summ = [s.run_round(e) for e in rounds]
        comm = [{k: int(v) for k, v in r.get("comm_bytes", {}).items()} for r in summ]
        torch.save({"state": s.global_state.cpu(), "acc": [r.get("global_acc") for r in summ],
                    "asr": [r.get("global_asr") for r in summ],
                    "comm": [[c.get("all_reduce", 0), c.get("all_gather", 0), c.get("broadcast", 0)] for c in comm],
                    "S": s.spec.S, "n_snapshots": [0]},
                   os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        shutdown(dctx)


def rccl_check(n_elems: int = 2_802_430, reps: int = 10) -> Dict[str, Any]:
    """RCCL self-check of the framework's collectives (run one rank per GPU under torchrun)."""
    import time
    from ..parallel.dist import init_distributed, shutdown
    dctx = init_distributed(prefer_gpu=True)
    out: Dict[str, Any] = {"rank": dctx.rank, "world": dctx.world, "backend": dctx.backend}
    try:
        dev = dctx.device
        W, r = dctx.world, dctx.rank
        rows = torch.full((2, 1000), float(r + 1), device=dev)
        g = dctx.all_gather_rows(rows[:1 + (r % 2)], 2)
        want = torch.cat([torch.full((2, 1000), float(q + 1), device=dev) * torch.tensor(
            [[1.0], [float(q % 2)]], device=dev) for q in range(W)])
        out["all_gather_ok"] = bool(torch.equal(g, want))
        buf = dctx.padded(n_elems, torch.float64)
        buf[:n_elems] = float(r + 1)
        dctx.all_reduce_(buf)
        out["all_reduce_ok"] = bool(torch.all(buf[:n_elems] == W * (W + 1) / 2).item())
        out["padded_elems"] = buf.numel()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dctx.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            dctx.all_reduce_(buf)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / reps
        out["fedavg_allreduce_us"] = round(dt * 1e6, 1)
        out["busbw_GBps"] = round(2 * (W - 1) / W * buf.numel() * 8 / dt / 1e9, 2) if W > 1 else None
    finally:
        shutdown(dctx)
    return out


def run_world(world: int, outdir: str, cfg: str, over: Dict[str, Any], rounds: List[int]) -> List[Dict[str, Any]]:
    os.makedirs(outdir, exist_ok=True)
    port = free_port()
    if world == 1:
        _worker(0, 1, port, outdir, cfg, over, rounds)
    else:
        mp.spawn(_worker, args=(world, port, outdir, cfg, over, rounds), nprocs=world, join=True)
    return [torch.load(os.path.join(outdir, f"rank{r}.pt"), weights_only=True) for r in range(world)]


if __name__ == "__main__":
    import argparse
    import json
    ap = argparse.ArgumentParser()
    ap.add_argument("--rccl", action="store_true", help="collective self-check (torchrun, one rank per GPU)")
    args = ap.parse_args()
    if args.rccl:
        print(json.dumps(rccl_check()), flush=True)
