"""Multi-process rehearsal of the distributed round (gloo on CPU, or RCCL on GPUs).

Used by tests/test_distributed.py:  python -m dba_mod_amd.tools.dist_check is not needed —
tests call :func:`run_world` which spawns ``world`` ranks over 127.0.0.1.
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
        torch.save({"state": s.global_state.cpu(), "acc": [r.get("global_acc") for r in summ],
                    "asr": [r.get("global_asr") for r in summ]}, os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        shutdown(dctx)


def run_world(world: int, outdir: str, cfg: str, over: Dict[str, Any], rounds: List[int]) -> List[Dict[str, Any]]:
    os.makedirs(outdir, exist_ok=True)
    port = free_port()
    if world == 1:
        _worker(0, 1, port, outdir, cfg, over, rounds)
    else:
        mp.spawn(_worker, args=(world, port, outdir, cfg, over, rounds), nprocs=world, join=True)
    return [torch.load(os.path.join(outdir, f"rank{r}.pt"), weights_only=True) for r in range(world)]
