"""One process per GPU over ``torch.distributed`` (RCCL over xGMI on MI355X, Gloo on CPU).

The reference is single-process/single-GPU with no collective at all.
This framework's distributed round (client-parallel DP):

1. every rank computes the identical round plan (same seeded RNG; no communication);
2. clients are placed on ranks by LPT (:func:`dba_mod_amd.utils.native.lpt_assign`);
3. each rank trains its clients concurrently, then ONE all-gather moves the packed client
   snapshot slots (flat fp32 buckets, one row per snapshot) to every rank — 10 CIFAR
   clients ≈ 112 MB, a fraction of a millisecond of xGMI time;
4. aggregation is applied redundantly on every rank (bit-identical global model, no
   broadcast);
5. a client's local tests run on its owner rank as soon as it finishes training (the longest
   clients' and the global model's tests are image-sharded across ranks); ONE all-reduce of
   the ``[jobs, 3]`` counters combines both.

On a one-GPU box the multi-rank path is rehearsed with ``DBA_SHARE_GPU=1`` (every rank on
device 0) and ``DBA_DIST_BACKEND=gloo`` (``tests/test_gpu_dist.py``).

Bucket policy: payloads are single contiguous flat buffers (never per-layer calls); rows
are padded so every rank contributes the same ``[k_max, S]`` block, which is what RCCL's
``all_gather_into_tensor`` needs.  The int64 BN counters never enter a float bucket.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


@dataclass
class DistCtx:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def enabled(self) -> bool:
        return self.world > 1

    def barrier(self) -> None:
        if self.enabled:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.enabled:
            dist.all_reduce(t)
        return t

    def all_reduce_max(self, value: float) -> float:
        if not self.enabled:
            return value
        t = torch.tensor([value], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_gather_rows(self, local: torch.Tensor, k_max: int) -> torch.Tensor:
        """Gather each rank's ``[k_r, W]`` rows (k_r <= k_max) into ``[world * k_max, W]``
        (rank-major, zero-padded rows) with one flat collective."""
        W = local.shape[1]
        if not self.enabled:
            out = torch.zeros(k_max, W, dtype=local.dtype, device=local.device)
            out[:local.shape[0]] = local
            return out
        send = torch.zeros(k_max, W, dtype=local.dtype, device=local.device)
        if local.shape[0]:
            send[:local.shape[0]] = local
        out = torch.empty(self.world * k_max, W, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, send)
        return out

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.enabled:
            dist.broadcast(t, src)
        return t


def init_distributed(prefer_gpu: bool = True, timeout_s: int = 1800) -> DistCtx:
    """Initialise from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*); world 1 otherwise."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    # rehearsal knobs for a one-GPU box: DBA_SHARE_GPU=1 puts every rank on device 0 and
    # DBA_DIST_BACKEND=gloo replaces RCCL (which refuses two ranks on one GPU)
    dev_index = 0 if os.environ.get("DBA_SHARE_GPU") == "1" else local
    if use_gpu:
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    if world <= 1:
        return DistCtx(0, 1, 0, device, "none")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    backend = os.environ.get("DBA_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")   # "nccl" is RCCL
    kw = dict(backend=backend, rank=rank, world_size=world,
              timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl":
        kw["device_id"] = device
    if not dist.is_initialized():
        dist.init_process_group(**kw)
    return DistCtx(rank, world, dev_index, device, backend)


def shutdown(ctx: DistCtx) -> None:
    if ctx.enabled and dist.is_initialized():
        dist.destroy_process_group()
