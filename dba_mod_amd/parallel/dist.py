"""One process per GPU over ``torch.distributed`` (RCCL over xGMI on MI355X, Gloo on CPU).

The reference is single-process/single-GPU with no collective at all (its
logical reduction points are ``helper.py:218-257`` FedAvg, ``:320-352`` Weiszfeld,
``:537-570`` FoolsGold).  This framework's distributed round (client-parallel DP):

1. every rank computes the identical round plan (same seeded RNG; no communication);
2. clients are placed on ranks by LPT (:func:`dba_mod_amd.utils.native.lpt_assign`); a
   client's snapshots stay on its owner rank;
3. aggregation reduces instead of gathering (``fl/server.py`` ``_aggregate``):
   * FedAvg — each rank sums its own clients' deltas in fp64, ONE all-reduce of S values;
   * FoolsGold — ONE all-reduce of the ``[n, d]`` final-layer features (each row owned by
     one rank), weights computed identically everywhere, ONE all-reduce of the wv-weighted
     P-vector;
   * RFA — distributed Weiszfeld (per iteration an all-reduce of the S-vector partial
     weighted sum + an all-reduce of the n distances) when that moves fewer bytes than an
     all-gather of the n final states, else the all-gather (``rfa_mode``);
4. aggregation is applied redundantly on every rank (bit-identical global model, no
   broadcast);
5. a client's local tests run on its owner rank as soon as it finishes training; only the
   snapshots of the clients whose tests are image-sharded across ranks (the round's longest
   clients) are broadcast from their owners; the image-sharded tests are split by
   water-filling over every rank's load in the window (``Server._eval_shares``); ONE
   all-reduce of the ``[jobs, 3]`` counters combines the tests.

Bucket policy: every collective moves one contiguous flat buffer (never
per-layer calls); the all-reduce buckets are padded to a multiple of world x 7 xGMI links x
4 KiB so each ring chunk is equal and 4 KiB aligned, and issued in pieces of at most 64 MB
(a snapshot broadcast is one unpadded model row, <= 45 MB for the largest model).  ``bytes`` counts the
payload of every collective (per kind) for tests and the round metrics.  The int64 BN
counters never enter a float bucket.

On a one-GPU box the multi-rank path is rehearsed with ``DBA_SHARE_GPU=1`` (every rank on
device 0) and ``DBA_DIST_BACKEND=gloo`` (``tests/test_gpu_dist.py``).  ``emulate_rank``
(:func:`emulated_ctx`, ``bench.py --emulate-rank R --emulate-world N``) runs exactly rank R's
share of an N-rank round in ONE process: collectives are local no-ops that still count their
bytes, so the per-rank critical path can be timed on one GPU (the numerics are not those of
the real N-rank run: the other ranks' contributions are missing).

``init_distributed`` ends with a one-element all-reduce self-check (``selfcheck_ok``), and
``DBA_FORCE_PG=1`` creates the process group even at world 1 (RCCL initialisation evidence
on a one-GPU box).
"""
from __future__ import annotations

import collections
import datetime
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist


XGMI_LINKS = 7                 # point-to-point xGMI links per MI355X
PAD_BYTES = 4096               # per-link chunk alignment
SPLIT_BYTES = 64 << 20         # largest single collective


@dataclass
class DistCtx:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    bytes: Dict[str, int] = field(default_factory=lambda: collections.Counter())
    emulated: bool = False          # rank R of an N-rank round, alone: collectives are no-ops
    selfcheck_ok: Optional[bool] = None   # init-time all-reduce self-check (None: no group)
    pg: bool = False                # a torch.distributed process group exists
    affinity_changed: Optional[bool] = None   # the backend's init re-pinned the host thread
    hw_queues: Optional[str] = None           # GPU_MAX_HW_QUEUES of this process (GPU groups)
    queue_policy: bool = False                # configure_hip_queues applied

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def enabled(self) -> bool:
        return self.world > 1

    @property
    def comm(self) -> bool:
        """Collectives really run (a real multi-rank group, not an emulated rank)."""
        return self.world > 1 and not self.emulated

    def barrier(self) -> None:
        if self.comm:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def pad_unit(self, itemsize: int) -> int:
        """Elements per padding unit: world x links x 4 KiB."""
        return max(1, self.world * XGMI_LINKS * PAD_BYTES // itemsize)

    def padded(self, n: int, dtype: torch.dtype) -> torch.Tensor:
        """A zeroed flat buffer of ``n`` elements rounded up to the padding unit; fill
        ``buf[:n]`` and hand the whole buffer to :meth:`all_reduce_`."""
        unit = self.pad_unit(torch.empty(0, dtype=dtype).element_size())
        return torch.zeros((n + unit - 1) // unit * unit, dtype=dtype, device=self.device)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """Sum-all-reduce ``t`` in place (one flat buffer; pieces of <= 64 MB)."""
        if self.enabled:
            flat = t.view(-1) if t.is_contiguous() else None
            if flat is None:
                raise ValueError("all_reduce_ needs a contiguous buffer")
            if self.comm:
                step = max(1, SPLIT_BYTES // flat.element_size())
                for i in range(0, flat.numel(), step):
                    dist.all_reduce(flat[i:i + step])
            self.bytes["all_reduce"] += flat.numel() * flat.element_size()
        return t

    def all_reduce_max(self, value: float) -> float:
        if not self.comm:
            return value
        t = torch.tensor([value], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_gather_rows(self, local: torch.Tensor, k_max: int) -> torch.Tensor:
        """Gather each rank's ``[k_r, W]`` rows (k_r <= k_max) into ``[world * k_max, W]``
        (rank-major, zero-padded rows).  Each row is padded to the §5.8 unit and the rows
        go out in all-gathers of at most 64 MB of output each (a CIFAR RFA gather of 10
        final states is ~112 MB: two pieces)."""
        W = local.shape[1]
        if not self.enabled:
            out = torch.zeros(k_max, W, dtype=local.dtype, device=local.device)
            out[:local.shape[0]] = local
            return out
        unit = self.pad_unit(local.element_size())
        Wp = (W + unit - 1) // unit * unit
        send = torch.zeros(k_max, Wp, dtype=local.dtype, device=local.device)
        if local.shape[0]:
            send[:local.shape[0], :W] = local
        out = torch.zeros(self.world, k_max, Wp, dtype=local.dtype, device=local.device)
        if self.comm:
            rows = max(1, SPLIT_BYTES // (self.world * Wp * local.element_size()))
            for i in range(0, k_max, rows):
                j = min(k_max, i + rows)
                piece = torch.empty(self.world * (j - i), Wp, dtype=local.dtype, device=local.device)
                dist.all_gather_into_tensor(piece, send[i:j].contiguous())
                out[:, i:j] = piece.view(self.world, j - i, Wp)
        else:
            out[self.rank] = send
        self.bytes["all_gather"] += out.numel() * out.element_size()
        return out[:, :, :W].reshape(self.world * k_max, W)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.enabled:
            if self.comm:
                dist.broadcast(t, src)
            self.bytes["broadcast"] += t.numel() * t.element_size()
        return t

    def gather_strings(self, s: str) -> List[str]:
        """Every rank's ``s`` (rank order), e.g. its device; one object all-gather."""
        if not self.comm:
            return [s]
        out: List[Any] = [None] * self.world
        dist.all_gather_object(out, s)
        return [str(x) for x in out]

    def take_bytes(self) -> Dict[str, int]:
        """Collective payload bytes since the last call (and reset)."""
        out = dict(self.bytes)
        self.bytes.clear()
        return out


_STREAMS: Dict[int, tuple] = {}


def framework_streams(device: torch.device):
    """The process's (train, eval, early-eval) streams, created once per device: training on a
    HIGH-priority stream, the two evaluation streams at default priority (``fl/server.py``).

    ``torch.cuda.Stream`` hands out streams round-robin from PyTorch's per-priority pools, and
    HIP maps those streams onto the process's few hardware queues (``GPU_MAX_HW_QUEUES``, 4 on
    the box).  :func:`init_distributed` takes these three before the process group exists
    (``DBA_STREAMS_FIRST=0``: after), so RCCL's own pool streams cannot shift the training and
    evaluation streams onto a shared hardware queue."""
    key = device.index if device.index is not None else torch.cuda.current_device()
    if key not in _STREAMS:
        pri = int(os.environ.get("DBA_TRAIN_STREAM_PRIORITY", "-1"))
        _STREAMS[key] = (torch.cuda.Stream(device, priority=pri), torch.cuda.Stream(device, priority=0),
                         torch.cuda.Stream(device, priority=0))
    return _STREAMS[key]


# Hardware queues and stream priorities of a process that holds an RCCL communicator.  A live
# communicator stops a high-priority stream from running concurrently with a default-priority
# one (tools/launch_probe two-stream check: overlap 1.23x without a communicator, 0.82x with
# one — slower than serial), which costs the overlapped round (evaluation under latency-bound
# training) 26 %: world-1 group 2.04 vs 2.75 rounds/s.  Measured on one box
# (profiles/prio_r3/, 12 rounds each): with the communicator, default-priority streams on 6 or
# 8 hardware queues run at 2.83 (= no communicator, 2.75-2.82); 4 queues 2.44, 16 queues 2.09,
# high priority on 8 queues 1.99.  Without a communicator the HIP defaults (4 queues, high-
# priority training) are the best (8 queues: 2.04-2.07).  So ranks that create a communicator
# take 8 queues and default priority; the variable must be set before HIP initialises.
PG_HW_QUEUES = "8"


def configure_hip_queues(world: int, force_pg: bool) -> bool:
    """Apply the communicator-process queue / priority policy (before any HIP call).  Returns
    whether it was applied.  ``DBA_HW_QUEUES=keep`` leaves the environment alone."""
    if not (world > 1 or force_pg) or os.environ.get("DBA_HW_QUEUES") == "keep":
        return False
    if torch.cuda.is_initialized():
        return False                      # too late: HIP read its queue count at init
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("DBA_HW_QUEUES", PG_HW_QUEUES)
    os.environ.setdefault("DBA_TRAIN_STREAM_PRIORITY", "0")
    return True


def init_distributed(prefer_gpu: bool = True, timeout_s: int = 1800) -> DistCtx:
    """Initialise from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*); world 1 otherwise."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    force_pg = os.environ.get("DBA_FORCE_PG") == "1" and "MASTER_PORT" in os.environ
    backend_env = os.environ.get("DBA_DIST_BACKEND")
    queues = (configure_hip_queues(world, force_pg) if prefer_gpu and backend_env in (None, "nccl")
              else False)
    use_gpu = prefer_gpu and torch.cuda.is_available()
    # rehearsal knobs for a one-GPU box: DBA_SHARE_GPU=1 puts every rank on device 0 and
    # DBA_DIST_BACKEND=gloo replaces RCCL (which refuses two ranks on one GPU)
    dev_index = 0 if os.environ.get("DBA_SHARE_GPU") == "1" else local
    if use_gpu:
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    if world <= 1 and not force_pg:
        return DistCtx(0, 1, 0, device, "none")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    backend = os.environ.get("DBA_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")   # "nccl" is RCCL
    kw = dict(backend=backend, rank=rank, world_size=world,
              timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl" and os.environ.get("DBA_PG_LAZY") != "1":
        kw["device_id"] = device   # eager communicator (DBA_PG_LAZY=1: created at the first collective)
    # RCCL binds the initialising thread to the GPU's NUMA-local cores; inside a container
    # whose cgroup CPU set does not match, that pins the one host thread that enqueues every
    # kernel onto a few (shared) cores — measured: the 1-GPU bench with a world-1 RCCL group
    # ran at 2.18 rounds/s vs 2.94 without (profiles/bench_r3_rccl_affinity.md).  Keep the
    # affinity the process started with (DBA_KEEP_RCCL_AFFINITY=1 keeps RCCL's choice).
    aff = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    if use_gpu and os.environ.get("DBA_STREAMS_FIRST", "1") != "0":
        framework_streams(device)
    if not dist.is_initialized():
        dist.init_process_group(**kw)
    ctx = DistCtx(rank, world, dev_index, device, backend, pg=True)
    ctx.hw_queues = os.environ.get("GPU_MAX_HW_QUEUES") if use_gpu else None
    ctx.queue_policy = queues
    ctx.selfcheck_ok = selfcheck(ctx) if os.environ.get("DBA_PG_SKIP_SELFCHECK") != "1" else None
    if aff is not None and os.environ.get("DBA_KEEP_RCCL_AFFINITY") != "1":
        ctx.affinity_changed = os.sched_getaffinity(0) != aff
        os.sched_setaffinity(0, aff)
    if ctx.selfcheck_ok is False:
        raise RuntimeError(f"rank {rank}: {backend} all-reduce self-check failed (world {world})")
    return ctx


def selfcheck(ctx: DistCtx) -> bool:
    """One all-reduce of ``rank + 1`` on the rank's device; the closed form is w(w+1)/2.
    With backend "nccl" this is the first RCCL collective of the run."""
    t = torch.full((4,), float(ctx.rank + 1), dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t)
    return bool(torch.all(t == ctx.world * (ctx.world + 1) / 2).item())


def emulated_ctx(rank: int, world: int, prefer_gpu: bool = True) -> DistCtx:
    """Rank ``rank`` of a ``world``-rank round, run alone (no process group): every
    collective is a local no-op that counts its bytes (``DistCtx.emulated``)."""
    if not 0 <= rank < world:
        raise ValueError(f"emulate rank {rank} of world {world}")
    use_gpu = prefer_gpu and torch.cuda.is_available()
    device = torch.device("cuda", 0) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(0)
    return DistCtx(rank, world, 0, device, "emulated", emulated=True)


def shutdown(ctx: DistCtx) -> None:
    if ctx.pg and dist.is_initialized():
        dist.destroy_process_group()
