"""Batched, sharded evaluation of every test the round needs.

The reference runs each test as its own full pass over the test set, one model at a time,
with a host sync per batch (``test.py:7-239``), and one CIFAR round runs ~15 such passes
(evaluation is ~84 % of a round's FLOPs).  Here a round's tests are *jobs*
``(model snapshot, clean | triggered, trigger id)`` evaluated together:

* all model snapshots are BN-folded once (:func:`dba_mod_amd.models.program.fold_bank`);
* jobs are grouped: one grouped forward covers up to ``max_groups`` jobs x ``chunk`` images,
  each job selecting its weights through ``wsel`` and its trigger through the fused gather;
* every job's image list is sharded across ranks (``[rank::world]``) and the
  ``[jobs, 3]`` (loss sum, correct, count) counters are all-reduced once.

Semantics per job (``Mytest`` / ``Mytest_poison*``): clean = CE(sum) and accuracy over the
full test set; poison = every sample of the non-target subset triggered and relabelled to
``poison_label_swap``, accuracy = ASR.
"""
from __future__ import annotations

import logging
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..models import program as prog
from ..utils import native
from ..utils.devcopy import to_device
from .plan import EvalJob
from .workload import Workload

log = logging.getLogger("logger")


class Evaluator:
    def __init__(self, wl: Workload, compute_dtype: torch.dtype, chunk: int = 1024,
                 max_groups: int = 24) -> None:
        self.wl = wl
        self.dtype = compute_dtype
        self.chunk = int(chunk)
        self.max_groups = int(max_groups)
        self.target = int(wl.params["poison_label_swap"])

    def run(self, bank: torch.Tensor, jobs: Sequence[EvalJob], rank: int = 0, world: int = 1,
            shares: Optional[Sequence[float]] = None) -> torch.Tensor:
        """bank [M, S] model states -> device tensor [J, 3] (loss_sum, correct, count), this
        rank's shard only (caller all-reduces).  ``shares`` (one per rank, summing to 1): rank
        r takes a contiguous ``shares[r]`` fraction of every test list (load-balanced sharding,
        :meth:`Server._eval_shares`) instead of the strided ``[rank::world]`` shard."""
        wl = self.wl
        dev = wl.device
        J = len(jobs)
        acc = torch.zeros(J, 3, dtype=torch.float64, device=dev)
        if J == 0:
            return acc
        # only fold the snapshots the jobs use
        used = sorted({j.model for j in jobs})
        remap = {m: i for i, m in enumerate(used)}
        sub = (bank[to_device(used, bank.device, torch.int64)] if len(used) != bank.shape[0] else bank)
        folded = prog.fold_bank(wl.spec, sub, self.dtype)
        lists = {}
        for kind, idx in (("clean", wl.test_clean_idx), ("poison", wl.test_poison_idx)):
            if world <= 1:
                lists[kind] = idx
            elif shares is not None:
                lo, hi = native.share_range(len(idx), shares, rank)
                lists[kind] = idx[lo:hi]
            else:
                lists[kind] = native.shard_index(idx, rank, world)
        for j0 in range(0, J, self.max_groups):
            grp = list(range(j0, min(J, j0 + self.max_groups)))
            self._run_group(folded, [jobs[j] for j in grp], [remap[jobs[j].model] for j in grp],
                            lists, acc[j0:j0 + len(grp)])
        return acc

    def _run_group(self, folded, jobs: List[EvalJob], slots: List[int], lists, acc: torch.Tensor) -> None:
        wl = self.wl
        dev = wl.device
        G = len(jobs)
        idx_lists = [lists[j.kind] for j in jobs]
        n_max = max(len(a) for a in idx_lists)
        if n_max == 0:
            return
        B = min(self.chunk, n_max)
        # every upload is pinned + async: a pageable copy here would block the host until the
        # whole queue of this (overlapped) evaluation stream had drained
        wsel = to_device(slots, dev, torch.int32)
        trig = to_device([j.trig if j.kind == "poison" else -1 for j in jobs], dev, torch.int32)
        pn = to_device([B if j.kind == "poison" else 0 for j in jobs], dev, torch.int32)
        # one upload of every chunk's index table: [n_chunks, G, B]
        n_chunks = (n_max + B - 1) // B
        table = -np.ones((n_chunks, G, B), dtype=np.int32)
        nval = np.zeros((n_chunks, G), dtype=np.int32)
        for g, a in enumerate(idx_lists):
            n = len(a)
            padded = -np.ones(n_chunks * B, dtype=np.int32)
            padded[:n] = a
            table[:, g, :] = padded.reshape(n_chunks, B)
            for c in range(n_chunks):
                nval[c, g] = max(0, min(B, n - c * B))
        table_d = to_device(table, dev)
        nval_d = to_device(nval, dev)
        for c in range(n_chunks):
            idx = table_d[c]
            # (one zeroed allocation for the chunk's fp16-pair operand-max slots)
            with ops.amax_arena(G, dev):
                if wl.kind == "image":
                    x, y = ops.gather_images(wl.test_store.images, wl.test_store.labels, idx, wl.trig_masks,
                                             trig, pn, self.target, None, self.dtype)
                else:
                    x, y = ops.gather_rows(wl.test_store.rows, wl.test_store.labels, idx, wl.trig_cols,
                                           wl.trig_vals, trig, pn, self.target, self.dtype)
                ctx = prog.Ctx(wl.spec, None, None, wsel, train=False, folded=folded, nvalid=nval_d[c],
                               act_dtype=self.dtype)
                logits = prog.forward(ctx, x)
            loss, correct, _ = ops.softmax_xent(logits, y, False, False, loss_dtype=torch.float64)
            acc[:, 0] += loss.double()
            acc[:, 1] += correct.double()
        acc[:, 2] += to_device([len(a) for a in idx_lists], dev, torch.float64)
