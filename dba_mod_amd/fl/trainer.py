"""Grouped client trainer: all of a rank's clients train *concurrently* as one replica group.

The reference trains the round's clients one after another on one shared model with a
fresh optimizer each (``image_train.py:21-36``), synchronising with the host on every batch
(``.item()`` at ``:105,223``).  Here a rank's G clients are G rows of flat ``[G, S]`` replica
buffers; each grouped step gathers every client's next batch (one kernel), runs the
grouped forward/backward (every conv launch covers all G clients — this is what fills 256
CUs at batch 64), and applies a per-client SGD step with per-client learning rate and
momentum-reset flags.  Clients with fewer steps simply go inactive (``nvalid = 0``: every
kernel skips them) — the control flow is static, so on GPU the whole step is captured once
into a HIP graph and replayed; per-step inputs are one packed descriptor row copied
device-to-device before each replay.  Loss/accuracy counters stay on the device and are
read once per round.
"""
from __future__ import annotations

import logging
import math
import os
import struct
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import config as C
from .. import ops
from ..ops import reference as ref_ops
from ..models import program as prog
from ..models.spec import ModelSpec
from ..utils import native
from ..utils.devcopy import to_device
from .plan import ClientPlan, RoundPlan
from .workload import Workload

log = logging.getLogger("logger")

# arrival counters per training step for the in-launch split-K combines of the fp32 convs
# (xconv.hpp sk_combine, lone-client launches): a ResNet-18 step needs 14 launches x <= 128;
# zeroed with the step's operand-max arena (no extra launch).  0: separate reduce launches
SK_COUNTERS = int(os.environ.get("DBA_SK_COUNTERS", str(1 << 15)))


@dataclass
class ClientResult:
    name: Any
    snapshots: Dict[int, torch.Tensor]        # snapshot slot -> state [S] (device)
    fg_grad: Optional[torch.Tensor]           # [P] summed gradients (FoolsGold)
    stats: np.ndarray                         # [n_slots, 3] loss_sum(batch-mean), correct, count
    scale_dist: Dict[int, float] = field(default_factory=dict)   # phase epoch -> distance
    num_samples: int = 0
    steps: int = 0
    # per-step (batch loss, distance to the round's global model) when vis_train_batch_loss /
    # batch_track_distance are set (model.train_batch_vis / track_distance_batch_vis)
    batch_trace: Optional[np.ndarray] = None
    # phase epoch -> (global norm, norm before scaling, distance before scaling, scaled norm):
    # the reference's poison-phase log lines (helper.model_global_norm / model_dist_norm,
    # image_train.py:144-146,172-183; loan_train.py:148-168)
    scale_norms: Dict[int, Tuple[float, float, float, float]] = field(default_factory=dict)


class _GroupBuffers:
    """Static per-G buffers (and the captured graph) reused across rounds."""

    def __init__(self, spec: ModelSpec, G: int, B: int, max_slots: int, device: torch.device,
                 fg: bool) -> None:
        S, P = spec.S, spec.P
        self.G, self.B, self.max_slots = G, B, max_slots
        self.state = torch.zeros(G, S, dtype=torch.float32, device=device)
        self.grads = torch.zeros(G, P, dtype=torch.float32, device=device)
        self.mom = torch.zeros(G, P, dtype=torch.float32, device=device)
        self.fg = torch.zeros(G, P, dtype=torch.float32, device=device) if fg else None
        self.base = torch.zeros(G, S, dtype=torch.float32, device=device)   # phase-start states
        self.stats = torch.zeros(3, G * max_slots, dtype=torch.float32, device=device)
        self.nan_flag = torch.zeros(1, dtype=torch.float32, device=device)
        # packed descriptor: idx[G*B] poison_n[G] trig[G] first[G] active[G] nvalid[G] slot[G] seed[G] lr[G]
        self.D = G * B + 8 * G
        self.desc = torch.zeros(self.D, dtype=torch.int32, device=device)
        o = G * B
        self.idx = self.desc[:o].view(G, B)
        names = ["poison_n", "trig", "first", "active", "nvalid", "slot", "seed", "lr_bits"]
        for k, n in enumerate(names):
            setattr(self, n, self.desc[o + k * G:o + (k + 1) * G])
        self.lr = self.lr_bits.view(torch.float32)
        self.graph: Optional[torch.cuda.CUDAGraph] = None


class _TrainHandle:
    """Training enqueued by :meth:`GroupTrainer.train_async`; ``collect()`` waits for it."""

    def __init__(self, trainer: "GroupTrainer", done: List[ClientResult], last) -> None:
        self.trainer, self.done, self.last = trainer, done, last

    def collect(self) -> List[ClientResult]:
        out = self.done + self.trainer._wave_collect(self.last)
        self.last = None
        return out


class GroupTrainer:
    def __init__(self, wl: Workload, params: C.Params, compute_dtype: torch.dtype,
                 max_groups: int = 16) -> None:
        self.wl, self.params, self.spec = wl, params, wl.spec
        self.device = wl.device
        self.dtype = compute_dtype
        self.max_groups = max_groups
        self._bufs: Dict[Tuple[int, int], _GroupBuffers] = {}
        self.use_graph = (self.device.type == "cuda" and bool(params["graph_capture"])
                          and ops.backend_name(self.device) == "hip")
        self.fg = params["aggregation_methods"] == C.AGGR_FOOLSGOLD
        self.momentum = float(params["momentum"])
        self.wd = float(params["decay"])
        self.B = int(params["batch_size"])
        self.target = int(params["poison_label_swap"])
        # anomaly-evasion distance term; every shipped config has alpha_loss = 1 (term off)
        self.alpha = float(params["alpha_loss"])
        # per-batch loss / distance tracing for the Visdom batch plots: eager steps (the
        # per-step values are read back), off in every shipped config
        self.trace = bool(params["vis_train_batch_loss"]) or bool(params["batch_track_distance"])
        if self.trace:
            self.use_graph = False
        self._last_loss: Optional[torch.Tensor] = None
        # LoanNet: every client's steps between two phase events run in ONE persistent launch
        # (csrc/kernels/mlp.hip, one workgroup per client) instead of a graph replay per step;
        # DBA_MLP_PERSIST=0 keeps the per-step graph
        self.persistent = (self.spec.arch == "loan" and self.device.type == "cuda" and self.alpha == 1.0
                           and not self.trace and ops.backend_name(self.device) == "hip"
                           and os.environ.get("DBA_MLP_PERSIST", "1") != "0")
        # per-client epoch slots of the step statistics: sized once for the longest phase the
        # config can run (benign and poison rounds then share one buffer set and one captured
        # graph per group size, so a poison round captures nothing new)
        ep = max(1, int(params["internal_epochs"]), int(params["internal_poison_epochs"]))
        self.min_slots = 1 << (ep - 1).bit_length()

    # ------------------------------------------------------------------ step
    def _step(self, b: _GroupBuffers) -> None:
        # one zeroed arena for the step's operand-max slots and split-K counters (re-zeroed by
        # the captured fill at every graph replay)
        with ops.amax_arena(b.state.shape[0], self.device, counters=SK_COUNTERS):
            self._step_ops(b)

    def _step_ops(self, b: _GroupBuffers) -> None:
        wl = self.wl
        if wl.kind == "image":
            x, y = ops.gather_images(wl.train_store.images, wl.train_store.labels, b.idx, wl.trig_masks,
                                     b.trig, b.poison_n, self.target, b.seed if wl.flip_train else None,
                                     self.dtype)
        else:
            x, y = ops.gather_rows(wl.train_store.rows, wl.train_store.labels, b.idx, wl.trig_cols,
                                   wl.trig_vals, b.trig, b.poison_n, self.target, self.dtype)
        ctx = prog.Ctx(self.spec, b.state, b.state, None, train=True, grads=b.grads,
                       nvalid=b.nvalid, dropout_seed=b.seed, act_dtype=self.dtype)
        fused = self.alpha == 1.0     # stats straight from the loss kernel (no extra launches)
        # the opt-in fused classifier head (pool + linear + loss + the head's backward in two
        # launches, models/program.py Ctx.fused_head, DBA_FUSED_HEAD=1) writes its gradients
        # during the forward
        ctx.head = {"labels": y, "stats": b.stats if fused else None, "slot": b.slot}
        b.grads.zero_()
        out = prog.forward(ctx, x)
        if ctx.head_out is not None:
            loss, correct = ctx.head_out
            ctx.tape.backward(out, out)   # (the head node ignores the seed)
        else:
            loss, correct, dl = ops.softmax_xent(out, y, True, True, *((b.stats, b.slot, b.nvalid) if fused else ()),
                                                 grad_dtype=x.dtype)
            if self.spec.arch == "loan":   # reference LoanNet raises on NaN outputs (loan_model.py:25-26)
                b.nan_flag += torch.isnan(loss).any().float()
            ctx.tape.backward(out, dl)
        if self.alpha != 1.0:
            # poison phases train on a*CE + (1-a)*||w - w_g|| with w_g the interval-start
            # model (image_train.py:52-54,87-90; loan_train.py:61-63,114-117)
            dist = ops.dist_loss_grad(b.state, b.base, b.grads, b.trig, b.active, self.alpha)
            loss = torch.where(b.trig >= 0, self.alpha * loss + (1.0 - self.alpha) * dist, loss)
        ops.sgd_step(b.state[:, :self.spec.P], b.grads, b.mom, b.lr, b.first, b.active, self.momentum,
                     self.wd, fg_accum=b.fg)
        if not fused:
            ref_ops.accumulate_step_stats(b.stats, b.slot, loss, correct, b.nvalid)
        self._last_loss = loss

    def _buffers(self, G: int, max_slots: int) -> _GroupBuffers:
        key = (G, max_slots)
        if key not in self._bufs:
            self._bufs[key] = _GroupBuffers(self.spec, G, self.B, max_slots, self.device, self.fg)
        return self._bufs[key]

    def prewarm(self, G: int) -> None:
        """Allocate the G-client buffers and capture their step graph ahead of use (an
        all-inactive descriptor: every kernel skips every replica).  The server does this for
        the lone-client shape at start-up, so the first poison round's lone attacker tail does
        not pay the capture (~45 ms) inside the attack window."""
        if not self.use_graph or self.persistent:
            return
        b = self._buffers(G, self.min_slots)
        if b.graph is None:
            b._cur = torch.zeros(b.D, dtype=torch.int32, device=self.device)
            self._run_step(b)

    def _run_step(self, b: _GroupBuffers) -> None:
        if not self.use_graph:
            self._step(b)
            return
        if b.graph is None:
            b.desc.copy_(b._cur)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):   # warm-up outside capture (allocator, lazy init)
                self._step(b)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._step(b)
            b.graph = g
            # the warm-up and capture executed the step twice: replay state is restored by
            # the caller (train() re-initialises before the real loop).
            return
        b.graph.replay()

    # ----------------------------------------------------------------- train
    def train(self, clients: List[ClientPlan], global_state: torch.Tensor,
              on_client_done: Optional[Callable[[ClientPlan, Dict[int, torch.Tensor]], None]] = None
              ) -> List[ClientResult]:
        """Train ``clients`` from ``global_state``.  ``on_client_done(client, snapshots)`` is
        called (host side, in stream order) the moment a client's last phase has ended, so its
        local tests can be enqueued while the other clients are still training."""
        return self.train_async(clients, global_state, on_client_done).collect()

    def train_async(self, clients: List[ClientPlan], global_state: torch.Tensor,
                    on_client_done=None) -> "_TrainHandle":
        """Enqueue the training of ``clients`` and return without waiting for the GPU (only
        earlier waves of a rank holding more than ``max_groups`` clients are collected
        synchronously: they share buffers with the next wave).  ``collect()`` synchronises
        and returns the results."""
        done: List[ClientResult] = []
        last = None
        for w0 in range(0, len(clients), self.max_groups):
            if last is not None:
                done.extend(self._wave_collect(last))
            last = self._wave_enqueue(clients[w0:w0 + self.max_groups], global_state, on_client_done)
        return _TrainHandle(self, done, last)

    def _wave_enqueue(self, clients: List[ClientPlan], global_state: torch.Tensor,
                      on_client_done=None) -> Optional[Dict[str, Any]]:
        G = len(clients)
        if G == 0:
            return None
        max_slots = max(sum(ph.internal_epochs for ph in c.phases) for c in clients)
        max_slots = max(self.min_slots, 1 << (max_slots - 1).bit_length())
        b = self._buffers(G, max_slots)
        T = max(len(c.steps) for c in clients)
        host = native.pack_steps(clients, G, self.B, T, max_slots)   # [T, D] int32 (C++ runtime)
        sched = to_device(host, self.device)
        if self.persistent:
            res = self._persistent_enqueue(clients, b, sched, T, global_state, on_client_done)
            if res is not None:
                return res
            # the kernel declined the shape (a batch size / layer width other than the
            # reference LoanNet's, or a device without its LDS budget) before launching
            # anything: this trainer keeps the per-step graph path from now on
            self.persistent = False
        if self.use_graph and b.graph is None:
            b._cur = sched[0]
            self._reset(b, global_state)
            self._run_step(b)            # capture (mutates buffers; reset below)
        self._reset(b, global_state)

        events = self._events(clients)
        snaps: Dict[int, Dict[int, torch.Tensor]] = {g: {} for g in range(G)}
        pend_dist: List[Tuple[int, int, torch.Tensor]] = []
        trace: List[torch.Tensor] = []
        gstate = global_state[None, :self.spec.P]
        solo = self._solo_tail(clients, T)
        cur, row_of, cur_sched = b, list(range(G)), sched
        # the round's global model norm (helper.model_global_norm(target_model),
        # image_train.py:144, loan_train.py:148), once per wave, for the poison-phase log lines
        gn2 = (ops.sq_dists(global_state[None, :self.spec.P], self._zeros_p())[0]
               if any(ph.pre_scale_snap is not None for c in clients for ph in c.phases) else None)
        for t in range(T):
            if solo is not None and t == solo[0]:
                # only client solo[1] is left: its remaining steps run in the G=1 graph
                # (every launch sized for one replica) instead of a G-replica graph whose other
                # replicas are idle — identical bits (per-replica kernel decisions only)
                cur, cur_sched = self._solo_enter(b, solo[1], clients, T, max_slots, global_state)
                row_of = [0 if g == solo[1] else -1 for g in range(G)]
            cur.desc.copy_(cur_sched[t], non_blocking=True)
            self._run_step(cur)
            if self.trace:
                dist = (b.state[:, :self.spec.P] - gstate).float().pow(2).sum(1).sqrt()
                trace.append(torch.stack([self._last_loss.float(), dist], 1))
            for (g, ph) in events.get(t + 1, []):
                self._phase_end(cur, row_of[g], ph, snaps[g], pend_dist, g, gn2)
                if on_client_done is not None and ph is clients[g].phases[-1]:
                    on_client_done(clients[g], snaps[g])
        if cur is not b:
            self._solo_leave(cur, b, solo[1])
        return {"b": b, "clients": clients, "snaps": snaps, "pend_dist": pend_dist, "sched": sched,
                "trace": torch.stack(trace) if trace else None}

    def _persistent_enqueue(self, clients: List[ClientPlan], b: _GroupBuffers, sched: torch.Tensor, T: int,
                            global_state: torch.Tensor, on_client_done=None) -> Optional[Dict[str, Any]]:
        """LoanNet: one persistent launch per segment of steps between phase events (the
        snapshots / scaling of :meth:`_phase_end` run between launches, as between graph
        replays).  None when the kernel declines the shape at the first segment (nothing was
        launched: the caller takes the per-step path)."""
        self._reset(b, global_state)
        G = len(clients)
        events = self._events(clients)
        snaps: Dict[int, Dict[int, torch.Tensor]] = {g: {} for g in range(G)}
        pend_dist: List[Tuple[int, int, torch.Tensor]] = []
        gn2 = (ops.sq_dists(global_state[None, :self.spec.P], self._zeros_p())[0]
               if any(ph.pre_scale_snap is not None for c in clients for ph in c.phases) else None)
        wl = self.wl
        hip = ops.hip_module()
        t0 = 0
        for t1 in sorted(set(events) | {T}):
            if t1 > t0:
                rc = hip.mlp_train(self.spec, sched, t0, t1, self.B, b.state, b.mom, b.fg, wl.train_store.rows,
                                   wl.train_store.labels, wl.trig_cols, wl.trig_vals, self.target, b.stats,
                                   b.max_slots, b.nan_flag, self.momentum, self.wd)
                if rc == hip.NOT_HANDLED and t0 == 0:
                    return None
                if rc != 0:
                    raise RuntimeError(f"persistent LoanNet trainer failed mid-wave ({rc})")
                t0 = t1
            for (g, ph) in events.get(t1, []):
                self._phase_end(b, g, ph, snaps[g], pend_dist, g, gn2)
                if on_client_done is not None and ph is clients[g].phases[-1]:
                    on_client_done(clients[g], snaps[g])
        return {"b": b, "clients": clients, "snaps": snaps, "pend_dist": pend_dist, "sched": sched, "trace": None}

    # a lone client's tail shorter than this stays in the group graph
    SOLO_MIN_STEPS = int(os.environ.get("DBA_SOLO_MIN_STEPS", "4"))

    def _solo_tail(self, clients: List[ClientPlan], T: int) -> Optional[Tuple[int, int]]:
        """(t0, g) when from step t0 on only client g trains (the 6-epoch attacker after the
        2-epoch clients finished) for at least SOLO_MIN_STEPS steps; graph mode, G > 1 only."""
        if not self.use_graph or len(clients) < 2 or self.SOLO_MIN_STEPS <= 0:
            return None
        # bit-identical: the fp32 family decides every summation order from the per-replica
        # geometry (split-K, fused BN groups), so moving a client to the one-replica graph
        # changes no rounding (tests/test_gpu_e2e.py test_solo_tail_bitwise)
        lens = sorted(((len(c.steps), g) for g, c in enumerate(clients)), reverse=True)
        (n0, g0), (n1, _) = lens[0], lens[1]
        if n0 != T or n0 - n1 < self.SOLO_MIN_STEPS:
            return None
        return n1, g0

    def _solo_enter(self, b: _GroupBuffers, g: int, clients: List[ClientPlan], T: int, max_slots: int,
                    global_state: torch.Tensor):
        b1 = self._buffers(1, max_slots)
        sched1 = to_device(native.pack_steps([clients[g]], 1, self.B, T, max_slots), self.device)
        if b1.graph is None:
            b1._cur = sched1[T - 1]
            self._reset(b1, global_state)
            self._run_step(b1)            # capture (mutates b1: overwritten below)
        self._copy_row(b, g, b1, 0)
        b1.nan_flag.zero_()
        return b1, sched1

    def _solo_leave(self, b1: _GroupBuffers, b: _GroupBuffers, g: int) -> None:
        self._copy_row(b1, 0, b, g)
        b.nan_flag += b1.nan_flag

    @staticmethod
    def _copy_row(src: _GroupBuffers, i: int, dst: _GroupBuffers, j: int) -> None:
        dst.state[j].copy_(src.state[i])
        dst.base[j].copy_(src.base[i])
        dst.mom[j].copy_(src.mom[i])
        if dst.fg is not None:
            dst.fg[j].copy_(src.fg[i])
        ms = dst.max_slots
        dst.stats.view(3, -1, ms)[:, j].copy_(src.stats.view(3, -1, ms)[:, i])

    def _wave_collect(self, w: Optional[Dict[str, Any]]) -> List[ClientResult]:
        if w is None:
            return []
        b, clients, snaps = w["b"], w["clients"], w["snaps"]
        G = len(clients)
        res: List[ClientResult] = []
        stats = b.stats.view(3, G, b.max_slots).permute(1, 2, 0).cpu().numpy()
        if self.spec.arch == "loan" and float(b.nan_flag.item()) > 0:
            raise ValueError("NaN in LoanNet forward (reference loan_model.py:25-26)")
        dists: Dict[int, Dict[int, float]] = {g: {} for g in range(G)}
        norms: Dict[int, Dict[int, Tuple[float, float, float, float]]] = {g: {} for g in range(G)}
        for g, e, d in w["pend_dist"]:
            # read as scalars and finished on the host: the device form (stack / fp64 clamp /
            # sqrt) launched torch kernels no benign round uses, and their first launch — in
            # the first poison round — stalled the host ~100 ms each while ROCm loaded them
            # (profiles/r5/first_poison/); IEEE sqrt, so the same values
            v = [math.sqrt(max(float(x.item()), 0.0)) for x in d]
            dists[g][e] = float(v[0])
            norms[g][e] = (v[1], v[2], v[3], v[4])
        tr = w["trace"].cpu().numpy() if w["trace"] is not None else None    # [T, G, 2]
        for g, c in enumerate(clients):
            nsl = sum(ph.internal_epochs for ph in c.phases)
            res.append(ClientResult(c.name, snaps[g], b.fg[g].clone() if b.fg is not None else None,
                                    stats[g, :nsl].copy(), dists[g], c.num_samples, len(c.steps),
                                    tr[:len(c.steps), g].copy() if tr is not None else None, norms[g]))
        return res

    def _reset(self, b: _GroupBuffers, global_state: torch.Tensor) -> None:
        b.state.copy_(global_state[None].expand_as(b.state))
        b.base.copy_(b.state)
        b.mom.zero_()
        b.stats.zero_()
        b.nan_flag.zero_()
        if b.fg is not None:
            b.fg.zero_()

    def _zeros_p(self) -> torch.Tensor:
        z = getattr(self, "_zp", None)
        if z is None:
            z = self._zp = torch.zeros(self.spec.P, dtype=torch.float32, device=self.device)
        return z

    @staticmethod
    def _events(clients: List[ClientPlan]) -> Dict[int, List[Tuple[int, Any]]]:
        ev: Dict[int, List[Tuple[int, Any]]] = {}
        for g, c in enumerate(clients):
            for ph in c.phases:
                ev.setdefault(ph.end_step, []).append((g, ph))
        return ev

    def _phase_end(self, b: _GroupBuffers, g: int, ph, snaps, pend_dist, client: int,
                   gn2: Optional[torch.Tensor] = None) -> None:
        """End of a local round: optional model-replacement scaling + snapshots.  ``g``: the
        client's row in ``b``; ``snaps``: the client's snapshot dict; ``client``: its index in
        the wave (the key of its pending distances); ``gn2``: the round's squared global
        model norm."""
        P = self.spec.P
        if ph.pre_scale_snap is not None:
            pre = b.state[g].clone()
            snaps[ph.pre_scale_snap] = pre
            gamma = float(self.params["scale_weights_poison"])
            scaled = ops.scale_from_base(b.state[g], b.base[g], gamma)
            b.state[g].copy_(scaled)
            # norms / distances over parameters only (helper.model_global_norm /
            # model_dist_norm, helper.py:59-71): scaled distance, the round's global model norm,
            # norm and distance before scaling, scaled norm — squared, on device, read once at
            # collect
            zero = self._zeros_p()
            if gn2 is None:
                gn2 = ops.sq_dists(b.base[g:g + 1, :P], zero)[0]
            pend_dist.append((client, ph.epoch, [
                ops.sq_dists(b.state[g:g + 1, :P], b.base[g, :P])[0], gn2,
                ops.sq_dists(pre[None, :P], zero)[0], ops.sq_dists(pre[None, :P], b.base[g, :P])[0],
                ops.sq_dists(b.state[g:g + 1, :P], zero)[0]]))
        snaps[ph.post_snap] = b.state[g].clone()
        b.base[g].copy_(b.state[g])
