"""The FL round orchestrator — equivalent of the reference's ``main.py`` round loop
(``main.py:135-235``), re-designed for one process per GPU.

Per round: select clients (identically on every rank) → plan → LPT-place clients on ranks →
grouped concurrent local training → one all-gather of client snapshots → aggregation
(FedAvg / RFA / FoolsGold, redundantly on every rank) → batched, image-sharded evaluation
with one counter all-reduce → CSV rows / checkpoint / metrics on rank 0.
"""
from __future__ import annotations

import dataclasses
import datetime
import logging
import os
import time
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch
import yaml

from .. import config as C
from .. import ops
from ..parallel.dist import DistCtx, framework_streams
from ..utils import checkpoint as ckpt
from ..utils import native
from ..utils.csv_record import CsvRecorder
from ..utils.devcopy import to_device
from ..utils.observability import MetricsStream, PhaseTimer, Plotter, dict_html, setup_logger
from . import aggregate as agg
from .evaluate import Evaluator
from .plan import ClientPlan, RoundPlan, build_round_plan, select_clients
from .trainer import ClientResult, GroupTrainer
from .workload import Workload, build_workload

log = logging.getLogger("logger")


class _EarlyEval:
    """Enqueues a client's local tests (``image_train.py:139-160,268-299``: clean / poison /
    own-trigger tests of its own snapshots) the moment its last phase ends.

    Benign clients finish long before a 6-epoch attacker: their local tests then run on the
    eval stream underneath the latency-bound tail of the round's training instead of after
    it.  They are evaluated by the client's owner rank over the WHOLE test set (the snapshot
    exists only there before the gather); the global-model tests stay image-sharded
    (:meth:`Server._launch_eval_impl`).  Either way the ``[jobs, 3]`` counters are summed
    across ranks by the one all-reduce in :meth:`Server._finish`."""

    def __init__(self, server: "Server", plan: RoundPlan) -> None:
        self.server, self.plan = server, plan
        self.acc = torch.zeros(len(plan.jobs), 3, dtype=torch.float64, device=server.device)
        self.done: set = set()
        self.keep: List[torch.Tensor] = []     # mini-banks read by the eval stream
        self.event: Optional[torch.cuda.Event] = None   # recorded once the last one is enqueued
        owner: Dict[int, Any] = {}
        for c in plan.clients:
            for ph in c.phases:
                for sl in (ph.pre_scale_snap, ph.post_snap):
                    if sl is not None:
                        owner[sl] = c.name
        self.by_client: Dict[Any, List[int]] = {}
        for j, job in enumerate(plan.jobs):
            if job.model != 0:
                self.by_client.setdefault(owner[job.model], []).append(j)
        # on N > 1 ranks the round's longest clients (the 6-epoch attackers) finish last and
        # their owner would evaluate them alone while the other ranks idle: their tests go
        # through the image-sharded path instead (on one GPU early is still better: -2 %)
        longest = max((len(c.steps) for c in plan.clients), default=0)
        self.late = ({c.name for c in plan.clients if len(c.steps) == longest}
                     if server.d.world > 1 else set())
        # every rank marks the SAME jobs as early (the owner runs them over the whole test
        # set, the other ranks skip them), so no test image is counted twice in the
        # cross-rank counter all-reduce
        self.done = {j for name, js in self.by_client.items() if name not in self.late for j in js}

    def __call__(self, client: ClientPlan, snaps: Dict[int, torch.Tensor]) -> None:
        js = self.by_client.get(client.name)
        if not js or client.name in self.late:
            return
        slots = sorted({self.plan.jobs[j].model for j in js})
        remap = {sl: i for i, sl in enumerate(slots)}
        bank = torch.stack([snaps[sl] for sl in slots])
        jobs = [dataclasses.replace(self.plan.jobs[j], model=remap[self.plan.jobs[j].model]) for j in js]
        self.server._enqueue_eval(bank, jobs, js, self.acc, sharded=False, stream=self.server._early_stream)
        self.keep.append(bank)


def compute_dtype_for(params: C.Params, device: torch.device) -> torch.dtype:
    """Activation / GEMM precision: fp32, the reference's precision (the fp32 kernel family on
    GPU, csrc/kernels/xconv*.hip).  The round-1 bf16 fast mode and its kernel family were removed
    in round 4 (one deterministic conv family)."""
    cd = str(params["compute_dtype"]).lower()
    if cd in ("bf16", "bfloat16"):
        raise ValueError("compute_dtype bf16 was removed (round 4): the kernels are the fp32 family")
    if cd not in ("auto", "fp32", "float32"):
        raise ValueError(f"compute_dtype {cd!r}: expected fp32")
    return torch.float32


class Server:
    def __init__(self, params: C.Params, dctx: DistCtx, write_outputs: bool = True,
                 folder: Optional[str] = None) -> None:
        self.params = params
        self.d = dctx
        self.device = dctx.device
        self.dtype = compute_dtype_for(params, self.device)
        self.current_time = datetime.datetime.now().strftime("%b.%d_%H.%M.%S")
        self.name = params.get("name", C.default_dataset_name(params.type))
        self.write = write_outputs and dctx.is_main
        self.folder = folder or os.path.join(params["save_dir"], f"model_{self.name}_{self.current_time}")
        if self.write:
            os.makedirs(self.folder, exist_ok=True)
        setup_logger(self.folder if self.write else None, dctx.is_main)
        log.info(f"current path: {self.folder}")
        if not params.get("environment_name"):
            params["environment_name"] = self.name
        params["current_time"] = self.current_time
        params["folder_path"] = self.folder

        self.wl: Workload = build_workload(params, self.device)
        self.spec = self.wl.spec
        log.info("load data done")
        self._init_model()
        log.info("create model done")
        if params["is_poison"]:
            log.info(f"Poisoned following participants: {params.adversary_list}")
        self.trainer = GroupTrainer(self.wl, params, self.dtype,
                                    max_groups=int(params.get("max_concurrent_clients", 16)))
        self.evaluator = Evaluator(self.wl, self.dtype, chunk=int(params["eval_batch_size"]),
                                   max_groups=int(params.get("eval_max_groups", 24)))
        self.fg = agg.FoolsGold(bool(params["fg_use_memory"]))
        if getattr(self, "_fg_aux", None):
            self.fg.load_state(self._fg_aux)
        self.csv = CsvRecorder(self.folder, enabled=self.write)
        self.metrics = MetricsStream(os.path.join(self.folder, "metrics.jsonl")
                                     if (self.write and params["metrics_jsonl"]) else None)
        self.plot = Plotter(params["environment_name"],
                            os.path.join(self.folder, "vis_events.jsonl") if self.write else None,
                            live=bool(params["visdom"]) and self.write)
        self.plot.text(dict_html(params, self.current_time))
        self.best_loss = float("inf")
        self.timer = PhaseTimer(self.device)
        self._completed: List[Dict[str, Any]] = []    # rounds finished inside _train_half (LOAN)
        self._eval_stream = None
        self._early_stream = None
        self._unlaunched: Optional[Dict[str, Any]] = None    # trained + aggregated, eval not enqueued
        self._launched: List[Dict[str, Any]] = []             # eval enqueued, not yet recorded
        self.train_done_t: List[float] = []   # host time each round's training was collected
        if self.device.type == "cuda" and bool(params.get("overlap_eval", True)):
            # training runs on a HIGH-priority stream (its kernels are small and latency-bound,
            # they win every CU that frees up); evaluation fills the rest at default priority
            # local tests of clients that finished training get their own low-priority stream,
            # so the global tests of round r (ready at once) never queue behind the local tests
            # of round r+1 (each waiting for its client to finish)
            torch.cuda.synchronize(self.device)
            self._main_stream, self._eval_stream, self._early_stream = framework_streams(self.device)
            torch.cuda.set_stream(self._main_stream)
        if self.write:
            with open(os.path.join(self.folder, "params.yaml"), "w") as f:
                yaml.safe_dump(params.to_plain(), f)
        self.last_round: Dict[str, Any] = {}
        if not params["resumed_model"] and int(params["pretrain_central_epochs"]) > 0:
            plr = params["pretrain_lr"]
            self.pretrain_central(int(params["pretrain_central_epochs"]), float(plr) if plr is not None else None)
        if not params["resumed_model"] and int(params["pretrain_rounds"]) > 0:
            plr = params["pretrain_lr"]
            self.pretrain(int(params["pretrain_rounds"]), float(params["pretrain_eta"]),
                          float(plr) if plr is not None else None)
        if params["is_poison"]:
            # the lone-client graph (a poison round's attacker tail) captured before round 1
            self.trainer.prewarm(1)

    # ------------------------------------------------------------------ model
    def _init_model(self) -> None:
        p = self.params
        self.counter = 0
        if p["resumed_model"]:
            path = os.path.join(p["save_dir"], str(p["resumed_model_name"]))
            if not os.path.exists(path):
                raise FileNotFoundError(
                    f"resumed_model: {path} not found (pretrained checkpoints are not shipped); "
                    f"run with resumed_model=false [start_epoch=N] or pretrain first")
            flat, ep, lr, self.counter = ckpt.load_checkpoint(path, self.spec)
            self.start_epoch = ep + 1
            if lr is not None:
                p["lr"] = float(lr)
            log.info(f"Loaded parameters from saved model: LR is {p['lr']} and current epoch is {self.start_epoch}")
            aux = ckpt.load_aux(path + ".aux")
            if aux is not None:
                ckpt.restore_rng(aux["rng"], self.wl.py_rng, self.wl.np_rng)
                self._fg_aux = aux.get("foolsgold")
        else:
            flat = self.spec.init_flat(int(p["seed"]))
            self.start_epoch = int(p.get("start_epoch") or 1)
        self.global_state = flat.to(self.device)
        if self.d.enabled:   # identical by construction; make it bit-identical anyway
            self.d.broadcast_(self.global_state, 0)
        self.init_comm_bytes = self.d.take_bytes()   # one-time; rounds report their own

    def pretrain(self, rounds: int, eta: float = 1.0, lr: Optional[float] = None) -> None:
        """Benign FedAvg warm start: ``rounds`` clean rounds (no attackers, no evaluation,
        no CSV rows) with server rate ``eta`` and client learning rate ``lr`` (default: the
        config's ``lr``; the attack-phase recipes of LOAN / Tiny use a fine-tuning rate of
        1e-3 that would need hundreds of rounds to reach a converged starting point).

        The reference never trains from scratch: every shipped config resumes a pretrained
        checkpoint (``resumed_model: true``, e.g. ``cifar_pretrain/...epoch_200``) whose
        weights and BN running statistics have converged.  Those checkpoints are not in the
        repository, so a run from random init would spend its attack window with running
        statistics still far from the activations' (eval accuracy at chance).  This builds the
        equivalent starting point on the configured (real or synthetic) data; the result can
        be written with :func:`dba_mod_amd.utils.checkpoint.save_checkpoint` and resumed like a
        reference checkpoint (``dba_mod_amd.tools.pretrain``)."""
        if rounds <= 0:
            return
        p = self.params
        saved = {k: p[k] for k in ("is_poison", "eta", "aggregation_methods", "lr")}
        p.update({"is_poison": False, "eta": float(eta), "aggregation_methods": C.AGGR_MEAN})
        if lr is not None:
            p["lr"] = float(lr)
        try:
            for e in range(1, rounds + 1):
                self._train_half(e, evaluate=False)
        finally:
            p.update(saved)
            self.timer.reset()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        log.info(f"pretrained {rounds} benign rounds (eta {eta}, lr {lr if lr is not None else p['lr']})")

    def pretrain_central(self, epochs: int, lr: Optional[float] = None) -> None:
        """Centralised warm start: ``epochs`` passes of one pseudo-client holding the WHOLE
        training set (no attackers, no evaluation, no CSV rows), then the global model takes
        its weights.  This is how the reference's resumed checkpoints were made (e.g.
        ``tiny_64_pretrain/tiny-resnet.epoch_20``: 20 centralised epochs, ``utils/
        tiny_params.yaml``), and it is the only practical warm start when the federated split
        is very non-IID (Tiny: 200 Dirichlet clients at alpha 0.01 hold ~1-2 classes each).
        On N ranks every rank trains the same pseudo-client (identical by construction)."""
        if epochs <= 0:
            return
        p = self.params
        wl = self.wl
        name = "__central__"
        wl.client_indices[name] = np.arange(int(wl.train_store.labels.numel()), dtype=np.int64)
        wl.client_sizes[name] = int(wl.client_indices[name].shape[0])
        saved = {k: p[k] for k in ("is_poison", "eta", "aggregation_methods", "lr", "internal_epochs", "no_models")}
        p.update({"is_poison": False, "eta": 1.0, "aggregation_methods": C.AGGR_MEAN, "internal_epochs": int(epochs),
                  "no_models": 1})
        if lr is not None:
            p["lr"] = float(lr)
        world = self.d.world
        try:
            plan = build_round_plan(p, wl, 1, [name], [])
            handle = self.trainer.train_async(plan.clients, self.global_state)
            res = handle.collect()
            self.global_state.copy_(res[0].snapshots[plan.clients[0].final_snap])
        finally:
            p.update(saved)
            self.timer.reset()
            del wl.client_indices[name]
            del wl.client_sizes[name]
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        log.info(f"central warm start: {epochs} epochs over {len(plan.clients[0].steps)} steps "
                 f"(lr {lr if lr is not None else p['lr']}, {world} rank(s))")

    # ------------------------------------------------------------------ round
    # A round is split in two halves so consecutive rounds can overlap on the GPU:
    #   _train_half(r): select -> plan -> train -> gather -> aggregate   (training stream)
    #   _eval_half(r):  batched evaluation of round r's snapshots + the new global model,
    #                   enqueued on a LOW-priority stream, then CSV/checkpoint once it lands.
    # Round r+1's training needs only the aggregated weights, never round r's test results,
    # so the eval of round r runs underneath the (latency-bound) training of round r+1.
    def _train_begin(self, epoch: int, evaluate: bool = True) -> Dict[str, Any]:
        """Select, plan and ENQUEUE the round's local training (returns while the GPU trains)."""
        p = self.params
        t0 = time.perf_counter()
        with self.timer.phase("select"):
            agents, adversarial = select_clients(p, self.wl, epoch)
        log.info(f"Server Epoch:{epoch} choose agents : {agents}.")
        pre_acc = None
        if p.type == C.TYPE_LOAN and p["is_poison"] and not p["baseline"] and adversarial:
            self._completed.extend(self.flush())
            pre_acc = self._loan_preeval()
        with self.timer.phase("plan", sync=False):
            plan = build_round_plan(p, self.wl, epoch, agents, adversarial, pre_acc)
            costs = [c.cost for c in plan.clients]
            owners, _ = native.lpt_assign(costs, self.d.world)
            mine = [c for c, o in zip(plan.clients, owners) if o == self.d.rank]
        early = _EarlyEval(self, plan) if (evaluate and p["early_local_eval"]) else None
        load = self._window_loads(plan, owners, early) if self.d.world > 1 else None
        with self.timer.phase("train_enqueue", sync=False):
            handle = self.trainer.train_async(mine, self.global_state, on_client_done=early)
        return {"epoch": epoch, "plan": plan, "owners": owners, "adversarial": adversarial, "t0": t0,
                "handle": handle, "early": early, "clients_on_rank": len(mine), "evaluate": evaluate,
                "load": load}

    def _job_images(self, job) -> int:
        return len(self.wl.test_clean_idx if job.kind == "clean" else self.wl.test_poison_idx)

    def _window_loads(self, plan: RoundPlan, owners: List[int], early: Optional["_EarlyEval"]) -> List[float]:
        """Each rank's GPU work while round r's image-sharded tests run (round r+1's training
        and its clients' early local tests), in eval image-forward units — the base of the
        water-filling split of those tests (:meth:`_eval_shares`).  Identical on every rank
        (a pure function of the plan).  A grouped step costs ``balance_step_latency +
        balance_step_per_client * active``: the latency floor of a lone client's step
        (1.75 ms at fp32 on MI355X, ~1.2k image forwards of evaluation) is weighted double: evaluation
        kernels running beside it stretch the latency-bound chain (emulated same-box sweep:
        profiles/balance_sweep_r3/)."""
        p = self.params
        lat, per = float(p["balance_step_latency"]), float(p["balance_step_per_client"])
        world = self.d.world
        load = [0.0] * world
        lens: List[List[int]] = [[] for _ in range(world)]
        for c, o in zip(plan.clients, owners):
            lens[o].append(len(c.steps))
        for r in range(world):
            ls = sorted(lens[r], reverse=True)
            prev = 0
            for k in range(len(ls), 0, -1):      # steps with k active clients
                n = ls[k - 1] - prev
                if n > 0:
                    load[r] += n * (lat + per * k)
                    prev = ls[k - 1]
        if early is not None:
            owner_of = {c.name: o for c, o in zip(plan.clients, owners)}
            for name, js in early.by_client.items():
                if name in early.late:
                    continue
                load[owner_of[name]] += sum(self._job_images(plan.jobs[j]) for j in js)
        return load

    def _eval_balance(self) -> bool:
        """Water-filled eval shares (config ``eval_balance``; None: on where the step-cost
        constants are calibrated — the CIFAR ResNets)."""
        eb = self.params["eval_balance"]
        return self.params["type"] == C.TYPE_CIFAR if eb is None else bool(eb)

    def _eval_shares(self, jobs, base: Optional[List[float]]) -> Optional[List[float]]:
        """Per-rank shares of the image-sharded tests ``jobs``: water-filling over ``base``
        (None: the strided even split)."""
        if self.d.world <= 1 or base is None or not self._eval_balance():
            return None
        work = float(sum(self._job_images(j) for j in jobs))
        return native.balance_shares(base, work)

    def _train_end(self, st: Dict[str, Any]) -> Dict[str, Any]:
        """Wait for the round's training, gather the snapshots, aggregate."""
        p = self.params
        plan, epoch, early = st["plan"], st["epoch"], st["early"]
        with self.timer.phase("train"):
            results = st["handle"].collect()
        self.train_done_t.append(time.perf_counter())   # per-round pacing (bench "round_ms")
        if early is not None and self._early_stream is not None:
            early.event = torch.cuda.Event()        # every local test of this round is enqueued
            early.event.record(self._early_stream)
        if self.trainer.trace and self.write:
            self._plot_batches(plan, results)
        with self.timer.phase("gather"):
            bank, local, cstats = self._gather(plan, st["owners"], results, early, st.get("evaluate", True))
        with self.timer.phase("aggregate"):
            self._aggregate(plan, bank, local, st["adversarial"])
            bank[0].copy_(self.global_state)
            if p["nan_check"] and not bool(torch.isfinite(self.global_state).all()):
                # fail fast: a non-finite global model poisons every later round
                raise FloatingPointError(f"round {epoch}: aggregated global model is not finite "
                                         f"(aggregation={p['aggregation_methods']})")
        return {"epoch": epoch, "plan": plan, "bank": bank, "cstats": cstats, "t0": st["t0"],
                "clients_on_rank": st["clients_on_rank"], "phases": self.timer.reset(), "early": early,
                "comm_bytes": self.d.take_bytes()}

    def _train_half(self, epoch: int, evaluate: bool = True) -> Dict[str, Any]:
        return self._train_end(self._train_begin(epoch, evaluate))

    def _launch_eval(self, pend: Dict[str, Any], base: Optional[List[float]] = None) -> None:
        """Enqueue the round's evaluation on the eval stream (returns immediately).  ``base``:
        every rank's load in the window the tests run in (:meth:`_window_loads`)."""
        t0 = time.perf_counter()
        try:
            self._launch_eval_impl(pend, base)
        finally:
            pend["phases"]["launch_eval"] = time.perf_counter() - t0

    def _enqueue_eval(self, bank: torch.Tensor, jobs: List[Any], rows: List[int], acc: torch.Tensor,
                      sharded: bool, stream=None, shares: Optional[List[float]] = None) -> None:
        """Evaluate ``jobs`` (models = rows of ``bank``) into ``acc[rows]`` on the eval stream,
        ordered after everything already enqueued on the current (training) stream.
        ``sharded``: this rank takes its ``[rank::world]`` image shard (the all-reduce in
        :meth:`_finish` sums the shards); otherwise it evaluates every image."""
        rank, world = (self.d.rank, self.d.world) if sharded else (0, 1)
        stream = stream if stream is not None else self._eval_stream
        if stream is None:
            acc.index_add_(0, to_device(rows, self.device, torch.int64),
                           self.evaluator.run(bank, jobs, rank, world, shares))
            return
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(stream):
            # everything this eval allocates lives on the eval stream; the only training-stream
            # tensors it reads (bank, acc) are kept referenced until _finish has waited for it
            # (a freed training-stream block is reused at once by the training stream)
            stream.wait_event(ready)
            idx = to_device(rows, self.device, torch.int64)
            acc.index_add_(0, idx, self.evaluator.run(bank, jobs, rank, world, shares))

    def _launch_eval_impl(self, pend: Dict[str, Any], base: Optional[List[float]] = None) -> None:
        plan = pend["plan"]
        early = pend.get("early")
        if early is not None:
            acc, done = early.acc, early.done
        else:
            acc, done = torch.zeros(len(plan.jobs), 3, dtype=torch.float64, device=self.device), set()
        pend["acc"] = acc
        rest = [j for j in range(len(plan.jobs)) if j not in done]
        if rest:
            rjobs = [plan.jobs[j] for j in rest]
            self._enqueue_eval(pend["bank"], rjobs, rest, acc, sharded=True, shares=self._eval_shares(rjobs, base))
        if self._eval_stream is not None:
            pend["done"] = torch.cuda.Event()
            pend["done"].record(self._eval_stream)
            if early is not None and getattr(early, "event", None) is not None:
                pend["done_early"] = early.event

    def _finish(self, pend: Dict[str, Any]) -> Dict[str, Any]:
        p = self.params
        t_wait = time.perf_counter()
        acc = pend["acc"]
        for ev in ("done", "done_early"):
            if ev in pend:
                torch.cuda.current_stream(self.device).wait_event(pend[ev])
        self.d.all_reduce_(acc)
        res = acc.cpu().numpy()
        comm = dict(pend.get("comm_bytes", {}))
        for k, v in self.d.take_bytes().items():
            comm[k] = comm.get(k, 0) + v
        t_io = time.perf_counter()
        summary = self._record(pend["plan"], res, pend["cstats"])
        self._save_model(pend["epoch"], summary["val_loss"], pend["bank"][0])
        self.csv.save(bool(p["is_poison"]))
        now = time.perf_counter()
        phases = dict(pend["phases"])
        phases["eval_wait"] = t_io - t_wait
        phases["io"] = now - t_io
        summary.update({"epoch": pend["epoch"], "round_s": now - pend["t0"], "phases": phases,
                        "clients_on_rank": pend["clients_on_rank"], "backend": ops.backend_name(self.device),
                        "comm_bytes": comm})
        self.metrics.emit(summary)
        log.info(f"Done in {now - pend['t0']} sec.")
        self.last_round = summary
        return summary

    def run_round(self, epoch: int) -> Dict[str, Any]:
        """One complete round, evaluated before returning (no overlap)."""
        self.flush()
        pend = self._train_half(epoch)
        self._completed = []
        self._launch_eval(pend)
        return self._finish(pend)

    def run_rounds(self, epochs) -> List[Dict[str, Any]]:
        """Pipelined rounds.  Per iteration: enqueue round r's training (the GPU starts at
        once); then, while it runs, enqueue round r-1's global tests and record round r-2
        (its tests ran underneath round r-1's training); then wait for round r's training and
        aggregate.  The host work between two rounds' training is only gather + aggregate +
        select + plan.  Every rank runs this same sequence, so collectives stay ordered."""
        out: List[Dict[str, Any]] = []
        for epoch in epochs:
            st = self._train_begin(epoch)
            out.extend(self._completed)
            self._completed = []
            if self._unlaunched is not None:
                # round r-1's tests share the GPUs with round r's training and local tests
                self._launch_eval(self._unlaunched, base=st.get("load"))
                self._launched.append(self._unlaunched)
                self._unlaunched = None
            while len(self._launched) > 1:
                out.append(self._finish(self._launched.pop(0)))
            self._unlaunched = self._train_end(st)
        out.extend(self.flush())
        return out

    def flush(self) -> List[Dict[str, Any]]:
        """Enqueue and record every round still in flight, oldest first."""
        if self._unlaunched is not None:
            self._launch_eval(self._unlaunched)
            self._launched.append(self._unlaunched)
            self._unlaunched = None
        out = []
        while self._launched:
            out.append(self._finish(self._launched.pop(0)))
        return out

    def run(self) -> None:
        p = self.params
        epochs = list(range(self.start_epoch, int(p["epochs"]) + 1, int(p["aggr_epoch_interval"])))
        if p["max_rounds"] is not None:
            epochs = epochs[:int(p["max_rounds"])]
        self.run_rounds(epochs)
        log.info("Saving all the graphs.")
        log.info(f"This run has a label: {p['current_time']}. Visdom environment: {p['environment_name']}")

    # ---------------------------------------------------------------- helpers
    def _loan_preeval(self) -> float:
        from .plan import EvalJob
        job = EvalJob(0, "poison", self.wl.global_trigger_id, "preeval")
        acc = self.evaluator.run(self.global_state[None], [job], self.d.rank, self.d.world)
        self.d.all_reduce_(acc)
        r = acc[0].cpu().numpy()
        v = 100.0 * r[1] / max(r[2], 1)
        log.info(v)
        return float(v)

    def _rfa_gather(self, n_clients: int) -> bool:
        """RFA on the gathered final states (True) or distributed Weiszfeld (False).  Per rank,
        a ring all-gather of the n final states moves ~n*S*4 bytes, distributed Weiszfeld
        ~(maxiter+1) * 2 * (S*4 + n*8): it pays only above ~2 (maxiter+1) clients per round
        (the reference configs run 10 clients with maxiter 10 -> gather)."""
        mode = str(self.params["rfa_mode"]).lower()
        if mode not in ("auto", "gather", "distributed"):
            raise ValueError(f"rfa_mode {mode!r}: expected auto | gather | distributed")
        if self.d.world == 1 or mode == "gather":
            return True
        if mode == "distributed":
            return False
        return n_clients <= 2 * (int(self.params["geom_median_maxiter"]) + 1)

    def _gather(self, plan: RoundPlan, owners: List[int], results: List[ClientResult],
                early: Optional["_EarlyEval"], evaluate: bool
                ) -> Tuple[torch.Tensor, Dict[str, Any], Dict[Any, Dict[str, Any]]]:
        """Snapshot bank + this rank's aggregation inputs + per-client scalars on every rank.

        Client snapshots stay on their owner rank.  Only the rows some other rank reads are
        broadcast from their owners: the snapshots of clients whose tests are image-sharded across ranks
        (the round's longest clients, or every client without early local tests) and, for
        RFA in gather mode, the final states.  Aggregation itself reduces (``_aggregate``)."""
        S, P = self.spec.S, self.spec.P
        world, rank = self.d.world, self.d.rank
        by_name = {r.name: r for r in results}
        slot_owner: Dict[int, int] = {}
        for c, o in zip(plan.clients, owners):
            for ph in c.phases:
                for s in (ph.pre_scale_snap, ph.post_snap):
                    if s is not None:
                        slot_owner[s] = o
        bank = torch.zeros(plan.n_snapshots, S, dtype=torch.float32, device=self.device)
        local_snaps: Dict[int, torch.Tensor] = {}
        for r in results:
            local_snaps.update(r.snapshots)
        if world == 1:
            for s, t in local_snaps.items():
                bank[s] = t
        else:
            shared: set = set()
            if evaluate:
                done_early = early.done if early is not None else set()
                shared.update(plan.jobs[j].model for j in range(len(plan.jobs))
                              if j not in done_early and plan.jobs[j].model != 0)
            if (self.params["aggregation_methods"] == C.AGGR_GEO_MED and self._rfa_gather(len(plan.clients))):
                shared.update(c.final_snap for c in plan.clients)
            for s, t in local_snaps.items():
                bank[s] = t
            # each shared row is broadcast from its owner straight into the bank (every rank
            # receives each row once; a zero-padded all-gather of [world, k_max] rows would
            # move world x the bytes when one rank owns the round's long clients)
            for s in sorted(shared):
                self.d.broadcast_(bank[s], slot_owner[s])
        mine = [i for i, c in enumerate(plan.clients) if c.name in by_name]
        local_in: Dict[str, Any] = {
            "idx": mine,
            "finals": (torch.stack([local_snaps[plan.clients[i].final_snap] for i in mine]) if mine
                       else torch.zeros(0, S, device=self.device)),
            "fg": ({i: by_name[plan.clients[i].name].fg_grad for i in mine}
                   if self.params["aggregation_methods"] == C.AGGR_FOOLSGOLD else None),
        }
        # per-client scalars: stats [max_slots, 3] + scale distances [interval] (one small all-reduce)
        n = len(plan.clients)
        max_slots = max(sum(ph.internal_epochs for ph in c.phases) for c in plan.clients)
        interval = int(self.params["aggr_epoch_interval"])
        W = max_slots * 3 + interval * 5
        o_n = max_slots * 3 + interval
        sc = torch.zeros(n, W, dtype=torch.float64)
        for i, c in enumerate(plan.clients):
            r = by_name.get(c.name)
            if r is None:
                continue
            st = torch.from_numpy(r.stats.astype(np.float64))
            sc[i, :st.numel()] = st.reshape(-1)
            for k, ph in enumerate(c.phases):
                sc[i, max_slots * 3 + k] = r.scale_dist.get(ph.epoch, 0.0)
                nr = r.scale_norms.get(ph.epoch)
                if nr is not None:
                    sc[i, o_n + 4 * k:o_n + 4 * k + 4] = torch.tensor(nr, dtype=torch.float64)
        if self.d.enabled:
            scd = sc.to(self.device)
            self.d.all_reduce_(scd)
            sc = scd.cpu()
        cstats: Dict[Any, Dict[str, Any]] = {}
        for i, c in enumerate(plan.clients):
            st = sc[i, :max_slots * 3].reshape(max_slots, 3).numpy()
            dists = {ph.epoch: float(sc[i, max_slots * 3 + k]) for k, ph in enumerate(c.phases)}
            norms = {ph.epoch: tuple(float(v) for v in sc[i, o_n + 4 * k:o_n + 4 * k + 4])
                     for k, ph in enumerate(c.phases)}
            cstats[c.name] = {"stats": st, "dist": dists, "norms": norms}
        return bank, local_in, cstats

    def _reduce(self, t: torch.Tensor) -> torch.Tensor:
        """Sum ``t`` over ranks through a §5.8-padded flat buffer (no-op at world 1)."""
        if not self.d.enabled:
            return t
        buf = self.d.padded(t.numel(), t.dtype)
        buf[:t.numel()] = t.reshape(-1)
        self.d.all_reduce_(buf)
        return buf[:t.numel()].view(t.shape)

    def _reduce_max(self, v: float) -> float:
        """Max of a host float over ranks (no-op at world 1)."""
        return self.d.all_reduce_max(v) if self.d.enabled else v

    def _aggregate(self, plan: RoundPlan, bank: torch.Tensor, local: Dict[str, Any],
                   adversarial: List[Any]) -> None:
        p = self.params
        method = p["aggregation_methods"]
        n_upd = self.spec.S if p["aggregate_bn_buffers"] else self.spec.P
        names = [c.name for c in plan.clients]
        dp_seed = (int(p["seed"]) * 7919 + plan.epoch) & 0x7FFFFFFF
        if method == C.AGGR_MEAN:
            # each rank sums its own clients' deltas (fp64), one all-reduce of S values
            part = ops.delta_sum(local["finals"][:, :n_upd], self.global_state[:n_upd])
            agg.fedavg_apply(self.global_state, self._reduce(part), float(p["eta"]), int(p["no_models"]),
                             bool(p["diff_privacy"]), float(p["sigma"]), dp_seed, n_upd)
        elif method == C.AGGR_GEO_MED:
            ns = [c.num_samples for c in plan.clients]
            self._log_poison_ratio("rfa", names, ns)
            mun = p["max_update_norm"]
            kw = dict(max_update_norm=float(mun) if mun is not None else None)
            if self._rfa_gather(len(plan.clients)):
                finals = bank[[c.final_snap for c in plan.clients]]
                updated, wv, alphas, calls = agg.geometric_median(
                    self.global_state, finals, ns, float(p["eta"]), int(p["geom_median_maxiter"]),
                    bool(p["diff_privacy"]), float(p["sigma"]), dp_seed, n_upd, **kw)
            else:
                updated, wv, alphas, calls = agg.geometric_median_distributed(
                    self.global_state, local["finals"], local["idx"], ns, float(p["eta"]),
                    int(p["geom_median_maxiter"]), bool(p["diff_privacy"]), float(p["sigma"]), dp_seed, n_upd,
                    reduce=self._reduce, reduce_max=self._reduce_max, **kw)
            self.csv.add_weight_result(names, wv, alphas)
            self._plot_weights(names, wv, alphas, adversarial, plan.epoch)
        elif method == C.AGGR_FOOLSGOLD:
            ns = [c.num_samples for c in plan.clients]
            self._log_poison_ratio("foolsgold", names, ns)
            t0 = time.time()
            lo, hi = self.spec.fg_feature_slice()
            n = len(plan.clients)
            feats = torch.zeros(n, hi - lo, dtype=torch.float32, device=self.device)
            for i, g in local["fg"].items():
                feats[i] = g[lo:hi]
            # ONE all-reduce of the [n, d] features (each row owned by one rank: exact)
            wv, alpha = self.fg.weights_from(self._reduce(feats), names)
            idx = local["idx"]
            grads = torch.stack([local["fg"][i] for i in idx]) if idx else None
            # the fixed grid's exponent from the max |gradient| over every rank's clients
            E = agg.fixed_exponent(self._reduce_max(agg.max_abs(grads)), n)
            if idx:
                wl = torch.tensor([wv[i] / n for i in idx], dtype=torch.float32, device=self.device)
                part = agg.wsum_part(grads, wl, E)
            else:
                part = agg.wsum_zero(self.spec.P, E, self.device)
            # ONE all-reduce of the wv-weighted P-vector's int64 limbs: exact, so the aggregate's
            # bits do not depend on the world size (fp64 partials if a gradient is not finite)
            agg_grad = agg.wsum_decode(self._reduce(part), E)
            log.info(f"[foolsgold agg] wv: {wv}")
            agg.foolsgold_server_step(self.global_state, agg_grad, self.spec.P, float(p["eta"]),
                                      float(p["lr"]), float(p["decay"]))
            print("model aggregation took {}s".format(time.time() - t0))
            self.csv.add_weight_result(names, wv.tolist(), alpha.tolist())
            self._plot_weights(names, wv.tolist(), alpha.tolist(), adversarial, plan.epoch)

    def _log_poison_ratio(self, tag: str, names: List[Any], ns: List[int]) -> None:
        p = self.params
        adv = sum(n for nm, n in zip(names, ns) if p.is_adversary(nm)) / max(1, sum(ns))
        log.info(f"[{tag} agg] training data poison_ratio: {adv}  data num: {ns}")
        log.info(f"[{tag} agg] considering poison per batch poison_fraction: "
                 f"{adv * p['poisoning_per_batch'] / p['batch_size']}")

    def _plot_batches(self, plan: RoundPlan, results: List[ClientResult]) -> None:
        """Per-batch loss (benign phases: image_train.py:225-234) and distance-to-global points
        (every phase; poison phases tagged ``_poisoned``: image_train.py:107-116, 235-249)."""
        p = self.params
        by = {r.name: r for r in results}
        for c in plan.clients:
            r = by.get(c.name)
            if r is None or r.batch_trace is None:
                continue
            t = 0
            for ph in c.phases:
                n_b = (ph.end_step - t) // max(1, ph.internal_epochs)
                for ie in range(ph.internal_epochs):
                    tle = (ph.epoch - 1) * ph.internal_epochs + ie + 1
                    for bi in range(n_b):
                        loss, dist = r.batch_trace[t + ie * n_b + bi]
                        if p["vis_train_batch_loss"] and not ph.poison:
                            self.plot.line(f"train_batch_loss_{self.current_time}", (tle - 1) * n_b + bi,
                                           float(loss), str(c.name))
                        if p["batch_track_distance"]:
                            # poison phases too, tagged like simple.py:46-49 (image_train.py:107-116)
                            tag = f"{c.name}_poisoned" if ph.poison else str(c.name)
                            self.plot.line(f"global_dist_{self.current_time}", (tle - 1) * n_b + bi + 1,
                                           float(dist), tag)
                t = ph.end_step

    def _plot_weights(self, names, wv, alphas, adversarial, epoch) -> None:
        for nm, w, a in zip(names, wv, alphas):
            tag = f"{nm}_poisoned" if any(C._same_client(nm, x) for x in adversarial) else str(nm)
            self.plot.line(f"aggregation_weight_{self.current_time}", epoch, float(w), tag)
            self.plot.line(f"fg_alpha_{self.current_time}", epoch, float(a), tag)

    def _record(self, plan: RoundPlan, res: np.ndarray, cstats: Dict[Any, Dict[str, Any]]) -> Dict[str, Any]:
        p = self.params
        loan = p.type == C.TYPE_LOAN
        csv = self.csv
        out: Dict[str, Any] = {"val_loss": None}

        def jres(j: int) -> Tuple[float, float, int, int]:
            ls, corr, tot = res[j]
            tot_i = int(round(tot))
            corr_i = int(round(corr))
            loss = ls / tot if tot else 0.0
            acc = 100.0 * corr / tot if tot else 0.0
            return float(loss), float(acc), corr_i, tot_i

        cum_internal: Dict[Any, int] = {}
        for kind, payload in plan.rows:
            if kind == "train":
                name, ph, ie = payload
                st = cstats[name]["stats"][ph.stat_slot0 + ie]
                size = int(round(st[2]))
                total_l = float(st[0]) / size if size else 0.0
                acc = 100.0 * float(st[1]) / size if size else 0.0
                if loan:
                    cum_internal[name] = cum_internal.get(name, 0) + 1
                    tle = plan.epoch - 1 + cum_internal[name]
                else:
                    tle = (ph.epoch - 1) * ph.internal_epochs + ie + 1
                tag = "PoisonTrain" if ph.poison else "Train"
                log.info(f"___{tag} {self.spec.arch},  epoch {ph.epoch:3d}, local model {name}, "
                         f"internal_epoch {ie + 1:3d},  Average loss: {total_l:.4f}, "
                         f"Accuracy: {int(round(st[1]))}/{size} ({acc:.4f}%)")
                csv.train_result.append([name, tle, ph.epoch, ie + 1, total_l, acc, int(round(st[1])), size])
                if p["vis_train"]:   # model.train_vis (models/simple.py:18-30)
                    tag = f"{name}_poisoned" if ph.poison else str(name)
                    self.plot.line(f"train_acc_{self.current_time}", tle, acc, tag)
                    self.plot.line(f"train_loss_{self.current_time}", tle, total_l, tag)
            elif kind in ("test", "poison"):
                name, ep, j = payload
                loss, acc, corr, tot = jres(j)
                row = [name, ep, loss, acc, corr, tot]
                (csv.test_result if kind == "test" else csv.posiontest_result).append(row)
                log.info(f"___Test {name} poisoned: {kind == 'poison'}, epoch: {ep}: Average loss: {loss:.4f}, "
                         f"Accuracy: {corr}/{tot} ({acc:.4f}%)")
                if name == "global":
                    if kind == "test":
                        out["global_acc"], out["global_loss"] = acc, loss
                        self.plot.line(f"test_acc_{self.current_time}", ep, acc, "global")
                    else:
                        out["global_asr"], out["poison_loss"] = acc, loss
                        self.plot.line(f"poison_test_acc_{self.current_time}", ep, acc, "global")
            elif kind == "trigger":
                name, tname, ep, j = payload
                loss, acc, corr, tot = jres(j)
                csv.poisontriggertest_result.append([name, tname, "", ep, loss, acc, corr, tot])
                if name == "global":
                    out.setdefault("trigger_asr", {})[tname] = acc
                if p["vis_trigger_split_test"]:
                    self.plot.line(f"poison_trigger_acc_{self.current_time}", ep, acc, tname)
            elif kind == "scale":
                name, ph = payload
                dist = cstats[name]["dist"].get(ph.epoch, 0.0)
                g_n, pre_n, pre_d, post_n = cstats[name]["norms"].get(ph.epoch, (0.0, 0.0, 0.0, 0.0))
                csv.scale_temp_one_row.append(ph.epoch)
                csv.scale_temp_one_row.append(round(dist, 4))
                # the reference's poison-phase norm lines (image_train.py:144-146,166-183;
                # loan_train.py:148-168)
                log.info(f"Global model norm: {g_n}.")
                log.info(f"Norm before scaling: {pre_n}. Distance: {pre_d}")
                if not loan:
                    log.info("will scale.")
                log.info(f"Scaling by  {p['scale_weights_poison']}")
                log.info(f"Scaled Norm after poisoning: {post_n}, distance: {dist}")
                n_adv = sum(1 for c in plan.clients if any(q.poison for q in c.phases))
                log.info(f"Total norm for {n_adv} adversaries is: {post_n}. distance: {dist}")
            elif kind == "scale_acc":
                if csv.scale_temp_one_row:
                    csv.scale_temp_one_row.append(round(out.get("global_acc", 0.0), 4))
        if p["is_poison"] and not p["best_on_clean_loss"]:
            out["val_loss"] = out.get("poison_loss", out.get("global_loss"))   # D6
        else:
            out["val_loss"] = out.get("global_loss")
        return out

    def _save_model(self, epoch: int, val_loss: Optional[float], state: Optional[torch.Tensor] = None) -> None:
        p = self.params
        if not (self.write and p["save_model"]):
            return
        state = self.global_state if state is None else state
        log.info("saving model")
        name = os.path.join(self.folder, "model_last.pt.tar")
        ckpt.save_checkpoint(name, self.spec, state, epoch, float(p["lr"]), self.counter)
        aux = {"rng": ckpt.rng_state(self.wl.py_rng, self.wl.np_rng), "foolsgold": self.fg.state(),
               "epoch": int(epoch)}
        ckpt.save_aux(name + ".aux", aux)
        if epoch in list(p["save_on_epochs"] or []):
            log.info(f"Saving model on epoch {epoch}")
            ckpt.save_checkpoint(f"{name}.epoch_{epoch}", self.spec, state, epoch, float(p["lr"]), self.counter)
            ckpt.save_aux(f"{name}.epoch_{epoch}.aux", aux)
        if val_loss is not None and val_loss < self.best_loss:
            ckpt.save_checkpoint(f"{name}.best", self.spec, state, epoch, float(p["lr"]), self.counter)
            self.best_loss = val_loss
