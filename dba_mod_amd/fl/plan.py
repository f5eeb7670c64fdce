"""Per-round plan: client selection, per-client step schedules, snapshots, eval jobs.

Every rank computes the identical plan from the identical RNG streams (no communication);
the plan is what makes the round *data-parallel over clients*: each client is a fixed list
of SGD steps that can run on any rank, concurrently with other clients.

Reference semantics reproduced here:

* selection — ``main.py:139-165`` (three modes; python ``random.sample`` on the same lists in
  the same order, so the selected ids match the reference for the same seed);
* per-client local rounds ``[epoch, epoch + aggr_epoch_interval)`` — ``image_train.py:50``;
* poison phase — ``internal_poison_epochs`` epochs at ``poison_lr`` with the reference's
  ``MultiStepLR([0.2E, 0.8E], 0.1)`` quirk (float milestones only fire when integral; the
  image trainer steps the scheduler after each internal epoch, the LOAN trainer before,
  ``image_train.py:118-120`` / ``loan_train.py:90-92``), fresh momentum, the first
  ``poisoning_per_batch`` samples of each batch stamped (``image_helper.py:306-319``);
* benign phase — ``internal_epochs`` epochs at ``lr`` (momentum persists across benign
  phases of the same client, ``image_train.py:33-35``);
* the evaluation jobs and CSV rows of ``image_train.py:148-299`` / ``loan_train.py:219-261``
  and ``main.py:198-231``.
"""
from __future__ import annotations

import copy
import zlib
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .. import config as C
from .workload import Workload


# ---------------------------------------------------------------------- selection
def select_clients(params: C.Params, wl: Workload, epoch: int) -> Tuple[List[Any], List[Any]]:
    """Returns (agent_name_keys, adversarial_name_keys) for the round starting at ``epoch``."""
    rng = wl.py_rng
    agents = list(wl.participants_list)
    adversarial: List[Any] = []
    adv_list = params.adversary_list
    if params["is_random_namelist"]:
        if params["is_random_adversary"]:
            agents = rng.sample(wl.participants_list, int(params["no_models"]))
            adversarial = [a for a in agents if any(C._same_client(a, x) for x in adv_list)]
        else:
            ongoing = list(range(epoch, epoch + int(params["aggr_epoch_interval"])))
            for idx, adv in enumerate(adv_list):
                for oe in ongoing:
                    if oe in params.poison_epochs_of(idx) and adv not in adversarial:
                        adversarial.append(adv)
            nonattacker = [copy.deepcopy(a) for a in adv_list if a not in adversarial]
            benign_num = int(params["no_models"]) - len(adversarial)
            picked = rng.sample(list(wl.benign_namelist) + nonattacker, benign_num)
            agents = adversarial + picked
    else:
        if not params["is_random_adversary"]:
            adversarial = copy.deepcopy(adv_list)
    return agents, adversarial


# --------------------------------------------------------------------------- plan
@dataclass
class StepRec:
    idx: np.ndarray           # int32 sample indices (<= batch_size)
    poison_n: int
    trig: int                 # trigger-bank slot, -1 = none
    lr: float
    first: bool               # fresh optimizer -> momentum buffer := d_p
    slot: int                 # train-stat slot (one per internal epoch)


@dataclass
class PhasePlan:
    epoch: int
    poison: bool
    internal_epochs: int
    stat_slot0: int
    end_step: int = 0
    pre_scale_snap: Optional[int] = None   # snapshot slot of the pre-scale model
    post_snap: Optional[int] = None        # snapshot slot of the model at phase end
    lr_schedule: List[float] = field(default_factory=list)


@dataclass
class ClientPlan:
    name: Any
    order: int
    adv_index: int            # index in adversary_list (or -1)
    train_trigger: int        # trigger-bank slot used while poisoning
    agent_trigger: int        # trigger-bank slot of this agent's own local trigger
    in_adv_list: bool
    phases: List[PhasePlan]
    steps: List[StepRec]
    num_samples: int
    seed: int
    final_snap: int = -1

    @property
    def cost(self) -> int:
        return sum(len(s.idx) for s in self.steps) or 1


@dataclass
class EvalJob:
    model: int                # snapshot slot (0 = new global model)
    kind: str                 # 'clean' | 'poison'
    trig: int                 # trigger-bank slot for poison jobs
    tag: str                  # human label


@dataclass
class RoundPlan:
    epoch: int
    agents: List[Any]
    adversarial: List[Any]
    clients: List[ClientPlan]
    n_snapshots: int          # snapshot slots (slot 0 reserved for the new global model)
    jobs: List[EvalJob]
    rows: List[Tuple[str, Any]]   # deferred CSV rows: (kind, payload with job ids)
    needs_preeval_asr: bool = False


def _multistep_lrs(base: float, n: int, step_before: bool) -> List[float]:
    """lr used in each internal epoch under the reference's MultiStepLR quirk."""
    milestones = {0.2 * n: 1, 0.8 * n: 1}
    out, lr, last = [], base, 0

    def advance(lr_: float, last_: int) -> Tuple[float, int]:
        last_ += 1
        hits = sum(c for m, c in milestones.items() if m == last_)
        return lr_ * (0.1 ** hits), last_

    for _ in range(n):
        if step_before:
            lr, last = advance(lr, last)
            out.append(lr)
        else:
            out.append(lr)
            lr, last = advance(lr, last)
    return out


def _client_seed(base: int, epoch: int, name: Any) -> int:
    return zlib.crc32(f"{base}|{epoch}|{name}".encode()) & 0x7FFFFFFF


def build_round_plan(params: C.Params, wl: Workload, epoch: int,
                     agents: List[Any], adversarial: List[Any],
                     loan_preeval_acc: Optional[float] = None) -> RoundPlan:
    is_poison = bool(params["is_poison"])
    adv_list = params.adversary_list
    bs = int(params["batch_size"])
    ppb = int(params["poisoning_per_batch"])
    interval = int(params["aggr_epoch_interval"])
    loan = params.type == C.TYPE_LOAN
    baseline = bool(params["baseline"])

    n_snap = 1
    clients: List[ClientPlan] = []
    needs_pre = False
    for order, name in enumerate(agents):
        adv_index = -1
        poison_epochs = list(params.get("poison_epochs") or [])
        in_adv = is_poison and any(C._same_client(name, a) for a in adv_list)
        if in_adv:
            adv_index = params.adversary_index(name)
            poison_epochs = params.poison_epochs_of(adv_index)
        train_adv_index = -1 if (in_adv and len(adv_list) == 1) else adv_index
        agent_trig_index = params.adversary_index(name)   # Mytest_poison_agent_trigger
        seed = _client_seed(int(params["seed"]), epoch, name)
        shard = wl.client_indices[name]
        rs = np.random.RandomState(seed)
        phases: List[PhasePlan] = []
        steps: List[StepRec] = []
        slot = 0
        benign_started = False
        for e in range(epoch, epoch + interval):
            poison = in_adv and (e in poison_epochs)
            if poison:
                n_int = int(params["internal_poison_epochs"])
                base_lr = float(params["poison_lr"])
                if loan and not baseline:
                    needs_pre = True
                    acc = loan_preeval_acc if loan_preeval_acc is not None else 0.0
                    if acc > 20:
                        base_lr /= 5
                    if acc > 60:
                        base_lr /= 10
                lrs = (_multistep_lrs(base_lr, n_int, step_before=loan) if params["poison_step_lr"]
                       else [base_lr] * n_int)
                first_of_phase = True
            else:
                n_int = int(params["internal_epochs"])
                lrs = [float(params["lr"])] * n_int
                first_of_phase = not benign_started
                benign_started = True
            ph = PhasePlan(e, poison, n_int, slot, lr_schedule=lrs)
            for ie in range(n_int):
                perm = shard[rs.permutation(shard.shape[0])] if shard.shape[0] else shard
                for b0 in range(0, perm.shape[0], bs):
                    bidx = perm[b0:b0 + bs].astype(np.int32)
                    pn = min(ppb, bidx.shape[0]) if poison else 0
                    trig = wl.trigger_id(train_adv_index) if poison else -1
                    steps.append(StepRec(bidx, pn, trig, lrs[ie], first_of_phase, slot))
                    first_of_phase = False
                slot += 1
            ph.end_step = len(steps)
            if poison and not baseline:
                ph.pre_scale_snap = n_snap
                n_snap += 1
            ph.post_snap = n_snap
            n_snap += 1
            phases.append(ph)
        cp = ClientPlan(name, order, adv_index, wl.trigger_id(train_adv_index),
                        wl.trigger_id(agent_trig_index), in_adv, phases, steps,
                        int(shard.shape[0]), seed)
        cp.final_snap = phases[-1].post_snap
        clients.append(cp)

    jobs: List[EvalJob] = []
    rows: List[Tuple[str, Any]] = []

    def job(model: int, kind: str, trig: int, tag: str) -> int:
        jobs.append(EvalJob(model, kind, trig, tag))
        return len(jobs) - 1

    gtrig = wl.global_trigger_id
    local_eval = bool(params["local_eval"])
    for cp in clients:
        for ph in cp.phases:
            for ie in range(ph.internal_epochs):
                rows.append(("train", (cp.name, ph, ie)))
            if local_eval:
                if ph.poison and not baseline and not loan:
                    rows.append(("test", (cp.name, ph.epoch, job(ph.pre_scale_snap, "clean", -1, f"{cp.name}/pre"))))
                    rows.append(("poison", (cp.name, ph.epoch, job(ph.pre_scale_snap, "poison", gtrig, f"{cp.name}/pre-p"))))
                if ph.poison and not baseline:
                    rows.append(("scale", (cp.name, ph)))
                if (not ph.poison) or loan:
                    rows.append(("test", (cp.name, ph.epoch, job(ph.post_snap, "clean", -1, f"{cp.name}/clean"))))
                if is_poison:
                    if ph.poison:
                        rows.append(("poison", (cp.name, ph.epoch, job(ph.post_snap, "poison", gtrig, f"{cp.name}/p"))))
                    if cp.in_adv_list:
                        rows.append(("trigger", (cp.name, f"{cp.name}_trigger", ph.epoch,
                                                 job(ph.post_snap, "poison", cp.agent_trigger, f"{cp.name}/agent"))))
            elif ph.poison and not baseline:
                rows.append(("scale", (cp.name, ph)))

    temp_global_epoch = epoch + interval - 1
    rows.append(("test", ("global", temp_global_epoch, job(0, "clean", -1, "global/clean"))))
    rows.append(("scale_acc", None))
    if is_poison:
        pj = job(0, "poison", gtrig, "global/combine")
        rows.append(("poison", ("global", temp_global_epoch, pj)))
        rows.append(("trigger", ("global", "combine", temp_global_epoch, pj)))
        if len(adv_list) == 1:
            if params["centralized_test_trigger"]:
                for j in range(int(params["trigger_num"])):
                    rows.append(("trigger", ("global", f"global_in_index_{j}_trigger", epoch,
                                             job(0, "poison", j, f"global/t{j}"))))
        else:
            for a in adv_list:
                ai = params.adversary_index(a)
                rows.append(("trigger", ("global", f"global_in_{a}_trigger", epoch,
                                         job(0, "poison", wl.trigger_id(ai), f"global/{a}"))))
    return RoundPlan(epoch, list(agents), list(adversarial), clients, n_snap, jobs, rows, needs_pre)
