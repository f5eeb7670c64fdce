"""Times the grouped training step (HIP-graph replay) of one real FL round, per step, and
groups the step times by the number of active clients — the latency-bound regime (a lone
attacker finishing its 6 poison epochs) vs the throughput regime (10 clients).

    python -m dba_mod_amd.tools.bench_step [--config configs/cifar_params.yaml] [--epoch 203]
"""
from __future__ import annotations

import argparse
import collections
import json
import os

import numpy as np
import torch

from .. import config as C
from ..fl.plan import build_round_plan, select_clients
from ..fl.server import Server
from ..parallel.dist import DistCtx
from ..utils import native
from ..utils.devcopy import to_device

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=os.path.join(ROOT, "configs", "cifar_params.yaml"))
    ap.add_argument("--epoch", type=int, default=203)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--clients", type=int, default=0,
                    help="keep only the k longest clients (k=1: the lone-attacker latency regime)")
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32")
    ap.add_argument("--split", default=None,
                    help="split-K policy target,min_k,max_s,kslab_max (ops.hip.set_split_policy)")
    ap.add_argument("--rccl", action="store_true",
                    help="create a world-1 RCCL communicator first (one all-reduce): its effect on step time")
    args = ap.parse_args(argv)
    dev = torch.device("cuda")
    if args.split:
        from ..ops import hip as H
        H.set_split_policy(*[int(v) for v in args.split.split(",")])
    if args.rccl:
        from ..parallel.dist import init_distributed
        os.environ.update(DBA_FORCE_PG="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29561"))
        assert init_distributed().selfcheck_ok
    p = C.load_params(args.config, {"resumed_model": False, "synthetic_data": True, "overlap_eval": False,
                                    "start_epoch": args.epoch, "compute_dtype": args.dtype})
    s = Server(p, DistCtx(device=dev), write_outputs=False)
    tr = s.trainer
    agents, adv = select_clients(p, s.wl, args.epoch)
    plan = build_round_plan(p, s.wl, args.epoch, agents, adv)
    clients = plan.clients
    if args.clients > 0:
        clients = sorted(clients, key=lambda c: -len(c.steps))[:args.clients]
    G = len(clients)
    max_slots = max(sum(ph.internal_epochs for ph in c.phases) for c in clients)
    max_slots = 1 << (max_slots - 1).bit_length()
    b = tr._buffers(G, max_slots)
    T = max(len(c.steps) for c in clients)
    host = native.pack_steps(clients, G, tr.B, T, max_slots)
    sched = to_device(host, dev)
    active = host[:, G * tr.B + 3 * G:G * tr.B + 4 * G].sum(1)
    b._cur = sched[0]
    tr._reset(b, s.global_state)
    tr._run_step(b)                       # capture
    tr._reset(b, s.global_state)
    times = collections.defaultdict(list)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(T)]
    for _ in range(args.reps):
        for t in range(T):
            b.desc.copy_(sched[t], non_blocking=True)
            ev[t][0].record()
            tr._run_step(b)
            ev[t][1].record()
        torch.cuda.synchronize()
        for t in range(T):
            times[int(active[t])].append(ev[t][0].elapsed_time(ev[t][1]))
    out = {"steps": int(T), "groups": G, "dtype": args.dtype, "split": args.split,
           "ms_per_step_by_active": {k: round(float(np.median(v)), 3) for k, v in sorted(times.items())},
           "steps_by_active": {k: len(v) // args.reps for k, v in sorted(times.items())}}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
