"""Headline benchmark: FL rounds/s on the BASELINE.json config.

CIFAR-10 half-width ResNet-18, 100 clients (10 per round), single-shot DBA with 4
distributed attackers (rounds 203/205/207/209), FedAvg — ``configs/cifar_params.yaml`` —
on synthetic CIFAR-shaped data and random-init weights (no network: no dataset download,
no pretrained checkpoint).  One "step" is one complete FL round exactly as the reference
defines it: client selection, every client's local training (benign 2 epochs, attackers 6
poisoned epochs + model-replacement scaling), every local and global test the reference
runs (per-client clean tests, attacker poison/trigger tests, global clean + combined
trigger + 4 per-trigger ASR tests), aggregation, CSV output.  Nothing is skipped.

The reference resumes every config from a pretrained checkpoint (CIFAR: round 200) that is
not shipped; the bench builds the equivalent starting point with ``--pretrain-rounds``
(default 40) benign FedAvg rounds before the warmup (untimed, :meth:`Server.pretrain`).
Rounds then start at 201, so with the default ``--warmup 2`` the timed window 203..210
contains all four poison rounds.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     # one rank per GPU over RCCL
    python bench.py --emulate-rank R --emulate-world N    # rank R's share of N, on one GPU

Launch forms.  Under a launcher (``WORLD_SIZE`` set, torchrun) every process is one rank and
``--gpus`` must equal ``WORLD_SIZE`` (checked; a mismatch fails loudly).  Without a launcher
and ``--gpus N > 1`` this process is only a PARENT: it never imports the framework or touches
the GPU, starts ``python -m torch.distributed.run --nproc-per-node N`` as a child (N fresh
rank processes), relays rank 0's JSON line and exits with the child's status.

Strong scaling: the round's work is fixed; N GPUs split its clients (LPT) and its
evaluation images.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from typing import Optional

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "FL rounds/sec + backdoor ASR & main-task acc, ResNet-18 CIFAR-10 100 clients"
# reference design, CIFAR FL throughput ≈ 0.0085 rounds/s (8-vCPU estimate;
# the reference repo publishes no number of its own)
BASELINE_ROUNDS_PER_S = 0.0085
MODEL_NAMES = {"cifar": "ResNet-18 (half-width, CIFAR-10)", "tiny-imagenet-200": "ResNet-18 (Tiny-ImageNet-200)",
               "mnist": "MnistNet (MNIST)", "loan": "LoanNet MLP (LOAN)"}


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn_ranks(n: int, argv) -> int:
    """Parent of an N-rank run: no framework import, no GPU call, no exec.  The child
    launcher starts N fresh ranks; their stdout is streamed (non-JSON lines to stderr so
    progress stays visible) and exactly one JSON line (rank 0's) is relayed to stdout."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env, cwd=ROOT)
    lines = []
    assert proc.stdout is not None
    for ln in proc.stdout:
        if ln.startswith("{") and '"metric"' in ln:
            lines.append(ln.strip())
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = proc.wait()
    if rc != 0:
        print(f"bench.py: {n}-rank launch failed (exit {rc})", file=sys.stderr)
        return rc
    if len(lines) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 1
    out = json.loads(lines[0])
    if out.get("n_gpus") != n or out.get("world") != n:
        print(f"bench.py: ranks reported world {out.get('world')} for --gpus {n}", file=sys.stderr)
        return 1
    print(lines[0], flush=True)
    return 0


def _split_label(server) -> Optional[dict]:
    """The fp32 family's operand split on the HIP backend: the scaled fp16 pair (3 MFMAs per
    product, fp32-level error: tests/test_gpu_f32.py) on every conv pass, training and
    evaluation."""
    import torch
    from dba_mod_amd import ops
    if server.dtype != torch.float32 or ops.backend_name(server.device) != "hip":
        return None
    return {"train": "scaled fp16x2 (3 MFMA)", "eval": "scaled fp16x2 (3 MFMA)"}


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default=os.path.join(ROOT, "configs", "cifar_params.yaml"))
    ap.add_argument("--aggregation", default=None, help="override: mean | geom_median | foolsgold")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--pretrain-rounds", type=int, default=40,
                    help="benign FedAvg warm start before warmup (stand-in for the reference's "
                         "pretrained checkpoint; untimed)")
    ap.add_argument("--start-epoch", type=int, default=None,
                    help="first (warmup) round; default: first poison round - warmup")
    ap.add_argument("--dtype", choices=("fp32",), default="fp32",
                    help="compute precision: fp32, the reference's (fp32 operands split for the 16-bit MFMA)")
    ap.add_argument("--set", dest="overrides", nargs="*", default=[])
    ap.add_argument("--emulate-rank", type=int, default=None,
                    help="run only rank R's share of an --emulate-world N round on one device "
                         "(collectives are counted no-ops; per-rank critical-path timing)")
    ap.add_argument("--emulate-world", type=int, default=None)
    ap.add_argument("--dump-state", default=None,
                    help="rank 0 saves the final global model here (torch.save; cross-world tests)")
    ap.add_argument("--round-phases", action="store_true",
                    help="add every timed round's host phase times (s) to the JSON line")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    args = _args(argv)
    emulate = args.emulate_world is not None
    if emulate and args.emulate_rank is None:
        raise SystemExit("--emulate-world needs --emulate-rank")
    if "WORLD_SIZE" in os.environ:
        world_env = int(os.environ["WORLD_SIZE"])
        if emulate or world_env != args.gpus:
            raise SystemExit(f"bench.py: launched with WORLD_SIZE={world_env} but --gpus {args.gpus}"
                             + (" (--emulate-* runs without a launcher)" if emulate else ""))
    elif args.gpus > 1 and not emulate:
        return _spawn_ranks(args.gpus, argv)
    elif emulate and args.gpus != 1:
        raise SystemExit("bench.py: --emulate-* runs on one device (--gpus 1)")
    return _run(args)


def _run(args) -> int:
    import torch
    from dba_mod_amd import config as C
    from dba_mod_amd import ops
    from dba_mod_amd.fl.server import Server
    from dba_mod_amd.parallel.dist import emulated_ctx, init_distributed, shutdown

    if args.emulate_world is not None:
        dctx = emulated_ctx(args.emulate_rank, args.emulate_world, prefer_gpu=not args.cpu)
    else:
        dctx = init_distributed(prefer_gpu=not args.cpu)
    devices = dctx.gather_strings(f"{dctx.device}" + (f" ({torch.cuda.get_device_name(dctx.device)})"
                                                      if dctx.device.type == "cuda" else ""))
    over = {"resumed_model": False, "synthetic_data": True, "save_model": False,
            "pretrain_rounds": args.pretrain_rounds, "compute_dtype": args.dtype}
    if args.aggregation:
        over["aggregation_methods"] = args.aggregation
    over.update(C.parse_override(args.overrides))
    params = C.load_params(args.config, over)
    if args.start_epoch is not None:
        params["start_epoch"] = args.start_epoch
    elif "start_epoch" not in over:
        # the reference resumes from a pretrain checkpoint just before the attack window: time
        # the window (CIFAR: warmup 201-202, timed 203-210 holds all four poison rounds)
        poison = [e for i in range(len(params.adversary_list)) for e in params.poison_epochs_of(i)]
        params["start_epoch"] = max(1, (min(poison) if poison else 1 + args.warmup) - args.warmup)
    tmp = tempfile.mkdtemp(prefix="dba_bench_")
    server = Server(params, dctx, write_outputs=True, folder=tmp)
    import logging
    logging.getLogger("logger").setLevel(logging.WARNING)

    epoch = server.start_epoch
    server.run_rounds(range(epoch, epoch + args.warmup))      # pipelined, flushed at the end
    epoch += args.warmup

    def sync():
        if dctx.device.type == "cuda":
            torch.cuda.synchronize(dctx.device)
        dctx.barrier()

    sync()
    t0 = time.perf_counter()
    n_done0 = len(server.train_done_t)
    # round r's evaluation overlaps round r+1's training; the last round is fully evaluated
    # (flushed) inside the timed region, so exactly K complete rounds are timed
    done = server.run_rounds(range(epoch, epoch + args.steps))
    epoch += args.steps
    last = done[-1] if done else {}
    sync()
    elapsed = dctx.all_reduce_max(time.perf_counter() - t0)
    rps = args.steps / elapsed if elapsed > 0 else 0.0
    import hashlib
    state_sha = hashlib.sha256(server.global_state.detach().cpu().numpy().tobytes()).hexdigest()[:16]
    if args.dump_state and (dctx.is_main or dctx.emulated):
        torch.save(server.global_state.detach().cpu(), args.dump_state)
    comm_kinds = sorted({k for r in done for k in r.get("comm_bytes", {})})
    comm_mean = {k: int(round(sum(r.get("comm_bytes", {}).get(k, 0) for r in done) / max(1, len(done))))
                 for k in comm_kinds}
    if dctx.is_main or dctx.emulated:
        metric = METRIC if params.type == "cifar" else (
            f"FL rounds/sec + backdoor ASR & main-task acc, {MODEL_NAMES.get(params.type, params.type)} "
            f"{int(params['number_of_total_participants'])} clients")
        out = {
            "metric": metric, "value": round(rps, 4), "unit": "rounds/s",
            "n_gpus": 1 if dctx.emulated else dctx.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / max(1, args.steps), 2),
            "higher_is_better": True, "scaling": "strong",
            "vs_baseline": round(rps / BASELINE_ROUNDS_PER_S, 2) if params.type == "cifar" else None,
            # the kernels' precision: the server's compute dtype selects the kernel family
            # (ops/hip.py dispatches on the activation dtype and never converts)
            "dtype": {torch.bfloat16: "bf16", torch.float32: "fp32"}[server.dtype],
            "data": (f"synthetic ({params.type} shapes/class sizes); random-init weights warm-started by "
                     + (f"{int(params['pretrain_central_epochs'])} centralised epochs + "
                        if int(params["pretrain_central_epochs"]) > 0 else "")
                     + f"{args.pretrain_rounds} benign FedAvg rounds (untimed)"),
            "config": {"model": MODEL_NAMES.get(params.type, params.type),
                       "global_batch": int(params["batch_size"]) * int(params["no_models"]),
                       "seq_len": None,
                       "parallelism": (f"emulated rank {dctx.rank} of client-dp{dctx.world}" if dctx.emulated
                                       else f"client-dp{dctx.world}"),
                       "clients_total": int(params["number_of_total_participants"]),
                       "clients_per_round": int(params["no_models"]),
                       "attackers": params.adversary_list, "aggregation": params["aggregation_methods"],
                       "rounds_timed": f"{epoch - args.steps}..{epoch - 1}",
                       "baseline_source": "BASELINE.md §4 reference-design estimate 0.0085 rounds/s"},
            "world": dctx.world,
            "emulated": bool(dctx.emulated),
            "dist_backend": dctx.backend,
            "devices": devices,
            "rccl_ok": dctx.selfcheck_ok if dctx.backend == "nccl" else None,
            "collective_selfcheck_ok": dctx.selfcheck_ok,
            "backend_repinned_cpu_affinity": dctx.affinity_changed,
            "hw_queues": dctx.hw_queues, "train_stream_priority": os.environ.get("DBA_TRAIN_STREAM_PRIORITY", "-1"),
            "comm_bytes_per_round": comm_mean,
            "ops_backend": ops.backend_name(dctx.device),
            "fp32_split": _split_label(server),
            # host time between consecutive rounds' training completions (the first from the
            # window start): where in the window a rank's critical path lies (poison rounds)
            "round_ms": [round(1000.0 * (b - a), 1) for a, b in
                         zip([t0] + server.train_done_t[n_done0:-1], server.train_done_t[n_done0:])],
            "global_acc": round(float(last.get("global_acc", 0.0)), 3),
            "global_asr": round(float(last.get("global_asr", 0.0)), 3),
            "rounds": [[int(r["epoch"]), round(float(r.get("global_acc", 0.0)), 2), round(float(r.get("global_asr", 0.0)), 2)]
                       for r in done],
            # the final global model's bytes (untimed): equal across world sizes (bitwise contract)
            "state_sha": state_sha,
            "phases_mean_s": {k: round(sum(r.get("phases", {}).get(k, 0.0) for r in done) / max(1, len(done)), 4)
                              for k in (done[0].get("phases", {}) if done else {})},
        }
        if args.round_phases:
            out["phases_by_round"] = [[int(r["epoch"]), {k: round(v, 4) for k, v in r.get("phases", {}).items()}]
                                      for r in done]
        print(json.dumps(out), flush=True)
    shutdown(dctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
