"""Build a pretrained starting checkpoint (stand-in for the reference's shipped-elsewhere
``*_pretrain/...`` checkpoints that every config resumes from).

Runs ``--rounds`` benign FedAvg rounds (no attackers, no evaluation) on the configured data
and writes a reference-layout checkpoint ``{'state_dict','epoch','lr'}`` (+ ``.aux`` RNG
state) that ``resumed_model: true`` / ``resumed_model_name`` resumes exactly like a
reference checkpoint:

    python -m dba_mod_amd.tools.pretrain --params configs/cifar_params.yaml --rounds 200 \\
        --out saved_models/cifar_pretrain/model_last.pt.tar.epoch_200
"""
from __future__ import annotations

import argparse
import os
import sys

from .. import config as C
from ..fl.server import Server
from ..parallel.dist import init_distributed, shutdown
from ..utils import checkpoint as ckpt


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--params", required=True)
    ap.add_argument("--rounds", type=int, default=50)
    ap.add_argument("--eta", type=float, default=1.0)
    ap.add_argument("--lr", type=float, default=None, help="client lr of the warm start (default: pretrain_lr / lr)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--set", dest="overrides", nargs="*", default=[])
    args = ap.parse_args(argv)
    over = {"resumed_model": False, "pretrain_rounds": 0}
    over.update(C.parse_override(args.overrides))
    params = C.load_params(args.params, over)
    dctx = init_distributed(prefer_gpu=not args.cpu)
    server = Server(params, dctx, write_outputs=False)
    plr = args.lr if args.lr is not None else params["pretrain_lr"]
    server.pretrain(args.rounds, args.eta, float(plr) if plr is not None else None)
    if dctx.is_main:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        ckpt.save_checkpoint(args.out, server.spec, server.global_state, args.rounds, float(params["lr"]),
                             server.counter)
        ckpt.save_aux(args.out + ".aux", {"rng": ckpt.rng_state(server.wl.py_rng, server.wl.np_rng),
                                          "foolsgold": None, "epoch": int(args.rounds)})
        print(f"wrote {args.out} (epoch {args.rounds})")
    shutdown(dctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
