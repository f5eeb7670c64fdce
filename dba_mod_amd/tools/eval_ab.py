"""A/B check of the round pipeline on one GPU: the same CIFAR attack window run with early
local evaluation on and off (and twice off, for run-to-run determinism); prints every
evaluation row of the attacker and the global model so the variants can be diffed.

    python -m dba_mod_amd.tools.eval_ab [--rounds 201 202 203]
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import tempfile

import torch

from .. import config as C
from ..fl.server import Server
from ..parallel.dist import DistCtx

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(early: bool, rounds, pretrain: int) -> dict:
    tmp = tempfile.mkdtemp(prefix="dba_ab_")
    p = C.load_params(os.path.join(ROOT, "configs", "cifar_params.yaml"),
                      {"resumed_model": False, "synthetic_data": True, "pretrain_rounds": pretrain,
                       "start_epoch": rounds[0], "save_dir": tmp, "early_local_eval": early})
    s = Server(p, DistCtx(device=torch.device("cuda")), write_outputs=True)
    pre = s.global_state.clone()
    s.run_rounds(rounds)
    out = {"pretrained_norm": float(pre.norm()), "final_norm": float(s.global_state.norm())}
    for name in ("test_result.csv", "posiontest_result.csv"):
        with open(os.path.join(s.folder, name)) as f:
            out[name] = [[r["model"], r["epoch"], round(float(r["accuracy"]), 4)] for r in csv.DictReader(f)]
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, nargs="*", default=[201, 202, 203])
    ap.add_argument("--pretrain", type=int, default=40)
    args = ap.parse_args(argv)
    res = {"off1": run(False, args.rounds, args.pretrain), "off2": run(False, args.rounds, args.pretrain),
           "on": run(True, args.rounds, args.pretrain)}
    for k, v in res.items():
        print(k, json.dumps(v))
    print("off1==off2", res["off1"] == res["off2"], "off1==on", res["off1"] == res["on"])
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
