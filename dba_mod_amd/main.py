"""CLI: ``python main.py --params configs/cifar_params.yaml [--set key=value ...]``.

Same entry point and YAML schema as the reference (``main.py:84-111``).  Launch one process
per GPU with ``torchrun --nproc-per-node N main.py --params ...`` for client-parallel runs.
"""
from __future__ import annotations

import argparse
import random
import sys
import time

import numpy as np
import torch

from . import config as C
from .fl.server import Server
from .parallel.dist import init_distributed, shutdown


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description="DBA federated backdoor simulator (MI355X-native)")
    ap.add_argument("--params", dest="params", required=True, help="YAML config (reference schema)")
    ap.add_argument("--set", dest="overrides", nargs="*", default=[], help="key=value overrides")
    ap.add_argument("--cpu", action="store_true", help="run on CPU even if a GPU is visible")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    args = parse_args(argv)
    print("Start training")
    t0 = time.time()
    params = C.load_params(args.params, C.parse_override(args.overrides))
    # reference seeding: python random / torch = 1 at import, numpy = 1 in __main__
    random.seed(int(params["seed"]))
    np.random.seed(int(params["seed"]))
    torch.manual_seed(int(params["seed"]))
    dctx = init_distributed(prefer_gpu=not args.cpu)
    try:
        server = Server(params, dctx)
        server.run()
    finally:
        shutdown(dctx)
    if dctx.is_main:
        print(f"total {time.time() - t0:.1f}s")
    return 0


if __name__ == "__main__":
    sys.exit(main())
