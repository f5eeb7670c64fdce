"""Per-step time of the persistent LoanNet trainer (csrc/kernels/mlp.hip): G clients x T
synthetic steps in one launch, timed with HIP events (one warm-up launch first).

    python -m dba_mod_amd.tools.bench_mlp [--G 10] [--T 400] [--fg]
"""
from __future__ import annotations

import argparse
import json

import numpy as np
import torch

from dba_mod_amd.models.spec import get_spec
from dba_mod_amd.ops import hip as H


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=10)
    ap.add_argument("--T", type=int, default=400)
    ap.add_argument("--rows", type=int, default=200000)
    ap.add_argument("--fg", action="store_true")
    ap.add_argument("--prof", action="store_true", help="per-phase clock deltas of client 0 (cycles)")
    args = ap.parse_args(argv)
    dev = torch.device("cuda")
    spec = get_spec("loan")
    G, T, B = args.G, args.T, 64
    rng = np.random.default_rng(0)
    D = G * B + 8 * G
    sched = np.zeros((T, D), dtype=np.int32)
    sched[:, :G * B] = rng.integers(0, args.rows, size=(T, G * B))
    f8 = sched[:, G * B:].reshape(T, 8, G)
    f8[:, 0] = 10          # poison_n
    f8[:, 1] = -1          # trig
    f8[0, 2] = 1           # first
    f8[:, 3] = 1           # active
    f8[:, 4] = B           # nvalid
    f8[:, 5] = 0           # slot
    f8[:, 6] = rng.integers(0, 2 ** 31 - 1, size=(T, G))
    f8[:, 7] = np.float32(0.001).view(np.int32)
    sched_d = torch.from_numpy(sched).to(dev)
    state = spec.init_flat(0)[None].repeat(G, 1).to(dev).contiguous()
    mom = torch.zeros(G, spec.P, device=dev)
    fg = torch.zeros(G, spec.P, device=dev) if args.fg else None
    rows = torch.rand(args.rows, 91, device=dev)
    labels = torch.randint(0, 9, (args.rows,), dtype=torch.int32, device=dev)
    tc = torch.zeros(1, 2, dtype=torch.int32, device=dev)
    tv = torch.zeros(1, 2, device=dev)
    stats = torch.zeros(3, G, device=dev)
    nan = torch.zeros(1, device=dev)

    prof = torch.zeros(T, 8, dtype=torch.int64, device=dev) if args.prof else None

    def run(t1, p=None):
        return H.mlp_train(spec, sched_d, 0, t1, B, state, mom, fg, rows, labels, tc, tv, 7, stats, 1, nan, 0.9, 5e-4,
                           prof=p)

    assert run(min(T, 8)) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run(T)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    print(json.dumps({"G": G, "T": T, "fg": bool(args.fg), "ms": round(ms, 3), "us_per_step": round(1e3 * ms / T, 2)}))
    if prof is not None:
        run(T, prof)
        torch.cuda.synchronize()
        c = prof.cpu().numpy().astype(np.float64)
        d = np.diff(np.concatenate([c[:-1, 6:7], c[1:, :7]], 1), axis=1)   # phase k: clock[k] - clock[k-1]
        names = ["gather/stage+sync", "layer1", "layer2", "layer3+loss", "d(layer2)", "d(layer1)+W3", "W1/W2 grads+SGD"]
        print(json.dumps({"phase_cycles_median": {n: float(np.median(d[:, i])) for i, n in enumerate(names)}}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
