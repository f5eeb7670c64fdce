"""Kernel microbenchmarks on the real ResNet-18 (CIFAR) layer shapes.

Times each HIP conv kernel family on the shapes the FL round actually runs — evaluation
(17 folded-BN client models x 1024 images) and grouped training (10 clients x 64 images) —
and prints achieved TFLOP/s, so kernel changes are judged on the chip, not guessed.

    python -m dba_mod_amd.tools.bench_kernels [--reps 20] [--json out.json]
"""
from __future__ import annotations

import argparse
import json

import torch

from dba_mod_amd.ops import hip as H

# name, G, N, H, Cin, Cout, k, stride, pad
SHAPES = [
    ("eval.layer1", 17, 1024, 32, 32, 32, 3, 1, 1),
    ("eval.layer2", 17, 1024, 16, 64, 64, 3, 1, 1),
    ("eval.layer3", 17, 1024, 8, 128, 128, 3, 1, 1),
    ("eval.layer4", 17, 1024, 4, 256, 256, 3, 1, 1),
    ("eval.l2.0.conv1", 17, 1024, 32, 32, 64, 3, 2, 1),
    ("eval.l3.0.conv1", 17, 1024, 16, 64, 128, 3, 2, 1),
    ("eval.l4.0.conv1", 17, 1024, 8, 128, 256, 3, 2, 1),
    ("eval.l2.0.sc", 17, 1024, 32, 32, 64, 1, 2, 0),
    ("eval.l3.0.sc", 17, 1024, 16, 64, 128, 1, 2, 0),
    ("eval.l4.0.sc", 17, 1024, 8, 128, 256, 1, 2, 0),
    ("eval.stem", 17, 1024, 32, 3, 32, 3, 1, 1),
    ("train.layer1", 10, 64, 32, 32, 32, 3, 1, 1),
    ("train.layer2", 10, 64, 16, 64, 64, 3, 1, 1),
    ("train.layer3", 10, 64, 8, 128, 128, 3, 1, 1),
    ("train.layer4", 10, 64, 4, 256, 256, 3, 1, 1),
    ("train.stem", 10, 64, 32, 3, 32, 3, 1, 1),
    ("train.l2.0.conv1", 10, 64, 32, 32, 64, 3, 2, 1),
    ("train.l2.0.sc", 10, 64, 32, 32, 64, 1, 2, 0),
    ("train.l3.0.conv1", 10, 64, 16, 64, 128, 3, 2, 1),
    ("train.l3.0.sc", 10, 64, 16, 64, 128, 1, 2, 0),
    ("train.l4.0.conv1", 10, 64, 8, 128, 256, 3, 2, 1),
    ("train.l4.0.sc", 10, 64, 8, 128, 256, 1, 2, 0),
    ("eval.tiny.stem", 1, 1024, 64, 3, 64, 7, 2, 3),  # Tiny-ImageNet 7x7/2 stem, an eval chunk
    ("tiny.stem", 1, 64, 64, 3, 64, 7, 2, 3),       # Tiny-ImageNet 7x7/2 stem, a lone client
    ("tiny.stem10", 10, 64, 64, 3, 64, 7, 2, 3),    # ... 10 clients
]


def _time(fn, reps, inner=10):
    """GPU time per call: `inner` calls are captured in one HIP graph and replayed (the FL
    round replays its kernels the same way), so host and graph-launch overhead do not count."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(inner):
            fn()
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * inner) * 1e-3


def _bench_fp32(name, G, N, Hh, Cin, Cout, k, s, p, reps, dev):
    """fwd / dgrad / wgrad of the fp16-pair fp32 family; TFLOP/s counts the real fp32 work."""
    torch.manual_seed(0)
    x = torch.randn(G, N, Hh, Hh, Cin, device=dev)
    w = torch.randn(G, Cout, k, k, Cin, device=dev) * 0.05
    Ho = (Hh + 2 * p - k) // s + 1
    dy = torch.randn(G, N, Ho, Ho, Cout, device=dev)
    flops = 2.0 * G * N * Ho * Ho * Cout * k * k * Cin
    rec = {"shape": name, "dtype": "fp32"}
    if name.startswith("eval"):
        # evaluation weights are static: split into fp16-pair planes once (as bn_fold does)
        per = Cout * k * k * Cin
        H.split_weights(w, per, per, H._amax_w(w, per, per))
    ops = [("fwd", lambda: H.conv2d(x, w, None, s, p, relu=True))]
    if name == "eval.tiny.stem":   # the exact-FMA stem kernel it replaces in evaluation

        def fma_fwd():
            prev, H._EVAL_STEM_MFMA = H._EVAL_STEM_MFMA, False
            try:
                return H.conv2d(x, w, None, s, p, relu=True)
            finally:
                H._EVAL_STEM_MFMA = prev
        ops.append(("fwd_fma", fma_fwd))

        def nopad_fwd():
            prev, H._EVAL_STEM_PAD = H._EVAL_STEM_PAD, False
            try:
                return H.conv2d(x, w, None, s, p, relu=True)
            finally:
                H._EVAL_STEM_PAD = prev
        ops.append(("fwd_nopad", nopad_fwd))
    block_flops = None
    if name.startswith("eval") and H.basic_block_ok(x, w, w):
        # the whole identity BasicBlock (two convs, the mid activation in LDS: xblock.hip); its
        # TFLOP/s counts both convs' fp32 work
        xb = torch.relu(x)
        w2 = torch.randn(G, Cout, k, k, Cin, device=dev) * 0.05
        H.split_weights(w2, per, per, H._amax_w(w2, per, per))
        b1, b2 = torch.randn(G, Cout, device=dev) * 0.1, torch.randn(G, Cout, device=dev) * 0.1
        xb._dba_amax = H._amax_act(xb, None)
        block_flops = 2 * flops
        ops.append(("block", lambda: H.basic_block_eval(xb, w, b1, w2, b2)))
    if name == "eval.stem":
        # the stem + layer1.0 (xblock.hip STEM variant) vs the stem launch + fused block; their
        # TFLOP/s count the stem's and both block convs' fp32 work
        wb = [torch.randn(G, 32, 3, 3, 32, device=dev) * 0.05 for _ in range(2)]
        for wi in wb:
            H.split_weights(wi, 9216, 9216, H._amax_w(wi, 9216, 9216))
        b0, b1, b2 = [torch.randn(G, 32, device=dev) * 0.1 for _ in range(3)]
        if H.stem_block_ok(x, w, *wb):
            block_flops = flops + 2 * 2.0 * G * N * 32 * 32 * 32 * 9 * 32
            ops += [("stem_then_block", lambda: H.basic_block_eval(H.conv2d(x, w, None, 1, 1, bias=b0, relu=True),
                                                                 wb[0], b1, wb[1], b2)),
                    ("stem_block", lambda: H.stem_block_eval(x, w, b0, wb[0], b1, wb[1], b2))]
    if name.startswith("train"):
        wt = H.prepare_dgrad_weights(w, [(w, None, s, p, (Hh, Hh), None, G)])[0]
        dw = torch.zeros(G, Cout, k, k, Cin, device=dev)
        ops += [("dgrad", lambda: H.conv2d_dgrad(dy, w, None, s, p, (Hh, Hh), wt=wt)),
                ("wgrad", lambda: H.conv2d_wgrad(dy, x, s, p, k, k, dw))]
    if name.startswith("tiny.stem"):   # the stem's weight gradient (the stem has no data gradient)
        dw = torch.zeros(G, Cout, k, k, Cin, device=dev)
        ops.append(("wgrad", lambda: H.conv2d_wgrad(dy, x, s, p, k, k, dw)))
    for tag, fn in ops:
        t = _time(fn, reps)
        rec[tag + "_us"] = round(t * 1e6, 1)
        rec[tag + "_tflops"] = round((block_flops if tag in ("block", "stem_block", "stem_then_block") else flops)
                                     / t / 1e12, 1)
    return rec


def _bench_down(name, G, N, W, C, C2, reps, dev):
    """A downsampling block's conv2 + 1x1 stride-2 shortcut: fused (one launch, xconv.hpp
    dba_xdown_fwd) vs the shortcut conv + conv2 with a residual epilogue; TFLOP/s counts both
    convs' fp32 work."""
    torch.manual_seed(0)
    a = torch.relu(torch.randn(G, N, W, W, C, device=dev))
    x2 = torch.relu(torch.randn(G, N, 2 * W, 2 * W, C2, device=dev))
    w2 = torch.randn(G, C, 3, 3, C, device=dev) * 0.03
    wsc = torch.randn(G, C, 1, 1, C2, device=dev) * 0.1
    for w in (w2, wsc):
        per = w[0].numel()
        H.split_weights(w, per, per, H._amax_w(w, per, per))
    b2, bsc = torch.randn(G, C, device=dev) * 0.1, torch.randn(G, C, device=dev) * 0.1
    a._dba_amax, x2._dba_amax = H._amax_act(a, None), H._amax_act(x2, None)
    flops = 2.0 * G * N * W * W * C * (9 * C + C2)
    rec = {"shape": name, "dtype": "fp32"}
    ops = [("fused", lambda: H.down_block_eval(a, w2, b2, x2, wsc, bsc)),
           ("two", lambda: H.conv2d(a, w2, None, 1, 1, bias=b2, relu=True,
                                    residual=H.conv2d(x2, wsc, None, 2, 0, bias=bsc)))]
    for tag, fn in ops:
        t = _time(fn, reps)
        rec[tag + "_us"] = round(t * 1e6, 1)
        rec[tag + "_tflops"] = round(flops / t / 1e12, 1)
    return rec


def _bench_eval_chunk(G, N, reps, dev):
    """The whole BN-folded CIFAR ResNet-18 evaluation forward of G models x N images (the
    evaluator's chunk: 17 x 1024), through the model program as the round runs it."""
    from dba_mod_amd.models import program as P
    from dba_mod_amd.models.spec import get_spec
    spec = get_spec("resnet18_cifar")
    torch.manual_seed(0)
    bank = torch.stack([spec.init_flat(i) for i in range(G)]).to(dev)
    bank[:, spec.P:] += 0.05 * torch.rand_like(bank[:, spec.P:])
    folded = P.fold_bank(spec, bank, torch.float32)
    x = torch.rand(G, N, 32, 32, 3, device=dev)
    x._dba_amax = H._unit_amax(G, dev)
    sel = torch.arange(G, dtype=torch.int32, device=dev)
    nval = torch.full((G,), N, dtype=torch.int32, device=dev)

    def fwd():
        ctx = P.Ctx(spec, None, None, sel, train=False, folded=folded, nvalid=nval, act_dtype=torch.float32)
        with H.amax_arena(G, dev):
            return P.forward(ctx, x)

    t = _time(fwd, reps, inner=1)
    return {"shape": f"eval.chunk.{G}x{N}", "dtype": "fp32", "fwd_ms": round(t * 1e3, 3),
            "fwd_tflops": round(G * N * 17.83e9 / 64 / t / 1e12, 1)}


DOWN = [("eval.l2.0.down", 17, 1024, 16, 64, 32)]

# softmax cross-entropy (loss.hip): G groups x B rows x C classes — Tiny-ImageNet's evaluation
# chunk and training step, CIFAR's evaluation chunk and training step
XENT = [("xent.tiny.eval", 1, 1024, 200), ("xent.tiny.train", 10, 64, 200), ("xent.cifar.eval", 17, 1024, 10),
        ("xent.cifar.train", 10, 64, 10)]


def _bench_xent(name, G, B, C, reps, dev):
    torch.manual_seed(0)
    logits = torch.randn(G, B, C, device=dev) * 3
    labels = torch.randint(0, C, (G, B), device=dev, dtype=torch.int32)
    t_grad = _time(lambda: H.softmax_xent(logits, labels, True, True, grad_dtype=torch.float32), reps)
    t_eval = _time(lambda: H.softmax_xent(logits, labels, False, False), reps)
    prev = H._L.dba_xent_r5_set(1)   # the round-5 kernel form (a thread per row, a block per group)
    try:
        t_grad5 = _time(lambda: H.softmax_xent(logits, labels, True, True, grad_dtype=torch.float32), reps)
        t_eval5 = _time(lambda: H.softmax_xent(logits, labels, False, False), reps)
    finally:
        H._L.dba_xent_r5_set(prev)
    return {"shape": name, "G": G, "B": B, "C": C, "train_us": round(t_grad * 1e6, 2),
            "eval_us": round(t_eval * 1e6, 2), "r5_train_us": round(t_grad5 * 1e6, 2),
            "r5_eval_us": round(t_eval5 * 1e6, 2)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default="", help="substring filter on shape names")
    args = ap.parse_args(argv)
    dev = torch.device("cuda")
    rows = []
    for name, G, N, Hh, Cin, Cout, k, s, p in SHAPES:
        if args.only not in name:
            continue
        rows.append(_bench_fp32(name, G, N, Hh, Cin, Cout, k, s, p, args.reps, dev))
        print(json.dumps(rows[-1]), flush=True)
    for name, G, N, W, C, C2 in DOWN:
        if args.only in name:
            rows.append(_bench_down(name, G, N, W, C, C2, args.reps, dev))
            print(json.dumps(rows[-1]), flush=True)
    for name, G, B, C in XENT:
        if args.only in name:
            rows.append(_bench_xent(name, G, B, C, args.reps, dev))
            print(json.dumps(rows[-1]), flush=True)
    if args.only in "eval.chunk":
        rows.append(_bench_eval_chunk(17, 1024, max(3, args.reps // 4), dev))
        print(json.dumps(rows[-1]), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
