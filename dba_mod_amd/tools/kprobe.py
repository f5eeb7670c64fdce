"""Runs a few kernels on fixed shapes for rocprofv3 PMC counter collection: conv shapes
(``f32:<shape>``: the fp32 family on a ``tools.bench_kernels`` shape) and the fused training
BN conv ``bn1``-``bn3`` (10 replicas x 64 images; ResNet stages 1-3: 32x32 x 32, 16x16 x 64,
8x8 x 128 channels: a 3x3 conv with the BN statistics in its epilogue, the lazy BN+ReLU
consumed by a second conv, and the fused backward finish), as ``scripts/gpu/pmc_bn.sh``
profiles them; ``blk`` / ``stemblk``: the fused evaluation BasicBlock of the 32-wide stage /
the stem + layer1.0 block on 17 x 1024 images (``xblock.hip``)."""
from __future__ import annotations

import sys

import torch

from dba_mod_amd.ops import bnstate as bs
from dba_mod_amd.ops import hip as H


def _bn_probe(name: str, dev) -> None:
    Hh, C = {"bn1": (32, 32), "bn2": (16, 64), "bn3": (8, 128)}[name]
    G, N = 10, 64
    x = torch.randn(G, N, Hh, Hh, C, device=dev)
    w = torch.randn(G, C, 3, 3, C, device=dev) * (1.0 / (9 * C) ** 0.5)
    per = C * 9 * C
    H.split_weights(w, per, per, H._amax_w(w, per, per))
    nv = torch.full((G,), N, dtype=torch.int32, device=dev)
    p = bs.BnParams(torch.ones(G, C, device=dev), torch.zeros(G, C, device=dev), torch.zeros(G, C, device=dev),
                    torch.ones(G, C, device=dev), torch.zeros(G, C, device=dev), torch.zeros(G, C, device=dev),
                    0.1, 1e-5)
    for _ in range(3):
        with H.amax_arena(G, dev):
            y, st = H.conv_bn_stats(x, w, None, 1, 1, nv, p, True)
            H.conv_bn_stats(bs.LazyBN(y, st, True), w, None, 1, 1, nv, p, True)
            H.bn_apply(bs.LazyBN(y, st, True), None, True, nv)


def main() -> int:
    dev = torch.device("cuda")
    which = sys.argv[1:] or ["bn1", "bn2", "bn3"]
    torch.manual_seed(0)
    for name in which:
        if name.startswith("bn"):
            _bn_probe(name, dev)
        elif name in ("blk", "stemblk"):
            G, N, C = 17, 1024, 32
            w1, w2 = [torch.randn(G, C, 3, 3, C, device=dev) * 0.06 for _ in range(2)]
            for w in (w1, w2):
                H.split_weights(w, C * 9 * C, C * 9 * C, H._amax_w(w, C * 9 * C, C * 9 * C))
            b1, b2 = torch.zeros(G, C, device=dev), torch.zeros(G, C, device=dev)
            if name == "blk":
                x = torch.relu(torch.randn(G, N, 32, 32, C, device=dev))
                for _ in range(3):
                    with H.amax_arena(G, dev):
                        H.basic_block_eval(x, w1, b1, w2, b2)
            else:
                img = torch.rand(G, N, 32, 32, 3, device=dev)
                w0 = torch.randn(G, C, 3, 3, 3, device=dev) * 0.3
                H.split_weights(w0, C * 27, C * 27, H._amax_w(w0, C * 27, C * 27))
                b0 = torch.zeros(G, C, device=dev)
                for _ in range(3):
                    with H.amax_arena(G, dev):
                        H.stem_block_eval(img, w0, b0, w1, b1, w2, b2)
        elif name.startswith("f32:"):
            # fp32-family forward of a bench_kernels shape (e.g. f32:eval.layer1), 3 calls
            from dba_mod_amd.tools.bench_kernels import SHAPES
            _, G, N, Hh, Cin, Cout, k, s, p = next(r for r in SHAPES if r[0] == name[4:])
            x = torch.randn(G, N, Hh, Hh, Cin, device=dev)
            w = torch.randn(G, Cout, k, k, Cin, device=dev) * 0.05
            per = Cout * k * k * Cin
            H.split_weights(w, per, per, H._amax_w(w, per, per))
            for _ in range(3):
                H.conv2d(x, w, None, s, p, relu=True)
        else:
            raise SystemExit(f"unknown probe {name!r} (bn1-bn3 or f32:<bench_kernels shape>)")
    torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
