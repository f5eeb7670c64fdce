"""Runs a few kernels on fixed shapes for rocprofv3 PMC counter collection: conv shapes (``f32:<shape>``:
the fp32 family on a ``tools.bench_kernels`` shape) and the
training BN forward / backward ``bn1``-``bn3`` (10 replicas x 64 images; ResNet stages 1-3:
32x32 x 32, 16x16 x 64, 8x8 x 128 channels), as ``scripts/gpu/pmc_bn.sh`` profiles them."""
from __future__ import annotations

import sys

import torch

from dba_mod_amd.ops import hip as H


def main() -> int:
    dev = torch.device("cuda")
    which = sys.argv[1:] or ["pconv1", "pconv2", "pw2", "pw3", "pw4"]
    torch.manual_seed(0)
    for name in which:
        if name.startswith("bn"):
            # training-mode BN forward + backward at a 10-client group's stage shapes
            Hh, C = {"bn1": (32, 32), "bn2": (16, 64), "bn3": (8, 128)}[name]
            G, N = 10, 64
            y = torch.randn(G, N, Hh, Hh, C, device=dev).bfloat16()
            gamma = torch.ones(G, C, device=dev)
            beta = torch.zeros(G, C, device=dev)
            rm = torch.zeros(G, C, device=dev)
            rv = torch.ones(G, C, device=dev)
            nv = torch.full((G,), N, dtype=torch.int32, device=dev)
            dout = torch.randn_like(y)
            dg = torch.zeros(G, C, device=dev)
            db = torch.zeros(G, C, device=dev)
            for _ in range(3):
                out, mean, invstd = H.bn_train(y, gamma, beta, rm, rv, nv, 0.1, 1e-5, True, None)
                H.bn_train_bwd(dout, y, out, mean, invstd, gamma, nv, True, dg, db)
        elif name.startswith("f32:"):
            # fp32-family forward of a bench_kernels shape (e.g. f32:eval.layer1), 3 calls
            from dba_mod_amd.tools.bench_kernels import SHAPES
            _, G, N, Hh, Cin, Cout, k, s, p = next(r for r in SHAPES if r[0] == name[4:])
            H.set_fp32_planes(H.F16_PAIR)
            x = torch.randn(G, N, Hh, Hh, Cin, device=dev)
            w = torch.randn(G, Cout, k, k, Cin, device=dev) * 0.05
            per = Cout * k * k * Cin
            H.split_weights(w, per, per, H._amax_w(w, per, per))
            for _ in range(3):
                H.conv2d(x, w, None, s, p, relu=True)
        elif name.startswith("pconv"):
            G, N, Hh, C = (17, 1024, 32, 32) if name == "pconv1" else (17, 1024, 16, 64)
            x = torch.randn(G, N, Hh, Hh, C, device=dev).bfloat16()
            w = (torch.randn(G, C, 3, 3, C, device=dev) * 0.05).bfloat16()
            for _ in range(3):
                H.conv2d(x, w, None, 1, 1, relu=True)
        else:
            Hh, C = {"pw1": (32, 32), "pw2": (16, 64), "pw3": (8, 128), "pw4": (4, 256)}[name]
            G, N = 10, 64
            x = torch.randn(G, N, Hh, Hh, C, device=dev).bfloat16()
            dy = torch.randn(G, N, Hh, Hh, C, device=dev).bfloat16()
            dw = torch.zeros(G, C, 3, 3, C, device=dev)
            for _ in range(3):
                H.conv2d_wgrad(dy, x, 1, 1, 3, 3, dw)
    torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
