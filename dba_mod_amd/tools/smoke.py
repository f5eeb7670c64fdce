"""One tiny grouped train step + eval forward of the CIFAR ResNet-18 (driver smoke test)."""
from __future__ import annotations

import time

import torch

from .. import ops
from ..models import program as prog
from ..models.spec import get_spec


def run_smoke(device: torch.device, G: int = 2, N: int = 8) -> dict:
    spec = get_spec("resnet18_cifar")
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    state = spec.init_flat(0).to(device)[None].repeat(G, 1).contiguous()
    wcomp = state if dtype == torch.float32 else state[:, :spec.P].to(dtype).contiguous()
    grads = torch.zeros(G, spec.P, device=device)
    mom = torch.zeros(G, spec.P, device=device)
    src = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device=device)
    labels = torch.randint(0, 10, (64,), dtype=torch.int32, device=device)
    idx = torch.arange(G * N, dtype=torch.int32, device=device).view(G, N)
    masks = torch.zeros(1, 32, 32, dtype=torch.uint8, device=device)
    masks[0, 0, :6] = 1
    trig = torch.tensor([0, -1], dtype=torch.int32, device=device)[:G]
    pn = torch.tensor([3, 0], dtype=torch.int32, device=device)[:G]
    nvalid = torch.full((G,), N, dtype=torch.int32, device=device)
    t0 = time.time()
    x, y = ops.gather_images(src, labels, idx, masks, trig, pn, 2, None, dtype)
    ctx = prog.Ctx(spec, state, wcomp, None, train=True, grads=grads, nvalid=nvalid, act_dtype=dtype)
    logits = prog.forward(ctx, x)
    loss, correct, dl = ops.softmax_xent(logits, y, True, True)
    ctx.tape.backward(logits, dl)
    lr = torch.full((G,), 0.1, device=device)
    one = torch.ones(G, dtype=torch.int32, device=device)
    ops.sgd_step(state[:, :spec.P], grads, mom, lr, one, one, 0.9, 5e-4,
                 shadow=(wcomp if wcomp is not state else None))
    folded = prog.fold_bank(spec, state, dtype)
    ectx = prog.Ctx(spec, None, None, torch.arange(G, dtype=torch.int32, device=device), train=False,
                    folded=folded, nvalid=nvalid, act_dtype=dtype)
    el = prog.forward(ectx, x)
    if device.type == "cuda":
        torch.cuda.synchronize()
    out = {"device": str(device), "backend": ops.backend_name(device), "loss": loss.float().tolist(),
           "grad_norm": float(grads.norm()), "eval_logits_finite": bool(torch.isfinite(el.float()).all()),
           "seconds": round(time.time() - t0, 3)}
    assert all(torch.isfinite(loss.float())), out
    assert out["grad_norm"] > 0 and out["eval_logits_finite"], out
    return out
