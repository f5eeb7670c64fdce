"""Tiny-ResNet train step vs fp64 over several input seeds: BN statistics folded into the conv
epilogue vs the separate reduce pass (is a failure a near-tie flip or systematic?)."""
import torch
from dba_mod_amd import ops
from dba_mod_amd.ops import hip as H
from dba_mod_amd.ops import reference as R
from dba_mod_amd.models import program as P
from dba_mod_amd.models.spec import get_spec

H.set_fp32_planes(3)
dev = torch.device("cuda")
G, N = 3, 16
for arch, shp in (("resnet18_tiny", (64, 64, 3)), ("resnet18_cifar", (32, 32, 3))):
    spec = get_spec(arch)
    for seed in range(5):
        torch.manual_seed(seed)
        flat = spec.init_flat(3)
        nval = torch.tensor([N, 9, 0], dtype=torch.int32)
        x = torch.rand(G, N, *shp)
        lab = torch.randint(0, spec.num_classes, (G, N)).int()
        lab = torch.where(torch.arange(N)[None] < nval[:, None].long(), lab, torch.full_like(lab, -1))
        seeds = torch.tensor([1, 2, 3], dtype=torch.int32)

        def run(mod, d, dt):
            state = flat.to(d, dt)[None].repeat(G, 1).contiguous()
            grads = torch.zeros(G, spec.P, device=d, dtype=dt)
            saved = {k: getattr(ops, k) for k in ops._OPS}
            for k in ops._OPS:
                setattr(ops, k, getattr(mod, k))
            try:
                ctx = P.Ctx(spec, state, state, None, train=True, grads=grads, nvalid=nval.to(d),
                            dropout_seed=seeds.to(d), act_dtype=dt)
                logits = P.forward(ctx, x.to(d, dt))
                loss, _, dl = ops.softmax_xent(logits, lab.to(d), True, True, grad_dtype=dt)
                ctx.tape.backward(logits, dl)
            finally:
                for k, v in saved.items():
                    setattr(ops, k, v)
            return grads.double().cpu()

        def rel(a, b):
            return ((a - b).norm() / b.norm().clamp(min=1e-300)).item()

        H._BN_FUSED_STATS = True
        gf = run(H, dev, torch.float32)
        H._BN_FUSED_STATS = False
        gu = run(H, dev, torch.float32)
        R.COMPUTE_DTYPE = torch.float64
        gr = run(R, torch.device("cpu"), torch.float64)
        R.COMPUTE_DTYPE = torch.float32
        g32 = run(R, torch.device("cpu"), torch.float32)
        print(arch, seed, " ".join(f"g{g}: fused {rel(gf[g], gr[g]):.1e} unfused {rel(gu[g], gr[g]):.1e} "
                                   f"torch32 {rel(g32[g], gr[g]):.1e}" for g in range(2)), flush=True)
