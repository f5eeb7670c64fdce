"""Per-tensor comparison of one Tiny-ResNet training step (as test_fp32_train_step_vs_fp64):
BN statistics folded into the conv epilogue vs the separate reduce pass, both against the
fp64 reference on the CPU (GPU diagnostic)."""
import torch
from dba_mod_amd import ops
from dba_mod_amd.ops import hip as H
from dba_mod_amd.ops import reference as R
from dba_mod_amd.models import program as P
from dba_mod_amd.models.spec import get_spec

H.set_fp32_planes(3)
spec = get_spec("resnet18_tiny")
dev = torch.device("cuda")
G, N = 3, 16
torch.manual_seed(0)
flat = spec.init_flat(3)
nval = torch.tensor([N, 9, 0], dtype=torch.int32)
x = torch.rand(G, N, 64, 64, 3)
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
    return loss.double().cpu(), grads.double().cpu(), state.double().cpu()


import os
H._BN_FUSED_STATS = True
os.environ["DBA_BN_FUSED_DRY"] = "1"
ld, gd, sd = run(H, dev, torch.float32)
os.environ["DBA_BN_FUSED_DRY"] = "0"
lf, gf, sf = run(H, dev, torch.float32)
H._BN_FUSED_STATS = False
lu, gu, su = run(H, dev, torch.float32)
R.COMPUTE_DTYPE = torch.float64
lr, gr, sr = run(R, torch.device("cpu"), torch.float64)


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp(min=1e-300)).item()


print("loss", lf[:2].tolist(), lu[:2].tolist(), lr[:2].tolist())
for g in range(2):
    print("g", g, "grad fused", rel(gf[g], gr[g]), "unfused", rel(gu[g], gr[g]), "dry", rel(gd[g], gr[g]))
for e in spec.params + spec.buffers:
    for g in range(2):
        src = (gf, gu, gr) if e.offset < spec.P else (sf, su, sr)
        a, b, c = (t[g, e.offset:e.offset + e.numel] for t in src)
        print(g, e.name, e.kind, f"fused {rel(a, c):.2e} unfused {rel(b, c):.2e}")

# per-BN-call mean / invstd: dry (separate reduce) vs fused (epilogue partials)
rec = {}
orig = H.bn_train


def spy(tag):
    def f(y, *a, **k):
        out, mean, invstd = orig(y, *a, **k)
        rec.setdefault(tag, []).append((mean.clone(), invstd.clone(), out.clone(), hasattr(y, "_dba_bnpart")))
        return out, mean, invstd
    return f


H._BN_FUSED_STATS = True
for tag, dry in (("dry", "1"), ("fused", "0")):
    os.environ["DBA_BN_FUSED_DRY"] = dry
    H.bn_train = spy(tag)
    run(H, dev, torch.float32)
H.bn_train = orig
for i, (a, b) in enumerate(zip(rec["dry"], rec["fused"])):
    for g in range(2):
        n = int(nval[g])
        dm = ((a[0][g] - b[0][g]).abs() / a[0][g].abs().clamp(min=1e-30)).max().item()
        di = ((a[1][g] - b[1][g]).abs() / a[1][g].abs().clamp(min=1e-30)).max().item()
        do = ((a[2][g, :n] - b[2][g, :n]).abs().max()).item()
        print("bn", i, "g", g, "fusedflag", b[3], f"mean {dm:.2e} invstd {di:.2e} out {do:.2e}")
