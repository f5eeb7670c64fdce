"""Which backward op of the Tiny-ResNet step first diverges for the partly valid replica when
the BN statistics are folded into the conv epilogue (fused) vs not (dry)?"""
import os
import torch
from dba_mod_amd import ops
from dba_mod_amd.ops import hip as H
from dba_mod_amd.models import program as P
from dba_mod_amd.models.spec import get_spec

H.set_fp32_planes(3)
import sys
ARCH = sys.argv[1] if len(sys.argv) > 1 else "resnet18_tiny"
spec = get_spec(ARCH)
SHP = (64, 64, 3) if "tiny" in ARCH else (32, 32, 3)
dev = torch.device("cuda")
G, N = 3, 16
torch.manual_seed(0)
flat = spec.init_flat(3)
nval = torch.tensor([N, 9, 0], dtype=torch.int32, device=dev)
x = torch.rand(G, N, *SHP).to(dev)
lab = torch.randint(0, spec.num_classes, (G, N)).int()
lab = torch.where(torch.arange(N)[None] < nval.cpu()[:, None].long(), lab, torch.full_like(lab, -1)).to(dev)
seeds = torch.tensor([1, 2, 3], dtype=torch.int32, device=dev)
names = ["conv2d", "bn_train", "conv2d_dgrad", "bn_train_bwd", "maxpool2d", "maxpool2d_bwd", "relu_mask_bwd"]
rec = {}


def spy(tag, name):
    f0 = getattr(H, name)

    def f(*a, **k):
        r = f0(*a, **k)
        t = r[0] if isinstance(r, tuple) else r
        rec.setdefault(tag, []).append((name, t.clone()))
        return r
    return f


H._BN_FUSED_STATS = True
for tag, dry in (("dry", "1"), ("fused", "0")):
    os.environ["DBA_BN_FUSED_DRY"] = dry
    saved = {n: getattr(H, n) for n in names}
    for n in names:
        setattr(H, n, spy(tag, n))
    state = flat.to(dev)[None].repeat(G, 1).contiguous()
    grads = torch.zeros(G, spec.P, device=dev)
    ctx = P.Ctx(spec, state, state, None, train=True, grads=grads, nvalid=nval, dropout_seed=seeds)
    logits = P.forward(ctx, x)
    loss, _, dl = ops.softmax_xent(logits, lab, True, True, grad_dtype=torch.float32)
    ctx.tape.backward(logits, dl)
    torch.cuda.synchronize()
    for n, f in saved.items():
        setattr(H, n, f)
for i, ((n, a), (_, b)) in enumerate(zip(rec["dry"], rec["fused"])):
    row = [n, str(tuple(a.shape))]
    for g in range(2):
        nv = int(nval[g])
        av, bv = a[g, :nv].double(), b[g, :nv].double()
        row.append(f"g{g} {((av - bv).norm() / av.norm().clamp(min=1e-30)).item():.2e}")
    print(i, *row)
first = None
for i, ((n, a), (_, b)) in enumerate(zip(rec["dry"], rec["fused"])):
    for g in range(2):
        nv = int(nval[g])
        av, bv = a[g, :nv].double(), b[g, :nv].double()
        if ((av - bv).norm() / av.norm().clamp(min=1e-30)).item() > 1e-4 and first is None:
            first = (i, g)
print("first divergent op", first)
if first is not None:
    i0, g = first
    for i in (i0 - 1, i0):
        (n, a), (_, b) = rec["dry"][i], rec["fused"][i]
        nv = int(nval[g])
        d = (a[g, :nv] - b[g, :nv]).abs()
        print(i, n, "max diff per image", [f"{v:.1e}" for v in d.flatten(1).max(1).values.tolist()])
        flat = d.flatten()
        top = flat.topk(5)
        print(i, n, "top-5 diffs", [f"{v:.2e}" for v in top.values.tolist()],
              "n > 1e-5:", int((flat > 1e-5).sum()), "of", flat.numel())
