"""Diagnostic: one training step of an architecture through the HIP kernels vs the fp64
reference under branch replay (as tests/test_gpu_f32.py test_fp32_train_step_vs_fp64), for a
list of replica fills; prints per-replica gradient error, torch-fp32's band, flips / hard."""
import sys
import torch
from dba_mod_amd import ops
from dba_mod_amd.models import program as P
from dba_mod_amd.models.spec import get_spec
from dba_mod_amd.ops import hip, reference as R
from dba_mod_amd.ops.branches import BranchReplay


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp(min=1e-30)).item()


def main(arch, shp, fills, N=16):
    spec = get_spec(arch)
    G = len(fills)
    torch.manual_seed(0)
    flat = spec.init_flat(3)
    nval = torch.tensor(fills, dtype=torch.int32)
    x = torch.rand(G, N, *shp)
    lab = torch.randint(0, spec.num_classes, (G, N)).int()
    lab = torch.where(torch.arange(N)[None] < nval[:, None].long(), lab, torch.full_like(lab, -1))
    seeds = torch.arange(1, G + 1, dtype=torch.int32)

    def run(mod, d, dt, over=None):
        state = flat.to(d, dt)[None].repeat(G, 1).contiguous()
        grads = torch.zeros(G, spec.P, device=d, dtype=dt)
        saved = {k: getattr(ops, k) for k in ops._OPS}
        for k in ops._OPS:
            setattr(ops, k, (over or {}).get(k, getattr(mod, k)))
        try:
            ctx = P.Ctx(spec, state, state, None, train=True, grads=grads, nvalid=nval.to(d), dropout_seed=seeds.to(d),
                        act_dtype=dt)
            logits = P.forward(ctx, x.to(d, dt))
            loss, _, dl = ops.softmax_xent(logits, lab.to(d), True, True, grad_dtype=dt)
            ctx.tape.backward(logits, dl)
        finally:
            for k, v in saved.items():
                setattr(ops, k, v)
        return loss, grads, state

    br = BranchReplay(nval)
    lh, gh, sh = run(hip, torch.device("cuda"), torch.float32, br.wrap(hip))
    br.start_replay()
    R.COMPUTE_DTYPE = torch.float64
    lr_, gr, sr = run(R, torch.device("cpu"), torch.float64, br.wrap(R))
    print(arch, fills, "flips", br.flips, "hard", br.hard, "elements", br.elements)
    R.COMPUTE_DTYPE = torch.float32
    br.start_replay()
    _, g32, _ = run(R, torch.device("cpu"), torch.float32, br.wrap(R))
    R.COMPUTE_DTYPE = torch.float64
    for g in range(G):
        if fills[g] == 0:
            continue
        e, band = rel(gh[g], gr[g]), rel(g32[g], gr[g])
        worst = []
        for p in spec.params:
            sl = slice(p.offset, p.offset + p.numel)
            worst.append((rel(gh[g, sl], gr[g, sl]), p.name))
        worst.sort(reverse=True)
        print(f"  g{g} fill {fills[g]}: err {e:.3e} band {band:.3e} loss {lh[g].item():.6f}/{lr_[g].item():.6f} "
              f"worst {[(f'{a:.1e}', n) for a, n in worst[:4]]}")


if __name__ == "__main__":
    arch = sys.argv[1] if len(sys.argv) > 1 else "resnet50_cifar"
    shp = (64, 64, 3) if "tiny" in arch else (32, 32, 3)
    for fills in ([16, 9, 0], [9], [16], [12, 9]):
        main(arch, shp, fills)
