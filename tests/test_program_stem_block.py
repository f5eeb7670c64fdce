"""Evaluation wiring of the fused stem + first BasicBlock (``Ctx.stem_block``) on CPU: with a
backend that takes the fused op (here the reference composition standing in for
``ops.hip.stem_block_eval``), the CIFAR ResNet program skips layer1.0 in its block loop and
produces the same logits as the unfused program (reference ``models/resnet_cifar.py:80-94``)."""
import torch

from dba_mod_amd import ops
from dba_mod_amd.models import program as P
from dba_mod_amd.models.spec import get_spec
from dba_mod_amd.ops import reference


def _logits(spec, bank, x, sel, nval, fused, monkeypatch):
    calls = []
    if fused:
        monkeypatch.setattr(ops, "stem_block_ok", lambda x, w0, w1, w2: True)

        def eval_(*a, **k):
            calls.append(a[0].shape)
            return reference.stem_block_eval(*a, **k)
        monkeypatch.setattr(ops, "stem_block_eval", eval_)
    ctx = P.Ctx(spec, None, None, sel, train=False, folded=P.fold_bank(spec, bank, torch.float32),
                nvalid=nval, act_dtype=torch.float32)
    out = P.forward(ctx, x)
    monkeypatch.undo()
    return out, calls


def test_stem_block_wiring_matches_unfused(monkeypatch):
    spec = get_spec("resnet18_cifar")
    torch.manual_seed(0)
    bank = torch.stack([spec.init_flat(1), spec.init_flat(2)])
    g = torch.Generator().manual_seed(3)
    for e in spec.params:
        if e.kind not in ("conv_w", "lin_w"):
            v = spec.view(bank, e.name)
            v += 0.1 * torch.randn(v.shape, generator=g)
    bank[:, spec.P:] = bank[:, spec.P:] + 0.05 * torch.rand(bank[:, spec.P:].shape, generator=g)
    x = torch.rand(2, 3, 32, 32, 3)
    sel = torch.tensor([0, 1], dtype=torch.int32)
    nval = torch.tensor([3, 2], dtype=torch.int32)
    ref, _ = _logits(spec, bank, x, sel, nval, False, monkeypatch)
    got, calls = _logits(spec, bank, x, sel, nval, True, monkeypatch)
    assert calls == [x.shape], "the fused op runs once, on the images"
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1, :2], ref[1, :2])
