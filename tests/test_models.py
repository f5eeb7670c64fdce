"""Functional grouped programs vs the torch.nn mirrors (reference architectures):
forward, loss, every parameter gradient, BN running stats, eval-mode BN folding, and the
checkpoint key/layout round trip."""
import pytest
import torch
import torch.nn.functional as F

from dba_mod_amd import ops
from dba_mod_amd.models import program as P
from dba_mod_amd.models.mirror import build_mirror
from dba_mod_amd.models.spec import get_spec

CASES = [("mnist", (28, 28, 1)), ("resnet18_cifar", (32, 32, 3)), ("resnet18_tiny", (64, 64, 3)),
         ("resnet34_cifar", (32, 32, 3)), ("resnet50_cifar", (32, 32, 3))]


@pytest.fixture
def fp64_reference():
    from dba_mod_amd.ops import reference
    old = reference.COMPUTE_DTYPE
    reference.COMPUTE_DTYPE = torch.float64
    yield
    reference.COMPUTE_DTYPE = old


@pytest.mark.parametrize("arch,shp", CASES)
def test_train_step_matches_autograd(arch, shp, fp64_reference):
    torch.manual_seed(0)
    spec = get_spec(arch)
    sd = build_mirror(arch).state_dict()
    flat = spec.flat_from_state_dict(sd).double()
    G, N = 2, 6
    nval = torch.tensor([N, N - 2])
    state = flat[None].repeat(G, 1).contiguous()
    x = torch.rand(G, N, *shp, dtype=torch.float64)
    lab = torch.randint(0, spec.num_classes, (G, N)).int()
    lab_m = torch.where(torch.arange(N)[None] < nval[:, None], lab, -1)
    grads = torch.zeros(G, spec.P, dtype=torch.float64)
    ctx = P.Ctx(spec, state, state, None, train=True, grads=grads, nvalid=nval, act_dtype=torch.float64)
    logits = P.forward(ctx, x)
    loss, _, dl = ops.softmax_xent(logits, lab_m, True, True)
    ctx.tape.backward(logits, dl)
    for g in range(G):
        n = int(nval[g])
        m = build_mirror(arch).double()
        m.load_state_dict(sd)
        m.train()
        out = m(x[g, :n].permute(0, 3, 1, 2))
        ref = F.cross_entropy(out, lab[g, :n].long())
        ref.backward()
        assert abs(ref.item() - loss[g].item()) < 1e-10
        gref = torch.zeros(spec.P, dtype=torch.float64)
        for name, p in m.named_parameters():
            e = spec.by_name[name]
            t = e.to_k(p.grad) if e.to_k else p.grad
            gref[e.offset:e.offset + e.numel] = t.reshape(-1)
        torch.testing.assert_close(grads[g], gref, rtol=1e-8, atol=1e-10)
        new_flat = spec.flat_from_state_dict(m.state_dict()).double()
        torch.testing.assert_close(state[g, spec.P:], new_flat[spec.P:], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("arch,shp", CASES + [("loan", (91,))])
def test_eval_folding_matches_eval_mode(arch, shp):
    torch.manual_seed(1)
    spec = get_spec(arch)
    m = build_mirror(arch)
    with torch.no_grad():   # non-trivial running stats
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.2, 0.2)
                mod.running_var.uniform_(0.5, 1.5)
    m.eval()
    flat = spec.flat_from_state_dict(m.state_dict())
    bank = torch.stack([flat, flat * 0.5])
    x = torch.rand(3, 4, *shp)
    x[2] = x[0]
    ctx = P.Ctx(spec, None, None, torch.tensor([0, 1, 0], dtype=torch.int32), train=False,
                folded=P.fold_bank(spec, bank, torch.float32))
    out = P.forward(ctx, x)
    xin = x[0] if len(shp) == 1 else x[0].permute(0, 3, 1, 2)
    ref = m(xin)
    torch.testing.assert_close(torch.log_softmax(out[0], -1), torch.log_softmax(ref, -1), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out[0], out[2])


@pytest.mark.parametrize("arch", ["mnist", "resnet18_cifar", "resnet18_tiny", "loan", "resnet34_cifar",
                                  "resnet50_cifar", "resnet101_cifar", "resnet152_cifar"])
def test_state_dict_roundtrip_and_keys(arch):
    spec = get_spec(arch)
    m = build_mirror(arch)
    sd = m.state_dict()
    flat = spec.flat_from_state_dict(sd)
    back = spec.state_dict_from_flat(flat, counter=7)
    assert list(back.keys()) == list(sd.keys())
    for k, v in sd.items():
        if k.endswith("num_batches_tracked"):
            assert int(back[k]) == 7
        else:
            assert torch.equal(back[k], v), k
    # FoolsGold feature = second-to-last parameter = final FC weight (helper.py:544)
    assert spec.params[-2].name.endswith(("linear.weight", "fc.weight", "fc2.weight", "layer3.0.weight"))


def test_param_counts_match_survey():
    # SURVEY §2.3 [measured]: parameter counts of the reference classes
    assert get_spec("mnist").n_params == 431_080
    assert get_spec("resnet18_cifar").n_params == 2_797_610
    assert sum(e.numel for e in get_spec("resnet18_cifar").buffers) == 4_800
    assert get_spec("resnet18_tiny").n_params == 11_279_112
    assert get_spec("loan").n_params == 5_529
    # rest of the CIFAR family (resnet_cifar.py:106-116), counted on the reference classes;
    # the state_dict key order/shapes were checked equal to them as well
    for a, n in (("resnet34_cifar", 5_326_506), ("resnet50_cifar", 5_899_050),
                 ("resnet101_cifar", 10_660_138), ("resnet152_cifar", 14_582_570)):
        assert get_spec(a).n_params == n, a
    for a in ("mnist", "resnet18_cifar", "resnet18_tiny", "loan"):
        s = get_spec(a)
        assert all(e.offset % 64 == 0 for e in s.params + s.buffers) and s.P % 64 == 0 and s.S % 64 == 0


def test_model_arch_selection():
    from dba_mod_amd.models.spec import arch_for_type
    assert arch_for_type("cifar") == "resnet18_cifar"
    assert arch_for_type("cifar", "resnet50_cifar") == "resnet50_cifar"
    with pytest.raises(ValueError):
        arch_for_type("mnist", "resnet50_cifar")
    with pytest.raises(ValueError):
        arch_for_type("cifar", "resnet200_cifar")
