"""torch.library registration (ops/library.py): every ``torch.ops.dba.*`` op runs the CPU
reference for CPU tensors and matches a direct call of the reference implementation."""
import torch

from dba_mod_amd import ops  # noqa: F401  (registers the dba:: ops)
from dba_mod_amd.ops import library as L
from dba_mod_amd.ops import reference as R


def test_registered_schemas():
    for name in L.OPS:
        assert hasattr(torch.ops.dba, name), name
    sch = str(torch.ops.dba.sgd_step.default._schema)
    assert "Tensor(a0!) params" in sch and "Tensor(a2!) mom" in sch, sch   # declared mutations


def test_cpu_dispatch_matches_reference():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 3, 8, 8, 4, generator=g)
    w = torch.randn(3, 5, 3, 3, 4, generator=g) * 0.2
    wsel = torch.tensor([2, 0], dtype=torch.int32)
    b = torch.randn(3, 5, generator=g)
    nv = torch.tensor([3, 2], dtype=torch.int32)
    y = torch.ops.dba.conv2d(x, w, wsel, 1, 1, b, None, True, nv)
    assert torch.equal(y, R.conv2d(x, w, wsel, 1, 1, bias=b, relu=True, nvalid=nv))
    dy = torch.randn(y.shape, generator=g)
    assert torch.equal(torch.ops.dba.conv2d_dgrad(dy, w, wsel, 1, 1, 8, 8, nv, None),
                       R.conv2d_dgrad(dy, w, wsel, 1, 1, (8, 8), nvalid=nv))
    dw1, dw2 = torch.zeros(2, 5, 3, 3, 4), torch.zeros(2, 5, 3, 3, 4)
    torch.ops.dba.conv2d_wgrad(dy, x, 1, 1, 3, 3, dw1, None, nv)
    R.conv2d_wgrad(dy, x, 1, 1, 3, 3, dw2, None, nvalid=nv)
    assert torch.equal(dw1, dw2) and dw1.abs().sum() > 0
    logits = torch.randn(2, 6, 10, generator=g)
    lab = torch.randint(0, 10, (2, 6), generator=g).int()
    for a, r in zip(torch.ops.dba.softmax_xent(logits, lab, True), R.softmax_xent(logits, lab, True, True)):
        assert torch.equal(a, r)
    pts = torch.randn(4, 300, generator=g)
    m = torch.randn(300, generator=g)
    assert torch.equal(torch.ops.dba.sq_dists(pts, m), R.sq_dists(pts, m))
    wts = torch.rand(4, generator=g)
    assert torch.equal(torch.ops.dba.weighted_sum(pts, wts), R.weighted_sum(pts, wts))
    assert torch.equal(torch.ops.dba.gram(pts), R.gram(pts))
    assert torch.equal(torch.ops.dba.delta_sum(pts, m), R.delta_sum(pts, m))


def test_mutating_ops():
    g = torch.Generator().manual_seed(1)
    p1 = torch.randn(2, 50, generator=g)
    p2 = p1.clone()
    grads = torch.randn(2, 50, generator=g)
    m1, m2 = torch.zeros(2, 50), torch.zeros(2, 50)
    lr = torch.tensor([0.1, 0.05])
    one = torch.ones(2, dtype=torch.int32)
    torch.ops.dba.sgd_step(p1, grads, m1, lr, one, one, 0.9, 5e-4)
    R.sgd_step(p2, grads, m2, lr, one, one, 0.9, 5e-4)
    assert torch.equal(p1, p2) and torch.equal(m1, m2)
    x = torch.randn(2, 3, 4, 4, 8, generator=g)
    w = torch.randn(2, 8, 3, 3, 8, generator=g) * 0.2
    gamma, beta = torch.rand(2, 8, generator=g) + 0.5, torch.randn(2, 8, generator=g) * 0.1
    rm1, rv1, rm2, rv2 = torch.zeros(2, 8), torch.ones(2, 8), torch.zeros(2, 8), torch.ones(2, 8)
    nv = torch.tensor([3, 2], dtype=torch.int32)
    y1, c1 = torch.ops.dba.conv_bn_stats(x, w, None, 1, 1, nv, gamma, beta, rm1, rv1, 0.1, 1e-5)
    from dba_mod_amd.ops.bnstate import BnParams, BnStat, LazyBN
    z = torch.zeros(2, 8)
    y2, st2 = R.conv_bn_stats(x, w, None, 1, 1, nv, BnParams(gamma, beta, rm2, rv2, z, z.clone(), 0.1, 1e-5), False)
    assert torch.equal(y1, y2) and torch.equal(c1, st2.coef)
    assert torch.equal(rm1, rm2) and torch.equal(rv1, rv2) and rm1.abs().sum() > 0
    o1 = torch.ops.dba.bn_apply(y1, c1, None, True, nv)
    o2 = R.bn_apply(LazyBN(y2, BnStat(st2.coef, None), False), None, True, nv)
    assert torch.equal(o1, o2)
