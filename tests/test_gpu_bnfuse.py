"""Training BatchNorm fused into the fp32 conv family (csrc/kernels/bnfuse.hpp) vs the fp64
oracle, and its determinism contract (GPU only).

* forward: conv + BN statistics in one launch (halo, implicit-GEMM, split-K in-launch and
  separate-reduce, stem), lazy BN(+ReLU) A operands, the stored block output;
* backward: the fused ReLU mask + BN reductions in the data-gradient epilogue (stride 1) and
  the standalone pass (stride 2, pooled gradient), the weight gradient staging dy = A d + B y + K
  from (d, y) and x from a lazy BN output;
* bits: a replica's statistics and coefficients do not depend on how many replicas share the
  launch (G = 1 vs G = 3), and repeated launches are bitwise equal.
Reference semantics: BatchNorm2d train mode, /root/reference/models/resnet_cifar.py:31-36.
"""
import pytest
import torch

from dba_mod_amd.ops import bnstate as bs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dba_mod_amd.ops import hip
    yield hip


@pytest.fixture()
def R64():
    from dba_mod_amd.ops import reference
    old = reference.COMPUTE_DTYPE
    reference.COMPUTE_DTYPE = torch.float64
    yield reference
    reference.COMPUTE_DTYPE = old


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp(min=1e-30)).item()


def _params(G, C, dev, dt, seed=1):
    g = torch.Generator().manual_seed(seed)
    flat = torch.zeros(G, 4 * C + 8, dtype=dt)
    flat[:, :C] = torch.rand(G, C, generator=g, dtype=torch.float64).to(dt) + 0.5
    flat[:, C:2 * C] = torch.randn(G, C, generator=g, dtype=torch.float64).to(dt) * 0.1
    flat[:, 2 * C:3 * C] = torch.randn(G, C, generator=g, dtype=torch.float64).to(dt) * 0.1
    flat[:, 3 * C:4 * C] = torch.rand(G, C, generator=g, dtype=torch.float64).to(dt) + 0.5
    flat = flat.to(dev)
    grads = torch.zeros(G, 2 * C + 8, dtype=dt, device=dev)
    return flat, grads, bs.BnParams(flat[:, :C], flat[:, C:2 * C], flat[:, 2 * C:3 * C], flat[:, 3 * C:4 * C],
                                    grads[:, :C], grads[:, C:2 * C], 0.1, 1e-5)


# G, N, H, W, Cin, Cout, k, stride, pad
FWD = [
    (2, 4, 32, 32, 32, 32, 3, 1, 1),     # stage-1 halo conv
    (2, 3, 16, 16, 64, 64, 3, 1, 1),     # stage-2 halo conv
    (2, 4, 32, 32, 32, 64, 3, 2, 1),     # strided implicit GEMM
    (2, 4, 32, 32, 32, 64, 1, 2, 0),     # 1x1 shortcut
    (1, 64, 8, 8, 128, 128, 3, 1, 1),    # lone client stage 3: split-K, in-launch combine
    (3, 64, 4, 4, 256, 256, 3, 1, 1),    # grouped stage 4: split-K, separate reduce + standalone pass
    (3, 5, 32, 32, 3, 32, 3, 1, 1),      # CIFAR stem
    (2, 3, 64, 64, 3, 64, 7, 2, 3),      # Tiny stem
]


def _x(case, dev, seed=0):
    G, N, Hh, Ww, Cin, Cout, k, s, p = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(G, N, Hh, Ww, Cin, generator=g).to(dev)
    w = (torch.randn(G, Cout, k, k, Cin, generator=g) * (1.0 / (k * k * Cin) ** 0.5)).to(dev)
    nvalid = torch.tensor([N] + [max(1, N - 3)] * (G - 1), dtype=torch.int32, device=dev)
    return x, w, nvalid


@pytest.mark.parametrize("case", FWD)
@pytest.mark.parametrize("lazy_in", [False, True])
def test_conv_bn_stats_and_lazy_operand(H, R64, case, lazy_in):
    """conv + fused statistics (mean / 1/std / running stats / scale / shift / max / min), with
    the input a lazy BN+ReLU output; then the stored output relu(BN(y) + residual)."""
    G, N, Hh, Ww, Cin, Cout, k, s, p = case
    if lazy_in and Cin < 4:
        pytest.skip("the stem reads images")
    dev = torch.device("cuda")
    x, w, nvalid = _x(case, dev)
    xin, xin_r = x, x.double().cpu()
    if lazy_in:   # x is relu(BN(x0)) of a previous BN, never stored
        _, _, p0 = _params(G, Cin, dev, torch.float32, seed=7)
        st0 = H._bnf_fwd(p0, True, G, N * Hh * Ww, Cin, dev)[1]
        _, _, p0r = _params(G, Cin, "cpu", torch.float64, seed=7)
        # the previous BN's coefficients: same values on both sides
        coef = torch.zeros(G, bs.ROWS, Cin)
        coef[:, bs.SCALE] = torch.rand(G, Cin) + 0.5
        coef[:, bs.SHIFT] = torch.randn(G, Cin) * 0.3
        st0.coef.copy_(coef.to(dev))
        xr = (x * coef[:, bs.SCALE].to(dev).view(G, 1, 1, 1, Cin) + coef[:, bs.SHIFT].to(dev).view(G, 1, 1, 1, Cin))
        am = xr.relu().abs().amax(dim=(1, 2, 3, 4))
        st0.bound[0, :G] = am.float().view(torch.int32)
        xin = bs.LazyBN(x, st0, True)
        xin_r = bs.LazyBN(x.double().cpu(), bs.BnStat(coef.double(), p0r), True)
    flat, grads, prm = _params(G, Cout, dev, torch.float32)
    flat_r, grads_r, prm_r = _params(G, Cout, "cpu", torch.float64)
    y, st = H.conv_bn_stats(xin, w, None, s, p, nvalid, prm, True)
    yr, str_ = R64.conv_bn_stats(xin_r, w.double().cpu(), None, s, p, nvalid.cpu(), prm_r, True)
    for g in range(G):
        n = int(nvalid[g])
        assert _rel(y[g, :n], yr[g, :n]) < 2e-6, g
        for row in (bs.MEAN, bs.INV, bs.SCALE, bs.SHIFT, bs.YMAX, bs.YMIN):
            assert _rel(st.coef[g, row], str_.coef[g, row]) < 1e-5, (g, row)
        assert _rel(flat[g, 2 * Cout:4 * Cout], flat_r[g, 2 * Cout:4 * Cout]) < 1e-6, g   # running stats
        # the bound slot: max |relu(y * scale + shift)| over the valid rows (exact up to rounding)
        a_r = R64.lazy_value(bs.LazyBN(yr, str_, True), nvalid.cpu())
        bound = torch.tensor(int(st.bound[:, g].max()), dtype=torch.int32).view(torch.float32).item()
        assert abs(bound - a_r[g].abs().max().item()) <= 1e-5 * a_r[g].abs().max().item(), g
    # stored output with an identity residual and with a BN branch
    res = torch.randn_like(y)
    out = H.bn_apply(bs.LazyBN(y, st, False), res, True, nvalid)
    out_r = R64.bn_apply(bs.LazyBN(yr, str_, False), res.double().cpu(), True, nvalid.cpu())
    out2 = H.bn_apply(bs.LazyBN(y, st, False), bs.LazyBN(y, st, False), True, nvalid)
    out2_r = R64.bn_apply(bs.LazyBN(yr, str_, False), bs.LazyBN(yr, str_, False), True, nvalid.cpu())
    for g in range(G):
        n = int(nvalid[g])
        assert _rel(out[g, :n], out_r[g, :n]) < 2e-6 and _rel(out2[g, :n], out2_r[g, :n]) < 2e-6, g
    # bitwise repeatable (the tickets pick which block sums, never the order)
    _, _, prm2 = _params(G, Cout, dev, torch.float32)
    y2, st2 = H.conv_bn_stats(xin, w, None, s, p, nvalid, prm2, True)
    for g in range(G):   # (rows of invalid images are never written)
        n = int(nvalid[g])
        assert torch.equal(y[g, :n], y2[g, :n]) and torch.equal(st.coef[g, :bs.A], st2.coef[g, :bs.A]), g


@pytest.mark.parametrize("case", [(3, 64, 8, 8, 128, 128, 3, 1, 1), (3, 64, 4, 4, 256, 256, 3, 1, 1),
                                  (3, 16, 32, 32, 32, 32, 3, 1, 1), (3, 16, 16, 16, 64, 64, 3, 1, 1)])
def test_bn_stats_group_size_independent(H, case):
    """A replica's fused statistics are bitwise the same whether it runs alone (G = 1: 32-row
    tiles, in-launch split-K) or beside two others (G = 3: larger tiles, separate split-K
    reduce + the standalone pass) — the solo tail and world-size independence."""
    G, N, Hh, Ww, Cin, Cout, k, s, p = case
    dev = torch.device("cuda")
    x, w, nvalid = _x(case, dev, seed=3)
    _, _, prm = _params(G, Cout, dev, torch.float32)
    y3, st3 = H.conv_bn_stats(x, w, None, s, p, nvalid, prm, True)
    for g in range(G):
        _, _, p1 = _params(G, Cout, dev, torch.float32)
        p1 = bs.BnParams(*(t[g:g + 1] for t in (p1.gamma, p1.beta, p1.rmean, p1.rvar, p1.dgamma, p1.dbeta)),
                         0.1, 1e-5)
        y1, st1 = H.conv_bn_stats(x[g:g + 1].contiguous(), w[g:g + 1].contiguous(), None, s, p, nvalid[g:g + 1], p1,
                                  True)
        n = int(nvalid[g])
        assert torch.equal(y1[0, :n], y3[g, :n]), g
        assert torch.equal(st1.coef[0, :bs.A], st3.coef[g, :bs.A]), g


BWD = [
    (2, 4, 32, 32, 32, 32, 3, 1, 1, False),   # stage-1 halo dgrad, mask from a stored output
    (2, 3, 16, 16, 64, 64, 3, 1, 1, True),    # stage-2 halo dgrad, lazy mask
    (1, 64, 8, 8, 128, 128, 3, 1, 1, True),   # lone stage 3: split-K dgrad, in-launch combine
    (3, 64, 4, 4, 256, 256, 3, 1, 1, False),  # grouped stage 4: separate reduce + standalone pass
    (2, 4, 16, 16, 32, 64, 3, 2, 1, False),   # stride-2 dgrad: standalone pass
]


@pytest.mark.parametrize("case", BWD)
def test_backward_finish_and_lazy_grad(H, R64, case):
    """dgrad(dy) finished for a BN output (mask + sums of two BNs: a block output with a
    shortcut BN branch, or a lazy BN+ReLU), then the weight gradient of the conv below staging
    dy = A d + B y + K (stored for its dgrad) and x from a lazy BN output."""
    G, N, Hh, Ww, Cin, Cout, k, s, p, lazy = case
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(11)
    nvalid = torch.tensor([N] + [max(1, N - 3)] * (G - 1), dtype=torch.int32, device=dev)
    # the BN whose output's gradient the dgrad produces: C = Cin channels at the dgrad output
    C = Cin
    ya = torch.randn(G, N, Hh, Ww, C, generator=gen).to(dev)
    yb = torch.randn(G, N, Hh, Ww, C, generator=gen).to(dev)
    flat, grads, pa = _params(G, C, dev, torch.float32, seed=2)
    flat_r, grads_r, pa_r = _params(G, C, "cpu", torch.float64, seed=2)
    fb, gb, pb = _params(G, C, dev, torch.float32, seed=3)
    fb_r, gb_r, pb_r = _params(G, C, "cpu", torch.float64, seed=3)
    sa = H._bnf_fwd(pa, lazy, G, 1, C, dev)[1]
    sb = H._bnf_fwd(pb, False, G, 1, C, dev)[1]
    coef_a = torch.zeros(G, bs.ROWS, C)
    coef_b = torch.zeros(G, bs.ROWS, C)
    for cf, y in ((coef_a, ya), (coef_b, yb)):
        for g in range(G):
            n = int(nvalid[g])
            yy = y[g, :n].double().cpu().reshape(-1, C)
            cf[g, bs.MEAN], cf[g, bs.INV] = yy.mean(0).float(), torch.rsqrt(yy.var(0, unbiased=False) + 1e-5).float()
            cf[g, bs.YMAX], cf[g, bs.YMIN] = yy.max(0).values.float(), yy.min(0).values.float()
        cf[:, bs.SCALE] = torch.rand(G, C) + 0.5
        cf[:, bs.SHIFT] = torch.randn(G, C) * 0.2
    sa.coef.copy_(coef_a.to(dev))
    sb.coef.copy_(coef_b.to(dev))
    sa_r, sb_r = bs.BnStat(coef_a.double(), pa_r), bs.BnStat(coef_b.double(), pb_r)
    if lazy:
        fin = bs.Finish(ya=ya, sa=sa, lazy=True)
        fin_r = bs.Finish(ya=ya.double().cpu(), sa=sa_r, lazy=True)
    else:
        out = torch.relu(torch.randn(G, N, Hh, Ww, C, generator=gen)).to(dev)
        fin = bs.Finish(ya=ya, sa=sa, mask_out=out, yb=yb, sb=sb)
        fin_r = bs.Finish(ya=ya.double().cpu(), sa=sa_r, mask_out=out.double().cpu(), yb=yb.double().cpu(), sb=sb_r)
    Ho, Wo = (Hh + 2 * p - k) // s + 1, (Ww + 2 * p - k) // s + 1
    dy = torch.randn(G, N, Ho, Wo, Cout, generator=gen).to(dev)
    dy.mul_((torch.arange(N, device=dev)[None, :] < nvalid[:, None]).view(G, N, 1, 1, 1))
    w = (torch.randn(G, Cout, k, k, Cin, generator=gen) * (1.0 / (k * k * Cin) ** 0.5)).to(dev)
    acc = torch.randn(G, N, Hh, Ww, Cin, generator=gen).to(dev)
    dy._dba_amax = H._amax(dy, dy.stride(0), dy[0].numel())
    r = H.conv2d_dgrad(dy, w, None, s, p, (Hh, Ww), nvalid=nvalid, accum=acc, finish=fin)
    rr = R64.conv2d_dgrad(dy.double().cpu(), w.double().cpu(), None, s, p, (Hh, Ww), nvalid=nvalid.cpu(),
                          accum=acc.double().cpu(), finish=fin_r)
    assert isinstance(r, bs.Fin) and isinstance(rr, bs.Fin)
    for g in range(G):
        n = int(nvalid[g])
        assert _rel(r.d[g, :n], rr.d[g, :n]) < 2e-6, g
        for row in (bs.A, bs.B, bs.K):
            assert _rel(sa.coef[g, row], sa_r.coef[g, row]) < 1e-5, (g, row)
            if not lazy:
                assert _rel(sb.coef[g, row], sb_r.coef[g, row]) < 1e-5, (g, row)
        assert _rel(grads[g, :2 * C], grads_r[g, :2 * C]) < 1e-5, g        # dgamma, dbeta
        if not lazy:
            assert _rel(gb[g, :2 * C], gb_r[g, :2 * C]) < 1e-5, g
    # the weight gradient of a conv whose output is BN a's input (ya = conv(x2)): dy from (d, ya),
    # its input x2 a lazy BN+ReLU output
    k2, C2 = 3, 32
    x2 = torch.randn(G, N, Hh, Ww, C2, generator=gen).to(dev)
    sx = H._bnf_fwd(_params(G, C2, dev, torch.float32, seed=5)[2], True, G, 1, C2, dev)[1]
    cx = torch.zeros(G, bs.ROWS, C2)
    cx[:, bs.SCALE], cx[:, bs.SHIFT] = torch.rand(G, C2) + 0.5, torch.randn(G, C2) * 0.2
    sx.coef.copy_(cx.to(dev))
    xv = torch.relu(x2 * sx.coef[:, bs.SCALE].view(G, 1, 1, 1, C2) + sx.coef[:, bs.SHIFT].view(G, 1, 1, 1, C2))
    sx.bound[0, :G] = xv.abs().amax(dim=(1, 2, 3, 4)).float().view(torch.int32)
    dw = torch.zeros(G, C, k2, k2, C2, device=dev)
    dyv = H.conv2d_wgrad(bs.LazyGrad(r.d, ya, sa), bs.LazyBN(x2, sx, True), 1, 1, k2, k2, dw, nvalid=nvalid)
    dw_r = torch.zeros(G, C, k2, k2, C2, dtype=torch.float64)
    dyv_r = R64.conv2d_wgrad(bs.LazyGrad(rr.d, ya.double().cpu(), sa_r), bs.LazyBN(x2.double().cpu(),
                             bs.BnStat(cx.double(), None), True), 1, 1, k2, k2, dw_r, nvalid=nvalid.cpu())
    for g in range(G):
        n = int(nvalid[g])
        assert _rel(dyv[g, :n], dyv_r[g, :n]) < 1e-5, g
        assert _rel(dw[g], dw_r[g]) < 1e-5, g


def test_pooled_gradient_finish(H, R64):
    """The global average pool's gradient finished in the same pass (the last block)."""
    G, N, C = 2, 16, 256
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(5)
    nvalid = torch.tensor([N, 9], dtype=torch.int32, device=dev)
    ya = torch.randn(G, N, 4, 4, C, generator=gen).to(dev)
    _, grads, pa = _params(G, C, dev, torch.float32)
    _, grads_r, pa_r = _params(G, C, "cpu", torch.float64)
    sa = H._bnf_fwd(pa, False, G, 1, C, dev)[1]
    cf = torch.zeros(G, bs.ROWS, C)
    cf[:, bs.MEAN], cf[:, bs.INV] = torch.randn(G, C) * 0.1, torch.rand(G, C) + 0.5
    cf[:, bs.YMAX], cf[:, bs.YMIN] = 3.0, -3.0
    sa.coef.copy_(cf.to(dev))
    out = torch.relu(torch.randn(G, N, 4, 4, C, generator=gen)).to(dev)
    pool = torch.randn(G, N, 1, 1, C, generator=gen).to(dev)
    r = H.bn_finish(None, bs.Finish(ya=ya, sa=sa, mask_out=out), nvalid, pool=pool, hw=(4, 4))
    rr = R64.bn_finish(None, bs.Finish(ya=ya.double().cpu(), sa=bs.BnStat(cf.double(), pa_r),
                                       mask_out=out.double().cpu()), nvalid.cpu(), pool=pool.double().cpu(), hw=(4, 4))
    for g in range(G):
        n = int(nvalid[g])
        assert _rel(r.d[g, :n], rr.d[g, :n]) < 1e-6
        assert _rel(grads[g, :2 * C], grads_r[g, :2 * C]) < 1e-5

