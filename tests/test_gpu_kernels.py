"""HIP kernels vs the plain-PyTorch fp32 reference of the same op (GPU only).

Every test runs the gfx950 kernel from ``libdba_kernels.so`` (never a fallback: the hip
module raises if the library is missing) and compares against
:mod:`dba_mod_amd.ops.reference` evaluated in fp32 on the same inputs.  The convolution family (fp32 and its fp16-pair
split, fused training BN) is covered in ``test_gpu_f32.py`` / ``test_gpu_bnfuse.py``; this
file holds the data, elementwise, loss, optimizer and aggregation kernels.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dba_mod_amd.ops import hip
    return hip


@pytest.fixture(scope="module")
def R():
    from dba_mod_amd.ops import reference
    return reference


def _close(a, b, rtol, atol, what=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{what}: {bad}/{a.numel()} out of tol, max err {err.max().item():.3e}"


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp(min=1e-12)).item()


def test_bn_fold(H, R):
    dev = torch.device("cuda")
    slots, Cout, K = 3, 64, 288
    S = Cout * K + 4 * Cout + 64
    st = torch.randn(slots, S, device=dev)
    w = st[:, :Cout * K].view(slots, Cout, 3, 3, 32)
    o = Cout * K
    gamma, beta, rm, rv = (st[:, o + i * Cout:o + (i + 1) * Cout] for i in range(4))
    rv.abs_()
    wf, bf = H.bn_fold(w, None, gamma, beta, rm, rv, 1e-5, torch.float32)
    wf_r, bf_r = R.bn_fold(w, None, gamma, beta, rm, rv, 1e-5, torch.float32)
    _close(wf, wf_r, 1e-5, 1e-5, "wf")
    _close(bf, bf_r, 1e-4, 1e-4, "bf")
    # the fold kernel's max |w'| per slot (the folded weights' fp16-pair scale) is exact
    import struct
    for sl in range(slots):
        got = struct.unpack("<f", struct.pack("<i", int(wf._dba_amax[:, sl].max().item())))[0]
        assert got == wf[sl].abs().max().item(), sl
    # one zeroed buffer for a whole model's folds (program.fold_bank)
    buf = H.amax_slots(2, slots, dev)
    wf2, _ = H.bn_fold(w, None, gamma, beta, rm, rv, 1e-5, torch.float32, amax_slot=buf[1])
    assert torch.equal(wf2, wf) and torch.equal(buf[1], wf._dba_amax) and buf[0].abs().sum().item() == 0
    # a model fold's splits in one launch == one split per conv (bits of the fp16 planes)
    wf3, _ = H.bn_fold(w, None, gamma, beta, rm, rv, 1e-5, torch.float32, amax_slot=buf[0], split=False)
    w_small = wf3[:, :16].contiguous()
    w_small._dba_amax = H._amax(w_small, w_small[0].numel(), w_small[0].numel())
    H.split_weights_batch([(wf3, Cout * K, Cout * K, wf3._dba_amax), (w_small, w_small[0].numel(), w_small[0].numel(),
                                                                     w_small._dba_amax)])
    assert torch.equal(wf3._dba_planes, wf._dba_planes)
    ref = H.split_weights(w_small.clone(), w_small[0].numel(), w_small[0].numel(), w_small._dba_amax)
    assert torch.equal(w_small._dba_planes, ref)


def test_bn_fold_batch(H):
    """A model fold in two launches (program.fold_bank: every BN fold, then every split) ==
    one bn_fold per conv, bit for bit (folded weights, biases, max |w'|, fp16-pair planes);
    sizes off the 2048 / 4096-element chunk grid."""
    dev = torch.device("cuda")
    slots, shapes = 3, [(16, 3, 3, 3), (64, 3, 3, 32), (40, 1, 1, 129), (8, 1, 1, 5)]
    S = sum(c * kh * kw * ci + 4 * c for c, kh, kw, ci in shapes) + 7
    st = torch.randn(slots, S, device=dev)
    convs, o = [], 0
    for c, kh, kw, ci in shapes:
        w = st[:, o:o + c * kh * kw * ci].view(slots, c, kh, kw, ci)
        o += c * kh * kw * ci
        g, b, rm, rv = (st[:, o + i * c:o + (i + 1) * c] for i in range(4))
        o += 4 * c
        rv.abs_()
        convs.append((w, g, b, rm, rv))
    buf = H.amax_slots(len(convs), slots, dev)
    got = H.bn_fold_batch([cv + (buf[i],) for i, cv in enumerate(convs)], 1e-5)
    H.split_weights_batch([(wf, wf[0].numel(), wf[0].numel(), wf._dba_amax) for wf, _ in got])
    for (w, g, b, rm, rv), (wf, bf) in zip(convs, got):
        wr, br = H.bn_fold(w, None, g, b, rm, rv, 1e-5, torch.float32)
        assert torch.equal(wf, wr) and torch.equal(bf, br)
        assert torch.equal(wf._dba_amax.max(0).values, wr._dba_amax.max(0).values)
        assert torch.equal(wf._dba_planes, wr._dba_planes)


def test_gather_and_triggers(H, R):
    dev = torch.device("cuda")
    src = torch.randint(0, 256, (50, 32, 32, 3), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 10, (50,), dtype=torch.int32, device=dev)
    idx = torch.randint(0, 50, (3, 8), dtype=torch.int32, device=dev)
    idx[2, 5:] = -1
    masks = torch.zeros(2, 32, 32, dtype=torch.uint8, device=dev)
    masks[0, 0, :6] = 1
    masks[1, 4, 9:15] = 1
    trig = torch.tensor([0, -1, 1], dtype=torch.int32, device=dev)
    pn = torch.tensor([3, 0, 8], dtype=torch.int32, device=dev)
    seeds = torch.tensor([11, 22, 33], dtype=torch.int32, device=dev)
    for fs in (None, seeds):
        for dt in (torch.float32,):
            x, y = H.gather_images(src, labels, idx, masks, trig, pn, 2, fs, dt)
            xr, yr = R.gather_images(src, labels, idx, masks, trig, pn, 2, fs, torch.float32)
            _close(x, xr, 1e-6, 1e-6, "gather x")
            assert torch.equal(y.cpu(), yr.cpu())
    rows = torch.randn(50, 91, device=dev)          # idx above indexes rows 0..49
    lab = torch.randint(0, 9, (50,), dtype=torch.int32, device=dev)
    cols = torch.tensor([[0, 1], [2, -1]], dtype=torch.int32, device=dev)
    vals = torch.tensor([[10.0, 80.0], [20.0, 0.0]], device=dev)
    x, y = H.gather_rows(rows, lab, idx, cols, vals, trig, pn, 7, torch.float32)
    xr, yr = R.gather_rows(rows, lab, idx, cols, vals, trig, pn, 7, torch.float32)
    _close(x, xr, 0, 1e-6, "rows")
    assert torch.equal(y.cpu(), yr.cpu())


def test_pool_dropout_relu(H, R):
    dev = torch.device("cuda")
    x = torch.randn(2, 3, 24, 24, 20, device=dev)
    for k, s, p in ((2, 2, 0), (3, 2, 1)):
        y, ind = H.maxpool2d(x, k, s, p)
        yr, indr = R.maxpool2d(x.float(), k, s, p)
        _close(y, yr, 0, 0, "maxpool")
        dy = torch.randn_like(y)
        dx = H.maxpool2d_bwd(dy, ind, tuple(x.shape), k, s, p)
        dxr = R.maxpool2d_bwd(dy.float(), ind, tuple(x.shape), k, s, p)
        _close(dx, dxr, 1e-6, 1e-6, "maxpool bwd")
    a = torch.randn(2, 5, 4, 4, 64, device=dev)
    _close(H.avgpool_global(a), R.avgpool_global(a), 1e-5, 1e-5, "gap")
    d = torch.randn(2, 5, 1, 1, 64, device=dev)
    _close(H.avgpool_global_bwd(d, (4, 4)), R.avgpool_global_bwd(d, (4, 4)), 1e-6, 1e-6, "gap bwd")
    seeds = torch.tensor([5, 9], dtype=torch.int32, device=dev)
    h = torch.randn(2, 7, 46, device=dev)
    _close(H.dropout(h, 0.5, seeds, 3), R.dropout(h, 0.5, seeds, 3), 0, 1e-6, "dropout")
    o = torch.randn(3, 1001, device=dev)
    dd = torch.randn(3, 1001, device=dev)
    _close(H.relu_mask_bwd(dd, o), R.relu_mask_bwd(dd, o), 0, 0, "relu mask")


def test_softmax_xent(H, R):
    dev = torch.device("cuda")
    for C in (10, 200, 9):
        logits = torch.randn(4, 70, C, device=dev) * 3
        labels = torch.randint(0, C, (4, 70), dtype=torch.int32, device=dev)
        labels[1, 40:] = -1
        labels[3] = -1
        for mean in (True, False):
            l, c, d = H.softmax_xent(logits, labels, mean, True, grad_dtype=torch.float32)
            lr_, cr, dr = R.softmax_xent(logits, labels, mean, True)
            _close(l, lr_, 1e-4, 1e-4, "loss")
            assert torch.equal(c.cpu(), cr.cpu())
            _close(d, dr, 1e-5, 1e-6, "dlogits")
        # fused per-client statistics accumulation (trainer step)
        G, ms = 4, 8
        slot = torch.tensor([0, 3, 7, 2], dtype=torch.int32, device=dev)
        nvalid = (labels >= 0).sum(1).int()
        sh = torch.rand(3, G * ms, device=dev)
        sr = sh.clone()
        H.softmax_xent(logits, labels, True, True, sh, slot, nvalid)
        R.softmax_xent(logits, labels, True, True, sr, slot, nvalid)
        _close(sh, sr, 1e-4, 1e-4, "stats")
    # eval-sized batches (one block handles >256 rows)
    logits = torch.randn(3, 1000, 10, device=dev) * 3
    labels = torch.randint(0, 10, (3, 1000), dtype=torch.int32, device=dev)
    labels[2, 600:] = -1
    l, c, _ = H.softmax_xent(logits, labels, False, False)
    lr_, cr, _ = R.softmax_xent(logits, labels, False, False)
    _close(l, lr_, 1e-4, 1e-4, "loss (eval)")
    assert torch.equal(c.cpu(), cr.cpu())
    # evaluation chunks of the Tiny head (1024 x 200: 64-row slices + the finish launch), wider
    # heads (several classes per lane), fp64 loss sums; argmax ties resolve to the first class
    for B, C in ((1024, 200), (300, 1000), (257, 3)):
        logits = (torch.randn(3, B, C, device=dev) * 3).round()     # many exact ties
        labels = torch.randint(0, C, (3, B), dtype=torch.int32, device=dev)
        labels[1, B // 3:] = -1
        l, c, _ = H.softmax_xent(logits, labels, False, False, loss_dtype=torch.float64)
        lr_, cr, _ = R.softmax_xent(logits, labels, False, False, loss_dtype=torch.float64)
        _close(l, lr_, 1e-6, 1e-4, f"loss (eval {B}x{C})")
        assert torch.equal(c.cpu(), cr.cpu()), (B, C)
        # a group's bits do not depend on the other groups of the launch
        l1, c1, _ = H.softmax_xent(logits[1:2].contiguous(), labels[1:2].contiguous(), False, False,
                                   loss_dtype=torch.float64)
        assert torch.equal(l1.cpu(), l[1:2].cpu()) and torch.equal(c1.cpu(), c[1:2].cpu())


def test_sgd_step(H, R):
    dev = torch.device("cuda")
    G, P, S = 3, 1024, 1088
    st = torch.randn(G, S, device=dev)
    gr = torch.randn(G, P, device=dev)
    mom = torch.randn(G, P, device=dev)
    lr = torch.tensor([0.1, 0.05, 0.2], device=dev)
    first = torch.tensor([1, 0, 0], dtype=torch.int32, device=dev)
    act = torch.tensor([1, 1, 0], dtype=torch.int32, device=dev)
    fg = torch.zeros(G, P, device=dev)
    st_r, mom_r, fg_r = st.clone(), mom.clone(), fg.clone()
    H.sgd_step(st[:, :P], gr, mom, lr, first, act, 0.9, 5e-4, fg_accum=fg)
    R.sgd_step(st_r[:, :P], gr, mom_r, lr, first, act, 0.9, 5e-4, fg_accum=fg_r)
    _close(st, st_r, 1e-6, 1e-6, "params")
    _close(mom, mom_r, 1e-6, 1e-6, "momentum")
    _close(fg, fg_r, 0, 0, "fg accum")


def test_dist_loss_grad(H, R):
    dev = torch.device("cuda")
    G, P, S = 4, 5000, 5120
    st = torch.randn(G, S, device=dev)
    base = st + 0.01 * torch.randn(G, S, device=dev)
    base[3] = st[3]                                   # w == base: zero subgradient
    trig = torch.tensor([0, -1, 2, 1], dtype=torch.int32, device=dev)
    act = torch.tensor([1, 1, 1, 1], dtype=torch.int32, device=dev)
    gr = torch.randn(G, P, device=dev)
    g2 = gr.clone()
    d1 = H.dist_loss_grad(st, base, gr, trig, act, 0.7)
    d2 = R.dist_loss_grad(st, base, g2, trig, act, 0.7)
    _close(d1, d2, 1e-4, 1e-6, "distance")
    _close(gr, g2, 1e-4, 1e-5, "grads")


def test_flat_aggregation_ops(H, R):
    dev = torch.device("cuda")
    n, L = 10, 100_003
    pts = torch.randn(n, L + 64, device=dev)[:, :L]
    m = torch.randn(L, device=dev)
    _close(H.sq_dists(pts, m), R.sq_dists(pts, m), 1e-5, 1e-3, "sq_dists")
    wts = torch.rand(n, device=dev)
    _close(H.weighted_sum(pts, wts), R.weighted_sum(pts, wts), 1e-4, 1e-4, "wsum")
    base = torch.randn(L, device=dev)
    w = torch.randn(L, device=dev)
    _close(H.scale_from_base(w, base, 100.0), R.scale_from_base(w, base, 100.0), 1e-5, 1e-4, "scale")
    for noise in (False, True):
        d1 = torch.randn(L, device=dev)
        d2 = d1.clone()
        upd = torch.randn(L, device=dev)
        H.add_noise_scaled(d1, upd, 0.01, 0.01, 1234, noise)
        R.add_noise_scaled(d2, upd, 0.01, 0.01, 1234, noise)
        _close(d1, d2, 1e-4, 1e-5, "noise add")
    for nn_, d in ((10, 2560), (37, 5000), (4, 207)):
        f = torch.randn(nn_, d, device=dev)
        _close(H.gram(f), R.gram(f), 1e-4, 1e-2, "gram")


def test_torch_library_ops_run_hip():
    """torch.ops.dba.* on GPU tensors dispatch to the HIP kernels (same bits as the direct
    launcher call) — ops/library.py."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dba_mod_amd.ops import hip as H
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 4, 16, 16, 32, generator=g).to(dev)
    w = (torch.randn(2, 32, 3, 3, 32, generator=g) * 0.05).to(dev)
    y = torch.ops.dba.conv2d(x, w, None, 1, 1, None, None, True, None)
    assert torch.equal(y, H.conv2d(x, w, None, 1, 1, relu=True))
    pts = torch.randn(5, 10000, generator=g).to(dev)
    assert torch.equal(torch.ops.dba.gram(pts), H.gram(pts))
    assert torch.equal(torch.ops.dba.sq_dists(pts, pts[0]), H.sq_dists(pts, pts[0]))


def test_weighted_sum_fixed_matches_reference_bitwise():
    """flat.hip wsum_fixed_kernel: the same int64 limbs as the CPU reference (every step is an
    exact fp64 operation or a floor), so the fixed-point RFA / FoolsGold sums agree across
    devices as well as across world sizes."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dba_mod_amd.fl import aggregate as agg
    from dba_mod_amd.ops import hip as H
    from dba_mod_amd.ops import reference as R
    g = torch.Generator().manual_seed(1)
    n, L = 7, 100003
    pts = torch.randn(n, L, generator=g) * torch.exp(2 * torch.randn(n, 1, generator=g))
    w = torch.rand(n, generator=g).float()
    w = w / w.sum()
    E = agg.fixed_exponent(float(pts.abs().max()), n)
    got = H.weighted_sum_fixed(pts.cuda(), w.cuda(), E).cpu()
    assert torch.equal(got, R.weighted_sum_fixed(pts, w, E))


def test_weight_amax_segments(H):
    """Per-replica max |w| of many flat-row segments in one launch (chunked, 16-B loads, scalar
    tails): odd lengths, a segment past 64 chunks, unaligned offsets, the exact float bits."""
    import struct
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(3)
    G, S = 3, 600_000
    flat = (torch.randn(G, S, generator=g) * torch.logspace(-3, 3, S)[None, :]).to(dev)
    segs = [(0, 864), (896, 9216), (10176, 1), (10240, 295_000), (305_408, 261_000), (566_410, 33_589)]
    slots = H.weight_amax(flat, segs)
    torch.cuda.synchronize()
    for (o, n), sl in zip(segs, slots):
        for r in range(G):
            want = flat[r, o:o + n].abs().max().item()
            got = struct.unpack("<f", struct.pack("<i", int(sl[:, r].max().item())))[0]
            assert got == want, (o, n, r, got, want)
