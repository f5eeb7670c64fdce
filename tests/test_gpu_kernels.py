"""HIP kernels vs the plain-PyTorch fp32 reference of the same op (GPU only).

Every test runs the gfx950 kernel from ``libdba_kernels.so`` (never a fallback: the hip
module raises if the library is missing) and compares against
:mod:`dba_mod_amd.ops.reference` evaluated in fp32 on the same inputs.  Tolerances reflect
bf16 operands with fp32 accumulation.
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


CONV_CASES = [
    # G, N, H, W, Cin, Cout, k, stride, pad
    (3, 5, 32, 32, 3, 32, 3, 1, 1),      # CIFAR stem (small-Cin kernel, staged 16-B epilogue)
    (2, 3, 32, 32, 3, 40, 3, 1, 1),      # small-Cin kernel, second column tile partly valid
    (2, 3, 32, 32, 3, 32, 3, 2, 1),      # small-Cin kernel without the LDS halo (stride 2)
    (2, 3, 16, 16, 3, 32, 3, 1, 1),      # LDS-halo stem, 16 output rows per block
    (2, 4, 32, 32, 32, 32, 3, 1, 1),     # layer1
    (2, 4, 32, 32, 32, 64, 3, 2, 1),     # layer2.0.conv1 (stride 2)
    (2, 4, 32, 32, 32, 64, 1, 2, 0),     # shortcut 1x1 s2
    (2, 3, 8, 8, 128, 256, 3, 2, 1),     # layer4.0.conv1
    (2, 3, 64, 64, 3, 64, 7, 2, 3),      # Tiny stem
    (2, 6, 28, 28, 1, 20, 5, 1, 0),      # MnistNet conv1
    (2, 64, 28, 28, 1, 20, 5, 1, 0),     # MnistNet conv1, full batch (multi-block bias grad)
    (2, 6, 12, 12, 20, 50, 5, 1, 0),     # MnistNet conv2
    (3, 7, 1, 1, 800, 500, 1, 1, 0),     # fc1 as 1x1
    (3, 7, 1, 1, 256, 10, 1, 1, 0),      # CIFAR linear
    (2, 5, 8, 8, 128, 128, 3, 1, 1),     # layer3 (halo kernel, 2 images per block)
    (2, 4, 16, 16, 64, 64, 3, 1, 1),     # layer2 (halo kernel)
    (3, 4, 32, 32, 32, 32, 1, 1, 0),     # 1x1 stride 1 (halo kernel)
    (2, 3, 4, 4, 256, 256, 3, 1, 1),     # layer4 (halo does not fit LDS -> gen-2 GEMM)
    (5, 40, 32, 32, 32, 32, 3, 1, 1),    # persistent kernel: block runs cross group boundaries
    (3, 20, 32, 32, 32, 64, 3, 2, 1),    # persistent kernel, stride 2 (de-interleaved halo)
    (3, 18, 16, 16, 64, 128, 3, 2, 1),   # persistent kernel, stride 2, 128 outputs
    (2, 3, 8, 8, 128, 256, 1, 2, 0),     # gen-3 GEMM small path, K = 2 k-steps (< ring depth)
    (2, 40, 8, 8, 128, 128, 3, 1, 1),    # gen-3 GEMM, 128x128 tiles
    (4, 70, 16, 16, 64, 64, 3, 1, 1),    # persistent kernel, 64-channel geometry
    (16, 64, 8, 8, 128, 256, 3, 2, 1),   # gen-3 wgrad without split-K (sole-writer epilogue)
    (2, 9, 16, 16, 64, 128, 1, 2, 0),    # gen-3 wgrad, shortcut (J = 64)
    (16, 6, 8, 8, 256, 256, 3, 2, 1),    # gen-3 wgrad 128x128 tiles (launch fills the chip)
    (1, 64, 4, 4, 256, 256, 3, 1, 1),    # lone client, stage 4: gen-3 split-K (8 slabs) + reduce
    (2, 64, 8, 8, 128, 128, 3, 1, 1),    # two clients, stage 3: gen-3 split-K (2 slabs)
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(H, R, case):
    G, N, Hh, Ww, Cin, Cout, k, s, p = case
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(G, N, Hh, Ww, Cin, device=dev).bfloat16()
    w = (torch.randn(G + 1, Cout, k, k, Cin, device=dev) * (1.0 / (k * k * Cin) ** 0.5)).bfloat16()
    wsel = torch.tensor([(g + 1) % (G + 1) for g in range(G)], dtype=torch.int32, device=dev)
    bias = torch.randn(G + 1, Cout, device=dev)
    nvalid = torch.tensor([N] + [max(1, N - 2)] * (G - 1), dtype=torch.int32, device=dev)
    Ho = (Hh + 2 * p - k) // s + 1
    res = torch.randn(G, N, Ho, Ho, Cout, device=dev).bfloat16()
    y = H.conv2d(x, w, wsel, s, p, bias=bias, residual=res, relu=True, nvalid=nvalid)
    yr = R.conv2d(x.float(), w.float(), wsel, s, p, bias=bias, residual=res.float(), relu=True)
    for g in range(G):
        n = int(nvalid[g])
        _close(y[g, :n], yr[g, :n], 2e-2, 3e-2, f"fwd g{g}")
    # data gradient
    dy = torch.randn(G, N, Ho, Ho, Cout, device=dev).bfloat16()
    for g in range(G):
        dy[g, int(nvalid[g]):] = 0
    dx = H.conv2d_dgrad(dy, w, wsel, s, p, (Hh, Ww), nvalid=nvalid)
    dxr = R.conv2d_dgrad(dy.float(), w.float(), wsel, s, p, (Hh, Ww))
    for g in range(G):
        n = int(nvalid[g])
        assert _rel(dx[g, :n], dxr[g, :n]) < 1e-2, f"dgrad g{g}"
    # residual-branch gradient fused into the dgrad epilogue
    acc = torch.randn(G, N, Hh, Ww, Cin, device=dev).bfloat16()
    dx2 = H.conv2d_dgrad(dy, w, wsel, s, p, (Hh, Ww), nvalid=nvalid, accum=acc)
    for g in range(G):
        n = int(nvalid[g])
        assert _rel(dx2[g, :n], dxr[g, :n] + acc[g, :n].float()) < 1e-2, f"dgrad+accum g{g}"
    # weight gradient (+ bias grad), accumulated into a strided flat buffer view
    P = Cout * k * k * Cin + 64
    flat = torch.zeros(G, P, device=dev)
    dw = flat[:, :Cout * k * k * Cin].view(G, Cout, k, k, Cin)
    db = torch.zeros(G, Cout, device=dev)
    H.conv2d_wgrad(dy, x, s, p, k, k, dw, db, nvalid=nvalid)
    dwr = torch.zeros(G, Cout, k, k, Cin, device=dev)
    dbr = torch.zeros(G, Cout, device=dev)
    R.conv2d_wgrad(dy.float(), x.float(), s, p, k, k, dwr, dbr)
    for g in range(G):
        assert _rel(dw[g], dwr[g]) < 1e-2, f"wgrad g{g}"
        assert _rel(db[g], dbr[g]) < 1e-3, f"bias grad g{g}"
    H.conv2d_wgrad(dy, x, s, p, k, k, dw, None, nvalid=nvalid)   # accumulates
    for g in range(G):
        assert _rel(dw[g], 2 * dwr[g]) < 1e-2, f"wgrad accumulate g{g}"
    assert flat[:, Cout * k * k * Cin:].abs().max().item() == 0.0, "wgrad wrote past its view"


@pytest.mark.parametrize("C,HW", [(32, 32), (64, 16)])
def test_pconv_inactive_groups_and_slots(H, R, C, HW):
    """Persistent conv: zero-valid groups in the middle, shared weight slots, fwd + dgrad."""
    dev = torch.device("cuda")
    torch.manual_seed(1)
    G, N = 7, 9
    x = torch.randn(G, N, HW, HW, C, device=dev).bfloat16()
    w = (torch.randn(3, C, 3, 3, C, device=dev) * (1.0 / (9 * C) ** 0.5)).bfloat16()
    wsel = torch.tensor([2, 0, 1, 1, 2, 0, 1], dtype=torch.int32, device=dev)
    nvalid = torch.tensor([9, 0, 4, 0, 0, 9, 1], dtype=torch.int32, device=dev)
    y = H.conv2d(x, w, wsel, 1, 1, nvalid=nvalid)
    yr = R.conv2d(x.float(), w.float(), wsel, 1, 1)
    dy = torch.randn(G, N, HW, HW, C, device=dev).bfloat16()
    dx = H.conv2d_dgrad(dy, w, wsel, 1, 1, (HW, HW), nvalid=nvalid)
    dxr = R.conv2d_dgrad(dy.float(), w.float(), wsel, 1, 1, (HW, HW))
    for g in range(G):
        n = int(nvalid[g])
        if n:
            _close(y[g, :n], yr[g, :n], 2e-2, 3e-2, f"fwd g{g}")
            assert _rel(dx[g, :n], dxr[g, :n]) < 1e-2, f"dgrad g{g}"


@pytest.mark.parametrize("code", [0, 1, 2, 3, 4, 5, 6])
def test_gemm3_tile_variants(H, R, code):
    """Every selectable gen-3 tile (small and large launch class) on a stage-4 3x3 conv, a
    ragged-M stage-3 conv and a 1x1 stride-2 shortcut, with bias/residual/ReLU and a short group."""
    dev = torch.device("cuda")
    torch.manual_seed(2)
    prev = H.set_gemm3_tiles(code, code)
    try:
        # small class without split-K (>= 192 64-row blocks) x3, then the large class
        for G, N, Hh, Cin, Cout, k, s, p in ((2, 301, 4, 256, 256, 3, 1, 1), (3, 91, 8, 128, 128, 3, 1, 1),
                                             (2, 301, 8, 128, 256, 1, 2, 0), (2, 601, 8, 128, 128, 3, 1, 1)):
            x = torch.randn(G, N, Hh, Hh, Cin, device=dev).bfloat16()
            w = (torch.randn(G, Cout, k, k, Cin, device=dev) * (1.0 / (k * k * Cin) ** 0.5)).bfloat16()
            bias = torch.randn(G, Cout, device=dev)
            nvalid = torch.tensor([N] + [max(1, N - 3)] * (G - 1), dtype=torch.int32, device=dev)
            Ho = (Hh + 2 * p - k) // s + 1
            res = torch.randn(G, N, Ho, Ho, Cout, device=dev).bfloat16()
            y = H.conv2d(x, w, None, s, p, bias=bias, residual=res, relu=True, nvalid=nvalid)
            yr = R.conv2d(x.float(), w.float(), None, s, p, bias=bias, residual=res.float(), relu=True)
            for g in range(G):
                n = int(nvalid[g])
                _close(y[g, :n], yr[g, :n], 2e-2, 3e-2, f"tile {code} G{G} N{N} C{Cin}->{Cout} g{g}")
    finally:
        H.set_gemm3_tiles(*prev)


def test_conv_fp32_out_and_inactive_group(H, R):
    dev = torch.device("cuda")
    x = torch.randn(2, 4, 1, 1, 512, device=dev).bfloat16()
    w = torch.randn(2, 200, 1, 1, 512, device=dev).bfloat16() * 0.05
    nv = torch.tensor([4, 0], dtype=torch.int32, device=dev)
    y = H.conv2d(x, w, None, 1, 0, nvalid=nv, out_dtype=torch.float32)
    assert y.dtype == torch.float32
    yr = R.conv2d(x.float(), w.float(), None, 1, 0)
    assert _rel(y[0], yr[0]) < 1e-2


@pytest.mark.parametrize("C,relu,with_res", [(32, True, False), (64, True, True), (256, False, False), (512, True, True)])
def test_bn_train_fwd_bwd(H, R, C, relu, with_res):
    dev = torch.device("cuda")
    torch.manual_seed(1)
    G, N, Hh = 3, 6, 4
    y = (torch.randn(G, N, Hh, Hh, C, device=dev) * 2 + 0.5).bfloat16()
    nvalid = torch.tensor([6, 3, 0], dtype=torch.int32, device=dev)
    S = 4 * C + 64
    st = torch.zeros(G, S, device=dev)
    gamma, beta, rm, rv = (st[:, i * C:(i + 1) * C] for i in range(4))
    gamma.copy_(torch.rand(G, C) + 0.5)
    beta.copy_(torch.randn(G, C) * 0.1)
    rv.fill_(1.0)
    st_ref = st.clone()
    res = torch.randn(G, N, Hh, Hh, C, device=dev).bfloat16() if with_res else None
    out, mean, invstd = H.bn_train(y, gamma, beta, rm, rv, nvalid, 0.1, 1e-5, relu, res)
    g_r, b_r, rm_r, rv_r = (st_ref[:, i * C:(i + 1) * C] for i in range(4))
    out_r, mean_r, inv_r = R.bn_train(y.float(), g_r, b_r, rm_r, rv_r, nvalid, 0.1, 1e-5, relu,
                                      res.float() if res is not None else None)
    for g in range(2):
        n = int(nvalid[g])
        _close(out[g, :n], out_r[g, :n], 2e-2, 2e-2, "bn out")
        _close(mean[g], mean_r[g], 1e-4, 1e-4, "mean")
        _close(invstd[g], inv_r[g], 1e-3, 1e-4, "invstd")
    _close(st[:, 2 * C:], st_ref[:, 2 * C:], 1e-4, 1e-5, "running stats")
    # padded rows / inactive replicas are not touched (every consumer gates on nvalid)
    dout = torch.randn_like(out.float()).bfloat16()
    gr = torch.zeros(G, 2 * C + 64, device=dev)
    dy, dres = H.bn_train_bwd(dout, y, out, mean, invstd, gamma, nvalid, relu, gr[:, :C], gr[:, C:2 * C],
                              want_dres=True)
    gr_r = torch.zeros_like(gr)
    dy_r, dres_r = R.bn_train_bwd(dout.float(), y.float(), out.float(), mean, invstd, gamma, nvalid, relu,
                                  gr_r[:, :C], gr_r[:, C:2 * C], want_dres=True)
    for g in range(2):
        n = int(nvalid[g])
        assert _rel(dy[g, :n], dy_r[g, :n]) < 2e-2
        assert _rel(dres[g, :n], dres_r[g, :n]) < 1e-2
    _close(gr, gr_r, 2e-2, 2e-2, "dgamma/dbeta")


@pytest.mark.parametrize("C,Hh", [(32, 32), (64, 16), (128, 12), (256, 12), (512, 12)])
def test_bn_train_large_multiblock(H, R, C, Hh):
    """Multi-block reduce path (rows > the single-launch limit: partials, finalize, apply),
    fwd + bwd, repeated eager calls and a HIP-graph replay against the fp32 reference."""
    from dba_mod_amd.ops import hip as hip_ops
    dev = torch.device("cuda")
    torch.manual_seed(2)
    G, N = 3, 10
    if N * Hh * Hh <= hip_ops._BN_SMALL_ROWS:
        pytest.skip("rows within the single-launch limit (DBA_BN_SMALL_ROWS raised)")
    y = (torch.randn(G, N, Hh, Hh, C, device=dev) * 1.5 - 0.3).bfloat16()
    nvalid = torch.tensor([10, 4, 0], dtype=torch.int32, device=dev)
    gamma = torch.rand(G, C, device=dev) + 0.5
    beta = torch.randn(G, C, device=dev) * 0.1
    dout = torch.randn(G, N, Hh, Hh, C, device=dev).bfloat16()

    def run():
        rm = torch.zeros(G, C, device=dev)
        rv = torch.ones(G, C, device=dev)
        out, mean, invstd = H.bn_train(y, gamma, beta, rm, rv, nvalid, 0.1, 1e-5, True, None)
        dg = torch.zeros(G, C, device=dev)
        db = torch.zeros(G, C, device=dev)
        dy = H.bn_train_bwd(dout, y, out, mean, invstd, gamma, nvalid, True, dg, db)
        return out, mean, invstd, rm, rv, dg, db, dy

    rm_r = torch.zeros(G, C, device=dev)
    rv_r = torch.ones(G, C, device=dev)
    out_r, mean_r, inv_r = R.bn_train(y.float(), gamma, beta, rm_r, rv_r, nvalid, 0.1, 1e-5, True, None)
    dg_r = torch.zeros(G, C, device=dev)
    db_r = torch.zeros(G, C, device=dev)
    dy_r = R.bn_train_bwd(dout.float(), y.float(), out_r, mean_r, inv_r, gamma, nvalid, True, dg_r, db_r)

    def check(res, tag):
        out, mean, invstd, rm, rv, dg, db, dy = res
        for g in range(2):
            n = int(nvalid[g])
            _close(out[g, :n], out_r[g, :n], 2e-2, 2e-2, f"{tag} bn out")
            _close(mean[g], mean_r[g], 1e-4, 1e-4, f"{tag} mean")
            _close(invstd[g], inv_r[g], 1e-3, 1e-4, f"{tag} invstd")
            assert _rel(dy[g, :n], dy_r[g, :n]) < 2e-2, tag
        _close(rm, rm_r, 1e-4, 1e-5, f"{tag} running mean")
        _close(rv, rv_r, 1e-3, 1e-4, f"{tag} running var")
        _close(dg, dg_r, 2e-2, 2e-2, f"{tag} dgamma")
        _close(db, db_r, 2e-2, 2e-2, f"{tag} dbeta")

    for i in range(3):
        check(run(), f"eager{i}")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        res = run()
    for i in range(3):
        g.replay()
        torch.cuda.synchronize()
        check(res, f"graph{i}")


def test_bn_fold(H, R):
    dev = torch.device("cuda")
    slots, Cout, K = 3, 64, 288
    S = Cout * K + 4 * Cout + 64
    st = torch.randn(slots, S, device=dev)
    w = st[:, :Cout * K].view(slots, Cout, 3, 3, 32)
    o = Cout * K
    gamma, beta, rm, rv = (st[:, o + i * Cout:o + (i + 1) * Cout] for i in range(4))
    rv.abs_()
    wf, bf = H.bn_fold(w, None, gamma, beta, rm, rv, 1e-5, torch.bfloat16)
    wf_r, bf_r = R.bn_fold(w, None, gamma, beta, rm, rv, 1e-5, torch.float32)
    _close(wf, wf_r, 1e-2, 1e-3, "wf")
    _close(bf, bf_r, 1e-4, 1e-4, "bf")


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
        for dt in (torch.bfloat16, torch.float32):
            x, y = H.gather_images(src, labels, idx, masks, trig, pn, 2, fs, dt)
            xr, yr = R.gather_images(src, labels, idx, masks, trig, pn, 2, fs, torch.float32)
            _close(x, xr, 1e-2, 1e-6, "gather x")
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
    x = torch.randn(2, 3, 24, 24, 20, device=dev).bfloat16()
    for k, s, p in ((2, 2, 0), (3, 2, 1)):
        y, ind = H.maxpool2d(x, k, s, p)
        yr, indr = R.maxpool2d(x.float(), k, s, p)
        _close(y, yr, 0, 0, "maxpool")
        dy = torch.randn_like(y.float()).bfloat16()
        dx = H.maxpool2d_bwd(dy, ind, tuple(x.shape), k, s, p)
        dxr = R.maxpool2d_bwd(dy.float(), ind, tuple(x.shape), k, s, p)
        _close(dx, dxr, 1e-2, 1e-2, "maxpool bwd")
    a = torch.randn(2, 5, 4, 4, 64, device=dev).bfloat16()
    _close(H.avgpool_global(a), R.avgpool_global(a.float()), 1e-2, 1e-2, "gap")
    d = torch.randn(2, 5, 1, 1, 64, device=dev).bfloat16()
    _close(H.avgpool_global_bwd(d, (4, 4)), R.avgpool_global_bwd(d.float(), (4, 4)), 1e-2, 1e-3, "gap bwd")
    seeds = torch.tensor([5, 9], dtype=torch.int32, device=dev)
    h = torch.randn(2, 7, 46, device=dev)
    _close(H.dropout(h, 0.5, seeds, 3), R.dropout(h, 0.5, seeds, 3), 0, 1e-6, "dropout")
    o = torch.randn(3, 1001, device=dev).bfloat16()
    dd = torch.randn(3, 1001, device=dev).bfloat16()
    _close(H.relu_mask_bwd(dd, o), R.relu_mask_bwd(dd.float(), o.float()), 0, 0, "relu mask")


def test_softmax_xent(H, R):
    dev = torch.device("cuda")
    for C in (10, 200, 9):
        logits = torch.randn(4, 70, C, device=dev) * 3
        labels = torch.randint(0, C, (4, 70), dtype=torch.int32, device=dev)
        labels[1, 40:] = -1
        labels[3] = -1
        for mean in (True, False):
            l, c, d = H.softmax_xent(logits, labels, mean, True)
            lr_, cr, dr = R.softmax_xent(logits, labels, mean, True)
            _close(l, lr_, 1e-4, 1e-4, "loss")
            assert torch.equal(c.cpu(), cr.cpu())
            _close(d, dr, 1e-2, 1e-3, "dlogits")
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


def test_sgd_step(H, R):
    dev = torch.device("cuda")
    G, P, S = 3, 1024, 1088
    st = torch.randn(G, S, device=dev)
    gr = torch.randn(G, P, device=dev)
    mom = torch.randn(G, P, device=dev)
    lr = torch.tensor([0.1, 0.05, 0.2], device=dev)
    first = torch.tensor([1, 0, 0], dtype=torch.int32, device=dev)
    act = torch.tensor([1, 1, 0], dtype=torch.int32, device=dev)
    sh = torch.zeros(G, P, dtype=torch.bfloat16, device=dev)
    fg = torch.zeros(G, P, device=dev)
    st_r, mom_r, fg_r = st.clone(), mom.clone(), fg.clone()
    H.sgd_step(st[:, :P], gr, mom, lr, first, act, 0.9, 5e-4, shadow=sh, fg_accum=fg)
    R.sgd_step(st_r[:, :P], gr, mom_r, lr, first, act, 0.9, 5e-4, fg_accum=fg_r)
    _close(st, st_r, 1e-6, 1e-6, "params")
    _close(mom, mom_r, 1e-6, 1e-6, "momentum")
    _close(fg, fg_r, 0, 0, "fg accum")
    _close(sh[:2], st[:2, :P], 1e-2, 1e-6, "bf16 shadow")


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
