"""The patch-reuse weight gradient of the narrow stages' 3x3 stride-1 convs
(``csrc/kernels/xwgrad_halo.hip``) vs an fp64 oracle and vs the implicit-GEMM weight gradient it
replaces (GPU only).

dW[co][tap][ci] = sum_p dy[p][co] x[p + off(tap)][ci] for the 32-wide stage (32 -> 32 channels)
and the 16-wide stage (64 -> 64), the reference's autograd of ``models/resnet_cifar.py:19-21``:
partly valid replicas, a plain and a lazy BN(+ReLU) input (x = relu(y * scale + shift), the
fused training BN's consumer form), the deferred batched slab reduction, accumulation into a
strided flat-buffer view, group-size independence and run-to-run bits.  The operands reach the
MFMAs through the transposing LDS read ``ds_read_b64_tr_b16``, so a wrong lane map would show
here as an O(1) error.
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
    hip.set_wgrad_halo(1)


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


def _lazy(H, y, g, relu):
    """A lazy BN output of y with random per-channel scale / shift (coefficient rows as the
    fused BN writes them) and its operand-max slot; returns (LazyBN, its fp32 value)."""
    G, C = y.shape[0], y.shape[-1]
    coef = torch.zeros(G, bs.ROWS, C, device=y.device)
    coef[:, bs.SCALE] = (torch.rand(G, C, generator=g) + 0.5).to(y.device)
    coef[:, bs.SHIFT] = (torch.randn(G, C, generator=g) * 0.2).to(y.device)
    sh = (G, 1, 1, 1, C)
    v = torch.addcmul(coef[:, bs.SHIFT].reshape(sh), y, coef[:, bs.SCALE].reshape(sh))
    if relu:
        v = torch.relu(v)
    st = bs.BnStat(coef, None, H._amax_act(v.clone(), None))
    return bs.LazyBN(y, st, relu), v


# (G, N, valid images, W, C, lazy x)
CASES = [(2, 3, (3, 1), 32, 32, False), (3, 2, (2, 2, 1), 16, 64, False), (2, 4, (4, 3), 32, 32, True),
         (2, 3, (3, 2), 16, 64, True), (1, 64, (64,), 32, 32, True), (1, 64, (64,), 16, 64, False)]


@pytest.mark.parametrize("G,N,nv,W,C,lazy", CASES)
def test_wgrad_halo_vs_fp64_and_implicit_gemm(H, R64, G, N, nv, W, C, lazy):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(G * 100 + N + W + C)
    y = torch.randn(G, N, W, W, C, generator=g).to(dev)
    dy = torch.randn(G, N, W, W, C, generator=g).to(dev)
    nvalid = torch.tensor(nv, dtype=torch.int32, device=dev)
    for i in range(G):
        dy[i, nv[i]:] = 0
    if lazy:
        xin, xval = _lazy(H, y, g, relu=True)
    else:
        xin, xval = y, y
    outs = {}
    for on in (1, 0):
        H.set_wgrad_halo(on)
        flat = torch.zeros(G, C * 9 * C + 64, device=dev)
        dw = flat[:, :C * 9 * C].view(G, C, 3, 3, C)
        defer = []
        H.conv2d_wgrad(dy, xin, 1, 1, 3, 3, dw, None, nvalid=nvalid, defer=defer)
        H.wgrad_flush(defer)
        H.conv2d_wgrad(dy, xin, 1, 1, 3, 3, dw, None, nvalid=nvalid)   # accumulates (own reduce)
        outs[on] = flat.clone()
        assert flat[:, C * 9 * C:].abs().max().item() == 0.0, "wrote past its view"
    H.set_wgrad_halo(1)
    ref = torch.zeros(G, C, 3, 3, C, dtype=torch.float64)
    R64.conv2d_wgrad(dy.double().cpu(), xval.double().cpu(), 1, 1, 3, 3, ref, None)
    for i in range(G):
        got = outs[1][i, :C * 9 * C].view(C, 3, 3, C)
        old = outs[0][i, :C * 9 * C].view(C, 3, 3, C)
        e1, e0 = _rel(got, 2 * ref[i]), _rel(old, 2 * ref[i])
        assert e1 < 1e-5, f"replica {i}: patch-reuse {e1:.2e} (implicit GEMM {e0:.2e})"
        assert e1 < max(1e-5, 4 * e0), (i, e1, e0)


@pytest.mark.parametrize("W,C", [(32, 32), (16, 64)])
def test_wgrad_halo_deterministic_and_group_size_independent(H, W, C):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(W + C)
    G, N = 3, 4
    x = torch.randn(G, N, W, W, C, generator=g).to(dev)
    dy = torch.randn(G, N, W, W, C, generator=g).to(dev)

    def run(sl):
        xs, dys = x[sl].contiguous(), dy[sl].contiguous()
        dw = torch.zeros(xs.shape[0], C, 3, 3, C, device=dev)
        H.conv2d_wgrad(dys, xs, 1, 1, 3, 3, dw, None)
        return dw

    full = run(slice(0, G))
    assert torch.equal(full, run(slice(0, G)))
    for i in range(G):
        assert torch.equal(run(slice(i, i + 1))[0], full[i]), i


# ------------------------------------------------------------------ the 3-channel stem
def _stem_case(dev, G, N, nv, W, seed, lazy):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(G, N, W, W, 3, generator=g).to(dev)           # image values in [0, 1]
    d = torch.randn(G, N, W, W, 32, generator=g).to(dev)
    for i in range(G):
        d[i, nv[i]:] = 0
    if not lazy:
        return x, d, d.double()
    y = torch.randn(G, N, W, W, 32, generator=g).to(dev) * 2 + 0.5
    coef = torch.zeros(G, bs.ROWS, 32, device=dev)
    coef[:, bs.A] = (torch.rand(G, 32, generator=g) + 0.5).to(dev)
    coef[:, bs.B] = (torch.randn(G, 32, generator=g) * 0.1).to(dev)
    coef[:, bs.K] = (torch.randn(G, 32, generator=g) * 0.1).to(dev)
    sh = (G, 1, 1, 1, 32)
    dyv = coef[:, bs.A].double().reshape(sh) * d.double() + coef[:, bs.B].double().reshape(sh) * y.double() \
        + coef[:, bs.K].double().reshape(sh)
    for i in range(G):
        dyv[i, nv[i]:] = 0
    st = bs.BnStat(coef, None, None)
    return x, bs.LazyGrad(d, y, st), dyv


@pytest.mark.parametrize("G,N,nv,W,lazy", [(2, 3, (3, 1), 32, False), (3, 2, (2, 0, 1), 32, True),
                                           (1, 64, (64,), 32, True), (2, 2, (2, 1), 64, False),
                                           (2, 2, (1, 2), 64, True)])
def test_stem_wgrad_vs_fp64_and_implicit_gemm(H, R64, G, N, nv, W, lazy):
    """dW of the 3 -> 32 stem (CIFAR 32-wide, Tiny 64-wide images), stored or lazy BN input
    gradient, partly valid / empty replicas, deferred and immediate slab reduction into a
    strided flat view (accumulating)."""
    dev = torch.device("cuda")
    x, dy, dyv = _stem_case(dev, G, N, nv, W, 300 + G * 10 + N + W, lazy)
    nvalid = torch.tensor(nv, dtype=torch.int32, device=dev)
    per = 32 * 27
    flat = torch.zeros(G, per + 64, device=dev)
    dw = flat[:, :per].view(G, 32, 3, 3, 3)
    assert H.set_stem_wgrad(-1) == 1
    defer = []
    assert H.conv2d_wgrad(dy, x, 1, 1, 3, 3, dw, None, nvalid=nvalid, defer=defer) is None
    assert len(defer) == 1
    H.wgrad_flush(defer)
    H.conv2d_wgrad(dy, x, 1, 1, 3, 3, dw, None, nvalid=nvalid)             # immediate reduce
    assert flat[:, per:].abs().max().item() == 0.0, "wrote past its view"
    ref = torch.zeros(G, 32, 3, 3, 3, dtype=torch.float64)
    R64.conv2d_wgrad(dyv.cpu(), x.double().cpu(), 1, 1, 3, 3, ref, None)
    # the implicit-GEMM weight gradient of the same (stored) dy
    old = torch.zeros(G, 32, 3, 3, 3, device=dev)
    prev = H.set_stem_wgrad(0)
    try:
        H.conv2d_wgrad(dyv.float().contiguous(), x, 1, 1, 3, 3, old, None, nvalid=nvalid)
    finally:
        H.set_stem_wgrad(prev)
    for i in range(G):
        if nv[i] == 0:
            assert flat[i].abs().max().item() == 0.0
            continue
        e1, e0 = _rel(dw[i], 2 * ref[i]), _rel(old[i], ref[i])
        assert e1 < 1e-6, f"replica {i}: stem wgrad {e1:.2e} (implicit GEMM {e0:.2e})"


def test_stem_wgrad_deterministic_and_group_size_independent(H):
    dev = torch.device("cuda")
    G, N = 3, 4
    x, dy, _ = _stem_case(dev, G, N, (N,) * G, 32, 77, True)

    def run(sl):
        lg = bs.LazyGrad(dy.d[sl].contiguous(), dy.y[sl].contiguous(),
                         bs.BnStat(dy.stat.coef[sl].contiguous(), None, None))
        dw = torch.zeros(lg.d.shape[0], 32, 3, 3, 3, device=dev)
        H.conv2d_wgrad(lg, x[sl].contiguous(), 1, 1, 3, 3, dw, None)
        return dw

    full = run(slice(0, G))
    assert torch.equal(full, run(slice(0, G)))
    for i in range(G):
        assert torch.equal(run(slice(i, i + 1))[0], full[i]), i
