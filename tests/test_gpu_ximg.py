"""The whole-image halo conv of the 16 / 8 / 4-wide evaluation stages (``xconv_fwd.hip ximg_kernel``)
vs an fp64 oracle and vs the implicit GEMM it replaces (GPU only).

3x3 stride-1 pad-1 forwards with BN-folded, pre-split weights (the stage-2 / 3 / 4 convs of the
reference ``models/resnet_cifar.py`` in evaluation): bias, residual and ReLU in the epilogue,
partly valid replicas, image counts that leave a partial tile, a slot map.  The kernel runs
the reduction chunk-major (32 channels x 9 taps per chunk) where the implicit GEMM runs it
tap-major, so the two agree at fp32 level, not bitwise.
"""
import struct

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dba_mod_amd.ops import hip
    yield hip
    hip.set_ximg(1)


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


@pytest.mark.parametrize("G,N,nv,W,Cin,Cout,res", [
    (3, 5, (5, 2, 4), 8, 128, 128, True), (2, 9, (9, 6), 4, 256, 256, True),
    (2, 7, (7, 3), 8, 64, 64, False), (1, 11, (11,), 4, 128, 64, False),
    (2, 5, (5, 3), 16, 64, 64, True), (1, 3, (3,), 16, 32, 32, False)])
def test_ximg_vs_fp64_and_implicit_gemm(H, R64, G, N, nv, W, Cin, Cout, res):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(G * 1000 + N * 10 + W)
    slots = 2
    x = torch.relu(torch.randn(G, N, W, W, Cin, generator=g)).to(dev)
    w = (torch.randn(slots, Cout, 3, 3, Cin, generator=g) / (3 * Cin ** 0.5)).to(dev)
    per = Cout * 9 * Cin
    H.split_weights(w, per, per, H._amax_w(w, per, per))
    b = (torch.randn(slots, Cout, generator=g) * 0.1).to(dev)
    r = torch.randn(G, N, W, W, Cout, generator=g).to(dev) if res else None
    wsel = torch.tensor([min(i, slots - 1) for i in range(G)], dtype=torch.int32, device=dev)
    nvalid = torch.tensor(nv, dtype=torch.int32, device=dev)
    outs = {}
    for on in (1, 0):
        H.set_ximg(on)
        with H.amax_arena(G, dev):
            y = H.conv2d(x, w, wsel, 1, 1, bias=b, residual=r, relu=True, nvalid=nvalid)
            outs[on] = (y, y._dba_amax.clone())
    H.set_ximg(1)
    torch.cuda.synchronize()
    yr = R64.conv2d(x.double().cpu(), w.double().cpu(), wsel.cpu(), 1, 1, bias=b.double().cpu(),
                    residual=None if r is None else r.double().cpu(), relu=True)
    y1, amax = outs[1]
    y0 = outs[0][0]
    for i in range(G):
        n = nv[i]
        e1, e0 = _rel(y1[i, :n], yr[i, :n]), _rel(y0[i, :n], yr[i, :n])
        assert e1 < 2e-6, f"replica {i}: whole-image {e1:.2e} (implicit GEMM {e0:.2e})"
        assert e1 < max(2e-6, 2 * e0), f"replica {i}: whole-image {e1:.2e} vs implicit GEMM {e0:.2e}"
        m = y1[i, :n].abs().max().item()
        assert struct.unpack("<f", struct.pack("<i", int(amax[:, i].max().item())))[0] == m


def test_ximg_is_deterministic(H):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(5)
    x = torch.relu(torch.randn(2, 6, 8, 8, 128, generator=g)).to(dev)
    w = (torch.randn(2, 128, 3, 3, 128, generator=g) * 0.03).to(dev)
    per = 128 * 9 * 128
    H.split_weights(w, per, per, H._amax_w(w, per, per))
    outs = []
    for _ in range(3):
        with H.amax_arena(2, dev):
            outs.append(H.conv2d(x, w, None, 1, 1, relu=True))
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("W,C", [(8, 128), (4, 256)])
def test_ximg_group_size_independent_bits(H, W, C):
    """A replica's output bits do not depend on how many replicas share the launch (world-1 vs
    world-N runs group models differently)."""
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(W + C)
    G = 3
    x = torch.relu(torch.randn(G, 5, W, W, C, generator=g)).to(dev)
    w = (torch.randn(G, C, 3, 3, C, generator=g) / (3 * C ** 0.5)).to(dev)
    per = C * 9 * C
    H.split_weights(w, per, per, H._amax_w(w, per, per))
    b = (torch.randn(G, C, generator=g) * 0.1).to(dev)
    with H.amax_arena(G, dev):
        yall = H.conv2d(x, w, None, 1, 1, bias=b, relu=True)
    for i in range(G):
        wi = w[i:i + 1].clone()
        H.split_weights(wi, per, per, H._amax_w(wi, per, per))
        with H.amax_arena(1, dev):
            yi = H.conv2d(x[i:i + 1].contiguous(), wi, None, 1, 1, bias=b[i:i + 1].contiguous(), relu=True)
        assert torch.equal(yi[0], yall[i]), i
