"""The fused downsampling block (``xconv_fwd.hip dba_xdown_fwd``: conv2 of a stride-2 BasicBlock with
its 1x1 stride-2 shortcut as extra k-steps of the same launch) vs an fp64 oracle and vs the
two-launch form it replaces (GPU only).

relu(conv3x3(a, w2) + b2 + conv1x1_s2(x2, wsc) + bsc) with BN folded into the weights — the
second half of the downsampling BasicBlock of the reference ``models/resnet_cifar.py:24-36``
(layer2.0) in evaluation; the 8 / 4-wide stages keep two launches (measured faster).  The
shortcut's products accumulate with their own fp16 scales (the accumulators are rescaled
exactly) and its output is never stored, so the fused form agrees with the two launches at fp32
level, not bitwise.  Wide dynamic ranges between the two
operand pairs exercise the rescale.
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


def _split(H, w):
    per = w[0].numel()
    H.split_weights(w, per, per, H._amax_w(w, per, per))
    return w


def _case(H, dev, G, N, W, C, C2, sa, sx, seed):
    g = torch.Generator().manual_seed(seed)
    slots = 2
    a = torch.relu(torch.randn(G, N, W, W, C, generator=g) * sa).to(dev)
    x2 = torch.relu(torch.randn(G, N, 2 * W, 2 * W, C2, generator=g) * sx).to(dev)
    w2 = _split(H, (torch.randn(slots, C, 3, 3, C, generator=g) / (3 * C ** 0.5)).to(dev))
    wsc = _split(H, (torch.randn(slots, C, 1, 1, C2, generator=g) / C2 ** 0.5).to(dev))
    b2 = (torch.randn(slots, C, generator=g) * 0.1 * sa).to(dev)
    bsc = (torch.randn(slots, C, generator=g) * 0.1 * sx).to(dev)
    wsel = torch.tensor([min(i, slots - 1) for i in range(G)], dtype=torch.int32, device=dev)
    return a, x2, w2, wsc, b2, bsc, wsel


# (G, N, valid images, W, C, C2, scale of a, scale of x2): layer2.0 of the CIFAR ResNets, partial
# tiles, operand ranges far apart (both directions)
@pytest.mark.parametrize("G,N,nv,W,C,C2,sa,sx", [
    (3, 5, (5, 2, 4), 16, 64, 32, 1.0, 1.0), (2, 4, (4, 1), 16, 64, 32, 1e-3, 30.0),
    (2, 9, (9, 6), 16, 64, 32, 30.0, 1e-3), (1, 7, (7,), 16, 64, 32, 1e-4, 1.0)])
def test_down_block_vs_fp64_and_two_launches(H, R64, G, N, nv, W, C, C2, sa, sx):
    dev = torch.device("cuda")
    a, x2, w2, wsc, b2, bsc, wsel = _case(H, dev, G, N, W, C, C2, sa, sx, G * 100 + N + W)
    nvalid = torch.tensor(nv, dtype=torch.int32, device=dev)
    assert H.down_block_ok(a, w2, x2, wsc)
    with H.amax_arena(G, dev):
        y = H.down_block_eval(a, w2, b2, x2, wsc, bsc, wsel, nvalid)
        amax = y._dba_amax.clone()
        sc = H.conv2d(x2, wsc, wsel, 2, 0, bias=bsc, nvalid=nvalid)
        y2 = H.conv2d(a, w2, wsel, 1, 1, bias=b2, residual=sc, relu=True, nvalid=nvalid)
    torch.cuda.synchronize()
    c = lambda t: t.double().cpu()  # noqa: E731
    yr = R64.down_block_eval(c(a), c(w2), c(b2), c(x2), c(wsc), c(bsc), wsel.cpu())
    for i in range(G):
        n = nv[i]
        e1, e0 = _rel(y[i, :n], yr[i, :n]), _rel(y2[i, :n], yr[i, :n])
        assert e1 < 2e-6, f"replica {i}: fused {e1:.2e} (two launches {e0:.2e})"
        assert e1 < max(2e-6, 2 * e0), f"replica {i}: fused {e1:.2e} vs two launches {e0:.2e}"
        m = y[i, :n].abs().max().item()
        assert struct.unpack("<f", struct.pack("<i", int(amax[:, i].max().item())))[0] == m


@pytest.mark.parametrize("W,C,C2", [(16, 64, 32)])
def test_down_block_deterministic_and_group_size_independent(H, W, C, C2):
    """Repeated launches are bitwise identical, and a replica's bits do not depend on how many
    replicas share the launch (world-1 vs world-N runs group models differently)."""
    dev = torch.device("cuda")
    G = 3
    a, x2, w2, wsc, b2, bsc, _ = _case(H, dev, G, 5, W, C, C2, 1.0, 1.0, W + C)
    sel = torch.tensor([0, 1, 1], dtype=torch.int32, device=dev)
    with H.amax_arena(G, dev):
        y0 = H.down_block_eval(a, w2, b2, x2, wsc, bsc, sel)
        y1 = H.down_block_eval(a.clone(), w2, b2, x2.clone(), wsc, bsc, sel)
    assert torch.equal(y0, y1)
    for i in range(G):
        s = int(sel[i])
        wi = _split(H, w2[s:s + 1].clone())
        wsi = _split(H, wsc[s:s + 1].clone())
        with H.amax_arena(1, dev):
            yi = H.down_block_eval(a[i:i + 1].contiguous(), wi, b2[s:s + 1].contiguous(), x2[i:i + 1].contiguous(),
                                   wsi, bsc[s:s + 1].contiguous())
        assert torch.equal(yi[0], y0[i]), i
