"""The fused evaluation BasicBlock (``csrc/kernels/xblock.hip``) vs an fp64 oracle and vs the
two-launch form it replaces (GPU only).

relu(conv2(relu(conv1(x) + b1)) + b2 + x) for the 32-wide stage with BN folded into the
weights — the identity BasicBlock of the reference ``models/resnet_cifar.py:14-37`` in
evaluation.  The kernel keeps the mid activation in LDS (split with the block's own scale), so
it is compared to the fp64 reference at fp32 level and to the two halo-conv launches to the
same level, not bitwise.  The STEM variant (stem + layer1.0 in one launch, the stem computed
on the MFMAs from the image rows) is compared to the fp64 stem + block and to the stem launch
followed by the fused block.
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


def _weights(H, slots, dev, g, scale, C=32):
    w = (torch.randn(slots, C, 3, 3, C, generator=g) * scale).to(dev)
    per = C * 9 * C
    H.split_weights(w, per, per, H._amax_w(w, per, per))
    return w


@pytest.mark.parametrize("G,N,nv,scale,W,C", [
    (3, 5, (5, 3, 5), 1.0, 32, 32), (2, 4, (4, 1), 1e-3, 32, 32), (1, 9, (9,), 30.0, 32, 32)])
def test_basic_block_eval_vs_fp64_and_two_launches(H, R64, G, N, nv, scale, W, C):
    """The 32-wide stage (8 output rows per workgroup, halo rows recomputed), partly valid
    replicas, a slot map and wide dynamic range."""
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(G * 100 + N + W)
    slots = 2
    x = torch.relu(torch.randn(G, N, W, W, C, generator=g) * scale).to(dev)
    w1 = _weights(H, slots, dev, g, 1.0 / (3 * C ** 0.5), C)
    w2 = _weights(H, slots, dev, g, 1.0 / (3 * C ** 0.5), C)
    b1 = (torch.randn(slots, C, generator=g) * 0.1 * scale).to(dev)
    b2 = (torch.randn(slots, C, generator=g) * 0.1 * scale).to(dev)
    wsel = torch.tensor([min(i, slots - 1) for i in range(G)], dtype=torch.int32, device=dev)
    nvalid = torch.tensor(nv, dtype=torch.int32, device=dev)
    assert H.basic_block_ok(x, w1, w2)
    with H.amax_arena(G, dev):
        y = H.basic_block_eval(x, w1, b1, w2, b2, wsel, nvalid)
        h = H.conv2d(x, w1, wsel, 1, 1, bias=b1, relu=True, nvalid=nvalid)
        y2 = H.conv2d(h, w2, wsel, 1, 1, bias=b2, residual=x, relu=True, nvalid=nvalid)
        amax = y._dba_amax.clone()
    torch.cuda.synchronize()
    yr = R64.basic_block_eval(x.double().cpu(), w1.double().cpu(), b1.double().cpu(), w2.double().cpu(),
                              b2.double().cpu(), wsel.cpu())
    for i in range(G):
        n = nv[i]
        e, e2 = _rel(y[i, :n], yr[i, :n]), _rel(y2[i, :n], yr[i, :n])
        assert e < 2e-6, f"replica {i}: fused {e:.2e} (two launches {e2:.2e})"
        assert e < max(2e-6, 2 * e2), f"replica {i}: fused {e:.2e} vs two launches {e2:.2e}"
        # the output's max |y| folded for its consumers (exact integer max of float bits)
        m = y[i, :n].abs().max().item()
        assert struct.unpack("<f", struct.pack("<i", int(amax[:, i].max().item())))[0] == m


def test_basic_block_eval_is_deterministic(H):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(7)
    x = torch.relu(torch.randn(2, 6, 32, 32, 32, generator=g)).to(dev)
    w1, w2 = _weights(H, 2, dev, g, 0.06), _weights(H, 2, dev, g, 0.06)
    b1, b2 = torch.randn(2, 32, generator=g).to(dev) * 0.1, torch.randn(2, 32, generator=g).to(dev) * 0.1
    outs = []
    for _ in range(3):
        with H.amax_arena(2, dev):
            outs.append(H.basic_block_eval(x, w1, b1, w2, b2))
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def _stem_weights(H, slots, dev, g, C=32):
    w = (torch.randn(slots, C, 3, 3, 3, generator=g) * 0.3).to(dev)
    per = C * 27
    H.split_weights(w, per, per, H._amax_w(w, per, per))
    return w


@pytest.mark.parametrize("G,N,nv,scale", [(3, 5, (5, 2, 5), 1.0), (2, 4, (4, 3), 1e-3), (1, 9, (9,), 40.0)])
def test_stem_block_eval_vs_fp64_and_separate_launches(H, R64, G, N, nv, scale):
    """The stem recomputed in the block (x = relu(stem(img) + b0) never stored): signed image
    values over a wide range, partly valid replicas, a slot map."""
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(1000 + G * 10 + N)
    slots = 2
    img = (torch.randn(G, N, 32, 32, 3, generator=g) * scale).to(dev)
    w0 = _stem_weights(H, slots, dev, g)
    w1 = _weights(H, slots, dev, g, 1.0 / (3 * 32 ** 0.5))
    w2 = _weights(H, slots, dev, g, 1.0 / (3 * 32 ** 0.5))
    b0, b1, b2 = [(torch.randn(slots, 32, generator=g) * 0.1 * scale).to(dev) for _ in range(3)]
    wsel = torch.tensor([min(i, slots - 1) for i in range(G)], dtype=torch.int32, device=dev)
    nvalid = torch.tensor(nv, dtype=torch.int32, device=dev)
    assert H.stem_block_ok(img, w0, w1, w2)
    with H.amax_arena(G, dev):
        y = H.stem_block_eval(img, w0, b0, w1, b1, w2, b2, wsel, nvalid)
        s = H.conv2d(img, w0, wsel, 1, 1, bias=b0, relu=True, nvalid=nvalid)
        y2 = H.basic_block_eval(s, w1, b1, w2, b2, wsel, nvalid)
        amax = y._dba_amax.clone()
    torch.cuda.synchronize()
    cpu = [t.double().cpu() for t in (img, w0, b0, w1, b1, w2, b2)]
    yr = R64.stem_block_eval(*cpu, wsel.cpu())
    for i in range(G):
        n = nv[i]
        e, e2 = _rel(y[i, :n], yr[i, :n]), _rel(y2[i, :n], yr[i, :n])
        assert e < 2e-6, f"replica {i}: fused {e:.2e} (separate {e2:.2e})"
        assert e < max(2e-6, 2 * e2), f"replica {i}: fused {e:.2e} vs separate {e2:.2e}"
        m = y[i, :n].abs().max().item()
        assert struct.unpack("<f", struct.pack("<i", int(amax[:, i].max().item())))[0] == m


def test_stem_block_eval_is_deterministic(H):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(11)
    img = torch.randn(2, 6, 32, 32, 3, generator=g).to(dev)
    w0 = _stem_weights(H, 2, dev, g)
    w1, w2 = _weights(H, 2, dev, g, 0.06), _weights(H, 2, dev, g, 0.06)
    b0, b1, b2 = [torch.randn(2, 32, generator=g).to(dev) * 0.1 for _ in range(3)]
    outs = []
    for _ in range(3):
        with H.amax_arena(2, dev):
            outs.append(H.stem_block_eval(img, w0, b0, w1, b1, w2, b2))
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])

