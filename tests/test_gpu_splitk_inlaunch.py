"""In-launch split-K combine of the fp32 convs (``csrc/kernels/xconv.hpp`` ``sk_combine``) vs
the separate ``xsplitk_reduce`` launch it replaces (GPU only).

The K-slice blocks of a split launch (a lone client's stage-3/4 convs and data gradients,
``xsplitk``) store write-through slabs and draw arrival tickets; the last arriver sums the
slabs in z order — the reduce kernel's order — so every output bit must equal the two-launch
path: forward with bias / residual / ReLU, the data gradient with its accumulated input, for
a lone client with a full and a partly valid batch.  The combine also
lets the epilogue fold training-BN statistics of a split conv (previously a separate BN
reduce + finalize): those match fp64 statistics of the output to fp32 rounding.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dba_mod_amd.ops import hip
    yield hip


SHAPES = [
    # G, N, Hh, Cin, Cout, valid images (the combine runs for a lone client's 32 x 128 tiles)
    (1, 64, 4, 256, 256, 64),    # lone client, stage 4
    (1, 64, 8, 128, 128, 64),    # lone client, stage 3
    (1, 64, 8, 128, 128, 23),    # lone client, last (partial) batch
    (1, 40, 4, 256, 256, 40),
    # round 6: launches of up to 3 clients take the 32 x 128 tiles and the combine too
    (2, 64, 8, 128, 128, None),  # two clients, stage 3 (one partly valid)
    (3, 64, 4, 256, 256, None),  # three clients, stage 4 (full, partial, inactive)
]


def test_inlaunch_combine_scope(H):
    """Launches of up to 3 clients' stage-3/4 convs take the combine; larger groups take 64 /
    128-row tiles, where the separate reduce launch is cheaper."""
    assert int(H._L.dba_xconv_sk_ints(3, 64, 8, 8, 128, 128, 3, 3)) > 0
    assert int(H._L.dba_xconv_sk_ints(4, 64, 8, 8, 128, 128, 3, 3)) == 0
    assert int(H._L.dba_xconv_sk_ints(10, 64, 4, 4, 256, 256, 3, 3)) == 0
    assert int(H._L.dba_xconv_sk_ints(1, 64, 16, 16, 64, 64, 3, 3)) == 0   # no split


def _data(G, N, Hh, Cin, Cout, dev, seed=0, nv=None):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(G, N, Hh, Hh, Cin, generator=g).to(dev)
    w = (torch.randn(G, Cout, 3, 3, Cin, generator=g) / (9 * Cin) ** 0.5).to(dev)
    bias = torch.randn(G, Cout, generator=g).to(dev)
    res = torch.randn(G, N, Hh, Hh, Cout, generator=g).to(dev)
    dy = torch.randn(G, N, Hh, Hh, Cout, generator=g).to(dev)
    acc = torch.randn(G, N, Hh, Hh, Cin, generator=g).to(dev)
    nvalid = torch.tensor([N, N // 2 + 1, 0, N - 3][:G] if nv is None else [nv], dtype=torch.int32, device=dev)
    for i in range(G):
        dy[i, int(nvalid[i]):] = 0
    return x, w, bias, res, dy, acc, nvalid


def _valid_equal(a, b, nvalid):
    for g in range(a.shape[0]):
        n = int(nvalid[g])
        assert torch.equal(a[g, :n], b[g, :n]), g


@pytest.mark.parametrize("shape", SHAPES)
def test_inlaunch_combine_bitwise(H, shape):
    G, N, Hh, Cin, Cout, nv = shape
    dev = torch.device("cuda")
    x, w, bias, res, dy, acc, nvalid = _data(G, N, Hh, Cin, Cout, dev, nv=nv)
    assert int(H._L.dba_xconv_sk_ints(G, N, Hh, Hh, Cin, Cout, 3, 3)) > 0, "shape does not split"
    assert int(H._L.dba_xconv_sk_ints(G, N, Hh, Hh, Cout, Cin, 3, 3)) > 0, "dgrad does not split"

    def run(counters):
        with H.amax_arena(G, dev, counters=counters):
            y = H.conv2d(x, w, None, 1, 1, bias=bias, residual=res, relu=True, nvalid=nvalid)
            dx = H.conv2d_dgrad(dy, w, None, 1, 1, (Hh, Hh), nvalid=nvalid, accum=acc)
        torch.cuda.synchronize()
        return y, dx

    y0, dx0 = run(0)                  # separate reduce launches
    for _ in range(3):                # in-launch combine, repeated (ticket order varies)
        y1, dx1 = run(1 << 15)
        _valid_equal(y0, y1, nvalid)
        _valid_equal(dx0, dx1, nvalid)
    # fp32-level agreement with an fp64 conv (the bits above are the reduce path's)
    xd = x.double().permute(0, 1, 4, 2, 3)
    for g in range(G):
        n = int(nvalid[g])
        if n == 0:
            continue
        ref = torch.nn.functional.conv2d(xd[g, :n].cpu(), w[g].double().permute(0, 3, 1, 2).cpu(),
                                         bias[g].double().cpu(), padding=1).permute(0, 2, 3, 1)
        ref = (ref + res[g, :n].double().cpu()).clamp(min=0)
        err = ((y1[g, :n].double().cpu() - ref).norm() / ref.norm()).item()
        assert err < 1e-5, (g, err)


def test_inlaunch_combine_graph_replay(H):
    """Inside a captured graph the arena's fill re-zeroes the counters every replay."""
    G, N, Hh, Cin, Cout = 1, 64, 4, 256, 256
    dev = torch.device("cuda")
    x, w, bias, res, dy, acc, nvalid = _data(G, N, Hh, Cin, Cout, dev, seed=1)
    with H.amax_arena(G, dev, counters=0):
        ref = H.conv2d(x, w, None, 1, 1, bias=bias, relu=True, nvalid=nvalid)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):   # warm up the allocator outside the capture
            with H.amax_arena(G, dev, counters=1 << 12):
                H.conv2d(x, w, None, 1, 1, bias=bias, relu=True, nvalid=nvalid)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        with H.amax_arena(G, dev, counters=1 << 12):
            out = H.conv2d(x, w, None, 1, 1, bias=bias, relu=True, nvalid=nvalid)
    for _ in range(4):
        out.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)


def test_inlaunch_combine_many_launches_in_one_graph(H):
    """Eight consecutive in-launch split-K combines (a chain of lone-client stage-3/4 convs and
    their data gradients, each reading the previous output) captured in ONE graph and replayed
    repeatedly: every replay is bitwise equal to the same chain on the separate reduce kernel.
    Each launch's hand-off (sc1 slab stores, vmcnt(0), a relaxed agent ticket, sc1 loads) must
    hold while the previous launch's blocks drain and the next one's start (xconv_fwd.hip
    sk_combine; MI355X_MICROARCH.md § visibility, hand-off table row 1)."""
    G, N = 1, 64
    dev = torch.device("cuda")
    layers = []
    g = torch.Generator().manual_seed(3)
    for Hh, C in ((8, 128), (8, 128), (4, 256), (4, 256)):
        w = (torch.randn(G, C, 3, 3, C, generator=g) / (9 * C) ** 0.5).to(dev)
        layers.append((Hh, C, w))
    x0 = torch.randn(G, N, 8, 8, 128, generator=g).to(dev)
    x1 = torch.randn(G, N, 4, 4, 256, generator=g).to(dev)
    nvalid = torch.tensor([N], dtype=torch.int32, device=dev)

    def chain(counters):
        outs = []
        with H.amax_arena(G, dev, counters=counters):
            for i, (Hh, C, w) in enumerate(layers):
                src = (x0 if Hh == 8 else x1) if i in (0, 2) else outs[-1]
                y = H.conv2d(src, w, None, 1, 1, relu=True, nvalid=nvalid)
                dx = H.conv2d_dgrad(y, w, None, 1, 1, (Hh, Hh), nvalid=nvalid)
                outs += [y, dx]
        return outs

    for Hh, C, _ in layers:
        assert int(H._L.dba_xconv_sk_ints(G, N, Hh, Hh, C, C, 3, 3)) > 0, "shape does not split"
    ref = [t.clone() for t in chain(0)]          # separate reduce launches
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            chain(1 << 14)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        outs = chain(1 << 14)
    for _ in range(6):
        for t in outs:
            t.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        for a, b in zip(outs, ref):
            assert torch.equal(a, b)

