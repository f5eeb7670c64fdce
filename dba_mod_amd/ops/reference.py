"""Plain-PyTorch fp32 reference implementation of every framework op.

This is (a) the implementation used for CPU tensors (the world_size=1 plumbing config and
the unit tests) and (b) the numerics oracle the HIP kernels are tested against.  Layouts
are the device layouts: activations ``[G, N, H, W, C]`` (group = client replica / eval job),
conv weights ``[Gm, Cout, KH, KW, Cin]`` (possibly a strided view into a flat parameter
buffer), per-group model selection ``wsel`` (group -> weight slot).

Semantics follow the reference's stock-PyTorch ops: BatchNorm2d in
train mode (biased var to normalise, unbiased var into running stats, momentum 0.1),
cross-entropy mean/sum reductions, ``torch.optim.SGD`` with momentum + weight decay.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from . import bnstate as bs
from . import rng

Tensor = torch.Tensor


def _sel(w: Tensor, wsel: Optional[Tensor], g: int) -> Tensor:
    return w[int(wsel[g])] if wsel is not None else w[g]


def _nchw(x: Tensor) -> Tensor:
    return x.permute(0, 3, 1, 2)


def _nhwc(x: Tensor) -> Tensor:
    return x.permute(0, 2, 3, 1)


# Compute dtype of the reference implementation: fp32 (the kernels' accumulation dtype);
# tests switch it to fp64 to get an oracle free of fp32 ReLU-mask flips.
COMPUTE_DTYPE = torch.float32


def _cdt() -> torch.dtype:
    return COMPUTE_DTYPE


def _rows_valid(nvalid: Optional[Tensor], g: int, n: int) -> int:
    return n if nvalid is None else int(nvalid[g])


# ------------------------------------------------------------------------- data ingest
def gather_images(src: Tensor, labels: Tensor, idx: Tensor, trig_masks: Tensor, trig_id: Tensor,
                  poison_n: Tensor, target: int, flip_seeds: Optional[Tensor], out_dtype: torch.dtype
                  ) -> Tuple[Tensor, Tensor]:
    """uint8 NHWC gather + /255 + optional h-flip + pixel trigger + relabel (K17/K19).

    Row ``b`` of group ``g`` is flipped iff ``hash2(flip_seeds[g], b) & 1`` (per-client
    seeds keep the result independent of how clients are placed on ranks/groups).
    """
    G, B = idx.shape
    _, H, W, C = src.shape
    valid = idx >= 0
    safe = idx.clamp(min=0).long()
    x = src[safe.reshape(-1)].reshape(G, B, H, W, C).to(torch.float32)
    y = labels.long()[safe.reshape(-1)].reshape(G, B)
    if flip_seeds is not None:
        ctr = torch.arange(B, dtype=torch.int64, device=src.device)[None, :].expand(G, B)
        flip = (rng.hash2(flip_seeds.to(torch.int64)[:, None], ctr) & 1).bool()
        x = torch.where(flip[..., None, None, None], x.flip(3), x)
    b_ar = torch.arange(B, device=src.device)[None, :]
    tid = trig_id.long()
    pois = (b_ar < poison_n.long()[:, None]) & (tid[:, None] >= 0) & valid
    if trig_masks.numel() > 0:
        m = trig_masks[tid.clamp(min=0)].bool()  # [G, H, W]
        pm = pois[:, :, None, None] & m[:, None, :, :]
        x = torch.where(pm[..., None], torch.full_like(x, 255.0), x)
    y = torch.where(pois, torch.full_like(y, int(target)), y)
    x = x * (1.0 / 255.0)
    x = torch.where(valid[..., None, None, None], x, torch.zeros_like(x))
    y = torch.where(valid, y, torch.full_like(y, -1))
    return x.to(out_dtype), y.to(torch.int32)


def gather_rows(src: Tensor, labels: Tensor, idx: Tensor, trig_cols: Tensor, trig_vals: Tensor,
                trig_id: Tensor, poison_n: Tensor, target: int, out_dtype: torch.dtype
                ) -> Tuple[Tensor, Tensor]:
    """Tabular (LOAN) gather + feature trigger (K18): x[:, col] = value for poisoned rows."""
    G, B = idx.shape
    Fd = src.shape[1]
    valid = idx >= 0
    safe = idx.clamp(min=0).long()
    x = src[safe.reshape(-1)].reshape(G, B, Fd).to(torch.float32).clone()
    y = labels.long()[safe.reshape(-1)].reshape(G, B)
    b_ar = torch.arange(B, device=src.device)[None, :]
    tid = trig_id.long()
    pois = (b_ar < poison_n.long()[:, None]) & (tid[:, None] >= 0) & valid
    for g in range(G):
        if int(tid[g]) < 0:
            continue
        cols = trig_cols[int(tid[g])]
        vals = trig_vals[int(tid[g])]
        rows = pois[g].nonzero().flatten()
        for k in range(cols.shape[0]):
            c = int(cols[k])
            if c >= 0:
                x[g, rows, c] = float(vals[k])
    y = torch.where(pois, torch.full_like(y, int(target)), y)
    x = torch.where(valid[..., None], x, torch.zeros_like(x))
    y = torch.where(valid, y, torch.full_like(y, -1))
    return x.to(out_dtype), y.to(torch.int32)


# ------------------------------------------------------------------------------ conv
def conv2d(x: Tensor, w: Tensor, wsel: Optional[Tensor], stride: int, pad: int,
           bias: Optional[Tensor] = None, residual: Optional[Tensor] = None,
           relu: bool = False, nvalid: Optional[Tensor] = None,
           out_dtype: Optional[torch.dtype] = None, bn_stats: bool = False) -> Tensor:
    """y = act(conv(x, w) + bias + residual); NHWC in/out (K1, K3, K4, K8).  ``bn_stats`` (a
    hint that y feeds a training BN) only matters to the HIP backend."""
    G = x.shape[0]
    outs = []
    for g in range(G):
        wg = _sel(w, wsel, g).to(_cdt()).permute(0, 3, 1, 2)  # [Cout, Cin, KH, KW]
        bg = _sel(bias, wsel, g).to(_cdt()) if bias is not None else None
        yg = F.conv2d(_nchw(x[g].to(_cdt())), wg, bg, stride=stride, padding=pad)
        yg = _nhwc(yg)
        if residual is not None:
            yg = yg + residual[g].to(_cdt())
        if relu:
            yg = torch.relu(yg)
        outs.append(yg)
    if out_dtype == torch.float32 and _cdt() == torch.float64:
        out_dtype = torch.float64
    return torch.stack(outs).to(out_dtype or x.dtype)


def basic_block_ok(x: Tensor, w1: Tensor, w2: Tensor) -> bool:
    """Whether the backend runs an evaluation BasicBlock as one fused op (HIP: xblock.hip);
    the reference runs the two convs."""
    return False


def basic_block_eval(x: Tensor, w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor,
                     wsel: Optional[Tensor] = None, nvalid: Optional[Tensor] = None) -> Tensor:
    """relu(conv2(relu(conv1(x) + b1)) + b2 + x), 3x3 stride-1 convs with BN folded into w / b
    (the identity BasicBlock of the reference models/resnet_cifar.py:14-37, evaluated)."""
    h = conv2d(x, w1, wsel, 1, 1, bias=b1, relu=True, nvalid=nvalid)
    return conv2d(h, w2, wsel, 1, 1, bias=b2, residual=x, relu=True, nvalid=nvalid)


def stem_block_ok(x: Tensor, w0: Tensor, w1: Tensor, w2: Tensor) -> bool:
    """Whether the backend runs the stem + first BasicBlock as one fused op (HIP: xblock.hip
    STEM variant); the reference runs the three convs."""
    return False


def stem_block_eval(x: Tensor, w0: Tensor, b0: Tensor, w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor,
                    wsel: Optional[Tensor] = None, nvalid: Optional[Tensor] = None) -> Tensor:
    """The CIFAR ResNet stem relu(conv(x) + b0) (3x3, pad 1) followed by the identity
    BasicBlock of :func:`basic_block_eval`, BN folded (reference models/resnet_cifar.py:80-88)."""
    s = conv2d(x, w0, wsel, 1, 1, bias=b0, relu=True, nvalid=nvalid)
    return basic_block_eval(s, w1, b1, w2, b2, wsel, nvalid)


def down_block_ok(a: Tensor, w2: Tensor, x2: Tensor, wsc: Tensor) -> bool:
    """Whether the backend runs a downsampling block's conv2 with its 1x1 stride-2 shortcut as
    one fused op (HIP: xconv_fwd.hip dba_xdown_fwd); the reference runs the two convs."""
    return False


def down_block_eval(a: Tensor, w2: Tensor, b2: Tensor, x2: Tensor, wsc: Tensor, bsc: Tensor,
                    wsel: Optional[Tensor] = None, nvalid: Optional[Tensor] = None) -> Tensor:
    """relu(conv3x3(a, w2) + b2 + conv1x1_s2(x2, wsc) + bsc), BN folded: the second half of a
    downsampling BasicBlock with its shortcut (reference models/resnet_cifar.py:24-36), evaluated."""
    sc = conv2d(x2, wsc, wsel, 2, 0, bias=bsc, nvalid=nvalid)
    return conv2d(a, w2, wsel, 1, 1, bias=b2, residual=sc, relu=True, nvalid=nvalid)


def _valid_mask(t: Tensor, nvalid: Optional[Tensor]) -> Tensor:
    """[G, N, 1, 1, 1] (bool) of the valid images of each replica."""
    G, N = t.shape[:2]
    n = torch.full((G,), N, dtype=torch.int64) if nvalid is None else nvalid.long().cpu()
    v = torch.arange(N)[None, :] < n[:, None]
    return v.view(G, N, *([1] * (t.dim() - 2))).to(t.device)


def _coef(st: "bs.BnStat", row: int, t: Tensor) -> Tensor:
    """Row ``row`` of a BN's coefficients broadcast over ``t`` [G, N, H, W, C]."""
    return st.coef[:, row].view(t.shape[0], *([1] * (t.dim() - 2)), t.shape[-1]).to(t.dtype)


def lazy_value(a: "bs.LazyBN", nvalid: Optional[Tensor] = None) -> Tensor:
    """relu?(y * scale + shift) of a lazy training-BN output (zero on invalid images).  A
    replayed ReLU decision (``ops.branches``) is taken from ``a.stat.relu_mask``."""
    v = a.y * _coef(a.stat, bs.SCALE, a.y) + _coef(a.stat, bs.SHIFT, a.y)
    if a.relu:
        m = getattr(a.stat, "relu_mask", None)   # replayed decisions (ops.branches)
        tiny = 1e-300 if v.dtype == torch.float64 else 1e-30
        v = torch.relu(v) if m is None else torch.where(m.to(v.device), v.clamp(min=tiny), torch.zeros_like(v))
    return torch.where(_valid_mask(v, nvalid), v, torch.zeros_like(v))


def lazy_grad_value(lg: "bs.LazyGrad", nvalid: Optional[Tensor] = None) -> Tensor:
    """dy = A * d + B * y + K of a training BN's input gradient (zero on invalid images)."""
    st = lg.stat
    v = _coef(st, bs.A, lg.d) * lg.d + _coef(st, bs.B, lg.y) * lg.y + _coef(st, bs.K, lg.d)
    return torch.where(_valid_mask(v, nvalid), v, torch.zeros_like(v)).to(lg.d.dtype)


def conv_bn_stats(x, w: Tensor, wsel: Optional[Tensor], stride: int, pad: int, nvalid: Optional[Tensor],
                  p: "bs.BnParams", relu: bool):
    """y = conv(x, w) and the training-BN statistics of y (running stats updated in place);
    x may be a lazy BN output.  Returns (y, BnStat) — the fused conv + BN forward
    (csrc/kernels/bnfuse.hpp); the BN output is :func:`lazy_value` of ``LazyBN(y, stat, relu)``."""
    xv = lazy_value(x, nvalid) if isinstance(x, bs.LazyBN) else x
    y = conv2d(xv, w, wsel, stride, pad, nvalid=nvalid)
    G, N = y.shape[:2]
    C = y.shape[-1]
    coef = torch.zeros(G, bs.ROWS, C, dtype=_cdt(), device=y.device)
    for g in range(G):
        n = _rows_valid(nvalid, g, N)
        if n == 0:
            continue
        flat = y[g, :n].to(_cdt()).reshape(-1, C)
        cnt = flat.shape[0]
        mean = flat.mean(0)
        var = flat.var(0, unbiased=False)
        invstd = torch.rsqrt(var + p.eps)
        unbiased = var * (cnt / max(cnt - 1, 1))
        p.rmean[g] = (1 - p.momentum) * p.rmean[g] + p.momentum * mean
        p.rvar[g] = (1 - p.momentum) * p.rvar[g] + p.momentum * unbiased
        sc = invstd * p.gamma[g].to(_cdt())
        coef[g, bs.MEAN], coef[g, bs.INV] = mean, invstd
        coef[g, bs.SCALE], coef[g, bs.SHIFT] = sc, p.beta[g].to(_cdt()) - mean * sc
        coef[g, bs.YMAX], coef[g, bs.YMIN] = flat.max(0).values, flat.min(0).values
    return y, bs.BnStat(coef, p)


def bn_apply(a: "bs.LazyBN", residual, relu: bool, nvalid: Optional[Tensor] = None) -> Tensor:
    """out = relu?(lazy BN value of ``a`` (its own ReLU not applied) + residual), residual a
    tensor, a lazy BN output or None: the stored output of a BasicBlock / the stem."""
    v = a.y * _coef(a.stat, bs.SCALE, a.y) + _coef(a.stat, bs.SHIFT, a.y)
    if isinstance(residual, bs.LazyBN):
        v = v + lazy_value(residual, nvalid)
    elif residual is not None:
        v = v + residual.to(v.dtype)
    if relu:
        v = torch.relu(v)
    return torch.where(_valid_mask(v, nvalid), v, torch.zeros_like(v)).to(a.y.dtype)


def bn_finish(g: Optional[Tensor], fin: "bs.Finish", nvalid: Optional[Tensor] = None,
              pool: Optional[Tensor] = None, hw: Optional[Tuple[int, int]] = None) -> "bs.Fin":
    """Finish the gradient of a BN output: d = g where the output is > 0, then the backward
    sums of BN a (and BN b) -> dbeta += sum d, dgamma += sum d * xhat and the coefficients A, B,
    K of dy = A d + B y + K (bn_train_bwd's arithmetic).  ``pool`` ([G, N, 1, 1, C]): g is the
    global average pool's gradient of it (``avgpool_global_bwd``)."""
    if pool is not None:
        g = avgpool_global_bwd(pool, hw)
    ya = fin.ya
    d = g.to(_cdt())
    if fin.mask_out is not None:
        d = d * (fin.mask_out.to(_cdt()) > 0)
    elif fin.lazy:
        m = getattr(fin.sa, "relu_mask", None)
        pre = ya.to(_cdt()) * _coef(fin.sa, bs.SCALE, ya).to(_cdt()) + _coef(fin.sa, bs.SHIFT, ya).to(_cdt())
        d = d * ((pre > 0) if m is None else m.to(d.device))
    d = torch.where(_valid_mask(d, nvalid), d, torch.zeros_like(d))
    G, N = d.shape[:2]
    C = d.shape[-1]
    for y, st in ((ya, fin.sa), (fin.yb, fin.sb)):
        if st is None:
            continue
        p = st.params
        for gg in range(G):
            n = _rows_valid(nvalid, gg, N)
            if n == 0:
                continue
            dg = d[gg, :n].reshape(-1, C)
            mean, inv = st.coef[gg, bs.MEAN].to(_cdt()), st.coef[gg, bs.INV].to(_cdt())
            xhat = (y[gg, :n].to(_cdt()).reshape(-1, C) - mean) * inv
            cnt = dg.shape[0]
            sd, sdx = dg.sum(0), (dg * xhat).sum(0)
            p.dbeta[gg] += sd.to(p.dbeta.dtype)
            p.dgamma[gg] += sdx.to(p.dgamma.dtype)
            A = p.gamma[gg].to(_cdt()) * inv
            B = -A * inv * sdx / cnt
            st.coef[gg, bs.A], st.coef[gg, bs.B] = A, B
            st.coef[gg, bs.K] = -A * sd / cnt - B * mean
    return bs.Fin(d.to(g.dtype), fin.stats())


def wgrad_prepare(dy, x, nvalid=None):
    """HIP backend: attaches the operands' fp16-pair maxima before the weight gradient moves to
    a side stream.  Nothing to prepare here."""
    return None


def wgrad_flush(defer: list) -> None:
    """Backend hook for deferred weight-gradient reductions; the reference has none."""
    if defer:
        defer.clear()


def prepare_dgrad_weights(ref: Tensor, items: list) -> dict:
    """Backend hook for pre-transposed data-gradient weights; the reference needs none."""
    return {}


def conv2d_dgrad(dy: Tensor, w: Tensor, wsel: Optional[Tensor], stride: int, pad: int,
                 in_hw: Tuple[int, int], nvalid: Optional[Tensor] = None,
                 out_dtype: Optional[torch.dtype] = None, accum: Optional[Tensor] = None,
                 wt: Optional[Tensor] = None, finish: Optional["bs.Finish"] = None):
    """dX of a conv; ``accum`` (the input's gradient from another branch) is added in.
    ``wt`` (a backend's pre-transposed weights) is ignored here.  ``finish``: dX is the complete
    gradient of a training-BN output — return it finished (:func:`bn_finish`, a ``Fin``)."""
    if finish is not None:
        dx = conv2d_dgrad(dy, w, wsel, stride, pad, in_hw, nvalid, out_dtype, accum, wt)
        return bn_finish(dx, finish, nvalid)
    G, N = dy.shape[:2]
    cin = w.shape[-1]
    outs = []
    for g in range(G):
        wg = _sel(w, wsel, g).to(_cdt()).permute(0, 3, 1, 2)
        dx = torch.nn.grad.conv2d_input((N, cin, in_hw[0], in_hw[1]), wg, _nchw(dy[g].to(_cdt())),
                                        stride=stride, padding=pad)
        outs.append(_nhwc(dx))
    dx = torch.stack(outs)
    if accum is not None:
        dx = dx + accum.to(dx.dtype)
    return dx.to(out_dtype or dy.dtype)


def conv2d_wgrad(dy, x, stride: int, pad: int, kh: int, kw: int,
                 dw: Tensor, dbias: Optional[Tensor] = None, nvalid: Optional[Tensor] = None,
                 defer: Optional[list] = None) -> Optional[Tensor]:
    """dw[g] += sum_rows dy (x) x  (fp32 accumulate into the flat grad buffer view).
    ``defer`` (a backend's batched-reduction queue) is unused here: the sum is immediate.
    ``dy`` may be a :class:`LazyGrad` (its value is returned, for the data gradient) and ``x`` a
    :class:`LazyBN`."""
    out = None
    if isinstance(dy, bs.LazyGrad):
        dy = out = lazy_grad_value(dy, nvalid)
    if isinstance(x, bs.LazyBN):
        x = lazy_value(x, nvalid)
    G = dy.shape[0]
    cout = dy.shape[-1]
    cin = x.shape[-1]
    for g in range(G):
        gw = torch.nn.grad.conv2d_weight(_nchw(x[g].to(_cdt())), (cout, cin, kh, kw),
                                         _nchw(dy[g].to(_cdt())), stride=stride, padding=pad)
        dw[g] += gw.permute(0, 2, 3, 1)
        if dbias is not None:
            dbias[g] += dy[g].to(_cdt()).sum(dim=(0, 1, 2))
    return out


# ------------------------------------------------------------------------ batch norm
def relu_mask_bwd(dout: Tensor, out: Tensor) -> Tensor:
    return (dout.to(_cdt()) * (out.to(_cdt()) > 0)).to(dout.dtype)


def bn_fold(w: Tensor, conv_bias: Optional[Tensor], gamma: Tensor, beta: Tensor,
            rmean: Tensor, rvar: Tensor, eps: float, out_dtype: torch.dtype,
            amax_slot: Optional[Tensor] = None, split: bool = True) -> Tuple[Tensor, Tensor]:
    """Eval-mode BN folded into the preceding conv: w' = w*s, b' = (b - mean)*s + beta.
    (``amax_slot`` / ``split``: the HIP backend's operand-max slot and fp16-pair split; unused here.)"""
    s = gamma.to(_cdt()) * torch.rsqrt(rvar.to(_cdt()) + eps)  # [Gm, Cout]
    wf = w.to(_cdt()) * s[:, :, None, None, None]
    b0 = conv_bias.to(_cdt()) if conv_bias is not None else torch.zeros_like(s)
    bf = (b0 - rmean.to(_cdt())) * s + beta.to(_cdt())
    return wf.to(out_dtype), bf.contiguous()


# --------------------------------------------------------------------------- pooling
def maxpool2d(x: Tensor, k: int, s: int, p: int, want_ind: bool = True) -> Tuple[Tensor, Optional[Tensor]]:
    """K7 max-pool; ``want_ind`` is a HIP hint (evaluation stores no indices): the reference
    always returns them."""
    G, N, H, W, C = x.shape
    y, ind = F.max_pool2d(_nchw(x.to(_cdt()).reshape(G * N, H, W, C)), k, s, p, return_indices=True)
    return (_nhwc(y).reshape(G, N, y.shape[2], y.shape[3], C).to(x.dtype),
            _nhwc(ind).reshape(G, N, y.shape[2], y.shape[3], C).to(torch.int32))


def maxpool2d_bwd(dy: Tensor, ind: Tensor, in_shape: Sequence[int], k: int, s: int, p: int) -> Tensor:
    G, N, H, W, C = in_shape
    Ho, Wo = dy.shape[2], dy.shape[3]
    dyn = _nchw(dy.to(_cdt()).reshape(G * N, Ho, Wo, C)).contiguous()
    indn = _nchw(ind.long().reshape(G * N, Ho, Wo, C)).contiguous()
    dx = torch.zeros(G * N, C, H * W, dtype=_cdt(), device=dy.device)
    dx.scatter_add_(2, indn.reshape(G * N, C, -1), dyn.reshape(G * N, C, -1))
    return _nhwc(dx.reshape(G * N, C, H, W)).reshape(G, N, H, W, C).to(dy.dtype)


def avgpool_global(x: Tensor) -> Tensor:
    return x.to(_cdt()).mean(dim=(2, 3), keepdim=True).to(x.dtype)


def avgpool_global_bwd(dy: Tensor, hw: Tuple[int, int]) -> Tensor:
    H, W = hw
    return (dy.to(_cdt()).expand(-1, -1, H, W, -1) / (H * W)).to(dy.dtype).contiguous()


# --------------------------------------------------------------------------- dropout
def dropout(x: Tensor, p: float, seeds: Tensor, salt: int) -> Tensor:
    """Inverted dropout; element i of group g kept iff uniform(salted(seeds[g]), i) >= p."""
    G = x.shape[0]
    per = x[0].numel()
    ctr = torch.arange(per, dtype=torch.int64, device=x.device)[None, :].expand(G, per)
    s = rng.salted(seeds.to(torch.int64), salt)[:, None]
    keep = (rng.uniform01(s, ctr) >= p).reshape(x.shape)
    return (x.to(_cdt()) * keep / (1.0 - p)).to(x.dtype)


def dropout_bwd(dy: Tensor, p: float, seeds: Tensor, salt: int) -> Tensor:
    return dropout(dy, p, seeds, salt)


# ---------------------------------------------------------------------------- loss
def softmax_xent(logits: Tensor, labels: Tensor, mean: bool, want_grad: bool,
                 stats: Optional[Tensor] = None, slot: Optional[Tensor] = None,
                 nvalid: Optional[Tensor] = None, grad_dtype: Optional[torch.dtype] = None,
                 loss_dtype: Optional[torch.dtype] = None) -> Tuple[Tensor, Tensor, Optional[Tensor]]:
    """Per-group CE (mean over valid rows or sum) + correct count + dlogits (K9).

    ``grad_dtype``: dtype of dlogits (default: the logits' dtype).  ``loss_dtype`` fp64: the
    per-row losses are summed in fp64 (the sum then does not depend on how rows are grouped
    into chunks or sharded over ranks).

    Rows with label < 0 are padding.  dlogits corresponds to the *mean* loss when
    ``mean`` (training) and to the sum otherwise.  With ``stats`` ([3, G*max_slots] fp32),
    also accumulates (loss, correct, nvalid) of group g into column g*max_slots + slot[g]
    (the per-client per-internal-epoch training statistics).
    """
    G, B, C = logits.shape
    lf = logits.to(_cdt())
    lab = labels.long()
    valid = lab >= 0
    logp = torch.log_softmax(lf, dim=-1)
    nll = -logp.gather(-1, lab.clamp(min=0)[..., None]).squeeze(-1)
    nll = torch.where(valid, nll, torch.zeros_like(nll))
    cnt = valid.sum(1).clamp(min=1).to(_cdt())
    if loss_dtype == torch.float64:
        nll = nll.to(torch.float64)
        cnt = cnt.to(torch.float64)
    loss = nll.sum(1) / cnt if mean else nll.sum(1)
    pred = lf.argmax(-1)
    correct = ((pred == lab) & valid).sum(1).to(_cdt())
    dl = None
    if want_grad:
        dl = torch.softmax(lf, -1)
        dl = dl - F.one_hot(lab.clamp(min=0), C).to(_cdt())
        dl = torch.where(valid[..., None], dl, torch.zeros_like(dl))
        if mean:
            dl = dl / cnt[:, None, None]
        dl = dl.to(grad_dtype or logits.dtype)
    if stats is not None:
        accumulate_step_stats(stats, slot, loss, correct, nvalid)
    return loss, correct, dl


def accumulate_step_stats(stats: Tensor, slot: Tensor, loss: Tensor, correct: Tensor, nvalid: Tensor) -> None:
    """stats[:, g*max_slots + slot[g]] += (loss[g], correct[g], nvalid[g])."""
    G = loss.shape[0]
    ms = stats.shape[1] // G
    col = torch.arange(G, device=stats.device, dtype=torch.int64) * ms + slot.long()
    stats[0].index_add_(0, col, loss.to(stats.dtype))
    stats[1].index_add_(0, col, correct.to(stats.dtype))
    stats[2].index_add_(0, col, nvalid.to(stats.dtype))


# ------------------------------------------------------------------------- optimizer
def sgd_step(params: Tensor, grads: Tensor, mom: Tensor, lr: Tensor, first: Tensor, active: Tensor,
             momentum: float, wd: float, fg_accum: Optional[Tensor] = None) -> None:
    """torch.optim.SGD(momentum, weight_decay) on [G, P] flat buffers (K10).

    ``first[g]`` marks the first step of a freshly created optimizer (buffer := d_p).
    ``fg_accum`` (FoolsGold) accumulates the raw per-batch gradients (image_train.py:94-100).
    """
    for g in range(params.shape[0]):
        if int(active[g]) == 0:
            continue
        gr = grads[g]
        if fg_accum is not None:
            fg_accum[g] += gr
        dp = gr + wd * params[g]
        if int(first[g]):
            mom[g] = dp
        else:
            mom[g] = momentum * mom[g] + dp
        params[g] -= float(lr[g]) * mom[g]


def dist_loss_grad(w: Tensor, base: Tensor, grads: Tensor, trig: Tensor, active: Tensor,
                   alpha: float) -> Tensor:
    """Anomaly-evasion loss a*CE + (1-a)*||w - w_g||_2 (helper.py:111-123, image_train.py:87-90).

    For replicas in a poison phase (``trig >= 0``) rewrites ``grads`` (the CE gradient) to
    ``a*g + (1-a)(w - base)/||w - base||`` (0 where w == base, torch's norm subgradient);
    returns the per-replica distance ``||w - base||`` over the parameter region.
    """
    G, P = grads.shape
    out = torch.zeros(G, dtype=torch.float32, device=grads.device)
    for g in range(G):
        if int(trig[g]) < 0 or int(active[g]) == 0:
            continue
        d = w[g, :P] - base[g, :P]
        nr = torch.linalg.vector_norm(d.double()).float()
        out[g] = nr
        c = (1.0 - alpha) / nr if float(nr) > 0 else 0.0
        grads[g] = alpha * grads[g] + c * d
    return out


# ---------------------------------------------------------------- flat / aggregation
def scale_from_base(w: Tensor, base: Tensor, gamma: float) -> Tensor:
    """Model-replacement scaling w' = base + gamma (w - base) (K11, image_train.py:166-171)."""
    return base + (w - base) * gamma


def add_noise_scaled(dst: Tensor, upd: Tensor, coef: float, sigma: float, seed: int,
                     noise: bool) -> None:
    """dst += coef*upd (+ N(0, sigma) per element if noise)  (K12, helper.py:240-257).
    ``upd`` may be fp64 (the FedAvg delta sum): the product is rounded to fp32 once."""
    u = (upd * coef).to(dst.dtype)
    if noise:
        ctr = torch.arange(u.numel(), dtype=torch.int64, device=u.device).reshape(u.shape)
        u = u + sigma * rng.normal(seed, ctr)
    dst += u


def delta_sum(rows: Tensor, base: Tensor) -> Tensor:
    """sum_r (rows[r] - base) in fp64 (FedAvg's per-rank Σ-delta, K12; helper.py:218-222).
    fp32 deltas summed in fp64 are exact, so a cross-rank all-reduce of the partial sums
    gives the same total as one rank summing all clients."""
    n = base.numel()
    if rows.shape[0] == 0:
        return torch.zeros(n, dtype=torch.float64, device=base.device)
    return (rows[:, :n].double() - base.double()[None]).sum(0)


def sq_dists(points: Tensor, m: Tensor) -> Tensor:
    """||points[i] - m||^2 for all i in one pass (K13)."""
    d = points.double() - m.double()[None]
    return (d * d).sum(1)


def weighted_sum(points: Tensor, wts: Tensor, out_dtype: Optional[torch.dtype] = None) -> Tensor:
    """sum_i wts[i] * points[i] (K14/K16); ``out_dtype`` fp64 keeps a partial sum unrounded."""
    return (wts.double()[:, None] * points.double()).sum(0).to(out_dtype or points.dtype)


def weighted_sum_fixed(points: Tensor, wts: Tensor, E: int) -> Tensor:
    """[2, L] int64 limb sums of sum_i wts[i] * points[i] on the fixed grid 2^-(E + 53): each
    product (exact in fp64) quantised on its own, hi = floor(q), lo = floor((q - hi) 2^53), q =
    w p 2^E, then summed exactly (order-free; flat.hip wsum_fixed_kernel is the GPU form)."""
    q = (wts.float().double()[:, None] * points.double()) * (2.0 ** E)
    hi = torch.floor(q)
    lo = torch.floor((q - hi) * 2.0 ** 53)
    return torch.stack([hi.to(torch.int64).sum(0), lo.to(torch.int64).sum(0)])


def gram(feats: Tensor) -> Tensor:
    """F F^T in float64 (K15)."""
    f = feats.double()
    return f @ f.t()
