"""Functional model programs over grouped replicas, with a minimal reverse-mode tape.

One forward definition per architecture serves three modes:

* ``train`` — BatchNorm with batch statistics (running stats updated in place), every op
  records a backward closure on a :class:`Tape`; ``Tape.backward`` writes parameter
  gradients straight into the flat ``[G, P]`` gradient buffer (no autograd, no per-tensor
  ``.grad``), so the whole step is a fixed launch sequence that a HIP graph can capture.
* ``eval`` — BatchNorm folded into the conv weights/bias (:func:`fold_bank`), so every conv
  is one kernel with a fused bias + residual + ReLU epilogue.

All activations are ``[G, N, H, W, C]``: G client replicas (training) or G eval jobs, each
selecting its weights through ``wsel``.  Reference forward definitions: see
:mod:`dba_mod_amd.models.mirror`.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Tuple

import torch

from .. import ops
from .mirror import CIFAR_RESNETS
from .spec import ModelSpec

Tensor = torch.Tensor
BN_EPS = 1e-5
BN_MOMENTUM = 0.1


class Tape:
    """Reverse-mode tape: nodes hold (outputs, inputs, backward closure)."""

    def __init__(self) -> None:
        self.nodes: List[Tuple[Tuple[Tensor, ...], Tuple[Optional[Tensor], ...], Callable]] = []
        self._produced: set = set()
        self._grads: Optional[Dict[int, Tensor]] = None
        self.on_begin: Optional[Callable[[], None]] = None
        self.on_end: Optional[Callable[[], None]] = None

    def record(self, outputs: Tuple[Tensor, ...], inputs: Tuple[Optional[Tensor], ...], bwd: Callable) -> None:
        self.nodes.append((outputs, inputs, bwd))
        for o in outputs:
            self._produced.add(id(o))

    def needs_grad(self, t: Optional[Tensor]) -> bool:
        return t is not None and id(t) in self._produced

    def pop_grad(self, t: Tensor) -> Optional[Tensor]:
        """Take the gradient already accumulated for ``t`` (during backward), so a backward
        closure can fuse it into the kernel that produces ``t``'s remaining gradient
        (residual-branch sums land in the dgrad epilogue instead of a separate add)."""
        return self._grads.pop(id(t), None) if self._grads is not None else None

    def backward(self, out: Tensor, grad: Tensor) -> None:
        if self.on_begin is not None:
            self.on_begin()
        grads: Dict[int, Tensor] = {id(out): grad}
        self._grads = grads
        for outputs, inputs, bwd in reversed(self.nodes):
            gouts = [grads.pop(id(o), None) for o in outputs]
            if all(g is None for g in gouts):
                continue
            gins = bwd(*gouts)
            for inp, gi in zip(inputs, gins):
                if gi is None or inp is None or not self.needs_grad(inp):
                    continue
                k = id(inp)
                grads[k] = grads[k] + gi if k in grads else gi
        self.nodes.clear()
        self._produced.clear()
        self._grads = None
        if self.on_end is not None:
            self.on_end()


_WGRAD_STREAMS: Dict[int, "torch.cuda.Stream"] = {}


def _wgrad_stream(device: torch.device) -> Optional["torch.cuda.Stream"]:
    """The per-device side stream weight gradients run on (``DBA_WGRAD_STREAM=1``; default off:
    launch on the caller's stream).  Same priority as the training stream."""
    if os.environ.get("DBA_WGRAD_STREAM", "0") == "0":
        return None
    key = device.index if device.index is not None else torch.cuda.current_device()
    if key not in _WGRAD_STREAMS:
        pri = int(os.environ.get("DBA_TRAIN_STREAM_PRIORITY", "-1"))
        _WGRAD_STREAMS[key] = torch.cuda.Stream(device, priority=pri)
    return _WGRAD_STREAMS[key]


class Ctx:
    """Per-forward context: where the weights live, which mode, the tape.

    ``state``   fp32 ``[Gm, S]`` (params | BN buffers) — master weights and running stats.
    ``wcomp``   weights in compute dtype ``[Gm, >=P]`` (bf16 shadow on GPU; = state on CPU).
    ``grads``   fp32 ``[G, P]`` gradient buffer (train mode only).
    ``folded``  eval mode: {conv name: (w', b')} from :func:`fold_bank`.
    """

    def __init__(self, spec: ModelSpec, state: Tensor, wcomp: Tensor, wsel: Optional[Tensor],
                 train: bool, grads: Optional[Tensor] = None, nvalid: Optional[Tensor] = None,
                 folded: Optional[Dict[str, Tuple[Tensor, Tensor]]] = None,
                 dropout_seed: Optional[Tensor] = None,
                 act_dtype: torch.dtype = torch.float32) -> None:
        self.spec, self.state, self.wcomp, self.wsel = spec, state, wcomp, wsel
        self.train, self.grads, self.nvalid, self.folded = train, grads, nvalid, folded
        self.tape = Tape() if train else None
        # data-gradient weight transposes of the whole step, issued as one batched launch
        # when the backward pass starts (ops.prepare_dgrad_weights)
        self._dgrad_items: List[tuple] = []
        self._wt: Dict[int, Tensor] = {}
        # weight-gradient slab reductions of the whole backward pass, run as one launch when
        # it ends (ops.wgrad_flush)
        self._wdefer: List[tuple] = []
        # weight gradients on a side stream (GPU training): they feed only the end-of-pass slab
        # reduction and the SGD, so they run beside the data-gradient / BN chain that bounds a
        # latency-bound step; joined before the reduction (_end_backward)
        self._side = _wgrad_stream(state.device) if (train and state is not None and state.is_cuda) else None
        self._side_used = False
        self._side_keep: List[Tensor] = []
        if self.tape is not None:
            self.tape.on_begin = self._prepare_dgrad
            self.tape.on_end = self._end_backward
        self.dropout_seed = dropout_seed
        self._drop_ctr = 0
        self.act_dtype = act_dtype
        self._wamax = self._weight_scales() if train else None
        # evaluation forwards of the fp32 family on the HIP backend may keep conv-to-conv
        # activations as fp16 pairs (ops.hip PairAct, DBA_EVAL_PAIRS=1).  OFF by default: same-box
        # A/B of the round-4 tree, 20 timed rounds after 5 warm-up rounds, twice each: 2.924 /
        # 2.976 rounds/s with pairs vs 3.022 / 3.024 without (profiles/r4/bench_pairs*.json) —
        # faster per conv in isolation (profiles/kbench_r3_eval_pairs.log), slower in the round
        self.eval_pairs = (not train and folded is not None and act_dtype == torch.float32
                           and any(t.is_cuda for t, _ in folded.values())
                           and ops.backend_name(next(iter(folded.values()))[0].device) == "hip"
                           and os.environ.get("DBA_EVAL_PAIRS", "0") == "1")

    def _weight_scales(self) -> Optional[Dict[str, Tensor]]:
        """fp32 kernels on the fp16 pair (ops.hip F16_PAIR): every conv / linear weight's
        per-replica max |w| in ONE launch at the start of the step (their operand scales)."""
        wc = self.wcomp
        if (wc is None or not wc.is_cuda or wc.dtype != torch.float32 or ops.backend_name(wc.device) != "hip"
                or ops.hip_module().fp32_mode() != ops.hip_module().F16_PAIR):
            return None
        names = [e.name for e in self.spec.params if e.kind in ("conv_w", "lin_w")]
        slots = ops.hip_module().weight_amax(wc, [(self.spec.by_name[n].offset, self.spec.by_name[n].numel)
                                                  for n in names])
        return dict(zip(names, slots))

    def _want_dgrad(self, w: Tensor, stride: int, pad: int, in_hw: Tuple[int, int], G: int) -> int:
        self._dgrad_items.append((w, self.wsel, stride, pad, in_hw, self.nvalid, G))
        return len(self._dgrad_items) - 1

    def _end_backward(self) -> None:
        if self._side_used:
            torch.cuda.current_stream(self._side.device).wait_stream(self._side)
            self._side_used = False
        if self._wdefer:
            ops.backend_for(self.state).wgrad_flush(self._wdefer)
        self._side_keep.clear()     # the operands the side stream read (alive until the join)

    def _wgrad(self, dy: Tensor, x: Tensor, fn: Callable[[], None]) -> None:
        """Run the weight-gradient launch ``fn`` (reading ``dy`` and ``x``) on the side stream."""
        if self._side is None:
            fn()
            return
        ops.wgrad_prepare(dy, x, self.nvalid)      # operand maxima on the main stream
        self._side.wait_stream(torch.cuda.current_stream(self._side.device))
        with torch.cuda.stream(self._side):
            fn()
        self._side_used = True
        self._side_keep.extend((dy, x))

    def _prepare_dgrad(self) -> None:
        if self._dgrad_items:
            self._wt = ops.prepare_dgrad_weights(self._dgrad_items[0][0], self._dgrad_items)
        self._dgrad_items = []

    # ----------------------------------------------------------------- weights
    def w(self, name: str) -> Tensor:
        v = self.spec.view(self.wcomp, name)
        if self._wamax is not None and name in self._wamax:
            v._dba_amax = self._wamax[name]
        return v

    def m(self, name: str) -> Tensor:
        return self.spec.view(self.state, name)

    def g(self, name: str) -> Tensor:
        assert self.grads is not None
        return self.spec.view(self.grads, name)

    # ------------------------------------------------------------------ layers
    def conv_bn(self, x: Tensor, conv: str, bn: str, stride: int, pad: int, relu: bool,
                residual: Optional[Tensor] = None, to_conv: bool = True) -> Tensor:
        """``to_conv``: the output only feeds convs (A operand or residual), so an evaluation
        forward may keep it as fp16-pair activations (ops.hip PairAct); False where a pooling
        or a linear layer reads it."""
        if not self.train:
            wf, bf = self.folded[conv]
            kw = {"out_pairs": True} if (to_conv and self.eval_pairs) else {}
            return ops.conv2d(x, wf, self.wsel, stride, pad, bias=bf, residual=residual, relu=relu,
                              nvalid=self.nvalid, **kw)
        w = self.w(conv)
        y = ops.conv2d(x, w, self.wsel, stride, pad, nvalid=self.nvalid, bn_stats=True)
        gamma, beta = self.m(bn + ".weight"), self.m(bn + ".bias")
        out, mean, invstd = ops.bn_train(y, gamma, beta, self.m(bn + ".running_mean"),
                                         self.m(bn + ".running_var"), self.nvalid, BN_MOMENTUM,
                                         BN_EPS, relu, residual)
        in_hw = (x.shape[2], x.shape[3])
        kh, kw = w.shape[2], w.shape[3]
        need_dx = self.tape.needs_grad(x)
        k = self._want_dgrad(w, stride, pad, in_hw, x.shape[0]) if need_dx else -1

        def bwd(dout: Tensor):
            r = ops.bn_train_bwd(dout, y, out, mean, invstd, gamma, self.nvalid, relu,
                                 self.g(bn + ".weight"), self.g(bn + ".bias"),
                                 want_dres=residual is not None)
            dy, dres = r if residual is not None else (r, None)
            self._wgrad(dy, x, lambda: ops.conv2d_wgrad(dy, x, stride, pad, kh, kw, self.g(conv), nvalid=self.nvalid,
                                                        defer=self._wdefer))
            dx = None
            if need_dx:
                # the other consumer of x (shortcut branch) already delivered its gradient
                acc = self.tape.pop_grad(x)
                dx = ops.conv2d_dgrad(dy, w, self.wsel, stride, pad, in_hw, nvalid=self.nvalid, accum=acc,
                                      wt=self._wt.get(k))
            return dx, dres

        self.tape.record((out,), (x, residual), bwd)
        return out

    def conv(self, x: Tensor, name: str, stride: int, pad: int, bias: Optional[str], relu: bool) -> Tensor:
        """Conv with its own bias (MnistNet); also used for linear layers as 1x1 convs."""
        if not self.train and self.folded is not None and name in self.folded:
            w, b = self.folded[name]
        else:
            w, b = self.w(name), (self.m(bias) if bias is not None else None)
        y = ops.conv2d(x, w, self.wsel, stride, pad, bias=b, relu=relu, nvalid=self.nvalid)
        if not self.train:
            return y
        in_hw = (x.shape[2], x.shape[3])
        kh, kw = w.shape[2], w.shape[3]
        need_dx = self.tape.needs_grad(x)
        k = self._want_dgrad(w, stride, pad, in_hw, x.shape[0]) if need_dx else -1

        def bwd(dout: Tensor):
            d = ops.relu_mask_bwd(dout, y) if relu else dout
            self._wgrad(d, x, lambda: ops.conv2d_wgrad(d, x, stride, pad, kh, kw, self.g(name),
                                                       self.g(bias) if bias is not None else None, nvalid=self.nvalid,
                                                       defer=self._wdefer))
            return (ops.conv2d_dgrad(d, w, self.wsel, stride, pad, in_hw, nvalid=self.nvalid, wt=self._wt.get(k))
                    if need_dx else None,)

        self.tape.record((y,), (x,), bwd)
        return y

    def linear(self, x: Tensor, name: str, bias: str, relu: bool, final: bool = False) -> Tensor:
        """x [G, N, F] -> [G, N, Out] via the 1x1-conv kernel (weights [Out, 1, 1, F]).
        ``final``: the logits layer writes fp32 (loss/argmax precision)."""
        G, N, Fd = x.shape
        x4 = self.reshape(x, (G, N, 1, 1, Fd))
        y4 = self._lin_conv(x4, name, bias, relu, torch.float32 if final else None)
        return self.reshape(y4, (G, N, y4.shape[-1]))

    def _lin_conv(self, x4: Tensor, name: str, bias: str, relu: bool,
                  out_dtype: Optional[torch.dtype] = None) -> Tensor:
        if not self.train and self.folded is not None and name in self.folded:
            w, b = self.folded[name]
        else:
            wv = self.w(name)
            w = wv.reshape(wv.shape[0], wv.shape[1], 1, 1, wv.shape[2])
            if hasattr(wv, "_dba_amax"):
                w._dba_amax = wv._dba_amax
            b = self.m(bias)
        y = ops.conv2d(x4, w, self.wsel, 1, 0, bias=b, relu=relu, nvalid=self.nvalid, out_dtype=out_dtype)
        if not self.train:
            return y
        need_dx = self.tape.needs_grad(x4)
        gv = self.g(name)
        k = self._want_dgrad(w, 1, 0, (1, 1), x4.shape[0]) if need_dx else -1

        def bwd(dout: Tensor):
            d = ops.relu_mask_bwd(dout, y) if relu else dout
            self._wgrad(d, x4, lambda: ops.conv2d_wgrad(d, x4, 1, 0, 1, 1,
                                                        gv.reshape(gv.shape[0], gv.shape[1], 1, 1, gv.shape[2]),
                                                        self.g(bias), nvalid=self.nvalid, defer=self._wdefer))
            return (ops.conv2d_dgrad(d, w, self.wsel, 1, 0, (1, 1), nvalid=self.nvalid, wt=self._wt.get(k))
                    if need_dx else None,)

        self.tape.record((y,), (x4,), bwd)
        return y

    def reshape(self, x: Tensor, shape: Tuple[int, ...]) -> Tensor:
        y = x.reshape(shape)
        if self.train and y is not x:
            in_shape = x.shape
            self.tape.record((y,), (x,), lambda d: (d.reshape(in_shape),))
        return y

    def maxpool(self, x: Tensor, k: int, s: int, p: int) -> Tensor:
        y, ind = ops.maxpool2d(x, k, s, p)
        if self.train:
            shp = tuple(x.shape)
            self.tape.record((y,), (x,), lambda d: (ops.maxpool2d_bwd(d, ind, shp, k, s, p),))
        return y

    def gap(self, x: Tensor) -> Tensor:
        y = ops.avgpool_global(x)
        if self.train:
            hw = (x.shape[2], x.shape[3])
            self.tape.record((y,), (x,), lambda d: (ops.avgpool_global_bwd(d, hw),))
        return y

    def dropout(self, x: Tensor, p: float) -> Tensor:
        if not self.train:
            return x
        seeds, salt = self.dropout_seed, self._drop_ctr
        self._drop_ctr += 1
        y = ops.dropout(x, p, seeds, salt)
        self.tape.record((y,), (x,), lambda d: (ops.dropout_bwd(d, p, seeds, salt),))
        return y


# ------------------------------------------------------------------- architectures
def _resnet_cifar(ctx: Ctx, x: Tensor) -> Tensor:
    """Any member of the half-width CIFAR family (``mirror.CIFAR_RESNETS``)."""
    bottleneck, blocks = CIFAR_RESNETS[ctx.spec.arch]
    exp = 4 if bottleneck else 1
    out = ctx.conv_bn(x, "conv1.weight", "bn1", 1, 1, relu=True)
    cin = 32
    for li, w in enumerate((32, 64, 128, 256)):
        for bi in range(blocks[li]):
            stride = 2 if (li > 0 and bi == 0) else 1
            pre = f"layer{li + 1}.{bi}."
            if bottleneck:
                a = ctx.conv_bn(out, pre + "conv1.weight", pre + "bn1", 1, 0, relu=True)
                a = ctx.conv_bn(a, pre + "conv2.weight", pre + "bn2", stride, 1, relu=True)
                last, p = "3", 0
            else:
                a = ctx.conv_bn(out, pre + "conv1.weight", pre + "bn1", stride, 1, relu=True)
                last, p = "2", 1
            if stride != 1 or cin != w * exp:
                sc = ctx.conv_bn(out, pre + "shortcut.0.weight", pre + "shortcut.1", stride, 0, relu=False)
            else:
                sc = out
            final = li == 3 and bi == blocks[li] - 1
            out = ctx.conv_bn(a, pre + f"conv{last}.weight", pre + f"bn{last}", 1, p, relu=True, residual=sc,
                              to_conv=not final)
            cin = w * exp
    out = ctx.gap(out)
    G, N = out.shape[:2]
    return ctx.linear(ctx.reshape(out, (G, N, out.shape[-1])), "linear.weight", "linear.bias", relu=False, final=True)


def _resnet_tiny(ctx: Ctx, x: Tensor) -> Tensor:
    out = ctx.conv_bn(x, "conv1.weight", "bn1", 2, 3, relu=True, to_conv=False)   # -> max-pool
    out = ctx.maxpool(out, 3, 2, 1)
    cin = 64
    for li, w in enumerate((64, 128, 256, 512)):
        for bi in range(2):
            stride = 2 if (li > 0 and bi == 0) else 1
            pre = f"layer{li + 1}.{bi}."
            if stride != 1 or cin != w:
                sc = ctx.conv_bn(out, pre + "downsample.0.weight", pre + "downsample.1", stride, 0, relu=False)
            else:
                sc = out
            a = ctx.conv_bn(out, pre + "conv1.weight", pre + "bn1", stride, 1, relu=True)
            out = ctx.conv_bn(a, pre + "conv2.weight", pre + "bn2", 1, 1, relu=True, residual=sc,
                              to_conv=not (li == 3 and bi == 1))
            cin = w
    out = ctx.gap(out)
    G, N = out.shape[:2]
    return ctx.linear(ctx.reshape(out, (G, N, out.shape[-1])), "fc.weight", "fc.bias", relu=False, final=True)


def _mnist(ctx: Ctx, x: Tensor) -> Tensor:
    a = ctx.conv(x, "conv1.weight", 1, 0, "conv1.bias", relu=True)
    a = ctx.maxpool(a, 2, 2, 0)
    b = ctx.conv(a, "conv2.weight", 1, 0, "conv2.bias", relu=True)
    b = ctx.maxpool(b, 2, 2, 0)
    G, N = b.shape[:2]
    f = ctx.reshape(b, (G, N, -1))
    h = ctx.linear(f, "fc1.weight", "fc1.bias", relu=True)
    # log_softmax of the reference is folded into the loss (idempotent, quirk D7)
    return ctx.linear(h, "fc2.weight", "fc2.bias", relu=False, final=True)


def _loan(ctx: Ctx, x: Tensor) -> Tensor:
    h = ctx.linear(x, "layer1.0.weight", "layer1.0.bias", relu=True)
    h = ctx.dropout(h, 0.5)
    h = ctx.linear(h, "layer2.0.weight", "layer2.0.bias", relu=True)
    h = ctx.dropout(h, 0.5)
    return ctx.linear(h, "layer3.0.weight", "layer3.0.bias", relu=False, final=True)


FORWARDS: Dict[str, Callable[[Ctx, Tensor], Tensor]] = {
    "resnet18_tiny": _resnet_tiny, "mnist": _mnist, "loan": _loan,
    **{arch: _resnet_cifar for arch in CIFAR_RESNETS},
}


def forward(ctx: Ctx, x: Tensor) -> Tensor:
    return FORWARDS[ctx.spec.arch](ctx, x)


# ------------------------------------------------------------------------ BN folding
def _conv_bn_pairs(spec: ModelSpec) -> List[Tuple[str, str]]:
    pairs = []
    for e in spec.params:
        if e.kind != "conv_w":
            continue
        n = e.name
        if n.endswith("shortcut.0.weight"):
            pairs.append((n, n.replace("shortcut.0.weight", "shortcut.1")))
        elif n.endswith("downsample.0.weight"):
            pairs.append((n, n.replace("downsample.0.weight", "downsample.1")))
        else:
            bn = n.replace("conv", "bn").replace(".weight", "")
            if bn + ".weight" in spec.by_name:
                pairs.append((n, bn))
    return pairs


def fold_bank(spec: ModelSpec, state: Tensor, dtype: torch.dtype) -> Dict[str, Tuple[Tensor, Tensor]]:
    """Eval weights for a ``[Gm, S]`` bank of model states: BN folded into each conv; plain
    convs/linears converted to the compute dtype with their fp32 bias."""
    out: Dict[str, Tuple[Tensor, Tensor]] = {}
    for conv, bn in _conv_bn_pairs(spec):
        out[conv] = ops.bn_fold(spec.view(state, conv), None, spec.view(state, bn + ".weight"),
                                spec.view(state, bn + ".bias"), spec.view(state, bn + ".running_mean"),
                                spec.view(state, bn + ".running_var"), BN_EPS, dtype)
    for e in spec.params:
        if e.name in out or e.kind not in ("conv_w", "lin_w"):
            continue
        bias = e.name.replace(".weight", ".bias")
        w = spec.view(state, e.name)
        if w.dim() == 3:  # linear [Gm, Out, In] -> [Gm, Out, 1, 1, In]
            w = w.reshape(w.shape[0], w.shape[1], 1, 1, w.shape[2])
        b = spec.view(state, bias).contiguous() if bias in spec.by_name else None
        out[e.name] = (w.to(dtype).contiguous(), b)
    return out
