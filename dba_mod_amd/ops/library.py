"""``torch.library`` registration of the framework's device ops (namespace ``dba``).

SURVEY §7.1 asks for one custom op per kernel with a HIP implementation (gfx950) and a CPU
implementation behind PyTorch's own device dispatch.  Importing this module registers the
schema of every op below; the ``cuda`` kernel of each calls the hand-written HIP launcher
(:mod:`dba_mod_amd.ops.hip`, ``libdba_kernels.so``) and the ``cpu`` kernel the plain-PyTorch
reference (:mod:`dba_mod_amd.ops.reference`), so ``torch.ops.dba.conv2d(x, w, ...)`` runs
the MFMA kernel for a GPU tensor and the reference for a CPU tensor — one call site, no
duplicated model code.  Mutating ops declare what they write (``mutates_args``).

This registration is the framework's EXTERNAL tensor API: the model programs
(``models/program.py`` via :mod:`dba_mod_amd.ops`) call the same two implementations directly,
because their training path passes values a schema cannot carry — lazy BN outputs and finished
gradients (:mod:`dba_mod_amd.ops.bnstate`), operand-max slots and fp16-pair activations attached
to tensors — so a ``torch.ops.dba`` call there would have to materialise what the fused kernels
never store.  ``tests/test_library.py`` (CPU) and
``tests/test_gpu_kernels.py::test_torch_library_ops_run_hip`` check that both entry points give
the same results.

Reference call sites of the ops (stock PyTorch there): conv ``models/resnet_cifar.py:19-33``,
BN ``:32-35``, CE ``image_train.py:85``, SGD ``image_train.py:33-35,102``, trigger
``image_helper.py:298-350``, FedAvg ``helper.py:240-257``, Weiszfeld ``helper.py:376-418``,
FoolsGold cosine ``helper.py:574-580``.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from . import reference as _ref

Tensor = torch.Tensor
NS = "dba"


def _hip():
    from . import hip   # raises if libdba_kernels.so is missing (no silent fallback)
    return hip


_IMPLS = {}


def _impl(name: str, t: Tensor):
    """The (cpu, cuda) implementation pair of ``name`` for ``t``'s device (the default kernel
    of an op; PyTorch's device dispatch normally picks the registered kernel first)."""
    cpu, gpu = _IMPLS[name]
    return gpu if t.is_cuda else cpu


def _both(name: str, fn_cpu, fn_gpu, schema_fn, mutates=()):
    """Register ``dba::name`` with the schema of ``schema_fn`` and one kernel per device."""
    _IMPLS[name] = (fn_cpu, fn_gpu)
    op = torch.library.custom_op(f"{NS}::{name}", mutates_args=mutates)(schema_fn)
    op.register_kernel("cpu")(fn_cpu)
    op.register_kernel("cuda")(fn_gpu)
    return op


# ----------------------------------------------------------------------------- conv
def _conv2d(x: Tensor, w: Tensor, wsel: Optional[Tensor], stride: int, pad: int, bias: Optional[Tensor],
            residual: Optional[Tensor], relu: bool, nvalid: Optional[Tensor]) -> Tensor:
    """y = act(conv(x, w[wsel]) + bias + residual) (K1/K3/K4/K8), NHWC [G, N, H, W, C]."""
    return _impl("conv2d", x)(x, w, wsel, stride, pad, bias, residual, relu, nvalid)


conv2d = _both(
    "conv2d",
    lambda x, w, wsel, stride, pad, bias, residual, relu, nvalid: _ref.conv2d(
        x, w, wsel, stride, pad, bias=bias, residual=residual, relu=relu, nvalid=nvalid),
    lambda x, w, wsel, stride, pad, bias, residual, relu, nvalid: _hip().conv2d(
        x, w, wsel, stride, pad, bias=bias, residual=residual, relu=relu, nvalid=nvalid),
    _conv2d)


def _conv2d_dgrad(dy: Tensor, w: Tensor, wsel: Optional[Tensor], stride: int, pad: int, in_h: int, in_w: int,
                  nvalid: Optional[Tensor], accum: Optional[Tensor]) -> Tensor:
    """dX of a conv (K2), ``accum`` added in."""
    return _impl("conv2d_dgrad", dy)(dy, w, wsel, stride, pad, in_h, in_w, nvalid, accum)


conv2d_dgrad = _both(
    "conv2d_dgrad",
    lambda dy, w, wsel, stride, pad, in_h, in_w, nvalid, accum: _ref.conv2d_dgrad(
        dy, w, wsel, stride, pad, (in_h, in_w), nvalid=nvalid, accum=accum),
    lambda dy, w, wsel, stride, pad, in_h, in_w, nvalid, accum: _hip().conv2d_dgrad(
        dy, w, wsel, stride, pad, (in_h, in_w), nvalid=nvalid, accum=accum),
    _conv2d_dgrad)


def _conv2d_wgrad(dy: Tensor, x: Tensor, stride: int, pad: int, kh: int, kw: int, dw: Tensor,
                  dbias: Optional[Tensor], nvalid: Optional[Tensor]) -> None:
    """dw (+= per replica) and dbias (+=) of a conv (K2)."""
    return _impl("conv2d_wgrad", dy)(dy, x, stride, pad, kh, kw, dw, dbias, nvalid)


conv2d_wgrad = _both(
    "conv2d_wgrad",
    lambda dy, x, stride, pad, kh, kw, dw, dbias, nvalid: _ref.conv2d_wgrad(
        dy, x, stride, pad, kh, kw, dw, dbias, nvalid=nvalid),
    lambda dy, x, stride, pad, kh, kw, dw, dbias, nvalid: _hip().conv2d_wgrad(
        dy, x, stride, pad, kh, kw, dw, dbias, nvalid=nvalid),
    _conv2d_wgrad, mutates=("dw", "dbias"))


# ------------------------------------------------------------------------ batch norm
def _bn_params(gamma, beta, rmean, rvar, momentum, eps):
    from .bnstate import BnParams
    z = torch.zeros_like(gamma)
    return BnParams(gamma, beta, rmean, rvar, z, z.clone(), momentum, eps)


def _conv_bn_stats(x: Tensor, w: Tensor, wsel: Optional[Tensor], stride: int, pad: int, nvalid: Optional[Tensor],
                   gamma: Tensor, beta: Tensor, rmean: Tensor, rvar: Tensor, momentum: float,
                   eps: float) -> Tuple[Tensor, Tensor]:
    """Training conv + BatchNorm statistics in one pass (K1/K5, csrc/kernels/bnfuse.hpp):
    y = conv(x, w[wsel]) and the BN's coefficient rows [G, 9, C] (mean, 1/std, scale, shift,
    max y, min y, ...); running stats updated in place.  The BN output is
    relu?(y * scale + shift) (``bn_apply``)."""
    return _impl("conv_bn_stats", x)(x, w, wsel, stride, pad, nvalid, gamma, beta, rmean, rvar, momentum, eps)


def _cbs(mod, x, w, wsel, stride, pad, nvalid, gamma, beta, rmean, rvar, momentum, eps):
    y, st = mod.conv_bn_stats(x, w, wsel, stride, pad, nvalid, _bn_params(gamma, beta, rmean, rvar, momentum, eps),
                              False)
    return y, st.coef.float().clone()


conv_bn_stats = _both("conv_bn_stats", lambda *a: _cbs(_ref, *a), lambda *a: _cbs(_hip(), *a), _conv_bn_stats,
                      mutates=("rmean", "rvar"))


def _bn_apply(y: Tensor, coef: Tensor, residual: Optional[Tensor], relu: bool, nvalid: Optional[Tensor]) -> Tensor:
    """relu?(y * scale + shift + residual) of a training BN from its coefficient rows (K6)."""
    return _impl("bn_apply", y)(y, coef, residual, relu, nvalid)


def _bapp(mod, y, coef, residual, relu, nvalid):
    from .bnstate import BnStat, LazyBN
    return mod.bn_apply(LazyBN(y, BnStat(coef.to(y.dtype), None), False), residual, relu, nvalid)


bn_apply = _both("bn_apply", lambda *a: _bapp(_ref, *a), lambda *a: _bapp(_hip(), *a), _bn_apply)


# ------------------------------------------------------------------ data / loss / optim
def _gather_images(src: Tensor, labels: Tensor, idx: Tensor, trig_masks: Tensor, trig_id: Tensor,
                   poison_n: Tensor, target: int, flip_seeds: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    """Fused uint8 gather + /255 + flip + pixel trigger + relabel (K17/K19), fp32 out."""
    return _impl("gather_images", src)(src, labels, idx, trig_masks, trig_id, poison_n, target, flip_seeds)


gather_images = _both(
    "gather_images",
    lambda src, labels, idx, masks, tid, pn, target, fs: _ref.gather_images(
        src, labels, idx, masks, tid, pn, target, fs, torch.float32),
    lambda src, labels, idx, masks, tid, pn, target, fs: _hip().gather_images(
        src, labels, idx, masks, tid, pn, target, fs, torch.float32),
    _gather_images)


def _softmax_xent(logits: Tensor, labels: Tensor, mean: bool) -> Tuple[Tensor, Tensor, Tensor]:
    """Per-group CE (mean or sum), correct count and dlogits (K9)."""
    return _impl("softmax_xent", logits)(logits, labels, mean)


softmax_xent = _both(
    "softmax_xent",
    lambda logits, labels, mean: tuple(_ref.softmax_xent(logits, labels, mean, True)),
    lambda logits, labels, mean: tuple(_hip().softmax_xent(logits, labels, mean, True)),
    _softmax_xent)


def _sgd_step(params: Tensor, grads: Tensor, mom: Tensor, lr: Tensor, first: Tensor, active: Tensor,
              momentum: float, wd: float) -> None:
    """Per-replica fused SGD with momentum + weight decay on flat buffers (K10)."""
    return _impl("sgd_step", params)(params, grads, mom, lr, first, active, momentum, wd)


sgd_step = _both(
    "sgd_step",
    lambda p, g, m, lr, first, active, mo, wd: _ref.sgd_step(p, g, m, lr, first, active, mo, wd),
    lambda p, g, m, lr, first, active, mo, wd: _hip().sgd_step(p, g, m, lr, first, active, mo, wd),
    _sgd_step, mutates=("params", "mom"))


# ------------------------------------------------------------------------- aggregation
def _delta_sum(rows: Tensor, base: Tensor) -> Tensor:
    """fp64 sum over clients of (row - base) (K11/K12, FedAvg)."""
    return _impl("delta_sum", rows)(rows, base)


delta_sum = _both("delta_sum", lambda r, b: _ref.delta_sum(r, b), lambda r, b: _hip().delta_sum(r, b), _delta_sum)


def _sq_dists(points: Tensor, m: Tensor) -> Tensor:
    """Squared L2 distance of every row to m, one pass (K13, Weiszfeld / norms)."""
    return _impl("sq_dists", points)(points, m)


sq_dists = _both("sq_dists", lambda p, m: _ref.sq_dists(p, m), lambda p, m: _hip().sq_dists(p, m), _sq_dists)


def _weighted_sum(points: Tensor, wts: Tensor) -> Tensor:
    """sum_i wts[i] * points[i] (K14/K16, Weiszfeld / FoolsGold)."""
    return _impl("weighted_sum", points)(points, wts)


weighted_sum = _both("weighted_sum", lambda p, w: _ref.weighted_sum(p, w), lambda p, w: _hip().weighted_sum(p, w),
                     _weighted_sum)


def _gram(feats: Tensor) -> Tensor:
    """F F^T of the FoolsGold features (K15)."""
    return _impl("gram", feats)(feats)


gram = _both("gram", lambda f: _ref.gram(f), lambda f: _hip().gram(f), _gram)


OPS: List[str] = ["conv2d", "conv2d_dgrad", "conv2d_wgrad", "conv_bn_stats", "bn_apply", "gather_images",
                  "softmax_xent", "sgd_step", "delta_sum", "sq_dists", "weighted_sum", "gram"]
