"""Value types of the fused training BatchNorm (``csrc/kernels/bnfuse.hpp``), shared by both
backends.

A training BN's output is not stored when only convs consume it: the producing conv reduces
its statistics, and consumers apply ``relu?(y * scale + shift)`` while staging (:class:`LazyBN`).
In the backward pass the gradient of a BN output is *finished* — masked by the ReLU and reduced
into the BN's backward coefficients — by the kernel that produces it (:class:`Finish` says how),
and the BN input gradient ``dy = A * d + B * y + K`` is applied by the weight gradient that
consumes it (:class:`LazyGrad`).

Reference semantics: ``BatchNorm2d`` in train mode + ReLU / residual add,
``/root/reference/models/resnet_cifar.py:31-36`` (``image_train.py:84-102``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, List, Optional

import torch

Tensor = torch.Tensor

# rows of BnStat.coef (bnfuse.hpp kC*)
MEAN, INV, SCALE, SHIFT, YMAX, YMIN, A, B, K = range(9)
ROWS = 9


@dataclass
class BnParams:
    """Views of one BN layer's parameters / buffers / gradients in the flat replica rows."""
    gamma: Tensor
    beta: Tensor
    rmean: Tensor
    rvar: Tensor
    dgamma: Tensor
    dbeta: Tensor
    momentum: float
    eps: float


class BnStat:
    """A training BN's per-step state: ``coef [G, ROWS, C]`` (forward: mean, 1/std, scale,
    shift, max / min of y; backward: A, B, K) and, on the HIP backend, the operand-max slots of
    its lazy output (``bound``) and of its input gradient (``dbound``)."""

    def __init__(self, coef: Tensor, params: BnParams, bound: Any = None) -> None:
        self.coef, self.params, self.bound = coef, params, bound
        self.dbound: Any = None

    @property
    def C(self) -> int:
        return self.coef.shape[-1]


class LazyBN:
    """``relu?(y * scale + shift)`` of a training BN — consumed by convs (A operand, weight
    gradient x operand) and residual adds without being stored."""

    def __init__(self, y: Tensor, stat: BnStat, relu: bool) -> None:
        self.y, self.stat, self.relu = y, stat, relu

    @property
    def shape(self):
        return self.y.shape

    @property
    def dtype(self):
        return self.y.dtype

    @property
    def device(self):
        return self.y.device

    @property
    def is_cuda(self) -> bool:
        return self.y.is_cuda


@dataclass
class Finish:
    """How the gradient of a BN output is finished: d = g where the output is > 0 (``mask_out``
    the stored output, or ``lazy`` = the ReLU of BN a's lazy output), then the backward sums of
    BN a (input ``ya``) and, for a residual sum of two BNs, BN b (input ``yb``)."""
    ya: Tensor
    sa: BnStat
    mask_out: Optional[Tensor] = None
    lazy: bool = False
    yb: Optional[Tensor] = None
    sb: Optional[BnStat] = None

    def stats(self) -> List[BnStat]:
        return [self.sa] + ([self.sb] if self.sb is not None else [])


class Fin:
    """A finished gradient: ``d`` (masked) with the backward coefficients of ``stats`` ready."""

    def __init__(self, d: Tensor, stats: List[BnStat]) -> None:
        self.d, self.stats = d, stats

    def for_stat(self, st: BnStat) -> "Fin":
        assert any(s is st for s in self.stats), "gradient finished for another BN"
        return Fin(self.d, [st])


class LazyGrad:
    """``dy = A * d + B * y + K`` of a training BN's input (d: the finished gradient of its
    output, y: its input, A/B/K: ``stat.coef``)."""

    def __init__(self, d: Tensor, y: Tensor, stat: BnStat) -> None:
        self.d, self.y, self.stat = d, y, stat

    @property
    def shape(self):
        return self.d.shape
