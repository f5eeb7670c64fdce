"""Flat, device-resident parameter layout of a model replica.

A replica's whole float state is ONE contiguous fp32 vector ``state[S]``:

    [ parameters (P floats, named_parameters() order) | BN running mean/var (B floats) ]

so client deltas, model-replacement scaling, FedAvg/RFA/FoolsGold and the RCCL collectives
all act on a single flat bucket instead of 122 per-layer tensors.
``G`` replicas are a ``[G, S]`` matrix.  The integer ``num_batches_tracked`` counters are
kept out of the float bucket (quirk D1) as one int64 per replica.

Conv weights are stored in the kernels' layout ``[Cout, KH, KW, Cin]`` (NHWC implicit GEMM,
K-contiguous); ``to_state_dict`` / ``load_state_dict`` convert to and from the reference's
``[Cout, Cin, KH, KW]`` checkpoint layout.  Element permutations are irrelevant to every
aggregation (sums, norms, dot products), so nothing else ever needs the reference layout.
The FoolsGold feature (reference ``client_grads[-2]``, the final FC weight) is the
second-to-last parameter, exactly as in the reference.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from .mirror import CIFAR_RESNETS, build_mirror


@dataclass
class Entry:
    name: str
    sd_shape: Tuple[int, ...]
    k_shape: Tuple[int, ...]
    offset: int
    numel: int
    kind: str                      # conv_w | lin_w | bias | bn_w | bn_b | bn_mean | bn_var
    to_k: Optional[Callable[[torch.Tensor], torch.Tensor]] = None
    to_sd: Optional[Callable[[torch.Tensor], torch.Tensor]] = None


ALIGN = 64   # every entry starts on a 64-element boundary (256 B fp32 / 128 B bf16), so
             # the kernels' 16-byte vector loads of weight rows are always aligned


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class ModelSpec:
    arch: str
    params: List[Entry]
    buffers: List[Entry]
    counters: List[str]
    sd_order: List[str]
    input_hwc: Tuple[int, ...]
    num_classes: int
    P: int = 0
    B: int = 0
    n_params: int = 0              # true parameter count (P includes alignment padding)
    by_name: Dict[str, Entry] = field(default_factory=dict)

    @property
    def S(self) -> int:
        return self.P + self.B

    # ------------------------------------------------------------------ views
    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        """Strided view ``[G, *k_shape]`` of entry ``name`` in a ``[G, >=S]`` flat matrix."""
        e = self.by_name[name]
        return flat[:, e.offset:e.offset + e.numel].view(flat.shape[0], *e.k_shape)

    def fg_feature_slice(self) -> Tuple[int, int]:
        e = self.params[-2]
        return e.offset, e.offset + e.numel

    # --------------------------------------------------------------- conversion
    def flat_from_state_dict(self, sd: Dict[str, torch.Tensor]) -> torch.Tensor:
        out = torch.zeros(self.S, dtype=torch.float32)
        for e in self.params + self.buffers:
            t = sd[e.name].detach().to(torch.float32).cpu()
            if e.to_k is not None:
                t = e.to_k(t)
            out[e.offset:e.offset + e.numel] = t.reshape(-1)
        return out

    def state_dict_from_flat(self, flat: torch.Tensor, counter: int = 0) -> "OrderedDict[str, torch.Tensor]":
        flat = flat.detach().to(torch.float32).cpu()
        sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        for name in self.sd_order:
            if name in self.by_name:
                e = self.by_name[name]
                t = flat[e.offset:e.offset + e.numel].reshape(e.k_shape)
                if e.to_sd is not None:
                    t = e.to_sd(t)
                sd[name] = t.contiguous().clone()
            else:
                sd[name] = torch.tensor(int(counter), dtype=torch.int64)
        return sd

    def init_flat(self, seed: int) -> torch.Tensor:
        torch.manual_seed(seed)
        m = build_mirror(self.arch)
        return self.flat_from_state_dict(m.state_dict())


def _conv_to_k(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 2, 3, 1).contiguous()


def _conv_to_sd(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 3, 1, 2)


def _make_spec(arch: str, input_hwc: Tuple[int, ...], num_classes: int,
               special: Optional[Dict[str, Tuple[Tuple[int, ...], Callable, Callable]]] = None) -> ModelSpec:
    m = build_mirror(arch)
    special = special or {}
    params: List[Entry] = []
    off = 0
    for name, p in m.named_parameters():
        shp = tuple(p.shape)
        to_k = to_sd = None
        if name in special:
            kshape, to_k, to_sd = special[name]
            kind = "lin_w"
        elif p.dim() == 4:
            kshape, to_k, to_sd, kind = (shp[0], shp[2], shp[3], shp[1]), _conv_to_k, _conv_to_sd, "conv_w"
        elif p.dim() == 2:
            kshape, kind = shp, "lin_w"
        else:
            kshape = shp
            kind = "bias"
            if ".bn" in name or name.startswith("bn") or ".shortcut.1." in name or ".downsample.1." in name:
                kind = "bn_w" if name.endswith("weight") else "bn_b"
        params.append(Entry(name, shp, kshape, off, p.numel(), kind, to_k, to_sd))
        off = _align(off + p.numel())
    P = off
    buffers: List[Entry] = []
    counters: List[str] = []
    for name, b in m.named_buffers():
        if name.endswith("num_batches_tracked"):
            counters.append(name)
            continue
        kind = "bn_mean" if name.endswith("running_mean") else "bn_var"
        buffers.append(Entry(name, tuple(b.shape), tuple(b.shape), off, b.numel(), kind))
        off = _align(off + b.numel())
    spec = ModelSpec(arch, params, buffers, counters, list(m.state_dict().keys()), input_hwc,
                     num_classes, P=P, B=off - P, n_params=sum(e.numel for e in params))
    spec.by_name = {e.name: e for e in params + buffers}
    return spec


def _mnist_fc1_special():
    # reference flattens NCHW [50,4,4] (c-major); our activations are NHWC (c-minor)
    def to_k(t):
        return t.view(500, 50, 4, 4).permute(0, 2, 3, 1).reshape(500, 800).contiguous()

    def to_sd(t):
        return t.view(500, 4, 4, 50).permute(0, 3, 1, 2).reshape(500, 800)
    return {"fc1.weight": ((500, 800), to_k, to_sd)}


_SPECS: Dict[str, ModelSpec] = {}


def get_spec(arch: str) -> ModelSpec:
    if arch not in _SPECS:
        if arch == "mnist":
            _SPECS[arch] = _make_spec(arch, (28, 28, 1), 10, _mnist_fc1_special())
        elif arch in CIFAR_RESNETS:
            _SPECS[arch] = _make_spec(arch, (32, 32, 3), 10)
        elif arch == "resnet18_tiny":
            _SPECS[arch] = _make_spec(arch, (64, 64, 3), 200)
        elif arch == "loan":
            _SPECS[arch] = _make_spec(arch, (91,), 9)
        else:
            raise ValueError(arch)
    return _SPECS[arch]


def arch_for_type(t: str, model_arch: Optional[str] = None) -> str:
    """Dataset type -> architecture; ``model_arch`` picks another member of the CIFAR ResNet
    family (the reference always builds ResNet18 for CIFAR, ``image_helper.py:33-38``)."""
    arch = {"mnist": "mnist", "cifar": "resnet18_cifar", "tiny-imagenet-200": "resnet18_tiny",
            "loan": "loan"}[t]
    if model_arch:
        if t != "cifar" or model_arch not in CIFAR_RESNETS:
            raise ValueError(f"model_arch {model_arch!r} is not available for type {t!r} "
                             f"(cifar: {sorted(CIFAR_RESNETS)})")
        arch = model_arch
    return arch
