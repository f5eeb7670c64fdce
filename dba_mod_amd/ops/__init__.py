"""Framework ops: one entry point per kernel, dispatched by the tensors' device.

* GPU tensors run the hand-written CDNA4 HIP kernels of ``csrc/kernels`` (gfx950), loaded
  from the in-tree ``libdba_kernels.so`` through :mod:`dba_mod_amd.ops.hip`.  If that
  library is missing on a GPU box the call fails loudly — there is no silent fallback.
* CPU tensors run :mod:`dba_mod_amd.ops.reference` (plain PyTorch fp32), which is also the
  numerics oracle of the GPU tests.

``DBA_OPS=reference`` forces the reference implementation on GPU tensors too (explicit
A/B baselining only; bench.py reports which backend ran).
"""
from __future__ import annotations

import contextlib
import os
from typing import Any

import torch

from . import reference as _ref

_FORCE_REF = os.environ.get("DBA_OPS", "").lower() == "reference"
_hip_mod = None


def hip_module():
    global _hip_mod
    if _hip_mod is None:
        from . import hip as _h  # raises with a clear message if the .so is missing
        _hip_mod = _h
    return _hip_mod


def backend_for(t: torch.Tensor):
    if t.is_cuda and not _FORCE_REF:
        return hip_module()
    return _ref


def backend_name(device: torch.device) -> str:
    return "hip" if (device.type == "cuda" and not _FORCE_REF) else "reference"


def _dispatch(name: str):
    def fn(*args: Any, **kw: Any):
        first = next(a for a in list(args) + list(kw.values()) if isinstance(a, torch.Tensor))
        return getattr(backend_for(first), name)(*args, **kw)
    fn.__name__ = name
    fn.__doc__ = getattr(_ref, name).__doc__
    return fn


_OPS = ["gather_images", "gather_rows", "conv2d", "conv2d_dgrad", "conv2d_wgrad", "relu_mask_bwd", "bn_fold", "maxpool2d", "maxpool2d_bwd", "avgpool_global",
        "avgpool_global_bwd", "dropout", "dropout_bwd", "softmax_xent", "sgd_step", "dist_loss_grad",
        "scale_from_base", "add_noise_scaled", "delta_sum", "sq_dists", "weighted_sum", "weighted_sum_fixed", "gram", "prepare_dgrad_weights", "wgrad_flush",
        "wgrad_prepare", "conv_bn_stats", "bn_apply", "bn_finish", "basic_block_ok", "basic_block_eval",
        "stem_block_ok", "stem_block_eval", "down_block_ok", "down_block_eval"]

for _n in _OPS:
    globals()[_n] = _dispatch(_n)


def amax_arena(G: int, device: torch.device, counters: int = 0):
    """Context: one zeroed allocation for the fp16-pair operand-max slots of the enclosed
    launches (``ops.hip.amax_arena``), plus ``counters`` arrival counters for their in-launch
    split-K combines; a no-op off the HIP backend."""
    if backend_name(device) == "hip":
        return hip_module().amax_arena(G, device, counters=counters)
    return contextlib.nullcontext()


__all__ = list(_OPS) + ["backend_for", "backend_name", "hip_module", "amax_arena"]

from . import library  # noqa: E402,F401  (torch.library registration of the dba:: ops)
