"""GPU implementation of every framework op: thin ctypes bindings to ``libdba_kernels.so``.

Each wrapper checks layouts, allocates outputs with the torch caching allocator and launches
the hand-written gfx950 kernel on torch's *current* stream (so every launch is captured by
``torch.cuda.graph``).  Signatures mirror :mod:`dba_mod_amd.ops.reference` exactly.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional, Sequence, Tuple

import torch

from . import bnstate as bs
from . import build

Tensor = torch.Tensor
_F32 = torch.float32

if not os.path.exists(build.kernels_path()):
    raise ImportError(f"HIP kernel library missing: {build.kernels_path()} — run "
                      f"`python -m dba_mod_amd.ops.build` (or __graft_entry__.build())")
_L = ctypes.CDLL(build.kernels_path())

_P = ctypes.c_void_p
_I = ctypes.c_int
_LL = ctypes.c_longlong
_F = ctypes.c_float
_U = ctypes.c_uint
_D = ctypes.c_double

_SIGS = {
    "dba_gather_images": [_P, _P, _P, _P, _P, _P, _I, _P, _P, _I, _P, _I, _I, _I, _I, _I, _P],
    "dba_gather_rows": [_P, _P, _P, _P, _P, _I, _P, _P, _I, _P, _I, _P, _I, _I, _I, _P],
    "dba_xcolsum": [_P, _LL, _I, _P, _I, _I, _I, _P, _LL, _P, _P],
    "dba_xcolsum_part_doubles": [_I, _I, _I, _I],
    "dba_amax_segments": [_P, _LL, _P, _I, _I, _P, _I, _P],
    "dba_bn_fold": [_P, _LL, _P, _P, _P, _P, _P, _LL, _F, _P, _P, _I, _I, _I, _I, _P, _I, _P],
    "dba_relu_mask_bwd": [_P, _P, _P, _LL, _I, _P],
    "dba_maxpool": [_P, _P, _P, _LL, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "dba_maxpool_bwd": [_P, _P, _P, _LL, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "dba_avgpool": [_P, _P, _LL, _I, _I, _I, _P],
    "dba_avgpool_bwd": [_P, _P, _LL, _I, _I, _I, _P],
    "dba_dropout": [_P, _P, _I, _P, _U, _F, _LL, _I, _P],
    "dba_softmax_xent": [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _LL, _P, _I, _P, _I, _P, _P, _P],
    "dba_softmax_xent_part_doubles": [_I, _I],
    "dba_xent_r5_set": [_I],
    "dba_head_train": [_P, _LL, _I, _I, _I, _I, _P, _LL, _P, _LL, _I, _P, _P, _P, _P, _P, _P, _LL, _P, _LL, _P, _P,
                       _P, _P, _LL, _P, _I, _I, _P],
    "dba_head_part_doubles": [_I, _I],
    "dba_sgd_step": [_P, _LL, _P, _P, _P, _P, _P, _F, _F, _P, _I, _I, _P],
    "dba_scale_from_base": [_P, _P, _F, _P, _LL, _P],
    "dba_add_noise_scaled": [_P, _P, _LL, _F, _F, _U, _I, _I, _P],
    "dba_delta_sum": [_P, _LL, _I, _P, _LL, _P, _P],
    "dba_sqdist_blocks": [_LL],
    "dba_gram_chunks": [_I],
    "dba_sq_dists": [_P, _LL, _P, _I, _LL, _P, _P, _P],
    "dba_weighted_sum": [_P, _LL, _P, _I, _P, _LL, _I, _P],
    "dba_weighted_sum_fixed": [_P, _LL, _P, _I, _P, _LL, _D, _P],
    "dba_gram": [_P, _LL, _I, _I, _P, _P, _P],
    "dba_dist_loss_grad": [_P, _LL, _P, _LL, _P, _LL, _I, _P, _P, _F, _P, _P, _P],
    # reference-precision (fp32) family: csrc/kernels/xconv*.hip, xwgrad.hip, xbn.hip, xaux.hip
    "dba_ximg_set": [_I],
    "dba_xwgrad_halo_set": [_I],
    "dba_xconv_ws_floats": [_I] * 8,
    "dba_xconv_fwd": [_P, _LL, _P, _LL, _P, _P, _LL, _P, _P, _LL, _P] + [_I] * 13 + [_P, _I] * 3 + [_P, _LL] * 2
    + [_P, _LL, _P, _P, _I, _P],
    "dba_xconv_sk_ints": [_I] * 8,
    "dba_xconv_dgrad": [_P, _LL, _P, _LL, _P, _P, _P, _LL, _P] + [_I] * 12 + [_P, _I] * 2 + [_P, _LL] * 3 + [_P, _P],
    "dba_xsplit_w": [_P, _LL, _LL, _I, _P, _I, _P, _P],
    "dba_amax": [_P, _LL, _LL, _P, _LL, _I, _P, _I, _P],
    "dba_xtranspose": [_P, _I, _I, _LL, _P, _P],
    "dba_xwgrad_ws_floats": [_I] * 8 + [_P],
    "dba_xwgrad_stem_ws_floats": [_I] * 6,
    "dba_xsplit_policy": [_I] * 5,
    "dba_xsplit_w_batch": [_P, _I, _I, _P],
    "dba_bn_fold_batch": [_P, _I, _I, _F, _P],
    "dba_xwgrad": [_P, _LL, _P, _LL, _P, _LL, _P] + [_I] * 12 + [_P, _I] * 2 + [_P, _LL, _I] + [_P, _I, _P],
    # fused training BN (csrc/kernels/bnfuse.hpp)
    "dba_bnx_rows": [_P, _P, _P, _LL, _P, _I, _I, _I, _P, _F, _P],
    "dba_bnx_apply": [_P, _P, _P, _P, _P, _I, _I, _P, _LL, _P, _I, _I, _I, _I, _P, _I, _P],
    "dba_bnfuse_size": [],
    "dba_xwgrad_stem": [_P, _LL, _P, _P, _P, _LL, _P, _P, _I, _I, _I, _I, _P],
    "dba_bnx_dy": [_P, _P, _P, _P, _LL, _P, _I, _I, _I, _I, _P, _I, _P],
    "dba_xwgrad_reduce_batch": [_P, _I, _I, _LL, _P],
    # fused evaluation BasicBlock, with or without the image stem (csrc/kernels/xblock.hip)
    "dba_xblock_fwd": [_P, _LL, _P, _LL, _P, _P, _P, _LL, _P, _P, _LL, _P] + [_I] * 6
    + [_P, _I, _P, _P, _I, _P, _I, _P],
    "dba_xblock_stem_fwd": [_P, _LL, _P, _LL, _P, _P, _LL, _P, _LL, _P, _P, _LL, _P, _P, _LL, _P] + [_I] * 6
    + [_P, _P, _P, _I, _P, _I, _P],
    "dba_mlp_train": [_P, _I, _I, _I, _I, _I, _P, _LL, _P, _P, _I, _P, _I, _I, _I, _I, _P, _P, _P, _P, _I, _I,
                      _P, _LL, _I, _P, _F, _F, _P, _P],
    "dba_xdown_fwd": [_P, _LL, _P, _LL, _P, _LL, _P, _P, _LL, _P, _LL, _P, _LL, _P, _LL, _P, _LL, _P] + [_I] * 8
    + [_P, _I] * 5 + [_P],
    "dba_xstem_fwd": [_P, _LL, _P, _LL, _P, _P, _LL, _P, _P, _LL, _P] + [_I] * 13 + [_P, _I, _P, _P],
}
for _name, _args in _SIGS.items():
    _fn = getattr(_L, _name)
    _fn.argtypes = _args
    _fn.restype = ctypes.c_int
_L.dba_xconv_ws_floats.restype = ctypes.c_longlong
_L.dba_xconv_sk_ints.restype = ctypes.c_longlong
_L.dba_xwgrad_ws_floats.restype = ctypes.c_longlong
_L.dba_xwgrad_stem_ws_floats.restype = ctypes.c_longlong
_L.dba_xcolsum_part_doubles.restype = ctypes.c_longlong
_L.dba_softmax_xent_part_doubles.restype = ctypes.c_longlong
_L.dba_head_part_doubles.restype = ctypes.c_longlong


class _BnFuse(ctypes.Structure):
    """Mirror of csrc/kernels/bnfuse.hpp ``BnFuse`` (passed by host pointer, copied by value
    into the kernel arguments at launch: graph-capture safe)."""
    _fields_ = [("mode", _I), ("C", _I), ("ngrp", _I),
                ("rec0", _P),
                ("coef_a", _P), ("gamma_a", _P), ("beta_a", _P), ("rm_a", _P), ("rv_a", _P),
                ("p_gstride", _LL), ("momentum", _F), ("eps", _F), ("relu", _I),
                ("amax_a", _P), ("amax_ld", _I),
                ("ya", _P), ("yb", _P), ("y_gstride", _LL),
                ("coef_b", _P), ("gamma_b", _P), ("amax_b", _P),
                ("dgamma_a", _P), ("dbeta_a", _P), ("dgamma_b", _P), ("dbeta_b", _P), ("gr_gstride", _LL),
                ("mask_out", _P), ("mask_lazy", _I)]


assert ctypes.sizeof(_BnFuse) == int(_L.dba_bnfuse_size()), "BnFuse layout mismatch (rebuild the kernels)"


NOT_HANDLED = -100   # an entry point declining a shape (the stem kernel: not a stem)
F16_PAIR = 16        # the fp32 family's operand split: the scaled fp16 pair (xconv.hpp header)


def _call(name: str, *args) -> int:
    rc = getattr(_L, name)(*args)
    if rc != 0 and rc != NOT_HANDLED:
        raise RuntimeError(f"{name}: HIP error {rc}")
    return rc


def _ptr(t: Optional[Tensor]):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _i32(t: Optional[Tensor]) -> Optional[Tensor]:
    if t is None:
        return None
    return t if (t.dtype == torch.int32 and t.is_contiguous()) else t.to(torch.int32).contiguous()


def _inner_contig(t: Tensor) -> bool:
    """True if all dims but the first are densely packed (a strided row view)."""
    exp = 1
    for d in range(t.dim() - 1, 0, -1):
        if t.shape[d] != 1 and t.stride(d) != exp:
            return False
        exp *= t.shape[d]
    return True


def _rowview(t: Tensor) -> Tuple[Tensor, int]:
    if not _inner_contig(t):
        t = t.contiguous()
    return t, (t.stride(0) if t.shape[0] > 1 else int(torch.tensor(t.shape[1:]).prod()))


def _act(t: Tensor, dt: Optional[torch.dtype] = None, what: str = "activation") -> Tensor:
    """An activation operand, contiguous and NEVER converted: every kernel computes in fp32
    (split into fp16 pairs for the MFMA family).  ``dt`` pins the dtype (every operand of
    one op must agree)."""
    if t.dtype != _F32:
        raise TypeError(f"{what}: unsupported dtype {t.dtype} (fp32 only)")
    if dt is not None and t.dtype != dt:
        raise TypeError(f"{what}: dtype {t.dtype} does not match the op's {dt} operands "
                        f"(no silent precision conversion)")
    return t.contiguous()


def _f32(t: Tensor) -> int:
    return int(t.dtype == _F32)


# ------------------------------------------------------------------------- data ingest
_UNIT_AMAX = {}


def _unit_amax(G: int, device):
    """A constant max-|x| slot holding 1.0: gathered images are in [0, 1] (x / 255)."""
    key = (G, device)
    if key not in _UNIT_AMAX:
        a = torch.zeros(AMAX_SUB, _amax_ld(G), dtype=torch.int32, device=device)
        a[0, :G] = 0x3F800000
        _UNIT_AMAX[key] = a
    return _UNIT_AMAX[key]


def gather_images(src, labels, idx, trig_masks, trig_id, poison_n, target, flip_seeds, out_dtype):
    G, B = idx.shape
    _, H, W, C = src.shape
    x = torch.empty(G, B, H, W, C, dtype=out_dtype, device=src.device)
    y = torch.empty(G, B, dtype=torch.int32, device=src.device)
    idx, trig_id, poison_n, fs = _i32(idx), _i32(trig_id), _i32(poison_n), _i32(flip_seeds)
    _call("dba_gather_images", src.data_ptr(), _i32(labels).data_ptr(), idx.data_ptr(),
          trig_masks.contiguous().data_ptr(), trig_id.data_ptr(), poison_n.data_ptr(), int(target), _ptr(fs),
          x.data_ptr(), int(out_dtype == torch.float32), y.data_ptr(), G, B, H, W, C, _stream())
    if out_dtype == _F32:
        x._dba_amax = _unit_amax(G, x.device)   # an upper bound is all the scale needs
    return x, y


def gather_rows(src, labels, idx, trig_cols, trig_vals, trig_id, poison_n, target, out_dtype):
    G, B = idx.shape
    Fd = src.shape[1]
    x = torch.empty(G, B, Fd, dtype=out_dtype, device=src.device)
    y = torch.empty(G, B, dtype=torch.int32, device=src.device)
    tc = _i32(trig_cols)
    _call("dba_gather_rows", src.contiguous().data_ptr(), _i32(labels).data_ptr(), _i32(idx).data_ptr(),
          tc.data_ptr(), trig_vals.float().contiguous().data_ptr(), int(tc.shape[1]), _i32(trig_id).data_ptr(),
          _i32(poison_n).data_ptr(), int(target), x.data_ptr(), int(out_dtype == torch.float32), y.data_ptr(),
          G, B, Fd, _stream())
    return x, y


_MLP_LAYERS = ("layer1.0.weight", "layer1.0.bias", "layer2.0.weight", "layer2.0.bias", "layer3.0.weight",
               "layer3.0.bias")


def mlp_train(spec, sched, t0, t1, B, state, mom, fg, rows, labels, trig_cols, trig_vals, target, stats,
              max_slots, nan_flag, momentum, wd, prof=None) -> int:
    """Steps [t0, t1) of the step table ``sched`` [T, G*B + 8G] for every client of a LoanNet
    group in ONE launch, one workgroup per client (csrc/kernels/mlp.hip): parameters and
    momentum LDS-resident, written back to ``state`` / ``mom`` at the end.  Returns -100
    (nothing launched) for other shapes."""
    G = state.shape[0]
    es = [spec.by_name[n] for n in _MLP_LAYERS]
    offs = torch.tensor([e.offset for e in es], dtype=torch.int32)   # host table, read at launch
    (H1, F), (H2, _), (C, _) = es[0].k_shape[:2], es[2].k_shape[:2], es[4].k_shape[:2]
    assert sched.dtype == torch.int32 and sched.is_contiguous() and state.stride(1) == 1
    tc = _i32(trig_cols)
    return _call("dba_mlp_train", sched.data_ptr(), sched.shape[1], int(t0), int(t1), G, B, state.data_ptr(),
                 state.stride(0), mom.data_ptr(), _ptr(fg), spec.P, offs.data_ptr(), F, H1, H2, C,
                 rows.contiguous().data_ptr(), _i32(labels).data_ptr(), tc.data_ptr(),
                 trig_vals.float().contiguous().data_ptr(), int(tc.shape[1]), int(target), stats.data_ptr(),
                 stats.shape[1], max_slots, nan_flag.data_ptr(), float(momentum), float(wd), _ptr(prof), _stream())


# ------------------------------------------------------------------------------ conv
def _check_w(w: Tensor, dt: torch.dtype = _F32) -> Tuple[Tensor, int]:
    if w.dtype != dt:
        raise TypeError(f"conv weights: dtype {w.dtype} does not match the {dt} activations "
                        f"(no silent precision conversion)")
    return _rowview(w)


def set_ximg(on: int) -> int:
    """Whole-image halo conv of the 8 / 4-wide evaluation stages (xconv_fwd.hip ximg_kernel) on /
    off; -1 queries.  Returns the previous setting (tests: A/B against the implicit GEMM)."""
    return int(_L.dba_ximg_set(int(on)))


def set_wgrad_halo(on: int) -> int:
    """Patch-reuse weight gradient of the narrow stages' 3x3 convs (xwgrad_halo.hip) on / off;
    -1 queries.  Returns the previous setting (tests: A/B against the implicit GEMM)."""
    return int(_L.dba_xwgrad_halo_set(int(on)))


def set_split_policy(target: int = -1, min_k: int = -1, max_s: int = -1, kslab_max: int = -1,
                     dgrad_ks: int = -1) -> None:
    """Split-K policy of the small forward / data-gradient launches (xconv.hpp ``xsplitk``:
    target tiles per replica, minimum k-steps per slab, maximum slabs, maximum in-block
    slabs, grouped data gradients as in-block slabs 1 / 0); negative keeps a value.  Any
    setting is deterministic and group-size independent."""
    _call("dba_xsplit_policy", int(target), int(min_k), int(max_s), int(kslab_max), int(dgrad_ks))


_STEM_WGRAD = True


def set_stem_wgrad(on: int) -> int:
    """The stem's own weight gradient (xwgrad_stem.hip) on / off; -1 queries.  Returns the
    previous setting (tests: A/B against the implicit GEMM)."""
    global _STEM_WGRAD
    prev = int(_STEM_WGRAD)
    if on >= 0:
        _STEM_WGRAD = bool(on)
    return prev


def fp32_mode() -> int:
    """The fp32 family's operand split (one since round 5: the scaled fp16 pair)."""
    return F16_PAIR


# ---- operand max |x| slots of the fp16 pair (csrc/kernels/common.hpp): int32 [16, ld]
AMAX_SUB = 16


def _amax_ld(G: int) -> int:
    return max(32, (G + 31) // 32 * 32)


class _AmaxArena:
    """One zeroed allocation for all the slots of a forward / backward pass: a single fill
    (captured into the training step's graph: re-zeroed at every replay) instead of one per
    producer."""

    def __init__(self, G: int, device, n: int, counters: int = 0) -> None:
        self.G, self.ld, self.next = G, _amax_ld(G), 0
        slots = n * AMAX_SUB * self.ld
        flat = torch.zeros(slots + counters, dtype=torch.int32, device=device)
        self.buf = flat[:slots].view(n, AMAX_SUB, self.ld)
        # arrival counters of the in-launch split-K combines (xconv.hpp sk_combine), zeroed by
        # the same fill
        self.cnt, self.cnt_next = flat[slots:], 0

    def counters(self, n: int, device):
        if n <= 0 or device != self.cnt.device or self.cnt_next + n > self.cnt.numel():
            return None
        self.cnt_next += n
        return self.cnt[self.cnt_next - n:self.cnt_next]

    def take(self, G: int, device):
        if G != self.G or self.next >= self.buf.shape[0] or device != self.buf.device:
            return None
        self.next += 1
        return self.buf[self.next - 1]


_ARENA: list = []


@contextlib.contextmanager
def amax_arena(G: int, device, n: int = 256, counters: int = 0):
    """Slots for the enclosed launches' fp16-pair operand maxima, and ``counters`` zeroed ints
    for their in-launch split-K combines (:func:`_sk_counters`)."""
    _ARENA.append(_AmaxArena(G, device, n, counters))
    try:
        yield
    finally:
        _ARENA.pop()


def amax_slots(n: int, G: int, device):
    """``n`` zeroed operand-max slots in one allocation ([n][AMAX_SUB][ld])."""
    return torch.zeros(n, AMAX_SUB, _amax_ld(G), dtype=torch.int32, device=device)


def _amax_new(G: int, device):
    a = _ARENA[-1].take(G, device) if _ARENA else None
    return a if a is not None else torch.zeros(AMAX_SUB, _amax_ld(G), dtype=torch.int32, device=device)


def _sk_counters(n: int, device):
    """``n`` zeroed arrival counters for an in-launch split-K combine (xconv.hpp sk_combine)
    from the enclosing arena (None: no arena / exhausted — the launch then runs the separate
    reduce kernel, same bits)."""
    if n <= 0 or not _ARENA:
        return None
    return _ARENA[-1].counters(n, device)


def _aptr(a):
    """(pointer, leading dimension) of an amax slot (None: no slot)."""
    return (None, 0) if a is None else (a.data_ptr(), a.shape[-1])


def _amax(t, gstride, n_per_g, nvalid=None, per_item=0):
    """Per-replica max |t| slot of the fp16-pair operand scales; rows of invalid images are
    excluded (their contents are undefined)."""
    G = t.shape[0]
    out = _amax_new(G, t.device)
    _call("dba_amax", t.data_ptr(), gstride, n_per_g, _ptr(_i32(nvalid)), per_item, G, out.data_ptr(), out.shape[1],
          _stream())
    return out


def _amax_out(t):
    """Zeroed slot for a producer to fold its fp32 output's max into, attached to ``t`` for its
    consumers."""
    if t.dtype != _F32:
        return None
    a = _amax_new(t.shape[0], t.device)
    t._dba_amax = a
    return a


def weight_amax(flat, segments):
    """Max |w| slots of ``segments = [(offset, length)]`` of the ``[G, S]`` flat replica rows, in
    one launch (a training step's conv weights): a list of slots."""
    G, n = flat.shape[0], len(segments)
    ar = _ARENA[-1] if _ARENA else None
    if ar is not None and ar.G == G and ar.buf.device == flat.device and ar.next + n <= ar.buf.shape[0]:
        buf, ar.next = ar.buf[ar.next:ar.next + n], ar.next + n
    else:
        buf = torch.zeros(n, AMAX_SUB, _amax_ld(G), dtype=torch.int32, device=flat.device)
    slots, base = list(buf), buf.data_ptr()
    d = torch.tensor(segments, dtype=torch.int64)   # host table, passed by value
    _call("dba_amax_segments", flat.data_ptr(), flat.stride(0), d.data_ptr(), len(segments), G, base,
          slots[0].shape[1], _stream())
    return slots


def split_weights(w, sstride: int, per: int, amax):
    """fp16-pair planes of a weight operand ([slots][2][per] fp16, scaled by the slot's max |w|,
    csrc/kernels/xaux.hip xsplit_w_kernel), attached as ``w._dba_planes``: every block of every
    launch that stages these weights then loads the planes instead of re-splitting them."""
    slots = w.shape[0]
    out = torch.empty(slots, 2, per, dtype=torch.int16, device=w.device)
    _call("dba_xsplit_w", w.data_ptr(), sstride, per, slots, amax.data_ptr(), amax.shape[1], out.data_ptr(), _stream())
    w._dba_planes = out
    return out


def split_weights_batch(items) -> None:
    """:func:`split_weights` of ``items = [(w, sstride, per, amax)]`` (same slot count) in one
    launch (per 24): a model fold's 20 weight splits."""
    if not items:
        return
    slots = items[0][0].shape[0]
    desc, outs = [], []
    for w, sstride, per, amax in items:
        assert w.shape[0] == slots and w.dtype == torch.float32
        out = torch.empty(slots, 2, per, dtype=torch.int16, device=w.device)
        desc.append([w.data_ptr(), sstride, per, amax.data_ptr(), amax.shape[1], out.data_ptr(), 0])
        outs.append(out)
    d = torch.tensor(desc, dtype=torch.int64)   # host table, passed by value
    _call("dba_xsplit_w_batch", d.data_ptr(), len(items), slots, _stream())
    for (w, *_), out in zip(items, outs):
        w._dba_planes = out


def _wplanes(w):
    """(pointer, slot stride) of ``w``'s fp16-pair planes, if split."""
    p = getattr(w, "_dba_planes", None)
    return (None, 0) if p is None else (p.data_ptr(), p.stride(0))


def _amax_w(w, gstride, n):
    a = getattr(w, "_dba_amax", None)
    if a is None:
        a = _amax(w, gstride, n)
        w._dba_amax = a   # weights are not written while this view is alive
    return a


def _amax_act(t, nvalid):
    """[G][N][...] activation (contiguous per replica); a producer that already folded its
    output's max into ``t._dba_amax`` (conv epilogue, BN apply) saves the pass."""
    a = getattr(t, "_dba_amax", None)
    if a is not None:
        return a
    per_item = t[0, 0].numel()
    a = _amax(t, t.stride(0), t.shape[1] * per_item, nvalid, per_item)
    t._dba_amax = a   # activations are never written in place: the fwd / wgrad pair shares it
    return a


_EVAL_STEM_MFMA = os.environ.get("DBA_EVAL_STEM7_MFMA", "1") != "0"
_EVAL_STEM_PAD = True   # (the kernel bench's A/B of the channel padding)


def _xconv_fwd(x, w, wsel, stride, pad, bias, residual, relu, nvalid, out_dtype, bnf=None, lz=None):
    """Reference-precision conv (fp32 in / fp32 out, fp16-pair MFMA: xconv.hpp).  ``bnf``: the
    fused training-BN statistics of the output (bnfuse.hpp); ``lz``: the input is a lazy BN
    output (its coefficients, ReLU, bound slot)."""
    if out_dtype not in (None, _F32):
        raise TypeError(f"fp32 conv cannot emit {out_dtype} (no silent precision conversion)")
    G, N, H, W, Cin = x.shape
    attrs = {k: getattr(w, k) for k in ("_dba_amax", "_dba_planes") if hasattr(w, k)}
    w, ws = _check_w(w, _F32)
    for k, v in attrs.items():
        setattr(w, k, v)
    Cout, KH, KW = w.shape[1], w.shape[2], w.shape[3]
    assert w.shape[4] == Cin, (w.shape, x.shape)
    Ho = (H + 2 * pad - KH) // stride + 1
    Wo = (W + 2 * pad - KW) // stride + 1
    y = torch.empty(G, N, Ho, Wo, Cout, dtype=_F32, device=x.device)
    bs = 0
    if bias is not None:
        if bias.dtype != _F32:
            raise TypeError(f"conv bias must be fp32 (got {bias.dtype})")
        bias, bs = _rowview(bias)
    res = _act(residual, _F32, "residual") if residual is not None else None
    ay = _amax_out(y) if bnf is None else None   # the output's max, for its consumers
    bnf_p = ctypes.byref(bnf) if bnf is not None else None
    # evaluation of a wide stem (Tiny-ImageNet's 7x7, K = 147; its weights pre-split at the
    # eval fold) runs on the fp16-pair MFMAs: the exact-FMA stem kernel reaches ~64 TFLOP/s of
    # VALU there and took 15 % of a Tiny round's GPU time (profiles/r6/tiny/).  Training keeps
    # the exact kernel (the training bits; on the MFMAs a Tiny lone step was 2.126 vs 2.142 ms,
    # profiles/r6/tiny/train_stem_ab.md), and so do the K = 27 / 25 stems, whose one-k-step MFMA
    # tiles are all prologue and epilogue.
    eval_mfma = (_EVAL_STEM_MFMA and "_dba_planes" in attrs and bnf is None and KH * KW * Cin > 64)
    if eval_mfma and Cin % 4 and _EVAL_STEM_PAD and lz is None:
        # ... with the channels zero-padded to a multiple of 4: the implicit GEMM then stages
        # one 16-B load per tap instead of Cin scalar loads (the zero channel adds K, never a bit
        # of the sums beyond the fp16-pair grid: 0 * w = 0)
        cp = 4 - Cin % 4
        x4 = torch.nn.functional.pad(x, (0, cp))
        x4._dba_amax = _amax_act(x, nvalid)
        w4 = torch.nn.functional.pad(w, (0, cp)).contiguous()
        per4 = w4[0].numel()
        a4 = attrs.get("_dba_amax")
        split_weights(w4, per4, per4, a4 if a4 is not None else _amax_w(w4, per4, per4))
        if a4 is not None:
            w4._dba_amax = a4
        return _xconv_fwd(x4, w4, wsel, stride, pad, bias, residual, relu, nvalid, out_dtype)
    if Cin <= 4 and not eval_mfma:
        # few-channel image stems: exact-fp32 direct conv (stem.hip), -100 = not a stem shape
        rc = _call("dba_xstem_fwd", x.data_ptr(), N * H * W * Cin, w.data_ptr(), ws, _ptr(_i32(wsel)), _ptr(bias), bs,
                   _ptr(res), y.data_ptr(), N * Ho * Wo * Cout, _ptr(_i32(nvalid)), G, N, H, W, Cin, Ho, Wo, Cout,
                   KH, KW, stride, pad, int(relu), *_aptr(ay), bnf_p, _stream())
        if rc != NOT_HANDLED:
            return y
    n = int(_L.dba_xconv_ws_floats(G, N, Ho, Wo, Cin, Cout, KH, KW))
    wsb = torch.empty(n, dtype=_F32, device=x.device) if n > 0 else None
    # split-K launch: slabs combined in the launch when the arena has counters for it
    ncnt = int(_L.dba_xconv_sk_ints(G, N, Ho, Wo, Cin, Cout, KH, KW)) if n > 0 else 0
    cnt = _sk_counters(ncnt, x.device)
    ax = lz[2] if lz is not None else _amax_act(x, nvalid)
    aw = _amax_w(w, ws, Cout * KH * KW * Cin)
    lz_coef, lz_relu = (lz[0].data_ptr(), int(lz[1])) if lz is not None else (None, 0)
    _call("dba_xconv_fwd", x.data_ptr(), N * H * W * Cin, w.data_ptr(), ws, _ptr(_i32(wsel)), _ptr(bias), bs,
          _ptr(res), y.data_ptr(), N * Ho * Wo * Cout, _ptr(_i32(nvalid)), G, N, H, W, Cin, Ho, Wo, Cout, KH, KW,
          stride, pad, int(relu), *_aptr(ax), *_aptr(aw), *_aptr(ay), *_wplanes(w), _ptr(wsb), n,
          _ptr(cnt), 0 if cnt is None else cnt.numel(), bnf_p, lz_coef, lz_relu, _stream())
    return y


_EVAL_BLOCK = os.environ.get("DBA_EVAL_BLOCK", "1") != "0"
# (width, channels) of the fused BasicBlock kernel (xblock.hip): the 32-wide stage.  Whole-image
# forms for the 16 / 8 / 4-wide stages were measured slower than the two launches (block /
# 2 x conv: 1.13, 1.07, 2.15 — per-workgroup row counts of 256 / 64 / 32 re-read the weights
# from L2 far more often than the 128-row implicit GEMM tiles: profiles/r4/xblock/README.md)
_BLOCK_SHAPES = {(32, 32)}


def basic_block_ok(x, w1, w2) -> bool:
    """The fused evaluation BasicBlock (csrc/kernels/xblock.hip) takes this block: fp32
    [G, N, W, W, C] input of a CIFAR ResNet stage, C -> C 3x3 weights pre-split at the eval fold.
    ``DBA_EVAL_BLOCK=0``: off (the two convs run; the A/B of profiles/r4/xblock/)."""
    if not (_EVAL_BLOCK and x.dtype == _F32 and x.dim() == 5):
        return False
    H, W, C = x.shape[2:]
    return (H == W and (W, C) in _BLOCK_SHAPES
            and all(w.dtype == _F32 and tuple(w.shape[1:]) == (C, 3, 3, C)
                    and getattr(w, "_dba_planes", None) is not None for w in (w1, w2)))


def basic_block_eval(x, w1, b1, w2, b2, wsel=None, nvalid=None):
    """relu(conv2(relu(conv1(x) + b1)) + b2 + x) in one launch (BN folded into w / b; the mid
    activation stays in LDS): xblock.hip.  Callers check :func:`basic_block_ok` first."""
    x = _act(x, _F32, "conv input")
    G, N, _, W, C = x.shape
    per = C * 9 * C
    (w1c, ws1), (w2c, ws2) = _check_w(w1), _check_w(w2)
    aw1, aw2 = _amax_w(w1, ws1, per), _amax_w(w2, ws2, per)
    p1, p2 = w1._dba_planes, w2._dba_planes
    assert p1.stride(0) == p2.stride(0) and aw1.shape[1] == aw2.shape[1]
    (b1c, bs1), (b2c, bs2) = _rowview(b1), _rowview(b2)
    assert bs1 == bs2 and b1c.dtype == b2c.dtype == _F32
    ax = _amax_act(x, nvalid)
    y = torch.empty_like(x)
    ay = _amax_out(y)
    rc = _call("dba_xblock_fwd", x.data_ptr(), x.stride(0), y.data_ptr(), y.stride(0), _ptr(_i32(wsel)),
               p1.data_ptr(), p2.data_ptr(), p1.stride(0), b1c.data_ptr(), b2c.data_ptr(), bs1, _ptr(_i32(nvalid)),
               G, N, W, W, C, C, *_aptr(ax), aw1.data_ptr(), aw2.data_ptr(), aw1.shape[1], *_aptr(ay), _stream())
    if rc == NOT_HANDLED:
        raise RuntimeError("xblock_fwd declined a shape basic_block_ok accepted")
    return y


_EVAL_STEM = os.environ.get("DBA_EVAL_STEM", "1") != "0"


def stem_block_ok(x, w0, w1, w2) -> bool:
    """The stem + first BasicBlock of the 32-wide stage run as one launch (xblock.hip STEM
    variant): [G, N, 32, 32, 3] fp32 images, a 3x3 3 -> 32 stem and the block's weights all
    pre-split at the eval fold.  ``DBA_EVAL_STEM=0``: off (stem launch + fused block)."""
    if not (_EVAL_STEM and _EVAL_BLOCK and x.dtype == _F32 and x.dim() == 5 and tuple(x.shape[2:]) == (32, 32, 3)):
        return False
    return (w0.dtype == _F32 and tuple(w0.shape[1:]) == (32, 3, 3, 3) and getattr(w0, "_dba_planes", None) is not None
            and all(w.dtype == _F32 and tuple(w.shape[1:]) == (32, 3, 3, 32)
                    and getattr(w, "_dba_planes", None) is not None for w in (w1, w2)))


def stem_block_eval(x, w0, b0, w1, b1, w2, b2, wsel=None, nvalid=None):
    """relu(conv2(h) + b2 + s), h = relu(conv1(s) + b1), s = relu(stem(x) + b0): the CIFAR
    ResNet stem and layer1.0 (BN folded) in one launch; the stem output stays on chip
    (xblock.hip).  Callers check :func:`stem_block_ok` first."""
    x = _act(x, _F32, "image")
    G, N, _, W, Ci = x.shape
    C = w1.shape[1]
    per = C * 9 * C
    (w0c, ws0), (w1c, ws1), (w2c, ws2) = _check_w(w0), _check_w(w1), _check_w(w2)
    aw0 = _amax_w(w0, ws0, C * 9 * Ci)
    aw1, aw2 = _amax_w(w1, ws1, per), _amax_w(w2, ws2, per)
    p0, p1, p2 = w0._dba_planes, w1._dba_planes, w2._dba_planes
    assert p1.stride(0) == p2.stride(0) and aw0.shape[1] == aw1.shape[1] == aw2.shape[1]
    (b0c, bs0), (b1c, bs1), (b2c, bs2) = _rowview(b0), _rowview(b1), _rowview(b2)
    assert bs1 == bs2 and b0c.dtype == b1c.dtype == b2c.dtype == _F32
    y = torch.empty(G, N, W, W, C, dtype=_F32, device=x.device)
    ay = _amax_out(y)
    rc = _call("dba_xblock_stem_fwd", x.data_ptr(), x.stride(0), y.data_ptr(), y.stride(0), _ptr(_i32(wsel)),
               p0.data_ptr(), p0.stride(0), b0c.data_ptr(), bs0, p1.data_ptr(), p2.data_ptr(), p1.stride(0),
               b1c.data_ptr(), b2c.data_ptr(), bs1, _ptr(_i32(nvalid)), G, N, W, W, Ci, C, aw0.data_ptr(),
               aw1.data_ptr(), aw2.data_ptr(), aw1.shape[1], *_aptr(ay), _stream())
    if rc == NOT_HANDLED:
        raise RuntimeError("xblock_stem_fwd declined a shape stem_block_ok accepted")
    return y


def down_block_ok(a, w2, x2, wsc) -> bool:
    """The downsampling block's conv2 + 1x1 stride-2 shortcut run as one launch (xconv_fwd.hip
    dba_xdown_fwd: the shortcut as an extra k-step of the W-16 halo conv): fp32 [G, N, 16, 16, 64]
    ``a``, shortcut input [G, N, 32, 32, 32], both weights pre-split at the eval fold — the CIFAR
    ResNets' layer2.0.  ``DBA_EVAL_DOWN=0``: off (two launches; the same-box A/B of
    profiles/r5/down/).  (The 8 / 4-wide stages' fused form measured slower than two launches.)"""
    if not (_EVAL_DOWN and a.dtype == _F32 and x2.dtype == _F32 and a.dim() == 5 and x2.dim() == 5):
        return False
    H, W, C = a.shape[2:]
    H2, W2, C2 = x2.shape[2:]
    # the 1x1 stride-2 shortcut's output grid must be conv2's
    if H != W or (H2 - 1) // 2 + 1 != H or (W2 - 1) // 2 + 1 != W or a.shape[:2] != x2.shape[:2]:
        return False
    if any(getattr(t, "_dba_planes", None) is None for t in (w2, wsc)):
        return False
    if tuple(w2.shape[1:]) != (C, 3, 3, C) or tuple(wsc.shape[1:]) != (C, 1, 1, C2):
        return False
    return W == 16 and C == 64 and C2 == 32


def down_block_eval(a, w2, b2, x2, wsc, bsc, wsel=None, nvalid=None):
    """relu(conv3x3(a, w2) + b2 + conv1x1_s2(x2, wsc) + bsc) in one launch (BN folded); callers
    check :func:`down_block_ok` first."""
    a = _act(a, _F32, "conv input")
    x2 = _act(x2, _F32, "shortcut input")
    G, N, Ho, Wo, C = a.shape
    _, _, H2, W2, C2 = x2.shape
    (w2c, ws2), (wscc, wss) = _check_w(w2), _check_w(wsc)
    aw2, awsc = _amax_w(w2, ws2, C * 9 * C), _amax_w(wsc, wss, C * C2)
    p2, psc = w2._dba_planes, wsc._dba_planes
    (b2c, bs2), (bscc, bss) = _rowview(b2), _rowview(bsc)
    aa, ax2 = _amax_act(a, nvalid), _amax_act(x2, nvalid)
    y = torch.empty_like(a)
    ay = _amax_out(y)
    rc = _call("dba_xdown_fwd", a.data_ptr(), a.stride(0), w2c.data_ptr(), ws2, p2.data_ptr(), p2.stride(0),
               _ptr(_i32(wsel)), b2c.data_ptr(), bs2, x2.data_ptr(), x2.stride(0), psc.data_ptr(), psc.stride(0),
               bscc.data_ptr(), bss, y.data_ptr(), y.stride(0), _ptr(_i32(nvalid)), G, N, Ho, Wo, C, H2, W2, C2,
               *_aptr(aa), *_aptr(aw2), *_aptr(ax2), *_aptr(awsc), *_aptr(ay), _stream())
    if rc == NOT_HANDLED:
        raise RuntimeError("xdown_fwd declined a shape down_block_ok accepted")
    return y


_EVAL_DOWN = os.environ.get("DBA_EVAL_DOWN", "1") != "0"


def conv2d(x, w, wsel, stride, pad, bias=None, residual=None, relu=False, nvalid=None, out_dtype=None,
           bn_stats=False):
    """``bn_stats`` is a reference-API hint (training BN goes through :func:`conv_bn_stats`)."""
    return _xconv_fwd(_act(x, _F32, "conv input"), w, wsel, stride, pad, bias, residual, relu, nvalid, out_dtype)


def _xtranspose(items) -> list:
    """Parity-class packed fp32 data-gradient weights (xconv_dgrad.hip xtranspose_kernel) of
    ``items = [(w, stride, pad, nvalid_or_None)]`` (same slot count) in ONE launch."""
    outs, desc, max_per, nv = [], [], 0, None
    slots = items[0][0].shape[0]
    for w, stride, pad, nvalid in items:
        wv, ws = _check_w(w, _F32)
        _, Cout, KH, KW, Cin = wv.shape
        per = Cout * KH * KW * Cin
        wt = torch.empty(slots, per, dtype=_F32, device=wv.device)
        outs.append(wt)
        desc.append([wv.data_ptr(), wt.data_ptr(), ws, Cout, KH, KW, Cin, stride, pad, 0])
        max_per = max(max_per, per)
        nv = nvalid
    d = torch.tensor(desc, dtype=torch.int64)    # host table: the launcher passes it by value
    _call("dba_xtranspose", d.data_ptr(), len(desc), slots, max_per, _ptr(_i32(nv)), _stream())
    return outs


def prepare_dgrad_weights(ref, items):
    """All of a training step's data-gradient weight transposes in ONE launch.

    ``items``: list of ``(w, wsel, stride, pad, in_hw, nvalid, G)`` for every conv whose input
    gradient the backward pass will compute.  Returns ``{index: wt}`` to be handed to
    :func:`conv2d_dgrad` as ``wt=`` (every data gradient reads class-packed transposed weights;
    items of another slot count are transposed by their own dgrad)."""
    if not items:
        return {}
    slots = items[0][0].shape[0]
    sel = [k for k, it in enumerate(items) if it[0].shape[0] == slots]
    it0 = items[sel[0]]
    nv = it0[5] if (it0[1] is None and it0[5] is not None and slots == it0[6]) else None
    wts = _xtranspose([(items[k][0], items[k][2], items[k][3], nv) for k in sel])
    return dict(zip(sel, wts))


def _xconv_dgrad(dy, w, wsel, stride, pad, in_hw, nvalid, out_dtype, accum, wt, finish=None):
    if out_dtype not in (None, _F32):
        raise TypeError(f"fp32 dgrad cannot emit {out_dtype} (no silent precision conversion)")
    G, N, Ho, Wo, Cout = dy.shape
    wv, _ = _check_w(w, _F32)
    slots, _, KH, KW, Cin = wv.shape
    H, W = in_hw
    if wt is None:
        nv = nvalid if (wsel is None and nvalid is not None and slots == G) else None
        wt = _xtranspose([(wv, stride, pad, nv)])[0]
    per = Cout * KH * KW * Cin
    assert wt.dtype == _F32 and wt.is_contiguous() and wt.numel() == slots * per
    dx = torch.empty(G, N, H, W, Cin, dtype=_F32, device=dy.device)
    acc = _act(accum, _F32, "dgrad accum") if accum is not None else None
    if acc is not None:
        assert acc.shape == dx.shape
    n = int(_L.dba_xconv_ws_floats(G, N, H, W, Cout, Cin, KH, KW)) if stride == 1 else 0
    wsb = torch.empty(n, dtype=_F32, device=dy.device) if n > 0 else None
    cnt = _sk_counters(int(_L.dba_xconv_sk_ints(G, N, H, W, Cout, Cin, KH, KW)) if n > 0 else 0, dy.device)
    a0 = getattr(w, "_dba_amax", None)   # the forward weights' max is the transpose's
    ad, aw = _amax_act(dy, nvalid), (a0 if a0 is not None else _amax(wt, per, per))
    bnf = _bnf_bwd(finish, G, N * H * W, dx.device) if (finish is not None and stride == 1) else None
    _call("dba_xconv_dgrad", dy.data_ptr(), N * Ho * Wo * Cout, wt.data_ptr(), per, _ptr(_i32(wsel)), _ptr(acc),
          dx.data_ptr(), N * H * W * Cin, _ptr(_i32(nvalid)), G, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad,
          *_aptr(ad), *_aptr(aw), *_wplanes(wt), _ptr(wsb), n, _ptr(cnt), 0 if cnt is None else cnt.numel(),
          ctypes.byref(bnf) if bnf is not None else None, _stream())
    if finish is None:
        return dx
    if bnf is not None:
        return bs.Fin(dx, finish.stats())
    return bn_finish(dx, finish, nvalid)   # stride-s data gradient: the standalone pass


def conv2d_dgrad(dy, w, wsel, stride, pad, in_hw, nvalid=None, out_dtype=None, accum=None, wt=None, finish=None):
    return _xconv_dgrad(_act(dy, _F32, "dgrad dy"), w, wsel, stride, pad, in_hw, nvalid, out_dtype, accum, wt, finish)


def conv2d_wgrad(dy, x, stride, pad, kh, kw, dw, dbias=None, nvalid=None, defer=None):
    """``defer`` (a list, fp32 family): the slab reduction is queued there and run for the whole
    backward pass by :func:`wgrad_flush` (one launch instead of one per conv).  ``dy`` may be a
    ``LazyGrad`` (a training BN's input gradient, staged from (d, y); its value is stored once
    and returned for the data gradient — except for the 3-channel stem, whose input has no
    gradient: its weight gradient forms dy while staging and returns None) and ``x`` a ``LazyBN``
    (a training BN's output, staged from y)."""
    if _stem_wgrad_ok(dy, x, stride, pad, kh, kw, dbias):
        return _stem_wgrad(dy, x, dw, nvalid, defer)
    if isinstance(dy, bs.LazyGrad):
        # the BN input gradient stored by one elementwise pass (bnx_dy_kernel; staging it from
        # (d, y) in the weight gradient was slower: profiles/r4/bnx/ab_steps.md), then the plain
        # weight gradient; returned for the data gradient
        dy = _bnx_dy(dy, nvalid)
        conv2d_wgrad(dy, x, stride, pad, kh, kw, dw, dbias, nvalid, defer)
        return dy
    lx = x if isinstance(x, bs.LazyBN) else None
    dy = _act(dy, _F32, "wgrad dy")
    x = _act(lx.y if lx is not None else x, _F32, "wgrad x")
    G, N, Ho, Wo, Cout = dy.shape
    _, _, H, W, Cin = x.shape
    assert dw.dtype == torch.float32 and _inner_contig(dw)
    mchunk = ctypes.c_int(0)
    n = int(_L.dba_xwgrad_ws_floats(G, N, Ho, Wo, Cin, Cout, kh, kw, ctypes.byref(mchunk)))
    wsb = torch.empty(n, dtype=_F32, device=dy.device) if n > 0 else None
    nv = _i32(nvalid)
    ad = _amax_act(dy, nvalid)
    ax = lx.stat.bound if lx is not None else _amax_act(x, nvalid)
    _call("dba_xwgrad", dy.data_ptr(), N * Ho * Wo * Cout, x.data_ptr(), N * H * W * Cin, dw.data_ptr(),
          dw.stride(0), _ptr(nv), G, N, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pad, *_aptr(ad), *_aptr(ax),
          _ptr(wsb), n, int(defer is not None and n > 0),
          _ptr(lx.stat.coef) if lx is not None else None, int(lx.relu) if lx is not None else 0, _stream())
    if defer is not None and n > 0:
        per = Cout * kh * kw * Cin
        # (keeps the slab workspace and nvalid alive until the flush)
        defer.append(([wsb.data_ptr(), dw.data_ptr(), dw.stride(0), per, _ptr(nv) or 0, N, Ho * Wo,
                       mchunk.value, G, 0], wsb, nv))
    if dbias is not None:
        assert dbias.dtype == torch.float32 and dbias.stride(1) == 1
        part = torch.empty(int(_L.dba_xcolsum_part_doubles(G, N, Ho * Wo, Cout)), dtype=torch.float64,
                           device=dy.device)
        _call("dba_xcolsum", dy.data_ptr(), N * Ho * Wo * Cout, Ho * Wo, _ptr(_i32(nvalid)), G, N, Cout,
              dbias.data_ptr(), dbias.stride(0), part.data_ptr(), _stream())
    return None


_STEM_PER = 32 * 27   # the stem weight gradient's [32][3][3][3] elements


def _stem_wgrad_ok(dy, x, stride, pad, kh, kw, dbias) -> bool:
    """The 3 -> 32 channel 3x3 stride-1 stem (xwgrad_stem.hip) of a stored input."""
    if not _STEM_WGRAD or dbias is not None or isinstance(x, bs.LazyBN) or (stride, pad, kh, kw) != (1, 1, 3, 3):
        return False
    d = dy.d if isinstance(dy, bs.LazyGrad) else dy
    if x.dim() != 5 or x.shape[-1] != 3 or x.dtype != _F32 or d.dtype != _F32 or d.shape[-1] != 32:
        return False
    G, N, H, W, _ = x.shape
    return tuple(d.shape) == (G, N, H, W, 32) and int(_L.dba_xwgrad_stem_ws_floats(G, N, H, W, 3, 32)) > 0


def _stem_wgrad(dy, x, dw, nvalid, defer):
    """Stem weight gradient: one 256-pixel slab per workgroup (exact fp32 FMAs), reduced by the
    batched slab reduction with ``mchunk`` 256; a ``LazyGrad`` dy is formed while staging."""
    lg = dy if isinstance(dy, bs.LazyGrad) else None
    d = _act(lg.d if lg is not None else dy, _F32, "wgrad dy")
    y = None
    if lg is not None:
        y = _act(lg.y, _F32, "BN input")
        assert y.shape == d.shape and y.stride(0) == d.stride(0)
    x = _act(x, _F32, "wgrad x")
    assert dw.dtype == torch.float32 and _inner_contig(dw) and dw[0].numel() == _STEM_PER
    G, N, H, W, _ = x.shape
    wsb = torch.empty(int(_L.dba_xwgrad_stem_ws_floats(G, N, H, W, 3, 32)), dtype=_F32, device=x.device)
    nv = _i32(nvalid)
    _call("dba_xwgrad_stem", d.data_ptr(), d.stride(0), _ptr(y), _ptr(lg.stat.coef) if lg is not None else None,
          x.data_ptr(), x.stride(0), wsb.data_ptr(), _ptr(nv), G, N, H, W, _stream())
    entry = ([wsb.data_ptr(), dw.data_ptr(), dw.stride(0), _STEM_PER, _ptr(nv) or 0, N, H * W, 256, G, 0], wsb, nv)
    if defer is not None:
        defer.append(entry)
    else:
        wgrad_flush([entry])
    return None


# ------------------------------------------------------------ fused training BN (bnfuse.hpp)
def _bnf_common(mode: int, G: int, M: int, C: int, device):
    """A fused BN pass (bnfuse.hpp) over M rows per replica: its level-0 record workspace."""
    ngrp = (M + 31) // 32
    rec0 = torch.empty(G * C * ngrp * 4, dtype=torch.float64, device=device)
    f = _BnFuse()
    f.mode, f.C, f.ngrp, f.rec0 = mode, C, ngrp, rec0.data_ptr()
    f._keep = (rec0,)   # alive until the launches have been enqueued
    return f


def _bnf_fwd(p: "bs.BnParams", relu: bool, G: int, M: int, C: int, device):
    """Forward statistics (mode 1) of a conv output feeding BN ``p``: the BnStat it fills."""
    coef = torch.empty(G, bs.ROWS, C, dtype=_F32, device=device)
    bound = _amax_new(G, device)
    st = bs.BnStat(coef, p, bound)
    f = _bnf_common(1, G, M, C, device)
    ps = _same_stride(p.gamma, p.beta, p.rmean, p.rvar)
    f.coef_a, f.gamma_a, f.beta_a = coef.data_ptr(), p.gamma.data_ptr(), p.beta.data_ptr()
    f.rm_a, f.rv_a, f.p_gstride = p.rmean.data_ptr(), p.rvar.data_ptr(), ps
    f.momentum, f.eps, f.relu = float(p.momentum), float(p.eps), int(relu)
    f.amax_a, f.amax_ld = bound.data_ptr(), bound.shape[1]
    return f, st


def _bnf_bwd(fin: "bs.Finish", G: int, M: int, device):
    """Backward mask + reduce (mode 2) of a BN output's gradient (``fin``); allocates the dy
    bound slots of its BNs."""
    sa, sb = fin.sa, fin.sb
    C = sa.C
    f = _bnf_common(2, G, M, C, device)
    ya = _act(fin.ya, _F32, "BN input")
    pa = sa.params
    f.coef_a, f.gamma_a, f.p_gstride = sa.coef.data_ptr(), pa.gamma.data_ptr(), _same_stride(pa.gamma)
    f.ya, f.y_gstride = ya.data_ptr(), ya.stride(0)
    f.dgamma_a, f.dbeta_a, f.gr_gstride = pa.dgamma.data_ptr(), pa.dbeta.data_ptr(), _same_stride(pa.dgamma, pa.dbeta)
    sa.dbound = _amax_new(G, device)
    f.amax_a, f.amax_ld = sa.dbound.data_ptr(), sa.dbound.shape[1]
    keep = [ya]
    if sb is not None:
        yb = _act(fin.yb, _F32, "BN input")
        assert yb.stride(0) == ya.stride(0) and sb.C == C
        pb = sb.params
        assert _same_stride(pb.gamma) == f.p_gstride and _same_stride(pb.dgamma, pb.dbeta) == f.gr_gstride
        f.yb, f.coef_b, f.gamma_b = yb.data_ptr(), sb.coef.data_ptr(), pb.gamma.data_ptr()
        f.dgamma_b, f.dbeta_b = pb.dgamma.data_ptr(), pb.dbeta.data_ptr()
        sb.dbound = _amax_new(G, device)
        f.amax_b = sb.dbound.data_ptr()
        keep.append(yb)
    if fin.mask_out is not None:
        mo = _act(fin.mask_out, _F32, "BN output")
        assert mo.stride(0) == ya.stride(0)
        f.mask_out = mo.data_ptr()
        keep.append(mo)
    f.mask_lazy = int(bool(fin.lazy))
    f._keep = f._keep + tuple(keep)
    return f


def _bnx_dy(lg, nvalid):
    """dy = A d + B y + K of a training BN's input, stored (its max slot: the finalize's bound)."""
    d = _act(lg.d, _F32, "BN output gradient")
    y = _act(lg.y, _F32, "BN input")
    G, N, H, W, C = d.shape
    assert y.shape == d.shape
    dy = torch.empty_like(d)
    am = lg.stat.dbound
    _call("dba_bnx_dy", d.data_ptr(), y.data_ptr(), lg.stat.coef.data_ptr(), dy.data_ptr(), d.stride(0),
          _ptr(_i32(nvalid)), G, N, H * W, C, *_aptr(None), _stream())
    dy._dba_amax = am
    return dy


def conv_bn_stats(x, w, wsel, stride, pad, nvalid, p, relu):
    """y = conv(x, w) with the training-BN statistics of y reduced and finalised in the same
    launch (running stats updated); x may be a ``LazyBN`` (staged as relu?(y*scale+shift)).
    Returns (y, BnStat)."""
    lz = None
    if isinstance(x, bs.LazyBN):
        if x.stat.bound is None:
            raise RuntimeError("lazy BN operand without its bound slot")
        lz = (x.stat.coef, x.relu, x.stat.bound)
        x = x.y
    x = _act(x, _F32, "conv input")
    G, N, H, W, Cin = x.shape
    Cout, KH, KW = w.shape[1], w.shape[2], w.shape[3]
    Ho = (H + 2 * pad - KH) // stride + 1
    Wo = (W + 2 * pad - KW) // stride + 1
    f, st = _bnf_fwd(p, relu, G, N * Ho * Wo, Cout, x.device)
    y = _xconv_fwd(x, w, wsel, stride, pad, None, None, False, nvalid, None, bnf=f, lz=lz)
    return y, st


def bn_apply(a, residual, relu, nvalid=None):
    """out = relu?(y_a * scale_a + shift_a + r), r = residual (tensor), a lazy BN output's value
    (its own ReLU off), or 0 — one elementwise pass (xbn.hip bnx_apply_kernel); folds max |out|."""
    y = _act(a.y, _F32, "BN input")
    G, N, H, W, C = y.shape
    out = torch.empty_like(y)
    am = _amax_out(out)
    res = yb = cb = None
    relu_b = 0
    if isinstance(residual, bs.LazyBN):
        yb, cb, relu_b = _act(residual.y, _F32, "BN input"), residual.stat.coef, int(residual.relu)
        assert yb.shape == y.shape
    elif residual is not None:
        res = _act(residual, _F32, "residual")
        assert res.shape == y.shape
    _call("dba_bnx_apply", y.data_ptr(), a.stat.coef.data_ptr(), _ptr(res), _ptr(yb), _ptr(cb), relu_b, int(relu),
          out.data_ptr(), y.stride(0), _ptr(_i32(nvalid)), G, N, H * W, C, *_aptr(am), _stream())
    return out


def bn_finish(g, fin, nvalid=None, pool=None, hw=None):
    """Finish a BN output's gradient in one standalone pass (xbn.hip bnx_tile_kernel): d = g
    where the output is > 0 plus the backward sums / coefficients of its BN(s).  ``pool``
    ([G, N, 1, 1, C]): g is the global average pool's gradient of it.  Returns a ``Fin``."""
    ya = _act(fin.ya, _F32, "BN input")
    G, N, H, W, C = ya.shape
    f = _bnf_bwd(fin, G, N * H * W, ya.device)
    d = torch.empty_like(ya)
    src = None
    if pool is not None:
        pool = _act(pool, _F32, "pooled gradient").reshape(G, N, C)
        assert hw == (H, W)
    else:
        src = _act(g, _F32, "BN output gradient")
        assert src.shape == ya.shape
    inv_hw = float(torch.tensor(1.0, dtype=torch.float32) / torch.tensor(float(H * W), dtype=torch.float32))
    _call("dba_bnx_rows", ctypes.byref(f), _ptr(src), d.data_ptr(), ya.stride(0), _ptr(_i32(nvalid)), G, N, H * W,
          _ptr(pool), inv_hw, _stream())
    return bs.Fin(d, fin.stats())


def wgrad_prepare(dy, x, nvalid=None):
    """Attach the fp16-pair operand maxima of a weight gradient's ``dy`` and ``x`` on the
    CURRENT stream.  Called before the weight gradient moves to the side stream
    (models/program.py): a max computed there would be read unordered by the data gradient,
    which runs on the main stream and shares ``dy``'s max slot."""
    if dy.dtype == _F32:
        _amax_act(_act(dy, None, "wgrad dy"), nvalid)
        _amax_act(_act(x, _F32, "wgrad x"), nvalid)


def wgrad_flush(defer):
    """Run the weight-gradient slab reductions queued by ``conv2d_wgrad(..., defer=)``."""
    if not defer:
        return
    d = torch.tensor([e[0] for e in defer], dtype=torch.int64)
    Gmax = max(e[0][8] for e in defer)
    max_per = max(e[0][3] for e in defer)
    _call("dba_xwgrad_reduce_batch", d.data_ptr(), len(defer), Gmax, max_per, _stream())
    defer.clear()


# ------------------------------------------------------------------------ batch norm
def _same_stride(*ts: Tensor) -> int:
    s = ts[0].stride(0)
    for t in ts:
        assert t.dtype == torch.float32 and t.stride(-1) == 1 and (t.shape[0] == 1 or t.stride(0) == s)
    return s


def relu_mask_bwd(dout, out):
    dout = _act(dout, None, "relu dout")
    out = _act(out, dout.dtype, "relu output")
    din = torch.empty_like(dout)
    _call("dba_relu_mask_bwd", dout.data_ptr(), out.data_ptr(), din.data_ptr(), dout.numel(), _f32(dout), _stream())
    return din


def bn_fold(w, conv_bias, gamma, beta, rmean, rvar, eps, out_dtype, amax_slot=None, split=True):
    """``amax_slot``: a zeroed operand-max slot for the folded weights (callers folding a whole
    model hand out slices of one zeroed buffer: one fill per fold, not one per conv).
    ``split`` False: the caller splits the folded weights itself (:func:`split_weights_batch`)."""
    assert w.dtype == torch.float32 and _inner_contig(w)
    if out_dtype != _F32:
        raise TypeError(f"bn_fold: fp32 weights only (got {out_dtype})")
    slots, Cout = w.shape[0], w.shape[1]
    K = int(torch.tensor(w.shape[2:]).prod())
    ss = _same_stride(gamma, beta, rmean, rvar)
    wf = torch.empty(w.shape, dtype=out_dtype, device=w.device)
    bf = torch.empty(slots, Cout, dtype=torch.float32, device=w.device)
    cb = None
    if conv_bias is not None:
        cb = conv_bias
        assert _same_stride(cb) == ss
    am = amax_slot if amax_slot is not None else _amax_new(slots, w.device)
    assert am.shape[0] == AMAX_SUB and am.shape[1] >= slots
    _call("dba_bn_fold", w.data_ptr(), w.stride(0), _ptr(cb), gamma.data_ptr(), beta.data_ptr(), rmean.data_ptr(),
          rvar.data_ptr(), ss, float(eps), wf.data_ptr(), bf.data_ptr(), slots, Cout, K, int(out_dtype == _F32),
          am.data_ptr(), am.shape[1], _stream())
    wf._dba_amax = am   # the folded weights' scale (max |wf| folded by the fold kernel), once per fold
    if split:
        split_weights(wf, Cout * K, Cout * K, wf._dba_amax)   # and their fp16 planes
    return wf, bf


def bn_fold_batch(items, eps: float):
    """:func:`bn_fold` (no conv bias, fp32) of ``items = [(w, gamma, beta, rmean, rvar,
    amax_slot)]`` of one model bank in one launch (per 24), max |w'| folded into each zeroed
    slot; returns ``[(wf, bf)]`` (planes not split: :func:`split_weights_batch`)."""
    if not items:
        return []
    slots = items[0][0].shape[0]
    desc, outs = [], []
    for w, gamma, beta, rmean, rvar, am in items:
        assert w.dtype == torch.float32 and _inner_contig(w) and w.shape[0] == slots
        Cout = w.shape[1]
        K = int(torch.tensor(w.shape[2:]).prod())
        ss = _same_stride(gamma, beta, rmean, rvar)
        assert am.shape[0] == AMAX_SUB and am.shape[1] >= slots
        wf = torch.empty(w.shape, dtype=_F32, device=w.device)
        bf = torch.empty(slots, Cout, dtype=torch.float32, device=w.device)
        desc.append([w.data_ptr(), w.stride(0), gamma.data_ptr(), beta.data_ptr(), rmean.data_ptr(), rvar.data_ptr(),
                     ss, wf.data_ptr(), bf.data_ptr(), Cout, K, am.data_ptr(), am.shape[1], 0])
        wf._dba_amax = am
        outs.append((wf, bf))
    d = torch.tensor(desc, dtype=torch.int64)   # host table, passed by value
    _call("dba_bn_fold_batch", d.data_ptr(), len(items), slots, float(eps), _stream())
    return outs


# --------------------------------------------------------------------------- pooling
def maxpool2d(x, k, s, p, want_ind=True):
    """``want_ind`` False (evaluation): no argmax indices are stored (returns (y, None))."""
    x = _act(x, None, "maxpool input")
    G, N, H, W, C = x.shape
    Ho = (H + 2 * p - k) // s + 1
    Wo = (W + 2 * p - k) // s + 1
    y = torch.empty(G, N, Ho, Wo, C, dtype=x.dtype, device=x.device)
    ind = torch.empty(G, N, Ho, Wo, C, dtype=torch.int32, device=x.device) if want_ind else None
    _call("dba_maxpool", x.data_ptr(), y.data_ptr(), _ptr(ind), G * N, H, W, C, Ho, Wo, k, s, p, _f32(x),
          _stream())
    return y, ind


def maxpool2d_bwd(dy, ind, in_shape, k, s, p):
    dy = _act(dy, None, "maxpool dy")
    G, N, H, W, C = in_shape
    Ho, Wo = dy.shape[2], dy.shape[3]
    dx = torch.empty(G, N, H, W, C, dtype=dy.dtype, device=dy.device)
    _call("dba_maxpool_bwd", dy.data_ptr(), ind.data_ptr(), dx.data_ptr(), G * N, H, W, C, Ho, Wo, k, s, p, _f32(dy),
          _stream())
    return dx


def avgpool_global(x):
    x = _act(x, None, "avgpool input")
    G, N, H, W, C = x.shape
    y = torch.empty(G, N, 1, 1, C, dtype=x.dtype, device=x.device)
    _call("dba_avgpool", x.data_ptr(), y.data_ptr(), G * N, H * W, C, _f32(x), _stream())
    return y


def avgpool_global_bwd(dy, hw):
    dy = _act(dy, None, "avgpool dy")
    G, N = dy.shape[:2]
    C = dy.shape[-1]
    H, W = hw
    dx = torch.empty(G, N, H, W, C, dtype=dy.dtype, device=dy.device)
    _call("dba_avgpool_bwd", dy.data_ptr(), dx.data_ptr(), G * N, H * W, C, _f32(dy), _stream())
    return dx


# --------------------------------------------------------------------------- dropout
def dropout(x, p, seeds, salt):
    x = _act(x, None, "dropout input")
    y = torch.empty_like(x)
    G = x.shape[0]
    _call("dba_dropout", x.data_ptr(), y.data_ptr(), _f32(x), _i32(seeds).data_ptr(),
          int(salt) & 0xFFFFFFFF, float(p), x.numel() // G, G, _stream())
    return y


def dropout_bwd(dy, p, seeds, salt):
    return dropout(dy, p, seeds, salt)


# ---------------------------------------------------------------------------- loss
def softmax_xent(logits, labels, mean, want_grad, stats=None, slot=None, nvalid=None, grad_dtype=None,
                 loss_dtype=None):
    """``grad_dtype``: dtype of dlogits (fp32, the compute dtype of the backward pass).  ``loss_dtype`` fp64 returns the per-group loss unrounded (evaluation sums)."""
    if logits.dtype != _F32:
        raise TypeError("softmax_xent: logits must be fp32 (the final layer emits fp32)")
    lf = logits.contiguous()
    G, B, C = lf.shape
    gdt = grad_dtype or _F32
    if gdt != _F32:
        raise TypeError(f"softmax_xent: unsupported grad dtype {gdt}")
    loss = torch.empty(G, dtype=torch.float32, device=lf.device)
    loss64 = torch.empty(G, dtype=torch.float64, device=lf.device) if loss_dtype == torch.float64 else None
    correct = torch.empty(G, dtype=torch.float32, device=lf.device)
    dl = torch.empty(G, B, C, dtype=gdt, device=lf.device) if want_grad else None
    sp, ss, slp, ms, nvp = None, 0, None, 0, None
    if stats is not None:
        assert stats.dtype == torch.float32 and stats.is_contiguous() and stats.shape[0] == 3
        ms = stats.shape[1] // G
        assert ms * G == stats.shape[1]
        slot_, nv_ = _i32(slot), _i32(nvalid)
        sp, ss, slp, nvp = stats.data_ptr(), stats.shape[1], slot_.data_ptr(), nv_.data_ptr()
    npart = int(_L.dba_softmax_xent_part_doubles(G, B))   # large groups: 32-row slices, one block each
    part = torch.empty(npart, dtype=torch.float64, device=lf.device) if npart > 0 else None
    _call("dba_softmax_xent", lf.data_ptr(), _i32(labels).data_ptr(), G, B, C, int(bool(mean)), _ptr(dl),
          loss.data_ptr(), correct.data_ptr(), sp, ss, slp, ms, nvp, int(gdt == _F32), _ptr(loss64), _ptr(part),
          _stream())
    return (loss64 if loss64 is not None else loss), correct, dl


_FUSED_HEAD = os.environ.get("DBA_FUSED_HEAD", "0") == "1"


def head_ok(x, w) -> bool:
    """The fused classifier head (loss.hip head_rows_kernel) takes this training head: fp32 last
    block output [G, N, H, W, C] (C <= 512, N <= 256, H * W <= 64) and a linear layer of <= 16 classes.
    Opt-in (``DBA_FUSED_HEAD=1``): its logits are fp32 FMA chains, not the fp16-pair MFMA of the
    unfused 1x1 conv, so a step's bits differ from the default path's."""
    return (_FUSED_HEAD and x.dtype == _F32 and x.dim() == 5 and x.shape[-1] <= 512 and x.shape[-1] % 4 == 0 and x.shape[1] <= 256
            and x.shape[2] * x.shape[3] <= 64
            and w.dim() == 3 and w.shape[1] <= 16 and w.shape[2] == x.shape[-1] and w.dtype == _F32
            and w.stride(2) == 1 and w.stride(1) == w.shape[2])


def head_train(x, w, b, labels, nvalid, dw, db, stats=None, slot=None, mean=True):
    """The training head in two launches (loss.hip head_rows_kernel / head_fin_kernel): pooled = avgpool(x), logits =
    pooled W^T + b, softmax cross-entropy (mean over valid rows) + correct count (+ ``stats``
    slots), and its backward: ``dw`` / ``db`` overwritten for the active replicas, the pooled
    features' gradient returned.  Returns (loss [G], correct [G], dpool [G, N, 1, 1, C])."""
    x = _act(x, _F32, "head input")
    G, N, H, W_, C = x.shape
    K = w.shape[1]
    assert head_ok(x, w) and b.stride(-1) == 1 and dw.stride(-1) == 1 and db.stride(-1) == 1
    pooled = torch.empty(G, N, C, dtype=_F32, device=x.device)
    dlog = torch.empty(G, N, 16, dtype=_F32, device=x.device)
    part = torch.empty(int(_L.dba_head_part_doubles(G, N)), dtype=torch.float64, device=x.device)
    dpool = torch.empty(G, N, 1, 1, C, dtype=_F32, device=x.device)
    loss = torch.empty(G, dtype=_F32, device=x.device)
    correct = torch.empty(G, dtype=_F32, device=x.device)
    sp, ss, slp, ms = None, 0, None, 0
    if stats is not None:
        ms = stats.shape[1] // G
        sp, ss, slp = stats.data_ptr(), stats.shape[1], _i32(slot).data_ptr()
    rc = _call("dba_head_train", x.data_ptr(), x.stride(0), G, N, H * W_, C, w.data_ptr(), w.stride(0), b.data_ptr(),
               b.stride(0), K, _i32(labels).data_ptr(), _ptr(_i32(nvalid)), pooled.data_ptr(), dlog.data_ptr(),
               part.data_ptr(), dw.data_ptr(),
               dw.stride(0), db.data_ptr(), db.stride(0), dpool.data_ptr(), loss.data_ptr(), correct.data_ptr(), sp, ss,
               slp, ms, int(bool(mean)), _stream())
    if rc == NOT_HANDLED:
        raise RuntimeError("head_train declined a shape head_ok accepted")
    return loss, correct, dpool


# ------------------------------------------------------------------------- optimizer
def sgd_step(params, grads, mom, lr, first, active, momentum, wd, fg_accum=None):
    G, P = grads.shape
    assert params.dtype == torch.float32 and params.stride(1) == 1 and params.stride(0) % 4 == 0
    assert grads.is_contiguous() and mom.is_contiguous() and P % 4 == 0
    _call("dba_sgd_step", params.data_ptr(), params.stride(0), grads.data_ptr(), mom.data_ptr(),
          lr.float().contiguous().data_ptr(), _i32(first).data_ptr(), _i32(active).data_ptr(), float(momentum),
          float(wd), _ptr(fg_accum), G, P, _stream())


def dist_loss_grad(w, base, grads, trig, active, alpha):
    G, P = grads.shape
    assert w.dtype == torch.float32 and w.stride(1) == 1 and base.stride(1) == 1 and grads.is_contiguous()
    assert w.shape[0] >= G and base.shape[0] >= G and w.shape[1] >= P and base.shape[1] >= P
    nrm2 = torch.zeros(G, dtype=torch.float32, device=grads.device)
    part = torch.empty(G, 256, dtype=torch.float32, device=grads.device)
    _call("dba_dist_loss_grad", w.data_ptr(), w.stride(0), base.data_ptr(), base.stride(0), grads.data_ptr(), P, G,
          _i32(trig).data_ptr(), _i32(active).data_ptr(), float(alpha), nrm2.data_ptr(), part.data_ptr(), _stream())
    return nrm2.sqrt()


# ---------------------------------------------------------------- flat / aggregation
def scale_from_base(w, base, gamma):
    w = w.contiguous()
    base = base.contiguous()
    out = torch.empty_like(w)
    _call("dba_scale_from_base", w.data_ptr(), base.data_ptr(), float(gamma), out.data_ptr(), w.numel(), _stream())
    return out


def add_noise_scaled(dst, upd, coef, sigma, seed, noise):
    assert dst.is_contiguous() and dst.dtype == torch.float32
    if upd.dtype not in (torch.float32, torch.float64):
        upd = upd.float()
    upd = upd.contiguous()
    _call("dba_add_noise_scaled", dst.data_ptr(), upd.data_ptr(), dst.numel(), float(coef), float(sigma),
          int(seed) & 0xFFFFFFFF, int(bool(noise)), int(upd.dtype == torch.float64), _stream())


def delta_sum(rows, base):
    assert rows.dtype == torch.float32 and base.dtype == torch.float32
    n = base.numel()
    out = torch.empty(n, dtype=torch.float64, device=base.device)
    if rows.shape[0] == 0:
        out.zero_()
        return out
    assert rows.stride(-1) == 1 and rows.shape[1] >= n
    base = base.contiguous()
    _call("dba_delta_sum", rows.data_ptr(), rows.stride(0), rows.shape[0], base.data_ptr(), n, out.data_ptr(),
          _stream())
    return out


def sq_dists(points, m):
    assert points.stride(1) == 1 and points.dtype == torch.float32
    m = m.float().contiguous()
    n, L = points.shape
    out = torch.empty(n, dtype=torch.float64, device=points.device)
    part = torch.empty(n * int(_L.dba_sqdist_blocks(L)), dtype=torch.float64, device=points.device)
    _call("dba_sq_dists", points.data_ptr(), points.stride(0), m.data_ptr(), n, L, out.data_ptr(), part.data_ptr(),
          _stream())
    return out


def weighted_sum(points, wts, out_dtype=None):
    assert points.stride(1) == 1 and points.dtype == torch.float32
    odt = out_dtype or torch.float32
    n, L = points.shape
    out = torch.empty(L, dtype=odt, device=points.device)
    _call("dba_weighted_sum", points.data_ptr(), points.stride(0), wts.float().contiguous().data_ptr(), n,
          out.data_ptr(), L, int(odt == torch.float64), _stream())
    return out


def weighted_sum_fixed(points, wts, E):
    """[2, L] int64 fixed-point limb sums of sum_i wts[i] * points[i] at scale 2^E (flat.hip
    wsum_fixed_kernel): order-free, so rank partials all-reduce to world-invariant bits."""
    assert points.stride(1) == 1 and points.dtype == torch.float32
    n, L = points.shape
    out = torch.empty(2, L, dtype=torch.int64, device=points.device)
    _call("dba_weighted_sum_fixed", points.data_ptr(), points.stride(0), wts.float().contiguous().data_ptr(), n,
          out.data_ptr(), L, float(2.0 ** E), _stream())
    return out


def gram(feats):
    f = feats.float()
    if f.stride(1) != 1:
        f = f.contiguous()
    n, d = f.shape
    out = torch.empty(n, n, dtype=torch.float64, device=f.device)
    slab = torch.empty(int(_L.dba_gram_chunks(d)) * n * n, dtype=torch.float32, device=f.device)
    _call("dba_gram", f.data_ptr(), f.stride(0), n, d, out.data_ptr(), slab.data_ptr(), _stream())
    return out
