"""ctypes bindings of the native host runtime (``csrc/runtime/runtime.cpp``).

The shared object is built in-tree (``dba_mod_amd/_lib/libdba_runtime.so``) by
:func:`dba_mod_amd.ops.build.build_runtime`; if it is missing it is built on first use
(g++ is part of the image on every box).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Any, List, Sequence, Tuple

import numpy as np

_LIB = None
_LOCK = threading.Lock()
_I64P = ctypes.POINTER(ctypes.c_int64)
_I32P = ctypes.POINTER(ctypes.c_int32)
_U32P = ctypes.POINTER(ctypes.c_uint32)
_F32P = ctypes.POINTER(ctypes.c_float)
_F64P = ctypes.POINTER(ctypes.c_double)


def lib():
    global _LIB
    if _LIB is None:
        with _LOCK:
            if _LIB is None:
                from ..ops import build
                path = build.runtime_path()
                if not os.path.exists(path) or build.runtime_stale():
                    build.build_runtime()
                L = ctypes.CDLL(path)
                L.dba_pack_steps.restype = ctypes.c_int
                L.dba_pack_steps.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             _I64P, _I64P, _I32P, _I32P, _I32P, _I32P, _I32P, _F32P,
                                             _U32P, _I32P]
                L.dba_lpt_assign.restype = None
                L.dba_lpt_assign.argtypes = [ctypes.c_int, _F64P, ctypes.c_int, _I32P, _F64P]
                L.dba_shard_index.restype = ctypes.c_int64
                L.dba_shard_index.argtypes = [_I64P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _I64P]
                L.dba_balance_shares.restype = None
                L.dba_balance_shares.argtypes = [ctypes.c_int, _F64P, ctypes.c_double, _F64P]
                L.dba_hash2.restype = ctypes.c_uint32
                L.dba_hash2.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
                _LIB = L
    return _LIB


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


def pack_steps(clients: Sequence[Any], G: int, B: int, T: int, max_slots: int) -> np.ndarray:
    """Packed [T, G*B + 8G] int32 step-descriptor table for the grouped trainer."""
    steps = [s for c in clients for s in c.steps]
    n_steps = np.array([len(c.steps) for c in clients], dtype=np.int64)
    step_off = np.zeros(G + 1, dtype=np.int64)
    step_off[1:] = np.cumsum(n_steps)
    lens = np.array([len(s.idx) for s in steps], dtype=np.int64)
    idx_off = np.zeros(len(steps) + 1, dtype=np.int64)
    idx_off[1:] = np.cumsum(lens)
    idx_flat = (np.concatenate([s.idx for s in steps]).astype(np.int32) if steps
                else np.zeros(1, dtype=np.int32))
    pn = np.array([s.poison_n for s in steps] or [0], dtype=np.int32)
    trig = np.array([s.trig for s in steps] or [0], dtype=np.int32)
    first = np.array([int(s.first) for s in steps] or [0], dtype=np.int32)
    slot = np.array([s.slot for s in steps] or [0], dtype=np.int32)
    lr = np.array([s.lr for s in steps] or [0], dtype=np.float32)
    seeds = np.array([c.seed for c in clients], dtype=np.uint32)
    D = G * B + 8 * G
    out = np.empty((max(T, 1), D), dtype=np.int32)
    rc = lib().dba_pack_steps(G, B, T, max_slots, _p(step_off, _I64P), _p(idx_off, _I64P),
                              _p(idx_flat, _I32P), _p(pn, _I32P), _p(trig, _I32P), _p(first, _I32P),
                              _p(slot, _I32P), _p(lr, _F32P), _p(seeds, _U32P), _p(out, _I32P))
    if rc != 0:
        raise RuntimeError(f"dba_pack_steps failed ({rc})")
    return out[:T]


def lpt_assign(costs: Sequence[float], world: int) -> Tuple[List[int], List[float]]:
    c = np.asarray(costs, dtype=np.float64)
    owner = np.zeros(len(c), dtype=np.int32)
    load = np.zeros(world, dtype=np.float64)
    lib().dba_lpt_assign(len(c), _p(c, _F64P), world, _p(owner, _I32P), _p(load, _F64P))
    return owner.tolist(), load.tolist()


def shard_index(idx: np.ndarray, rank: int, world: int) -> np.ndarray:
    a = np.ascontiguousarray(idx, dtype=np.int64)
    out = np.empty(max(1, (a.shape[0] + world - 1) // world), dtype=np.int64)
    k = lib().dba_shard_index(_p(a, _I64P), a.shape[0], rank, world, _p(out, _I64P))
    return out[:k]


def balance_shares(base: Sequence[float], work: float) -> List[float]:
    """Water-filling shares of ``work`` over ranks already loaded with ``base`` (same units):
    the least-loaded ranks take the work first, shares sum to 1 (runtime.cpp)."""
    b = np.ascontiguousarray(base, dtype=np.float64)
    out = np.zeros(b.shape[0], dtype=np.float64)
    lib().dba_balance_shares(int(b.shape[0]), _p(b, _F64P), float(work), _p(out, _F64P))
    return out.tolist()


def share_range(n: int, shares: Sequence[float], rank: int) -> Tuple[int, int]:
    """[lo, hi) of an n-element list owned by ``rank`` under ``shares`` (contiguous blocks,
    boundaries floor(n * cumulative share), the last one n): every rank computes the same
    boundaries, so the blocks tile the list exactly."""
    cum = np.concatenate([[0.0], np.cumsum(np.asarray(shares, dtype=np.float64))])
    edges = np.minimum(np.floor(cum * n).astype(np.int64), n)
    edges[-1] = n
    return int(edges[rank]), int(edges[rank + 1])


def hash2(seed: int, counter: int) -> int:
    return int(lib().dba_hash2(seed & 0xFFFFFFFF, counter & 0xFFFFFFFF))
