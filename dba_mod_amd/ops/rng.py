"""Counter-based hash RNG shared bit-for-bit by the HIP kernels and the torch reference.

Every random decision on the device (dropout masks, horizontal flips, DP Gaussian noise)
is a pure function of ``(seed, counter)`` so a step can be replayed inside a HIP graph and
the reference implementation reproduces the kernel exactly.  The mixer is the 32-bit
"lowbias32" integer hash; ``csrc/kernels/common.hpp`` holds the identical device version.
"""
from __future__ import annotations

import math

import torch

M32 = 0xFFFFFFFF


def hash_u32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 on an int64 tensor holding uint32 values; returns uint32 values (int64)."""
    x = x & M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & M32
    x = x ^ (x >> 16)
    return x


def hash2(seed, counter: torch.Tensor) -> torch.Tensor:
    """hash(seed, counter) = lowbias32(counter ^ lowbias32(seed)).

    ``seed``: python int or an int tensor broadcastable against ``counter``.
    """
    if not isinstance(seed, torch.Tensor):
        seed = torch.tensor(int(seed) & M32, dtype=torch.int64)
    s = hash_u32(seed.to(torch.int64).to(counter.device))
    return hash_u32((counter.to(torch.int64) & M32) ^ s)


def salted(seed, salt: int):
    """Per-launch sub-stream of a seed: (seed + salt * 0x9E3779B9) mod 2^32."""
    if isinstance(seed, torch.Tensor):
        return (seed.to(torch.int64) + int(salt) * 0x9E3779B9) & M32
    return (int(seed) + int(salt) * 0x9E3779B9) & M32


def uniform01(seed, counter: torch.Tensor) -> torch.Tensor:
    """Uniform in (0, 1): ((h >> 8) + 0.5) / 2^24, as float32."""
    h = hash2(seed, counter)
    return (((h >> 8).to(torch.float32)) + 0.5) * (1.0 / 16777216.0)


def normal(seed, counter: torch.Tensor) -> torch.Tensor:
    """Standard normal via Box-Muller on counters (2c, 2c+1)."""
    c = counter.to(torch.int64) * 2
    u1 = uniform01(seed, c)
    u2 = uniform01(seed, c + 1)
    return torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * math.pi * u2)
