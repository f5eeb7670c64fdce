"""Device-resident datasets.

The reference streams every batch through DataLoader worker processes, ``ToTensor`` and a
per-image Python trigger loop, then copies it host→device (``image_helper.py:252-263,
289-326``).  Here the whole dataset lives in HBM once (CIFAR train = 150 MB uint8, Tiny =
1.2 GB — trivial against 288 GB), clients are index arrays, and one fused kernel
(:func:`dba_mod_amd.ops.gather_images`) gathers a batch, converts uint8→compute dtype,
flips, stamps the trigger and relabels it.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch


@dataclass
class DeviceImages:
    images: torch.Tensor      # [N, H, W, C] uint8
    labels: torch.Tensor      # [N] int32

    @staticmethod
    def from_numpy(images: np.ndarray, labels: np.ndarray, device: torch.device) -> "DeviceImages":
        return DeviceImages(torch.from_numpy(np.ascontiguousarray(images)).to(device),
                            torch.from_numpy(labels.astype(np.int32)).to(device))

    def __len__(self) -> int:
        return int(self.labels.shape[0])


@dataclass
class DeviceRows:
    rows: torch.Tensor        # [N, F] float32
    labels: torch.Tensor      # [N] int32

    @staticmethod
    def from_numpy(x: np.ndarray, y: np.ndarray, device: torch.device) -> "DeviceRows":
        return DeviceRows(torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(device),
                          torch.from_numpy(y.astype(np.int32)).to(device))

    def __len__(self) -> int:
        return int(self.labels.shape[0])


def pixel_trigger_bank(patterns: List[List[List[int]]], h: int, w: int) -> np.ndarray:
    """[T, H, W] uint8 masks, one per trigger pattern ((row, col) pixel lists)."""
    bank = np.zeros((max(1, len(patterns)), h, w), dtype=np.uint8)
    for t, pat in enumerate(patterns):
        for r, c in pat:
            bank[t, int(r), int(c)] = 1
    return bank


def feature_trigger_bank(triggers: List[List[tuple]], feature_index: dict) -> tuple:
    """LOAN triggers -> ([T, K] int32 columns (-1 pad), [T, K] float32 values)."""
    k = max([len(t) for t in triggers] + [1])
    cols = -np.ones((max(1, len(triggers)), k), dtype=np.int32)
    vals = np.zeros((max(1, len(triggers)), k), dtype=np.float32)
    for ti, trig in enumerate(triggers):
        for j, (name, value) in enumerate(trig):
            cols[ti, j] = feature_index[name]
            vals[ti, j] = float(value)
    return cols, vals
