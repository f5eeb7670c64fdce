"""Readers for the real datasets when their files are present under ``data_dir``.

Layouts follow what the reference expects on disk:

* MNIST: torchvision's raw idx files ``{data_dir}/MNIST/raw/{train,t10k}-images-idx3-ubyte[.gz]``
  (reference ``image_helper.py:191-201``).
* CIFAR-10: the *binary* distribution ``{data_dir}/cifar-10-batches-bin/data_batch_{1..5}.bin``
  / ``test_batch.bin`` (3073-byte records; no pickle is ever loaded).
* Tiny-ImageNet: ``{data_dir}/tiny-imagenet-200/{train,val}/<wnid>/**.JPEG`` after the
  reference's ``tinyimagenet_reformat.py``; classes sorted like ``ImageFolder``.
* LOAN: ``{data_dir}/loan/loan_<ST>.csv`` written by ``loan_preprocess.py``; label column
  ``loan_status``; per-state ``train_test_split(test_size=0.2, random_state=42)``
  (``loan_helper.py:148-181``).  Files are sorted by name (quirk D10: the reference used the
  unsorted ``os.listdir`` order).
"""
from __future__ import annotations

import gzip
import os
from typing import List, Optional, Tuple

import numpy as np

from .synthetic import ImageDataset, TabularDataset


def _open_maybe_gz(path: str):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    raise FileNotFoundError(path)


def _read_idx(path: str) -> np.ndarray:
    with _open_maybe_gz(path) as f:
        raw = f.read()
    magic = int.from_bytes(raw[0:4], "big")
    ndim = magic & 0xFF
    dims = [int.from_bytes(raw[4 + 4 * i: 8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(raw, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def mnist_available(data_dir: str) -> bool:
    p = os.path.join(data_dir, "MNIST", "raw", "train-images-idx3-ubyte")
    return os.path.exists(p) or os.path.exists(p + ".gz")


def read_mnist(data_dir: str) -> Tuple[ImageDataset, ImageDataset]:
    raw = os.path.join(data_dir, "MNIST", "raw")
    out = []
    for split, pref in (("train", "train"), ("test", "t10k")):
        x = _read_idx(os.path.join(raw, f"{pref}-images-idx3-ubyte"))
        y = _read_idx(os.path.join(raw, f"{pref}-labels-idx1-ubyte")).astype(np.int64)
        out.append(ImageDataset(np.ascontiguousarray(x[..., None]), y, 10, f"mnist-{split}"))
    return out[0], out[1]


def cifar_available(data_dir: str) -> bool:
    return os.path.exists(os.path.join(data_dir, "cifar-10-batches-bin", "test_batch.bin"))


def _read_cifar_bin(paths: List[str]) -> Tuple[np.ndarray, np.ndarray]:
    recs = [np.fromfile(p, dtype=np.uint8).reshape(-1, 3073) for p in paths]
    r = np.concatenate(recs)
    y = r[:, 0].astype(np.int64)
    x = r[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    return np.ascontiguousarray(x), y


def read_cifar(data_dir: str) -> Tuple[ImageDataset, ImageDataset]:
    base = os.path.join(data_dir, "cifar-10-batches-bin")
    xtr, ytr = _read_cifar_bin([os.path.join(base, f"data_batch_{i}.bin") for i in range(1, 6)])
    xte, yte = _read_cifar_bin([os.path.join(base, "test_batch.bin")])
    return ImageDataset(xtr, ytr, 10, "cifar-train"), ImageDataset(xte, yte, 10, "cifar-test")


def tiny_available(data_dir: str) -> bool:
    return os.path.isdir(os.path.join(data_dir, "tiny-imagenet-200", "train"))


def _read_image_folder(root: str, classes: Optional[List[str]] = None) -> Tuple[np.ndarray, np.ndarray, List[str]]:
    from PIL import Image  # PIL is in the image; only needed for real Tiny-ImageNet
    if classes is None:
        classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
    xs, ys = [], []
    exts = (".jpeg", ".jpg", ".png")
    for ci, c in enumerate(classes):
        cdir = os.path.join(root, c)
        if not os.path.isdir(cdir):
            continue
        files = []
        for dp, _, fns in os.walk(cdir):
            files.extend(os.path.join(dp, fn) for fn in fns if fn.lower().endswith(exts))
        for fp in sorted(files):
            with Image.open(fp) as im:
                xs.append(np.asarray(im.convert("RGB"), dtype=np.uint8))
            ys.append(ci)
    return np.stack(xs), np.asarray(ys, dtype=np.int64), classes


def read_tiny(data_dir: str) -> Tuple[ImageDataset, ImageDataset]:
    base = os.path.join(data_dir, "tiny-imagenet-200")
    xtr, ytr, classes = _read_image_folder(os.path.join(base, "train"))
    xte, yte, _ = _read_image_folder(os.path.join(base, "val"), classes)
    return (ImageDataset(xtr, ytr, len(classes), "tiny-train"),
            ImageDataset(xte, yte, len(classes), "tiny-test"))


def loan_available(data_dir: str) -> bool:
    d = os.path.join(data_dir, "loan")
    return os.path.isdir(d) and any(f.endswith(".csv") for f in os.listdir(d))


def read_loan(data_dir: str) -> List[TabularDataset]:
    import pandas as pd
    from sklearn.model_selection import train_test_split
    d = os.path.join(data_dir, "loan")
    out: List[TabularDataset] = []
    for fn in sorted(f for f in os.listdir(d) if f.endswith(".csv")):
        df = pd.read_csv(os.path.join(d, fn))
        feats = [c for c in df.columns if c != "loan_status"]
        x = df[feats]
        y = df["loan_status"].astype("int")
        xtr, xte, ytr, yte = train_test_split(x, y, test_size=0.2, random_state=42)
        out.append(TabularDataset(fn[5:7], xtr.values.astype(np.float32), ytr.values.astype(np.int64),
                                  xte.values.astype(np.float32), yte.values.astype(np.int64),
                                  list(xtr.columns)))
    return out
