"""Synthetic datasets with the reference workloads' exact shapes and class sizes.

There is no network in this environment, so the torchvision downloads of the reference
(``image_helper.py:176-220``) and the Kaggle LendingClub CSVs (``utils/process_loan_data.sh``)
cannot be fetched.  These generators produce *learnable* stand-ins:

* every class owns a smooth random template (low-frequency field, per-channel tint);
* every image is its class template, randomly shifted by a few pixels, contrast-jittered
  and corrupted by pixel noise, quantised to uint8 (the reference feeds ``ToTensor``
  = uint8/255 images with no normalisation, ``image_helper.py:176-201``).

Class sizes match the real datasets so the Dirichlet partitioner reproduces the reference's
annotated shard sizes: CIFAR-10 5000/1000 per class, MNIST's real per-class
counts, Tiny-ImageNet 500/50 per class for 200 classes.

Images are stored NHWC uint8 — the device-resident layout the gather kernel reads.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

# real per-class counts of MNIST train / test (digits 0..9)
MNIST_TRAIN_COUNTS = [5923, 6742, 5958, 6131, 5842, 5421, 5918, 6265, 5851, 5949]
MNIST_TEST_COUNTS = [980, 1135, 1032, 1010, 982, 892, 958, 1028, 974, 1009]


@dataclass
class ImageDataset:
    """Host-side image dataset: uint8 NHWC images + int64 labels."""
    images: np.ndarray          # [N, H, W, C] uint8
    labels: np.ndarray          # [N] int64
    num_classes: int
    name: str = ""

    def __len__(self) -> int:
        return int(self.labels.shape[0])

    @property
    def shape(self) -> Tuple[int, int, int]:
        return tuple(self.images.shape[1:])  # type: ignore[return-value]


@dataclass
class TabularDataset:
    """One LOAN state: float features + int labels, train/test already split."""
    name: str
    train_x: np.ndarray         # [Ntr, F] float32
    train_y: np.ndarray         # [Ntr] int64
    test_x: np.ndarray
    test_y: np.ndarray
    columns: List[str] = field(default_factory=list)


def _class_order_labels(counts: List[int], rng: np.random.RandomState) -> np.ndarray:
    labels = np.concatenate([np.full(c, k, dtype=np.int64) for k, c in enumerate(counts)])
    rng.shuffle(labels)  # interleave classes like a real dataset file
    return labels


def _smooth_field(rng: np.random.RandomState, h: int, w: int, c: int, coarse: int) -> np.ndarray:
    """Low-frequency random field in [0,1] of shape [h, w, c] (bilinear upsample)."""
    g = rng.rand(coarse + 1, coarse + 1, c).astype(np.float32)
    ys = np.linspace(0, coarse, h, dtype=np.float32)
    xs = np.linspace(0, coarse, w, dtype=np.float32)
    y0 = np.floor(ys).astype(int).clip(0, coarse - 1)
    x0 = np.floor(xs).astype(int).clip(0, coarse - 1)
    fy = (ys - y0)[:, None, None]
    fx = (xs - x0)[None, :, None]
    a = g[y0][:, x0]
    b = g[y0][:, x0 + 1]
    cc = g[y0 + 1][:, x0]
    d = g[y0 + 1][:, x0 + 1]
    return (a * (1 - fy) * (1 - fx) + b * (1 - fy) * fx + cc * fy * (1 - fx) + d * fy * fx)


def _smooth_fields(rng: np.random.RandomState, n: int, h: int, w: int, c: int, coarse: int) -> np.ndarray:
    """``n`` independent low-frequency fields in [0,1], [n, h, w, c] (vectorised bilinear)."""
    g = rng.rand(n, coarse + 1, coarse + 1, c).astype(np.float32)
    ys = np.linspace(0, coarse, h, dtype=np.float32)
    xs = np.linspace(0, coarse, w, dtype=np.float32)
    y0 = np.floor(ys).astype(int).clip(0, coarse - 1)
    x0 = np.floor(xs).astype(int).clip(0, coarse - 1)
    fy = (ys - y0)[None, :, None, None]
    fx = (xs - x0)[None, None, :, None]
    a = g[:, y0][:, :, x0]
    b = g[:, y0][:, :, x0 + 1]
    cc = g[:, y0 + 1][:, :, x0]
    d = g[:, y0 + 1][:, :, x0 + 1]
    return a * (1 - fy) * (1 - fx) + b * (1 - fy) * fx + cc * fy * (1 - fx) + d * fy * fx


def make_image_dataset(counts: List[int], h: int, w: int, c: int, seed: int,
                       noise: float = 0.15, shift: int = 3, coarse: int = 4,
                       shared: float = 0.75, clutter: float = 0.0, strokes: bool = False,
                       sky: float = 0.0, sky_rows: int = 3, margin: int = 0,
                       contrast: Tuple[float, float] = (0.6, 1.2),
                       templates: Optional[np.ndarray] = None, blend: float = 0.0,
                       name: str = "") -> Tuple[ImageDataset, np.ndarray]:
    """Generate a dataset; returns (dataset, class templates) so train/test share templates.

    ``sky``: fraction of images whose top ``sky_rows`` rows fade to saturated white (row 0
    exactly 255), like the bright sky at the top of many natural photographs.  ``margin``: an
    exactly black border of that many pixels (MNIST digits are size-normalised into the central
    20 x 20 box of the 28 x 28 frame, so its 4-pixel border is always 0).  Both shape what a pixel
    trigger in the top rows competes with: a white trigger is invisible on a white sky, and a
    trigger in a border that benign data never lights is never unlearned by benign updates.
    ``blend``: fraction of AMBIGUOUS images, their class template mixed half and half with
    another class's (like the badly written digits of the real MNIST test set): an irreducible
    error of about blend / 2, so the main-task accuracy does not saturate at 100 %.  Drawn from
    a stream of its own (every other draw is unchanged)."""
    rng = np.random.RandomState(seed)
    brng = np.random.RandomState(seed * 104729 + 3) if blend > 0 else None
    k = len(counts)
    if templates is None:
        trng = np.random.RandomState(seed * 7919 + 17)
        # classes share 75% of their template: separable, but not trivially so.  Pixel noise is
        # kept moderate (like natural images, saturated pixels are rare), so a pixel trigger
        # is as salient as on the real datasets and the backdoor is learnable.
        base = _smooth_field(trng, h + 2 * shift, w + 2 * shift, c, coarse)
        templates = np.stack([shared * base + (1.0 - shared) * _smooth_field(trng, h + 2 * shift, w + 2 * shift, c, coarse)
                              for _ in range(k)]).astype(np.float32)
        if strokes:
            # MNIST-like: bright sparse structures on a black background
            templates = np.clip((templates - 0.5) * 5.0, 0.0, 1.0).astype(np.float32)
    labels = _class_order_labels(counts, rng)
    n = labels.shape[0]
    contrast_lo, contrast_hi = float(contrast[0]), float(contrast[1])
    out = np.empty((n, h, w, c), dtype=np.uint8)
    chunk = 4096
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        lab = labels[s:e]
        dy = rng.randint(0, 2 * shift + 1, size=e - s)
        dx = rng.randint(0, 2 * shift + 1, size=e - s)
        contrast = rng.uniform(contrast_lo, contrast_hi, size=(e - s, 1, 1, 1)).astype(np.float32)
        bright = rng.uniform(-0.15, 0.15, size=(e - s, 1, 1, 1)).astype(np.float32)
        imgs = np.empty((e - s, h, w, c), dtype=np.float32)
        amb = brng.rand(e - s) < blend if brng is not None else None
        other = (lab + brng.randint(1, k, size=e - s)) % k if brng is not None else None
        for i in range(e - s):
            t = templates[lab[i]]
            imgs[i] = t[dy[i]:dy[i] + h, dx[i]:dx[i] + w]
            if amb is not None and amb[i]:
                imgs[i] = 0.5 * imgs[i] + 0.5 * templates[other[i]][dy[i]:dy[i] + h, dx[i]:dx[i] + w]
        if clutter > 0:
            # per-image background content: masks the class signal the way natural-image
            # variability does (moderate margins), while staying smooth so a pixel trigger
            # remains a salient, learnable feature
            imgs = (1.0 - clutter) * imgs + clutter * _smooth_fields(rng, e - s, h, w, c, 2 * coarse)
        if strokes:
            imgs = imgs * contrast
        else:
            imgs = (imgs - 0.5) * contrast + 0.5 + bright
        imgs += rng.randn(e - s, h, w, c).astype(np.float32) * noise
        if sky > 0:
            # (drawn from the shared stream after the pixel noise: the first chunk's other draws
            # are unchanged by it, every later chunk's are not — BASELINE numbers before the
            # round-5 calibration came from different data)
            bright = rng.rand(e - s) < sky
            fade = np.maximum(0.0, 1.0 - np.arange(h, dtype=np.float32) / float(sky_rows))[None, :, None, None]
            imgs = np.where(bright[:, None, None, None], imgs + (1.0 - imgs) * fade, imgs)
        if margin > 0:
            imgs[:, :margin] = 0.0
            imgs[:, h - margin:] = 0.0
            imgs[:, :, :margin] = 0.0
            imgs[:, :, w - margin:] = 0.0
        out[s:e] = np.clip(imgs * 255.0 + 0.5, 0, 255).astype(np.uint8)
    return ImageDataset(out, labels, k, name), templates


def _scaled_counts(counts: List[int], total: Optional[int]) -> List[int]:
    if total is None:
        return list(counts)
    s = sum(counts)
    return [max(1, int(round(c * total / s))) for c in counts]


def synthetic_image_pair(kind: str, seed: int = 1, train_size: Optional[int] = None,
                         test_size: Optional[int] = None, noise: Optional[float] = None,
                         shared: Optional[float] = None, clutter: Optional[float] = None,
                         sky: Optional[float] = None, margin: Optional[int] = None,
                         sky_rows: Optional[int] = None,
                         contrast: Optional[Tuple[float, float]] = None) -> Tuple[ImageDataset, ImageDataset]:
    """(train, test) synthetic datasets for 'mnist' | 'cifar' | 'tiny-imagenet-200'.

    ``noise`` (pixel-noise sigma) and ``shared`` (template fraction common to all classes) set
    the task difficulty; ``None`` keeps the per-dataset defaults."""
    if kind == "mnist":
        tr_c, te_c, hwc = MNIST_TRAIN_COUNTS, MNIST_TEST_COUNTS, (28, 28, 1)
    elif kind == "cifar":
        tr_c, te_c, hwc = [5000] * 10, [1000] * 10, (32, 32, 3)
    elif kind == "tiny-imagenet-200":
        tr_c, te_c, hwc = [500] * 200, [50] * 200, (64, 64, 3)
    else:
        raise ValueError(kind)
    tr_c = _scaled_counts(tr_c, train_size)
    te_c = _scaled_counts(te_c, test_size)
    h, w, c = hwc
    coarse = 3 if kind == "mnist" else 4
    # Calibrated so the DBA attack window behaves like the real datasets (measured on MI355X,
    # profiles/asr_r1_synthetic_calibration.md): a warm-started global model at ~85-90% clean
    # accuracy with moderate margins, attackers reaching ~100% local ASR in their poison
    # epochs.  Low-clutter/high-noise images are separable with huge logit margins and a
    # pixel trigger then never beats the clean evidence (local ASR < 10%).
    #
    # Attack window (round 5, profiles/r5/calib/): the DBA triggers must compose the way the
    # paper's do — a single local trigger partial, the union of four near-complete — and a
    # MNIST backdoor must outlive a few benign rounds.  CIFAR: 15 % of the images have a
    # saturated white top row (bright sky), on which the row-0 local triggers are invisible, so
    # no single local trigger carries the global one (ASR 13 / 12 / 22 % after the first three
    # poison rounds, 100 % after the fourth, on two warm-start lengths; a 3-row or 30 % sky
    # kills the attack, none lets the first trigger reach 93-100 %).  MNIST: digits are
    # size-normalised into the central 20 x 20 box like the real set (a 4-pixel black border:
    # the trigger rows are never lit by benign data, so benign updates do not unlearn the
    # backdoor) and classes share half their template (smaller margins): global ASR 84-86 %
    # after round 12, 47-56 % still at round 19 (was 7 %).
    kw = {"coarse": coarse, "noise": 0.05, "shared": 0.6, "clutter": 0.5}
    if kind == "cifar":
        kw.update({"sky": 0.15, "sky_rows": 1})
    if kind == "mnist":
        # (round 6: 6 % ambiguous digits, half one class, half another — main accuracy ~97 %
        # instead of a saturated 100 %)
        kw = {"coarse": 5, "noise": 0.05, "shared": 0.5, "clutter": 0.0, "strokes": True, "shift": 2, "margin": 4,
              "blend": 0.06}
    if noise is not None:
        kw["noise"] = float(noise)
    if shared is not None:
        kw["shared"] = float(shared)
    if clutter is not None:
        kw["clutter"] = float(clutter)
    if sky is not None:
        kw["sky"] = float(sky)
    if margin is not None:
        kw["margin"] = int(margin)
    if sky_rows is not None:
        kw["sky_rows"] = int(sky_rows)
    if contrast is not None:
        kw["contrast"] = (float(contrast[0]), float(contrast[1]))
    train, tmpl = make_image_dataset(tr_c, h, w, c, seed=seed * 1000 + 1, name=f"{kind}-train", **kw)
    test, _ = make_image_dataset(te_c, h, w, c, seed=seed * 1000 + 2, templates=tmpl,
                                 name=f"{kind}-test", **kw)
    return train, test


# ---------------------------------------------------------------------------- LOAN
US_STATES = ["AK", "AL", "AR", "AZ", "CA", "CO", "CT", "DC", "DE", "FL", "GA", "HI", "IA",
             "ID", "IL", "IN", "KS", "KY", "LA", "MA", "MD", "ME", "MI", "MN", "MO", "MS",
             "MT", "NC", "ND", "NE", "NH", "NJ", "NM", "NV", "NY", "OH", "OK", "OR", "PA",
             "RI", "SC", "SD", "TN", "TX", "UT", "VA", "VT", "WA", "WI", "WV", "WY"]
# trigger features named in utils/loan_params.yaml (low/high importance sets)
LOAN_NAMED_FEATURES = ["num_tl_120dpd_2m", "num_tl_90g_dpd_24m", "pub_rec_bankruptcies",
                       "pub_rec", "acc_now_delinq", "tax_liens", "out_prncp",
                       "total_pymnt_inv", "out_prncp_inv", "total_rec_prncp",
                       "last_pymnt_amnt", "all_util"]
LOAN_COUNT_FEATURES = ["num_tl_120dpd_2m", "num_tl_90g_dpd_24m", "pub_rec_bankruptcies", "pub_rec",
                       "acc_now_delinq", "tax_liens"]
# approximate share of each state's loans in the LendingClub dump (population-like: CA, NY,
# TX, FL lead; the DBA attackers CT / MO / TN hold ~1.5 % each), in US_STATES order
LOAN_STATE_SHARE = [0.0023, 0.0123, 0.0074, 0.0240, 0.1390, 0.0217, 0.0152, 0.0024, 0.0029, 0.0718,
                    0.0325, 0.0050, 0.0001, 0.0012, 0.0399, 0.0163, 0.0083, 0.0097, 0.0113, 0.0229,
                    0.0236, 0.0018, 0.0262, 0.0180, 0.0161, 0.0054, 0.0029, 0.0280, 0.0016, 0.0033,
                    0.0049, 0.0362, 0.0054, 0.0149, 0.0829, 0.0330, 0.0090, 0.0122, 0.0340, 0.0044,
                    0.0120, 0.0021, 0.0156, 0.0822, 0.0071, 0.0280, 0.0021, 0.0212, 0.0131, 0.0037,
                    0.0022]
LENDINGCLUB_ROWS = 2_260_668
LOAN_NUM_FEATURES = 91   # reference loan_model.py:11 in_dim
LOAN_NUM_CLASSES = 9     # loan_helper.py:149-152


def loan_columns() -> List[str]:
    cols = list(LOAN_NAMED_FEATURES)
    k = 0
    while len(cols) < LOAN_NUM_FEATURES:
        cols.append(f"feat_{k:02d}")
        k += 1
    return cols


def synthetic_loan(seed: int = 1, total_rows: int = LENDINGCLUB_ROWS) -> List[TabularDataset]:
    """51 per-state tabular datasets (91 features, 9 classes), 80/20 split.

    Feature scales mimic the reference preprocessing (``loan_preprocess.py``: values
    divided down to roughly O(1-10)).  Labels come from a fixed random linear teacher so
    the task is learnable; class priors are skewed like LendingClub's.

    Size: by default the LendingClub dump's row count, split by approximate state shares
    (``LOAN_STATE_SHARE``).  The size matters to the attack: the reference recipe's
    MultiStepLR (``loan_train.py:83-92``, milestones 0.2E / 0.8E stepped at the start of each
    internal epoch) runs ONE of the 10 poison epochs at ``poison_lr`` and the rest at 1/10 and
    1/100 of it, so the attacker's trigger is learned from about 1.7 epochs' worth of
    full-rate SGD steps over its state's rows.  A 20x smaller dataset leaves it 20x fewer
    steps and the trigger unlearned (LOAN ASR 0 in every round:
    profiles/asr_r1_synthetic_calibration.md, profiles/loan_attack_r3.md).
    """
    rng = np.random.RandomState(seed * 31 + 5)
    gen = np.random.default_rng(seed * 31 + 7)      # bulk float32 draws (2.3 M x 91)
    cols = loan_columns()
    f = len(cols)
    teacher = rng.randn(f, LOAN_NUM_CLASSES).astype(np.float32)
    # delinquency / public-record counts (the DBA trigger features) are sparse, mostly-zero
    # and nearly uninformative in LendingClub data: Poisson counts with no teacher weight, so
    # a trigger writes an outlier value the clean model has no strong opinion about
    counts = [cols.index(c) for c in LOAN_COUNT_FEATURES]
    teacher[counts] = 0.0
    prior = np.log(np.array([40, 35, 3, 2, 12, 1.5, 0.5, 3, 3], dtype=np.float32))
    weights = np.array(LOAN_STATE_SHARE, dtype=np.float64)
    weights = weights / weights.sum()
    scale = rng.uniform(0.2, 3.0, size=(1, f)).astype(np.float32)
    out: List[TabularDataset] = []
    for si, st in enumerate(US_STATES):
        n = max(60, int(total_rows * weights[si]))
        x = np.abs(gen.standard_normal((n, f), dtype=np.float32))
        x *= scale
        x[:, counts] = gen.poisson(0.05, size=(n, len(counts))).astype(np.float32)
        logits = x @ teacher * 0.6 + prior + gen.standard_normal((n, LOAN_NUM_CLASSES), dtype=np.float32) * 0.5
        y = logits.argmax(1).astype(np.int64)
        perm = np.random.RandomState(42 + si).permutation(n)  # stands in for random_state=42
        n_te = int(np.ceil(n * 0.2))
        te, tr = perm[:n_te], perm[n_te:]
        out.append(TabularDataset(st, x[tr], y[tr], x[te], y[te], cols))
    return out
