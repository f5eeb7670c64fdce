"""Workload construction: datasets, client partition, name lists, triggers, test subsets.

Equivalent of the reference's ``ImageHelper.load_data`` / ``LoanHelper.load_data``
(``image_helper.py:173-250``, ``loan_helper.py:111-145``), re-designed around device-resident
data: every client is an index array into one HBM-resident training set.
"""
from __future__ import annotations

import logging
import random
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from .. import config as C
from ..data import partition, readers, synthetic
from ..data.store import DeviceImages, DeviceRows, feature_trigger_bank, pixel_trigger_bank
from ..models.spec import ModelSpec, arch_for_type, get_spec

log = logging.getLogger("logger")


@dataclass
class Workload:
    params: C.Params
    spec: ModelSpec
    device: torch.device
    kind: str                                  # 'image' | 'tabular'
    train_store: Any                           # DeviceImages | DeviceRows
    test_store: Any
    client_indices: Dict[Any, np.ndarray]      # client name -> train indices (int64)
    participants_list: List[Any]
    benign_namelist: List[Any]
    adversarial_namelist: List[Any]
    test_clean_idx: np.ndarray                 # all test indices
    test_poison_idx: np.ndarray                # test indices with label != target
    trig_masks: torch.Tensor                   # image: [T, H, W] uint8; T = trigger_num + 1
    trig_cols: torch.Tensor                    # tabular: [T, K]
    trig_vals: torch.Tensor
    py_rng: random.Random                      # reference's python `random` stream
    np_rng: np.random.RandomState
    flip_train: bool = False                   # Tiny: RandomHorizontalFlip on train
    synthetic: bool = True
    feature_index: Dict[str, int] = field(default_factory=dict)
    client_sizes: Dict[Any, int] = field(default_factory=dict)

    @property
    def global_trigger_id(self) -> int:
        """Trigger-bank slot of the global (union) trigger."""
        return int(self.params["trigger_num"])

    def trigger_id(self, adv_index: int) -> int:
        """Bank slot for an adversarial index (-1 = global trigger)."""
        return self.global_trigger_id if adv_index == -1 else int(adv_index)


def _use_synthetic(params: C.Params, available: bool) -> bool:
    s = params["synthetic_data"]
    if s == "auto":
        return not available
    return bool(s)


def build_workload(params: C.Params, device: torch.device) -> Workload:
    seed = int(params["seed"])
    py_rng = random.Random(seed)
    np_rng = np.random.RandomState(seed)
    t = params.type
    spec = get_spec(arch_for_type(t, params["model_arch"]))
    data_dir = params["data_dir"]
    if t == C.TYPE_LOAN:
        return _build_loan(params, spec, device, py_rng, np_rng, data_dir)

    avail = {C.TYPE_MNIST: readers.mnist_available, C.TYPE_CIFAR: readers.cifar_available,
             C.TYPE_TINYIMAGENET: readers.tiny_available}[t](data_dir)
    synth = _use_synthetic(params, avail)
    if synth:
        train, test = synthetic.synthetic_image_pair(t, seed=seed, train_size=params["synthetic_train_size"],
                                                     test_size=params["synthetic_test_size"],
                                                     noise=params["synthetic_noise"],
                                                     shared=params["synthetic_shared"],
                                                     clutter=params["synthetic_clutter"],
                                                     sky=params["synthetic_sky"],
                                                     margin=params["synthetic_margin"],
                                                     sky_rows=params["synthetic_sky_rows"],
                                                     contrast=params["synthetic_contrast"])
    else:
        train, test = {C.TYPE_MNIST: readers.read_mnist, C.TYPE_CIFAR: readers.read_cifar,
                       C.TYPE_TINYIMAGENET: readers.read_tiny}[t](data_dir)
    log.info(f"data: {'synthetic' if synth else 'real'} {t} train={len(train)} test={len(test)}")

    n_total = int(params["number_of_total_participants"])
    if params["sampling_dirichlet"]:
        per = partition.sample_dirichlet(train.labels, n_total, float(params["dirichlet_alpha"]), py_rng, np_rng)
        client_indices = {pos: np.asarray(per.get(pos, []), dtype=np.int64) for pos in range(n_total)}
    else:
        per = partition.equal_split(len(train), n_total, py_rng)
        client_indices = {pos: np.asarray(v, dtype=np.int64) for pos, v in per.items()}

    adversaries = params.adversary_list
    if params["is_random_namelist"]:
        participants = list(range(n_total))
    else:
        participants = list(params["participants_namelist"])
    benign = sorted(set(participants) - set(adversaries))  # D10: explicit order

    h, w, _ = train.shape
    patterns = [params.poison_pattern(i) for i in range(int(params["trigger_num"]))]
    patterns.append(params.poison_pattern(-1))
    masks = pixel_trigger_bank(patterns, h, w)

    target = int(params["poison_label_swap"])
    wl = Workload(
        params=params, spec=spec, device=device, kind="image",
        train_store=DeviceImages.from_numpy(train.images, train.labels, device),
        test_store=DeviceImages.from_numpy(test.images, test.labels, device),
        client_indices=client_indices, participants_list=participants, benign_namelist=benign,
        adversarial_namelist=list(adversaries),
        test_clean_idx=np.arange(len(test), dtype=np.int64),
        test_poison_idx=partition.poison_test_indices(test.labels, target),
        trig_masks=torch.from_numpy(masks).to(device),
        trig_cols=torch.zeros(1, 1, dtype=torch.int32, device=device),
        trig_vals=torch.zeros(1, 1, dtype=torch.float32, device=device),
        py_rng=py_rng, np_rng=np_rng, flip_train=(t == C.TYPE_TINYIMAGENET), synthetic=synth)
    wl.client_sizes = {k: int(v.shape[0]) for k, v in client_indices.items()}
    return wl


def _build_loan(params: C.Params, spec: ModelSpec, device: torch.device, py_rng: random.Random,
                np_rng: np.random.RandomState, data_dir: str) -> Workload:
    synth = _use_synthetic(params, readers.loan_available(data_dir))
    rows = params["synthetic_loan_rows"]
    if rows is None and params["synthetic_train_size"] is not None:   # small test / smoke runs
        rows = int(params["synthetic_train_size"]) * 5 // 4
    states = (synthetic.synthetic_loan(seed=int(params["seed"]),
                                       **({"total_rows": int(rows)} if rows is not None else {}))
              if synth else readers.read_loan(data_dir))
    feature_index = {name: k for k, name in enumerate(states[0].columns)}
    tr_x, tr_y, te_x, te_y = [], [], [], []
    client_indices: Dict[Any, np.ndarray] = {}
    off = 0
    for st in states:
        n = st.train_x.shape[0]
        client_indices[st.name] = np.arange(off, off + n, dtype=np.int64)
        off += n
        tr_x.append(st.train_x)
        tr_y.append(st.train_y)
        te_x.append(st.test_x)
        te_y.append(st.test_y)
    adversaries = [str(a) for a in params.adversary_list]
    names = [st.name for st in states]
    n_total = int(params["number_of_total_participants"])
    benign = [s for s in names[:n_total] if s not in adversaries]
    if params["is_random_namelist"]:
        participants = benign + adversaries          # loan_helper.py:145
    else:
        participants = [str(s) for s in params["participants_namelist"]]
    test_y = np.concatenate(te_y)
    triggers = [params.trigger_features(i) for i in range(int(params["trigger_num"]))]
    triggers.append(params.trigger_features(-1))
    cols, vals = feature_trigger_bank(triggers, feature_index)
    target = int(params["poison_label_swap"])
    wl = Workload(
        params=params, spec=spec, device=device, kind="tabular",
        train_store=DeviceRows.from_numpy(np.concatenate(tr_x), np.concatenate(tr_y), device),
        test_store=DeviceRows.from_numpy(np.concatenate(te_x), test_y, device),
        client_indices=client_indices, participants_list=participants, benign_namelist=benign,
        adversarial_namelist=adversaries,
        test_clean_idx=np.arange(test_y.shape[0], dtype=np.int64),
        # LOAN poison tests run over ALL test rows (test.py:62-81 relabels every row)
        test_poison_idx=np.arange(test_y.shape[0], dtype=np.int64),
        trig_masks=torch.zeros(1, 1, 1, dtype=torch.uint8, device=device),
        trig_cols=torch.from_numpy(cols).to(device), trig_vals=torch.from_numpy(vals).to(device),
        py_rng=py_rng, np_rng=np_rng, synthetic=synth, feature_index=feature_index)
    wl.client_sizes = {k: int(v.shape[0]) for k, v in client_indices.items()}
    log.info(f"data: {'synthetic' if synth else 'real'} loan states={len(states)} "
             f"train={off} test={test_y.shape[0]}")
    return wl
