"""Client data partitioning: non-IID Dirichlet and equal split.

Semantics (and RNG consumption) are kept identical to the reference so that, given the
same per-class sizes and the reference's seeds (python ``random`` and numpy both seeded
with 1, ``main.py:36-38,86``), the per-client shards — and therefore the annotated attacker
shard sizes of the YAMLs — are reproduced exactly:

* ``sample_dirichlet`` — reference ``image_helper.py:82-110``: for each class in label
  order, ``shuffle`` the class's index list with python ``random``; draw
  ``class_size * Dirichlet([alpha]*N)`` with numpy where ``class_size`` is the size of
  **class 0** for every class; client ``u`` takes ``round(p_u)`` indices from the head.
* ``equal_split`` — reference ``image_helper.py:231-236,265-280``.
* ``poison_test_indices`` — reference ``image_helper.py:148-172``: test indices whose label
  differs from the backdoor target.

Dedicated ``random.Random`` / ``numpy.random.RandomState`` objects replace the reference's
global generators; seeded identically they yield the same streams.
"""
from __future__ import annotations

import random
from collections import defaultdict
from typing import Dict, List

import numpy as np


def build_classes_dict(labels: np.ndarray) -> Dict[int, List[int]]:
    """label -> list of dataset indices in dataset order (reference image_helper.py:72-80)."""
    classes: Dict[int, List[int]] = {}
    for ind, lab in enumerate(labels.tolist()):
        classes.setdefault(int(lab), []).append(ind)
    return classes


def sample_dirichlet(labels: np.ndarray, no_participants: int, alpha: float,
                     py_rng: random.Random, np_rng: np.random.RandomState) -> Dict[int, List[int]]:
    classes = build_classes_dict(labels)
    class_size = len(classes[0])
    no_classes = len(classes.keys())
    per_participant: Dict[int, List[int]] = defaultdict(list)
    for n in range(no_classes):
        cls = classes[n]
        py_rng.shuffle(cls)
        probs = class_size * np_rng.dirichlet(np.array(no_participants * [alpha]))
        for user in range(no_participants):
            take = min(len(cls), int(round(probs[user])))
            per_participant[user].extend(cls[:take])
            cls = cls[take:]
        classes[n] = cls
    return dict(per_participant)


def equal_split(n_items: int, no_participants: int, py_rng: random.Random) -> Dict[int, List[int]]:
    all_range = list(range(n_items))
    py_rng.shuffle(all_range)
    per = n_items // no_participants
    return {pos: all_range[pos * per:(pos + 1) * per] for pos in range(no_participants)}


def poison_test_indices(test_labels: np.ndarray, target_label: int) -> np.ndarray:
    return np.nonzero(test_labels != target_label)[0].astype(np.int64)


def shard_class_histogram(labels: np.ndarray, shard: List[int], num_classes: int) -> np.ndarray:
    """Per-client class histogram (the reference's ``__main__`` self-check, image_helper.py:352-378)."""
    return np.bincount(labels[np.asarray(shard, dtype=np.int64)], minlength=num_classes)
