"""Checkpoints in the reference's layout (``helper.py:420-435``, ``image_helper.py:56-67``).

``{folder}/model_last.pt.tar`` every round (when ``save_model``), ``.epoch_{e}`` for
``e in save_on_epochs`` and ``.best`` when the tracked loss improves; payload
``{'state_dict', 'epoch', 'lr'}`` with the reference's key names and NCHW conv layout, so
checkpoints interchange with the reference.  New: a sibling ``.aux`` file with what the
reference never saved (FoolsGold history, RNG streams) so a resumed run continues exactly.
Everything is loaded with ``torch.load(weights_only=True)`` — nothing executable is
ever unpickled.
"""
from __future__ import annotations

import os
import random
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from ..models.spec import ModelSpec


def save_checkpoint(path: str, spec: ModelSpec, state: torch.Tensor, epoch: int, lr: float,
                    counter: int) -> None:
    sd = spec.state_dict_from_flat(state, counter)
    tmp = path + ".tmp"
    torch.save({"state_dict": sd, "epoch": int(epoch), "lr": float(lr)}, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str, spec: ModelSpec) -> Tuple[torch.Tensor, int, Optional[float], int]:
    """-> (flat state [S] fp32 cpu, epoch, lr, num_batches_tracked)."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = ck["state_dict"] if isinstance(ck, dict) and "state_dict" in ck else ck
    flat = spec.flat_from_state_dict(sd)
    counter = 0
    for k in spec.counters:
        if k in sd:
            counter = int(sd[k])
            break
    return flat, int(ck.get("epoch", 0)), ck.get("lr"), counter


def rng_state(py: random.Random, npr: np.random.RandomState) -> Dict[str, Any]:
    v, st, gauss = py.getstate()
    name, keys, pos, has_gauss, cached = npr.get_state()
    return {"py_version": int(v), "py_state": torch.tensor(st, dtype=torch.int64),
            "py_gauss": float(gauss) if gauss is not None else None,
            "np_keys": torch.from_numpy(keys.astype(np.int64)), "np_pos": int(pos),
            "np_has_gauss": int(has_gauss), "np_cached": float(cached)}


def restore_rng(d: Dict[str, Any], py: random.Random, npr: np.random.RandomState) -> None:
    py.setstate((d["py_version"], tuple(int(x) for x in d["py_state"].tolist()), d["py_gauss"]))
    npr.set_state(("MT19937", d["np_keys"].numpy().astype(np.uint32), d["np_pos"], d["np_has_gauss"],
                   d["np_cached"]))


def save_aux(path: str, payload: Dict[str, Any]) -> None:
    tmp = path + ".tmp"
    torch.save(payload, tmp)
    os.replace(tmp, path)


def load_aux(path: str) -> Optional[Dict[str, Any]]:
    if not os.path.exists(path):
        return None
    return torch.load(path, map_location="cpu", weights_only=True)
