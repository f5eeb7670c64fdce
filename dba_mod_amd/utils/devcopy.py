"""Host -> device uploads that never stall the host.

``torch.tensor(data, device="cuda")`` and ``.to(device)`` from pageable host memory are
synchronous copies ordered on the current stream: issued in the middle of an enqueued
evaluation (or training round) they block the host until every kernel already queued on
that stream has finished — which silently serialises the two-stream round pipeline
(:mod:`dba_mod_amd.fl.server`).  These helpers stage through pinned memory (torch's caching
host allocator keeps the buffer alive until the copy has executed) and copy asynchronously.
"""
from __future__ import annotations

from typing import Any, Optional

import numpy as np
import torch


def to_device(data: Any, device: torch.device, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    if isinstance(data, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(data))
        if dtype is not None:
            t = t.to(dtype)
    else:
        t = torch.as_tensor(data, dtype=dtype)
    if device.type != "cuda":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)
