"""Logging, phase timers (with roctx ranges), JSONL metrics and optional Visdom plots.

* Logger: the reference's single ``logging.getLogger("logger")`` writing ``{folder}/log.txt``
  and the console at DEBUG (``helper.py:40-42``); only rank 0 writes the file.
* :class:`PhaseTimer`: per-phase wall time (select / train / gather / aggregate / eval / io)
  measured between device synchronisations, each phase also emitted as a roctx range so
  ``rocprofv3 --marker-trace`` shows the round structure around the kernels.
* :class:`Plotter`: the reference's Visdom windows (``models/simple.py:18-200``) become an
  event stream (``vis_events.jsonl``); a live Visdom server is used only when
  ``visdom: true`` and the ``visdom`` package is importable — the run never depends on it.
"""
from __future__ import annotations

import ctypes
import json
import logging
import os
import time
from contextlib import contextmanager
from typing import Any, Dict, Iterator, List, Optional

import torch

LOGGER_NAME = "logger"


def setup_logger(folder: Optional[str], is_main: bool, level: int = logging.DEBUG) -> logging.Logger:
    log = logging.getLogger(LOGGER_NAME)
    log.setLevel(level if is_main else logging.WARNING)
    for h in list(log.handlers):
        log.removeHandler(h)
    if is_main:
        sh = logging.StreamHandler()
        sh.setFormatter(logging.Formatter("%(message)s"))
        log.addHandler(sh)
        if folder:
            fh = logging.FileHandler(os.path.join(folder, "log.txt"))
            log.addHandler(fh)
    log.propagate = False
    return log


class _Roctx:
    def __init__(self) -> None:
        self.lib = None
        for name in ("librocprofiler-sdk-roctx.so", "libroctx64.so"):
            try:
                self.lib = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if self.lib is not None:
            try:
                self.push = self.lib.roctxRangePushA
                self.push.argtypes = [ctypes.c_char_p]
                self.pop = self.lib.roctxRangePop
            except AttributeError:
                self.lib = None

    def range_push(self, msg: str) -> None:
        if self.lib is not None:
            self.push(msg.encode())

    def range_pop(self) -> None:
        if self.lib is not None:
            self.pop()


_ROCTX: Optional[_Roctx] = None


def roctx() -> _Roctx:
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = _Roctx()
    return _ROCTX


class PhaseTimer:
    def __init__(self, device: torch.device, sync: bool = True) -> None:
        self.device = device
        self.sync = sync
        self.t: Dict[str, float] = {}

    def _sync(self) -> None:
        # only the CURRENT stream: a device-wide sync would serialise the overlapped eval stream
        if self.sync and self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    @contextmanager
    def phase(self, name: str, sync: bool = True) -> Iterator[None]:
        """Time a phase; ``sync=False`` for host-only phases (no device synchronisation)."""
        if sync:
            self._sync()
        roctx().range_push(name)
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if sync:
                self._sync()
            roctx().range_pop()
            self.t[name] = self.t.get(name, 0.0) + time.perf_counter() - t0

    def reset(self) -> Dict[str, float]:
        out, self.t = self.t, {}
        return out


class MetricsStream:
    def __init__(self, path: Optional[str]) -> None:
        self.path = path

    def emit(self, rec: Dict[str, Any]) -> None:
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(rec, default=float) + "\n")


class Plotter:
    """Visdom-compatible line plots; records every point, sends to Visdom if enabled."""

    def __init__(self, env: str, path: Optional[str], live: bool = False) -> None:
        self.env = env
        self.path = path
        self.vis = None
        if live:
            try:
                import visdom  # type: ignore
                self.vis = visdom.Visdom(port=8098)
            except Exception:  # visdom not installed / no server: stream only
                self.vis = None

    def line(self, win: str, x: float, y: float, name: str) -> None:
        rec = {"env": self.env, "win": win, "x": x, "y": y, "name": name}
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(rec, default=float) + "\n")
        if self.vis is not None:
            import numpy as np
            self.vis.line(X=np.array([x]), Y=np.array([y]), name=name, win=win, env=self.env,
                          update="append" if self.vis.win_exists(win, env=self.env) else None,
                          opts=dict(showlegend=True, title=win))

    def text(self, html: str) -> None:
        if self.vis is not None:
            self.vis.text(text=html, env=self.env, opts=dict(width=300, height=400))


def dict_html(d: Dict[str, Any], current_time: str) -> str:
    """reference utils/utils.py:8-19 (params table for the Visdom text pane)."""
    skip = {"poisoning_test", "test_batch_size", "discount_size", "folder_path", "log_interval",
            "coefficient_transfer", "grad_threshold"}
    rows = "".join(f"<tr><td>{k}</td><td>{v}</td></tr>" for k, v in d.items() if k not in skip)
    return f"<h4>Params for model: {current_time}:</h4><table>{rows}</table>"
