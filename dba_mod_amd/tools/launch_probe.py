"""Eager launch cost with / without a live RCCL communicator (round-3 diagnosis of the
world-1 RCCL slowdown): times a chunk-like sequence of eager fp32 conv launches (host wall,
synchronised) and the same sequence replayed from a captured HIP graph.

    python -m dba_mod_amd.tools.launch_probe [--rccl]
"""
from __future__ import annotations

import argparse
import json
import os
import time

import torch


_LIMITS = {"stack": 0, "malloc_heap": 2}


def _hip():
    import ctypes
    return ctypes.CDLL("libamdhip64.so")


def device_state() -> dict:
    """HIP device limits and flags of the current device (what a communicator init may change)."""
    import ctypes
    L = _hip()
    out = {}
    for k, v in _LIMITS.items():
        n = ctypes.c_size_t(0)
        rc = L.hipDeviceGetLimit(ctypes.byref(n), ctypes.c_int(v))
        L.hipGetLastError()            # an unsupported limit must not leave a sticky error for torch
        out[k] = int(n.value) if rc == 0 else f"rc{rc}"
    f = ctypes.c_uint(0)
    rc = L.hipGetDeviceFlags(ctypes.byref(f))
    out["flags"] = int(f.value) if rc == 0 else f"rc{rc}"
    return out


def restore_device_state(before: dict, after: dict) -> None:
    import ctypes
    L = _hip()
    for k, v in _LIMITS.items():
        if isinstance(before.get(k), int) and before[k] != after.get(k):
            L.hipDeviceSetLimit(ctypes.c_int(v), ctypes.c_size_t(before[k]))
            L.hipGetLastError()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rccl", action="store_true")
    ap.add_argument("--gloo", action="store_true", help="a world-1 gloo group instead (control)")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--restore-limits", action="store_true",
                    help="put the device limits / flags back to their pre-group values after the group init")
    ap.add_argument("--same-prio", action="store_true", help="both probe streams at default priority")
    ap.add_argument("--streams-first", action="store_true", help="create the probe streams before the group")
    args = ap.parse_args(argv)
    torch.cuda.init()
    pri = (0, 0) if args.same_prio else (-1, 0)
    early = (torch.cuda.Stream(priority=pri[0]), torch.cuda.Stream(priority=pri[1])) if args.streams_first else None
    before = device_state()
    if args.rccl or args.gloo:
        from ..parallel.dist import init_distributed
        os.environ.update(DBA_FORCE_PG="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29591"))
        if args.gloo:
            os.environ["DBA_DIST_BACKEND"] = "gloo"
        ok = init_distributed().selfcheck_ok
        assert ok or ok is None
    after = device_state()
    if args.restore_limits:
        restore_device_state(before, after)
    from ..ops import hip as H
    dev = torch.device("cuda")
    out = {"rccl": args.rccl, "gloo": args.gloo, "lazy": os.environ.get("DBA_PG_LAZY") == "1",
           "state_before": before, "state_after": after, "restored": args.restore_limits,
           "same_prio": args.same_prio, "streams_first": args.streams_first,
           "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}
    graphs = {}
    for name, (G, N, Hh, C) in {"small": (2, 64, 8, 128), "large": (4, 512, 16, 64)}.items():
        x = torch.randn(G, N, Hh, Hh, C, device=dev)
        w = torch.randn(G, C, 3, 3, C, device=dev) * 0.05

        def seq():
            y = x
            for _ in range(20):
                y = H.conv2d(y, w, None, 1, 1, relu=True)
            return y
        for _ in range(3):
            seq()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            seq()
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / args.reps
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            seq()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            seq()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            g.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t0) / args.reps
        out[name] = {"eager_ms": round(eager * 1e3, 3), "graph_ms": round(graph * 1e3, 3)}
        # the graph reads x / w by address: keep them (and the graph) alive for the two-stream
        # replay below (the next capture empties the allocator cache)
        graphs[name] = (g, x, w)
    # two streams at the bench's priorities (training high, evaluation default): the small
    # sequence's graph replayed on one while the large one runs on the other.  Overlapped
    # time vs the sum of the two alone shows whether the streams still run concurrently.
    hi, lo = early if early is not None else (torch.cuda.Stream(priority=pri[0]), torch.cuda.Stream(priority=pri[1]))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        with torch.cuda.stream(lo):
            graphs["large"][0].replay()
        with torch.cuda.stream(hi):
            for _ in range(4):
                graphs["small"][0].replay()
    torch.cuda.synchronize()
    both = (time.perf_counter() - t0) / args.reps
    alone = out["large"]["graph_ms"] + 4 * out["small"]["graph_ms"]
    out["two_streams"] = {"overlapped_ms": round(both * 1e3, 3), "serial_sum_ms": round(alone, 3),
                          "overlap_gain": round(alone / (both * 1e3), 3)}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
