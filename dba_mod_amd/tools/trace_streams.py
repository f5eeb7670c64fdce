"""Per-stream kernel-time summary of a ``rocprofv3 --kernel-trace --output-format csv`` trace.

``python -m dba_mod_amd.tools.trace_streams gpurun_out/prof/bench_kernel_trace.csv
[--last-ms 750] [--top 12]`` prints a markdown report: for every HIP stream, the kernels that
took the most time (ms, share of the stream, launches), then the union of all kernel
intervals over the window — how much of the wall time the GPU had any kernel in flight.
The window is the last ``--last-ms`` of the trace (the timed bench rounds; the warm start
and the first warm-up round are before it).
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict
from typing import Dict, List, Tuple


def _short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)", name)
    return m.group(1) if m else name[:60]


def summarize(path: str, last_ms: float = 750.0, top: int = 12) -> str:
    rows: List[Tuple[int, int, int, str]] = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]),
                         _short(r["Kernel_Name"])))
    if not rows:
        return "empty trace\n"
    t_end = max(r[1] for r in rows)
    t0 = t_end - int(last_ms * 1e6)
    win = [r for r in rows if r[0] >= t0]
    per: Dict[int, Dict[str, List[float]]] = defaultdict(lambda: defaultdict(lambda: [0.0, 0]))
    for s, e, st, k in win:
        acc = per[st][k]
        acc[0] += (e - s) / 1e6
        acc[1] += 1
    out = [f"Window: last {last_ms:.0f} ms of the trace, {len(win)} kernels.\n"]
    for st in sorted(per):
        tot = sum(v[0] for v in per[st].values())
        out.append(f"\n## stream {st}: {tot:.1f} ms of kernels\n\n| kernel | ms | % | launches |\n|---|---|---|---|")
        for k, (ms, n) in sorted(per[st].items(), key=lambda kv: -kv[1][0])[:top]:
            out.append(f"| `{k}` | {ms:.1f} | {100 * ms / max(tot, 1e-9):.1f} | {n} |")
    iv = sorted((s, e, k) for s, e, _, k in win)
    busy, cur_s, cur_e, last_k = 0, iv[0][0], iv[0][1], iv[0][2]
    gaps: List[Tuple[int, str, str, int]] = []   # (idle ns, kernel before, kernel after, start ns)
    for s, e, k in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, last_k, k, cur_e))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= cur_e:
            last_k = k
    busy += cur_e - cur_s
    span = (t_end - min(s for s, _, _ in iv)) / 1e6
    out.append(f"\nUnion of kernel intervals: {busy / 1e6:.0f} ms of {span:.0f} ms "
               f"({100 * busy / 1e6 / max(span, 1e-9):.0f} % of the window has a kernel in flight).\n")
    if gaps:
        big = sorted(gaps, reverse=True)[:top]
        idle = sum(g[0] for g in gaps) / 1e6
        n1 = sum(1 for g in gaps if g[0] >= 1e6)
        out.append(f"Idle: {idle:.1f} ms in {len(gaps)} gaps ({n1} of >= 1 ms, "
                   f"{sum(g[0] for g in gaps if g[0] >= 1e6) / 1e6:.1f} ms).  Largest:\n\n"
                   "| idle ms | starts, ms before the trace end | last kernel before | first kernel after |\n"
                   "|---|---|---|---|")
        for g, a, b, t in big:
            out.append(f"| {g / 1e6:.2f} | {(t_end - t) / 1e6:.1f} | `{a}` | `{b}` |")
    return "\n".join(out) + "\n"


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("trace")
    ap.add_argument("--last-ms", type=float, default=750.0)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    print(summarize(a.trace, a.last_ms, a.top), end="")


if __name__ == "__main__":
    main()
