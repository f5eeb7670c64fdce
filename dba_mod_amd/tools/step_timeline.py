"""Training-step timeline of a ``rocprofv3 --kernel-trace --output-format csv`` trace.

``python -m dba_mod_amd.tools.step_timeline TRACE.csv [--last-ms 3000] [--min-gap-ms 4]``
marks every training step by its ``sgd_kernel`` (one per step) and prints, for the window's
runs of consecutive steps, each run's step count, wall time, per-step time and the kernel time
of the training stream vs the other streams inside it; then the steps slower than the run's
median by more than ``--slow`` x, with what ran in their interval.  It answers "is a slow
round's training chain slow per step (contention, a missing graph) or waiting between steps
(host)".
"""
from __future__ import annotations

import argparse
import csv
import re
import statistics
from collections import defaultdict
from typing import List, Tuple


def _short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)", name)
    return m.group(1) if m else name[:60]


def timeline(path: str, last_ms: float = 3000.0, min_gap_ms: float = 4.0, slow: float = 1.5) -> str:
    rows: List[Tuple[int, int, int, str]] = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]),
                         _short(r["Kernel_Name"])))
    if not rows:
        return "empty trace\n"
    rows.sort()
    t_end = max(r[1] for r in rows)
    t0 = t_end - int(last_ms * 1e6)
    win = [r for r in rows if r[1] >= t0]
    sgd = [r for r in win if r[3].startswith("sgd_kernel")]
    if not sgd:
        return "no sgd_kernel in the window\n"
    train_stream = sgd[0][2]
    # runs: consecutive steps closer than min_gap_ms
    runs: List[List[Tuple[int, int, int, str]]] = [[sgd[0]]]
    for r in sgd[1:]:
        if (r[1] - runs[-1][-1][1]) / 1e6 > min_gap_ms:
            runs.append([r])
        else:
            runs[-1].append(r)
    out = [f"window: last {last_ms:.0f} ms, {len(win)} kernels, {len(sgd)} steps, training stream {train_stream}", "",
           "| run | start ms | steps | wall ms | ms / step (median) | train-stream kernel ms | other-stream kernel ms |",
           "|---|---|---|---|---|---|---|"]
    slow_rows = []
    for i, run in enumerate(runs):
        a = run[0][1]
        b = run[-1][1]
        ivs = [(run[k][1] - run[k - 1][1]) / 1e6 for k in range(1, len(run))]
        med = statistics.median(ivs) if ivs else 0.0
        tk = sum((min(e, b) - max(s, a)) for s, e, st, _ in win if st == train_stream and e > a and s < b) / 1e6
        ok = sum((min(e, b) - max(s, a)) for s, e, st, _ in win if st != train_stream and e > a and s < b) / 1e6
        out.append(f"| {i} | {(a - t0) / 1e6:.1f} | {len(run)} | {(b - a) / 1e6:.1f} | {med:.3f} | {tk:.1f} | {ok:.1f} |")
        for k in range(1, len(run)):
            if med > 0 and ivs[k - 1] > slow * med:
                slow_rows.append((i, k, ivs[k - 1], med, run[k - 1][1], run[k][1]))
    if slow_rows:
        out += ["", f"steps slower than {slow} x their run's median (up to 20):", "",
                "| run | step | ms | median | largest train-stream kernels in the interval | other streams' kernel ms |",
                "|---|---|---|---|---|---|"]
        for i, k, dt, med, a, b in slow_rows[:20]:
            ks = defaultdict(float)
            other = 0.0
            for s, e, st, name in win:
                if e > a and s < b:
                    if st == train_stream:
                        ks[name] += (min(e, b) - max(s, a)) / 1e6
                    else:
                        other += (min(e, b) - max(s, a)) / 1e6
            top = ", ".join(f"{n} {v:.2f}" for n, v in sorted(ks.items(), key=lambda x: -x[1])[:3])
            out.append(f"| {i} | {k} | {dt:.2f} | {med:.2f} | {top} | {other:.2f} |")
    return "\n".join(out) + "\n"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-ms", type=float, default=3000.0)
    ap.add_argument("--min-gap-ms", type=float, default=4.0)
    ap.add_argument("--slow", type=float, default=1.5)
    a = ap.parse_args()
    print(timeline(a.trace, a.last_ms, a.min_gap_ms, a.slow), end="")


if __name__ == "__main__":
    main()
