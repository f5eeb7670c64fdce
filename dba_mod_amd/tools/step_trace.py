"""Per-training-step kernel breakdown of a rocprofv3 kernel trace of ``tools.bench_step``.

Steps are delimited by the SGD launch that ends every grouped step; the summary averages the
steps in the second half of the trace (after capture / warm-up):

    python -m dba_mod_amd.tools.step_trace gpurun_out/prof/step1_kernel_trace.csv [--top 25]

Prints kernels per step, summed kernel time per step, and a per-kernel table (µs per step,
launches per step, mean duration) as Markdown.
"""
from __future__ import annotations

import argparse
import collections
import csv


def summarize(path: str, top: int = 25) -> str:
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
    late = [r for r in rows if int(r["Start_Timestamp"]) > t0 + (t1 - t0) // 2]
    ends = [i for i, r in enumerate(late) if "sgd_kernel" in r["Kernel_Name"]]
    if len(ends) < 2:
        raise SystemExit("fewer than two complete steps in the trace")
    seg = late[ends[0] + 1:ends[-1] + 1]
    n = len(ends) - 1
    agg = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = name.split("(")[0][:80]
        agg[name][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[name][1] += 1
    busy = sum(v[0] for v in agg.values()) / 1e3 / n
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3 / n
    out = [f"{n} steps: {len(seg) / n:.0f} kernels/step, {busy:.0f} us of kernels/step, "
           f"{span:.0f} us/step wall", "", "| kernel | us/step | launches/step | us/launch |",
           "|---|---|---|---|"]
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        out.append(f"| `{k}` | {t / 1e3 / n:.1f} | {c / n:.1f} | {t / c / 1e3:.1f} |")
    return "\n".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args(argv)
    print(summarize(a.trace, a.top))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
