"""Summarise rocprofv3 PMC / kernel-trace CSVs per kernel (median over dispatches).

    python -m dba_mod_amd.tools.pmc_summary gpurun_out/pmc_eval [--match xconv]

Reads every ``*counter_collection.csv`` (one row per dispatch x counter) and
``*kernel_trace.csv`` under the directory; prints one markdown table row per kernel with the
median of each counter and the median duration."""
from __future__ import annotations

import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def _short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:90]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args(argv)
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = _short(r.get("Kernel_Name", ""))
            if a.match in k:
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = _short(r.get("Kernel_Name", ""))
            if a.match in k and "Kernel_Name" in r:
                vals[k]["dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    cols = sorted({c for v in vals.values() for c in v})
    print("| kernel | " + " | ".join(cols) + " |")
    print("|---" * (len(cols) + 1) + "|")
    for k, v in sorted(vals.items()):
        print(f"| `{k}` | " + " | ".join(f"{statistics.median(v[c]):.4g}" if v.get(c) else "" for c in cols) + " |")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
