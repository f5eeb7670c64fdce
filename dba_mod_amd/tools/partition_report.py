"""Per-client data-split report: the reference's split self-check and its Dirichlet plot.

* prints, per participant, the class histogram, shard size and majority class, then the mean
  shard size — the reference's ``image_helper.py`` ``__main__`` block (``:352-378``);
* ``--csv``: the same table as CSV;
* ``--plot``: the stacked horizontal bar chart of images per (label, participant) of the
  reference's ``draw_dirichlet_plot`` (``image_helper.py:112-146``, whose call is commented
  out there), saved as ``Num_Img_Dirichlet_Alpha{alpha}.pdf`` (or the given path).

    python -m dba_mod_amd.tools.partition_report --params configs/cifar_params.yaml [--plot out.pdf]
"""
from __future__ import annotations

import argparse
import csv
import os
import sys
from typing import List

import numpy as np
import torch

from .. import config as C
from ..data.partition import shard_class_histogram
from ..fl.workload import build_workload


def histogram_table(params: C.Params) -> tuple:
    wl = build_workload(params, torch.device("cpu"))
    if wl.kind != "image":
        raise SystemExit("partition_report covers the image workloads (LOAN splits by US state)")
    labels = wl.train_store.labels.cpu().numpy().astype(np.int64)
    k = int(wl.spec.num_classes)
    names = sorted(wl.client_indices, key=lambda n: (str(type(n)), n))
    hist = np.stack([shard_class_histogram(labels, list(wl.client_indices[n]), k) for n in names])
    return names, hist


def plot(hist: np.ndarray, path: str) -> None:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    n_part, n_cls = hist.shape
    fig = plt.figure(figsize=(10, 5))
    colors = plt.get_cmap("RdYlGn")(np.linspace(0.15, 0.85, n_part))
    labels = [f"Label {c}" for c in range(n_cls)]
    left = np.zeros(n_cls)
    for p in range(n_part):
        plt.barh(labels, hist[p], left=left, label=str(p), color=colors[p])
        left = left + hist[p]
    plt.legend(ncol=20, loc="lower left", bbox_to_anchor=(0, 1), fontsize=4)
    plt.xlabel("Number of Images", fontsize=16)
    fig.tight_layout(pad=0.1)
    fig.savefig(path)
    plt.close(fig)


def main(argv: List[str] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--params", required=True)
    ap.add_argument("--set", dest="overrides", nargs="*", default=[])
    ap.add_argument("--csv", default=None)
    ap.add_argument("--plot", default=None, nargs="?", const="",
                    help="write the stacked bar chart (default name: Num_Img_Dirichlet_Alpha{alpha}.pdf)")
    args = ap.parse_args(argv)
    over = {"resumed_model": False}
    over.update(C.parse_override(args.overrides))
    params = C.load_params(args.params, over)
    names, hist = histogram_table(params)
    for n, h in zip(names, hist):
        print(n, {c: int(v) for c, v in enumerate(h)}, int(h.sum()), (int(h.max()), int(h.argmax())))
    print("avg", float(hist.sum(1).mean()))
    if args.csv:
        with open(args.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["participant"] + [f"class_{c}" for c in range(hist.shape[1])] + ["total"])
            for n, h in zip(names, hist):
                w.writerow([n] + [int(v) for v in h] + [int(h.sum())])
    if args.plot is not None:
        path = args.plot or f"Num_Img_Dirichlet_Alpha{params['dirichlet_alpha']}.pdf"
        plot(hist, path)
        print(f"wrote {os.path.abspath(path)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
