"""Offline Tiny-ImageNet-200 reformat: ``val/images/*`` -> ``val/<wnid>/*`` (ImageFolder layout).

Behaviour of reference ``utils/tinyimagenet_reformat.py:1-33`` (+ ``process_tiny_data.sh``):
read ``val/val_annotations.txt`` (tab-separated: file, wnid, bbox...), move each validation
image into its class folder, then delete the annotation file and the emptied ``images/``
directory.  Idempotent: a second run on an already reformatted tree does nothing.

    python -m dba_mod_amd.tools.prep_tiny --root data/tiny-imagenet-200
"""
from __future__ import annotations

import argparse
import os
import shutil
from typing import Dict


def reformat_val(root: str) -> int:
    val = os.path.join(root, "val")
    ann = os.path.join(val, "val_annotations.txt")
    img_dir = os.path.join(val, "images")
    if not os.path.exists(ann):
        return 0
    label_of: Dict[str, str] = {}
    with open(ann) as f:
        for line in f:
            parts = line.rstrip("\n").split("\t")
            if len(parts) >= 2:
                label_of[parts[0]] = parts[1]
    moved = 0
    if os.path.isdir(img_dir):
        for fn in sorted(os.listdir(img_dir)):
            wnid = label_of.get(fn)
            if wnid is None:
                raise KeyError(f"{fn} has no entry in {ann}")
            os.makedirs(os.path.join(val, wnid), exist_ok=True)
            shutil.move(os.path.join(img_dir, fn), os.path.join(val, wnid, fn))
            moved += 1
        os.rmdir(img_dir)
    os.remove(ann)
    return moved


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--root", default="data/tiny-imagenet-200")
    args = ap.parse_args(argv)
    n = reformat_val(args.root)
    print(f"moved {n} validation images into class folders under {args.root}/val")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
