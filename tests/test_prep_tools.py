"""Offline dataset preparation tools (reference utils/loan_preprocess.py, tinyimagenet_reformat.py)."""
import os

import numpy as np
import pandas as pd

from dba_mod_amd.data import readers
from dba_mod_amd.tools import prep_loan, prep_tiny

from conftest import ROOT


def test_loan_preprocess_encodes_scales_and_splits(tmp_path):
    n = 60
    rng = np.random.default_rng(0)
    df = pd.DataFrame({
        "id": np.arange(n), "url": ["u"] * n,                       # dropped
        "loan_amnt": rng.uniform(1000, 30000, n),                    # mean > 1000   -> /10000
        "int_rate": rng.uniform(11, 20, n),                          # (10, 100]     -> /10
        "installment": rng.uniform(150, 900, n),                     # (100, 1000]   -> /100
        "pub_rec": rng.integers(0, 3, n).astype(np.int64),           # <= 10         -> unchanged
        "term": rng.choice([" 36 months", " 60 months"], n),         # object -> first-appearance codes
        "loan_status": rng.choice(["Current", "Fully Paid", "Charged Off"], n),
        "addr_state": rng.choice(["CA", "NY", "TX"], n),
        "mths_since_last_delinq": [np.nan] * n,                      # dropped
    })
    df.loc[3, "int_rate"] = np.nan                                   # fillna(0) before scaling
    out = prep_loan.preprocess(df)
    assert "id" not in out and "url" not in out and "mths_since_last_delinq" not in out
    np.testing.assert_allclose(out["loan_amnt"], df["loan_amnt"] / 10000)
    np.testing.assert_allclose(out["installment"], df["installment"] / 100)
    np.testing.assert_allclose(out["int_rate"], df["int_rate"].fillna(0) / 10)
    assert (out["pub_rec"] == df["pub_rec"]).all()
    first = list(dict.fromkeys(df["loan_status"]))
    assert [first[c] for c in out["loan_status"]] == list(df["loan_status"])
    files = prep_loan.split_by_state(out, str(tmp_path / "loan"))
    assert sorted(os.path.basename(f) for f in files) == ["loan_CA.csv", "loan_NY.csv", "loan_TX.csv"]
    # the framework's LOAN reader consumes the output directly
    parts = readers.read_loan(str(tmp_path))
    assert sum(len(p.train_y) + len(p.test_y) for p in parts) == n


def test_tiny_reformat_moves_val_images(tmp_path):
    root = tmp_path / "tiny-imagenet-200"
    img = root / "val" / "images"
    img.mkdir(parents=True)
    ann = []
    for i, wnid in enumerate(["n01", "n02", "n01"]):
        (img / f"val_{i}.JPEG").write_bytes(b"x")
        ann.append(f"val_{i}.JPEG\t{wnid}\t0\t0\t63\t63")
    (root / "val" / "val_annotations.txt").write_text("\n".join(ann) + "\n")
    assert prep_tiny.reformat_val(str(root)) == 3
    assert sorted(os.listdir(root / "val")) == ["n01", "n02"]
    assert sorted(os.listdir(root / "val" / "n01")) == ["val_0.JPEG", "val_2.JPEG"]
    assert prep_tiny.reformat_val(str(root)) == 0                  # idempotent


def test_partition_report_reproduces_attacker_shards(tmp_path):
    """Split self-check / Dirichlet plot tool (reference image_helper.py:112-146,352-378):
    the CIFAR attackers' shard sizes are the ones annotated in cifar_params.yaml."""
    import csv as _csv
    from dba_mod_amd.tools import partition_report
    out = tmp_path / "split.csv"
    pdf = tmp_path / "split.pdf"
    assert partition_report.main(["--params", os.path.join(ROOT, "configs", "cifar_params.yaml"),
                                  "--set", "synthetic_data=true", "--csv", str(out), "--plot", str(pdf)]) == 0
    rows = {r["participant"]: int(r["total"]) for r in _csv.DictReader(open(out))}
    assert [rows[k] for k in ("17", "33", "77", "11")] == [526, 527, 496, 546]
    assert pdf.stat().st_size > 0


def test_trace_streams_summary(tmp_path):
    """rocprofv3 kernel-trace CSV -> per-stream markdown (tools/trace_streams.py)."""
    from dba_mod_amd.tools.trace_streams import summarize
    p = tmp_path / "k.csv"
    hdr = '"Kind","Stream_Id","Kernel_Name","Start_Timestamp","End_Timestamp"\n'
    rows = [("1", "void (anonymous namespace)::xconv_kernel<32, 128, 1, 4, 2, 32, true, false>(XArgs)", 0, 2_000_000),
            ("1", "(anonymous namespace)::bnx_finalize_kernel(BnFuse)", 2_000_000, 3_000_000),
            ("4", "void (anonymous namespace)::xhalo_kernel<32, 32, 128, 32>(XArgs)", 1_000_000, 5_000_000)]
    p.write_text(hdr + "".join(f'"KERNEL_DISPATCH",{s},"{k}",{a},{b}\n' for s, k, a, b in rows))
    md = summarize(str(p), last_ms=100)
    assert "## stream 1: 3.0 ms" in md and "## stream 4: 4.0 ms" in md
    assert "`xconv_kernel<32, 128, 1, 4, 2, 32, true, false>` | 2.0 | 66.7 | 1 |" in md
    assert "Union of kernel intervals: 5 ms of 5 ms" in md
