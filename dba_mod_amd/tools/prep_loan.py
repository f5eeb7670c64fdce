"""Offline LOAN preprocessing: Kaggle ``loan.csv`` -> one ``loan_<STATE>.csv`` per US state.

Behaviour of reference ``utils/loan_preprocess.py:1-58`` (+ ``process_loan_data.sh``), as a
vectorised pandas pipeline (the reference assigns codes one value at a time and writes rows
one ``iloc`` at a time — hours on the 2.26 M-row file):

1. drop the identifier / free-text / date / sparse joint-application / hardship /
   settlement columns (``DROP_COLUMNS``), then ``fillna(0)``;
2. every object column except ``addr_state`` -> ordinal codes in order of first
   appearance (``pd.factorize(sort=False)`` == the reference's ``drop_duplicates`` order);
3. numeric columns rescaled by the magnitude of their mean:
   (10, 100] -> /10, (100, 1000] -> /100, > 1000 -> /10000, <= 10 unchanged;
4. split by ``addr_state`` (column dropped) into ``{out_dir}/loan_<ST>.csv``.

The output is exactly what :func:`dba_mod_amd.data.readers.read_loan` consumes.

    python -m dba_mod_amd.tools.prep_loan --src data/lending-club-loan-data/loan.csv --out data/loan
"""
from __future__ import annotations

import argparse
import os
from typing import Dict, List

import numpy as np
import pandas as pd

# reference loan_preprocess.py:8-12 (two drop() calls)
DROP_COLUMNS: List[str] = [
    "id", "member_id", "emp_title", "issue_d", "zip_code", "emp_length", "title", "earliest_cr_line",
    "last_pymnt_d", "hardship_start_date", "desc", "hardship_end_date", "payment_plan_start_date",
    "next_pymnt_d", "settlement_date", "last_credit_pull_d", "debt_settlement_flag_date",
    "sec_app_earliest_cr_line",
    "url", "mths_since_last_delinq", "mths_since_last_major_derog", "mths_since_last_record",
    "annual_inc_joint", "dti_joint", "verification_status_joint", "mths_since_recent_bc_dlq",
    "mths_since_recent_revol_delinq", "revol_bal_joint", "sec_app_inq_last_6mths", "sec_app_mort_acc",
    "sec_app_open_acc", "sec_app_revol_util", "sec_app_open_act_il", "sec_app_num_rev_accts",
    "sec_app_chargeoff_within_12_mths", "sec_app_collections_12_mths_ex_med",
    "sec_app_mths_since_last_major_derog", "hardship_type", "hardship_reason", "hardship_status",
    "deferral_term", "hardship_amount", "hardship_length", "hardship_dpd", "hardship_loan_status",
    "orig_projected_additional_accrued_interest", "hardship_payoff_balance_amount",
    "hardship_last_payment_amount", "settlement_status", "settlement_amount", "settlement_percentage",
    "settlement_term",
]
STATE_COLUMN = "addr_state"


def _scale_of(mean: float) -> float:
    if 10.0 < mean <= 100.0:
        return 10.0
    if 100.0 < mean <= 1000.0:
        return 100.0
    if mean > 1000.0:
        return 10000.0
    return 1.0


def preprocess(df: pd.DataFrame) -> pd.DataFrame:
    """Steps 1-3 on an in-memory frame (kept separate for testing)."""
    df = df.drop(columns=[c for c in DROP_COLUMNS if c in df.columns]).fillna(0)
    out: Dict[str, pd.Series] = {}
    for col in df.columns:
        s = df[col]
        if s.dtype == object and col != STATE_COLUMN:
            codes, _ = pd.factorize(s, sort=False)
            out[col] = pd.Series(codes.astype(np.int64), index=s.index)
        elif s.dtype in (np.float64, np.int64):
            k = _scale_of(float(s.mean()))
            out[col] = s / k if k != 1.0 else s
        else:
            out[col] = s
    return pd.DataFrame(out, index=df.index)


def split_by_state(df: pd.DataFrame, out_dir: str) -> List[str]:
    os.makedirs(out_dir, exist_ok=True)
    written = []
    for state, part in df.groupby(STATE_COLUMN, sort=True):
        path = os.path.join(out_dir, f"loan_{state}.csv")
        part.drop(columns=[STATE_COLUMN]).to_csv(path, index=False)
        written.append(path)
    return written


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--src", default="data/lending-club-loan-data/loan.csv")
    ap.add_argument("--out", default="data/loan")
    args = ap.parse_args(argv)
    df = pd.read_csv(args.src, low_memory=False)
    files = split_by_state(preprocess(df), args.out)
    print(f"wrote {len(files)} state files to {args.out}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
