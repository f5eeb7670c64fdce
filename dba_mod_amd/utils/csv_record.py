"""CSV result files, byte-compatible with the reference (``utils/csv_record.py:1-66``).

Same six files, same headers (including the ``posiontest`` spelling), same row shapes, and
the same full-rewrite-every-round behaviour; only rank 0 writes.  Unlike the reference's
module-global lists, the rows live on a :class:`CsvRecorder` instance.
"""
from __future__ import annotations

import copy
import csv
import os
from typing import Any, List

TRAIN_HEADER = ["local_model", "round", "epoch", "internal_epoch", "average_loss", "accuracy",
                "correct_data", "total_data"]
TEST_HEADER = ["model", "epoch", "average_loss", "accuracy", "correct_data", "total_data"]
TRIGGER_HEADER = ["model", "trigger_name", "trigger_value", "epoch", "average_loss", "accuracy",
                  "correct_data", "total_data"]


class CsvRecorder:
    def __init__(self, folder: str, enabled: bool = True) -> None:
        self.folder = folder
        self.enabled = enabled
        self.train_result: List[list] = []
        self.test_result: List[list] = []
        self.posiontest_result: List[list] = []
        self.poisontriggertest_result: List[list] = []
        self.weight_result: List[list] = []
        self.scale_result: List[list] = []
        self.scale_temp_one_row: List[Any] = []

    def add_weight_result(self, names: list, weights: list, alphas: list) -> None:
        self.weight_result.append(list(names))
        self.weight_result.append(list(weights))
        self.weight_result.append(list(alphas))

    def _write(self, name: str, rows: List[list], header: List[str] = None) -> None:
        with open(os.path.join(self.folder, name), "w", newline="") as f:
            w = csv.writer(f, lineterminator="\r\n")
            if header is not None:
                w.writerow(header)
            w.writerows(rows)

    def save(self, is_poison: bool) -> None:
        """reference save_result_csv(epoch, is_posion, folder_path)."""
        if self.scale_temp_one_row:
            self.scale_result.append(copy.deepcopy(self.scale_temp_one_row))
            self.scale_temp_one_row.clear()
            has_scale = True
        else:
            has_scale = bool(self.scale_result)
        if not self.enabled:
            return
        self._write("train_result.csv", self.train_result, TRAIN_HEADER)
        self._write("test_result.csv", self.test_result, TEST_HEADER)
        if self.weight_result:
            self._write("weight_result.csv", self.weight_result)
        if has_scale:
            self._write("scale_result.csv", self.scale_result)
        if is_poison:
            self._write("posiontest_result.csv", self.posiontest_result, TEST_HEADER)
            self._write("poisontriggertest_result.csv", self.poisontriggertest_result, TRIGGER_HEADER)
