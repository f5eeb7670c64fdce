"""Client-parallel distributed rounds on the gloo backend (CPU, world 2 and 3) must give the
same global model and metrics as world 1 — placement (LPT), the snapshot all-gather and the
image-sharded evaluation + counter all-reduce are all exercised."""
import os

import pytest
import torch

from dba_mod_amd.tools.dist_check import run_world

from conftest import ROOT

CFG = os.path.join(ROOT, "configs", "mnist_params.yaml")


@pytest.mark.parametrize("agg", ["mean", "geom_median", "foolsgold"])
def test_world2_matches_world1(tmp_path, agg):
    over = {"resumed_model": False, "start_epoch": 11, "synthetic_data": True, "synthetic_train_size": 3000,
            "synthetic_test_size": 400, "save_dir": str(tmp_path), "eval_batch_size": 200,
            "aggregation_methods": agg}
    rounds = [11, 12]
    one = run_world(1, str(tmp_path / "w1"), CFG, over, rounds)
    two = run_world(2, str(tmp_path / "w2"), CFG, over, rounds)
    assert torch.equal(two[0]["state"], two[1]["state"])           # every rank holds the same model
    torch.testing.assert_close(two[0]["state"], one[0]["state"], rtol=1e-5, atol=1e-6)
    for a, b in zip(two[0]["acc"], one[0]["acc"]):
        assert abs(a - b) < 1e-6
    for a, b in zip(two[0]["asr"], one[0]["asr"]):
        assert abs(a - b) < 1e-6


def test_world3_uneven_placement(tmp_path):
    over = {"resumed_model": False, "start_epoch": 12, "synthetic_data": True, "synthetic_train_size": 3000,
            "synthetic_test_size": 400, "save_dir": str(tmp_path), "eval_batch_size": 200}
    one = run_world(1, str(tmp_path / "w1"), CFG, over, [12])
    three = run_world(3, str(tmp_path / "w3"), CFG, over, [12])
    torch.testing.assert_close(three[2]["state"], one[0]["state"], rtol=1e-5, atol=1e-6)
