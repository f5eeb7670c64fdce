"""Client-parallel distributed rounds on the gloo backend (CPU, world 2, 3, 4, 8) must give the
same global model and metrics as world 1 — placement (LPT), the reduction-based aggregation
(fp64 FedAvg delta all-reduce, FoolsGold feature + weighted-sum all-reduces, RFA gather or
distributed Weiszfeld), the sharded-test snapshot all-gather and the image-sharded evaluation
+ counter all-reduce are all exercised, and the per-round collective bytes are pinned."""
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
    # bitwise: FedAvg's fp64 delta sums, RFA / FoolsGold through the exact fixed-point limb sums
    assert torch.equal(two[0]["state"], one[0]["state"])
    for a, b in zip(two[0]["acc"], one[0]["acc"]):
        assert abs(a - b) < 1e-6
    for a, b in zip(two[0]["asr"], one[0]["asr"]):
        assert abs(a - b) < 1e-6


def test_world3_uneven_placement(tmp_path):
    over = {"resumed_model": False, "start_epoch": 12, "synthetic_data": True, "synthetic_train_size": 3000,
            "synthetic_test_size": 400, "save_dir": str(tmp_path), "eval_batch_size": 200}
    one = run_world(1, str(tmp_path / "w1"), CFG, over, [12])
    three = run_world(3, str(tmp_path / "w3"), CFG, over, [12])
    assert torch.equal(three[2]["state"], one[0]["state"])


def _over(tmp_path, **kw):
    o = {"resumed_model": False, "start_epoch": 11, "synthetic_data": True, "synthetic_train_size": 3000,
         "synthetic_test_size": 400, "save_dir": str(tmp_path), "eval_batch_size": 200}
    o.update(kw)
    return o


def _csv_rows(folder):
    import csv
    import glob
    out = {}
    for f in sorted(glob.glob(os.path.join(folder, "run", "*.csv"))):
        with open(f) as fh:
            out[os.path.basename(f)] = list(csv.reader(fh))
    return out


def _same_rows(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert len(a[k]) == len(b[k]), k
        for ra, rb in zip(a[k], b[k]):
            assert len(ra) == len(rb), (k, ra, rb)
            for x, y in zip(ra, rb):
                try:
                    fx, fy = float(x), float(y)
                except ValueError:
                    assert x == y, (k, ra, rb)
                    continue
                # counts / accuracies are exact; a loss is a sum of per-chunk fp32 loss sums, and
                # sharding the test images changes the chunks (fp32 rounding, ~1e-7)
                if fx == int(fx) and fy == int(fy):
                    assert fx == fy, (k, ra, rb)
                else:
                    assert abs(fx - fy) <= 1e-6 * max(1.0, abs(fy)), (k, ra, rb)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_fedavg_bitwise_and_bytes(tmp_path, world):
    """FedAvg at world W: bit-identical global model and equal CSV rows vs world 1; the round's
    aggregation moves ONE §5.8-padded fp64 S-vector all-reduce (no snapshot all-gather of the
    aggregated clients); only the image-sharded clients' snapshots are broadcast, each once,
    from their owner rank."""
    from dba_mod_amd.parallel.dist import DistCtx
    over = _over(tmp_path)
    rounds = [11, 12]
    one = run_world(1, str(tmp_path / "w1"), CFG, over, rounds)
    many = run_world(world, str(tmp_path / f"w{world}"), CFG, over, rounds)
    for r in range(world):
        assert torch.equal(many[r]["state"], one[0]["state"]), r
    _same_rows(_csv_rows(str(tmp_path / f"w{world}")), _csv_rows(str(tmp_path / "w1")))
    S = one[0]["S"]
    unit = DistCtx(world=world).pad_unit(8)
    fedavg = (S + unit - 1) // unit * unit * 8
    for ar, ag, bc in many[0]["comm"]:
        assert ar >= fedavg and ar < fedavg + 64 * 1024, (ar, fedavg)   # + small stats / eval counters
        assert ag == 0
    # round 12: the attacker (41) is the round's only long client; only its two snapshots
    # (pre-scaling, final) are broadcast for its image-sharded tests.  (Round 11's clients are
    # all equally long, so all their tests are sharded and their snapshots broadcast.)
    bc12 = many[0]["comm"][1][2]
    assert bc12 == 2 * S * 4, (bc12, S)
    assert one[0]["comm"] == [[0, 0, 0]] * len(rounds)


@pytest.mark.parametrize("agg", ["foolsgold", "geom_median"])
def test_reduction_aggregators_world4(tmp_path, agg):
    """FoolsGold moves the [n, d] features + one weighted P-vector (no [n, P] gradients);
    RFA in distributed mode runs Weiszfeld on rank-resident deltas."""
    over = _over(tmp_path, aggregation_methods=agg, rfa_mode="distributed")
    rounds = [11, 12]
    one = run_world(1, str(tmp_path / "w1"), CFG, over, rounds)
    four = run_world(4, str(tmp_path / "w4"), CFG, over, rounds)
    for r in range(4):
        assert torch.equal(four[r]["state"], four[0]["state"])
    assert torch.equal(four[0]["state"], one[0]["state"])   # world-invariant bits (fixed-point sums)
    for a, b in zip(four[0]["acc"], one[0]["acc"]):
        assert abs(a - b) < 1e-6
    S = one[0]["S"]
    for ar, ag, bc in four[0]["comm"]:
        assert ag <= 4 * 4 * S * 4      # no all-gather of every client's state
        if agg == "foolsgold":
            # features (10 x 5000) + P-vector (fp64) + small counters; NOT 10 x P gradients
            assert ar < 3 * S * 8, (ar, S)
