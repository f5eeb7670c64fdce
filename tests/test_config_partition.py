"""Config parsing (reference YAML schema) and the bit-compatible Dirichlet partitioner."""
import os
import random

import numpy as np
import pytest

from dba_mod_amd import config as C
from dba_mod_amd.data import partition, synthetic

from conftest import REFERENCE, ROOT


@pytest.mark.parametrize("name", ["cifar_params.yaml", "mnist_params.yaml", "tiny_params.yaml", "loan_params.yaml"])
def test_reference_yamls_load_unchanged(name):
    path = os.path.join(REFERENCE, "utils", name)
    if not os.path.exists(path):
        pytest.skip("reference not mounted")
    p = C.load_params(path)
    assert p.type in C.TYPES
    assert p["aggregation_methods"] in C.AGGREGATIONS
    for i in range(int(p["trigger_num"])):
        assert p.poison_epochs_of(i)
    if p.type != C.TYPE_LOAN:
        g = p.poison_pattern(-1)
        assert len(g) == sum(len(p.poison_pattern(i)) for i in range(int(p["trigger_num"])))
    else:
        assert len(p.trigger_features(-1)) == 6


@pytest.mark.parametrize("name", ["cifar_params.yaml", "mnist_params.yaml", "cifar_centralized.yaml"])
def test_own_configs_load(name):
    p = C.load_params(os.path.join(ROOT, "configs", name))
    assert p["no_models"] == 10


def test_overrides_and_validation():
    assert C.parse_override(["a=1", "b=[1,2]", "c=true"]) == {"a": 1, "b": [1, 2], "c": True}
    with pytest.raises(ValueError):
        C.Params({"type": "cifar", "aggregation_methods": "median"})
    with pytest.raises(ValueError):
        C.Params({"type": "cifar", "aggregation_methods": "foolsgold", "aggr_epoch_interval": 2})


def _labels(counts):
    return np.concatenate([np.full(c, k) for k, c in enumerate(counts)])


@pytest.mark.parametrize("counts,adv,alpha,expect", [
    ([5000] * 10, [17, 33, 77, 11, 45], 0.5, [526, 527, 496, 546, 529]),          # cifar_params.yaml:33-36
    (synthetic.MNIST_TRAIN_COUNTS, [41, 73, 51, 74, 95], 0.5, [606, 591, 568, 557, 602]),  # mnist_params.yaml:33-36
    ([500] * 200, [0, 20, 74, 95, 17], 0.5, [990, 993, 983, 993, 999]),           # tiny_params.yaml:32-35 (alpha .5)
])
def test_dirichlet_reproduces_reference_shard_sizes(counts, adv, alpha, expect):
    per = partition.sample_dirichlet(_labels(counts), 100, alpha, random.Random(1), np.random.RandomState(1))
    assert [len(per[a]) for a in adv] == expect
    allidx = np.concatenate([np.asarray(v) for v in per.values()])
    assert len(np.unique(allidx)) == len(allidx)        # disjoint shards


def test_equal_split_and_poison_subset():
    per = partition.equal_split(1000, 10, random.Random(1))
    assert all(len(v) == 100 for v in per.values())
    lab = np.array([0, 2, 1, 2, 3])
    assert partition.poison_test_indices(lab, 2).tolist() == [0, 2, 4]


def test_synthetic_shapes():
    tr, te = synthetic.synthetic_image_pair("cifar", 1, 2000, 500)
    assert tr.images.shape[1:] == (32, 32, 3) and tr.images.dtype == np.uint8
    assert np.bincount(te.labels).tolist() == [50] * 10
    states = synthetic.synthetic_loan(1, total_rows=5000)
    assert len(states) == 51 and states[0].train_x.shape[1] == 91


@pytest.mark.parametrize("name", ["mnist_params", "cifar_params", "cifar_centralized", "tiny_params", "loan_params"])
def test_shipped_configs_plan_their_poison_rounds(name):
    """Every shipped config loads, builds its (synthetic) workload and plans its attack rounds."""
    import torch
    from dba_mod_amd.fl.plan import build_round_plan, select_clients
    from dba_mod_amd.fl.workload import build_workload
    p = C.load_params(os.path.join(ROOT, "configs", f"{name}.yaml"),
                      {"resumed_model": False, "synthetic_data": True, "synthetic_train_size": 3000,
                       "synthetic_test_size": 300})
    wl = build_workload(p, torch.device("cpu"))
    assert len(wl.participants_list) >= int(p["no_models"])
    rounds = sorted({e for i in range(len(p.adversary_list)) for e in p.poison_epochs_of(i)})
    assert rounds
    agents, adversarial = select_clients(p, wl, rounds[0])
    plan = build_round_plan(p, wl, rounds[0], agents, adversarial, loan_preeval_acc=0.0)
    poisoners = [c for c in plan.clients if any(ph.poison for ph in c.phases)]
    assert poisoners, name
