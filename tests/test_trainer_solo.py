"""The grouped trainer's solo-tail rule (fl/trainer.py GroupTrainer._solo_tail): when one
client outlasts every other by at least SOLO_MIN_STEPS steps (the 6-epoch attacker after the
2-epoch clients), its tail moves to the G=1 graph.  Pure host logic — the GPU equivalence of
the two paths is covered by the bitwise world-1 / world-2 and reproducibility GPU tests."""
from types import SimpleNamespace

import torch

from dba_mod_amd.fl.trainer import GroupTrainer


def _tail(lens, use_graph=True, min_steps=4, dtype=torch.float32):
    self = SimpleNamespace(use_graph=use_graph, SOLO_MIN_STEPS=min_steps, dtype=dtype)
    clients = [SimpleNamespace(steps=[None] * n) for n in lens]
    return GroupTrainer._solo_tail(self, clients, max(lens))


def test_solo_tail_attacker_outlasts_benign():
    # 9 benign clients with 18 steps, the attacker (index 3) with 54: steps 18..53 run solo
    assert _tail([18, 18, 18, 54, 18, 18, 18, 18, 18, 18]) == (18, 3)


def test_solo_tail_needs_a_long_enough_gap():
    assert _tail([18, 20]) is None                 # 2-step tail: stays in the group graph
    assert _tail([18, 22]) == (18, 1)
    assert _tail([54, 54, 18]) is None             # two clients until the end


def test_solo_tail_off_without_graphs_or_group():
    assert _tail([18, 54], use_graph=False) is None
    assert _tail([54]) is None
    assert _tail([18, 54], min_steps=0) is None
