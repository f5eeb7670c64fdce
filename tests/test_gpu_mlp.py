"""Persistent LoanNet trainer (``csrc/kernels/mlp.hip``) vs the per-step graph path (GPU only).

One round of the LOAN config (synthetic per-state shards; a benign round and the round where
attacker MO poisons with 10 internal epochs and model replacement) trained both ways from the
same global model: every snapshot (post-phase and pre-scaling), the per-epoch statistics and
the FoolsGold gradient sums agree to fp32 rounding.  The persistent kernel computes the three
linear layers in exact fp32 FMA while the graph path uses the split-fp16 MFMA family, so the
two are not bitwise; the same dropout masks, trigger rows and step order make them agree to
a few ulps per step (reference loan_train.py:98-127).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dba_mod_amd.ops import hip  # noqa: F401  (must load: no silent fallback)
    return torch.device("cuda:0")


def _params(tmp_path, **kw):
    from dba_mod_amd import config as C
    base = {"resumed_model": False, "pretrain_rounds": 0, "synthetic_data": True, "synthetic_train_size": 60000,
            "synthetic_test_size": 4000, "save_model": False, "save_dir": str(tmp_path)}
    base.update(kw)
    return C.load_params(os.path.join(ROOT, "configs", "loan_params.yaml"), base)


def _round(dev, tmp_path, persistent, epoch, agg):
    from dba_mod_amd.fl.server import Server
    from dba_mod_amd.parallel.dist import DistCtx
    s = Server(_params(tmp_path, aggregation_methods=agg), DistCtx(device=dev), write_outputs=False)
    assert s.trainer.persistent, "the LOAN config should take the persistent trainer by default"
    s.trainer.persistent = persistent
    st = s._train_begin(epoch)
    res = {r.name: r for r in st["handle"].collect()}
    return res, max(len(c.steps) for c in st["plan"].clients)


@pytest.mark.parametrize("epoch,agg", [(12, "mean"), (13, "foolsgold")])
def test_persistent_matches_graph_path(dev, tmp_path, epoch, agg):
    a, T = _round(dev, tmp_path / "graph", False, epoch, agg)
    b, _ = _round(dev, tmp_path / "pers", True, epoch, agg)
    assert T > 10 and a.keys() == b.keys()
    for name in a:
        ra, rb = a[name], b[name]
        assert ra.snapshots.keys() == rb.snapshots.keys()
        for k in ra.snapshots:
            x, y = ra.snapshots[k].double(), rb.snapshots[k].double()
            rel = ((x - y).norm() / x.norm()).item()
            assert rel < 1e-4, (name, k, rel)
        # per-epoch (loss sum, correct, count): counts exact, losses to fp32 rounding, correct
        # counts to a row or two per epoch (argmax near-ties)
        assert np.array_equal(ra.stats[:, 2], rb.stats[:, 2]), name
        np.testing.assert_allclose(ra.stats[:, 0], rb.stats[:, 0], rtol=1e-3, atol=1e-3)
        assert np.abs(ra.stats[:, 1] - rb.stats[:, 1]).max() <= 0.002 * max(1.0, ra.stats[:, 2].max()) + 2
        if agg == "foolsgold":
            # the raw-gradient sums see every ReLU near-tie the two arithmetics decide
            # differently (a flipped unit moves its whole row of the layer's gradient), so
            # they agree to ~1e-3 where the weights agree to ~1e-6
            x, y = ra.fg_grad.double(), rb.fg_grad.double()
            assert ((x - y).norm() / x.norm()).item() < 1e-2, name


def test_persistent_is_deterministic(dev, tmp_path):
    a, _ = _round(dev, tmp_path / "a", True, 12, "mean")
    b, _ = _round(dev, tmp_path / "b", True, 12, "mean")
    for name in a:
        for k in a[name].snapshots:
            assert torch.equal(a[name].snapshots[k], b[name].snapshots[k]), (name, k)
        assert np.array_equal(a[name].stats, b[name].stats)


def test_other_batch_size_falls_back(dev, tmp_path):
    """A LOAN run with a batch size the persistent kernel does not take (it is built for the
    reference's 64) trains on the per-step graph path instead of failing mid-round."""
    from dba_mod_amd.fl.server import Server
    from dba_mod_amd.parallel.dist import DistCtx
    s = Server(_params(tmp_path, batch_size=32), DistCtx(device=dev), write_outputs=False)
    assert s.trainer.persistent
    st = s._train_begin(12)
    res = st["handle"].collect()
    assert not s.trainer.persistent and res
    for r in res:
        for v in r.snapshots.values():
            assert torch.isfinite(v).all()
