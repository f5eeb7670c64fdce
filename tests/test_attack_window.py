"""The calibrated synthetic attack window (verdict r4 item 7; ``data/synthetic.py``).

The reference's DBA experiments resume pretrained checkpoints on the real datasets; here the
data are synthetic, so the generator is calibrated until the attack window behaves like the
paper's (``/root/reference/image_helper.py:298-350``: pixel triggers, ``utils/
cifar_params.yaml`` / ``mnist_params.yaml``: four local triggers in rounds 203/205/207/209 and
12/14/16/18, model replacement x100):

* CIFAR: no single local trigger carries the global one (ASR < 80 % after the first poison
  round) and the four compose (>= 90 % after the fourth) — the mechanism is a saturated white
  top row on 15 % of the images, on which the row-0 local triggers are invisible;
* MNIST: the backdoor survives the benign rounds to round 19 — the mechanism is MNIST's empty
  4-pixel border (digits size-normalised into the central 20 x 20 box), which benign data
  never light, so benign updates do not unlearn the trigger rows.

These are DATA-CALIBRATION tests: the ASR bounds pin properties the generator was tuned to
reproduce, not parity with the reference (whose real-data trajectory is not in-tree, so attack
parity is unpinned).  A correct change that makes one trigger land faster fails here only
because the calibration target moved; retune the generator, not the trainer.

CPU tests pin the mechanisms on the generated data and the MNIST trajectory at CPU scale (the
reference backend, a 12k-image subset); the GPU tests pin both full bench windows (the driver's
protocol: 40 warm-start rounds, 5 warm-up rounds, the 8 rounds that hold the four poison rounds).
"""
import json

import numpy as np
import pytest

from dba_mod_amd.data import synthetic


@pytest.fixture(scope="module")
def cifar():
    return synthetic.synthetic_image_pair("cifar", seed=1, train_size=4000, test_size=2000)


@pytest.fixture(scope="module")
def mnist():
    return synthetic.synthetic_image_pair("mnist", seed=1, train_size=4000, test_size=2000)


def test_cifar_sky_hides_only_row0_triggers(cifar):
    for ds in cifar:
        img = ds.images                                   # [N, 32, 32, 3] uint8
        white0 = (img[:, 0] == 255).all(axis=(1, 2))      # whole top row saturated
        assert 0.12 < white0.mean() < 0.18, white0.mean()
        # the band is one row: row 4 (the other two local triggers) is never saturated whole,
        # so triggers 2 / 3 stay visible on every image
        assert not (img[:, 4, :15] == 255).all(axis=(1, 2)).any()
        # and the non-sky images' top rows are ordinary content (a visible white trigger)
        assert (img[~white0, 0, :15] < 255).any(axis=(1, 2)).mean() > 0.99


def test_mnist_trigger_rows_never_lit_by_benign_data(mnist):
    for ds in mnist:
        img = ds.images[..., 0]                           # [N, 28, 28]
        border = np.ones((28, 28), dtype=bool)
        border[4:24, 4:24] = False
        assert img[:, border].max() == 0                  # exactly black, like real MNIST
        # every pixel of the four local triggers (rows 0 / 3, columns 0-3 / 6-9) is in it
        for r, c in [(0, 0), (0, 3), (0, 6), (0, 9), (3, 0), (3, 3), (3, 6), (3, 9)]:
            assert border[r, c]
        assert img[:, 4:24, 4:24].max() > 200             # with bright strokes inside


def _bench(argv, capsys):
    import bench
    assert bench.main(argv) == 0
    line = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1]
    j = json.loads(line)
    return {r: (a, s) for r, a, s in j["rounds"]}


def test_mnist_backdoor_survives_cpu_scale(capsys):
    """MnistNet on the CPU (reference ops) over a 12k / 1k-image subset, 10 warm-start rounds:
    the first attacker's backdoor lands and the global-trigger ASR is still well above the
    clean rate at round 19 (the pre-calibration generator fell to ~7 % on the GPU bench)."""
    r = _bench(["--cpu", "--config", "configs/mnist_params.yaml", "--steps", "8", "--warmup", "2",
                "--pretrain-rounds", "10", "--set", "synthetic_train_size=12000", "synthetic_test_size=1000"], capsys)
    assert r[12][1] > 60, r
    assert r[19][1] > 20, r


@pytest.mark.gpu
def test_cifar_dba_triggers_compose_gpu(capsys):
    """The BASELINE.json bench window on one GPU: ASR < 80 % after the first local trigger,
    >= 90 % after the fourth."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = _bench(["--steps", "8", "--warmup", "5"], capsys)
    assert r[203][1] < 80, r
    assert r[209][1] >= 90 and r[210][1] >= 90, r


@pytest.mark.gpu
def test_mnist_backdoor_survives_to_round_19_gpu(capsys):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = _bench(["--config", "configs/mnist_params.yaml", "--steps", "8", "--warmup", "5"], capsys)
    assert r[12][1] > 60, r
    assert r[19][1] > 30, r
