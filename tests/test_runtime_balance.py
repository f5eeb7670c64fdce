"""Native runtime scheduling helpers (csrc/runtime/runtime.cpp): LPT client placement, the
water-filling split of a round's image-sharded tests, and the contiguous share ranges."""
import numpy as np
import pytest

from dba_mod_amd.utils import native


def test_lpt_assign_deterministic_and_balanced():
    owner, load = native.lpt_assign([54, 16, 16, 15, 14, 16, 12, 16, 18, 16], 4)
    assert owner[0] == 0                      # the longest client opens rank 0
    assert sorted(set(owner)) == [0, 1, 2, 3]
    assert sum(load) == 54 + 16 * 5 + 15 + 14 + 12 + 18
    assert native.lpt_assign([54, 16, 16, 15, 14, 16, 12, 16, 18, 16], 4) == (owner, load)


@pytest.mark.parametrize("base,work", [([5, 1, 1, 0], 4.0), ([100, 1, 1, 0], 4.0), ([0, 0, 0], 9.0),
                                       ([3, 3, 3, 3, 3, 3, 3, 40], 100.0), ([7], 3.0)])
def test_balance_shares_water_filling(base, work):
    sh = native.balance_shares(base, work)
    assert len(sh) == len(base) and abs(sum(sh) - 1.0) < 1e-12 and min(sh) >= 0.0
    fin = [b + s * work for b, s in zip(base, sh)]
    level = max(f for f, s in zip(fin, sh) if s > 0)
    for f, b, s in zip(fin, base, sh):
        if s > 0:
            assert abs(f - level) < 1e-9 * max(1.0, level)   # every receiving rank ends level
        else:
            assert b >= level - 1e-9                         # a rank left out was already above it


def test_balance_shares_no_work_is_even():
    assert native.balance_shares([9, 1, 1, 1], 0.0) == [0.25] * 4


def test_share_ranges_tile_the_list():
    rng = np.random.default_rng(0)
    for n in (0, 1, 7, 9000, 10000):
        for world in (2, 3, 8):
            sh = rng.dirichlet(np.ones(world))
            sh[rng.integers(world)] = 0.0
            sh = (sh / sh.sum()).tolist()
            rs = [native.share_range(n, sh, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[r][1] == rs[r + 1][0] for r in range(world - 1))
            assert all(hi >= lo for lo, hi in rs)
