"""Per-rank HBM / pinned budgets when ranks share one device (exec/hbm_budget.py).  Four ranks
on one MI355X in the round-5 rehearsal each reserved a 64 GB arena and a 160 GB cache budget
from an unsynchronized ``mem_get_info``; these checks pin that the co-resident ranks' summed
reservations fit the device, for any sharing."""
import pytest

from hyperspace_amd.exec import hbm_budget as HB

GB = 1 << 30
MI355X = 288 * GB
ARENA, CACHE = 64 * GB, 160 * GB      # the configured defaults (index/constants.py)


def test_ranks_sharing_device_follow_local_rank_modulo_devices():
    assert HB.ranks_sharing_device(0, 4, 1) == 4          # 4 ranks on a 1-GPU box
    assert HB.ranks_sharing_device(3, 8, 8) == 1          # one process per GPU
    assert HB.ranks_sharing_device(1, 6, 4) == 2          # ranks 1 and 5 on device 1
    assert HB.ranks_sharing_device(3, 6, 4) == 1


@pytest.mark.parametrize("share", [1, 2, 4, 8, 16])
def test_co_resident_ranks_fit_one_device(share):
    b = HB.plan(MI355X, share, ARENA, CACHE)
    assert b.share == share
    # what the ranks hold at once: each rank's arena, or its cache plus one build in flight
    per_rank = max(b.arena, b.cache + b.build(0, MI355X) if share > 1 else b.arena)
    assert share * per_rank <= MI355X, (share, b)
    assert share * b.arena <= MI355X * HB.HBM_USABLE
    assert share * b.pinned <= HB.PINNED_BYTES or b.pinned == 256 << 20


def test_one_rank_per_device_keeps_the_configured_budgets():
    b = HB.plan(MI355X, 1, ARENA, CACHE)
    assert (b.arena, b.cache) == (ARENA, CACHE)
    assert b.build(0, 100 * GB) == 60 * GB            # 60% of the free HBM, as before
    assert b.build(7 * GB, 100 * GB) == 7 * GB        # an explicit budget stands
    four = HB.plan(MI355X, 4, ARENA, CACHE)
    assert four.arena < ARENA and four.cache < CACHE
    assert four.build(0, 280 * GB) == four.build_cap   # capped by the share, not the free HBM
