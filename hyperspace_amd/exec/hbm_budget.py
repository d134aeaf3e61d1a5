"""Per-rank memory budgets when several ranks share one MI355X.

One process per GPU is the production layout, but multi-rank rehearsals (gloo, ``LOCAL_RANK %
device_count``) and tests put 2-8 ranks on one device.  Every budget the engine sizes at start
or per build - the HBM arena handed to the caching allocator (``spark.hyperspace.mi.
hbmReserveBytes``), the resident-table cache (``deviceCacheBytes``), a build's working set
(``build.hbmBudgetBytes``) and the pinned host staging pool - was sized as if the rank owned the
device, from an unsynchronized ``mem_get_info``: ranks starting together each saw the whole
device free and reserved up to 64 GB of arena plus a 160 GB cache budget apiece, so four
co-resident ranks could commit more than the 288 GB of HBM between them, and the first
allocation past it killed a rank mid-collective (the round-5 "Connection closed by peer" at the
first ``createIndex`` barrier of the 4-rank tests).

Here every budget is capped by the rank's deterministic share of the device,
``HBM_USABLE x total_memory / ranks_sharing_device`` (the device's total memory, not its
momentary free memory, so co-starting ranks agree), with fixed fractions of the share for the
arena, the cache and a build; a single rank per device keeps the configured values.
``plan(...)`` is pure (no device queries), so the CPU tests check the sums for any sharing.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional

HBM_USABLE = 0.90        # of a device's total memory, for all ranks on it together
ARENA_FRAC = 0.80        # of a rank's share: the engine-start arena (a pool the others carve)
CACHE_FRAC = 0.55        # of a rank's share: resident index tables
BUILD_FRAC = 0.35        # of a rank's share: one build's decoded columns + sort workspace
PINNED_BYTES = 8 << 30   # pinned host staging per device (split among its ranks)


def ranks_sharing_device(local_rank: Optional[int] = None, local_world: Optional[int] = None,
                         ndev: Optional[int] = None) -> int:
    """How many ranks of this node use this rank's device: local ranks map to devices
    ``local_rank % ndev`` (``parallel/dist.py``).  ``LOCAL_WORLD_SIZE`` (torchrun) or, without
    it, ``WORLD_SIZE`` (single-node spawns) gives the node's rank count."""
    env = os.environ
    if local_world is None:
        local_world = int(env.get("LOCAL_WORLD_SIZE") or env.get("WORLD_SIZE") or 1)
    if local_rank is None:
        local_rank = int(env.get("LOCAL_RANK") or env.get("RANK") or 0)
    if ndev is None:
        try:
            import torch
            ndev = torch.cuda.device_count() if torch.cuda.is_available() else 1
        except Exception:  # noqa: BLE001
            ndev = 1
    ndev = max(int(ndev), 1)
    local_world = max(int(local_world), 1)
    mine = local_rank % ndev
    return max(1, sum(1 for r in range(local_world) if r % ndev == mine))


@dataclasses.dataclass(frozen=True)
class RankBudget:
    share: int          # ranks on this device
    rank_bytes: int     # this rank's share of the device's usable HBM
    arena: int          # engine-start arena
    cache: int          # resident-table cache budget
    build_cap: int      # cap of one build's HBM budget
    pinned: int         # pinned host staging pool

    def build(self, configured: int, free_bytes: int) -> int:
        """A build's HBM budget: the configured one (0 = 60% of the free HBM now), capped by
        this rank's share when the device is shared."""
        b = configured if configured > 0 else int(free_bytes * 0.6)
        return b if self.share == 1 else min(b, self.build_cap)


def plan(total_bytes: int, share: int, arena_conf: int, cache_conf: int) -> RankBudget:
    """The budgets of one of ``share`` ranks on a device of ``total_bytes``.  With one rank the
    configured arena and cache stand (the arena is still capped by the device)."""
    share = max(int(share), 1)
    rank = int(total_bytes * HBM_USABLE) // share
    if share == 1:
        return RankBudget(1, rank, min(int(arena_conf), int(rank * ARENA_FRAC)),
                          int(cache_conf), rank, PINNED_BYTES)
    return RankBudget(share, rank, min(int(arena_conf), int(rank * ARENA_FRAC)),
                      min(int(cache_conf), int(rank * CACHE_FRAC)), int(rank * BUILD_FRAC),
                      max(PINNED_BYTES // share, 256 << 20))


_CACHED: dict = {}
# (conf, conf version, device) -> budget: the query path asks per query (gpu_agg._stream_chunks)
# and the rank's environment and the device's size do not change within a process
_FAST: dict = {}


def rank_budget(conf, device=None) -> RankBudget:
    """This process's budgets for ``device`` (the current one by default), from the session
    conf (arena and cache keys) and the device's total memory."""
    fk = (id(conf), getattr(conf, "version", None), device)
    hit = _FAST.get(fk)
    if hit is not None and hit[0] is conf:
        return hit[1]
    from ..utils.conf import HyperspaceConf
    import torch
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    total = int(torch.cuda.get_device_properties(dev).total_memory)
    share = ranks_sharing_device()
    key = (str(dev), total, share, HyperspaceConf.hbm_reserve_bytes(conf),
           HyperspaceConf.device_cache_bytes(conf))
    b = _CACHED.get(key)
    if b is None:
        b = _CACHED[key] = plan(total, share, key[3], key[4])
    if device is not None:      # (the current device may change between calls)
        if len(_FAST) >= 64:
            _FAST.clear()
        _FAST[fk] = (conf, b)
    return b
