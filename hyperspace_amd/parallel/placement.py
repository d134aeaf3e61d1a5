"""Bucket -> rank ownership for the sharded placement (one process per MI355X).

Hyperspace's bucketing hashes each row's indexed key to one of ``numBuckets`` buckets
(``CreateActionBase.scala:129-130``) and JoinIndexRule joins two indexes bucket by bucket with no
exchange (``JoinIndexRule.scala:63-69``).  Spread over W GPUs, bucket b must live on the same rank
for every index with that bucket count, or a co-located join would need a shuffle.  The plain
rule ``b % W`` has that property but ignores size: a low-cardinality or skewed key puts one
heavy bucket (and everything else ``b % W`` sends there) on one GPU, which then bounds every
query (the reference FAQ on skew: ``docs/_docs/04-ug-faqs.md:107-132``).

``OwnerMap`` is an explicit table ``owners[b]``.  ``balanced`` assigns buckets by decreasing
weight to the least-loaded rank (LPT; ties to the lower bucket id / rank), so with equal weights
it reproduces ``b % W`` exactly, and a heavy bucket ends up alone on its rank.  The session keeps
ONE map per (bucket count, world) - "sticky": decided from the bucket sizes of the first index
with that bucket count the session queries (index metadata, identical on every rank, so every
rank computes the same map with no collective), then shared by every index and query-time
shuffle with that bucket count, so any two of them stay co-partitioned.  Builds keep writing
bucket ``b`` from rank ``b % W``: which rank writes a bucket file does not matter to queries,
only which rank holds it in HBM.

``spark.hyperspace.mi.bucketPlacement`` = ``balanced`` (default) | ``modulo``.
"""
from __future__ import annotations

import heapq
import threading
from typing import Dict, Optional, Sequence

import numpy as np

BUCKET_PLACEMENT = "spark.hyperspace.mi.bucketPlacement"
BUCKET_PLACEMENT_DEFAULT = "balanced"


class OwnerMap:
    """``owners[b]`` = rank holding bucket b."""
    __slots__ = ("owners", "world", "key", "_luts")

    def __init__(self, owners: Sequence[int], world: int):
        self.owners = np.asarray(owners, dtype=np.int32)
        self.world = int(world)
        if len(self.owners) and (self.owners.min() < 0 or self.owners.max() >= self.world):
            raise ValueError("OwnerMap: owner outside [0, world)")
        self.key = (self.world, self.owners.tobytes())
        self._luts: Dict[str, object] = {}

    @property
    def num_buckets(self) -> int:
        return len(self.owners)

    @staticmethod
    def modulo(num_buckets: int, world: int) -> "OwnerMap":
        return OwnerMap(np.arange(num_buckets, dtype=np.int64) % max(world, 1), max(world, 1))

    @staticmethod
    def balanced(weights: Sequence[float], world: int) -> "OwnerMap":
        return OwnerMap(lpt(weights, world), max(world, 1))

    def owner(self, b: int) -> int:
        return int(self.owners[b])

    def owned(self, rank: int):
        return [int(b) for b in np.nonzero(self.owners == rank)[0]]

    def is_modulo(self) -> bool:
        return bool((self.owners == np.arange(len(self.owners)) % self.world).all())

    def loads(self, weights: Sequence[float]) -> np.ndarray:
        """Per-rank total weight under this map."""
        out = np.zeros(self.world, dtype=np.float64)
        np.add.at(out, self.owners, np.asarray(weights, dtype=np.float64))
        return out

    def lut(self, device):
        """``owners`` as an int32 tensor on ``device`` (cached): dest = lut[bucket]."""
        import torch
        k = str(device)
        t = self._luts.get(k)
        if t is None:
            t = torch.from_numpy(self.owners.copy()).to(device)
            self._luts[k] = t
        return t

    def dest(self, bucket):
        """Destination rank of every row of an int32 bucket-id tensor."""
        if self.is_modulo():
            return bucket % self.world if self.world > 1 else bucket * 0
        return self.lut(bucket.device).index_select(0, bucket.long())


def lpt(weights: Sequence[float], world: int) -> np.ndarray:
    """Longest-processing-time-first assignment: buckets by decreasing weight (ties: lower id
    first) each go to the currently least-loaded rank (ties: lower rank).  Equal weights give
    ``b % world``."""
    w = np.asarray(weights, dtype=np.float64)
    world = max(int(world), 1)
    owners = np.zeros(len(w), dtype=np.int32)
    order = sorted(range(len(w)), key=lambda b: (-w[b], b))
    heap = [(0.0, r) for r in range(world)]
    for b in order:
        load, r = heapq.heappop(heap)
        owners[b] = r
        heapq.heappush(heap, (load + w[b], r))
    return owners


_LOCK = threading.Lock()


def placement_mode(session) -> str:
    v = str(session.conf.get(BUCKET_PLACEMENT, BUCKET_PLACEMENT_DEFAULT)).lower()
    if v not in ("balanced", "modulo"):
        raise ValueError(f"{BUCKET_PLACEMENT} must be balanced or modulo, got {v}")
    return v


def session_map(session, num_buckets: int, world: int,
                weights: Optional[Sequence[float]] = None) -> OwnerMap:
    """The session's owner map for ``num_buckets`` buckets over ``world`` ranks: decided on its
    first request (``weights``: that index's per-bucket sizes; None or the ``modulo`` mode:
    ``b % world``), then returned unchanged to every later request."""
    maps = session.__dict__.setdefault("_hs_owner_maps", {})
    mode = placement_mode(session)
    key = (int(num_buckets), int(world), mode)
    with _LOCK:
        m = maps.get(key)
        if m is None:
            if world <= 1 or mode == "modulo" or weights is None or not np.any(weights):
                m = OwnerMap.modulo(num_buckets, world)
            else:
                m = OwnerMap.balanced(weights, world)
            maps[key] = m
    return m


def bucket_weights(files, num_buckets: int) -> np.ndarray:
    """Per-bucket bytes of an index's bucket files (``..._<bucket:05d>.c000...`` names)."""
    from ..io.writer import get_bucket_id
    from ..utils import path_utils as P
    w = np.zeros(num_buckets, dtype=np.float64)
    for f in files:
        b = get_bucket_id(P.get_name(f.path))
        if b is not None and 0 <= b < num_buckets:
            w[b] += float(f.length)
    return w
