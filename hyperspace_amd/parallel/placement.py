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

Heavy buckets (``spark.hyperspace.mi.heavyBucketSplit.enabled``, default true).  LPT still
leaves a bucket heavier than total/W on one GPU, bounding every sharded query.  Such a bucket is
cut into key ranges - ``m = ceil(weight / (total/W))`` pieces, split keys taken from the index
files' row-group statistics of the leading indexed column (rows are sorted by it inside a
bucket, so row groups are key ranges) - and the pieces go to distinct ranks in the same LPT
pass.  Every index and shuffle with that bucket count cuts bucket b at the same key values, so
a join on the bucket key stays co-located piece by piece, and every row still has exactly one
owner.  One hot key cannot be cut (its rows are one key range): its bucket stays whole.
"""
from __future__ import annotations

import heapq
import math
import threading
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

BUCKET_PLACEMENT = "spark.hyperspace.mi.bucketPlacement"
BUCKET_PLACEMENT_DEFAULT = "balanced"


class OwnerMap:
    """``owners[b]`` = rank holding bucket b; ``splits[b]`` = (ranks of its key-range pieces,
    the ``len(ranks) - 1`` increasing split keys) for a bucket cut across ranks - piece i holds
    the keys in ``[bounds[i - 1], bounds[i])``, open at both ends - and ``owners[b]`` is then
    its first piece's rank."""
    __slots__ = ("owners", "world", "key", "_luts", "splits", "_unsplit")

    def __init__(self, owners: Sequence[int], world: int,
                 splits: Optional[Dict[int, Tuple[Sequence[int], Sequence[int]]]] = None):
        self.owners = np.asarray(owners, dtype=np.int32)
        self.world = int(world)
        if len(self.owners) and (self.owners.min() < 0 or self.owners.max() >= self.world):
            raise ValueError("OwnerMap: owner outside [0, world)")
        self.splits: Dict[int, Tuple[np.ndarray, np.ndarray]] = {}
        for b, (ranks, bounds) in sorted((splits or {}).items()):
            ranks = np.asarray(ranks, dtype=np.int32)
            bounds = np.asarray(bounds, dtype=np.int64)
            if len(ranks) != len(bounds) + 1 or len(set(ranks.tolist())) != len(ranks) or \
                    (len(bounds) > 1 and not (np.diff(bounds) > 0).all()):
                raise ValueError(f"OwnerMap: bad split of bucket {b}")
            self.splits[int(b)] = (ranks, bounds)
            self.owners[b] = ranks[0]
        self.key = (self.world, self.owners.tobytes(),
                    tuple((b, r.tobytes(), k.tobytes()) for b, (r, k) in self.splits.items()))
        self._luts: Dict[str, object] = {}
        self._unsplit: Optional["OwnerMap"] = None

    def unsplit(self) -> "OwnerMap":
        """This map without key-range cuts: a split bucket lives whole on its first piece's rank.
        The split keys are values of the integer key the cuts were computed from, so a table or
        shuffle whose leading key is of another type (string codes are rank-local, float values
        would truncate) must not route by them; it uses this map instead (``routes_by_key``) -
        every table keyed by that type agrees on it, so joins on such keys stay co-located."""
        if not self.splits:
            return self
        if self._unsplit is None:
            self._unsplit = OwnerMap(self.owners.copy(), self.world)
        return self._unsplit

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

    def owned(self, rank: int) -> List[int]:
        """Buckets rank ``rank`` holds rows of: whole, or a key range (``ranges``)."""
        out = {int(b) for b in np.nonzero(self.owners == rank)[0] if int(b) not in self.splits}
        out |= {b for b, (ranks, _) in self.splits.items() if rank in ranks.tolist()}
        return sorted(out)

    def ranges(self, rank: int) -> Dict[int, Tuple[Optional[int], Optional[int]]]:
        """The key range ``[lo, hi)`` (None: open) rank ``rank`` holds of each split bucket."""
        out = {}
        for b, (ranks, bounds) in self.splits.items():
            for i, r in enumerate(ranks.tolist()):
                if r == rank:
                    out[b] = (int(bounds[i - 1]) if i > 0 else None,
                              int(bounds[i]) if i < len(bounds) else None)
        return out

    def is_modulo(self) -> bool:
        return not self.splits and \
            bool((self.owners == np.arange(len(self.owners)) % self.world).all())

    def loads(self, weights: Sequence[float]) -> np.ndarray:
        """Per-rank total weight under this map (a split bucket's pieces weigh equally)."""
        w = np.asarray(weights, dtype=np.float64)
        out = np.zeros(self.world, dtype=np.float64)
        whole = np.array([b not in self.splits for b in range(len(self.owners))], dtype=bool)
        np.add.at(out, self.owners[whole], w[whole])
        for b, (ranks, _) in self.splits.items():
            out[ranks] += w[b] / len(ranks)
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

    def dest(self, bucket, key=None, valid=None):
        """Destination rank of every row of an int32 bucket-id tensor; rows of a split bucket
        go by their (leading bucketing) key, ``key`` (an integer tensor of the same rows), and a
        row whose key is null (``valid`` == 0) to the bucket's first piece - nulls sort first,
        so an index's null keys are in that piece's key range (``device_cache._cut_buckets``)."""
        if self.is_modulo():
            return bucket % self.world if self.world > 1 else bucket * 0
        out = self.lut(bucket.device).index_select(0, bucket.long())
        if self.splits:
            import torch
            if key is None:
                raise ValueError("OwnerMap.dest: a split bucket routes rows by key")
            k = key.long()
            nonnull = valid.bool() if valid is not None else None
            for b, (ranks, bounds) in self.splits.items():
                m = bucket == b
                if nonnull is not None:
                    m = m & nonnull
                piece = torch.bucketize(k, torch.from_numpy(bounds).to(k.device), right=True)
                r = torch.from_numpy(ranks.astype(np.int64)).to(k.device)[piece].to(out.dtype)
                out = torch.where(m, r, out)
        return out


def routes_by_key(atype) -> bool:
    """Whether rows keyed by a column of arrow type ``atype`` follow a map's key-range cuts:
    integer keys only (the domain split keys are taken from, ``bucket_bounds``)."""
    import pyarrow as pa
    if pa.types.is_dictionary(atype):
        return False
    return pa.types.is_integer(atype)


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


def split_heavy(weights: Sequence[float], world: int,
                bounds_of: Callable[[int, int], Optional[Sequence[int]]],
                slack: float = 1.05, max_piece: float = 0.75) -> OwnerMap:
    """LPT over whole buckets and the key-range pieces of heavy ones: a bucket heavier than
    ``slack`` x total/W asks ``bounds_of(b, m)`` for ``m - 1`` increasing split keys - or
    (keys, each piece's fraction of the rows) - and its pieces go to distinct ranks, weighted
    by their fractions.  None, or a piece keeping more than ``max_piece`` of the rows (a hot
    key), leaves the bucket whole."""
    w = np.asarray(weights, dtype=np.float64)
    world = max(int(world), 1)
    cap = float(w.sum()) / world
    items = []      # (weight, bucket, piece index, pieces)
    cuts: Dict[int, np.ndarray] = {}
    for b in range(len(w)):
        m = min(world, int(math.ceil(w[b] / cap))) if cap > 0 and w[b] > slack * cap else 1
        got = bounds_of(b, m) if m > 1 else None
        bounds, frac = got if isinstance(got, tuple) else (got, None)
        if bounds is not None and len(bounds):
            bounds = np.asarray(bounds, dtype=np.int64)
            m = len(bounds) + 1
            frac = np.full(m, 1.0 / m) if frac is None else np.asarray(frac, dtype=np.float64)
            if frac.max() > max_piece:
                m = 1          # one key range keeps most rows (a hot key): not worth a cut
        else:
            m = 1
        if m > 1:
            cuts[b] = bounds
            items += [(w[b] * frac[i], b, i, m) for i in range(m)]
        else:
            items.append((w[b], b, 0, 1))
    owners = np.zeros(len(w), dtype=np.int32)
    pieces: Dict[int, List[int]] = {}
    loads = [0.0] * world
    for wt, b, i, m in sorted(items, key=lambda x: (-x[0], x[1], x[2])):
        taken = set(pieces.get(b, []))
        r = min((r for r in range(world) if r not in taken), key=lambda r: (loads[r], r))
        loads[r] += wt
        if m == 1:
            owners[b] = r
        else:
            pieces.setdefault(b, []).append(r)
    splits = {b: (pieces[b], cuts[b]) for b in cuts}
    return OwnerMap(owners, world, splits)


def bucket_bounds(files, num_buckets: int, key: str) -> Callable[[int, int], Optional[List[int]]]:
    """``bounds_of(b, m)`` for ``split_heavy`` from an index's bucket files: ``m - 1`` split
    keys of the leading indexed column ``key`` at the row quantiles of bucket b - from the row
    groups' integer minimum statistics when every row group has them (footers only), else
    from the bucket's key column itself (read once, for a heavy bucket only) - or None (no
    integer key, or a single key value).  Every rank reads the same files: identical maps."""
    from ..io.writer import get_bucket_id
    from ..utils import path_utils as P
    by_bucket: Dict[int, list] = {}
    for f in files:
        b = get_bucket_id(P.get_name(f.path))
        if b is not None and 0 <= b < num_buckets:
            by_bucket.setdefault(b, []).append(f.path)

    def from_stats(paths) -> Optional[List[tuple]]:
        import pyarrow.parquet as pq
        starts = []     # (min key, rows) per row group
        for path in paths:
            md = pq.ParquetFile(P.to_local(path)).metadata
            names = [md.schema.column(j).name for j in range(md.num_columns)]
            if key not in names:
                return None
            j = names.index(key)
            for g in range(md.num_row_groups):
                st = md.row_group(g).column(j).statistics
                if st is None or not st.has_min_max or not isinstance(st.min, (int, np.integer)):
                    return None
                starts.append((int(st.min), md.row_group(g).num_rows))
        return starts if len(starts) >= 2 else None

    def bounds_of(b: int, m: int) -> Optional[List[int]]:
        import pyarrow as pa
        import pyarrow.parquet as pq
        paths = sorted(by_bucket.get(b, []))
        if not paths:
            return None
        starts = from_stats(paths)
        vals = None
        if starts is not None:
            starts.sort()
            total = sum(n for _, n in starts)
            cum = np.cumsum([0] + [n for _, n in starts[:-1]])
            cands = [starts[int(np.argmin(np.abs(cum - total * i / m)))][0] for i in range(1, m)]
            lo = starts[0][0]
        else:
            col = pa.concat_arrays([pq.read_table(P.to_local(p), columns=[key]).column(key)
                                    .combine_chunks() for p in paths]) if paths else None
            if col is None or not pa.types.is_integer(col.type) or col.null_count:
                return None
            vals = np.sort(np.asarray(col.to_numpy(), dtype=np.int64))
            if len(vals) < 2:
                return None
            cands = [int(vals[int(len(vals) * i / m)]) for i in range(1, m)]
            lo = int(vals[0])
        out = []
        for k in cands:
            if k > lo and (not out or k > out[-1]):
                out.append(int(k))
        if not out:
            return None
        # each piece's share of the rows: exact from the key column, else from the row groups
        if vals is not None:
            cnt = np.diff(np.concatenate([[0], np.searchsorted(vals, out), [len(vals)]]))
        else:
            ks = np.array([k for k, _ in starts], dtype=np.int64)
            rows = np.array([n for _, n in starts], dtype=np.float64)
            piece = np.searchsorted(np.asarray(out, dtype=np.int64), ks, side="right")
            cnt = np.bincount(piece, weights=rows, minlength=len(out) + 1)
        return out, (cnt / max(float(cnt.sum()), 1.0)).tolist()
    return bounds_of


_LOCK = threading.Lock()


def placement_mode(session) -> str:
    v = str(session.conf.get(BUCKET_PLACEMENT, BUCKET_PLACEMENT_DEFAULT)).lower()
    if v not in ("balanced", "modulo"):
        raise ValueError(f"{BUCKET_PLACEMENT} must be balanced or modulo, got {v}")
    return v


HEAVY_SPLIT = "spark.hyperspace.mi.heavyBucketSplit.enabled"


def session_map(session, num_buckets: int, world: int,
                weights: Optional[Sequence[float]] = None,
                bounds_of: Optional[Callable[[int, int], Optional[Sequence[int]]]] = None
                ) -> OwnerMap:
    """The session's owner map for ``num_buckets`` buckets over ``world`` ranks: decided on its
    first request (``weights``: that index's per-bucket sizes; None or the ``modulo`` mode:
    ``b % world``; ``bounds_of``: split keys of a heavy bucket, ``bucket_bounds``), then
    returned unchanged to every later request."""
    maps = session.__dict__.setdefault("_hs_owner_maps", {})
    mode = placement_mode(session)
    key = (int(num_buckets), int(world), mode)
    with _LOCK:
        m = maps.get(key)
        if m is None:
            if world <= 1 or mode == "modulo" or weights is None or not np.any(weights):
                m = OwnerMap.modulo(num_buckets, world)
            elif bounds_of is not None and \
                    str(session.conf.get(HEAVY_SPLIT, "true")).lower() == "true":
                m = split_heavy(weights, world, bounds_of)
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
