"""MI355X executor: runs physical plans on HIP kernels over HBM-resident tables.

Plans are evaluated into lazy device relations (``DRel``): a device table, an attribute -> column
map, pending filter conjuncts and optional row ranges.  Nothing is materialized until a consumer
needs rows, so the hot shapes compile into single fused launches:

* ``Aggregate <- Filter <- IndexScan``            -> range search + ``hs_scan_agg`` (Q6 shape)
* ``Aggregate <- SortMergeJoin(IndexScan, IndexScan)`` -> ``hs_join_agg`` (co-located, no shuffle)
* ``Filter/Project <- Scan``                       -> ``hs_scan_select`` + ``hs_gather``
* ``SortMergeJoin``                                 -> ``hs_join_count/emit`` + gathers
* ``Exchange(hashpartitioning) <- Scan``           -> Murmur3 + radix sort on the device

Under ``torch.distributed`` each rank owns the buckets the session's owner map gives it
(``parallel/placement.py``: size-balanced, ``b % world`` for equal sizes; co-partitioned, so a
bucketed join needs no data movement); partial aggregates are combined with one RCCL all-reduce
and row results with an all-gather.  Shapes outside the kernel templates raise ``Unsupported``
and the whole query runs on the host oracle (recorded in ``last_path``).
"""
from __future__ import annotations

import logging
import time
from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa

from ..index import constants as C
from ..ops import _lib as NL
from ..ops import kernels as K
from ..plan import expressions as E
from ..plan import physical as X
from ..utils import murmur3
from ..utils.conf import HyperspaceConf
from ..utils.tracing import TRACER, stage
from . import compile as CP
from . import jit, jit_runs, join_index
from .arrow_eval import key
from .device_cache import (DeviceTableCache, _files_key, load_bucketed_index, load_flat,
                           seeded_index)
from .device_table import DeviceColumn, DeviceTable
from .graphs import GraphCache, ScanAggGraph, range_bounds
from .graphs import GraphPending as _GraphPending, _cbuf

log = logging.getLogger(__name__)

# per-wavefront list size of a run top-K aggregate (hash_agg.TopKPlan.K): LIMIT must be below
H_TOPK_K = 32
Unsupported = CP.Unsupported
MAX_GROUPS_SCAN = 3000
MAX_GROUPS_JOIN = 2400
# LDS bytes a dense aggregate's group table may take (32 bytes per group x aggregate: sum, min,
# max, count) beside the rest of the kernel's LDS (160 KiB per CU on gfx950)
GROUP_LDS_SCAN = 144 << 10
GROUP_LDS_JOIN = 112 << 10


def _group_limit(limit: int, lds: int, naggs: int) -> int:
    """Most groups a dense aggregate of ``naggs`` aggregates (+ COUNT(*)) keeps in LDS."""
    return max(1, min(limit, lds // (32 * (naggs + 1))))
# a grouped aggregate with more groups than this returns candidates of ORDER BY ... LIMIT from
# the device top-k instead of copying every group to the host
TOPK_MIN_GROUPS = 4096


class _NeedHash(CP.Unsupported):
    """The dense (LDS) grouped aggregate does not apply; run the hash-mode aggregate
    (exec/hash_agg.py) instead of falling back to the host."""


class DRel:
    def __init__(self, table: DeviceTable, colmap: Dict[int, str], attrs: List[E.Attribute],
                 conds: Optional[list] = None, bucketed: bool = False,
                 sort_attrs: Optional[List[E.Attribute]] = None,
                 bucket_attrs: Optional[List[E.Attribute]] = None, num_buckets: int = 0,
                 parts: Optional[List["DRel"]] = None, split: bool = False):
        self.table = table
        self.colmap = colmap
        self.attrs = attrs
        self.conds = list(conds or [])
        self.bucketed = bucketed
        self.sort_attrs = list(sort_attrs or [])
        self.bucket_attrs = list(bucket_attrs or [])
        self.num_buckets = num_buckets
        # BucketUnion: co-partitioned parts (each sorted within its buckets); table is None
        self.parts = parts
        # distributed: this rank holds a file split of a non-index relation (rows not yet routed
        # to their bucket owners)
        self.split = split
        # computed projection columns of this query (exec/project.py), by colmap name
        self.extra: Dict[str, DeviceColumn] = {}

    def col(self, a: E.Attribute) -> DeviceColumn:
        if self.parts:
            raise Unsupported("column access on a bucket union")
        name = self.colmap.get(a.expr_id)
        if name is None:
            raise Unsupported(f"attribute {a.sql()} not available on device")
        c = self.extra.get(name)
        return c if c is not None else self.table.columns[name]

    def is_computed(self, a: E.Attribute) -> bool:
        return self.colmap.get(a.expr_id) in self.extra

    def copy(self, **kw) -> "DRel":
        d = DRel(self.table, dict(self.colmap), list(self.attrs), list(self.conds), self.bucketed,
                 self.sort_attrs, self.bucket_attrs, self.num_buckets, self.parts, self.split)
        d.extra = dict(self.extra)
        for k, v in kw.items():
            setattr(d, k, v)
        return d


class GpuBackend:
    name = "gpu"
    # QueryExecution may submit a plan-cache entry's own plan with a query's literals bound in
    # place (plan/plan_cache.py): everything literal-dependent is read during collect_async
    supports_bound_plans = True

    def __init__(self, session):
        import torch
        NL.lib()  # fail loudly if the kernels are not built
        self.session = session
        # the generated kernels' tunables: spark.hyperspace.mi.kernel.* over HS_JIT_* over the
        # measured defaults (exec/kernel_config.py)
        from . import kernel_config
        cfg = kernel_config.base().with_conf(session.conf)
        if cfg != kernel_config.active():
            kernel_config.bind(cfg)
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.cache = DeviceTableCache(HyperspaceConf.device_cache_bytes(session.conf))
        self.last_path = None
        self.fallback_reason = None
        self.last_stream_passes = 0      # bucket-range passes of the last aggregate (0: resident)
        self.metrics: Dict[str, float] = {}
        self._cpu = None
        self._domains: Dict[tuple, tuple] = {}
        self._gdomains: Dict[tuple, tuple] = {}   # (table global key, column) -> all-rank domain
        self._unions: Dict[tuple, tuple] = {}     # string join keys: dictionary pair -> union
        self._groups_agreed = False
        self.graphs = GraphCache()
        # plan object id -> (plan, _AggProgram): prepared re-submission of plan-cache hits
        self._programs: Dict[int, tuple] = {}
        self._prog_candidate = None
        from .hash_agg import TablePool
        self.htables = TablePool()
        # engine start: size the pinned staging pool once (pinning GBs is the slow part of a
        # cold build), as the HBM side is sized by the device table cache
        from .staging import pinned_pool
        pinned_pool().reserve()
        self._engine_start()

    def _engine_start(self) -> None:
        """Bring the engine up once, outside any query or build: the HBM arena (one large
        allocation handed back to torch's caching allocator, which later builds and queries
        carve up instead of calling hipMalloc per multi-GB column), the staging threads and
        copy streams, and the kernel code objects."""
        import torch
        from . import staging
        # pyarrow's lazily imported dataset layer (pulled in by the first Parquet read of a
        # build) costs ~0.45 s of one-time import: pay it here, not inside the first build
        import pyarrow.compute  # noqa: F401
        import pyarrow.dataset  # noqa: F401
        import pyarrow.parquet  # noqa: F401
        reserve = HyperspaceConf.hbm_reserve_bytes(self.session.conf)
        if reserve > 0:
            free, _ = torch.cuda.mem_get_info(self.device)
            reserve = min(reserve, int(free * 0.8))
            if reserve > (1 << 30):
                block = torch.empty(reserve, dtype=torch.uint8, device=self.device)
                del block   # stays cached in the allocator as one segment
        pool = staging.io_pool()
        list(pool.map(lambda _: None, range(pool._max_workers)))   # spawn the workers now
        staging.copy_streams(self.device)
        if staging.native_decode_enabled():
            staging._warm_decode_kernels()
        _warm_torch_kernels(self.device)

    # ------------------------------------------------------------------------------------------
    @property
    def cpu(self):
        if self._cpu is None:
            from .cpu import CpuBackend
            self._cpu = CpuBackend(self.session)
        return self._cpu

    def _dist(self):
        """The process group queries run over, or None when this rank answers alone: single
        process, or replicated placement (every rank holds every bucket; builds still shard
        through ``session.dist`` in exec/device_build.py)."""
        d = getattr(self.session, "dist", None)
        if d is not None and HyperspaceConf.index_placement(self.session.conf) == "replicated":
            return None
        return d

    def collect(self, plan: X.SparkPlan) -> pa.Table:
        return self.collect_async(plan).result()

    def collect_async(self, plan: X.SparkPlan) -> "QueryFuture":
        """Submit a query; ``.result()`` returns its table.  Fused aggregates (the indexed
        filter / join hot paths) return before the device finishes, so a caller that keeps
        several queries in flight overlaps host planning with device execution.  A shape the
        device cannot run falls back to the host oracle (recorded in ``path``)."""
        t0 = time.perf_counter()
        hit = self._programs.get(id(plan))
        if hit is not None and hit[0] is plan:
            fut = hit[1].submit(self, plan, t0)
            if fut is not None:
                self.last_path, self.fallback_reason = "native", None
                return fut
        TRACER.configure(self.session.conf)
        self._prog_candidate = None
        try:
            with stage("query"):
                finish = self._collect_native(plan)
            fut = QueryFuture(self, plan, finish, "native", None, t0)
            self._register_program(plan)
        except Unsupported as e:
            fut = self._fallback(plan, e, t0)
        self.last_path, self.fallback_reason = fut.path, fut.reason
        return fut

    def _register_program(self, plan) -> None:
        """After a native submission that ran a prepared lowering (``_ScanPrep`` /
        ``_JoinPrep``) for the plan's top aggregate, keep an ``_AggProgram`` for the plan
        object: a plan-cache hit re-submits the same plan with new literals bound into it, and
        the program replays the prepared kernels / hipGraph directly."""
        cand = self._prog_candidate
        self._prog_candidate = None
        if cand is None or not HyperspaceConf.prepared_submit_enabled(self.session.conf):
            return
        m = self._match_agg(plan)
        if m is None or m[0] is not cand[0]:
            return
        if len(self._programs) >= 256:
            self._programs.clear()
        self._programs[id(plan)] = (plan, _AggProgram(self, *cand))

    def _fallback(self, plan, e, t0) -> "QueryFuture":
        log.info("device executor fallback: %s", e)
        out = self.cpu.collect(plan)
        return QueryFuture(self, plan, lambda: out, "fallback", str(e), t0)

    def _collect_native(self, plan: X.SparkPlan):
        """``finish() -> pa.Table`` of a plan (aggregates deferred, row results computed now).
        ``[CollectLimit] <- [Sort(global) <- Exchange(single)] <- plan``: a grouped aggregate
        below takes the ORDER BY / LIMIT into its device top-k; the final ordering of the (few)
        result rows runs on the host."""
        limit = None
        order = None
        if isinstance(plan, X.CollectLimitExec):
            limit = plan.n
            plan = plan.child
        if isinstance(plan, X.SortExec) and plan.global_sort:
            order = plan.order
            plan = plan.child
            if isinstance(plan, X.ShuffleExchangeExec) and \
                    isinstance(plan.partitioning, X.SinglePartition):
                plan = plan.child
        out_attrs = list(plan.output)
        agg = self._match_agg(plan)
        if agg is not None:
            finish = self._exec_agg(*agg, order=order, limit=limit)
        else:
            self.last_stream_passes = 0
            chunks = self._stream_chunks(plan)
            d = self._dist()
            if chunks is None and order is not None and (d is None or d.world == 1) and \
                    all(isinstance(o.child, E.Attribute) and
                        o.child.expr_id in {a.expr_id for a in out_attrs} for o in order):
                # row ORDER BY on one rank: sorted on the device, no host sort of the rows
                r = self._sort_rel(self._rel(plan), order, True, out_attrs)
                t = self._to_arrow(r, out_attrs)
                if limit is not None:
                    t = t.slice(0, limit)
                return lambda: t
            if chunks is None:
                t = self._to_arrow_ranks(self._rel(plan), plan.output)
            else:
                # rows of an index larger than the HBM budget: bucket range by bucket range,
                # in the bucket-major order of the resident run
                self.last_stream_passes = len(chunks)
                pieces = []
                try:
                    for ch in chunks:
                        self._bucket_chunk = ch
                        self._drop_resident()
                        pieces.append(self._to_arrow_ranks(self._rel(plan), plan.output))
                finally:
                    self._bucket_chunk = None
                    self._drop_resident()
                t = pa.concat_tables(pieces) if len(pieces) > 1 else pieces[0]
            finish = (lambda: t)
        if order is None and limit is None:
            return finish

        def ordered() -> pa.Table:
            t = finish()
            if order is not None:
                t = self._sort_rows(t, out_attrs, order)
            return t if limit is None else t.slice(0, limit)
        return ordered

    def _sort_rows(self, t: pa.Table, attrs, order) -> pa.Table:
        """Host sort of a (small) result table by SortOrders over its output attributes."""
        if t.num_rows <= 1:
            return t
        names = t.column_names
        keyed = t.rename_columns([key(a) for a in attrs])
        return self.cpu._sort_table(keyed, order).rename_columns(names)

    # ------------------------------------------------------------------------------------------
    # Relations
    # ------------------------------------------------------------------------------------------
    def _rel(self, p: X.SparkPlan) -> DRel:
        if isinstance(p, X.FileSourceScanExec):
            return self._scan_memo(p)
        if isinstance(p, X.BucketUnionExec):
            return self._bucket_union(p)
        if isinstance(p, X.ProjectExec):
            sj = self._semi_project(p)
            if sj is not None:
                return sj
        if isinstance(p, (X.FilterExec, X.ProjectExec)):
            r = self._rel(p.child)
            if r.parts:
                parts = [self._unary(p, x) for x in r.parts]
                return r.copy(parts=parts, attrs=list(p.output), colmap=dict(parts[0].colmap))
            return self._unary(p, r)
        if isinstance(p, X.SortExec):
            r = self._rel(p.child)
            if not p.global_sort and r.bucketed and _prefix_sorted(r, [o.child for o in p.order]):
                return r
            return self._sort_rel(r, p.order, p.global_sort, list(p.output))
        if isinstance(p, X.ShuffleExchangeExec) and isinstance(p.partitioning, X.HashPartitioning):
            return self._repartition(self._rel(p.child), p.partitioning)
        if isinstance(p, X.SortMergeJoinExec):
            return self._join_rel(p)
        if isinstance(p, X.UnionExec):
            # UNION ALL: every child's rows (its pending filters applied) concatenated into one
            # flat device relation, columns by position
            out_attrs = list(p.output)
            pieces = []
            for child in p.children:
                r = self._rel(child)
                if r.parts:
                    raise Unsupported("union of a bucket union")
                got = self._materialize(r, list(child.output))
                pieces.append([got[a.expr_id] for a in child.output])
            for ai in range(len(out_attrs)):
                if len({str(x[ai].atype) for x in pieces}) > 1 or \
                        len({x[ai].data.dtype for x in pieces}) > 1:
                    raise Unsupported("union of differently typed columns")
            return self._concat_rels(pieces, out_attrs)
        if isinstance(p, X.ReusedExchangeExec):
            # the device repartition of a resident table is cached, so the original subtree
            # replays the first exchange's result
            return self._rel(p.equivalent)
        raise Unsupported(f"operator {p.node_name}")

    def _sort_rel(self, r: DRel, order, global_sort: bool, attrs) -> DRel:
        """The rows of ``r`` sorted on the device (``K.sort_permutation``: the LSD radix sort of
        csrc/kernels/radix_sort.hip over order-preserving key images): by ``order`` within each
        bucket (a local sort - the result stays bucketed, e.g. a join side Spark would sort
        after its shuffle) or over all rows (a global ORDER BY).  ASC sorts NULLS FIRST; DESC
        sorts NULLS LAST through two keys: a null flag, then the value reversed (``~x`` for
        integers and sorted-dictionary string codes, ``-x`` for floats - NaN, the largest value,
        comes first)."""
        import torch
        if any(not isinstance(o.child, E.Attribute) for o in order):
            raise Unsupported("device sort by an expression")
        if r.parts:
            if not global_sort:
                raise Unsupported("local device sort of a bucket union")
            mats = [self._materialize(x, attrs) for x in r.parts]
            r = self._concat_rels([[m[a.expr_id] for a in attrs] for m in mats], attrs)
        t = r.table
        local = not global_sort and r.bucketed and t.bucket_offsets is not None and \
            t.num_buckets > 1
        rows = self._selected_rows(r) if r.conds else None
        cols = {a.expr_id: (r.col(a) if rows is None else None) for a in attrs}
        if rows is not None:
            got = K.gather_columns([r.col(a) for a in attrs], rows)
            cols = {a.expr_id: c for a, c in zip(attrs, got)}
        n = int(rows.numel()) if rows is not None else int(t.num_rows)
        keys = []
        for o in order:
            c = cols[o.child.expr_id]
            if o.ascending:
                keys.append(c)
                continue
            d = c.data
            if d.dtype.is_floating_point:
                rev = -d
            elif d.dtype == torch.bool:
                rev = (~d).to(torch.uint8)
            else:
                rev = torch.bitwise_not(d)
            if c.valid is not None:
                nullf = (c.valid == 0).to(torch.int32)
                keys.append(DeviceColumn(nullf, None, pa.int32()))
                rev = torch.where(c.valid.bool(), rev, torch.zeros_like(rev))
            keys.append(DeviceColumn(rev.contiguous(), None, c.atype))
        lead = None
        new_off = np.array([0, n], dtype=np.int64)
        if local:
            off = t.bucket_offsets
            if rows is None:
                counts = torch.diff(off)
                bid = torch.repeat_interleave(torch.arange(t.num_buckets, dtype=torch.int32,
                                                           device=self.device), counts)
            else:
                bid = (torch.searchsorted(off[1:], rows, right=True)).to(torch.int32)
            lead = (bid, max(1, int(t.num_buckets - 1).bit_length()))
            cnt = torch.bincount(bid.long(), minlength=t.num_buckets)
            new_off = np.concatenate([[0], np.cumsum(cnt.cpu().numpy())]).astype(np.int64)
        if n > 1:
            perm = K.sort_permutation(keys, extra_leading=lead).long()
            got = K.gather_columns([cols[a.expr_id] for a in attrs], perm)
        else:
            got = [cols[a.expr_id] for a in attrs]
        out = {}
        for a, c in zip(attrs, got):
            c.hs_transient = True
            out[key(a)] = c
        table = DeviceTable(out, n, torch.from_numpy(new_off).to(self.device), new_off)
        asc = all(o.ascending for o in order)
        return DRel(table, {a.expr_id: key(a) for a in attrs}, attrs, [], bucketed=local,
                    sort_attrs=[o.child for o in order] if asc else [],
                    bucket_attrs=r.bucket_attrs if local else [],
                    num_buckets=r.num_buckets if local else 0)

    def _holds(self, t) -> bool:
        """Whether resident table ``t`` is still current: in the device cache, or derived from
        tables that are (a merged Hybrid Scan union, a cached repartition of appended rows)."""
        src = getattr(t, "_hs_sources", None)
        if src is not None:
            return all(self._holds(x) for x in src)
        return self.cache.holds(t)

    def _bucket_union(self, p: X.BucketUnionExec) -> DRel:
        nb = p.bucket_spec.num_buckets
        parts = []
        for child in p.children:
            r = self._rel(child)
            if r.parts or not r.bucketed or r.num_buckets != nb:
                raise Unsupported("bucket union of non co-partitioned inputs")
            colmap = dict(r.colmap)
            for u, c in zip(p.output, child.output):   # BucketUnion output = child 0's attrs
                if c.expr_id in r.colmap:
                    colmap[u.expr_id] = r.colmap[c.expr_id]
            parts.append(r.copy(colmap=colmap))
        first = parts[0]
        merged = self._merged_union(p, parts, [c.output for c in p.children])
        if merged is not None:
            return merged
        return DRel(None, dict(first.colmap), list(p.output), [], True, first.sort_attrs,
                    first.bucket_attrs, nb, parts)

    @staticmethod
    def _union_conds(p: X.BucketUnionExec, parts: List[DRel], outputs):
        """(predicates, extra attributes) when every part carries the same pending predicates (a
        filter pushed below the union into each child), over the union's output attributes plus
        ``extra``: columns the filter reads that a projection above it dropped, present under
        the same attribute in every part (a Hybrid Scan's branches share the relation's
        attributes).  None when the parts' predicates differ."""
        keys, conds0 = None, None
        extra: Dict[int, E.Attribute] = {}
        for x, out in zip(parts, outputs):
            sub = {c.expr_id: u for u, c in zip(p.output, out)}
            missing = []

            def ren(e, sub=sub, missing=missing, x=x):
                if isinstance(e, E.Attribute):
                    u = sub.get(e.expr_id)
                    if u is None:
                        if all(e.expr_id in y.colmap for y in parts):
                            extra.setdefault(e.expr_id, e)
                            return e
                        missing.append(e)
                    return u
                return None
            conds = [c.transform_up(ren) for c in x.conds]
            if missing:
                return None
            k = sorted(repr(c.canonical_key()) for c in conds)
            if keys is None:
                keys, conds0 = k, conds
            elif k != keys:
                return None
        return conds0, list(extra.values())

    def _merged_union(self, p: X.BucketUnionExec, parts: List[DRel],
                      outputs=None) -> Optional[DRel]:
        """A Hybrid Scan's bucket union as ONE resident table: the index rows and the appended
        rows (already bucketed and sorted by the device shuffle) of every bucket merged into
        bucket-major order sorted by the index key, built once per (index table, appended
        table) and kept while both stay resident - so queries over an index with appended
        files take the single-table paths (prepared lowering, graph replays, the run-keyed
        merge join) instead of one launch per (part, part) pair.  None when the parts carry
        their own predicates (a deleted-files filter), computed columns, differently encoded
        columns, or would take more than a quarter of the device cache."""
        import torch
        conf = self.session.conf

        def skip(why: str):
            self.metrics["hybrid_merge_skip"] = why
            return None
        if str(conf.get("spark.hyperspace.mi.hybridMerge.enabled", "true")).lower() != "true":
            return skip("disabled")
        d = self._dist()
        if d is not None and d.world > 1:
            return skip("world > 1")
        for x in parts:
            if x.table is None or x.extra or x.split or x.parts:
                return skip("part: " + ", ".join(
                    n for n, v in (("no table", x.table is None), ("extra", x.extra),
                                   ("split", x.split), ("parts", x.parts)) if v))
        # the same filter in every part (pushed below the union) applies to the merged rows
        uc = self._union_conds(p, parts, outputs) if outputs is not None else \
            (([], []) if not any(x.conds for x in parts) else None)
        if uc is None:
            return skip("parts carry different predicates")
        conds, extra = uc
        first = parts[0]
        visible = list(p.output)
        outs = visible + [a for a in extra if a.expr_id not in {u.expr_id for u in visible}]
        ids = {u.expr_id for u in outs}
        if not first.sort_attrs or any(a.expr_id not in ids for a in first.sort_attrs):
            return skip("sort attributes not in the output")
        key = tuple(id(x.table) for x in parts) + tuple(u.expr_id for u in outs)
        memo = self.__dict__.setdefault("_hybrid_unions", {})
        hit = memo.get(key)
        if hit is not None and all(a is b for a, b in zip(hit[0], [x.table for x in parts])) \
                and self._holds(hit[1]):
            table = hit[1]
        else:
            cols = []
            for u in outs:
                cs = [x.col(u) for x in parts]
                c0 = cs[0]
                if any(c.data.dtype != c0.data.dtype or str(c.atype) != str(c0.atype) or
                       c.offsets is not None or
                       (c.dictionary is None) != (c0.dictionary is None) or
                       (c.dictionary is not None and not c.dictionary.equals(c0.dictionary))
                       for c in cs):
                    return skip(f"column {u.name}: parts differ in type or dictionary")
                cols.append(cs)
            nbytes = sum(c.data.numel() * c.data.element_size() for cs in cols for c in cs)
            if nbytes > HyperspaceConf.device_cache_bytes(conf) // 4:
                return skip("over a quarter of the device cache")
            nb = first.num_buckets
            with stage("hybrid.merge"):
                bucket = torch.cat([torch.repeat_interleave(
                    torch.arange(nb, dtype=torch.int32, device=self.device),
                    x.table.bucket_offsets[1:] - x.table.bucket_offsets[:-1]) for x in parts])
                merged = {}
                for j, cs in enumerate(cols):
                    data = torch.cat([c.data for c in cs])
                    valid = None
                    if any(c.valid is not None for c in cs):
                        valid = torch.cat([c.valid if c.valid is not None else
                                           torch.ones(c.data.shape[0], dtype=torch.uint8,
                                                      device=self.device) for c in cs])
                    merged[f"u{j}"] = DeviceColumn(data, valid, cs[0].atype, cs[0].dictionary)
                pos = {u.expr_id: j for j, u in enumerate(outs)}
                keys = [merged[f"u{pos[a.expr_id]}"] for a in first.sort_attrs]
                perm = K.sort_permutation(keys, extra_leading=(bucket, 16))
                names = list(merged)
                gathered = K.gather_columns([merged[n] for n in names], perm)
                off_host = sum(np.asarray(x.table.bucket_offsets_host, dtype=np.int64) for x in parts)
                n = int(off_host[-1])
                table = DeviceTable(dict(zip(names, gathered)), n,
                                    torch.from_numpy(off_host).to(self.device), off_host)
            table._hs_sources = [x.table for x in parts]
            table._hs_cache_key = ("hybrid-union",) + key
            table.global_key = ("hybrid-union",) + tuple(
                getattr(x.table, "global_key", None) for x in parts)
            if len(memo) > 8:
                memo.clear()
            memo[key] = ([x.table for x in parts], table)
        self.metrics.pop("hybrid_merge_skip", None)
        colmap = {u.expr_id: f"u{j}" for j, u in enumerate(outs)}
        return DRel(table, colmap, visible, conds, True, first.sort_attrs, first.bucket_attrs,
                    first.num_buckets)

    def _unary(self, p: X.SparkPlan, r: DRel) -> DRel:
        if isinstance(p, X.FilterExec):
            conds = E.split_conjuncts(p.condition)
            computed = [c for c in conds if _needs_eval(c)]
            if not computed:
                return r.copy(conds=r.conds + conds)
            # conjuncts over computed values (``a * 2 > 500``, pushed below a projection by the
            # optimizer): one generated kernel evaluates them to 0/1 columns, and the scan
            # kernels test those like any column
            from . import project
            out = r.copy()
            refs = {a.expr_id: r.col(a) for c in computed for a in c.references()}
            n = r.table.num_rows if r.table.num_rows is not None else \
                len(next(iter(r.table.columns.values())))
            with stage("project"):
                vals = project.evaluate([E.Cast(c, pa.int8()) for c in computed], refs, n,
                                        self.device)
            rest = [c for c in conds if not _needs_eval(c)]
            for c, v in zip(computed, vals):
                v.hs_transient = True
                at = E.Attribute(f"__hs_pred", pa.int8(), True)
                name = f"__hs_pred_{at.expr_id}"
                out.colmap[at.expr_id] = name
                out.extra[name] = v
                rest.append(E.GreaterThan(at, E.Literal(0)))
            out.conds = r.conds + rest
            return out
        if isinstance(p, X.ProjectExec):
            colmap = dict(r.colmap)
            attrs = []
            computed = []
            for e in p.project_list:
                if isinstance(e, E.Attribute):
                    attrs.append(e)
                elif isinstance(e, E.Alias) and isinstance(e.child, E.Attribute):
                    if e.child.expr_id not in colmap:
                        raise Unsupported("alias of unknown column")
                    colmap[e.expr_id] = colmap[e.child.expr_id]
                    attrs.append(e.to_attribute())
                elif isinstance(e, E.Alias):
                    computed.append(e)
                    attrs.append(e.to_attribute())
                else:
                    raise Unsupported("computed projection without a name")
            out = r.copy(colmap=colmap, attrs=attrs)
            if computed:
                # one generated elementwise kernel over the relation's rows (pending filters
                # still apply afterwards, on the computed columns too)
                from . import project
                refs = {a.expr_id: r.col(a) for e in computed for a in e.child.references()}
                n = r.table.num_rows if r.table.num_rows is not None else \
                    len(next(iter(r.table.columns.values())))
                with stage("project"):
                    vals = project.evaluate([e.child for e in computed], refs, n, self.device)
                for e, c in zip(computed, vals):
                    c.hs_transient = True     # per query: no domain / encoding caches
                    name = f"__hs_expr_{e.expr_id}"
                    colmap[e.expr_id] = name
                    out.extra[name] = c
            return out
        raise Unsupported(f"operator {p.node_name}")

    def _scan_memo(self, p: X.FileSourceScanExec) -> DRel:
        """``_scan`` of a plan leaf, reused while the device cache still holds its table: a
        plan-cache hit re-runs the same scan nodes with new literals above them, so the file
        listing, placement and cache-key work of the scan happen once per (node, placement)."""
        d = self._dist()
        tag = (d.rank, d.world, self.session.conf.get(
            "spark.hyperspace.mi.bucketPlacement", "balanced")) if d is not None else None
        tag = (tag, getattr(self, "_bucket_chunk", None))
        memo = self.__dict__.setdefault("_scans", {})
        m = memo.get(id(p))
        if m is not None and m[0] is p and m[2] == tag and m[1].table is not None and \
                self._holds(m[1].table):
            return m[1].copy()
        r = self._scan(p)
        if getattr(r.table, "_hs_cache_key", None) is not None:
            if len(memo) > 256:
                memo.clear()
            memo[id(p)] = (p, r, tag)
            return r.copy()
        return r

    def _scan(self, p: X.FileSourceScanExec, files=None, bucketed: Optional[bool] = None) -> DRel:
        """The device relation of a scan leaf: its index bucket files as a bucket-sorted table,
        anything else as a flat table.  ``files`` / ``bucketed``: a subset of the leaf's files
        and which path it takes (``_mixed_index_agg``)."""
        rel = p.relation
        if files is None:
            files = rel.location.all_files()
        d = self._dist()
        rank, world = (d.rank, d.world) if d is not None else (0, 1)
        names = [a.name for a in p.output]
        if bucketed is None:
            bucketed = rel.is_index() and \
                self._all_bucket_files(rel.location, files, rel.index.num_buckets)
        if bucketed:
            idx = rel.index
            ncol = {n.lower(): n for n in idx.schema.names}
            cols = [ncol[a.name.lower()] for a in p.output]
            sort_cols = [ncol[c.lower()] for c in idx.indexed_columns]
            load_cols = list(dict.fromkeys(cols + sort_cols))
            owners = self._owner_map(idx.num_buckets, world, files)
            owned = owners.owned(rank)
            chunk = getattr(self, "_bucket_chunk", None)
            if chunk is not None:
                # bucket-range streaming (_streamed_agg): this pass holds buckets [lo, hi) only
                owned = [b for b in owned if chunk[0] <= b < chunk[1]]
            table = self.cache.get(
                files, load_cols, ("bucketed", rank, world, owners.key, chunk),
                lambda: seeded_index(files, load_cols, idx.num_buckets, rank, world, owned) or
                load_bucketed_index(files, load_cols, idx.num_buckets, sort_cols, self.device,
                                    rank, world, owned))
            # rank-independent identity (every rank scans the same file list)
            table.global_key = ("bucketed", _files_key(files), tuple(load_cols), world)
            colmap = {a.expr_id: c for a, c in zip(p.output, cols)}
            sort_attrs = []
            for c in sort_cols:
                a = next((x for x in p.output if x.name.lower() == c.lower()), None)
                if a is None:
                    a = E.Attribute(c, idx.schema.field(c).type)
                    colmap[a.expr_id] = c
                sort_attrs.append(a)
            return DRel(table, colmap, list(p.output), [], True, sort_attrs, sort_attrs,
                        idx.num_buckets)
        fmt = "parquet" if (rel.is_index() or rel.file_format == "delta") else rel.file_format
        gkey = ("flat", _files_key(files), tuple(names), world)
        if world > 1:
            # a file split per rank, like Spark's scan tasks; a following hash Exchange moves rows
            # to their owners with an all-to-all (_repartition), aggregates all-reduce
            files = sorted(files, key=lambda f: f.path)[rank::world]
        table = self.cache.get(files, names, ("flat", fmt, rank, world),
                               lambda: load_flat(files, fmt, names, rel.data_schema, rel.options,
                                                 rel.location.partition_spec, self.device))
        table.global_key = gkey
        return DRel(table, {a.expr_id: a.name for a in p.output}, list(p.output),
                    split=world > 1)

    def _owner_map(self, num_buckets: int, world: int, files=None):
        """The session's bucket -> rank map for this bucket count (parallel/placement.py):
        size-balanced from the first index queried with it, shared by every later index and
        query-time shuffle with that bucket count (co-partitioned)."""
        from ..parallel.placement import bucket_weights, session_map
        if world <= 1:
            return session_map(self.session, num_buckets, 1)
        w = bucket_weights(files, num_buckets) if files is not None else None
        return session_map(self.session, num_buckets, world, w)

    @staticmethod
    def _all_bucket_files(location, files, nb) -> bool:
        v = getattr(location, "_hs_all_bucket_files", None)
        if v is None or v[0] != nb:
            from ..io.writer import get_bucket_id
            from ..utils import path_utils as P
            ok = True
            for f in files:
                b = get_bucket_id(P.get_name(f.path))
                if b is None or b >= nb:
                    ok = False
                    break
            v = (nb, ok)
            location._hs_all_bucket_files = v
        return v[1]

    # -- lowering helpers ----------------------------------------------------------------------
    def _ranges(self, r: DRel, conds: list, implied: Optional[set] = None):
        """Row ranges after bucket / sort-key pruning on the leading indexed column.

        When ``implied`` is given it receives ``id(c)`` of every conjunct the ranges already
        guarantee (comparisons of the sort key with literals, and ``isnotnull(key)`` since range
        search skips the null prefix), so kernels do not re-evaluate them per row."""
        spec = self._range_spec(r, conds, implied)
        if spec is None:
            return self._full_ranges(r.table)
        kc, lo, lo_incl, hi, hi_incl, buckets = spec
        return K.range_search(kc, r.table.bucket_offsets, buckets, lo, lo_incl, hi, hi_incl)

    def _range_spec(self, r: DRel, conds: list, implied: Optional[set] = None):
        """(key column, lo, lo_incl, hi, hi_incl, buckets) of the range search ``_ranges``
        runs, or None when every row of every bucket is in range."""
        t = r.table
        if not (r.bucketed and r.sort_attrs):
            return None
        lead = r.sort_attrs[0]
        kc = r.col(lead)
        lo = hi = None
        lo_incl = hi_incl = True
        eq_bucket = None
        used = []
        notnull = [c for c in conds if isinstance(c, E.IsNotNull) and
                   isinstance(c.child, E.Attribute) and c.child.expr_id == lead.expr_id]
        for c in conds:
            if not isinstance(c, E.BinaryComparison) or isinstance(c, E.NotEqual):
                continue
            leaf = None
            try:
                leaf = CP._leaf(c)
            except Unsupported:
                continue
            if leaf.kind != "cmp_lit" or leaf.attr.expr_id != lead.expr_id or leaf.value is None:
                continue
            v = leaf.value
            if kc.dictionary is not None or isinstance(v, str):
                continue
            if kc.is_float:
                v = float(v)
            elif isinstance(v, float):
                if not float(v).is_integer():
                    continue
                v = int(v)
            img = K.sortable_image(v, kc.hs_type)
            used.append(c)
            if leaf.op in (NL.OP_GT, NL.OP_GE, NL.OP_EQ):
                inc = leaf.op != NL.OP_GT
                if lo is None or img > lo or (img == lo and not inc):
                    lo, lo_incl = img, inc
            if leaf.op in (NL.OP_LT, NL.OP_LE, NL.OP_EQ):
                inc = leaf.op != NL.OP_LT
                if hi is None or img < hi or (img == hi and not inc):
                    hi, hi_incl = img, inc
            if leaf.op == NL.OP_EQ and len(r.bucket_attrs) == 1 and not kc.is_float:
                eq_bucket = self._bucket_of_literal(leaf.value, lead.data_type, r.num_buckets)
        buckets = None
        if eq_bucket is not None:
            import torch
            buckets = torch.tensor([eq_bucket], dtype=torch.int32, device=self.device)
        if lo is None and hi is None and buckets is None:
            if notnull and kc.valid is None:
                # isnotnull(key) on a key column without nulls: the full ranges already satisfy
                # it (and stay the cached full-range object, which keys cached join spans)
                if implied is not None:
                    implied.update(id(c) for c in notnull)
                return None
            if not notnull:
                return None
        if implied is not None:
            implied.update(id(c) for c in used + notnull)
        return kc, lo, lo_incl, hi, hi_incl, buckets

    def _full_ranges(self, t: DeviceTable):
        fr = getattr(t, "_full_ranges", None)
        if fr is None:
            fr = K.full_ranges(t.bucket_offsets_host, self.device)
            t._full_ranges = fr
        return fr

    @staticmethod
    def _bucket_of_literal(v, dtype, nb) -> int:
        arr = pa.array([v], type=dtype)
        return int(murmur3.bucket_ids([arr], nb)[0])

    def _column_infos(self, rels_slots):
        """rels_slots: list of (DRel, slot_base). Returns col_info(attr) and the ColDesc list."""
        slot_map: Dict[int, int] = {}
        descs: Dict[int, DeviceColumn] = {}
        counters = {base: 0 for _, base in rels_slots}

        def col_info(a: E.Attribute) -> CP.ColumnInfo:
            if a.expr_id not in slot_map:
                for rel, base in rels_slots:
                    if a.expr_id in rel.colmap:
                        i = counters[base]
                        limit = 8 if len(rels_slots) > 1 else NL.MAX_COLS
                        if i >= limit:
                            raise Unsupported("too many columns for one kernel")
                        counters[base] = i + 1
                        slot_map[a.expr_id] = base + i
                        descs[base + i] = rel.col(a)
                        break
                else:
                    raise Unsupported(f"unknown column {a.sql()}")
            s = slot_map[a.expr_id]
            c = descs[s]
            return CP.ColumnInfo(s, c.hs_type, c.atype, c.dictionary)
        return col_info, descs

    # ------------------------------------------------------------------------------------------
    # Materialization
    # ------------------------------------------------------------------------------------------
    def _materialize(self, r: DRel, attrs: List[E.Attribute]) -> Dict[int, DeviceColumn]:
        """Apply pending predicates; return expr_id -> gathered DeviceColumn."""
        if r.parts:
            raise Unsupported("materialize a bucket union")
        if not r.conds:
            t = r.table
            full = t.num_rows
            return {a.expr_id: r.col(a) for a in attrs} if full is not None else {}
        rows = self._selected_rows(r, attrs)
        cols = [r.col(a) for a in attrs]
        g = K.gather_columns(cols, rows)
        return {a.expr_id: c for a, c in zip(attrs, g)}

    def _selected_rows(self, r: DRel, attrs: List[E.Attribute] = ()):
        """Row ids (int64, ascending) of ``r``'s rows that pass its pending predicates."""
        implied: set = set()
        rstart, rlen, _ = self._ranges(r, r.conds, implied)
        col_info, descs = self._column_infos([(r, 0)])
        bound = CP.bind(CP.to_cnf([c for c in r.conds if id(c) not in implied]), col_info,
                        self.device)
        for a in attrs:
            col_info(a)
        p = NL.ScanParams()
        for s, c in descs.items():
            p.cols[s] = c.desc()
        for i, pr in enumerate(bound.preds):
            p.preds[i] = pr
        p.npreds = len(bound.preds)
        p.naggs, p.group_col = 0, -1
        import torch
        if bound.always_false:
            rows = torch.empty(0, dtype=torch.int64, device=self.device)
        else:
            tp = K.ranges_to_tiles(rlen)
            max_tiles = r.table.num_rows // NL.lib().hs_scan_tile_rows() + rlen.numel() + 1
            rows = K.scan_select(p, rstart, rlen, tp, max_tiles)
        return rows

    # a filtered right side drives the join when it keeps fewer than 1 / PROBE_RATIO of the left
    # rows; only tried when the right table itself is this much smaller than the left
    PROBE_RATIO = 64
    PROBE_MAX = 1 << 20

    def _probe_ranges(self, left: DRel, right: DRel, lk, rk):
        """Key-probe ranges of ``left`` for a selective, filtered ``right`` (a dimension filtered
        down to a few keys against a large fact index sorted by the join key): the right rows
        passing their predicates are selected first, and each distinct (bucket, key) of them
        becomes one equality range search in the left's bucket, so the join scans only the
        matching key runs of the left instead of every left row.  None when the shape does not
        qualify (then the left's own ranges drive the join).  Left-side predicates are not
        applied by these ranges; the caller evaluates all of them per row."""
        import torch
        if left.parts or right.parts or not right.conds or not left.bucketed:
            return None
        nl, nr = left.table.num_rows or 0, right.table.num_rows or 0
        if nl < (1 << 20) or nr * 8 > nl:
            return None
        lc, rc = left.col(lk), right.col(rk)
        if lc.is_float or rc.is_float or lc.dictionary is not None or \
                rc.dictionary is not None or lc.offsets is not None:
            return None
        width = {NL.I8: 8, NL.I16: 16, NL.I32: 32, NL.I64: 64}.get(lc.hs_type)
        if width is None or rc.hs_type not in (NL.I8, NL.I16, NL.I32, NL.I64):
            return None
        # a pair whose filtered side turned out not selective twice is not probed again (the
        # selection costs a scan of the right side and a host sync per query)
        pk_ = (id(left.table), id(right.table))
        misses = self.__dict__.setdefault("_probe_misses", {})
        if misses.get(pk_, 0) >= 2:
            return None
        with stage("join.probe_select"):
            rows = self._selected_rows(right)
            npass = int(rows.numel())
        if npass * self.PROBE_RATIO > nl or npass > self.PROBE_MAX:
            if len(misses) > 4096:
                misses.clear()
            misses[pk_] = misses.get(pk_, 0) + 1
            return None
        with stage("join.probe_ranges"):
            g = K.gather_columns([rc], rows)[0]
            vals = g.data.to(torch.int64).cpu().numpy()
            ok = np.ones(len(vals), dtype=bool)
            if g.valid is not None:
                ok &= g.valid.cpu().numpy().astype(bool)
            rows_h = rows.cpu().numpy()
            off = right.table.bucket_offsets_host
            bk = np.searchsorted(off, rows_h, side="right") - 1
            lo, hi = -(1 << (width - 1)), (1 << (width - 1)) - 1
            ok &= (vals >= lo) & (vals <= hi)
            vals, bk = vals[ok], bk[ok]
            if width == 64:
                u = (vals.view(np.uint64) ^ np.uint64(1 << 63))
            else:
                u = (vals + (1 << (width - 1))).astype(np.uint64)
            probes = np.unique(np.stack([bk.astype(np.uint64), u], axis=1), axis=0) \
                if len(u) else np.zeros((0, 2), np.uint64)
            self.last_join_probes = len(probes)
            pb = torch.from_numpy(probes[:, 0].astype(np.int32)).to(self.device)
            pk = torch.from_numpy(probes[:, 1].view(np.int64).copy()).to(self.device)
            if len(probes) == 0:
                z = torch.zeros(0, dtype=torch.int64, device=self.device)
                return z, z.clone(), torch.zeros(0, dtype=torch.int32, device=self.device)
            return K.probe_ranges(lc, left.table.bucket_offsets, pb, pk)

    def _domain_pruned_ranges(self, left: DRel, right: DRel, lk, rk):
        """Left ranges restricted to the right join key's [min, max] when that domain is
        narrower than the left's (a zone-map join filter on the sorted left key): e.g. the
        Hybrid Scan pair (index lineitem, appended orders) whose keys are disjoint costs a range
        search instead of a scan.  None when the left has its own key ranges, the shape is not
        integer / resident, or the domains do not prune."""
        if left.parts or right.parts or not left.bucketed or not left.sort_attrs:
            return None
        if self._range_spec(left, left.conds) is not None:
            return None
        lc, rc = left.col(lk), right.col(rk)
        if lc.is_float or rc.is_float or lc.dictionary is not None or \
                rc.dictionary is not None or lc.hs_transient or rc.hs_transient:
            return None
        width = {NL.I8: 8, NL.I16: 16, NL.I32: 32, NL.I64: 64}.get(lc.hs_type)
        if width is None or rc.hs_type not in (NL.I8, NL.I16, NL.I32, NL.I64):
            return None
        llo, lspan = self._local_domain(lc)
        rlo, rspan = self._local_domain(rc)
        if lspan == 0:
            return None
        lhi, rhi = llo + lspan - 1, rlo + rspan - 1
        if rspan > 0 and rlo <= llo and rhi >= lhi:
            return None                     # the right covers the left's keys: nothing to prune
        import torch
        tmin, tmax = -(1 << (width - 1)), (1 << (width - 1)) - 1
        if rspan == 0 or rlo > min(lhi, tmax) or rhi < max(llo, tmin):
            z = torch.zeros(0, dtype=torch.int64, device=self.device)
            return z, z.clone(), torch.zeros(0, dtype=torch.int32, device=self.device)
        lo = K.sortable_image(max(rlo, tmin), lc.hs_type)
        hi = K.sortable_image(min(rhi, tmax), lc.hs_type)
        with stage("join.domain_prune"):
            return K.range_search(lc, left.table.bucket_offsets, None, lo, True, hi, True)

    def _to_arrow(self, r: DRel, out_attrs: List[E.Attribute]) -> pa.Table:
        if r.parts:  # rows of a bucket union: each part's rows, concatenated
            return pa.concat_tables([self._to_arrow(x, out_attrs) for x in r.parts])
        cols = self._materialize(r, out_attrs)
        arrays = [cols[a.expr_id].to_arrow() for a in out_attrs]
        fixed = []
        for a, arr in zip(out_attrs, arrays):
            if not arr.type.equals(a.data_type):
                try:
                    arr = arr.cast(a.data_type)
                except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                    pass
            fixed.append(arr)
        return pa.Table.from_arrays(fixed, names=[a.name for a in out_attrs])

    def _to_arrow_ranks(self, r: DRel, out_attrs: List[E.Attribute]) -> pa.Table:
        """Rows of ``r`` from every rank (sharded placement): this rank's rows are materialized
        as device columns (bucket-union parts concatenated, their string dictionaries unified)
        and cross ranks with one packed device all-gather (``parallel/gather.py``) — no
        pickled tables."""
        d = self._dist()
        if d is None or d.world == 1:
            return self._to_arrow(r, out_attrs)
        import torch
        from ..parallel.gather import gather_device_columns
        parts = r.parts or [r]
        mats = [self._materialize(x, out_attrs) for x in parts]
        cols = []
        for a in out_attrs:
            cs = [m[a.expr_id] for m in mats]
            if len(cs) == 1:
                cols.append(cs[0])
                continue
            dicts = [c.dictionary for c in cs]
            if any(x is not None for x in dicts):
                import pyarrow.compute as pc
                from ..parallel.dictionary import remap_table
                union = pc.unique(pa.concat_arrays([x.cast(pa.string()) for x in dicts])).sort()
                datas = []
                for c in cs:
                    t_ = torch.from_numpy(remap_table(c.dictionary, union)).to(self.device)
                    datas.append(K.lookup_i32(t_, c.data) if len(c.dictionary) and len(c)
                                 else torch.zeros_like(c.data))
            else:
                union, datas = None, [c.data for c in cs]
            valid = None
            if any(c.valid is not None for c in cs):
                valid = torch.cat([c.valid if c.valid is not None else
                                   torch.ones(len(c), dtype=torch.uint8, device=self.device)
                                   for c in cs])
            cols.append(DeviceColumn(torch.cat(datas), valid, cs[0].atype, union))
        n = len(cols[0]) if cols else 0
        with stage("rows.gather_ranks"):
            allc = gather_device_columns(d, cols, n)
        arrays = []
        for a, c in zip(out_attrs, allc):
            arr = c.to_arrow()
            if not arr.type.equals(a.data_type):
                try:
                    arr = arr.cast(a.data_type)
                except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                    pass
            arrays.append(arr)
        return pa.Table.from_arrays(arrays, names=[a.name for a in out_attrs])

    # ------------------------------------------------------------------------------------------
    # Repartition (device shuffle for non-index inputs)
    # ------------------------------------------------------------------------------------------
    def _repartition(self, r: DRel, part: X.HashPartitioning) -> DRel:
        """Hash Exchange (K3) on the device: Spark-compatible Murmur3 bucket ids, then one
        (bucket, keys) sort so the result is bucketed and sorted like an index.  With several
        ranks, rows first move to their bucket's owner (``b % world``) with RCCL all-to-all, so
        the output is co-partitioned with the index tables of the same bucket count."""
        d = self._dist()
        if not all(isinstance(e, E.Attribute) for e in part.expressions):
            raise Unsupported("hash partitioning on expressions")
        keys = list(part.expressions)
        if (r.bucketed and not r.parts and not r.split and r.num_buckets == part.num_partitions
                and [a.expr_id for a in r.bucket_attrs] == [k.expr_id for k in keys]
                and _prefix_sorted(r, keys)):
            # an index table loaded bucket-major is already hash-partitioned by these keys into
            # this many buckets (same Murmur3 + pmod) and sorted inside each bucket — the
            # exchange the planner asked for would reproduce exactly this layout
            return r
        if (d is None or d.world == 1) and not r.parts and not r.split and \
                getattr(r.table, "global_key", None) is not None:
            cached = self._repartition_cached(r, keys, part.num_partitions)
            if cached is not None:
                return cached
        cols = self._materialize(r, list(dict.fromkeys(r.attrs + keys)))
        kcols = [cols[k.expr_id] for k in keys]
        import torch
        B = part.num_partitions
        with stage("shuffle.hash"):
            bucket, counts = K.murmur3_bucket(kcols, B)
        if d is not None and d.world > 1:
            with stage("shuffle.all_to_all"):
                cols, bucket = self._exchange_rows(d, cols, bucket,
                                                   self._owner_map(B, d.world).dest(bucket))
            kcols = [cols[k.expr_id] for k in keys]
            counts = K.histogram(bucket, B)
        n = int(bucket.numel())
        with stage("shuffle.sort"):
            perm = K.sort_permutation(kcols, extra_leading=(bucket, 16))
        names = list(cols.keys())
        gathered = K.gather_columns([cols[i] for i in names], perm)
        for c in gathered:
            c.hs_transient = True       # built for this query only (not the cached repartition)
        off_host = np.concatenate([[0], np.cumsum(counts.cpu().numpy())]).astype(np.int64)
        table = DeviceTable({f"c{i}": c for i, c in zip(names, gathered)}, n,
                            torch.from_numpy(off_host).to(self.device), off_host)
        colmap = {i: f"c{i}" for i in names}
        return DRel(table, colmap, list(r.attrs), [], True, keys, keys, B)

    def _repartition_cached(self, r: DRel, keys, B: int) -> Optional[DRel]:
        """Single rank, resident source table (e.g. the appended files of a Hybrid Scan): the
        bucketed + sorted layout of the *unfiltered* rows depends only on the table, so it is
        built once and cached on the table; the query's filters stay pending on the result
        and run inside the consuming kernel.  Queries with new literals reuse the layout."""
        need = list(dict.fromkeys(list(r.attrs) + list(keys) +
                                  [a for c in r.conds for a in c.references()]))
        if any(a.expr_id not in r.colmap or r.is_computed(a) for a in need):
            return None
        names = sorted({r.colmap[a.expr_id] for a in need})
        knames = tuple(r.colmap[k.expr_id] for k in keys)
        t = r.table
        cache = t.__dict__.setdefault("_repart", {})
        ck = (tuple(names), knames, B)
        nt = cache.get(ck)
        if nt is None:
            import torch
            kcols = [t.columns[n] for n in knames]
            with stage("shuffle.hash"):
                bucket, counts = K.murmur3_bucket(kcols, B)
            with stage("shuffle.sort"):
                perm = K.sort_permutation(kcols, extra_leading=(bucket, 16))
            gathered = K.gather_columns([t.columns[n] for n in names], perm)
            off_host = np.concatenate([[0], np.cumsum(counts.cpu().numpy())]).astype(np.int64)
            nt = DeviceTable(dict(zip(names, gathered)), t.num_rows,
                             torch.from_numpy(off_host).to(self.device), off_host)
            nt.global_key = ("repartition", t.global_key, ck)
            nt._hs_sources = [t]      # current while the source table is resident
            nt._hs_cache_key = nt.global_key
            cache[ck] = nt
        colmap = {a.expr_id: r.colmap[a.expr_id] for a in need}
        return DRel(nt, colmap, list(r.attrs), list(r.conds), True, list(keys), list(keys), B)

    def _exchange_rows(self, d, cols: Dict[int, DeviceColumn], bucket, dest=None):
        """Route every row to its bucket's owner rank (``dest``, default ``bucket % world``:
        parallel/placement.py) with ONE packed all-to-all
        (``parallel/exchange.py``).  Ranks first agree on column layouts: a validity mask exists
        on every rank if it exists on any (one small all-reduce), and string dictionaries are
        unified (raw-buffer all-gather, ``parallel/dictionary.py``) with codes remapped on the
        device."""
        import torch
        from ..parallel.dictionary import remap_table, union_sorted
        from ..parallel.exchange import RowExchange
        ids = list(cols)
        need_valid = d.agree_any([cols[i].valid is not None for i in ids])
        datas, valids, dicts = [], [], []
        for j, i in enumerate(ids):
            c = cols[i]
            data = c.data
            gdict = None
            if c.dictionary is not None:
                gdict = union_sorted(c.dictionary, d)
                if len(c.dictionary) == 0:
                    data = torch.zeros_like(data)
                elif not c.dictionary.equals(gdict):
                    remap = torch.from_numpy(remap_table(c.dictionary, gdict)).to(self.device)
                    data = K.lookup_i32(remap, data)
            v = c.valid
            if need_valid[j] and v is None:
                v = torch.ones(data.shape[0], dtype=torch.uint8, device=self.device)
            datas.append(data)
            valids.append(v if need_valid[j] else None)
            dicts.append(gdict)
        send = datas + [v for v in valids if v is not None] + [bucket]
        moved = RowExchange(d, [t.dtype for t in send], self.device)
        moved.add(send, bucket, dest)
        got = moved.finish()
        out = {}
        vi = len(ids)
        for j, i in enumerate(ids):
            mv = None
            if valids[j] is not None:
                mv = got[vi]
                vi += 1
            out[i] = DeviceColumn(got[j], mv, cols[i].atype, dicts[j])
        return out, got[-1]

    # ------------------------------------------------------------------------------------------
    # Joins
    # ------------------------------------------------------------------------------------------
    JOIN_TYPES = ("inner", "left", "right", "full", "leftsemi", "leftanti")

    def _join_inputs(self, p: X.SortMergeJoinExec):
        if p.join_type not in self.JOIN_TYPES:
            raise Unsupported(f"{p.join_type} join on device")
        if not all(isinstance(k, E.Attribute) for k in list(p.left_keys) + list(p.right_keys)):
            raise Unsupported("expression join keys")
        left, right = self._rel(p.left), self._rel(p.right)
        if not (left.bucketed and right.bucketed) or left.num_buckets != right.num_buckets:
            raise Unsupported("join inputs not co-partitioned on device")
        if not _prefix_sorted(left, list(p.left_keys)):
            raise Unsupported("left not sorted by join key")
        if not _prefix_sorted(right, list(p.right_keys)):
            raise Unsupported("right not sorted by join key")
        if len(p.left_keys) > 1:
            return self._packed_join_keys(left, right, list(p.left_keys), list(p.right_keys))
        lk, rk = p.left_keys[0], p.right_keys[0]
        kinds = set()
        strings = []
        for side, k in ((left, lk), (right, rk)):
            for part in side.parts or [side]:
                c = part.col(k)
                strings.append(c.dictionary is not None)
                kinds.add(c.is_float)
        if any(strings):
            if not all(strings):
                raise Unsupported("mixed string / non-string join keys")
            left, right = self._string_join_keys(left, right, lk, rk)
        elif len(kinds) > 1:
            raise Unsupported("mixed int/float join keys")
        return left, right, lk, rk

    def _packed_join_keys(self, left: DRel, right: DRel, lks, rks):
        """Multi-column equi-join (e.g. ``(l_partkey, l_suppkey) = (ps_partkey, ps_suppkey)``):
        both sides are sorted by the key columns inside every bucket, so packing the integer
        keys into one 64-bit value — ``(k1 - lo1) << bits2 | (k2 - lo2)`` with the SAME bases
        and widths on both sides — preserves the lexicographic order and equality.  The packed
        column (null if any component is null) is cached on each table, and the single-key join
        machinery (merge join or join index) runs on it."""
        # string key components: codes into the sorted union of every part's dictionary (the
        # same remap as a single string key, _string_join_keys), so they compare across sides
        # and keep each bucket's order; then they pack like integers
        for lk, rk in zip(lks, rks):
            strs = [x.col(k).dictionary is not None
                    for side, k in ((left, lk), (right, rk)) for x in (side.parts or [side])]
            if any(strs):
                if not all(strs):
                    raise Unsupported("mixed string / non-string join keys")
                left, right = self._string_join_keys(left, right, lk, rk)
        lparts, rparts = left.parts or [left], right.parts or [right]
        lcols = [[x.col(k) for x in lparts] for k in lks]
        rcols = [[x.col(k) for x in rparts] for k in rks]
        if any(c.is_float for cs in lcols + rcols for c in cs):
            raise Unsupported("multi-key join on float keys")
        spans = []
        for lcs, rcs in zip(lcols, rcols):
            doms = [d for d in (self._local_domain(c) for c in lcs + rcs) if d[1] > 0]
            lo = min((d[0] for d in doms), default=0)
            hi = max((d[0] + d[1] - 1 for d in doms), default=0)
            # codes: 0 = null on the left, 1 = null on the right, 2 + (v - lo) = value
            spans.append((lo, max(1, int(hi - lo + 2).bit_length())))
        if sum(b for _, b in spans) > 62:
            raise Unsupported("multi-key join keys do not pack into 64 bits")
        spec = tuple(spans)
        la = E.Attribute("__hs_jkey", pa.int64(), True)
        ra = E.Attribute("__hs_jkey", pa.int64(), True)

        def pack(side, keys, code, attr):
            parts = [self._packed(x, keys, spec, code) for x in (side.parts or [side])]
            for x in parts:
                x.colmap[attr.expr_id] = "__hs_jkey"
                x.sort_attrs = [attr]
            if side.parts:
                return side.copy(parts=parts)
            return parts[0]
        return pack(left, lks, 0, la), pack(right, rks, 1, ra), la, ra

    def _packed(self, r: DRel, keys, spec, side: int) -> DRel:
        """``side`` 0/1 = the code of a null component on this side: nulls sort first within
        their prefix (the index order, NULLS FIRST) and never equal anything on the other side,
        so the packed column is sorted per bucket and needs no validity mask."""
        import torch
        t = r.table
        names = tuple(r.colmap[k.expr_id] for k in keys)
        cache = t.__dict__.setdefault("_packed_keys", {})
        nt = cache.get((names, spec, side))
        if nt is None:
            packed = torch.zeros(t.num_rows, dtype=torch.int64, device=self.device)
            for name, (lo, bits) in zip(names, spec):
                c = t.columns[name]
                code = c.data.long() - (lo - 2)
                if c.valid is not None:
                    code = torch.where(c.valid.bool(), code, torch.full_like(code, side))
                packed = (packed << bits) | code
            cols = dict(t.columns)
            cols["__hs_jkey"] = DeviceColumn(packed, None, pa.int64())
            nt = DeviceTable(cols, t.num_rows, t.bucket_offsets, t.bucket_offsets_host)
            for a in ("global_key", "_full_ranges"):
                if a in t.__dict__:
                    nt.__dict__[a] = t.__dict__[a]
            cache[(names, spec, side)] = nt
        return r.copy(table=nt, colmap=dict(r.colmap))

    def _string_join_keys(self, left: DRel, right: DRel, lk, rk):
        """Join on string keys.  Strings live in HBM as codes into per-table *sorted*
        dictionaries, so codes of different tables are not comparable — but codes into the
        sorted union of all their dictionaries are, and they keep each bucket's sort order
        (code order == string order).  Every part's key column (both sides; a Hybrid Scan side
        is a bucket union of the index and its shuffled appended rows) is remapped once (one
        int32 gather) into the union's code space; the remapped tables are cached on the
        originals, so the join index and span caches see stable tables across queries."""
        sides = [(left, lk), (right, rk)]
        dicts = []
        for side, k in sides:
            for part in side.parts or [side]:
                dicts.append(part.col(k).dictionary)
        if all(d is dicts[0] or d.equals(dicts[0]) for d in dicts[1:]):
            return left, right
        ukey = tuple(id(d) for d in dicts)
        hit = self._unions.get(ukey)
        if hit is None or any(a is not b for a, b in zip(hit[0], dicts)):
            import pyarrow.compute as pc
            union = pc.unique(pa.concat_arrays([d.cast(pa.string()) for d in dicts])).sort()
            hit = (tuple(dicts), union)
            self._unions[ukey] = hit
        union = hit[1]

        def remap(side, k):
            if side.parts:
                return side.copy(parts=[self._remapped(x, k, union) for x in side.parts])
            return self._remapped(side, k, union)
        return remap(left, lk), remap(right, rk)

    def _remapped(self, r: DRel, attr, union) -> DRel:
        import pyarrow.compute as pc
        import torch
        name = r.colmap[attr.expr_id]
        t = r.table
        cache = t.__dict__.setdefault("_remap", {})
        hit = cache.get((name, id(union)))
        if hit is None or hit[0] is not union:
            c = t.columns[name]
            pos = pc.index_in(c.dictionary.cast(pa.string()), value_set=union)
            remap = torch.from_numpy(pos.to_numpy(zero_copy_only=False).astype(np.int32)) \
                .to(self.device)
            data = remap[c.data.long()] if len(pos) else torch.zeros_like(c.data)
            cols = dict(t.columns)
            cols[name] = DeviceColumn(data, c.valid, c.atype, union)
            nt = DeviceTable(cols, t.num_rows, t.bucket_offsets, t.bucket_offsets_host)
            for a in ("global_key", "_full_ranges"):
                if a in t.__dict__:
                    nt.__dict__[a] = t.__dict__[a]
            hit = (union, nt)
            cache[(name, id(union))] = hit
        return r.copy(table=hit[1])

    def _join_params(self, left: DRel, right: DRel, lk, rk, residual, extra_attrs=(),
                     lconds=None, slots=None):
        col_info, descs = slots if slots is not None else \
            self._column_infos([(left, 0), (right, 8)])
        lslot = col_info(lk).slot
        rslot = col_info(rk).slot
        lb = CP.bind(CP.to_cnf(left.conds if lconds is None else lconds), col_info, self.device, 0)
        rconds = list(right.conds) + ([residual] if residual is not None else [])
        rb = CP.bind(CP.to_cnf(rconds), col_info, self.device, 1000)
        for a in extra_attrs:
            col_info(a)
        p = NL.JoinParams()
        preds = lb.preds + rb.preds
        if len(preds) > NL.MAX_PREDS:
            raise Unsupported("too many join predicates")
        for i, pr in enumerate(preds):
            p.preds[i] = pr
        p.nlp, p.npreds = len(lb.preds), len(preds)
        p.lkey, p.rkey = lslot, rslot
        p.key_is_float = 1 if left.col(lk).is_float else 0
        p.group_col = -1
        return p, col_info, descs, (lb, rb)

    def _join_rel(self, p: X.SortMergeJoinExec) -> DRel:
        """Row-producing co-located join: matched (left row, right row) pairs from the join
        kernels, then per join type — inner: the pairs; left/right/full outer: plus the
        unmatched rows of the preserved side(s) (rows passing that side's own filters, marked
        by a scatter of the matched ids and selected in order) padded with NULLs (gather index
        -1); left semi / anti: the left rows that do / do not appear in a pair.  Reference: the
        rule rewrites any join type (JoinIndexRule.scala:58), Spark's bucketed SortMergeJoin
        runs it."""
        left, right, lk, rk = self._join_inputs(p)
        if left.parts or right.parts:
            return self._join_rel_union(p, left, right, lk, rk)
        return self._join_rel_pair(p, left, right, lk, rk)

    def _join_rel_union(self, p: X.SortMergeJoinExec, left: DRel, right: DRel, lk, rk) -> DRel:
        """Inner join rows over BucketUnion inputs (Hybrid Scan: index buckets plus appended
        rows shuffled by the index bucket spec): an inner join distributes over union, so each
        (left part, right part) pair runs as its own co-located join and the row sets are
        concatenated; string columns whose parts carry different dictionaries are re-coded
        over the union of the dictionaries."""
        out_attrs = list(p.output)
        if p.join_type == "inner":
            pieces = [self._join_rel_pair(p, lp, rp, lk, rk)
                      for lp in (left.parts or [left]) for rp in (right.parts or [right])]
            return self._concat_rels([[x.col(a) for a in out_attrs] for x in pieces], out_attrs)
        return self._join_rel_parts_outer(p, left.parts or [left], right.parts or [right],
                                          lk, rk)

    def _join_rel_parts_outer(self, p: X.SortMergeJoinExec, lparts, rparts, lk, rk) -> DRel:
        """Outer / semi / anti join rows over BucketUnion parts (Hybrid Scan of either side): the
        matched pairs of every (left part, right part) pair, and a row of a preserved side is
        unmatched only if NO part of the other side matched it - its match marks are OR-ed over
        the other side's parts before the unmatched rows (passing the row's own side filters)
        are selected and padded with NULLs.  Same rows as the join of the unions
        (JoinIndexRule.scala:57-58 rewrites any join type; RuleUtils.scala:439-441 puts the
        BucketUnion under it)."""
        import torch
        jt = p.join_type
        out_attrs = list(p.output)
        lset = {a.expr_id for a in p.left.output}
        lattrs = [a for a in out_attrs if a.expr_id in lset]
        rattrs = [a for a in out_attrs if a.expr_id not in lset]
        inner = X.SortMergeJoinExec(p.left_keys, p.right_keys, "inner", p.condition, p.left,
                                    p.right)
        lmarks: List = [None] * len(lparts)
        rmarks: List = [None] * len(rparts)
        pieces = []
        for i, lp in enumerate(lparts):
            for j, rp in enumerate(rparts):
                ol, orr = self._pair_rows(inner, lp, rp, lk, rk)
                if jt in ("left", "full", "leftsemi", "leftanti"):
                    m = K.mark_rows(ol, int(lp.table.num_rows or 0))
                    lmarks[i] = m if lmarks[i] is None else torch.maximum(lmarks[i], m)
                if jt in ("right", "full"):
                    m = K.mark_rows(orr, int(rp.table.num_rows or 0))
                    rmarks[j] = m if rmarks[j] is None else torch.maximum(rmarks[j], m)
                if jt in ("left", "right", "full"):
                    lg = K.gather_columns([lp.col(a) for a in lattrs], ol)
                    rg = K.gather_columns([rp.col(a) for a in rattrs], orr)
                    pieces.append(lg + rg)
        ncols = len(rattrs)
        for i, lp in enumerate(lparts):
            if jt not in ("left", "full", "leftsemi", "leftanti"):
                break
            sel = self._selected_rows(lp)
            want = 1 if jt == "leftsemi" else 0
            rows = K.select_marked(sel, lmarks[i], want)
            lg = K.gather_columns([lp.col(a) for a in lattrs], rows)
            if jt in ("leftsemi", "leftanti"):
                pieces.append(lg)
                continue
            pad = torch.full_like(rows, -1)
            rg = K.gather_columns([rparts[0].col(a) for a in rattrs], pad, padded=True) \
                if ncols else []
            pieces.append(lg + rg)
        if jt in ("right", "full"):
            for j, rp in enumerate(rparts):
                sel = self._selected_rows(rp)
                rows = K.select_marked(sel, rmarks[j], 0)
                pad = torch.full_like(rows, -1)
                lg = K.gather_columns([lparts[0].col(a) for a in lattrs], pad, padded=True) \
                    if lattrs else []
                rg = K.gather_columns([rp.col(a) for a in rattrs], rows)
                pieces.append(lg + rg)
        attrs = lattrs + rattrs if jt not in ("leftsemi", "leftanti") else lattrs
        rel = self._concat_rels(pieces, attrs)
        if [a.expr_id for a in attrs] != [a.expr_id for a in out_attrs]:
            rel.attrs = out_attrs
        return rel

    def _pair_rows(self, p: X.SortMergeJoinExec, left: DRel, right: DRel, lk, rk):
        """(left row ids, right row ids) of the inner join pairs of one part pair (each side's
        own predicates applied, the join condition evaluated)."""
        import torch
        implied: set = set()
        probed = self._probe_ranges(left, right, lk, rk)
        if probed is None:
            probed = self._domain_pruned_ranges(left, right, lk, rk)
        if probed is not None:
            rstart, rlen, rbk = probed
        else:
            rstart, rlen, rbk = self._ranges(left, left.conds, implied)
        jp, col_info, descs, keep = self._join_params(
            left, right, lk, rk, p.condition,
            lconds=[c for c in left.conds if id(c) not in implied])
        for s_, c in descs.items():
            jp.cols[s_] = c.desc()
        if keep[0].always_false or keep[1].always_false:
            e = torch.empty(0, dtype=torch.int64, device=self.device)
            return e, e
        max_tiles = K.join_max_tiles(left.table.num_rows, rlen.numel())
        return K.join_pairs(jp, rstart, rlen, rbk, right.table.bucket_offsets, max_tiles)

    def _concat_rels(self, pieces: List[List[DeviceColumn]], out_attrs) -> DRel:
        """One flat device relation over ``out_attrs`` from row sets ``pieces`` (per piece the
        columns in ``out_attrs`` order); string columns with different dictionaries are
        re-coded over their union."""
        import torch
        from ..parallel.dictionary import remap_table
        cols = {}
        for ai, a in enumerate(out_attrs):
            cs = [x[ai] for x in pieces]
            dicts = [c.dictionary for c in cs]
            gd = None
            if any(d is not None for d in dicts):
                gd = dicts[0]
                if not all(d is not None and d.equals(gd) for d in dicts):
                    import pyarrow.compute as pc
                    allv = pa.concat_arrays([d.cast(pa.string()) for d in dicts if d is not None])
                    gd = pc.unique(allv).sort()
            datas = []
            for c in cs:
                d = c.data
                if gd is not None and c.dictionary is not None and not c.dictionary.equals(gd) \
                        and d.numel():
                    tab = torch.from_numpy(remap_table(c.dictionary, gd)).to(self.device)
                    d = K.lookup_i32(tab, d)
                datas.append(d)
            valid = None
            if any(c.valid is not None for c in cs):
                valid = torch.cat([c.valid if c.valid is not None else
                                   torch.ones(c.data.numel(), dtype=torch.uint8,
                                              device=self.device) for c in cs])
            col = DeviceColumn(torch.cat(datas), valid, cs[0].atype, gd)
            col.hs_transient = True
            cols[key(a)] = col
        n = sum(int(x[0].data.numel()) for x in pieces) if out_attrs else 0
        off = np.array([0, n], dtype=np.int64)
        table = DeviceTable(cols, n, torch.from_numpy(off).to(self.device), off)
        return DRel(table, {a.expr_id: key(a) for a in out_attrs}, out_attrs)

    def _join_rel_pair(self, p: X.SortMergeJoinExec, left: DRel, right: DRel, lk, rk) -> DRel:
        jt = p.join_type
        out_attrs = list(p.output)
        implied: set = set()
        probed = self._probe_ranges(left, right, lk, rk) if jt in ("inner", "leftsemi") else None
        if probed is None and jt in ("inner", "leftsemi", "right"):
            probed = self._domain_pruned_ranges(left, right, lk, rk)
        if probed is not None:
            rstart, rlen, rbk = probed
        else:
            with stage("join.ranges"):
                rstart, rlen, rbk = self._ranges(left, left.conds, implied)
        jp, col_info, descs, keep = self._join_params(
            left, right, lk, rk, p.condition,
            lconds=[c for c in left.conds if id(c) not in implied])
        for s, c in descs.items():
            jp.cols[s] = c.desc()
        if keep[0].always_false or keep[1].always_false:
            import torch
            ol = orr = torch.empty(0, dtype=torch.int64, device=self.device)
        else:
            max_tiles = K.join_max_tiles(left.table.num_rows, rlen.numel())
            ol, orr = K.join_pairs(jp, rstart, rlen, rbk, right.table.bucket_offsets, max_tiles)
        lset = {a.expr_id for a in p.left.output}
        lattrs = [a for a in out_attrs if a.expr_id in lset]
        rattrs = [a for a in out_attrs if a.expr_id not in lset]
        padded = jt in ("left", "right", "full")
        if jt != "inner":
            import torch
            with stage("join.outer_rows"):
                if jt in ("left", "full", "leftsemi", "leftanti"):
                    lsel = self._selected_rows(left)
                    lmark = K.mark_rows(ol, int(left.table.num_rows or 0))
                if jt in ("leftsemi", "leftanti"):
                    ol = K.select_marked(lsel, lmark, 1 if jt == "leftsemi" else 0)
                    orr = ol[:0]
                    rattrs = []
                else:
                    extra_l, extra_r = [], []
                    if jt in ("left", "full"):
                        um = K.select_marked(lsel, lmark, 0)
                        extra_l.append(um)
                        extra_r.append(torch.full_like(um, -1))
                    if jt in ("right", "full"):
                        rsel = self._selected_rows(right)
                        rmark = K.mark_rows(orr, int(right.table.num_rows or 0))
                        um = K.select_marked(rsel, rmark, 0)
                        extra_l.append(torch.full_like(um, -1))
                        extra_r.append(um)
                    ol = torch.cat([ol] + extra_l)
                    orr = torch.cat([orr] + extra_r)
        lg = K.gather_columns([left.col(a) for a in lattrs], ol,
                              padded=padded and jt in ("right", "full"))
        rg = K.gather_columns([right.col(a) for a in rattrs], orr,
                              padded=padded and jt in ("left", "full"))
        cols = {}
        for a, c in list(zip(lattrs, lg)) + list(zip(rattrs, rg)):
            c.hs_transient = True
            cols[key(a)] = c
        n = int(ol.numel())
        import torch
        off = np.array([0, n], dtype=np.int64)
        table = DeviceTable(cols, n, torch.from_numpy(off).to(self.device), off)
        return DRel(table, {a.expr_id: key(a) for a in out_attrs}, out_attrs)

    # ------------------------------------------------------------------------------------------
    # Aggregation
    # ------------------------------------------------------------------------------------------
    def _match_agg(self, plan):
        if not (isinstance(plan, X.HashAggregateExec) and plan.mode == "final"):
            return None
        ex = plan.child
        if not isinstance(ex, X.ShuffleExchangeExec):
            return None
        partial = ex.child
        if not (isinstance(partial, X.HashAggregateExec) and partial.mode == "partial"):
            return None
        return plan, partial.child

    def _exec_agg(self, final: X.HashAggregateExec, child: X.SparkPlan, order=None,
                  limit=None):
        """Queue a fused aggregate and return ``finish() -> pa.Table``: the dense LDS
        aggregate for one small integer group column, else the hash-mode aggregate
        (``_hash_agg``)."""
        if any(not isinstance(g, E.Attribute) for g in final.grouping):
            final, child = self._named_groups(final, child)
        try:
            return self._dense_agg(final, child)
        except _NeedHash as e:
            log.debug("hash-mode aggregate: %s", e)
        return self._hash_agg(final, child, order, limit)

    @staticmethod
    def _named_groups(final: X.HashAggregateExec, child: X.SparkPlan):
        """GROUP BY expressions: each named grouping expression becomes a computed column of a
        projection over the aggregate's input (exec/project.py) and the aggregate groups on
        that column; result expressions that repeat a grouping expression read the column."""
        groups, extra = [], []
        for gi, g in enumerate(final.grouping):
            if isinstance(g, E.Attribute):
                groups.append(g)
            elif isinstance(g, E.Alias):
                extra.append(g)
                groups.append(g.to_attribute())
            else:
                # an unnamed grouping expression (SQL ``GROUP BY a % 3``): a hidden computed
                # column; result expressions repeating it read that column (swap below)
                a = E.Alias(g, f"__hs_g{gi}")
                extra.append(a)
                groups.append(a.to_attribute())

        def swap(x):
            for g in extra:
                if x.semantic_equals(g.child):
                    return g.to_attribute()
            return None
        aggs = []
        for e in final.aggregates:
            hit = next((g for g in extra if g.expr_id == getattr(e, "expr_id", None)), None)
            if hit is not None:
                aggs.append(hit.to_attribute())
            else:
                aggs.append(e.transform_up(swap))
        proj = X.ProjectExec(list(child.output) + extra, child)
        return X.HashAggregateExec(groups, aggs, final.mode, final.child, final.result_attrs), proj

    # ------------------------------------------------------------------------------------------
    # Bucket-range streaming: indexes larger than the HBM budget
    # ------------------------------------------------------------------------------------------
    def _stream_chunks(self, child) -> Optional[List[tuple]]:
        """Bucket ranges an aggregate over ``child`` runs in, one resident range at a time, when
        its index scans would not fit ``deviceCacheBytes`` together; None when they fit or the
        plan cannot be split by bucket (a non-index scan, indexes of different bucket counts,
        a Hybrid Scan union, several ranks).  Every index of the plan is cut at the same bucket
        boundaries, so a co-partitioned join joins bucket range to bucket range
        (BucketUnionExec.scala:61-74 runs a bucketed plan partition by partition)."""
        if self._dist() is not None:
            return None
        budget = HyperspaceConf.device_cache_bytes(self.session.conf)
        memo = self.__dict__.setdefault("_stream_memo", {})
        hit = memo.get(id(child))
        if hit is not None and hit[0] is child and hit[1] == budget:
            return hit[2]       # a plan-cache hit re-submits the same nodes: decided once
        chunks = self._stream_plan(child, budget)
        if len(memo) > 256:
            memo.clear()
        memo[id(child)] = (child, budget, chunks)
        return chunks

    def _stream_plan(self, child, budget: int) -> Optional[List[tuple]]:
        scans = child.collect(lambda x: isinstance(x, X.FileSourceScanExec))
        # only operators that keep bucket b's rows inside bucket b: an Exchange (a join of
        # sides bucketed on other keys) or a union would pair rows across bucket ranges
        if not scans or child.collect(lambda x: not isinstance(
                x, (X.FileSourceScanExec, X.FilterExec, X.ProjectExec, X.SortExec,
                    X.SortMergeJoinExec))):
            return None
        nbs, per_bucket = set(), None
        total = 0
        for sc in scans:
            rel = sc.relation
            if not rel.is_index():
                return None
            files = rel.location.all_files()
            nb = rel.index.num_buckets
            if not self._all_bucket_files(rel.location, files, nb):
                return None
            nbs.add(nb)
            memo = getattr(rel.location, "_hs_bucket_weights", None)
            if memo is None or memo[0] != nb or memo[1] is not files:
                from ..parallel.placement import bucket_weights
                memo = (nb, files, bucket_weights(files, nb) * self.STREAM_EXPANSION)
                rel.location._hs_bucket_weights = memo
            w = memo[2]
            per_bucket = w if per_bucket is None or len(per_bucket) != nb else per_bucket + w
            total += float(w.sum())
        if len(nbs) != 1 or total <= budget:
            return None
        return bucket_chunks(per_bucket, budget)

    # decoded bytes per byte of a (compressed, dictionary-encoded) index file: the resident
    # estimate of a bucket for the streaming plan
    STREAM_EXPANSION = 4.0

    def _streamed_agg(self, final, child, fns, group, chunks):
        """The aggregate as one pass per bucket range: each pass loads its range of every
        index (evicting the previous one), runs the fused kernels and brings its partials to
        the host, where they combine by group value."""
        import torch
        A = len(fns) + 1
        acc: Dict[object, list] = {}
        gtype = None
        gdict_all = None
        self.last_stream_passes = len(chunks)
        try:
            for ch in chunks:
                self._bucket_chunk = ch
                self._drop_resident()
                node = child
                while isinstance(node, X.ProjectExec) and \
                        all(isinstance(e, E.Attribute) for e in node.project_list):
                    node = node.child
                if isinstance(node, X.SortMergeJoinExec) and node.join_type == "inner":
                    res = self._join_agg(node, fns, group)
                else:
                    res = self._scan_agg(self._rel(child), fns, group)
                sums, cnts, mins, maxs, G, gbase, gdict, gt = res
                if isinstance(sums, _GraphPending):
                    host = sums.result()
                elif isinstance(sums, np.ndarray):
                    host = (sums, cnts, mins, maxs)
                else:
                    host = K.agg_to_host_async(sums, cnts, mins, maxs)()
                gtype = gt if gt is not None else gtype
                s_, c_, mn_, mx_ = (np.asarray(x).reshape(G, A) for x in host)
                for g in range(G):
                    if c_[g, A - 1] == 0 and group is not None:
                        continue
                    key = None
                    if group is not None:
                        key = gdict[gbase + g].as_py() if gdict is not None else gbase + g
                    cur = acc.get(key)
                    if cur is None:
                        acc[key] = [s_[g].copy(), c_[g].copy(), mn_[g].copy(), mx_[g].copy()]
                    else:
                        cur[0] += s_[g]
                        cur[1] += c_[g]
                        cur[2] = np.minimum(cur[2], mn_[g])
                        cur[3] = np.maximum(cur[3], mx_[g])
                del res, sums, cnts, mins, maxs
                torch.cuda.current_stream().synchronize()
        finally:
            self._bucket_chunk = None
            self._drop_resident()
        if group is None:
            if None not in acc:
                acc[None] = [np.zeros(A), np.zeros(A, np.int64), np.full(A, np.inf),
                             np.full(A, -np.inf)]
            keys = [None]
        else:
            keys = sorted(acc)
            if gtype is not None and pa.types.is_string(gtype):
                gdict_all = pa.array(keys, type=pa.string())
        G = max(len(keys), 1)
        host = tuple(np.concatenate([acc[k][i] for k in keys]) if keys else
                     np.zeros(A) for i in range(4))
        if group is not None and gdict_all is None:
            # integer group values: lay the rows out over their own domain order
            gvals = keys
            gbase = 0

            def finish() -> pa.Table:
                return self._agg_table_values(final, fns, group, host, G, A, gvals, gtype)
            return finish
        gbase = 0
        gd = gdict_all

        def finish() -> pa.Table:
            return self._agg_table(final, fns, group, host, G, A, gbase, gd, gtype)
        return finish

    def _drop_resident(self) -> None:
        """Release every device table this backend holds: the cache and the per-table memos
        (scan nodes, null flags, domains, prepared submissions) that keep tables alive."""
        self.cache.clear()
        for memo in ("_scans", "_nulls_memo"):
            self.__dict__.pop(memo, None)
        self._domains.clear()
        preps = getattr(self, "_agg_preps", None)
        if preps:
            preps.clear()
        self._join_rec = None

    def _agg_table_values(self, final, fns, group, host, G, A, gvals, gtype) -> pa.Table:
        """``_agg_table`` over explicit integer group values (row g has group ``gvals[g]``)."""
        s, c, mn, mx = (x.reshape(G, A) for x in host)
        rows = [g for g in range(G) if c[g, A - 1] > 0]
        vals = {}
        for i, fn in enumerate(fns):
            vals[id(fn)] = [CP.finalize_value(fn, s[g, i], c[g, i], mn[g, i], mx[g, i]) for g in rows]
        raw = [gvals[g] for g in rows]
        if pa.types.is_date32(gtype):
            gv = pa.array(np.array(raw, dtype=np.int32)).view(pa.date32()).to_pylist()
        else:
            gv = raw
        out_cols = [self._agg_output(e, group, gv, vals, len(rows)) for e in final.aggregates]
        arrays = []
        for a, vlist in zip(final.output, out_cols):
            try:
                arrays.append(pa.array(vlist, type=a.data_type))
            except (pa.ArrowInvalid, pa.ArrowTypeError):
                arrays.append(pa.array(vlist))
        return pa.Table.from_arrays(arrays, names=[a.name for a in final.output])

    def _agg_prep_get(self, final) -> Optional["_ScanPrep"]:
        """The prepared scan of a fused aggregate node submitted before (plan-cache hits
        submit the same node objects with new literal values), while its table is resident."""
        preps = self.__dict__.get("_agg_preps")
        if not preps:
            return None
        pr = preps.get(id(final))
        if pr is None or pr.final is not final or pr.placement != self._placement_tag() or \
                not all(self._holds(t) for t in pr.tables()):
            return None
        return pr

    def _agg_prep_put(self, final, r: DRel) -> None:
        """Keep what the fused scan of ``final`` lowered, for its next submission: only for a
        relation of one resident table with no computed columns (their values are literal
        dependent) whose lowering completed."""
        st = getattr(self, "_scan_gs", None)
        if st is None or r.parts or r.extra or r.split or \
                getattr(r.table, "_hs_cache_key", None) is None:
            return
        col_info, descs, gs, p = st
        preps = self.__dict__.setdefault("_agg_preps", {})
        if len(preps) > 256:
            preps.clear()
        preps[id(final)] = _ScanPrep(final, r, col_info, descs, gs, p,
                                     getattr(self, "_last_graph_prep", None),
                                     self._placement_tag())

    def _join_prep_put(self, final, node, res) -> None:
        """Keep a co-located merge join aggregate's lowering (one left x right pair over full
        bucket ranges, resident tables) for its next submission."""
        rec = getattr(self, "_join_rec", None)
        self._join_rec = None
        if rec is None or res is None or rec[6] is None:
            return
        left, right, lk, rk, col_info, descs, launcher, specs, lconds = rec
        for t in (left.table, right.table):
            if getattr(t, "_hs_cache_key", None) is None:
                return
        preps = self.__dict__.setdefault("_agg_preps", {})
        if len(preps) > 256:
            preps.clear()
        preps[id(final)] = _JoinPrep(final, node, left, right, lk, rk, col_info, descs,
                                     launcher, res[4:], self._placement_tag(),
                                     self._groups_agreed, lconds)

    def _placement_tag(self):
        d = self._dist()
        return None if d is None else (d.rank, d.world, self.session.conf.get(
            "spark.hyperspace.mi.bucketPlacement", "balanced"))

    def _dense_agg(self, final: X.HashAggregateExec, child: X.SparkPlan):
        """Queue a fused aggregate and return ``finish() -> pa.Table``.  Nothing here waits on
        the device: kernels, the cross-rank combine and the D2H of the tiny result block are
        stream-ordered, so the host can plan and submit the next query while this one runs
        (``collect_async``)."""
        fns = [fn for _, fn in X.agg_functions(final.aggregates)]
        if len(final.grouping) > 1:
            raise _NeedHash("multi-column group by")
        group = final.grouping[0] if final.grouping else None
        if group is not None and not isinstance(group, E.Attribute):
            raise Unsupported("group by expression")
        node = child
        while isinstance(node, X.ProjectExec) and all(isinstance(e, E.Attribute) for e in node.project_list):
            node = node.child
        self._groups_agreed = False
        self.last_stream_passes = 0
        chunks = self._stream_chunks(child)
        if chunks is not None:
            return self._streamed_agg(final, child, fns, group, chunks)
        res = None
        prep = self._agg_prep_get(final)
        if prep is not None:
            try:
                res = prep.run(self, fns, group)
            except _Stale:
                self._agg_preps.pop(id(final), None)
                res = None
            if res is not None:
                self._prog_candidate = (final, fns, group, prep, self.cache.epoch)
        if res is not None:
            pass
        elif isinstance(node, X.SortMergeJoinExec) and node.join_type == "inner":
            res = self._semi_join_agg(node, fns, group)
        if res is not None:
            pass
        elif isinstance(node, X.SortMergeJoinExec) and node.join_type == "inner":
            self._join_rec = None
            res = self._join_agg(node, fns, group)
            self._join_prep_put(final, node, res)
        elif group is None and isinstance(node, X.UnionExec) and \
                str(self.session.conf.get("spark.hyperspace.mi.unionAgg.enabled", "true")).lower() \
                == "true":
            res = self._union_agg(node, fns)
        elif group is None and (res := self._mixed_index_agg(child, fns)) is not None:
            pass
        else:
            r = self._rel(child)
            self._scan_gs = None
            self._last_graph_prep = None
            res = self._scan_agg(r, fns, group)
            self._agg_prep_put(final, r)
        return self._agg_finish(final, fns, group, res)

    def _agg_finish(self, final, fns, group, res):
        """``finish() -> pa.Table`` of a queued fused aggregate ``res`` = (sums, counts, mins,
        maxs, G, gbase, gdict, gtype): the cross-rank combine (sharded placement) is queued
        now, stream-ordered behind the kernels; the result is read when ``finish`` runs."""
        sums, cnts, mins, maxs, G, gbase, gdict, gtype = res
        d = self._dist()
        A = len(fns) + 1  # + implicit count(*)
        if isinstance(sums, _GraphPending) and d is not None and d.world > 1:
            # sharded: combine this rank's partials straight from the graph's device output
            # (stream-ordered after the replay; the next replay is ordered after the collective)
            if sums.graph.on_side:
                import torch
                # the replay ran on the side stream: the collective on this stream waits for it
                torch.cuda.current_stream().wait_stream(self._side)
            sums, cnts, mins, maxs = sums.graph.out
        if isinstance(sums, _GraphPending):
            fetch = sums.result
        elif d is not None and d.world > 1:
            with stage("agg.combine_ranks"):
                if group is not None and not self._groups_agreed:
                    sums, cnts, mins, maxs, G, gbase, gdict, gtype = self._agree_groups(
                        d, sums, cnts, mins, maxs, G, gbase, gdict, gtype, A)
                fetch = d.combine_aggs_async(sums, cnts, mins, maxs)
        elif isinstance(sums, np.ndarray):
            host = (sums, cnts, mins, maxs)
            fetch = (lambda: host)
        else:
            fetch = K.agg_to_host_async(sums, cnts, mins, maxs)

        def finish() -> pa.Table:
            with stage("agg.result"):
                host = fetch()
            return self._agg_table(final, fns, group, host, G, A, gbase, gdict, gtype)
        return finish

    def _agg_table(self, final, fns, group, host, G, A, gbase, gdict, gtype) -> pa.Table:
        s, c, mn, mx = (x.reshape(G, A) for x in host)
        rows = [g for g in range(G) if c[g, A - 1] > 0] if group is not None else [0]
        vals = {}
        for i, fn in enumerate(fns):
            vals[id(fn)] = [CP.finalize_value(fn, s[g, i], c[g, i], mn[g, i], mx[g, i]) for g in rows]
        gvals = None
        if group is not None:
            raw = [gbase + g for g in rows]
            if gdict is not None:
                gvals = [gdict[int(v)].as_py() for v in raw]
            elif pa.types.is_date32(gtype):
                gvals = pa.array(np.array(raw, dtype=np.int32)).view(pa.date32()).to_pylist()
            else:
                gvals = raw
        out_cols = []
        for e in final.aggregates:
            out_cols.append(self._agg_output(e, group, gvals, vals, len(rows)))
        arrays = []
        for a, vlist in zip(final.output, out_cols):
            try:
                arrays.append(pa.array(vlist, type=a.data_type))
            except (pa.ArrowInvalid, pa.ArrowTypeError):
                arrays.append(pa.array(vlist))
        return pa.Table.from_arrays(arrays, names=[a.name for a in final.output])

    def _agree_groups(self, d, sums, cnts, mins, maxs, G, gbase, gdict, gtype, A):
        """Re-key grouped partials onto the union group domain of all ranks.

        Every rank aggregated only its own buckets (index) or files (non-index), so its [G, A]
        partials are laid out over its *local* domain — integer range ``[gbase, gbase+G)`` or the
        rank's own string dictionary.  The ranks exchange those domains with tensor collectives
        (an all-gather of (G, base, live) and, for string keys, the raw-buffer dictionary union
        of ``parallel/dictionary.py`` — nothing is pickled), scatter their rows into the union
        layout, and only then run the element-wise all-reduce.  Ranks that saw no rows do not
        contribute an integer domain."""
        import torch
        from ..parallel.dictionary import union_sorted
        from ..parallel.gather import _all_gather_flat
        live_here = bool(cnts.view(G, A)[:, A - 1].sum().item() > 0)
        cdev = d.device if d.backend == "nccl" else torch.device("cpu")
        info = torch.tensor([G, gbase, 1 if live_here else 0, 1 if gdict is not None else 0],
                            dtype=torch.int64, device=cdev)
        allinfo = _all_gather_flat(d, info).view(d.world, 4).cpu().numpy()
        live = [x for x in allinfo if x[2]]
        if any(x[3] for x in allinfo):
            local = gdict if (live_here and gdict is not None) else pa.array([], pa.string())
            new_dict = union_sorted(local, d)       # collective: every rank calls it
            if not live:
                z = self._empty_agg(A, 1)
                return (*z, 1, 0, None, gtype)
            Gg, base = max(len(new_dict), 1), 0
            if live_here and gdict is not None and len(gdict):
                import pyarrow.compute as pc
                idx = pc.index_in(gdict.cast(pa.string()), value_set=new_dict).to_numpy(
                    zero_copy_only=False).astype(np.int64).tolist()
            else:
                idx = []
        else:
            if not live:
                z = self._empty_agg(A, 1)
                return (*z, 1, 0, None, gtype)
            base = int(min(x[1] for x in live))
            Gg = int(max(x[1] + x[0] for x in live)) - base
            new_dict = None
            idx = list(range(gbase - base, gbase - base + G)) if live_here else []
        s2, c2, mn2, mx2 = self._empty_agg(A, Gg)
        if idx:
            it = torch.tensor(idx, dtype=torch.int64, device=self.device)
            for dst, src in ((s2, sums), (c2, cnts), (mn2, mins), (mx2, maxs)):
                dst.view(Gg, A)[it] = src.view(G, A)[:len(idx)]
        return s2, c2, mn2, mx2, Gg, base, new_dict, gtype

    def _agg_output(self, e, group, gvals, vals, nrows):
        inner = e.child if isinstance(e, E.Alias) else e
        if isinstance(inner, E.AggregateFunction):
            return vals[id(inner)]
        if group is not None and isinstance(inner, E.Attribute) and inner.expr_id == group.expr_id:
            return gvals
        # arithmetic over aggregates (e.g. sum(a)/count(b)) evaluated on the host
        out = []
        for r in range(nrows):
            out.append(_eval_scalar(inner, lambda fn: vals[id(fn)][r],
                                    lambda a: gvals[r] if group is not None and a.expr_id == group.expr_id
                                    else None))
        return out

    def _group_spec(self, r: DRel, group, limit):
        """(agreed, G, base, dictionary, arrow type) of a group column, or None when empty.

        ``agreed`` is True when ``[base, base+G)`` is the domain over ALL ranks: partials laid
        out over it combine with a plain element-wise reduction, no per-query domain exchange.
        It is agreed once per (table identity, column) — a key every rank computes identically,
        unlike device-cache residency — and cached, so steady-state queries run no collective
        here."""
        if group is None:
            return -1, 1, 0, None, None
        c = r.col(group)
        if c.is_float:
            raise _NeedHash("float group key")
        d = self._dist()
        multi = d is not None and d.world > 1
        if c.valid is not None:
            nulls = self._has_nulls(c)
            if multi:
                nulls = d.agree_any([nulls])[0]
            if nulls:
                # NULL is a group of its own (Spark): the hash-mode aggregate keys it
                raise _NeedHash("nullable group key")
        gkey = getattr(r.table, "global_key", None) if r.table is not None else None
        if c.dictionary is not None:
            G = len(c.dictionary)
            base = 0
        else:
            base, G = self._local_domain(c)
            if multi and gkey is not None and not getattr(c, "hs_transient", False):
                k = (gkey, r.colmap.get(group.expr_id))
                dom = self._gdomains.get(k)
                if dom is None:
                    # (min, max) over ranks with one small all-reduce (no object collective)
                    import torch
                    cdev = d.device if d.backend == "nccl" else torch.device("cpu")
                    big = 1 << 62
                    t = torch.tensor([-base if G > 0 else -big, base + G - 1 if G > 0 else -big],
                                     dtype=torch.int64, device=cdev)
                    d.all_reduce(t, "max")
                    lo, hi = -int(t[0].item()), int(t[1].item())
                    dom = (lo, hi - lo + 1) if hi >= lo else (0, 0)
                    self._gdomains[k] = dom
                base, G = dom
                # identical on every rank, so the fallback decision is unanimous by construction
                if G > limit:
                    raise _NeedHash("group domain too large for LDS aggregation")
                return (True, G, base, None, c.atype) if G > 0 else None
        too_big = G > limit
        if multi:
            # data-dependent fallbacks must be unanimous, or ranks diverge in their collectives
            too_big = d.agree_any([too_big])[0]
        if too_big:
            raise _NeedHash("group domain too large for LDS aggregation")
        if G == 0:
            return None
        return None, max(G, 1), base, c.dictionary, c.atype

    def _has_nulls(self, c: DeviceColumn) -> bool:
        """Whether a device column holds a null (cached per resident column)."""
        memo = self.__dict__.setdefault("_nulls_memo", {})
        hit = memo.get(id(c))
        if hit is not None and hit[0] is c:
            return hit[1]
        v = bool((c.valid == 0).any().item())
        if not getattr(c, "hs_transient", False):
            if len(memo) > 4096:
                memo.clear()
            memo[id(c)] = (c, v)
        return v

    def _local_domain(self, c: DeviceColumn):
        """(min, max - min + 1) of an integer column on this rank; tables are immutable, so it
        is computed once per column."""
        ck = id(c)
        hit = self._domains.get(ck)
        if hit is not None and hit[0] is c:
            return hit[1]
        transient = getattr(c, "hs_transient", False)   # a per-query column: not cached
        import torch
        vals = c.data if c.valid is None else c.data[c.valid.bool()]
        if vals.numel() == 0:
            dom = (0, 0)
        else:
            lo, hi = torch.aminmax(vals)
            dom = (int(lo.item()), int(hi.item()) - int(lo.item()) + 1)
        if not transient:
            self._domains[ck] = (c, dom)
        return dom

    def _agg_specs(self, fns, col_info):
        specs = [CP.agg_spec(fn, lambda a: col_info(a).slot) for fn in fns]
        star = NL.AggSpec()
        star.kind, star.nterms = NL.AK_COUNT_STAR, 0
        specs.append(star)
        if len(specs) > NL.MAX_AGGS:
            raise Unsupported("too many aggregates")
        return specs

    def _mixed_index_agg(self, child: X.SparkPlan, fns):
        """An ungrouped aggregate over Filter / Project of an index scan whose file list also
        holds appended source files (FilterIndexRule's Hybrid Scan appends them to the index
        relation, ``RuleUtils`` same-scan appended files): the index bucket files load as the
        bucket-sorted table - so the scan keeps its leading-key range pruning - and the appended
        files as a flat table; one fused scan aggregate each, partials combined on the device.
        None when the shape does not qualify (one flat table of every file then)."""
        import torch
        if str(self.session.conf.get("spark.hyperspace.mi.mixedScanAgg.enabled", "true")).lower() \
                != "true":
            return None
        d = self._dist()
        if d is not None and d.world > 1:
            return None
        chain, node = [], child
        while isinstance(node, (X.FilterExec, X.ProjectExec)):
            chain.append(node)
            node = node.child
        if not isinstance(node, X.FileSourceScanExec) or not node.relation.is_index():
            return None
        rel = node.relation
        nb = rel.index.num_buckets
        files = rel.location.all_files()
        if self._all_bucket_files(rel.location, files, nb):
            return None
        from ..io.writer import get_bucket_id
        from ..utils import path_utils as P

        def is_bucket(f) -> bool:
            b = get_bucket_id(P.get_name(f.path))
            return b is not None and b < nb
        bfiles = [f for f in files if is_bucket(f)]
        afiles = [f for f in files if not is_bucket(f)]
        if not bfiles or not afiles:
            return None
        res = []
        for fs, bk in ((bfiles, True), (afiles, False)):
            r = self._scan(node, fs, bk)
            for n in reversed(chain):
                r = self._unary(n, r)
            res.append(self._scan_agg(r, fns, None, graph_ok=False))
            if bk:
                pruned = self.metrics.get("scan_key_ranges")
        self.metrics["scan_key_ranges"] = pruned     # the bucket files' scan, not the flat one
        sums, cnts, mins, maxs = (t.clone() for t in res[0][:4])
        x = res[1]
        sums.add_(x[0])
        cnts.add_(x[1])
        torch.minimum(mins, x[2], out=mins)
        torch.maximum(maxs, x[3], out=maxs)
        self.metrics["mixed_scan_agg"] = (len(bfiles), len(afiles))
        return sums, cnts, mins, maxs, 1, 0, None, None

    def _union_agg(self, node: X.UnionExec, fns):
        """An ungrouped aggregate over UNION ALL (a Hybrid Scan filter query: the index scan
        plus the appended files, FilterIndexRule's hybrid union) as one fused scan aggregate
        per branch - the index branch keeps its key-range pruning - with the partial results
        combined on the device (an aggregate distributes over UNION ALL), instead of
        materializing and concatenating every branch's rows first."""
        import torch
        res = []
        for child in node.children:
            r = self._rel(child)
            if r.parts or r.table is None:
                raise Unsupported("union branch is a bucket union")
            colmap = dict(r.colmap)
            for u, c in zip(node.output, child.output):
                if c.expr_id in r.colmap:
                    colmap[u.expr_id] = r.colmap[c.expr_id]
            res.append(self._scan_agg(r.copy(colmap=colmap), fns, None, graph_ok=False))
        sums, cnts, mins, maxs = (t.clone() for t in res[0][:4])
        for x in res[1:]:
            sums.add_(x[0])
            cnts.add_(x[1])
            torch.minimum(mins, x[2], out=mins)
            torch.maximum(maxs, x[3], out=maxs)
        return sums, cnts, mins, maxs, 1, 0, None, None

    def _scan_agg(self, r: DRel, fns, group, prep: Optional["_ScanPrep"] = None,
                  graph_ok: bool = True):
        """Fused scan + filter + aggregate.  ``prep`` (a plan-cache hit submitting the same plan
        nodes again, ``_dense_agg``) carries what does not depend on literal values - column
        slots, group domain, compact encodings, the generated kernel, the captured graph and
        the column argument slots - so only the literal-dependent work runs: range bounds,
        predicate values, aggregate terms, the args block and the launch."""
        if prep is None:
            col_info, descs = self._column_infos([(r, 0)])
        else:
            col_info, descs = prep.col_info, prep.descs
        nd = len(descs)
        lkey = prep.literal_key() if prep is not None else None
        low = prep.lowered.get(lkey) if lkey is not None else None
        if low is None:
            implied: set = set()
            spec = self._range_spec(r, r.conds, implied)
            bound = CP.bind(CP.to_cnf([c for c in r.conds if id(c) not in implied]), col_info,
                            self.device)
            specs = self._agg_specs(fns, col_info)
            if lkey is not None:
                if len(prep.lowered) >= 1024:
                    prep.lowered.clear()
                prep.lowered[lkey] = (spec, bound, specs)
        else:
            spec, bound, specs = low
        graph = graph_ok and self._graph_eligible(spec, descs)
        self.metrics["scan_key_ranges"] = spec is not None   # leading-key range pruning
        if not graph:
            with stage("scan.ranges"):
                rstart, rlen, _ = self._ranges(r, r.conds) if spec is not None else \
                    self._full_ranges(r.table)
        if prep is None:
            gs = self._group_spec(r, group, _group_limit(MAX_GROUPS_SCAN, GROUP_LDS_SCAN,
                                                         len(fns)))
        else:
            gs = prep.gs
            if len(descs) != nd or (prep.graph is not None) != graph:
                raise _Stale()
        if gs is None:  # empty group column
            return (*self._empty_agg(len(specs)), 1, 0, None, None)
        agreed, G, gbase, gdict, gtype = gs
        self._groups_agreed = agreed is True
        if prep is None:
            p = NL.ScanParams()
            # a single-valued group key runs the register-accumulating (ungrouped) kernel
            p.group_col = col_info(group).slot if (group is not None and G > 1) else -1
            p.num_groups, p.group_base = G, gbase
            for s_, c in descs.items():
                p.cols[s_] = c.desc()
        else:
            p = prep.params
        for i, pr in enumerate(bound.preds):
            p.preds[i] = pr
        p.npreds = len(bound.preds)
        for i, a in enumerate(specs):
            p.aggs[i] = a
        p.naggs = len(specs)
        self._scan_gs = (col_info, descs, gs, p)
        if bound.always_false:
            out = self._empty_agg(len(specs), G)
        elif graph:
            with stage("scan.graph"):
                out = self._scan_agg_graph(r, p, spec,
                                           p.naggs * (p.num_groups if p.group_col >= 0 else 1),
                                           descs, keep=bound.buffers,
                                           prep=prep.graph if prep is not None else None,
                                           lkey=lkey)
        else:
            with stage("scan.agg_kernel"):
                tp = K.ranges_to_tiles(rlen)
                if HyperspaceConf.codegen_enabled(self.session.conf):
                    out = jit.scan_agg(p, rstart, rlen, tp, self._compacts(descs),
                                       nrows=r.table.num_rows)
                else:
                    out = K.scan_agg(p, rstart, rlen, tp)
        return (*out, G, gbase, gdict, gtype)

    def _graph_eligible(self, spec, descs) -> bool:
        """Replay a captured hipGraph for this scan (exec/graphs.py): generated kernels and a
        range search over all of this rank's buckets (equality bucket pruning changes the
        launch shape)."""
        if spec is None or spec[5] is not None:
            return False
        conf = self.session.conf
        return HyperspaceConf.codegen_enabled(conf) and HyperspaceConf.hipgraph_enabled(conf)

    def _scan_agg_graph(self, r: DRel, p: NL.ScanParams, spec, GA: int, descs=None, keep=(),
                        prep: Optional["_GraphPrep"] = None, lkey=None):
        kc, lo, lo_incl, hi, hi_incl, _ = spec
        if prep is None or prep.GA != GA or self.graphs.peek(prep.key) is not prep.g:
            prep = self._graph_prep(r, p, kc, GA, descs)
            self._last_graph_prep = prep
        g, k, compacts = prep.g, prep.k, prep.compacts
        hit = prep.packed.get(lkey) if lkey is not None else None
        if hit is None:
            values = dict(prep.values)
            jit.fill_preds_aggs(values, [(i, p.preds[i]) for i in range(p.npreds)],
                                [p.aggs[i] for i in range(p.naggs)], compacts)
            # (the per-query predicate buffers the block points to stay referenced with it)
            hit = (range_bounds(lo, lo_incl, hi, hi_incl), _cbuf(k.args.pack(values)),
                   list(keep))
            if lkey is not None:
                if len(prep.packed) >= 1024:
                    prep.packed.clear()
                prep.packed[lkey] = hit
        bounds, packed, _ = hit
        side = self._scan_side_stream(g)
        if side is None:
            if g.on_side:
                import torch
                # side-stream scans were switched off after this pipeline replayed there: its
                # shared intermediates are free only once those replays are done
                torch.cuda.current_stream().wait_stream(g.side_stream)
            handle = g.launch(bounds, packed)
            return (_GraphPending(g, handle), None, None, None)
        import torch
        # a warm pipeline (replays only: no module load, capture or cache fill left) runs on
        # the side stream, after everything queued so far, so it overlaps the queries queued
        # next on this stream (a Q6 scan beside a Q3 merge join: profiles/bench_side_stream_r3).
        # Every replay of the pipeline goes there (its intermediates stay ordered); the
        # buffers it reads are marked in use by that stream, so memory the caller frees
        # meanwhile is not handed out again before the replay is done.
        side.wait_stream(torch.cuda.current_stream())
        if prep.marked is not side:
            for c in list((descs or {}).values()) + [kc]:
                for x in (c.data, c.valid):
                    if x is not None:
                        _use_on(x, side)
            # the generated kernel reads the compact codes (jit._fill_common) rather than
            # c.data: those buffers are in use by the side stream too (a device-cache eviction
            # between this launch and its fetch must not hand their memory to query-stream
            # allocations).  One record per buffer and stream covers every later replay.
            for enc in (compacts or {}).values():
                for x in _compact_buffers(enc):
                    _use_on(x, side)
            for x in g.buffers():
                _use_on(x, side)
            prep.marked = side
        for x in keep:      # per-query predicate buffers (IN sets, key bitmaps)
            _use_on(x, side)
        with torch.cuda.stream(side):
            handle = g.launch(bounds, packed)
        return (_GraphPending(g, handle), None, None, None)

    def _graph_prep(self, r: DRel, p: NL.ScanParams, kc, GA: int, descs) -> "_GraphPrep":
        """The literal-independent part of a graph-replayed scan: kernel, graph, and the args
        slots of the columns and the graph's own buffers."""
        t = r.table
        nb = t.num_buckets
        grid = jit.SCAN_GRID or NL.lib().hs_scan_grid()
        compacts = self._compacts(descs or {})
        vec = jit.scan_vec(p, compacts, t.num_rows)
        shape = jit.scan_agg_shape(p, compacts, vec)
        k = jit.kernel_for(shape, lambda: jit.gen_scan_agg(p, compacts, vec))
        key = (shape, kc.data.data_ptr(), kc.valid.data_ptr() if kc.valid is not None else 0,
               kc.hs_type, t.bucket_offsets.data_ptr(), nb, grid, GA)
        shmem = GA * 32 if p.group_col >= 0 else 0
        g = self.graphs.get(key, lambda: ScanAggGraph(k, kc.desc(), t.bucket_offsets, nb, grid,
                                                      GA, shmem, self.device, vec))
        values = g.values_template()
        values.update({"num_groups": p.num_groups, "group_base": p.group_base,
                       "nrows": t.num_rows})
        jit._fill_cols(values, p.cols, compacts)
        return _GraphPrep(key, g, k, compacts, values, GA)

    def _scan_side_stream(self, g):
        """The side stream warm scan pipelines replay on (None: replay on the current stream)."""
        if not HyperspaceConf.side_stream_scans(self.session.conf):
            return None
        if not (g.on_side or g.replays > 0):
            return None
        import torch
        s = getattr(self, "_side", None)
        if s is None:
            s = self._side = torch.cuda.Stream(device=self.device)
        g.on_side = True
        g.side_stream = s
        return s

    def _compacts(self, descs: Dict[int, DeviceColumn]) -> Optional[dict]:
        """Compact HBM encodings (exec/encoding.py) the generated kernels read instead."""
        if not HyperspaceConf.hbm_compression_enabled(self.session.conf):
            return None
        from .encoding import compact_of
        out = {}
        for s, c in descs.items():
            if getattr(c, "hs_transient", False):
                continue    # a per-query intermediate: analysing it costs more than it saves
            enc = compact_of(c)
            if enc is not None:
                out[s] = enc
        return out

    def _empty_agg(self, A, G=1):
        import torch
        z = torch.zeros(G * A, dtype=torch.float64, device=self.device)
        zc = torch.zeros(G * A, dtype=torch.int64, device=self.device)
        return z, zc, torch.full_like(z, float("inf")), torch.full_like(z, float("-inf"))

    # ------------------------------------------------------------------------------------------
    # Semi-join through a key-domain bitmap (csrc/kernels/key_bitmap.hip)
    # ------------------------------------------------------------------------------------------
    def _semi_join_agg(self, node: X.SortMergeJoinExec, fns, group):
        """An inner equi-join whose aggregate reads only one side (the probe) and whose other
        side (the build) needs an Exchange - it is not co-partitioned with the probe, e.g. the
        output of another join (TPC-H Q3: (customer x orders) x lineitem; JoinIndexRule cannot
        rewrite a join whose side is a join, JoinIndexRule.scala:100-105,149-150) - runs as a
        scan of the probe side filtered by a bitmap of the build keys, when those keys are
        unique (then the join matches each probe row at most once and multiplies nothing).
        That replaces the Exchange + Sort of both sides and the merge join.  None when the
        shape does not qualify (or the build keys repeat): the general join runs instead."""
        if node.condition is not None or len(node.left_keys) != 1:
            return None
        conf = self.session.conf
        if not HyperspaceConf.codegen_enabled(conf) or \
                str(conf.get("spark.hyperspace.mi.semiJoinBitmap.enabled", "true")).lower() != "true":
            return None
        failed = self.__dict__.setdefault("_semi_failed", {})
        fkey = _semi_fail_key(node)
        if failed.get(fkey) is node:
            return None
        need = set()
        for fn in fns:
            need.update(a.expr_id for a in fn.references())
        if group is not None:
            need.add(group.expr_id)
        lk, rk = node.left_keys[0], node.right_keys[0]
        if not (isinstance(lk, E.Attribute) and isinstance(rk, E.Attribute)):
            return None
        sides = []
        for probe, build, pk, bk in ((node.right, node.left, rk, lk), (node.left, node.right, lk, rk)):
            if not need <= {a.expr_id for a in probe.output}:
                continue
            binner = _strip_exchange(build)
            if binner is None:
                continue
            sides.append((_plan_bytes(build), probe, binner, pk, bk))
        if not sides:
            return None
        _, probe, binner, pk, bk = min(sides, key=lambda x: x[0])
        if not all(pa.types.is_integer(a.data_type) for a in (pk, bk)):
            return None
        pinner = _strip_exchange(probe) or probe
        out = self._copart_semi(pinner, pk, binner, bk, fns, group)
        if out is not None:
            return out
        with stage("semi.build"):
            brel = self._rel(binner)
            if brel.parts:
                return None
            keys = self._materialize(brel, [bk])[bk.expr_id]
            bm = self._semi_bitmap(keys)
        if bm is None:
            if len(failed) > 256:
                failed.clear()
            failed[fkey] = node
            return None
        words, lo, nbits = bm
        prel = self._rel(pinner)
        if prel.parts:
            return None
        cond = CP.KeyBitmap(pk, words, lo, nbits)
        self.last_semi_join = {"build_keys": int(keys.data.numel()), "bitmap_bits": nbits,
                               "probe": "scan"}
        with stage("semi.probe"):
            out = self._semi_runs(prel, pk, words, lo, nbits, fns, group)
            if out is not None:
                self.last_semi_join["probe"] = "runs"
                return out
            return self._scan_agg(prel.copy(conds=prel.conds + [cond]), fns, group)

    def _copart_semi(self, pinner, pk, binner, bk, fns, group):
        """The semi-join's build as a co-partitioned join: a build ``Project/Filter <- inner
        join(orders side, customer side)`` whose kept key ``bk`` comes from the orders side
        (TPC-H Q3: ``(customer x orders) x lineitem``), when another index over the same orders
        files is bucketed by ``bk`` like the probe index is by ``pk`` and covers the orders
        side's columns.  Then the probe joins that index bucket by bucket - the two-phase
        run-keyed merge join of ``_join_agg_pair`` - with the orders side's own filters plus
        ``o_custkey`` in a bitmap of the (unique) customer keys as right-side predicates: one
        small bitmap (the customer key domain, L2-resident) instead of the orders-key bitmap
        (75 MB at SF100, probed at random) and no all-gather of it across ranks.  An inner join
        with unique customer keys pairs every passing orders row with exactly one customer, so
        ``(C x O) x L = L x (O where o_custkey in C)``.  None when the shape or the indexes do
        not qualify."""
        conf = self.session.conf
        if str(conf.get("spark.hyperspace.mi.coPartitionedSemiJoin.enabled", "true")).lower() \
                != "true" or not HyperspaceConf.codegen_enabled(conf):
            return None
        above, node = [], binner
        while isinstance(node, (X.ProjectExec, X.FilterExec)):
            if isinstance(node, X.ProjectExec) and \
                    not all(isinstance(e, E.Attribute) for e in node.project_list):
                return None
            above.append(node)
            node = node.child
        if not (isinstance(node, X.SortMergeJoinExec) and node.join_type == "inner" and
                node.condition is None and len(node.left_keys) == 1):
            return None
        pick = None
        for o, c, ok, ck in ((node.left, node.right, node.left_keys[0], node.right_keys[0]),
                             (node.right, node.left, node.right_keys[0], node.left_keys[0])):
            if any(a.expr_id == bk.expr_id for a in o.output):
                pick = (o, c, ok, ck)
        if pick is None:
            return None
        oside, cside, ojk, cjk = pick
        if not all(isinstance(k, E.Attribute) and pa.types.is_integer(k.data_type)
                   for k in (ojk, cjk)):
            return None
        oids = {a.expr_id for a in oside.output}
        upper = [f for f in above if isinstance(f, X.FilterExec)]
        if any(not {a.expr_id for a in f.condition.references()} <= oids for f in upper):
            return None
        chain, leaf = [], _strip_exchange(oside) or oside
        while isinstance(leaf, (X.ProjectExec, X.FilterExec)):
            chain.append(leaf)
            leaf = leaf.child
        if not isinstance(leaf, X.FileSourceScanExec) or not leaf.relation.is_index():
            return None
        ascan = self._copart_scan(leaf, bk, pinner)
        if ascan is None:
            return None
        prel = self._rel(pinner)
        if prel.parts or not prel.bucketed or prel.num_buckets != ascan.relation.index.num_buckets \
                or not prel.sort_attrs or prel.sort_attrs[0].expr_id != pk.expr_id or \
                pk.data_type != bk.data_type:
            return None
        gs = (None, 1, 0, None, None)
        if group is not None:
            if group.expr_id not in prel.colmap:
                return None
            gs = self._group_spec(prel, group, _group_limit(MAX_GROUPS_JOIN, GROUP_LDS_JOIN,
                                                            len(fns)))
            if gs is None:
                return (*self._empty_agg(len(fns) + 1), 1, 0, None, None)
        with stage("semi.build"):
            crel = self._rel(_strip_exchange(cside) or cside)
            if crel.parts:
                return None
            keys = self._materialize(crel, [cjk])[cjk.expr_id]
            bm = self._semi_bitmap(keys)
        if bm is None:
            return None
        words, lo, nbits = bm
        orel = self._scan_memo(ascan)
        for n in reversed(chain):
            orel = self._unary(n, orel)
        for f in reversed(upper):
            orel = self._unary(f, orel)
        orel = orel.copy(conds=orel.conds + [CP.KeyBitmap(ojk, words, lo, nbits)])
        self.last_semi_join = {"build_keys": int(keys.data.numel()), "bitmap_bits": nbits,
                               "probe": "copart", "index": ascan.relation.index.name}
        agreed, G, gbase, gdict, gtype = gs
        self._groups_agreed = agreed is True
        self._join_rec = None
        with stage("semi.probe"):
            out = self._join_agg_pair(_NoCondition, prel, orel, pk, bk, fns, group, G, gbase)
        self._join_rec = None
        return (*out, G, gbase, gdict, gtype)

    def _copart_scan(self, scan: X.FileSourceScanExec, key, pinner):
        """A scan of an index over the same source files as ``scan``'s index, bucketed by
        ``key`` alone with the probe index's bucket count and holding every column ``scan``
        outputs (``_copart_semi``); the scan node is kept per (scan, index) so the device
        cache and scan memo see one node.  None when no index qualifies."""
        from ..hyperspace import get_context
        from ..actions import states
        from ..rules import rule_utils as RU
        from ..index import tags as T
        from ..plan import logical as L
        idx = scan.relation.index
        probe_scans = pinner.collect(lambda x: isinstance(x, X.FileSourceScanExec))
        if len(probe_scans) != 1 or not probe_scans[0].relation.is_index():
            return None
        nb = probe_scans[0].relation.index.num_buckets
        names = {a.name.lower() for a in scan.output}
        if C.DATA_FILE_NAME_ID.lower() in names:
            return None        # lineage ids are per index: a hybrid-scan delete filter stays
        found = None
        for e in get_context(self.session).index_collection_manager.get_indexes([states.ACTIVE]):
            if e.name == idx.name or e.num_buckets != nb or \
                    [c.lower() for c in e.indexed_columns] != [key.name.lower()] or \
                    not names <= {n.lower() for n in e.schema.names} or \
                    e.source_file_info_set != idx.source_file_info_set:
                continue
            found = e
            break
        if found is None:
            return None
        memo = self.__dict__.setdefault("_copart_scans", {})
        mk = (id(scan), found.name)
        hit = memo.get(mk)
        if hit is not None and hit[0] is scan and hit[1] is found:
            return hit[2]
        loc = found.with_cached_tag(None, T.INMEMORYFILEINDEX_INDEX_ONLY,
                                    lambda: RU._index_file_index(found))
        k, v = C.INDEX_RELATION_IDENTIFIER
        schema = pa.schema([f for f in found.schema if f.name != C.DATA_FILE_NAME_ID])
        rel = L.HadoopFsRelation(loc, None, schema, found.bucket_spec, "parquet", {k: v},
                                 index=found)
        ascan = X.FileSourceScanExec(rel, list(scan.output), [], [], True)
        if len(memo) > 64:
            memo.clear()
        memo[mk] = (scan, found, ascan)
        return ascan

    def _semi_runs(self, r: DRel, key, words, lo: int, nbits: int, fns, group):
        """The semi-join probe over the probe key's run form (``jit_runs.semi_runs_agg``): a
        resident index relation sorted by the key (an index's bucket-sorted indexed column, so
        its rows form runs of equal keys) tests the build bitmap once per run and scans its
        own predicates and aggregates bit-parallel.  None when the shape does not qualify (the
        plain scan with a per-row bitmap predicate runs instead)."""
        conf = self.session.conf
        if not (jit_runs.RS_BITS and HyperspaceConf.codegen_enabled(conf)) or \
                str(conf.get("spark.hyperspace.mi.semiRuns.enabled", "true")).lower() != "true":
            return None
        if r.table is None or r.parts or r.extra or r.split or not r.bucketed or \
                not r.sort_attrs or r.sort_attrs[0].expr_id != key.expr_id:
            return None
        col_info, descs = self._column_infos([(r, 0)])
        kslot = col_info(key).slot
        implied: set = set()
        spec = self._range_spec(r, r.conds, implied)
        bound = CP.bind(CP.to_cnf([c for c in r.conds if id(c) not in implied]), col_info,
                        self.device)
        specs = self._agg_specs(fns, col_info)
        gs = self._group_spec(r, group, _group_limit(MAX_GROUPS_SCAN, GROUP_LDS_SCAN, len(fns)))
        if gs is None:
            return None
        agreed, G, gbase, gdict, gtype = gs
        gslot = col_info(group).slot if (group is not None and G > 1) else -1
        if any(sl >= jit_runs.SPLIT for sl in descs) or len(bound.preds) > NL.MAX_PREDS:
            return None
        comp = self._compacts(descs)
        if not comp or kslot not in comp or r.col(key).valid is not None:
            return None
        from .encoding import key_runs
        runs = key_runs(comp[kslot])
        if runs is None:
            return None
        comp = dict(comp)
        comp[kslot] = runs
        rstart, rlen, _ = self._ranges(r, r.conds) if spec is not None else \
            self._full_ranges(r.table)
        self._groups_agreed = agreed is True
        if bound.always_false:
            return (*self._empty_agg(len(specs), G), G, gbase, gdict, gtype)
        p = NL.JoinParams()
        for s_, c in descs.items():
            p.cols[s_] = c.desc()
        for i, pr in enumerate(bound.preds):
            p.preds[i] = pr
        p.nlp = p.npreds = len(bound.preds)
        for i, a in enumerate(specs):
            p.aggs[i] = a
        p.naggs = len(specs)
        p.lkey, p.rkey, p.key_is_float = kslot, kslot, 0
        p.group_col, p.num_groups, p.group_base = gslot, G, gbase
        out = jit_runs.semi_runs_agg(p, rstart, rlen, comp, runs, r.table.num_rows, words, lo,
                                     nbits)
        return (*out, G, gbase, gdict, gtype)

    def _semi_project(self, p: X.ProjectExec) -> Optional[DRel]:
        """``Project <- Filter* <- inner join`` whose projection and filters read one side only:
        that side filtered by a bitmap of the other side's (unique) keys - a semi-join, no
        row pairs materialized (TPC-H Q3's customer x orders feeding the lineitem join).  None
        when the shape does not qualify or the other side's keys repeat."""
        filters, node = [], p.child
        while isinstance(node, X.FilterExec):
            filters.append(node)
            node = node.child
        if not (isinstance(node, X.SortMergeJoinExec) and node.join_type == "inner" and
                node.condition is None and len(node.left_keys) == 1):
            return None
        conf = self.session.conf
        if not HyperspaceConf.codegen_enabled(conf) or \
                str(conf.get("spark.hyperspace.mi.semiJoinBitmap.enabled", "true")).lower() != "true" \
                or str(conf.get("spark.hyperspace.mi.semiProject.enabled", "true")).lower() != "true":
            return None
        failed = self.__dict__.setdefault("_semi_failed", {})
        fkey = _semi_fail_key(node)
        if failed.get(fkey) is node:
            return None
        need = set()
        for e in p.project_list:
            need.update(a.expr_id for a in e.references())
        for f in filters:
            need.update(a.expr_id for a in f.condition.references())
        lk, rk = node.left_keys[0], node.right_keys[0]
        if not (isinstance(lk, E.Attribute) and isinstance(rk, E.Attribute)) or \
                not all(pa.types.is_integer(a.data_type) for a in (lk, rk)):
            return None
        cands = []
        for probe, build, pk, bk in ((node.right, node.left, rk, lk),
                                     (node.left, node.right, lk, rk)):
            if need <= {a.expr_id for a in probe.output}:
                cands.append((_plan_bytes(build), probe, build, pk, bk))
        if not cands:
            return None
        _, probe, build, pk, bk = min(cands, key=lambda x: x[0])
        binner = _strip_exchange(build) or build
        pinner = _strip_exchange(probe) or probe
        with stage("semi.build"):
            brel = self._rel(binner)
            if brel.parts:
                return None
            keys = self._materialize(brel, [bk])[bk.expr_id]
            bm = self._semi_bitmap(keys)
        if bm is None:
            if len(failed) > 256:
                failed.clear()
            failed[fkey] = node
            return None
        words, lo, nbits = bm
        r = self._rel(pinner)
        if r.parts:
            return None
        r = r.copy(conds=r.conds + [CP.KeyBitmap(pk, words, lo, nbits)])
        for f in reversed(filters):
            r = self._unary(f, r)
        return self._unary(p, r)

    def _semi_bitmap(self, keys: DeviceColumn):
        """(words, lo, nbits) of the build keys over every rank's keys, or None when they are
        not unique, not integer, empty everywhere or span more than K.MAX_BITMAP_BITS."""
        import torch
        d = self._dist()
        dom = K.key_domain(keys)
        if d is None or d.world == 1:
            if dom is None:
                return None
            lo, hi, n = dom
            if hi - lo + 1 > K.MAX_BITMAP_BITS:
                return None
            words, dup = K.key_bitmap(keys, lo, hi - lo + 1)
            return None if dup else (words, lo, hi - lo + 1)
        # every rank: the global domain (one all-reduce), its own keys' bits, then the OR of all
        # ranks' bitmaps (all-gather) and a uniqueness check by population count
        big = 1 << 62
        lo, hi, n = dom if dom is not None else (big, -big, 0)
        t = torch.tensor([lo, -hi, 0], dtype=torch.int64, device=self.device)
        t2 = torch.tensor([n], dtype=torch.int64, device=self.device)
        d.all_reduce(t, "min")
        d.all_reduce(t2, "sum")
        glo, ghi, gn = int(t[0].item()), -int(t[1].item()), int(t2[0].item())
        if gn == 0 or ghi - glo + 1 > K.MAX_BITMAP_BITS:
            return None
        nbits = ghi - glo + 1
        if dom is not None:
            words, _ = K.key_bitmap(keys, glo, nbits)
        else:
            words = torch.zeros((nbits + 63) // 64, dtype=torch.int64, device=self.device)
        allw = d.all_gather_tensor(words).view(d.world, -1)
        words = allw[0].clone()
        for r in range(1, d.world):
            words.bitwise_or_(allw[r])
        if K.bitmap_popcount(words) != gn:
            return None
        return words, glo, nbits

    def _join_agg(self, node: X.SortMergeJoinExec, fns, group):
        """Fused join + aggregate.  A side that is a BucketUnion (Hybrid Scan: index buckets plus
        appended rows shuffled by the index bucket spec) is a list of co-partitioned sorted parts;
        an inner join distributes over union, so every (left part, right part) pair runs as its
        own co-located join and the partial aggregates combine — the index side is never
        re-sorted together with the appended rows."""
        left, right, lk, rk = self._join_inputs(node)
        lparts, rparts = left.parts or [left], right.parts or [right]
        gs = (None, 1, 0, None, None)
        if group is not None:
            side = lparts if any(group.expr_id in x.colmap for x in lparts) else rparts
            gs = self._group_spec_parts(side, group, _group_limit(MAX_GROUPS_JOIN, GROUP_LDS_JOIN,
                                                                  len(fns)))
            if gs is None:
                return (*self._empty_agg(len(fns) + 1), 1, 0, None, None)
        agreed, G, gbase, gdict, gtype = gs
        self._groups_agreed = agreed is True
        out = None
        for lp in lparts:
            for rp in rparts:
                part = self._join_agg_pair(node, lp, rp, lk, rk, fns, group, G, gbase)
                out = part if out is None else _combine_aggs(out, part)
        if len(lparts) * len(rparts) > 1:
            self._join_rec = None       # a bucket union: no single replayable launch
        return (*out, G, gbase, gdict, gtype)

    def _group_spec_parts(self, parts, group, limit):
        specs = [self._group_spec(x, group, limit) for x in parts if group.expr_id in x.colmap]
        specs = [s for s in specs if s is not None]
        if not specs:
            return None
        if len(specs) == 1:
            return specs[0]
        if any(s[3] is not None for s in specs):
            raise _NeedHash("string group key over a bucket union")
        lo = min(s[2] for s in specs)
        hi = max(s[2] + s[1] for s in specs)
        if hi - lo > limit:
            raise _NeedHash("group domain too large for LDS aggregation")
        return (True if all(s[0] is True for s in specs) else None), hi - lo, lo, None, specs[0][4]

    def _join_agg_pair(self, node, left: DRel, right: DRel, lk, rk, fns, group, G, gbase):
        # drive the kernel from a much smaller side (the appended part of a hybrid scan).  Only
        # then: one work item per driving row is cheapest when each finds few matches, so a
        # many-to-one pair like lineitem⋈orders (4:1) keeps the many side driving — swapping it
        # made TPC-H Q3 2.5x slower on MI355X (profiles/bench_sf100_r1_v5.json)
        if right.table.num_rows * 64 < left.table.num_rows:
            left, right, lk, rk = right, left, rk, lk
        implied: set = set()
        probed = self._probe_ranges(left, right, lk, rk)
        if probed is None:
            probed = self._domain_pruned_ranges(left, right, lk, rk)
        if probed is not None:
            rstart, rlen, rbk = probed
        else:
            rstart, rlen, rbk = self._ranges(left, left.conds, implied)
        jp, col_info, descs, keep = self._join_params(
            left, right, lk, rk, node.condition,
            lconds=[c for c in left.conds if id(c) not in implied])
        specs = self._agg_specs(fns, col_info)
        if group is not None:
            col_info(group)
            jp.group_col = col_info(group).slot if G > 1 else -1
            jp.num_groups, jp.group_base = G, gbase
        for s, c in descs.items():
            jp.cols[s] = c.desc()
        for i, a in enumerate(specs):
            jp.aggs[i] = a
        jp.naggs = len(specs)
        if keep[0].always_false or keep[1].always_false or left.table.num_rows == 0 or \
                right.table.num_rows == 0:
            return self._empty_agg(len(specs), G)
        max_tiles = K.join_max_tiles(left.table.num_rows, rlen.numel())
        conf = self.session.conf
        if HyperspaceConf.codegen_enabled(conf) and HyperspaceConf.join_index_enabled(conf) and \
                getattr(left.table, "global_key", None) is not None and \
                getattr(right.table, "global_key", None) is not None and \
                join_index.eligible(left.table, right.table, left.col(lk), right.col(rk)):
            # both sides are resident index tables: join through the cached join index
            with stage("join.index"):
                fs, fl, fb = self._full_ranges(left.table)
                jidx = join_index.get_join_index(jp, left.table, right.table, left.col(lk),
                                                 right.col(rk), fs, fl, fb)
            with stage("join.index_agg_kernel"):
                return jit.join_index_agg(jp, rstart, rlen, jidx, self._compacts(descs),
                                          nrows=left.table.num_rows,
                                          rnrows=right.table.num_rows)
        with stage("join.agg_kernel"):
            if HyperspaceConf.codegen_enabled(self.session.conf):
                fr = getattr(left.table, "_full_ranges", None)
                comp = self._compacts(descs)
                if jit.merge_join_ok(jp, comp, right.table.num_rows, left.table.num_rows):
                    jit.LAST_MJ_LAUNCHER[0] = None
                    out = jit.merge_join_agg(jp, rstart, rlen, rbk, right.table.bucket_offsets,
                                             comp, nrows=left.table.num_rows,
                                             cache_spans=fr is not None and rstart is fr[0],
                                             rdup=jit.key_has_dups(right.col(rk)))
                    if fr is not None and rstart is fr[0] and probed is None:
                        # full ranges, no probing: the launch can be replayed for this pair
                        # (``implied`` then holds only isnotnull(key) conjuncts the full ranges
                        # satisfy; the replay binds the same left conjuncts as this launch)
                        self._join_rec = (left, right, lk, rk, col_info, descs,
                                          jit.LAST_MJ_LAUNCHER[0], specs,
                                          [c for c in left.conds if id(c) not in implied])
                    return out
                return jit.join_agg(jp, rstart, rlen, rbk, right.table.bucket_offsets, max_tiles,
                                    self._compacts(descs),
                                    cache_spans=fr is not None and rstart is fr[0])
            return K.join_agg(jp, rstart, rlen, rbk, right.table.bucket_offsets, max_tiles)

    # ------------------------------------------------------------------------------------------
    # Hash-mode aggregation (multi-column / high-cardinality / float keys; exec/hash_agg.py)
    # ------------------------------------------------------------------------------------------
    def _hash_agg(self, final: X.HashAggregateExec, child: X.SparkPlan, order, limit):
        """GROUP BY through the device hash table: every (part) launch of the fused scan or
        merge-join kernel inserts into one table, ``hs_hagg_extract`` compacts it, ranks merge
        their groups, and ORDER BY ... LIMIT picks its candidates on the device.  Kernels and the
        extract are queued now; ``finish`` reads the group count (re-running with a 4x table if
        the size guess overflowed) and copies the result."""
        from . import hash_agg as H
        if not HyperspaceConf.codegen_enabled(self.session.conf):
            raise Unsupported("hash aggregate needs code generation")
        fns = [fn for _, fn in X.agg_functions(final.aggregates)]
        grouping = list(final.grouping)
        if not all(isinstance(g, E.Attribute) for g in grouping):
            raise Unsupported("group by expression")
        node = child
        while isinstance(node, X.ProjectExec) and \
                all(isinstance(e, E.Attribute) for e in node.project_list):
            node = node.child
        fd = None
        if isinstance(node, X.SortMergeJoinExec) and node.join_type == "inner":
            left, right, lk, rk = self._join_inputs(node)
            lparts, rparts = left.parts or [left], right.parts or [right]
            rels = lparts + rparts
            launches = [("join", lp, rp) for lp in lparts for rp in rparts]
            fd = self._fd_grouping(final, grouping, left, right, lk, rk, order, limit)
            if fd is not None:
                grouping = fd[0]
        else:
            r = self._rel(child)
            rels = r.parts or [r]
            launches = [("scan", x, None) for x in rels]
        doms = {g.expr_id: self._union_domain(rels, g) for g in grouping}
        A = len(fns) + 1
        minmax = any(isinstance(fn, (E.Min, E.Max)) for fn in fns)
        shape_key = (tuple(g.name for g in grouping), tuple(fn.sql() for fn in fns),
                     tuple(id(x.table) for x in rels))
        est = min(sum(x.table.num_rows or 0 for x in rels), 1 << 40)
        span = 1
        for g in grouping:
            span *= max(1, doms[g.expr_id][1]) + 1 if doms[g.expr_id][1] else (1 << 32)
        est = max(1, min(est, span))
        hk_box: list = []
        tk_box: list = []
        # ORDER BY <sum / count> LIMIT k over the key-run hash walk: whole keys compete in the
        # walk's per-wavefront top-K lists and only split keys use the table (TopKPlan)
        tk_req = self._topk_request(final, fns, order, limit, minmax) if fd is not None else None

        def run(M: int, use_tk: bool = True):
            table = self.htables.get(M, A, minmax, self.device)
            tk_box.clear()
            with stage("hagg.kernels"):
                for kind, a, b in launches:
                    if kind == "join":
                        self._join_hash_pair(node, a, b, lk, rk, fns, grouping, doms, table, hk_box,
                                             tk_req=tk_req if use_tk else None, tk_box=tk_box)
                    else:
                        self._scan_hash(a, fns, grouping, doms, table, hk_box)
            with stage("hagg.extract"):
                return table.extract(A - 1)

        M = self.htables.slots_for(shape_key, est)
        groups = run(M)
        d = self._dist()

        def finish() -> pa.Table:
            if fd is not None and d is not None and d.world > 1:
                # keys partitioned by bucket: this rank's top candidates, then result rows
                # from every rank (one exchange; the caller sorts and cuts)
                t = local()
                with stage("hagg.gather_rows"):
                    return _gather_tables(d, t)
            return local()

        def local() -> pa.Table:
            nonlocal groups, M
            with stage("hagg.result"):
                hk = hk_box[0] if hk_box else None
                tk = tk_box[0] if tk_box and tk_box[0].used else None
                if tk is not None and hk is not None:
                    # run top-K: candidates, the table's size and the candidates' right
                    # columns in one copy (_topk_fast, _fd_device)
                    fdd = self._fd_device(hk, right, rk, fd) if fd is not None else None
                    st, host, G = self._topk_fast(tk, groups, hk, A, int(limit), fdd)
                    while st == "over":
                        if M >= H.MAX_SLOTS:
                            raise Unsupported("hash aggregate table too large")
                        M *= 4
                        groups = run(M)
                        st, host, G = self._topk_fast(tk_box[0], groups, hk, A, int(limit), fdd)
                    self.htables.record(shape_key, M, G)
                    if st == "ok":
                        self.metrics["run_topk"] = 1
                        ex = None
                        if fd is not None and "fd" in host:
                            def ex(gmap, host):
                                _fd_columns(fd[1], fdd["cols"], host["fd"], gmap)
                        elif fd is not None:
                            def ex(gmap, host):
                                self._fd_lookup(right, rk, fd[1], gmap[fd[0][0].expr_id], gmap)
                        return self._hash_table_out(final, fns, grouping, hk, host, A, ex)
                    # a dropped value may tie the k-th one (or ties flood the copy): exact path
                    self.metrics["run_topk"] = 0
                    groups = run(M, use_tk=False)
                G, over = groups.count()
                while over:
                    if M >= H.MAX_SLOTS:
                        raise Unsupported("hash aggregate table too large")
                    M *= 4
                    groups = run(M, use_tk=False)
                    G, over = groups.count()
                self.htables.record(shape_key, M, G)
                extra = None
                if fd is not None:
                    def extra(gmap, host):
                        self._fd_lookup(right, rk, fd[1], gmap[fd[0][0].expr_id], gmap)
                if d is not None and d.world > 1 and fd is None:
                    groups, G = self._hash_combine_ranks(d, groups, G, A, minmax)
                if hk is None or G == 0:
                    return self._hash_table_out(final, fns, grouping, hk, None, A)
                src = self._topk_source(final, fns, grouping, hk, order, limit, G)
                if src is not None:
                    groups, G = H.topk_candidates(groups, G, src, int(limit))
                return self._hash_table_out(final, fns, grouping, hk, groups.to_host(G), A,
                                            extra)
        return finish

    # keys per functional-dependency lookup (one probe per key, in the key's bucket)
    FD_MAX_KEYS = 1 << 22

    def _fd_grouping(self, final, grouping, left: DRel, right: DRel, lk, rk, order, limit):
        """GROUP BY (left join key, right columns...) over an inner join whose right key is
        unique: every right column is a function of the key (TPC-H Q3's ``l_orderkey,
        o_orderdate, o_shippriority``), so the groups are the left key's and the right columns
        are looked up for the result groups only (``_fd_lookup``).  The reduced grouping lets
        the run-keyed two-phase join aggregate into the hash table (jit_runs hash walk).  Returns
        ([the key attribute], [right attributes]) or None.  Applies when the result is bounded
        by an ORDER BY <aggregate> LIMIT k (device top-k).  Sharded across ranks the key is
        both sides' bucket key, so every key's groups live on one rank: each rank finishes its
        own top candidates and the ranks exchange result rows only (``_gather_tables``); the
        table-dependent checks are agreed once per table pair, so every rank takes the same
        path."""
        if not HyperspaceConf.fd_group_enabled(self.session.conf):
            return None
        if left.parts or right.parts or not order or limit is None or \
                not 0 < int(limit) <= 1024:
            return None
        d = self._dist()
        if d is not None and d.world > 1:
            gk = (getattr(left.table, "global_key", None), getattr(right.table, "global_key", None),
                  lk.name, rk.name, tuple(g.name for g in grouping))
            if gk[0] is None or gk[1] is None:
                return None
            memo = self.__dict__.setdefault("_fd_agreed", {})
            ok = memo.get(gk)
            if ok is None:
                local = self._fd_grouping_local(final, grouping, left, right, lk, rk, order)
                ok = not d.agree_any([local is None])[0]
                memo[gk] = ok
            return self._fd_grouping_local(final, grouping, left, right, lk, rk, order,
                                           check=False) if ok else None
        return self._fd_grouping_local(final, grouping, left, right, lk, rk, order)

    def _fd_grouping_local(self, final, grouping, left: DRel, right: DRel, lk, rk, order,
                           check: bool = True):
        """``_fd_grouping`` on this rank's tables (``check``: the data-dependent checks too)."""
        if check and (right.table.num_rows or 0) * 64 < (left.table.num_rows or 0):
            return None          # _join_hash_pair would swap the sides
        keyg = [g for g in grouping if g.expr_id in (lk.expr_id, rk.expr_id)]
        rest = [g for g in grouping if g.expr_id not in (lk.expr_id, rk.expr_id)]
        if len(keyg) != 1 or not rest:
            return None
        if any(g.expr_id not in right.colmap or g.expr_id in left.colmap for g in rest):
            return None
        lc, rc = left.col(lk), right.col(rk)
        if lc.is_float or rc.is_float or lc.dictionary is not None or \
                rc.dictionary is not None or lc.valid is not None or \
                rc.hs_type not in (NL.I8, NL.I16, NL.I32, NL.I64):
            return None
        e = order[0].child
        if not isinstance(e, E.Attribute):
            return None
        ok = False
        for agg in final.aggregates:
            a = agg if isinstance(agg, E.Attribute) else agg.to_attribute()
            if a.expr_id == e.expr_id:
                inner = agg.child if isinstance(agg, E.Alias) else agg
                ok = isinstance(inner, E.AggregateFunction)
        if not ok or (check and jit.key_has_dups(rc)):
            return None
        g = keyg[0]
        if g.expr_id != lk.expr_id:      # the right key's attribute: group by the left's
            g = lk
        return [g], rest

    def _fd_lookup(self, right: DRel, rk, attrs, keys: pa.Array, gmap: dict) -> None:
        """``gmap[attr] = right[attr]`` at the right row of each key (unique right keys; the
        row is found by one equality probe in the key's bucket, as ``_probe_ranges``)."""
        import torch
        G = len(keys)
        if G == 0:
            for a in attrs:
                gmap[a.expr_id] = pa.array([], type=a.data_type)
            return
        if G > self.FD_MAX_KEYS:
            raise RuntimeError(f"functional-dependency lookup of {G} keys")
        rc = right.col(rk)
        width = {NL.I8: 8, NL.I16: 16, NL.I32: 32, NL.I64: 64}[rc.hs_type]
        vals = np.asarray(keys.cast(pa.int64()).to_numpy(zero_copy_only=False), dtype=np.int64)
        if width == 64:
            img = vals.view(np.uint64) ^ np.uint64(1 << 63)
        else:
            img = (vals + (1 << (width - 1))).astype(np.uint64)
        nb = len(right.table.bucket_offsets_host) - 1
        # each key probes only its own bucket (the index's Murmur3 bucketing of the right key)
        bids = np.asarray(murmur3.bucket_ids([keys.cast(rk.data_type)], nb), dtype=np.int32)
        # one upload (bucket ids and key images), rows picked on the device, one check after
        # the gathers are queued: the lookup synchronizes once before its column copies
        both = torch.from_numpy(np.concatenate([bids.astype(np.int64), img.view(np.int64)]))
        both = both.to(self.device)
        pb, pk = both[:G].to(torch.int32), both[G:]
        rstart, rlen, _ = K.probe_ranges(rc, right.table.bucket_offsets, pb, pk)
        idx = torch.where(rlen > 0, rstart, torch.zeros_like(rstart))
        cols = K.gather_columns([right.col(a) for a in attrs], idx)
        if int((rlen <= 0).sum().item()):
            raise RuntimeError("functional-dependency lookup: a group key has no right row")
        for a, c in zip(attrs, cols):
            arr = c.to_arrow()
            if not arr.type.equals(a.data_type):
                try:
                    arr = arr.cast(a.data_type)
                except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                    pass
            gmap[a.expr_id] = arr

    def _union_domain(self, rels, g: E.Attribute):
        """(lo, span, scale) of group column ``g`` over every part holding it and every rank.
        Integer columns: their value range (scale None).  float64 columns: the range of the
        exact decimal integers q = x * scale of their compact encoding (exec/encoding.py), so
        such a column packs into a multi-column key; scale 0.0 = no usable encoding (a float
        key then only runs alone, as raw bits).  Dictionary columns need none."""
        from .encoding import compact_of
        lo, hi, seen = None, None, False
        dicts = []
        scale = None
        for x in rels:
            if g.expr_id not in x.colmap:
                continue
            c = x.col(g)
            if c.dictionary is not None:
                dicts.append(c.dictionary)
                continue
            if c.is_float:
                enc = compact_of(c) if c.hs_type == NL.F64 else None
                if enc is None or enc.scale is None or enc.lo is None or \
                        (scale is not None and enc.scale != scale):
                    return (0, 0, 0.0)
                scale = enc.scale
                seen = True
                l0, sp = int(enc.lo), int(enc.hi) - int(enc.lo) + 1
            else:
                seen = True
                l0, sp = self._local_domain(c)
            if sp == 0:
                continue
            lo = l0 if lo is None else min(lo, l0)
            hi = l0 + sp - 1 if hi is None else max(hi, l0 + sp - 1)
        if len(dicts) > 1 and not all(dd.equals(dicts[0]) for dd in dicts[1:]):
            raise Unsupported("string group key with different dictionaries per part")
        d = self._dist()
        if seen and d is not None and d.world > 1:
            import torch
            dev = d.device if d.backend == "nccl" else "cpu"
            big = 1 << 62
            t = torch.tensor([-(lo if lo is not None else big), hi if hi is not None else -big],
                             dtype=torch.int64, device=dev)
            d.all_reduce(t, "max")
            nlo, nhi = -int(t[0].item()), int(t[1].item())
            if nhi < nlo:
                return (0, 0, scale)
            return (nlo, nhi - nlo + 1, scale)
        if lo is None:
            return (0, 0, scale)
        return (lo, hi - lo + 1, scale)

    def _hash_keyplan(self, grouping, col_info, fns, doms, specs, descs):
        from . import hash_agg as H
        items = []
        for g in grouping:
            ci = col_info(g)
            items.append((ci.slot, g, descs[ci.slot], doms[g.expr_id]))
        own = []
        for a in specs:
            own.append(a.kind != NL.AK_COUNT_STAR and
                       any(descs[a.col[t]].valid is not None for t in range(a.nterms)))
        need_star = any(isinstance(fn, (E.Count, E.Avg)) for fn in fns)
        return H.plan_keys(items, tuple(own), need_star)

    def _scan_hash(self, r: DRel, fns, grouping, doms, table, hk_box) -> None:
        col_info, descs = self._column_infos([(r, 0)])
        implied: set = set()
        spec = self._range_spec(r, r.conds, implied)
        with stage("scan.ranges"):
            rstart, rlen, _ = self._ranges(r, r.conds) if spec is not None else \
                self._full_ranges(r.table)
        bound = CP.bind(CP.to_cnf([c for c in r.conds if id(c) not in implied]), col_info,
                        self.device)
        specs = self._agg_specs(fns, col_info)
        hk = self._hash_keyplan(grouping, col_info, fns, doms, specs, descs)
        if not hk_box:
            hk_box.append(hk)
        p = NL.ScanParams()
        p.group_col, p.num_groups, p.group_base = -1, 1, 0
        for s, c in descs.items():
            p.cols[s] = c.desc()
        for i, pr in enumerate(bound.preds):
            p.preds[i] = pr
        p.npreds = len(bound.preds)
        for i, a in enumerate(specs):
            p.aggs[i] = a
        p.naggs = len(specs)
        if bound.always_false or (r.table.num_rows or 0) == 0:
            return
        with stage("scan.hash_agg_kernel"):
            tp = K.ranges_to_tiles(rlen)
            jit.scan_agg(p, rstart, rlen, tp, self._compacts(descs), nrows=r.table.num_rows,
                         hk=hk, htab=table)

    def _topk_request(self, final, fns, order, limit, minmax):
        """(aggregate index, by count, descending, limit) when the query orders by one SUM /
        COUNT aggregate with a small LIMIT (a ``TopKPlan`` can serve it), else None."""
        if not order or limit is None or minmax or not 0 < int(limit) < H_TOPK_K or \
                not HyperspaceConf.run_topk_enabled(self.session.conf):
            return None
        e = order[0].child
        if not isinstance(e, E.Attribute):
            return None
        for agg in final.aggregates:
            a = agg if isinstance(agg, E.Attribute) else agg.to_attribute()
            if a.expr_id != e.expr_id:
                continue
            inner = agg.child if isinstance(agg, E.Alias) else agg
            if not isinstance(inner, (E.Sum, E.Count)):
                return None
            i = next((k for k, fn in enumerate(fns) if fn is inner), None)
            if i is None:
                return None
            return (i, isinstance(inner, E.Count), not order[0].ascending, int(limit))
        return None

    def _topk_plan(self, req, hk, A: int):
        """The cached TopKPlan of a request (buffers reused across queries), or None when the
        order aggregate keeps its own non-null count (a NULL sum has no order value there)."""
        from . import hash_agg as H
        i, by_count, desc, limit = req
        if (hk.own_counts[i] and not by_count) or any(c.nullable for c in hk.cols):
            return None
        plans = self.__dict__.setdefault("_tkplans", {})
        K = 16 if limit <= 16 else 32
        key = (i, by_count, desc, A, K)
        tk = plans.get(key)
        if tk is None:
            tk = plans[key] = H.TopKPlan(i, by_count, desc, A, K)
        return tk

    def _fd_device(self, hk, right: DRel, rk, fd) -> Optional[dict]:
        """The device functional-dependency lookup of run top-K candidates
        (``TopKPlan.gather``'s ``fd``): a single non-null integer key column and at most
        ``TopKPlan.FD_COLS`` fixed-width right columns; None otherwise (``_fd_lookup``)."""
        from . import hash_agg as H
        if len(hk.cols) != 1 or hk.mode not in ("packed", "raw_int") or len(fd[1]) > \
                H.TopKPlan.FD_COLS:
            return None
        c = hk.cols[0]
        if c.kind != "int" or c.nullable or c.dictionary is not None:
            return None
        key = right.col(rk)
        if key.hs_type not in (NL.I8, NL.I16, NL.I32, NL.I64) or key.valid is not None or \
                right.table.bucket_offsets is None:
            return None
        cols = [right.col(a) for a in fd[1]]
        if any(x.offsets is not None for x in cols):
            return None
        raw = hk.mode == "raw_int"
        mask = ((1 << c.bits) - 1) if c.bits < 64 else (1 << 64) - 1
        return {"raw": raw, "lo": 0 if raw else int(c.lo), "shift": 0 if raw else int(c.shift),
                "mask": mask, "key": key, "off": right.table.bucket_offsets,
                "nb": len(right.table.bucket_offsets_host) - 1, "cols": cols}

    def _topk_fast(self, tk, groups, hk, A: int, limit: int, fdd: Optional[dict] = None):
        """(status, host group arrays, table groups) of a run top-K query from one packed copy
        (``TopKPlan.gather``): "ok" with the top-``limit`` candidates of the slots and the
        table (split keys); "over" when the table overflowed (grow and re-run); "exact" when
        the largest value the slots do not hold reaches the k-th best value (a dropped tie is
        possible) or ties of the k-th value overflow the copy (the caller re-runs exactly)."""
        i = tk.agg
        cs = i if hk.own_counts[i] else (A - 1 if hk.need_star else -1)
        r = tk.unpack(tk.gather(groups, cs, limit, fdd), len(fdd["cols"]) if fdd else 0)
        if r["over"]:
            return "over", None, r["G"]
        host = r["host"]
        if host is None:
            return "exact", None, r["G"]
        n = len(host["keys"])
        if r["empty"] and n < limit:
            return "exact", None, r["G"]     # a live entry may share the empty pattern
        if n >= limit:
            vals = np.sort(tk.image(host["sums"], host["cnts"]))[::-1]
            kth = float(vals[limit - 1])
        else:
            kth = -np.inf
        self.metrics["run_topk_guard"] = (float(r["bound"]), kth, n, r["G"])
        if r["bound"] >= kth:
            return "exact", None, r["G"]
        if "fd" in r:
            host["fd"] = r["fd"]
        return "ok", host, r["G"]

    def _join_hash_pair(self, node, left: DRel, right: DRel, lk, rk, fns, grouping, doms,
                        table, hk_box, tk_req=None, tk_box=None) -> None:
        if right.table.num_rows * 64 < left.table.num_rows:
            left, right, lk, rk = right, left, rk, lk
        implied: set = set()
        probed = self._probe_ranges(left, right, lk, rk)
        if probed is None:
            probed = self._domain_pruned_ranges(left, right, lk, rk)
        if probed is not None:
            rstart, rlen, rbk = probed
        else:
            rstart, rlen, rbk = self._ranges(left, left.conds, implied)
        jp, col_info, descs, keep = self._join_params(
            left, right, lk, rk, node.condition,
            lconds=[c for c in left.conds if id(c) not in implied])
        specs = self._agg_specs(fns, col_info)
        hk = self._hash_keyplan(grouping, col_info, fns, doms, specs, descs)
        if not hk_box:
            hk_box.append(hk)
        jp.group_col, jp.num_groups, jp.group_base = -1, 1, 0
        for s, c in descs.items():
            jp.cols[s] = c.desc()
        for i, a in enumerate(specs):
            jp.aggs[i] = a
        jp.naggs = len(specs)
        if keep[0].always_false or keep[1].always_false or left.table.num_rows == 0 or \
                right.table.num_rows == 0:
            return
        comp = self._compacts(descs)
        if not jit.merge_join_ok(jp, comp, right.table.num_rows, left.table.num_rows):
            raise Unsupported("hash aggregate over a join the merge-join kernel cannot run")
        fr = getattr(left.table, "_full_ranges", None)
        tk = self._topk_plan(tk_req, hk, len(specs)) if tk_req is not None else None
        if tk is not None:
            tk.used = False
            tk_box.append(tk)
        with stage("join.hash_agg_kernel"):
            jit.merge_join_agg(jp, rstart, rlen, rbk, right.table.bucket_offsets, comp,
                               nrows=left.table.num_rows,
                               cache_spans=fr is not None and rstart is fr[0],
                               rdup=jit.key_has_dups(right.col(rk)), hk=hk, htab=table, tk=tk)

    def _hash_combine_ranks(self, d, groups, G: int, A: int, minmax: bool):
        """Every rank's groups to every rank (one variable-size all-gather of packed rows, no
        pickling), merged in a device table: ranks may share groups (any key not led by the
        bucket key)."""
        from . import hash_agg as H
        with stage("hagg.combine_ranks"):
            host = groups.to_host(G)
            parts = [host["keys"].view(np.int64).reshape(G, 1),
                     host["nulls"].astype(np.int64).reshape(G, 1),
                     host["sums"].view(np.int64), host["cnts"],
                     host["mins"].view(np.int64), host["maxs"].view(np.int64)]
            rows = np.ascontiguousarray(np.concatenate(parts, axis=1)) if G else \
                np.zeros((0, 2 + 4 * A), np.int64)
            allr = d.all_gather_rows(rows)
            n = allr.shape[0]
            if n == 0:
                return groups, 0

            def col(j):
                return np.ascontiguousarray(allr[:, 2 + j * A: 2 + (j + 1) * A])
            merged_in = H.Groups.from_host(
                {"keys": allr[:, 0].copy().view(np.uint64), "nulls": allr[:, 1].astype(np.uint8),
                 "sums": col(0).view(np.float64), "cnts": col(1),
                 "mins": col(2).view(np.float64), "maxs": col(3).view(np.float64)},
                A, minmax, self.device)
            M = H.next_pow2(max(H.MIN_SLOTS, 2 * n))
            table = self.htables.get(M, A, minmax, self.device)
            g = merged_in
            NL.check(NL.lib().hs_hagg_merge(NL.ptr(g.keys), NL.ptr(g.nulls), NL.ptr(g.sums),
                                            NL.ptr(g.cnts), NL.ptr(g.mins), NL.ptr(g.maxs), n,
                                            g.cap, NL.ptr(table.keys), NL.ptr(table.sums),
                                            NL.ptr(table.cnts), NL.ptr(table.mins),
                                            NL.ptr(table.maxs), M, A, NL.ptr(table.flag),
                                            NL.stream_ptr()), "hs_hagg_merge")
            merged = table.extract(A - 1)
            Gm, over = merged.count()
            if over:
                raise Unsupported("rank merge table overflow")
            return merged, Gm

    def _topk_source(self, final, fns, grouping, hk, order, limit, G):
        """The device top-k image of the primary ORDER BY key, or None (host sort of all)."""
        from . import hash_agg as H
        if not order or limit is None or G <= max(TOPK_MIN_GROUPS, 4 * int(limit)) or \
                int(limit) > 1024 or int(limit) <= 0:
            return None
        o = order[0]
        e = o.child
        if not isinstance(e, E.Attribute):
            return None
        desc = not o.ascending
        A = len(fns) + 1
        for agg in final.aggregates:
            a = agg if isinstance(agg, E.Attribute) else agg.to_attribute()
            if a.expr_id != e.expr_id:
                continue
            inner = agg.child if isinstance(agg, E.Alias) else agg
            if isinstance(inner, E.AggregateFunction):
                i = next(k for k, fn in enumerate(fns) if fn is inner)
                cs = i if hk.own_counts[i] else (A - 1 if hk.need_star else -1)
                src = {E.Sum: H.SRC_SUM, E.Count: H.SRC_COUNT, E.Min: H.SRC_MIN,
                       E.Max: H.SRC_MAX, E.Avg: H.SRC_AVG}.get(type(inner))
                if src is None:
                    return None
                return H.OrderSource(src, i, cs, desc=desc)
            if isinstance(inner, E.Attribute):
                e = inner
                break
            return None
        for j, g in enumerate(grouping):
            if g.expr_id != e.expr_id:
                continue
            c = hk.cols[j]
            if hk.mode == "raw_int":
                return H.OrderSource(H.SRC_RAWINT, desc=desc)
            if hk.mode == "raw_float":
                return H.OrderSource(H.SRC_RAWFLT, desc=desc)
            if c.kind == "f32":
                return None
            mask = (1 << c.bits) - 1 if c.bits < 64 else (1 << 64) - 1
            return H.OrderSource(H.SRC_KEYFIELD, shift=c.shift, mask=mask,
                                 nullable=c.nullable, desc=desc)
        return None

    def _hash_table_out(self, final, fns, grouping, hk, host, A, extra=None) -> pa.Table:
        """Result table of a hash-mode aggregate from its host group arrays (vectorized
        finalize; arithmetic over aggregates with pyarrow.compute).  ``extra(gmap, host)`` adds
        group columns not in the key (``_fd_grouping``)."""
        G = 0 if host is None else len(host["keys"])
        if G and hk is not None and not hk.need_star:
            host["cnts"][:, A - 1] = 1     # COUNT(*) not accumulated: every group has rows
        gmap = {}
        if hk is not None and G:
            for g, arr in zip(grouping, hk.unpack(host["keys"], host["nulls"])):
                gmap[g.expr_id] = arr
        else:
            for g in grouping:
                gmap[g.expr_id] = pa.array([], type=g.data_type)
        if extra is not None:
            extra(gmap, host)
        vals = {}
        for i, fn in enumerate(fns):
            if G:
                cnt = host["cnts"][:, i] if (hk.own_counts[i]) else host["cnts"][:, A - 1]
                vals[id(fn)] = _finalize_array(fn, host["sums"][:, i], cnt, host["mins"][:, i],
                                               host["maxs"][:, i])
            else:
                vals[id(fn)] = pa.array([], type=fn.data_type)
        arrays = []
        for e, a in zip(final.aggregates, final.output):
            arr = _eval_vec(e.child if isinstance(e, E.Alias) else e, vals, gmap, G)
            if not arr.type.equals(a.data_type):
                try:
                    arr = arr.cast(a.data_type)
                except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                    pass
            arrays.append(arr)
        return pa.Table.from_arrays(arrays, names=[a.name for a in final.output])


def _finalize_array(fn, s, c, mn, mx) -> pa.Array:
    """Vectorized ``CP.finalize_value`` over the groups of a hash-mode aggregate."""
    c = np.asarray(c, dtype=np.int64)
    if isinstance(fn, E.Count):
        return pa.array(c, type=pa.int64())
    null = c == 0
    if isinstance(fn, E.Avg):
        with np.errstate(divide="ignore", invalid="ignore"):
            return pa.array(np.where(null, 0.0, s / np.maximum(c, 1)), mask=null)
    v = s if isinstance(fn, E.Sum) else (mn if isinstance(fn, E.Min) else mx)
    v = np.where(null, 0.0, v)
    if CP.int_result(fn):
        return pa.array(np.rint(v).astype(np.int64), mask=null)
    t = fn.child.data_type
    if isinstance(fn, (E.Min, E.Max)) and pa.types.is_date32(t):
        return pa.array(np.rint(v).astype(np.int32), mask=null).view(pa.date32())
    if isinstance(fn, (E.Min, E.Max)) and CP._int_coded(t):
        return pa.array(np.rint(v).astype(np.int64), mask=null).cast(t)
    if isinstance(fn, (E.Min, E.Max)) and pa.types.is_decimal(t):
        return pa.array([CP.finalize_value(fn, 0.0, 1, x, x) if not nl else None
                         for x, nl in zip(v, null)], type=t)
    return pa.array(v.astype(np.float64), mask=null)


def _eval_vec(e, vals, gmap, n: int) -> pa.Array:
    """Output expression of an aggregate over whole result columns."""
    import pyarrow.compute as pc
    if isinstance(e, E.AggregateFunction):
        return vals[id(e)]
    if isinstance(e, E.Attribute):
        if e.expr_id in gmap:
            return gmap[e.expr_id]
        raise Unsupported(f"result column {e.sql()}")
    if isinstance(e, E.Literal):
        return pa.array([e.value] * n)
    if isinstance(e, E.Alias):
        return _eval_vec(e.child, vals, gmap, n)
    if isinstance(e, E.Cast):
        return _eval_vec(e.child, vals, gmap, n).cast(e.data_type)
    if isinstance(e, E.BinaryArithmetic):
        a = _eval_vec(e.left, vals, gmap, n)
        b = _eval_vec(e.right, vals, gmap, n)
        if isinstance(e, E.Add):
            return pc.add(a, b)
        if isinstance(e, E.Subtract):
            return pc.subtract(a, b)
        if isinstance(e, E.Multiply):
            return pc.multiply(a, b)
        a = pc.cast(a, pa.float64())
        b = pc.cast(b, pa.float64())
        return pc.if_else(pc.equal(b, 0.0), pa.scalar(None, pa.float64()), pc.divide(a, b))
    raise Unsupported(f"result expression {type(e).__name__}")


def _combine_aggs(a, b):
    """Merge two (sum, count, min, max) partial aggregate tuples in place of ``a``."""
    import torch
    a[0].add_(b[0])
    a[1].add_(b[1])
    torch.minimum(a[2], b[2], out=a[2])
    torch.maximum(a[3], b[3], out=a[3])
    return a


def _warm_torch_kernels(device) -> None:
    """Run the PyTorch elementwise / reduction / scan kernels the query paths use once, on
    tiny tensors: ROCm loads a kernel's code object on its first launch (tens of ms each),
    which would otherwise land in the first query that needs it (profiled: floor_divide,
    cumsum, compare + any of the join setup, ~250 ms of a cold Q3)."""
    import torch
    for dt in (torch.int64, torch.int32):
        x = torch.arange(64, dtype=dt, device=device)
        y = x.flip(0)
        (x // 3, x % 3, x + y, x - y, x * y, x == y, x != y, x < y, x <= y, x > y, x >= y,
         torch.cumsum(x, 0), torch.cumsum((x + 1) // 2, 0, out=torch.empty_like(x)),
         torch.aminmax(x), x.max(), x.min(), x.sum(), (x == y).any(), (x == y).all(),
         torch.nonzero(x > 3), x.index_select(0, y.long()), torch.where(x > 3, x, y),
         x.clamp(0, 9), torch.repeat_interleave(x[:4].long(), 2), x.long(), x.int(),
         x.to(torch.float64), torch.minimum(x, y), torch.maximum(x, y), x[1:] == x[:-1],
         (x[1:] != 0) & (x[:-1] != 0), torch.zeros_like(x), torch.full_like(x, 7))
    v = torch.ones(64, dtype=torch.uint8, device=device)
    (v.bool(), v & v, v == 0, v.any(), v.sum(), v.bool().any(), torch.nonzero(v))
    f = torch.linspace(0, 1, 64, dtype=torch.float64, device=device)
    (f + f, f * f, f / 3, f < 0.5, torch.aminmax(f), f.sum(), torch.minimum(f, f),
     torch.maximum(f, f), torch.isnan(f), f.to(torch.int64))
    torch.cuda.synchronize(device)


def _needs_eval(c: E.Expression) -> bool:
    """A predicate over computed values (arithmetic, or a cast that changes a column's values):
    the scan kernels' predicate compiler takes column / literal comparisons (it looks through
    value-preserving casts only), so such a conjunct is evaluated as a computed column."""
    for x in c.iter_tree():
        if isinstance(x, E.BinaryArithmetic):
            return True
        if isinstance(x, E.Cast) and not isinstance(x.child, E.Literal) and \
                not _lossless_cast(x.child.data_type, x.dtype):
            return True
    return False


def _lossless_cast(src: pa.DataType, dst: pa.DataType) -> bool:
    if src == dst:
        return True
    if pa.types.is_integer(src) and pa.types.is_integer(dst):
        return dst.bit_width >= src.bit_width and \
            pa.types.is_signed_integer(dst) >= pa.types.is_signed_integer(src)
    if pa.types.is_float64(dst):
        return pa.types.is_floating(src) or \
            (pa.types.is_integer(src) and src.bit_width <= 32) or pa.types.is_decimal(src)
    return False


def _prefix_sorted(r: DRel, exprs) -> bool:
    if r.parts:
        return all(_prefix_sorted(x, exprs) for x in r.parts)
    if len(exprs) > len(r.sort_attrs):
        return False
    for e, s in zip(exprs, r.sort_attrs):
        if not isinstance(e, E.Attribute):
            return False
        if r.colmap.get(e.expr_id) != r.colmap.get(s.expr_id):
            return False
    return True


def _eval_scalar(e, agg_val, attr_val):
    if isinstance(e, E.AggregateFunction):
        return agg_val(e)
    if isinstance(e, E.Attribute):
        return attr_val(e)
    if isinstance(e, E.Literal):
        return e.value
    if isinstance(e, E.Alias):
        return _eval_scalar(e.child, agg_val, attr_val)
    if isinstance(e, E.Cast):
        return _eval_scalar(e.child, agg_val, attr_val)
    if isinstance(e, E.BinaryArithmetic):
        a = _eval_scalar(e.left, agg_val, attr_val)
        b = _eval_scalar(e.right, agg_val, attr_val)
        if a is None or b is None:
            return None
        if isinstance(e, E.Add):
            return a + b
        if isinstance(e, E.Subtract):
            return a - b
        if isinstance(e, E.Multiply):
            return a * b
        return None if b == 0 else a / b
    raise Unsupported(f"result expression {type(e).__name__}")


def _semi_fail_key(node) -> tuple:
    """Memo key of a semi-join whose build keys repeated: the join node AND the literal values
    under it - a plan-cache hit re-submits the same nodes with other literals, whose filtered
    build side may well be unique."""
    from ..plan.plan_cache import _iter_literals
    lits: list = []
    _iter_literals(node, lits, set())
    try:
        vals = tuple(x.value for x in lits)
        hash(vals)
    except TypeError:
        vals = tuple(id(x) for x in lits)
    return (id(node), vals)


class _Stale(Exception):
    """A prepared lowering no longer matches the query (the normal path runs instead)."""


class _GraphPrep:
    __slots__ = ("key", "g", "k", "compacts", "values", "GA", "packed", "marked")

    def __init__(self, key, g, k, compacts, values, GA):
        self.key, self.g, self.k, self.compacts, self.values, self.GA = \
            key, g, k, compacts, values, GA
        self.packed: Dict[tuple, tuple] = {}     # literal vector -> (range bounds, args block)
        self.marked = None    # the side stream every persistent buffer was marked in use by


def bucket_chunks(per_bucket, budget: int) -> List[tuple]:
    """Contiguous bucket ranges [lo, hi) whose estimated resident bytes (``per_bucket``, the
    decoded bytes of every index of a plan per bucket) stay within half of ``budget`` - the
    pass's tables plus what its kernels derive - one bucket at least per range."""
    cap = max(budget // 2, 1)
    chunks, lo, acc = [], 0, 0.0
    for b, wb in enumerate(per_bucket):
        if acc and acc + wb > cap:
            chunks.append((lo, b))
            lo, acc = b, 0.0
        acc += float(wb)
    chunks.append((lo, len(per_bucket)))
    return chunks


def _literals(exprs) -> list:
    """The Literal nodes under ``exprs`` (depth first)."""
    out = []
    stack = list(reversed(list(exprs)))
    while stack:
        e = stack.pop()
        if isinstance(e, E.Literal):
            out.append(e)
        else:
            stack.extend(reversed(getattr(e, "children", ()) or ()))
    return out


class _ScanPrep:
    """Literal-independent lowering of a fused scan aggregate (GpuBackend._dense_agg), plus
    the literal-dependent part per literal vector (``lowered``): the plan cache binds a query's
    literals into the same Literal nodes of the cached plan, so their values key the range
    bounds, bound predicates and aggregate terms - a repeated parameter set (a dashboard's
    queries) skips predicate compilation altogether."""
    __slots__ = ("final", "r", "col_info", "descs", "gs", "params", "graph", "placement",
                 "lits", "lowered")

    def __init__(self, final, r, col_info, descs, gs, params, graph, placement):
        self.final, self.r, self.col_info, self.descs, self.gs = final, r, col_info, descs, gs
        self.params, self.graph, self.placement = params, graph, placement
        self.lits = _literals(list(r.conds) + list(final.aggregates))
        self.lowered: Dict[tuple, tuple] = {}

    def literal_key(self):
        try:
            k = tuple(x.value for x in self.lits)
            hash(k)
            return k
        except TypeError:
            return None

    def tables(self):
        return (self.r.table,)

    def run(self, be, fns, group):
        return be._scan_agg(self.r, fns, group, self)

    def fast(self, be, fns, group):
        """``run`` for a literal vector whose lowering and graph block are cached, with no
        re-validation beyond the graph's (``_AggProgram`` checked residency); None otherwise."""
        gp = self.graph
        if gp is None:
            return None
        lkey = self.literal_key()
        low = self.lowered.get(lkey) if lkey is not None else None
        hit = gp.packed.get(lkey) if low is not None else None
        if hit is None or low[1].always_false or be.graphs.peek(gp.key) is not gp.g:
            return None
        g = gp.g
        side = gp.marked
        if side is None and (g.on_side or HyperspaceConf.side_stream_scans(be.session.conf)):
            return None     # the full path moves warm replays to the side stream first
        agreed, G, gbase, gdict, gtype = self.gs
        be._groups_agreed = agreed is True
        if side is None:
            handle = g.launch(hit[0], hit[1])
        else:
            import torch
            side.wait_stream(torch.cuda.current_stream())
            for x in hit[2]:
                _use_on(x, side)
            with torch.cuda.stream(side):
                handle = g.launch(hit[0], hit[1])
        return (_GraphPending(g, handle), None, None, None, G, gbase, gdict, gtype)


class _JoinPrep:
    """Literal-independent lowering of a co-located merge-join aggregate: the two resident
    relations, column slots, group domain and the kernel launcher (jit.MergeJoinLauncher).
    A submission re-binds the predicates and aggregate terms and launches."""
    __slots__ = ("final", "node", "left", "right", "lk", "rk", "col_info", "descs", "launcher",
                 "gtail", "placement", "agreed", "lits", "lowered", "lconds")

    def __init__(self, final, node, left, right, lk, rk, col_info, descs, launcher, gtail,
                 placement, agreed, lconds=None):
        self.final, self.node, self.left, self.right = final, node, left, right
        self.lk, self.rk, self.col_info, self.descs = lk, rk, col_info, descs
        self.launcher, self.gtail, self.placement, self.agreed = launcher, gtail, placement, agreed
        # the left conjuncts the recorded launch bound (same order: predicate slots match)
        self.lconds = list(left.conds) if lconds is None else list(lconds)
        conds = list(left.conds) + list(right.conds) + \
            ([node.condition] if node.condition is not None else [])
        self.lits = _literals(conds + list(final.aggregates))
        self.lowered: Dict[tuple, tuple] = {}   # literal vector -> (params, keep, specs)

    literal_key = _ScanPrep.literal_key

    def tables(self):
        return (self.left.table, self.right.table)

    def run(self, be, fns, group):
        left = self.left
        lkey = self.literal_key()
        low = self.lowered.get(lkey) if lkey is not None else None
        if low is None and be._range_spec(left, left.conds) is not None:
            raise _Stale()        # the new literals bound the left key: ranges change
        nd = len(self.descs)
        with stage("join.agg_kernel"):
            if low is None:
                jp, col_info, descs, keep = be._join_params(
                    left, self.right, self.lk, self.rk, self.node.condition,
                    lconds=self.lconds, slots=(self.col_info, self.descs))
                specs = be._agg_specs(fns, col_info)
                if len(descs) != nd:
                    raise _Stale()
                if lkey is not None:
                    if len(self.lowered) >= 1024:
                        self.lowered.clear()
                    self.lowered[lkey] = (jp, keep, specs)
            else:
                jp, keep, specs = low
                col_info = self.col_info
            G, gbase = self.gtail[0], self.gtail[1]
            if keep[0].always_false or keep[1].always_false:
                out = be._empty_agg(len(specs), G)
            else:
                for i, a in enumerate(specs):
                    jp.aggs[i] = a
                jp.naggs = len(specs)
                if group is not None:
                    jp.group_col = col_info(group).slot if G > 1 else -1
                    jp.num_groups, jp.group_base = G, gbase
                if isinstance(self.launcher, jit_runs.TwoPhaseLauncher):
                    out = self.launcher.launch(
                        jp, lkey, graph=HyperspaceConf.join_graph_enabled(be.session.conf))
                    if isinstance(out, _GraphPending):
                        out = (out, None, None, None)
                else:
                    out = self.launcher.launch(jp)
        be._groups_agreed = self.agreed
        return (*out, *self.gtail)

    def fast(self, be, fns, group):
        """``run`` replaying the captured two-phase pipeline for a cached literal vector; None
        when that does not apply (the full ``run`` / planning path runs instead)."""
        launcher = self.launcher
        if not isinstance(launcher, jit_runs.TwoPhaseLauncher) or launcher.graph is None:
            return None
        lkey = self.literal_key()
        low = self.lowered.get(lkey) if lkey is not None else None
        if low is None or lkey not in launcher.gblocks:
            return None
        jp, keep, specs = low
        if keep[0].always_false or keep[1].always_false:
            return None
        out = launcher.launch(jp, lkey, graph=True)
        be._groups_agreed = self.agreed
        return (out, None, None, None, *self.gtail)


class _AggProgram:
    """Prepared re-submission of a fused aggregate plan (GpuBackend._register_program): a
    plan-cache hit binds its literals into the cached plan's nodes and the program replays the
    prepared lowering of its literal vector - a captured hipGraph (scan: ``ScanAggGraph``;
    two-phase merge join: ``TwoPhaseGraph``) - and queues the cross-rank combine, skipping the
    executor's plan walk and every per-query lowering check.  Valid while the device-table
    cache has evicted nothing since it was made (``epoch``); any miss (new literal vector,
    eviction, graph dropped) returns None and the full path runs (and re-registers)."""
    __slots__ = ("final", "fns", "group", "prep", "epoch", "n")

    def __init__(self, be, final, fns, group, prep, epoch):
        self.final, self.fns, self.group, self.prep, self.epoch = final, fns, group, prep, epoch
        self.n = 0

    def submit(self, be, plan, t0):
        if be.cache.epoch != self.epoch:
            return None
        self.n += 1
        if self.n % 64 == 0 and not all(be._holds(t) for t in self.prep.tables()):
            return None      # (also keeps the tables recent in the cache's LRU)
        res = self.prep.fast(be, self.fns, self.group)
        if res is None:
            return None
        finish = be._agg_finish(self.final, self.fns, self.group, res)
        return QueryFuture(be, plan, finish, "native", None, t0)


def _gather_tables(d, t: pa.Table) -> pa.Table:
    """Every rank's (small) result table, concatenated in rank order: Arrow IPC bytes through
    one row all-gather (``DistContext.all_gather_rows``), no pickling."""
    import pyarrow.ipc as ipc
    sink = pa.BufferOutputStream()
    with ipc.new_stream(sink, t.schema) as w:
        w.write_table(t)
    b = sink.getvalue().to_pybytes()
    n = len(b)
    words = np.frombuffer(b + b"\0" * ((-n) % 8), dtype=np.int64)
    allr = d.all_gather_rows(np.concatenate([[n], words]).astype(np.int64).reshape(-1, 1))
    allr = allr.reshape(-1)
    out, i = [], 0
    while i < len(allr):
        nb = int(allr[i])
        nw = (nb + 7) // 8
        out.append(ipc.open_stream(pa.py_buffer(allr[i + 1:i + 1 + nw].tobytes()[:nb])).read_all())
        i += 1 + nw
    out = [x if x.schema.equals(t.schema) else x.cast(t.schema) for x in out]
    return pa.concat_tables(out)


def _fd_columns(attrs, cols, fd, gmap: dict) -> None:
    """``gmap[attr]`` from the device functional-dependency lookup (``TopKPlan.unpack``'s
    rows, 64-bit values and validity per right column)."""
    import torch
    rows, vals, valid = fd
    if (rows < 0).any():
        raise RuntimeError("functional-dependency lookup: a group key has no right row")
    for a, c, v, ok in zip(attrs, cols, vals, valid):
        nd = np.dtype(str(c.data.dtype).replace("torch.", ""))
        x = v.view(np.float64).astype(nd) if c.is_float else v.astype(nd)
        dc = DeviceColumn(torch.from_numpy(x), None if ok.all() else
                          torch.from_numpy(ok.astype(np.uint8)), c.atype, c.dictionary)
        arr = dc.to_arrow()
        if not arr.type.equals(a.data_type):
            try:
                arr = arr.cast(a.data_type)
            except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                pass
        gmap[a.expr_id] = arr


class _NoCondition:
    """A join node stand-in without a residual condition (``_copart_semi``'s derived join)."""
    condition = None


def _strip_exchange(p):
    """The child below a [Sort(local) <-] hash Exchange (a join side Spark would shuffle), or
    None when ``p`` does not start with one."""
    if isinstance(p, X.SortExec) and not p.global_sort:
        p = p.child
    if isinstance(p, X.ShuffleExchangeExec) and isinstance(p.partitioning, X.HashPartitioning):
        return p.child
    return None


def _plan_bytes(p) -> int:
    """Bytes of the files under a physical plan's scans (the build side of a semi-join is the
    side with fewer)."""
    n = 0
    for s in p.collect(lambda x: isinstance(x, X.FileSourceScanExec)):
        try:
            n += sum(int(f.length) for f in s.relation.location.all_files())
        except Exception:  # noqa: BLE001 - a relation without a file listing counts 0
            pass
    return n


def _use_on(x, stream) -> None:
    """``x.record_stream(stream)`` once per (tensor, stream): the caching allocator keeps the
    streams a block was used on until the block is freed, and then waits for the work queued
    on each of them by that time, so one record covers every later use on the stream."""
    if getattr(x, "_hs_used_on", None) is not stream:
        x.record_stream(stream)
        x._hs_used_on = stream


def _compact_buffers(enc) -> list:
    """Device tensors of a compact encoding whose pointers go into a kernel's argument block
    (codes, and a grouped 16-bit form's group bases and wide codes)."""
    out = [enc.codes]
    g = getattr(enc, "g16", None)
    for e in (enc, g if g else None):
        if e is None:
            continue
        for name in ("gbase", "wide", "codes"):
            x = getattr(e, name, None)
            if x is not None and hasattr(x, "record_stream") and all(x is not y for y in out):
                out.append(x)
    return out


class QueryFuture:
    """Handle of a submitted query (``GpuBackend.collect_async``)."""

    def __init__(self, backend, plan, finish, path: str, reason, t0: float):
        self.backend, self.plan = backend, plan
        self.plan_fn = None         # builds the plan when ``plan`` was a bound cached plan
        self._finish = finish
        self.path, self.reason = path, reason
        self._t0 = t0
        self._value = None
        self._done = False

    def result(self) -> pa.Table:
        if not self._done:
            try:
                self._value = self._finish()
            except Unsupported as e:   # e.g. a result expression the device path cannot finish
                plan = self.plan if self.plan is not None else self.plan_fn()
                f = self.backend._fallback(plan, e, self._t0)
                self._value, self.path, self.reason = f.result(), f.path, f.reason
                self.backend.last_path, self.backend.fallback_reason = self.path, self.reason
            self._done = True
            self._finish = None
            self.backend.metrics["last_query_s"] = time.perf_counter() - self._t0
        return self._value


__all__ = ["GpuBackend", "QueryFuture", "C"]
