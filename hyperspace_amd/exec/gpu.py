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

``GpuBackend`` is composed from one module per operator family: ``gpu_agg`` (fused scan
aggregates, prepared lowerings, streaming, cross-rank combine), ``gpu_join`` (co-partitioned
joins and the device shuffle), ``gpu_semi`` (bitmap and co-partitioned semi-joins) and
``gpu_hash`` (hash-mode GROUP BY, run top-K); shared names live in ``gpu_common``.  This module
keeps the query entry points, relations, scans and row output."""
from __future__ import annotations

import time
import weakref
from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa

from ..ops import _lib as NL, kernels as K
from ..plan import expressions as E, physical as X
from ..parallel.placement import routes_by_key
from ..utils import murmur3
from ..utils.conf import HyperspaceConf
from ..utils.tracing import stage, TRACER
from . import compile as CP
from .arrow_eval import key
from .device_cache import (_files_key, DeviceTableCache, load_bucketed_index, load_flat,
                           seeded_index)
from .device_table import DeviceColumn, DeviceTable
from .graphs import GraphCache
from .hbm_budget import rank_budget
from .staging import RESERVE_BLOCK as _RESERVE_BLOCK
from .gpu_common import (arrow_table, _AggProgram, _needs_eval, _prefix_sorted,
                         _warm_torch_kernels, DRel, log, QueryFuture, Unsupported)
from .gpu_agg import AggOps
from .gpu_hash import HashAggOps
from .gpu_join import JoinOps
from .gpu_semi import SemiJoinOps
# re-exported for tests and diagnostics scripts
from .gpu_common import _strip_exchange, bucket_chunks  # noqa: F401


# every live backend of the process (release_process_device_memory)
_BACKENDS: "weakref.WeakSet" = weakref.WeakSet()


def release_process_device_memory() -> None:
    """``GpuBackend.release_device_memory`` for every backend of the process plus the
    process-wide derived caches (build seeds, cached two-phase lowerings, row-packed aggregate
    inputs), then the caching allocator's free blocks: sessions created one after another in
    one process (e.g. ``bench.py``'s side configs) each size their cache for the whole device."""
    import torch
    from . import device_cache, jit_join, jit_runs
    for be in list(_BACKENDS):
        be.release_device_memory()
    device_cache.clear_seeds()
    jit_join._RUNS_LOWERED.clear()
    jit_join._RUNS_HASH_LOWERED.clear()
    jit_runs._PACKS.clear()
    jit_runs._P12.clear()
    jit_join.LAST_MJ_LAUNCHER[0] = None
    # a plain gc.collect() skips what utils/hostgc.py froze: the released sessions' cycles
    # (and the device tensors they hold) are only found after an unfreeze
    from ..utils import hostgc
    hostgc.settle(full=True)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


class GpuBackend(AggOps, JoinOps, SemiJoinOps, HashAggOps):
    name = "gpu"
    # QueryExecution may submit a plan-cache entry's own plan with a query's literals bound in
    # place (plan/plan_cache.py): everything literal-dependent is read during collect_async
    supports_bound_plans = True

    def __init__(self, session):
        import torch
        NL.lib()  # fail loudly if the kernels are not built
        self.session = session
        _BACKENDS.add(self)
        # the generated kernels' tunables: spark.hyperspace.mi.kernel.* over HS_JIT_* over the
        # measured defaults (exec/kernel_config.py)
        from . import kernel_config
        cfg = kernel_config.base().with_conf(session.conf)
        if cfg != kernel_config.active():
            kernel_config.bind(cfg)
        self.device = torch.device("cuda", torch.cuda.current_device())
        # HBM / pinned budgets of this rank: its share of the device when ranks share one
        # (exec/hbm_budget.py), the configured values otherwise
        self.budget = rank_budget(session.conf, self.device)
        self.cache = DeviceTableCache(self.budget.cache)
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
        pool = pinned_pool()
        pool.limit = min(pool.limit, self.budget.pinned)
        pool.reserve(count=max(1, min(32, pool.limit // (2 * _RESERVE_BLOCK))))
        self._engine_start()

    def release_device_memory(self) -> None:
        """Drop everything this backend keeps resident in HBM - index tables, derived join
        indexes and packed columns (with the tables), captured graphs, prepared lowerings - so
        another session of the same process can use the device.  The next query reloads."""
        import torch
        torch.cuda.synchronize(self.device)
        self.cache.clear()
        self._programs.clear()
        self.graphs._lru.clear()
        for k in ("_agg_preps", "_stream_memo", "_side"):
            self.__dict__.pop(k, None)
        from .hash_agg import TablePool
        self.htables = TablePool()

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
        reserve = self.budget.arena
        if reserve > 0:
            free, _ = torch.cuda.mem_get_info(self.device)
            reserve = min(reserve, int(free * 0.8))
            if reserve > (1 << 30):
                try:
                    block = torch.empty(reserve, dtype=torch.uint8, device=self.device)
                    del block   # stays cached in the allocator as one segment
                except torch.OutOfMemoryError:
                    # ranks sharing the device reserve at the same time: the free memory read
                    # above may already be gone - the arena is only a head start, go without
                    pass
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
        new_shape = id(plan) not in self._programs
        self._programs[id(plan)] = (plan, _AggProgram(self, *cand))
        if new_shape and HyperspaceConf.gc_freeze_enabled(self.session.conf):
            from ..utils import hostgc
            hostgc.settle()

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
        """The device relation of a BucketUnion (Hybrid Scan): its parts, or one merged table
        (``_merged_union``).  A merged result is kept per union node while its tables stay
        resident: a plan-cache hit re-submits the same node with its literals rebound in place
        (the kept predicates hold those same literal objects), so the parts' relations, the
        predicate check across parts and the merge lookup run once per node."""
        memo = self.__dict__.setdefault("_union_memo", {})
        tag = self._placement_tag()
        hit = memo.get(id(p))
        if hit is not None and hit[0] is p and hit[2] == tag and self._holds(hit[1].table):
            return hit[1].copy()
        r = self._bucket_union_eval(p)
        if r.table is not None and getattr(r.table, "_hs_sources", None) is not None:
            if len(memo) > 64:
                memo.clear()
            memo[id(p)] = (p, r, tag)
            return r.copy()
        return r

    def _bucket_union_eval(self, p: X.BucketUnionExec) -> DRel:
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
            if nbytes > rank_budget(conf, self.device).cache // 4:
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
        tag = (tag, getattr(self, "_bucket_chunk", None),
               self.session.conf.get("spark.hyperspace.mi.hybridScanMerge.enabled", "true"))
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
            if not bucketed and rel.is_index() and world == 1:
                hy = self._hybrid_scan(p, files)
                if hy is not None:
                    return hy
        if bucketed:
            idx = rel.index
            ncol = {n.lower(): n for n in idx.schema.names}
            cols = [ncol[a.name.lower()] for a in p.output]
            sort_cols = [ncol[c.lower()] for c in idx.indexed_columns]
            load_cols = list(dict.fromkeys(cols + sort_cols))
            owners = self._owner_map(idx.num_buckets, world, files, sort_cols[0])
            if owners.splits and not routes_by_key(idx.schema.field(sort_cols[0]).type):
                owners = owners.unsplit()   # cut keys are integer values (placement.py)
            owned = owners.owned(rank)
            cuts = owners.ranges(rank)      # key ranges of heavy buckets cut across ranks
            chunk = getattr(self, "_bucket_chunk", None)
            if chunk is not None:
                # bucket-range streaming (_streamed_agg): this pass holds buckets [lo, hi) only
                owned = [b for b in owned if chunk[0] <= b < chunk[1]]
            table = self.cache.get(
                files, load_cols, ("bucketed", rank, world, owners.key, chunk),
                lambda: (None if cuts else
                         seeded_index(files, load_cols, idx.num_buckets, rank, world, owned)) or
                load_bucketed_index(files, load_cols, idx.num_buckets, sort_cols, self.device,
                                    rank, world, owned, cuts))
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

    def _hybrid_split(self, p: X.FileSourceScanExec, files):
        """(bucket files, appended files, load columns, sort columns, output columns) of an
        index scan whose file list also holds appended source files (FilterIndexRule's Hybrid
        Scan), or None when they cannot share one device table (string columns: every load has
        its own dictionary; a column missing from the index)."""
        if str(self.session.conf.get("spark.hyperspace.mi.hybridScanMerge.enabled", "true")) \
                .lower() != "true":
            return None
        from ..io.writer import get_bucket_id
        from ..utils import path_utils as P
        from .device_table import is_string
        idx = p.relation.index
        nb = idx.num_buckets
        bfiles, afiles = [], []
        for f in files:
            b = get_bucket_id(P.get_name(f.path))
            (bfiles if b is not None and b < nb else afiles).append(f)
        if not bfiles or not afiles:
            return None
        ncol = {n.lower(): n for n in idx.schema.names}
        cols = [ncol.get(a.name.lower()) for a in p.output]
        if any(c is None for c in cols):
            return None
        sort_cols = [ncol[c.lower()] for c in idx.indexed_columns]
        load_cols = list(dict.fromkeys(cols + sort_cols))
        types = {f.name: f.type for f in idx.schema}
        if any(is_string(types[c]) for c in load_cols):
            return None
        return bfiles, afiles, load_cols, sort_cols, cols

    def _hybrid_scan(self, p: X.FileSourceScanExec, files) -> Optional[DRel]:
        """An index scan with same-scan appended files (Hybrid Scan) as ONE resident table: the
        index buckets as loaded (bucket-sorted), then the appended rows sorted once by the
        indexed columns as one more bucket range.  Every bucket range is sorted by the key,
        so a filter's key-range search prunes the appended rows too, and the query takes the
        single-table paths (prepared lowering, captured graph) like a refreshed index.  The
        extra range carries no bucket identity (``bucket_attrs`` empty): no equality-bucket
        pruning and no co-partitioned join read it as a hash partition."""
        sp = self._hybrid_split(p, files)
        if sp is None:
            return None
        bfiles, afiles, load_cols, sort_cols, cols = sp
        rel = p.relation
        idx = rel.index
        nb = idx.num_buckets
        dev = self.device

        def load():
            import torch
            bt = load_bucketed_index(bfiles, load_cols, nb, sort_cols, dev)
            at = load_flat(afiles, "parquet", load_cols, rel.data_schema, rel.options,
                           rel.location.partition_spec, dev)
            perm = K.sort_permutation([at.columns[c] for c in sort_cols]) if at.num_rows else None
            ag = K.gather_columns([at.columns[c] for c in load_cols], perm) if perm is not None \
                else [at.columns[c] for c in load_cols]
            merged = {}
            for c, a in zip(load_cols, ag):
                b = bt.columns[c]
                if b.data.dtype != a.data.dtype:
                    raise Unsupported(f"hybrid scan: column {c} differs in type")
                valid = None
                if b.valid is not None or a.valid is not None:
                    ones = lambda x: torch.ones(x.data.shape[0], dtype=torch.uint8,  # noqa: E731
                                                device=dev)
                    valid = torch.cat([b.valid if b.valid is not None else ones(b),
                                       a.valid if a.valid is not None else ones(a)])
                merged[c] = DeviceColumn(torch.cat([b.data, a.data]), valid, b.atype, None)
            off = np.concatenate([np.asarray(bt.bucket_offsets_host, dtype=np.int64),
                                  [bt.num_rows + at.num_rows]]).astype(np.int64)
            return DeviceTable(merged, int(off[-1]), torch.from_numpy(off).to(dev), off)
        table = self.cache.get(files, load_cols, ("hybrid-scan", nb), load)
        table.global_key = ("hybrid-scan", _files_key(files), tuple(load_cols))
        colmap = {a.expr_id: c for a, c in zip(p.output, cols)}
        sort_attrs = []
        for c in sort_cols:
            a = next((x for x in p.output if x.name.lower() == c.lower()), None)
            if a is None:
                a = E.Attribute(c, idx.schema.field(c).type)
                colmap[a.expr_id] = c
            sort_attrs.append(a)
        self.metrics["hybrid_scan_merged"] = (len(bfiles), len(afiles))
        return DRel(table, colmap, list(p.output), [], True, sort_attrs, [], nb + 1)

    def _owner_map(self, num_buckets: int, world: int, files=None, key: str = None):
        """The session's bucket -> rank map for this bucket count (parallel/placement.py):
        size-balanced from the first index queried with it (heavy buckets cut into key ranges
        of its leading indexed column ``key``), shared by every later index and query-time
        shuffle with that bucket count (co-partitioned)."""
        from ..parallel.placement import bucket_bounds, bucket_weights, session_map
        if world <= 1:
            return session_map(self.session, num_buckets, 1)
        w = bucket_weights(files, num_buckets) if files is not None else None
        bounds = bucket_bounds(files, num_buckets, key) if files is not None and key else None
        return session_map(self.session, num_buckets, world, w, bounds)

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
        return arrow_table(fixed, [a.name for a in out_attrs])

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
        return arrow_table(arrays, [a.name for a in out_attrs])


__all__ = ["GpuBackend", "QueryFuture", "DRel", "bucket_chunks", "release_process_device_memory"]
