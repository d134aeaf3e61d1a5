"""Host (pyarrow) executor — the correctness oracle for the MI355X executor.

Executes the shared physical plan with Spark's partitioning semantics: a bucketed index scan
yields one partition per bucket, ShuffleExchange(hashpartitioning) re-buckets with Spark Murmur3,
SortMergeJoin zips co-partitioned children, BucketUnion concatenates partition *i* of every
child (``BucketUnionExec.scala:61-74``).
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from ..io.reader import read_files
from ..io.writer import get_bucket_id
from ..plan import expressions as E
from ..plan import physical as X
from ..utils import murmur3
from .arrow_eval import eval_expr, eval_predicate, key


def _schema(attrs) -> pa.Schema:
    return pa.schema([pa.field(key(a), a.data_type, True) for a in attrs])


def _empty(attrs) -> pa.Table:
    return _schema(attrs).empty_table()


def _concat(tables: List[pa.Table], attrs) -> pa.Table:
    tables = [t for t in tables if t is not None]
    if not tables:
        return _empty(attrs)
    sch = _schema(attrs)
    return pa.concat_tables([t.select(sch.names).cast(sch) for t in tables])


class CpuBackend:
    name = "cpu"

    def __init__(self, session):
        self.session = session
        self.metrics: Dict[str, float] = {}
        self.last_path = None         # "host" once a query ran (GpuBackend: native / fallback)
        self.fallback_reason = None

    # -- public -------------------------------------------------------------------------------
    def collect(self, plan: X.SparkPlan) -> pa.Table:
        self._reuse_memo = {}
        try:
            parts = self.execute(plan)
        finally:
            self._reuse_memo = {}
        t = _concat(parts, plan.output)
        self.last_path = "host"
        return pa.Table.from_arrays(t.columns, names=[a.name for a in plan.output])

    def execute(self, p: X.SparkPlan) -> List[pa.Table]:
        fn = getattr(self, "_exec_" + type(p).__name__)
        memo = getattr(self, "_reuse_memo", None)
        if memo is None or not isinstance(p, (X.ShuffleExchangeExec, X.BroadcastExchangeExec)):
            return fn(p)
        hit = memo.get(id(p))
        if hit is None or hit[0] is not p:
            hit = memo[id(p)] = (p, fn(p))
        return hit[1]

    # -- scans ----------------------------------------------------------------------------------
    def _read(self, p: X.FileSourceScanExec, files: List[str]) -> pa.Table:
        rel = p.relation
        cols = [a.name for a in p.output]
        # index data and Delta data files are parquet
        fmt = "parquet" if rel.is_index() or rel.file_format == "delta" else rel.file_format
        data_schema = rel.data_schema
        t = read_files(fmt, files, data_schema, rel.options, rel.location.partition_spec, cols)
        arrays = []
        for a in p.output:
            c = t.column(a.name) if a.name in t.column_names else pa.nulls(t.num_rows, a.data_type)
            if not c.type.equals(a.data_type):
                c = c.cast(a.data_type)
            arrays.append(c)
        return pa.Table.from_arrays(arrays, schema=_schema(p.output))

    def _exec_FileSourceScanExec(self, p):
        files = [f.path for f in p.relation.location.all_files()]
        if p.use_bucketing:
            n = p.relation.bucket_spec.num_buckets
            groups: Dict[int, list] = {}
            for f in files:
                b = get_bucket_id(f.rsplit("/", 1)[-1])
                groups.setdefault(b, []).append(f)
            out = []
            for b in range(n):
                if b in groups and (p.selected_buckets is None or b in p.selected_buckets):
                    out.append(self._read(p, groups[b]))
                else:
                    out.append(_empty(p.output))
            return out
        if not files:
            return [_empty(p.output)]
        return [self._read(p, [f]) for f in files]

    def _exec_LocalTableScanExec(self, p):
        t = p.table
        return [pa.Table.from_arrays(t.columns, schema=_schema(p.output))]

    # -- row operators --------------------------------------------------------------------------
    def _exec_FilterExec(self, p):
        return [eval_predicate(p.condition, t) for t in self.execute(p.child)]

    def _project(self, exprs, t: pa.Table, out_attrs) -> pa.Table:
        arrays = []
        for e, a in zip(exprs, out_attrs):
            c = eval_expr(e, t)
            if isinstance(c, pa.ChunkedArray) and c.num_chunks == 0:
                c = pa.array([], a.data_type)
            if not c.type.equals(a.data_type):
                try:
                    c = c.cast(a.data_type)
                except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                    pass
            arrays.append(c)
        return pa.Table.from_arrays(arrays, names=[key(a) for a in out_attrs])

    def _exec_ProjectExec(self, p):
        out = p.output
        return [self._project(p.project_list, t, out) for t in self.execute(p.child)]

    def _exec_CollectLimitExec(self, p):
        t = _concat(self.execute(p.child), p.output)
        return [t.slice(0, p.n)]

    # -- exchange / sort ------------------------------------------------------------------------
    def _hash_partition(self, t: pa.Table, exprs, n: int) -> List[pa.Table]:
        if t.num_rows == 0:
            return [t.slice(0, 0) for _ in range(n)]
        cols = [eval_expr(e, t) for e in exprs]
        bids = murmur3.bucket_ids(cols, n)
        order = np.argsort(bids, kind="stable")
        bounds = np.searchsorted(bids[order], np.arange(n + 1))
        st = t.take(pa.array(order))
        return [st.slice(int(bounds[i]), int(bounds[i + 1] - bounds[i])) for i in range(n)]

    def _exec_ShuffleExchangeExec(self, p):
        parts = self.execute(p.child)
        t = _concat(parts, p.child.output)
        part = p.partitioning
        if isinstance(part, X.HashPartitioning):
            return self._hash_partition(t, part.expressions, part.num_partitions)
        return [t]

    def _exec_ReusedExchangeExec(self, p):
        # the reused exchange runs once per query; its partitions are renamed positionally
        names = [key(a) for a in p.output]
        return [t.rename_columns(names) for t in self.execute(p.exchange)]

    def _exec_BroadcastExchangeExec(self, p):
        return [_concat(self.execute(p.child), p.child.output)]

    def _sort_table(self, t: pa.Table, order) -> pa.Table:
        if t.num_rows <= 1:
            return t
        tmp = t
        keys = []
        for i, o in enumerate(order):
            name = f"__sort{i}"
            tmp = tmp.append_column(name, eval_expr(o.child, t))
            keys.append((name, "ascending" if o.ascending else "descending",
                         "at_start" if o.ascending else "at_end"))
        idx = pc.sort_indices(tmp, sort_keys=keys)
        return t.take(idx)

    def _exec_SortExec(self, p):
        return [self._sort_table(t, p.order) for t in self.execute(p.child)]

    # -- joins ----------------------------------------------------------------------------------
    def _join_tables(self, lt, rt, lkeys, rkeys, join_type, condition, out_attrs, lattrs, rattrs):
        lt = lt.combine_chunks() if lt.num_rows else lt
        rt = rt.combine_chunks() if rt.num_rows else rt
        lnames, rnames = [], []
        for i, (lk, rk) in enumerate(zip(lkeys, rkeys)):
            lc, rc = eval_expr(lk, lt), eval_expr(rk, rt)
            if not lc.type.equals(rc.type):
                lc, rc = _align_keys(lc, rc)
            lt = lt.append_column(f"__lk{i}", lc)
            rt = rt.append_column(f"__rk{i}", rc)
            lnames.append(f"__lk{i}")
            rnames.append(f"__rk{i}")
        jt = {"inner": "inner", "left": "left outer", "right": "right outer",
              "full": "full outer", "leftsemi": "left semi", "leftanti": "left anti"}[join_type]
        # arrow's hash join: keep both key sets; suffix collisions impossible (unique keys)
        lt = lt.append_column("__lrow", pa.array(np.arange(lt.num_rows, dtype=np.int64)))
        rt = rt.append_column("__rrow", pa.array(np.arange(rt.num_rows, dtype=np.int64)))
        j = lt.join(rt, keys=lnames, right_keys=rnames, join_type=jt, coalesce_keys=False,
                    use_threads=True)
        if join_type in ("leftsemi", "leftanti"):
            res = j.select([key(a) for a in lattrs])
        else:
            res = j.select([key(a) for a in lattrs] + [key(a) for a in rattrs])
        if condition is not None and join_type == "inner":
            res = eval_predicate(condition, res)
        return res

    def _exec_SortMergeJoinExec(self, p):
        lparts = self.execute(p.left)
        rparts = self.execute(p.right)
        assert len(lparts) == len(rparts), (len(lparts), len(rparts))
        return [self._join_tables(l, r, p.left_keys, p.right_keys, p.join_type, p.condition,
                                  p.output, p.left.output, p.right.output)
                for l, r in zip(lparts, rparts)]

    def _exec_BroadcastHashJoinExec(self, p):
        if p.build_side == "right":
            build = _concat(self.execute(p.right), p.right.output)
            return [self._join_tables(l, build, p.left_keys, p.right_keys, p.join_type,
                                      p.condition, p.output, p.left.output, p.right.output)
                    for l in self.execute(p.left)]
        build = _concat(self.execute(p.left), p.left.output)
        return [self._join_tables(build, r, p.left_keys, p.right_keys, p.join_type, p.condition,
                                  p.output, p.left.output, p.right.output)
                for r in self.execute(p.right)]

    def _exec_NestedLoopJoinExec(self, p):
        l = _concat(self.execute(p.children[0]), p.children[0].output)
        r = _concat(self.execute(p.children[1]), p.children[1].output)
        li = np.repeat(np.arange(l.num_rows), r.num_rows)
        ri = np.tile(np.arange(r.num_rows), l.num_rows)
        lt = l.take(pa.array(li))
        rt = r.take(pa.array(ri))
        t = pa.Table.from_arrays(lt.columns + rt.columns, names=lt.column_names + rt.column_names)
        if p.condition is not None:
            t = eval_predicate(p.condition, t)
        return [t]

    # -- aggregation ----------------------------------------------------------------------------
    def _exec_HashAggregateExec(self, p):
        parts = self.execute(p.child)
        if p.mode == "partial":
            return [self._partial_agg(p, t) for t in parts]
        t = _concat(parts, p.child.output) if parts else _empty(p.child.output)
        return [self._final_agg(p, t)]

    def _partial_agg(self, p, t: pa.Table) -> pa.Table:
        fns = X.agg_functions(p.aggregates)
        g_names = [f"g{i}" for i in range(len(p.grouping))]
        cols = {n: eval_expr(g, t) for n, g in zip(g_names, p.grouping)}
        aggs = []
        for i, (_, fn) in enumerate(fns):
            if fn.child is None:
                cols[f"a{i}"] = pa.array(np.ones(t.num_rows, dtype=np.int64))
            else:
                v = eval_expr(fn.child, t)
                if pa.types.is_decimal(v.type):
                    v = pc.cast(v, pa.float64())
                cols[f"a{i}"] = v
            if isinstance(fn, E.Avg):
                aggs += [(f"a{i}", "sum"), (f"a{i}", "count")]
            elif isinstance(fn, E.Count):
                aggs.append((f"a{i}", "count"))
            else:
                aggs.append((f"a{i}", fn.name))
        tt = pa.table(cols) if cols else pa.table({"__x": pa.array(np.zeros(t.num_rows))})
        if g_names:
            r = tt.group_by(g_names, use_threads=False).aggregate(aggs)
            r = r.select([f"{c}_{a}" for c, a in aggs] + g_names)
        else:
            arrays = []
            for c, a in aggs:
                col = tt.column(c)
                if a == "count":
                    arrays.append(pa.array([pc.count(col).as_py()], pa.int64()))
                else:
                    s = getattr(pc, {"sum": "sum", "min": "min", "max": "max"}[a])(col)
                    arrays.append(pa.array([s.as_py()], s.type if s.type != pa.null() else pa.float64()))
            r = pa.Table.from_arrays(arrays, names=[f"{c}_{a}" for c, a in aggs]) if arrays else \
                pa.table({"__x": pa.array([0])})
        names = g_names + [f"{c}_{a}" for c, a in aggs]
        return pa.Table.from_arrays([r.column(n) for n in names if n in r.column_names],
                                    names=[key(a) for a in p.partial_output()])

    def _final_agg(self, p, t: pa.Table) -> pa.Table:
        fns = X.agg_functions(p.aggregates)
        child_out = p.child.output
        ng = len(p.grouping)
        g_keys = [key(a) for a in child_out[:ng]]
        buf = [key(a) for a in child_out[ng:]]
        merges, names = [], []
        bi = 0
        for i, (_, fn) in enumerate(fns):
            if isinstance(fn, E.Avg):
                merges += [(buf[bi], "sum"), (buf[bi + 1], "sum")]
                names.append((f"avg", bi))
                bi += 2
            else:
                merges.append((buf[bi], {"count": "sum", "sum": "sum", "min": "min",
                                         "max": "max"}[fn.name]))
                names.append((fn.name, bi))
                bi += 1
        if ng:
            r = t.group_by(g_keys, use_threads=False).aggregate(merges)
            merged = {c: r.column(f"{c}_{a}") for c, a in merges}
            groups = [r.column(k) for k in g_keys]
            nrows = r.num_rows
        else:
            merged = {}
            for c, a in merges:
                col = t.column(c)
                s = getattr(pc, a)(col) if col.null_count < len(col) else pa.scalar(None)
                v = s.as_py()
                if a == "sum" and v is None and "count" in c:
                    v = 0
                merged[c] = pa.array([v])
            groups = []
            nrows = 1
        # evaluate the result expressions with aggregate results substituted
        env_cols, env_names = [], []
        for gi, g in enumerate(p.grouping):
            env_cols.append(groups[gi])
            env_names.append(f"__g{gi}")
        agg_vals = {}
        for i, ((kind, b), (_, fn)) in enumerate(zip(names, fns)):
            if kind == "avg":
                s, c = merged[buf[b]], merged[buf[b + 1]]
                v = pc.divide(pc.cast(s, pa.float64()), pc.cast(c, pa.float64()))
            else:
                v = merged[buf[b]]
                if kind == "count":
                    v = pc.fill_null(pc.cast(v, pa.int64()), 0)
            agg_vals[id(fn)] = v
        out_arrays = []
        for e in p.aggregates:
            inner = e.child if isinstance(e, E.Alias) else e
            out_arrays.append(self._eval_agg_result(inner, p.grouping, groups, agg_vals, nrows))
        out_attrs = p.output
        fixed = []
        for a, arr in zip(out_attrs, out_arrays):
            if isinstance(arr, pa.ChunkedArray):
                arr = arr.combine_chunks()
            if not arr.type.equals(a.data_type):
                try:
                    arr = arr.cast(a.data_type)
                except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                    pass
            fixed.append(arr)
        return pa.Table.from_arrays(fixed, names=[key(a) for a in out_attrs])

    def _eval_agg_result(self, e, grouping, groups, agg_vals, nrows):
        if isinstance(e, E.AggregateFunction):
            return agg_vals[id(e)]
        # a named grouping expression matches its own expression (the result column)
        grouping = [g.child if isinstance(g, E.Alias) else g for g in grouping]
        for gi, g in enumerate(grouping):
            if e.semantic_equals(g) or (isinstance(e, E.Attribute) and isinstance(g, E.Attribute)
                                        and e.expr_id == g.expr_id):
                return groups[gi]
        # composite expression over aggregates/groups
        cols, subst = {}, {}
        i = [0]

        def fn(x):
            if isinstance(x, E.AggregateFunction) or any(
                    x.semantic_equals(g) for g in grouping):
                nm = f"__r{i[0]}"
                i[0] += 1
                cols[nm] = self._eval_agg_result(x, grouping, groups, agg_vals, nrows)
                att = E.Attribute(nm, cols[nm].type)
                subst[att.expr_id] = nm
                return att
            return None
        rewritten = e.transform_up(fn)
        t = pa.table({f"{n}#{eid}": cols[n] for eid, n in subst.items()}) if cols else \
            pa.table({"__x": pa.array(np.zeros(nrows))})
        return eval_expr(rewritten, t)

    # -- unions ---------------------------------------------------------------------------------
    def _rename_like(self, t: pa.Table, src_attrs, dst_attrs) -> pa.Table:
        return pa.Table.from_arrays(t.columns, names=[key(a) for a in dst_attrs])

    def _exec_UnionExec(self, p):
        out = []
        for c in p.children:
            out += [self._rename_like(t, c.output, p.output) for t in self.execute(c)]
        return out

    def _exec_BucketUnionExec(self, p):
        child_parts = [[self._rename_like(t, c.output, p.output) for t in self.execute(c)]
                       for c in p.children]
        n = p.bucket_spec.num_buckets
        assert all(len(cp) == n for cp in child_parts)
        return [_concat([cp[i] for cp in child_parts], p.output) for i in range(n)]


def _align_keys(a, b):
    ta, tb = a.type, b.type
    if pa.types.is_integer(ta) and pa.types.is_integer(tb):
        return pc.cast(a, pa.int64()), pc.cast(b, pa.int64())
    if (pa.types.is_floating(ta) or pa.types.is_integer(ta)) and \
            (pa.types.is_floating(tb) or pa.types.is_integer(tb)):
        return pc.cast(a, pa.float64()), pc.cast(b, pa.float64())
    return pc.cast(a, pa.string()), pc.cast(b, pa.string())
