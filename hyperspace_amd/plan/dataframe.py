"""Lazy DataFrame over logical plans (the SparkSession/Dataset analog the Hyperspace API needs).

A DataFrame is an immutable (session, analyzed logical plan) pair.  Actions (``collect``,
``to_arrow``, ``count``) run the plan through ``QueryExecution``: optimizer (incl. the Hyperspace
rules when enabled) -> physical planner -> executor (HIP device executor or the pyarrow oracle).
"""
from __future__ import annotations

import weakref
from typing import List, Sequence

import pyarrow as pa

from ..exceptions import HyperspaceException
from . import expressions as E
from . import logical as L
from .column import Column, col
from .parser import parse_expression

_RESOLVED: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def _name_map(plan, cs: bool) -> dict:
    """name -> first output attribute of that name (lower-cased names when not case
    sensitive), built once per plan: a serving loop resolves the same names against the same
    base relations on every query (plans are immutable; the weak map dies with the plan)."""
    memo = _RESOLVED.get(plan)
    if memo is None:
        memo = _RESOLVED[plan] = {}
    m = memo.get(cs)
    if m is None:
        t = type(plan)
        if t is L.Filter or t is L.Sort:         # output = the child's output
            m = _name_map(plan.children[0], cs)
        elif t is L.Join and plan.join_type == "inner":
            # left's attributes first, then right's (the order of Join.output)
            m = dict(_name_map(plan.children[0], cs))
            for k, a in _name_map(plan.children[1], cs).items():
                m.setdefault(k, a)
        else:
            m = {}
            for a in plan.output:
                m.setdefault(a.name if cs else a.name.lower(), a)
        memo[cs] = m
    return m


def _resolve_name(cs: bool, name: str, plan) -> E.Attribute:
    a = _name_map(plan, cs).get(name if cs else name.lower())
    if a is None:
        raise HyperspaceException(
            f"cannot resolve '{name}' given input columns: [{', '.join(x.name for x in plan.output)}]")
    return a


def _native_resolve():
    from .plan_cache import _NATIVE
    return _NATIVE.resolve if _NATIVE is not None else None


_NATIVE_RESOLVE = _native_resolve()


def _resolve_walk(x, names: dict, cs: bool, plan):
    """``x`` with every UnresolvedAttribute replaced by its attribute in ``names``
    (``_name_map``)."""
    if isinstance(x, E.UnresolvedAttribute):
        a = names.get(x.name if cs else x.name.lower())
        if a is None:
            raise HyperspaceException(
                f"cannot resolve '{x.name}' given input columns: "
                f"[{', '.join(y.name for y in plan.output)}]")
        return a
    ch = x.children
    if not ch:
        return x
    new = tuple([_resolve_walk(c, names, cs, plan) for c in ch])
    for a, b in zip(new, ch):
        if a is not b:
            return x.with_children(new)
    return x


class Row(tuple):
    """Result row: tuple with attribute / key access, like ``pyspark.sql.Row``."""

    def __new__(cls, values, fields):
        r = super().__new__(cls, values)
        r._fields = tuple(fields)
        return r

    def __getattr__(self, name):
        try:
            return self[self._fields.index(name)]
        except ValueError:
            raise AttributeError(name) from None

    def __getitem__(self, k):
        if isinstance(k, str):
            return tuple.__getitem__(self, self._fields.index(k))
        return tuple.__getitem__(self, k)

    def asDict(self):
        return dict(zip(self._fields, self))

    def __repr__(self):
        return "Row(" + ", ".join(f"{f}={v!r}" for f, v in zip(self._fields, self)) + ")"


class DataFrame:
    def __init__(self, session, plan: L.LogicalPlan):
        self.session = session
        self.plan = plan

    # -- metadata ----------------------------------------------------------------------------
    @property
    def sparkSession(self):
        return self.session

    @property
    def columns(self) -> List[str]:
        return [a.name for a in self.plan.output]

    @property
    def schema(self) -> pa.Schema:
        return pa.schema([pa.field(a.name, a.data_type, a.nullable) for a in self.plan.output])

    @property
    def queryExecution(self):
        from .execution import QueryExecution
        return QueryExecution(self.session, self.plan)

    def _resolve_name(self, name: str, plan: L.LogicalPlan = None) -> E.Attribute:
        return _resolve_name(self.session.case_sensitive, name, plan or self.plan)

    def __getitem__(self, name) -> Column:
        if isinstance(name, str):
            return Column(self._resolve_name(name))
        raise TypeError(name)

    def __getattr__(self, name):
        if name.startswith("_") or name in ("session", "plan"):
            raise AttributeError(name)
        try:
            return self[name]
        except HyperspaceException as e:  # PySpark semantics: unknown attribute -> AttributeError
            raise AttributeError(str(e)) from None

    def _resolve(self, e: E.Expression, plan: L.LogicalPlan = None) -> E.Expression:
        """``e`` with its unresolved column names bound to ``plan``'s attributes; subtrees
        without one are kept as they are (a serving loop builds a fresh expression per query,
        so this walk is on its host path)."""
        plan = plan or self.plan
        cs = self.session.case_sensitive
        names = _name_map(plan, cs)
        if _NATIVE_RESOLVE is not None:
            return _NATIVE_RESOLVE(e, names, cs, E.UnresolvedAttribute,
                                   lambda n: _resolve_name(cs, n, plan))
        return _resolve_walk(e, names, cs, plan)

    def _to_expr(self, c) -> E.Expression:
        if isinstance(c, str):
            if c == "*":
                raise ValueError("*")
            return parse_expression(c) if not c.isidentifier() else E.UnresolvedAttribute(c)
        if isinstance(c, Column):
            return c.expr
        if isinstance(c, E.Expression):
            return c
        raise TypeError(f"unsupported column spec {c!r}")

    # -- transformations ---------------------------------------------------------------------
    def filter(self, condition) -> "DataFrame":
        e = parse_expression(condition) if isinstance(condition, str) else self._to_expr(condition)
        return DataFrame(self.session, L.Filter(self._resolve(e), self.plan))

    where = filter

    def select(self, *cols) -> "DataFrame":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        exprs: List[E.Expression] = []
        for c in cols:
            if isinstance(c, str) and c == "*":
                exprs.extend(self.plan.output)
                continue
            e = self._resolve(self._to_expr(c))
            if not isinstance(e, (E.Attribute, E.Alias)):
                e = E.Alias(e, e.sql())
            exprs.append(e)
        if any(E.contains_aggregate(e) for e in exprs):
            return DataFrame(self.session, L.Aggregate([], exprs, self.plan))
        return DataFrame(self.session, L.Project(exprs, self.plan))

    def toDF(self, *names) -> "DataFrame":
        if len(names) != len(self.plan.output):
            raise HyperspaceException("toDF: number of column names does not match")
        exprs = [a if a.name == n else E.Alias(a, n) for a, n in zip(self.plan.output, names)]
        if all(isinstance(e, E.Attribute) for e in exprs):
            return self
        return DataFrame(self.session, L.Project(exprs, self.plan))

    def withColumnRenamed(self, old: str, new: str) -> "DataFrame":
        exprs = [E.Alias(a, new) if a.name == old else a for a in self.plan.output]
        return DataFrame(self.session, L.Project(exprs, self.plan))

    def withColumn(self, name: str, c) -> "DataFrame":
        e = self._resolve(self._to_expr(c))
        exprs = [a for a in self.plan.output if a.name != name] + [E.Alias(e, name)]
        return DataFrame(self.session, L.Project(exprs, self.plan))

    def drop(self, *names) -> "DataFrame":
        keep = [a for a in self.plan.output if a.name not in names]
        return DataFrame(self.session, L.Project(keep, self.plan))

    def crossJoin(self, other: "DataFrame") -> "DataFrame":
        return self.join(other, None, "cross")

    def join(self, other: "DataFrame", on=None, how: str = "inner") -> "DataFrame":
        how = {"left_outer": "left", "leftouter": "left", "right_outer": "right",
               "rightouter": "right", "outer": "full", "full_outer": "full",
               "fullouter": "full", "semi": "leftsemi", "left_semi": "leftsemi",
               "anti": "leftanti", "left_anti": "leftanti"}.get(how.lower(), how.lower())
        left = self.plan
        right = other.plan
        # Self-join / shared lineage: re-instance the right side's attributes (Catalyst's dedupRight).
        lids = left.output_set()
        remap = {}
        if lids & right.output_set():
            right, remap = _dedup(right, lids)
        if on is None:
            return DataFrame(self.session, L.Join(left, right, how, None))
        if isinstance(on, str) or (isinstance(on, (list, tuple)) and on and isinstance(on[0], str)):
            names = [on] if isinstance(on, str) else list(on)
            conds = [E.EqualTo(self._resolve_name(n, left), self._resolve_name(n, right)) for n in names]
            j = L.Join(left, right, how, E.conjoin(conds))
            # USING join: keep one copy of the key columns
            rkeys = {self._resolve_name(n, right).expr_id for n in names}
            proj = [a for a in j.output if a.expr_id not in rkeys]
            return DataFrame(self.session, L.Project(proj, j))
        cond = self._to_expr(on)
        if remap:
            cond = _fix_self_join_condition(cond, remap)
        combined = L.Join(left, right, how, None)
        cond = self._resolve(cond, combined)
        return DataFrame(self.session, L.Join(left, right, how, cond))

    def groupBy(self, *cols) -> "GroupedData":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        return GroupedData(self, [self._resolve(self._to_expr(c)) for c in cols])

    groupby = groupBy

    def agg(self, *aggs) -> "DataFrame":
        return GroupedData(self, []).agg(*aggs)

    def union(self, other: "DataFrame") -> "DataFrame":
        return DataFrame(self.session, L.Union([self.plan, other.plan]))

    unionAll = union

    def orderBy(self, *cols, ascending=True) -> "DataFrame":
        """``ascending``: one flag or one per column; ``col(x).desc()`` / ``.asc()`` override it
        per column (mixed orders such as TPC-H Q3's ``revenue DESC, o_orderdate``)."""
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        flags = list(ascending) if isinstance(ascending, (list, tuple)) else [ascending] * len(cols)
        orders = [L.SortOrder(self._resolve(self._to_expr(c)),
                              bool(getattr(c, "sort_ascending", f)))
                  for c, f in zip(cols, flags)]
        return DataFrame(self.session, L.Sort(orders, True, self.plan))

    sort = orderBy

    def limit(self, n: int) -> "DataFrame":
        return DataFrame(self.session, L.Limit(n, self.plan))

    def repartition(self, num: int, *cols) -> "DataFrame":
        exprs = [self._resolve(self._to_expr(c)) for c in cols]
        return DataFrame(self.session, L.RepartitionByExpression(exprs, self.plan, num))

    def hint(self, *_):
        return self

    # -- catalog -------------------------------------------------------------------------------
    def createOrReplaceTempView(self, name: str) -> None:
        self.session.catalog.create_temp_view(name, self.plan, replace=True)

    def createTempView(self, name: str) -> None:
        self.session.catalog.create_temp_view(name, self.plan, replace=False)

    registerTempTable = createOrReplaceTempView

    def cache(self):
        return self

    # -- actions -------------------------------------------------------------------------------
    def to_arrow(self) -> pa.Table:
        return self.queryExecution.to_arrow()

    toArrow = to_arrow

    def collect(self) -> List[Row]:
        return _rows(self.to_arrow())

    def collect_async(self) -> "RowsFuture":
        """Submit this query and return at once; ``.result()`` gives ``collect()``'s rows.
        Keeping several queries in flight lets the MI355X executor run one query's kernels
        while the host plans the next (``GpuBackend.collect_async``)."""
        return RowsFuture(self.queryExecution.to_arrow_async())

    def count(self) -> int:
        return self.to_arrow().num_rows

    def toPandas(self):
        return self.to_arrow().to_pandas()

    def show(self, n: int = 20, truncate: bool = True) -> None:
        print(show_string(self.limit(n).to_arrow(), truncate))

    def explain(self, extended: bool = False) -> None:
        print(self.queryExecution.explain_string(extended))

    @property
    def write(self):
        from ..io.writer import DataFrameWriter
        return DataFrameWriter(self)


class GroupedData:
    def __init__(self, df: DataFrame, grouping: Sequence[E.Expression]):
        import re
        self.df = df
        # an unnamed grouping expression is an output column too: name it like Spark does,
        # after its SQL text ("(a * 2)")
        self.grouping = [g if isinstance(g, (E.Attribute, E.Alias)) else
                         E.Alias(g, re.sub(r"#\d+", "", g.sql())) for g in grouping]

    def agg(self, *aggs) -> DataFrame:
        exprs: List[E.Expression] = list(self.grouping)
        if len(aggs) == 1 and isinstance(aggs[0], dict):
            from .column import Column as _C
            items = []
            for c, fn in aggs[0].items():
                f = {"sum": E.Sum, "count": E.Count, "min": E.Min, "max": E.Max,
                     "avg": E.Avg, "mean": E.Avg}[fn.lower()]
                items.append(_C(E.Alias(f(E.UnresolvedAttribute(c)), f"{fn}({c})")))
            aggs = tuple(items)
        for a in aggs:
            e = self.df._resolve(self.df._to_expr(a))
            if not isinstance(e, (E.Alias, E.Attribute)):
                e = E.Alias(e, e.sql().replace("#", "_"))
            exprs.append(e)
        return DataFrame(self.df.session, L.Aggregate(self.grouping, exprs, self.df.plan))

    def count(self) -> DataFrame:
        return self.agg(Column(E.Alias(E.Count(None), "count")))

    def sum(self, *cols) -> DataFrame:
        return self.agg(*[Column(E.Alias(E.Sum(col(c).expr), f"sum({c})")) for c in cols])


def _dedup(plan: L.LogicalPlan, conflicting: set):
    """Give every attribute produced by ``plan`` that conflicts a fresh expr id."""
    mapping = {}

    def fresh(a: E.Attribute) -> E.Attribute:
        if a.expr_id in conflicting or a.expr_id in mapping:
            if a.expr_id not in mapping:
                mapping[a.expr_id] = a.new_instance()
            return mapping[a.expr_id]
        return a

    def rewrite_expr(e):
        def fn(x):
            if isinstance(x, E.Attribute) and x.expr_id in mapping:
                return mapping[x.expr_id]
            if isinstance(x, E.Alias) and x.expr_id in conflicting:
                na = E.Alias(x.child, x.name)
                mapping[x.expr_id] = na.to_attribute()
                return na
            return None
        return e.transform_up(fn)

    def fn(p):
        if isinstance(p, L.LogicalRelation):
            return p.copy(output=[fresh(a) for a in p.output])
        if isinstance(p, L.LocalRelation):
            return L.LocalRelation(p.table, [fresh(a) for a in p.output])
        if isinstance(p, L.Filter):
            return L.Filter(rewrite_expr(p.condition), p.child)
        if isinstance(p, L.Project):
            return L.Project([rewrite_expr(e) for e in p.project_list], p.child)
        if isinstance(p, L.Aggregate):
            return L.Aggregate([rewrite_expr(e) for e in p.grouping],
                               [rewrite_expr(e) for e in p.aggregates], p.child)
        if isinstance(p, L.Join) and p.condition is not None:
            return L.Join(p.left, p.right, p.join_type, rewrite_expr(p.condition))
        if isinstance(p, L.Sort):
            return L.Sort([L.SortOrder(rewrite_expr(o.child), o.ascending) for o in p.order],
                          p.global_sort, p.child)
        if isinstance(p, L.RepartitionByExpression):
            return L.RepartitionByExpression([rewrite_expr(e) for e in p.partition_expressions],
                                             p.child, p.num_partitions)
        return None

    new_plan = plan.transform_up(fn)
    return new_plan, {k: v for k, v in mapping.items()}


def _fix_self_join_condition(cond: E.Expression, remap: dict) -> E.Expression:
    """``df.join(df, df("a") === df("a"))``: map the right operand of a trivially-true equality
    onto the right side's re-instanced attribute (Catalyst's self-join condition resolution)."""
    def fn(x):
        if isinstance(x, E.EqualTo) and isinstance(x.left, E.Attribute) and \
                isinstance(x.right, E.Attribute) and x.left.expr_id == x.right.expr_id and \
                x.right.expr_id in remap:
            return E.EqualTo(x.left, remap[x.right.expr_id])
        return None
    return cond.transform_up(fn)


def _cell(v) -> str:
    """Spark's cell rendering: null, arrays as ``[a, b]``, booleans lower-case."""
    if v is None:
        return "null"
    if isinstance(v, (list, tuple)):
        return "[" + ", ".join(_cell(x) for x in v) + "]"
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def show_string(t: pa.Table, truncate: bool = True) -> str:
    """Spark ``Dataset.showString`` table layout (right-aligned cells)."""
    names = t.column_names
    rows = [[_cell(v) for v in r] for r in
            zip(*[c.to_pylist() for c in t.columns])] if t.num_columns else []
    if truncate:
        rows = [[v if len(v) <= 20 else v[:17] + "..." for v in r] for r in rows]
    widths = [max([3, len(n)] + [len(r[i]) for r in rows]) for i, n in enumerate(names)]
    sep = "+" + "+".join("-" * w for w in widths) + "+"
    lines = [sep, "|" + "|".join(n.rjust(w) for n, w in zip(names, widths)) + "|", sep]
    for r in rows:
        lines.append("|" + "|".join(v.rjust(w) for v, w in zip(r, widths)) + "|")
    lines.append(sep)
    return "\n".join(lines) + "\n"


def _rows(t: pa.Table) -> List[Row]:
    names = t.column_names
    cols = [c.to_pylist() for c in t.columns]
    return [Row(vals, names) for vals in zip(*cols)] if cols else []


class RowsFuture:
    """Pending ``collect()`` of a submitted query; ``path`` is the executor path that ran."""

    def __init__(self, fut):
        self._fut = fut

    @property
    def path(self) -> str:
        return self._fut.path

    @property
    def reason(self):
        return self._fut.reason

    def result(self) -> List[Row]:
        return _rows(self._fut.result())
