"""Physical plans + planner + EnsureRequirements.

The operator set mirrors what the reference makes Spark run: file scans (plain or
bucketed index scans), Filter, Project, ShuffleExchange(hashpartitioning), Sort, SortMergeJoin,
BroadcastHashJoin, HashAggregate, Union and BucketUnion (``BucketUnionExec.scala:52-121``).
Execution is delegated to a backend (``exec.cpu.CpuBackend`` — pyarrow oracle — or
``exec.gpu.GpuBackend`` — HIP kernels on MI355X); both honour the same partitioning semantics so
plans are interchangeable and results comparable row-for-row.

``EnsureRequirements`` inserts Exchange/Sort only when a child's output partitioning/ordering does
not already satisfy the join: two bucketed index scans with equal bucket counts on the join keys
need neither (ExplainTest.scala:142-172: ShuffleExchange 1->0, Sort 2->0).
"""
from __future__ import annotations

import re
from typing import List, Optional

import pyarrow as pa

from ..utils.conf import HyperspaceConf
from . import expressions as E
from . import logical as L
from .types import struct_string


# ---------------------------------------------------------------------------------------------
# Partitioning
# ---------------------------------------------------------------------------------------------
class Partitioning:
    num_partitions: int = 1

    def satisfies_clustering(self, exprs: List[E.Expression], n: Optional[int] = None) -> bool:
        return False


class UnknownPartitioning(Partitioning):
    def __init__(self, n: int):
        self.num_partitions = n


class SinglePartition(Partitioning):
    num_partitions = 1

    def satisfies_clustering(self, exprs, n=None):
        return True


class HashPartitioning(Partitioning):
    def __init__(self, exprs: List[E.Expression], n: int):
        self.expressions = list(exprs)
        self.num_partitions = int(n)

    def satisfies_clustering(self, exprs, n=None):
        if n is not None and n != self.num_partitions:
            return False
        if len(exprs) != len(self.expressions):
            return False
        return all(a.semantic_equals(b) for a, b in zip(self.expressions, exprs))

    def sql(self):
        return f"hashpartitioning({', '.join(e.sql() for e in self.expressions)}, {self.num_partitions})"


# ---------------------------------------------------------------------------------------------
# Operators
# ---------------------------------------------------------------------------------------------
class SparkPlan:
    children: tuple = ()

    @property
    def output(self) -> List[E.Attribute]:
        raise NotImplementedError

    @property
    def node_name(self) -> str:
        return type(self).__name__.replace("Exec", "")

    @property
    def output_partitioning(self) -> Partitioning:
        return self.children[0].output_partitioning if self.children else UnknownPartitioning(1)

    @property
    def output_ordering(self) -> List[L.SortOrder]:
        return []

    def with_children(self, children) -> "SparkPlan":
        raise NotImplementedError

    def simple_string(self) -> str:
        return self.node_name

    def iter_pre(self):
        yield self
        for c in self.children:
            yield from c.iter_pre()

    def collect(self, pred):
        return [p for p in self.iter_pre() if pred(p)]

    def transform_up(self, fn):
        new_children = tuple(c.transform_up(fn) for c in self.children)
        node = self.with_children(new_children) if any(
            a is not b for a, b in zip(new_children, self.children)) else self
        r = fn(node)
        return node if r is None else r

    def tree_string(self) -> str:
        lines: list = []
        self._tree(lines, [])
        return "\n".join(lines)

    def tree_lines(self):
        """[(prefix, node)] pre-order with Spark's ``:- / +-`` tree prefixes."""
        out: list = []
        self._tree_nodes(out, [])
        return out

    def _tree_nodes(self, out, flags):
        prefix = ""
        if flags:
            prefix = "".join("   " if f else ":  " for f in flags[:-1])
            prefix += "+- " if flags[-1] else ":- "
        out.append((prefix, self))
        for i, c in enumerate(self.children):
            c._tree_nodes(out, flags + [i == len(self.children) - 1])

    def _tree(self, lines, flags):
        for prefix, node in self.tree_lines():
            lines.append(prefix + node.simple_string())

    def __repr__(self):
        return self.tree_string()


class FileSourceScanExec(SparkPlan):
    def __init__(self, relation: L.HadoopFsRelation, output: List[E.Attribute],
                 data_filters: List[E.Expression], partition_filters: List[E.Expression],
                 use_bucketing: bool, logical: L.LogicalRelation = None,
                 selected_buckets: Optional[set] = None):
        self.relation = relation
        self._output = list(output)
        self.data_filters = list(data_filters)
        self.partition_filters = list(partition_filters)
        self.use_bucketing = use_bucketing and relation.bucket_spec is not None
        self.logical = logical
        self.selected_buckets = selected_buckets

    @property
    def output(self):
        return self._output

    def with_children(self, children):
        return self

    @property
    def node_name(self):
        return f"Scan {self.relation!r}"

    @property
    def bucket_spec(self) -> Optional[L.BucketSpec]:
        return self.relation.bucket_spec if self.use_bucketing else None

    @property
    def output_partitioning(self):
        bs = self.bucket_spec
        if bs is not None:
            attrs = []
            for n in bs.bucket_column_names:
                a = next((x for x in self._output if x.name.lower() == n.lower()), None)
                if a is None:
                    return UnknownPartitioning(bs.num_buckets)
                attrs.append(a)
            return HashPartitioning(attrs, bs.num_buckets)
        return UnknownPartitioning(max(1, len(self.relation.location.all_files())))

    @property
    def output_ordering(self):
        bs = self.bucket_spec
        if bs is None or not bs.sort_column_names:
            return []
        # Sorted output only when every bucket has at most one file (E2EHyperspaceRulesTest:455-479).
        if not self.relation.location.one_file_per_bucket():
            return []
        out = []
        for n in bs.sort_column_names:
            a = next((x for x in self._output if x.name.lower() == n.lower()), None)
            if a is None:
                break
            out.append(L.SortOrder(a, True))
        return out

    def pushed_filters_string(self):
        out = []
        for f in self.data_filters:
            s = _source_filter(f)
            if s:
                out.append(s)
        return out

    def simple_string(self):
        rel = self.relation
        fmt = "Parquet" if rel.is_index() else rel.file_format.capitalize()
        if rel.file_format == "csv":
            fmt = "CSV"
        elif rel.file_format == "json":
            fmt = "JSON"
        elif rel.file_format == "orc":
            fmt = "ORC"
        read_schema = pa.schema([pa.field(a.name, a.data_type) for a in self._output
                                 if a.name not in rel.partition_schema.names])
        loc = f"{rel.location.kind}[{', '.join(rel.location.root_paths)}]"
        s = (f"FileScan {rel!r} [{','.join(a.sql() for a in self._output)}] Batched: true, "
             f"Format: {fmt}, Location: {loc}, "
             f"PartitionFilters: [{', '.join(p.sql() for p in self.partition_filters)}], "
             f"PushedFilters: [{', '.join(self.pushed_filters_string())}], "
             f"ReadSchema: {struct_string(read_schema)}")
        if self.use_bucketing:
            n = self.relation.bucket_spec.num_buckets
            sel = n if self.selected_buckets is None else len(self.selected_buckets)
            s += f", SelectedBucketsCount: {sel} out of {n}"
        return s


def _source_filter(e: E.Expression) -> Optional[str]:
    def name(x):
        return x.name if isinstance(x, E.Attribute) else None
    if isinstance(e, E.IsNotNull) and name(e.child):
        return f"IsNotNull({name(e.child)})"
    if isinstance(e, E.IsNull) and name(e.child):
        return f"IsNull({name(e.child)})"
    if isinstance(e, E.BinaryComparison) and name(e.left) and isinstance(e.right, E.Literal):
        op = {E.EqualTo: "EqualTo", E.LessThan: "LessThan", E.LessThanOrEqual: "LessThanOrEqual",
              E.GreaterThan: "GreaterThan", E.GreaterThanOrEqual: "GreaterThanOrEqual"}.get(type(e))
        if op:
            return f"{op}({name(e.left)},{e.right.sql()})"
    if isinstance(e, (E.In, E.InSet)) and name(e.value):
        return f"In({name(e.value)}, [...])"
    return None


class LocalTableScanExec(SparkPlan):
    def __init__(self, table: pa.Table, output: List[E.Attribute]):
        self.table = table
        self._output = output

    @property
    def output(self):
        return self._output

    def with_children(self, children):
        return self

    def simple_string(self):
        return f"LocalTableScan [{', '.join(a.sql() for a in self._output)}]"


class UnaryExec(SparkPlan):
    @property
    def child(self) -> SparkPlan:
        return self.children[0]

    @property
    def output(self):
        return self.child.output


class FilterExec(UnaryExec):
    def __init__(self, condition: E.Expression, child: SparkPlan):
        self.condition = condition
        self.children = (child,)

    def with_children(self, children):
        return FilterExec(self.condition, children[0])

    @property
    def output_ordering(self):
        return self.child.output_ordering

    def simple_string(self):
        return f"Filter {self.condition.sql()}"


class ProjectExec(UnaryExec):
    def __init__(self, project_list: List[E.Expression], child: SparkPlan):
        self.project_list = list(project_list)
        self.children = (child,)

    @property
    def output(self):
        return [e if isinstance(e, E.Attribute) else e.to_attribute() for e in self.project_list]

    def with_children(self, children):
        return ProjectExec(self.project_list, children[0])

    @property
    def output_partitioning(self):
        p = self.child.output_partitioning
        if isinstance(p, HashPartitioning):
            ids = {a.expr_id for a in self.output}
            if all(isinstance(x, E.Attribute) and x.expr_id in ids for x in p.expressions):
                return p
            return UnknownPartitioning(p.num_partitions)
        return p

    @property
    def output_ordering(self):
        ids = {a.expr_id for a in self.output}
        out = []
        for o in self.child.output_ordering:
            if isinstance(o.child, E.Attribute) and o.child.expr_id in ids:
                out.append(o)
            else:
                break
        return out

    def simple_string(self):
        return f"Project [{', '.join(e.sql() for e in self.project_list)}]"


class ShuffleExchangeExec(UnaryExec):
    def __init__(self, partitioning: Partitioning, child: SparkPlan):
        self.partitioning = partitioning
        self.children = (child,)

    @property
    def node_name(self):
        return "ShuffleExchange"

    @property
    def output_partitioning(self):
        return self.partitioning

    def with_children(self, children):
        return ShuffleExchangeExec(self.partitioning, children[0])

    def simple_string(self):
        if isinstance(self.partitioning, HashPartitioning):
            return f"Exchange {self.partitioning.sql()}"
        return "Exchange SinglePartition"


class ReusedExchangeExec(SparkPlan):
    """Leaf standing for an exchange whose result another, identical exchange of the same plan
    already produces (Spark's ``ReuseExchange`` rule; golden: ``ExplainTest.scala:142-172``,
    ``ReusedExchange [Col1#21, Col2#22], Exchange hashpartitioning(Col1#11, 5)``).

    ``exchange`` is the reused node (its output attributes map positionally onto ``output``);
    ``equivalent`` is the original subtree this leaf replaced, for a backend that prefers to
    execute it instead of sharing the result."""

    def __init__(self, output: List[E.Attribute], exchange: SparkPlan, equivalent: SparkPlan):
        self._output = list(output)
        self.exchange = exchange
        self.equivalent = equivalent

    @property
    def output(self):
        return self._output

    @property
    def node_name(self):
        return "ReusedExchange"

    @property
    def output_partitioning(self):
        return self.equivalent.output_partitioning

    @property
    def output_ordering(self):
        return self.equivalent.output_ordering

    def with_children(self, children):
        return self

    def simple_string(self):
        return (f"ReusedExchange [{', '.join(a.sql() for a in self._output)}], "
                f"{self.exchange.simple_string()}")


class BroadcastExchangeExec(UnaryExec):
    def __init__(self, child: SparkPlan):
        self.children = (child,)

    @property
    def node_name(self):
        return "BroadcastExchange"

    def with_children(self, children):
        return BroadcastExchangeExec(children[0])

    def simple_string(self):
        return "BroadcastExchange HashedRelationBroadcastMode"


class SortExec(UnaryExec):
    def __init__(self, order: List[L.SortOrder], global_sort: bool, child: SparkPlan):
        self.order = list(order)
        self.global_sort = global_sort
        self.children = (child,)

    def with_children(self, children):
        return SortExec(self.order, self.global_sort, children[0])

    @property
    def output_ordering(self):
        return self.order

    def simple_string(self):
        return f"Sort [{', '.join(o.sql() for o in self.order)}], {str(self.global_sort).lower()}, 0"


class SortMergeJoinExec(SparkPlan):
    def __init__(self, left_keys, right_keys, join_type: str, condition, left, right):
        self.left_keys = list(left_keys)
        self.right_keys = list(right_keys)
        self.join_type = join_type
        self.condition = condition
        self.children = (left, right)

    @property
    def left(self):
        return self.children[0]

    @property
    def right(self):
        return self.children[1]

    @property
    def output(self):
        return L.Join(_Out(self.left.output), _Out(self.right.output), self.join_type).output

    @property
    def output_partitioning(self):
        return self.left.output_partitioning

    def with_children(self, children):
        return SortMergeJoinExec(self.left_keys, self.right_keys, self.join_type, self.condition,
                                 children[0], children[1])

    def simple_string(self):
        s = (f"SortMergeJoin [{', '.join(k.sql() for k in self.left_keys)}], "
             f"[{', '.join(k.sql() for k in self.right_keys)}], {self.join_type.capitalize()}")
        if self.condition is not None:
            s += f", {self.condition.sql()}"
        return s


class BroadcastHashJoinExec(SparkPlan):
    def __init__(self, left_keys, right_keys, join_type, build_side, condition, left, right):
        self.left_keys = list(left_keys)
        self.right_keys = list(right_keys)
        self.join_type = join_type
        self.build_side = build_side
        self.condition = condition
        self.children = (left, right)

    @property
    def left(self):
        return self.children[0]

    @property
    def right(self):
        return self.children[1]

    @property
    def output(self):
        return L.Join(_Out(self.left.output), _Out(self.right.output), self.join_type).output

    @property
    def output_partitioning(self):
        stream = self.left if self.build_side == "right" else self.right
        return stream.output_partitioning

    def with_children(self, children):
        return BroadcastHashJoinExec(self.left_keys, self.right_keys, self.join_type,
                                     self.build_side, self.condition, children[0], children[1])

    def simple_string(self):
        return (f"BroadcastHashJoin [{', '.join(k.sql() for k in self.left_keys)}], "
                f"[{', '.join(k.sql() for k in self.right_keys)}], {self.join_type.capitalize()}, "
                f"Build{self.build_side.capitalize()}")


class NestedLoopJoinExec(SparkPlan):
    def __init__(self, join_type, condition, left, right):
        self.join_type = join_type
        self.condition = condition
        self.children = (left, right)

    @property
    def output(self):
        return L.Join(_Out(self.children[0].output), _Out(self.children[1].output),
                      self.join_type).output

    @property
    def output_partitioning(self):
        return UnknownPartitioning(1)

    def with_children(self, children):
        return NestedLoopJoinExec(self.join_type, self.condition, children[0], children[1])

    def simple_string(self):
        return f"BroadcastNestedLoopJoin {self.join_type.capitalize()}"


class HashAggregateExec(UnaryExec):
    def __init__(self, grouping, aggregates, mode: str, child: SparkPlan, result_attrs=None):
        self.grouping = list(grouping)
        self.aggregates = list(aggregates)   # Alias(AggFn) | Attribute(grouping col)
        self.mode = mode                     # "partial" | "final" | "complete"
        self.children = (child,)
        self.result_attrs = result_attrs
        # attributes of unnamed grouping expressions (SQL ``GROUP BY a % 7``), made once: the
        # exchange above partitions by them and the final aggregate reads them by id
        self._unnamed: dict = {}

    @property
    def output(self):
        if self.mode == "partial":
            return self.partial_output()
        return [e if isinstance(e, E.Attribute) else e.to_attribute() for e in self.aggregates]

    def partial_output(self):
        # a named grouping expression keeps its alias's id: the exchange above partitions by,
        # and the final aggregate groups on, these same attributes
        out = []
        for i, g in enumerate(self.grouping):
            if isinstance(g, E.Attribute):
                out.append(g)
            elif isinstance(g, E.Alias):
                out.append(g.to_attribute())
            else:
                if i not in self._unnamed:
                    self._unnamed[i] = E.Attribute(g.sql(), g.data_type, True)
                out.append(self._unnamed[i])
        for i, (_, fn) in enumerate(agg_functions(self.aggregates)):
            for j, (nm, dt) in enumerate(_buffer_fields(fn)):
                out.append(E.Attribute(f"{nm}#{i}_{j}", dt, True, expr_id=-(1000 * (i + 1) + j)))
        return out

    def with_children(self, children):
        n = HashAggregateExec(self.grouping, self.aggregates, self.mode, children[0],
                              self.result_attrs)
        n._unnamed = self._unnamed
        return n

    @property
    def output_partitioning(self):
        return self.child.output_partitioning

    def simple_string(self):
        fns = ", ".join(f"{self.mode}_{fn.sql()}" if self.mode == "partial" else fn.sql()
                        for _, fn in agg_functions(self.aggregates))
        return (f"HashAggregate(keys=[{', '.join(g.sql() for g in self.grouping)}], "
                f"functions=[{fns}])")


def agg_functions(aggregates):
    out = []
    for e in aggregates:
        for x in e.iter_tree():
            if isinstance(x, E.AggregateFunction):
                out.append((e, x))
    return out


def _buffer_fields(fn):
    if isinstance(fn, E.Avg):
        return [("sum", pa.float64()), ("count", pa.int64())]
    return [(fn.name, fn.data_type)]


class UnionExec(SparkPlan):
    def __init__(self, children):
        self.children = tuple(children)

    @property
    def output(self):
        return self.children[0].output

    @property
    def output_partitioning(self):
        return UnknownPartitioning(sum(c.output_partitioning.num_partitions for c in self.children))

    def with_children(self, children):
        return UnionExec(children)

    def simple_string(self):
        return "Union"


class BucketUnionExec(SparkPlan):
    def __init__(self, children, bucket_spec: L.BucketSpec):
        self.children = tuple(children)
        self.bucket_spec = bucket_spec

    @property
    def output(self):
        return self.children[0].output

    @property
    def output_partitioning(self):
        parts = [c.output_partitioning for c in self.children]
        assert all(isinstance(p, HashPartitioning) for p in parts)
        assert all(p.num_partitions == self.bucket_spec.num_buckets for p in parts)
        return parts[0]

    def with_children(self, children):
        return BucketUnionExec(children, self.bucket_spec)

    def simple_string(self):
        return (f"BucketUnion {self.bucket_spec.num_buckets} buckets, bucket columns: "
                f"[{', '.join(self.bucket_spec.bucket_column_names)}]")


class CollectLimitExec(UnaryExec):
    def __init__(self, n: int, child):
        self.n = n
        self.children = (child,)

    def with_children(self, children):
        return CollectLimitExec(self.n, children[0])

    def simple_string(self):
        return f"CollectLimit {self.n}"


class _Out(L.LeafNode):
    def __init__(self, output):
        self._o = output

    @property
    def output(self):
        return self._o


# ---------------------------------------------------------------------------------------------
# Planner
# ---------------------------------------------------------------------------------------------
def extract_equi_join_keys(join: L.Join):
    if join.condition is None:
        return [], [], None
    lset, rset = join.left.output_set(), join.right.output_set()
    lk, rk, rest = [], [], []
    for c in E.split_conjuncts(join.condition):
        if isinstance(c, E.EqualTo):
            l_refs = {a.expr_id for a in c.left.references()}
            r_refs = {a.expr_id for a in c.right.references()}
            if l_refs and r_refs and l_refs <= lset and r_refs <= rset:
                lk.append(c.left)
                rk.append(c.right)
                continue
            if l_refs and r_refs and l_refs <= rset and r_refs <= lset:
                lk.append(c.right)
                rk.append(c.left)
                continue
        rest.append(c)
    return lk, rk, E.conjoin(rest)


def estimate_size(plan: L.LogicalPlan) -> int:
    if isinstance(plan, L.LogicalRelation):
        return max(1, plan.relation.location.size_in_bytes())
    if isinstance(plan, L.LocalRelation):
        return max(1, plan.table.nbytes)
    if not plan.children:
        return 1 << 62
    return sum(estimate_size(c) for c in plan.children)


class Planner:
    def __init__(self, session):
        self.session = session

    def plan(self, p: L.LogicalPlan) -> SparkPlan:
        for strategy in self.session.extra_strategies:
            r = strategy(self, p)
            if r is not None:
                return r
        if isinstance(p, (L.Project, L.Filter, L.LogicalRelation)):
            scan = self._plan_scan_operation(p)
            if scan is not None:
                return scan
        if isinstance(p, L.Project):
            return ProjectExec(p.project_list, self.plan(p.child))
        if isinstance(p, L.Filter):
            return FilterExec(p.condition, self.plan(p.child))
        if isinstance(p, L.LocalRelation):
            return LocalTableScanExec(p.table, p.output)
        if isinstance(p, L.Join):
            return self._plan_join(p)
        if isinstance(p, L.Aggregate):
            child = self.plan(p.child)
            partial = HashAggregateExec(p.grouping, p.aggregates, "partial", child)
            if p.grouping:
                n = HyperspaceConf.shuffle_partitions(self.session.conf)
                exch = ShuffleExchangeExec(HashPartitioning(partial.partial_output()[:len(p.grouping)], n),
                                           partial)
            else:
                exch = ShuffleExchangeExec(SinglePartition(), partial)
            return HashAggregateExec(p.grouping, p.aggregates, "final", exch)
        if isinstance(p, L.Union):
            return UnionExec([self.plan(c) for c in p.children])
        if isinstance(p, L.RepartitionByExpression):
            return ShuffleExchangeExec(HashPartitioning(p.partition_expressions, p.num_partitions),
                                       self.plan(p.child))
        if isinstance(p, L.Sort):
            child = self.plan(p.child)
            if p.global_sort:
                child = ShuffleExchangeExec(SinglePartition(), child)
            return SortExec(p.order, p.global_sort, child)
        if isinstance(p, L.Limit):
            return CollectLimitExec(p.n, self.plan(p.child))
        if isinstance(p, L.BucketUnion):
            return BucketUnionExec([self.plan(c) for c in p.children], p.bucket_spec)
        raise NotImplementedError(f"no physical plan for {p.node_name}")

    def _plan_scan_operation(self, p):
        """``FileSourceStrategy``: Project? -> Filter? -> LogicalRelation becomes one scan with
        pushed filters + Filter/Project on top."""
        project = None
        node = p
        if isinstance(node, L.Project):
            project = node
            node = node.child
        filt = None
        if isinstance(node, L.Filter):
            filt = node
            node = node.child
        if not isinstance(node, L.LogicalRelation):
            return None
        rel = node.relation
        conds = E.split_conjuncts(filt.condition) if filt is not None else []
        part_names = set(rel.partition_schema.names)
        part_filters = [c for c in conds if c.references() and
                        all(a.name in part_names for a in c.references())]
        data_filters = [c for c in conds if c not in part_filters]
        if project is not None:
            needed = {a.expr_id for e in project.project_list for a in e.references()}
        else:
            needed = {a.expr_id for a in node.output}
        if filt is not None:
            needed |= {a.expr_id for a in filt.condition.references()}
        scan_out = [a for a in node.output if a.expr_id in needed] or node.output[:1]
        if rel.bucket_spec is not None:
            # bucketed scans must expose the bucket columns to report HashPartitioning
            for n in rel.bucket_spec.bucket_column_names:
                a = next((x for x in node.output if x.name.lower() == n.lower()), None)
                if a is not None and a not in scan_out and project is None:
                    scan_out.append(a)
        scan = FileSourceScanExec(rel, scan_out, data_filters, part_filters,
                                  use_bucketing=rel.bucket_spec is not None, logical=node)
        out: SparkPlan = scan
        if filt is not None:
            out = FilterExec(filt.condition, out)
        if project is not None:
            if [a.expr_id for a in out.output] != [
                    (e.expr_id if isinstance(e, E.Attribute) else None) for e in project.project_list]:
                out = ProjectExec(project.project_list, out)
        return out

    def _plan_join(self, j: L.Join) -> SparkPlan:
        lk, rk, rest = extract_equi_join_keys(j)
        left, right = self.plan(j.left), self.plan(j.right)
        if not lk:
            return NestedLoopJoinExec(j.join_type, j.condition, left, right)
        thr = HyperspaceConf.auto_broadcast_join_threshold(self.session.conf)
        if thr >= 0 and j.join_type in ("inner", "left", "leftsemi", "leftanti") and \
                estimate_size(j.right) <= thr:
            return BroadcastHashJoinExec(lk, rk, j.join_type, "right", rest, left,
                                         BroadcastExchangeExec(right))
        if thr >= 0 and j.join_type in ("inner", "right") and estimate_size(j.left) <= thr:
            return BroadcastHashJoinExec(lk, rk, j.join_type, "left", rest,
                                         BroadcastExchangeExec(left), right)
        return SortMergeJoinExec(lk, rk, j.join_type, rest, left, right)


def ensure_requirements(plan: SparkPlan, session) -> SparkPlan:
    n_default = HyperspaceConf.shuffle_partitions(session.conf)

    def fn(p):
        if isinstance(p, SortMergeJoinExec):
            lp, rp = p.left.output_partitioning, p.right.output_partitioning
            l_ok = isinstance(lp, HashPartitioning) and lp.satisfies_clustering(p.left_keys)
            r_ok = isinstance(rp, HashPartitioning) and rp.satisfies_clustering(p.right_keys)
            left, right = p.left, p.right
            if l_ok and r_ok and lp.num_partitions == rp.num_partitions:
                pass
            elif l_ok and r_ok:
                # keep the side with more buckets, reshuffle the other one into it
                if lp.num_partitions >= rp.num_partitions:
                    right = ShuffleExchangeExec(HashPartitioning(p.right_keys, lp.num_partitions), right)
                else:
                    left = ShuffleExchangeExec(HashPartitioning(p.left_keys, rp.num_partitions), left)
            elif l_ok:
                right = ShuffleExchangeExec(HashPartitioning(p.right_keys, lp.num_partitions), right)
            elif r_ok:
                left = ShuffleExchangeExec(HashPartitioning(p.left_keys, rp.num_partitions), left)
            else:
                left = ShuffleExchangeExec(HashPartitioning(p.left_keys, n_default), left)
                right = ShuffleExchangeExec(HashPartitioning(p.right_keys, n_default), right)
            left = _ensure_sorted(left, p.left_keys)
            right = _ensure_sorted(right, p.right_keys)
            if left is not p.left or right is not p.right:
                return p.with_children((left, right))
        if isinstance(p, BucketUnionExec):
            return None
        return None
    return plan.transform_up(fn)


_EXPR_ID = re.compile(r"#(\d+)")


def canonical_string(plan: SparkPlan) -> str:
    """Expression-id-free rendering of a subtree: ids are renumbered by first appearance, so
    two subtrees that differ only in the ids of their (deduplicated self-join) attributes
    render identically (the role of Spark's ``QueryPlan.canonicalized``)."""
    seen: dict = {}

    def sub(m):
        return "#" + str(seen.setdefault(m.group(1), len(seen)))

    lines = []
    for prefix, node in plan.tree_lines():
        s = prefix + node.simple_string()
        # leaves carry their data identity: local rows by object, scans by their file list
        if isinstance(node, LocalTableScanExec):
            s += f" @{id(node.table)}"
        elif isinstance(node, FileSourceScanExec):
            s += f" @{hash(tuple(sorted(repr(f) for f in node.relation.location.all_files())))}"
            s += f" {sorted(node.selected_buckets) if node.selected_buckets else ''}"
        lines.append(s)
    # literal values verbatim (not renumbered): a string literal such as 'item#5' renders like
    # an attribute id, so two subtrees differing only in such literals would otherwise match
    from .plan_cache import _iter_literals
    lits: list = []
    _iter_literals(plan, lits, set())
    tail = "\n#literals " + repr([(str(x.dtype), x.value) for x in lits])
    return _EXPR_ID.sub(sub, "\n".join(lines)) + tail


def reuse_exchanges(plan: SparkPlan, session) -> SparkPlan:
    """Spark's ``ReuseExchange``: the second and later exchanges whose canonical subtrees equal
    an earlier one become ``ReusedExchange`` leaves (``spark.sql.exchange.reuse``, default
    true).  Index scans of a bucketed self-join have no exchange left to reuse."""
    v = str(session.conf.get("spark.sql.exchange.reuse", "true")).lower()
    if v != "true":
        return plan
    seen: dict = {}

    def fn(p):
        if not isinstance(p, (ShuffleExchangeExec, BroadcastExchangeExec)):
            return None
        k = (type(p).__name__, canonical_string(p))
        first = seen.get(k)
        if first is None:
            seen[k] = p
            return None
        if len(first.output) != len(p.output):
            return None
        return ReusedExchangeExec(p.output, first, p)
    return plan.transform_up(fn)


def _ensure_sorted(child: SparkPlan, keys) -> SparkPlan:
    ordering = child.output_ordering
    if len(ordering) >= len(keys) and all(o.child.semantic_equals(k) and o.ascending
                                          for o, k in zip(ordering, keys)):
        return child
    return SortExec([L.SortOrder(k, True) for k in keys], False, child)
