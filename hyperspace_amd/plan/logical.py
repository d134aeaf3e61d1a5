"""Logical plans of the query front-end (Catalyst's node set, reduced to what the index rules and
executors need): LogicalRelation over a file-based HadoopFsRelation, Filter, Project, Join,
Aggregate, Union, BucketUnion, RepartitionByExpression, Sort, Limit.

Reference analogs: Spark's LogicalRelation/HadoopFsRelation, Hyperspace's
``IndexHadoopFsRelation`` (``index/plans/logical/IndexHadoopFsRelation.scala:29-50``) and
``BucketUnion`` (``index/plans/logical/BucketUnion.scala:31-68``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import pyarrow as pa

from . import expressions as E


@dataclass(frozen=True)
class BucketSpec:
    num_buckets: int
    bucket_column_names: tuple
    sort_column_names: tuple

    def __init__(self, num_buckets, bucket_column_names, sort_column_names=()):
        object.__setattr__(self, "num_buckets", int(num_buckets))
        object.__setattr__(self, "bucket_column_names", tuple(bucket_column_names))
        object.__setattr__(self, "sort_column_names", tuple(sort_column_names))

    def copy(self, **kw):
        return BucketSpec(kw.get("num_buckets", self.num_buckets),
                          kw.get("bucket_column_names", self.bucket_column_names),
                          kw.get("sort_column_names", self.sort_column_names))


@dataclass
class PartitionSpec:
    """Hive-style partitioning discovered from ``key=value`` directories."""
    columns: pa.Schema = field(default_factory=lambda: pa.schema([]))
    # qualified partition directory path -> {col: python value}
    partitions: dict = field(default_factory=dict)
    base_path: Optional[str] = None


class FileIndex:
    """``InMemoryFileIndex``: a fixed list of leaf files plus partition info."""

    kind = "InMemoryFileIndex"

    def __init__(self, root_paths: List[str], files: list, partition_spec: PartitionSpec = None):
        self.root_paths = list(root_paths)
        self._files = list(files)
        self.partition_spec = partition_spec or PartitionSpec()

    def all_files(self) -> list:
        return self._files

    def refresh(self) -> None:
        pass

    @property
    def partition_schema(self) -> pa.Schema:
        return self.partition_spec.columns

    def size_in_bytes(self) -> int:
        return sum(f.length for f in self.all_files())

    def one_file_per_bucket(self) -> bool:
        """True iff no two files carry the same bucket id (cached; the file list is fixed)."""
        v = getattr(self, "_one_per_bucket", None)
        if v is None:
            from ..io.writer import get_bucket_id
            from ..utils import path_utils as P
            ids = [get_bucket_id(P.get_name(f.path)) for f in self.all_files()]
            v = len(ids) == len(set(ids))
            self._one_per_bucket = v
        return v

    def __repr__(self):
        return f"{self.kind}[{', '.join(self.root_paths)}]"


class HadoopFsRelation:
    def __init__(self, location: FileIndex, partition_schema: pa.Schema, data_schema: pa.Schema,
                 bucket_spec: Optional[BucketSpec], file_format: str, options: dict,
                 index=None):
        self.location = location
        self.partition_schema = partition_schema if partition_schema is not None else pa.schema([])
        self.data_schema = data_schema
        self.bucket_spec = bucket_spec
        self.file_format = file_format
        self.options = dict(options or {})
        self.index = index  # IndexLogEntry when this is an IndexHadoopFsRelation

    @property
    def schema(self) -> pa.Schema:
        fields = list(self.data_schema)
        names = {f.name for f in fields}
        fields += [f for f in self.partition_schema if f.name not in names]
        return pa.schema(fields)

    def copy(self, **kw) -> "HadoopFsRelation":
        return HadoopFsRelation(kw.get("location", self.location),
                                kw.get("partition_schema", self.partition_schema),
                                kw.get("data_schema", self.data_schema),
                                kw.get("bucket_spec", self.bucket_spec),
                                kw.get("file_format", self.file_format),
                                kw.get("options", self.options),
                                kw.get("index", self.index))

    def is_index(self) -> bool:
        return self.index is not None

    def __repr__(self):
        if self.index is not None:
            # IndexHadoopFsRelation.toString (IndexHadoopFsRelation.scala:44-48)
            return (f"Hyperspace(Type: {self.index.derived_dataset.kind_abbr}, "
                    f"Name: {self.index.name}, LogVersion: {self.index.id})")
        return self.file_format


# ---------------------------------------------------------------------------------------------
class LogicalPlan:
    children: tuple = ()

    @property
    def output(self) -> List[E.Attribute]:
        raise NotImplementedError

    @property
    def node_name(self) -> str:
        return type(self).__name__

    def expressions(self) -> List[E.Expression]:
        return []

    def references(self) -> List[E.Attribute]:
        out, seen = [], set()
        for e in self.expressions():
            for a in e.references():
                if a.expr_id not in seen:
                    seen.add(a.expr_id)
                    out.append(a)
        return out

    def with_children(self, children) -> "LogicalPlan":
        raise NotImplementedError(type(self).__name__)

    def output_set(self) -> set:
        return {a.expr_id for a in self.output}

    # -- tree traversal --------------------------------------------------------------------------
    def transform_up(self, fn) -> "LogicalPlan":
        new_children = tuple(c.transform_up(fn) for c in self.children)
        node = self.with_children(new_children) if any(
            a is not b for a, b in zip(new_children, self.children)) else self
        r = fn(node)
        return node if r is None else r

    def transform_down(self, fn) -> "LogicalPlan":
        r = fn(self)
        node = self if r is None else r
        if node.children:
            new_children = tuple(c.transform_down(fn) for c in node.children)
            if any(a is not b for a, b in zip(new_children, node.children)):
                node = node.with_children(new_children)
        return node

    def iter_pre(self):
        yield self
        for c in self.children:
            yield from c.iter_pre()

    def collect(self, pred) -> list:
        return [p for p in self.iter_pre() if pred(p)]

    def collect_leaves(self) -> list:
        return [p for p in self.iter_pre() if not p.children]

    def foreach_up(self, fn) -> None:
        for c in self.children:
            c.foreach_up(fn)
        fn(self)

    def find(self, pred):
        for p in self.iter_pre():
            if pred(p):
                return p
        return None

    # -- printing ------------------------------------------------------------------------------
    def simple_string(self) -> str:
        return self.node_name

    def tree_string(self) -> str:
        lines: list = []
        self._tree(lines, [], True)
        return "\n".join(lines)

    def _tree(self, lines, last_flags, is_root):
        prefix = ""
        if last_flags:
            prefix = "".join("   " if f else ":  " for f in last_flags[:-1])
            prefix += "+- " if last_flags[-1] else ":- "
        lines.append(prefix + self.simple_string())
        for i, c in enumerate(self.children):
            c._tree(lines, last_flags + [i == len(self.children) - 1], False)

    def __repr__(self):
        return self.tree_string()


class LeafNode(LogicalPlan):
    def with_children(self, children):
        return self


class LogicalRelation(LeafNode):
    def __init__(self, relation: HadoopFsRelation, output: List[E.Attribute] = None):
        self.relation = relation
        if output is None:
            output = [E.Attribute(f.name, f.type, f.nullable) for f in relation.schema]
        self._output = list(output)

    @property
    def output(self):
        return self._output

    def copy(self, relation=None, output=None) -> "LogicalRelation":
        return LogicalRelation(relation or self.relation, output if output is not None else self._output)

    @property
    def schema(self) -> pa.Schema:
        return self.relation.schema

    def simple_string(self):
        return f"Relation[{','.join(a.sql() for a in self.output)}] {self.relation!r}"


class LocalRelation(LeafNode):
    """In-memory table (``spark.createDataFrame``)."""

    def __init__(self, table: pa.Table, output: List[E.Attribute] = None):
        self.table = table
        self._output = output or [E.Attribute(f.name, f.type, f.nullable) for f in table.schema]

    @property
    def output(self):
        return self._output

    def simple_string(self):
        return f"LocalRelation [{', '.join(a.sql() for a in self.output)}]"


class UnaryNode(LogicalPlan):
    @property
    def child(self) -> LogicalPlan:
        return self.children[0]


class Filter(UnaryNode):
    def __init__(self, condition: E.Expression, child: LogicalPlan):
        self.condition = condition
        self.children = (child,)

    @property
    def output(self):
        return self.child.output

    def expressions(self):
        return [self.condition]

    def with_children(self, children):
        return Filter(self.condition, children[0])

    def simple_string(self):
        return f"Filter {self.condition.sql()}"


class Project(UnaryNode):
    def __init__(self, project_list: List[E.Expression], child: LogicalPlan):
        self.project_list = list(project_list)
        self.children = (child,)

    @property
    def output(self):
        out = []
        for e in self.project_list:
            if isinstance(e, E.Attribute):
                out.append(e)
            elif isinstance(e, E.Alias):
                out.append(e.to_attribute())
            else:
                raise ValueError(f"unnamed project expression {e}")
        return out

    def expressions(self):
        return list(self.project_list)

    def with_children(self, children):
        return Project(self.project_list, children[0])

    def simple_string(self):
        return f"Project [{', '.join(e.sql() for e in self.project_list)}]"


class Join(LogicalPlan):
    def __init__(self, left: LogicalPlan, right: LogicalPlan, join_type: str = "inner",
                 condition: Optional[E.Expression] = None):
        self.children = (left, right)
        self.join_type = join_type
        self.condition = condition

    @property
    def left(self):
        return self.children[0]

    @property
    def right(self):
        return self.children[1]

    @property
    def output(self):
        jt = self.join_type
        if jt in ("leftsemi", "leftanti"):
            return self.left.output
        lo = self.left.output
        ro = self.right.output
        if jt in ("right", "full"):
            lo = [a.with_nullability(True) for a in lo]
        if jt in ("left", "full"):
            ro = [a.with_nullability(True) for a in ro]
        return lo + ro

    def expressions(self):
        return [self.condition] if self.condition is not None else []

    def with_children(self, children):
        return Join(children[0], children[1], self.join_type, self.condition)

    def copy(self, left=None, right=None, condition="__keep__"):
        return Join(left or self.left, right or self.right, self.join_type,
                    self.condition if condition == "__keep__" else condition)

    def simple_string(self):
        cond = f", {self.condition.sql()}" if self.condition is not None else ""
        return f"Join {self.join_type.capitalize()}{cond}"


class Aggregate(UnaryNode):
    def __init__(self, grouping: List[E.Expression], aggregates: List[E.Expression],
                 child: LogicalPlan):
        self.grouping = list(grouping)
        self.aggregates = list(aggregates)
        self.children = (child,)

    @property
    def output(self):
        out = []
        for e in self.aggregates:
            out.append(e if isinstance(e, E.Attribute) else e.to_attribute())
        return out

    def expressions(self):
        return self.grouping + self.aggregates

    def with_children(self, children):
        return Aggregate(self.grouping, self.aggregates, children[0])

    def simple_string(self):
        return (f"Aggregate [{', '.join(g.sql() for g in self.grouping)}], "
                f"[{', '.join(a.sql() for a in self.aggregates)}]")


class Union(LogicalPlan):
    def __init__(self, children: List[LogicalPlan]):
        self.children = tuple(children)

    @property
    def output(self):
        first = self.children[0].output
        nullable = [any(c.output[i].nullable for c in self.children) for i in range(len(first))]
        return [a.with_nullability(n) for a, n in zip(first, nullable)]

    def with_children(self, children):
        return Union(list(children))


class BucketUnion(LogicalPlan):
    """Bucket-preserving union (``BucketUnion.scala:31-68``): all children must have the same
    column count/types; the result keeps the index's HashPartitioning."""

    def __init__(self, children: List[LogicalPlan], bucket_spec: BucketSpec):
        if len(children) < 2:
            raise ValueError("BucketUnion requires at least two children")
        first = children[0].output
        for c in children[1:]:
            co = c.output
            if len(co) != len(first) or any(not a.data_type.equals(b.data_type)
                                            for a, b in zip(co, first)):
                raise ValueError("BucketUnion children must have compatible outputs")
        self.children = tuple(children)
        self.bucket_spec = bucket_spec

    @property
    def output(self):
        return self.children[0].output

    def with_children(self, children):
        return BucketUnion(list(children), self.bucket_spec)

    def simple_string(self):
        bs = self.bucket_spec
        return (f"BucketUnion {bs.num_buckets} buckets, bucket columns: "
                f"[{', '.join(bs.bucket_column_names)}]")


class RepartitionByExpression(UnaryNode):
    def __init__(self, partition_expressions: List[E.Expression], child: LogicalPlan,
                 num_partitions: int):
        self.partition_expressions = list(partition_expressions)
        self.children = (child,)
        self.num_partitions = int(num_partitions)

    @property
    def output(self):
        return self.child.output

    def expressions(self):
        return list(self.partition_expressions)

    def with_children(self, children):
        return RepartitionByExpression(self.partition_expressions, children[0], self.num_partitions)

    def simple_string(self):
        return (f"RepartitionByExpression [{', '.join(e.sql() for e in self.partition_expressions)}]"
                f", {self.num_partitions}")


@dataclass
class SortOrder:
    child: E.Expression
    ascending: bool = True

    def sql(self):
        return f"{self.child.sql()} {'ASC NULLS FIRST' if self.ascending else 'DESC NULLS LAST'}"


class Sort(UnaryNode):
    def __init__(self, order: List[SortOrder], global_sort: bool, child: LogicalPlan):
        self.order = list(order)
        self.global_sort = global_sort
        self.children = (child,)

    @property
    def output(self):
        return self.child.output

    def expressions(self):
        return [o.child for o in self.order]

    def with_children(self, children):
        return Sort(self.order, self.global_sort, children[0])

    def simple_string(self):
        return f"Sort [{', '.join(o.sql() for o in self.order)}], {str(self.global_sort).lower()}"


class Limit(UnaryNode):
    def __init__(self, n: int, child: LogicalPlan):
        self.n = int(n)
        self.children = (child,)

    @property
    def output(self):
        return self.child.output

    def with_children(self, children):
        return Limit(self.n, children[0])

    def simple_string(self):
        return f"GlobalLimit {self.n}"


def is_logical_relation(plan: LogicalPlan) -> bool:
    """``LogicalPlanUtils.isLogicalRelation`` (``util/LogicalPlanUtils.scala:25-38``)."""
    return isinstance(plan, LogicalRelation)
