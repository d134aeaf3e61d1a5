"""Expression trees of the query front-end (the subset of Catalyst the index rules need,
SURVEY §7.4 item 8): attributes, literals, comparisons, boolean logic, IN, null tests,
arithmetic, aliases and aggregate functions.

Attributes carry a unique ``expr_id`` (Catalyst's ``ExprId``); equality of attributes is by id,
which is what ``JoinIndexRule.ensureAttributeRequirements`` relies on when it canonicalizes
join-condition attributes (``JoinIndexRule.scala:232-271``).
"""
from __future__ import annotations

import datetime
import itertools
from typing import Iterable, List

import pyarrow as pa

from .types import common_numeric

_ids = itertools.count(1)


def new_expr_id() -> int:
    return next(_ids)


class Expression:
    children: tuple = ()

    # -- tree utilities -----------------------------------------------------------------------
    def references(self) -> List["Attribute"]:
        out: list = []
        seen = set()
        for e in self.iter_tree():
            if isinstance(e, Attribute) and e.expr_id not in seen:
                seen.add(e.expr_id)
                out.append(e)
        return out

    def iter_tree(self):
        yield self
        for c in self.children:
            yield from c.iter_tree()

    def with_children(self, children) -> "Expression":
        raise NotImplementedError(type(self).__name__)

    def transform_up(self, fn) -> "Expression":
        if self.children:
            new_children = tuple(c.transform_up(fn) for c in self.children)
            node = self.with_children(new_children) if any(
                a is not b for a, b in zip(new_children, self.children)) else self
        else:
            node = self
        r = fn(node)
        return node if r is None else r

    @property
    def data_type(self) -> pa.DataType:
        raise NotImplementedError

    @property
    def nullable(self) -> bool:
        return any(c.nullable for c in self.children)

    def semantic_equals(self, other) -> bool:
        return self.canonical_key() == other.canonical_key()

    def canonical_key(self):
        return (type(self).__name__,) + tuple(c.canonical_key() for c in self.children)

    def __repr__(self):
        return self.sql()

    def sql(self) -> str:
        raise NotImplementedError


class LeafExpression(Expression):
    def with_children(self, children):
        return self


class Attribute(LeafExpression):
    def __init__(self, name: str, dtype: pa.DataType, nullable: bool = True, expr_id: int = None,
                 qualifier: str = None):
        self.name = name
        self.dtype = dtype
        self._nullable = nullable
        self.expr_id = expr_id if expr_id is not None else new_expr_id()
        self.qualifier = qualifier

    @property
    def data_type(self):
        return self.dtype

    @property
    def nullable(self):
        return self._nullable

    def with_nullability(self, nullable: bool) -> "Attribute":
        return Attribute(self.name, self.dtype, nullable, self.expr_id, self.qualifier)

    def new_instance(self) -> "Attribute":
        return Attribute(self.name, self.dtype, self._nullable, None, self.qualifier)

    def canonical_key(self):
        return ("Attribute", self.expr_id)

    def __eq__(self, o):
        return isinstance(o, Attribute) and o.expr_id == self.expr_id

    def __hash__(self):
        return hash(("attr", self.expr_id))

    def sql(self):
        return f"{self.name}#{self.expr_id}"


class Literal(LeafExpression):
    def __init__(self, value, dtype: pa.DataType = None):
        if dtype is None:
            dtype = infer_literal_type(value)
        self.value = value
        self.dtype = dtype

    @property
    def data_type(self):
        return self.dtype

    @property
    def nullable(self):
        return self.value is None

    def canonical_key(self):
        return ("Literal", repr(self.value), str(self.dtype))

    def sql(self):
        v = self.value
        if v is None:
            return "null"
        if isinstance(v, str):
            return v
        if isinstance(v, datetime.date):
            return v.isoformat()
        return str(v)


def infer_literal_type(v) -> pa.DataType:
    if v is None:
        return pa.null()
    if isinstance(v, bool):
        return pa.bool_()
    if isinstance(v, int):
        return pa.int32() if -2 ** 31 <= v < 2 ** 31 else pa.int64()
    if isinstance(v, float):
        return pa.float64()
    if isinstance(v, str):
        return pa.string()
    if isinstance(v, datetime.datetime):
        return pa.timestamp("us")
    if isinstance(v, datetime.date):
        return pa.date32()
    if isinstance(v, bytes):
        return pa.binary()
    raise TypeError(f"unsupported literal {v!r}")


class Alias(Expression):
    def __init__(self, child: Expression, name: str, expr_id: int = None):
        self.children = (child,)
        self.name = name
        self.expr_id = expr_id if expr_id is not None else new_expr_id()

    @property
    def child(self):
        return self.children[0]

    def with_children(self, children):
        return Alias(children[0], self.name, self.expr_id)

    @property
    def data_type(self):
        return self.child.data_type

    def to_attribute(self) -> Attribute:
        return Attribute(self.name, self.data_type, self.child.nullable, self.expr_id)

    def canonical_key(self):
        return ("Alias", self.child.canonical_key())

    def sql(self):
        return f"{self.child.sql()} AS {self.name}#{self.expr_id}"


class UnresolvedAttribute(LeafExpression):
    """A column referenced by name before analysis (``col("a")``)."""

    def __init__(self, name: str):
        self.name = name

    @property
    def data_type(self):
        raise ValueError(f"unresolved attribute {self.name}")

    def canonical_key(self):
        return ("Unresolved", self.name)

    def sql(self):
        return f"'{self.name}"


# ---------------------------------------------------------------------------------------------
# Predicates
# ---------------------------------------------------------------------------------------------
class BinaryExpression(Expression):
    symbol = "?"

    def __init__(self, left: Expression, right: Expression):
        self.children = (left, right)

    @property
    def left(self):
        return self.children[0]

    @property
    def right(self):
        return self.children[1]

    def with_children(self, children):
        return type(self)(children[0], children[1])

    def sql(self):
        return f"({self.left.sql()} {self.symbol} {self.right.sql()})"


class Predicate(Expression):
    @property
    def data_type(self):
        return pa.bool_()


class BinaryComparison(BinaryExpression, Predicate):
    op = "?"


class EqualTo(BinaryComparison):
    symbol, op = "=", "eq"


class NotEqual(BinaryComparison):
    symbol, op = "!=", "ne"

    def sql(self):
        return f"NOT ({self.left.sql()} = {self.right.sql()})"


class LessThan(BinaryComparison):
    symbol, op = "<", "lt"


class LessThanOrEqual(BinaryComparison):
    symbol, op = "<=", "le"


class GreaterThan(BinaryComparison):
    symbol, op = ">", "gt"


class GreaterThanOrEqual(BinaryComparison):
    symbol, op = ">=", "ge"


FLIP = {EqualTo: EqualTo, NotEqual: NotEqual, LessThan: GreaterThan,
        LessThanOrEqual: GreaterThanOrEqual, GreaterThan: LessThan,
        GreaterThanOrEqual: LessThanOrEqual}


class And(BinaryExpression, Predicate):
    symbol = "AND"


class Or(BinaryExpression, Predicate):
    symbol = "OR"


class Not(Predicate):
    def __init__(self, child):
        self.children = (child,)

    @property
    def child(self):
        return self.children[0]

    def with_children(self, children):
        return Not(children[0])

    def sql(self):
        return f"NOT {self.child.sql()}"


class IsNull(Predicate):
    def __init__(self, child):
        self.children = (child,)

    @property
    def child(self):
        return self.children[0]

    @property
    def nullable(self):
        return False

    def with_children(self, children):
        return IsNull(children[0])

    def sql(self):
        return f"isnull({self.child.sql()})"


class IsNotNull(Predicate):
    def __init__(self, child):
        self.children = (child,)

    @property
    def child(self):
        return self.children[0]

    @property
    def nullable(self):
        return False

    def with_children(self, children):
        return IsNotNull(children[0])

    def sql(self):
        return f"isnotnull({self.child.sql()})"


class In(Predicate):
    def __init__(self, value: Expression, values: List[Expression]):
        self.children = (value, *values)

    @property
    def value(self):
        return self.children[0]

    @property
    def values(self):
        return self.children[1:]

    def with_children(self, children):
        return In(children[0], list(children[1:]))

    def sql(self):
        return f"{self.value.sql()} IN ({','.join(v.sql() for v in self.values)})"


class InSet(Predicate):
    """``OptimizeIn`` output for large literal lists (``HybridScanSuite.scala:138-165``)."""

    def __init__(self, value: Expression, hset: frozenset):
        self.children = (value,)
        self.hset = frozenset(hset)

    @property
    def value(self):
        return self.children[0]

    def with_children(self, children):
        return InSet(children[0], self.hset)

    def canonical_key(self):
        return ("InSet", self.value.canonical_key(), tuple(sorted(map(repr, self.hset))))

    def sql(self):
        return f"{self.value.sql()} INSET ({','.join(map(str, sorted(self.hset, key=repr)))})"


# ---------------------------------------------------------------------------------------------
# Arithmetic
# ---------------------------------------------------------------------------------------------
class BinaryArithmetic(BinaryExpression):
    op = "?"

    @property
    def data_type(self):
        return common_numeric(self.left.data_type, self.right.data_type)


class Add(BinaryArithmetic):
    symbol, op = "+", "add"


class Subtract(BinaryArithmetic):
    symbol, op = "-", "sub"


class Multiply(BinaryArithmetic):
    symbol, op = "*", "mul"


class Remainder(BinaryArithmetic):
    """``a % b``: Spark's (and the JVM's) remainder - the sign follows the dividend, NULL for a
    zero divisor; ``fmod`` for floating-point operands."""
    symbol, op = "%", "mod"


class Divide(BinaryArithmetic):
    symbol, op = "/", "div"

    @property
    def data_type(self):
        return pa.float64()


class Cast(Expression):
    def __init__(self, child, dtype: pa.DataType):
        self.children = (child,)
        self.dtype = dtype

    @property
    def child(self):
        return self.children[0]

    @property
    def data_type(self):
        return self.dtype

    def with_children(self, children):
        return Cast(children[0], self.dtype)

    def canonical_key(self):
        return ("Cast", str(self.dtype), self.child.canonical_key())

    def sql(self):
        return f"cast({self.child.sql()} as {self.dtype})"


# ---------------------------------------------------------------------------------------------
# Aggregates
# ---------------------------------------------------------------------------------------------
class AggregateFunction(Expression):
    name = "agg"

    def __init__(self, child: Expression = None):
        self.children = (child,) if child is not None else ()

    @property
    def child(self):
        return self.children[0] if self.children else None

    def with_children(self, children):
        return type(self)(children[0] if children else None)

    def sql(self):
        return f"{self.name}({self.child.sql() if self.child is not None else '1'})"


class Sum(AggregateFunction):
    name = "sum"

    @property
    def data_type(self):
        t = self.child.data_type
        return pa.int64() if pa.types.is_integer(t) else pa.float64()


class Count(AggregateFunction):
    name = "count"

    @property
    def data_type(self):
        return pa.int64()

    @property
    def nullable(self):
        return False


class Min(AggregateFunction):
    name = "min"

    @property
    def data_type(self):
        return self.child.data_type


class Max(AggregateFunction):
    name = "max"

    @property
    def data_type(self):
        return self.child.data_type


class Avg(AggregateFunction):
    name = "avg"

    @property
    def data_type(self):
        return pa.float64()


# ---------------------------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------------------------
def split_conjuncts(e: Expression) -> List[Expression]:
    if isinstance(e, And):
        return split_conjuncts(e.left) + split_conjuncts(e.right)
    return [e]


def conjoin(preds: Iterable[Expression]):
    preds = list(preds)
    if not preds:
        return None
    out = preds[0]
    for p in preds[1:]:
        out = And(out, p)
    return out


def attr_set(exprs) -> set:
    out = set()
    for e in exprs:
        for r in e.references():
            out.add(r.expr_id)
    return out


def contains_aggregate(e: Expression) -> bool:
    return any(isinstance(x, AggregateFunction) for x in e.iter_tree())
