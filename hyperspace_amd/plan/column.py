"""User-facing ``Column`` API (``col("a") > 5``, ``df["a"] == df2["b"]``, ``sum_("x")``)."""
from __future__ import annotations

from . import expressions as E


def _expr(v) -> E.Expression:
    if isinstance(v, Column):
        return v.expr
    if isinstance(v, E.Expression):
        return v
    return E.Literal(v)


class Column:
    def __init__(self, expr: E.Expression):
        self.expr = expr

    # comparisons
    def __eq__(self, o):  # noqa: D105
        return Column(E.EqualTo(self.expr, _expr(o)))

    def __ne__(self, o):
        return Column(E.NotEqual(self.expr, _expr(o)))

    def __lt__(self, o):
        return Column(E.LessThan(self.expr, _expr(o)))

    def __le__(self, o):
        return Column(E.LessThanOrEqual(self.expr, _expr(o)))

    def __gt__(self, o):
        return Column(E.GreaterThan(self.expr, _expr(o)))

    def __ge__(self, o):
        return Column(E.GreaterThanOrEqual(self.expr, _expr(o)))

    # boolean
    def __and__(self, o):
        return Column(E.And(self.expr, _expr(o)))

    def __or__(self, o):
        return Column(E.Or(self.expr, _expr(o)))

    def __invert__(self):
        return Column(E.Not(self.expr))

    # arithmetic
    def __add__(self, o):
        return Column(E.Add(self.expr, _expr(o)))

    def __radd__(self, o):
        return Column(E.Add(_expr(o), self.expr))

    def __sub__(self, o):
        return Column(E.Subtract(self.expr, _expr(o)))

    def __rsub__(self, o):
        return Column(E.Subtract(_expr(o), self.expr))

    def __mul__(self, o):
        return Column(E.Multiply(self.expr, _expr(o)))

    def __rmul__(self, o):
        return Column(E.Multiply(_expr(o), self.expr))

    def __mod__(self, o):
        return Column(E.Remainder(self.expr, _expr(o)))

    def __rmod__(self, o):
        return Column(E.Remainder(_expr(o), self.expr))

    def __truediv__(self, o):
        return Column(E.Divide(self.expr, _expr(o)))

    def __neg__(self):
        return Column(E.Subtract(E.Literal(0), self.expr))

    __hash__ = object.__hash__

    def isin(self, *values):
        if len(values) == 1 and isinstance(values[0], (list, tuple, set)):
            values = tuple(values[0])
        return Column(E.In(self.expr, [_expr(v) for v in values]))

    def isNull(self):
        return Column(E.IsNull(self.expr))

    def isNotNull(self):
        return Column(E.IsNotNull(self.expr))

    def between(self, lo, hi):
        return (self >= lo) & (self <= hi)

    def asc(self):
        """Sort order for ``orderBy`` (ascending, nulls first — Spark's default)."""
        c = Column(self.expr)
        c.sort_ascending = True
        return c

    def desc(self):
        """Sort order for ``orderBy`` (descending, nulls last)."""
        c = Column(self.expr)
        c.sort_ascending = False
        return c

    def alias(self, name: str):
        return Column(E.Alias(self.expr, name))

    def cast(self, dtype):
        """``dtype``: a pyarrow type or a Spark type name ("int", "bigint", "double", ...)."""
        if isinstance(dtype, str):
            import pyarrow as pa
            names = {"byte": pa.int8(), "tinyint": pa.int8(), "short": pa.int16(),
                     "smallint": pa.int16(), "int": pa.int32(), "integer": pa.int32(),
                     "long": pa.int64(), "bigint": pa.int64(), "float": pa.float32(),
                     "double": pa.float64(), "string": pa.string(), "boolean": pa.bool_(),
                     "date": pa.date32()}
            if dtype.lower() not in names:
                raise ValueError(f"unknown type name {dtype!r}")
            dtype = names[dtype.lower()]
        return Column(E.Cast(self.expr, dtype))

    def __repr__(self):
        return f"Column<{self.expr.sql()}>"


def col(name: str) -> Column:
    return Column(E.UnresolvedAttribute(name))


def lit(v) -> Column:
    return Column(E.Literal(v))


def sum_(c) -> Column:
    return Column(E.Sum(_expr(col(c) if isinstance(c, str) else c)))


def count(c="*") -> Column:
    if c == "*":
        return Column(E.Count(None))
    return Column(E.Count(_expr(col(c) if isinstance(c, str) else c)))


def min_(c) -> Column:
    return Column(E.Min(_expr(col(c) if isinstance(c, str) else c)))


def max_(c) -> Column:
    return Column(E.Max(_expr(col(c) if isinstance(c, str) else c)))


def avg(c) -> Column:
    return Column(E.Avg(_expr(col(c) if isinstance(c, str) else c)))


def input_file_name() -> Column:  # documented for API parity; lineage is attached natively.
    raise NotImplementedError("input_file_name() is computed natively by the index build (K2)")
