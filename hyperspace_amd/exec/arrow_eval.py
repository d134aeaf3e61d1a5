"""Expression evaluation over pyarrow tables (the CPU oracle's expression engine).

Columns inside executors are keyed ``<name>#<exprId>`` so self-joins never collide.
Comparison operands are coerced the way Spark's analyzer would (string literal vs date column ->
date, int vs double -> double).
"""
from __future__ import annotations

import datetime

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from ..plan import expressions as E


def key(a: E.Attribute) -> str:
    return f"{a.name}#{a.expr_id}"


def _coerce_literal(lit: E.Literal, target: pa.DataType):
    v = lit.value
    if v is None:
        return pa.scalar(None, target)
    if pa.types.is_date32(target) and isinstance(v, str):
        return pa.scalar(datetime.date.fromisoformat(v[:10]), pa.date32())
    if pa.types.is_timestamp(target) and isinstance(v, str):
        return pa.scalar(datetime.datetime.fromisoformat(v), target)
    if pa.types.is_timestamp(target) and isinstance(v, datetime.date) and \
            not isinstance(v, datetime.datetime):
        return pa.scalar(datetime.datetime(v.year, v.month, v.day), target)
    if (pa.types.is_string(target) or pa.types.is_large_string(target)) and not isinstance(v, str):
        return pa.scalar(str(v), pa.string())
    if pa.types.is_integer(target) and isinstance(v, float):
        return pa.scalar(v, pa.float64())
    if pa.types.is_floating(target) and isinstance(v, (int, float)) and not isinstance(v, bool):
        return pa.scalar(float(v), pa.float64())
    if pa.types.is_integer(target) and isinstance(v, int) and not isinstance(v, bool):
        return pa.scalar(v, pa.int64())
    if pa.types.is_decimal(target) and isinstance(v, (int, float)):
        return pa.scalar(float(v), pa.float64())
    return pa.scalar(v, lit.data_type)


def _numeric_align(a, b):
    ta, tb = a.type, b.type
    if pa.types.is_decimal(ta):
        a = pc.cast(a, pa.float64())
    if pa.types.is_decimal(tb):
        b = pc.cast(b, pa.float64())
    ta, tb = a.type, b.type
    if (pa.types.is_floating(ta) and pa.types.is_integer(tb)) or \
            (pa.types.is_integer(ta) and pa.types.is_floating(tb)):
        a, b = pc.cast(a, pa.float64()), pc.cast(b, pa.float64())
    elif pa.types.is_integer(ta) and pa.types.is_integer(tb) and ta != tb:
        a, b = pc.cast(a, pa.int64()), pc.cast(b, pa.int64())
    return a, b


def _operands(e: E.BinaryExpression, t: pa.Table):
    l, r = e.left, e.right
    if isinstance(r, E.Literal) and not isinstance(l, E.Literal):
        lv = eval_expr(l, t)
        return _numeric_align(lv, _coerce_literal(r, lv.type))
    if isinstance(l, E.Literal) and not isinstance(r, E.Literal):
        rv = eval_expr(r, t)
        return _numeric_align(_coerce_literal(l, rv.type), rv)
    return _numeric_align(eval_expr(l, t), eval_expr(r, t))


_CMP = {E.EqualTo: pc.equal, E.NotEqual: pc.not_equal, E.LessThan: pc.less,
        E.LessThanOrEqual: pc.less_equal, E.GreaterThan: pc.greater,
        E.GreaterThanOrEqual: pc.greater_equal}
_ARITH = {E.Add: pc.add, E.Subtract: pc.subtract, E.Multiply: pc.multiply}


def _is_num(t: pa.DataType) -> bool:
    return pa.types.is_integer(t) or pa.types.is_floating(t)


def eval_expr(e: E.Expression, t: pa.Table):
    if isinstance(e, E.Attribute):
        return t.column(key(e))
    if isinstance(e, E.Alias):
        return eval_expr(e.child, t)
    if isinstance(e, E.Literal):
        return pa.array([e.value] * t.num_rows, e.data_type if e.value is not None else pa.null())
    if type(e) in _CMP:
        a, b = _operands(e, t)
        return _CMP[type(e)](a, b)
    if isinstance(e, E.And):
        return pc.and_kleene(eval_expr(e.left, t), eval_expr(e.right, t))
    if isinstance(e, E.Or):
        return pc.or_kleene(eval_expr(e.left, t), eval_expr(e.right, t))
    if isinstance(e, E.Not):
        return pc.invert(eval_expr(e.child, t))
    if isinstance(e, E.IsNull):
        return pc.is_null(eval_expr(e.child, t))
    if isinstance(e, E.IsNotNull):
        return pc.is_valid(eval_expr(e.child, t))
    if isinstance(e, (E.In, E.InSet)):
        v = eval_expr(e.value, t)
        raw = [x.value for x in e.values] if isinstance(e, E.In) else list(e.hset)
        lits = [_coerce_literal(E.Literal(x), v.type).as_py() for x in raw if x is not None]
        vtype = v.type
        if pa.types.is_integer(vtype) and any(isinstance(x, float) for x in lits):
            v = pc.cast(v, pa.float64())
            vtype = pa.float64()
        vs = pa.array(lits, vtype if not pa.types.is_dictionary(vtype) else vtype.value_type)
        return pc.is_in(v, value_set=vs)
    if type(e) in _ARITH:
        a, b = _operands(e, t)
        return _ARITH[type(e)](a, b)
    if isinstance(e, E.Remainder):
        return _remainder(*_operands(e, t), t.num_rows, e.data_type)
    if isinstance(e, E.Divide):
        # Spark: a double division, NULL for a zero divisor
        a, b = _operands(e, t)
        b = pc.cast(b, pa.float64())
        q = pc.divide(pc.cast(a, pa.float64()), b)
        return pc.if_else(pc.equal(b, 0.0), pa.scalar(None, pa.float64()), q)
    if isinstance(e, E.Cast):
        v = eval_expr(e.child, t)
        if _is_num(v.type) and _is_num(e.dtype):
            if pa.types.is_floating(v.type) and pa.types.is_integer(e.dtype):
                return _float_to_int(v, e.dtype)
            # Spark's numeric casts truncate toward zero and wrap (non-ANSI)
            return pc.cast(v, e.dtype, safe=False)
        return pc.cast(v, e.dtype)
    raise NotImplementedError(f"cannot evaluate {type(e).__name__}")


def _remainder(a, b, n: int, dtype=None):
    """Spark ``%``: truncated remainder (sign of the dividend), NULL for a zero divisor or a
    NULL operand; ``fmod`` for floating-point operands; Long.MIN_VALUE % -1 = 0.  Either operand
    may be a scalar (a literal dividend or divisor): both are broadcast to the ``n`` rows first.
    The result takes the expression's type ``dtype``."""
    import numpy as np

    def arr(x):
        if isinstance(x, pa.Scalar):
            return pa.array([x.as_py()] * n, x.type)
        return x.combine_chunks() if isinstance(x, pa.ChunkedArray) else x
    a, b = arr(a), arr(b)
    f = pa.types.is_floating(a.type) or pa.types.is_floating(b.type)
    out_t = pa.float64() if f else pa.int64()
    av = np.asarray(pc.fill_null(pc.cast(a, out_t), 0).to_numpy(zero_copy_only=False))
    bv = np.asarray(pc.fill_null(pc.cast(b, out_t), 0).to_numpy(zero_copy_only=False))
    bad = np.asarray(pc.or_kleene(pc.is_null(a), pc.is_null(b)).to_numpy(zero_copy_only=False))
    bad = bad | (bv == 0)
    if f:
        with np.errstate(invalid="ignore"):
            r = np.fmod(av, np.where(bad, 1.0, bv))
    else:
        safe = np.where(bad | (bv == -1), 1, bv)
        r = np.fmod(av, safe)          # C / JVM truncated remainder
        r = np.where(bv == -1, 0, r)
    out = pa.array(r, out_t, mask=bad)
    if dtype is not None and out.type != dtype and (pa.types.is_integer(dtype) or
                                                    pa.types.is_floating(dtype)):
        out = pc.cast(out, dtype, safe=False)
    return out


def _float_to_int(v, dtype: pa.DataType):
    """Spark (non-ANSI) float -> integral cast: truncate toward zero, NaN -> 0, saturate to the
    long range (d2l) for a long target, to the int range (d2i) otherwise; a short / byte target
    then wraps (``toInt.toShort``).  Explicit clamps: an out-of-range ``pc.cast`` is undefined."""
    lo, hi = ((-2.0 ** 63, 2.0 ** 63) if pa.types.is_int64(dtype)
              else (-2147483648.0, 2147483647.0))
    f = pc.cast(v, pa.float64())
    f = pc.if_else(pc.is_nan(f), 0.0, f)
    f = pc.trunc(pc.min_element_wise(pc.max_element_wise(f, lo, skip_nulls=False), hi,
                                     skip_nulls=False))
    if pa.types.is_int64(dtype):
        big = pc.greater_equal(f, 2.0 ** 63)
        out = pc.cast(pc.if_else(big, 0.0, f), pa.int64(), safe=False)
        return pc.if_else(big, pa.scalar(2**63 - 1, pa.int64()), out)
    return pc.cast(pc.cast(f, pa.int64(), safe=False), dtype, safe=False)


def eval_predicate(e: E.Expression, t: pa.Table) -> pa.Table:
    mask = eval_expr(e, t)
    if isinstance(mask, pa.ChunkedArray):
        mask = mask.combine_chunks()
    return t.filter(mask, null_selection_behavior="drop")


def to_numpy(col) -> np.ndarray:
    if isinstance(col, pa.ChunkedArray):
        col = col.combine_chunks()
    return col.to_numpy(zero_copy_only=False)
