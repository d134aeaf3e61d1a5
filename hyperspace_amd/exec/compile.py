"""Lowering of filter / aggregate expressions onto the HIP kernel templates.

* Predicates -> CNF of leaf comparisons (``Pred`` structs): NOT is pushed into the leaves
  (De Morgan, operator flip), OR-of-ANDs is distributed, string literals become dictionary-code
  bounds, dates/timestamps become integers.
* Aggregate inputs -> products of affine terms ``prod(alpha + beta * col)``.
Anything outside these shapes raises ``Unsupported`` and the executor falls back.
"""
from __future__ import annotations

import bisect
import datetime
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import pyarrow as pa

from ..ops import _lib as NL
from ..plan import expressions as E


class Unsupported(Exception):
    pass


_OPS = {E.EqualTo: NL.OP_EQ, E.NotEqual: NL.OP_NE, E.LessThan: NL.OP_LT,
        E.LessThanOrEqual: NL.OP_LE, E.GreaterThan: NL.OP_GT, E.GreaterThanOrEqual: NL.OP_GE}
_NEG = {NL.OP_EQ: NL.OP_NE, NL.OP_NE: NL.OP_EQ, NL.OP_LT: NL.OP_GE, NL.OP_LE: NL.OP_GT,
        NL.OP_GT: NL.OP_LE, NL.OP_GE: NL.OP_LT}
_FLIP = {NL.OP_EQ: NL.OP_EQ, NL.OP_NE: NL.OP_NE, NL.OP_LT: NL.OP_GT, NL.OP_LE: NL.OP_GE,
         NL.OP_GT: NL.OP_LT, NL.OP_GE: NL.OP_LE}


# ------------------------------------------------------------------------------------------------
# Leaf representation before slot binding
# ------------------------------------------------------------------------------------------------
class Leaf:
    __slots__ = ("kind", "op", "attr", "attr2", "value", "values", "lit")

    def __init__(self, kind, op, attr, attr2=None, value=None, values=None, lit=None):
        self.kind, self.op, self.attr, self.attr2 = kind, op, attr, attr2
        self.value, self.values = value, values
        self.lit = lit      # cmp_lit: the Literal node ``value`` came from (``rebind``)

    def negate(self) -> "Leaf":
        if self.kind in ("cmp_lit", "cmp_col", "in", "bitmap"):
            return Leaf(self.kind, _NEG[self.op], self.attr, self.attr2, self.value, self.values,
                        self.lit)
        if self.kind == "isnull":
            return Leaf("notnull", 0, self.attr)
        if self.kind == "notnull":
            return Leaf("isnull", 0, self.attr)
        if self.kind == "const":
            return Leaf("const", 0, None, value=not self.value)
        raise Unsupported("negate")


_EPOCH = datetime.datetime(1970, 1, 1)
_UNIT_PER_US = {"us": (1, 1), "ns": (1000, 1), "ms": (1, 1000), "s": (1, 1_000_000)}


def _lit_value(v, dtype=None):
    """A literal in the device storage of the column it is compared with: dates as days,
    timestamps as integers in the column's own unit (exact integer arithmetic; tz-aware values
    are converted to UTC).  A literal the column's unit cannot represent exactly is
    ``Unsupported`` (the host path evaluates it)."""
    if isinstance(v, datetime.datetime):
        if v.tzinfo is not None:
            v = v.astimezone(datetime.timezone.utc).replace(tzinfo=None)
        us = (v - _EPOCH) // datetime.timedelta(microseconds=1)
        if dtype is not None and pa.types.is_date32(dtype):
            days, rem = divmod(us, 86_400_000_000)
            if rem:
                raise Unsupported("timestamp literal compared with a date column")
            return days
        if dtype is not None and pa.types.is_timestamp(dtype):
            mul, div = _UNIT_PER_US[dtype.unit]
            if us % div:
                raise Unsupported(f"timestamp literal finer than the column unit {dtype.unit}")
            return us * mul // div
        return us
    if isinstance(v, datetime.date):
        days = (v - datetime.date(1970, 1, 1)).days
        if dtype is not None and pa.types.is_timestamp(dtype):
            mul, div = _UNIT_PER_US[dtype.unit]
            return days * 86_400_000_000 * mul // div
        return days
    return v


def _to_nnf(e: E.Expression, negate: bool = False):
    """Negation normal form over And/Or with Leaf leaves."""
    if isinstance(e, E.Not):
        return _to_nnf(e.child, not negate)
    if isinstance(e, (E.And, E.Or)):
        l, r = _to_nnf(e.left, negate), _to_nnf(e.right, negate)
        is_and = isinstance(e, E.And) != negate
        return ("and" if is_and else "or", l, r)
    leaf = _leaf(e)
    return leaf.negate() if negate else leaf


class KeyBitmap(E.Expression):
    """Executor-internal predicate ``attr in <device key bitmap>``: bit (value - base) of
    ``words`` (int64 tensor, ``nbits`` bits) is set.  Built from a semi-join's build-side keys
    (GpuBackend._semi_join_agg) and bound as a PK_BITMAP predicate of the probe scan."""

    def __init__(self, attr: E.Attribute, words, base: int, nbits: int):
        self.attr, self.words, self.base, self.nbits = attr, words, int(base), int(nbits)
        self.children = (attr,)

    @property
    def data_type(self):
        return pa.bool_()

    @property
    def nullable(self) -> bool:
        return False

    def with_children(self, children):
        return KeyBitmap(children[0], self.words, self.base, self.nbits)

    def canonical_key(self):
        return ("KeyBitmap", self.attr.canonical_key(), id(self.words), self.base, self.nbits)

    def sql(self) -> str:
        return f"{self.attr.sql()} IN key_bitmap[{self.base}, {self.base + self.nbits})"


def _leaf(e: E.Expression) -> Leaf:
    if isinstance(e, KeyBitmap):
        return Leaf("bitmap", NL.OP_EQ, e.attr, value=e)
    if isinstance(e, E.Literal) and isinstance(e.value, bool):
        return Leaf("const", 0, None, value=e.value)
    if type(e) in _OPS:
        l, r = e.left, e.right
        op = _OPS[type(e)]
        if isinstance(l, E.Cast):
            l = l.child
        if isinstance(r, E.Cast):
            r = r.child
        if isinstance(l, E.Attribute) and isinstance(r, E.Literal):
            return Leaf("cmp_lit", op, l, value=_lit_value(r.value, l.data_type), lit=r)
        if isinstance(r, E.Attribute) and isinstance(l, E.Literal):
            return Leaf("cmp_lit", _FLIP[op], r, value=_lit_value(l.value, r.data_type), lit=l)
        if isinstance(l, E.Attribute) and isinstance(r, E.Attribute):
            return Leaf("cmp_col", op, l, r)
        raise Unsupported(f"comparison {e.sql()}")
    if isinstance(e, E.IsNull) and isinstance(e.child, E.Attribute):
        return Leaf("isnull", 0, e.child)
    if isinstance(e, E.IsNotNull) and isinstance(e.child, E.Attribute):
        return Leaf("notnull", 0, e.child)
    if isinstance(e, E.In) and isinstance(e.value, E.Attribute) and \
            all(isinstance(v, E.Literal) for v in e.values):
        return Leaf("in", NL.OP_EQ, e.value, values=[_lit_value(v.value, e.value.data_type) for v in e.values])
    if isinstance(e, E.InSet) and isinstance(e.value, E.Attribute):
        return Leaf("in", NL.OP_EQ, e.value, values=[_lit_value(v, e.value.data_type) for v in e.hset])
    raise Unsupported(f"predicate {type(e).__name__}")


def _cnf(node) -> List[List[Leaf]]:
    if isinstance(node, Leaf):
        return [[node]]
    kind, l, r = node
    lc, rc = _cnf(l), _cnf(r)
    if kind == "and":
        return lc + rc
    out = []
    for a in lc:
        for b in rc:
            out.append(a + b)
            if len(out) > 64:
                raise Unsupported("CNF blow-up")
    return out


def to_cnf(conds: List[E.Expression]) -> List[List[Leaf]]:
    clauses: List[List[Leaf]] = []
    for c in conds:
        clauses.extend(_cnf(_to_nnf(c)))
    # drop clauses that are trivially true, fail on trivially false
    out = []
    for cl in clauses:
        if any(l.kind == "const" and l.value for l in cl):
            continue
        cl = [l for l in cl if l.kind != "const"]
        out.append(cl)
    return out


# ------------------------------------------------------------------------------------------------
# Binding leaves to column slots
# ------------------------------------------------------------------------------------------------
class ColumnInfo:
    """What the compiler needs to know about a bound column."""

    def __init__(self, slot: int, hs_type: int, atype: pa.DataType, dictionary=None):
        self.slot = slot
        self.hs_type = hs_type
        self.atype = atype
        self.dictionary = dictionary

    @property
    def is_float(self):
        return self.hs_type in (NL.F32, NL.F64)


class Bound:
    """Kernel-ready predicates plus keep-alive buffers (IN sets).  ``lits``: for every
    predicate whose literal came from a Literal node, (predicate index, Literal, column type,
    float?) - what ``rebind`` rewrites for a new literal vector; ``rebindable`` is False when a
    predicate's shape depends on its value (dictionary codes, IN sets, string dates, NULLs)."""

    def __init__(self):
        self.preds: List[NL.Pred] = []
        self.buffers: list = []
        self.always_false = False
        self.lits: list = []
        self.rebindable = True


def _dict_code_bound(info: ColumnInfo, op: int, v: str) -> Tuple[str, int, int]:
    """Translate ``col <op> 'v'`` on a sorted-dictionary column into an int predicate."""
    d = info.dictionary.to_pylist()
    lo = bisect.bisect_left(d, v)
    present = lo < len(d) and d[lo] == v
    if op in (NL.OP_EQ, NL.OP_NE):
        if not present:
            return ("false", 0, 0) if op == NL.OP_EQ else ("notnull", 0, 0)
        return ("int", op, lo)
    if op == NL.OP_LT:
        return ("int", NL.OP_LT, lo)
    if op == NL.OP_GE:
        return ("int", NL.OP_GE, lo)
    hi = bisect.bisect_right(d, v)
    if op == NL.OP_LE:
        return ("int", NL.OP_LT, hi)
    return ("int", NL.OP_GE, hi)  # GT


def bind(clauses: List[List[Leaf]], col_info: Callable[[E.Attribute], ColumnInfo], device,
         group_start: int = 0) -> Bound:
    import torch
    b = Bound()
    group = group_start
    for cl in clauses:
        if not cl:
            b.always_false = True
            continue
        emitted = 0
        for leaf in cl:
            info = col_info(leaf.attr) if leaf.attr is not None else None
            if leaf.kind == "isnull":
                b.preds.append(NL.Pred(NL.PK_IS_NULL, 0, info.slot, 0, group, 0, 0, 0.0, None))
            elif leaf.kind == "notnull":
                b.preds.append(NL.Pred(NL.PK_NOT_NULL, 0, info.slot, 0, group, 0, 0, 0.0, None))
            elif leaf.kind == "cmp_col":
                info2 = col_info(leaf.attr2)
                if info.dictionary is not None or info2.dictionary is not None:
                    raise Unsupported("column compare on strings")
                kind = NL.PK_FLT_COL if (info.is_float or info2.is_float) else NL.PK_INT_COL
                b.preds.append(NL.Pred(kind, leaf.op, info.slot, info2.slot, group, 0, 0, 0.0, None))
            elif leaf.kind == "cmp_lit":
                v = leaf.value
                if v is None:
                    b.rebindable = False
                    continue  # comparison with NULL is never true
                if info.dictionary is not None or isinstance(v, str) or leaf.lit is None:
                    b.rebindable = False
                else:
                    b.lits.append((len(b.preds), leaf.lit, leaf.attr.data_type,
                                   bool(info.is_float or isinstance(v, float))))
                if info.dictionary is not None:
                    if not isinstance(v, str):
                        raise Unsupported("non-string literal vs string column")
                    what, op, code = _dict_code_bound(info, leaf.op, v)
                    if what == "false":
                        continue
                    if what == "notnull":
                        b.preds.append(NL.Pred(NL.PK_NOT_NULL, 0, info.slot, 0, group, 0, 0, 0.0, None))
                    else:
                        b.preds.append(NL.Pred(NL.PK_INT_LIT, op, info.slot, 0, group, 0, int(code),
                                               0.0, None))
                elif isinstance(v, str):
                    if pa.types.is_date32(info.atype):
                        v = (datetime.date.fromisoformat(v[:10]) - datetime.date(1970, 1, 1)).days
                    else:
                        raise Unsupported("string literal vs non-string column")
                    b.preds.append(NL.Pred(NL.PK_INT_LIT, leaf.op, info.slot, 0, group, 0, int(v), 0.0, None))
                elif info.is_float or isinstance(v, float):
                    b.preds.append(NL.Pred(NL.PK_FLT_LIT, leaf.op, info.slot, 0, group, 0, 0,
                                           float(v), None))
                else:
                    b.preds.append(NL.Pred(NL.PK_INT_LIT, leaf.op, info.slot, 0, group, 0, int(v), 0.0, None))
            elif leaf.kind == "bitmap":
                b.rebindable = False
                kb = leaf.value
                if info.dictionary is not None or info.is_float:
                    raise Unsupported("key bitmap on a non-integer column")
                b.buffers.append(kb.words)
                b.preds.append(NL.Pred(NL.PK_BITMAP, leaf.op, info.slot, 0, group,
                                       kb.words.numel(), kb.base, 0.0, kb.words.data_ptr()))
            elif leaf.kind == "in":
                b.rebindable = False
                vals = [v for v in leaf.values if v is not None]
                if info.dictionary is not None:
                    d = {s: i for i, s in enumerate(info.dictionary.to_pylist())}
                    ivals = sorted({d[v] for v in vals if v in d})
                elif info.is_float:
                    if len(vals) > 8:
                        raise Unsupported("large float IN")
                    for v in vals:
                        b.preds.append(NL.Pred(NL.PK_FLT_LIT, NL.OP_EQ if leaf.op == NL.OP_EQ else NL.OP_NE,
                                               info.slot, 0, group if leaf.op == NL.OP_EQ else group,
                                               0, 0, float(v), None))
                    if leaf.op == NL.OP_NE:
                        raise Unsupported("NOT IN over floats")
                    emitted += 1
                    continue
                else:
                    ivals = sorted({int(v) for v in vals})
                if not ivals:
                    if leaf.op == NL.OP_EQ:
                        continue
                    b.preds.append(NL.Pred(NL.PK_NOT_NULL, 0, info.slot, 0, group, 0, 0, 0.0, None))
                else:
                    buf = torch.tensor(ivals, dtype=torch.int64, device=device)
                    b.buffers.append(buf)
                    b.preds.append(NL.Pred(NL.PK_IN_SET, leaf.op, info.slot, 0, group, len(ivals), 0,
                                           0.0, buf.data_ptr()))
            else:
                raise Unsupported(leaf.kind)
            emitted += 1
        if emitted == 0:
            b.always_false = True
        group += 1
    if len(b.preds) > NL.MAX_PREDS:
        raise Unsupported("too many predicates")
    return b


def rebind(b: Bound) -> Optional[Bound]:
    """``b`` (a bound predicate list of a prepared lowering) with every literal predicate's
    value re-read from its Literal node - a plan-cache hit writes the new query's values into
    the cached plan's Literal nodes - so a new literal vector skips the CNF conversion and
    column binding; None when the new values could change the predicates' shape (a NULL, a
    type change) or ``b`` is not rebindable (the full ``bind`` runs instead)."""
    if not b.rebindable or b.always_false:
        return None
    out = Bound()
    out.preds = [NL.Pred.from_buffer_copy(p) for p in b.preds]
    out.buffers = b.buffers
    out.lits = b.lits
    for i, lit, dtype, flt in b.lits:
        v = lit.value
        if v is None or isinstance(v, (str, bool)):
            return None
        v = _lit_value(v, dtype)
        p = out.preds[i]
        if flt:
            p.flit = float(v)
        else:
            if isinstance(v, float) and not v.is_integer():
                return None
            p.ilit = int(v)
    return out


# ------------------------------------------------------------------------------------------------
# Aggregate values
# ------------------------------------------------------------------------------------------------
def affine_terms(e: E.Expression) -> Tuple[float, List[Tuple[float, float, E.Attribute]]]:
    """e == scale * prod(alpha_i + beta_i * attr_i)."""
    if isinstance(e, E.Cast):
        return affine_terms(e.child)
    if isinstance(e, E.Alias):
        return affine_terms(e.child)
    if isinstance(e, E.Attribute):
        return 1.0, [(0.0, 1.0, e)]
    if isinstance(e, E.Literal) and isinstance(e.value, (int, float)) and not isinstance(e.value, bool):
        return float(e.value), []
    if isinstance(e, E.Multiply):
        s1, t1 = affine_terms(e.left)
        s2, t2 = affine_terms(e.right)
        return s1 * s2, t1 + t2
    if isinstance(e, E.Divide) and isinstance(e.right, E.Literal):
        s1, t1 = affine_terms(e.left)
        return s1 / float(e.right.value), t1
    if isinstance(e, (E.Add, E.Subtract)):
        sign = 1.0 if isinstance(e, E.Add) else -1.0
        l, r = e.left, e.right
        if isinstance(l, E.Literal) and not isinstance(r, E.Literal):
            s, t = affine_terms(r)
            if len(t) != 1:
                raise Unsupported("affine over product")
            a, b, attr = t[0]
            return 1.0, [(float(l.value) + sign * s * a, sign * s * b, attr)]
        if isinstance(r, E.Literal) and not isinstance(l, E.Literal):
            s, t = affine_terms(l)
            if len(t) != 1:
                raise Unsupported("affine over product")
            a, b, attr = t[0]
            return 1.0, [(s * a + sign * float(r.value), s * b, attr)]
    raise Unsupported(f"aggregate input {e.sql()}")


def agg_spec(fn: E.AggregateFunction, slot_of: Callable[[E.Attribute], int]) -> NL.AggSpec:
    a = NL.AggSpec()
    if isinstance(fn, E.Count):
        if fn.child is None or isinstance(fn.child, E.Literal):
            a.kind, a.nterms = NL.AK_COUNT_STAR, 0
            return a
        if not isinstance(fn.child, E.Attribute):
            raise Unsupported("count(expr)")
        a.kind, a.nterms = NL.AK_COUNT, 1
        a.col[0], a.alpha[0], a.beta[0] = slot_of(fn.child), 0.0, 1.0
        return a
    kind = {E.Sum: NL.AK_SUM, E.Min: NL.AK_MIN, E.Max: NL.AK_MAX, E.Avg: NL.AK_SUM}.get(type(fn))
    if kind is None:
        raise Unsupported(type(fn).__name__)
    scale, terms = affine_terms(fn.child)
    if not terms:
        raise Unsupported("constant aggregate")
    if len(terms) > NL.MAX_TERMS:
        raise Unsupported("too many terms")
    if kind in (NL.AK_MIN, NL.AK_MAX) and scale < 0:
        kind = NL.AK_MAX if kind == NL.AK_MIN else NL.AK_MIN
    a.kind, a.nterms = kind, len(terms)
    for i, (al, be, attr) in enumerate(terms):
        if i == 0:
            al, be = al * scale, be * scale
        a.col[i], a.alpha[i], a.beta[i] = slot_of(attr), al, be
    return a


def int_result(fn: E.AggregateFunction) -> bool:
    if isinstance(fn, E.Count):
        return True
    if isinstance(fn, (E.Sum, E.Min, E.Max)):
        t = fn.child.data_type
        return pa.types.is_integer(t)
    return False


def finalize_value(fn: E.AggregateFunction, s: float, c: int, mn: float, mx: float, c2: int = None):
    if isinstance(fn, E.Count):
        return int(c)
    if c == 0:
        return None
    if isinstance(fn, E.Avg):
        return s / c
    v = s if isinstance(fn, E.Sum) else (mn if isinstance(fn, E.Min) else mx)
    if int_result(fn):
        return int(round(v))
    t = fn.child.data_type
    if isinstance(fn, (E.Min, E.Max)) and pa.types.is_date32(t):
        return datetime.date(1970, 1, 1) + datetime.timedelta(days=int(v))
    if isinstance(fn, (E.Min, E.Max)) and _int_coded(t):
        # timestamps / times / durations / date64 aggregate as their int64 counts
        return pa.array([int(round(v))], pa.int64()).cast(t)[0].as_py()
    if isinstance(fn, (E.Min, E.Max)) and pa.types.is_decimal(t):
        import decimal
        return decimal.Decimal(int(round(v * 10 ** t.scale))).scaleb(-t.scale)
    return float(v)


def _int_coded(t: pa.DataType) -> bool:
    """Arrow types stored as int64 counts of a unit (besides plain integers)."""
    return (pa.types.is_timestamp(t) or pa.types.is_date64(t) or pa.types.is_time(t) or
            pa.types.is_duration(t))


__all__ = ["Unsupported", "to_cnf", "bind", "ColumnInfo", "agg_spec", "finalize_value",
           "affine_terms", "np"]
