"""Computed projections on the device: ``select(a * 2 + b)``, ``select((x > 0) & (y < 5))``.

FilterIndexRule rewrites ``Project(Filter(Relation))`` with an arbitrary project list
(FilterIndexRule.scala:155-191); the reference leaves the expressions to Spark's executors.
Here every computed column of a projection is evaluated by ONE generated elementwise kernel
(hipRTC, ``exec/jit.py``) over the relation's rows: column loads, the expression trees with
Spark's semantics, and one store per output column.  The kernel is cached per expression
*shape* (operators, input types, nullability); literals are kernel arguments, so a new literal
reuses the compiled kernel.

Semantics (Spark non-ANSI, and the host oracle ``exec/arrow_eval.py``):

* arithmetic on integers wraps at the result width; a mixed integer / floating (or decimal)
  operation runs in double;
* ``/`` is a double division; a zero divisor gives NULL;
* casts between numeric types truncate toward zero (integer targets) and wrap;
* comparisons give booleans; AND / OR / NOT follow three-valued (Kleene) logic;
* NULL in, NULL out for everything else.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import pyarrow as pa

from ..ops import _lib as NL
from ..plan import expressions as E
from . import jit
from .compile import Unsupported
from .device_table import DeviceColumn

BLOCK = 256

_CTYPE = {NL.I8: "signed char", NL.I16: "short", NL.I32: "int", NL.I64: "long long",
          NL.F32: "float", NL.F64: "double", NL.BOOL: "unsigned char", NL.U32: "unsigned"}
_CMP = {E.EqualTo: "==", E.NotEqual: "!=", E.LessThan: "<", E.LessThanOrEqual: "<=",
        E.GreaterThan: ">", E.GreaterThanOrEqual: ">="}
_ARITH = {E.Add: "+", E.Subtract: "-", E.Multiply: "*"}


def _kind(t: pa.DataType) -> str:
    """'i' integral, 'f' double (floating / decimal), 'b' boolean; else unsupported."""
    if pa.types.is_boolean(t):
        return "b"
    if pa.types.is_integer(t):
        return "i"
    if pa.types.is_floating(t) or pa.types.is_decimal(t):
        return "f"
    raise Unsupported(f"computed projection over {t}")


def _out_storage(t: pa.DataType):
    import torch
    if pa.types.is_boolean(t):
        return torch.uint8, "unsigned char"
    if pa.types.is_integer(t):
        bw = t.bit_width
        return ({8: torch.int8, 16: torch.int16, 32: torch.int32, 64: torch.int64}[bw],
                {8: "signed char", 16: "short", 32: "int", 64: "long long"}[bw])
    if pa.types.is_float32(t):
        return torch.float32, "float"
    return torch.float64, "double"


class _Gen:
    """Expression -> C statements over row ``i``; every node yields (value var, valid var)."""

    def __init__(self, cols: Dict[int, DeviceColumn]):
        self.cols = cols            # expr_id -> device column
        self.slot: Dict[int, int] = {}
        self.args = jit.Args()
        self.lines: List[str] = []
        self.values: Dict[str, object] = {}
        self.shape: List[object] = []
        self.n = 0

    def _var(self) -> str:
        self.n += 1
        return f"t{self.n}"

    def attr(self, a: E.Attribute) -> Tuple[str, str, str]:
        c = self.cols.get(a.expr_id)
        if c is None:
            raise Unsupported(f"attribute {a.sql()} not on device")
        if c.dictionary is not None:
            raise Unsupported("computed projection over a string column")
        k = _kind(c.atype)
        s = self.slot.get(a.expr_id)
        if s is None:
            s = self.slot[a.expr_id] = len(self.slot)
            self.args.add("p", f"c{s}", f"const {_CTYPE[c.hs_type]}*")
            self.args.add("p", f"v{s}", "const unsigned char*")
            self.values[f"c{s}"] = c.data.data_ptr()
            self.values[f"v{s}"] = c.valid.data_ptr() if c.valid is not None else 0
            self.shape.append(("col", s, c.hs_type, c.valid is not None))
        v, ok = self._var(), self._var()
        ct = "double" if k == "f" else ("bool" if k == "b" else "long long")
        self.lines.append(f"const {ct} {v} = ({ct})a.c{s}[i];")
        self.lines.append(f"const bool {ok} = !a.v{s} || a.v{s}[i];" if c.valid is not None
                          else f"const bool {ok} = true;")
        return v, ok, k

    def lit(self, e: E.Literal) -> Tuple[str, str, str]:
        v, ok = self._var(), self._var()
        if e.value is None:
            self.shape.append(("null",))
            self.lines.append(f"const long long {v} = 0; const bool {ok} = false;")
            return v, ok, "i"
        val = e.value
        if isinstance(val, bool):
            k = "b"
        elif isinstance(val, int):
            k = "i"
        elif isinstance(val, float) or hasattr(val, "as_tuple"):
            k = "f"
        else:
            raise Unsupported(f"literal {val!r} in a computed projection")
        name = f"l{len(self.values)}"
        if k == "f":
            self.args.add("d", name, "double")
            self.values[name] = float(val)
            self.lines.append(f"const double {v} = a.{name};")
        else:
            self.args.add("q", name, "long long")
            self.values[name] = int(val)
            ct = "bool" if k == "b" else "long long"
            self.lines.append(f"const {ct} {v} = ({ct})a.{name};")
        self.shape.append(("lit", k))
        self.lines.append(f"const bool {ok} = true;")
        return v, ok, k

    def emit(self, e: E.Expression) -> Tuple[str, str, str]:
        if isinstance(e, E.Alias):
            return self.emit(e.child)
        if isinstance(e, E.Attribute):
            return self.attr(e)
        if isinstance(e, E.Literal):
            return self.lit(e)
        self.shape.append(type(e).__name__)
        if type(e) in _ARITH or isinstance(e, (E.Divide, E.Remainder)) or type(e) in _CMP:
            (a, av, ak), (b, bv, bk) = self.emit(e.left), self.emit(e.right)
            if "b" in (ak, bk):
                raise Unsupported("arithmetic / comparison on booleans")
            v, ok = self._var(), self._var()
            f = "f" in (ak, bk)
            if isinstance(e, E.Remainder):
                # Spark: sign of the dividend, NULL for a zero divisor; x % -1 = 0 (no trap on
                # LLONG_MIN % -1)
                if f:
                    self.lines.append(f"const bool {ok} = {av} && {bv} && (double){b} != 0.0;")
                    self.lines.append(f"const double {v} = {ok} ? fmod((double){a}, (double){b})"
                                      f" : 0.0;")
                    return v, ok, "f"
                self.lines.append(f"const bool {ok} = {av} && {bv} && (long long){b} != 0;")
                self.lines.append(f"const long long {v} = (!{ok} || (long long){b} == -1) ? 0 : "
                                  f"(long long){a} % (long long){b};")
                return v, ok, "i"
            if isinstance(e, E.Divide):
                self.lines.append(f"const bool {ok} = {av} && {bv} && (double){b} != 0.0;")
                self.lines.append(f"const double {v} = {ok} ? (double){a} / (double){b} : 0.0;")
                return v, ok, "f"
            self.lines.append(f"const bool {ok} = {av} && {bv};")
            if type(e) in _CMP:
                ct = "double" if f else "long long"
                self.lines.append(f"const bool {v} = ({ct}){a} {_CMP[type(e)]} ({ct}){b};")
                return v, ok, "b"
            op = _ARITH[type(e)]
            if f:
                self.lines.append(f"const double {v} = (double){a} {op} (double){b};")
                return v, ok, "f"
            # integers wrap: two's-complement arithmetic in unsigned 64 bits, narrowed at store
            self.lines.append(f"const long long {v} = (long long)((unsigned long long){a} {op} "
                              f"(unsigned long long){b});")
            return v, ok, "i"
        if isinstance(e, (E.And, E.Or)):
            (a, av, ak), (b, bv, bk) = self.emit(e.left), self.emit(e.right)
            if ak != "b" or bk != "b":
                raise Unsupported("AND / OR of non-booleans")
            v, ok = self._var(), self._var()
            if isinstance(e, E.And):
                # false wins over NULL
                self.lines.append(f"const bool {ok} = ({av} && {bv}) || ({av} && !{a}) || "
                                  f"({bv} && !{b});")
                self.lines.append(f"const bool {v} = {a} && {b} && {av} && {bv};")
            else:
                # true wins over NULL
                self.lines.append(f"const bool {ok} = ({av} && {bv}) || ({av} && {a}) || "
                                  f"({bv} && {b});")
                self.lines.append(f"const bool {v} = ({av} && {a}) || ({bv} && {b});")
            return v, ok, "b"
        if isinstance(e, E.Not):
            a, av, ak = self.emit(e.child)
            if ak != "b":
                raise Unsupported("NOT of a non-boolean")
            v = self._var()
            self.lines.append(f"const bool {v} = !{a};")
            return v, av, "b"
        if isinstance(e, (E.IsNull, E.IsNotNull)):
            a, av, _ = self.emit(e.child)
            v, ok = self._var(), self._var()
            self.lines.append(f"const bool {v} = {'!' if isinstance(e, E.IsNull) else ''}{av};")
            self.lines.append(f"const bool {ok} = true;")
            return v, ok, "b"
        if isinstance(e, E.Cast):
            a, av, ak = self.emit(e.child)
            tk = _kind(e.dtype)
            self.shape.append(str(e.dtype))
            v = self._var()
            if tk == "f":
                self.lines.append(f"const double {v} = (double){a};")
            elif tk == "b":
                self.lines.append(f"const bool {v} = {a} != 0;")
            elif ak == "f" and pa.types.is_int64(e.dtype):
                # truncation toward zero; NaN / out of range saturate like the JVM's d2l
                self.lines.append(f"const long long {v} = {a} != {a} ? 0LL : ({a} >= 9.2233720368547758e18 ? "
                                  f"0x7fffffffffffffffLL : ({a} <= -9.2233720368547758e18 ? "
                                  f"(-0x7fffffffffffffffLL - 1) : (long long){a}));")
            elif ak == "f":
                # Spark: d2i saturates to the int range (NaN -> 0); a short / byte target is
                # toInt then a wrapping narrow, which the store performs
                self.lines.append(f"const long long {v} = {a} != {a} ? 0LL : ({a} >= 2147483647.0 ? "
                                  f"2147483647LL : ({a} <= -2147483648.0 ? -2147483648LL : "
                                  f"(long long){a}));")
            else:
                self.lines.append(f"const long long {v} = (long long){a};")
            return v, av, tk
        raise Unsupported(f"computed projection of {type(e).__name__}")


def evaluate(exprs: List[E.Expression], cols: Dict[int, DeviceColumn], n: int,
             device) -> List[DeviceColumn]:
    """Device columns of ``exprs`` (over attributes in ``cols``: expr_id -> column of ``n``
    rows), all computed by one generated kernel launch."""
    k, values, outs = build(exprs, cols, n, device)
    if n:
        grid = max(1, min(4096, -(-n // BLOCK)))
        k.launch(grid, values, NL.stream_ptr(), 0)
    return outs


def build(exprs: List[E.Expression], cols: Dict[int, DeviceColumn], n: int, device):
    """(kernel, argument values, output columns) of ``evaluate`` without the launch."""
    import torch
    g = _Gen(cols)
    outs = []
    body: List[str] = []
    for j, e in enumerate(exprs):
        t = e.data_type
        if pa.types.is_integer(t) and e.data_type.bit_width > 64:
            raise Unsupported("wide integer result")
        v, ok, k = g.emit(e)
        tdt, ct = _out_storage(t)
        if (k == "b") != pa.types.is_boolean(t):
            raise Unsupported(f"result type {t} of {e.sql()}")
        data = torch.empty(n, dtype=tdt, device=device)
        valid = torch.empty(n, dtype=torch.uint8, device=device)
        g.args.add("p", f"o{j}", f"{ct}*")
        g.args.add("p", f"ov{j}", "unsigned char*")
        g.values[f"o{j}"] = data.data_ptr()
        g.values[f"ov{j}"] = valid.data_ptr()
        g.shape.append(("out", str(t)))
        g.lines.append(f"a.o{j}[i] = {v} ? ({ct}){v} : ({ct})0;" if k == "b" else
                       f"a.o{j}[i] = {ok} ? ({ct}){v} : ({ct})0;")
        g.lines.append(f"a.ov{j}[i] = {ok} ? 1 : 0;")
        outs.append((data, valid, t))
    g.args.add("q", "n", "long long")
    g.values["n"] = n
    body = ["  const long long stride = (long long)gridDim.x * blockDim.x;",
            "  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; "
            "i += stride) {"] + ["    " + x for x in g.lines] + ["  }"]
    shape = ("project", tuple(map(str, g.shape)), tuple(s for _, s, _ in g.args.slots))

    def make():
        src = (jit._PRELUDE + g.args.struct_src() +
               f'extern "C" __global__ __launch_bounds__({BLOCK}) void hs_jit_project(Args a) {{\n'
               + "\n".join(body) + "\n}\n")
        return jit.Kernel(src, "hs_jit_project", g.args, 0, BLOCK)
    k = jit.kernel_for(shape, make)
    return k, g.values, [DeviceColumn(data, valid, t) for data, valid, t in outs]


__all__ = ["evaluate"]
