"""Tiny SQL expression parser for ``df.filter("c3 == 'x' AND c1 > 5")`` style strings.

Grammar (precedence low->high): OR, AND, NOT, comparison / IN / BETWEEN / IS [NOT] NULL,
additive, multiplicative, unary minus, primary (literal, column, function call, parenthesised).
Produces expressions with ``UnresolvedAttribute`` leaves; the DataFrame resolves them.
"""
from __future__ import annotations

import datetime
import re

from . import expressions as E

_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<num>\d+\.\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?[LlDd]?)
  | (?P<str>'(?:[^'\\]|\\.|'')*'|"(?:[^"\\]|\\.)*")
  | (?P<bq>`[^`]+`)
  | (?P<op><=>|==|!=|<>|<=|>=|&&|\|\||[=<>+\-*/(),!%])
  | (?P<id>[A-Za-z_][A-Za-z0-9_.]*)
""", re.VERBOSE)

_KEYWORDS = {"AND", "OR", "NOT", "IN", "IS", "NULL", "TRUE", "FALSE", "BETWEEN", "DATE",
             "TIMESTAMP", "LIKE"}


def tokenize(s: str):
    pos, out = 0, []
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise SyntaxError(f"cannot parse expression at: {s[pos:]!r}")
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        text = m.group(kind)
        if kind == "id" and text.upper() in _KEYWORDS:
            out.append(("kw", text.upper()))
        elif kind == "bq":
            out.append(("id", text[1:-1]))
        else:
            out.append((kind, text))
    out.append(("eof", None))
    return out


class _Parser:
    def __init__(self, s: str):
        self.toks = tokenize(s)
        self.i = 0

    def peek(self, k=0):
        return self.toks[self.i + k]

    def take(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def accept(self, kind, text=None):
        t = self.peek()
        if t[0] == kind and (text is None or t[1] == text):
            self.i += 1
            return True
        return False

    def expect(self, kind, text=None):
        if not self.accept(kind, text):
            raise SyntaxError(f"expected {text or kind}, got {self.peek()[1]!r}")

    def parse(self):
        e = self.or_expr()
        if self.peek()[0] != "eof":
            raise SyntaxError(f"unexpected token {self.peek()[1]!r}")
        return e

    def or_expr(self):
        e = self.and_expr()
        while self.accept("kw", "OR") or self.accept("op", "||"):
            e = E.Or(e, self.and_expr())
        return e

    def and_expr(self):
        e = self.not_expr()
        while self.accept("kw", "AND") or self.accept("op", "&&"):
            e = E.And(e, self.not_expr())
        return e

    def not_expr(self):
        if self.accept("kw", "NOT") or self.accept("op", "!"):
            return E.Not(self.not_expr())
        return self.comparison()

    def comparison(self):
        left = self.additive()
        t = self.peek()
        if t[0] == "op" and t[1] in ("=", "==", "!=", "<>", "<", "<=", ">", ">=", "<=>"):
            self.take()
            right = self.additive()
            cls = {"=": E.EqualTo, "==": E.EqualTo, "<=>": E.EqualTo, "!=": E.NotEqual,
                   "<>": E.NotEqual, "<": E.LessThan, "<=": E.LessThanOrEqual,
                   ">": E.GreaterThan, ">=": E.GreaterThanOrEqual}[t[1]]
            return cls(left, right)
        negate = False
        if t == ("kw", "NOT") and self.peek(1)[1] in ("IN", "BETWEEN", "LIKE"):
            self.take()
            negate = True
        if self.accept("kw", "IN"):
            self.expect("op", "(")
            vals = [self.additive()]
            while self.accept("op", ","):
                vals.append(self.additive())
            self.expect("op", ")")
            e = E.In(left, vals)
            return E.Not(e) if negate else e
        if self.accept("kw", "BETWEEN"):
            lo = self.additive()
            self.expect("kw", "AND")
            hi = self.additive()
            e = E.And(E.GreaterThanOrEqual(left, lo), E.LessThanOrEqual(left, hi))
            return E.Not(e) if negate else e
        if self.accept("kw", "IS"):
            neg = self.accept("kw", "NOT")
            self.expect("kw", "NULL")
            return E.IsNotNull(left) if neg else E.IsNull(left)
        return left

    def additive(self):
        e = self.multiplicative()
        while True:
            if self.accept("op", "+"):
                e = E.Add(e, self.multiplicative())
            elif self.accept("op", "-"):
                e = E.Subtract(e, self.multiplicative())
            else:
                return e

    def multiplicative(self):
        e = self.unary()
        while True:
            if self.accept("op", "*"):
                e = E.Multiply(e, self.unary())
            elif self.accept("op", "/"):
                e = E.Divide(e, self.unary())
            elif self.accept("op", "%"):
                e = E.Remainder(e, self.unary())
            else:
                return e

    def unary(self):
        if self.accept("op", "-"):
            inner = self.unary()
            if isinstance(inner, E.Literal) and isinstance(inner.value, (int, float)):
                return E.Literal(-inner.value)
            return E.Subtract(E.Literal(0), inner)
        return self.primary()

    def primary(self):
        kind, text = self.take()
        if kind == "num":
            if text[-1] in "Ll":
                return E.Literal(int(text[:-1]), E.infer_literal_type(2 ** 40))
            if text[-1] in "Dd":
                return E.Literal(float(text[:-1]))
            if any(c in text for c in ".eE"):
                return E.Literal(float(text))
            return E.Literal(int(text))
        if kind == "str":
            body = text[1:-1].replace("''", "'")
            return E.Literal(bytes(body, "utf-8").decode("unicode_escape") if "\\" in body else body)
        if kind == "kw":
            if text == "NULL":
                return E.Literal(None)
            if text in ("TRUE", "FALSE"):
                return E.Literal(text == "TRUE")
            if text == "DATE":
                s = self.take()
                return E.Literal(datetime.date.fromisoformat(s[1][1:-1]))
            if text == "TIMESTAMP":
                s = self.take()
                return E.Literal(datetime.datetime.fromisoformat(s[1][1:-1]))
            raise SyntaxError(f"unexpected keyword {text}")
        if kind == "op" and text == "(":
            e = self.or_expr()
            self.expect("op", ")")
            return e
        if kind == "id":
            if self.peek() == ("op", "("):
                self.take()
                args = []
                if self.accept("op", "*"):
                    args = []
                elif not self.accept("op", ")"):
                    args.append(self.or_expr())
                    while self.accept("op", ","):
                        args.append(self.or_expr())
                    self.expect("op", ")")
                    return make_function(text, args)
                else:
                    return make_function(text, args)
                self.expect("op", ")")
                return make_function(text, args)
            return E.UnresolvedAttribute(text)
        raise SyntaxError(f"unexpected token {text!r}")


def make_function(name: str, args):
    n = name.lower()
    if n == "isnotnull":
        return E.IsNotNull(args[0])
    if n == "isnull":
        return E.IsNull(args[0])
    table = {"sum": E.Sum, "count": E.Count, "min": E.Min, "max": E.Max, "avg": E.Avg,
             "mean": E.Avg}
    if n in table:
        return table[n](args[0] if args else None)
    raise SyntaxError(f"unknown function {name}")


def parse_expression(s: str) -> E.Expression:
    return _Parser(s).parse()
