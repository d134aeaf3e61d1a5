"""SQL front-end: ``session.sql("SELECT ... FROM ... WHERE ...")`` over temporary views and
catalog tables (``hyperspace_amd/catalog.py``), planned into the same logical operators the
DataFrame API builds - so the Hyperspace rules rewrite SQL queries exactly like DataFrame ones.

Supported (the shapes the reference's tests and notebooks run through ``spark.sql``:
``E2EHyperspaceRulesTest.scala:230-341``, ``ExplainTest.scala:187,311``,
``python/hyperspace/tests/test_indexutilization.py:45-46``)::

    query   := select [UNION [ALL] select]*
    select  := SELECT [DISTINCT] item, ... FROM from [WHERE e] [GROUP BY e, ...] [HAVING e]
               [ORDER BY e [ASC|DESC], ...] [LIMIT n]
    item    := * | rel.* | e [[AS] alias]
    from    := ref [, ref | [INNER|CROSS|LEFT [OUTER]|RIGHT [OUTER]|FULL [OUTER]|LEFT SEMI|
               LEFT ANTI] JOIN ref [ON e]]*
    ref     := name [[AS] alias] | ( query ) [AS] alias

Expressions are ``plan/parser.py``'s grammar; ``rel.col`` resolves against the FROM scope (a
table's name or alias).  A comma join becomes an inner join on the WHERE conjuncts that link
the new relation to the ones before it (what Spark's ``ReorderJoin`` does for the same text);
the remaining conjuncts stay a filter, which the optimizer pushes down.
"""
from __future__ import annotations

import re
from typing import List, Optional, Tuple

from ..exceptions import HyperspaceException
from . import expressions as E
from . import logical as L
from .parser import _Parser, tokenize

_SQL_KW = {"SELECT", "FROM", "WHERE", "GROUP", "BY", "HAVING", "ORDER", "LIMIT", "AS", "JOIN",
           "INNER", "LEFT", "RIGHT", "FULL", "OUTER", "CROSS", "SEMI", "ANTI", "ON", "ASC",
           "DESC", "DISTINCT", "UNION", "ALL", "NULLS", "FIRST", "LAST"}


def _tokens(text: str):
    out = []
    for kind, t in tokenize(text):
        if kind == "id" and t.upper() in _SQL_KW:
            out.append(("kw", t.upper()))
        else:
            out.append((kind, t))
    return out


class _Scope:
    """The relations of a FROM clause: (qualifier, attributes) in order."""

    def __init__(self, case_sensitive: bool):
        self.rels: List[Tuple[Optional[str], List[E.Attribute]]] = []
        self.cs = case_sensitive

    def _eq(self, a: Optional[str], b: Optional[str]) -> bool:
        if a is None or b is None:
            return False
        return a == b if self.cs else a.lower() == b.lower()

    def add(self, qual: Optional[str], attrs) -> None:
        self.rels.append((qual, list(attrs)))

    def ids(self) -> set:
        return {a.expr_id for _, attrs in self.rels for a in attrs}

    def attrs(self) -> List[E.Attribute]:
        return [a for _, attrs in self.rels for a in attrs]

    def of(self, qual: str) -> List[E.Attribute]:
        for q, attrs in self.rels:
            if self._eq(q, qual):
                return attrs
        raise HyperspaceException(f"unknown relation '{qual}' in the FROM clause")

    def resolve(self, name: str) -> Optional[E.Attribute]:
        qual, _, col = name.rpartition(".")
        pool = self.of(qual) if qual else self.attrs()
        hits = {}
        for a in pool:
            if (a.name == col) if self.cs else (a.name.lower() == col.lower()):
                hits[a.expr_id] = a
        if len(hits) > 1:
            raise HyperspaceException(f"Reference '{name}' is ambiguous")
        return next(iter(hits.values())) if hits else None


class SqlPlanner(_Parser):
    def __init__(self, session, text: str):
        self.session = session
        self.toks = _tokens(text)
        self.i = 0

    # -- entry -------------------------------------------------------------------------------
    def plan(self) -> L.LogicalPlan:
        p = self.query()
        if self.peek()[0] != "eof":
            raise SyntaxError(f"unexpected token {self.peek()[1]!r}")
        return p

    def _union_ahead(self) -> bool:
        """Whether a UNION follows at this nesting level (before the closing parenthesis or
        the end): then a trailing ORDER BY / LIMIT belongs to the whole union, as in Spark."""
        depth = 0
        for kind, t in self.toks[self.i:]:
            if kind == "eof":
                return False
            if kind == "op" and t == "(":
                depth += 1
            elif kind == "op" and t == ")":
                if depth == 0:
                    return False
                depth -= 1
            elif depth == 0 and kind == "kw" and t == "UNION":
                return True
        return False

    def query(self) -> L.LogicalPlan:
        if not self._union_ahead():
            return self.select()
        p = self.select(tail=False)
        while self.accept("kw", "UNION"):
            all_ = self.accept("kw", "ALL")
            p = L.Union([p, self.select(tail=False)])
            if not all_:
                p = _distinct(p)
        orders, limit = self.order_limit()
        if orders:
            # names resolve against the union's output (the first branch's column names)
            scope = _Scope(self.session.case_sensitive)
            scope.add(None, p.output)
            p = L.Sort([L.SortOrder(self.resolve(e, scope), a) for e, a in orders], True, p)
        if limit is not None:
            p = L.Limit(limit, p)
        return p

    def order_limit(self):
        """A trailing ``ORDER BY ... [LIMIT n]``: ([(expression, ascending)], limit or None)."""
        orders = []
        if self.accept("kw", "ORDER"):
            self.expect("kw", "BY")
            orders = [self.order_item()]
            while self.accept("op", ","):
                orders.append(self.order_item())
        limit = None
        if self.accept("kw", "LIMIT"):
            kind, t = self.take()
            if kind != "num":
                raise SyntaxError("LIMIT needs a number")
            limit = int(t)
        return orders, limit

    # -- SELECT ------------------------------------------------------------------------------
    def select(self, tail: bool = True) -> L.LogicalPlan:
        """One SELECT; ``tail``: with its ORDER BY / LIMIT (False inside a UNION chain, whose
        trailing ORDER BY / LIMIT ``query`` applies to the whole union)."""
        if self.accept("op", "("):
            p = self.query()
            self.expect("op", ")")
            return p
        self.expect("kw", "SELECT")
        distinct = self.accept("kw", "DISTINCT")
        items = self.select_items()
        self.expect("kw", "FROM")
        scope = _Scope(self.session.case_sensitive)
        where_parts: List[E.Expression] = []
        plan = self.from_clause(scope, where_parts)
        if self.accept("kw", "WHERE"):
            where_parts.extend(E.split_conjuncts(self.resolve(self.or_expr(), scope)))
        plan = self.place_conjuncts(plan, scope, where_parts)
        grouping = []
        if self.accept("kw", "GROUP"):
            self.expect("kw", "BY")
            grouping = [self.or_expr()]
            while self.accept("op", ","):
                grouping.append(self.or_expr())
        having = None
        if self.accept("kw", "HAVING"):
            having = self.or_expr()
        orders, limit = self.order_limit() if tail else ([], None)
        plan = self.project(plan, scope, items, grouping, having, orders, distinct)
        if limit is not None:
            plan = L.Limit(limit, plan)
        return plan

    def select_items(self):
        items = [self.select_item()]
        while self.accept("op", ","):
            items.append(self.select_item())
        return items

    def select_item(self):
        if self.accept("op", "*"):
            return ("*", None)
        t = self.peek()
        if t[0] == "id" and t[1].endswith(".") and self.peek(1) == ("op", "*"):
            self.take()
            self.take()
            return ("rel*", t[1][:-1])
        e = self.or_expr()
        alias = None
        if self.accept("kw", "AS"):
            alias = self.take()[1]
        elif self.peek()[0] in ("id", "str") and not self.peek()[1].endswith("."):
            alias = self.take()[1]
            if alias[:1] in "'\"":
                alias = alias[1:-1]
        return ("expr", (e, alias))

    def order_item(self):
        e = self.or_expr()
        asc = True
        if self.accept("kw", "DESC"):
            asc = False
        else:
            self.accept("kw", "ASC")
        if self.accept("kw", "NULLS"):
            if self.accept("kw", "FIRST"):
                first = True
            elif self.accept("kw", "LAST"):
                first = False
            else:
                raise SyntaxError("NULLS FIRST | LAST")
            # SortOrder carries Spark's default null ordering only (ASC NULLS FIRST, DESC NULLS
            # LAST): an explicit other one must not be silently dropped
            if first != asc:
                raise HyperspaceException(
                    f"ORDER BY ... {'ASC' if asc else 'DESC'} NULLS {'FIRST' if first else 'LAST'}"
                    f" is not supported (only the default null ordering)")
        return e, asc

    # -- FROM --------------------------------------------------------------------------------
    def table_ref(self, scope: _Scope) -> L.LogicalPlan:
        if self.accept("op", "("):
            plan = self.query()
            self.expect("op", ")")
            alias = None
            if self.accept("kw", "AS") or self.peek()[0] == "id":
                kind, alias = self.take()
                if kind != "id":
                    raise SyntaxError(f"expected a subquery alias, got {alias!r}")
        else:
            kind, name = self.take()
            if kind != "id":
                raise SyntaxError(f"expected a table name, got {name!r}")
            plan = self.session.catalog.lookup(name).plan
            alias = name.rpartition(".")[2]
            if self.accept("kw", "AS"):
                alias = self.take()[1]
            elif self.peek()[0] == "id":
                alias = self.take()[1]
        ids = scope.ids()
        if ids & {a.expr_id for a in plan.output}:
            # the same view / table twice (a self join): fresh attribute ids for this instance
            from .dataframe import _dedup
            plan, _ = _dedup(plan, ids)
        scope.add(alias, plan.output)
        return plan

    def from_clause(self, scope: _Scope, where_parts) -> L.LogicalPlan:
        plan = self.table_ref(scope)
        while True:
            if self.accept("op", ","):
                right = self.table_ref(scope)
                plan = L.Join(plan, right, "cross", None)
                continue
            how = self.join_type()
            if how is None:
                return plan
            right = self.table_ref(scope)
            cond = None
            if self.accept("kw", "ON"):
                cond = self.resolve(self.or_expr(), scope)
            if how == "inner" and cond is None:
                how = "cross"
            plan = L.Join(plan, right, how, cond)

    def join_type(self) -> Optional[str]:
        if self.accept("kw", "JOIN"):
            return "inner"
        save = self.i
        how = None
        if self.accept("kw", "INNER"):
            how = "inner"
        elif self.accept("kw", "CROSS"):
            how = "cross"
        elif self.accept("kw", "LEFT"):
            how = "left"
            if self.accept("kw", "SEMI"):
                how = "leftsemi"
            elif self.accept("kw", "ANTI"):
                how = "leftanti"
            else:
                self.accept("kw", "OUTER")
        elif self.accept("kw", "RIGHT"):
            how = "right"
            self.accept("kw", "OUTER")
        elif self.accept("kw", "FULL"):
            how = "full"
            self.accept("kw", "OUTER")
        if how is None:
            return None
        if not self.accept("kw", "JOIN"):
            self.i = save
            return None
        return how

    def place_conjuncts(self, plan, scope, conds) -> L.LogicalPlan:
        """WHERE conjuncts over a join tree: each cross join takes the conjuncts linking its two
        sides as an inner-join condition (lowest join first), the rest filter on top."""
        left = list(conds)

        def walk(p):
            if not isinstance(p, L.Join):
                return p
            lp, rp = walk(p.children[0]), walk(p.children[1])
            if p.join_type != "cross":
                return L.Join(lp, rp, p.join_type, p.condition) \
                    if (lp is not p.children[0] or rp is not p.children[1]) else p
            lids = {a.expr_id for a in lp.output}
            rids = {a.expr_id for a in rp.output}
            take = []
            for c in list(left):
                refs = {a.expr_id for a in c.references()}
                if refs & lids and refs & rids and refs <= lids | rids:
                    take.append(c)
                    left.remove(c)
            if take:
                return L.Join(lp, rp, "inner", E.conjoin(take))
            return L.Join(lp, rp, "cross", None)
        plan = walk(plan)
        return L.Filter(E.conjoin(left), plan) if left else plan

    # -- projection / aggregation ------------------------------------------------------------
    def resolve(self, e: E.Expression, scope: _Scope, extra=None) -> E.Expression:
        def fn(x):
            if isinstance(x, E.UnresolvedAttribute):
                if extra is not None:
                    hit = extra(x.name)
                    if hit is not None:
                        return hit
                a = scope.resolve(x.name)
                if a is None:
                    raise HyperspaceException(
                        f"cannot resolve '{x.name}' given input columns: "
                        f"[{', '.join(b.name for b in scope.attrs())}]")
                return a
            return None
        return e.transform_up(fn)

    def project(self, plan, scope, items, grouping, having, orders, distinct) -> L.LogicalPlan:
        exprs: List[E.Expression] = []
        for kind, v in items:
            if kind == "*":
                exprs.extend(scope.attrs())
            elif kind == "rel*":
                exprs.extend(scope.of(v))
            else:
                e, alias = v
                e = self.resolve(e, scope)
                if alias is not None:
                    e = E.Alias(e, alias)
                elif not isinstance(e, (E.Attribute, E.Alias)):
                    e = E.Alias(e, re.sub(r"#\d+", "", e.sql()))
                exprs.append(e)
        aliases = {}
        for e in exprs:
            if isinstance(e, E.Alias):
                aliases.setdefault(e.name if self.session.case_sensitive else e.name.lower(), e)

        def alias_of(name):
            k = name if self.session.case_sensitive else name.lower()
            a = aliases.get(k)
            return a.to_attribute() if a is not None else None

        agg = bool(grouping) or any(E.contains_aggregate(e) for e in exprs) or \
            (having is not None)
        if agg:
            groups = []
            for g in grouping:
                g2 = self.resolve(g, scope, lambda n: (aliases[n.lower()].child
                                                       if scope.resolve(n) is None and
                                                       n.lower() in aliases else None))
                groups.append(g2)
            out = list(exprs)
            hidden: List[E.Alias] = []

            def lift(e):
                """An aggregate / input reference of HAVING or ORDER BY that is not an output
                column becomes a hidden output of the aggregate."""
                def fn(x):
                    if isinstance(x, E.AggregateFunction) or (
                            isinstance(x, E.Attribute) and
                            x.expr_id not in {o.expr_id for o in out + hidden
                                              if isinstance(o, (E.Attribute, E.Alias))}):
                        for o in out + hidden:
                            inner = o.child if isinstance(o, E.Alias) else o
                            if inner.semantic_equals(x):
                                return o.to_attribute() if isinstance(o, E.Alias) else o
                        h = E.Alias(x, f"_h{len(hidden)}")
                        hidden.append(h)
                        return h.to_attribute()
                    return None
                return _transform_down(e, fn)
            hav = None
            if having is not None:
                hav = lift(self.resolve(having, scope, alias_of))
            sort = [(lift(self.resolve(e, scope, alias_of)), asc) for e, asc in orders]
            plan = L.Aggregate(groups, out + hidden, plan)
            if hav is not None:
                plan = L.Filter(hav, plan)
            if sort:
                plan = L.Sort([L.SortOrder(e, a) for e, a in sort], True, plan)
            if hidden:
                plan = L.Project([e.to_attribute() if isinstance(e, E.Alias) else e
                                  for e in out], plan)
            return _distinct(plan) if distinct else plan
        proj = L.Project(exprs, plan)
        if distinct:
            proj = _distinct(proj)
        if not orders:
            return proj
        out_ids = {(e.to_attribute() if isinstance(e, E.Alias) else e).expr_id for e in exprs}
        sort = [(self.resolve(e, scope, alias_of), asc) for e, asc in orders]
        if all({a.expr_id for a in e.references()} <= out_ids for e, _ in sort):
            return L.Sort([L.SortOrder(e, a) for e, a in sort], True, proj)
        if distinct:
            raise HyperspaceException("ORDER BY of a column not in a SELECT DISTINCT list")
        # sort below the projection by the input columns (select aliases by their expressions)
        sub = {(e.to_attribute()).expr_id: e.child for e in exprs if isinstance(e, E.Alias)}

        def unalias(x):
            if isinstance(x, E.Attribute) and x.expr_id in sub:
                return sub[x.expr_id]
            return None
        below = L.Sort([L.SortOrder(e.transform_up(unalias), a) for e, a in sort], True, plan)
        return L.Project(exprs, below)


def _transform_down(e: E.Expression, fn) -> E.Expression:
    r = fn(e)
    if r is not None:
        return r
    if not e.children:
        return e
    new = tuple(_transform_down(c, fn) for c in e.children)
    if all(a is b for a, b in zip(new, e.children)):
        return e
    return e.with_children(new)


def _distinct(p: L.LogicalPlan) -> L.LogicalPlan:
    out = list(p.output)
    return L.Aggregate(out, out, p)


def sql(session, text: str):
    from .dataframe import DataFrame
    return DataFrame(session, SqlPlanner(session, text).plan())
