"""Logical optimizer: the Catalyst rules that shape plans the way the Hyperspace rules expect
(Project(Filter(Relation)) under joins, inferred ``isnotnull`` filters, pruned join children),
followed by the session's extra optimizations (``spark.experimental.extraOptimizations``), which is
where ``JoinIndexRule`` and ``FilterIndexRule`` are registered (``package.scala:35-54``).
"""
from __future__ import annotations

from typing import List

from . import expressions as E
from . import logical as L

IN_SET_THRESHOLD_DEFAULT = 10


def _substitute(e: E.Expression, aliases: dict) -> E.Expression:
    def fn(x):
        if isinstance(x, E.Attribute) and x.expr_id in aliases:
            return aliases[x.expr_id]
        return None
    return e.transform_up(fn)


def _alias_map(project_list) -> dict:
    return {e.expr_id: e.child for e in project_list if isinstance(e, E.Alias)}


def _deterministic_project(p: L.Project) -> bool:
    return all(not E.contains_aggregate(e) for e in p.project_list)


# ---------------------------------------------------------------------------------------------
def combine_filters(plan):
    def fn(p):
        if isinstance(p, L.Filter) and isinstance(p.child, L.Filter):
            conds = E.split_conjuncts(p.child.condition)
            keys = {c.canonical_key() for c in conds}
            conds += [c for c in E.split_conjuncts(p.condition) if c.canonical_key() not in keys]
            return L.Filter(E.conjoin(conds), p.child.child)
        return None
    return plan.transform_up(fn)


def push_down_predicates(plan):
    def fn(p):
        if not isinstance(p, L.Filter):
            return None
        c = p.child
        if isinstance(c, L.Project) and _deterministic_project(c):
            cond = _substitute(p.condition, _alias_map(c.project_list))
            return L.Project(c.project_list, L.Filter(cond, c.child))
        if isinstance(c, L.Join) and c.join_type in ("inner", "cross"):
            lset, rset = c.left.output_set(), c.right.output_set()
            lp, rp, keep = [], [], []
            for cond in E.split_conjuncts(p.condition):
                refs = {a.expr_id for a in cond.references()}
                if refs and refs <= lset:
                    lp.append(cond)
                elif refs and refs <= rset:
                    rp.append(cond)
                else:
                    keep.append(cond)
            left = L.Filter(E.conjoin(lp), c.left) if lp else c.left
            right = L.Filter(E.conjoin(rp), c.right) if rp else c.right
            jcond = E.conjoin(([c.condition] if c.condition is not None else []) + keep)
            return L.Join(left, right, c.join_type, jcond)
        if isinstance(c, L.Union):
            return None
        return None
    return plan.transform_down(fn)


def push_join_condition(plan):
    """Move single-side conjuncts of an inner join condition into filters on that side."""
    def fn(p):
        if isinstance(p, L.Join) and p.join_type == "inner" and p.condition is not None:
            lset, rset = p.left.output_set(), p.right.output_set()
            lp, rp, keep = [], [], []
            for cond in E.split_conjuncts(p.condition):
                refs = {a.expr_id for a in cond.references()}
                if refs and refs <= lset:
                    lp.append(cond)
                elif refs and refs <= rset:
                    rp.append(cond)
                else:
                    keep.append(cond)
            if not lp and not rp:
                return None
            left = L.Filter(E.conjoin(lp), p.left) if lp else p.left
            right = L.Filter(E.conjoin(rp), p.right) if rp else p.right
            return L.Join(left, right, p.join_type, E.conjoin(keep))
        return None
    return plan.transform_up(fn)


def _null_intolerant_attrs(cond: E.Expression) -> List[E.Attribute]:
    out = []
    for c in E.split_conjuncts(cond):
        if isinstance(c, (E.BinaryComparison, E.In, E.InSet)):
            for a in c.references():
                out.append(a)
        elif isinstance(c, E.IsNotNull) and isinstance(c.child, E.Attribute):
            out.append(c.child)
    return out


def infer_filters(plan):
    """``InferFiltersFromConstraints``: add ``isnotnull(a)`` for null-intolerant predicates and
    inner equi-join keys (this is what puts ``Filter isnotnull(Col1#11)`` into join plans)."""
    def add_not_null(child: L.LogicalPlan, attrs: List[E.Attribute]) -> L.LogicalPlan:
        present = set()
        base = child
        existing = []
        if isinstance(child, L.Filter):
            existing = E.split_conjuncts(child.condition)
            base = child.child
            for c in existing:
                if isinstance(c, E.IsNotNull) and isinstance(c.child, E.Attribute):
                    present.add(c.child.expr_id)
        out_ids = child.output_set()
        new = []
        for a in attrs:
            if a.expr_id in out_ids and a.expr_id not in present and a.nullable:
                present.add(a.expr_id)
                new.append(E.IsNotNull(a))
        if not new:
            return child
        return L.Filter(E.conjoin(new + existing), base)

    def fn(p):
        if isinstance(p, L.Filter):
            attrs = [a for a in _null_intolerant_attrs(p.condition)]
            conds = E.split_conjuncts(p.condition)
            have = {c.child.expr_id for c in conds
                    if isinstance(c, E.IsNotNull) and isinstance(c.child, E.Attribute)}
            new = []
            for a in attrs:
                if a.expr_id not in have and a.nullable and a.expr_id in p.child.output_set():
                    have.add(a.expr_id)
                    new.append(E.IsNotNull(a))
            if new:
                return L.Filter(E.conjoin(new + conds), p.child)
            return None
        if isinstance(p, L.Join) and p.join_type in ("inner", "leftsemi") and p.condition is not None:
            keys = [a for c in E.split_conjuncts(p.condition) if isinstance(c, E.EqualTo)
                    for a in c.references()]
            left = add_not_null(p.left, keys)
            right = add_not_null(p.right, keys) if p.join_type == "inner" else p.right
            if left is not p.left or right is not p.right:
                return L.Join(left, right, p.join_type, p.condition)
        return None
    return plan.transform_up(fn)


def column_pruning(plan, required=None):
    """Top-down required-attribute propagation; inserts Projects under joins/aggregates."""
    if required is None:
        required = plan.output_set()
    if isinstance(plan, L.Project):
        need = {a.expr_id for e in plan.project_list for a in e.references()}
        return L.Project(plan.project_list, _prune_child(plan.child, need, wrap=False))
    if isinstance(plan, L.Filter):
        need = set(required) | {a.expr_id for a in plan.condition.references()}
        return L.Filter(plan.condition, column_pruning(plan.child, need))
    if isinstance(plan, L.Join):
        cond_refs = {a.expr_id for a in plan.condition.references()} if plan.condition else set()
        need = set(required) | cond_refs
        return L.Join(_prune_child(plan.left, need, wrap=True),
                      _prune_child(plan.right, need, wrap=True), plan.join_type, plan.condition)
    if isinstance(plan, L.Aggregate):
        need = {a.expr_id for e in plan.expressions() for a in e.references()}
        return L.Aggregate(plan.grouping, plan.aggregates, _prune_child(plan.child, need, wrap=True))
    if isinstance(plan, (L.Sort, L.Limit, L.RepartitionByExpression)):
        need = set(required) | {a.expr_id for e in plan.expressions() for a in e.references()}
        return plan.with_children((column_pruning(plan.child, need),))
    if isinstance(plan, (L.Union, L.BucketUnion)):
        return plan.with_children(tuple(column_pruning(c) for c in plan.children))
    return plan


def _prune_child(child, need: set, wrap: bool):
    out = child.output
    keep = [a for a in out if a.expr_id in need]
    if wrap and not keep and isinstance(child, L.Filter):
        # COUNT(*) over a filter needs no column of its own: keep one the filter reads anyway,
        # so the scan below narrows to the filter's columns (Spark's empty Project) and a
        # covering index over them qualifies (FilterIndexRule.scala:59-65)
        refs = {a.expr_id for a in child.condition.references()}
        keep = [a for a in out if a.expr_id in refs][:1]
    if isinstance(child, L.Project):
        plist = [e for e in child.project_list
                 if (e.expr_id if isinstance(e, (E.Attribute, E.Alias)) else None) in need]
        if not plist:
            plist = child.project_list[:1]
        inner_need = {a.expr_id for e in plist for a in e.references()}
        return L.Project(plist, _prune_child(child.child, inner_need, wrap=False))
    pruned = column_pruning(child, {a.expr_id for a in keep} if keep else {out[0].expr_id})
    if wrap and len(keep) < len(out) and keep:
        return L.Project(keep, pruned)
    return pruned


def collapse_project(plan):
    def fn(p):
        if isinstance(p, L.Project) and isinstance(p.child, L.Project):
            amap = _alias_map(p.child.project_list)
            new = []
            for e in p.project_list:
                ne = _substitute(e, amap)
                if isinstance(e, E.Attribute) and not isinstance(ne, E.Attribute):
                    ne = E.Alias(ne, e.name, e.expr_id)
                new.append(ne)
            return L.Project(new, p.child.child)
        return None
    return plan.transform_up(fn)


def remove_redundant_project(plan):
    def fn(p):
        if isinstance(p, L.Project) and all(isinstance(e, E.Attribute) for e in p.project_list):
            if [a.expr_id for a in p.project_list] == [a.expr_id for a in p.child.output]:
                return p.child
        return None
    return plan.transform_up(fn)


def optimize_in(plan, threshold: int = IN_SET_THRESHOLD_DEFAULT):
    def efn(x):
        if isinstance(x, E.In) and all(isinstance(v, E.Literal) for v in x.values):
            vals = []
            seen = set()
            for v in x.values:
                if v.value not in seen:
                    seen.add(v.value)
                    vals.append(v)
            if len(vals) > threshold:
                return E.InSet(x.value, frozenset(v.value for v in vals))
            if len(vals) < len(x.values):
                return E.In(x.value, vals)
        return None

    def fn(p):
        if isinstance(p, L.Filter):
            c2 = p.condition.transform_up(efn)
            return None if c2 is p.condition else L.Filter(c2, p.child)
        return None
    return plan.transform_up(fn)


def optimize_in_plan(plan):
    return optimize_in(plan)


class Optimizer:
    def __init__(self, session):
        self.session = session

    def base_batches(self, plan):
        from ..index import constants as C
        thr = int(self.session.conf.get(C.SQL_IN_SET_CONVERSION_THRESHOLD, "10"))
        # fixed point by identity: every rule returns the very same tree when it changes nothing
        for _ in range(10):
            before = plan
            plan = combine_filters(plan)
            plan = push_down_predicates(plan)
            plan = push_join_condition(plan)
            plan = combine_filters(plan)
            plan = collapse_project(plan)
            plan = remove_redundant_project(plan)
            plan = optimize_in(plan, thr)
            if plan is before:
                break
        plan = infer_filters(plan)
        plan = column_pruning(plan)
        plan = collapse_project(plan)
        plan = remove_redundant_project(plan)
        plan = combine_filters(plan)
        return plan

    def execute(self, plan, with_extra: bool = True):
        plan = self.base_batches(plan)
        if with_extra:
            for rule in list(self.session.extra_optimizations):
                plan = rule(self.session, plan)
        return plan
