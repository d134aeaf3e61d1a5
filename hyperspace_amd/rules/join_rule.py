"""JoinIndexRule (reference ``index/rules/JoinIndexRule.scala:52-534``).

Rewrites both sides of an equi-join to bucketed covering-index scans so the join needs no
shuffle.  Applicability: the condition is a conjunction of ``attr = attr``; each side is linear
with exactly one relation not yet index-modified; join attributes map one-to-one between sides.
A usable index has indexed-column *set* == the side's join keys and covers every required column;
a pair is compatible when indexed-column *order* agrees with the key mapping.  On MI355X the
rewritten join is a co-located per-bucket merge join with zero inter-GPU traffic (K8).
"""
from __future__ import annotations

import logging
from typing import Dict, List, Optional

from ..actions import states
from ..plan import expressions as E
from ..plan import logical as L
from ..telemetry.events import (AppInfo, HyperspaceIndexUsageEvent, NoOpEventLogger,
                                get_event_logger)
from ..utils.resolver import resolve, resolve_one
from . import rule_utils as RU
from .rankers import rank_join

log = logging.getLogger(__name__)


def _is_condition_supported(cond) -> bool:
    if isinstance(cond, E.EqualTo):
        return isinstance(cond.left, E.Attribute) and isinstance(cond.right, E.Attribute)
    if isinstance(cond, E.And):
        return _is_condition_supported(cond.left) and _is_condition_supported(cond.right)
    return False


def _extract_conditions(cond) -> list:
    if isinstance(cond, E.EqualTo) and isinstance(cond.left, E.Attribute) and \
            isinstance(cond.right, E.Attribute):
        return [cond]
    if isinstance(cond, E.And):
        return _extract_conditions(cond.left) + _extract_conditions(cond.right)
    raise RuntimeError("Unsupported condition found")


def _is_linear(plan) -> bool:
    return len(plan.children) <= 1 and all(_is_linear(c) for c in plan.children)


def _is_modified(plan) -> bool:
    return plan.find(lambda p: isinstance(p, L.LogicalRelation) and
                     RU.is_index_applied(p.relation)) is not None


def _relation_outputs(plan) -> List[E.Attribute]:
    return [a for leaf in plan.collect_leaves() if isinstance(leaf, L.LogicalRelation)
            for a in leaf.output]


def _ensure_attribute_requirements(l, r, cond) -> bool:
    lbase = {a.expr_id for a in _relation_outputs(l)}
    rbase = {a.expr_id for a in _relation_outputs(r)}
    amap: Dict[int, int] = {}
    for c in _extract_conditions(cond):
        c1, c2 = c.left.expr_id, c.right.expr_id
        if not ((c1 in lbase and c2 in rbase) or (c2 in lbase and c1 in rbase)):
            return False
        if c1 in amap and c2 in amap:
            if amap[c1] != c2 or amap[c2] != c1:
                return False
        elif c1 not in amap and c2 not in amap:
            amap[c1] = c2
            amap[c2] = c1
        else:
            return False
    return True


def _is_applicable(l, r, cond) -> bool:
    return _is_condition_supported(cond) and RU.get_logical_relation(l) is not None and \
        RU.get_logical_relation(r) is not None and _is_linear(l) and _is_linear(r) and \
        not _is_modified(l) and not _is_modified(r) and _ensure_attribute_requirements(l, r, cond)


def _all_required_cols(plan) -> List[str]:
    refs = []
    for p in plan.iter_pre():
        if isinstance(p, L.LogicalRelation):
            continue
        refs.extend(p.references())
    out, seen = [], set()
    for a in refs + list(plan.output):
        if a.name not in seen:
            seen.add(a.name)
            out.append(a.name)
    return out


def _lr_column_mapping(session, lbase, rbase, cond) -> Dict[str, str]:
    cs = session.case_sensitive
    out = {}
    for c in _extract_conditions(cond):
        a1 = resolve_one(c.left.name, lbase, cs)
        b1 = resolve_one(c.right.name, rbase, cs)
        if a1 is not None and b1 is not None:
            out[a1] = b1
            continue
        a2 = resolve_one(c.right.name, lbase, cs)
        b2 = resolve_one(c.left.name, rbase, cs)
        if a2 is None or b2 is None:
            raise RuntimeError("Unexpected exception while using join rule")
        out[a2] = b2
    return out


def _usable(indexes, required_indexed, required_all) -> list:
    return [i for i in indexes
            if set(required_indexed) == set(i.indexed_columns) and
            all(c in list(i.indexed_columns) + list(i.included_columns) for c in required_all)]


def _is_compatible(li, ri, mapping) -> bool:
    return list(ri.indexed_columns) == [mapping[c] for c in li.indexed_columns]


def get_best_index_pair(session, left, right, cond):
    from ..hyperspace import get_context
    all_idx = get_context(session).index_collection_manager.get_indexes([states.ACTIVE])
    lbase = [a.name for a in _relation_outputs(left)]
    rbase = [a.name for a in _relation_outputs(right)]
    mapping = _lr_column_mapping(session, lbase, rbase, cond)
    cs = session.case_sensitive
    l_req_all = resolve(_all_required_cols(left), lbase, cs)
    r_req_all = resolve(_all_required_cols(right), rbase, cs)
    if l_req_all is None or r_req_all is None:
        return None
    l_usable = _usable(all_idx, list(mapping.keys()), l_req_all)
    r_usable = _usable(all_idx, list(mapping.values()), r_req_all)
    lrel, rrel = RU.get_logical_relation(left), RU.get_logical_relation(right)
    l_idx = RU.get_candidate_indexes(session, l_usable, lrel)
    r_idx = RU.get_candidate_indexes(session, r_usable, rrel)
    pairs = [(li, ri) for li in l_idx for ri in r_idx if _is_compatible(li, ri, mapping)]
    if not pairs:
        return None
    return rank_join(session, lrel, rrel, pairs)[0]


def JoinIndexRule(session, plan):
    def fn(p):
        if not (isinstance(p, L.Join) and p.condition is not None and
                _is_applicable(p.left, p.right, p.condition)):
            return None
        try:
            pair = get_best_index_pair(session, p.left, p.right, p.condition)
            if pair is None:
                return None
            li, ri = pair
            updated = p.copy(left=RU.transform_plan_to_use_index(session, li, p.left, True),
                             right=RU.transform_plan_to_use_index(session, ri, p.right, True))
            logger = get_event_logger(session.conf)
            if not isinstance(logger, NoOpEventLogger):  # plan strings only when someone listens
                logger.log_event(HyperspaceIndexUsageEvent(
                    AppInfo(session.user, session.app_id, session.app_name), [li, ri],
                    p.tree_string(), updated.tree_string(), "Join index rule applied."))
            return updated
        except Exception as e:  # noqa: BLE001
            log.warning("Non fatal exception in running join index rule: %s", e)
            return None
    return plan.transform_up(fn)
