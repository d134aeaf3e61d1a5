"""FilterIndexRule (reference ``index/rules/FilterIndexRule.scala:38-191``).

Replaces the relation under ``Project(Filter(Relation))`` / ``Filter(Relation)`` with a covering
index whose first indexed column appears in the predicate and which covers every referenced
column.  The index is read *without* its bucket spec to keep scan parallelism (``:59-65``).
Any exception leaves the plan unchanged — an index must never break a query.
"""
from __future__ import annotations

import logging

from ..actions import states
from ..plan import logical as L
from ..telemetry.events import (AppInfo, HyperspaceIndexUsageEvent, NoOpEventLogger,
                                get_event_logger)
from ..utils.resolver import resolve, resolve_one
from . import rule_utils as RU
from .rankers import rank_filter

log = logging.getLogger(__name__)


def extract_filter_node(plan):
    """Returns (original, filter, output_cols, filter_cols, relation) or None."""
    if isinstance(plan, L.Project) and isinstance(plan.child, L.Filter) and \
            isinstance(plan.child.child, L.LogicalRelation) and \
            not RU.is_index_applied(plan.child.child.relation):
        f = plan.child
        out_cols = [a.name for e in plan.project_list for a in e.references()]
        filt_cols = [a.name for a in f.condition.references()]
        return plan, f, out_cols, filt_cols, f.child
    if isinstance(plan, L.Filter) and isinstance(plan.child, L.LogicalRelation) and \
            not RU.is_index_applied(plan.child.relation):
        return plan, plan, [a.name for a in plan.child.output], \
            [a.name for a in plan.condition.references()], plan.child
    return None


def index_covers_plan(session, out_cols, filt_cols, indexed, included) -> bool:
    cs = session.case_sensitive
    return resolve_one(indexed[0], filt_cols, cs) is not None and \
        resolve(out_cols + filt_cols, list(indexed) + list(included), cs) is not None


def find_covering_indexes(session, filt, out_cols, filt_cols) -> list:
    from ..hyperspace import get_context
    rel = RU.get_logical_relation(filt)
    if rel is None:
        return []
    all_idx = get_context(session).index_collection_manager.get_indexes([states.ACTIVE])
    cands = [i for i in all_idx
             if index_covers_plan(session, out_cols, filt_cols, i.indexed_columns, i.included_columns)]
    return RU.get_candidate_indexes(session, cands, rel)


def FilterIndexRule(session, plan):
    def fn(p):
        m = extract_filter_node(p)
        if m is None:
            return None
        original, filt, out_cols, filt_cols, _ = m
        try:
            cands = find_covering_indexes(session, filt, out_cols, filt_cols)
            index = rank_filter(session, filt, cands)
            if index is None:
                return None
            transformed = RU.transform_plan_to_use_index(session, index, original, False)
            logger = get_event_logger(session.conf)
            if not isinstance(logger, NoOpEventLogger):  # plan strings only when someone listens
                logger.log_event(HyperspaceIndexUsageEvent(
                    AppInfo(session.user, session.app_id, session.app_name), [index],
                    filt.tree_string(), transformed.tree_string(), "Filter index rule applied."))
            return _Done(transformed)
        except Exception as e:  # noqa: BLE001
            log.warning("Non fatal exception in running filter index rule: %s", e)
            return None
    return _undone(plan.transform_down(fn))


class _Done(L.LogicalPlan):
    """Wraps a rewritten subtree so transform_down does not revisit it."""

    def __init__(self, inner):
        self.inner = inner
        self.children = ()

    @property
    def output(self):
        return self.inner.output

    def with_children(self, children):
        return self


def _undone(plan):
    return plan.transform_up(lambda p: p.inner if isinstance(p, _Done) else None)
