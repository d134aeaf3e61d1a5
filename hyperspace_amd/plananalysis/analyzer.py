"""``explain``: physical plans with and without indexes, highlighted diff, used indexes and
operator statistics (reference ``plananalysis/PlanAnalyzer.scala:35-412``,
``PhysicalOperatorAnalyzer.scala:22-58``).

Plans are flattened pre-order and walked in lock step; scan nodes are equal iff their root paths
match, other nodes iff their operator class matches; the first differing subtree on each side is
highlighted.  Nothing is executed.
"""
from __future__ import annotations

from collections import Counter
from typing import List

import pyarrow as pa

from ..plan import physical as X
from ..utils import path_utils as P
from .display import BufferStream, get_display_mode

SEP = "============================================================="


class _PlanContext:
    def __init__(self, plan: X.SparkPlan, mode):
        self.plan = plan
        self.lines = plan.tree_lines()   # [(prefix, node)]
        self.pos = 0
        self.stream = BufferStream(mode)

    def non_empty(self):
        return self.pos < len(self.lines)

    @property
    def cur(self):
        return self.lines[self.pos][1]

    def _depth(self, i):
        return len(self.lines[i][0])

    def move_next(self, writer):
        prefix, node = self.lines[self.pos]
        writer(self.stream, prefix, node)
        self.pos += 1

    def move_next_subtree(self, writer):
        start_depth = self._depth(self.pos)
        self.move_next(writer)
        while self.pos < len(self.lines) and self._depth(self.pos) > start_depth:
            self.move_next(writer)

    def text(self):
        return str(self.stream)


def _are_equal(a: X.SparkPlan, b: X.SparkPlan) -> bool:
    if isinstance(a, X.FileSourceScanExec) and isinstance(b, X.FileSourceScanExec):
        return a.relation.location.root_paths == b.relation.location.root_paths
    return type(a) is type(b)


def _with_hyperspace_state(session, enabled: bool, fn):
    was = session.isHyperspaceEnabled()
    try:
        if enabled:
            session.enableHyperspace()
        else:
            session.disableHyperspace()
        return fn()
    finally:
        if was:
            session.enableHyperspace()
        else:
            session.disableHyperspace()


def _executed_plan(session, df, enabled: bool) -> X.SparkPlan:
    from ..plan.execution import QueryExecution
    return _with_hyperspace_state(session, enabled,
                                  lambda: QueryExecution(session, df.plan).executed_plan)


def physical_operator_stats(plan: X.SparkPlan) -> Counter:
    c = Counter()
    for p in plan.iter_pre():
        c[p.node_name] += 1
    return c


def explain_string(df, session, indexes_df, verbose: bool) -> str:
    mode = get_display_mode(session.conf)
    with_ctx = _PlanContext(_executed_plan(session, df, True), mode)
    without_ctx = _PlanContext(_executed_plan(session, df, False), mode)

    def plain(stream, prefix, node):
        stream.write_line(prefix + node.simple_string())

    def hl(stream, prefix, node):
        # highlight only the node text; keep the tree prefix plain (PlanAnalyzer moveNextSubtree)
        stream.write(prefix).highlight(node.simple_string()).write_line()

    while with_ctx.non_empty() and without_ctx.non_empty():
        if not _are_equal(with_ctx.cur, without_ctx.cur):
            with_ctx.move_next_subtree(hl)
            without_ctx.move_next_subtree(hl)
        else:
            with_ctx.move_next(plain)
            without_ctx.move_next(plain)
    while with_ctx.non_empty():
        with_ctx.move_next(hl)
    while without_ctx.non_empty():
        without_ctx.move_next(hl)

    out = BufferStream(mode)

    def header(title):
        out.write_line(SEP).write_line(title).write_line(SEP)

    header("Plan with indexes:")
    out.write_line(with_ctx.text())
    header("Plan without indexes:")
    out.write_line(without_ctx.text())
    header("Indexes used:")
    _write_used_indexes(with_ctx.plan, indexes_df, out)
    out.write_line()
    if verbose:
        header("Physical operator stats:")
        _write_stats(with_ctx.plan, without_ctx.plan, out)
        out.write_line()
    return out.with_tag()


def _write_used_indexes(plan, indexes_df, out):
    paths = set()
    for p in plan.iter_pre():
        if isinstance(p, X.FileSourceScanExec):
            for r in p.relation.location.root_paths:
                paths.add(P.get_parent(r))
                paths.add(r)
    t: pa.Table = indexes_df.to_arrow()
    for name, loc in zip(t.column("name").to_pylist(), t.column("indexLocation").to_pylist()):
        if loc in paths or any(x.startswith(loc.rstrip("/") + "/") for x in paths):
            out.write_line(f"{name}:{loc}")


def _write_stats(with_plan, without_plan, out):
    a = physical_operator_stats(without_plan)
    b = physical_operator_stats(with_plan)
    names = sorted(set(a) | set(b))
    rows = [(n, str(a.get(n, 0)), str(b.get(n, 0)), str(b.get(n, 0) - a.get(n, 0))) for n in names]
    header = ("Physical Operator", "Hyperspace Disabled", "Hyperspace Enabled", "Difference")
    widths = [max(len(header[i]), *(len(r[i]) for r in rows)) if rows else len(header[i])
              for i in range(4)]
    sep = "+" + "+".join("-" * w for w in widths) + "+"
    out.write_line(sep)
    out.write_line("|" + "|".join(h.rjust(w) for h, w in zip(header, widths)) + "|")
    out.write_line(sep)
    for r in rows:
        out.write_line("|" + "|".join(v.rjust(w) for v, w in zip(r, widths)) + "|")
    out.write_line(sep)
