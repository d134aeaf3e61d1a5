"""QueryExecution: analyzed -> optimized -> physical -> executed plan, then run on a backend."""
from __future__ import annotations

import pyarrow as pa

from .optimizer import Optimizer
from .physical import Planner, ensure_requirements, reuse_exchanges


class QueryExecution:
    def __init__(self, session, logical):
        self.session = session
        self.logical = logical
        self._optimized = None
        self._spark_plan = None
        self._executed = None

    @property
    def analyzed(self):
        return self.logical

    @property
    def optimized_plan(self):
        if self._optimized is None:
            self._optimized = Optimizer(self.session).execute(self.logical)
        return self._optimized

    optimizedPlan = optimized_plan

    @property
    def spark_plan(self):
        if self._spark_plan is None:
            self._spark_plan = Planner(self.session).plan(self.optimized_plan)
        return self._spark_plan

    sparkPlan = spark_plan

    @property
    def executed_plan(self):
        if self._executed is None:
            from ..utils.conf import HyperspaceConf
            pc = None
            pend = getattr(self, "_pending_store", None)
            if pend is not None:        # _submit_bound already looked the query up: a miss
                pc, key, ctx = pend
                self._pending_store = None
            elif HyperspaceConf.plan_cache_enabled(self.session.conf):
                from .plan_cache import plan_cache
                pc = plan_cache(self.session)
                plan, key, ctx = pc.lookup(self.session, self.logical)
                if plan is not None:
                    if ctx.reuse:
                        plan = reuse_exchanges(plan, self.session)
                    self._executed = plan
                    return plan
            planned = ensure_requirements(self.spark_plan, self.session)
            self._executed = reuse_exchanges(planned, self.session)
            if pc is not None:
                pc.store(key, planned, ctx)
        return self._executed

    executedPlan = executed_plan

    def to_arrow(self) -> pa.Table:
        backend = self.session.backend()
        if self._executed is None and getattr(backend, "supports_bound_plans", False):
            # a plan-cache hit runs the cached plan with its literals bound in place, the same
            # path as ``to_arrow_async``: the executor's prepared lowerings (and captured graphs)
            # are keyed by the cached plan's nodes, which a materialized copy would not share
            fut = self._submit_bound(backend)
            if fut is not None:
                return fut.result()
        return backend.collect(self.executed_plan)

    def to_arrow_async(self):
        """Plan now, execute asynchronously: an object whose ``result()`` is the table.  The
        device backend returns before its kernels finish (``GpuBackend.collect_async``); the
        host backend runs the query here."""
        backend = self.session.backend()
        if self._executed is None and getattr(backend, "supports_bound_plans", False):
            fut = self._submit_bound(backend)
            if fut is not None:
                return fut
        plan = self.executed_plan
        if hasattr(backend, "collect_async"):
            return backend.collect_async(plan)
        return _Done(backend.collect(plan), getattr(backend, "last_path", "host"))

    def _submit_bound(self, backend):
        """Plan-cache hit fast path: submit the cached plan itself with this query's literal
        values bound into it for the duration of the submission (plan_cache._Entry).  None when
        the query is not a hit that allows it (then ``executed_plan`` plans / materializes)."""
        from ..utils.conf import HyperspaceConf
        if not HyperspaceConf.plan_cache_enabled(self.session.conf):
            return None
        from .plan_cache import plan_cache
        pc = plan_cache(self.session)
        entry, key, ctx = pc.lookup_entry(self.session, self.logical)
        if entry is None or ctx.reuse or not entry.inplace_ok:
            if entry is not None:
                plan = pc.materialize(entry, ctx)
                self._executed = reuse_exchanges(plan, self.session) if ctx.reuse else plan
            else:
                self._pending_store = (pc, key, ctx)
            return None
        with entry.lock:
            saved = entry.bind_literals(ctx.lits)
            try:
                fut = backend.collect_async(entry.plan)
            finally:
                entry.restore_literals(saved)
        # a result fallback later re-runs the query on the host: give it a plan of its own
        fut.plan = None
        fut.plan_fn = lambda: pc.materialize(entry, ctx)
        return fut

    def explain_string(self, extended: bool = False) -> str:
        parts = []
        if extended:
            parts += ["== Analyzed Logical Plan ==", self.logical.tree_string(),
                      "== Optimized Logical Plan ==", self.optimized_plan.tree_string()]
        parts += ["== Physical Plan ==", self.executed_plan.tree_string()]
        return "\n".join(parts)


class _Done:
    def __init__(self, table: pa.Table, path: str):
        self._t, self.path, self.reason = table, path, None

    def result(self) -> pa.Table:
        return self._t
