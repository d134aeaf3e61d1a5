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
            if HyperspaceConf.plan_cache_enabled(self.session.conf):
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
        return backend.collect(self.executed_plan)

    def to_arrow_async(self):
        """Plan now, execute asynchronously: an object whose ``result()`` is the table.  The
        device backend returns before its kernels finish (``GpuBackend.collect_async``); the
        host backend runs the query here."""
        backend = self.session.backend()
        plan = self.executed_plan
        if hasattr(backend, "collect_async"):
            return backend.collect_async(plan)
        return _Done(backend.collect(plan), getattr(backend, "last_path", "host"))

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
