"""``BucketUnionStrategy`` (reference ``index/execution/BucketUnionStrategy.scala:28-34``)."""
from __future__ import annotations

from ..plan import logical as L
from ..plan import physical as X


def BucketUnionStrategy(planner, plan):
    if isinstance(plan, L.BucketUnion):
        return X.BucketUnionExec([planner.plan(c) for c in plan.children], plan.bucket_spec)
    return None
