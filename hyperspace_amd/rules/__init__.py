"""Hyperspace optimizer rules and their registration (reference ``package.scala:25-79``).

``enable`` installs ``JoinIndexRule`` then ``FilterIndexRule`` (join first: order matters) plus
``BucketUnionStrategy``; it first removes existing entries so it is idempotent.
"""
from __future__ import annotations

from .filter_rule import FilterIndexRule
from .join_rule import JoinIndexRule
from .bucket_union_strategy import BucketUnionStrategy

HYPERSPACE_RULES = (JoinIndexRule, FilterIndexRule)


def enable(session) -> None:
    disable(session)
    session.extra_optimizations.extend(HYPERSPACE_RULES)
    session.extra_strategies.append(BucketUnionStrategy)


def disable(session) -> None:
    session.extra_optimizations[:] = [r for r in session.extra_optimizations
                                      if r not in HYPERSPACE_RULES]
    session.extra_strategies[:] = [s for s in session.extra_strategies if s is not BucketUnionStrategy]


def is_enabled(session) -> bool:
    return all(r in session.extra_optimizations for r in HYPERSPACE_RULES) and \
        BucketUnionStrategy in session.extra_strategies
