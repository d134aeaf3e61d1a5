"""Index rankers (reference ``index/rankers/FilterIndexRanker.scala:28-61``,
``JoinIndexRanker.scala:28-91``)."""
from __future__ import annotations

import functools

from ..index import tags as T
from ..utils.conf import HyperspaceConf


def rank_filter(session, plan, candidates: list):
    if not candidates:
        return None
    if HyperspaceConf.hybrid_scan_enabled(session.conf):
        return max(candidates, key=lambda i: i.get_tag_value(plan, T.COMMON_SOURCE_SIZE_IN_BYTES) or 0)
    return candidates[0]


def rank_join(session, left_child, right_child, pairs: list) -> list:
    hybrid = HyperspaceConf.hybrid_scan_enabled(session.conf)

    def common(plan, idx):
        return idx.get_tag_value(plan, T.COMMON_SOURCE_SIZE_IN_BYTES) or 0

    def before(p1, p2) -> bool:
        (l1, r1), (l2, r2) = p1, p2
        c1 = common(left_child, l1) + common(right_child, r1)
        c2 = common(left_child, l2) + common(right_child, r2)
        if l1.num_buckets == r1.num_buckets and l2.num_buckets == r2.num_buckets:
            if not hybrid or c1 == c2:
                return l1.num_buckets > l2.num_buckets
            return c1 > c2
        if l1.num_buckets == r1.num_buckets:
            return True
        if l2.num_buckets == r2.num_buckets:
            return False
        return (not hybrid) or c1 > c2

    def cmp(a, b):
        if before(a, b):
            return -1
        if before(b, a):
            return 1
        return 0
    return sorted(pairs, key=functools.cmp_to_key(cmp))
