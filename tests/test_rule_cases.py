"""JoinIndexRule / FilterIndexRule applicability cases and the rankers, mirroring the reference's
rule-level suites (``JoinIndexRuleTest.scala`` — CNF, aliases, one-to-one column mapping, included
columns, implicit outputs; ``FilterIndexRuleTest.scala``; ``FilterIndexRankerTest.scala``,
``JoinIndexRankerTest.scala``).  Plans come from the DataFrame API over two small Parquet tables
(the reference builds the same shapes from synthetic attributes)."""
from __future__ import annotations

import numpy as np
import pyarrow as pa
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, col, lit
from hyperspace_amd.index import tags as T
from hyperspace_amd.plan import physical as X
from hyperspace_amd.rules.join_rule import JoinIndexRule
from hyperspace_amd.rules.rankers import rank_filter, rank_join

from helpers import (count_nodes, index_names_used, make_session, verify_index_usage,
                     write_parquet_parts)


@pytest.fixture
def tables(tmp_path):
    """t1(t1c1..t1c4), t2(t2c1..t2c4) with the reference's index set: t1i1(t1c1; t1c3),
    t1i2(t1c1,t1c2; t1c3), t1i3(t1c2; t1c3), t2i1(t2c1; t2c3), t2i2(t2c1,t2c2; t2c3)."""
    s = make_session(tmp_path)
    rng = np.random.default_rng(11)
    n = 60
    for name in ("t1", "t2"):
        t = pa.table({f"{name}c1": rng.integers(0, 12, n).astype(np.int64),
                      f"{name}c2": pa.array([f"v{x}" for x in rng.integers(0, 5, n)]),
                      f"{name}c3": rng.integers(0, 100, n).astype(np.int32),
                      f"{name}c4": rng.random(n)})
        write_parquet_parts(t, str(tmp_path / name), parts=2)
    hs = Hyperspace(s)
    t1 = lambda: s.read.parquet(str(tmp_path / "t1"))  # noqa: E731
    t2 = lambda: s.read.parquet(str(tmp_path / "t2"))  # noqa: E731
    for name, df, idx, inc in (("t1i1", t1, ["t1c1"], ["t1c3"]),
                               ("t1i2", t1, ["t1c1", "t1c2"], ["t1c3"]),
                               ("t1i3", t1, ["t1c2"], ["t1c3"]),
                               ("t2i1", t2, ["t2c1"], ["t2c3"]),
                               ("t2i2", t2, ["t2c1", "t2c2"], ["t2c3"])):
        hs.createIndex(df(), IndexConfig(name, idx, inc))
    yield s, hs, t1, t2
    s.disableHyperspace()


def _no_index_join(s, df):
    s.enableHyperspace()
    assert not any(sc.use_bucketing for sc in
                   df.queryExecution.executed_plan.collect(
                       lambda p: isinstance(p, X.FileSourceScanExec))), \
        df.queryExecution.executed_plan.tree_string()


# ---------------------------------------------------------------------------------- applies
def test_join_rule_applies_with_matching_indexes(tables):
    s, _, t1, t2 = tables

    def q():
        a, b = t1(), t2()
        return a.join(b, a["t1c1"] == b["t2c1"]).select(a["t1c1"], a["t1c3"], b["t2c1"], b["t2c3"])
    df = verify_index_usage(s, q, {"t1i1", "t2i1"})
    assert count_nodes(df, X.ShuffleExchangeExec) == 0


def test_join_rule_case_insensitive_query(tables):
    s, _, t1, t2 = tables

    def q():
        a, b = t1(), t2()
        return a.join(b, a["T1C1"] == b["T2c1"]).select(a["T1c1"], a["t1C3"], b["t2c1"],
                                                         b["T2C3"])
    verify_index_usage(s, q, {"t1i1", "t2i1"})


@pytest.mark.parametrize("order", ["same", "reordered", "swapped", "repeated"])
def test_join_rule_composite_and_conditions(tables, order):
    s, _, t1, t2 = tables

    def q():
        a, b = t1(), t2()
        c1 = a["t1c1"] == b["t2c1"]
        c2 = a["t1c2"] == b["t2c2"]
        cond = {"same": c1 & c2, "reordered": c2 & c1,
                "swapped": (b["t2c1"] == a["t1c1"]) & (b["t2c2"] == a["t1c2"]),
                "repeated": c1 & c2 & c1}[order]
        return a.join(b, cond).select(a["t1c1"], a["t1c3"], b["t2c1"], b["t2c3"])
    verify_index_usage(s, q, {"t1i2", "t2i2"})


# ---------------------------------------------------------------------------------- does not apply
def test_join_rule_skips_cross_join(tables):
    s, _, t1, t2 = tables
    a, b = t1(), t2()
    _no_index_join(s, a.crossJoin(b).select(a["t1c1"], b["t2c1"]))
    _no_index_join(s, a.join(b).select(a["t1c1"], b["t2c1"]))


def test_join_rule_skips_non_equality_condition(tables):
    s, _, t1, t2 = tables
    a, b = t1(), t2()
    _no_index_join(s, a.join(b, a["t1c1"] > b["t2c1"]).select(a["t1c1"], b["t2c1"]))


def test_join_rule_skips_or_condition(tables):
    s, _, t1, t2 = tables
    a, b = t1(), t2()
    _no_index_join(s, a.join(b, (a["t1c1"] == b["t2c1"]) | (a["t1c2"] == b["t2c2"]))
                   .select(a["t1c1"], b["t2c1"]))


def test_join_rule_skips_literal_condition(tables):
    s, _, t1, t2 = tables
    a, b = t1(), t2()
    _no_index_join(s, a.join(b, a["t1c1"] == lit(10)).select(a["t1c1"], b["t2c1"]))


def test_join_rule_needs_indexes_on_both_sides(tables):
    s, hs, t1, t2 = tables
    for name in ("t2i1", "t2i2"):
        hs.deleteIndex(name)
    a, b = t1(), t2()
    _no_index_join(s, a.join(b, a["t1c1"] == b["t2c1"]).select(a["t1c1"], b["t2c1"]))


def test_join_rule_skips_when_included_columns_missing(tables):
    s, _, t1, t2 = tables
    a, b = t1(), t2()
    # t1c4 is in no index
    _no_index_join(s, a.join(b, a["t1c1"] == b["t2c1"]).select(a["t1c4"], b["t2c1"]))


def test_join_rule_implicit_output_columns(tables):
    s, hs, t1, t2 = tables
    a, b = t1(), t2()
    # no projection: every column of both sides is required, which no index covers
    _no_index_join(s, a.join(b, a["t1c1"] == b["t2c1"]))
    hs.createIndex(t1(), IndexConfig("t1all", ["t1c1"], ["t1c2", "t1c3", "t1c4"]))
    hs.createIndex(t2(), IndexConfig("t2all", ["t2c1"], ["t2c2", "t2c3", "t2c4"]))

    def q():
        x, y = t1(), t2()
        return x.join(y, x["t1c1"] == y["t2c1"])
    verify_index_usage(s, q, {"t1all", "t2all"})


def test_join_rule_requires_one_to_one_column_mapping(tables):
    s, _, t1, t2 = tables
    a, b = t1(), t2()
    _no_index_join(s, a.join(b, (a["t1c1"] == b["t2c1"]) & (a["t1c1"] == b["t2c2"]))
                   .select(a["t1c1"], b["t2c1"]))


def test_join_rule_not_reapplied_to_modified_plan(tables):
    s, _, t1, t2 = tables
    s.enableHyperspace()
    a, b = t1(), t2()
    df = a.join(b, a["t1c1"] == b["t2c1"]).select(a["t1c1"], a["t1c3"], b["t2c1"], b["t2c3"])
    once = df.queryExecution.optimized_plan
    assert index_names_used(df) == {"t1i1", "t2i1"}
    again = JoinIndexRule(s, once)
    assert again.tree_string() == once.tree_string()


# ---------------------------------------------------------------------------------- filter rule
def test_filter_rule_not_reapplied_and_alias_supported(tables):
    s, _, t1, _ = tables

    def q():
        return t1().filter(col("t1c2") == "v3").select(col("t1c2").alias("x"), col("t1c3"))
    verify_index_usage(s, q, {"t1i3"})


# ---------------------------------------------------------------------------------- rankers
class FakeIndex:
    def __init__(self, name, buckets, common=0):
        self.name = name
        self.num_buckets = buckets
        self._common = common

    def get_tag_value(self, plan, tag):
        return self._common if tag == T.COMMON_SOURCE_SIZE_IN_BYTES else None

    def __repr__(self):
        return self.name


def test_filter_ranker_head_by_default_and_largest_common_bytes_with_hybrid(tmp_path):
    s = make_session(tmp_path)
    a, b, c = FakeIndex("a", 10, 5), FakeIndex("b", 10, 50), FakeIndex("c", 10, 20)
    assert rank_filter(s, None, [a, b, c]) is a
    assert rank_filter(s, None, []) is None
    s.conf.set("spark.hyperspace.index.hybridscan.enabled", "true")
    assert rank_filter(s, None, [a, b, c]) is b


def test_join_ranker_prefers_equal_buckets_then_more_buckets(tmp_path):
    s = make_session(tmp_path)
    l10, l20, l30 = FakeIndex("l10", 10), FakeIndex("l20", 20), FakeIndex("l30", 30)
    r10, r20, r5 = FakeIndex("r10", 10), FakeIndex("r20", 20), FakeIndex("r5", 5)
    pairs = [(l30, r5), (l10, r10), (l20, r20)]
    ranked = rank_join(s, None, None, pairs)
    assert ranked[0] == (l20, r20) and ranked[1] == (l10, r10) and ranked[2] == (l30, r5)


def test_join_ranker_prefers_common_bytes_with_hybrid_scan(tmp_path):
    s = make_session(tmp_path)
    s.conf.set("spark.hyperspace.index.hybridscan.enabled", "true")
    l1, r1 = FakeIndex("l1", 10, 100), FakeIndex("r1", 10, 100)
    l2, r2 = FakeIndex("l2", 20, 10), FakeIndex("r2", 20, 10)
    ranked = rank_join(s, None, None, [(l2, r2), (l1, r1)])
    assert ranked[0] == (l1, r1)
