"""Computed projections and GROUP BY expressions on the device (exec/project.py): one
generated elementwise kernel per projection, Spark semantics (wrapping integer arithmetic,
NULL for a zero divisor, truncating casts, Kleene AND / OR), checked against the host oracle
with the native path asserted.  The reference covers Project(Filter(Relation)) with arbitrary
project lists (FilterIndexRule.scala:155-191)."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_

from test_gpu_e2e import _both, _close

pytestmark = pytest.mark.gpu


@pytest.fixture
def tbl(tmp_path, device):
    rng = np.random.default_rng(5)
    n = 200_000
    a = rng.integers(-1000, 1000, n).astype(np.int64)
    b = rng.integers(-5, 6, n).astype(np.int32)            # zeros: NULL quotients
    t = pa.table({"k": rng.integers(0, 50_000, n).astype(np.int64),
                  "a": pa.array(a, mask=rng.random(n) < 0.05),
                  "b": pa.array(b),
                  "i": pa.array(rng.integers(-2**31, 2**31 - 1, n).astype(np.int32)),
                  "x": np.round(rng.random(n) * 200 - 100, 3),
                  "q": pa.array(rng.integers(1, 51, n).astype(np.float64),
                                mask=rng.random(n) < 0.03)})
    os.makedirs(tmp_path / "t")
    for i in range(3):
        pq.write_table(t.slice(i * (n // 3), n // 3 + (n % 3 if i == 2 else 0)),
                       tmp_path / "t" / f"part-{i}.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "16",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=str(tmp_path / "wh"))
    hs = Hyperspace(s)
    df = s.read.parquet(str(tmp_path / "t"))
    hs.createIndex(df, IndexConfig("t_k", ["k"], ["a", "b", "i", "x", "q"]))
    Hyperspace.enable(s)
    return s, s.read.parquet(str(tmp_path / "t"))


def test_computed_projection_rows_native(tbl):
    s, df = tbl
    f = df.filter(col("k") < 4000)
    q = f.select(col("k"),
                 (col("a") * 3 + col("b")).alias("lin"),
                 (col("a") / col("b")).alias("quot"),
                 (col("i") + col("i")).alias("wrap32"),           # int32 overflow wraps
                 (col("x") * col("q") - 1.5).alias("fx"),
                 col("x").cast("int").alias("trunc"),
                 ((col("a") > col("b")) & (col("q") < 25)).alias("both"),
                 ((col("a") < 0) | (col("q") > 40)).alias("either"))
    plan = q.queryExecution.executed_plan.tree_string()
    assert "Name: t_k" in plan
    g, c, path = _both(s, q)
    assert path == "native", s.backend().fallback_reason
    assert g.num_rows > 0
    _close(g, c)


def test_filter_and_aggregate_over_computed_columns(tbl):
    s, df = tbl
    p = df.filter(col("k") > 100).select((col("a") * 2).alias("a2"), col("x"), col("k"))
    q = p.filter(col("a2") > 500).agg(sum_("x").alias("sx"), count("*").alias("n"),
                                      sum_("a2").alias("sa"))
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)


def test_group_by_expressions_native(tbl):
    s, df = tbl
    f = df.filter(col("k") < 20_000)
    # small integer domain (dense LDS aggregate)
    q1 = f.groupBy((col("b") * 2 + 1).alias("g")).agg(sum_("x").alias("sx"), count("*").alias("n"))
    # unnamed expression + a plain column (multi-column: hash aggregate)
    q2 = f.groupBy(col("a") / 100, col("b")).agg(sum_("q").alias("sq"))
    for q in (q1, q2):
        g, c, path = _both(s, q)
        assert path == "native", s.backend().fallback_reason
        _close(g, c)


def test_union_all_rows_and_aggregates_native(tbl):
    s, df = tbl
    lo = df.filter(col("k") < 3000).select("k", "a", "x")
    hi = df.filter(col("k") > 47_000).select("k", "a", "x")
    u = lo.union(hi)
    for q in (u,
              u.agg(sum_("x").alias("sx"), count("*").alias("n"), sum_("a").alias("sa")),
              u.groupBy((col("k") / 10_000).cast("int").alias("band"))
               .agg(count("*").alias("n"), sum_("x").alias("sx"))):
        g, c, path = _both(s, q)
        assert path == "native", s.backend().fallback_reason
        assert g.num_rows > 0
        _close(g, c)


def test_float_to_int_casts_saturate_like_spark(tbl):
    """d2i / d2l saturation (NaN -> 0, +-inf and 3e9 clamp) and the wrapping narrow of a short /
    byte target, device against the host oracle (the int target used to wrap)."""
    s, df = tbl
    f = df.filter(col("k") < 6000)
    big = col("x") * 1e8                    # up to +-1e10: outside the int range
    inf = col("x") * 1e307 * 100            # +-inf (0 stays 0)
    q = f.select(col("k"), big.cast("int").alias("i32"), big.cast("short").alias("i16"),
                 big.cast("byte").alias("i8"), big.cast("long").alias("i64"),
                 inf.cast("int").alias("inf32"), inf.cast("long").alias("inf64"))
    g, c, path = _both(s, q)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    i32 = g.column("i32").to_pylist()
    assert 2147483647 in i32 and -2147483648 in i32


def test_remainder_matches_host_oracle(tbl):
    """Spark ``%`` on the device against the host oracle: column % literal,
    literal % column, negative operands, zero divisors (NULL), LLONG_MIN % -1 and float fmod."""
    s, df = tbl
    f = df.filter(col("k") < 5000)
    q = f.select(col("k"),
                 (col("a") % 7).alias("a_mod_lit"),
                 (col("a") % -7).alias("a_mod_neg"),
                 (1000 % col("b")).alias("lit_mod_b"),        # b has zeros: NULLs
                 (-1000 % col("b")).alias("neg_lit_mod_b"),
                 (col("a") % col("b")).alias("a_mod_b"),
                 ((col("a") * 0 - 9223372036854775807 - 1) % -1).alias("min_mod_m1"),
                 (col("x") % 3.5).alias("fmod"),
                 (7.25 % col("x")).alias("lit_fmod"))
    g, c, path = _both(s, q)
    assert path == "native", s.backend().fallback_reason
    assert g.num_rows > 0
    _close(g, c)
