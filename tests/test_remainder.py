"""Spark ``%`` (``Remainder``) on the host engine: parser, literal operands on either side,
negative operands, zero divisors (NULL), ``Long.MIN_VALUE % -1`` and float ``fmod``, against
plain Python / numpy truth.  The device projection is checked against this oracle in
``tests/test_project_gpu.py::test_remainder_matches_host_oracle``."""
import math

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

from hyperspace_amd import Session, col


def _jmod(a, b):
    """JVM truncated remainder."""
    if a is None or b is None or b == 0:
        return None
    if b == -1:
        return 0
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def _session(tmp_path):
    return Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                         "spark.hyperspace.mi.execution.device": "cpu"},
                   warehouse_dir=str(tmp_path / "wh"))


def test_remainder_host_semantics(tmp_path):
    a = [7, -7, 13, -13, 0, None, -9223372036854775808, 5]
    b = [3, 3, -4, -4, 5, 2, -1, 0]
    x = [7.5, -7.5, 1.0, -0.0, 3.25, 2.0, 1e10, 5.5]
    (tmp_path / "t").mkdir()
    pq.write_table(pa.table({"a": pa.array(a, pa.int64()), "b": pa.array(b, pa.int32()),
                             "x": pa.array(x)}), tmp_path / "t" / "p.parquet")
    s = _session(tmp_path)
    df = s.read.parquet(str(tmp_path / "t"))
    t = df.select((col("a") % col("b")).alias("ab"), (col("a") % 4).alias("a4"),
                  (100 % col("b")).alias("lb"), (-100 % col("b")).alias("nlb"),
                  (col("x") % 2.5).alias("xf"), (9.0 % col("x")).alias("lx")).to_arrow()
    assert t.column("ab").to_pylist() == [_jmod(p, q) for p, q in zip(a, b)]
    assert t.column("a4").to_pylist() == [_jmod(p, 4) for p in a]
    assert t.column("lb").to_pylist() == [_jmod(100, q) for q in b]
    assert t.column("nlb").to_pylist() == [_jmod(-100, q) for q in b]
    assert t.column("ab").type == pa.int64() and t.column("lb").type in (pa.int32(), pa.int64())
    xf = t.column("xf").to_pylist()
    for v, want in zip(xf, [math.fmod(p, 2.5) for p in x]):
        assert v == want or (math.isnan(v) and math.isnan(want))
    lx = t.column("lx").to_pylist()
    for v, p in zip(lx, x):
        want = None if p == 0 else math.fmod(9.0, p)
        assert (v is None and want is None) or v == want


def test_remainder_parser(tmp_path):
    (tmp_path / "t").mkdir()
    pq.write_table(pa.table({"a": np.arange(-10, 10, dtype=np.int64)}), tmp_path / "t" / "p.parquet")
    s = _session(tmp_path)
    df = s.read.parquet(str(tmp_path / "t"))
    got = df.filter("a % 3 = -1").to_arrow().column("a").to_pylist()
    assert got == [a for a in range(-10, 10) if _jmod(a, 3) == -1]
