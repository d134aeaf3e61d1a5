"""HBM-budgeted streaming index build (the reference scales builds by bucket count
and streaming tasks, docs/_docs/04-ug-faqs.md:107-132): the pass / file-group planner on the
CPU, and on the GPU a build forced into many bucket-range passes whose bucket files are
equal to the one-pass build's (rows, order, schema, row groups)."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd.exec.device_build import plan_file_groups, plan_passes


def test_plan_passes_cover_buckets_contiguously():
    assert plan_passes(100, 1000, 200) == [(0, 200)]
    assert plan_passes(100, 0, 200) == [(0, 200)]          # 0 = no budget
    p = plan_passes(10_000, 1_000, 200)
    assert len(p) == 10 and p[0][0] == 0 and p[-1][1] == 200
    assert all(a[1] == b[0] for a, b in zip(p, p[1:]))
    assert {hi - lo for lo, hi in p} == {20}
    p = plan_passes(10 ** 12, 1, 7)                          # at most one bucket per pass
    assert p == [(i, i + 1) for i in range(7)]
    p = plan_passes(2_500, 1_000, 10)
    assert len(p) == 3 and sum(hi - lo for lo, hi in p) == 10


def test_plan_file_groups_respect_budget():
    assert plan_file_groups([10, 10, 10], 4, 1_000) == [(0, 3)]
    assert plan_file_groups([10, 10, 10, 10], 10, 250) == [(0, 2), (2, 4)]
    assert plan_file_groups([100, 1, 1], 10, 50) == [(0, 1), (1, 3)]   # oversized file alone
    assert plan_file_groups([], 8, 10) == []


@pytest.mark.gpu
def test_streaming_build_writes_same_files(tmp_path, device):
    from hyperspace_amd import Hyperspace, IndexConfig, Session
    from hyperspace_amd.exec import device_build
    rng = np.random.default_rng(3)
    src = tmp_path / "src"
    src.mkdir()
    for i in range(5):
        n = 40_000 + 1_000 * i
        t = pa.table({"k": pa.array(rng.integers(0, 5_000, n)),           # many equal keys
                      "d": pa.array(rng.integers(8000, 11000, n).astype(np.int32)),
                      "p": pa.array(np.round(rng.random(n) * 1e4, 2)),
                      "q": pa.array(np.where(rng.random(n) < 0.1, None,
                                             rng.integers(0, 50, n)).tolist(), pa.int64()),
                      # strings: per-file dictionaries differ; file 3 has nulls
                      "s": pa.array([f"s{x}" if i != 3 or x % 9 else None
                                     for x in rng.integers(0, 40 + 10 * i, n)], pa.string())})
        # file 4: PLAIN-encoded strings (decoded on the device, no dictionary pages)
        pq.write_table(t, src / f"part-{i}.parquet", row_group_size=16_000,
                       use_dictionary=(i != 4))

    def build(name, budget):
        s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "ix"),
                          "spark.hyperspace.index.numBuckets": "16",
                          "spark.hyperspace.mi.execution.device": "gpu",
                          "spark.hyperspace.mi.build.hbmBudgetBytes": str(budget)},
                    warehouse_dir=str(tmp_path / "wh"))
        Hyperspace(s).createIndex(s.read.parquet(str(src)), IndexConfig(name, ["k"], ["d", "p", "q", "s"]))
        stats = dict(device_build.LAST_BUILD_STATS)
        files = {}
        for root, _, fs in os.walk(tmp_path / "ix" / name):
            for f in fs:
                if f.endswith(".parquet"):
                    b = int(f.split("_")[-1].split(".")[0])
                    files[b] = open(os.path.join(root, f), "rb").read()
        return files, stats
    one, s1 = build("one_pass", 1 << 40)
    many, s2 = build("streamed", 600_000)
    assert "passes" not in s1 and s2["passes"] >= 4 and s2["file_groups"] >= 2, s2
    # every column - dictionary and PLAIN strings, nulls included - decoded on the device, the
    # streamed build's job-global string dictionary too
    assert s1.get("host_decoded") == [] and s2.get("host_decoded") == [], (s1, s2)
    assert sorted(one) == sorted(many) and len(one) == 16
    # compared decoded (same rows in the same order, schema and row groups): the dictionary vs
    # PLAIN choice per column follows the distinct values of the buckets one encode call covers
    for b in one:
        fx = pq.ParquetFile(pa.BufferReader(one[b]))
        fy = pq.ParquetFile(pa.BufferReader(many[b]))
        assert fx.read().equals(fy.read()), f"bucket {b} differs"
        assert fx.schema_arrow.equals(fy.schema_arrow)
        assert [fx.metadata.row_group(g).num_rows for g in range(fx.num_row_groups)] == \
            [fy.metadata.row_group(g).num_rows for g in range(fy.num_row_groups)]


def test_footer_info_marks_uncovered_columns_nullable(tmp_path):
    """Columns a Parquet footer does not cover (hive partition columns, columns missing from
    the file) may hold nulls: the multi-GPU batched exchange agrees on validity masks from
    this before its first collective batch (exec/device_build.py)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from hyperspace_amd.exec.device_build import _footer_info
    p = tmp_path / "f.parquet"
    pq.write_table(pa.table({"a": [1, 2, 3], "b": [1.0, None, 2.0]}), p)
    rows, maybe = _footer_info(str(p), ["a", "b", "part", "missing"])
    assert rows == 3
    assert maybe == {"b", "part", "missing"}
