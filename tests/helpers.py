"""Shared fixtures/helpers for the CPU end-to-end tiers (reference ``SampleData.scala:25-50``,
``TestUtils.scala:27-121``, ``E2EHyperspaceRulesTest.scala:1004-1019``)."""
from __future__ import annotations

import os
from typing import List

import pyarrow as pa
import pyarrow.parquet as pq

from hyperspace_amd import Session
from hyperspace_amd.plan import physical as X
from hyperspace_amd.utils import path_utils as P

SAMPLE_ROWS = [
    ("2017-09-03", "810a20a2", "donde", 1, 10),
    ("2017-09-03", "fd093f8a", "facebook", 2, 20),
    ("2017-09-03", "af3ed6a1", "ibraco", 3, 30),
    ("2018-09-03", "975134eb", "facebook", 4, 40),
    ("2018-09-03", "9ae2bbcd", "donde", 5, 50),
    ("2019-10-03", "3ee5b7cf", "miperro", 6, 60),
    ("2019-10-03", "fd093f8a", "facebook", 7, 70),
    ("2019-10-03", "810a20a2", "donde", 8, 80),
    ("2020-10-03", "af3ed6a1", "ibraco", 9, 90),
    ("2020-10-03", "3ee5b7cf", "miperro", 10, 100),
]
SAMPLE_COLS = ["Date", "RGUID", "Query", "imprs", "clicks"]


def sample_table() -> pa.Table:
    cols = list(zip(*SAMPLE_ROWS))
    return pa.table({"Date": pa.array(cols[0]), "RGUID": pa.array(cols[1]),
                     "Query": pa.array(cols[2]), "imprs": pa.array(cols[3], pa.int32()),
                     "clicks": pa.array(cols[4], pa.int64())})


def write_parquet_parts(t: pa.Table, directory: str, parts: int = 2, prefix: str = "part") -> List[str]:
    os.makedirs(directory, exist_ok=True)
    step = (t.num_rows + parts - 1) // parts
    out = []
    for i in range(parts):
        p = os.path.join(directory, f"{prefix}-{i:05d}.parquet")
        pq.write_table(t.slice(i * step, step), p)
        out.append(p)
    return out


def make_session(tmp_path, **extra) -> Session:
    conf = {"spark.hyperspace.system.path": str(tmp_path / "indexes"),
            "spark.hyperspace.index.numBuckets": "4",
            "spark.sql.autoBroadcastJoinThreshold": "-1",
            "spark.sql.shuffle.partitions": "5",
            "spark.hyperspace.mi.execution.device": "cpu"}
    conf.update({k.replace("__", "."): v for k, v in extra.items()})
    return Session(conf=conf, warehouse_dir=str(tmp_path / "wh"))


def scans(df) -> list:
    return df.queryExecution.executed_plan.collect(lambda p: isinstance(p, X.FileSourceScanExec))


def count_nodes(df, cls) -> int:
    return len(df.queryExecution.executed_plan.collect(lambda p: isinstance(p, cls)))


def index_names_used(df) -> set:
    return {s.relation.index.name for s in scans(df) if s.relation.index is not None}


def sorted_rows(df):
    def key(r):
        return tuple((v is None, str(type(v)), v if v is not None else 0) for v in r)
    return sorted(df.collect(), key=key)


def verify_index_usage(session, make_df, expected_indexes: set, index_files_only: bool = True):
    """Disabled-vs-enabled oracle: same schema and sorted rows; the enabled plan scans exactly
    the expected indexes, and (unless hybrid scan mixes in source files) only files under their
    ``v__=`` directories."""
    session.disableHyperspace()
    base = make_df()
    expected = sorted_rows(base)
    schema = base.schema
    session.enableHyperspace()
    df = make_df()
    assert df.schema == schema
    assert sorted_rows(df) == expected
    assert index_names_used(df) == set(expected_indexes)
    for s in scans(df):
        if s.relation.index is not None and index_files_only:
            for f in s.relation.location.all_files():
                parent = P.get_name(P.get_parent(f.path))
                assert parent.startswith("v__="), f.path
    return df
