#!/usr/bin/env python
"""A guided tour of hyperspace_amd, in the spirit of the reference's "Hitchhiker's Guide to
Hyperspace" notebook: create sample data, build covering indexes, watch the optimizer use them,
mutate the data, refresh, optimize and walk through the lifecycle.

    python examples/quickstart.py                 # host executor
    python examples/quickstart.py --device gpu    # MI355X executor (index builds + queries)
"""
import argparse
import os
import shutil
import sys
import tempfile

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_  # noqa: E402


def banner(msg):
    print(f"\n=== {msg} " + "=" * max(0, 70 - len(msg)))


def write_tables(root, rng):
    os.makedirs(f"{root}/departments")
    os.makedirs(f"{root}/employees")
    depts = pa.table({"deptId": np.arange(10, 50, 10, dtype=np.int64),
                      "deptName": ["Accounting", "Research", "Sales", "Operations"],
                      "location": ["New York", "Dallas", "Chicago", "Boston"]})
    pq.write_table(depts, f"{root}/departments/part-0.parquet")
    n = 2000
    emps = pa.table({"empId": np.arange(n, dtype=np.int64),
                     "empName": [f"emp{i:04d}" for i in range(n)],
                     "deptId": rng.choice(np.arange(10, 50, 10, dtype=np.int64), n),
                     "salary": rng.integers(1000, 9000, n).astype(np.float64)})
    for i in range(4):
        pq.write_table(emps.slice(i * n // 4, n // 4), f"{root}/employees/part-{i}.parquet")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu", choices=["cpu", "gpu"])
    ap.add_argument("--keep", action="store_true", help="keep the temporary lake directory")
    args = ap.parse_args()
    root = tempfile.mkdtemp(prefix="hs_quickstart_")
    rng = np.random.default_rng(0)
    write_tables(root, rng)
    s = Session(conf={"spark.hyperspace.system.path": f"{root}/indexes",
                      "spark.hyperspace.index.numBuckets": "8",
                      "spark.hyperspace.index.lineage.enabled": "true",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.hyperspace.mi.execution.device": args.device},
                warehouse_dir=f"{root}/wh")
    hs = Hyperspace(s)
    emp = s.read.parquet(f"{root}/employees")
    dept = s.read.parquet(f"{root}/departments")

    banner("1. create covering indexes")
    hs.createIndex(emp, IndexConfig("empIndex", ["deptId"], ["empName", "salary"]))
    hs.createIndex(dept, IndexConfig("deptIndex", ["deptId"], ["deptName"]))
    hs.createIndex(emp, IndexConfig("empNameIndex", ["empName"], ["salary"]))
    hs.indexes().show()

    banner("2. a filter query served by an index")
    Hyperspace.enable(s)
    f = emp.filter(col("empName") == "emp0042").select("empName", "salary")
    hs.explain(f, verbose=True)
    f.show()

    banner("3. an equi-join served by two co-bucketed indexes (no shuffle, no sort)")
    j = emp.join(dept, emp["deptId"] == dept["deptId"]) \
        .groupBy(dept["deptName"]).agg(sum_(col("salary")).alias("payroll"),
                                        count("*").alias("headcount"))
    hs.explain(j, verbose=True)
    j.show()
    print("executed on:", s.backend().last_path)

    banner("4. the data changes: append a file, delete a file")
    extra = pa.table({"empId": np.arange(5000, 5100, dtype=np.int64),
                      "empName": [f"new{i:03d}" for i in range(100)],
                      "deptId": np.full(100, 20, dtype=np.int64),
                      "salary": np.full(100, 4242.0)})
    pq.write_table(extra, f"{root}/employees/part-new.parquet")
    os.remove(f"{root}/employees/part-3.parquet")
    emp = s.read.parquet(f"{root}/employees")
    j2 = emp.join(dept, emp["deptId"] == dept["deptId"]).select(emp["empName"], dept["deptName"])
    print("index used while stale?",
          "Name: empIndex" in j2.queryExecution.executed_plan.tree_string())

    banner("5. Hybrid Scan: use the stale index plus the changed files")
    s.conf.set("spark.hyperspace.index.hybridscan.enabled", "true")
    s.conf.set("spark.hyperspace.index.hybridscan.maxDeletedRatio", "0.5")
    s.conf.set("spark.hyperspace.index.hybridscan.maxAppendedRatio", "0.5")
    j2 = emp.join(dept, emp["deptId"] == dept["deptId"]).select(emp["empName"], dept["deptName"])
    print(j2.queryExecution.executed_plan.tree_string())
    print("rows:", len(j2.collect()))
    s.conf.set("spark.hyperspace.index.hybridscan.enabled", "false")

    banner("6. incremental refresh, then optimize the small files away")
    hs.refreshIndex("empIndex", "incremental")
    hs.optimizeIndex("empIndex", "full")
    hs.index("empIndex").show()

    banner("7. lifecycle: delete (soft), restore, delete + vacuum (hard)")
    hs.deleteIndex("empNameIndex")
    hs.restoreIndex("empNameIndex")
    hs.deleteIndex("empNameIndex")
    hs.vacuumIndex("empNameIndex")
    hs.indexes().show()

    if args.keep:
        print("lake kept at", root)
    else:
        shutil.rmtree(root)


if __name__ == "__main__":
    main()
