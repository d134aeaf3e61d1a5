"""Which scan path (captured graph or plain launch) Q6 and COUNT(*)-only Q6 take, and why."""
import datetime, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_
from hyperspace_amd.exec import gpu as G
from hyperspace_amd.models import tpch
d = "/tmp/hs_diag"; data = os.path.join(d, "tpch")
tpch.generate(data, 1, 8)
s = Session(conf={"spark.hyperspace.system.path": os.path.join(d, "idx"),
                  "spark.hyperspace.index.numBuckets": "64",
                  "spark.hyperspace.mi.execution.device": "gpu"}, warehouse_dir=os.path.join(d, "wh"))
hs = Hyperspace(s)
li = s.read.parquet(os.path.join(data, "lineitem"))
hs.createIndex(li, IndexConfig("li_shipdate", ["l_shipdate"], ["l_discount", "l_quantity", "l_extendedprice"]))
Hyperspace.enable(s)
li = s.read.parquet(os.path.join(data, "lineitem"))
orig = G.GpuBackend._graph_eligible
def ge(self, spec, descs):
    out = orig(self, spec, descs)
    print("graph_eligible", out, "spec", None if spec is None else (spec[1], spec[3], spec[5]),
          "descs", sorted(descs), flush=True)
    return out
G.GpuBackend._graph_eligible = ge
f = li.filter((col("l_shipdate") >= datetime.date(1994, 1, 1)) & (col("l_shipdate") < datetime.date(1995, 1, 1)) &
              (col("l_discount") >= 0.05) & (col("l_discount") <= 0.07) & (col("l_quantity") < 24))
for name, q in (("sum", f.agg(sum_(col("l_extendedprice") * col("l_discount")).alias("r"))),
                ("count", f.agg(count("*").alias("n")))):
    print(name, q.collect(), s.backend().last_path if hasattr(s.backend(), "last_path") else "")
    print(q.queryExecution.executed_plan.tree_string())
