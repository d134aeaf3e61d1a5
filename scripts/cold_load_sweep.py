#!/usr/bin/env python
"""Cold HBM load of index bucket files (load_bucketed_index) under the decode-path knobs:
device page decode (HS_DEVICE_PARQUET) x host-inflate policy (hs_pq_set_host_inflate), for
Snappy and uncompressed index files of the bench's TPC-H lineitem indexes.  One JSON line per
(codec, mode).

    python scripts/cold_load_sweep.py --sf 100
"""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--data-dir", default=os.environ.get("HS_BENCH_DIR", "/tmp/hs_bench"))
    args = ap.parse_args()
    import torch
    from hyperspace_amd import Hyperspace, IndexConfig, Session
    from hyperspace_amd.exec import device_cache, staging
    from hyperspace_amd.io import native_parquet
    from hyperspace_amd.models import tpch
    from hyperspace_amd.ops import _lib as NL
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    nfiles = max(8, int(round(args.sf * 1.28)))
    data = os.path.join(args.data_dir, f"tpch_sf{args.sf:g}_f{nfiles}")
    tpch.generate(data, args.sf, nfiles, workers=16)
    for codec in ("snappy", "none"):
        root = os.path.join(args.data_dir, f"cl_{codec}")
        shutil.rmtree(root, ignore_errors=True)
        s = Session(conf={"spark.hyperspace.system.path": root,
                          "spark.hyperspace.index.numBuckets": "200",
                          "spark.hyperspace.mi.execution.device": "gpu",
                          "spark.hyperspace.mi.index.codec": codec})
        hs = Hyperspace(s)
        li = s.read.parquet(os.path.join(data, "lineitem"))
        hs.createIndex(li, IndexConfig("li_shipdate", ["l_shipdate"],
                                       ["l_discount", "l_quantity", "l_extendedprice"]))
        idir = os.path.join(root, "li_shipdate", "v__=0")
        from hyperspace_amd.utils.file_utils import list_leaf_files
        files = [f for f in list_leaf_files(idir) if f.path.endswith(".parquet")]
        cols = ["l_shipdate", "l_discount", "l_quantity", "l_extendedprice"]
        for dev_path in ("1", "0"):
            for hmode in (2, 1, 0):
                os.environ["HS_DEVICE_PARQUET"] = dev_path
                native_parquet.lib().hs_pq_set_host_inflate(hmode)
                staging.DEVICE_DECODED.clear()
                staging.HOST_DECODED.clear()
                native_parquet.PHASES.clear()
                torch.cuda.synchronize()
                t = time.perf_counter()
                tab = device_cache.load_bucketed_index(files, cols, 200, ["l_shipdate"], dev)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t
                print(json.dumps({"codec": codec, "device_parquet": dev_path, "host_inflate": hmode,
                                  "load_s": round(dt, 3), "rows": tab.num_rows,
                                  "device_decoded": sorted(staging.DEVICE_DECODED),
                                  "phases": {k: round(v, 3) for k, v in
                                             native_parquet.PHASES.items()}}), flush=True)
                del tab
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
