#!/usr/bin/env python
"""Index-build benchmark on the bench's TPC-H data: builds the bench's covering indexes (or
those named by --index) and prints one JSON line per build with its wall time, decoded-bytes
GB/s and the device build's stage breakdown (``LAST_BUILD_STATS``).

    python scripts/build_bench.py --sf 100 [--index li_shipdate]
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
    ap.add_argument("--buckets", type=int, default=200)
    ap.add_argument("--data-dir", default=os.environ.get("HS_BENCH_DIR", "/tmp/hs_bench"))
    ap.add_argument("--index", action="append", default=None)
    ap.add_argument("--codec", default="none")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--h2d-streams", type=int, default=None,
                    help="staging.UPLOAD_H2D_STREAMS for this run (0 = one stream per file)")
    ap.add_argument("--d2h-priority", type=int, default=None,
                    help="pq_encode.D2H_PRIORITY for this run (0 = ordinary copy streams)")
    ap.add_argument("--d2h-serial", type=int, default=None,
                    help="pq_encode.D2H_ON_COMPRESS_STREAM for this run")
    ap.add_argument("--cprofile", action="store_true",
                    help="main-thread cProfile of each build (top functions to stderr)")
    ap.add_argument("--conf", action="append", default=[],
                    help="extra session conf key=value (e.g. spark.hyperspace.mi.build.copyCUs=0)")
    args = ap.parse_args()
    import torch
    from hyperspace_amd import Hyperspace, IndexConfig, Session
    from hyperspace_amd.exec import device_build
    from hyperspace_amd.models import tpch
    torch.cuda.set_device(0)
    if args.h2d_streams is not None:
        from hyperspace_amd.exec import staging
        staging.UPLOAD_H2D_STREAMS = args.h2d_streams
    if args.d2h_serial is not None:
        from hyperspace_amd.exec import pq_encode
        pq_encode.D2H_ON_COMPRESS_STREAM = bool(args.d2h_serial)
    if args.d2h_priority is not None:
        from hyperspace_amd.exec import pq_encode
        pq_encode.D2H_PRIORITY = bool(args.d2h_priority)
    nfiles = max(8, int(round(args.sf * 1.28)))
    data = os.path.join(args.data_dir, f"tpch_sf{args.sf:g}_f{nfiles}")
    tpch.generate(data, args.sf, nfiles, workers=16)
    idx_root = os.path.join(args.data_dir, f"bb_indexes_sf{args.sf:g}")
    s = Session(conf={"spark.hyperspace.system.path": idx_root,
                      "spark.hyperspace.index.numBuckets": str(args.buckets),
                      "spark.hyperspace.mi.execution.device": "gpu",
                      "spark.hyperspace.mi.index.codec": args.codec,
                      **dict(kv.split("=", 1) for kv in args.conf)},
                warehouse_dir=os.path.join(args.data_dir, "wh"))
    hs = Hyperspace(s)
    s.backend()             # engine start outside the timed builds (as bench.py)
    li = s.read.parquet(os.path.join(data, "lineitem"))
    od = s.read.parquet(os.path.join(data, "orders"))
    builds = [(li, IndexConfig("li_shipdate", ["l_shipdate"],
                               ["l_discount", "l_quantity", "l_extendedprice"])),
              (li, IndexConfig("li_orderkey", ["l_orderkey"],
                               ["l_extendedprice", "l_discount", "l_shipdate"])),
              (od, IndexConfig("ord_orderkey", ["o_orderkey"], ["o_orderdate", "o_shippriority"]))]
    for rep in range(args.repeat):
        if os.path.exists(idx_root):
            shutil.rmtree(idx_root)
        for df, cfg in builds:
            if args.index and cfg.indexName not in args.index:
                continue
            torch.cuda.synchronize()
            prof = None
            if args.cprofile:
                import cProfile
                prof = cProfile.Profile()
                prof.enable()
            t = time.perf_counter()
            hs.createIndex(df, cfg)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            if prof is not None:
                import io
                import pstats
                prof.disable()
                buf = io.StringIO()
                pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(25)
                print(f"[build_bench] {cfg.indexName} cProfile\n{buf.getvalue()}", file=sys.stderr)
            st = dict(device_build.LAST_BUILD_STATS)
            print(json.dumps({"index": cfg.indexName, "rep": rep, "conf": args.conf,
                              "h2d_streams": args.h2d_streams, "d2h_serial": args.d2h_serial, "d2h_priority": args.d2h_priority,
                              "s": round(dt, 3),
                              "gbps": round(st.get("source_bytes", 0) / dt / 1e9, 3),
                              "stats": st}), flush=True)


if __name__ == "__main__":
    main()
