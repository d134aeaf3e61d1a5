"""cProfile of one SF-N index build on the device (the bench's li_shipdate index): where the
host time of a build goes (``python scripts/diag/build_profile.py --sf 100``)."""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--data-dir", default=os.environ.get("HS_BENCH_DIR", "/tmp/hs_bench"))
    ap.add_argument("--index", default="li_shipdate")
    args = ap.parse_args()
    import torch
    from hyperspace_amd import Hyperspace, IndexConfig, Session
    from hyperspace_amd.models import tpch
    nfiles = max(8, int(round(args.sf * 1.28)))
    data = os.path.join(args.data_dir, f"tpch_sf{args.sf:g}_f{nfiles}")
    tpch.generate(data, args.sf, nfiles, workers=16)
    cfgs = {"li_shipdate": ("lineitem", ["l_shipdate"], ["l_discount", "l_quantity",
                                                         "l_extendedprice"]),
            "li_orderkey": ("lineitem", ["l_orderkey"], ["l_extendedprice", "l_discount",
                                                         "l_shipdate"])}
    table, idx, inc = cfgs[args.index]
    for rep in range(2):
        root = os.path.join(args.data_dir, f"bprof_{rep}")
        s = Session(conf={"spark.hyperspace.system.path": root,
                          "spark.hyperspace.index.numBuckets": "200",
                          "spark.hyperspace.mi.execution.device": "gpu"})
        hs = Hyperspace(s)
        df = s.read.parquet(os.path.join(data, table))
        pr = cProfile.Profile() if rep == 1 else None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if pr is not None:
            pr.enable()
        hs.createIndex(df, IndexConfig(f"{args.index}_{rep}", idx, inc))
        torch.cuda.synchronize()
        if pr is not None:
            pr.disable()
        print(f"[build_profile] rep {rep}: {time.perf_counter() - t0:.3f}s", file=sys.stderr,
              flush=True)
        if pr is not None:
            buf = io.StringIO()
            st = pstats.Stats(pr, stream=buf)
            st.sort_stats("tottime").print_stats(40)
            st.sort_stats("cumulative").print_stats(70)
            print(buf.getvalue(), file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
