#!/usr/bin/env python
"""Kernel-level sweep for the fused join/scan aggregates on SF-shaped device tables.

Builds TPC-H-shaped bucketed, sorted columns directly in HBM (orders: sparse unique keys; lineitem:
1-7 rows per order), then times the generated (JIT) kernels over a parameter grid and the AOT
interpreter for reference.  Prints one JSON line per configuration.

    python scripts/microbench_join.py --sf 100 --buckets 200
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--buckets", type=int, default=200)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--items", default="2,4,8")
    ap.add_argument("--grids", default="1024,2048,4096")
    ap.add_argument("--blocks", default="256")
    ap.add_argument("--stage", default="1,0", help="stage right columns in LDS (1/0)")
    ap.add_argument("--pipe", default="1,0", help="software-pipelined tile loop (1/0)")
    ap.add_argument("--direct", default="1,0", help="direct-address LDS key table (1/0)")
    ap.add_argument("--quick", action="store_true", help="raw/lazy join variants only")
    ap.add_argument("--no-scan", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import pyarrow as pa
    import torch
    from hyperspace_amd.exec import jit
    from hyperspace_amd.exec import kernel_config
    base = kernel_config.active()
    from hyperspace_amd.exec.device_table import DeviceColumn
    from hyperspace_amd.ops import _lib as NL
    from hyperspace_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    B = args.buckets
    n_ord = int(1_500_000 * args.sf)
    okeys = torch.arange(n_ord, dtype=torch.int64, device=dev) * 4 + 1
    kc = DeviceColumn(okeys, None, pa.int64())
    ob, counts = K.murmur3_bucket([kc], B)
    perm = K.sort_permutation([DeviceColumn(ob, None, pa.int32())])
    okeys = okeys[perm.long()]
    ocounts = counts
    per = torch.randint(1, 8, (n_ord,), device=dev, generator=g)
    lkeys = torch.repeat_interleave(okeys, per)
    lb = torch.repeat_interleave(ob[perm.long()], per)
    n_li = lkeys.numel()
    lcounts = torch.bincount(lb.long(), minlength=B)
    loff = np.concatenate([[0], np.cumsum(lcounts.cpu().numpy())]).astype(np.int64)
    roff = torch.from_numpy(np.concatenate([[0], np.cumsum(ocounts.cpu().numpy())]).astype(np.int64)).to(dev)
    ship = torch.randint(8000, 10600, (n_li,), dtype=torch.int32, device=dev, generator=g)
    # TPC-H prices are DECIMAL(15,2): doubles that are exact 2-digit decimals
    price = torch.round(torch.rand(n_li, dtype=torch.float64, device=dev, generator=g) * 1e7) / 100
    disc = torch.randint(0, 11, (n_li,), device=dev, generator=g).double() / 100
    odate = torch.randint(8000, 10500, (n_ord,), dtype=torch.int32, device=dev, generator=g)
    del per, lb
    cols = {0: DeviceColumn(lkeys, None, pa.int64()), 1: DeviceColumn(ship, None, pa.int32()),
            2: DeviceColumn(price, None, pa.float64()), 3: DeviceColumn(disc, None, pa.float64()),
            8: DeviceColumn(okeys, None, pa.int64()), 9: DeviceColumn(odate, None, pa.int32())}
    p = NL.JoinParams()
    for s, c in cols.items():
        p.cols[s] = c.desc()
    p.preds[0] = NL.Pred(NL.PK_INT_LIT, NL.OP_GT, 1, 0, 0, 0, 9200, 0.0, None)
    p.preds[1] = NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 9, 0, 1000, 0, 9200, 0.0, None)
    p.nlp, p.npreds = 1, 2
    a = NL.AggSpec()
    a.kind, a.nterms = NL.AK_SUM, 2
    a.col[0], a.alpha[0], a.beta[0] = 2, 0.0, 1.0
    a.col[1], a.alpha[1], a.beta[1] = 3, 1.0, -1.0
    c = NL.AggSpec()
    c.kind = NL.AK_COUNT_STAR
    p.aggs[0], p.aggs[1] = a, c
    p.naggs, p.lkey, p.rkey, p.key_is_float, p.group_col = 2, 0, 8, 0, -1
    rstart, rlen, rbk = K.full_ranges(loff, dev)
    mt = K.join_max_tiles(n_li, B)
    nbytes = n_li * 28 + n_ord * 12

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            out = fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.iters, out

    ms, out = timed(lambda: K.join_agg(p, rstart, rlen, rbk, roff, mt))
    ref = out[0][0].item()
    print(json.dumps({"kernel": "aot_join", "ms": round(ms, 3), "GBps": round(nbytes / ms / 1e6, 1),
                      "rows": n_li}), flush=True)
    from hyperspace_amd.exec.encoding import encode
    comp = {s: e for s, e in ((s, encode(cc)) for s, cc in cols.items()) if e is not None}
    print(json.dumps({"compact_widths": {s: e.width for s, e in comp.items()}}), flush=True)
    modes = [("raw", False)] if args.quick else [("raw", False), ("raw", True), ("compact", False)]
    for cmode, eager in modes:
        cm = comp if cmode == "compact" else None
        for pipe, direct in [(p_ == "1", d_ == "1") for p_ in args.pipe.split(",")
                             for d_ in args.direct.split(",")]:
          for stage in [x == "1" for x in args.stage.split(",")]:
            for block in [int(x) for x in args.blocks.split(",")]:
                for items in [int(x) for x in args.items.split(",")]:
                    for grid in [int(x) for x in args.grids.split(",")]:
                        kernel_config.bind(base.replace(
                            join_items=items, join_grid=grid, join_eager=eager,
                            join_block=block, join_stage_right=stage, join_pipeline=pipe,
                            join_direct=direct))
                        ms, out = timed(lambda: jit.join_agg(p, rstart, rlen, rbk, roff, mt, cm))
                        ok = abs(out[0][0].item() - ref) <= 1e-9 * abs(ref)
                        print(json.dumps({"kernel": "jit_join", "enc": cmode, "eager": eager,
                                          "pipeline": pipe, "direct": direct,
                                          "stage_right": stage,
                                          "block": block, "items": items,
                                          "grid": grid, "ms": round(ms, 3),
                                          "GBps_logical": round(nbytes / ms / 1e6, 1),
                                          "match": ok}), flush=True)
    kernel_config.bind(base)
    if args.no_scan:
        return
    # scan (Q6 shape) over a shipdate-sorted copy: 1/7 of the rows in range
    order = torch.argsort(ship.view(-1), stable=True)
    s_ship, s_disc, s_price = ship[order], disc[order], price[order]
    qty = torch.randint(1, 51, (n_li,), device=dev, generator=g).double()
    lo = int(torch.searchsorted(s_ship, torch.tensor([8766], dtype=torch.int32, device=dev)).item())
    hi = int(torch.searchsorted(s_ship, torch.tensor([9131], dtype=torch.int32, device=dev)).item())
    sp = NL.ScanParams()
    scols = {0: DeviceColumn(s_disc, None, pa.float64()), 1: DeviceColumn(qty, None, pa.float64()),
             2: DeviceColumn(s_price, None, pa.float64())}
    for s, cc in scols.items():
        sp.cols[s] = cc.desc()
    sp.preds[0] = NL.Pred(NL.PK_FLT_LIT, NL.OP_GE, 0, 0, 0, 0, 0, 0.05, None)
    sp.preds[1] = NL.Pred(NL.PK_FLT_LIT, NL.OP_LE, 0, 0, 1, 0, 0, 0.07, None)
    sp.preds[2] = NL.Pred(NL.PK_FLT_LIT, NL.OP_LT, 1, 0, 2, 0, 0, 24.0, None)
    sp.npreds = 3
    a = NL.AggSpec()
    a.kind, a.nterms = NL.AK_SUM, 2
    a.col[0], a.alpha[0], a.beta[0] = 2, 0.0, 1.0
    a.col[1], a.alpha[1], a.beta[1] = 0, 0.0, 1.0
    sp.aggs[0] = a
    sp.aggs[1] = c
    sp.naggs, sp.group_col = 2, -1
    rs_ = torch.tensor([lo], dtype=torch.int64, device=dev)
    rl_ = torch.tensor([hi - lo], dtype=torch.int64, device=dev)
    sbytes = (hi - lo) * 24
    tp = K.ranges_to_tiles(rl_)
    ms, out = timed(lambda: K.scan_agg(sp, rs_, rl_, tp))
    ref = out[0][0].item()
    print(json.dumps({"kernel": "aot_scan", "ms": round(ms, 3), "GBps": round(sbytes / ms / 1e6, 1),
                      "rows": hi - lo}), flush=True)
    scomp = {s: e for s, e in ((s, encode(cc)) for s, cc in scols.items()) if e is not None}
    for cmode in ("raw", "compact"):
        cm = scomp if cmode == "compact" else None
        for eager in (True, False):
            for items in (4, 8):
                for grid in [int(x) for x in args.grids.split(",")]:
                    kernel_config.bind(base.replace(scan_items=items, scan_grid=grid,
                                                    scan_eager=eager))
                    ms, out = timed(lambda: jit.scan_agg(sp, rs_, rl_, None, cm))
                    ok = abs(out[0][0].item() - ref) <= 1e-9 * abs(ref)
                    print(json.dumps({"kernel": "jit_scan", "enc": cmode, "eager": eager,
                                      "items": items, "grid": grid, "ms": round(ms, 3),
                                      "GBps_logical": round(sbytes / ms / 1e6, 1), "match": ok}),
                          flush=True)


if __name__ == "__main__":
    main()
