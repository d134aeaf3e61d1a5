#!/usr/bin/env python
"""Merge-join kernel microbenchmark on SF-shaped device tables (no Parquet, no index build).

Builds TPC-H-shaped bucketed, sorted lineitem / orders columns directly in HBM (sparse unique
order keys, 1-7 lines per order, the bench's Q3 predicates and aggregate), compact-encodes them
like the executor, then times ``exec.jit.merge_join_agg`` for every configuration (a JSON dict
of ``exec.jit`` knobs) and checks every result against the first.  One JSON line per config.

    python scripts/mj_micro.py --sf 100 --configs '[{}, {"MJ_RUNS": false}]'
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(sf: float, B: int, dev):
    import numpy as np
    import pyarrow as pa
    import torch
    from hyperspace_amd.exec.device_table import DeviceColumn
    from hyperspace_amd.ops import kernels as K
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    n_ord = int(1_500_000 * sf)
    i = torch.arange(n_ord, dtype=torch.int64, device=dev)
    okeys = (i // 8) * 32 + (i % 8) + 1                      # TPC-H sparse order keys
    kc = DeviceColumn(okeys, None, pa.int64())
    ob, counts = K.murmur3_bucket([kc], B)
    perm = K.sort_permutation([DeviceColumn(ob, None, pa.int32()), kc]).long()
    okeys, ob = okeys[perm], ob[perm]
    per = torch.randint(1, 8, (n_ord,), device=dev, generator=g)
    lkeys = torch.repeat_interleave(okeys, per)
    lb = torch.repeat_interleave(ob, per)
    n_li = lkeys.numel()
    lcounts = torch.bincount(lb.long(), minlength=B)
    loff = np.concatenate([[0], np.cumsum(lcounts.cpu().numpy())]).astype(np.int64)
    roff = torch.from_numpy(np.concatenate([[0], np.cumsum(counts.cpu().numpy())])
                            .astype(np.int64)).to(dev)
    odate = torch.randint(8035, 10440, (n_ord,), dtype=torch.int32, device=dev, generator=g)
    ship = torch.repeat_interleave(odate, per) + \
        torch.randint(1, 122, (n_li,), dtype=torch.int32, device=dev, generator=g)
    qty = torch.randint(1, 51, (n_li,), device=dev, generator=g).double()
    price = torch.round(qty * (900 + torch.randint(0, 20000, (n_li,), device=dev,
                                                   generator=g).double() / 10) * 100) / 100
    disc = torch.randint(0, 11, (n_li,), device=dev, generator=g).double() / 100
    prio = torch.zeros(n_ord, dtype=torch.int32, device=dev)
    del per, lb, perm, i
    cols = {0: DeviceColumn(lkeys, None, pa.int64()), 1: DeviceColumn(ship, None, pa.date32()),
            2: DeviceColumn(price, None, pa.float64()), 3: DeviceColumn(disc, None, pa.float64()),
            8: DeviceColumn(okeys, None, pa.int64()), 9: DeviceColumn(odate, None, pa.date32()),
            10: DeviceColumn(prio, None, pa.int32())}
    return cols, loff, roff, n_li, n_ord


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--buckets", type=int, default=200)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--configs", default="[{}]")
    ap.add_argument("--day", type=int, default=9190)
    args = ap.parse_args()
    import torch
    from hyperspace_amd.exec import jit
    from hyperspace_amd.exec.encoding import encode
    from hyperspace_amd.ops import _lib as NL
    from hyperspace_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    cols, loff, roff, n_li, n_ord = build(args.sf, args.buckets, dev)
    comp = {s: e for s, e in ((s, encode(c)) for s, c in cols.items()) if e is not None}
    torch.cuda.synchronize()
    print(json.dumps({"built_s": round(time.perf_counter() - t0, 2), "lineitem": n_li,
                      "orders": n_ord, "widths": {s: e.width for s, e in comp.items()}}),
          flush=True)
    p = NL.JoinParams()
    for s, c in cols.items():
        p.cols[s] = c.desc()
    p.preds[0] = NL.Pred(NL.PK_INT_LIT, NL.OP_GT, 1, 0, 0, 0, args.day, 0.0, None)
    p.preds[1] = NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 9, 0, 1000, 0, args.day, 0.0, None)
    p.nlp, p.npreds = 1, 2
    a = NL.AggSpec()
    a.kind, a.nterms = NL.AK_SUM, 2
    a.col[0], a.alpha[0], a.beta[0] = 2, 0.0, 1.0
    a.col[1], a.alpha[1], a.beta[1] = 3, 1.0, -1.0
    c = NL.AggSpec()
    c.kind = NL.AK_COUNT_STAR
    p.aggs[0], p.aggs[1] = a, c
    p.naggs, p.lkey, p.rkey, p.key_is_float, p.group_col = 2, 0, 8, 0, -1
    p.num_groups, p.group_base = 1, 0
    rstart, rlen, rbk = K.full_ranges(loff, dev)
    from hyperspace_amd.exec import jit_runs
    configs = json.loads(args.configs)

    def mod(k):     # knobs of the two-phase form live in exec/jit_runs.py
        return jit_runs if hasattr(jit_runs, k) and not hasattr(jit, k) else jit
    base = {k: getattr(mod(k), k) for cfg in configs for k in cfg}
    ref = None
    for cfg in configs:
        for k, v in base.items():
            setattr(mod(k), k, v)
        for k, v in cfg.items():
            setattr(mod(k), k, v)
        jit._KERNELS.clear()

        def run():
            return jit.merge_join_agg(p, rstart, rlen, rbk, roff, comp, nrows=n_li,
                                      cache_spans=True, rdup=False)
        out = run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            out = run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        s_, n_ = float(out[0][0].item()), int(out[1][1].item())
        if ref is None:
            ref = (s_, n_)
        ok = n_ == ref[1] and abs(s_ - ref[0]) <= 1e-9 * abs(ref[0])
        print(json.dumps({"cfg": cfg, "ms": round(ms, 4), "sum": s_, "count": n_, "match": ok}),
              flush=True)
    for k, v in base.items():
        setattr(mod(k), k, v)


if __name__ == "__main__":
    main()
