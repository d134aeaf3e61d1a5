"""Competent CPU baseline for the headline step (one Q6 + one Q3), BASELINE.md "measure it on
the same synthetic TPC-H data": Apache Arrow's multithreaded C++ engine (Acero) over the SAME
covering-index files the MI355X engine serves from, used the way a CPU engine would use them.

* Q6 over ``li_shipdate`` (sorted by l_shipdate inside every bucket file): a dataset scan with
  the whole predicate pushed down, so row groups whose l_shipdate / l_discount / l_quantity
  statistics exclude the range are never read (row-group pruning), then one vectorized
  sum(l_extendedprice * l_discount).
* Q3 over ``li_orderkey`` x ``ord_orderkey`` (co-bucketed on the join key, 200 buckets): the
  bucketed join the reference's JoinIndexRule plans (no shuffle) - every bucket pair is filtered,
  hash-joined and partially aggregated by one task of a thread pool, partials merged at the end.
* The un-indexed alternative (the same queries over the source Parquet files) is measured too,
  and the baseline is the better of the two (VERDICT r2 "what's weak" 5).
* ``--warm`` (the default since round 4): the same two plans over Arrow tables already RESIDENT
  in host RAM (the index columns each query reads, loaded once before timing, split into
  record batches for the thread pool) - the CPU counterpart of the MI355X engine serving
  HBM-resident columns, with no file read or decode inside the timed queries.  Q6 is Acero's
  multithreaded filter + project over the in-memory dataset with the same row-group pruning
  done by the batches' min/max (batches are sorted by l_shipdate inside every bucket); Q3 is the
  bucketed hash join per resident bucket pair on the thread pool.  The baseline is the best of
  warm / cold / unindexed per query.

Writes ``profiles/cpu_baseline_sf<SF>.json`` (the ``vs_baseline`` denominator of bench.py).
Run it where the bench's data and indexes exist (the GPU box, after bench.py), e.g.
``python scripts/cpu_baseline.py --sf 100 --threads 16``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import datetime
import glob
import json
import os
import sys
import threading
import time

import pyarrow as pa
import pyarrow.compute as pc
import pyarrow.dataset as ds

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _heartbeat(stop: threading.Event) -> None:
    t0 = time.time()
    while not stop.wait(30):
        print(f"[cpu_baseline] running {time.time() - t0:.0f}s", file=sys.stderr, flush=True)


def q6_lits(i: int):
    year = 1993 + i % 5
    disc = 0.02 + (i % 8) * 0.01
    return (datetime.date(year, 1, 1), datetime.date(year + 1, 1, 1), round(disc - 0.01, 2),
            round(disc + 0.01, 2), 24 + (i % 2))


def q3_date(i: int):
    return datetime.date(1995, 3, 1) + datetime.timedelta(days=(i * 7) % 30)


def q6(dataset: ds.Dataset, i: int) -> float:
    lo, hi, dlo, dhi, qty = q6_lits(i)
    f = ((ds.field("l_shipdate") >= pa.scalar(lo)) & (ds.field("l_shipdate") < pa.scalar(hi)) &
         (ds.field("l_discount") >= dlo) & (ds.field("l_discount") <= dhi) &
         (ds.field("l_quantity") < qty))
    t = dataset.to_table(columns=["l_extendedprice", "l_discount"], filter=f, use_threads=True)
    return pc.sum(pc.multiply(t["l_extendedprice"], t["l_discount"])).as_py() or 0.0


def _q3_part(li_files, od_files, dd):
    li = ds.dataset(li_files, format="parquet").to_table(
        columns=["l_orderkey", "l_extendedprice", "l_discount"],
        filter=ds.field("l_shipdate") > pa.scalar(dd), use_threads=False)
    od = ds.dataset(od_files, format="parquet").to_table(
        columns=["o_orderkey", "o_shippriority"],
        filter=ds.field("o_orderdate") < pa.scalar(dd), use_threads=False)
    if not li.num_rows or not od.num_rows:
        return {}
    j = li.join(od, keys="l_orderkey", right_keys="o_orderkey", join_type="inner",
                use_threads=False)
    rev = pc.multiply(j["l_extendedprice"], pc.subtract(1.0, j["l_discount"]))
    g = pa.table({"p": j["o_shippriority"], "r": rev}).group_by("p").aggregate(
        [("r", "sum"), ("r", "count")])
    return {p: (r, n) for p, r, n in zip(g["p"].to_pylist(), g["r_sum"].to_pylist(),
                                         g["r_count"].to_pylist())}


def q3_bucketed(pool, li_buckets, od_buckets, i: int):
    dd = q3_date(i)
    tasks = [pool.submit(_q3_part, li_buckets[b], od_buckets[b], dd)
             for b in sorted(li_buckets) if b in od_buckets]
    out = {}
    for t in tasks:
        for p, (r, n) in t.result().items():
            a = out.get(p, (0.0, 0))
            out[p] = (a[0] + r, a[1] + n)
    return out


def q3_unindexed(li_ds, od_ds, i: int):
    dd = q3_date(i)
    li = li_ds.to_table(columns=["l_orderkey", "l_extendedprice", "l_discount"],
                        filter=ds.field("l_shipdate") > pa.scalar(dd))
    od = od_ds.to_table(columns=["o_orderkey", "o_shippriority"],
                        filter=ds.field("o_orderdate") < pa.scalar(dd))
    j = li.join(od, keys="l_orderkey", right_keys="o_orderkey", join_type="inner")
    rev = pc.multiply(j["l_extendedprice"], pc.subtract(1.0, j["l_discount"]))
    g = pa.table({"p": j["o_shippriority"], "r": rev}).group_by("p").aggregate(
        [("r", "sum"), ("r", "count")])
    return dict(zip(g["p"].to_pylist(), zip(g["r_sum"].to_pylist(), g["r_count"].to_pylist())))


class WarmQ6:
    """Resident ``li_shipdate`` columns as record batches with their l_shipdate ranges, so a
    query touches only batches that can hold its year (the in-memory form of row-group
    pruning)."""

    COLS = ["l_shipdate", "l_discount", "l_quantity", "l_extendedprice"]

    def __init__(self, files, batch_rows: int = 1 << 20):
        self.batches = []
        for f in sorted(files):
            t = ds.dataset(f, format="parquet").to_table(columns=self.COLS)
            for b in t.combine_chunks().to_batches(max_chunksize=batch_rows):
                mm = pc.min_max(b.column(0))
                self.batches.append((mm["min"].as_py(), mm["max"].as_py(), b))

    def __call__(self, pool, i: int) -> float:
        lo, hi, dlo, dhi, qty = q6_lits(i)

        def part(b):
            d = b.column(0)
            m = pc.and_(pc.and_(pc.greater_equal(d, pa.scalar(lo)), pc.less(d, pa.scalar(hi))),
                        pc.and_(pc.and_(pc.greater_equal(b.column(1), dlo),
                                        pc.less_equal(b.column(1), dhi)),
                                pc.less(b.column(2), qty)))
            t = b.filter(m)
            return pc.sum(pc.multiply(t.column(3), t.column(1))).as_py() or 0.0
        live = [b for mn, mx, b in self.batches if mx is not None and mx >= lo and mn < hi]
        return sum(pool.map(part, live))


class WarmQ3:
    """Resident bucket pairs of ``li_orderkey`` / ``ord_orderkey`` (the Q3 columns), joined
    bucket by bucket on the thread pool."""

    def __init__(self, li_buckets, od_buckets):
        self.pairs = []
        for b in sorted(li_buckets):
            if b not in od_buckets:
                continue
            li = ds.dataset(li_buckets[b], format="parquet").to_table(
                columns=["l_orderkey", "l_extendedprice", "l_discount", "l_shipdate"])
            od = ds.dataset(od_buckets[b], format="parquet").to_table(
                columns=["o_orderkey", "o_orderdate", "o_shippriority"])
            self.pairs.append((li.combine_chunks(), od.combine_chunks()))

    @staticmethod
    def _part(li, od, dd):
        li = li.filter(pc.greater(li["l_shipdate"], pa.scalar(dd)))
        od = od.filter(pc.less(od["o_orderdate"], pa.scalar(dd)))
        if not li.num_rows or not od.num_rows:
            return {}
        j = li.select(["l_orderkey", "l_extendedprice", "l_discount"]).join(
            od.select(["o_orderkey", "o_shippriority"]), keys="l_orderkey",
            right_keys="o_orderkey", join_type="inner", use_threads=False)
        rev = pc.multiply(j["l_extendedprice"], pc.subtract(1.0, j["l_discount"]))
        g = pa.table({"p": j["o_shippriority"], "r": rev}).group_by("p").aggregate(
            [("r", "sum"), ("r", "count")])
        return {p: (r, n) for p, r, n in zip(g["p"].to_pylist(), g["r_sum"].to_pylist(),
                                             g["r_count"].to_pylist())}

    def __call__(self, pool, i: int):
        dd = q3_date(i)
        out = {}
        for part in pool.map(lambda x: self._part(x[0], x[1], dd), self.pairs):
            for p, (r, n) in part.items():
                a = out.get(p, (0.0, 0))
                out[p] = (a[0] + r, a[1] + n)
        return out


def _bucket_files(index_dir: str):
    out = {}
    for f in glob.glob(os.path.join(index_dir, "**", "*.parquet"), recursive=True):
        b = int(os.path.basename(f).split("_")[-1].split(".")[0])
        out.setdefault(b, []).append(f)
    return out


def _timed(fn, reps: int):
    ts = []
    res = None
    for i in range(reps):
        t = time.perf_counter()
        res = fn(i)
        ts.append(time.perf_counter() - t)
    return sum(ts) / len(ts), res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100.0)
    ap.add_argument("--buckets", type=int, default=200)
    ap.add_argument("--data-dir", default=os.environ.get("HS_BENCH_DIR", "/tmp/hs_bench"))
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--skip-unindexed", action="store_true")
    ap.add_argument("--no-warm", action="store_true",
                    help="skip the resident-table (warm) plans")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    pa.set_cpu_count(args.threads)
    pa.set_io_thread_count(args.threads)
    stop = threading.Event()
    threading.Thread(target=_heartbeat, args=(stop,), daemon=True).start()
    sf = args.sf
    nfiles = max(8, int(round(sf * 1.28)))
    data = os.path.join(args.data_dir, f"tpch_sf{sf:g}_f{nfiles}")
    idx = os.path.join(args.data_dir, f"indexes_sf{sf:g}_b{args.buckets}_w1")
    ship = glob.glob(os.path.join(idx, "li_shipdate", "**", "*.parquet"), recursive=True)
    li_b = _bucket_files(os.path.join(idx, "li_orderkey"))
    od_b = _bucket_files(os.path.join(idx, "ord_orderkey"))
    if not ship or not li_b or not od_b:
        raise SystemExit(f"index files missing under {idx}: run bench.py first")
    res = {"sf": sf, "threads": args.threads}
    ship_ds = ds.dataset(ship, format="parquet")
    q6(ship_ds, 0)   # warm the page cache / footers
    res["q6_indexed_s"], _ = _timed(lambda i: q6(ship_ds, i), args.reps)
    print(f"[cpu_baseline] q6 indexed {res['q6_indexed_s']:.3f}s", file=sys.stderr, flush=True)
    with cf.ThreadPoolExecutor(args.threads) as pool:
        q3_bucketed(pool, li_b, od_b, 0)
        res["q3_indexed_s"], _ = _timed(lambda i: q3_bucketed(pool, li_b, od_b, i), args.reps)
    print(f"[cpu_baseline] q3 indexed {res['q3_indexed_s']:.3f}s", file=sys.stderr, flush=True)
    step = res["q6_indexed_s"] + res["q3_indexed_s"]
    source = "indexed"
    best6, best3 = res["q6_indexed_s"], res["q3_indexed_s"]
    if not args.no_warm:
        t0 = time.perf_counter()
        w6, w3 = WarmQ6(ship), WarmQ3(li_b, od_b)
        res["warm_load_s"] = time.perf_counter() - t0
        with cf.ThreadPoolExecutor(args.threads) as pool:
            # same answers as the cold plans
            a6 = q6(ship_ds, 1)
            assert abs(w6(pool, 1) - a6) <= 1e-9 * max(abs(a6), 1.0)
            c3 = q3_bucketed(pool, li_b, od_b, 1)
            g3 = w3(pool, 1)
            assert sorted(c3) == sorted(g3) and all(
                c3[k][1] == g3[k][1] and abs(c3[k][0] - g3[k][0]) <= 1e-9 * abs(c3[k][0])
                for k in c3), (c3, g3)
            res["q6_warm_s"], _ = _timed(lambda i: w6(pool, i), args.reps)
            res["q3_warm_s"], _ = _timed(lambda i: w3(pool, i), args.reps)
        print(f"[cpu_baseline] warm q6 {res['q6_warm_s']:.3f}s q3 {res['q3_warm_s']:.3f}s",
              file=sys.stderr, flush=True)
        best6, best3 = min(best6, res["q6_warm_s"]), min(best3, res["q3_warm_s"])
        del w6, w3
    if not args.skip_unindexed:
        li_ds = ds.dataset(os.path.join(data, "lineitem"), format="parquet")
        od_ds = ds.dataset(os.path.join(data, "orders"), format="parquet")
        res["q6_unindexed_s"], _ = _timed(lambda i: q6(li_ds, i), args.reps)
        print(f"[cpu_baseline] q6 unindexed {res['q6_unindexed_s']:.3f}s", file=sys.stderr,
              flush=True)
        res["q3_unindexed_s"], _ = _timed(lambda i: q3_unindexed(li_ds, od_ds, i), args.reps)
        print(f"[cpu_baseline] q3 unindexed {res['q3_unindexed_s']:.3f}s", file=sys.stderr,
              flush=True)
        # both plans answer the same queries
        a6, b6 = q6(ship_ds, 1), q6(li_ds, 1)
        assert abs(a6 - b6) <= 1e-9 * max(abs(b6), 1.0), (a6, b6)
        with cf.ThreadPoolExecutor(args.threads) as pool:
            a3 = q3_bucketed(pool, li_b, od_b, 1)
        b3 = q3_unindexed(li_ds, od_ds, 1)
        assert sorted(a3) == sorted(b3) and all(
            a3[k][1] == b3[k][1] and abs(a3[k][0] - b3[k][0]) <= 1e-9 * abs(b3[k][0])
            for k in b3), (a3, b3)
        res["results_match"] = True
        best6 = min(best6, res["q6_unindexed_s"])
        best3 = min(best3, res["q3_unindexed_s"])
    if best6 + best3 < step:
        # the best plan per query
        step, source = best6 + best3, "best of warm-resident / indexed / unindexed per query"
    stop.set()
    out = {"metric": "queries/s (CPU baseline: one Q6 + one Q3 per step)",
           "value": round(2.0 / step, 4), "unit": "queries/s", "ms_per_step": round(step * 1e3, 2),
           "source": f"scripts/cpu_baseline.py: pyarrow {pa.__version__} Acero, "
                     f"{args.threads} threads, row-group pruning, bucketed join ({source})",
           "detail": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}}
    line = json.dumps(out)
    print(line)
    path = args.out or os.path.join(ROOT, "profiles", f"cpu_baseline_sf{sf:g}.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(line + "\n")


if __name__ == "__main__":
    main()
