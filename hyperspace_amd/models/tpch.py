"""Synthetic TPC-H-shaped tables (``lineitem``, ``orders``) for the benchmark and tests.

No dbgen/network here, so data is generated with numpy following the TPC-H column domains:
sparse order keys (8 of every 32), 1-7 lines per order, dates in [1992-01-01, 1998-08-02],
ship = order + [1,121] days, commit = order + [30,90], receipt = ship + [1,30], quantity in
[1,50], discount in [0.00,0.10], tax in [0.00,0.08], extendedprice = quantity * part price.
Row counts match the scale factor: orders = 1.5M * SF, lineitem ~= 6M * SF (avg 4 lines/order).

Generation is embarrassingly parallel: file ``i`` holds orders chunk ``i`` and the lineitems of
exactly those orders (so the join key domains line up), seeded by ``(seed, i)``.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

ORDERS_PER_SF = 1_500_000
DATE_LO = 8035     # 1992-01-01 as days since epoch
DATE_HI = 10440    # 1998-08-02 - 121 (so ship dates stay in range)

LINEITEM_SCHEMA = pa.schema([
    ("l_orderkey", pa.int64()), ("l_partkey", pa.int64()), ("l_suppkey", pa.int64()),
    ("l_linenumber", pa.int32()), ("l_quantity", pa.float64()), ("l_extendedprice", pa.float64()),
    ("l_discount", pa.float64()), ("l_tax", pa.float64()), ("l_returnflag", pa.string()),
    ("l_linestatus", pa.string()), ("l_shipdate", pa.date32()), ("l_commitdate", pa.date32()),
    ("l_receiptdate", pa.date32())])

ORDERS_SCHEMA = pa.schema([
    ("o_orderkey", pa.int64()), ("o_custkey", pa.int64()), ("o_orderstatus", pa.string()),
    ("o_totalprice", pa.float64()), ("o_orderdate", pa.date32()), ("o_orderpriority", pa.string()),
    ("o_shippriority", pa.int32())])

_PRIORITIES = np.array(["1-URGENT", "2-HIGH", "3-MEDIUM", "4-NOT SPECIFIED", "5-LOW"])


def order_count(sf: float) -> int:
    return int(ORDERS_PER_SF * sf)


def _sparse_key(i: np.ndarray) -> np.ndarray:
    # TPC-H orderkeys: 8 consecutive keys used out of every 32
    return (i // 8) * 32 + (i % 8) + 1


def generate_chunk(sf: float, nfiles: int, i: int, seed: int = 42):
    """Orders chunk i and its lineitems as two pyarrow tables."""
    n_orders = order_count(sf)
    lo = n_orders * i // nfiles
    hi = n_orders * (i + 1) // nfiles
    rng = np.random.default_rng([seed, i])
    idx = np.arange(lo, hi, dtype=np.int64)
    n = len(idx)
    okey = _sparse_key(idx)
    odate = rng.integers(DATE_LO, DATE_HI, n).astype(np.int32)
    nlines = rng.integers(1, 8, n)
    m = int(nlines.sum())
    lkey = np.repeat(okey, nlines)
    ldate = np.repeat(odate, nlines)
    first = np.repeat(np.cumsum(nlines) - nlines, nlines)
    linenumber = (np.arange(m) - first + 1).astype(np.int32)
    partkey = rng.integers(1, int(200_000 * sf) + 1, m).astype(np.int64)
    suppkey = rng.integers(1, int(10_000 * sf) + 1, m).astype(np.int64)
    qty = rng.integers(1, 51, m).astype(np.float64)
    price = np.round(900.0 + (partkey % 20001) / 10.0 + (partkey // 1000 % 1000), 2)
    ext = np.round(qty * price, 2)
    disc = rng.integers(0, 11, m) / 100.0
    tax = rng.integers(0, 9, m) / 100.0
    ship = ldate + rng.integers(1, 122, m).astype(np.int32)
    commit = ldate + rng.integers(30, 91, m).astype(np.int32)
    receipt = ship + rng.integers(1, 31, m).astype(np.int32)
    current = 9298  # 1995-06-17
    rflag = np.where(receipt <= current, np.where(rng.random(m) < 0.5, "R", "A"), "N")
    lstatus = np.where(ship > current, "O", "F")
    li = pa.Table.from_arrays([
        pa.array(lkey), pa.array(partkey), pa.array(suppkey), pa.array(linenumber), pa.array(qty),
        pa.array(ext), pa.array(disc), pa.array(tax), pa.array(rflag), pa.array(lstatus),
        pa.array(ship).view(pa.date32()), pa.array(commit).view(pa.date32()),
        pa.array(receipt).view(pa.date32())], schema=LINEITEM_SCHEMA)
    tot = np.bincount(np.repeat(np.arange(n), nlines), weights=ext * (1 + tax) * (1 - disc),
                      minlength=n)
    od = pa.Table.from_arrays([
        pa.array(okey), pa.array(rng.integers(1, int(150_000 * sf) + 1, n).astype(np.int64)),
        pa.array(np.where(rng.random(n) < 0.5, "F", "O")), pa.array(np.round(tot, 2)),
        pa.array(odate).view(pa.date32()), pa.array(_PRIORITIES[rng.integers(0, 5, n)]),
        pa.array(np.zeros(n, dtype=np.int32))], schema=ORDERS_SCHEMA)
    return li, od


def write_chunk(root: str, sf: float, nfiles: int, i: int, seed: int = 42) -> int:
    """Write chunk i (idempotent: temp + rename). Returns lineitem rows."""
    li_path = os.path.join(root, "lineitem", f"part-{i:05d}.parquet")
    od_path = os.path.join(root, "orders", f"part-{i:05d}.parquet")
    if os.path.exists(li_path) and os.path.exists(od_path):
        return pq.ParquetFile(li_path).metadata.num_rows
    li, od = generate_chunk(sf, nfiles, i, seed)
    for t, path in ((li, li_path), (od, od_path)):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = os.path.join(os.path.dirname(path), f".tmp-{os.getpid()}-{os.path.basename(path)}")
        pq.write_table(t, tmp, compression="snappy", row_group_size=1 << 20)
        os.replace(tmp, path)
    return li.num_rows


def _write_chunk_args(args):
    return write_chunk(*args)


def generate(root: str, sf: float, nfiles: int, files: Optional[list] = None,
             workers: int = 8, seed: int = 42) -> int:
    """Generate (the given subset of) chunk files with a process pool."""
    files = list(range(nfiles)) if files is None else list(files)
    todo = [(root, sf, nfiles, i, seed) for i in files]
    if workers <= 1 or len(todo) <= 1:
        return sum(_write_chunk_args(a) for a in todo)
    import multiprocessing as mp
    ctx = mp.get_context("fork")
    with ctx.Pool(processes=min(workers, len(todo))) as pool:
        return sum(pool.map(_write_chunk_args, todo, chunksize=1))


CUSTOMERS_PER_SF = 150_000
SEGMENTS = np.array(["AUTOMOBILE", "BUILDING", "FURNITURE", "HOUSEHOLD", "MACHINERY"])

CUSTOMER_SCHEMA = pa.schema([("c_custkey", pa.int64()), ("c_nationkey", pa.int32()),
                             ("c_acctbal", pa.float64()), ("c_mktsegment", pa.string())])


def write_customers(root: str, sf: float, nfiles: int = 4, seed: int = 42) -> int:
    """``customer`` (c_custkey 1..150k*SF, the domain of o_custkey) in ``nfiles`` files —
    the third table of the TPC-H Q3 three-way join."""
    n = int(CUSTOMERS_PER_SF * sf)
    out_dir = os.path.join(root, "customer")
    os.makedirs(out_dir, exist_ok=True)
    for i in range(nfiles):
        path = os.path.join(out_dir, f"part-{i:05d}.parquet")
        if os.path.exists(path):
            continue
        lo, hi = n * i // nfiles, n * (i + 1) // nfiles
        rng = np.random.default_rng([seed, 10_000 + i])
        m = hi - lo
        t = pa.Table.from_arrays([
            pa.array(np.arange(lo + 1, hi + 1, dtype=np.int64)),
            pa.array(rng.integers(0, 25, m).astype(np.int32)),
            pa.array(np.round(rng.random(m) * 10_999 - 999, 2)),
            pa.array(SEGMENTS[rng.integers(0, 5, m)])], schema=CUSTOMER_SCHEMA)
        tmp = os.path.join(out_dir, f".tmp-{os.getpid()}-part-{i:05d}.parquet")
        pq.write_table(t, tmp, compression="snappy", row_group_size=1 << 20)
        os.replace(tmp, path)
    return n
