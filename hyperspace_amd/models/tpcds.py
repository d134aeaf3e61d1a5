"""Synthetic TPC-DS-shaped tables for BASELINE config #5 (incremental refresh + a three-way
star join): ``store_sales`` (fact), ``item`` and ``date_dim`` (dimensions).

No dsdgen offline, so the tables are generated with numpy following the TPC-DS column domains
and row counts:

* ``date_dim``: 73,049 days from 1900-01-02, ``d_date_sk`` = 2,415,022 + day (the spec's
  surrogate keys), with ``d_year`` / ``d_moy`` / ``d_dom`` / ``d_qoy`` / ``d_dow``;
* ``item``: rows by the spec's scale table (18k at SF1 ... 264k at SF300, 300k at SF1000),
  ``i_manufact_id`` in [1, 1000], ``i_brand_id`` = 1,001,001 + ..., ``i_category_id`` in [1, 10];
* ``store_sales``: 2,880,404 * SF rows (864M at SF300), sold dates in the spec's sales window
  [1998-01-02, 2003-01-02], item keys uniform over ``item``, quantity in [1, 100], list/sales
  prices with two decimals, ``ss_ext_sales_price`` = quantity * sales price.

Foreign keys are null-free (dsdgen leaves ~4% of them null; the device join paths handle null
keys, but the oracle here stays exact and simple).  Generation is embarrassingly parallel: fact
file ``i`` is seeded by ``(seed, i)``; ``write_store_sales_files(..., first=k)`` appends files
``k..`` (new rows for an incremental refresh) without touching existing ones.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

DATE_SK0 = 2_415_022               # d_date_sk of 1900-01-02
DATE_ROWS = 73_049
SALES_LO = DATE_SK0 + (datetime.date(1998, 1, 2) - datetime.date(1900, 1, 2)).days
SALES_HI = DATE_SK0 + (datetime.date(2003, 1, 2) - datetime.date(1900, 1, 2)).days
STORE_SALES_PER_SF = 2_880_404
_ITEM_ROWS = ((1, 18_000), (10, 102_000), (100, 204_000), (300, 264_000), (1000, 300_000))

STORE_SALES_SCHEMA = pa.schema([
    ("ss_sold_date_sk", pa.int64()), ("ss_item_sk", pa.int64()), ("ss_customer_sk", pa.int64()),
    ("ss_store_sk", pa.int32()), ("ss_quantity", pa.int32()), ("ss_list_price", pa.float64()),
    ("ss_sales_price", pa.float64()), ("ss_ext_sales_price", pa.float64()),
    ("ss_net_profit", pa.float64())])
ITEM_SCHEMA = pa.schema([
    ("i_item_sk", pa.int64()), ("i_brand_id", pa.int32()), ("i_class_id", pa.int32()),
    ("i_category_id", pa.int32()), ("i_manufact_id", pa.int32()),
    ("i_current_price", pa.float64())])
DATE_SCHEMA = pa.schema([
    ("d_date_sk", pa.int64()), ("d_date", pa.date32()), ("d_year", pa.int32()),
    ("d_moy", pa.int32()), ("d_dom", pa.int32()), ("d_qoy", pa.int32()), ("d_dow", pa.int32())])


def item_rows(sf: float) -> int:
    """Item rows at scale ``sf`` (log-linear between the spec's table points; tiny SFs keep a
    floor so every manufacturer has items)."""
    pts = _ITEM_ROWS
    if sf <= pts[0][0]:
        return max(2_000, int(pts[0][1] * sf))
    for (s0, n0), (s1, n1) in zip(pts, pts[1:]):
        if sf <= s1:
            w = (np.log(sf) - np.log(s0)) / (np.log(s1) - np.log(s0))
            return int(round(n0 + w * (n1 - n0)))
    return pts[-1][1]


def store_sales_rows(sf: float) -> int:
    return int(STORE_SALES_PER_SF * sf)


def date_dim() -> pa.Table:
    day = np.arange(DATE_ROWS, dtype=np.int64)
    dates = np.datetime64("1900-01-02") + day.astype("timedelta64[D]")
    y = dates.astype("datetime64[Y]").astype(np.int64) + 1970
    m = (dates.astype("datetime64[M]").astype(np.int64) % 12) + 1
    dom = (dates - dates.astype("datetime64[M]")).astype(np.int64) + 1
    epoch_days = dates.astype("datetime64[D]").astype(np.int64)
    return pa.Table.from_arrays([
        pa.array(DATE_SK0 + day), pa.array(epoch_days.astype(np.int32)).view(pa.date32()),
        pa.array(y.astype(np.int32)), pa.array(m.astype(np.int32)),
        pa.array(dom.astype(np.int32)), pa.array(((m - 1) // 3 + 1).astype(np.int32)),
        pa.array(((epoch_days + 4) % 7).astype(np.int32))], schema=DATE_SCHEMA)


def item(sf: float, seed: int = 42) -> pa.Table:
    n = item_rows(sf)
    rng = np.random.default_rng([seed, 7])
    cat = rng.integers(1, 11, n).astype(np.int32)
    cls = rng.integers(1, 17, n).astype(np.int32)
    return pa.Table.from_arrays([
        pa.array(np.arange(1, n + 1, dtype=np.int64)),
        pa.array((1_001_001 + cat.astype(np.int64) * 1000 + rng.integers(0, 10, n)).astype(np.int32)),
        pa.array(cls), pa.array(cat),
        pa.array(rng.integers(1, 1001, n).astype(np.int32)),
        pa.array(np.round(rng.random(n) * 99 + 0.09, 2))], schema=ITEM_SCHEMA)


def store_sales_chunk(sf: float, nfiles: int, i: int, seed: int = 42) -> pa.Table:
    """Fact file ``i`` of ``nfiles`` (files past ``nfiles`` are appended data of the same
    size and domains)."""
    total = store_sales_rows(sf)
    n = total // nfiles + (1 if i < total % nfiles else 0)
    rng = np.random.default_rng([seed, 1_000 + i])
    items = item_rows(sf)
    qty = rng.integers(1, 101, n).astype(np.int32)
    lp = np.round(rng.random(n) * 199 + 1.0, 2)
    sp = np.round(lp * rng.integers(20, 101, n) / 100.0, 2)
    ext = np.round(qty * sp, 2)
    cost = np.round(lp * rng.integers(10, 81, n) / 100.0, 2)
    return pa.Table.from_arrays([
        pa.array(rng.integers(SALES_LO, SALES_HI + 1, n).astype(np.int64)),
        pa.array(rng.integers(1, items + 1, n).astype(np.int64)),
        pa.array(rng.integers(1, int(100_000 * max(sf, 1.0) ** 0.7) + 1, n).astype(np.int64)),
        pa.array(rng.integers(1, 1 + max(12, int(sf * 4)), n).astype(np.int32)),
        pa.array(qty), pa.array(lp), pa.array(sp), pa.array(ext),
        pa.array(np.round(ext - qty * cost, 2))], schema=STORE_SALES_SCHEMA)


def _write(t: pa.Table, path: str, row_group: int = 1 << 20) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = os.path.join(os.path.dirname(path), f".tmp-{os.getpid()}-{os.path.basename(path)}")
    pq.write_table(t, tmp, compression="snappy", row_group_size=row_group)
    os.replace(tmp, path)


def _ss_file(args) -> int:
    root, sf, nfiles, i, seed = args
    path = os.path.join(root, "store_sales", f"part-{i:05d}.parquet")
    if os.path.exists(path):
        return pq.ParquetFile(path).metadata.num_rows
    t = store_sales_chunk(sf, nfiles, i, seed)
    _write(t, path)
    return t.num_rows


def write_store_sales_files(root: str, sf: float, nfiles: int, first: int = 0,
                            count: Optional[int] = None, workers: int = 8,
                            seed: int = 42) -> int:
    """Write fact files ``first .. first + count`` (default: the ``nfiles`` base files);
    idempotent per file.  Returns the rows written (or already present)."""
    count = nfiles - first if count is None else count
    todo = [(root, sf, nfiles, i, seed) for i in range(first, first + count)]
    if workers <= 1 or len(todo) <= 1:
        return sum(_ss_file(a) for a in todo)
    import multiprocessing as mp
    with mp.get_context("fork").Pool(processes=min(workers, len(todo))) as pool:
        return sum(pool.map(_ss_file, todo, chunksize=1))


def generate(root: str, sf: float, nfiles: int, workers: int = 8, seed: int = 42) -> None:
    """``store_sales`` (``nfiles`` files), ``item`` and ``date_dim`` under ``root``."""
    for name, make in (("item", lambda: item(sf, seed)), ("date_dim", date_dim)):
        path = os.path.join(root, name, "part-00000.parquet")
        if not os.path.exists(path):
            _write(make(), path)
    write_store_sales_files(root, sf, nfiles, workers=workers, seed=seed)
