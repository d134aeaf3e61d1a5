"""Numerics of every HIP kernel against a host reference (pyarrow / numpy / the Spark-compatible
Murmur3 oracle).  GPU-only."""
import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pytest

from hyperspace_amd.utils import murmur3

pytestmark = pytest.mark.gpu


def _col(arr, device, raw=False):
    from hyperspace_amd.exec.device_table import DeviceColumn
    return DeviceColumn.from_arrow(arr, device, raw_strings=raw)


def test_murmur3_bucket_matches_spark_oracle(device):
    from hyperspace_amd.ops import kernels as K
    rng = np.random.default_rng(1)
    n = 100_003
    i32 = pa.array(rng.integers(-2**31, 2**31 - 1, n).astype(np.int32),
                   mask=rng.random(n) < 0.05)
    i64 = pa.array(rng.integers(-2**62, 2**62, n).astype(np.int64))
    f64 = pa.array(np.where(rng.random(n) < 0.01, -0.0, rng.normal(size=n)))
    f32 = pa.array(rng.normal(size=n).astype(np.float32))
    s = pa.array([("k%d" % v) * (v % 5) for v in rng.integers(0, 1000, n)],
                 mask=rng.random(n) < 0.03)
    d = pa.array(rng.integers(0, 20000, n).astype(np.int32)).view(pa.date32())
    for cols in ([i32], [i64], [f64], [f32], [s], [d], [i64, s, f64], [s, i32]):
        dcols = [_col(c, device, raw=True) for c in cols]
        for nb in (1, 7, 200, 20000):
            b, counts = K.murmur3_bucket(dcols, nb)
            ref = murmur3.bucket_ids(cols, nb)
            got = b.cpu().numpy()
            assert np.array_equal(got, ref), (cols[0].type, nb)
            assert np.array_equal(counts.cpu().numpy(), np.bincount(ref, minlength=nb))
    # golden vectors (BucketUnionTest.scala:101-122)
    b, _ = K.murmur3_bucket([_col(pa.array([2, 3], pa.int32()), device)], 10)
    assert b.cpu().tolist() == [4, 1]


def test_murmur3_bucket_decimal_and_timestamp_match_host(device):
    """Device bucket ids equal the host/Spark hash for decimals (unscaled long from float64
    storage) and timestamps in every unit (microseconds, floor for ns)."""
    import decimal
    from hyperspace_amd.ops import kernels as K
    rng = np.random.default_rng(5)
    n = 50_000
    dec = pa.array([decimal.Decimal(int(v)).scaleb(-2) for v in rng.integers(-10**12, 10**12, n)],
                   pa.decimal128(15, 2))
    raw = rng.integers(-2**50, 2**50, n)
    cols = [dec, pa.array([decimal.Decimal("1.50"), decimal.Decimal("2.25"),
                           decimal.Decimal("100.00")], pa.decimal128(10, 2))]
    for unit in ("s", "ms", "us", "ns"):
        cols.append(pa.array(raw, pa.int64()).view(pa.timestamp(unit)))
    for c in cols:
        for nb in (200, 7):
            got = K.murmur3_bucket([_col(c, device)], nb)[0].cpu().numpy()
            assert np.array_equal(got, murmur3.bucket_ids([c], nb)), (c.type, nb)


def test_sort_permutation_stable_nulls_first(device):
    import torch
    from hyperspace_amd.ops import kernels as K
    rng = np.random.default_rng(2)
    n = 300_001
    a = rng.integers(-50, 50, n).astype(np.int64)
    amask = rng.random(n) < 0.02
    b = rng.normal(size=n)
    c = rng.integers(0, 2**31 - 1, n).astype(np.int32)
    bucket = rng.integers(0, 200, n).astype(np.int32)
    ca = _col(pa.array(a, mask=amask), device)
    cb = _col(pa.array(b), device)
    cc = _col(pa.array(c), device)
    perm = K.sort_permutation([ca, cb, cc],
                              extra_leading=(torch.from_numpy(bucket).to(device), 8)).cpu().numpy()
    # reference: lexsort (last key primary) - nulls first encoded via flag
    a_key = np.where(amask, np.iinfo(np.int64).min, a)
    a_flag = (~amask).astype(np.int8)
    ref = np.lexsort((np.arange(n), c, b, a_key, a_flag, bucket))
    assert np.array_equal(perm, ref)


def test_gather_and_scan_agg_q6_shape(device):
    import torch
    from hyperspace_amd.ops import _lib as NL, kernels as K
    rng = np.random.default_rng(3)
    B = 16
    per = rng.integers(1000, 40000, B)
    n = int(per.sum())
    ship = np.concatenate([np.sort(rng.integers(8000, 10500, k)) for k in per]).astype(np.int32)
    disc = rng.integers(0, 11, n) / 100.0
    qty = rng.integers(1, 51, n).astype(np.float64)
    price = rng.random(n) * 1e5
    off = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
    cs, cd, cq, cp = (_col(pa.array(x), device) for x in (ship, disc, qty, price))
    boff = torch.from_numpy(off).to(device)
    lo, hi = 8766, 9131
    rstart, rlen, rb = K.range_search(cs, boff, lo=K.sortable_image(lo, NL.I32), lo_incl=True,
                                      hi=K.sortable_image(hi, NL.I32), hi_incl=False)
    tp = K.ranges_to_tiles(rlen)
    p = NL.ScanParams()
    for i, c in enumerate((cs, cd, cq, cp)):
        p.cols[i] = c.desc()
    p.preds[0] = NL.Pred(NL.PK_FLT_LIT, NL.OP_GE, 1, 0, 0, 0, 0, 0.05, None)
    p.preds[1] = NL.Pred(NL.PK_FLT_LIT, NL.OP_LE, 1, 0, 1, 0, 0, 0.07, None)
    p.preds[2] = NL.Pred(NL.PK_FLT_LIT, NL.OP_LT, 2, 0, 2, 0, 0, 24.0, None)
    p.npreds = 3
    a = NL.AggSpec()
    a.kind, a.nterms = NL.AK_SUM, 2
    a.col[0], a.col[1] = 3, 1
    a.alpha[0], a.alpha[1] = 0.0, 0.0
    a.beta[0], a.beta[1] = 1.0, 1.0
    p.aggs[0] = a
    p.naggs = 1
    p.group_col = -1
    s, c, mn, mx = K.scan_agg(p, rstart, rlen, tp)
    m = (ship >= lo) & (ship < hi) & (disc >= 0.05) & (disc <= 0.07) & (qty < 24)
    ref = float((price[m] * disc[m]).sum())
    assert int(c[0].item()) == int(m.sum())
    assert abs(float(s[0].item()) - ref) <= 1e-9 * max(1.0, abs(ref))
    # selection path
    rows = K.scan_select(p, rstart, rlen, tp, max_tiles=n // 2048 + B + 1).cpu().numpy()
    assert np.array_equal(rows, np.nonzero(m)[0])
    g = K.gather_columns([cp, cd], torch.from_numpy(rows).to(device))
    assert np.allclose(g[0].data.cpu().numpy(), price[rows])


def test_grouped_scan_agg(device):
    from hyperspace_amd.ops import _lib as NL, kernels as K
    rng = np.random.default_rng(4)
    n = 200_000
    g = rng.integers(0, 37, n).astype(np.int32)
    v = rng.random(n)
    cg, cv = _col(pa.array(g), device), _col(pa.array(v), device)
    rstart, rlen, _ = K.full_ranges(np.array([0, n], np.int64), device)
    tp = K.ranges_to_tiles(rlen)
    p = NL.ScanParams()
    p.cols[0], p.cols[1] = cg.desc(), cv.desc()
    p.npreds = 0
    for k, kind in enumerate((NL.AK_SUM, NL.AK_MIN, NL.AK_MAX, NL.AK_COUNT_STAR)):
        a = NL.AggSpec()
        a.kind = kind
        a.nterms = 0 if kind == NL.AK_COUNT_STAR else 1
        a.col[0], a.alpha[0], a.beta[0] = 1, 0.0, 1.0
        p.aggs[k] = a
    p.naggs = 4
    p.group_col, p.num_groups, p.group_base = 0, 37, 0
    s, c, mn, mx = K.scan_agg(p, rstart, rlen, tp)
    s, c, mn, mx = (x.cpu().numpy().reshape(37, 4) for x in (s, c, mn, mx))
    for grp in range(37):
        sel = v[g == grp]
        assert abs(s[grp, 0] - sel.sum()) < 1e-9 * max(1, sel.sum())
        assert mn[grp, 1] == sel.min() and mx[grp, 2] == sel.max()
        assert c[grp, 3] == len(sel)


def test_join_agg_and_pairs(device):
    import torch
    from hyperspace_amd.ops import _lib as NL, kernels as K
    rng = np.random.default_rng(5)
    B = 8
    # right: unique keys per bucket (orders), left: ~4 rows per key (lineitem)
    rk = np.arange(0, 60_000, dtype=np.int64) * 3
    rb = murmur3.bucket_ids([pa.array(rk)], B)
    lk = np.repeat(rk, rng.integers(1, 7, len(rk)))
    lk = np.concatenate([lk, rng.integers(0, 180_000, 5000)])  # some keys without a match
    lb = murmur3.bucket_ids([pa.array(lk)], B)
    ro = np.lexsort((rk, rb)); rk, rb = rk[ro], rb[ro]
    lo_ = np.lexsort((lk, lb)); lk, lb = lk[lo_], lb[lo_]
    rdate = rng.integers(0, 1000, len(rk)).astype(np.int32)
    lprice = rng.random(len(lk)) * 100
    ldisc = rng.integers(0, 11, len(lk)) / 100.0
    loff = np.searchsorted(lb, np.arange(B + 1)).astype(np.int64)
    roff = np.searchsorted(rb, np.arange(B + 1)).astype(np.int64)
    clk, clp, cld = (_col(pa.array(x), device) for x in (lk, lprice, ldisc))
    crk, crd = _col(pa.array(rk), device), _col(pa.array(rdate), device)
    p = NL.JoinParams()
    p.cols[0], p.cols[1], p.cols[2] = clk.desc(), clp.desc(), cld.desc()
    p.cols[8], p.cols[9] = crk.desc(), crd.desc()
    p.lkey, p.rkey = 0, 8
    p.preds[0] = NL.Pred(NL.PK_FLT_LIT, NL.OP_GT, 2, 0, 0, 0, 0, 0.02, None)   # left pred
    p.preds[1] = NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 9, 0, 1, 0, 500, 0.0, None)  # right pred
    p.nlp, p.npreds = 1, 2
    a = NL.AggSpec()
    a.kind, a.nterms = NL.AK_SUM, 2
    a.col[0], a.alpha[0], a.beta[0] = 1, 0.0, 1.0
    a.col[1], a.alpha[1], a.beta[1] = 2, 1.0, -1.0
    p.aggs[0] = a
    p.naggs, p.group_col, p.key_is_float = 1, -1, 0
    rstart, rlen, rbk = K.full_ranges(loff, device)
    mt = K.join_max_tiles(len(lk), B)
    s, c, _, _ = K.join_agg(p, rstart, rlen, rbk, torch.from_numpy(roff).to(device), mt)
    # reference
    rmap = {int(k): i for i, k in enumerate(rk)}
    tot, cnt, pairs = 0.0, 0, []
    for i, k in enumerate(lk):
        j = rmap.get(int(k))
        if j is None or not (ldisc[i] > 0.02) or not (rdate[j] < 500):
            continue
        tot += lprice[i] * (1 - ldisc[i])
        cnt += 1
        pairs.append((i, j))
    assert int(c[0].item()) == cnt
    assert abs(float(s[0].item()) - tot) < 1e-9 * tot
    ol, orr = K.join_pairs(p, rstart, rlen, rbk, torch.from_numpy(roff).to(device), mt)
    got = sorted(zip(ol.cpu().tolist(), orr.cpu().tolist()))
    assert got == sorted(pairs)


def test_join_many_to_many_with_nulls_and_wide_spans(device):
    """Duplicate right keys (match rounds > 1), null left keys (sorted first), a right span wider
    than the LDS stage (global binary-search fallback) and a grouped aggregate on a right column."""
    import torch
    from hyperspace_amd.ops import _lib as NL, kernels as K
    rng = np.random.default_rng(11)
    B = 4
    rk = np.concatenate([np.repeat(np.arange(0, 3000, dtype=np.int64), 3),   # 3 dups per key
                         np.arange(10_000, 100_000, dtype=np.int64)])          # dense: wide spans
    rb = murmur3.bucket_ids([pa.array(rk)], B)
    lk = np.concatenate([rng.integers(0, 3000, 20_000), rng.integers(10_000, 100_000, 20_000)])
    lb = murmur3.bucket_ids([pa.array(lk)], B)
    ro = np.lexsort((rk, rb)); rk, rb = rk[ro], rb[ro]
    lo_ = np.lexsort((lk, lb)); lk, lb = lk[lo_], lb[lo_]
    lnull = np.zeros(len(lk), bool)
    # null keys must sit at the start of each bucket (nulls-first sort); null out the first 5
    loff = np.searchsorted(lb, np.arange(B + 1)).astype(np.int64)
    for b in range(B):
        lnull[loff[b]:loff[b] + 5] = True
    roff = np.searchsorted(rb, np.arange(B + 1)).astype(np.int64)
    rgrp = rng.integers(0, 5, len(rk)).astype(np.int32)
    lval = rng.random(len(lk))
    clk = _col(pa.array(lk, mask=lnull), device)
    clv = _col(pa.array(lval), device)
    crk, crg = _col(pa.array(rk), device), _col(pa.array(rgrp), device)
    p = NL.JoinParams()
    p.cols[0], p.cols[1] = clk.desc(), clv.desc()
    p.cols[8], p.cols[9] = crk.desc(), crg.desc()
    p.lkey, p.rkey = 0, 8
    p.nlp, p.npreds = 0, 0
    a = NL.AggSpec()
    a.kind, a.nterms = NL.AK_SUM, 1
    a.col[0], a.alpha[0], a.beta[0] = 1, 0.0, 1.0
    p.aggs[0] = a
    p.naggs, p.key_is_float = 1, 0
    p.group_col, p.num_groups, p.group_base = 9, 5, 0
    rstart, rlen, rbk = K.full_ranges(loff, device)
    mt = K.join_max_tiles(len(lk), B)
    roff_t = torch.from_numpy(roff).to(device)
    s, c, _, _ = K.join_agg(p, rstart, rlen, rbk, roff_t, mt)
    from collections import defaultdict
    rpos = defaultdict(list)
    for j, k in enumerate(rk):
        rpos[int(k)].append(j)
    exp_s, exp_c, pairs = np.zeros(5), np.zeros(5, np.int64), []
    for i, k in enumerate(lk):
        if lnull[i]:
            continue
        for j in rpos.get(int(k), []):
            exp_s[rgrp[j]] += lval[i]
            exp_c[rgrp[j]] += 1
            pairs.append((i, j))
    assert c.cpu().numpy().tolist() == exp_c.tolist()
    np.testing.assert_allclose(s.cpu().numpy(), exp_s, rtol=1e-9)
    ol, orr = K.join_pairs(p, rstart, rlen, rbk, roff_t, mt)
    assert sorted(zip(ol.cpu().tolist(), orr.cpu().tolist())) == sorted(pairs)
    # generated kernels (sampled span search + galloping, LDS stage or global fallback),
    # with and without the software-pipelined tile loop / right-column staging
    from hyperspace_amd.exec import jit
    from hyperspace_amd.exec import kernel_config
    for pipe in (True, False):
        for stage in (True, False):
            with kernel_config.use(join_pipeline=pipe, join_stage_right=stage):
                js, jc, _, _ = jit.join_agg(p, rstart, rlen, rbk, roff_t, mt)
                assert jc.cpu().numpy().tolist() == exp_c.tolist(), (pipe, stage)
                np.testing.assert_allclose(js.cpu().numpy(), exp_s, rtol=1e-9)


@pytest.mark.parametrize("world", [1, 3, 8, 64])
def test_packed_exchange_kernel_matches_reference(device, world):
    """hs_xch_pack writes the exact byte layout of the numpy oracle (stable per-destination
    segments, 16-byte aligned column runs) and hs_xch_unpack restores the columns."""
    import ctypes as C
    import torch
    from hyperspace_amd.ops import _lib as NL
    from hyperspace_amd.parallel.exchange import pack_reference, segment_bytes
    rng = np.random.default_rng(world)
    n = 3 * 4096 + 77
    bucket = rng.integers(0, 200, n).astype(np.int32)
    cols = [rng.integers(-2**62, 2**62, n).astype(np.int64), rng.random(n).astype(np.float32),
            rng.integers(0, 2, n).astype(np.uint8), rng.integers(0, 9, n).astype(np.int16), bucket]
    ref, counts, lay = pack_reference(cols, bucket, world)
    dcols = [torch.from_numpy(c).to(device) for c in cols]
    L = NL.lib()
    ntiles = (n + L.hs_xch_tile_rows() - 1) // L.hs_xch_tile_rows()
    tile = torch.empty(ntiles * world, dtype=torch.int64, device=device)
    meta = torch.zeros(2 * world + world * (len(cols) + 1), dtype=torch.int64, device=device)
    send = torch.zeros(n * sum(c.dtype.itemsize for c in cols) + 16 * world * len(cols),
                       dtype=torch.uint8, device=device)
    p = NL.XchParams()
    for i, c in enumerate(dcols):
        p.src[i] = c.data_ptr()
        p.elem_bytes[i] = c.element_size()
    p.ncols, p.world = len(cols), world
    NL.check(L.hs_xch_pack(C.byref(p), NL.ptr(dcols[-1]), n, NL.ptr(tile), NL.ptr(meta),
                           NL.ptr(send), NL.stream_ptr()), "pack")
    m = meta.cpu().numpy()
    assert np.array_equal(m[:world], counts)
    assert np.array_equal(m[2 * world:].reshape(world, -1), lay)
    got = send.cpu().numpy()[:len(ref)]
    # compare only the value bytes (alignment padding is unspecified)
    for d in range(world):
        for ci, c in enumerate(cols):
            o, k = int(lay[d, ci]), int(counts[d]) * c.dtype.itemsize
            assert np.array_equal(got[o:o + k], ref[o:o + k]), (d, ci)
    # unpack through the exchange's copy table (world-1 local "exchange")
    from hyperspace_amd.parallel.exchange import RowExchange
    if world == 1:
        ex = RowExchange(None, [c.dtype for c in dcols], device)
        ex.add(dcols, dcols[-1])
        outs = ex.finish()
        for o, c in zip(outs, cols):
            assert np.array_equal(o.cpu().numpy(), c)
    assert segment_bytes(int(counts[0]), [c.dtype.itemsize for c in cols]) == \
        int(lay[0, -1] - lay[0, 0])


def test_histogram_kernel(device):
    import torch
    from hyperspace_amd.ops import kernels as K
    rng = np.random.default_rng(2)
    for B in (1, 200, 16384):
        ids = rng.integers(0, B, 1_000_003).astype(np.int32)
        got = K.histogram(torch.from_numpy(ids).to(device), B).cpu().numpy()
        assert np.array_equal(got, np.bincount(ids, minlength=B))


@pytest.mark.parametrize("runs_per_bucket", [2, 3, 7])
def test_merge_runs_permutation_equals_stable_sort(device, runs_per_bucket):
    """K6 merge path: buckets made of sorted runs (ties across runs, nulls, a two-column key,
    empty runs) merge to exactly the stable (bucket, keys) sort permutation."""
    import torch
    from hyperspace_amd.ops import kernels as K
    rng = np.random.default_rng(runs_per_bucket)
    parts_a, parts_b, masks, off, grp = [], [], [], [0], []
    for bkt in range(37):
        for r in range(runs_per_bucket):
            m = int(rng.integers(0, 5000)) if (bkt + r) % 11 else 0
            a = rng.integers(-300, 300, m).astype(np.int64)
            b = rng.integers(0, 1000, m).astype(np.int32)
            mask = rng.random(m) < 0.03
            key = np.where(mask, np.iinfo(np.int64).min, a)
            o = np.lexsort((b, key, (~mask).astype(np.int8)))   # a sorted run, nulls first
            parts_a.append(a[o]); parts_b.append(b[o]); masks.append(mask[o])
            off.append(off[-1] + m)
            grp.append(bkt)
    a, b, mask = np.concatenate(parts_a), np.concatenate(parts_b), np.concatenate(masks)
    n = len(a)
    ca = _col(pa.array(a, mask=mask), device)
    cb = _col(pa.array(b), device)
    bucket = np.repeat(np.asarray(grp, np.int32), np.diff(off))
    perm = K.merge_runs_permutation([ca, cb], np.asarray(off), np.asarray(grp))
    assert perm is not None
    ref = K.sort_permutation([ca, cb], extra_leading=(torch.from_numpy(bucket).to(device), 8))
    assert np.array_equal(perm.cpu().numpy(), ref.cpu().numpy()), n
    # unsorted runs are detected: the caller falls back to the radix sort
    bad = _col(pa.array(rng.integers(0, 100, n).astype(np.int64)), device)
    assert K.merge_runs_permutation([bad], np.asarray(off), np.asarray(grp)) is None


@pytest.mark.parametrize("idx_bits", [32, 64])
def test_packed_row_gather_matches_per_column_gather(device, idx_bits):
    """Permutations of large tables through packed records (hs_gather_packed, HS_GATHER_PACKED=1):
    1-, 2-, 4- and 8-byte columns with and without validity give exactly what the per-column
    gather and torch indexing give."""
    import os
    import torch
    from hyperspace_amd.exec.device_table import DeviceColumn
    from hyperspace_amd.ops import kernels as K
    n = (1 << 20) + 4097
    g = torch.Generator(device=device)
    g.manual_seed(3)
    cols = [DeviceColumn(torch.randint(-2**62, 2**62, (n,), device=device, generator=g),
                         None, pa.int64()),
            DeviceColumn(torch.rand(n, device=device, dtype=torch.float64, generator=g),
                         (torch.rand(n, device=device, generator=g) < 0.9).to(torch.uint8),
                         pa.float64()),
            DeviceColumn(torch.randint(0, 2**31 - 1, (n,), device=device, generator=g)
                         .to(torch.int32), None, pa.int32()),
            DeviceColumn(torch.randint(0, 30000, (n,), device=device, generator=g)
                         .to(torch.int16), None, pa.int16()),
            DeviceColumn(torch.randint(0, 2, (n,), device=device, generator=g).to(torch.uint8),
                         (torch.rand(n, device=device, generator=g) < 0.5).to(torch.uint8),
                         pa.bool_())]
    perm = torch.randperm(n, device=device, generator=g)[: n - 1000]
    idx = perm.to(torch.int32 if idx_bits == 32 else torch.int64)
    lay = K._packed_layout(cols, True)
    assert lay is not None and lay[0] == 32
    ref = K.gather_columns(cols, idx)
    os.environ["HS_GATHER_PACKED"] = "1"
    try:
        got = K.gather_columns(cols, idx)
    finally:
        os.environ.pop("HS_GATHER_PACKED")
    for c, a, b in zip(cols, got, ref):
        assert torch.equal(a.data, b.data) and torch.equal(a.data, c.data[perm])
        if c.valid is None:
            assert a.valid is None and b.valid is None
        else:
            assert torch.equal(a.valid, b.valid) and torch.equal(a.valid, c.valid[perm])
