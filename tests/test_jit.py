"""Whole-stage codegen (exec/jit.py + csrc/runtime/hs_jit.cpp).

CPU tier: the generated sources for representative shapes compile for gfx950 with hipRTC (no GPU
needed).  GPU tier: generated kernels agree with the AOT interpreter kernels and a numpy fp64
reference on the same inputs (nulls, OR groups, IN sets, grouped min/max, joins with duplicates).
"""
import os

import numpy as np
import pyarrow as pa
import pytest

from hyperspace_amd.ops import _lib as NL
from hyperspace_amd.utils import murmur3


def _agg(kind, terms=()):
    a = NL.AggSpec()
    a.kind, a.nterms = kind, len(terms)
    for t, (c, al, be) in enumerate(terms):
        a.col[t], a.alpha[t], a.beta[t] = c, al, be
    return a


def _scan_params(descs, preds, aggs, group_col=-1, num_groups=1, group_base=0):
    p = NL.ScanParams()
    for s, d in descs.items():
        p.cols[s] = d
    for i, pr in enumerate(preds):
        p.preds[i] = pr
    p.npreds = len(preds)
    for i, a in enumerate(aggs):
        p.aggs[i] = a
    p.naggs = len(aggs)
    p.group_col, p.num_groups, p.group_base = group_col, num_groups, group_base
    return p


def _fake(t, valid=False):
    return NL.ColDesc(0x1000, 0x2000 if valid else 0, t, 0)


@pytest.fixture(scope="module")
def rt():
    import os
    from hyperspace_amd.exec import jit
    if not os.path.exists(jit.RUNTIME_PATH):
        pytest.skip("runtime library not built")
    return jit


def test_generated_sources_compile(rt, tmp_path):
    jit = rt
    cases = []
    cases.append(_scan_params(
        {0: _fake(NL.I32), 1: _fake(NL.F64), 2: _fake(NL.F64, True), 3: _fake(NL.F64)},
        [NL.Pred(NL.PK_FLT_LIT, NL.OP_GE, 1, 0, 0, 0, 0, 0.05, None),
         NL.Pred(NL.PK_FLT_LIT, NL.OP_LT, 2, 0, 1, 0, 0, 24.0, None),
         NL.Pred(NL.PK_INT_LIT, NL.OP_EQ, 0, 0, 2, 0, 7, 0.0, None),
         NL.Pred(NL.PK_IN_SET, NL.OP_NE, 0, 0, 2, 3, 0, 0.0, 0x5000)],
        [_agg(NL.AK_SUM, [(3, 0.0, 1.0), (1, 1.0, -1.0)]), _agg(NL.AK_COUNT_STAR)]))
    cases.append(_scan_params(
        {0: _fake(NL.I64, True), 1: _fake(NL.F32), 2: _fake(NL.BOOL)},
        [NL.Pred(NL.PK_IS_NULL, 0, 0, 0, 0, 0, 0, 0.0, None),
         NL.Pred(NL.PK_INT_COL, NL.OP_LT, 0, 2, 0, 0, 0, 0.0, None),
         NL.Pred(NL.PK_BITMAP, NL.OP_NE, 0, 0, 1, 4, 0, 0.0, 0x6000)],
        [_agg(NL.AK_MIN, [(1, 0.0, 1.0)]), _agg(NL.AK_MAX, [(1, 0.0, 2.0)]),
         _agg(NL.AK_COUNT, [(0, 0.0, 1.0)])], group_col=2, num_groups=2))
    for p in cases:
        for vec in (0, 8, 16):
            k = jit.gen_scan_agg(p, vec=vec)
            rc = jit.runtime().hs_jit_compile_to_cache(k.src.encode(), k.name.encode(),
                                                       b"gfx950", str(tmp_path).encode())
            assert rc == 0, jit.runtime().hs_jit_last_error().decode()
    j = NL.JoinParams()
    j.cols[0], j.cols[1], j.cols[2] = _fake(NL.I64), _fake(NL.I32), _fake(NL.F64, True)
    j.cols[8], j.cols[9], j.cols[10] = _fake(NL.I64), _fake(NL.I32), _fake(NL.I32, True)
    j.preds[0] = NL.Pred(NL.PK_INT_LIT, NL.OP_GT, 1, 0, 0, 0, 9000, 0.0, None)
    j.preds[1] = NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 9, 0, 1000, 0, 9000, 0.0, None)
    j.preds[2] = NL.Pred(NL.PK_INT_COL, NL.OP_LT, 1, 9, 1001, 0, 0, 0.0, None)
    j.nlp, j.npreds = 1, 3
    j.aggs[0] = _agg(NL.AK_SUM, [(2, 0.0, 1.0), (2, 1.0, -1.0)])
    j.aggs[1] = _agg(NL.AK_COUNT_STAR)
    j.naggs, j.lkey, j.rkey = 2, 0, 8
    for g, fl in ((-1, 0), (10, 0), (-1, 1)):
        j.group_col, j.num_groups, j.key_is_float = g, 3, fl
        ks = [jit.gen_join_agg(j), jit.gen_merge_join_agg(j)]
        if not fl:
            ks += [jit.gen_join_index_agg(j), jit.gen_join_index_agg(j, vec=4),
                   jit.gen_join_index_agg(j, vec=8, jw=1, jlog=7),
                   jit.gen_join_index_agg(j, vec=16, jw=1, jlog=7),
                   jit.gen_join_index_agg(j, jw=2, jlog=8)]
        for k in ks:
            rc = jit.runtime().hs_jit_compile_to_cache(k.src.encode(), k.name.encode(),
                                                       b"gfx950", str(tmp_path).encode())
            assert rc == 0, jit.runtime().hs_jit_last_error().decode()


def _decode(c):
    import torch
    v = c.codes.long() + c.base
    return v.double() / c.scale if c.scale else v


def test_hbm_encoding_round_trip_cpu():
    import torch
    from hyperspace_amd.exec.device_table import DeviceColumn
    from hyperspace_amd.exec.encoding import encode
    rng = np.random.default_rng(2)
    # int64 keys with a large base -> 4-byte FOR
    k = torch.from_numpy(rng.integers(10**12, 10**12 + 3_000_000_000, 5000))
    c = encode(DeviceColumn(k, None, pa.int64()))
    assert c.width == 4 and c.scale is None and torch.equal(_decode(c), k)
    # dates -> 2 bytes
    d = torch.from_numpy(rng.integers(8000, 10600, 5000).astype(np.int32))
    c = encode(DeviceColumn(d, None, pa.date32()))
    assert c.width == 2 and torch.equal(_decode(c), d.long())
    # TPC-H style decimals: discount 0.00..0.10 -> 1 byte, prices (2 digits) -> 4 bytes
    disc = torch.from_numpy(rng.integers(0, 11, 5000) / 100.0)
    c = encode(DeviceColumn(disc, None, pa.float64()))
    assert c.width == 1 and c.scale == 100.0
    assert torch.equal(_decode(c).view(torch.int64), disc.view(torch.int64))
    price = torch.from_numpy(np.round(rng.random(5000) * 1e5, 2))
    c = encode(DeviceColumn(price, None, pa.float64()))
    assert c.width == 4 and torch.equal(_decode(c).view(torch.int64), price.view(torch.int64))
    # arbitrary doubles and wide ranges stay uncompressed
    assert encode(DeviceColumn(torch.from_numpy(rng.random(100)), None, pa.float64())) is None
    assert encode(DeviceColumn(torch.tensor([0, 2**40], dtype=torch.int64), None, pa.int64())) is None
    # nulls: masked slots do not widen the range
    vals = torch.tensor([5, 0, 7, 6], dtype=torch.int64)
    valid = torch.tensor([1, 0, 1, 1], dtype=torch.uint8)
    c = encode(DeviceColumn(vals, valid, pa.int64()))
    assert c.width == 1
    dec = _decode(c)
    assert dec[0] == 5 and dec[2] == 7 and dec[3] == 6
    # -0.0 is not representable as a scaled integer bit-exactly
    assert encode(DeviceColumn(torch.tensor([-0.0, 1.0]), None, pa.float64())) is None


def test_generated_sources_compile_with_compact_columns(rt, tmp_path):
    from hyperspace_amd.exec.encoding import Compact
    jit = rt
    p = _scan_params({0: _fake(NL.F64), 1: _fake(NL.F64), 2: _fake(NL.I64, True)},
                     [NL.Pred(NL.PK_FLT_LIT, NL.OP_GE, 0, 0, 0, 0, 0, 0.05, None),
                      NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 2, 0, 1, 0, 9, 0.0, None)],
                     [_agg(NL.AK_SUM, [(1, 0.0, 1.0), (0, 1.0, -1.0)])])
    comp = {0: Compact(None, 1, 0, 100.0, NL.F64), 1: Compact(None, 4, 0, 100.0, NL.F64),
            2: Compact(None, 2, 5, None, NL.I64)}
    k = jit.gen_scan_agg(p, comp)
    # slot 0: its literal predicate runs on the stored codes (CL0/CH0), its SUM term decodes
    # with a reciprocal (R0); no exact division left for it
    assert "a.CL0" in k.src and "a.R0" in k.src and "a.Q0" not in k.src
    assert "a.CL1" in k.src and "a.L1" not in k.src    # integer compact column: code bounds
    assert "const signed char* c0" in k.src
    rc = jit.runtime().hs_jit_compile_to_cache(k.src.encode(), k.name.encode(), b"gfx950",
                                               str(tmp_path).encode())
    assert rc == 0, jit.runtime().hs_jit_last_error().decode()
    assert jit.scan_agg_shape(p, comp) != jit.scan_agg_shape(p, None)
    j = NL.JoinParams()
    j.cols[0], j.cols[1] = _fake(NL.I64), _fake(NL.F64)
    j.cols[8], j.cols[9] = _fake(NL.I64), _fake(NL.I32)
    j.preds[0] = NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 9, 0, 1000, 0, 9000, 0.0, None)
    j.nlp, j.npreds = 0, 1
    j.aggs[0] = _agg(NL.AK_SUM, [(1, 0.0, 1.0)])
    j.naggs, j.lkey, j.rkey, j.group_col = 1, 0, 8, -1
    comp = {0: Compact(None, 4, 1, None, NL.I64), 8: Compact(None, 4, 1, None, NL.I64),
            9: Compact(None, 2, 8000, None, NL.I32), 1: Compact(None, 4, 0, 100.0, NL.F64)}
    k = jit.gen_join_agg(j, comp)
    rc = jit.runtime().hs_jit_compile_to_cache(k.src.encode(), k.name.encode(), b"gfx950",
                                               str(tmp_path).encode())
    assert rc == 0, jit.runtime().hs_jit_last_error().decode()
    ks = [q3_join_index_kernel(jit, stage=True), q3_join_index_kernel(jit, bitmap=True),
          q3_join_index_kernel(jit, vec=0, bitmap=True), q3_bitmap_kernel(jit),
          jit.gen_merge_join_agg(_q3_params(), _q3_compacts())]
    c32 = dict(_q3_compacts())
    c32[0] = Compact(None, 4, 1 + (1 << 31), None, NL.I64, 1, 600_000_000)
    c32[8] = Compact(None, 4, 1 + (1 << 31), None, NL.I64, 1, 600_000_000)
    k32 = jit.gen_merge_join_agg(_q3_params(), c32)
    assert "unsigned skeys" in k32.src and "a.KOF" in k32.src    # 32-bit merge images
    assert "u64 skeys" in ks[-1].src
    ks.append(k32)
    from hyperspace_amd.exec.encoding import GroupedCompact
    c16 = dict(c32)
    c16[0] = GroupedCompact(None, None, None, 1 + (1 << 31), NL.I64, 1, 600_000_000)
    k16 = jit.gen_merge_join_agg(_q3_params(), c16)
    assert "const unsigned short* c0" in k16.src and "a.G0[" in k16.src   # 16-bit left keys
    assert jit.merge_join_shape(_q3_params(), c16) != jit.merge_join_shape(_q3_params(), c32)
    ks.append(k16)
    import torch
    from hyperspace_amd.exec.encoding import RunCompact
    cr = dict(c32)
    cr[0] = RunCompact(c32[0], torch.zeros(1, dtype=torch.int32), torch.zeros(1, dtype=torch.int64),
                       torch.zeros(1, dtype=torch.int32))
    kr = jit.gen_merge_join_agg(_q3_params(), cr)
    # run-keyed merge join: per-row run lookups, no per-row key stream of slot 0
    assert "a.GM0[" in kr.src and "a.RK0[" in kr.src and "lrk_[" in kr.src
    assert "vload<int, 8>(a.c0" not in kr.src and "a.rdup" not in kr.src
    assert jit.merge_join_shape(_q3_params(), cr) != jit.merge_join_shape(_q3_params(), c32)
    ks.append(kr)
    # two-phase form (exec/jit_runs.py): run tags, then the left scan with the tag test
    from hyperspace_amd.exec import jit_runs
    q3 = _q3_params()
    assert jit_runs.applies(q3) and jit_runs.tag_width(q3) == 1
    for g, G, W in ((-1, 1, 1), (10, 1, 1), (10, 3, 2), (10, 200, 8), (1, 4, 1)):
        q3.group_col, q3.num_groups = g, G
        if g == 10:
            q3.cols[10] = _fake(NL.I32)
        assert jit_runs.tag_width(q3) == W
        kt = jit_runs.gen_run_tags2(q3, cr, W)
        kq = jit_runs.gen_run_scan(q3, cr, W, 16)
        assert "a.RNG" in kt.src and "a.RK0[" in kt.src and "a.c2" not in kt.src
        assert "a.GM0[" in kq.src and "a.tags[w0_" in kq.src and "a.c8" not in kq.src
        ks += [kt, kq]
        # recorded-match phase 1: the verifying form stores the match, the match form reads it
        # (no run keys, no right key images, no range table)
        kr_ = jit_runs.gen_run_tags2(q3, cr, W, True, "rec")
        km = jit_runs.gen_run_tags2(q3, cr, W, True, "match")
        assert "a.MOUT[" in kr_.src and "a.MATCH[" in km.src
        assert "a.RK0[" not in km.src and "a.RNG" not in km.src and "a.c8" not in km.src
        # copy form: hit bits and run-order copies of the right columns, nothing at right rows
        klo = jit_runs.gen_run_tags2(q3, cr, W, True, "lo16")
        kpr = jit_runs.gen_run_tags2(q3, cr, W, True, "lo16prep")
        assert "a.LL[act" in klo.src and "cl0" in klo.src and "a.RL[i] =" in kpr.src
        ks += [klo, kpr]
        kc = jit_runs.gen_run_tags2(q3, cr, W, True, "copy")
        kgat = jit_runs.gen_match_gather(q3, cr)
        assert jit_runs.copy_ok(q3, cr) and "a.HIT[" in kc.src and "a.S9[" in kc.src
        assert "a.c9" not in kc.src and "a.MATCH" not in kc.src
        assert "a.S9[i] = a.c9[j_]" in kgat.src
        ks += [kr_, km, kc, kgat]
    q3.group_col, q3.num_groups = 10, 300
    assert not jit_runs.applies(q3)
    q3.group_col = -1
    assert "st9_s" in ks[0].src          # phase 2 staged through LDS
    assert "a.rbm" in ks[1].src and "a.c9" not in ks[1].src   # phase 2 = bitmap tests
    for k in ks:
        rc = jit.runtime().hs_jit_compile_to_cache(k.src.encode(), k.name.encode(), b"gfx950",
                                                   str(tmp_path).encode())
        assert rc == 0, jit.runtime().hs_jit_last_error().decode()


def test_hash_mode_sources_compile(rt, tmp_path):
    """Hash-mode grouping (exec/hash_agg.py): the Q3 full-shape merge join (3-column packed key
    over both sides), a scan with a nullable / exact-decimal / f32 packed key and MIN/MAX, and a
    raw float key compile for gfx950."""
    import types
    from hyperspace_amd.exec import hash_agg as H
    from hyperspace_amd.exec.encoding import Compact
    jit = rt

    def col(t, valid=False, dictionary=None):
        return types.SimpleNamespace(hs_type=t, valid=1 if valid else None, dictionary=dictionary,
                                     offsets=None, atype=pa.int64())
    j = _q3_params()
    j.cols[10] = _fake(NL.I32)
    comp = dict(_q3_compacts())
    comp[0] = Compact(None, 4, 1 + (1 << 31), None, NL.I64, 1, 600_000_000)
    comp[8] = Compact(None, 4, 1 + (1 << 31), None, NL.I64, 1, 600_000_000)
    hk = H.plan_keys([(0, None, col(NL.I64), (1, 600_000_000, None)),
                      (9, None, col(NL.I32), (8000, 2500, None)),
                      (10, None, col(NL.I32), (0, 1, None))], (False, False), False)
    assert hk.mode == "packed" and [c.shift for c in hk.cols] == [0, 30, 42]
    ks = [jit.gen_merge_join_agg(j, comp, hk), jit.gen_merge_join_agg(j, None, hk)]
    assert "atomicCAS" in ks[0].src and "hs_mix64" in ks[0].src and "_flush" not in ks[0].src
    p = _scan_params({0: _fake(NL.I64, True), 1: _fake(NL.F64), 2: _fake(NL.F32),
                      3: _fake(NL.F64)},
                     [NL.Pred(NL.PK_FLT_LIT, NL.OP_GE, 1, 0, 0, 0, 0, 0.05, None)],
                     [_agg(NL.AK_SUM, [(3, 0.0, 1.0)]), _agg(NL.AK_MIN, [(3, 0.0, 1.0)]),
                      _agg(NL.AK_MAX, [(3, 0.0, 1.0)]), _agg(NL.AK_COUNT_STAR)])
    hk2 = H.plan_keys([(0, None, col(NL.I64, True), (-5, 100, None)),
                       (1, None, col(NL.F64), (0, 11, 100.0)),
                       (2, None, col(NL.F32), (0, 0, None))], (False, False, False, False), True)
    assert [c.kind for c in hk2.cols] == ["int", "dec", "f32"]
    hk3 = H.plan_keys([(3, None, col(NL.F64), (0, 0, 0.0))], (False, False, False, False))
    assert hk3.mode == "raw_float"
    for vec in (0, 8):
        ks += [jit.gen_scan_agg(p, None, vec, hk2), jit.gen_scan_agg(p, None, vec, hk3)]
    for k in ks:
        rc = jit.runtime().hs_jit_compile_to_cache(k.src.encode(), k.name.encode(), b"gfx950",
                                                   str(tmp_path).encode())
        assert rc == 0, jit.runtime().hs_jit_last_error().decode()


def q3_join_index_kernel(jit, vec=8, stage=False, bitmap=False):
    """The TPC-H Q3 shape of the bench: left (lineitem) l_shipdate > d, right (orders)
    o_orderdate < d, SUM(price * (1 - disc)) + COUNT(*), compact HBM columns, 1-byte join index."""
    j = _q3_params()
    return jit.gen_join_index_agg(j, _q3_compacts(), vec=vec, jw=1, jlog=7, stage=stage,
                                  bitmap=bitmap)


def _q3_params():
    j = NL.JoinParams()
    j.cols[0], j.cols[1] = _fake(NL.I64), _fake(NL.I32)
    j.cols[2], j.cols[3] = _fake(NL.F64), _fake(NL.F64)
    j.cols[8], j.cols[9] = _fake(NL.I64), _fake(NL.I32)
    j.preds[0] = NL.Pred(NL.PK_INT_LIT, NL.OP_GT, 1, 0, 0, 0, 9000, 0.0, None)
    j.preds[1] = NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 9, 0, 1, 0, 9000, 0.0, None)
    j.nlp, j.npreds = 1, 2
    j.aggs[0] = _agg(NL.AK_SUM, [(2, 0.0, 1.0), (3, 1.0, -1.0)])
    j.aggs[1] = _agg(NL.AK_COUNT_STAR)
    j.naggs, j.lkey, j.rkey, j.group_col = 2, 0, 8, -1
    return j


def _q3_compacts():
    from hyperspace_amd.exec.encoding import Compact
    return {1: Compact(None, 2, 8000, None, NL.I32), 3: Compact(None, 1, 0, 100.0, NL.F64),
            9: Compact(None, 2, 8000, None, NL.I32)}


def q3_bitmap_kernel(jit):
    return jit.gen_pred_bitmap(_q3_params(), _q3_compacts())


def test_shape_key_ignores_literals():
    from hyperspace_amd.exec import jit
    a = _scan_params({0: _fake(NL.F64)}, [NL.Pred(NL.PK_FLT_LIT, NL.OP_LT, 0, 0, 0, 0, 0, 1.0, None)],
                     [_agg(NL.AK_SUM, [(0, 0.0, 1.0)])])
    b = _scan_params({0: _fake(NL.F64)}, [NL.Pred(NL.PK_FLT_LIT, NL.OP_LT, 0, 0, 0, 0, 0, 9.0, None)],
                     [_agg(NL.AK_SUM, [(0, 2.0, 3.0)])])
    assert jit.scan_agg_shape(a) == jit.scan_agg_shape(b)
    c = _scan_params({0: _fake(NL.F64)}, [NL.Pred(NL.PK_FLT_LIT, NL.OP_LE, 0, 0, 0, 0, 0, 1.0, None)],
                     [_agg(NL.AK_SUM, [(0, 0.0, 1.0)])])
    assert jit.scan_agg_shape(a) != jit.scan_agg_shape(c)


# ------------------------------------------------------------------------------------------------
# GPU numerics
# ------------------------------------------------------------------------------------------------
def _col(arr, device):
    from hyperspace_amd.exec.device_table import DeviceColumn
    return DeviceColumn.from_arrow(arr, device)


@pytest.mark.gpu
def test_jit_scan_agg_matches_aot_and_numpy(device):
    import torch
    from hyperspace_amd.exec import jit
    from hyperspace_amd.ops import kernels as K
    rng = np.random.default_rng(21)
    n = 300_001
    d = rng.integers(0, 2000, n).astype(np.int32)
    disc = rng.integers(0, 11, n) / 100.0
    qnull = rng.random(n) < 0.05
    qty = rng.integers(1, 51, n).astype(np.float64)
    price = rng.random(n) * 1000
    grp = rng.integers(0, 7, n).astype(np.int64)
    cols = {0: _col(pa.array(d), device), 1: _col(pa.array(disc), device),
            2: _col(pa.array(qty, mask=qnull), device), 3: _col(pa.array(price), device),
            4: _col(pa.array(grp), device)}
    iset = torch.tensor([3, 17, 500, 1999], dtype=torch.int64, device=device)
    preds = [NL.Pred(NL.PK_INT_LIT, NL.OP_GE, 0, 0, 0, 0, 100, 0.0, None),
             NL.Pred(NL.PK_FLT_LIT, NL.OP_GE, 1, 0, 1, 0, 0, 0.03, None),
             NL.Pred(NL.PK_IN_SET, NL.OP_EQ, 0, 0, 1, 4, 0, 0.0, iset.data_ptr()),
             NL.Pred(NL.PK_FLT_LIT, NL.OP_LT, 2, 0, 2, 0, 0, 30.0, None)]
    aggs = [_agg(NL.AK_SUM, [(3, 0.0, 1.0), (1, 1.0, -1.0)]), _agg(NL.AK_MIN, [(2, 0.0, 1.0)]),
            _agg(NL.AK_MAX, [(3, 0.0, 1.0)]), _agg(NL.AK_COUNT_STAR)]
    ok = (d >= 100) & ((disc >= 0.03) | np.isin(d, [3, 17, 500, 1999])) & (~qnull) & (qty < 30)
    rstart = torch.tensor([0, 1000], dtype=torch.int64, device=device)
    rlen = torch.tensor([1000, n - 1000], dtype=torch.int64, device=device)
    tp = K.ranges_to_tiles(rlen)
    for grouped in (False, True):
        p = _scan_params({s: c.desc() for s, c in cols.items()}, preds, aggs,
                         group_col=4 if grouped else -1, num_groups=7)
        got = [t.cpu().numpy() for t in jit.scan_agg(p, rstart, rlen, tp)]
        aot = [t.cpu().numpy() for t in K.scan_agg(p, rstart, rlen, tp)]
        G = 7 if grouped else 1
        for g in range(G):
            m = ok & ((grp == g) if grouped else True)
            exp_sum = (price * (1 - disc))[m].sum()
            base = g * 4
            assert abs(got[0][base] - exp_sum) <= 1e-9 * max(1.0, abs(exp_sum))
            assert got[1][base + 3] == m.sum()
            if m.any():
                assert got[2][base + 1] == qty[m].min()
                assert got[3][base + 2] == price[m].max()
        np.testing.assert_allclose(got[0], aot[0], rtol=1e-12)
        assert np.array_equal(got[1], aot[1])
        # compact HBM encodings give bit-identical inputs, hence identical results
        from hyperspace_amd.exec.encoding import encode
        comp = {s: e for s, e in ((s, encode(c)) for s, c in cols.items()) if e is not None}
        assert {1, 2, 4} <= set(comp)  # discount (dec2/u8), quantity (int/u8), group (u8)
        cg = [t.cpu().numpy() for t in jit.scan_agg(p, rstart, rlen, None, comp)]
        np.testing.assert_allclose(cg[0], got[0], rtol=1e-12)
        assert np.array_equal(cg[1], got[1])
        assert np.array_equal(cg[2], got[2]) and np.array_equal(cg[3], got[3])


@pytest.mark.gpu
def test_jit_join_agg_matches_aot(device):
    import torch
    from hyperspace_amd.exec import jit
    from hyperspace_amd.ops import kernels as K
    rng = np.random.default_rng(8)
    B = 8
    rk = np.concatenate([np.repeat(np.arange(0, 20_000, dtype=np.int64) * 3, 2),
                         np.arange(100_000, 130_000, dtype=np.int64)])
    rb = murmur3.bucket_ids([pa.array(rk)], B)
    lk = np.concatenate([np.repeat(rk[::2], rng.integers(1, 5, len(rk[::2]))),
                         rng.integers(0, 140_000, 20_000)])
    lb = murmur3.bucket_ids([pa.array(lk)], B)
    ro = np.lexsort((rk, rb)); rk, rb = rk[ro], rb[ro]
    lo_ = np.lexsort((lk, lb)); lk, lb = lk[lo_], lb[lo_]
    loff = np.searchsorted(lb, np.arange(B + 1)).astype(np.int64)
    roff = np.searchsorted(rb, np.arange(B + 1)).astype(np.int64)
    ldate = rng.integers(0, 1000, len(lk)).astype(np.int32)
    lprice = rng.random(len(lk)) * 100
    rdate = rng.integers(0, 1000, len(rk)).astype(np.int32)
    rgrp = rng.integers(0, 3, len(rk)).astype(np.int32)
    p = NL.JoinParams()
    cl = [_col(pa.array(x), device) for x in (lk, ldate, lprice)]
    cr = [_col(pa.array(x), device) for x in (rk, rdate, rgrp)]
    for i, c in enumerate(cl):
        p.cols[i] = c.desc()
    for i, c in enumerate(cr):
        p.cols[8 + i] = c.desc()
    p.preds[0] = NL.Pred(NL.PK_INT_LIT, NL.OP_GT, 1, 0, 0, 0, 300, 0.0, None)
    p.preds[1] = NL.Pred(NL.PK_INT_COL, NL.OP_LT, 9, 1, 1000, 0, 0, 0.0, None)
    p.nlp, p.npreds = 1, 2
    p.aggs[0] = _agg(NL.AK_SUM, [(2, 0.0, 1.0)])
    p.aggs[1] = _agg(NL.AK_COUNT_STAR)
    p.naggs, p.lkey, p.rkey, p.key_is_float = 2, 0, 8, 0
    rstart, rlen, rbk = K.full_ranges(loff, device)
    roff_t = torch.from_numpy(roff).to(device)
    mt = K.join_max_tiles(len(lk), B)
    for g in (-1, 10):
        p.group_col, p.num_groups, p.group_base = g, 3, 0
        got = [t.cpu().numpy() for t in jit.join_agg(p, rstart, rlen, rbk, roff_t, mt)]
        aot = [t.cpu().numpy() for t in K.join_agg(p, rstart, rlen, rbk, roff_t, mt)]
        np.testing.assert_allclose(got[0], aot[0], rtol=1e-12)
        assert np.array_equal(got[1], aot[1])
        assert got[1].sum() > 0
        from hyperspace_amd.exec.encoding import encode
        allc = dict(enumerate(cl))
        allc.update({8 + i: c for i, c in enumerate(cr)})
        comp = {s: e for s, e in ((s, encode(c)) for s, c in allc.items()) if e is not None}
        assert 0 in comp and 8 in comp  # both join keys FOR-encoded
        cg = [t.cpu().numpy() for t in jit.join_agg(p, rstart, rlen, rbk, roff_t, mt, comp)]
        np.testing.assert_allclose(cg[0], got[0], rtol=1e-12)
        assert np.array_equal(cg[1], got[1])
        # vectorized sort-merge join: staged spans, and every span searched in HBM
        from hyperspace_amd.exec import kernel_config
        for keys in (kernel_config.active().mj_lds_keys, 16):
            with kernel_config.use(mj_lds_keys=keys):
                for cmp in (None, comp):
                    mj = [t.cpu().numpy() for t in
                          jit.merge_join_agg(p, rstart, rlen, rbk, roff_t, cmp, nrows=len(lk))]
                    np.testing.assert_allclose(mj[0], got[0], rtol=1e-12)
                    assert np.array_equal(mj[1], got[1]), (keys, cmp is None)


@pytest.mark.gpu
def test_merge_join_agg_numpy_oracle(device):
    """Merge join with right-only predicates, a left predicate, duplicate right keys, null keys
    on both sides and sub-ranges (unaligned range starts) against a numpy fp64 oracle."""
    import torch
    from hyperspace_amd.exec import jit
    from hyperspace_amd.ops import kernels as K
    rng = np.random.default_rng(5)
    B = 4
    rk = rng.integers(0, 60_000, 50_000).astype(np.int64)
    rnull = rng.random(len(rk)) < 0.01
    lk = rng.integers(0, 60_000, 400_003).astype(np.int64)
    lnull = rng.random(len(lk)) < 0.01
    rb = murmur3.bucket_ids([pa.array(rk)], B)
    lb = murmur3.bucket_ids([pa.array(lk)], B)
    rb[rnull] = rng.integers(0, B, rnull.sum())
    lb[lnull] = rng.integers(0, B, lnull.sum())
    # sort: bucket, nulls first, key
    ro = np.lexsort((rk, ~rnull, rb)); rk, rb, rnull = rk[ro], rb[ro], rnull[ro]
    lo_ = np.lexsort((lk, ~lnull, lb)); lk, lb, lnull = lk[lo_], lb[lo_], lnull[lo_]
    loff = np.searchsorted(lb, np.arange(B + 1)).astype(np.int64)
    roff = np.searchsorted(rb, np.arange(B + 1)).astype(np.int64)
    ldate = rng.integers(0, 1000, len(lk)).astype(np.int32)
    lprice = np.round(rng.random(len(lk)) * 1000, 2)
    rdate = rng.integers(0, 1000, len(rk)).astype(np.int32)
    p = NL.JoinParams()
    cl = [_col(pa.array(lk, mask=lnull), device), _col(pa.array(ldate), device),
          _col(pa.array(lprice), device)]
    cr = [_col(pa.array(rk, mask=rnull), device), _col(pa.array(rdate), device)]
    for i, c in enumerate(cl):
        p.cols[i] = c.desc()
    for i, c in enumerate(cr):
        p.cols[8 + i] = c.desc()
    p.preds[0] = NL.Pred(NL.PK_INT_LIT, NL.OP_GT, 1, 0, 0, 0, 250, 0.0, None)
    p.preds[1] = NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 9, 0, 1, 0, 600, 0.0, None)
    p.nlp, p.npreds = 1, 2
    p.aggs[0] = _agg(NL.AK_SUM, [(2, 0.0, 1.0)])
    p.aggs[1] = _agg(NL.AK_COUNT_STAR)
    p.naggs, p.lkey, p.rkey, p.key_is_float = 2, 0, 8, 0
    p.group_col, p.num_groups, p.group_base = -1, 1, 0
    # oracle over sub-ranges of every bucket (unaligned starts)
    starts = loff[:-1] + 3
    lens = np.maximum(loff[1:] - starts - 5, 0)
    exp_sum, exp_cnt = 0.0, 0
    for b in range(B):
        rows = np.arange(starts[b], starts[b] + lens[b])
        rsel = np.arange(roff[b], roff[b + 1])
        rsel = rsel[(~rnull[rsel]) & (rdate[rsel] < 600)]
        cnt = {}
        for k in rk[rsel]:
            cnt[k] = cnt.get(k, 0) + 1
        for i in rows:
            if lnull[i] or ldate[i] <= 250:
                continue
            c = cnt.get(lk[i], 0)
            exp_cnt += c
            exp_sum += c * lprice[i]
    rstart = torch.from_numpy(starts.astype(np.int64)).to(device)
    rlen = torch.from_numpy(lens.astype(np.int64)).to(device)
    rbk = torch.arange(B, dtype=torch.int32, device=device)
    roff_t = torch.from_numpy(roff).to(device)
    from hyperspace_amd.exec.encoding import encode
    allc = dict(enumerate(cl))
    allc.update({8 + i: c for i, c in enumerate(cr)})
    comp = {s: e for s, e in ((s, encode(c)) for s, c in allc.items()) if e is not None}
    from hyperspace_amd.exec import kernel_config
    for keys in (kernel_config.active().mj_lds_keys, 32):
        with kernel_config.use(mj_lds_keys=keys):
            for cmp in (None, comp):
                got = [t.cpu().numpy() for t in
                       jit.merge_join_agg(p, rstart, rlen, rbk, roff_t, cmp, nrows=len(lk))]
                assert got[1][1] == exp_cnt and got[1][0] == exp_cnt, (keys, got[1], exp_cnt)
                assert abs(got[0][0] - exp_sum) <= 1e-9 * max(1.0, exp_sum)


@pytest.mark.gpu
def test_merge_join_key16_matches_oracle(device):
    """Merge join streaming the left key as grouped 16-bit codes (MJ_KEY16): TPC-H-like sparse
    unique right keys, 1-7 left rows per key, buckets sorted by key (groups straddling buckets
    read the 32-bit codes), full and partial tiles; equals the 32-bit-key kernel and numpy."""
    import torch
    from hyperspace_amd.exec import jit
    from hyperspace_amd.exec.encoding import GroupedCompact, encode
    rng = np.random.default_rng(8)
    B = 8
    ok = np.arange(1, 150_001, dtype=np.int64) * 4 + (1 << 20)
    rb = murmur3.bucket_ids([pa.array(ok)], B)
    per = rng.integers(1, 8, len(ok))
    lk = np.repeat(ok, per)
    lb = np.repeat(rb, per)
    ro = np.lexsort((ok, rb)); rk, rb = ok[ro], rb[ro]
    lo_ = np.lexsort((lk, lb)); lk, lb = lk[lo_], lb[lo_]
    loff = np.searchsorted(lb, np.arange(B + 1)).astype(np.int64)
    roff = np.searchsorted(rb, np.arange(B + 1)).astype(np.int64)
    ldate = rng.integers(0, 1000, len(lk)).astype(np.int32)
    lprice = np.round(rng.random(len(lk)) * 1000, 2)
    rdate = rng.integers(0, 1000, len(rk)).astype(np.int32)
    p = NL.JoinParams()
    cl = [_col(pa.array(lk), device), _col(pa.array(ldate), device), _col(pa.array(lprice), device)]
    cr = [_col(pa.array(rk), device), _col(pa.array(rdate), device)]
    for i, c in enumerate(cl):
        p.cols[i] = c.desc()
    for i, c in enumerate(cr):
        p.cols[8 + i] = c.desc()
    p.preds[0] = NL.Pred(NL.PK_INT_LIT, NL.OP_GT, 1, 0, 0, 0, 300, 0.0, None)
    p.preds[1] = NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 9, 0, 1, 0, 500, 0.0, None)
    p.nlp, p.npreds = 1, 2
    p.aggs[0] = _agg(NL.AK_SUM, [(2, 0.0, 1.0)])
    p.aggs[1] = _agg(NL.AK_COUNT_STAR)
    p.naggs, p.lkey, p.rkey, p.key_is_float = 2, 0, 8, 0
    p.group_col, p.num_groups, p.group_base = -1, 1, 0
    rpass = dict(zip(rk.tolist(), (rdate < 500).tolist()))
    m = np.array([rpass[k] for k in lk.tolist()]) & (ldate > 300)
    allc = dict(enumerate(cl))
    allc.update({8 + i: c for i, c in enumerate(cr)})
    comp = {s: e for s, e in ((s, encode(c)) for s, c in allc.items()) if e is not None}
    assert comp[0].width == 4
    from hyperspace_amd.exec import kernel_config
    with kernel_config.use(mj_key16=True):
        assert isinstance(jit._with_key16(p, comp)[0], GroupedCompact)
    assert int((comp[0].g16.gbase == -(1 << 31)).sum()) >= 1      # groups across buckets
    for starts, lens, exp in ((loff[:-1], loff[1:] - loff[:-1], m),
                              (loff[:-1] + 5, loff[1:] - loff[:-1] - 9, None)):
        if exp is None:
            exp = np.zeros(len(lk), bool)
            for b in range(B):
                exp[starts[b]:starts[b] + lens[b]] = m[starts[b]:starts[b] + lens[b]]
        rstart = torch.from_numpy(starts.astype(np.int64)).to(device)
        rlen = torch.from_numpy(lens.astype(np.int64)).to(device)
        rbk = torch.arange(B, dtype=torch.int32, device=device)
        roff_t = torch.from_numpy(roff).to(device)
        res = {}
        for k16 in (True, False):
            with kernel_config.use(mj_key16=k16, mj_runs=False):
                res[k16] = [t.cpu().numpy() for t in
                            jit.merge_join_agg(p, rstart, rlen, rbk, roff_t, comp, nrows=len(lk),
                                               rdup=False)]
        for r in res.values():
            assert r[1][0] == int(exp.sum())
            assert abs(r[0][0] - float(lprice[exp].sum())) <= 1e-9 * max(1.0, float(lprice[exp].sum()))


def test_code_bounds_match_value_compares():
    """Predicates on compact columns compare stored codes with host-computed int32 bounds; they
    must agree with the compare on the decoded value for every code, op and literal."""
    from hyperspace_amd.exec import jit
    rng = np.random.default_rng(3)
    codes = np.arange(-128, 128, dtype=np.int64)
    ops = {NL.OP_EQ: np.equal, NL.OP_NE: np.not_equal, NL.OP_LT: np.less, NL.OP_LE: np.less_equal,
           NL.OP_GT: np.greater, NL.OP_GE: np.greater_equal}
    for base in (0, 1000, -5, 2**40):
        for lit in list(base + rng.integers(-300, 300, 20)) + [2**62, -2**62]:
            for op, fn in ops.items():
                lo, hi = jit.code_bounds(*jit._int_lit_bounds(op, lit), base)
                assert -2**31 <= lo and hi <= 2**31 - 1
                inside = (codes >= lo) & (codes <= hi)
                got = ~inside if op == NL.OP_NE else inside
                assert (got == fn(base + codes, lit)).all(), (base, lit, op)


def test_int_bounds_match_decoded_double_compares():
    """Integer-code predicates on decimal-scaled compact columns select exactly the rows the
    decoded double comparison selects (all ops, literals on and between grid points)."""
    import random
    from hyperspace_amd.exec.jit import int_bounds
    rng = random.Random(7)
    ops = {NL.OP_EQ: lambda a, b: a == b, NL.OP_NE: lambda a, b: a != b,
           NL.OP_LT: lambda a, b: a < b, NL.OP_LE: lambda a, b: a <= b,
           NL.OP_GT: lambda a, b: a > b, NL.OP_GE: lambda a, b: a >= b}
    for scale in (1.0, 10.0, 100.0, 1000.0, 10000.0):
        qs = list(range(-3000, 3000))
        lits = [q / scale for q in rng.sample(qs, 40)] + [rng.uniform(-30, 30) for _ in range(40)]
        lits += [0.05, 0.07, -0.0, float("inf"), float("-inf"), float("nan")]
        for lit in lits:
            for op, f in ops.items():
                lo, hi = int_bounds(op, lit, scale)
                for q in qs[::7]:
                    inside = lo <= q <= hi
                    got = (not inside) if op == NL.OP_NE else inside
                    assert got == f(q / scale, lit), (scale, lit, op, q)


def test_timestamp_literals_exact_in_column_unit():
    import datetime
    import random
    from hyperspace_amd.exec.compile import Unsupported, _lit_value
    rnd = random.Random(3)
    epoch = datetime.datetime(1970, 1, 1)
    for _ in range(20000):
        us = rnd.randrange(-2**50, 2**50)
        v = epoch + datetime.timedelta(microseconds=us)
        assert _lit_value(v) == us
        assert _lit_value(v, pa.timestamp("ns")) == us * 1000
    tz = datetime.timezone(datetime.timedelta(hours=2))
    assert _lit_value(datetime.datetime(1970, 1, 1, 2, 0, 1, tzinfo=tz)) == 1_000_000
    assert _lit_value(datetime.datetime(1970, 1, 1, 0, 0, 5), pa.timestamp("s")) == 5
    assert _lit_value(datetime.datetime(1970, 1, 2), pa.date32()) == 1
    assert _lit_value(datetime.date(1970, 1, 2), pa.timestamp("ms")) == 86_400_000
    with pytest.raises(Unsupported):
        _lit_value(datetime.datetime(1970, 1, 1, 0, 0, 0, 5), pa.timestamp("ms"))
    with pytest.raises(Unsupported):
        _lit_value(datetime.datetime(1970, 1, 2, 1), pa.date32())


@pytest.mark.gpu
def test_hbm_encoding_device_matches_torch_reference(device):
    """hs_compact_probe / hs_compact_encode (csrc/kernels/compact.hip) take the same decisions
    and write the same codes as the PyTorch reference path on the host."""
    import torch
    from hyperspace_amd.exec.device_table import DeviceColumn
    from hyperspace_amd.exec.encoding import _encode_device, _encode_torch
    rng = np.random.default_rng(7)
    n = 300_001
    cases = [
        (torch.from_numpy(rng.integers(10**12, 10**12 + 3_000_000_000, n)), None, pa.int64()),
        (torch.from_numpy(rng.integers(8000, 10600, n).astype(np.int32)), None, pa.date32()),
        (torch.from_numpy(rng.integers(-100, 100, n).astype(np.int32)),
         torch.from_numpy((rng.random(n) < 0.9).astype(np.uint8)), pa.int32()),
        (torch.from_numpy(rng.integers(0, 11, n) / 100.0), None, pa.float64()),
        (torch.from_numpy(np.round(rng.random(n) * 1e5, 2)), None, pa.float64()),
        (torch.from_numpy(np.round(rng.random(n) * 1e3, 3)),
         torch.from_numpy((rng.random(n) < 0.5).astype(np.uint8)), pa.float64()),
        (torch.from_numpy(rng.random(n)), None, pa.float64()),                  # no scale
        (torch.tensor([-0.0, 1.0] * 100, dtype=torch.float64), None, pa.float64()),
        (torch.tensor([np.nan, 1.0] * 100, dtype=torch.float64), None, pa.float64()),
        (torch.tensor([1e17, 1.0] * 100, dtype=torch.float64), None, pa.float64()),
        (torch.tensor([0, 2**40] * 100, dtype=torch.int64), None, pa.int64()),
        (torch.tensor([3, 4], dtype=torch.int64), torch.tensor([0, 0], dtype=torch.uint8),
         pa.int64()),
    ]
    for data, valid, at in cases:
        ref = _encode_torch(DeviceColumn(data, valid, at))
        got = _encode_device(DeviceColumn(data.to(device),
                                          None if valid is None else valid.to(device), at))
        assert (ref is None) == (got is None), (at, ref, got)
        if ref is None:
            continue
        assert (got.width, got.base, got.scale, got.lo, got.hi) == \
            (ref.width, ref.base, ref.scale, ref.lo, ref.hi)
        vm = torch.ones(len(data), dtype=torch.bool) if valid is None else valid.bool()
        assert torch.equal(got.codes.cpu()[vm], ref.codes[vm])


def test_aot_sources_compile_into_cache(rt, tmp_path):
    """The committed kernel sources of the benchmark workload (hyperspace_amd/_native/aot,
    recorded with HS_JIT_RECORD) compile for gfx950 into a code-object cache on a machine without
    a GPU, one object per source, keyed the way hs_jit_get looks them up."""
    from hyperspace_amd.exec import jit
    n = jit.aot_compile(cache_dir=str(tmp_path))
    assert n >= 1
    assert len([f for f in os.listdir(tmp_path) if f.endswith(".co")]) == n
    # recording writes the exact generated text under <kernel>.<hash>.hip
    rec = tmp_path / "rec"
    jit._record_source(str(rec), "hs_jit_x", "int x;")
    (f,) = os.listdir(rec)
    assert f.startswith("hs_jit_x.") and f.endswith(".hip") and (rec / f).read_text() == "int x;"


def test_project_kernel_compiles(rt, tmp_path):
    """exec/project.py: the elementwise kernel of a computed projection (arithmetic with
    wrapping / division / casts / Kleene logic over nullable columns) compiles for gfx950."""
    import torch
    from hyperspace_amd.exec import project
    from hyperspace_amd.exec.device_table import DeviceColumn
    jit = rt
    from hyperspace_amd.plan import expressions as E
    a = E.Attribute("a", pa.int64())
    b = E.Attribute("b", pa.int32())
    x = E.Attribute("x", pa.float64())
    cols = {a.expr_id: DeviceColumn(torch.zeros(4, dtype=torch.int64),
                                    torch.ones(4, dtype=torch.uint8), pa.int64()),
            b.expr_id: DeviceColumn(torch.zeros(4, dtype=torch.int32), None, pa.int32()),
            x.expr_id: DeviceColumn(torch.zeros(4, dtype=torch.float64), None, pa.float64())}
    exprs = [E.Add(E.Multiply(a, E.Literal(3)), b), E.Divide(a, b), E.Cast(x, pa.int32()),
             E.Or(E.And(E.GreaterThan(a, b), E.LessThan(x, E.Literal(2.5))), E.IsNull(a)),
             E.Subtract(x, E.Cast(b, pa.float64()))]
    k, values, outs = project.build(exprs, cols, 4, torch.device("cpu"))
    assert [o.atype for o in outs] == [e.data_type for e in exprs]
    rc = jit.runtime().hs_jit_compile_to_cache(k.src.encode(), k.name.encode(), b"gfx950",
                                               str(tmp_path).encode())
    assert rc == 0, jit.runtime().hs_jit_last_error().decode()
    # literals are arguments: another literal reuses the kernel
    exprs[0] = E.Add(E.Multiply(a, E.Literal(7)), b)
    k2, _, _ = project.build(exprs, cols, 4, torch.device("cpu"))
    assert k2 is k


def test_grouped16_round_trips_sorted_keys():
    """encoding.grouped16: 16-bit codes over per-64-row group bases reproduce every 32-bit code
    of a bucket-sorted key column (uint16 bits in int16 storage); groups straddling two buckets
    are wide (read from the 32-bit codes); too many wide groups make the column ineligible."""
    import torch
    from hyperspace_amd.exec.encoding import Compact, grouped16
    rng = np.random.default_rng(5)
    runs = []
    for _ in range(8):              # sorted runs (buckets), restarting low
        runs.append(np.sort(rng.integers(0, 4_000_000, 20_000)))
    codes = torch.from_numpy(np.concatenate(runs).astype(np.int32))
    c = Compact(codes, 4, 100, None, NL.I64, 100, 4_000_100)
    g = grouped16(c)
    assert g is not None and g.codes.dtype == torch.int16
    assert g.gbase.numel() == (codes.numel() + 63) // 64
    gb = g.gbase.repeat_interleave(64)[:codes.numel()].long()
    wide = gb == -(1 << 31)
    assert 0 < int(wide.sum()) <= 8 * 64      # only groups across run boundaries
    back = torch.where(wide, g.wide.long(), gb + (g.codes.long() & 0xFFFF))
    assert torch.equal(back, codes.long())
    assert grouped16(c) is g and c.nbytes() == codes.numel() * 4 + g.nbytes()
    spread = torch.from_numpy(np.array([0, 1 << 17] * 64, dtype=np.int32))
    assert grouped16(Compact(spread, 4, 0, None, NL.I64, 0, 1 << 17)) is None


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["dense", "jumpy"])
def test_merge_join_runs_matches_oracle(device, layout):
    """Run-keyed merge join (MJ_RUNS, encoding.RunCompact): TPC-H-like unique right keys, 1-7
    left rows per key, right keys with no left rows and left keys with no right row, a grouped
    aggregate over a right column; full buckets and unaligned sub-ranges, staged (2048 LDS keys)
    and HBM-searched (32) spans; equals the per-row-key kernel and numpy.  The device run form
    equals the PyTorch reference."""
    import torch
    from hyperspace_amd.exec import jit
    from hyperspace_amd.exec.encoding import encode, key_runs, runs_torch
    rng = np.random.default_rng(11)
    B = 8
    ok = np.arange(1, 120_001, dtype=np.int64) * 4 + (1 << 20)
    if layout == "jumpy":
        # rare large key gaps: a few percent of the 64-key groups span >= 2^16 codes (the 16-bit
        # grouped key forms read those groups' 32-bit keys)
        gaps = np.where(rng.random(len(ok)) < 0.0001, 3_000_000, 4)
        ok = np.cumsum(gaps) + (1 << 20)
    per = rng.integers(1, 8, len(ok))
    per[rng.random(len(ok)) < 0.05] = 0                         # orders without lines
    lk = np.repeat(ok, per)
    orphan = rng.integers(1, 120_001, 3000) * 4 + (1 << 20) + 1  # lines without an order
    lk = np.concatenate([lk, orphan])
    rk = ok
    rb = murmur3.bucket_ids([pa.array(rk)], B)
    lb = murmur3.bucket_ids([pa.array(lk)], B)
    ro = np.lexsort((rk, rb)); rk, rb = rk[ro], rb[ro]
    lo_ = np.lexsort((lk, lb)); lk, lb = lk[lo_], lb[lo_]
    loff = np.searchsorted(lb, np.arange(B + 1)).astype(np.int64)
    roff = np.searchsorted(rb, np.arange(B + 1)).astype(np.int64)
    ldate = rng.integers(0, 1000, len(lk)).astype(np.int32)
    lprice = np.round(rng.random(len(lk)) * 1000, 2)
    rdate = rng.integers(0, 1000, len(rk)).astype(np.int32)
    rprio = rng.integers(0, 3, len(rk)).astype(np.int32)
    p = NL.JoinParams()
    cl = [_col(pa.array(lk), device), _col(pa.array(ldate), device), _col(pa.array(lprice), device)]
    cr = [_col(pa.array(rk), device), _col(pa.array(rdate), device), _col(pa.array(rprio), device)]
    for i, c in enumerate(cl):
        p.cols[i] = c.desc()
    for i, c in enumerate(cr):
        p.cols[8 + i] = c.desc()
    p.preds[0] = NL.Pred(NL.PK_INT_LIT, NL.OP_GT, 1, 0, 0, 0, 300, 0.0, None)
    p.preds[1] = NL.Pred(NL.PK_INT_LIT, NL.OP_LT, 9, 0, 1, 0, 500, 0.0, None)
    p.nlp, p.npreds = 1, 2
    # two aggregate input columns (price, date): the bits scan reads them row-packed
    p.aggs[0] = _agg(NL.AK_SUM, [(2, 0.0, 1.0), (1, 1.0, 0.001)])
    p.aggs[1] = _agg(NL.AK_COUNT_STAR)
    p.naggs, p.lkey, p.rkey, p.key_is_float = 2, 0, 8, 0
    p.group_col, p.num_groups, p.group_base = 10, 3, 0
    rmap = {k: (d < 500, g) for k, d, g in zip(rk.tolist(), rdate.tolist(), rprio.tolist())}
    allc = dict(enumerate(cl))
    allc.update({8 + i: c for i, c in enumerate(cr)})
    comp = {s: e for s, e in ((s, encode(c)) for s, c in allc.items()) if e is not None}
    rc = key_runs(comp[0])
    assert rc is not None and rc.nruns < len(lk) / 2
    ref = runs_torch(comp[0].codes.cpu())
    for a, b_ in zip((rc.runkeys, rc.gmask, rc.gruns), ref):
        assert torch.equal(a.cpu(), b_)
    from hyperspace_amd.exec import jit_runs, kernel_config
    lds_keys = kernel_config.active().mj_lds_keys
    alive = []
    try:
        for starts, lens in ((loff[:-1], loff[1:] - loff[:-1]),
                             (loff[:-1] + 5, loff[1:] - loff[:-1] - 9)):
            exp_s, exp_c = np.zeros(3), np.zeros(3, np.int64)
            for b in range(B):
                for i in range(starts[b], starts[b] + lens[b]):
                    m = rmap.get(int(lk[i]))
                    if m is not None and m[0] and ldate[i] > 300:
                        exp_s[m[1]] += lprice[i] * (1.0 + 0.001 * ldate[i])
                        exp_c[m[1]] += 1
            rstart = torch.from_numpy(starts.astype(np.int64)).to(device)
            rlen = torch.from_numpy(lens.astype(np.int64)).to(device)
            rbk = torch.arange(B, dtype=torch.int32, device=device)
            roff_t = torch.from_numpy(roff).to(device)
            alive.append((rstart, rlen, rbk, roff_t))   # cached lowerings key by tensor ids
            for keys, grouped in ((lds_keys, True), (32, True), (lds_keys, False)):
                # ungrouped: 1-bit tags (bit-parallel phase 2 unless rs_bits is off)
                p.group_col, p.num_groups = (10, 3) if grouped else (-1, 1)
                G = 3 if grouped else 1
                es = exp_s if grouped else exp_s.sum(keepdims=True)
                ec = exp_c if grouped else exp_c.sum(keepdims=True)
                for use_runs, two, sparse, pk12, match in ((True, True, True, True, True),
                                                           (True, True, True, True, False),
                                                           (True, True, True, False, True),
                                                           (True, True, False, True, True),
                                                           (True, False, False, True, True),
                                                           (False, False, False, True, True)):
                    # pk12: the date predicate reads the 12-bit packed copy (codes span < 4096);
                    # match: phase 1 reads the recorded per-run match (rt2_match), the first
                    # config with the right columns copied into run order (rt2_copy), the second
                    # through the match
                    cfg = (keys, grouped, use_runs, two, sparse, pk12, match)
                    with kernel_config.use(mj_lds_keys=keys, mj_runs=use_runs, mj_2p=two,
                                           rs_bits=sparse, rs_pack12=pk12, rt2_match=match,
                                           rt2_copy=pk12, rt2_lo16=match):
                        got = [t.cpu().numpy() for t in
                               jit.merge_join_agg(p, rstart, rlen, rbk, roff_t, comp,
                                                  nrows=len(lk), rdup=False, record=match,
                                                  cache_spans=match)]
                        s_, c_ = got[0].reshape(G, 2)[:, 0], got[1].reshape(G, 2)[:, 1]
                        assert (c_ == ec).all(), (cfg, c_, ec)
                        assert np.allclose(s_, es, rtol=1e-12), cfg
                        if two:
                            launcher = jit.LAST_MJ_LAUNCHER[0]
                            assert isinstance(launcher, jit_runs.TwoPhaseLauncher)
                            # a reused (cached) lowering compares 16-bit key halves (rt2_lo16)
                            assert ("a.LL[" in launcher.kt.src) == match, cfg
                            # the second launch of a lowering records the match (rt2_match)
                            got = [t.cpu().numpy() for t in launcher.launch(p)]
                            assert ("a.MATCH[" in launcher.kt.src or
                                    "a.HIT[" in launcher.kt.src) == match, cfg
                            s_, c_ = got[0].reshape(G, 2)[:, 0], got[1].reshape(G, 2)[:, 1]
                            assert (c_ == ec).all(), (cfg, "relaunch", c_, ec)
                            assert np.allclose(s_, es, rtol=1e-12), cfg
                            if sparse and not grouped:
                                assert jit_runs.pack_layout(p, comp) is not None
    finally:
        p.group_col, p.num_groups = 10, 3


def test_pack12_layout_decodes_like_the_kernel():
    """The 12-bit packed predicate copy (jit_runs.packed12, RS_PACK12): 8 codes per 3 dwords,
    stored relative to the column's smallest code; decoding with the generated kernel's shifts
    and masks gives back every code, and the packed 16-bit range test (hs_rng2 with the
    pair-clamped bounds shifted by the same offset) selects exactly the rows of the value
    compare, for ranges inside, across and outside the column's span."""
    import torch
    from hyperspace_amd.exec.encoding import Compact
    from hyperspace_amd.exec import jit_runs
    rng = np.random.default_rng(5)
    vals = rng.integers(8000, 10000, 1000).astype(np.int64)
    base = 8000 + 32768
    c = Compact(torch.from_numpy((vals - base).astype(np.int16)), 2, base, None, NL.I32,
                8000, 9999)
    assert jit_runs.pack12_ok(c)
    assert not jit_runs.pack12_ok(Compact(c.codes, 2, base, None, NL.I32, 8000, 8000 + 4096))
    w = jit_runs.packed12(c).numpy().view(np.uint32).astype(np.uint64)
    assert w.size == (1000 + 63) // 64 * 24
    a, b, cc = w[0::3], w[1::3], w[2::3]
    m = np.uint64(0xFFF)
    dec = np.stack([a & m, (a >> 12) & m, ((a >> 24) | (b << 8)) & m, (b >> 4) & m,
                    (b >> 16) & m, ((b >> 28) | (cc << 4)) & m, (cc >> 8) & m,
                    (cc >> 20) & m], axis=1).reshape(-1)[:1000].astype(np.int64)
    off = 8000 - base
    assert off == -32768 and np.array_equal(dec + off, vals - base)

    def sat16(x):
        return np.clip(x, -32768, 32767)

    def c16(lo, hi):        # hs_c16lo / hs_c16hi: ranges outside int16 never match
        if hi < -32768 or lo > 32767:
            return 32767, -32768
        return max(lo, -32768), min(hi, 32767)
    for vlo, vhi in ((8500, 9000), (7000, 8100), (9990, 12000), (100, 200), (20000, 30000),
                     (9000, 8000), (8000, 9999)):
        lo, hi = c16(vlo - base - off, vhi - base - off)
        fail = (sat16(dec - lo) < 0) | (sat16(hi - dec) < 0)    # sign of sub_sat | sub_sat
        assert np.array_equal(~fail, (vals >= vlo) & (vals <= vhi)), (vlo, vhi)


def test_run_topk_sources_compile(rt, tmp_path):
    """The key-run bits walk in hash mode (TPC-H Q3 full shape: GROUP BY l_orderkey) with and
    without the per-wavefront top-K lists (hash_agg.TopKPlan) compiles for gfx950, and the top-K
    form carries segments across windows and keeps the table probe only for keys that may
    continue into another wavefront's tiles."""
    import types
    from hyperspace_amd.exec import hash_agg as H
    from hyperspace_amd.exec import jit_runs
    jit = rt

    def col(t):
        return types.SimpleNamespace(hs_type=t, valid=None, dictionary=None, offsets=None,
                                     atype=pa.int64())
    j = _q3_params()
    comp = _q3_compacts()
    hk = H.plan_keys([(0, None, col(NL.I64), (1, 600_000_000, None))], (False, False), False)
    ks = []
    for desc in (True, False):
        for by_count in (False, True):
            tk = H.TopKPlan(1 if by_count else 0, by_count, desc, 2, 16 if desc else 32)
            k = jit_runs.gen_run_sparse_scan(j, comp, hk, tk)
            assert k.name == "hs_jit_run_bits_topk" and "hprb_" in k.src and "tcr_" in k.src
            assert "TKK" in k.src and "TKW" in k.src and "tkdmx" in k.src and "lrn_" in k.src
            assert "atomic" not in k.src.split("tkdmx")[-1]     # no atomics in the top-K flush
            ks.append(k)
    k0 = jit_runs.gen_run_sparse_scan(j, comp, hk)
    assert k0.name == "hs_jit_run_bits_hash" and "hcomp" not in k0.src
    assert jit_runs.sparse_shape(j, comp, hk, ks[0] and H.TopKPlan(0, False, True, 2)) != \
        jit_runs.sparse_shape(j, comp, hk)
    for k in ks + [k0]:
        rc = jit.runtime().hs_jit_compile_to_cache(k.src.encode(), k.name.encode(), b"gfx950",
                                                   str(tmp_path).encode())
        assert rc == 0, jit.runtime().hs_jit_last_error().decode()


def test_args_template_patch_equals_full_pack():
    """A new literal vector's argument block packed as template + patched literal slots
    (``Args.patch``: TwoPhaseLauncher / scan graph fresh path) equals packing every slot."""
    from hyperspace_amd.exec.jit import Args
    a = Args()
    for kind, name in (("p", "RK0"), ("q", "L0"), ("d", "F0"), ("q", "CL0"), ("q", "NRUNS"),
                       ("d", "A0_0"), ("p", "psum")):
        a.add(kind, name, "long long" if kind != "d" else "double")
    base = {"RK0": 1 << 40, "NRUNS": 123, "psum": 0, "L0": 5, "F0": 1.5, "CL0": -7,
            "A0_0": 2.0}
    lits = {"L0": 9, "F0": -0.25, "CL0": 3, "A0_0": 0.5, "X_not_a_slot": 1}
    full = dict(base)
    full.update({k: v for k, v in lits.items() if k != "X_not_a_slot"})
    tpl = bytearray(a.pack(base, default=0))
    assert bytes(a.patch(tpl, lits)) == a.pack(full)
    assert a.pack({"RK0": 1}, default=0) == a.pack({"RK0": 1, "L0": 0, "F0": 0.0, "CL0": 0,
                                                    "NRUNS": 0, "A0_0": 0.0, "psum": 0})


def test_rebind_matches_fresh_bind():
    """``compile.rebind``: a bound predicate list re-reads its literals from their Literal nodes
    (a plan-cache hit rewrites those in place) and equals a fresh CNF + bind of the same
    conditions; NULLs, strings and IN sets are not rebindable."""
    import datetime as dt
    from hyperspace_amd.exec import compile as CP
    from hyperspace_amd.plan import expressions as E
    d = E.Attribute("d", pa.date32())
    q = E.Attribute("q", pa.int64())
    x = E.Attribute("x", pa.float64())
    infos = {d.expr_id: CP.ColumnInfo(0, NL.I32, pa.date32()),
             q.expr_id: CP.ColumnInfo(1, NL.I64, pa.int64()),
             x.expr_id: CP.ColumnInfo(2, NL.F64, pa.float64())}
    lo, hi = E.Literal(dt.date(1994, 1, 1)), E.Literal(dt.date(1995, 1, 1))
    lq, lx = E.Literal(24), E.Literal(0.05)
    conds = [E.GreaterThanOrEqual(d, lo), E.LessThan(d, hi),
             E.Or(E.LessThan(q, lq), E.GreaterThan(lx, x)), E.Not(E.EqualTo(q, E.Literal(7)))]

    def fresh():
        return CP.bind(CP.to_cnf(conds), lambda a: infos[a.expr_id], None)

    def key(b):
        return [(p.kind, p.op, p.col, p.group, p.ilit, p.flit) for p in b.preds]
    b0 = fresh()
    assert b0.rebindable and len(b0.lits) == 5
    lo.value, hi.value, lq.value, lx.value = dt.date(1996, 3, 2), dt.date(1997, 1, 1), 25, 0.07
    rb = CP.rebind(b0)
    assert rb is not None and key(rb) == key(fresh()) and key(rb) != key(b0)
    lq.value = None
    assert CP.rebind(b0) is None
    s = E.Attribute("s", pa.string())
    infos[s.expr_id] = CP.ColumnInfo(3, NL.I32, pa.string(), pa.array(["a", "b"]))
    bs = CP.bind(CP.to_cnf([E.EqualTo(s, E.Literal("b"))]), lambda a: infos[a.expr_id], None)
    assert not bs.rebindable and CP.rebind(bs) is None
