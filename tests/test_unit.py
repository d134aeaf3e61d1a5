"""Pure unit tests (no data): IndexConfig, JSON/hash utils, Murmur3 golden vectors, display
buffers, conf accessors, caches, event logger wiring.

Mirrors the reference's pure-unit tier: ``IndexConfigTest``, ``JsonUtilsTest``,
``HashingUtilsTest``, ``BufferStreamTest``, ``DisplayModeTest``, ``HyperspaceConfTest``,
``IndexCacheTest`` (mock clock) and ``BucketUnionTest.scala:101-122`` (Murmur3 vectors).
"""
import os

import numpy as np
import pyarrow as pa
import pytest

from hyperspace_amd import IndexConfig
from hyperspace_amd.index import constants as C
from hyperspace_amd.index.cache import Clock, CreationTimeBasedIndexCache, IndexCacheFactoryImpl
from hyperspace_amd.plananalysis.display import (BufferStream, ConsoleMode, HTMLMode, PlainTextMode,
                                                 Tag, get_display_mode)
from hyperspace_amd.utils import hashing, json_utils, murmur3
from hyperspace_amd.utils import path_utils as P
from hyperspace_amd.utils.cache import CacheWithTransform
from hyperspace_amd.utils.conf import HyperspaceConf, RuntimeConf


# ------------------------------------------------------------------------------------------------
# IndexConfig (IndexConfigTest)
# ------------------------------------------------------------------------------------------------
def test_index_config_validation():
    with pytest.raises(ValueError):
        IndexConfig("", ["a"])
    with pytest.raises(ValueError):
        IndexConfig("i", [])
    with pytest.raises(ValueError):
        IndexConfig("i", ["a", "A"])
    with pytest.raises(ValueError):
        IndexConfig("i", ["a"], ["b", "B"])
    with pytest.raises(ValueError):
        IndexConfig("i", ["a"], ["A"])


def test_index_config_equality_ignores_case_and_included_order():
    a = IndexConfig("Idx", ["A", "b"], ["c", "D"])
    b = IndexConfig("idx", ["a", "B"], ["d", "C"])
    assert a == b and hash(a) == hash(b)
    # indexed order matters
    assert IndexConfig("i", ["a", "b"]) != IndexConfig("i", ["b", "a"])
    assert IndexConfig("i", ["a"]) != IndexConfig("j", ["a"])


def test_index_config_builder_guards():
    cfg = IndexConfig.builder().indexName("n").indexBy("a", "b").include("c").create()
    assert cfg == IndexConfig("n", ["a", "b"], ["c"])
    with pytest.raises(RuntimeError):
        IndexConfig.builder().indexName("n").indexName("m")
    with pytest.raises(RuntimeError):
        IndexConfig.builder().indexBy("a").indexBy("b")
    with pytest.raises(RuntimeError):
        IndexConfig.builder().include("a").include("b")
    with pytest.raises(ValueError):
        IndexConfig.builder().indexName("")
    with pytest.raises(ValueError):
        IndexConfig.builder().indexName("n").create()


# ------------------------------------------------------------------------------------------------
# JSON / hashing (JsonUtilsTest, HashingUtilsTest)
# ------------------------------------------------------------------------------------------------
def test_json_pretty_jackson_style():
    s = json_utils.to_json({"a": 1, "b": [1, 2], "c": {}, "d": [], "e": None, "f": "x"})
    assert s == ('{\n  "a" : 1,\n  "b" : [ 1, 2 ],\n  "c" : { },\n  "d" : [ ],\n'
                 '  "e" : null,\n  "f" : "x"\n}')
    assert json_utils.from_json(s) == {"a": 1, "b": [1, 2], "c": {}, "d": [], "e": None, "f": "x"}


def test_json_round_trip_nested():
    obj = {"x": [{"name": "f1", "size": 1}, {"name": "f2", "size": 2}], "y": {"z": True}}
    assert json_utils.from_json(json_utils.to_json(obj)) == obj


def test_md5_hex():
    assert hashing.md5_hex("") == "d41d8cd98f00b204e9800998ecf8427e"
    assert hashing.md5_hex("abc") == "900150983cd24fb0d6963f7d28e17f72"


# ------------------------------------------------------------------------------------------------
# Spark Murmur3 (Appendix D golden vectors)
# ------------------------------------------------------------------------------------------------
def test_murmur3_golden_ints():
    h = murmur3.hash_columns([pa.array([2, 3], pa.int32())])
    assert list(h) == [1765031574, -1823081949]
    assert list(murmur3.bucket_ids([pa.array([2, 3], pa.int32())], 10)) == [4, 1]


M32 = 0xFFFFFFFF


def _py_mix_k1(k):
    k = (k * 0xCC9E2D51) & M32
    k = ((k << 15) | (k >> 17)) & M32
    return (k * 0x1B873593) & M32


def _py_mix_h1(h, k):
    h ^= k
    h = ((h << 13) | (h >> 19)) & M32
    return (h * 5 + 0xE6546B64) & M32


def _py_fmix(h, n):
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    return h ^ (h >> 16)


def _signed(u):
    return u - (1 << 32) if u & 0x80000000 else u


def _py_hash_int(v, seed):
    return _signed(_py_fmix(_py_mix_h1(seed & M32, _py_mix_k1(v & M32)), 4))


def _py_hash_long(v, seed):
    v &= (1 << 64) - 1
    h = _py_mix_h1(seed & M32, _py_mix_k1(v & M32))
    h = _py_mix_h1(h, _py_mix_k1(v >> 32))
    return _signed(_py_fmix(h, 8))


def _py_hash_bytes(b, seed):
    """Spark ``hashUnsafeBytes``: 4-byte LE words, then each tail byte mixed on its own."""
    h = seed & M32
    n4 = len(b) // 4 * 4
    for i in range(0, n4, 4):
        h = _py_mix_h1(h, _py_mix_k1(int.from_bytes(b[i:i + 4], "little")))
    for i in range(n4, len(b)):
        sb = b[i] - 256 if b[i] >= 128 else b[i]
        h = _py_mix_h1(h, _py_mix_k1(sb & M32))
    return _signed(_py_fmix(h, len(b)))


def test_murmur3_spark_known_values():
    # Spark: SELECT hash(1) == -559580957
    assert murmur3.hash_columns([pa.array([1], pa.int32())])[0] == -559580957


def test_murmur3_matches_scalar_oracle():
    rng = np.random.default_rng(3)
    ints = rng.integers(-2**31, 2**31 - 1, 200).astype(np.int32)
    longs = rng.integers(-2**63, 2**63 - 1, 200, dtype=np.int64)
    strs = ["", "a", "ab", "abc", "abcd", "abcde", "héllo wörld", "x" * 37]
    assert list(murmur3.hash_columns([pa.array(ints)])) == [_py_hash_int(int(v), 42) for v in ints]
    assert list(murmur3.hash_columns([pa.array(longs)])) == [_py_hash_long(int(v), 42) for v in longs]
    assert list(murmur3.hash_columns([pa.array(strs)])) == \
        [_py_hash_bytes(s.encode(), 42) for s in strs]
    # dates hash as int, doubles as their long bits (Spark 2.4.2: -0.0 keeps its sign bit)
    assert murmur3.hash_columns([pa.array([19000], pa.date32())])[0] == _py_hash_int(19000, 42)
    bits = int(np.array([1.5]).view(np.int64)[0])
    assert murmur3.hash_columns([pa.array([1.5])])[0] == _py_hash_long(bits, 42)
    neg0 = int(np.array([-0.0]).view(np.int64)[0])
    assert murmur3.hash_columns([pa.array([-0.0])])[0] == _py_hash_long(neg0, 42)
    assert murmur3.hash_columns([pa.array([-0.0])])[0] != murmur3.hash_columns([pa.array([0.0])])[0]
    nan_bits = 0x7FF8000000000000
    assert murmur3.hash_columns([pa.array([float("nan")])])[0] == _py_hash_long(nan_bits, 42)


def test_murmur3_decimal_and_timestamp_logical_values():
    import datetime
    import decimal
    # decimal hashes its unscaled long (Spark Murmur3Hash on DecimalType(p<=18))
    d = pa.array([decimal.Decimal("1.50"), decimal.Decimal("-2.25")], pa.decimal128(10, 2))
    assert list(murmur3.hash_columns([d])) == [_py_hash_long(150, 42), _py_hash_long(-225, 42)]
    # timestamps hash microseconds whatever the storage unit (floor for ns)
    ts = datetime.datetime(2020, 1, 2, 3, 4, 5, 678901)
    us = pa.array([ts], pa.timestamp("us"))
    for unit in ("ms", "s"):
        v = pa.array([ts.replace(microsecond=0)], pa.timestamp(unit))
        ref = pa.array([ts.replace(microsecond=0)], pa.timestamp("us"))
        assert murmur3.hash_columns([v])[0] == murmur3.hash_columns([ref])[0]
    ns = pa.array([int(us.view(pa.int64())[0].as_py()) * 1000 + 999], pa.int64()).view(
        pa.timestamp("ns"))
    assert murmur3.hash_columns([ns])[0] == murmur3.hash_columns([us])[0]
    neg_ns = pa.array([-1], pa.int64()).view(pa.timestamp("ns"))  # floor(-1 ns) = -1 us
    assert murmur3.hash_columns([neg_ns])[0] == _py_hash_long(-1, 42)


def test_device_hash_xform_codes():
    from hyperspace_amd.ops import _lib as NL
    from hyperspace_amd.ops.kernels import hash_xform
    assert hash_xform(pa.decimal128(12, 2)) == NL.XF_DECIMAL | 2
    assert hash_xform(pa.timestamp("ns")) == NL.XF_FDIV | 3
    assert hash_xform(pa.timestamp("ms")) == NL.XF_MUL | 3
    assert hash_xform(pa.timestamp("us")) == NL.XF_NONE
    assert hash_xform(pa.float64()) == NL.XF_NONE
    with pytest.raises(ValueError):
        hash_xform(pa.decimal128(18, 2))


def test_murmur3_null_keeps_seed_and_chaining():
    # A null contributes nothing: hash(null) == seed.
    assert murmur3.hash_columns([pa.array([None], pa.int32())])[0] == 42
    # Chaining: hash(a, b) == hash_b(seed=hash_a(42)).
    a = pa.array([5, 6], pa.int32())
    b = pa.array([7, 8], pa.int64())
    ha = murmur3.hash_columns([a])
    hab = murmur3.hash_columns([a, b])
    assert list(hab) == [_py_hash_long(bv, int(s)) for bv, s in zip(b.to_pylist(), ha)]


def test_murmur3_pmod_non_negative():
    h = np.array([-7, -1, 0, 5], dtype=np.int32)
    assert list(murmur3.pmod(h, 4)) == [1, 3, 0, 1]


# ------------------------------------------------------------------------------------------------
# Paths (PathUtilsTest / DataPathFilter)
# ------------------------------------------------------------------------------------------------
def test_data_path_filter():
    assert P.data_path_filter("part-0.parquet")
    assert not P.data_path_filter("_SUCCESS")
    assert not P.data_path_filter(".hidden")
    assert P.data_path_filter("_col=1")  # partition dir with '='


def test_path_helpers(tmp_path):
    q = P.make_absolute(str(tmp_path))
    assert P.is_qualified(q) and q.startswith("file:/")
    assert P.to_local(q) == str(tmp_path)
    assert P.get_name(P.join(q, "x")) == "x"
    assert P.get_parent(P.join(q, "x")) == q


# ------------------------------------------------------------------------------------------------
# Display / BufferStream (DisplayModeTest, BufferStreamTest)
# ------------------------------------------------------------------------------------------------
def test_buffer_stream_highlight_preserves_whitespace():
    b = BufferStream(PlainTextMode())
    b.write("  ").highlight("  abc  ").write_line("x")
    assert str(b) == "    <----abc---->  x\n"
    b2 = BufferStream(PlainTextMode())
    b2.highlight("   ")
    assert str(b2) == "   "


def test_display_modes_and_conf_override():
    assert HTMLMode().new_line == "<br>"
    h = BufferStream(HTMLMode()).write_line("a")
    assert h.with_tag() == "<pre>a<br></pre>"
    assert ConsoleMode().highlight_tag.open == "\u001b[42m"
    conf = RuntimeConf({C.DISPLAY_MODE: "html", C.HIGHLIGHT_BEGIN_TAG: "<<",
                        C.HIGHLIGHT_END_TAG: ">>"})
    m = get_display_mode(conf)
    assert isinstance(m, HTMLMode) and m.highlight_tag.open == "<<"
    assert isinstance(get_display_mode(RuntimeConf({})), PlainTextMode)
    assert PlainTextMode(Tag("", "")).highlight_tag.open == "<----"


# ------------------------------------------------------------------------------------------------
# Conf (HyperspaceConfTest: legacy numBuckets key precedence)
# ------------------------------------------------------------------------------------------------
def test_num_buckets_legacy_key_precedence():
    assert HyperspaceConf.num_buckets_for_index(RuntimeConf({})) == 200
    assert HyperspaceConf.num_buckets_for_index(RuntimeConf({C.INDEX_NUM_BUCKETS_LEGACY: "7"})) == 7
    assert HyperspaceConf.num_buckets_for_index(
        RuntimeConf({C.INDEX_NUM_BUCKETS_LEGACY: "7", C.INDEX_NUM_BUCKETS: "9"})) == 9


def test_hybrid_scan_delete_enabled_follows_ratio():
    c = RuntimeConf({C.INDEX_HYBRID_SCAN_DELETED_RATIO_THRESHOLD: "0"})
    assert not HyperspaceConf.hybrid_scan_delete_enabled(c)
    c.set(C.INDEX_HYBRID_SCAN_DELETED_RATIO_THRESHOLD, "0.2")
    assert HyperspaceConf.hybrid_scan_delete_enabled(c)


def test_runtime_conf_basic():
    c = RuntimeConf({"a": 1})
    assert c.get("a") == "1" and c.contains("a")
    c.unset("a")
    assert c.get("a", "d") == "d" and not c.contains("a")


# ------------------------------------------------------------------------------------------------
# Caches (IndexCacheTest with a mock clock)
# ------------------------------------------------------------------------------------------------
class MockClock(Clock):
    def __init__(self):
        self.t = 1000

    def get_time(self):
        return self.t


class _S:
    def __init__(self, conf):
        self.conf = conf


def test_creation_time_cache_expiry():
    clock = MockClock()
    s = _S(RuntimeConf({C.INDEX_CACHE_EXPIRY_DURATION_SECONDS: "10"}))
    cache = CreationTimeBasedIndexCache(s, clock)
    assert cache.get() is None
    cache.set(["e1"])
    assert cache.get() == ["e1"]
    clock.t += 9_999
    assert cache.get() == ["e1"]
    clock.t += 1
    assert cache.get() is None
    cache.set(["e2"])
    cache.clear()
    assert cache.get() is None
    with pytest.raises(ValueError):
        IndexCacheFactoryImpl().create(s, "nope")


def test_cache_with_transform_recomputes_on_change():
    state = {"v": "a", "n": 0}

    def transform(v):
        state["n"] += 1
        return v.upper()
    c = CacheWithTransform(lambda: state["v"], transform)
    assert c.load() == "A" and c.load() == "A" and state["n"] == 1
    state["v"] = "b"
    assert c.load() == "B" and state["n"] == 2


# ------------------------------------------------------------------------------------------------
# Event logger reflection (SparkInvolvedSuite MockEventLogger wiring)
# ------------------------------------------------------------------------------------------------
class RecordingLogger:
    events = []

    def log_event(self, e):
        RecordingLogger.events.append(e)


def test_event_logger_by_class_name():
    from hyperspace_amd.exceptions import HyperspaceException
    from hyperspace_amd.telemetry.events import NoOpEventLogger, get_event_logger
    assert isinstance(get_event_logger(RuntimeConf({})), NoOpEventLogger)
    lg = get_event_logger(RuntimeConf({C.EVENT_LOGGER_CLASS_KEY: f"{__name__}.RecordingLogger"}))
    assert isinstance(lg, RecordingLogger)
    with pytest.raises(HyperspaceException):
        get_event_logger(RuntimeConf({C.EVENT_LOGGER_CLASS_KEY: "no.such.Logger"}))


def test_lint_gate_no_undefined_names():
    """scripts/lint_names.py: no function reads a name defined nowhere (dropped imports)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "lint_names.py")],
                       cwd=root, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout


def test_negative_zero_float_keys_bucket_like_spark_2_4():
    """Spark 2.4.2 (the reference's build.sbt:19) hashes a double's raw bits: 0.0 and -0.0 land
    in different buckets (SPARK-26021, fixed only in Spark 3.0).  Kept on purpose for bucket-id
    parity with reference-built indexes; documented in docs/user-guide.md."""
    import pyarrow as pa
    from hyperspace_amd.utils import murmur3
    b = murmur3.bucket_ids([pa.array([0.0, -0.0])], 200)
    assert int(b[0]) != int(b[1])


def test_float_to_int_cast_oracle_matches_spark():
    """Host oracle of Spark's non-ANSI float -> integral casts (exec/arrow_eval._float_to_int)."""
    import pyarrow as pa
    from hyperspace_amd.exec.arrow_eval import _float_to_int
    v = pa.array([float("nan"), float("inf"), -float("inf"), 3e9, -3e9, 2.9, -2.9, 70000.5, None])
    assert _float_to_int(v, pa.int32()).to_pylist() == \
        [0, 2**31 - 1, -2**31, 2**31 - 1, -2**31, 2, -2, 70000, None]
    # short / byte: toInt then a wrapping narrow
    assert _float_to_int(v, pa.int16()).to_pylist() == [0, -1, 0, -1, 0, 2, -2, 4464, None]
    assert _float_to_int(v, pa.int8()).to_pylist() == [0, -1, 0, -1, 0, 2, -2, 112, None]
    assert _float_to_int(v, pa.int64()).to_pylist() == \
        [0, 2**63 - 1, -2**63, 3000000000, -3000000000, 2, -2, 70000, None]


def test_owner_map_lpt_and_sticky_session_map():
    """parallel/placement.py: equal weights reproduce b % W; a heavy bucket gets a rank of its
    own; the session keeps the first map it decides per (bucket count, world, mode)."""
    import types
    import numpy as np
    from hyperspace_amd.parallel.placement import OwnerMap, lpt, session_map
    for w in (1, 2, 3, 8):
        assert lpt([5.0] * 200, w).tolist() == [b % w for b in range(200)]
        assert OwnerMap.modulo(200, w).is_modulo()
    wts = [1.0] * 16
    wts[5] = 100.0
    m = OwnerMap.balanced(wts, 4)
    assert m.owners.tolist().count(m.owner(5)) == 1
    loads = m.loads(wts)
    assert loads.max() == 100.0 and loads.min() >= 5.0
    assert sorted(b for r in range(4) for b in m.owned(r)) == list(range(16))
    import torch
    bt = torch.tensor([5, 0, 15, 5], dtype=torch.int32)
    assert m.dest(bt).tolist() == [m.owner(5), m.owner(0), m.owner(15), m.owner(5)]
    sess = types.SimpleNamespace(conf={})
    first = session_map(sess, 16, 4, wts)
    assert session_map(sess, 16, 4, [1.0] * 16) is first          # sticky
    assert session_map(sess, 16, 1, wts).owners.tolist() == [0] * 16
    sess.conf = {"spark.hyperspace.mi.bucketPlacement": "modulo"}
    assert session_map(sess, 16, 4, wts).is_modulo()
    assert np.array_equal(first.owners, m.owners)


def test_bucket_chunks_cover_buckets_within_budget():
    """Bucket-range streaming plan (exec/gpu.py bucket_chunks): contiguous ranges covering every
    bucket once, each within half the budget unless a single bucket alone exceeds it."""
    from hyperspace_amd.exec.gpu import bucket_chunks
    rng = np.random.default_rng(4)
    w = rng.integers(1, 100, 200).astype(float)
    for budget in (50, 400, 2000, 10**9):
        ch = bucket_chunks(w, budget)
        assert ch[0][0] == 0 and ch[-1][1] == 200
        assert all(a[1] == b[0] for a, b in zip(ch, ch[1:]))
        for lo, hi in ch:
            assert hi > lo
            assert hi - lo == 1 or w[lo:hi].sum() <= budget // 2
    assert bucket_chunks(w, 10**9) == [(0, 200)]


def test_hostgc_settle_freezes_live_objects():
    """utils/hostgc.settle: young garbage collected, everything alive moved to the permanent
    generation (gc.freeze) so later full collections skip it."""
    import gc
    from hyperspace_amd.utils import hostgc
    keep = [[i] for i in range(1000)]
    n0 = hostgc.STATS["settles"]
    hostgc.settle()
    try:
        assert gc.get_freeze_count() >= len(keep)
        assert hostgc.STATS["settles"] == n0 + 1
        # a full settle reclaims cyclic garbage frozen by an earlier one
        import weakref

        class Node:
            pass
        a, b = Node(), Node()
        a.b, b.a = b, a
        ref = weakref.ref(a)
        hostgc.settle()
        del a, b
        assert ref() is not None           # frozen: the young passes never see it
        hostgc.settle(full=True)
        assert ref() is None
    finally:
        gc.unfreeze()


def test_derived_buffers_shrink_the_table_cache_budget():
    """Buffers a lowering keeps outside any table (device_cache.track_derived: the recorded run
    matches of exec/jit_runs.py) count against the cache budget while they live."""
    import gc
    import torch
    from hyperspace_amd.exec import device_cache as DC
    base = DC.derived_bytes()
    t = torch.empty(1000, dtype=torch.int32)
    DC.track_derived(t)
    assert DC.derived_bytes() == base + 4000
    del t
    gc.collect()
    assert DC.derived_bytes() == base
