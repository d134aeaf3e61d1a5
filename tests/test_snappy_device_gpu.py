"""Device Snappy compressor (csrc/kernels/snappy_encode.hip) against pyarrow's decompressor:
every page of every segment must round-trip, over data that exercises the skip heuristic
(incompressible runs that switch the probe stride up, matches that drop it back to 1) and pages
spanning several 64 KiB chunks.  Reference behaviour: the index files are Snappy Parquet as
Spark writes them (DataFrameWriterExtensions.scala:57-66)."""
import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu


class _Seg:
    def __init__(self, payload, page_off):
        self.payload, self.page_off = payload, page_off


def _pages(rng):
    n = 1 << 16
    rand = rng.integers(0, 256, 3 * n + 777).astype(np.uint8).tobytes()
    keys = np.sort(rng.integers(0, 10 ** 9, 40_000)).astype(np.int64).tobytes()
    doubles = (rng.random(30_000) * 1e5).round(2).tobytes()
    # incompressible stretches long enough to reach the widest stride, then a repeat of an
    # earlier stretch (a match far back), then zeros
    head = rng.integers(0, 256, 5000).astype(np.uint8).tobytes()
    mixed = head + rng.integers(0, 256, 9000).astype(np.uint8).tobytes() + head + bytes(3000) + \
        head[:700] + rng.integers(0, 256, 100).astype(np.uint8).tobytes()
    small_codes = np.repeat(rng.integers(0, 16, 5000), rng.integers(1, 40, 5000)) \
        .astype(np.uint8).tobytes()
    return [b"", b"x", b"abcdabcdabcdabcdabcdabcdabcdabcd", rand, keys, doubles, mixed,
            small_codes, bytes(n + 5), rand[:n], rand[:n - 1] + b"\0" * 40]


def test_device_snappy_round_trips_through_pyarrow():
    import torch
    from hyperspace_amd.exec import pq_encode as PE
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(17)
    segs, raws = [], []
    for s in range(2):
        pages = _pages(rng) if s == 0 else list(reversed(_pages(rng)))
        off = np.concatenate([[0], np.cumsum([len(p) for p in pages])]).astype(np.int64)
        buf = np.frombuffer(b"".join(pages) + bytes(64), dtype=np.uint8).copy()
        segs.append(_Seg(torch.from_numpy(buf).to(dev), off))
        raws.append(pages)
    npg = len(raws[0])
    packed, zoff, zsize = PE.snappy_pages(segs, 0, npg, dev)
    torch.cuda.synchronize()
    host = packed.cpu().numpy().tobytes()
    for c, pages in enumerate(raws):
        for j, raw in enumerate(pages):
            el = host[int(zoff[c][j]):int(zoff[c][j]) + int(zsize[c][j])]
            z = PE._varint(len(raw)) + el
            got = pa.decompress(z, len(raw), codec="snappy", asbytes=True) if raw else b""
            assert got == raw, (c, j, len(raw))
            # incompressible input: literals only cost their tags
            assert len(el) <= len(raw) + len(raw) // 32 + 16, (c, j, len(el), len(raw))
    # compressible pages still compress: within 2x of the host's serial Snappy parse (the wave
    # parser caps a match at 64 bytes per window; runs of one code compress ~half as well)
    for j in (4, 5, 7, 8):     # sorted keys, rounded doubles, code runs, zeros
        raw = raws[0][j]
        host_n = len(PE.snappy_stream_host(np.frombuffer(raw, dtype=np.uint8)))
        assert int(zsize[0][j]) <= 2.0 * host_n + 64, (j, int(zsize[0][j]), host_n)
    assert int(zsize[0][8]) < 0.06 * len(raws[0][8])   # zeros: 64-byte copies, 3 bytes each
