#!/usr/bin/env python
"""AddressSanitizer + UBSan run of the native host I/O layer (SURVEY §5.2 race/memory checks).

Builds ``csrc/runtime/hs_parquet.cpp``, ``hs_parquet_write.cpp`` and ``hs_avro.cpp`` (pure host
C++: Thrift footer/page-header parsing, host Snappy, RLE/bit-packed run tables, the page
planner, the Parquet writer, the Avro block decoder) with ``g++ -fsanitize=address,undefined``
into a separate library, then drives it from a child Python process that preloads the
sanitizer runtimes:

* valid files: pyarrow-written Parquet (Snappy / uncompressed, dictionary / plain, data page
  v1 / v2, with and without nulls) read chunk by chunk, expanded on the host and planned for the
  device (page tables, host-inflated pages), plus files written by the native writer;
* corrupted files: random truncations, byte flips and footer-length damage of those files —
  every call must return an error code, never read or write out of bounds;
* Snappy: random and mutated streams through the host decompressor;
* Avro: mutated container files through the native block decoder.

    python scripts/sanitize_hostio.py [--iters 300]

Exit status 0 = no sanitizer report.  GPU code is not involved (GPU sanitizers are not
available on this pool); the HIP kernels are checked by the numerics tests instead.
"""
import argparse
import ctypes as C
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ["hs_parquet.cpp", "hs_parquet_write.cpp", "hs_avro.cpp"]


def _rt(name: str) -> str:
    r = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else ""


def build(out_dir: str, tsan: bool = False) -> str:
    lib = os.path.join(out_dir, "libhs_hostio_tsan.so" if tsan else "libhs_hostio_asan.so")
    san = ["-fsanitize=thread"] if tsan else \
        ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *san, "-shared", "-fPIC",
           *[os.path.join(ROOT, "csrc", "runtime", s) for s in SOURCES], "-lz", "-o", lib]
    subprocess.run(cmd, check=True)
    return lib


def parent(iters: int, seed: int, tsan: bool = False) -> int:
    if tsan:
        rt = _rt("libtsan.so")
        if not rt:
            print("sanitizer runtimes not found", file=sys.stderr)
            return 2
        preload = rt
    else:
        asan, ubsan = _rt("libasan.so"), _rt("libubsan.so")
        if not asan or not ubsan:
            print("sanitizer runtimes not found", file=sys.stderr)
            return 2
        preload = f"{asan}:{ubsan}"
    with tempfile.TemporaryDirectory() as d:
        lib = build(d, tsan)
        env = dict(os.environ)
        env["LD_PRELOAD"] = preload
        env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1:allocator_may_return_null=1"
        env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
        # races are reported for the instrumented library only (CPython is not instrumented);
        # any report fails the run
        # pyarrow (used to write the test files) is not instrumented: its own thread pool's
        # futures read as races to TSan, so reports whose stacks are inside Arrow are
        # suppressed; the library under test is never on this list
        supp = os.path.join(d, "tsan.supp")
        with open(supp, "w") as f:
            for lib_ in ("libarrow.so", "libarrow_dataset.so", "libparquet.so",
                         "libarrow_acero.so", "libarrow_python.so", "libarrow_substrait.so"):
                f.write(f"race:{lib_}\ncalled_from_lib:{lib_}\nmutex:{lib_}\n"
                        f"deadlock:{lib_}\nthread:{lib_}\n")
        env["TSAN_OPTIONS"] = (f"halt_on_error=1:exitcode=66:report_signal_unsafe=0:"
                               f"suppressions={supp}")
        cmd = [sys.executable, os.path.abspath(__file__), "--child", lib, d, "--iters",
               str(iters), "--seed", str(seed)]
        if tsan:
            # the test files are written by an uninstrumented process first: pyarrow's own
            # thread pool must not run inside the TSan process (it is not instrumented, its
            # futures read as races); the TSan child only calls the native library
            g = subprocess.run(cmd + ["--gen-only"], env=dict(os.environ))
            if g.returncode != 0:
                return g.returncode
            cmd += ["--threads", "8", "--reuse"]
        r = subprocess.run(cmd, env=env)
        if r.returncode == 0 and tsan:
            import pyarrow.parquet as pq
            ws = [x for x in os.listdir(d) if x.startswith("w")]
            for x in ws:   # the files the threads wrote concurrently are valid Parquet
                assert pq.read_table(os.path.join(d, x, "native.parquet")).num_rows == 1331
            print(f"verified {len(ws)} concurrently written files")
        return r.returncode


def child(lib_path: str, work: str, iters: int, seed: int, threads: int = 0,
          gen_only: bool = False, reuse: bool = False) -> int:
    sys.path.insert(0, ROOT)
    import numpy as np
    import pyarrow as pa
    import pyarrow.parquet as pq

    from hyperspace_amd.exec import jit
    if not gen_only:   # the generating process (no sanitizer runtime) uses the normal build
        jit._rt = C.CDLL(lib_path)      # host I/O symbols only; bound by the modules below
    from hyperspace_amd.exec import pq_encode as PE
    from hyperspace_amd.io import avro
    from hyperspace_amd.io import native_parquet as NP

    rng = np.random.default_rng(seed)
    n = 5000
    tab = pa.table({
        "i32": pa.array(rng.integers(-1000, 1000, n).astype(np.int32)),
        "i64": pa.array(np.sort(rng.integers(0, 10**12, n))),
        "f64": pa.array(np.round(rng.random(n) * 100, 2)),
        "low": pa.array(rng.integers(0, 7, n).astype(np.int64)),
        "d": pa.array(rng.integers(8000, 9000, n).astype(np.int32)).cast(pa.date32()),
        "s": pa.array([f"v{x}" for x in rng.integers(0, 50, n)]),
    })
    manifest = os.path.join(work, "files.txt")
    if reuse:
        with open(manifest) as fh:
            files = fh.read().split()
    else:
        nulls = tab.set_column(0, "i32", pa.array(
            np.where(rng.random(n) < 0.2, None, rng.integers(0, 100, n)).tolist(), pa.int32()))
        files = []
        for comp in ("snappy", "none"):
            for dic in (True, False):
                for ver in ("1.0", "2.0"):
                    for t, tag in ((tab, "nn"), (nulls, "nu")):
                        p = os.path.join(work, f"f_{comp}_{dic}_{ver}_{tag}.parquet")
                        pq.write_table(t, p, compression=comp, use_dictionary=dic,
                                       data_page_version=ver, row_group_size=1700,
                                       data_page_size=4096)
                        files.append(p)
        # native writer file (device encoder contract, host-packed payloads)
        files.append(_native_written(PE, work, rng))
        ap = os.path.join(work, "t.avro")
        avro.write_avro(ap, tab.drop(["d"]), codec="deflate", block_rows=500)
        with open(manifest, "w") as fh:
            fh.write("\n".join(files))
        if gen_only:
            return 0

    def exercise(path: str) -> None:
        f = NP.PqFile(path)
        try:
            if not f.ok:
                return
            ncol = int(f.L.hs_pq_num_columns(f.h))
            for c in range(ncol):
                ptype, _, eb = f.column_info(c)
                for g in range(f.num_row_groups):
                    rc, buf, info, vr, lr = f.read_chunk_host(g, c)
                    if rc == NP.OK and eb in (4, 8) and info.num_values >= 0:
                        try:
                            NP.expand_host(buf, info, vr, lr,
                                           np.dtype(np.int32 if eb == 4 else np.int64))
                        except Exception:
                            pass
                if eb in (4, 8):
                    plan = [(pa.field(f"c{c}", pa.int64()), c, eb)]
                    raw_cap = sum((int(f.L.hs_pq_chunk_raw_bytes(f.h, g, c)) + 15) // 16 * 16
                                  for g in range(f.num_row_groups)) + 64
                    host_cap = sum(int(f.L.hs_pq_chunk_host_bound(f.h, g, c)) + 16
                                   for g in range(f.num_row_groups))
                    if 0 <= raw_cap < (1 << 28) and 0 <= host_cap < (1 << 28):
                        raw = np.zeros(raw_cap, np.uint8)
                        hb = np.zeros(max(host_cap, 16), np.uint8)
                        try:
                            NP.plan_file(f, plan, raw_cap, raw.ctypes.data, host_cap,
                                         hb.ctypes.data)
                        except (IOError, OSError, ValueError):
                            pass
        finally:
            f.close()

    if threads:
        return _threaded(exercise, files, PE, avro, n, work, threads, iters)
    for p in files:
        exercise(p)
    blobs = [open(p, "rb").read() for p in files]
    bad = os.path.join(work, "bad.parquet")
    for it in range(iters):
        b = bytearray(blobs[it % len(blobs)])
        kind = it % 3
        if kind == 0:
            b = b[:int(rng.integers(0, len(b)))]
        elif kind == 1:
            for _ in range(int(rng.integers(1, 16))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        else:
            k = int(rng.integers(0, 4))
            b[-8 + k] = int(rng.integers(0, 256))
        with open(bad, "wb") as fh:
            fh.write(bytes(b))
        exercise(bad)

    # Snappy: valid streams, random bytes, mutated streams
    L = NP.lib()
    for it in range(iters):
        raw = rng.integers(0, 4, int(rng.integers(1, 5000))).astype(np.uint8)
        z = PE.snappy_stream_host(raw)
        zz = bytearray(z.tobytes())
        if it % 2:
            for _ in range(int(rng.integers(1, 8))):
                zz[int(rng.integers(0, len(zz)))] = int(rng.integers(0, 256))
        if it % 5 == 4:
            zz = bytearray(rng.integers(0, 256, int(rng.integers(1, 300))).astype(np.uint8))
        src = np.frombuffer(bytes(zz), dtype=np.uint8).copy()
        cap = len(raw)
        dst = np.zeros(cap, np.uint8)
        got = L.hs_pq_snappy_decompress(src.ctypes.data, len(src), dst.ctypes.data, cap)
        if it % 2 == 0 and it % 5 != 4:
            assert got == cap and bytes(dst) == raw.tobytes(), "snappy round trip"

    # Avro: mutated containers through the native block decoder
    ap = os.path.join(work, "a.avro")
    avro.write_avro(ap, tab.drop(["d"]), codec="deflate", block_rows=700)
    avro.write_avro(os.path.join(work, "b.avro"), tab.drop(["d"]), codec="null",
                    block_rows=700)
    ablobs = [open(ap, "rb").read(), open(os.path.join(work, "b.avro"), "rb").read()]
    assert avro.read_avro(ap).num_rows == n
    badavro = os.path.join(work, "bad.avro")
    for it in range(iters):
        b = bytearray(ablobs[it % 2])
        if it % 2:
            b = b[:int(rng.integers(0, len(b)))]
        else:
            for _ in range(int(rng.integers(1, 12))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        with open(badavro, "wb") as fh:
            fh.write(bytes(b))
        try:
            avro.read_avro(badavro)
        except Exception:
            pass
    print(f"sanitized host I/O: {len(files)} files, {iters} corrupt parquet, {iters} snappy, "
          f"{iters} avro cases: clean")
    return 0


def _threaded(exercise, files, PE, avro, nrows: int, work: str, threads: int, iters: int) -> int:
    """TSan mode: the staging pool's access pattern (exec/staging.py) — many threads decoding
    and planning chunks of the same and of different files at once (ctypes releases the GIL
    for every native call), plus concurrent Snappy streams, Avro block decodes and native
    Parquet writes, each thread with its own buffers."""
    import concurrent.futures as cf

    import numpy as np
    ap = os.path.join(work, "t.avro")          # written by the generating process
    abuf = open(ap, "rb").read()
    meta, sync, start = avro.read_header(abuf)
    fields, _ = avro.schema_of(meta)
    AL = avro._lib()

    def avro_native(rows_want: int) -> None:
        """The native block decode of read_avro, without building Arrow arrays (pyarrow is not
        instrumented; its internal atomics would read as races)."""
        body = np.frombuffer(abuf, dtype=np.uint8)[start:]
        types = np.array([f[1] for f in fields], dtype=np.int32)
        nulls = np.array([f[2] for f in fields], dtype=np.int32)
        syncb = np.frombuffer(sync, dtype=np.uint8)
        h = AL.hs_avro_decode(body.ctypes.data, len(body), syncb.ctypes.data, 1, len(fields),
                              types.ctypes.data, nulls.ctypes.data)
        try:
            assert not AL.hs_avro_error(h)
            assert int(AL.hs_avro_rows(h)) == rows_want
            for k in range(len(fields)):
                for which in (0, 1, 2):
                    avro._buf(AL, h, k, which)
        finally:
            AL.hs_avro_free(h)

    def job(i: int) -> int:
        rng = np.random.default_rng(1000 + i)
        exercise(files[i % len(files)])
        exercise(files[0])                      # every thread also shares one file
        raw = rng.integers(0, 4, 4096).astype(np.uint8)
        z = PE.snappy_stream_host(raw)
        src = np.frombuffer(z.tobytes(), np.uint8).copy()
        dst = np.zeros(len(raw), np.uint8)
        from hyperspace_amd.io import native_parquet as NP
        got = NP.lib().hs_pq_snappy_decompress(src.ctypes.data, len(src), dst.ctypes.data,
                                                len(raw))
        assert got == len(raw) and bytes(dst) == raw.tobytes()
        avro_native(nrows)
        d = os.path.join(work, f"w{i}")
        os.makedirs(d, exist_ok=True)
        _native_written(PE, d, rng, verify=False)
        return i
    n = max(threads * 4, min(iters, 64))
    with cf.ThreadPoolExecutor(threads) as ex:
        done = list(ex.map(job, range(n)))
    assert done == list(range(n))
    print(f"tsan host I/O: {n} jobs on {threads} threads over {len(files)} files: clean")
    return 0


def _native_written(PE, work: str, rng, verify: bool = True) -> str:
    import numpy as np
    L = PE._writer()
    rows = [900, 431]
    cols = (PE.WCol * (2 * len(rows)))()
    keep = []
    for g, nrow in enumerate(rows):
        plain = rng.integers(0, 10**9, nrow).astype(np.int64)
        codes = rng.integers(0, 4, nrow)
        dpage = np.arange(4, dtype=np.int32).tobytes()
        pad = (-nrow) % 8
        bits = ((np.concatenate([codes, np.zeros(pad, np.int64)]).astype(np.uint64)[:, None] >>
                 np.arange(2, dtype=np.uint64)) & 1).astype(np.uint8).reshape(-1)
        packed = np.packbits(bits, bitorder="little").tobytes()
        for c, (name, pt, dic, payload) in enumerate((("k", 2, 0, plain.tobytes()),
                                                       ("c", 1, 1, packed))):
            w = cols[g * 2 + c]
            w.name, w.ptype, w.logical, w.dict, w.bit_width = name.encode(), pt, 0, dic, 2
            w.codec = 1
            raw = np.frombuffer(payload, np.uint8)
            el = PE.snappy_stream_host(raw)[len(PE._varint(len(raw))):]
            keep.append(el)
            w.payload, w.payload_bytes = el.ctypes.data, el.nbytes
            w.payload_raw_bytes = len(raw)
            if dic:
                z = PE.snappy_stream_host(np.frombuffer(dpage, np.uint8))
                keep.append(z)
                w.dict_page, w.dict_bytes, w.dict_raw_bytes = z.ctypes.data, z.nbytes, len(dpage)
                w.dict_count = 4
    path = os.path.join(work, "native.parquet")
    rg = (C.c_int64 * len(rows))(*rows)
    assert L.hs_pq_write_file(path.encode(), 2, len(rows), rg, cols, b"asan") == 0
    if verify:
        import pyarrow.parquet as pq
        assert pq.read_table(path).num_rows == sum(rows)
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", nargs=2, metavar=("LIB", "WORKDIR"))
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--tsan", action="store_true",
                    help="ThreadSanitizer build, concurrent calls from a thread pool")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--gen-only", action="store_true")
    ap.add_argument("--reuse", action="store_true")
    a = ap.parse_args()
    if a.child:
        sys.exit(child(a.child[0], a.child[1], a.iters, a.seed, a.threads, a.gen_only,
                       a.reuse))
    sys.exit(parent(a.iters, a.seed, a.tsan))


if __name__ == "__main__":
    main()
