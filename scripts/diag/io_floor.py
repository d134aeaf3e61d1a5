#!/usr/bin/env python
"""Box I/O floors for the index build (docs/round6-status.md, build floor table): the rates the
build's phases cannot beat on this machine, measured the way the build uses them.

* ``pwrite``: THREADS writer threads pwrite 64 MiB blocks from pinned host memory into one file
  each (the build's writer threads, exec/pq_encode.write_buckets), page cache;
* ``pread``: the same files read back from the page cache by THREADS threads into pinned
  blocks (the build's source reader, io/native_parquet);
* ``h2d`` / ``d2h``: one pinned <-> device copy of 1 GiB (torch, async + synchronize).

    python scripts/diag/io_floor.py [GB] [THREADS]
"""
import concurrent.futures as cf
import json
import os
import sys
import tempfile
import time

import torch


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    nthreads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    blk = 64 << 20
    per = int(gb * (1 << 30)) // nthreads // blk * blk
    bufs = [torch.empty(blk, dtype=torch.uint8, pin_memory=True) for _ in range(nthreads)]
    for b in bufs:
        b.fill_(7)
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    paths = [os.path.join(d, f"f{i}") for i in range(nthreads)]
    out = {"bytes": per * nthreads, "threads": nthreads}

    def write(i):
        fd = os.open(paths[i], os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        mv = memoryview(bufs[i].numpy())
        for off in range(0, per, blk):
            os.pwrite(fd, mv, off)
        os.close(fd)

    def read(i):
        fd = os.open(paths[i], os.O_RDONLY)
        mv = memoryview(bufs[i].numpy())
        for off in range(0, per, blk):
            os.preadv(fd, [mv], off)
        os.close(fd)

    with cf.ThreadPoolExecutor(nthreads) as ex:
        for name, fn in (("pwrite", write), ("pread", read), ("pread_again", read)):
            t = time.perf_counter()
            list(ex.map(fn, range(nthreads)))
            out[f"{name}_gbps"] = round(per * nthreads / (time.perf_counter() - t) / 1e9, 2)
    for p in paths:
        os.unlink(p)
    os.rmdir(d)
    n = 1 << 30
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    g = torch.empty(n, dtype=torch.uint8, device="cuda")
    for name, fn in (("h2d", lambda: g.copy_(h, non_blocking=True)),
                     ("d2h", lambda: h.copy_(g, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
        out[f"{name}_gbps"] = round(4 * n / (time.perf_counter() - t) / 1e9, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
