#!/usr/bin/env python
"""Host-side write speed into the staging pool's pinned blocks vs pageable memory: one thread's
memcpy (numpy) and pread from a page-cached file, 256 MB each.  The build's reader preads every
column chunk into a pinned block (io/native_parquet.plan_file), so a pinned mapping that the
CPU writes slowly would bound the read phase.

    python scripts/diag/pinned_write_probe.py
"""
import json
import os
import tempfile
import time

import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rate(fn, nbytes, reps=5):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return round(nbytes * reps / (time.perf_counter() - t) / 1e9, 2)


def main():
    n = 256 << 20
    src = np.ones(n, np.uint8)
    page = np.empty(n, np.uint8)
    pin_t = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    pin = pin_t.numpy()
    from hyperspace_amd.exec.staging import pinned_pool
    pool_t = pinned_pool().acquire(n)
    pool = pool_t.numpy()[:n]
    fd, path = tempfile.mkstemp(dir=os.environ.get("TMPDIR", "/tmp"))
    os.write(fd, src.tobytes())
    os.fsync(fd)
    out = {}
    for name, dst in (("pageable", page), ("torch_pinned", pin), ("pool_pinned", pool)):
        out[f"memcpy_{name}_gbps"] = rate(lambda d=dst: np.copyto(d, src), n)
        out[f"pread_{name}_gbps"] = rate(lambda d=dst: os.preadv(fd, [memoryview(d)], 0), n)
    os.close(fd)
    os.unlink(path)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
