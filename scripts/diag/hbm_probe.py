#!/usr/bin/env python
"""HBM read-bandwidth roof of the box, for judging the query kernels' GB/s: device-wide reads
of a multi-GB tensor by torch's tuned reduction kernels and a device-to-device copy, timed with
HIP events (best of several repetitions).  One JSON line.

    python scripts/diag/hbm_probe.py [GB]
"""
import json
import sys

import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b)
        best = ms if best is None else min(best, ms)
    return best


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    n = int(gb * (1 << 30)) // 4
    x = torch.ones(n, dtype=torch.float32, device="cuda")
    y = torch.empty_like(x)
    h = x.view(torch.int16)
    out = {"bytes": x.numel() * 4}
    ms = timed(lambda: x.sum())
    out["sum_f32_read_tbps"] = round(out["bytes"] / ms / 1e9, 3)
    ms = timed(lambda: torch.amax(h))
    out["amax_i16_read_tbps"] = round(out["bytes"] / ms / 1e9, 3)
    ms = timed(lambda: y.copy_(x))
    out["copy_rw_tbps"] = round(2 * out["bytes"] / ms / 1e9, 3)
    ms = timed(lambda: torch.count_nonzero(h > 3))
    out["cmp_count_i16_tbps"] = round(out["bytes"] / ms / 1e9, 3)
    out["device"] = torch.cuda.get_device_name(0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
