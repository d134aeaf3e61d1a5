#!/usr/bin/env python
"""Which host<->device copy forms run on an SDMA engine and which as a blit kernel
(``__amd_rocclr_copyBuffer``) on this ROCm, and at what rate.  Run under
``rocprofv3 --kernel-trace --memory-copy-trace``: SDMA copies appear in the memory-copy
trace, blit kernels in the kernel trace.  Prints one JSON line per variant (GB/s by events).

    python scripts/diag/d2h_probe.py [--mb 96]
"""
import argparse
import ctypes
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=96)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    n = args.mb << 20
    dev = torch.device("cuda", 0)
    src = torch.randint(0, 255, (n + 8192,), dtype=torch.uint8, device=dev)
    pin = torch.empty(n + 8192, dtype=torch.uint8, pin_memory=True)
    page = torch.empty(n + 8192, dtype=torch.uint8)
    hip = ctypes.CDLL("libamdhip64.so")
    side = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()

    def timeit(name, fn, nbytes):
        with torch.cuda.stream(side):
            fn()
        side.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            e0.record(side)
            for _ in range(args.reps):
                fn()
            e1.record(side)
        side.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        print(json.dumps({"variant": name, "bytes": nbytes, "ms": round(ms, 4),
                          "gbps": round(nbytes / ms / 1e6, 2)}), flush=True)

    # torch copy_ D2H into pinned, various offsets / lengths
    for so, do, ln in ((0, 0, n), (256, 0, n), (0, 0, n - 100), (100, 0, n), (0, 100, n),
                       (4096, 4096, n)):
        timeit(f"torch_d2h_pinned so={so} do={do} len={ln}",
               lambda so=so, do=do, ln=ln: pin[do:do + ln].copy_(src[so:so + ln],
                                                                  non_blocking=True), ln)
    timeit("torch_h2d_pinned", lambda: src[:n].copy_(pin[:n], non_blocking=True), n)
    timeit("torch_d2h_pageable", lambda: page[:n].copy_(src[:n]), n)
    # hipMemcpyAsync directly, both kinds (2 = DeviceToHost, 4 = Default)
    for kind in (2, 4):
        def f(kind=kind):
            rc = hip.hipMemcpyAsync(ctypes.c_void_p(pin.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                    ctypes.c_size_t(n), ctypes.c_int(kind),
                                    ctypes.c_void_p(side.cuda_stream))
            assert rc == 0, rc
        timeit(f"hipMemcpyAsync kind={kind}", f, n)

    def g():
        rc = hip.hipMemcpyDtoHAsync(ctypes.c_void_p(pin.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                    ctypes.c_size_t(n), ctypes.c_void_p(side.cuda_stream))
        assert rc == 0, rc
    timeit("hipMemcpyDtoHAsync", g, n)
    # a hipHostMalloc'd block (flags 0) and a hipHostRegister'ed plain block
    hp = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(hp), ctypes.c_size_t(n), ctypes.c_uint(0)) == 0

    def h():
        rc = hip.hipMemcpyAsync(hp, ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(n),
                                ctypes.c_int(2), ctypes.c_void_p(side.cuda_stream))
        assert rc == 0, rc
    timeit("hipHostMalloc(0) hipMemcpyAsync D2H", h, n)
    reg = torch.empty(n, dtype=torch.uint8)
    assert hip.hipHostRegister(ctypes.c_void_p(reg.data_ptr()), ctypes.c_size_t(n),
                               ctypes.c_uint(0)) == 0

    def r():
        rc = hip.hipMemcpyAsync(ctypes.c_void_p(reg.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                ctypes.c_size_t(n), ctypes.c_int(2),
                                ctypes.c_void_p(side.cuda_stream))
        assert rc == 0, rc
    timeit("hipHostRegister D2H", r, n)
    # H2D while host threads copy memory (the build's preads into pinned blocks run beside its
    # uploads), and two H2D copies on two streams at once
    import threading
    import numpy as np
    stop = threading.Event()
    srcs = [np.ones(64 << 20, np.uint8) for _ in range(8)]
    dsts = [np.empty(64 << 20, np.uint8) for _ in range(8)]

    def churn(k):
        while not stop.is_set():
            np.copyto(dsts[k], srcs[k])
    for threads in (4, 8):
        stop.clear()
        th = [threading.Thread(target=churn, args=(k,)) for k in range(threads)]
        for t in th:
            t.start()
        timeit(f"torch_h2d_pinned with {threads} host memcpy threads",
               lambda: src[:n].copy_(pin[:n], non_blocking=True), n)
        stop.set()
        for t in th:
            t.join()
    side2 = torch.cuda.Stream(device=dev)
    pin2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    dst2 = torch.empty(n, dtype=torch.uint8, device=dev)

    def two():
        ev = torch.cuda.Event()
        ev.record(side)
        side2.wait_event(ev)
        src[:n].copy_(pin[:n], non_blocking=True)
        with torch.cuda.stream(side2):
            dst2.copy_(pin2, non_blocking=True)
        ev2 = torch.cuda.Event()
        ev2.record(side2)
        side.wait_event(ev2)
    timeit("torch_h2d_pinned two streams at once (bytes = both)", two, 2 * n)
    torch.cuda.synchronize()
    hip.hipHostUnregister(ctypes.c_void_p(reg.data_ptr()))
    hip.hipHostFree(hp)


if __name__ == "__main__":
    main()
