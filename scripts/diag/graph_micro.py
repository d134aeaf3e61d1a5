"""hipGraph replay overhead on this ROCm build: host time per replay and device time per
replay of (a) a captured [H2D param copy from pinned memory + 2 kernels], (b) the same without
the copy, (c) eager launches, (d) an explicit async H2D + replay of (b).  Usage:
python scripts/diag/graph_micro.py"""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from hyperspace_amd.exec import jit  # noqa: E402
from hyperspace_amd.exec.graphs import _Pinned  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    L = jit.runtime()
    x = torch.zeros(1 << 20, device=dev)
    y = torch.zeros(1 << 20, device=dev)
    d_params = torch.empty(1024, dtype=torch.uint8, device=dev)
    h = _Pinned(1024)
    out = {}

    def work(stream, copy=True):
        if copy:
            L.hs_memcpy_async(d_params.data_ptr(), h.ptr, 1024, 1, stream)
        x.add_(1.0)
        y.mul_(0.5)

    for name, copy in (("graph_copy", True), ("graph_nocopy", False)):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            work(s.cuda_stream, copy)
            g.capture_begin()
            work(s.cuda_stream, copy)
            g.capture_end()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        for _ in range(50):
            g.replay()
        torch.cuda.synchronize()
        n = 2000
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[name] = {"host_us": (t1 - t0) / n * 1e6, "wall_us": (t2 - t0) / n * 1e6}
        # single-replay latency
        lat = []
        for _ in range(50):
            ts = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - ts)
        out[name]["latency_us"] = sorted(lat)[25] * 1e6
        if name == "graph_nocopy":
            t0 = time.perf_counter()
            st = torch.cuda.current_stream().cuda_stream
            for _ in range(n):
                L.hs_memcpy_async(d_params.data_ptr(), h.ptr, 1024, 1, st)
                g.replay()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            out["copy_then_graph"] = {"host_us": (t1 - t0) / n * 1e6, "wall_us": (t2 - t0) / n * 1e6}
    st = torch.cuda.current_stream().cuda_stream
    n = 2000
    t0 = time.perf_counter()
    for _ in range(n):
        work(st, True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["eager_copy"] = {"host_us": (t1 - t0) / n * 1e6, "wall_us": (t2 - t0) / n * 1e6}
    t0 = time.perf_counter()
    for _ in range(n):
        work(st, False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["eager_nocopy"] = {"host_us": (t1 - t0) / n * 1e6, "wall_us": (t2 - t0) / n * 1e6}
    print(json.dumps({k: {a: round(b, 2) for a, b in v.items()} for k, v in out.items()}))


if __name__ == "__main__":
    main()
