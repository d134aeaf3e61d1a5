// Host memory + copy primitives for the graph-captured query pipelines (exec/graphs.py).
//
// Pinned parameter / result blocks are allocated here with hipHostMalloc (not through torch's
// caching host allocator, whose per-copy event bookkeeping is not capture-safe), and the H2D
// parameter copy and D2H result copy are issued with hipMemcpyAsync so that stream capture
// records them as memcpy nodes reading / writing those fixed pinned addresses on every replay.
#include <hip/hip_runtime.h>

#include <cstddef>

extern "C" {

void* hs_host_alloc(size_t n) {
  void* p = nullptr;
  if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void hs_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

// kind: 1 host->device, 2 device->host, 3 device->device
int hs_memcpy_async(void* dst, const void* src, size_t n, int kind, void* stream) {
  const hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice
                          : kind == 2 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
  return (int)hipMemcpyAsync(dst, src, n, k, (hipStream_t)stream);
}

int hs_stream_sync(void* stream) { return (int)hipStreamSynchronize((hipStream_t)stream); }

}  // extern "C"
