// Pipeline-stage markers for rocprofv3 (the reference has no tracer; its only
// observability is explain, PlanAnalyzer.scala:46-130).  Each executor / index-build stage
// (decode+H2D, hash, all-to-all, sort, gather, D2H+encode, probe) pushes a roctx range so that
// `rocprofv3 --marker-trace --kernel-trace` shows kernels nested under the stage that issued them.
//
// The roctx library is resolved with dlopen on first use, so the runtime has no link-time
// dependency on the profiler SDK and the markers cost one predictable branch when tracing is off.
#include <dlfcn.h>

#include <atomic>
#include <cstdint>
#include <mutex>

namespace {

using push_fn = int (*)(const char*);
using pop_fn = int (*)();
using mark_fn = void (*)(const char*);

std::once_flag g_once;
push_fn g_push = nullptr;
pop_fn g_pop = nullptr;
mark_fn g_mark = nullptr;
std::atomic<int> g_enabled{0};
std::atomic<int64_t> g_depth{0};

void resolve() {
  const char* libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                        "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "libroctx64.so.4",
                        "/opt/rocm/lib/libroctx64.so.4"};
  for (const char* name : libs) {
    void* h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
    if (!h) continue;
    g_push = (push_fn)dlsym(h, "roctxRangePushA");
    g_pop = (pop_fn)dlsym(h, "roctxRangePop");
    g_mark = (mark_fn)dlsym(h, "roctxMarkA");
    if (g_push && g_pop) return;
    g_push = nullptr;
    g_pop = nullptr;
    g_mark = nullptr;
  }
}

}  // namespace

extern "C" {

// Turns markers on (1) or off (0).  Returns 1 if a roctx library was found, 0 otherwise (the
// markers then stay no-ops, which is not an error: the stage timers still work).
int hs_trace_enable(int on) {
  std::call_once(g_once, resolve);
  g_enabled.store(on && g_push != nullptr);
  return g_push != nullptr ? 1 : 0;
}

int hs_trace_push(const char* name) {
  if (!g_enabled.load(std::memory_order_relaxed)) return -1;
  g_depth.fetch_add(1);
  return g_push(name);
}

int hs_trace_pop() {
  if (!g_enabled.load(std::memory_order_relaxed)) return -1;
  g_depth.fetch_sub(1);
  return g_pop();
}

void hs_trace_mark(const char* name) {
  if (g_enabled.load(std::memory_order_relaxed) && g_mark) g_mark(name);
}

// Open ranges (pushes minus pops) — a test hook that catches unbalanced instrumentation.
int64_t hs_trace_depth() { return g_depth.load(); }

}  // extern "C"
