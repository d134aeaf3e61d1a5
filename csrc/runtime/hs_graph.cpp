// Captured HIP graphs of query pipelines with per-replay kernel arguments.
//
// A fused query pipeline (exec/graphs.py: range search + tile map + generated scan kernel +
// final fold + result copy; or the two-phase merge join's tags + bits scan + fold + copy) is
// captured once from a stream and replayed per query.  The generated kernels take their literals
// in a by-value argument struct (kernarg segment): reading that struct from device memory instead
// would turn every column load of the kernel into a flat load (the compiler cannot prove a pointer
// read from memory is global), which measured ~2x slower on gfx950.  So instead of a parameter
// copy node, each replay rewrites the argument blocks of the captured kernel nodes
// (hipGraphExecKernelNodeSetParams) and launches the executable graph.
//
// C ABI (ctypes, hyperspace_amd/exec/graphs.py):
//   hs_graph_capture_begin(stream)
//   hs_graph_capture_end(stream, funcs, nfuncs) -> handle   (kernel node i = first node of funcs[i])
//   hs_graph_set_args(handle, i, args, size)                 (next launches use these arguments)
//   hs_graph_launch(handle, stream)
//   hs_graph_replay(handle, nblocks, blocks, stream, after, done)
//       one query's replay in one call: optionally order ``stream`` after ``after``'s queued
//       work, rewrite the first nblocks kernel nodes' argument blocks, launch, and record the
//       slot's ``done`` event (the Python side's per-call overhead was several torch stream /
//       event calls per query)
//   hs_graph_destroy(handle)
//   hs_event_create() / hs_event_record(ev, stream) / hs_event_query(ev) / hs_event_sync(ev) /
//   hs_event_destroy(ev)       (timing-disabled events of the replay slots)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

struct HsGraph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipEvent_t join = nullptr;               // hs_graph_replay's ``after`` ordering event
  std::vector<hipGraphNode_t> nodes;       // the kernel node of funcs[i]
  std::vector<hipKernelNodeParams> params;  // its captured launch configuration
};

int fail(const char* what, hipError_t e) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return (int)e;
}

}  // namespace

extern "C" {

const char* hs_graph_last_error() { return g_err.c_str(); }

int hs_graph_capture_begin(void* stream) {
  const hipError_t e = hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeThreadLocal);
  return e == hipSuccess ? 0 : fail("hipStreamBeginCapture", e);
}

// Ends the capture and instantiates.  funcs[i] (hipFunction_t of a generated kernel) names the
// kernel node whose arguments hs_graph_set_args(.., i, ..) rewrites: the first captured kernel
// node launching that function not already taken.  Returns nullptr on failure.
void* hs_graph_capture_end(void* stream, void** funcs, int nfuncs) {
  hipGraph_t graph = nullptr;
  hipError_t e = hipStreamEndCapture((hipStream_t)stream, &graph);
  if (e != hipSuccess || graph == nullptr) {
    fail("hipStreamEndCapture", e);
    return nullptr;
  }
  auto* g = new HsGraph();
  g->graph = graph;
  size_t n = 0;
  e = hipGraphGetNodes(graph, nullptr, &n);
  std::vector<hipGraphNode_t> all(n);
  if (e == hipSuccess && n) e = hipGraphGetNodes(graph, all.data(), &n);
  if (e != hipSuccess) {
    fail("hipGraphGetNodes", e);
    hipGraphDestroy(graph);
    delete g;
    return nullptr;
  }
  std::vector<char> taken(n, 0);
  for (int i = 0; i < nfuncs; ++i) {
    bool found = false;
    for (size_t k = 0; k < n && !found; ++k) {
      if (taken[k]) continue;
      hipGraphNodeType t;
      if (hipGraphNodeGetType(all[k], &t) != hipSuccess || t != hipGraphNodeTypeKernel) continue;
      hipKernelNodeParams p;
      std::memset(&p, 0, sizeof(p));
      if (hipGraphKernelNodeGetParams(all[k], &p) != hipSuccess) continue;
      if (p.func != funcs[i]) continue;
      taken[k] = 1;
      g->nodes.push_back(all[k]);
      g->params.push_back(p);
      found = true;
    }
    if (!found) {
      g_err = "hs_graph_capture_end: kernel node of function " + std::to_string(i) + " not found";
      hipGraphDestroy(graph);
      delete g;
      return nullptr;
    }
  }
  e = hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    fail("hipGraphInstantiate", e);
    hipGraphDestroy(graph);
    delete g;
    return nullptr;
  }
  return g;
}

// Kernel node i of the executable graph takes the argument block ``args`` (the generated kernels
// have ONE by-value struct parameter, so kernelParams = {args}) from its next launch on.
int hs_graph_set_args(void* handle, int i, void* args, size_t size) {
  auto* g = (HsGraph*)handle;
  if (i < 0 || (size_t)i >= g->nodes.size()) {
    g_err = "hs_graph_set_args: bad node index";
    return -1;
  }
  (void)size;
  hipKernelNodeParams p = g->params[i];
  void* kp[1] = {args};
  p.kernelParams = kp;
  p.extra = nullptr;
  const hipError_t e = hipGraphExecKernelNodeSetParams(g->exec, g->nodes[i], &p);
  return e == hipSuccess ? 0 : fail("hipGraphExecKernelNodeSetParams", e);
}

int hs_graph_launch(void* handle, void* stream) {
  auto* g = (HsGraph*)handle;
  const hipError_t e = hipGraphLaunch(g->exec, (hipStream_t)stream);
  return e == hipSuccess ? 0 : fail("hipGraphLaunch", e);
}

int hs_graph_replay(void* handle, int nblocks, void** blocks, void* stream, void* after,
                    void* done) {
  auto* g = (HsGraph*)handle;
  if (nblocks < 0 || (size_t)nblocks > g->nodes.size()) {
    g_err = "hs_graph_replay: bad block count";
    return -1;
  }
  hipError_t e;
  if (after != nullptr && after != stream) {
    if (g->join == nullptr) {
      e = hipEventCreateWithFlags(&g->join, hipEventDisableTiming);
      if (e != hipSuccess) return fail("hipEventCreateWithFlags", e);
    }
    e = hipEventRecord(g->join, (hipStream_t)after);
    if (e != hipSuccess) return fail("hipEventRecord", e);
    e = hipStreamWaitEvent((hipStream_t)stream, g->join, 0);
    if (e != hipSuccess) return fail("hipStreamWaitEvent", e);
  }
  for (int i = 0; i < nblocks; ++i) {
    if (blocks[i] == nullptr) continue;
    hipKernelNodeParams p = g->params[i];
    void* kp[1] = {blocks[i]};
    p.kernelParams = kp;
    p.extra = nullptr;
    e = hipGraphExecKernelNodeSetParams(g->exec, g->nodes[i], &p);
    if (e != hipSuccess) return fail("hipGraphExecKernelNodeSetParams", e);
  }
  e = hipGraphLaunch(g->exec, (hipStream_t)stream);
  if (e != hipSuccess) return fail("hipGraphLaunch", e);
  if (done != nullptr) {
    e = hipEventRecord((hipEvent_t)done, (hipStream_t)stream);
    if (e != hipSuccess) return fail("hipEventRecord", e);
  }
  return 0;
}

void* hs_event_create() {
  hipEvent_t ev = nullptr;
  const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    fail("hipEventCreateWithFlags", e);
    return nullptr;
  }
  return ev;
}

int hs_event_record(void* ev, void* stream) {
  const hipError_t e = hipEventRecord((hipEvent_t)ev, (hipStream_t)stream);
  return e == hipSuccess ? 0 : fail("hipEventRecord", e);
}

// 0: complete, 1: not ready, < 0: error
int hs_event_query(void* ev) {
  const hipError_t e = hipEventQuery((hipEvent_t)ev);
  if (e == hipSuccess) return 0;
  if (e == hipErrorNotReady) return 1;
  return -fail("hipEventQuery", e);
}

int hs_event_sync(void* ev) {
  const hipError_t e = hipEventSynchronize((hipEvent_t)ev);
  return e == hipSuccess ? 0 : fail("hipEventSynchronize", e);
}

void hs_event_destroy(void* ev) {
  if (ev != nullptr) hipEventDestroy((hipEvent_t)ev);
}

void hs_graph_destroy(void* handle) {
  auto* g = (HsGraph*)handle;
  if (g == nullptr) return;
  if (g->join) hipEventDestroy(g->join);
  if (g->exec) hipGraphExecDestroy(g->exec);
  if (g->graph) hipGraphDestroy(g->graph);
  delete g;
}

}  // extern "C"
