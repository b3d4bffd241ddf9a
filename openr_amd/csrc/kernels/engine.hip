// engine.hip — the default context, the thread's bound context and the
// launch scratch (engine.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "engine.h"

namespace ogs {

namespace {
thread_local EngineContext* t_ctx = nullptr;
std::mutex g_wsMutex;
std::map<std::pair<int, hipStream_t>, Workspace> g_ws;
std::vector<void*> g_retired;  // grown-out default-context blocks (never freed)
}  // namespace

EngineOptions& default_options() {
  static EngineOptions o;
  return o;
}

EngineContext* bound_context() { return t_ctx; }
void bind_context(EngineContext* ctx) { t_ctx = ctx; }

EngineContext::~EngineContext() {
  for (auto& [s, w] : ws) {
    if (w.ptr) (void)hipFree(w.ptr);  // device sync: no launch still reads it
  }
}

hipError_t workspace(size_t bytes, hipStream_t stream, void** out) {
  if (EngineContext* c = t_ctx) {
    Workspace& w = c->ws[stream];
    if (w.bytes < bytes) {
      if (w.ptr) {
        // the context's thread alone launches on it; a free waits for the
        // device, so no earlier launch of this context still reads it
        hipError_t e = hipFree(w.ptr);
        if (e != hipSuccess) return e;
        w.ptr = nullptr;
        w.bytes = 0;
      }
      hipError_t e = hipMalloc(&w.ptr, bytes);
      if (e != hipSuccess) return e;
      w.bytes = bytes;
    }
    *out = w.ptr;
    return hipSuccess;
  }
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lock(g_wsMutex);
  Workspace& w = g_ws[{dev, stream}];
  if (w.bytes < bytes) {
    // another host thread may hold the old pointer between its workspace()
    // and its launch: retire the block instead of freeing it
    // (geometric growth: the retired blocks never sum past the live one)
    if (w.ptr) g_retired.push_back(w.ptr);
    size_t grow = w.bytes ? std::max(bytes, 2 * w.bytes) : bytes;
    w.ptr = nullptr;
    w.bytes = 0;
    e = hipMalloc(&w.ptr, grow);
    if (e == hipErrorOutOfMemory && grow > bytes) {
      (void)hipGetLastError();  // clear the sticky OOM before the exact retry
      grow = bytes;
      e = hipMalloc(&w.ptr, grow);
    }
    if (e != hipSuccess) return e;
    w.bytes = grow;
  }
  *out = w.ptr;
  return hipSuccess;
}

}  // namespace ogs
