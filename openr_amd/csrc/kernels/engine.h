// engine.h — per-context engine state of libopenr_gpu.so: the
// ogs_set_option knobs (EngineOptions) and the launch scratch (workspace).
// A context (ogs_ctx_create, include/openr_gpu.h) owns both, so two host
// threads with their own contexts never share a knob or a scratch buffer;
// the legacy entry points use the process default context. A context is
// thread-compatible, not thread-safe: one host thread at a time (the SURVEY
// §8(b) contract). Every option is read on the host, at launch time.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

namespace ogs {

// The defaults and meaning of each knob are documented where it is read
// (the "EngineOptions::<name>" comments) and in include/openr_gpu.h.
struct EngineOptions {
  int kspWaveTrace = 1;
  int kspHbm = 0;
  int kspQueue = 1;
  int kspStage = -1;
  int kspPrune = 1;
  int routeStream = 5;
  int routeStoreNt = 2;
  int spfLaneWalk = -1;
  int spfPreload = 1;
  int spfSeedRow = 1;
  int spfPackedScan = 1;
  int spfQueue = -1;
  int spfNinfo = 1;
  int frontierBlock = 0;
  int frontierParts = 0;
  int frontierPartsWide = 0;
  int spfFrontier = 1;
  int c4Desc = 1;
  int spfGlobal = 0;
  int spfGlobalSync = 1;
  int spfGlobalLds = 1;
  int ldsParts = 0;
  int ldsGrid = 0;
  int ldsKey16 = 1;
  int ldsTail = 1;
  int ldsBfsExit = 1;
  int ldsPull = 6;
  int ldsLead = 0;
  int ldsTailParts = 0;
  int msGroup = 0;
  int waveWgLds = 0;
  int waveUpb = 4;
  int waveOpt = 2;  // OGS_WAVE_OPT_REG_ROUTES (spf_route_wave.hip)
  int unitWidth = [] {
    const char* e = std::getenv("OGS_UNIT_WIDTH");
    return e ? std::atoi(e) : -1;
  }();
};

struct Workspace {
  void* ptr = nullptr;
  size_t bytes = 0;
};

struct EngineContext {
  int device = 0;
  EngineOptions opts;
  std::map<hipStream_t, Workspace> ws;  // grow-only scratch per stream
  ~EngineContext();
};

// the process default options (ogs_set_option)
EngineOptions& default_options();
// the context bound to the calling thread for the current call (nullptr:
// the default context)
EngineContext* bound_context();
void bind_context(EngineContext* ctx);
inline const EngineOptions& opts() {
  EngineContext* c = bound_context();
  return c ? c->opts : default_options();
}

// Scratch of at least `bytes` for launches on `stream`: the bound context's
// own buffer (no lock: one host thread per context), else the default
// context's per-(device, stream) buffer under a mutex. A grown buffer's old
// block is retired, never freed while the process runs, so a pointer handed
// to another host thread stays valid (calls on ONE stream from several
// threads still share the buffer: give each thread its own context).
hipError_t workspace(size_t bytes, hipStream_t stream, void** out);

// RAII: sets the calling thread's HIP device to `device` for one scope and
// restores the thread's previous device on exit (only when it was changed)
class DeviceGuard {
 public:
  explicit DeviceGuard(int device) {
    if (device < 0) return;
    if (hipGetDevice(&prev_) != hipSuccess) {
      ok_ = false;
      return;
    }
    if (prev_ == device) return;
    set_ = hipSetDevice(device) == hipSuccess;
    ok_ = set_;
  }
  ~DeviceGuard() {
    if (set_) (void)hipSetDevice(prev_);
  }
  // false when the thread could not be switched to the device: the call
  // must not run (it would use the caller's device with the context's
  // pointers)
  bool ok() const { return ok_; }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;

 private:
  int prev_ = -1;
  bool set_ = false;
  bool ok_ = true;
};

// RAII: binds `ctx` (and its device) to the calling thread for one call; the
// thread's previous context binding AND its previous HIP device come back on
// exit, so a thread on device 1 calling a device-0 context stays on device 1
class BoundContext {
 public:
  explicit BoundContext(EngineContext* ctx)
      : prev_(bound_context()), dev_(ctx ? ctx->device : -1) {
    bind_context(ctx);
  }
  ~BoundContext() { bind_context(prev_); }
  bool ok() const { return dev_.ok(); }
  BoundContext(const BoundContext&) = delete;
  BoundContext& operator=(const BoundContext&) = delete;

 private:
  EngineContext* prev_;
  DeviceGuard dev_;
};

}  // namespace ogs
