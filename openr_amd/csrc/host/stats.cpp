// stats.cpp — fb303-style Decision counters of the drop-in.
//
// The reference exports its Decision timers and counters through
// fb303::fbData->addStatValue (SpfSolver.cpp:86-104 registers the keys;
// LinkState.cpp:727 / 818 decision.spf_runs / decision.spf_ms per runSpf,
// SpfSolver.cpp:327 / 450 decision.route_build_runs / decision.route_build_ms
// per buildRouteDb, 166 decision.get_route_for_prefix, 221 / 242
// decision.no_route_to_prefix). The drop-in keeps the same keys in one
// process-wide table (fb303 itself is not part of this engine) and adds the
// engine's own split of a single-area build: decision.gpu.prepare_ms (CSR
// flatten and uploads when stale), decision.gpu.launch_ms (kernels to stream
// sync, D2H included) and decision.gpu.materialize_ms (host RouteDb).
#include <mutex>

#include "decision.h"

namespace openr_amd {

namespace {

struct Stat {
  StatType type{StatType::COUNT};
  double sum{0};
  uint64_t samples{0};
};

std::mutex& statsMu() {
  static std::mutex mu;
  return mu;
}

std::map<std::string, Stat>& statsTable() {
  static std::map<std::string, Stat> t;
  return t;
}

}  // namespace

void addStatValue(const std::string& key, double value, StatType type) {
  std::lock_guard<std::mutex> lk(statsMu());
  Stat& s = statsTable()[key];
  s.type = type;
  s.sum += value;
  ++s.samples;
}

std::map<std::string, double> getDecisionCounters() {
  std::lock_guard<std::mutex> lk(statsMu());
  std::map<std::string, double> out;
  for (const auto& [key, s] : statsTable()) {
    if (s.type == StatType::COUNT) {
      out[key + ".count"] = s.sum;
    } else {
      out[key + ".avg"] = s.samples ? s.sum / double(s.samples) : 0.0;
      out[key + ".sum"] = s.sum;
      out[key + ".count"] = double(s.samples);
    }
  }
  return out;
}

void resetDecisionCounters() {
  std::lock_guard<std::mutex> lk(statsMu());
  statsTable().clear();
}

}  // namespace openr_amd
