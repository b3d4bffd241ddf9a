// ksp2_host.cpp — LinkState::getKthPaths (reference LinkState.cpp:674-703).
// Placeholder until the KSP2 kernel lands: fails loudly.
#include "decision.h"

namespace openr_amd {

const std::vector<LinkState::Path>& LinkState::getKthPaths(
    const std::string&, const std::string&, size_t) const {
  throw std::domain_error("getKthPaths: KSP2 GPU kernel not built yet");
}

}  // namespace openr_amd
