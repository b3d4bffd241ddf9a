// route_digest.h — layout-independent digest of unicast RouteDbs.
//
// The bench and the bench-size parity tests compare the engine's output with
// oracle-generated golden values without materialising hundreds of millions
// of routes as text (config C3: 2,080 sources x 208k prefixes). The digest is
// a function of the RouteDb's SEMANTIC content only -- the fields the
// reference's RibUnicastEntry / NextHopThrift carry (RibEntry.h:45-113,
// Network.thrift:61-92) -- so the oracle computes it from its DecisionRouteDb
// and the engine from its compact device records (prefix index, link-slot
// masks) with the same value. Spec (identical in oracle/refcpu/bindings.cpp):
//
//   fnv(s)   FNV-1a 64 of the bytes of s;  mix(x) splitmix64 finaliser
//   nh(n)    = mix(fnv(address "%" ifName "|" neighbor "|" area "|" act)
//                  ^ (u32(metric) << 32 | u32(weight)))
//              act = "" or "<action>:<swapLabel or -1>"
//   route(r) = h <- fnv(prefix); h <- mix(h ^ igpCost);
//              h <- mix(h ^ fnv(bestArea)); h <- mix(h ^ u32(best.drain_metric));
//              h <- mix(h ^ fnv(best.prefix));
//              h <- mix(h ^ (local ? 1 : 0) ^ (doNotInstall ? 2 : 0));
//              h <- mix(h ^ fnv(counterID or "-"));
//              h <- mix(h ^ sum over next hops of nh(n) mod 2^64)
//   unit(K, db) = XOR over routes of mix(fnv(K) ^ route(r));
//                 nullopt db: mix(fnv(K) ^ 0x4E4F4E45)
// MPLS routes are not part of it (off in the bench configs).
// XOR over routes makes the job digest independent of how prefixes or units
// are split over ranks.
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "decision.h"

namespace openr_amd {
namespace digest {

inline uint64_t fnv(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}
inline uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
inline uint64_t nhKey(const NextHopThrift& n) {
  std::string s = n.address + "%" + n.ifName.value_or("") + "|" +
      n.neighborNodeName.value_or("") + "|" + n.area.value_or("") + "|";
  if (n.mplsAction) {
    s += std::to_string(n.mplsAction->action) + ":" +
        std::to_string(n.mplsAction->swapLabel.value_or(-1));
  }
  return fnv(s);
}
inline uint64_t nhHash(uint64_t key, int32_t metric, int32_t weight) {
  return mix(key ^ (uint64_t(uint32_t(metric)) << 32 | uint32_t(weight)));
}
// route(r) with the next-hop sum supplied by the caller
inline uint64_t routeHash(uint64_t prefixHash, unsigned igpCost, uint64_t bestAreaHash,
                          int32_t drain, uint64_t bestPrefixHash, bool local,
                          bool doNotInstall, uint64_t counterHash, uint64_t nhSum) {
  uint64_t h = prefixHash;
  h = mix(h ^ igpCost);
  h = mix(h ^ bestAreaHash);
  h = mix(h ^ uint32_t(drain));
  h = mix(h ^ bestPrefixHash);
  h = mix(h ^ (local ? 1u : 0u) ^ (doNotInstall ? 2u : 0u));
  h = mix(h ^ counterHash);
  return mix(h ^ nhSum);
}
inline uint64_t route(const RibUnicastEntry& r) {
  uint64_t s = 0;
  for (const auto& n : r.nexthops) s += nhHash(nhKey(n), n.metric, n.weight);
  return routeHash(fnv(r.prefix), r.igpCost, fnv(r.bestArea),
                   r.bestPrefixEntry.metrics.drain_metric, fnv(r.bestPrefixEntry.prefix),
                   r.localRouteConsidered, r.doNotInstall, fnv(r.counterID.value_or("-")), s);
}
inline uint64_t unit(const std::string& key, const std::optional<DecisionRouteDb>& db) {
  const uint64_t k = fnv(key);
  if (!db) return mix(k ^ 0x4E4F4E45ull);
  uint64_t d = 0;
  for (const auto& [_, r] : db->unicastRoutes) d ^= mix(k ^ route(r));
  return d;
}

// Per-prefix-table hashes shared by every unit of a batch (fnv of each
// prefix, of each advertisement's prefix and area, its drain metric).
struct TableHashes {
  std::vector<uint64_t> prefix;     // [P]
  std::vector<uint8_t> isV4;        // [P]
  std::vector<uint64_t> advPrefix;  // [A]
  std::vector<uint64_t> advArea;    // [A]
  std::vector<int32_t> advDrain;    // [A]
  explicit TableHashes(const PrefixHostTable& pt);
};

// unit(K, db) straight from one unit's compact records (UnitView over the
// prefix table `pt` and the source `me` of flat topology `f`, single area,
// no RibPolicy / static routes / node labels) -- what materializeRouteDb
// would build, without building it.
uint64_t unitFromRecords(const std::string& key, const FlatTopology& f,
                         const std::string& me, const PrefixHostTable& pt,
                         const TableHashes& th, const UnitView& v,
                         bool v4OverV6Nexthop);

}  // namespace digest
}  // namespace openr_amd
