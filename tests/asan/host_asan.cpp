// host_asan.cpp — the drop-in's host code under AddressSanitizer and
// UndefinedBehaviorSanitizer (make asan). Linked with
// tests/asan/ogs_stub.cpp instead of libopenr_gpu.so: the device layer is
// host memory and no route is computed, so the harness drives exactly the
// host paths that own or recycle memory --
//   * KvStore publication decode + ingestion (LsdbIngest::processPublication,
//     per-key updateKeyInLsdb / deleteKeyFromLsdb, the hashed PrefixState
//     with inline / vector entry lists, DecisionPendingUpdates);
//   * LinkState adjacency updates (new / changed / removed links, overload
//     flips) and the CSR flatten, prefix tables (PrefixHostTable,
//     HostBatch::append);
//   * materializeRouteDb with synthetic records over the selection cache
//     (map / set node recycling between builds), DecisionRouteDb::toThrift,
//     calculateUpdate / update, and the threaded materialisation.
// Exit status 0 = every check passed (the sanitizers abort on a finding).
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "decision.h"
#include "lsdb_codec.h"
#include "lsdb_gen.h"

using namespace openr_amd;

namespace {

int failures = 0;
#define EXPECT(c)                                                   \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                   \
    }                                                               \
  } while (0)

topogen::Lsdb fabricLsdb(int pods, uint64_t seed) {
  topogen::FabricOpts o;
  o.pods = pods;
  o.planes = 4;
  o.sswPerPlane = 6;
  o.rswPerPod = 12;
  o.prefixesPerNode = 3;
  o.prefixSeed = seed;
  auto g = topogen::fabric(o);
  topogen::applyOverloads(g, 30, 20, seed + 1);
  topogen::PrefixMix m;
  m.v4Permille = 150;
  m.anycastPermille = 200;
  m.minNhPermille = 60;
  m.drainPermille = 50;
  m.tagPermille = 100;
  m.seed = seed + 2;
  topogen::applyPrefixMix(g, m);
  return g;
}

// publication ingest, then churn: metric flaps, withdrawn prefixes and
// expired keys, re-advertisements; the pending updates and the final state
// are checked against a second LSDB ingested key by key
void ingestAndChurn() {
  auto g = fabricLsdb(6, 0xA5);
  std::vector<std::string> keys, vals;
  lsdbPublication(g, keys, vals);
  std::vector<PublicationKeyVal> pub;
  for (size_t i = 0; i < keys.size(); ++i) pub.push_back(PublicationKeyVal{keys[i], vals[i]});
  // a repeated key (the last value wins) and a TTL-only key
  pub.push_back(PublicationKeyVal{keys[3], vals[3]});
  pub.push_back(PublicationKeyVal{"prefix:ttl-only", std::nullopt});
  AreaLinkStates als;
  PrefixState ps;
  LsdbIngest ing("test_node", {g.area});
  DecisionPendingUpdates pending("test_node");
  ing.processPublication(g.area, als, ps, pub, {}, pending);
  EXPECT(pending.needsRouteUpdate());
  EXPECT(!pending.updatedPrefixes().empty());
  // the same keys one by one into another state
  LinkState ls2(g.area, "test_node");
  PrefixState ps2;
  for (size_t i = 0; i < keys.size(); ++i) {
    auto u = ing.updateKeyInLsdb(g.area, ls2, ps2, keys[i], std::string_view(vals[i]));
    EXPECT(u.kind != LsdbKeyUpdate::kError);
  }
  EXPECT(ps.prefixes().size() == ps2.prefixes().size());
  LinkState& ls = als.at(g.area);
  std::mt19937_64 rng(7);
  for (int round = 0; round < 40; ++round) {
    // a metric flap / overload flip of a random node's adjacency DB
    auto d = g.adjDbs[rng() % g.adjDbs.size()];
    for (auto& a : d.adjs) {
      if (rng() % 3 == 0) a.metric = 1 + int(rng() % 9);
      if (rng() % 17 == 0) a.isOverloaded = !a.isOverloaded;
    }
    if (rng() % 5 == 0 && !d.adjs.empty()) d.adjs.pop_back();  // a link goes away
    std::vector<PublicationKeyVal> flap;
    flap.push_back(PublicationKeyVal{"adj:" + d.thisNodeName,
                                     writeAdjacencyDatabase(toAdjacencyDatabase(d, g.area))});
    // prefixes withdrawn / re-advertised
    std::vector<std::string> expired;
    for (int k = 0; k < 20; ++k) {
      const auto& p = g.prefixes[rng() % g.prefixes.size()];
      const std::string key = "prefix:" + p.node + ":[" + p.prefix + "]";
      if (rng() % 2) {
        expired.push_back(key);
      } else {
        PrefixDatabase db;
        db.thisNodeName = p.node;
        db.prefixEntries.push_back(toPrefixEntry(p));
        db.prefixEntries.back().metrics.distance = int32_t(rng() % 4);
        flap.push_back(PublicationKeyVal{key, writePrefixDatabase(db)});
      }
    }
    DecisionPendingUpdates pu("test_node");
    ing.processPublication(g.area, als, ps, flap, expired, pu);
    const FlatTopology& f = ls.flat();
    EXPECT(f.names.size() == g.adjDbs.size());
    PrefixHostTable pt;
    pt.build(ps);
    HostBatch hb;
    hb.append(f, ps, g.area);
  }
  // malformed values are dropped with an error, never crash
  for (size_t cut = 1; cut < vals[0].size(); cut += 7) {
    auto u = ing.updateKeyInLsdb(g.area, ls2, ps2, keys[0],
                                 std::string_view(vals[0]).substr(0, cut));
    (void)u;
  }
}

// PrefixState with many advertisers per prefix: inline -> vector -> inline
void prefixStateChurn() {
  PrefixState ps;
  std::mt19937_64 rng(11);
  std::map<std::pair<std::string, std::pair<std::string, std::string>>, int> model;
  for (int i = 0; i < 20000; ++i) {
    const std::string node = "n" + std::to_string(rng() % 7);
    const std::string area = rng() % 2 ? "a" : "b";
    const std::string pfx = "fc00::" + std::to_string(rng() % 50) + "/128";
    if (rng() % 3 == 0) {
      const bool had = model.erase({pfx, {node, area}}) != 0;
      EXPECT(!ps.deletePrefix(node, area, pfx).empty() == had);
    } else {
      PrefixEntry e;
      e.prefix = pfx;
      e.metrics.path_preference = int32_t(rng() % 3);
      auto& m = model[{pfx, {node, area}}];
      const bool changed = !ps.updatePrefix(node, area, e).empty();
      EXPECT(changed == (m != e.metrics.path_preference + 1));
      m = e.metrics.path_preference + 1;
    }
  }
  size_t entries = 0;
  for (const auto& [p, es] : ps.prefixes()) entries += es.size();
  EXPECT(entries == model.size());
}

// materializeRouteDb over synthetic records: the selection cache keeps its
// nodes between builds (recycled), the previous DecisionRouteDb is diffed
// and released; then the threaded form
void materialiseChurn() {
  auto g = fabricLsdb(8, 0xB7);
  LinkState ls(g.area, "test_node");
  PrefixState ps;
  loadLsdb(g, ls, ps);
  const FlatTopology& f = ls.flat();
  PrefixHostTable pt;
  pt.build(ps);
  const std::string me = g.adjDbs[5].thisNodeName;
  const uint32_t s = f.id.at(me);
  const uint32_t deg = f.rowPtr[s + 1] - f.rowPtr[s];
  const uint32_t P = uint32_t(pt.prefixes.size()), N = uint32_t(f.names.size());
  std::map<std::string, RibUnicastEntry> statics;
  std::map<std::string, RouteSelectionResult> cache;
  std::mt19937_64 rng(3);
  std::optional<DecisionRouteDb> prev;
  for (int rep = 0; rep < 12; ++rep) {
    std::vector<uint32_t> meta(P), mask(P), sel(P);
    std::vector<uint64_t> metric(P), dist(N);
    std::vector<uint32_t> nh(N);
    for (uint32_t p = 0; p < P; ++p) {
      const bool valid = rng() % 8 != 0;
      meta[p] = valid ? (OGS_ROUTE_VALID | OGS_ROUTE_SELECTED) : 0u;
      mask[p] = deg ? (1u << (rng() % std::min(deg, 32u))) : 0u;
      sel[p] = 1;
      metric[p] = 1 + rng() % 50;
    }
    for (uint32_t v = 0; v < N; ++v) {
      dist[v] = rng() % 6;
      nh[v] = deg ? (1u << (rng() % std::min(deg, 32u))) : 0u;
    }
    UnitView v;
    v.W = 1;
    v.N = N;
    v.P = P;
    v.dist = dist.data();
    v.nh = nh.data();
    v.nhStride = N;
    v.meta = meta.data();
    v.metric = metric.data();
    v.mask = mask.data();
    v.maskStride = P;
    v.sel = sel.data();
    g_materializeThreads = rep % 3 == 2 ? 4 : 1;
    DecisionRouteDb db = materializeRouteDb(ls, f, g.area, me, v, pt, rep % 2 == 0,
                                            rep % 4 == 1, statics, &cache);
    RouteDatabase t = db.toThrift();
    EXPECT(t.unicastRoutes.size() == db.unicastRoutes.size());
    if (prev) {
      DecisionRouteUpdate u = prev->calculateUpdate(db);
      prev->update(u);
      EXPECT(prev->unicastRoutes.size() == db.unicastRoutes.size());
    }
    prev = std::move(db);
  }
  g_materializeThreads = 0;
}

}  // namespace

int main() {
  ingestAndChurn();
  prefixStateChurn();
  materialiseChurn();
  std::printf("host_asan: %s (%d failed checks)\n", failures ? "FAILED" : "ok", failures);
  return failures ? 1 : 0;
}
