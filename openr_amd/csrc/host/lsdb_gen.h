// lsdb_gen.h — generated LSDBs (gen/topogen.h) as the drop-in's structs:
// the adjacency / prefix databases of a topogen::Lsdb, loaded into a
// LinkState / PrefixState or encoded as one KvStore publication (compact
// thrift values, lsdb_codec.h). Shared by the pybind test surface and the
// host-only sanitizer harness (tests/asan/host_asan.cpp).
#pragma once

#include <string>
#include <vector>

#include "decision.h"
#include "lsdb_codec.h"
#include "../gen/topogen.h"

namespace openr_amd {

inline AdjacencyDatabase toAdjacencyDatabase(const topogen::AdjDb& d, const std::string& area) {
  AdjacencyDatabase db;
  db.thisNodeName = d.thisNodeName;
  db.isOverloaded = d.isOverloaded;
  db.nodeLabel = d.nodeLabel;
  db.area = area;
  db.nodeMetricIncrementVal = d.nodeMetricIncrementVal;
  for (const auto& a : d.adjs) {
    Adjacency x;
    x.otherNodeName = a.otherNodeName;
    x.ifName = a.ifName;
    x.otherIfName = a.otherIfName;
    x.nextHopV6 = a.nextHopV6;
    x.nextHopV4 = a.nextHopV4;
    x.metric = a.metric;
    x.adjLabel = a.adjLabel;
    x.isOverloaded = a.isOverloaded;
    x.weight = a.weight;
    db.adjacencies.push_back(x);
  }
  return db;
}

inline PrefixEntry toPrefixEntry(const topogen::Prefix& p) {
  PrefixEntry e;
  e.prefix = p.prefix;
  e.type = 1;  // LOOPBACK (RoutingBenchmarkUtils.cpp:281)
  e.metrics.path_preference = p.path_preference;
  e.metrics.source_preference = p.source_preference;
  e.metrics.distance = p.distance;
  e.metrics.drain_metric = p.drain_metric;
  if (p.minNexthop >= 0) e.minNexthop = p.minNexthop;
  e.tags.insert(p.tags.begin(), p.tags.end());
  return e;
}

inline void loadLsdb(const topogen::Lsdb& g, LinkState& ls, PrefixState& ps) {
  for (const auto& d : g.adjDbs) ls.updateAdjacencyDatabase(toAdjacencyDatabase(d, g.area), g.area);
  for (const auto& p : g.prefixes) ps.updatePrefix(p.node, g.area, toPrefixEntry(p));
}

// A generated LSDB as one KvStore publication (§8(f) f4): "adj:<node>" ->
// compact AdjacencyDatabase, "prefix:<node>:[<prefix>]" -> compact
// PrefixDatabase holding that one entry (the per-prefix key format of
// PrefixKey, LsdbTypes.cpp:15-26).
inline void lsdbPublication(const topogen::Lsdb& g, std::vector<std::string>& keys,
                            std::vector<std::string>& vals) {
  for (const auto& d : g.adjDbs) {
    keys.push_back("adj:" + d.thisNodeName);
    vals.push_back(writeAdjacencyDatabase(toAdjacencyDatabase(d, g.area)));
  }
  for (const auto& p : g.prefixes) {
    PrefixDatabase db;
    db.thisNodeName = p.node;
    db.prefixEntries.push_back(toPrefixEntry(p));
    keys.push_back("prefix:" + p.node + ":[" + p.prefix + "]");
    vals.push_back(writePrefixDatabase(db));
  }
}

}  // namespace openr_amd
