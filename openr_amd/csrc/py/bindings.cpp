// openr_amd._decision — Python binding of the GPU drop-in (product path).
// Exposes the same surface as the CPU oracle binding so tests can drive one
// scenario through both. Every computation goes through libopenr_gpu.so.
#include <algorithm>
#include <array>
#include <chrono>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <optional>

#include <sstream>

#include "../gen/topogen.h"
#include "../host/decision.h"
#include "../host/lsdb_codec.h"
#include "../host/lsdb_gen.h"
#include "../host/route_digest.h"
#include <thread>

namespace py = pybind11;
using namespace openr_amd;

PYBIND11_MAKE_OPAQUE(openr_amd::AreaLinkStates)

namespace {

template <typename T>
T get(const py::dict& d, const char* k, T dflt) {
  if (d.contains(k) && !d[k].is_none()) return d[k].cast<T>();
  return dflt;
}

Adjacency toAdj(const py::dict& d) {
  Adjacency a;
  a.otherNodeName = get<std::string>(d, "otherNodeName", "");
  a.ifName = get<std::string>(d, "ifName", "");
  a.nextHopV6 = get<std::string>(d, "nextHopV6", "");
  a.nextHopV4 = get<std::string>(d, "nextHopV4", "");
  a.metric = get<int32_t>(d, "metric", 0);
  a.adjLabel = get<int32_t>(d, "adjLabel", 0);
  a.isOverloaded = get<bool>(d, "isOverloaded", false);
  a.rtt = get<int32_t>(d, "rtt", 0);
  a.timestamp = get<int64_t>(d, "timestamp", 0);
  a.weight = get<int64_t>(d, "weight", 1);
  a.otherIfName = get<std::string>(d, "otherIfName", "");
  a.adjOnlyUsedByOtherNode = get<bool>(d, "adjOnlyUsedByOtherNode", false);
  return a;
}

// perf events as [(nodeName, eventDescr, unixTs), ...] (None: absent)
std::optional<PerfEvents> toPerfEvents(const py::handle& h) {
  if (h.is_none()) return std::nullopt;
  PerfEvents evs;
  for (auto x : h) {
    py::tuple t = x.cast<py::tuple>();
    evs.push_back(PerfEvent{t[0].cast<std::string>(), t[1].cast<std::string>(),
                            t[2].cast<int64_t>()});
  }
  return evs;
}
py::object fromPerfEvents(const std::optional<PerfEvents>& evs) {
  if (!evs) return py::none();
  py::list out;
  for (const auto& e : *evs) out.append(py::make_tuple(e.nodeName, e.eventDescr, e.unixTs));
  return out;
}

AdjacencyDatabase toAdjDb(const py::dict& d) {
  AdjacencyDatabase db;
  db.thisNodeName = get<std::string>(d, "thisNodeName", "");
  db.isOverloaded = get<bool>(d, "isOverloaded", false);
  db.nodeLabel = get<int32_t>(d, "nodeLabel", 0);
  db.area = get<std::string>(d, "area", "");
  db.nodeMetricIncrementVal = get<int32_t>(d, "nodeMetricIncrementVal", 0);
  if (d.contains("adjacencies")) {
    for (auto h : d["adjacencies"]) db.adjacencies.push_back(toAdj(h.cast<py::dict>()));
  }
  if (d.contains("perfEvents")) db.perfEvents = toPerfEvents(d["perfEvents"]);
  return db;
}

PrefixEntry toEntry(const py::dict& d) {
  PrefixEntry e;
  e.prefix = get<std::string>(d, "prefix", "");
  e.type = get<int32_t>(d, "type", 0);
  e.forwardingType = get<int32_t>(d, "forwardingType", 0);
  e.forwardingAlgorithm = get<int32_t>(d, "forwardingAlgorithm", 0);
  if (d.contains("minNexthop") && !d["minNexthop"].is_none()) {
    e.minNexthop = d["minNexthop"].cast<int64_t>();
  }
  if (d.contains("metrics")) {
    py::dict m = d["metrics"];
    e.metrics.version = get<int32_t>(m, "version", 1);
    e.metrics.drain_metric = get<int32_t>(m, "drain_metric", 0);
    e.metrics.path_preference = get<int32_t>(m, "path_preference", 0);
    e.metrics.source_preference = get<int32_t>(m, "source_preference", 0);
    e.metrics.distance = get<int32_t>(m, "distance", 0);
  }
  if (d.contains("tags")) {
    for (auto t : d["tags"]) e.tags.insert(t.cast<std::string>());
  }
  if (d.contains("area_stack")) {
    for (auto t : d["area_stack"]) e.area_stack.push_back(t.cast<std::string>());
  }
  if (d.contains("weight") && !d["weight"].is_none()) e.weight = d["weight"].cast<int64_t>();
  return e;
}

py::dict fromEntry(const PrefixEntry& e) {
  py::dict d, m;
  d["prefix"] = e.prefix;
  d["type"] = e.type;
  d["forwardingType"] = e.forwardingType;
  d["forwardingAlgorithm"] = e.forwardingAlgorithm;
  d["minNexthop"] = e.minNexthop ? py::cast(*e.minNexthop) : py::none();
  m["version"] = e.metrics.version;
  m["drain_metric"] = e.metrics.drain_metric;
  m["path_preference"] = e.metrics.path_preference;
  m["source_preference"] = e.metrics.source_preference;
  m["distance"] = e.metrics.distance;
  d["metrics"] = m;
  d["tags"] = py::cast(std::vector<std::string>(e.tags.begin(), e.tags.end()));
  d["area_stack"] = py::cast(e.area_stack);
  d["weight"] = e.weight ? py::cast(*e.weight) : py::none();
  return d;
}

py::object optStr(const std::optional<std::string>& s) {
  return s ? py::cast(*s) : py::none();
}

py::tuple fromNh(const NextHopThrift& nh) {
  py::object act = py::none();
  if (nh.mplsAction) {
    py::object push = py::none();
    if (nh.mplsAction->pushLabels) push = py::tuple(py::cast(*nh.mplsAction->pushLabels));
    act = py::make_tuple(nh.mplsAction->action,
                         nh.mplsAction->swapLabel ? py::cast(*nh.mplsAction->swapLabel)
                                                  : py::none(),
                         push);
  }
  return py::make_tuple(nh.address, optStr(nh.ifName), nh.weight, act, nh.metric,
                        optStr(nh.area), optStr(nh.neighborNodeName));
}

NextHopThrift toNh(const py::tuple& t) {
  NextHopThrift nh;
  nh.address = t[0].cast<std::string>();
  if (!t[1].is_none()) nh.ifName = t[1].cast<std::string>();
  nh.weight = t[2].cast<int32_t>();
  if (!t[3].is_none()) {
    py::tuple a = t[3];
    MplsAction m;
    m.action = a[0].cast<int32_t>();
    if (!a[1].is_none()) m.swapLabel = a[1].cast<int32_t>();
    if (!a[2].is_none()) m.pushLabels = a[2].cast<std::vector<int32_t>>();
    nh.mplsAction = m;
  }
  nh.metric = t[4].cast<int32_t>();
  if (!t[5].is_none()) nh.area = t[5].cast<std::string>();
  if (!t[6].is_none()) nh.neighborNodeName = t[6].cast<std::string>();
  return nh;
}

py::frozenset fromNhSet(const NextHops& s) {
  py::set out;
  for (const auto& nh : s) out.add(fromNh(nh));
  return py::frozenset(out);
}

py::dict fromRoute(const RibUnicastEntry& r) {
  py::dict d;
  d["prefix"] = r.prefix;
  d["nexthops"] = fromNhSet(r.nexthops);
  d["igpCost"] = r.igpCost;
  d["bestPrefixEntry"] = fromEntry(r.bestPrefixEntry);
  d["bestArea"] = r.bestArea;
  d["doNotInstall"] = r.doNotInstall;
  d["counterID"] = optStr(r.counterID);
  d["localRouteConsidered"] = r.localRouteConsidered;
  return d;
}

RibUnicastEntry toRoute(const py::dict& d) {
  RibUnicastEntry r;
  r.prefix = d["prefix"].cast<std::string>();
  for (auto h : d["nexthops"]) r.nexthops.insert(toNh(h.cast<py::tuple>()));
  r.igpCost = get<unsigned>(d, "igpCost", 0);
  if (d.contains("bestPrefixEntry")) r.bestPrefixEntry = toEntry(d["bestPrefixEntry"]);
  r.bestArea = get<std::string>(d, "bestArea", "");
  r.doNotInstall = get<bool>(d, "doNotInstall", false);
  if (d.contains("counterID") && !d["counterID"].is_none()) {
    r.counterID = d["counterID"].cast<std::string>();
  }
  r.localRouteConsidered = get<bool>(d, "localRouteConsidered", false);
  return r;
}

py::dict fromChange(const LinkState::LinkStateChange& c) {
  py::dict d;
  d["topologyChanged"] = c.topologyChanged;
  d["linkAttributesChanged"] = c.linkAttributesChanged;
  d["nodeLabelChanged"] = c.nodeLabelChanged;
  d["addedLinks"] = c.addedLinks.size();
  return d;
}

py::dict fromAdjDb(const AdjacencyDatabase& db) {
  py::dict d;
  d["thisNodeName"] = db.thisNodeName;
  d["isOverloaded"] = db.isOverloaded;
  d["nodeLabel"] = db.nodeLabel;
  d["area"] = db.area;
  d["nodeMetricIncrementVal"] = db.nodeMetricIncrementVal;
  d["perfEvents"] = fromPerfEvents(db.perfEvents);
  py::list adjs;
  for (const auto& a : db.adjacencies) {
    py::dict x;
    x["otherNodeName"] = a.otherNodeName;
    x["ifName"] = a.ifName;
    x["otherIfName"] = a.otherIfName;
    x["nextHopV6"] = a.nextHopV6;
    x["nextHopV4"] = a.nextHopV4;
    x["metric"] = a.metric;
    x["adjLabel"] = a.adjLabel;
    x["isOverloaded"] = a.isOverloaded;
    x["rtt"] = a.rtt;
    x["timestamp"] = a.timestamp;
    x["weight"] = a.weight;
    x["adjOnlyUsedByOtherNode"] = a.adjOnlyUsedByOtherNode;
    adjs.append(x);
  }
  d["adjacencies"] = adjs;
  return d;
}

PrefixDatabase toPrefixDb(const py::dict& d) {
  PrefixDatabase db;
  db.thisNodeName = get<std::string>(d, "thisNodeName", "");
  db.deletePrefix = get<bool>(d, "deletePrefix", false);
  if (d.contains("prefixEntries")) {
    for (auto h : d["prefixEntries"]) db.prefixEntries.push_back(toEntry(h.cast<py::dict>()));
  }
  if (d.contains("perfEvents") && !d["perfEvents"].is_none()) {
    db.perfEvents.emplace();
    for (auto h : d["perfEvents"]) {
      py::tuple t = h.cast<py::tuple>();
      db.perfEvents->push_back(
          PerfEvent{t[0].cast<std::string>(), t[1].cast<std::string>(), t[2].cast<int64_t>()});
    }
  }
  return db;
}

py::dict fromPrefixDb(const PrefixDatabase& db) {
  py::dict d;
  d["thisNodeName"] = db.thisNodeName;
  d["deletePrefix"] = db.deletePrefix;
  py::list es;
  for (const auto& e : db.prefixEntries) es.append(fromEntry(e));
  d["prefixEntries"] = es;
  if (db.perfEvents) {
    py::list evs;
    for (const auto& ev : *db.perfEvents) evs.append(py::make_tuple(ev.nodeName, ev.eventDescr, ev.unixTs));
    d["perfEvents"] = evs;
  } else {
    d["perfEvents"] = py::none();
  }
  return d;
}

py::dict fromKeyUpdate(const LsdbKeyUpdate& u) {
  py::dict d;
  d["kind"] = int(u.kind);
  d["nodeName"] = u.nodeName;
  d["linkChange"] = u.kind == LsdbKeyUpdate::kAdjacency ? py::object(fromChange(u.linkChange))
                                                         : py::object(py::none());
  d["changedPrefixes"] = std::vector<std::string>(u.changedPrefixes.begin(),
                                                  u.changedPrefixes.end());
  d["perfEvents"] = fromPerfEvents(u.perfEvents);
  d["error"] = u.error;
  return d;
}

py::dict fromLink(const Link& l) {
  py::dict d;
  const auto& k = l.key();
  d["n1"] = k.first.first;
  d["if1"] = k.first.second;
  d["n2"] = k.second.first;
  d["if2"] = k.second.second;
  d["m1"] = l.getMetricFromNode(k.first.first);
  d["m2"] = l.getMetricFromNode(k.second.first);
  d["up"] = l.isUp();
  d["usable"] = l.getUsability();
  d["area"] = l.getArea();
  return d;
}

py::dict fromUpdate(const DecisionRouteUpdate& u) {
  py::dict d, uu, mu;
  for (const auto& [p, e] : u.unicastRoutesToUpdate) uu[py::str(p)] = fromRoute(e);
  for (const auto& [l, e] : u.mplsRoutesToUpdate) mu[py::int_(l)] = fromNhSet(e.nexthops);
  d["unicastRoutesToUpdate"] = uu;
  d["unicastRoutesToDelete"] = py::cast(u.unicastRoutesToDelete);
  d["mplsRoutesToUpdate"] = mu;
  d["mplsRoutesToDelete"] = py::cast(u.mplsRoutesToDelete);
  return d;
}

// Canonical text of a route DB: byte-identical format to the oracle's.
std::string canonical(const DecisionRouteDb& db) {
  std::ostringstream os;
  for (const auto& [p, r] : db.unicastRoutes) {
    os << "U " << p << " c=" << r.igpCost << " a=" << r.bestArea
       << " dm=" << r.bestPrefixEntry.metrics.drain_metric
       << " bp=" << r.bestPrefixEntry.prefix << " l=" << r.localRouteConsidered
       << " cid=" << r.counterID.value_or("-")
       << "\n";
    for (const auto& nh : r.nexthops) {
      os << "  " << nh.address << "%" << nh.ifName.value_or("") << " m=" << nh.metric
         << " w=" << nh.weight << " n=" << nh.neighborNodeName.value_or("")
         << " ar=" << nh.area.value_or("");
      if (nh.mplsAction) {
        os << " act=" << nh.mplsAction->action << ":"
           << nh.mplsAction->swapLabel.value_or(-1);
      }
      os << "\n";
    }
  }
  for (const auto& [l, r] : db.mplsRoutes) {
    os << "M " << l << "\n";
    for (const auto& nh : r.nexthops) {
      os << "  " << nh.address << "%" << nh.ifName.value_or("") << " m=" << nh.metric
         << " n=" << nh.neighborNodeName.value_or("");
      if (nh.mplsAction) {
        os << " act=" << nh.mplsAction->action << ":"
           << nh.mplsAction->swapLabel.value_or(-1);
      }
      os << "\n";
    }
  }
  return os.str();
}

// ------------------------------------------------------ generated LSDBs ---
// toAdjacencyDatabase / toPrefixEntry / loadLsdb / lsdbPublication: lsdb_gen.h

// The multi-area domain of MultiAreaOpts (config C5 defaults) + overloads
// and prefix mix per area, loaded into one LinkState per area.
void loadMultiArea(const py::dict& d, AreaLinkStates& als, PrefixState& ps) {
  topogen::MultiAreaOpts o;
  o.areas = get<int>(d, "areas", 8);
  o.nodesPerArea = get<int>(d, "nodesPerArea", 1250);
  o.abrs = get<int>(d, "abrs", 64);
  o.k = get<int>(d, "k", 3);
  o.seed = get<uint64_t>(d, "seed", 0xC5A0);
  o.prefixesPerNode = get<int>(d, "prefixesPerNode", 10);
  o.anycastPermille = get<int>(d, "anycastPermille", 50);
  auto lsdbs = topogen::multiArea(o);
  for (size_t a = 0; a < lsdbs.size(); ++a) {
    topogen::applyOverloads(lsdbs[a], get<int>(d, "adjOverloadPermille", 0),
                            get<int>(d, "nodeOverloadPermille", 0),
                            get<uint64_t>(d, "overloadSeed", 0x0F) + a);
    topogen::applySpecialMetrics(lsdbs[a], get<int>(d, "zeroMetricPermille", 0),
                                 get<int>(d, "negMetricPermille", 0),
                                 get<uint64_t>(d, "specialSeed", 0x5E) + a);
    topogen::PrefixMix m;
    m.v4Permille = get<int>(d, "v4Permille", 0);
    m.minNhPermille = get<int>(d, "minNhPermille", 0);
    m.drainPermille = get<int>(d, "drainPermille", 0);
    m.tagPermille = get<int>(d, "tagPermille", 0);
    m.seed = get<uint64_t>(d, "mixSeed", 0x3F) + a;
    topogen::applyPrefixMix(lsdbs[a], m);
    auto& ls = als.emplace(lsdbs[a].area, LinkState(lsdbs[a].area, "test_node"))
                   .first->second;
    loadLsdb(lsdbs[a], ls, ps);
  }
}

// Directed text of a link (KSP parity): n1/if1-n2/if2 in key order.
std::string linkText(const Link& l) {
  const auto& k = l.key();
  return k.first.first + "/" + k.first.second + "-" + k.second.first + "/" +
      k.second.second;
}

std::string pathsText(const std::vector<LinkState::Path>& paths) {
  std::string out;
  for (size_t i = 0; i < paths.size(); ++i) {
    if (i) out += " |";
    for (const auto& l : paths[i]) out += " " + linkText(*l);
  }
  return out;
}

topogen::GridOpts gridOpts(const py::dict& d) {
  topogen::GridOpts o;
  o.n = get<int>(d, "n", 10);
  o.prefixesPerNode = get<int>(d, "prefixesPerNode", 1);
  o.prefixSeed = get<uint64_t>(d, "prefixSeed", 0xC1);
  o.metricSeed = get<uint64_t>(d, "metricSeed", 0);
  o.metricMax = get<int>(d, "metricMax", 100);
  o.adjOverloadPermille = get<int>(d, "adjOverloadPermille", 0);
  o.nodeOverloadPermille = get<int>(d, "nodeOverloadPermille", 0);
  o.overloadSeed = get<uint64_t>(d, "overloadSeed", 0);
  return o;
}

topogen::Lsdb genLsdbRaw(const std::string& kind, const py::dict& d);

topogen::Lsdb genLsdb(const std::string& kind, const py::dict& d) {
  auto db = genLsdbRaw(kind, d);
  topogen::applySpecialMetrics(db, get<int>(d, "zeroMetricPermille", 0),
                               get<int>(d, "negMetricPermille", 0),
                               get<uint64_t>(d, "specialSeed", 0x5E));
  topogen::PrefixMix m;
  m.v4Permille = get<int>(d, "v4Permille", 0);
  m.anycastPermille = get<int>(d, "anycastPermille", 0);
  m.minNhPermille = get<int>(d, "minNhPermille", 0);
  m.drainPermille = get<int>(d, "drainPermille", 0);
  m.tagPermille = get<int>(d, "tagPermille", 0);
  m.seed = get<uint64_t>(d, "mixSeed", 0x3F);
  topogen::applyPrefixMix(db, m);
  return db;
}

topogen::Lsdb genLsdbRaw(const std::string& kind, const py::dict& d) {
  if (kind == "grid") return topogen::grid(gridOpts(d));
  if (kind == "fabric") {
    topogen::FabricOpts o;
    o.pods = get<int>(d, "pods", 32);
    o.planes = get<int>(d, "planes", 8);
    o.sswPerPlane = get<int>(d, "sswPerPlane", 36);
    o.rswPerPod = get<int>(d, "rswPerPod", 48);
    o.full = get<bool>(d, "full", true);
    o.prefixesPerNode = get<int>(d, "prefixesPerNode", 1);
    o.prefixSeed = get<uint64_t>(d, "prefixSeed", 0xC3);
    auto db = topogen::fabric(o);
    topogen::applyOverloads(db, get<int>(d, "adjOverloadPermille", 0),
                            get<int>(d, "nodeOverloadPermille", 0),
                            get<uint64_t>(d, "overloadSeed", 0x0F));
    return db;
  }
  if (kind == "wan") {
    topogen::WanOpts o;
    o.nodes = get<int>(d, "nodes", 2000);
    o.k = get<int>(d, "k", 3);
    o.seed = get<uint64_t>(d, "seed", 0xC4);
    o.prefixesPerNode = get<int>(d, "prefixesPerNode", 1);
    auto db = topogen::wan(o);
    topogen::applyOverloads(db, get<int>(d, "adjOverloadPermille", 0),
                            get<int>(d, "nodeOverloadPermille", 0),
                            get<uint64_t>(d, "overloadSeed", 0x0F));
    return db;
  }
  throw std::invalid_argument("unknown generator " + kind);
}

// ---------------------------------------------------------- BatchRunner ---
// Many (topology, source) units flattened into one graph batch and solved by
// one launch of the fused kernel. Owns its device memory.
class BatchRunner {
 public:
  BatchRunner(bool enableV4, bool sr, bool brs)
      : enableV4_(enableV4), sr_(sr), brs_(brs) {}

  void addLsdb(const topogen::Lsdb& g, const std::vector<std::string>& sources) {
    auto w = std::make_unique<Topo>();
    w->als.emplace(g.area, LinkState(g.area, "test_node"));
    w->area = g.area;
    LinkState& ls = w->als.at(g.area);
    loadLsdb(g, ls, w->ps);
    const FlatTopology& f = ls.flat();
    w->table.build(w->ps);
    const uint32_t t = uint32_t(topos_.size());
    hb_.append(f, w->ps, g.area);
    for (const auto& s : sources) {
      units_.push_back({t, f.id.at(s)});
      unitSrc_.push_back(s);
      const int deg = int(f.rowPtr[f.id.at(s) + 1] - f.rowPtr[f.id.at(s)]);
      W_ = std::max(W_, batchNhWords(deg, f.names.size(),
                                     wideDistancesNeeded(f) || f.hasZeroMetric ||
                                         f.hasWideMetric));
    }
    wide_ |= wideDistancesNeeded(f);
    exact_ |= f.hasZeroMetric || f.hasWideMetric;
    topos_.push_back(std::move(w));
  }

  void upload() {
    wide_ |= exact_;  // spf_exact.hip writes 64-bit distances
    dNodeBase_.upload(hb_.nodeBase.data(), hb_.nodeBase.size());
    dDesc_.upload(hb_.topoDesc.data(), hb_.topoDesc.size());
    dRow_.upload(hb_.rowPtr.data(), hb_.rowPtr.size());
    dEdges_.upload(hb_.edges.data(), hb_.edges.size());
    dEdgeSrc_.upload(hb_.edgeSrc.data(), hb_.edgeSrc.size());
    dFlags_.upload(hb_.nodeFlags.data(), hb_.nodeFlags.size());
    dPfxBase_.upload(hb_.pfxBase.data(), hb_.pfxBase.size());
    dAdvOff_.upload(hb_.advOff.data(), hb_.advOff.size());
    dAdvNode_.upload(hb_.advNode.data(), hb_.advNode.size());
    dAdvMetrics_.upload(hb_.advMetrics.data(), hb_.advMetrics.size());
    dAdvMinNh_.upload(hb_.advMinNh.data(), hb_.advMinNh.size());
    dPfxFlags_.upload(hb_.pfxFlags.data(), hb_.pfxFlags.size());
    std::vector<uint16_t> slots;
    std::vector<uint32_t> slotEdges;
    slotStride_ = slotOrder_ ? hb_.slotOrder(slots, &slotEdges, &slotDegree_) : 0;
    if (!slotStride_ || !slotEdgeImage_) slotDegree_ = 0;
    dSlot_.upload(slots.data(), slots.size());
    dSlotEdges_.upload(slotEdges.data(), slotEdges.size());
    dUnits_.upload(units_.data(), units_.size());
    const size_t U = units_.size(), db = wide_ ? 8 : 4;
    const size_t Sn = hb_.maxNodes, Sp = std::max(hb_.maxPrefixes, 1);
    dDist_.resize(U * Sn * db);
    dNh_.resize(U * W_ * Sn * 4);
    dMeta_.resize(U * Sp * 4);
    dMetric_.resize(U * Sp * db);
    dMask_.resize(U * W_ * Sp * 4);
    dSel_.resize(U * Sp * 4);
    dReach_.resize(std::max<size_t>(U * ((Sn + 31) / 32) * 4, 4));
  }

  void run() {
    ogs_graph g = graph();
    ogs_prefix_table pt = table();
    ogs_spf_out out{dDist_.get(), dNh_.as<uint32_t>(), dMeta_.as<uint32_t>(),
                    dMetric_.get(), dMask_.as<uint32_t>(),
                    selOut_ ? dSel_.as<uint32_t>() : nullptr,
                    exact_ ? dReach_.as<uint32_t>() : nullptr};
    ogsCheck(ogs_spf_routes(&g, hb_.maxPrefixes ? &pt : nullptr,
                            dUnits_.as<ogs_unit>(), int32_t(units_.size()),
                            flags(), W_, &out, nullptr),
             "ogs_spf_routes");
    ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
  }
  // the sel row (selected advertisers: only the best-route selection cache
  // reads it) is written unless turned off (the G1 bench's digest needs none)
  void setSelOutput(bool on) { selOut_ = on; }

  void download() {
    const size_t U = units_.size(), Sn = hb_.maxNodes,
                 Sp = std::max(hb_.maxPrefixes, 1);
    auto widen = [&](const DeviceBuffer& b, size_t n, std::vector<uint64_t>& v) {
      v.resize(n);
      if (wide_) {
        b.download(v.data(), n);
      } else {
        std::vector<uint32_t> t(n);
        b.download(t.data(), n);
        for (size_t i = 0; i < n; ++i) v[i] = t[i] == 0xFFFFFFFFu ? ~0ull : t[i];
      }
    };
    widen(dDist_, U * Sn, dist_);
    nh_.resize(U * W_ * Sn);
    dNh_.download(nh_.data(), nh_.size());
    meta_.resize(U * Sp);
    dMeta_.download(meta_.data(), meta_.size());
    widen(dMetric_, U * Sp, metric_);
    mask_.resize(U * W_ * Sp);
    dMask_.download(mask_.data(), mask_.size());
    sel_.assign(U * Sp, 0u);
    if (selOut_) dSel_.download(sel_.data(), sel_.size());
    reach_.assign(exact_ ? U * ((Sn + 31) / 32) : 0, 0u);
    if (exact_) dReach_.download(reach_.data(), reach_.size());
    ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
  }

  DecisionRouteDb routeDb(size_t u) const {
    const size_t Sn = hb_.maxNodes, Sp = std::max(hb_.maxPrefixes, 1);
    const Topo& t = *topos_.at(units_.at(u).topo);
    const LinkState& ls = t.als.at(t.area);
    UnitView v;
    v.W = W_;
    v.N = uint32_t(ls.flat().names.size());
    v.P = uint32_t(t.table.prefixes.size());
    v.dist = &dist_[u * Sn];
    v.nh = &nh_[u * W_ * Sn];
    v.nhStride = Sn;
    v.meta = &meta_[u * Sp];
    v.metric = &metric_[u * Sp];
    v.mask = &mask_[u * W_ * Sp];
    v.maskStride = Sp;
    v.sel = &sel_[u * Sp];
    v.reach = reach_.empty() ? nullptr : &reach_[u * ((Sn + 31) / 32)];
    static const std::map<std::string, RibUnicastEntry> kNoStatics;
    return materializeRouteDb(ls, ls.flat(), t.area, unitSrc_[u], v, t.table,
                              false, sr_, kNoStatics, nullptr);
  }

  uint32_t flags() const {
    return (enableV4_ ? OGS_F_ENABLE_V4 : 0u) |
        (brs_ ? OGS_F_BEST_ROUTE_SELECTION : 0u) |
        (wide_ ? OGS_F_WIDE_METRIC : 0u) | (exact_ ? OGS_F_EXACT_ORDER : 0u);
  }
  // route_digest.h unit(K, db) of every unit, straight from record arrays
  // laid out like this runner's outputs (meta / metric [U*Sp], mask
  // [U*W*Sp]; 32-bit metrics, all-ones = none): the bench digests the
  // buffers of its timed launches with this. keys[u] = the unit's key
  // (empty list: the unit's source name). Spread over `threads` threads.
  // rows (optional): row i of the arrays holds unit rows[i] -- the records
  // of a launch over a subset of this runner's units (a rank's shard).
  std::vector<uint64_t> recordsDigests(const std::vector<std::string>& keys,
                                       const uint32_t* meta, const uint32_t* metric,
                                       const uint32_t* mask, int W, int threads,
                                       const std::vector<int64_t>& rows = {}) const {
    const size_t U = rows.empty() ? units_.size() : rows.size();
    const size_t Sp = std::max(hb_.maxPrefixes, 1);
    if (!keys.empty() && keys.size() != units_.size()) {
      throw std::invalid_argument("keys: one per unit");
    }
    for (int64_t r : rows) {
      if (r < 0 || size_t(r) >= units_.size()) throw std::out_of_range("rows: unit index");
    }
    if (W != W_) throw std::invalid_argument("mask width differs from the runner's");
    for (const auto& t : topos_) {
      if (!t->hashes) t->hashes = std::make_unique<digest::TableHashes>(t->table);
    }
    std::vector<uint64_t> out(U, 0);
    threads = std::max(1, std::min<int>(threads, int(U)));
    auto work = [&](int th) {
      std::vector<uint64_t> m64(Sp);
      for (size_t i = th; i < U; i += threads) {
        const size_t u = rows.empty() ? i : size_t(rows[i]);
        const Topo& t = *topos_[units_[u].topo];
        const LinkState& ls = t.als.at(t.area);
        UnitView v;
        v.W = W;
        v.N = uint32_t(ls.flat().names.size());
        v.P = uint32_t(t.table.prefixes.size());
        v.meta = meta + i * Sp;
        for (size_t p = 0; p < v.P; ++p) m64[p] = metric[i * Sp + p];
        v.metric = m64.data();
        v.mask = mask + i * W * Sp;
        v.maskStride = Sp;
        out[i] = digest::unitFromRecords(keys.empty() ? unitSrc_[u] : keys[u], ls.flat(),
                                         unitSrc_[u], t.table, *t.hashes, v, false);
      }
    };
    std::vector<std::thread> pool;
    for (int th = 1; th < threads; ++th) pool.emplace_back(work, th);
    work(0);
    for (auto& p : pool) p.join();
    return out;
  }
  size_t numUnits() const { return units_.size(); }
  void setSlotOrder(bool on) { slotOrder_ = on; }
  bool selOut_{true};
  void setSlotEdgeImage(bool on) { slotEdgeImage_ = on; }
  const HostBatch& host() const { return hb_; }
  const std::vector<ogs_unit>& units() const { return units_; }
  int nhWords() const { return W_; }
  bool wide() const { return wide_; }
  const std::vector<uint64_t>& dist() const { return dist_; }
  const std::vector<uint32_t>& meta() const { return meta_; }
  const std::vector<uint64_t>& metric() const { return metric_; }
  const std::vector<uint32_t>& mask() const { return mask_; }

 private:
  ogs_graph graph() const {
    ogs_graph g{};
    g.num_topos = int32_t(topos_.size());
    g.max_nodes = hb_.maxNodes;
    g.max_edges = hb_.maxEdges;
    g.max_degree = hb_.maxDegree;
    g.topo_desc = dDesc_.as<uint32_t>();
    g.node_base = dNodeBase_.as<uint32_t>();
    g.row_ptr = dRow_.as<uint32_t>();
    g.edges = dEdges_.as<uint64_t>();
    g.node_flags = dFlags_.as<uint8_t>();
    g.slot_node = slotStride_ ? dSlot_.as<uint16_t>() : nullptr;
    g.slot_stride = slotStride_;
    g.slot_edges = slotDegree_ ? dSlotEdges_.as<uint32_t>() : nullptr;
    g.slot_degree = slotDegree_;
    g.edge_src = dEdgeSrc_.as<uint32_t>();
    return g;
  }
  ogs_prefix_table table() const {
    ogs_prefix_table pt{};
    pt.max_prefixes = hb_.maxPrefixes;
    pt.max_advertisements = hb_.maxAdvs;
    pt.pfx_base = dPfxBase_.as<uint32_t>();
    pt.adv_off = dAdvOff_.as<uint32_t>();
    pt.adv_node = dAdvNode_.as<uint32_t>();
    pt.adv_metrics = dAdvMetrics_.as<int32_t>();
    pt.adv_min_nh = dAdvMinNh_.as<int64_t>();
    pt.pfx_flags = dPfxFlags_.as<uint8_t>();
    return pt;
  }
  struct Topo {
    AreaLinkStates als;
    std::string area;
    PrefixState ps;
    PrefixHostTable table;
    mutable std::unique_ptr<digest::TableHashes> hashes;
  };
  bool enableV4_, sr_, brs_;
  bool slotOrder_{true}, slotEdgeImage_{true};
  int slotStride_{0}, slotDegree_{0};
  DeviceBuffer dSlot_, dSlotEdges_, dEdgeSrc_;
  std::vector<std::unique_ptr<Topo>> topos_;
  HostBatch hb_;
  std::vector<ogs_unit> units_;
  std::vector<std::string> unitSrc_;
  int W_{1};
  bool wide_{false}, exact_{false};
  DeviceBuffer dDesc_, dNodeBase_, dRow_, dEdges_, dFlags_, dPfxBase_, dAdvOff_,
      dAdvNode_, dAdvMetrics_, dAdvMinNh_, dPfxFlags_, dUnits_, dDist_, dNh_,
      dMeta_, dMetric_, dMask_, dSel_, dReach_;
  std::vector<uint64_t> dist_, metric_;
  std::vector<uint32_t> nh_, meta_, mask_, sel_, reach_;
};

// -------------------------------------------------------- VariantRunner ---
// Config C4: one generated topology, its base RouteDb from `source`, and
// `count` seeded link-failure variants (this rank's block [lo, hi)) solved in
// ONE launch with the route diff fused in -- a LinkFailureSweep (§8(f) f1)
// over a generated LSDB.
class VariantRunner {
 public:
  VariantRunner(bool enableV4, bool brs) : enableV4_(enableV4), brs_(brs) {}

  void setup(const std::string& kind, const py::dict& opts, const std::string& source,
             int count, uint64_t seed, int dualPermille, int lo, int hi) {
    g_ = genLsdb(kind, opts);
    auto variants = topogen::linkFailureVariants(g_, count, seed, dualPermille);
    // this rank's block [lo, hi) of the job's variants (hi < 0: to the end)
    hi = hi < 0 ? int(variants.size()) : std::min(hi, int(variants.size()));
    lo = std::max(0, std::min(lo, hi));
    std::vector<std::vector<LinkFailureSweep::LinkDown>> downs;
    for (int v = lo; v < hi; ++v) {
      auto& d = downs.emplace_back();
      for (const auto& l : variants[v]) d.push_back({l.a, l.ifA});
    }
    area_ = g_.area;
    sweep_.reset();
    als_.clear();
    ps_ = PrefixState();
    als_.emplace(area_, LinkState(area_, "test_node"));
    loadLsdb(g_, als_.at(area_), ps_);
    sweep_ = std::make_unique<LinkFailureSweep>(source, als_.at(area_), ps_, downs, enableV4_,
                                                brs_);
  }
  void runBase(uintptr_t stream) { sw().runBase(reinterpret_cast<void*>(stream)); }
  void setMode(int m) {
    if (m < 0 || m > 2) throw std::invalid_argument("mode must be 0, 1 or 2");
    sw().setMode(LinkFailureSweep::Mode(m));
  }
  int mode() const { return int(sw().mode()); }
  void launch(uintptr_t stream, bool records) {
    sw().launch(reinterpret_cast<void*>(stream), records);
  }
  void download() { sw().fetchRecords(); }
  void fetchUpdates(uintptr_t stream) { sw().fetchUpdates(reinterpret_cast<void*>(stream)); }
  std::string canonicalOf(size_t v) const { return canonical(sw().routeDb(v)); }
  std::string baseCanonical() const { return canonical(sw().baseRouteDb()); }
  // base RouteDb with variant v's DecisionRouteUpdate applied
  // (DecisionRouteDb::update, SpfSolver.cpp:58-72)
  std::string updatedCanonical(size_t v) const {
    DecisionRouteDb db = sw().baseRouteDb();
    db.update(sw().routeUpdate(v));
    return canonical(db);
  }
  // every variant's updated RouteDb from the parallel materialisation
  // (LinkFailureSweep::routeUpdates on `threads` host threads)
  std::vector<std::string> updatedCanonicalsAll(int threads) const {
    std::vector<std::string> out;
    const DecisionRouteDb& base = sw().baseRouteDb();
    for (const auto& u : sw().routeUpdates(threads)) {
      DecisionRouteDb db = base;
      db.update(u);
      out.push_back(canonical(db));
    }
    return out;
  }
  py::tuple updateOf(size_t v) const {
    const DecisionRouteUpdate u = sw().routeUpdate(v);
    py::list upd;
    for (const auto& [p, _] : u.unicastRoutesToUpdate) upd.append(p);
    py::list del;
    for (const auto& p : u.unicastRoutesToDelete) del.append(p);
    return py::make_tuple(upd, del);
  }
  // every variant's DecisionRouteUpdate materialised (host cost of the
  // update path): (route changes, ms to build them on `threads` host threads;
  // the updates' later destruction -- the consumer's -- is not timed)
  std::pair<uint64_t, double> materializeAll(int threads) const {
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<DecisionRouteUpdate> ups = sw().routeUpdates(threads);
    const double ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    uint64_t n = 0;
    for (const auto& u : ups) n += u.unicastRoutesToUpdate.size() + u.unicastRoutesToDelete.size();
    return {n, ms};
  }
  std::vector<std::string> changedOf(size_t v) const { return sw().changedPrefixes(v); }
  std::pair<uint32_t, uint32_t> countsOf(size_t v) const { return sw().counts(v); }
  size_t numVariants() const { return sw().numVariants(); }
  uint64_t totalChanges() const { return sw().totalChanges(); }
  py::dict shape() const {
    const HostBatch& hb = sw().batch();
    py::dict d;
    d["nodes"] = hb.maxNodes;
    d["directed_edges"] = hb.maxEdges;
    d["prefixes"] = hb.maxPrefixes;
    d["advertisements"] = hb.maxAdvs;
    d["nh_words"] = sw().nhWords();
    d["variants"] = sw().numVariants();
    return d;
  }

 private:
  LinkFailureSweep& sw() const {
    if (!sweep_) throw std::logic_error("VariantRunner: setup() first");
    return *sweep_;
  }
  bool enableV4_, brs_;
  topogen::Lsdb g_;
  std::string area_;
  AreaLinkStates als_;
  PrefixState ps_;
  std::unique_ptr<LinkFailureSweep> sweep_;
};

template <typename T>
py::array_t<T> npcopy(const std::vector<T>& v) {
  py::array_t<T> a(v.size());
  std::copy(v.begin(), v.end(), a.mutable_data());
  return a;
}

}  // namespace

namespace {
std::vector<RibPolicyStatementSpec> parseStatements(py::list stmts) {
  std::vector<RibPolicyStatementSpec> v;
  for (auto h : stmts) {
    py::dict d = h.cast<py::dict>();
    RibPolicyStatementSpec s;
    s.name = get<std::string>(d, "name", "");
    if (d.contains("prefixes") && !d["prefixes"].is_none())
      s.prefixes = d["prefixes"].cast<std::vector<std::string>>();
    if (d.contains("tags") && !d["tags"].is_none())
      s.tags = d["tags"].cast<std::vector<std::string>>();
    if (d.contains("set_weight") && !d["set_weight"].is_none()) {
      py::dict w = d["set_weight"];
      RibRouteActionWeight a;
      a.default_weight = get<int32_t>(w, "default_weight", 0);
      if (w.contains("area_to_weight"))
        a.area_to_weight = w["area_to_weight"].cast<std::map<std::string, int32_t>>();
      if (w.contains("neighbor_to_weight"))
        a.neighbor_to_weight =
            w["neighbor_to_weight"].cast<std::map<std::string, int32_t>>();
      s.set_weight = a;
    }
    if (d.contains("counterID") && !d["counterID"].is_none())
      s.counterID = d["counterID"].cast<std::string>();
    v.push_back(s);
  }
  return v;
}

// ------------------------------------------------------------ C5Runner ---
// Config C5: one multi-area domain, source `source`; a job
// = the source's multi-area RouteDb with the UCMP RibPolicy
// (SpfSolver::enqueueRouteDb, results left on the device) + getKthPaths(src,
// d, 1) and (src, d, 2) for every other node d of every area holding the
// source (one Ksp2Batch per area). Rank r of `world` keeps block r of the
// prefix table and of the destinations: routes and KSP2 units are
// independent, so there is no exchange.
class C5Runner {
 public:
  void setup(const py::dict& opts, const std::string& source, py::list policy,
             bool brs, int rank, int world) {
    loadMultiArea(opts, als_, ps_);
    if (world > 1) {
      // the rank's block of the prefixes in sorted order
      std::vector<std::string> all;
      for (const auto& [pfx, _] : ps_.prefixes()) all.push_back(pfx);
      std::sort(all.begin(), all.end());
      const size_t P = all.size();
      const size_t lo = P * rank / world, hi = P * (rank + 1) / world;
      PrefixState sub;
      for (size_t i = lo; i < hi; ++i) {
        for (const auto& [na, e] : ps_.prefixes().at(all[i])) {
          sub.updatePrefixKeyed(na.first, na.second, all[i], *e);
        }
      }
      ps_ = std::move(sub);
    }
    source_ = source;
    solver_ = std::make_unique<SpfSolver>(source, true, false, brs);
    if (!policy.empty()) {
      pol_.emplace(parseStatements(policy), 3600);
      solver_->setRibPolicy(&*pol_);
    }
    std::vector<std::pair<std::string, std::string>> all;  // (area, dest)
    for (const auto& [area, ls] : als_) {
      if (!ls.hasNode(source)) continue;
      for (const auto& n : ls.flat().names) {
        if (n != source) all.emplace_back(area, n);
      }
    }
    totalDests_ = all.size();
    const size_t lo = all.size() * rank / world, hi = all.size() * (rank + 1) / world;
    // every area's destinations in ONE Ksp2Batch (one pair of launches)
    std::vector<const LinkState*> lss;
    std::vector<std::vector<std::string>> dests;
    for (const auto& [area, ls] : als_) {
      std::vector<std::string> d;
      for (size_t i = lo; i < hi; ++i) {
        if (all[i].first == area) d.push_back(all[i].second);
      }
      if (d.empty()) continue;
      areas_.push_back(area);
      lss.push_back(&ls);
      dests.push_back(std::move(d));
    }
    if (!lss.empty()) batches_.push_back(std::make_unique<Ksp2Batch>(lss, source, dests));
  }

  void setPolicy(py::list policy) {
    solver_->setRibPolicy(nullptr);
    pol_.reset();
    if (!policy.empty()) {
      pol_.emplace(parseStatements(policy), 3600);
      solver_->setRibPolicy(&*pol_);
    }
  }
  // the source's neighbours over all areas (UCMP neighbor_to_weight keys)
  std::vector<std::string> sourceNeighbors() const {
    std::set<std::string> out;
    for (const auto& [area, ls] : als_) {
      if (!ls.hasNode(source_)) continue;
      for (const auto& l : ls.linksFromNode(source_)) {
        out.insert(l->getOtherNodeName(source_));
      }
    }
    return {out.begin(), out.end()};
  }
  std::vector<std::string> areaNames() const {
    std::vector<std::string> out;
    for (const auto& [area, _] : als_) out.push_back(area);
    return out;
  }

  void launchRoutes(uintptr_t stream) {
    solver_->enqueueRouteDb(source_, als_, ps_, reinterpret_cast<void*>(stream));
  }
  void launchKsp(uintptr_t stream) {
    for (const auto& b : batches_) b->launch(reinterpret_cast<void*>(stream));
  }
  void fetch() {
    for (const auto& b : batches_) b->fetch();
  }
  py::bytes routes() {
    auto db = solver_->buildRouteDb(source_, als_, ps_);
    return py::bytes(db ? canonical(*db) : std::string("NONE"));
  }
  // "area dest k:" + the paths, one line per (destination, k), batch order
  std::vector<std::string> kspText() const {
    std::vector<std::string> out;
    for (const auto& b : batches_) {
      for (size_t i = 0; i < b->size(); ++i) {
        for (int k = 1; k <= 2; ++k) {
          out.push_back(areas_[b->areaOf(i)] + " " + b->dests()[i] + " " +
                        std::to_string(k) + ":" + pathsText(b->paths(i, k)));
        }
      }
    }
    return out;
  }
  std::vector<std::pair<std::string, std::string>> kspDests() const {
    std::vector<std::pair<std::string, std::string>> out;
    for (const auto& b : batches_) {
      for (size_t i = 0; i < b->size(); ++i) {
        out.emplace_back(areas_[b->areaOf(i)], b->dests()[i]);
      }
    }
    return out;
  }
  // route_digest.h unit(source, RouteDb) of the last launch_routes (its
  // device results downloaded and materialised; rank-invariant: the ranks'
  // prefix blocks XOR to the whole job's)
  uint64_t routesDigest(uintptr_t stream) {
    return digest::unit(source_, solver_->collectRouteDb(source_, als_,
                                                         reinterpret_cast<void*>(stream)));
  }
  py::dict shape() const {
    py::dict d;
    size_t nodes = 0, edges = 0, srcNodes = 0, srcEdges = 0, units = 0, adv = 0;
    for (const auto& [area, ls] : als_) {
      const FlatTopology& f = ls.flat();
      nodes += f.names.size();
      edges += f.edges.size();
      if (ls.hasNode(source_)) {
        srcNodes += f.names.size();
        srcEdges += f.edges.size();
      }
    }
    for (const auto& b : batches_) units += b->numUnits();
    for (const auto& [p, e] : ps_.prefixes()) adv += e.size();
    uint64_t pe1 = 0, pe2 = 0;
    for (const auto& b : batches_) {
      pe1 += b->totalPathEdges(1);
      pe2 += b->totalPathEdges(2);
    }
    d["areas"] = als_.size();
    d["nodes"] = nodes;
    d["directed_edges"] = edges;
    d["source_area_nodes"] = srcNodes;
    d["source_area_edges"] = srcEdges;
    d["prefixes"] = ps_.prefixes().size();
    d["advertisements"] = adv;
    d["ksp_units"] = units;
    d["ksp_batches"] = batches_.size();  // launch pairs per job
    d["total_dests"] = totalDests_;
    d["path_edges_k1"] = pe1;
    d["path_edges_k2"] = pe2;
    return d;
  }

 private:
  AreaLinkStates als_;
  PrefixState ps_;
  std::string source_;
  std::optional<RibPolicy> pol_;
  std::unique_ptr<SpfSolver> solver_;
  std::vector<std::string> areas_;
  std::vector<std::unique_ptr<Ksp2Batch>> batches_;
  size_t totalDests_{0};
};

}  // namespace

PYBIND11_MODULE(_decision, m) {
  m.doc() = "MI355X (gfx950) SPF + RouteDb engine: Open/R Decision drop-in";

  m.def("device_count", []() {
    int n = 0;
    ogs_device_count(&n);
    return n;
  });
  m.def("version", []() { return std::string(ogs_version()); });
  // fb303-style Decision counters (stats.cpp)
  m.def("decision_counters", []() { return getDecisionCounters(); });
  m.def("reset_decision_counters", []() { resetDecisionCounters(); });
  // growHashTable's factor (decision.h), process-wide; for A/B runs
  m.def("set_hash_growth_factor", [](int k) { setHashGrowthFactor(k); });
  m.def("hash_growth_factor", []() { return hashGrowthFactor(); });

  py::class_<LinkState>(m, "LinkState")
      .def(py::init<const std::string&, const std::string&>())
      .def("updateAdjacencyDatabase",
           [](LinkState& s, py::dict db, const std::string& area, bool init) {
             return fromChange(s.updateAdjacencyDatabase(toAdjDb(db), area, init));
           },
           py::arg("db"), py::arg("area"), py::arg("inInitialization") = false)
      .def("deleteAdjacencyDatabase",
           [](LinkState& s, const std::string& n) {
             return fromChange(s.deleteAdjacencyDatabase(n));
           })
      .def("getSpfResult",
           [](const LinkState& s, const std::string& n, bool ulm) {
             py::dict out;
             for (const auto& [name, r] : s.getSpfResult(n, ulm)) {
               std::vector<std::string> nh(r.nextHops().begin(), r.nextHops().end());
               out[py::str(name)] = py::make_tuple(r.metric(), nh);
             }
             return out;
           },
           py::arg("node"), py::arg("useLinkMetric") = true)
      .def("prefetchKthPaths", &LinkState::prefetchKthPaths, py::arg("src"),
           py::arg("dests"))
      .def("getKthPaths",
           [](const LinkState& s, const std::string& a, const std::string& b, size_t k) {
             py::list out;
             for (const auto& p : s.getKthPaths(a, b, k)) {
               py::list path;
               for (const auto& l : p) path.append(fromLink(*l));
               out.append(path);
             }
             return out;
           })
      .def("getMetricFromAToB",
           [](const LinkState& s, const std::string& a, const std::string& b) {
             return s.getMetricFromAToB(a, b);
           })
      .def("hasNode", &LinkState::hasNode)
      .def("isNodeOverloaded", &LinkState::isNodeOverloaded)
      .def("getNodeMetricIncrement", &LinkState::getNodeMetricIncrement)
      .def("numLinks", &LinkState::numLinks)
      .def("flatBuilds", &LinkState::flatBuilds)
      .def("flatPatches", &LinkState::flatPatches)
      .def("edgesPatched", &LinkState::edgesPatched)
      .def("flat_image", [](const LinkState& s) {  // host CSR image (tests)
        const FlatTopology& f = s.flat();
        py::dict d;
        d["names"] = f.names;
        d["row_ptr"] = f.rowPtr;
        d["edges"] = f.edges;
        d["node_flags"] = f.nodeFlags;
        d["max_metric"] = f.maxMetric;
        d["max_degree"] = f.maxDegree;
        d["has_zero_metric"] = f.hasZeroMetric;
        d["has_wide_metric"] = f.hasWideMetric;
        return d;
      })
      .def("device_edges", [](const LinkState& s) {  // device CSR edge words (tests)
        const FlatTopology& f = s.flatOnDevice();
        std::vector<uint64_t> out(f.edges.size());
        if (!out.empty()) f.dEdges.download(out.data(), out.size());
        ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
        std::vector<uint8_t> fl(f.nodeFlags.size());
        if (!fl.empty()) f.dFlags.download(fl.data(), fl.size());
        ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
        return py::make_tuple(out, fl);
      })
      .def("numNodes", &LinkState::numNodes)
      .def("spfRuns", &LinkState::spfRuns)
      .def("getArea", &LinkState::getArea)
      .def("linksFromNode", [](const LinkState& s, const std::string& n) {
        py::list out;
        for (const auto& l : s.linksFromNode(n)) out.append(fromLink(*l));
        return out;
      });

  py::class_<AreaLinkStates>(m, "AreaLinkStates")
      .def(py::init<>())
      .def("add",
           [](AreaLinkStates& a, const std::string& area, const std::string& me)
               -> LinkState& {
             return a.emplace(area, LinkState(area, me)).first->second;
           },
           py::return_value_policy::reference_internal)
      .def("__getitem__",
           [](AreaLinkStates& a, const std::string& area) -> LinkState& {
             return a.at(area);
           },
           py::return_value_policy::reference_internal)
      .def("areas", [](const AreaLinkStates& a) {
        std::vector<std::string> v;
        for (auto& [k, _] : a) v.push_back(k);
        return v;
      });

  py::class_<PrefixState>(m, "PrefixState")
      .def(py::init<>())
      .def("updatePrefix",
           [](PrefixState& s, const std::string& node, const std::string& area,
              py::dict e) { return s.updatePrefix(node, area, toEntry(e)); })
      .def("deletePrefix", &PrefixState::deletePrefix)
      .def("prefixes", [](const PrefixState& s) {
        py::dict out;
        for (const auto& [p, es] : s.prefixes()) {
          std::vector<NodeAndArea> keys;
          for (const auto& [k, _] : es) keys.push_back(k);
          out[py::str(p)] = keys;
        }
        return out;
      });

  // ---- f4: KvStore publication decode (lsdb_codec.h) ----
  m.def("encodeAdjDb", [](py::dict d) { return py::bytes(writeAdjacencyDatabase(toAdjDb(d))); });
  m.def("decodeAdjDb", [](py::bytes b) {
    std::string_view v = b;
    return fromAdjDb(readAdjacencyDatabase(v));
  });
  m.def("encodePrefixDb", [](py::dict d) { return py::bytes(writePrefixDatabase(toPrefixDb(d))); });
  m.def("decodePrefixDb", [](py::bytes b) {
    std::string_view v = b;
    return fromPrefixDb(readPrefixDatabase(v));
  });
  m.def("getNodeNameFromKey", &getNodeNameFromKey);
  py::register_exception<LsdbDecodeError>(m, "LsdbDecodeError", PyExc_ValueError);

  py::class_<DecisionPendingUpdates>(m, "DecisionPendingUpdates")
      .def(py::init<std::string>())
      .def("needsFullRebuild", &DecisionPendingUpdates::needsFullRebuild)
      .def("needsRouteUpdate", &DecisionPendingUpdates::needsRouteUpdate)
      .def("updatedPrefixes", &DecisionPendingUpdates::updatedPrefixes)
      .def("getCount", &DecisionPendingUpdates::getCount)
      .def("reset", &DecisionPendingUpdates::reset)
      .def("applyLinkStateChange",
           [](DecisionPendingUpdates& p, const std::string& node, py::dict change,
              py::object perf) {
             LinkState::LinkStateChange c;
             c.topologyChanged = get<bool>(change, "topologyChanged", false);
             c.linkAttributesChanged = get<bool>(change, "linkAttributesChanged", false);
             c.nodeLabelChanged = get<bool>(change, "nodeLabelChanged", false);
             p.applyLinkStateChange(node, c, toPerfEvents(perf));
           },
           py::arg("nodeName"), py::arg("change"), py::arg("perfEvents") = py::none())
      .def("applyPrefixStateChange",
           [](DecisionPendingUpdates& p, const std::vector<std::string>& change,
              py::object perf) { p.applyPrefixStateChange(change, toPerfEvents(perf)); },
           py::arg("change"), py::arg("perfEvents") = py::none())
      .def("addEvent", &DecisionPendingUpdates::addEvent)
      .def("perfEvents",
           [](const DecisionPendingUpdates& p) { return fromPerfEvents(p.perfEvents()); })
      .def("moveOutEvents",
           [](DecisionPendingUpdates& p) { return fromPerfEvents(p.moveOutEvents()); });
  m.def("addPerfEvent", [](py::list evs, const std::string& node, const std::string& descr) {
    PerfEvents e = *toPerfEvents(evs);
    addPerfEvent(e, node, descr);
    return fromPerfEvents(e);
  });
  m.def("sprintPerfEvents", [](py::list evs) { return sprintPerfEvents(*toPerfEvents(evs)); });
  m.def("getTotalPerfEventsDuration",
        [](py::list evs) { return getTotalPerfEventsDuration(*toPerfEvents(evs)); });
  m.def("getDurationBetweenPerfEvents",
        [](py::list evs, const std::string& a, const std::string& b) -> py::object {
          std::string err;
          auto d = getDurationBetweenPerfEvents(*toPerfEvents(evs), a, b, &err);
          if (!d) return py::make_tuple(py::none(), err);
          return py::make_tuple(*d, py::none());
        });

  py::class_<LsdbIngest>(m, "LsdbIngest")
      .def(py::init<std::string, std::set<std::string>>(), py::arg("myNodeName"),
           py::arg("areas"))
      .def("updateKeyInLsdb",
           [](const LsdbIngest& g, const std::string& area, LinkState& ls, PrefixState& ps,
              const std::string& key, py::object val, bool init) {
             std::optional<std::string_view> v;
             std::string hold;
             if (!val.is_none()) {
               hold = val.cast<py::bytes>();
               v = hold;
             }
             return fromKeyUpdate(g.updateKeyInLsdb(area, ls, ps, key, v, init));
           },
           py::arg("area"), py::arg("linkState"), py::arg("prefixState"), py::arg("key"),
           py::arg("value"), py::arg("inInitialization") = false)
      .def("deleteKeyFromLsdb",
           [](const LsdbIngest& g, const std::string& area, LinkState& ls, PrefixState& ps,
              const std::string& key) {
             return fromKeyUpdate(g.deleteKeyFromLsdb(area, ls, ps, key));
           })
      .def("processPublicationKeyVals",
           [](LsdbIngest& g, const std::string& area, AreaLinkStates& als, PrefixState& ps,
              py::list keyVals, const std::vector<std::string>& expired,
              DecisionPendingUpdates& pending, bool init) {
             std::vector<PublicationKeyVal> kvs;
             for (auto h : keyVals) {
               py::tuple t = h.cast<py::tuple>();
               PublicationKeyVal kv;
               kv.key = t[0].cast<std::string>();
               if (!t[1].is_none()) kv.value = std::string(t[1].cast<py::bytes>());
               kvs.push_back(std::move(kv));
             }
             g.processPublication(area, als, ps, kvs, expired, pending, init);
           },
           py::arg("area"), py::arg("areaLinkStates"), py::arg("prefixState"),
           py::arg("keyVals"), py::arg("expiredKeys"), py::arg("pending"),
           py::arg("inInitialization") = false)
      // one publication's key/value pairs applied in C++ (bench / bulk load):
      // returns per-kind counts and the wall time of the loop alone
      .def("processPublication",
           [](const LsdbIngest& g, const std::string& area, LinkState& ls, PrefixState& ps,
              const std::vector<std::string>& keys, const std::vector<py::bytes>& vals,
              bool init) {
             if (keys.size() != vals.size()) throw std::invalid_argument("keys/values size");
             std::vector<std::string> raw;
             raw.reserve(vals.size());
             size_t bytes = 0;
             for (const auto& b : vals) {
               raw.emplace_back(b);
               bytes += raw.back().size();
             }
             size_t counts[4] = {0, 0, 0, 0};
             size_t topo = 0;
             auto t0 = std::chrono::steady_clock::now();
             for (size_t i = 0; i < keys.size(); ++i) {
               auto u = g.updateKeyInLsdb(area, ls, ps, keys[i], std::string_view(raw[i]), init);
               counts[u.kind]++;
               topo += u.kind == LsdbKeyUpdate::kAdjacency && u.linkChange.topologyChanged;
             }
             double ns = std::chrono::duration<double, std::nano>(
                             std::chrono::steady_clock::now() - t0).count();
             py::dict d;
             d["skipped"] = counts[0];
             d["adjacency"] = counts[1];
             d["prefix"] = counts[2];
             d["error"] = counts[3];
             d["topologyChanged"] = topo;
             d["bytes"] = bytes;
             d["ns"] = ns;
             return d;
           },
           py::arg("area"), py::arg("linkState"), py::arg("prefixState"), py::arg("keys"),
           py::arg("values"), py::arg("inInitialization") = false);

  py::class_<RouteDbBatch>(m, "RouteDbBatch")
      .def(py::init<const SpfSolver&, const AreaLinkStates&, const PrefixState&,
                    const std::vector<std::string>&>(),
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>(), py::keep_alive<1, 4>())
      .def("launch", [](RouteDbBatch& b, uintptr_t stream) {
             b.launch(reinterpret_cast<void*>(stream));
           }, py::arg("stream") = 0)
      .def("routeDb", [](const RouteDbBatch& b, const std::string& n) { return b.routeDb(n); })
      .def("getRouteDbComputed", [](const RouteDbBatch& b, const std::string& n) {
        const RouteDatabase r = b.getRouteDbComputed(n);
        py::list uni, mpls;
        for (const auto& u : r.unicastRoutes) {
          py::list nhs;
          for (const auto& nh : u.nextHops) nhs.append(fromNh(nh));
          uni.append(py::make_tuple(u.dest, nhs, u.counterID ? py::object(py::str(*u.counterID))
                                                            : py::object(py::none())));
        }
        for (const auto& mr : r.mplsRoutes) {
          py::list nhs;
          for (const auto& nh : mr.nextHops) nhs.append(fromNh(nh));
          mpls.append(py::make_tuple(mr.topLabel, nhs));
        }
        py::dict d;
        d["thisNodeName"] = r.thisNodeName;
        d["unicastRoutes"] = uni;
        d["mplsRoutes"] = mpls;
        return d;
      })
      .def("numSources", &RouteDbBatch::numSources)
      .def("numGroups", &RouteDbBatch::numGroups);

  py::class_<DecisionRouteDb>(m, "DecisionRouteDb")
      .def(py::init<>())
      .def("unicastRoutes",
           [](const DecisionRouteDb& db) {
             py::dict out;
             for (const auto& [p, r] : db.unicastRoutes) out[py::str(p)] = fromRoute(r);
             return out;
           })
      .def("mplsRoutes",
           [](const DecisionRouteDb& db) {
             py::dict out;
             for (const auto& [l, r] : db.mplsRoutes) out[py::int_(l)] = fromNhSet(r.nexthops);
             return out;
           })
      .def("calculateUpdate",
           [](const DecisionRouteDb& a, const DecisionRouteDb& b) {
             return fromUpdate(a.calculateUpdate(b));
           })
      .def("canonical", [](const DecisionRouteDb& db) { return py::bytes(canonical(db)); })
      .def("digest", [](const DecisionRouteDb& db, const std::string& key) {
        return digest::unit(key, db);
      });

  py::class_<SpfSolver>(m, "SpfSolver")
      .def(py::init<const std::string&, bool, bool, bool, bool>(), py::arg("myNodeName"),
           py::arg("enableV4"), py::arg("enableNodeSegmentLabel"),
           py::arg("enableBestRouteSelection") = false, py::arg("v4OverV6Nexthop") = false)
      .def("buildRouteDb",
           [](SpfSolver& s, const std::string& me, const AreaLinkStates& a,
              const PrefixState& ps) { return s.buildRouteDb(me, a, ps); })
      .def("createRouteForPrefixOrGetStaticRoute",
           [](SpfSolver& s, const std::string& me, const AreaLinkStates& a,
              const PrefixState& ps, const std::string& prefix) -> py::object {
             auto r = s.createRouteForPrefixOrGetStaticRoute(me, a, ps, prefix);
             if (!r) return py::none();
             return fromRoute(*r);
           })
      .def("createRoutesForPrefixes",
           [](SpfSolver& s, const std::string& me, const AreaLinkStates& a,
              const PrefixState& ps, const std::set<std::string>& prefixes) {
             py::dict out;
             for (const auto& [p, r] : s.createRoutesForPrefixes(me, a, ps, prefixes)) {
               out[py::str(p)] = r ? py::object(fromRoute(*r)) : py::object(py::none());
             }
             return out;
           })
      .def("incrementalBatches", &SpfSolver::incrementalBatches)
      .def("incrementalBatchPrefixes", &SpfSolver::incrementalBatchPrefixes)
      .def("updateStaticUnicastRoutes",
           [](SpfSolver& s, py::dict upd, std::vector<std::string> del) {
             std::map<std::string, RibUnicastEntry> u;
             for (auto kv : upd) u[kv.first.cast<std::string>()] = toRoute(kv.second.cast<py::dict>());
             s.updateStaticUnicastRoutes(u, del);
           })
      .def("setRibPolicy",
           [](SpfSolver& s, const RibPolicy* p) { s.setRibPolicy(p); },
           py::arg("policy").none(true), py::keep_alive<1, 2>())
      .def("getBestRoutesCache", [](const SpfSolver& s) {
        py::dict out;
        for (const auto& [p, r] : s.getBestRoutesCache()) {
          py::dict d;
          d["allNodeAreas"] = std::vector<NodeAndArea>(r.allNodeAreas.begin(), r.allNodeAreas.end());
          d["bestNodeArea"] = r.bestNodeArea;
          d["isBestNodeDrained"] = r.isBestNodeDrained;
          out[py::str(p)] = d;
        }
        return out;
      });

  py::class_<RibPolicy>(m, "RibPolicy")
      .def(py::init([](py::list stmts, int64_t ttl) {
             return RibPolicy(parseStatements(stmts), ttl);
           }),
           py::arg("statements"), py::arg("ttl_secs") = 3600)
      .def("isActive", &RibPolicy::isActive)
      .def("match", [](const RibPolicy& p, py::dict r) { return p.match(toRoute(r)); })
      .def("applyAction",
           [](const RibPolicy& p, py::dict r) {
             auto e = toRoute(r);
             bool ok = p.applyAction(e);
             return py::make_tuple(ok, fromRoute(e));
           })
      .def("applyPolicy", [](const RibPolicy& p, DecisionRouteDb& db) {
        return p.applyPolicy(db.unicastRoutes);
      });

  m.def("pathAInPathB", [](py::list a, py::list b) {
    auto conv = [](py::list l) {
      LinkState::Path p;
      for (auto h : l) {
        py::tuple t = h.cast<py::tuple>();
        p.push_back(std::make_shared<Link>("", t[0].cast<std::string>(), t[1].cast<std::string>(),
                                           t[2].cast<std::string>(), t[3].cast<std::string>()));
      }
      return p;
    };
    return LinkState::pathAInPathB(conv(a), conv(b));
  });

  // ---- bulk workloads ------------------------------------------------------
  // Multi-area domain (topogen::multiArea): canonical RouteDbs per source.
  m.def("gen_route_dbs_multiarea",
        [](py::dict d, std::vector<std::string> sources, bool enableV4, bool sr,
           bool brs, py::list policy) {
          AreaLinkStates als;
          PrefixState ps;
          loadMultiArea(d, als, ps);
          SpfSolver solver("test_node", enableV4, sr, brs);
          std::optional<RibPolicy> pol;
          if (!policy.empty()) {
            pol.emplace(parseStatements(policy), 3600);
            solver.setRibPolicy(&*pol);
          }
          std::vector<py::bytes> out;
          for (const auto& s : sources) {
            auto db = solver.buildRouteDb(s, als, ps);
            out.push_back(py::bytes(db ? canonical(*db) : std::string("NONE")));
          }
          return out;
        },
        py::arg("opts"), py::arg("sources"), py::arg("enableV4") = true,
        py::arg("sr") = false, py::arg("brs") = false, py::arg("policy") = py::list());

  // §8(f) f3 measurement: mean host+device cost of one link-metric flap
  // (updateAdjacencyDatabase of one node with one adjacency metric changed,
  // then the CSR made current on the device and the stream drained), with the
  // in-place patch and with a full re-flatten + upload. Returns
  // (patch_us, rebuild_us, edges, flaps).
  m.def("flap_update_bench",
        [](const std::string& kind, py::dict opts, int flaps, uint64_t seed) {
          const topogen::Lsdb g = genLsdb(kind, opts);
          auto run = [&](bool incremental) {
            py::gil_scoped_release nogil;
            LinkState ls(g.area, "test_node");
            PrefixState ps;
            loadLsdb(g, ls, ps);
            ls.setIncrementalFlatten(incremental);
            ls.flatOnDevice();
            ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
            std::vector<AdjacencyDatabase> dbs;
            for (const auto& [_, db] : ls.getAdjacencyDatabases()) dbs.push_back(db);
            uint64_t s = seed;
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < flaps; ++i) {
              AdjacencyDatabase& db = dbs[topogen::splitmix64(s) % dbs.size()];
              if (db.adjacencies.empty()) continue;
              Adjacency& a = db.adjacencies[topogen::splitmix64(s) % db.adjacencies.size()];
              a.metric = 1 + int32_t(topogen::splitmix64(s) % 1000);
              ls.updateAdjacencyDatabase(db, g.area);
              ls.flatOnDevice();
              ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
            }
            const double us = std::chrono::duration<double, std::micro>(
                                  std::chrono::steady_clock::now() - t0).count();
            return std::make_pair(us / std::max(flaps, 1), ls.flat().edges.size());
          };
          const auto [patchUs, edges] = run(true);
          const auto [rebuildUs, _] = run(false);
          return py::make_tuple(patchUs, rebuildUs, edges, flaps);
        });
  // §8(f) f4 + f3 end to end: the same flaps arriving as KvStore values
  // (compact AdjacencyDatabase bytes, encoded before timing, as the sender
  // would) -> LsdbIngest::updateKeyInLsdb -> in-place CSR patch -> device
  // current. Returns (us per flap, flaps applied, digest of the final device
  // edge words == digest of a fresh flatten of the same LSDB).
  m.def("publication_flap_bench",
        [](const std::string& kind, py::dict opts, int flaps, uint64_t seed) {
          const topogen::Lsdb g = genLsdb(kind, opts);
          std::optional<py::gil_scoped_release> nogil(std::in_place);
          LinkState ls(g.area, "test_node");
          PrefixState ps;
          loadLsdb(g, ls, ps);
          ls.flatOnDevice();
          ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
          std::vector<AdjacencyDatabase> dbs;
          for (const auto& [_, db] : ls.getAdjacencyDatabases()) dbs.push_back(db);
          std::vector<std::pair<std::string, std::string>> pubs;
          uint64_t s = seed;
          for (int i = 0; i < flaps; ++i) {
            AdjacencyDatabase& db = dbs[topogen::splitmix64(s) % dbs.size()];
            if (db.adjacencies.empty()) continue;
            Adjacency& a = db.adjacencies[topogen::splitmix64(s) % db.adjacencies.size()];
            a.metric = 1 + int32_t(topogen::splitmix64(s) % 1000);
            pubs.emplace_back("adj:" + db.thisNodeName, writeAdjacencyDatabase(db));
          }
          LsdbIngest ing("test_node", {g.area});
          const auto t0 = std::chrono::steady_clock::now();
          for (const auto& [key, val] : pubs) {
            auto u = ing.updateKeyInLsdb(g.area, ls, ps, key, std::string_view(val));
            if (u.kind != LsdbKeyUpdate::kAdjacency) throw std::runtime_error(u.error);
            ls.flatOnDevice();
            ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
          }
          const double us = std::chrono::duration<double, std::micro>(
                                std::chrono::steady_clock::now() - t0).count();
          auto digest = [](const std::vector<uint64_t>& v) {
            uint64_t h = 0xcbf29ce484222325ull;
            for (uint64_t x : v) h = (h ^ x) * 0x100000001b3ull;
            return h;
          };
          const FlatTopology& f = ls.flatOnDevice();
          std::vector<uint64_t> dev(f.edges.size());
          if (!dev.empty()) f.dEdges.download(dev.data(), dev.size());
          ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
          LinkState fresh(g.area, "test_node");
          for (const auto& db : dbs) fresh.updateAdjacencyDatabase(db, g.area);
          const uint64_t dDev = digest(dev), dFresh = digest(fresh.flat().edges);
          nogil.reset();  // the GIL is needed again to build the result
          return py::make_tuple(us / std::max<size_t>(pubs.size(), 1), pubs.size(), dDev, dFresh);
        });
  // f1 incremental branch after a prefix publication: `n` changed prefixes
  // answered by createRoutesForPrefixes (one build) vs the reference's loop
  // of createRouteForPrefixOrGetStaticRoute; returns (batch ms, loop ms,
  // identical results)
  m.def("incremental_routes_bench",
        [](const std::string& kind, py::dict opts, const std::string& me, int n) {
          auto g = genLsdb(kind, opts);
          py::gil_scoped_release nogil;
          AreaLinkStates als;
          auto& ls = als.emplace(g.area, LinkState(g.area, "test_node")).first->second;
          PrefixState ps;
          loadLsdb(g, ls, ps);
          std::set<std::string> changed;  // every stride-th in sorted order (refcpu's too)
          std::vector<std::string> all;
          for (const auto& [p, _] : ps.prefixes()) all.push_back(p);
          std::sort(all.begin(), all.end());
          const size_t stride = std::max<size_t>(1, all.size() / std::max(n, 1));
          for (size_t i = 0; i < all.size(); ++i) {
            if (i % stride == 0 && int(changed.size()) < n) changed.insert(all[i]);
          }
          SpfSolver a("test_node", true, false, false, false), b("test_node", true, false, false, false);
          // Decision's flow (Decision.cpp:912-951): a full build, then
          // publications change the prefixes (a tag added to each entry),
          // then the incremental branch over the changed set
          a.buildRouteDb(me, als, ps);
          b.buildRouteDb(me, als, ps);
          std::vector<std::tuple<NodeAndArea, std::string, PrefixEntry>> upd;
          for (const auto& p : changed) {
            for (const auto& [na, e] : ps.prefixes().at(p)) {
              PrefixEntry e2 = *e;
              e2.tags.insert("incremental");
              upd.emplace_back(na, p, std::move(e2));
            }
          }
          for (auto& [na, p, e] : upd) ps.updatePrefixKeyed(na.first, na.second, p, std::move(e));
          // both solvers warm (device sub-table buffers allocated, as the
          // reference's loop runs with its SPF memo warm); createRoutesForPrefixes
          // leaves the per-prefix path's change-log cursor alone
          a.createRoutesForPrefixes(me, als, ps, changed);
          b.createRoutesForPrefixes(me, als, ps, changed);
          const char* kSplit[4] = {"decision.gpu.inc_spf_ms.sum", "decision.gpu.inc_table_ms.sum",
                                   "decision.gpu.inc_device_ms.sum",
                                   "decision.gpu.inc_materialize_ms.sum"};
          auto sums = [&](std::array<double, 4>& acc, double sign) {
            const auto c = getDecisionCounters();
            for (int i = 0; i < 4; ++i) {
              auto it = c.find(kSplit[i]);
              acc[i] += sign * (it == c.end() ? 0.0 : it->second);
            }
          };
          std::array<double, 4> split{};
          sums(split, -1.0);
          auto t0 = std::chrono::steady_clock::now();
          auto batch = a.createRoutesForPrefixes(me, als, ps, changed);
          auto t1 = std::chrono::steady_clock::now();
          sums(split, 1.0);
          std::vector<std::optional<RibUnicastEntry>> loop;
          loop.reserve(changed.size());
          for (const auto& p : changed) {
            loop.push_back(b.createRouteForPrefixOrGetStaticRoute(me, als, ps, p));
          }
          auto t2 = std::chrono::steady_clock::now();
          bool same = true;  // compared after the timed loop
          size_t i = 0;
          for (const auto& p : changed) {
            const auto& r = loop[i++];
            same &= (r.has_value() == batch[p].has_value()) && (!r || *r == *batch[p]);
          }
          return std::make_tuple(std::chrono::duration<double, std::milli>(t1 - t0).count(),
                                 std::chrono::duration<double, std::milli>(t2 - t1).count(),
                                 same, changed.size(), split[0], split[1], split[2], split[3]);
        });
  m.def("gen_publication",
        [](const std::string& kind, py::dict opts) {
          auto g = genLsdb(kind, opts);
          std::vector<std::string> keys, vals;
          lsdbPublication(g, keys, vals);
          std::vector<py::bytes> out;
          out.reserve(vals.size());
          for (auto& v : vals) out.emplace_back(v);
          return py::make_tuple(g.area, keys, out);
        });
  // f4 bench: encode a generated LSDB, then decode + ingest every key into a
  // fresh LinkState / PrefixState (Decision::updateKeyInLsdb per key), and
  // decode alone; medians over `reps`. Host-only (no device call).
  m.def("publication_ingest_bench",
        [](const std::string& kind, py::dict opts, int reps) {
          auto g = genLsdb(kind, opts);
          std::vector<std::string> keys, vals;
          lsdbPublication(g, keys, vals);
          size_t bytes = 0, adjBytes = 0, nAdj = g.adjDbs.size();
          for (size_t i = 0; i < vals.size(); ++i) {
            bytes += vals[i].size();
            if (i < nAdj) adjBytes += vals[i].size();
          }
          std::vector<double> ingest, decode, keyedDecode, insert, publication;
          size_t routesKept = 0;
          std::vector<PublicationKeyVal> pub(keys.size());
          for (size_t i = 0; i < keys.size(); ++i) pub[i] = PublicationKeyVal{keys[i], vals[i]};
          // in key order, as Decision receives it (thrift::Publication's
          // keyVals is a std::map, Decision.cpp:821-846); processPublication
          // sorts an unsorted vector itself
          std::sort(pub.begin(), pub.end(), [](const PublicationKeyVal& a,
                                               const PublicationKeyVal& b) { return a.key < b.key; });
          for (int r = 0; r < reps; ++r) {
            {
              // the whole publication through processPublication (one host
              // thread: each key decoded and applied in key order, streamed)
              AreaLinkStates als;
              PrefixState ps0;
              LsdbIngest ing0("test_node", {g.area});
              DecisionPendingUpdates pending("test_node");
              auto p0 = std::chrono::steady_clock::now();
              ing0.processPublication(g.area, als, ps0, pub, {}, pending);
              publication.push_back(std::chrono::duration<double, std::milli>(
                                        std::chrono::steady_clock::now() - p0).count());
              if (ps0.prefixes().size() != keys.size() - nAdj) {
                throw std::runtime_error("processPublication lost prefixes");
              }
            }
            LinkState ls(g.area, "test_node");
            PrefixState ps;
            LsdbIngest ing("test_node", {g.area});
            auto t0 = std::chrono::steady_clock::now();
            for (size_t i = 0; i < keys.size(); ++i) {
              auto u = ing.updateKeyInLsdb(g.area, ls, ps, keys[i], std::string_view(vals[i]));
              if (u.kind == LsdbKeyUpdate::kError) throw std::runtime_error(u.error);
            }
            auto t1 = std::chrono::steady_clock::now();
            size_t sink = 0;
            for (size_t i = 0; i < keys.size(); ++i) {
              if (i < nAdj) sink += readAdjacencyDatabase(vals[i]).adjacencies.size();
              else sink += readPrefixDatabase(vals[i]).prefixEntries.size();
            }
            auto t2 = std::chrono::steady_clock::now();
            // split of the prefix-key ingest: decode with the keyed network,
            // then PrefixState inserts of the decoded entries
            std::vector<std::pair<std::string, PrefixDatabase>> decoded;
            decoded.reserve(keys.size() - nAdj);
            for (size_t i = nAdj; i < keys.size(); ++i) {
              std::vector<std::string> nets;
              PrefixDatabase db = readPrefixDatabase(vals[i], &nets);
              decoded.emplace_back(nets.front(), std::move(db));
            }
            auto t3 = std::chrono::steady_clock::now();
            PrefixState ps2;
            for (auto& [net, db] : decoded) {
              sink += ps2.updatePrefixKeyed(db.thisNodeName, g.area, net,
                                            std::move(db.prefixEntries.front())).size();
            }
            auto t4 = std::chrono::steady_clock::now();
            routesKept = ps.prefixes().size() + (sink & 0);
            ingest.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
            decode.push_back(std::chrono::duration<double, std::milli>(t2 - t1).count());
            keyedDecode.push_back(std::chrono::duration<double, std::milli>(t3 - t2).count());
            insert.push_back(std::chrono::duration<double, std::milli>(t4 - t3).count());
          }
          std::sort(keyedDecode.begin(), keyedDecode.end());
          std::sort(publication.begin(), publication.end());
          std::sort(insert.begin(), insert.end());
          std::sort(ingest.begin(), ingest.end());
          std::sort(decode.begin(), decode.end());
          py::dict d;
          d["adj_dbs"] = nAdj;
          d["prefix_keys"] = keys.size() - nAdj;
          d["bytes"] = bytes;
          d["adj_bytes"] = adjBytes;
          d["prefixes"] = routesKept;
          d["ingest_ms"] = ingest[ingest.size() / 2];
          d["decode_ms"] = decode[decode.size() / 2];
          d["prefix_keyed_decode_ms"] = keyedDecode[keyedDecode.size() / 2];
          d["prefix_insert_ms"] = insert[insert.size() / 2];
          d["publication_ms"] = publication[publication.size() / 2];
          return d;
        },
        py::arg("kind"), py::arg("opts"), py::arg("reps") = 3);
  m.def("gen_route_dbs",
        [](const std::string& kind, py::dict opts, std::vector<std::string> sources,
           bool enableV4, bool sr, bool brs, py::list policy) {
          auto g = genLsdb(kind, opts);
          AreaLinkStates als;
          auto& ls = als.emplace(g.area, LinkState(g.area, "test_node")).first->second;
          PrefixState ps;
          loadLsdb(g, ls, ps);
          SpfSolver solver("test_node", enableV4, sr, brs);
          std::optional<RibPolicy> pol;
          if (!policy.empty()) {
            pol.emplace(parseStatements(policy), 3600);
            solver.setRibPolicy(&*pol);
          }
          std::vector<py::bytes> out;
          for (const auto& s : sources) {
            auto db = solver.buildRouteDb(s, als, ps);
            out.push_back(py::bytes(db ? canonical(*db) : std::string("NONE")));
          }
          return out;
        },
        py::arg("kind"), py::arg("opts"), py::arg("sources"), py::arg("enableV4") = true,
        py::arg("sr") = false, py::arg("brs") = false, py::arg("policy") = py::list());

  // §8(f) f2 parity: a generated topology's RouteDbs for `sources` from ONE
  // RouteDbBatch (resident records, per-node materialisation); canonical text
  // per source ("NONE" without a RouteDb) and the getRouteDbComputed shape
  // (thisNodeName, unicast routes, mpls routes, next hops in total)
  // f2 over a multi-area domain (loadMultiArea): RouteDbBatch served per node
  // (canonical text per source, and whether getRouteDbComputed equals
  // routeDb(node)->toThrift() with thisNodeName = node)
  m.def("gen_route_db_batch_multiarea",
        [](py::dict opts, std::vector<std::string> sources, bool enableV4, bool sr, bool brs) {
          AreaLinkStates als;
          PrefixState ps;
          loadMultiArea(opts, als, ps);
          SpfSolver solver("test_node", enableV4, sr, brs);
          RouteDbBatch batch(solver, als, ps, sources);
          batch.launch();
          std::vector<py::bytes> out;
          py::list same;
          for (const auto& s : sources) {
            auto db = batch.routeDb(s);
            out.push_back(py::bytes(db ? canonical(*db) : std::string("NONE")));
            const RouteDatabase r = batch.getRouteDbComputed(s);
            RouteDatabase want;
            if (db) want = db->toThrift();
            bool eq = r.thisNodeName == s &&
                r.unicastRoutes.size() == want.unicastRoutes.size() &&
                r.mplsRoutes.size() == want.mplsRoutes.size();
            for (size_t i = 0; eq && i < r.unicastRoutes.size(); ++i) {
              eq = r.unicastRoutes[i].dest == want.unicastRoutes[i].dest &&
                  r.unicastRoutes[i].nextHops == want.unicastRoutes[i].nextHops;
            }
            same.append(eq);
          }
          return py::make_tuple(out, same);
        },
        py::arg("opts"), py::arg("sources"), py::arg("enableV4") = true, py::arg("sr") = false,
        py::arg("brs") = false);
  m.def("gen_route_db_batch",
        [](const std::string& kind, py::dict opts, std::vector<std::string> sources,
           bool enableV4, bool sr, bool brs) {
          auto g = genLsdb(kind, opts);
          AreaLinkStates als;
          auto& ls = als.emplace(g.area, LinkState(g.area, "test_node")).first->second;
          PrefixState ps;
          loadLsdb(g, ls, ps);
          SpfSolver solver("test_node", enableV4, sr, brs);
          RouteDbBatch batch(solver, als, ps, sources);
          batch.launch();
          std::vector<py::bytes> out;
          py::list shapes;
          for (const auto& s : sources) {
            auto db = batch.routeDb(s);
            out.push_back(py::bytes(db ? canonical(*db) : std::string("NONE")));
            const RouteDatabase r = batch.getRouteDbComputed(s);
            size_t nhs = 0;
            for (const auto& u : r.unicastRoutes) nhs += u.nextHops.size();
            for (const auto& mr : r.mplsRoutes) nhs += mr.nextHops.size();
            // the direct thrift build equals toThrift() of the materialised
            // DecisionRouteDb, route for route, next hop for next hop
            RouteDatabase want;
            if (db) want = db->toThrift();
            bool same = r.unicastRoutes.size() == want.unicastRoutes.size() &&
                r.mplsRoutes.size() == want.mplsRoutes.size();
            for (size_t i = 0; same && i < r.unicastRoutes.size(); ++i) {
              const auto &a = r.unicastRoutes[i], &b = want.unicastRoutes[i];
              same = a.dest == b.dest && a.nextHops == b.nextHops && a.counterID == b.counterID;
            }
            for (size_t i = 0; same && i < r.mplsRoutes.size(); ++i) {
              same = r.mplsRoutes[i].topLabel == want.mplsRoutes[i].topLabel &&
                  r.mplsRoutes[i].nextHops == want.mplsRoutes[i].nextHops;
            }
            shapes.append(py::make_tuple(r.thisNodeName, r.unicastRoutes.size(),
                                         r.mplsRoutes.size(), nhs, same));
          }
          return py::make_tuple(out, shapes, batch.numGroups());
        },
        py::arg("kind"), py::arg("opts"), py::arg("sources"), py::arg("enableV4") = true,
        py::arg("sr") = false, py::arg("brs") = false);

  // §8(f) f2 measurement: RouteDbBatch over ALL nodes of a generated
  // topology (one launch per width group, records resident), then
  // getRouteDbComputed for `serve` nodes (D2H of that node's records + host
  // materialisation + toThrift). Returns (launch_ms, serve_ms_mean,
  // routes_per_served_node_mean, sources).
  // Config C1 latency of the drop-in SpfSolver::buildRouteDb(source) as a
  // Decision caller sees it. cold: fresh LinkState / PrefixState / solver per
  // repetition (CSR flatten + uploads, launch, D2H, materialisation; the
  // ingestion of the adjacency / prefix databases is untimed); warm: the same
  // objects again (device tables cached, the SPF + RouteDb launch, D2H and
  // materialisation still run every call). Returns (cold us, warm us, routes).
  m.def("build_latency_bench",
        [](const std::string& kind, py::dict opts, const std::string& me, int reps) {
          auto g = genLsdb(kind, opts);
          py::gil_scoped_release nogil;
          std::vector<double> cold, warm;
          size_t routes = 0;
          uint64_t dCold = 0, dWarm = 0;  // route_digest.h unit(me, db)
          // the drop-in's split timers (decision.gpu.*_ms) of EACH timed
          // build (counter deltas around it), so a caller can report the
          // split of the same rep as its total
          const char* kSplit[3] = {"decision.gpu.prepare_ms.sum", "decision.gpu.launch_ms.sum",
                                   "decision.gpu.materialize_ms.sum"};
          auto snap = [&]() {
            std::array<double, 3> a{};
            const auto c = getDecisionCounters();
            for (int i = 0; i < 3; ++i) {
              auto it = c.find(kSplit[i]);
              a[i] = it == c.end() ? 0.0 : it->second;
            }
            return a;
          };
          auto delta = [](const std::array<double, 3>& a, const std::array<double, 3>& b) {
            return std::array<double, 3>{b[0] - a[0], b[1] - a[1], b[2] - a[2]};
          };
          std::vector<std::array<double, 3>> splitCold, splitWarm;
          for (int r = 0; r < reps + 1; ++r) {
            AreaLinkStates als;
            auto& ls = als.emplace(g.area, LinkState(g.area, "test_node")).first->second;
            PrefixState ps;
            loadLsdb(g, ls, ps);
            SpfSolver solver("test_node", true, false, false);
            const auto c0 = snap();
            auto t0 = std::chrono::steady_clock::now();
            auto db = solver.buildRouteDb(me, als, ps);
            const double us = std::chrono::duration<double, std::micro>(
                                  std::chrono::steady_clock::now() - t0).count();
            const auto c1 = snap();
            if (!db) throw std::runtime_error("no RouteDb for " + me);
            routes = db->unicastRoutes.size();
            if (r) {  // rep 0 warms code objects / workspace
              cold.push_back(us);
              splitCold.push_back(delta(c0, c1));
            }
            if (r == reps) {
              dCold = digest::unit(me, *db);
              for (int k = 0; k < reps; ++k) {
                db.reset();  // the previous result is released untimed, as before a cold build
                const auto w0 = snap();
                t0 = std::chrono::steady_clock::now();
                db = solver.buildRouteDb(me, als, ps);
                warm.push_back(std::chrono::duration<double, std::micro>(
                                   std::chrono::steady_clock::now() - t0).count());
                splitWarm.push_back(delta(w0, snap()));
              }
              dWarm = digest::unit(me, *db);
            }
          }
          return std::make_tuple(cold, warm, routes, dCold, dWarm, splitCold, splitWarm);
        },
        py::arg("kind"), py::arg("opts"), py::arg("me"), py::arg("reps"));
  // Host-only f1 materialisation harness (no device): synthetic changed
  // records of `variants` variants x `perVariant` prefixes of a generated
  // topology's source `me` (about 10 % deletions, random next-hop subsets of
  // the source's links) through materializeUpdates on `threads` host threads.
  // Returns (ms per rep, changes) -- destruction of the updates untimed.
  m.def("materialize_updates_bench",
        [](const std::string& kind, py::dict opts, const std::string& me, size_t variants,
           size_t perVariant, int threads, int reps) {
          auto g = genLsdb(kind, opts);
          py::gil_scoped_release nogil;
          LinkState ls(g.area, "test_node");
          PrefixState ps;
          loadLsdb(g, ls, ps);
          const FlatTopology& f = ls.flat();
          PrefixHostTable pt;
          pt.build(ps);
          const uint32_t s = f.id.at(me);
          const uint32_t deg = f.rowPtr[s + 1] - f.rowPtr[s];
          const int W = std::max(1, int((deg + 31) / 32));
          const size_t P = pt.prefixes.size();
          std::vector<uint32_t> off(variants + 1, 0), pfx, meta, metric;
          uint64_t x = 0x9E3779B97F4A7C15ull;
          auto rnd = [&] {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            return x;
          };
          for (size_t v = 0; v < variants; ++v) {
            std::vector<uint32_t> ps_;
            for (size_t k = 0; k < perVariant; ++k) ps_.push_back(uint32_t(rnd() % P));
            std::sort(ps_.begin(), ps_.end());
            ps_.erase(std::unique(ps_.begin(), ps_.end()), ps_.end());
            for (uint32_t p : ps_) {
              pfx.push_back(p);
              meta.push_back(rnd() % 10 == 0 ? 0u : OGS_ROUTE_VALID);
              metric.push_back(uint32_t(10 + rnd() % 1000));
            }
            off[v + 1] = uint32_t(pfx.size());
          }
          const size_t T = pfx.size();
          std::vector<uint32_t> mask(T * W, 0);
          for (size_t i = 0; i < T; ++i) {
            for (int k = 0; k < 2; ++k) {
              const uint32_t j = uint32_t(rnd() % deg);
              mask[size_t(j / 32) * T + i] |= 1u << (j % 32);
            }
          }
          ChangeRecords c;
          c.offsets = off.data();
          c.variants = variants;
          c.prefix = pfx.data();
          c.meta = meta.data();
          c.metric = metric.data();
          c.mask = mask.data();
          c.total = T;
          c.W = W;
          std::vector<double> ms;
          for (int r = 0; r < reps; ++r) {
            auto t0 = std::chrono::steady_clock::now();
            auto ups = materializeUpdates(f, me, pt, c, false, threads);
            ms.push_back(std::chrono::duration<double, std::milli>(
                             std::chrono::steady_clock::now() - t0).count());
          }
          return std::make_pair(ms, T);
        },
        py::arg("kind"), py::arg("opts"), py::arg("me"), py::arg("variants"),
        py::arg("per_variant"), py::arg("threads"), py::arg("reps"));
  // Host-only RouteDb materialisation harness (no device): every prefix of
  // a generated topology a VALID single-advertiser record with a random
  // next-hop subset of `me`'s links, through materializeRouteDb on
  // `threads` threads (0: automatic). Returns (build ms, destroy ms) per rep.
  m.def("materialize_routedb_bench",
        [](const std::string& kind, py::dict opts, const std::string& me, int threads,
           int reps) {
          auto g = genLsdb(kind, opts);
          py::gil_scoped_release nogil;
          LinkState ls(g.area, "test_node");
          PrefixState ps;
          loadLsdb(g, ls, ps);
          const FlatTopology& f = ls.flat();
          PrefixHostTable pt;
          pt.build(ps);
          const uint32_t s = f.id.at(me);
          const uint32_t deg = f.rowPtr[s + 1] - f.rowPtr[s];
          const uint32_t P = uint32_t(pt.prefixes.size());
          std::vector<uint32_t> meta(P, OGS_ROUTE_VALID | OGS_ROUTE_SELECTED), mask(P), sel(P, 1);
          std::vector<uint64_t> metric(P);
          uint64_t x = 0x9E3779B97F4A7C15ull;
          for (uint32_t p = 0; p < P; ++p) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            mask[p] = (1u << (x % std::min(deg, 32u))) | (1u << ((x >> 8) % std::min(deg, 32u)));
            metric[p] = 10 + x % 1000;
          }
          UnitView v;
          v.W = 1;
          v.P = P;
          v.N = uint32_t(f.names.size());
          v.meta = meta.data();
          v.metric = metric.data();
          v.mask = mask.data();
          v.maskStride = P;
          v.sel = sel.data();
          const int saved = g_materializeThreads;
          g_materializeThreads = threads;
          std::vector<std::pair<double, double>> out;
          std::map<std::string, RibUnicastEntry> statics;
          std::map<std::string, RouteSelectionResult> cache;
          for (int r = 0; r < reps; ++r) {
            auto t0 = std::chrono::steady_clock::now();
            auto* db = new DecisionRouteDb(materializeRouteDb(ls, f, g.area, me, v, pt, false,
                                                              false, statics, &cache));
            const double b = msSince(t0);
            t0 = std::chrono::steady_clock::now();
            delete db;
            out.emplace_back(b, msSince(t0));
          }
          g_materializeThreads = saved;
          return out;
        },
        py::arg("kind"), py::arg("opts"), py::arg("me"), py::arg("threads"), py::arg("reps"));
  // Host-only split of a cold single-area build's preparation (no device):
  // LinkState::flat() (CSR flatten), PrefixHostTable::build and
  // HostBatch::appendPrefixes (the packed prefix table) in ms, per rep on a
  // fresh LinkState / PrefixState (ingestion untimed).
  m.def("prepare_split_bench",
        [](const std::string& kind, py::dict opts, int reps) {
          auto g = genLsdb(kind, opts);
          py::gil_scoped_release nogil;
          std::vector<std::tuple<double, double, double>> out;
          for (int r = 0; r < reps; ++r) {
            LinkState ls(g.area, "test_node");
            PrefixState ps;
            loadLsdb(g, ls, ps);
            auto t0 = std::chrono::steady_clock::now();
            const FlatTopology& f = ls.flat();
            const double a = msSince(t0);
            t0 = std::chrono::steady_clock::now();
            PrefixHostTable pt;
            pt.build(ps);
            const double b = msSince(t0);
            t0 = std::chrono::steady_clock::now();
            HostBatch hb;
            hb.appendPrefixes(f, ps, g.area);
            out.emplace_back(a, b, msSince(t0));
          }
          return out;
        },
        py::arg("kind"), py::arg("opts"), py::arg("reps"));
  m.def("route_db_batch_serve_bench",
        [](const std::string& kind, py::dict opts, int serve) {
          auto g = genLsdb(kind, opts);
          py::gil_scoped_release nogil;
          AreaLinkStates als;
          auto& ls = als.emplace(g.area, LinkState(g.area, "test_node")).first->second;
          PrefixState ps;
          loadLsdb(g, ls, ps);
          SpfSolver solver("test_node", true, false, false);
          const std::vector<std::string> names = ls.flat().names;
          RouteDbBatch batch(solver, als, ps, names);
          batch.launch();  // warm-up (workspace, code objects)
          ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
          auto t0 = std::chrono::steady_clock::now();
          batch.launch();
          ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
          const double launchMs = std::chrono::duration<double, std::milli>(
                                      std::chrono::steady_clock::now() - t0).count();
          uint64_t routes = 0;
          const int n = std::max(1, std::min<int>(serve, int(names.size())));
          // one untimed serve first: a serving process runs warm (the first
          // call in a process also pays its heap growth, 108 vs 50-65 ms)
          (void)batch.getRouteDbComputed(names.back());
          t0 = std::chrono::steady_clock::now();
          for (int i = 0; i < n; ++i) {
            const RouteDatabase r = batch.getRouteDbComputed(names[(size_t(i) * 7919) % names.size()]);
            routes += r.unicastRoutes.size();
          }
          const double serveMs = std::chrono::duration<double, std::milli>(
                                     std::chrono::steady_clock::now() - t0).count() / n;
          return std::make_tuple(launchMs, serveMs, double(routes) / n, names.size());
        });

  py::class_<VariantRunner>(m, "VariantRunner")
      .def(py::init<bool, bool>(), py::arg("enableV4") = true,
           py::arg("enableBestRouteSelection") = false)
      .def("setup", &VariantRunner::setup, py::arg("kind"), py::arg("opts"),
           py::arg("source"), py::arg("count"), py::arg("seed") = 0xC4F,
           py::arg("dualPermille") = 500, py::arg("lo") = 0, py::arg("hi") = -1)
      .def("run_base", [](VariantRunner& r, uintptr_t stream) {
             py::gil_scoped_release nogil;
             r.runBase(stream);
           }, py::arg("stream") = 0)
      .def("launch", [](VariantRunner& r, uintptr_t stream, bool records) {
             py::gil_scoped_release nogil;
             r.launch(stream, records);
           }, py::arg("stream") = 0, py::arg("records") = true)
      .def("download", &VariantRunner::download)
      .def("set_mode", &VariantRunner::setMode, py::arg("mode"))
      .def("mode", &VariantRunner::mode)
      .def("fetch_updates", [](VariantRunner& r, uintptr_t stream) { r.fetchUpdates(stream); },
           py::arg("stream") = 0)
      .def("base_canonical", [](const VariantRunner& r) { return py::bytes(r.baseCanonical()); })
      .def("updated_canonical",
           [](const VariantRunner& r, size_t v) { return py::bytes(r.updatedCanonical(v)); })
      .def("updated_canonicals_all", [](const VariantRunner& r, int threads) {
        py::list out;
        for (auto& c : r.updatedCanonicalsAll(threads)) out.append(py::bytes(c));
        return out;
      }, py::arg("threads") = 0)
      .def("update", &VariantRunner::updateOf)
      .def("total_changes", &VariantRunner::totalChanges)
      .def("materialize_all", &VariantRunner::materializeAll, py::arg("threads") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("num_variants", &VariantRunner::numVariants)
      .def("canonical", [](const VariantRunner& r, size_t v) { return py::bytes(r.canonicalOf(v)); })
      .def("changed", &VariantRunner::changedOf)
      .def("counts", &VariantRunner::countsOf)
      .def("shape", &VariantRunner::shape);

  py::class_<C5Runner>(m, "C5Runner")
      .def(py::init<>())
      .def("setup", &C5Runner::setup, py::arg("opts"), py::arg("source"),
           py::arg("policy") = py::list(), py::arg("brs") = true, py::arg("rank") = 0,
           py::arg("world") = 1)
      .def("launch_routes", [](C5Runner& r, uintptr_t stream) {
             py::gil_scoped_release nogil;
             r.launchRoutes(stream);
           }, py::arg("stream") = 0)
      .def("launch_ksp", [](C5Runner& r, uintptr_t stream) {
             py::gil_scoped_release nogil;
             r.launchKsp(stream);
           }, py::arg("stream") = 0)
      .def("set_policy", &C5Runner::setPolicy, py::arg("policy"))
      .def("source_neighbors", &C5Runner::sourceNeighbors)
      .def("area_names", &C5Runner::areaNames)
      .def("fetch", &C5Runner::fetch)
      .def("routes", &C5Runner::routes)
      .def("ksp_text", &C5Runner::kspText)
      .def("ksp_dests", &C5Runner::kspDests)
      .def("routes_digest", &C5Runner::routesDigest, py::arg("stream") = 0)
      .def("shape", &C5Runner::shape);

  py::class_<BatchRunner>(m, "BatchRunner")
      .def(py::init<bool, bool, bool>(), py::arg("enableV4") = true,
           py::arg("enableNodeSegmentLabel") = false,
           py::arg("enableBestRouteSelection") = false)
      .def("add_generated",
           [](BatchRunner& b, const std::string& kind, py::dict opts,
              std::vector<std::string> sources) { b.addLsdb(genLsdb(kind, opts), sources); })
      .def("add_grid_batch",
           [](BatchRunner& b, py::dict opts, int lo, int hi, const std::string& source) {
             // topology t: metric seed base+t, prefix seed base+t (config C2)
             auto base = gridOpts(opts);
             for (int t = lo; t < hi; ++t) {
               auto o = base;
               o.metricSeed = base.metricSeed + t;
               o.prefixSeed = base.prefixSeed + t;
               if (o.overloadSeed) o.overloadSeed = base.overloadSeed + t;
               b.addLsdb(topogen::grid(o), {source});
             }
           })
      .def("upload", &BatchRunner::upload)
      .def("set_sel_output", &BatchRunner::setSelOutput)
      .def("run", [](BatchRunner& b) {
        py::gil_scoped_release nogil;
        b.run();
      })
      .def("download", &BatchRunner::download)
      .def("num_units", &BatchRunner::numUnits)
      .def("canonical", [](const BatchRunner& b, size_t u) { return py::bytes(canonical(b.routeDb(u))); })
      .def("unit_digest",  // route_digest.h unit() of the materialised RouteDb
           [](const BatchRunner& b, size_t u, const std::string& key) {
             return digest::unit(key, b.routeDb(u));
           })
      .def("records_digests",
           [](const BatchRunner& b, const std::vector<std::string>& keys, py::array meta,
              py::array metric, py::array mask, int W, int threads,
              const std::vector<int64_t>& rows) {
             auto words = [](const py::array& a, size_t n, const char* what) {
               if (a.itemsize() != 4 || !(a.flags() & py::array::c_style) ||
                   size_t(a.size()) < n) {
                 throw std::invalid_argument(std::string(what) +
                                             ": contiguous 32-bit array of the runner's shape");
               }
               return static_cast<const uint32_t*>(a.data());
             };
             const size_t U = rows.empty() ? b.numUnits() : rows.size();
             const size_t Sp = std::max(b.host().maxPrefixes, 1);
             const uint32_t* me = words(meta, U * Sp, "meta");
             const uint32_t* mt = words(metric, U * Sp, "metric");
             const uint32_t* mk = words(mask, U * W * Sp, "mask");
             py::gil_scoped_release nogil;
             return b.recordsDigests(keys, me, mt, mk, W, threads, rows);
           },
           py::arg("keys"), py::arg("meta"), py::arg("metric"), py::arg("mask"),
           py::arg("nh_words"), py::arg("threads") = 8,
           py::arg("rows") = std::vector<int64_t>{})
      .def("route_counts",
           [](const BatchRunner& b) {
             std::vector<size_t> c;
             for (size_t u = 0; u < b.numUnits(); ++u) c.push_back(b.routeDb(u).unicastRoutes.size());
             return c;
           })
      .def("flags", &BatchRunner::flags)
      .def("set_slot_order", &BatchRunner::setSlotOrder,
           "use the 2-colour relaxation order (default on; takes effect at upload)")
      .def("set_slot_edge_image", &BatchRunner::setSlotEdgeImage,
           "hand the wave kernel the per-position edge image (default on)")
      .def("nh_words", &BatchRunner::nhWords)
      .def("wide", &BatchRunner::wide)
      .def("host_arrays", [](const BatchRunner& b) {
        // the exact HBM image the kernel consumes (bench.py uploads it)
        const HostBatch& h = b.host();
        py::dict d;
        d["node_base"] = npcopy(h.nodeBase);
        d["topo_desc"] = npcopy(h.topoDesc);
        d["row_ptr"] = npcopy(h.rowPtr);
        d["edges"] = npcopy(h.edges);
        d["edge_src"] = npcopy(h.edgeSrc);
        d["node_flags"] = npcopy(h.nodeFlags);
        d["pfx_base"] = npcopy(h.pfxBase);
        d["adv_off"] = npcopy(h.advOff);
        d["adv_node"] = npcopy(h.advNode);
        d["adv_metrics"] = npcopy(h.advMetrics);
        d["adv_min_nh"] = npcopy(h.advMinNh);
        d["pfx_flags"] = npcopy(h.pfxFlags);
        std::vector<uint16_t> slots;
        std::vector<uint32_t> slotEdges;
        int slotDegree = 0;
        d["slot_stride"] = h.slotOrder(slots, &slotEdges, &slotDegree);
        d["slot_node"] = npcopy(slots);
        d["slot_edges"] = npcopy(slotEdges);
        d["slot_degree"] = slotDegree;
        std::vector<uint32_t> u;
        for (const auto& x : b.units()) {
          u.push_back(x.topo);
          u.push_back(x.src);
        }
        d["units"] = npcopy(u);
        d["max_nodes"] = h.maxNodes;
        d["max_edges"] = h.maxEdges;
        d["max_prefixes"] = h.maxPrefixes;
        d["max_advertisements"] = h.maxAdvs;
        d["max_degree"] = h.maxDegree;
        d["num_topos"] = int(h.nodeBase.size() - 1);
        d["nh_words"] = b.nhWords();
        d["flags"] = b.flags();
        return d;
      })
      .def("dist", [](const BatchRunner& b) { return npcopy(b.dist()); })
      .def("meta", [](const BatchRunner& b) { return npcopy(b.meta()); })
      .def("metric", [](const BatchRunner& b) { return npcopy(b.metric()); })
      .def("mask", [](const BatchRunner& b) { return npcopy(b.mask()); });
}
