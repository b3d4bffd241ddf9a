// route_db_batch.cpp — RouteDbBatch: many sources' RouteDbs resident in HBM,
// served per node, and DecisionRouteDb::toThrift.
//
// Reference: Decision::getDecisionRouteDb (Decision.cpp:341-360) answers
// OpenrCtrl getRouteDbComputed(node) (OpenrCtrlHandler.cpp:640-643) with
// SpfSolver::buildRouteDb(node) -> DecisionRouteDb::toThrift
// (SpfSolver.h:82-94, RibEntry.h:95-103, 144-151) and thisNodeName = node.
// The batch runs that build for every listed source in one launch per
// next-hop width group (the C3 all-sources kernels), leaves the compact
// records in HBM and materialises a node's RouteDb only when it is asked for.
#include <thread>
#include <algorithm>
#include <memory>
#include <stdexcept>

#include "decision.h"

namespace openr_amd {

RouteDatabase DecisionRouteDb::toThrift() const {
  RouteDatabase db;
  for (const auto& [_, e] : unicastRoutes) {  // RibEntry.h:95-103
    db.unicastRoutes.push_back(
        UnicastRoute{e.prefix, std::vector<NextHopThrift>(e.nexthops.begin(), e.nexthops.end()),
                     e.counterID});
  }
  for (const auto& [_, e] : mplsRoutes) {  // RibEntry.h:144-151
    db.mplsRoutes.push_back(
        MplsRoute{e.label, std::vector<NextHopThrift>(e.nexthops.begin(), e.nexthops.end())});
  }
  return db;
}

RouteDbBatch::RouteDbBatch(const SpfSolver& solver, const AreaLinkStates& als,
                           const PrefixState& ps, const std::vector<std::string>& sources)
    : solver_(solver), sources_(sources) {
  if (als.size() != 1) {
    // multi-area domain: each served node is a multi-area buildRouteDb
    // (route_multiarea_kernel over every area's SPF) on a private solver with
    // the caller's settings and static routes -- getDecisionRouteDb exactly
    multiArea_ = true;
    als_ = &als;
    ps_ = &ps;
    for (size_t i = 0; i < sources_.size(); ++i) {
      if (!index_.emplace(sources_[i], i).second) {
        throw std::invalid_argument("RouteDbBatch: duplicate source " + sources_[i]);
      }
    }
    multi_ = std::make_unique<SpfSolver>(solver.myNodeName_, solver.enableV4_,
                                         solver.enableNodeSegmentLabel_,
                                         solver.enableBestRouteSelection_,
                                         solver.v4OverV6Nexthop_);
    multi_->staticUnicastRoutes_ = solver.staticUnicastRoutes_;
    return;
  }
  area_ = als.begin()->first;
  ls_ = &als.begin()->second;
  const FlatTopology& f = ls_->flatOnDevice();
  // zero / negative metrics: the reference's extraction order (spf_exact.hip)
  exact_ = f.hasZeroMetric || f.hasWideMetric;
  wide_ = exact_ || wideDistancesNeeded(f);
  table_.build(ps);
  hb_.append(f, ps, area_);
  // group sources by next-hop bitset width so each launch writes masks of
  // its own width (C3: FSW rows need 3 words, the rest 1)
  units_.assign(sources_.size(), {SIZE_MAX, 0});
  for (size_t i = 0; i < sources_.size(); ++i) {
    if (!index_.emplace(sources_[i], i).second) {
      throw std::invalid_argument("RouteDbBatch: duplicate source " + sources_[i]);
    }
    auto it = f.id.find(sources_[i]);
    if (it == f.id.end()) continue;  // no adjacency database: nullopt
    const uint32_t s = it->second;
    const int W = batchNhWords(int(f.rowPtr[s + 1] - f.rowPtr[s]), f.names.size(), wide_);
    auto g = std::find_if(groups_.begin(), groups_.end(), [&](const Group& x) { return x.W == W; });
    if (g == groups_.end()) {
      groups_.emplace_back();
      groups_.back().W = W;
      g = groups_.end() - 1;
    }
    units_[i] = {size_t(g - groups_.begin()), g->members.size()};
    g->members.push_back(uint32_t(i));
  }
  dDesc_.upload(hb_.topoDesc.data(), hb_.topoDesc.size());
  dPfxBase_.upload(hb_.pfxBase.data(), hb_.pfxBase.size());
  dAdvOff_.upload(hb_.advOff.data(), hb_.advOff.size());
  dAdvNode_.upload(hb_.advNode.data(), hb_.advNode.size());
  dAdvMetrics_.upload(hb_.advMetrics.data(), hb_.advMetrics.size());
  dAdvMinNh_.upload(hb_.advMinNh.data(), hb_.advMinNh.size());
  dPfxFlags_.upload(hb_.pfxFlags.data(), hb_.pfxFlags.size());
  const size_t Sn = size_t(std::max(hb_.maxNodes, 1)), Sp = size_t(std::max(hb_.maxPrefixes, 1));
  const size_t db = wide_ ? 8 : 4;
  for (Group& g : groups_) {
    const size_t U = g.members.size();
    std::vector<ogs_unit> units(U);
    for (size_t k = 0; k < U; ++k) units[k] = ogs_unit{0, f.id.at(sources_[g.members[k]])};
    g.units.upload(units.data(), units.size());
    g.dist.resize(U * Sn * db);
    g.nh.resize(U * g.W * Sn * 4);
    g.meta.resize(U * Sp * 4);
    g.metric.resize(U * Sp * db);
    g.mask.resize(U * g.W * Sp * 4);
    g.sel.resize(U * Sp * 4);
    g.reach.resize(std::max<size_t>(U * ((Sn + 31) / 32) * 4, 4));
  }
}

ogs_graph RouteDbBatch::graph() const {
  const FlatTopology& f = ls_->flatOnDevice();
  ogs_graph g{};
  g.num_topos = 1;
  g.max_nodes = int32_t(f.names.size());
  g.max_edges = int32_t(f.edges.size());
  g.max_degree = f.maxDegree;
  g.topo_desc = dDesc_.as<uint32_t>();
  g.node_base = f.dNodeBase.as<uint32_t>();
  g.row_ptr = f.dRow.as<uint32_t>();
  g.edges = f.dEdges.as<uint64_t>();
  g.node_flags = f.dFlags.as<uint8_t>();
  g.slot_node = f.slotStride ? f.dSlot.as<uint16_t>() : nullptr;
  g.slot_stride = f.slotStride;
  g.slot_edges = f.slotDegree ? f.dSlotEdges.as<uint32_t>() : nullptr;
  g.slot_degree = f.slotDegree;
  g.edge_src = f.dEdgeSrc.as<uint32_t>();
  return g;
}

ogs_prefix_table RouteDbBatch::table() const {
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

void RouteDbBatch::launch(void* stream) {
  if (multiArea_) {  // built per served node (routeDb)
    launched_ = true;
    return;
  }
  const ogs_graph g = graph();
  const ogs_prefix_table pt = table();
  const uint32_t flags = (solver_.enableV4_ ? OGS_F_ENABLE_V4 : 0u) |
      (solver_.v4OverV6Nexthop_ ? OGS_F_V4_OVER_V6 : 0u) |
      (solver_.enableBestRouteSelection_ ? OGS_F_BEST_ROUTE_SELECTION : 0u) |
      (wide_ ? OGS_F_WIDE_METRIC : 0u) | (exact_ ? OGS_F_EXACT_ORDER : 0u);
  // every width group in one call (one prep + one persistent launch for
  // all of them on the large-topology form, ogs_spf_routes_groups)
  std::vector<ogs_route_group> rg;
  rg.reserve(groups_.size());
  for (Group& G : groups_) {
    ogs_spf_out out{G.dist.get(), G.nh.as<uint32_t>(), G.meta.as<uint32_t>(),
                    G.metric.get(), G.mask.as<uint32_t>(), G.sel.as<uint32_t>(),
                    exact_ ? G.reach.as<uint32_t>() : nullptr};
    rg.push_back(ogs_route_group{G.units.as<ogs_unit>(), int32_t(G.members.size()), G.W, out});
  }
  ogsCheck(ogs_spf_routes_groups(&g, hb_.maxPrefixes ? &pt : nullptr, rg.data(),
                                 int32_t(rg.size()), flags, stream),
           "ogs_spf_routes_groups(batch)");
  for (Group& G : groups_) {
    for (uint32_t m : G.members) ls_->noteSpf(sources_[m]);
    addStatValue("decision.gpu.spf_launches", double(G.members.size()), StatType::COUNT);
  }
  launched_ = true;
}

// one unit's records D2H (its slices only: dist[u*Sn], nh[(u*W+w)*Sn],
// meta/metric/sel[u*Sp], mask[(u*W+w)*Sp]), distances widened
struct RouteDbBatch::UnitRecords {
  std::vector<uint64_t> dist, metric;
  std::vector<uint32_t> nh, meta, mask, sel;
  std::vector<uint32_t> reach;  // exact-order settled bitset (else empty)
  int W{1};
  size_t Sn{1}, Sp{1};
};

bool RouteDbBatch::fetchUnit(const std::string& node, void* stream, UnitRecords& r) const {
  auto it = index_.find(node);
  if (it == index_.end()) throw std::out_of_range("RouteDbBatch: not a source: " + node);
  if (!launched_) throw std::logic_error("RouteDbBatch: launch() first");
  const auto [gi, u] = units_[it->second];
  if (gi == SIZE_MAX) return false;  // SpfSolver.cpp:318-324
  const Group& G = groups_[gi];
  const FlatTopology& f = ls_->flat();
  const size_t N = f.names.size(), P = table_.prefixes.size();
  r.Sn = size_t(std::max(hb_.maxNodes, 1));
  r.Sp = size_t(std::max(hb_.maxPrefixes, 1));
  const size_t db = wide_ ? 8 : 4, Sn = r.Sn, Sp = r.Sp;
  const int W = r.W = G.W;
  auto fetch = [&](const DeviceBuffer& b, size_t elemOff, size_t n, size_t esz, void* host) {
    if (n == 0) return;
    ogsCheck(ogs_memcpy_d2h(host, static_cast<const char*>(b.get()) + elemOff * esz, n * esz,
                            stream),
             "ogs_memcpy_d2h");
  };
  r.dist.resize(N);
  r.metric.resize(P);
  std::vector<uint32_t> d32(wide_ ? 0 : N), m32(wide_ ? 0 : P);
  r.nh.resize(W * Sn);
  r.meta.resize(P);
  r.mask.resize(W * Sp);
  r.sel.resize(P);
  fetch(G.dist, u * Sn, N, db, wide_ ? static_cast<void*>(r.dist.data()) : d32.data());
  fetch(G.nh, u * W * Sn, W * Sn, 4, r.nh.data());
  fetch(G.meta, u * Sp, P, 4, r.meta.data());
  fetch(G.metric, u * Sp, P, db, wide_ ? static_cast<void*>(r.metric.data()) : m32.data());
  fetch(G.mask, u * W * Sp, W * Sp, 4, r.mask.data());
  fetch(G.sel, u * Sp, P, 4, r.sel.data());
  if (exact_) {
    const size_t RW = (Sn + 31) / 32;
    r.reach.resize(RW);
    fetch(G.reach, u * RW, RW, 4, r.reach.data());
  }
  ogsCheck(ogs_stream_sync(stream), "ogs_stream_sync");
  if (!wide_) {
    for (size_t i = 0; i < N; ++i) r.dist[i] = d32[i] == 0xFFFFFFFFu ? ~0ull : d32[i];
    for (size_t i = 0; i < P; ++i) r.metric[i] = m32[i] == 0xFFFFFFFFu ? ~0ull : m32[i];
  }
  return true;
}

std::optional<DecisionRouteDb> RouteDbBatch::routeDb(const std::string& node,
                                                     void* stream) const {
  if (multiArea_) {
    if (!index_.count(node)) throw std::out_of_range("RouteDbBatch: not a source: " + node);
    if (!launched_) throw std::logic_error("RouteDbBatch: launch() first");
    std::lock_guard<std::mutex> lk(multiMu_);
    return multi_->buildRouteDb(node, *als_, *ps_);
  }
  UnitRecords r;
  if (!fetchUnit(node, stream, r)) return std::nullopt;
  const FlatTopology& f = ls_->flat();
  UnitView view;
  view.W = r.W;
  view.N = uint32_t(f.names.size());
  view.P = uint32_t(table_.prefixes.size());
  view.dist = r.dist.data();
  view.nh = r.nh.data();
  view.nhStride = r.Sn;
  view.meta = r.meta.data();
  view.metric = r.metric.data();
  view.mask = r.mask.data();
  view.maskStride = r.Sp;
  view.sel = r.sel.data();
  view.reach = r.reach.empty() ? nullptr : r.reach.data();
  return materializeRouteDb(*ls_, f, area_, node, view, table_, solver_.v4OverV6Nexthop_,
                            solver_.enableNodeSegmentLabel_, solver_.staticUnicastRoutes_,
                            nullptr);
}

// getDecisionRouteDb + toThrift (Decision.cpp:341-360, SpfSolver.h:82-94,
// RibEntry.h:95-103 / 144-151) straight from the records: the thrift form
// carries only prefix, next hops and counterID, so no DecisionRouteDb /
// RibUnicastEntry (best entry, area, ...) is built. Next hops come from
// per-link-slot templates pre-sorted in NextHopThrift order (a route's next
// hops share its metric, so slot order = set order), prefixes in table
// order (= the DecisionRouteDb map order), built in parallel chunks and
// merged with the static routes. Equal to routeDb(node)->toThrift()
// (tests/test_gpu_route_db_batch.py).
RouteDatabase RouteDbBatch::getRouteDbComputed(const std::string& node, void* stream) const {
  RouteDatabase out;  // Decision.cpp:341-360
  const std::string& n = node.empty() ? solver_.myNodeName_ : node;
  out.thisNodeName = n;
  if (multiArea_) {
    if (auto db = routeDb(n, stream)) {
      RouteDatabase t = db->toThrift();
      out.unicastRoutes = std::move(t.unicastRoutes);
      out.mplsRoutes = std::move(t.mplsRoutes);
    }
    return out;
  }
  UnitRecords r;
  if (!fetchUnit(n, stream, r)) return out;
  const FlatTopology& f = ls_->flat();
  const uint32_t s = f.id.at(n);
  const uint32_t rb = f.rowPtr[s], deg = f.rowPtr[s + 1] - rb;
  const size_t P = table_.prefixes.size();
  // next-hop templates per link slot, v6 (0) and v4 (1) address flavours,
  // and the slots of each flavour in NextHopThrift order
  std::vector<NextHopThrift> tmpl[2];
  std::vector<uint32_t> order[2];
  for (int fl = 0; fl < 2; ++fl) {
    tmpl[fl].reserve(deg);
    for (uint32_t j = 0; j < deg; ++j) {
      const Link& l = *f.edgeLink[rb + j];
      NextHopThrift nh;
      nh.address = fl ? l.getNhV4FromNode(n) : l.getNhV6FromNode(n);
      nh.ifName = l.getIfaceFromNode(n);
      nh.area = l.getArea();
      nh.neighborNodeName = l.getOtherNodeName(n);
      tmpl[fl].push_back(std::move(nh));
    }
    order[fl].resize(deg);
    for (uint32_t j = 0; j < deg; ++j) order[fl][j] = j;
    std::stable_sort(order[fl].begin(), order[fl].end(),
                     [&](uint32_t a, uint32_t b) { return tmpl[fl][a] < tmpl[fl][b]; });
  }
  const int W = r.W;
  const size_t Sp = r.Sp;
  // routes in prefix order (the DecisionRouteDb map's), merged with the
  // statics below
  const std::vector<uint32_t>& sorted = table_.sortedOrder();
  auto build = [&](size_t i0, size_t i1, std::vector<UnicastRoute>& dst) {
    for (size_t i = i0; i < i1; ++i) {
      const size_t p = sorted[i];
      if (!(r.meta[p] & OGS_ROUTE_VALID)) continue;
      const std::string& prefix = table_.prefixes[p];
      const int fl = (isV4Prefix(prefix) && !solver_.v4OverV6Nexthop_) ? 1 : 0;
      const int32_t m32 = static_cast<int32_t>(r.metric[p]);
      UnicastRoute ur;
      ur.dest = prefix;
      for (uint32_t j : order[fl]) {
        if (!((r.mask[size_t(j / 32) * Sp + p] >> (j % 32)) & 1u)) continue;
        NextHopThrift nh = tmpl[fl][j];
        nh.metric = m32;
        ur.nextHops.push_back(std::move(nh));
      }
      dst.push_back(std::move(ur));
    }
  };
  (void)W;
  const size_t T = std::max<size_t>(
      1, std::min<size_t>({16, std::max(1u, std::thread::hardware_concurrency()), P / 8192 + 1}));
  std::vector<std::vector<UnicastRoute>> parts(T);
  {
    std::vector<std::thread> pool;
    for (size_t t = 1; t < T; ++t) {
      pool.emplace_back(build, P * t / T, P * (t + 1) / T, std::ref(parts[t]));
    }
    build(0, P / T, parts[0]);
    for (auto& th : pool) th.join();
  }
  // merge with the statics (a computed route wins, SpfSolver.cpp:343-349)
  const auto& statics = solver_.staticUnicastRoutes_;
  size_t total = statics.size();
  for (const auto& part : parts) total += part.size();
  out.unicastRoutes.reserve(total);
  auto st = statics.begin();
  auto emitStatic = [&](const RibUnicastEntry& e) {
    out.unicastRoutes.push_back(UnicastRoute{
        e.prefix, std::vector<NextHopThrift>(e.nexthops.begin(), e.nexthops.end()), e.counterID});
  };
  for (auto& part : parts) {
    for (auto& ur : part) {
      while (st != statics.end() && st->first < ur.dest) emitStatic((st++)->second);
      if (st != statics.end() && st->first == ur.dest) ++st;
      out.unicastRoutes.push_back(std::move(ur));
    }
  }
  for (; st != statics.end(); ++st) emitStatic(st->second);
  // node-label MPLS routes (SpfSolver.cpp:354-445), label order
  if (solver_.enableNodeSegmentLabel_) {
    LabelRoutes labelToNode;
    addNodeLabelRoutes(*ls_, f, area_, n, r.dist.data(), r.nh.data(), r.Sn, r.W, labelToNode,
                       r.reach.empty() ? nullptr : r.reach.data());
    for (auto& [label, ne] : labelToNode) {
      out.mplsRoutes.push_back(MplsRoute{
          label, std::vector<NextHopThrift>(ne.second.nexthops.begin(), ne.second.nexthops.end())});
    }
  }
  return out;
}

}  // namespace openr_amd
