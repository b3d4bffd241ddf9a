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
#include <algorithm>
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
    throw std::domain_error("RouteDbBatch: one area (multi-area builds go through buildRouteDb)");
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
    const int W = std::max(1, ogs_nh_words_for_degree(int(f.rowPtr[s + 1] - f.rowPtr[s])));
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
  const ogs_graph g = graph();
  const ogs_prefix_table pt = table();
  const uint32_t flags = (solver_.enableV4_ ? OGS_F_ENABLE_V4 : 0u) |
      (solver_.v4OverV6Nexthop_ ? OGS_F_V4_OVER_V6 : 0u) |
      (solver_.enableBestRouteSelection_ ? OGS_F_BEST_ROUTE_SELECTION : 0u) |
      (wide_ ? OGS_F_WIDE_METRIC : 0u) | (exact_ ? OGS_F_EXACT_ORDER : 0u);
  for (Group& G : groups_) {
    ogs_spf_out out{G.dist.get(), G.nh.as<uint32_t>(), G.meta.as<uint32_t>(),
                    G.metric.get(), G.mask.as<uint32_t>(), G.sel.as<uint32_t>()};
    ogsCheck(ogs_spf_routes(&g, hb_.maxPrefixes ? &pt : nullptr, G.units.as<ogs_unit>(),
                            int32_t(G.members.size()), flags, G.W, &out, stream),
             "ogs_spf_routes(batch)");
    ls_->noteSpfRuns(G.members.size());
  }
  launched_ = true;
}

std::optional<DecisionRouteDb> RouteDbBatch::routeDb(const std::string& node,
                                                     void* stream) const {
  auto it = index_.find(node);
  if (it == index_.end()) throw std::out_of_range("RouteDbBatch: not a source: " + node);
  if (!launched_) throw std::logic_error("RouteDbBatch: launch() first");
  const auto [gi, u] = units_[it->second];
  if (gi == SIZE_MAX) return std::nullopt;  // SpfSolver.cpp:318-324
  const Group& G = groups_[gi];
  const FlatTopology& f = ls_->flat();
  const size_t N = f.names.size(), P = table_.prefixes.size();
  const size_t Sn = size_t(std::max(hb_.maxNodes, 1)), Sp = size_t(std::max(hb_.maxPrefixes, 1));
  const size_t db = wide_ ? 8 : 4;
  const int W = G.W;
  // this unit's slices only: dist[u*Sn], nh[(u*W+w)*Sn], meta/metric/sel[u*Sp],
  // mask[(u*W+w)*Sp]
  auto fetch = [&](const DeviceBuffer& b, size_t elemOff, size_t n, size_t esz, void* host) {
    if (n == 0) return;
    ogsCheck(ogs_memcpy_d2h(host, static_cast<const char*>(b.get()) + elemOff * esz, n * esz,
                            stream),
             "ogs_memcpy_d2h");
  };
  std::vector<uint64_t> dist(N), metric(P);
  std::vector<uint32_t> d32(wide_ ? 0 : N), m32(wide_ ? 0 : P);
  std::vector<uint32_t> nh(W * Sn), meta(P), mask(W * Sp), sel(P);
  fetch(G.dist, u * Sn, N, db, wide_ ? static_cast<void*>(dist.data()) : d32.data());
  fetch(G.nh, u * W * Sn, W * Sn, 4, nh.data());
  fetch(G.meta, u * Sp, P, 4, meta.data());
  fetch(G.metric, u * Sp, P, db, wide_ ? static_cast<void*>(metric.data()) : m32.data());
  fetch(G.mask, u * W * Sp, W * Sp, 4, mask.data());
  fetch(G.sel, u * Sp, P, 4, sel.data());
  ogsCheck(ogs_stream_sync(stream), "ogs_stream_sync");
  if (!wide_) {
    for (size_t i = 0; i < N; ++i) dist[i] = d32[i] == 0xFFFFFFFFu ? ~0ull : d32[i];
    for (size_t i = 0; i < P; ++i) metric[i] = m32[i] == 0xFFFFFFFFu ? ~0ull : m32[i];
  }
  UnitView view;
  view.W = W;
  view.N = uint32_t(N);
  view.P = uint32_t(P);
  view.dist = dist.data();
  view.nh = nh.data();
  view.nhStride = Sn;
  view.meta = meta.data();
  view.metric = metric.data();
  view.mask = mask.data();
  view.maskStride = Sp;
  view.sel = sel.data();
  return materializeRouteDb(*ls_, f, area_, node, view, table_, solver_.v4OverV6Nexthop_,
                            solver_.enableNodeSegmentLabel_, solver_.staticUnicastRoutes_,
                            nullptr);
}

RouteDatabase RouteDbBatch::getRouteDbComputed(const std::string& node, void* stream) const {
  RouteDatabase out;  // Decision.cpp:341-360
  const std::string& n = node.empty() ? solver_.myNodeName_ : node;
  if (auto db = routeDb(n, stream)) out = db->toThrift();
  out.thisNodeName = n;
  return out;
}

}  // namespace openr_amd
