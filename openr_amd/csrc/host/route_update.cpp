// route_update.cpp — LinkFailureSweep: batched what-if route updates
// (SURVEY.md §8(f) f1 over config C4).
//
// Reference: Decision::rebuildRoutes (Decision.cpp:912-951) rebuilds the
// RouteDb after a topology change and publishes
// DecisionRouteDb::calculateUpdate(old, new) (SpfSolver.cpp:21-56) to Fib.
// Here the "new" RouteDbs of many link-failure variants come out of one
// ogs_spf_routes_variants launch with that diff fused in; the changed records
// are gathered on the device and only those are materialised into
// DecisionRouteUpdate (unicastRoutesToUpdate / unicastRoutesToDelete).
#include <algorithm>
#include <atomic>
#include <exception>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "decision.h"

namespace openr_amd {

LinkFailureSweep::LinkFailureSweep(
    const std::string& myNodeName, const LinkState& ls, const PrefixState& ps,
    const std::vector<std::vector<LinkDown>>& variants, bool enableV4,
    bool enableBestRouteSelection, bool v4OverV6Nexthop)
    : ls_(ls),
      ps_(ps),
      me_(myNodeName),
      area_(ls.getArea()),
      enableV4_(enableV4),
      brs_(enableBestRouteSelection),
      v4OverV6_(v4OverV6Nexthop) {
  const FlatTopology& f = ls.flat();
  auto sIt = f.id.find(me_);
  if (sIt == f.id.end()) {
    throw std::invalid_argument("LinkFailureSweep: " + me_ + " is not in area " + area_);
  }
  const bool wide = wideDistancesNeeded(f);
  table_.build(ps);
  hb_.append(f, ps, area_);
  // zero / negative link metrics (extraction-order replay) or path sums past
  // 32 bits: the variants kernel's packed 32-bit {dist, nh} repair does not
  // apply, every variant runs as a topology of its own (exactLaunch)
  exact_ = wide || hb_.hasZeroMetric;
  exactOrder_ = f.hasZeroMetric || f.hasWideMetric;
  const uint32_t s = sIt->second;
  W_ = std::max(1, ogs_nh_words_for_degree(int(f.rowPtr[s + 1] - f.rowPtr[s])));
  // next-hop sets of more than 4 words (source degree > 128): past the
  // variants kernel, ogs_spf_routes takes up to 16
  if (W_ > 4) exact_ = true;

  // dead directed edges: both directions of every failed link
  auto edgeOf = [&](const std::string& node, auto&& pred) -> uint32_t {
    auto it = f.id.find(node);
    if (it == f.id.end()) throw std::invalid_argument("LinkFailureSweep: unknown node " + node);
    for (uint32_t e = f.rowPtr[it->second]; e < f.rowPtr[it->second + 1]; ++e) {
      if (pred(*f.edgeLink[e])) return e;
    }
    return OGS_NODE_NONE;
  };
  dead_.assign(variants.size() * kDeadMax, OGS_NODE_NONE);
  for (size_t v = 0; v < variants.size(); ++v) {
    if (variants[v].size() * 2 > size_t(kDeadMax)) {
      throw std::invalid_argument("LinkFailureSweep: more than 2 links in a variant");
    }
    size_t k = 0;
    for (const auto& d : variants[v]) {
      const Link* link = nullptr;
      const uint32_t e = edgeOf(d.node, [&](const Link& l) {
        if (l.getIfaceFromNode(d.node) != d.ifName) return false;
        link = &l;
        return true;
      });
      if (e == OGS_NODE_NONE) {
        throw std::invalid_argument("LinkFailureSweep: no link " + d.node + "%" + d.ifName);
      }
      const std::string other = link->getOtherNodeName(d.node);
      const uint32_t r = edgeOf(other, [&](const Link& l) { return &l == link; });
      dead_[v * kDeadMax + k++] = e;
      if (r != OGS_NODE_NONE) dead_[v * kDeadMax + k++] = r;
    }
  }

  const size_t U = variants.size(), Sn = size_t(std::max(hb_.maxNodes, 1));
  Sp_ = size_t(std::max(hb_.maxPrefixes, 1));
  words_ = (Sp_ + 31) / 32;
  std::vector<ogs_unit> units(U, ogs_unit{0, s});
  const ogs_unit base{0, s};
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
  dUnits_.upload(units.data(), units.size());
  dBaseUnit_.upload(&base, 1);
  dDead_.upload(dead_.data(), dead_.size());
  // best-entry equality classes for the diff (ogs_route_diff.adv_class):
  // per prefix, the list [entries as is, entries with the drain override]
  // of materialised best entries (weight cleared, RibEntry.h:77), each
  // numbered by the first equal one
  {
    std::vector<uint32_t> cls(std::max<size_t>(2 * table_.advEntry.size(), 1), 0);
    for (size_t p = 0; p + 1 < table_.advOff.size(); ++p) {
      const uint32_t a0 = table_.advOff[p], k = table_.advOff[p + 1] - a0;
      std::vector<PrefixEntry> eff;
      eff.reserve(2 * k);
      for (int drained = 0; drained < 2; ++drained) {
        for (uint32_t i = 0; i < k; ++i) {
          PrefixEntry e = *table_.advEntry[a0 + i];
          e.weight = std::nullopt;
          if (drained) e.metrics.drain_metric = 1;
          eff.push_back(std::move(e));
        }
      }
      for (uint32_t j = 0; j < 2 * k; ++j) {
        uint32_t c = j;
        for (uint32_t i = 0; i < j; ++i) {
          if (eff[i] == eff[j]) {
            c = i;
            break;
          }
        }
        const uint32_t i = j % k, drained = j / k;
        cls[2 * (a0 + i) + drained] = c;
      }
    }
    dAdvClass_.upload(cls.data(), cls.size());
  }
  bDist_.resize(Sn * 4);
  bNh_.resize(W_ * Sn * 4);
  for (auto* b : {&bMeta_, &bMetric_, &bSel_}) b->resize(Sp_ * 4);
  bMask_.resize(W_ * Sp_ * 4);
  const size_t Uc = std::max<size_t>(U, 1);
  dDist_.resize(Uc * Sn * 4);
  dNh_.resize(Uc * W_ * Sn * 4);
  for (auto* b : {&dMeta_, &dMetric_, &dSel_}) b->resize(Uc * Sp_ * 4);
  dMask_.resize(Uc * W_ * Sp_ * 4);
  dChanged_.resize(Uc * words_ * 4);
  dCounts_.resize(Uc * 2 * 4);
}

// Variants outside the repair kernel's domain: ogs_spf_routes launches over
// the base (topology 0) and every variant's own topology copy (the failed
// links' edges marked down, the same skip the variants kernel applies to its
// dead-edge list), kExactChunk topologies per launch so that device and host
// copies stay bounded, in the exact extraction order when the area has zero
// or negative metrics, with 64-bit distances. fetch materialises the records and
// the update is DecisionRouteDb::calculateUpdate (SpfSolver.cpp:21-56) of the
// base and variant RouteDbs, as Decision::rebuildRoutes computes it.
void LinkFailureSweep::exactLaunch(void* stream) {
  const size_t U = numVariants(), T = U + 1;
  const FlatTopology& f = ls_.flat();
  const uint32_t s = f.id.at(me_);
  const uint32_t fl = flags() | OGS_F_WIDE_METRIC | (exactOrder_ ? OGS_F_EXACT_ORDER : 0u);
  xMeta_.assign(T * Sp_, 0);
  xMetric_.assign(T * Sp_, 0);
  xMask_.assign(T * W_ * Sp_, 0);
  DeviceBuffer nodeBase, desc, row, edges, edgeSrc, nflags, pfxBase, advOff, advNode,
      advMetrics, advMinNh, pfxFlags, units, meta, metric, mask;
  for (size_t c0 = 0; c0 < T; c0 += kExactChunk) {
    const size_t c1 = std::min(T, c0 + kExactChunk), n = c1 - c0;
    HostBatch hb;  // topology t - c0 = the base (t = 0) or variant t - 1
    for (size_t t = c0; t < c1; ++t) {
      const uint32_t e0 = uint32_t(hb.edges.size());
      hb.append(f, ps_, area_);
      if (t == 0) continue;
      for (int k = 0; k < kDeadMax; ++k) {
        const uint32_t e = dead_[(t - 1) * kDeadMax + k];
        if (e != OGS_NODE_NONE) hb.edges[e0 + e] |= OGS_EDGE_DOWN;
      }
    }
    std::vector<ogs_unit> us(n);
    for (size_t i = 0; i < n; ++i) us[i] = ogs_unit{uint32_t(i), s};
    nodeBase.upload(hb.nodeBase.data(), hb.nodeBase.size(), stream);
    desc.upload(hb.topoDesc.data(), hb.topoDesc.size(), stream);
    row.upload(hb.rowPtr.data(), hb.rowPtr.size(), stream);
    edges.upload(hb.edges.data(), hb.edges.size(), stream);
    edgeSrc.upload(hb.edgeSrc.data(), hb.edgeSrc.size(), stream);
    nflags.upload(hb.nodeFlags.data(), hb.nodeFlags.size(), stream);
    pfxBase.upload(hb.pfxBase.data(), hb.pfxBase.size(), stream);
    advOff.upload(hb.advOff.data(), hb.advOff.size(), stream);
    advNode.upload(hb.advNode.data(), hb.advNode.size(), stream);
    advMetrics.upload(hb.advMetrics.data(), hb.advMetrics.size(), stream);
    advMinNh.upload(hb.advMinNh.data(), hb.advMinNh.size(), stream);
    pfxFlags.upload(hb.pfxFlags.data(), hb.pfxFlags.size(), stream);
    units.upload(us.data(), us.size(), stream);
    meta.resize(n * Sp_ * 4);
    metric.resize(n * Sp_ * 8);
    mask.resize(n * W_ * Sp_ * 4);
    ogs_graph g{};
    g.num_topos = int32_t(n);
    g.max_nodes = hb.maxNodes;
    g.max_edges = hb.maxEdges;
    g.max_degree = hb.maxDegree;
    g.topo_desc = desc.as<uint32_t>();
    g.node_base = nodeBase.as<uint32_t>();
    g.row_ptr = row.as<uint32_t>();
    g.edges = edges.as<uint64_t>();
    g.node_flags = nflags.as<uint8_t>();
    g.edge_src = edgeSrc.as<uint32_t>();
    ogs_prefix_table pt{};
    pt.max_prefixes = hb.maxPrefixes;
    pt.max_advertisements = hb.maxAdvs;
    pt.pfx_base = pfxBase.as<uint32_t>();
    pt.adv_off = advOff.as<uint32_t>();
    pt.adv_node = advNode.as<uint32_t>();
    pt.adv_metrics = advMetrics.as<int32_t>();
    pt.adv_min_nh = advMinNh.as<int64_t>();
    pt.pfx_flags = pfxFlags.as<uint8_t>();
    ogs_spf_out out{nullptr, nullptr, meta.as<uint32_t>(), metric.get(), mask.as<uint32_t>(),
                    nullptr};
    ogsCheck(ogs_spf_routes(&g, &pt, units.as<ogs_unit>(), int32_t(n), fl, W_, &out, stream),
             "ogs_spf_routes(variant topologies)");
    meta.download(xMeta_.data() + c0 * Sp_, n * Sp_, stream);
    metric.download(xMetric_.data() + c0 * Sp_, n * Sp_, stream);
    // mask rows [(i * W + w) * Sp + p] of the chunk follow the previous ones
    mask.download(xMask_.data() + c0 * W_ * Sp_, n * W_ * Sp_, stream);
    ogsCheck(ogs_stream_sync(stream), "ogs_stream_sync");  // buffers reused
  }
  baseRun_ = recordsRun_ = true;
  changedOnlyRun_ = false;
}

void LinkFailureSweep::exactFetch(void* /*stream*/) {
  if (!recordsRun_) throw std::logic_error("LinkFailureSweep: launch() first");
  const size_t U = numVariants();
  const std::vector<uint32_t>& meta = xMeta_;
  const std::vector<uint32_t>& mask = xMask_;
  const std::vector<uint64_t>& metric = xMetric_;
  const FlatTopology& f = ls_.flat();
  auto dbOf = [&](size_t t) {
    DecisionRouteDb db;
    for (uint32_t p = 0; p < uint32_t(table_.prefixes.size()); ++p) {
      auto e = materializeRoute(f, me_, table_, p, meta[t * Sp_ + p], metric[t * Sp_ + p],
                                &mask[t * W_ * Sp_ + p], Sp_, W_, v4OverV6_, nullptr, OGS_POLICY_NONE,
                                OGS_POLICY_NONE);
      if (e) db.unicastRoutes.emplace(e->prefix, std::move(*e));
    }
    return db;
  };
  base_ = dbOf(0);
  xDb_.clear();
  xUpd_.clear();
  counts_.assign(2 * U, 0);
  offsets_.assign(U + 1, 0);
  for (size_t v = 0; v < U; ++v) {
    xDb_.push_back(dbOf(v + 1));
    xUpd_.push_back(base_->calculateUpdate(xDb_.back()));
    counts_[2 * v] = uint32_t(xUpd_.back().unicastRoutesToUpdate.size());
    counts_[2 * v + 1] = uint32_t(xUpd_.back().unicastRoutesToDelete.size());
    offsets_[v + 1] = offsets_[v] + counts_[2 * v] + counts_[2 * v + 1];
  }
}

uint32_t LinkFailureSweep::flags() const {
  return (enableV4_ ? OGS_F_ENABLE_V4 : 0u) | (brs_ ? OGS_F_BEST_ROUTE_SELECTION : 0u);
}

ogs_graph LinkFailureSweep::graph() const {
  ogs_graph g{};
  g.num_topos = 1;
  g.max_nodes = hb_.maxNodes;
  g.max_edges = hb_.maxEdges;
  g.max_degree = hb_.maxDegree;
  g.topo_desc = dDesc_.as<uint32_t>();
  g.node_base = dNodeBase_.as<uint32_t>();
  g.row_ptr = dRow_.as<uint32_t>();
  g.edges = dEdges_.as<uint64_t>();
  g.node_flags = dFlags_.as<uint8_t>();
  g.edge_src = dEdgeSrc_.as<uint32_t>();
  return g;
}

ogs_prefix_table LinkFailureSweep::table() const {
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

void LinkFailureSweep::runBase(void* stream) {
  if (exact_) return exactLaunch(stream);
  ogs_graph g = graph();
  ogs_prefix_table pt = table();
  ogs_spf_out out{bDist_.get(), bNh_.as<uint32_t>(), bMeta_.as<uint32_t>(),
                  bMetric_.get(), bMask_.as<uint32_t>(), bSel_.as<uint32_t>()};
  ogsCheck(ogs_spf_routes(&g, &pt, dBaseUnit_.as<ogs_unit>(), 1, flags(), W_, &out, stream),
           "ogs_spf_routes(base)");
  baseRun_ = true;
  descValid_ = false;  // a new base SPF: its descendant rows are rebuilt
  base_.reset();
}

void LinkFailureSweep::launch(void* stream, bool records) {
  if (exact_) return exactLaunch(stream);  // records are always written
  if (!baseRun_) runBase(stream);
  offsets_.clear();  // results of an earlier launch are stale now
  changed_.clear();
  meta_.clear();
  counts_.clear();
  ogs_graph g = graph();
  ogs_prefix_table pt = table();
  const bool changedOnly = mode_ == kChangedOnly && W_ == 1;
  ogs_spf_out out{};
  if (records) {
    out = ogs_spf_out{dDist_.get(), dNh_.as<uint32_t>(), dMeta_.as<uint32_t>(),
                      dMetric_.get(), dMask_.as<uint32_t>(), dSel_.as<uint32_t>()};
    if (changedOnly) out.dist = out.nh = nullptr;  // records of changed routes only
  }
  ogs_unit_mods mods{dDead_.as<uint32_t>(), kDeadMax};
  // the base's tight-DAG descendant rows: built by the first repair launch
  // after runBase, reused by the next ones (same topology, source, base SPF)
  const size_t Sn = size_t(std::max(hb_.maxNodes, 1));
  if (Sn <= kDescMaxNodes) bDesc_.resize(Sn * ((Sn + 31) / 32) * 4);
  ogs_route_diff diff{bMeta_.as<uint32_t>(), bMetric_.as<uint32_t>(), bMask_.as<uint32_t>(),
                      dChanged_.as<uint32_t>(), dCounts_.as<uint32_t>(),
                      bDist_.as<uint32_t>(), bNh_.as<uint32_t>(), dAdvClass_.as<uint32_t>(),
                      Sn <= kDescMaxNodes ? bDesc_.as<uint32_t>() : nullptr,
                      descValid_ ? 1 : 0};
  uint32_t fl = flags();
  if (mode_ != kFull) fl |= OGS_F_INCREMENTAL;
  if (changedOnly) fl |= OGS_F_CHANGED_ONLY;
  ogsCheck(ogs_spf_routes_variants(&g, &pt, dUnits_.as<ogs_unit>(), int32_t(numVariants()),
                                   &mods, &diff, fl, W_, &out, stream),
           "ogs_spf_routes_variants");
  descValid_ = diff.base_desc_valid != 0;  // set by the library when it wrote the rows
  recordsRun_ = records;
  changedOnlyRun_ = records && changedOnly;
}

void LinkFailureSweep::fetchUpdates(void* stream) {
  if (exact_) return exactFetch(stream);
  if (!recordsRun_) {
    throw std::logic_error("LinkFailureSweep::fetchUpdates: launch(records=true) first");
  }
  const size_t U = numVariants();
  counts_.resize(U * 2);
  if (U) dCounts_.download(counts_.data(), U * 2, stream);
  ogsCheck(ogs_stream_sync(stream), "ogs_stream_sync");
  offsets_.assign(U + 1, 0);
  uint64_t total = 0;
  for (size_t v = 0; v < U; ++v) {
    offsets_[v] = uint32_t(total);
    total += uint64_t(counts_[2 * v]) + counts_[2 * v + 1];
    if (total > 0xFFFFFFFFull) throw std::length_error("LinkFailureSweep: > 2^32 changes");
  }
  offsets_[U] = uint32_t(total);
  const size_t T = std::max<size_t>(total, 1);
  dOffsets_.upload(offsets_.data(), offsets_.size(), stream);
  cPrefix_.resize(T * 4);
  cMeta_.resize(T * 4);
  cMetric_.resize(T * 4);
  cMask_.resize(T * W_ * 4);
  ogs_spf_out rec{nullptr, nullptr, dMeta_.as<uint32_t>(), dMetric_.get(),
                  dMask_.as<uint32_t>(), nullptr};
  ogs_route_changes ch{dOffsets_.as<uint32_t>(), size_t(total), cPrefix_.as<uint32_t>(),
                       cMeta_.as<uint32_t>(), cMetric_.as<uint32_t>(),
                       cMask_.as<uint32_t>()};
  ogsCheck(ogs_route_changes_gather(dChanged_.as<uint32_t>(), int32_t(U), int32_t(Sp_), &rec,
                                    W_, &ch, stream),
           "ogs_route_changes_gather");
  cPrefixH_.resize(total);
  cMetaH_.resize(total);
  cMetricH_.resize(total);
  cMaskH_.resize(total * W_);
  if (total) {
    cPrefix_.download(cPrefixH_.data(), total, stream);
    cMeta_.download(cMetaH_.data(), total, stream);
    cMetric_.download(cMetricH_.data(), total, stream);
    cMask_.download(cMaskH_.data(), total * W_, stream);
  }
  baseMeta_.resize(Sp_);
  baseMetric_.resize(Sp_);
  baseMask_.resize(W_ * Sp_);
  bMeta_.download(baseMeta_.data(), Sp_, stream);
  bMetric_.download(baseMetric_.data(), Sp_, stream);
  bMask_.download(baseMask_.data(), W_ * Sp_, stream);
  ogsCheck(ogs_stream_sync(stream), "ogs_stream_sync");
  base_.reset();
}

void LinkFailureSweep::fetchRecords(void* stream) {
  if (exact_) return exactFetch(stream);
  // the diff (bitmap + counts) always; the records when the launch wrote them
  const size_t U = numVariants();
  const size_t R = (recordsRun_ && !changedOnlyRun_) ? U : 0;
  counts_.resize(U * 2);
  changed_.resize(U * words_);
  meta_.resize(R * Sp_);
  metric_.resize(R * Sp_);
  mask_.resize(R * W_ * Sp_);
  if (U) {
    dCounts_.download(counts_.data(), U * 2, stream);
    dChanged_.download(changed_.data(), U * words_, stream);
  }
  if (R) {
    dMeta_.download(meta_.data(), U * Sp_, stream);
    dMetric_.download(metric_.data(), U * Sp_, stream);
    dMask_.download(mask_.data(), U * W_ * Sp_, stream);
  }
  baseMeta_.resize(Sp_);
  baseMetric_.resize(Sp_);
  baseMask_.resize(W_ * Sp_);
  bMeta_.download(baseMeta_.data(), Sp_, stream);
  bMetric_.download(baseMetric_.data(), Sp_, stream);
  bMask_.download(baseMask_.data(), W_ * Sp_, stream);
  ogsCheck(ogs_stream_sync(stream), "ogs_stream_sync");
  base_.reset();
}

const DecisionRouteDb& LinkFailureSweep::baseRouteDb() const {
  if (exact_) {
    if (!base_) throw std::logic_error("LinkFailureSweep: nothing fetched yet");
    return *base_;
  }
  if (baseMeta_.empty()) throw std::logic_error("LinkFailureSweep: nothing fetched yet");
  if (!base_) {
    DecisionRouteDb db;
    const FlatTopology& f = ls_.flat();
    for (uint32_t p = 0; p < uint32_t(table_.prefixes.size()); ++p) {
      auto e = materializeRoute(f, me_, table_, p, baseMeta_[p], baseMetric_[p],
                                &baseMask_[p], Sp_, W_, v4OverV6_, nullptr, OGS_POLICY_NONE, OGS_POLICY_NONE);
      if (e) db.unicastRoutes.emplace(e->prefix, std::move(*e));
    }
    base_ = std::move(db);
  }
  return *base_;
}

namespace {

// SpfSolver.cpp:21-56 for one variant, prefixes in table order
DecisionRouteUpdate updateOf(const FlatTopology& f, uint32_t rb, const std::string& me,
                             const PrefixHostTable& pt, const ChangeRecords& c, size_t v,
                             bool v4OverV6) {
  DecisionRouteUpdate u;
  for (uint32_t i = c.offsets[v]; i < c.offsets[v + 1]; ++i) {
    const uint32_t p = c.prefix[i];
    auto e = materializeRouteAt(f, rb, me, pt, p, c.meta[i], c.metric[i], &c.mask[i], c.total,
                                c.W, v4OverV6, nullptr, OGS_POLICY_NONE, OGS_POLICY_NONE);
    if (e) {
      u.unicastRoutesToUpdate.emplace_hint(u.unicastRoutesToUpdate.end(), e->prefix,
                                           std::move(*e));
    } else {
      u.unicastRoutesToDelete.push_back(pt.prefixes.at(p));
    }
  }
  return u;
}

}  // namespace

std::vector<DecisionRouteUpdate> materializeUpdates(const FlatTopology& f, const std::string& me,
                                                    const PrefixHostTable& pt,
                                                    const ChangeRecords& c, bool v4OverV6,
                                                    int threads) {
  const size_t V = c.variants;
  const uint32_t rb = f.rowPtr[f.id.at(me)];
  std::vector<DecisionRouteUpdate> out(V);
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  constexpr size_t kBlockV = 16;  // variants per work item
  const size_t T = std::min<size_t>(threads > 0 ? size_t(threads) : std::min(16u, hw),
                                    (V + kBlockV - 1) / kBlockV);
  std::atomic<size_t> next{0};
  std::exception_ptr err;
  std::mutex errMu;
  auto work = [&] {
    try {
      for (size_t b; (b = next.fetch_add(kBlockV)) < V;) {
        for (size_t v = b; v < std::min(V, b + kBlockV); ++v) {
          out[v] = updateOf(f, rb, me, pt, c, v, v4OverV6);
        }
      }
    } catch (...) {
      std::lock_guard<std::mutex> lk(errMu);
      if (!err) err = std::current_exception();
    }
  };
  std::vector<std::thread> pool;
  for (size_t t = 1; t < T; ++t) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  if (err) std::rethrow_exception(err);
  return out;
}

ChangeRecords LinkFailureSweep::changeRecords() const {
  ChangeRecords c;
  c.offsets = offsets_.data();
  c.variants = numVariants();
  c.prefix = cPrefixH_.data();
  c.meta = cMetaH_.data();
  c.metric = cMetricH_.data();
  c.mask = cMaskH_.data();
  c.total = cPrefixH_.size();
  c.W = W_;
  return c;
}

DecisionRouteUpdate LinkFailureSweep::routeUpdate(size_t v) const {
  if (v >= numVariants() || offsets_.size() != numVariants() + 1) {
    throw std::out_of_range("LinkFailureSweep::routeUpdate: variant / fetchUpdates");
  }
  if (exact_) return xUpd_.at(v);
  const FlatTopology& f = ls_.flat();
  return updateOf(f, f.rowPtr[f.id.at(me_)], me_, table_, changeRecords(), v, v4OverV6_);
}

std::vector<DecisionRouteUpdate> LinkFailureSweep::routeUpdates(int threads) const {
  const size_t V = numVariants();
  if (offsets_.size() != V + 1) {
    throw std::out_of_range("LinkFailureSweep::routeUpdates: fetchUpdates first");
  }
  if (exact_) return xUpd_;
  return materializeUpdates(ls_.flat(), me_, table_, changeRecords(), v4OverV6_, threads);
}

DecisionRouteDb LinkFailureSweep::routeDb(size_t v) const {
  if (exact_) {
    if (v >= xDb_.size()) throw std::out_of_range("LinkFailureSweep::routeDb: variant / fetch");
    return xDb_[v];
  }
  if (v >= numVariants() || meta_.size() != numVariants() * Sp_) {
    throw std::out_of_range("LinkFailureSweep::routeDb: variant / fetchRecords");
  }
  DecisionRouteDb db;
  const FlatTopology& f = ls_.flat();
  for (uint32_t p = 0; p < uint32_t(table_.prefixes.size()); ++p) {
    auto e = materializeRoute(f, me_, table_, p, meta_[v * Sp_ + p], metric_[v * Sp_ + p],
                              &mask_[v * W_ * Sp_ + p], Sp_, W_, v4OverV6_, nullptr, OGS_POLICY_NONE,
                              OGS_POLICY_NONE);
    if (e) db.unicastRoutes.emplace(e->prefix, std::move(*e));
  }
  return db;
}

std::vector<std::string> LinkFailureSweep::changedPrefixes(size_t v) const {
  if (v >= numVariants()) throw std::out_of_range("LinkFailureSweep: variant");
  std::vector<std::string> out;
  if (exact_) {
    if (v >= xUpd_.size()) throw std::logic_error("LinkFailureSweep: nothing fetched yet");
    for (const auto& [p, _] : xUpd_[v].unicastRoutesToUpdate) out.push_back(p);
    out.insert(out.end(), xUpd_[v].unicastRoutesToDelete.begin(),
               xUpd_[v].unicastRoutesToDelete.end());
  } else if (offsets_.size() == numVariants() + 1) {
    for (uint32_t i = offsets_[v]; i < offsets_[v + 1]; ++i) {
      out.push_back(table_.prefixes.at(cPrefixH_[i]));
    }
  } else if (changed_.size() == numVariants() * words_) {
    for (size_t p = 0; p < table_.prefixes.size(); ++p) {
      if (changed_[v * words_ + p / 32] >> (p % 32) & 1u) out.push_back(table_.prefixes[p]);
    }
  } else {
    throw std::logic_error("LinkFailureSweep: nothing fetched yet");
  }
  std::sort(out.begin(), out.end());
  return out;
}

std::pair<uint32_t, uint32_t> LinkFailureSweep::counts(size_t v) const {
  if (v >= numVariants() || counts_.size() != 2 * numVariants()) {
    throw std::out_of_range("LinkFailureSweep::counts: variant / fetch");
  }
  return {counts_[2 * v], counts_[2 * v + 1]};
}

}  // namespace openr_amd
