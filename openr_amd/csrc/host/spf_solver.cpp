// spf_solver.cpp — SpfSolver::buildRouteDb on the GPU (reference:
// openr/decision/SpfSolver.cpp:139-767). The host flattens PrefixState into
// the C-ABI prefix table, launches the fused SPF+RouteDb kernel for the
// source and materialises the compact route records into RibUnicastEntry /
// RibMplsEntry objects.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>

#include "decision.h"
#include "slot_order.h"

namespace openr_amd {

namespace {
struct PinnedPool {
  std::mutex mu;
  std::multimap<size_t, void*> free;  // capacity -> block
  size_t bytes{0};
  static constexpr size_t kMaxBytes = size_t(256) << 20, kMaxBlock = size_t(64) << 20;
  ~PinnedPool() {
    for (auto& [_, p] : free) ogs_host_free(p);
  }
};
PinnedPool& pinnedPool() {
  static PinnedPool* pool = new PinnedPool;  // outlives static destructors
  return *pool;
}
}  // namespace

void* pinnedAcquire(size_t bytes, size_t* cap) {
  // power-of-two classes from 4 KiB: a recycled block fits the next request
  size_t c = 4096;
  while (c < bytes) c <<= 1;
  PinnedPool& P = pinnedPool();
  {
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.free.lower_bound(c);
    if (it != P.free.end() && it->first <= 4 * c) {
      void* p = it->second;
      *cap = it->first;
      P.bytes -= it->first;
      P.free.erase(it);
      return p;
    }
  }
  void* p = nullptr;
  ogsCheck(ogs_host_alloc(&p, c), "ogs_host_alloc");
  *cap = c;
  return p;
}

void pinnedRelease(void* p, size_t cap) {
  if (!p) return;
  PinnedPool& P = pinnedPool();
  {
    std::lock_guard<std::mutex> g(P.mu);
    if (cap <= PinnedPool::kMaxBlock && P.bytes + cap <= PinnedPool::kMaxBytes) {
      P.free.emplace(cap, p);
      P.bytes += cap;
      return;
    }
  }
  ogs_host_free(p);
}

uint64_t nextVersionStamp() {
  static std::atomic<uint64_t> stamp{0};
  return ++stamp;
}

// ----------------------------------------------------------- PrefixState --
void PrefixState::logChange(const std::string& network) {
  if (!tracking_) return;
  if (changeLog_.size() >= kChangeLogCap) {
    const size_t drop = changeLog_.size() / 2;
    changeLog_.erase(changeLog_.begin(), changeLog_.begin() + drop);
    changeLogBase_ += drop;
  }
  changeLog_.push_back(network);
}

const std::string* PrefixState::updatePrefixInPlace(const std::string& node,
                                                    const std::string& area,
                                                    std::string&& network, PrefixEntry&& entry) {
  // PrefixState.cpp:15-38
  // one lookup: the key moves in only when inserted
  growHashTable(prefixes_);
  auto mapIt = prefixes_.try_emplace(std::move(network)).first;
  auto& entries = mapIt->second;
  auto [it, inserted] = entries.try_emplace(NodeAndArea(node, area));
  if (!inserted && *it->second == entry) return nullptr;
  it->second = std::make_shared<PrefixEntry>(std::move(entry));
  version_ = nextVersionStamp();
  logChange(mapIt->first);
  return &mapIt->first;
}

std::set<std::string> PrefixState::updatePrefixKeyed(const std::string& node,
                                                     const std::string& area,
                                                     const std::string& network,
                                                     PrefixEntry entry) {
  std::set<std::string> changed;
  std::string key = network;
  if (updatePrefixInPlace(node, area, std::move(key), std::move(entry))) changed.insert(network);

  return changed;
}

std::set<std::string> PrefixState::updatePrefix(const std::string& node,
                                                const std::string& area,
                                                const PrefixEntry& entry) {
  return updatePrefixKeyed(node, area, prefixNetworkKey(entry.prefix), entry);
}

std::set<std::string> PrefixState::updatePrefix(const std::string& node,
                                                const std::string& area,
                                                PrefixEntry&& entry) {
  std::string network = prefixNetworkKey(entry.prefix);
  return updatePrefixKeyed(node, area, network, std::move(entry));
}

bool PrefixState::deletePrefixInPlace(const std::string& node, const std::string& area,
                                      const std::string& prefix, std::string* network) {
  // PrefixState.cpp:40-57
  auto it = prefixes_.find(prefixNetworkKey(prefix, /*applyMask=*/false));
  if (it == prefixes_.end() || !it->second.erase(std::make_pair(node, area))) return false;
  if (network) *network = it->first;
  logChange(it->first);
  if (it->second.empty()) prefixes_.erase(it);
  version_ = nextVersionStamp();
  return true;
}

std::set<std::string> PrefixState::deletePrefix(const std::string& node,
                                                const std::string& area,
                                                const std::string& prefix) {
  std::set<std::string> changed;
  std::string network;
  if (deletePrefixInPlace(node, area, prefix, &network)) changed.insert(std::move(network));
  return changed;
}

// ------------------------------------------------------- DecisionRouteDb --
DecisionRouteUpdate DecisionRouteDb::calculateUpdate(
    const DecisionRouteDb& newDb) const {  // SpfSolver.cpp:21-56
  DecisionRouteUpdate d;
  for (const auto& [p, e] : newDb.unicastRoutes) {
    auto it = unicastRoutes.find(p);
    if (it == unicastRoutes.end() || it->second != e) d.unicastRoutesToUpdate[p] = e;
  }
  for (const auto& [p, _] : unicastRoutes) {
    if (!newDb.unicastRoutes.count(p)) d.unicastRoutesToDelete.push_back(p);
  }
  for (const auto& [l, e] : newDb.mplsRoutes) {
    auto it = mplsRoutes.find(l);
    if (it == mplsRoutes.end() || it->second != e) d.mplsRoutesToUpdate[l] = e;
  }
  for (const auto& [l, _] : mplsRoutes) {
    if (!newDb.mplsRoutes.count(l)) d.mplsRoutesToDelete.push_back(l);
  }
  return d;
}

void DecisionRouteDb::update(const DecisionRouteUpdate& u) {
  for (const auto& p : u.unicastRoutesToDelete) unicastRoutes.erase(p);
  for (const auto& [p, e] : u.unicastRoutesToUpdate) unicastRoutes[p] = e;
  for (const auto& l : u.mplsRoutesToDelete) mplsRoutes.erase(l);
  for (const auto& [l, e] : u.mplsRoutesToUpdate) mplsRoutes[l] = e;
}

// ------------------------------------------------------------ HostBatch --
void HostBatch::append(const FlatTopology& t, const PrefixState& ps,
                       const std::string& area) {
  const uint32_t N = uint32_t(t.names.size());
  const uint32_t e0 = rowPtr.back();
  const uint32_t n0 = nodeBase.back(), pb0 = pfxBase.back();
  const uint32_t ab0 = uint32_t(advNode.size());
  for (uint32_t v = 0; v < N; ++v) {
    rowPtr.push_back(e0 + t.rowPtr[v + 1]);
    edgeSrc.insert(edgeSrc.end(), t.rowPtr[v + 1] - t.rowPtr[v], v);
  }
  edges.insert(edges.end(), t.edges.begin(), t.edges.end());
  nodeFlags.insert(nodeFlags.end(), t.nodeFlags.begin(), t.nodeFlags.end());
  nodeBase.push_back(nodeBase.back() + N);
  const auto c = colorNodes(t.rowPtr.data(), t.edges.data(), N);
  color.insert(color.end(), c.begin(), c.end());
  maxNodes = std::max<int>(maxNodes, int(N));
  maxEdges = std::max<int>(maxEdges, int(t.edges.size()));
  maxDegree = std::max(maxDegree, t.maxDegree);
  maxMetric = std::max(maxMetric, t.maxMetric);
  hasZeroMetric |= t.hasZeroMetric;
  const size_t a0 = advNode.size();
  const uint32_t np = appendPrefixes(t, ps, area);
  topoDesc.insert(topoDesc.end(),
                  {n0, N, e0, uint32_t(t.edges.size()), pb0, np, ab0,
                   uint32_t(advNode.size() - a0)});
}

uint32_t HostBatch::appendPrefixes(const FlatTopology& t, const PrefixState& ps,
                                   const std::string& area) {
  uint32_t np = 0;
  const size_t a0 = advNode.size();
  for (const auto& [prefix, entries] : ps.prefixes()) {
    bool anyMinNh = false;
    for (const auto& [na, e] : entries) {
      if (na.second != area) {
        throw std::out_of_range("prefix advertised in unknown area " + na.second);
      }
      auto it = t.id.find(na.first);
      advNode.push_back(it == t.id.end() ? OGS_NODE_NONE : it->second);
      advMetrics.insert(advMetrics.end(),
                        {e->metrics.drain_metric, e->metrics.path_preference,
                         e->metrics.source_preference, e->metrics.distance});
      advMinNh.push_back(e->minNexthop ? *e->minNexthop : INT64_MIN);
      anyMinNh |= e->minNexthop.has_value();
    }
    advOff.push_back(uint32_t(advNode.size()));
    pfxFlags.push_back((isV4Prefix(prefix) ? OGS_PFX_V4 : 0u) |
                       (anyMinNh ? OGS_PFX_HAS_MIN_NH : 0u));
    ++np;
  }
  pfxBase.push_back(pfxBase.back() + np);
  maxPrefixes = std::max<int>(maxPrefixes, int(np));
  maxAdvs = std::max<int>(maxAdvs, int(advNode.size() - a0));
  return np;
}

int HostBatch::slotOrder(std::vector<uint16_t>& out,
                         std::vector<uint32_t>* edgesOut,
                         int* degreeOut) const {
  const int stride = slotStrideFor(maxNodes);
  const int degree = slotDegreeFor(maxDegree, maxMetric, stride);
  out.clear();
  if (edgesOut) edgesOut->clear();
  if (degreeOut) *degreeOut = edgesOut ? degree : 0;
  if (!stride) return 0;
  const size_t T = nodeBase.size() - 1;
  out.resize(T * stride);
  if (edgesOut && degree) edgesOut->resize(T * size_t(degree) * stride);
  for (size_t t = 0; t < T; ++t) {
    const std::vector<uint8_t> c(color.begin() + nodeBase[t],
                                 color.begin() + nodeBase[t + 1]);
    placeSlots(c, stride, &out[t * stride]);
    if (edgesOut && degree) {
      placeSlotEdges(&out[t * stride], stride, &rowPtr[nodeBase[t]],
                     edges.data(), nodeBase[t + 1] - nodeBase[t], degree,
                     &(*edgesOut)[t * size_t(degree) * stride]);
    }
  }
  return stride;
}

// ------------------------------------------------------------- SpfSolver --
// device tables of a RibPolicy compiled for one source (runPolicyOnDevice):
// one ogs_rib_policy per chunk of <= 32 statements (statement_base = 32c)
struct PolicyDevice {
  struct Chunk {
    DeviceBuffer pfxMatch, tagMatch, nonzero;
    ogs_rib_policy rp{};
  };
  std::vector<Chunk> chunks;
  DeviceBuffer applied, counter;
  // what the matcher tables were compiled for (recompiled on change)
  struct Key {
    uint64_t policy{0}, tableGen{0};
    const PrefixHostTable* table{nullptr};
    std::vector<std::tuple<const FlatTopology*, uint64_t, uint32_t>> src;
    int W{0};
    std::string me;
    bool operator==(const Key& o) const {
      return policy == o.policy && tableGen == o.tableGen && table == o.table &&
          src == o.src && W == o.W && me == o.me;
    }
  } key;
};

// Byte layout of a single-topology prefix table packed into one block (one
// H2D), and of one unit's result records (one D2H): 256-byte aligned spans.
inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

struct TableImage {
  size_t desc{0}, pfxBase{0}, advOff{0}, advNode{0}, advMetrics{0}, advMinNh{0},
      pfxFlags{0}, end{0};
  uint32_t P{0}, A{0};
  // packs hb (one topology, appendPrefixes) + its topoDesc into `h`
  void pack(const HostBatch& hb, const uint32_t desc8[8], PinnedBuffer& h) {
    P = uint32_t(hb.pfxFlags.size());
    A = uint32_t(hb.advNode.size());
    desc = 0;
    pfxBase = al256(desc + 8 * 4);
    advOff = al256(pfxBase + 2 * 4);
    advNode = al256(advOff + (P + 1) * 4);
    advMetrics = al256(advNode + std::max<size_t>(A, 1) * 4);
    advMinNh = al256(advMetrics + std::max<size_t>(A, 1) * 16);
    pfxFlags = al256(advMinNh + std::max<size_t>(A, 1) * 8);
    end = al256(pfxFlags + std::max<size_t>(P, 1));
    h.resize(end);
    std::memcpy(h.at<uint32_t>(desc), desc8, 8 * 4);
    std::memcpy(h.at<uint32_t>(pfxBase), hb.pfxBase.data(), 2 * 4);
    std::memcpy(h.at<uint32_t>(advOff), hb.advOff.data(), (P + 1) * 4);
    std::memcpy(h.at<uint32_t>(advNode), hb.advNode.data(), A * 4);
    std::memcpy(h.at<int32_t>(advMetrics), hb.advMetrics.data(), A * 16);
    std::memcpy(h.at<int64_t>(advMinNh), hb.advMinNh.data(), A * 8);
    std::memcpy(h.at<uint8_t>(pfxFlags), hb.pfxFlags.data(), P);
  }
  ogs_prefix_table view(const DeviceBuffer& d) const {
    ogs_prefix_table pt{};
    pt.max_prefixes = int32_t(P);
    pt.max_advertisements = int32_t(A);
    pt.pfx_base = devAt<uint32_t>(d, pfxBase);
    pt.adv_off = devAt<uint32_t>(d, advOff);
    pt.adv_node = devAt<uint32_t>(d, advNode);
    pt.adv_metrics = devAt<int32_t>(d, advMetrics);
    pt.adv_min_nh = devAt<int64_t>(d, advMinNh);
    pt.pfx_flags = devAt<uint8_t>(d, pfxFlags);
    return pt;
  }
};

// dist [N] | nh [W][N] | reach [ceil(N/32)] (exact-order settled bitset) |
// meta [P] | metric [P] | mask [W][P] | sel [P]  (the SPF spans depend on N
// and W only: the memo's layout is the same with or without a table)
struct ResultImage {
  size_t dist{0}, nh{0}, reach{0}, meta{0}, metric{0}, mask{0}, sel{0}, end{0};
  ResultImage() = default;
  ResultImage(uint32_t N, uint32_t P, int W, size_t db) {
    const size_t P1 = std::max<uint32_t>(P, 1);
    nh = al256(size_t(N) * db);
    reach = nh + al256(size_t(N) * W * 4);
    meta = reach + al256((size_t(N) + 31) / 32 * 4 + 4);
    metric = meta + al256(P1 * 4);
    mask = metric + al256(P1 * db);
    sel = mask + al256(P1 * W * 4);
    end = sel + al256(P1 * 4);
  }
};

struct SpfSolver::Impl {
  // ---- single-area buildRouteDb ----
  // prefix table of (cachedPs, cachedTopo), packed: one H2D per change
  DeviceBuffer tab;
  PinnedBuffer hTab;
  TableImage tabImg;
  const PrefixState* cachedPs{nullptr};
  uint64_t cachedPsVersion{~0ull}, cachedTopoVersion{~0ull};
  const FlatTopology* cachedTopo{nullptr};
  PrefixHostTable table;
  // the unit (uploaded when the source changes) and the result block: one
  // D2H per build (the SPF part only when node-label routes need it)
  DeviceBuffer unit, res;
  PinnedBuffer hRes;
  uint32_t unitSrc{~0u};
  // createRoutesForPrefixes: the changed prefixes' sub-table and records
  DeviceBuffer subTab, subRes, spfDesc;
  PinnedBuffer hSubTab, hSubRes;
  PrefixHostTable subTable;
  PolicyDevice policy;

  // multi-area domain (buildRouteDbMultiArea): the areas' CSR as one graph
  // batch + the domain prefix table with per-entry area / node-name ids
  struct MultiArea {
    std::vector<std::pair<const FlatTopology*, uint64_t>> topoKey;
    const PrefixState* ps{nullptr};
    uint64_t psVersion{~0ull};
    std::vector<std::string> areas;  // area index -> name (map order)
    std::vector<const FlatTopology*> flats;
    HostBatch hb;
    std::unordered_map<std::string, uint32_t> nameId;
    uint32_t maxPrefixes{0}, numNames{0};
    PrefixHostTable table;
    DeviceBuffer nodeBase, rowPtr, edges, flags, edgeSrc, desc;
    DeviceBuffer pfxBase, advOff, advNode, advMetrics, advMinNh, pfxFlags,
        advArea, advName, nameLocal;
    DeviceBuffer units, srcName, spfRow, dist, nh, meta, metric, mask, sel, reach;
    bool exact{false}, wide{false};  // domain needs OGS_F_EXACT_ORDER / u64
  } ma;
  // shape of the last enqueueRouteDb (collectRouteDb downloads its results)
  std::optional<MultiAreaResult> enqueued;
  std::string enqueuedMe;
};

SpfSolver::SpfSolver(const std::string& me, bool enableV4, bool sr, bool brs,
                     bool v4OverV6)
    : impl_(std::make_unique<Impl>()),
      myNodeName_(me),
      enableV4_(enableV4),
      enableNodeSegmentLabel_(sr),
      enableBestRouteSelection_(brs),
      v4OverV6Nexthop_(v4OverV6) {}
SpfSolver::~SpfSolver() = default;

void SpfSolver::updateStaticUnicastRoutes(
    const std::map<std::string, RibUnicastEntry>& toUpdate,
    const std::vector<std::string>& toDelete) {  // SpfSolver.cpp:109-137
  for (const auto& [p, e] : toUpdate) staticUnicastRoutes_[p] = e;
  for (const auto& p : toDelete) staticUnicastRoutes_.erase(p);
}

namespace {

const LinkState& singleArea(const AreaLinkStates& als, std::string& area) {
  if (als.size() != 1) {
    throw std::domain_error(
        "SpfSolver: multi-area route computation is not on the GPU path yet");
  }
  area = als.begin()->first;
  return als.begin()->second;
}

NextHopThrift makeNh(const Link& l, const std::string& me, bool useV4,
                     int32_t metric, std::optional<MplsAction> act) {
  NextHopThrift nh;  // createNextHop (LsdbUtil.cpp:600-618)
  nh.address = useV4 ? l.getNhV4FromNode(me) : l.getNhV6FromNode(me);
  nh.ifName = l.getIfaceFromNode(me);
  nh.metric = metric;
  nh.mplsAction = std::move(act);
  nh.area = l.getArea();
  nh.neighborNodeName = l.getOtherNodeName(me);
  nh.weight = 0;
  return nh;
}

// RibPolicy compiled on the host against the prefix table and the source's
// links (per area) -- cached until the policy, table or topology changes --
// and applied on the device (ogs_rib_policy_apply): next hops of weight 0
// dropped in the device masks, statement choices left in D.applied /
// D.counter (downloadPolicy).
void runPolicyOnDevice(const RibPolicy& pol, const PrefixHostTable& table,
                       const ogs_prefix_table& pt,
                       const std::vector<std::pair<const FlatTopology*, uint32_t>>& src,
                       const std::string& me, int W, uint32_t* dMeta, uint32_t* dMask,
                       PolicyDevice& D, void* stream) {
  const size_t K = pol.numStatements();
  // applied / counter are u16 statement indexes with OGS_POLICY_NONE = none
  // (RibPolicy.cpp:231-249 walks any number of statements)
  if (K >= OGS_POLICY_NONE) throw std::domain_error("RibPolicy: more than 65,534 statements");
  const size_t P = table.prefixes.size(), A = src.size();
  PolicyDevice::Key key{pol.uid(), table.generation, &table, {}, W, me};
  for (const auto& [f, s] : src) key.src.emplace_back(f, f->version, s);
  if (!(key == D.key)) {
    D.chunks.clear();
    D.chunks.resize((K + 31) / 32);
    // source link slots' next hops (weight 0, v6 form: the weight rules
    // read only the area and the neighbour name, RibPolicy.cpp:122-137)
    std::vector<std::vector<NextHopThrift>> slots(A);
    for (size_t a = 0; a < A; ++a) {
      const FlatTopology* f = src[a].first;
      const uint32_t s = src[a].second;
      if (s == OGS_NODE_NONE) continue;
      const uint32_t rb = f->rowPtr[s], deg = f->rowPtr[s + 1] - rb;
      for (uint32_t j = 0; j < deg && j < 32u * uint32_t(W); ++j) {
        slots[a].push_back(makeNh(*f->edgeLink[rb + j], me, false, 0, std::nullopt));
      }
    }
    for (size_t c = 0; c < D.chunks.size(); ++c) {
      const size_t k0 = 32 * c, kn = std::min<size_t>(32, K - k0);
      std::vector<uint32_t> pm(std::max<size_t>(P, 1), 0),
          tm(std::max<size_t>(table.advEntry.size(), 1), 0);
      std::vector<uint32_t> nz(std::max<size_t>(kn * A * W, 1), 0);
      uint32_t active = 0;
      for (size_t k = 0; k < kn; ++k) {
        if (pol.hasMatcher(k0 + k)) active |= 1u << k;
      }
      for (size_t p = 0; p < P; ++p) {
        for (size_t k = 0; k < kn; ++k) {
          if (pol.matchesPrefix(k0 + k, table.prefixes[p])) pm[p] |= 1u << k;
        }
      }
      for (size_t a = 0; a < table.advEntry.size(); ++a) {
        for (size_t k = 0; k < kn; ++k) {
          if (pol.matchesTags(k0 + k, table.advEntry[a]->tags)) tm[a] |= 1u << k;
        }
      }
      for (size_t a = 0; a < A; ++a) {
        for (size_t j = 0; j < slots[a].size(); ++j) {
          for (size_t k = 0; k < kn; ++k) {
            if (pol.weightOf(k0 + k, slots[a][j]) > 0) {
              nz[(k * A + a) * W + j / 32] |= 1u << (j % 32);
            }
          }
        }
      }
      PolicyDevice::Chunk& C = D.chunks[c];
      C.pfxMatch.upload(pm.data(), pm.size(), stream);
      C.tagMatch.upload(tm.data(), tm.size(), stream);
      C.nonzero.upload(nz.data(), nz.size(), stream);
      C.rp = ogs_rib_policy{int32_t(kn), active, C.pfxMatch.as<uint32_t>(),
                            C.tagMatch.as<uint32_t>(), C.nonzero.as<uint32_t>(),
                            int32_t(k0)};
    }
    D.applied.resize(2 * std::max<size_t>(P, 1));
    D.counter.resize(2 * std::max<size_t>(P, 1));
    D.key = std::move(key);
  }
  // chunks in statement order; a later chunk continues the routes no
  // earlier statement transformed (first transforming statement wins,
  // RibPolicy.cpp:222-229)
  for (const auto& C : D.chunks) {
    ogsCheck(ogs_rib_policy_apply(&pt, &C.rp, int32_t(A), 1, W, dMeta, dMask,
                                  D.applied.as<uint16_t>(), D.counter.as<uint16_t>(), stream),
             "ogs_rib_policy_apply");
  }
}

void downloadPolicy(const PolicyDevice& D, size_t P, std::vector<uint16_t>& applied,
                    std::vector<uint16_t>& counter) {
  applied.assign(P, OGS_POLICY_NONE);
  counter.assign(P, OGS_POLICY_NONE);
  if (P) {
    D.applied.download(applied.data(), P);
    D.counter.download(counter.data(), P);
  }
}

// Route-level effect of the device policy: counterID of the last matching
// statement, weights of the applied one (RibPolicy.cpp:115-160).
void finishPolicy(const RibPolicy* pol, uint16_t applied, uint16_t counter,
                  RibUnicastEntry& e) {
  if (!pol) return;
  if (counter != OGS_POLICY_NONE) e.counterID = pol->counterIDOf(counter);
  if (applied == OGS_POLICY_NONE) return;
  NextHops w;
  for (NextHopThrift nh : e.nexthops) {
    nh.weight = pol->weightOf(applied, nh);
    w.insert(std::move(nh));
  }
  e.nexthops = std::move(w);
}

}  // namespace

// decision.no_route_to_prefix (SpfSolver.cpp:221 no reachable advertiser,
// :242 empty selection, :579 no next hop): the records whose reason code is
// one of those
static bool noRouteReason(uint32_t meta) {
  if (meta & OGS_ROUTE_VALID) return false;
  const uint32_t r = (meta >> OGS_ROUTE_REASON_SHIFT) & 0xFu;
  return r == OGS_REASON_UNREACHABLE || r == OGS_REASON_NO_NEXTHOP;
}

bool wideDistancesNeeded(const FlatTopology& f) {
  const uint64_t n = f.names.empty() ? 0 : f.names.size() - 1;
  // 32-bit kernels cap "unreachable" at 2^31 - 1 inside their loops
  return f.maxMetric != 0 && n != 0 && f.maxMetric > 0x7FFFFFFEull / n;
}

void PrefixHostTable::build(const PrefixState& ps) {
  ++generation;
  prefixes.clear();
  advEntry.clear();
  advKey.clear();
  advOff.assign(1, 0);
  for (const auto& [prefix, entries] : ps.prefixes()) {
    prefixes.push_back(prefix);
    for (const auto& [na, e] : entries) {
      advEntry.push_back(e.get());
      advKey.push_back(na);
    }
    advOff.push_back(uint32_t(advEntry.size()));
  }
}

const std::vector<uint32_t>& PrefixHostTable::sortedOrder() const {
  std::lock_guard<std::mutex> lock(sortedMutex_);
  if (sortedGen_ != generation || sorted_.size() != prefixes.size()) {
    sorted_.resize(prefixes.size());
    for (uint32_t i = 0; i < uint32_t(prefixes.size()); ++i) sorted_[i] = i;
    std::sort(sorted_.begin(), sorted_.end(),
              [&](uint32_t a, uint32_t b) { return prefixes[a] < prefixes[b]; });
    sortedGen_ = generation;
  }
  return sorted_;
}

// One prefix's route from the unit's compact records (RibUnicastEntry of
// createRouteForPrefix, SpfSolver.cpp:160-311 + addBestPaths 595-639).
// `meta`, `metric` and the link-slot mask words (word w at mask[w * stride])
// are the record of prefix p; nullopt when the record holds no route.
std::optional<RibUnicastEntry> materializeRoute(
    const FlatTopology& f, const std::string& me, const PrefixHostTable& pt,
    uint32_t p, uint32_t meta, uint64_t metric, const uint32_t* mask,
    size_t maskStride, int W, bool v4OverV6Nexthop, const RibPolicy* policy,
    uint16_t applied, uint16_t counter) {
  if (!(meta & OGS_ROUTE_VALID)) return std::nullopt;
  return materializeRouteAt(f, f.rowPtr[f.id.at(me)], me, pt, p, meta, metric, mask,
                            maskStride, W, v4OverV6Nexthop, policy, applied, counter);
}

std::optional<RibUnicastEntry> materializeRouteAt(
    const FlatTopology& f, uint32_t rb, const std::string& me, const PrefixHostTable& pt,
    uint32_t p, uint32_t meta, uint64_t metric, const uint32_t* mask,
    size_t maskStride, int W, bool v4OverV6Nexthop, const RibPolicy* policy,
    uint16_t applied, uint16_t counter) {
  if (!(meta & OGS_ROUTE_VALID)) return std::nullopt;
  const uint32_t best = pt.advOff[p] + (meta >> OGS_ROUTE_BEST_SHIFT);
  RibUnicastEntry e;
  e.prefix = pt.prefixes[p];
  const bool useV4 = isV4Prefix(e.prefix) && !v4OverV6Nexthop;
  const int32_t m32 = static_cast<int32_t>(metric);
  for (int w = 0; w < W; ++w) {
    uint32_t bits = mask[w * maskStride];
    while (bits) {
      const int b = __builtin_ctz(bits);
      bits &= bits - 1;
      e.nexthops.insert(makeNh(*f.edgeLink[rb + w * 32 + b], me, useV4, m32, std::nullopt));
    }
  }
  e.bestPrefixEntry = *pt.advEntry[best];
  if (meta & OGS_ROUTE_DRAINED) e.bestPrefixEntry.metrics.drain_metric = 1;
  e.bestPrefixEntry.weight = std::nullopt;  // RibEntry.h:77
  e.bestArea = pt.advKey[best].second;
  e.igpCost = static_cast<unsigned int>(metric);
  e.localRouteConsidered = meta & OGS_ROUTE_LOCAL;
  if (policy) finishPolicy(policy, applied, counter, e);
  return e;
}

int g_materializeThreads = 0;

DecisionRouteDb materializeRouteDb(
    const LinkState& ls, const FlatTopology& f, const std::string& area,
    const std::string& me, const UnitView& r, const PrefixHostTable& pt,
    bool v4OverV6Nexthop, bool enableNodeSegmentLabel,
    const std::map<std::string, RibUnicastEntry>& statics,
    std::map<std::string, RouteSelectionResult>* bestRoutesCache) {
  DecisionRouteDb rdb;
  // SpfSolver.cpp:98 clears the cache per build; the single-threaded build
  // refills it from the previous build's nodes (keys and selection sets
  // reassigned in place) instead of freeing and allocating ~20k of them
  std::map<std::string, RouteSelectionResult> spare;
  if (bestRoutesCache) spare.swap(*bestRoutesCache);
  const auto meIt = f.id.find(me);
  const uint32_t rb = meIt == f.id.end() ? 0u : f.rowPtr[meIt->second];
  // sorted positions [i0, i1) into `routes` / `sel`: walked in prefix order
  // (the table follows the hashed PrefixState), so appending at the end is
  // the map's hint
  const std::vector<uint32_t>& sorted = pt.sortedOrder();
  std::atomic<uint64_t> noRoute{0};  // decision.no_route_to_prefix (SpfSolver.cpp:221, 242)
  bool recycle = false;  // spare nodes are reused by the single-threaded build only
  auto build = [&](uint32_t i0, uint32_t i1, std::map<std::string, RibUnicastEntry>& routes,
                   std::map<std::string, RouteSelectionResult>* cache) {
    uint64_t unreachable = 0;
    for (uint32_t i = i0; i < i1; ++i) {
      const uint32_t p = sorted[i];
      const uint32_t meta = r.meta[p];
      unreachable += noRouteReason(meta);
      if (cache && (meta & OGS_ROUTE_SELECTED)) {  // SpfSolver.cpp:247
        const uint32_t a0 = pt.advOff[p];
        const uint32_t a1 = pt.advOff[p + 1];
        if (recycle && !spare.empty()) {
          auto nh = spare.extract(spare.begin());
          nh.key() = pt.prefixes[p];
          RouteSelectionResult& sel = nh.mapped();
          auto& areas = sel.allNodeAreas;
          decltype(areas.extract(areas.begin())) keep;
          if (!areas.empty()) keep = areas.extract(areas.begin());
          areas.clear();
          for (uint32_t a = a0; a < std::min(a1, a0 + 32); ++a) {
            if (!(r.sel[p] >> (a - a0) & 1u)) continue;
            if (keep) {
              keep.value() = pt.advKey[a];
              areas.insert(areas.end(), std::move(keep));
            } else {
              areas.insert(pt.advKey[a]);
            }
          }
          sel.bestNodeArea = pt.advKey[a0 + (meta >> OGS_ROUTE_BEST_SHIFT)];
          sel.isBestNodeDrained = meta & OGS_ROUTE_DRAINED;
          cache->insert(cache->end(), std::move(nh));
        } else {
          RouteSelectionResult sel;
          for (uint32_t a = a0; a < std::min(a1, a0 + 32); ++a) {
            if (r.sel[p] >> (a - a0) & 1u) sel.allNodeAreas.insert(pt.advKey[a]);
          }
          sel.bestNodeArea = pt.advKey[a0 + (meta >> OGS_ROUTE_BEST_SHIFT)];
          sel.isBestNodeDrained = meta & OGS_ROUTE_DRAINED;
          cache->insert_or_assign(cache->end(), pt.prefixes[p], std::move(sel));
        }
      }
      if (!(meta & OGS_ROUTE_VALID)) continue;
      auto e = materializeRouteAt(f, rb, me, pt, p, meta, r.metric[p], &r.mask[p],
                                  r.maskStride, r.W, v4OverV6Nexthop, r.policy,
                                  r.policy ? r.applied[p] : OGS_POLICY_NONE,
                                  r.policy ? r.counter[p] : OGS_POLICY_NONE);
      if (e) routes.emplace_hint(routes.end(), e->prefix, std::move(*e));
    }
    noRoute += unreachable;
  };
  // With g_materializeThreads > 1 the prefixes are built in chunks on host
  // threads into per-chunk maps whose nodes are then spliced, in order, into
  // the result (no copies). Off by default: on the GPU box's 16-core share
  // the G1 warm build (20k routes) took 34 ms with 5 threads against 21 ms
  // on one (the routes are freed later on the caller's thread, across the
  // workers' malloc arenas).
  const size_t T = g_materializeThreads > 0 ? size_t(g_materializeThreads) : 1;
  recycle = T <= 1;
  if (T <= 1) {
    build(0, r.P, rdb.unicastRoutes, bestRoutesCache);
  } else {
    std::vector<std::map<std::string, RibUnicastEntry>> routes(T);
    std::vector<std::map<std::string, RouteSelectionResult>> sels(T);
    std::vector<std::exception_ptr> errs(T);
    auto part = [&](size_t t) {
      try {
        build(uint32_t(r.P * t / T), uint32_t(r.P * (t + 1) / T), routes[t],
              bestRoutesCache ? &sels[t] : nullptr);
      } catch (...) {
        errs[t] = std::current_exception();
      }
    };
    std::vector<std::thread> pool;
    for (size_t t = 1; t < T; ++t) pool.emplace_back(part, t);
    part(0);
    for (auto& th : pool) th.join();
    for (auto& e : errs) {
      if (e) std::rethrow_exception(e);
    }
    for (size_t t = 0; t < T; ++t) {
      while (!routes[t].empty()) {
        rdb.unicastRoutes.insert(rdb.unicastRoutes.end(), routes[t].extract(routes[t].begin()));
      }
      if (bestRoutesCache) {
        while (!sels[t].empty()) {
          bestRoutesCache->insert(bestRoutesCache->end(), sels[t].extract(sels[t].begin()));
        }
      }
    }
  }
  if (noRoute) addStatValue("decision.no_route_to_prefix", double(noRoute), StatType::COUNT);
  for (const auto& [prefix, e] : statics) {  // SpfSolver.cpp:343-349
    if (rdb.unicastRoutes.count(prefix)) continue;
    auto it = rdb.unicastRoutes.emplace(prefix, e).first;
    if (r.policy) r.policy->applyAction(it->second);  // policy covers statics too
  }

  // node-label MPLS routes from the SPF result (SpfSolver.cpp:354-445)
  if (enableNodeSegmentLabel) {
    LabelRoutes labelToNode;
    addNodeLabelRoutes(ls, f, area, me, r.dist, r.nh, r.nhStride, r.W,
                       labelToNode, r.reach);
    for (auto& [label, ne] : labelToNode) {
      rdb.mplsRoutes.emplace(label, std::move(ne.second));
    }
  }
  return rdb;
}

void addNodeLabelRoutes(const LinkState& ls, const FlatTopology& f,
                        const std::string& area, const std::string& me,
                        const uint64_t* dist, const uint32_t* nhWords,
                        size_t nhStride, int W, LabelRoutes& labelToNode,
                        const uint32_t* reach) {
  // SpfSolver.cpp:357-437, one area; dist == nullptr: the source has no
  // SPF in this area (no adjacency database), every other owner unreachable
  const auto sIt = f.id.find(me);
  for (const auto& [node, adjDb] : ls.getAdjacencyDatabases()) {
    const int32_t label = adjDb.nodeLabel;
    const bool valid =
        (static_cast<uint32_t>(label) & 0xfff00000u) == 0 && label != 0;
    if (!valid) continue;
    auto it = labelToNode.find(label);
    if (it != labelToNode.end() && it->second.first < node) continue;
    if (node == me) {
      NextHopThrift nh;
      nh.address = "::";
      nh.area = area;
      nh.mplsAction = MplsAction{POP_AND_LOOKUP, std::nullopt, std::nullopt};
      labelToNode.erase(label);
      labelToNode.emplace(label, std::make_pair(me, RibMplsEntry{label, {nh}}));
      continue;
    }
    if (!dist || sIt == f.id.end()) continue;
    const uint32_t v = f.id.at(node);
    if (reach ? !bitAt(reach, v) : dist[v] == ~0ull) continue;  // no route to the owner
    RibMplsEntry entry{label, {}};
    const int32_t m32 = static_cast<int32_t>(dist[v]);
    const uint32_t rb = f.rowPtr[sIt->second];
    for (int w = 0; w < W; ++w) {
      uint32_t bits = nhWords[w * nhStride + v];
      while (bits) {
        const int b = __builtin_ctz(bits);
        bits &= bits - 1;
        const Link& l = *f.edgeLink[rb + w * 32 + b];
        const bool php = l.getOtherNodeName(me) == node;
        entry.nexthops.insert(makeNh(
            l, me, false, m32,
            php ? MplsAction{PHP, std::nullopt, std::nullopt}
                : MplsAction{SWAP, label, std::nullopt}));
      }
    }
    if (entry.nexthops.empty()) continue;
    labelToNode.erase(label);
    labelToNode.emplace(label, std::make_pair(node, std::move(entry)));
  }
}

namespace {

ogs_graph singleGraph(const FlatTopology& f, const uint32_t* desc) {
  ogs_graph g{};
  g.num_topos = 1;
  g.max_nodes = int32_t(f.names.size());
  g.max_edges = int32_t(f.edges.size());
  g.max_degree = f.maxDegree;
  g.topo_desc = desc;
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

// host widening of a u32 / u64 record span (all-ones = unreachable)
void widenSpan(const void* src, size_t n, bool wide, std::vector<uint64_t>& v) {
  v.resize(n);
  if (wide) {
    std::memcpy(v.data(), src, n * 8);
    return;
  }
  const uint32_t* t = static_cast<const uint32_t*>(src);
  for (size_t i = 0; i < n; ++i) v[i] = t[i] == 0xFFFFFFFFu ? ~0ull : t[i];
}

}  // namespace

void SpfSolver::prepareSingleArea(const FlatTopology& f, const PrefixState& ps,
                                  const std::string& area) {
  Impl& I = *impl_;
  // prefix table (cached on PrefixState / topology version): one packed H2D
  if (I.cachedPs == &ps && I.cachedPsVersion == ps.version() && I.cachedTopo == &f &&
      I.cachedTopoVersion == f.version) {
    return;
  }
  HostBatch hb;
  const uint32_t np = hb.appendPrefixes(f, ps, area);
  const uint32_t desc[8] = {0, uint32_t(f.names.size()), 0, uint32_t(f.edges.size()),
                            0, np, 0, uint32_t(hb.advNode.size())};
  I.table.build(ps);
  I.tabImg.pack(hb, desc, I.hTab);
  I.tab.resize(I.tabImg.end);
  ogsCheck(ogs_memcpy_h2d(I.tab.get(), I.hTab.get(), I.tabImg.end, nullptr), "ogs_memcpy_h2d");
  I.cachedPs = &ps;
  I.cachedPsVersion = ps.version();
  I.cachedTopo = &f;
  I.cachedTopoVersion = f.version;
}

std::optional<DecisionRouteDb> SpfSolver::buildRouteDb(
    const std::string& me, const AreaLinkStates& als, const PrefixState& ps) {
  bool exists = false;  // SpfSolver.cpp:318-324
  for (const auto& [_, l] : als) exists |= l.hasNode(me);
  if (!exists) return std::nullopt;
  const auto t0 = std::chrono::steady_clock::now();
  if (!quietStats_) {
    addStatValue("decision.route_build_runs", 1, StatType::COUNT);  // SpfSolver.cpp:327
    // SpfSolver.cpp:334-339: one createRouteForPrefix per known prefix
    addStatValue("decision.get_route_for_prefix", double(ps.prefixes().size()),
                 StatType::COUNT);
  }
  auto db = als.size() > 1 ? buildRouteDbMultiArea(me, als, ps)
                           : buildRouteDbSingleArea(me, als, ps);
  // every change so far is in this build: the next incremental loop's
  // batch starts after it
  ps.trackChanges();
  incPs_ = &ps;
  incLogCursor_ = ps.changeLogEnd();
  if (!quietStats_) {
    addStatValue("decision.route_build_ms", msSince(t0), StatType::AVG);  // SpfSolver.cpp:450
  }
  return db;
}

std::optional<DecisionRouteDb> SpfSolver::buildRouteDbSingleArea(
    const std::string& me, const AreaLinkStates& als, const PrefixState& ps) {
  const auto tPrep = std::chrono::steady_clock::now();
  std::string area;
  const LinkState& ls = singleArea(als, area);
  const FlatTopology& f = ls.flatOnDevice();
  // zero / negative link metrics: the reference's extraction order replayed
  // on the device (spf_exact.hip), 64-bit distances
  const bool exact = f.hasZeroMetric || f.hasWideMetric;
  Impl& I = *impl_;
  prepareSingleArea(f, ps, area);
  // flatten / device CSR + prefix table when stale (cached otherwise)
  addStatValue("decision.gpu.prepare_ms", msSince(tPrep), StatType::AVG);
  const auto tLaunch = std::chrono::steady_clock::now();

  // ---- launch the fused kernel for (topology, me) -------------------------
  const uint32_t s = f.id.at(me);
  const uint32_t N = uint32_t(f.names.size());
  const uint32_t P = uint32_t(I.table.prefixes.size());
  const int degree = int(f.rowPtr[s + 1] - f.rowPtr[s]);
  const int W = std::max(1, ogs_nh_words_for_degree(degree));
  const bool wide = exact || wideDistancesNeeded(f);
  const size_t db = wide ? 8 : 4;
  if (I.unitSrc != s) {
    const ogs_unit u{0, s};
    I.unit.upload(&u, 1);
    I.unitSrc = s;
  }
  const ResultImage L(N, P, W, db);
  I.res.resize(L.end);
  I.hRes.resize(L.end);

  const ogs_graph g = singleGraph(f, devAt<uint32_t>(I.tab, I.tabImg.desc));
  const ogs_prefix_table pt = I.tabImg.view(I.tab);
  ogs_spf_out out{};
  out.meta = devAt<uint32_t>(I.res, L.meta);
  out.metric = devAt<void>(I.res, L.metric);
  out.mask = devAt<uint32_t>(I.res, L.mask);
  out.sel = devAt<uint32_t>(I.res, L.sel);
  const uint32_t flags = (enableV4_ ? OGS_F_ENABLE_V4 : 0u) |
      (v4OverV6Nexthop_ ? OGS_F_V4_OVER_V6 : 0u) |
      (enableBestRouteSelection_ ? OGS_F_BEST_ROUTE_SELECTION : 0u) |
      (wide ? OGS_F_WIDE_METRIC : 0u) | (exact ? OGS_F_EXACT_ORDER : 0u);
  // SPF memo (LinkState::getSpfResult, LinkState.cpp:705-715): the
  // LinkState's device rows of this source -> the route pass alone, no SPF
  // relaunch (ogs_routes_from_spf); else ONE fused launch writes the SPF
  // into a new memo slot and the records into res
  LinkState::DeviceSpf* memo = ls.findDeviceSpf(s, true, N, W, db, exact);
  if (memo) {
    if (P) {
      ogsCheck(ogs_routes_from_spf(&g, &pt, I.unit.as<ogs_unit>(), 1, memo->dist(),
                                   memo->nh(), exact ? memo->reach() : nullptr, flags, W, &out,
                                   nullptr),
               "ogs_routes_from_spf");
    }
  } else {
    LinkState::DeviceSpf& slot = ls.newDeviceSpf(s, true, N, W, db, exact);
    out.dist = slot.dist();
    out.nh = slot.nh();
    out.reached = exact ? slot.reach() : nullptr;
    ogsCheck(ogs_spf_routes(&g, P ? &pt : nullptr, I.unit.as<ogs_unit>(), 1,
                            flags, W, &out, nullptr),
             "ogs_spf_routes");
    ls.commitDeviceSpf(slot, me, true);
    memo = &slot;
  }
  const RibPolicy* policy = (ribPolicy_ && ribPolicy_->isActive()) ? ribPolicy_ : nullptr;
  std::vector<uint16_t> applied, counter;
  if (policy && P) {
    runPolicyOnDevice(*policy, I.table, pt, {{&f, s}}, me, W, out.meta, out.mask,
                      I.policy, nullptr);
    downloadPolicy(I.policy, P, applied, counter);
  }
  // ONE D2H of the records (+ the SPF rows when node-label routes read them)
  ogsCheck(ogs_memcpy_d2h(I.hRes.at<char>(L.meta), devAt<char>(I.res, L.meta),
                          L.end - L.meta, nullptr),
           "ogs_memcpy_d2h");
  if (enableNodeSegmentLabel_) {
    ogsCheck(ogs_memcpy_d2h(I.hRes.at<char>(L.dist), memo->dist(), L.nh - L.dist, nullptr),
             "ogs_memcpy_d2h");
    ogsCheck(ogs_memcpy_d2h(I.hRes.at<char>(L.nh), memo->nh(), L.reach - L.nh, nullptr),
             "ogs_memcpy_d2h");
    if (exact) {
      ogsCheck(ogs_memcpy_d2h(I.hRes.at<char>(L.reach), memo->reach(), L.meta - L.reach,
                              nullptr),
               "ogs_memcpy_d2h");
    }
  }
  ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
  addStatValue("decision.gpu.launch_ms", msSince(tLaunch), StatType::AVG);
  const auto tMat = std::chrono::steady_clock::now();

  std::vector<uint64_t> dist, metric;
  if (enableNodeSegmentLabel_) widenSpan(I.hRes.at<void>(L.dist), N, wide, dist);
  widenSpan(I.hRes.at<void>(L.metric), P, wide, metric);
  UnitView view;
  view.W = W;
  view.N = N;
  view.P = P;
  view.dist = enableNodeSegmentLabel_ ? dist.data() : nullptr;
  view.nh = I.hRes.at<uint32_t>(L.nh);
  view.nhStride = N;
  view.meta = I.hRes.at<uint32_t>(L.meta);
  view.metric = metric.data();
  view.mask = I.hRes.at<uint32_t>(L.mask);
  view.maskStride = P;
  view.sel = I.hRes.at<uint32_t>(L.sel);
  view.reach = exact && enableNodeSegmentLabel_ ? I.hRes.at<uint32_t>(L.reach) : nullptr;
  if (policy && P) {
    view.policy = policy;
    view.applied = applied.data();
    view.counter = counter.data();
  }
  auto rdb = materializeRouteDb(ls, f, area, me, view, I.table, v4OverV6Nexthop_,
                                enableNodeSegmentLabel_, staticUnicastRoutes_,
                                &bestRoutesCache_);
  addStatValue("decision.gpu.materialize_ms", msSince(tMat), StatType::AVG);
  return rdb;
}

// The incremental branch's routes (createRoutesForPrefixes) of a single-area
// source: the SPF memo of the last build (SPF-only launch on a miss), the
// changed prefixes' sub-table in one H2D, ogs_routes_from_spf, one D2H.
void SpfSolver::routesFromSpfMemo(const std::string& me, const LinkState& ls,
                                  const std::string& area, const PrefixState& /*ps*/,
                                  const PrefixState& sub,
                                  std::map<std::string, std::optional<RibUnicastEntry>>& out) {
  Impl& I = *impl_;
  const auto tIn = std::chrono::steady_clock::now();
  const FlatTopology& f = ls.flatOnDevice();
  const bool exact = f.hasZeroMetric || f.hasWideMetric;
  const uint32_t s = f.id.at(me);
  const uint32_t N = uint32_t(f.names.size());
  const int degree = int(f.rowPtr[s + 1] - f.rowPtr[s]);
  const int W = std::max(1, ogs_nh_words_for_degree(degree));
  const bool wide = exact || wideDistancesNeeded(f);
  const size_t db = wide ? 8 : 4;
  const uint32_t flags = (enableV4_ ? OGS_F_ENABLE_V4 : 0u) |
      (v4OverV6Nexthop_ ? OGS_F_V4_OVER_V6 : 0u) |
      (enableBestRouteSelection_ ? OGS_F_BEST_ROUTE_SELECTION : 0u) |
      (wide ? OGS_F_WIDE_METRIC : 0u) | (exact ? OGS_F_EXACT_ORDER : 0u);
  if (I.unitSrc != s) {
    const ogs_unit u{0, s};
    I.unit.upload(&u, 1);
    I.unitSrc = s;
  }
  LinkState::DeviceSpf* memo = ls.findDeviceSpf(s, true, N, W, db, exact);
  if (!memo) {
    // SPF only into a memo slot: the topology's descriptor without a prefix
    // table (the full table is not needed to answer a few prefixes)
    const uint32_t desc[8] = {0, N, 0, uint32_t(f.edges.size()), 0, 0, 0, 0};
    I.spfDesc.upload(desc, 8);
    LinkState::DeviceSpf& slot = ls.newDeviceSpf(s, true, N, W, db, exact);
    const ogs_graph g = singleGraph(f, I.spfDesc.as<uint32_t>());
    ogs_spf_out so{};
    so.dist = slot.dist();
    so.nh = slot.nh();
    so.reached = exact ? slot.reach() : nullptr;
    ogsCheck(ogs_spf_routes(&g, nullptr, I.unit.as<ogs_unit>(), 1, flags, W, &so, nullptr),
             "ogs_spf_routes");
    ls.commitDeviceSpf(slot, me, true);
    memo = &slot;
  }
  const auto tSpf = std::chrono::steady_clock::now();

  // the changed prefixes' table: one packed H2D
  HostBatch hb;
  const uint32_t np = hb.appendPrefixes(f, sub, area);
  const uint32_t desc[8] = {0, N, 0, uint32_t(f.edges.size()), 0, np, 0,
                            uint32_t(hb.advNode.size())};
  I.subTable.build(sub);
  TableImage T;
  T.pack(hb, desc, I.hSubTab);
  I.subTab.resize(T.end);
  ogsCheck(ogs_memcpy_h2d(I.subTab.get(), I.hSubTab.get(), T.end, nullptr), "ogs_memcpy_h2d");
  const auto tTab = std::chrono::steady_clock::now();
  const ResultImage R(0, np, W, db);  // records only (dist / nh spans empty)
  I.subRes.resize(R.end);
  I.hSubRes.resize(R.end);
  const ogs_graph g = singleGraph(f, devAt<uint32_t>(I.subTab, T.desc));
  const ogs_prefix_table pt = T.view(I.subTab);
  ogs_spf_out ro{};
  ro.meta = devAt<uint32_t>(I.subRes, R.meta);
  ro.metric = devAt<void>(I.subRes, R.metric);
  ro.mask = devAt<uint32_t>(I.subRes, R.mask);
  ro.sel = devAt<uint32_t>(I.subRes, R.sel);
  ogsCheck(ogs_routes_from_spf(&g, &pt, I.unit.as<ogs_unit>(), 1, memo->dist(), memo->nh(),
                               exact ? memo->reach() : nullptr, flags, W, &ro, nullptr),
           "ogs_routes_from_spf");
  ogsCheck(ogs_memcpy_d2h(I.hSubRes.at<char>(R.meta), devAt<char>(I.subRes, R.meta),
                          R.end - R.meta, nullptr),
           "ogs_memcpy_d2h");
  ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
  const auto tDev = std::chrono::steady_clock::now();

  std::vector<uint64_t> metric;
  widenSpan(I.hSubRes.at<void>(R.metric), np, wide, metric);
  const uint32_t* meta = I.hSubRes.at<uint32_t>(R.meta);
  const uint32_t* mask = I.hSubRes.at<uint32_t>(R.mask);
  const uint32_t* sel = I.hSubRes.at<uint32_t>(R.sel);
  const PrefixHostTable& st = I.subTable;
  uint64_t noRoute = 0;
  for (uint32_t p = 0; p < np; ++p) {
    const std::string& prefix = st.prefixes[p];
    noRoute += noRouteReason(meta[p]);
    if (meta[p] & OGS_ROUTE_SELECTED) {  // SpfSolver.cpp:247
      RouteSelectionResult rs;
      const uint32_t a0 = st.advOff[p], a1 = st.advOff[p + 1];
      for (uint32_t a = a0; a < std::min(a1, a0 + 32); ++a) {
        if (sel[p] >> (a - a0) & 1u) rs.allNodeAreas.insert(st.advKey[a]);
      }
      rs.bestNodeArea = st.advKey[a0 + (meta[p] >> OGS_ROUTE_BEST_SHIFT)];
      rs.isBestNodeDrained = meta[p] & OGS_ROUTE_DRAINED;
      bestRoutesCache_[prefix] = std::move(rs);
    } else {
      bestRoutesCache_.erase(prefix);
    }
    out[prefix] = materializeRoute(f, me, st, p, meta[p], metric[p], &mask[p], np, W,
                                   v4OverV6Nexthop_, nullptr, OGS_POLICY_NONE,
                                   OGS_POLICY_NONE);
  }
  if (noRoute) addStatValue("decision.no_route_to_prefix", double(noRoute), StatType::COUNT);
  // split of the per-prefix path (decision.gpu.inc_*_ms): SPF memo check /
  // run, sub-table build + H2D, route launch + D2H + sync, materialisation
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const auto tEnd = std::chrono::steady_clock::now();
  addStatValue("decision.gpu.inc_spf_ms", ms(tIn, tSpf), StatType::AVG);
  addStatValue("decision.gpu.inc_table_ms", ms(tSpf, tTab), StatType::AVG);
  addStatValue("decision.gpu.inc_device_ms", ms(tTab, tDev), StatType::AVG);
  addStatValue("decision.gpu.inc_materialize_ms", ms(tDev, tEnd), StatType::AVG);
}

// Domain tables of a multi-area buildRouteDb: the areas' CSR as one graph
// batch (cached on the areas' topology versions) and the domain prefix table
// with per-entry area and node-name ids (cached on the PrefixState version).
void SpfSolver::prepareMultiArea(const AreaLinkStates& als, const PrefixState& ps) {
  Impl::MultiArea& M = impl_->ma;
  const uint32_t A = uint32_t(als.size());
  std::vector<std::pair<const FlatTopology*, uint64_t>> key;
  for (const auto& [area, ls] : als) {
    const FlatTopology& f = ls.flat();
    key.emplace_back(&f, f.version);
  }
  // zero / negative metrics anywhere: the whole domain's SPF launch replays
  // the reference's extraction order (spf_exact.hip); 64-bit distances then
  // or when a 32-bit path sum could overflow
  M.exact = false;
  M.wide = false;
  for (const auto& [area, ls] : als) {
    const FlatTopology& f = ls.flat();
    M.exact |= f.hasZeroMetric || f.hasWideMetric;
    M.wide |= wideDistancesNeeded(f);
  }
  M.wide |= M.exact;
  const bool topoChanged = key != M.topoKey;
  if (topoChanged) {
    static const PrefixState kNoPrefixes;
    M.areas.clear();
    M.flats.clear();
    M.hb = HostBatch();
    for (const auto& [area, ls] : als) {
      M.areas.push_back(area);
      M.flats.push_back(&ls.flat());
      M.hb.append(ls.flat(), kNoPrefixes, area);
    }
    M.nodeBase.upload(M.hb.nodeBase.data(), M.hb.nodeBase.size());
    M.rowPtr.upload(M.hb.rowPtr.data(), M.hb.rowPtr.size());
    M.edges.upload(M.hb.edges.data(), M.hb.edges.size());
    M.flags.upload(M.hb.nodeFlags.data(), M.hb.nodeFlags.size());
    M.edgeSrc.upload(M.hb.edgeSrc.data(), M.hb.edgeSrc.size());
    M.desc.upload(M.hb.topoDesc.data(), M.hb.topoDesc.size());
    M.topoKey = key;
  }
  if (!topoChanged && M.ps == &ps && M.psVersion == ps.version()) return;
  M.nameId.clear();
  std::vector<std::string> names;
  auto nid = [&](const std::string& n) {
    auto [it, fresh] = M.nameId.emplace(n, uint32_t(names.size()));
    if (fresh) names.push_back(n);
    return it->second;
  };
  for (const FlatTopology* f : M.flats) {
    for (const auto& n : f->names) nid(n);
  }
  M.table.build(ps);
  std::vector<uint32_t> advOff{0}, advNode, advArea, advName;
  std::vector<int32_t> advMetrics;
  std::vector<int64_t> advMinNh;
  std::vector<uint8_t> pfxFlags;
  for (const auto& [prefix, entries] : ps.prefixes()) {
    bool anyMinNh = false;
    for (const auto& [na, e] : entries) {
      auto ait = std::find(M.areas.begin(), M.areas.end(), na.second);
      if (ait == M.areas.end()) {  // areaLinkStates.at(area) throws there
        throw std::out_of_range("prefix advertised in unknown area " + na.second);
      }
      const uint32_t a = uint32_t(ait - M.areas.begin());
      const auto lit = M.flats[a]->id.find(na.first);
      advNode.push_back(lit == M.flats[a]->id.end() ? OGS_NODE_NONE : lit->second);
      advArea.push_back(a);
      advName.push_back(nid(na.first));
      advMetrics.insert(advMetrics.end(),
                        {e->metrics.drain_metric, e->metrics.path_preference,
                         e->metrics.source_preference, e->metrics.distance});
      advMinNh.push_back(e->minNexthop ? *e->minNexthop : INT64_MIN);
      anyMinNh |= e->minNexthop.has_value();
    }
    advOff.push_back(uint32_t(advNode.size()));
    pfxFlags.push_back((isV4Prefix(prefix) ? OGS_PFX_V4 : 0u) |
                       (anyMinNh ? OGS_PFX_HAS_MIN_NH : 0u));
  }
  M.numNames = uint32_t(names.size());
  std::vector<uint32_t> nameLocal(size_t(M.numNames) * A, OGS_NODE_NONE);
  for (uint32_t g = 0; g < M.numNames; ++g) {
    for (uint32_t a = 0; a < A; ++a) {
      auto it = M.flats[a]->id.find(names[g]);
      if (it != M.flats[a]->id.end()) nameLocal[size_t(g) * A + a] = it->second;
    }
  }
  M.maxPrefixes = uint32_t(pfxFlags.size());
  const uint32_t pfxBase[2] = {0, M.maxPrefixes};
  M.pfxBase.upload(pfxBase, 2);
  M.advOff.upload(advOff.data(), advOff.size());
  M.advNode.upload(advNode.data(), advNode.size());
  M.advArea.upload(advArea.data(), advArea.size());
  M.advName.upload(advName.data(), advName.size());
  M.advMetrics.upload(advMetrics.data(), advMetrics.size());
  M.advMinNh.upload(advMinNh.data(), advMinNh.size());
  M.pfxFlags.upload(pfxFlags.data(), pfxFlags.size());
  M.nameLocal.upload(nameLocal.data(), nameLocal.size());
  M.ps = &ps;
  M.psVersion = ps.version();
}

// Per-area masks -> next hops over that area's links; MPLS node labels of
// every area in map order (SpfSolver.cpp:354-445).
DecisionRouteDb SpfSolver::materializeMultiArea(const std::string& me,
                                                const AreaLinkStates& als,
                                                const MultiAreaResult& R) {
  Impl::MultiArea& M = impl_->ma;
  const uint32_t A = uint32_t(als.size());
  const int W = R.W;
  const size_t Sn = R.Sn, P = R.P;
  DecisionRouteDb rdb;
  bestRoutesCache_.clear();
  const PrefixHostTable& pt = M.table;
  uint64_t noRoute = 0;
  for (uint32_t p = 0; p < P; ++p) {
    const uint32_t m = R.meta[p];
    noRoute += noRouteReason(m);
    const uint32_t a0 = pt.advOff[p];
    const uint32_t best = a0 + (m >> OGS_ROUTE_BEST_SHIFT);
    if (m & OGS_ROUTE_SELECTED) {  // SpfSolver.cpp:247
      RouteSelectionResult rs;
      for (uint32_t a = a0; a < std::min(pt.advOff[p + 1], a0 + 32); ++a) {
        if (R.sel[p] >> (a - a0) & 1u) rs.allNodeAreas.insert(pt.advKey[a]);
      }
      rs.bestNodeArea = pt.advKey[best];
      rs.isBestNodeDrained = m & OGS_ROUTE_DRAINED;
      bestRoutesCache_[pt.prefixes[p]] = std::move(rs);
    }
    if (!(m & OGS_ROUTE_VALID)) continue;
    RibUnicastEntry e;
    e.prefix = pt.prefixes[p];
    const bool useV4 = isV4Prefix(e.prefix) && !v4OverV6Nexthop_;
    const int32_t m32 = static_cast<int32_t>(R.metric[p]);
    for (uint32_t a = 0; a < A; ++a) {
      if (R.row[a] == OGS_NODE_NONE) continue;
      const FlatTopology& f = *M.flats[a];
      const uint32_t rb = f.rowPtr[f.id.at(me)];
      for (int w = 0; w < W; ++w) {
        uint32_t bits = R.mask[(size_t(a) * W + w) * P + p];
        while (bits) {
          const int b = __builtin_ctz(bits);
          bits &= bits - 1;
          e.nexthops.insert(makeNh(*f.edgeLink[rb + w * 32 + b], me, useV4, m32,
                                   std::nullopt));
        }
      }
    }
    e.bestPrefixEntry = *pt.advEntry[best];
    if (m & OGS_ROUTE_DRAINED) e.bestPrefixEntry.metrics.drain_metric = 1;
    e.bestPrefixEntry.weight = std::nullopt;  // RibEntry.h:77
    e.bestArea = pt.advKey[best].second;
    e.igpCost = static_cast<unsigned int>(R.metric[p]);
    e.localRouteConsidered = m & OGS_ROUTE_LOCAL;
    if (!R.applied.empty()) finishPolicy(ribPolicy_, R.applied[p], R.counter[p], e);
    rdb.unicastRoutes.emplace(e.prefix, std::move(e));
  }
  // counted also on the probe solver of the incremental path (the
  // reference counts it per createRouteForPrefix call)
  if (noRoute) addStatValue("decision.no_route_to_prefix", double(noRoute), StatType::COUNT);
  for (const auto& [prefix, e] : staticUnicastRoutes_) {  // SpfSolver.cpp:343-349
    if (rdb.unicastRoutes.count(prefix)) continue;
    auto it = rdb.unicastRoutes.emplace(prefix, e).first;
    if (ribPolicy_ && ribPolicy_->isActive()) ribPolicy_->applyAction(it->second);
  }
  if (enableNodeSegmentLabel_) {
    LabelRoutes labelToNode;
    std::vector<uint64_t> d64(Sn);
    uint32_t a = 0;
    for (const auto& [area, ls] : als) {
      const uint64_t* dist = nullptr;
      const uint32_t* nhw = nullptr;
      const uint32_t* reach = nullptr;
      if (R.row[a] != OGS_NODE_NONE) {
        for (size_t v = 0; v < Sn; ++v) d64[v] = R.dist[R.row[a] * Sn + v];
        dist = d64.data();
        nhw = &R.nh[size_t(R.row[a]) * W * Sn];
        if (!R.reach.empty()) reach = &R.reach[size_t(R.row[a]) * ((Sn + 31) / 32)];
      }
      addNodeLabelRoutes(ls, *M.flats[a], area, me, dist, nhw, Sn, W, labelToNode, reach);
      ++a;
    }
    for (auto& [label, ne] : labelToNode) {
      rdb.mplsRoutes.emplace(label, std::move(ne.second));
    }
  }
  return rdb;
}

// Kernels of a multi-area build on `stream`: SPF of the source in every
// area holding it (one launch), the multi-area RouteDb, the RibPolicy.
// Fills R's shape fields (row, W, Sn, P); results stay on the device.
void SpfSolver::enqueueMultiArea(const std::string& me, const AreaLinkStates& als,
                                 const PrefixState& ps, void* stream,
                                 MultiAreaResult& R) {
  prepareMultiArea(als, ps);
  Impl::MultiArea& M = impl_->ma;
  const uint32_t A = uint32_t(als.size());

  // ---- SPF of the source in every area holding it (one launch) -----------
  std::vector<ogs_unit> su;
  R.row.assign(A, OGS_NODE_NONE);
  for (uint32_t a = 0; a < A; ++a) {
    const FlatTopology& f = *M.flats[a];
    auto it = f.id.find(me);
    if (it == f.id.end()) continue;
    R.row[a] = uint32_t(su.size());
    su.push_back({a, it->second});
    const int deg = int(f.rowPtr[it->second + 1] - f.rowPtr[it->second]);
    R.W = std::max(R.W, std::max(1, ogs_nh_words_for_degree(deg)));
  }
  const int W = R.W;
  R.Sn = size_t(std::max(M.hb.maxNodes, 1));
  R.P = M.maxPrefixes;
  const size_t Sn = R.Sn, P = R.P, P1 = std::max<size_t>(P, 1);
  const uint32_t S = M.nameId.at(me);
  M.units.upload(su.data(), su.size(), stream);
  M.spfRow.upload(R.row.data(), R.row.size(), stream);
  M.srcName.upload(&S, 1, stream);
  R.wide = M.wide;
  const size_t db = M.wide ? 8 : 4;
  M.dist.resize(su.size() * Sn * db);
  M.nh.resize(su.size() * W * Sn * 4);
  M.meta.resize(P1 * 4);
  M.metric.resize(P1 * db);
  M.mask.resize(P1 * A * W * 4);
  M.sel.resize(P1 * 4);
  const size_t RW = (Sn + 31) / 32;
  M.reach.resize(std::max<size_t>(su.size() * RW * 4, 4));
  ogs_graph g{};
  g.num_topos = int32_t(A);
  g.max_nodes = int32_t(Sn);
  g.max_edges = M.hb.maxEdges;
  g.max_degree = M.hb.maxDegree;
  g.node_base = M.nodeBase.as<uint32_t>();
  g.row_ptr = M.rowPtr.as<uint32_t>();
  g.edges = M.edges.as<uint64_t>();
  g.node_flags = M.flags.as<uint8_t>();
  g.topo_desc = M.desc.as<uint32_t>();
  g.edge_src = M.edgeSrc.as<uint32_t>();
  const uint32_t flags = (enableV4_ ? OGS_F_ENABLE_V4 : 0u) |
      (v4OverV6Nexthop_ ? OGS_F_V4_OVER_V6 : 0u) |
      (enableBestRouteSelection_ ? OGS_F_BEST_ROUTE_SELECTION : 0u) |
      (M.wide ? OGS_F_WIDE_METRIC : 0u) | (M.exact ? OGS_F_EXACT_ORDER : 0u);
  ogs_spf_out spf{};
  spf.dist = M.dist.get();
  spf.nh = M.nh.as<uint32_t>();
  spf.reached = M.exact ? M.reach.as<uint32_t>() : nullptr;
  ogsCheck(ogs_spf_routes(&g, nullptr, M.units.as<ogs_unit>(), int32_t(su.size()),
                          flags, W, &spf, stream),
           "ogs_spf_routes");
  // one SPF per area holding `me` (SpfSolver.cpp:595-639 calls getSpfResult
  // per area); the multi-area batch does not use the per-area row memos
  addStatValue("decision.gpu.spf_launches", double(su.size()), StatType::COUNT);
  for (const auto& [area, ls] : als) {
    if (ls.flat().id.count(me)) ls.noteSpf(me);
  }

  // ---- multi-area RouteDb --------------------------------------------------
  if (P) {
    ogs_prefix_table pt{};
    pt.max_prefixes = int32_t(P);
    pt.max_advertisements = int32_t(M.table.advEntry.size());
    pt.pfx_base = M.pfxBase.as<uint32_t>();
    pt.adv_off = M.advOff.as<uint32_t>();
    pt.adv_node = M.advNode.as<uint32_t>();
    pt.adv_metrics = M.advMetrics.as<int32_t>();
    pt.adv_min_nh = M.advMinNh.as<int64_t>();
    pt.pfx_flags = M.pfxFlags.as<uint8_t>();
    ogs_area_table at{int32_t(A), int32_t(M.numNames), M.nameLocal.as<uint32_t>(),
                      M.advArea.as<uint32_t>(), M.advName.as<uint32_t>(),
                      M.exact ? M.reach.as<uint32_t>() : nullptr};
    ogs_spf_out out{};
    out.meta = M.meta.as<uint32_t>();
    out.metric = M.metric.get();
    out.mask = M.mask.as<uint32_t>();
    out.sel = M.sel.as<uint32_t>();
    ogsCheck(ogs_routes_multiarea(&g, &pt, &at, M.srcName.as<uint32_t>(), 1,
                                  M.spfRow.as<uint32_t>(), M.dist.get(),
                                  M.nh.as<uint32_t>(), flags, W, &out, stream),
             "ogs_routes_multiarea");
    if (ribPolicy_ && ribPolicy_->isActive()) {
      std::vector<std::pair<const FlatTopology*, uint32_t>> src;
      for (uint32_t a = 0; a < A; ++a) {
        auto it = M.flats[a]->id.find(me);
        src.emplace_back(M.flats[a], it == M.flats[a]->id.end() ? OGS_NODE_NONE : it->second);
      }
      runPolicyOnDevice(*ribPolicy_, M.table, pt, src, me, W, M.meta.as<uint32_t>(),
                        M.mask.as<uint32_t>(), impl_->policy, stream);
    }
  }
}

bool SpfSolver::enqueueRouteDb(const std::string& me, const AreaLinkStates& als,
                               const PrefixState& ps, void* stream) {
  bool found = false;
  for (const auto& [_, ls] : als) found |= ls.hasNode(me);
  if (!found) return false;
  impl_->enqueued.emplace();
  impl_->enqueuedMe = me;
  enqueueMultiArea(me, als, ps, stream, *impl_->enqueued);
  return true;
}

std::optional<DecisionRouteDb> SpfSolver::collectRouteDb(const std::string& me,
                                                         const AreaLinkStates& als,
                                                         void* stream) {
  if (!impl_->enqueued || impl_->enqueuedMe != me) {
    throw std::logic_error("collectRouteDb: no enqueueRouteDb(" + me + ") to collect");
  }
  ogsCheck(ogs_stream_sync(stream), "ogs_stream_sync");
  MultiAreaResult R = *impl_->enqueued;
  return downloadMultiArea(me, als, R);
}

std::optional<DecisionRouteDb> SpfSolver::buildRouteDbMultiArea(
    const std::string& me, const AreaLinkStates& als, const PrefixState& ps) {
  MultiAreaResult R;
  enqueueMultiArea(me, als, ps, nullptr, R);
  return downloadMultiArea(me, als, R);
}

// D2H of a multi-area build's device results (default stream after the
// launches) + materialisation.
DecisionRouteDb SpfSolver::downloadMultiArea(const std::string& me,
                                             const AreaLinkStates& als,
                                             MultiAreaResult& R) {
  Impl::MultiArea& M = impl_->ma;
  const uint32_t A = uint32_t(als.size());
  const int W = R.W;
  const size_t Sn = R.Sn, P = R.P;
  const size_t nSpf = size_t(std::count_if(R.row.begin(), R.row.end(),
                                           [](uint32_t r) { return r != OGS_NODE_NONE; }));
  if (P && ribPolicy_ && ribPolicy_->isActive()) {
    downloadPolicy(impl_->policy, P, R.applied, R.counter);
  }
  R.nh.resize(nSpf * W * Sn);
  R.meta.resize(P);
  R.mask.resize(P * A * W);
  R.sel.resize(P);
  // distances / route metrics widened to 64 bits, all-ones = unreachable
  auto widen = [&](const DeviceBuffer& b, size_t n, std::vector<uint64_t>& v) {
    v.resize(n);
    if (!n) return;
    if (R.wide) {
      b.download(v.data(), n);
    } else {
      std::vector<uint32_t> t(n);
      b.download(t.data(), n);
      for (size_t i = 0; i < n; ++i) v[i] = t[i] == 0xFFFFFFFFu ? ~0ull : t[i];
    }
  };
  widen(M.dist, nSpf * Sn, R.dist);
  M.nh.download(R.nh.data(), R.nh.size());
  R.reach.clear();
  if (M.exact && nSpf) {
    R.reach.resize(nSpf * ((Sn + 31) / 32));
    M.reach.download(R.reach.data(), R.reach.size());
  }
  if (P) {
    M.meta.download(R.meta.data(), P);
    widen(M.metric, P, R.metric);
    M.mask.download(R.mask.data(), R.mask.size());
    M.sel.download(R.sel.data(), P);
  }
  ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
  return materializeMultiArea(me, als, R);
}

std::optional<RibUnicastEntry> SpfSolver::createRouteForPrefixOrGetStaticRoute(
    const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
    const std::string& prefix) {  // SpfSolver.cpp:139-158
  addStatValue("decision.get_route_for_prefix", 1.0, StatType::COUNT);  // :166
  std::vector<std::pair<const FlatTopology*, uint64_t>> topo;
  for (const auto& [_, l] : als) {
    const FlatTopology& f = l.flat();
    topo.emplace_back(&f, f.version);
  }
  if (incMe_ != me || incPsVersion_ != ps.version() || incTopo_ != topo) {
    incCache_.clear();
    incMe_ = me;
    incPsVersion_ = ps.version();
    incTopo_ = std::move(topo);
  }
  auto hit = incCache_.find(prefix);
  if (hit == incCache_.end()) {
    // this call and every prefix changed since the last build / batch
    // (Decision's pending updatedPrefixes, the loop this call is part of)
    std::set<std::string> batch{prefix};
    ps.trackChanges();
    if (incPs_ != &ps || incLogCursor_ < ps.changeLogBase()) {
      incPs_ = &ps;
      incLogCursor_ = ps.changeLogBase();  // unknown position: the whole log
    }
    const auto& log = ps.changeLog();
    for (size_t i = size_t(incLogCursor_ - ps.changeLogBase()); i < log.size(); ++i) {
      batch.insert(log[i]);
    }
    incLogCursor_ = ps.changeLogEnd();
    ++incBatches_;
    incBatchPrefixes_ += batch.size();
    // the batch's selections go into the entries; bestRoutesCache_ keeps
    // the pre-batch state until each prefix is asked
    std::vector<std::pair<std::string, std::optional<RouteSelectionResult>>> pre;
    for (const auto& p : batch) {
      auto b = bestRoutesCache_.find(p);
      pre.emplace_back(p, b == bestRoutesCache_.end()
                              ? std::nullopt
                              : std::optional<RouteSelectionResult>(b->second));
    }
    auto routes = computeRoutes(me, als, ps, batch);
    for (auto& [p, before] : pre) {
      IncEntry& e = incCache_[p];
      e.route = std::move(routes[p]);
      auto b = bestRoutesCache_.find(p);
      e.sel = b == bestRoutesCache_.end() ? std::nullopt
                                          : std::optional<RouteSelectionResult>(b->second);
      // SpfSolver.cpp:170-185: a gated or unknown prefix returns before the
      // selection cache is touched
      e.touched = ps.prefixes().count(p) && !(isV4Prefix(p) && !enableV4_ && !v4OverV6Nexthop_);
      if (before) {
        bestRoutesCache_[p] = std::move(*before);
      } else if (b != bestRoutesCache_.end()) {
        bestRoutesCache_.erase(b);
      }
    }
    hit = incCache_.find(prefix);
  }
  if (hit->second.touched) {  // SpfSolver.cpp:185, :239 for this prefix
    if (hit->second.sel) {
      bestRoutesCache_[prefix] = *hit->second.sel;
    } else {
      bestRoutesCache_.erase(prefix);
    }
  }
  if (hit->second.route) {
    // handed out by move: Decision asks each changed prefix once per
    // rebuild; asking it again recomputes it (a batch of just that prefix
    // plus whatever changed since)
    std::optional<RibUnicastEntry> r = std::move(hit->second.route);
    incCache_.erase(hit);
    return r;
  }
  auto it = staticUnicastRoutes_.find(prefix);  // static routes as the fallback
  if (it != staticUnicastRoutes_.end()) return it->second;
  return std::nullopt;
}

std::map<std::string, std::optional<RibUnicastEntry>> SpfSolver::createRoutesForPrefixes(
    const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
    const std::set<std::string>& prefixes) {
  // SpfSolver.cpp:166: one createRouteForPrefix per asked prefix
  addStatValue("decision.get_route_for_prefix", double(prefixes.size()), StatType::COUNT);
  auto out = computeRoutes(me, als, ps, prefixes);
  for (auto& [prefix, route] : out) {  // static routes as the fallback
    if (route) continue;
    auto it = staticUnicastRoutes_.find(prefix);
    if (it != staticUnicastRoutes_.end()) route = it->second;
  }
  return out;
}

std::map<std::string, std::optional<RibUnicastEntry>> SpfSolver::computeRoutes(
    const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
    const std::set<std::string>& prefixes) {
  std::map<std::string, std::optional<RibUnicastEntry>> out;
  bool exists = false;  // SpfSolver.cpp:139-158 per prefix
  for (const auto& [_, l] : als) exists |= l.hasNode(me);
  PrefixState sub;  // the changed prefixes through one route launch
  std::set<std::string> asked;
  for (const auto& prefix : prefixes) {
    out[prefix] = std::nullopt;
    auto pit = ps.prefixes().find(prefix);
    const bool gated = isV4Prefix(prefix) && !enableV4_ && !v4OverV6Nexthop_;
    // gated or unknown prefix: returned before the selection cache is
    // touched (SpfSolver.cpp:170-182); known prefix: its entry is cleared,
    // then set again only by a successful selection (:185, :239)
    if (gated || pit == ps.prefixes().end()) continue;
    if (!exists) {
      bestRoutesCache_.erase(prefix);
      continue;
    }
    for (const auto& [na, e] : pit->second) sub.updatePrefixKeyed(na.first, na.second, pit->first, *e);
    asked.insert(prefix);
  }
  if (!asked.empty() && als.size() == 1) {
    std::string area;
    const LinkState& ls = singleArea(als, area);
    routesFromSpfMemo(me, ls, area, ps, sub, out);
  } else if (!asked.empty()) {
    // several areas: the multi-area build over the sub-table on a private
    // solver kept across calls (its domain CSR stays on the device while the
    // topology is unchanged); its builds are not Decision's route builds
    if (!probe_) {
      probe_ = std::make_unique<SpfSolver>(myNodeName_, enableV4_, false,
                                           enableBestRouteSelection_, v4OverV6Nexthop_);
      probe_->quietStats_ = true;
    }
    SpfSolver& probe = *probe_;
    auto db = probe.buildRouteDb(me, als, sub);
    const auto& bcache = probe.getBestRoutesCache();
    for (const auto& prefix : asked) {
      if (db) {
        auto it = db->unicastRoutes.find(prefix);
        if (it != db->unicastRoutes.end()) out[prefix] = it->second;
      }
      auto bc = bcache.find(prefix);
      if (bc != bcache.end()) bestRoutesCache_[prefix] = bc->second;
      else bestRoutesCache_.erase(prefix);
    }
  }
  return out;
}

// ------------------------------------------------------------- RibPolicy --
RibPolicy::RibPolicy(const std::vector<RibPolicyStatementSpec>& statements,
                     int64_t ttlSecs)
    : validUntil_(std::chrono::steady_clock::now() + std::chrono::seconds(ttlSecs)) {  // RibPolicy.cpp:20-50, 167-182
  static std::atomic<uint64_t> nextUid{1};
  uid_ = nextUid++;
  if (statements.empty()) {
    throw std::invalid_argument("Missing policy.statements attribute");
  }
  for (const auto& s : statements) {
    if (!s.set_weight) {
      throw std::invalid_argument(
          "Missing policy_statement.action.set_weight attribute");
    }
    if (!s.prefixes && !s.tags) {
      throw std::invalid_argument(
          "Missing policy_statement.matcher.prefixes or "
          "policy_statement.matcher.tags attribute");
    }
    Stmt st;
    st.name = s.name;
    if (s.prefixes) st.prefixes.insert(s.prefixes->begin(), s.prefixes->end());
    if (s.tags) st.tags.insert(s.tags->begin(), s.tags->end());
    st.weight = *s.set_weight;
    st.counterID = s.counterID;
    stmts_.push_back(std::move(st));
  }
}

bool RibPolicy::matchStmt(const Stmt& s, const RibUnicastEntry& r) const {
  if (s.tags.empty() && s.prefixes.empty()) return false;  // RibPolicy.cpp:74-107
  bool tag = s.tags.empty();
  for (const auto& t : s.tags) {
    if (r.bestPrefixEntry.tags.count(t)) {
      tag = true;
      break;
    }
  }
  return tag && (s.prefixes.empty() || s.prefixes.count(r.prefix));
}

bool RibPolicy::matchesTags(size_t k, const std::set<std::string>& tags) const {
  const Stmt& s = stmts_[k];
  if (s.tags.empty()) return true;
  for (const auto& t : s.tags) {
    if (tags.count(t)) return true;
  }
  return false;
}

int32_t RibPolicy::weightOf(size_t k, const NextHopThrift& nh) const {
  const Stmt& s = stmts_[k];  // neighbor > area > default (RibPolicy.cpp:122-137)
  int32_t w = s.weight.default_weight;
  if (nh.area) {
    if (auto it = s.weight.area_to_weight.find(*nh.area);
        it != s.weight.area_to_weight.end()) {
      w = it->second;
    }
  }
  if (nh.neighborNodeName) {
    if (auto it = s.weight.neighbor_to_weight.find(*nh.neighborNodeName);
        it != s.weight.neighbor_to_weight.end()) {
      w = it->second;
    }
  }
  return w;
}

bool RibPolicy::match(const RibUnicastEntry& r) const {
  for (const auto& s : stmts_) {
    if (matchStmt(s, r)) return true;
  }
  return false;
}

bool RibPolicy::applyAction(RibUnicastEntry& r) const {
  for (const auto& s : stmts_) {  // first statement that transforms wins
    if (!matchStmt(s, r)) continue;
    r.counterID = s.counterID;
    NextHops next;
    for (const auto& nh : r.nexthops) {  // neighbor > area > default
      int32_t w = s.weight.default_weight;
      if (nh.area) {
        if (auto it = s.weight.area_to_weight.find(*nh.area);
            it != s.weight.area_to_weight.end()) {
          w = it->second;
        }
      }
      if (nh.neighborNodeName) {
        if (auto it = s.weight.neighbor_to_weight.find(*nh.neighborNodeName);
            it != s.weight.neighbor_to_weight.end()) {
          w = it->second;
        }
      }
      if (w > 0) {
        NextHopThrift n = nh;
        n.weight = w;
        next.insert(std::move(n));
      }
    }
    if (next.empty()) continue;  // keep the old next-hops (RibPolicy.cpp:148-158)
    r.nexthops = std::move(next);
    return true;
  }
  return false;
}

std::vector<std::string> RibPolicy::applyPolicy(
    std::map<std::string, RibUnicastEntry>& entries) const {
  std::vector<std::string> updated;  // RibPolicy.cpp:231-249
  if (!isActive()) return updated;
  for (auto& [p, e] : entries) {
    if (applyAction(e)) updated.push_back(p);
  }
  return updated;
}

}  // namespace openr_amd
