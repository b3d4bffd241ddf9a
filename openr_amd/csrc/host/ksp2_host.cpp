// ksp2_host.cpp — LinkState::getKthPaths on the GPU (reference
// LinkState.cpp:674-703): the k-th call masks every link of the paths for
// 1..k-1 and launches one KSP unit (masked SPF + greedy trace).
#include <algorithm>
#include <stdexcept>
#include <unordered_map>

#include "decision.h"

namespace openr_amd {

const std::vector<LinkState::Path>& LinkState::getKthPaths(
    const std::string& src, const std::string& dest, size_t k) const {
  if (k < 1) throw std::invalid_argument("getKthPaths: k must be >= 1");
  auto key = std::make_tuple(src, dest, k);
  if (auto it = kthMemo_.find(key); it != kthMemo_.end()) return it->second;

  std::vector<const Link*> ignore;
  for (size_t i = 1; i < k; ++i) {
    for (const auto& p : getKthPaths(src, dest, i)) {
      for (const auto& l : p) ignore.push_back(l.get());
    }
  }
  const FlatTopology& f = flatOnDevice();
  std::vector<Path> paths;
  auto sIt = f.id.find(src), dIt = f.id.find(dest);
  if (sIt == f.id.end() || dIt == f.id.end() || src == dest) {
    // unknown endpoints or src == dest: the reference finds no path (after
    // its SPF, which it counts)
    if (ignore.empty()) {
      noteSpf(src);
    } else {
      noteSpfRuns(1);
    }
    return kthMemo_.emplace(key, std::move(paths)).first->second;
  }
  const uint32_t E = uint32_t(f.edges.size());
  const uint32_t maskWords = std::max<uint32_t>(1, (E + 31) / 32);
  std::vector<uint32_t> mask;
  if (!ignore.empty()) {
    std::unordered_map<const Link*, uint32_t> canon;  // link -> min edge id
    for (uint32_t e = 0; e < E; ++e) canon.emplace(f.edgeLink[e], e);
    mask.assign(maskWords, 0u);
    for (const Link* l : ignore) {
      // links are re-flattened objects of this LinkState; match by key
      const uint32_t e = canon.at(links_.at(l->key()).get());
      mask[e >> 5] |= 1u << (e & 31u);
    }
  }
  const uint32_t t = dIt->second;
  const uint32_t maxPaths = f.rowPtr[t + 1] - f.rowPtr[t] + 1;
  const uint32_t maxEdges = E / 2 + 1;

  DeviceBuffer dUnit, dMask, dCount, dLen, dEdges;
  const ogs_path_unit u{0, sIt->second, t, 0};
  dUnit.upload(&u, 1);
  if (!mask.empty()) dMask.upload(mask.data(), mask.size());
  dCount.resize(4);
  dLen.resize(maxPaths * 4);
  dEdges.resize(maxEdges * 4);
  ogs_graph g{};
  g.num_topos = 1;
  g.max_nodes = int32_t(f.names.size());
  g.max_edges = int32_t(E);
  g.max_degree = f.maxDegree;
  g.node_base = f.dNodeBase.as<uint32_t>();
  g.row_ptr = f.dRow.as<uint32_t>();
  g.edges = f.dEdges.as<uint64_t>();
  g.node_flags = f.dFlags.as<uint8_t>();
  g.rslot_ext = f.rslotExtDev();  // rows of 512+ edges
  ogs_path_out out{dCount.as<uint32_t>(), dLen.as<uint32_t>(),
                   dEdges.as<uint32_t>(), maxPaths, maxEdges};
  // zero / negative metrics: pathLinks follow the reference's extraction
  // order (ksp.hip, HBM-state path with OGS_F_EXACT_ORDER)
  const bool exact = f.hasZeroMetric || f.hasWideMetric;
  const uint32_t flags = (exact || wideDistancesNeeded(f) ? OGS_F_WIDE_METRIC : 0u) |
      (exact ? OGS_F_EXACT_ORDER : 0u);
  ogsCheck(ogs_ksp_paths(&g, dUnit.as<ogs_path_unit>(), 1,
                         mask.empty() ? nullptr : dMask.as<uint32_t>(),
                         maskWords, flags, &out, nullptr),
           "ogs_ksp_paths");
  // k = 1 traces the memoised getSpfResult(src), k > 1 a masked runSpf
  // (LinkState.cpp:690-692)
  if (ignore.empty()) {
    noteSpf(src);
  } else {
    noteSpfRuns(1);
  }
  uint32_t count = 0;
  dCount.download(&count, 1);
  ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
  if (count >> 31) throw std::runtime_error("getKthPaths: path buffer overflow");
  std::vector<uint32_t> len(count), edges;
  if (count) {
    dLen.download(len.data(), count);
    uint32_t total = 0;
    for (auto x : len) total += x;
    edges.resize(total);
    dEdges.download(edges.data(), total);
    ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
  }
  size_t pos = 0;
  for (uint32_t i = 0; i < count; ++i) {
    Path p;
    for (uint32_t j = 0; j < len[i]; ++j) {
      p.push_back(links_.at(f.edgeLink[edges[pos++]]->key()));
    }
    paths.push_back(std::move(p));
  }
  return kthMemo_.emplace(key, std::move(paths)).first->second;
}

// ---- Ksp2Batch ----------------------------------------------------------
Ksp2Batch::Ksp2Batch(const LinkState& ls, const std::string& src,
                     const std::vector<std::string>& dests)
    : ls_{&ls} {
  init(src, {dests});
}

Ksp2Batch::Ksp2Batch(const std::vector<const LinkState*>& areas,
                     const std::string& src,
                     const std::vector<std::vector<std::string>>& destinations)
    : ls_(areas) {
  if (areas.size() != destinations.size()) {
    throw std::invalid_argument("Ksp2Batch: one destination list per topology");
  }
  init(src, destinations);
}

void Ksp2Batch::init(const std::string& src,
                     const std::vector<std::vector<std::string>>& destinations) {
  const size_t T = ls_.size();
  std::vector<const FlatTopology*> fl(T);
  for (size_t a = 0; a < T; ++a) {
    fl[a] = T == 1 ? &ls_[a]->flatOnDevice() : &ls_[a]->flat();
    for (const auto& d : destinations[a]) {
      dests_.push_back(d);
      destArea_.push_back(a);
    }
  }
  unitOf_.assign(dests_.size(), -1);
  std::vector<ogs_unit> sources;
  std::vector<int64_t> srcOf(T, -1);
  for (size_t a = 0; a < T; ++a) {
    auto it = fl[a]->id.find(src);
    if (it == fl[a]->id.end()) continue;  // no source there: no paths there
    if (fl[a]->hasZeroMetric || fl[a]->hasWideMetric) {
      flags_ |= OGS_F_EXACT_ORDER | OGS_F_WIDE_METRIC;  // extraction order
    }
    srcOf[a] = int64_t(sources.size());
    sources.push_back(ogs_unit{uint32_t(a), it->second});
  }
  std::vector<ogs_path_unit> units;
  for (size_t i = 0; i < dests_.size(); ++i) {
    const size_t a = destArea_[i];
    if (srcOf[a] < 0) continue;
    auto dIt = fl[a]->id.find(dests_[i]);
    if (dIt == fl[a]->id.end()) continue;
    unitOf_[i] = int64_t(units.size());
    units.push_back(ogs_path_unit{uint32_t(a), sources[srcOf[a]].src, dIt->second,
                                  uint32_t(srcOf[a])});
  }
  nUnits_ = units.size();
  nSources_ = sources.size();
  if (!nUnits_) return;
  uint32_t maxN = 0, maxE = 0;
  int maxDeg = 0;
  for (const auto* f : fl) {
    maxN = std::max<uint32_t>(maxN, uint32_t(f->names.size()));
    maxE = std::max<uint32_t>(maxE, uint32_t(f->edges.size()));
    maxDeg = std::max(maxDeg, f->maxDegree);
    if (wideDistancesNeeded(*f)) flags_ |= OGS_F_WIDE_METRIC;
  }
  // edge-disjoint paths into d: at most deg(d) of them, at most E/2 links
  maxPaths_ = uint32_t(maxDeg) + 1;
  maxEdges_ = maxE / 2 + 1;
  dSrc_.upload(sources.data(), sources.size());
  dUnits_.upload(units.data(), units.size());
  for (int k = 0; k < 2; ++k) {
    dCount_[k].resize(nUnits_ * 4);
    dLen_[k].resize(nUnits_ * maxPaths_ * 4);
    dEdges2_[k].resize(nUnits_ * maxEdges_ * 4);
  }
  g_.num_topos = int32_t(T);
  g_.max_nodes = int32_t(maxN);
  g_.max_edges = int32_t(maxE);
  g_.max_degree = maxDeg;
  if (T == 1) {  // the LinkState's own device CSR
    g_.node_base = fl[0]->dNodeBase.as<uint32_t>();
    g_.row_ptr = fl[0]->dRow.as<uint32_t>();
    g_.edges = fl[0]->dEdges.as<uint64_t>();
    g_.node_flags = fl[0]->dFlags.as<uint8_t>();
    g_.rslot_ext = fl[0]->rslotExtDev();
    return;
  }
  // concatenated batch: global row offsets, topology-local edge targets
  std::vector<uint32_t> nodeBase{0}, row;
  std::vector<uint64_t> edges;
  std::vector<uint8_t> flags;
  for (const auto* f : fl) {
    const uint32_t eb = uint32_t(edges.size());
    for (size_t v = 0; v + 1 < f->rowPtr.size(); ++v) row.push_back(eb + f->rowPtr[v]);
    edges.insert(edges.end(), f->edges.begin(), f->edges.end());
    flags.insert(flags.end(), f->nodeFlags.begin(), f->nodeFlags.end());
    nodeBase.push_back(nodeBase.back() + uint32_t(f->names.size()));
  }
  row.push_back(uint32_t(edges.size()));
  dNodeBase_.upload(nodeBase.data(), nodeBase.size());
  dRow_.upload(row.data(), row.size());
  dEdges_.upload(edges.data(), edges.size());
  dFlags_.upload(flags.data(), flags.size());
  if (maxDeg >= OGS_MAX_DEGREE) {  // exact reverse slots, concatenated
    std::vector<uint32_t> ext;
    ext.reserve(edges.size());
    for (const auto* f : fl) {
      if (!f->rslotExt.empty()) {
        ext.insert(ext.end(), f->rslotExt.begin(), f->rslotExt.end());
      } else {
        for (uint64_t x : f->edges) {
          ext.push_back((uint32_t(x) >> OGS_EDGE_RSLOT_SHIFT) & OGS_EDGE_RSLOT_MASK);
        }
      }
    }
    dRslot_.upload(ext.data(), ext.size());
    g_.rslot_ext = dRslot_.as<uint32_t>();
  }
  g_.node_base = dNodeBase_.as<uint32_t>();
  g_.row_ptr = dRow_.as<uint32_t>();
  g_.edges = dEdges_.as<uint64_t>();
  g_.node_flags = dFlags_.as<uint8_t>();
}

void Ksp2Batch::launch(void* stream) const {
  if (!nUnits_) return;
  ogs_path_out o[2];
  for (int k = 0; k < 2; ++k) {
    o[k] = ogs_path_out{const_cast<DeviceBuffer&>(dCount_[k]).as<uint32_t>(),
                        const_cast<DeviceBuffer&>(dLen_[k]).as<uint32_t>(),
                        const_cast<DeviceBuffer&>(dEdges2_[k]).as<uint32_t>(),
                        maxPaths_, maxEdges_};
  }
  ogsCheck(ogs_ksp2_paths(&g_, const_cast<DeviceBuffer&>(dSrc_).as<ogs_unit>(),
                          int32_t(nSources_),
                          const_cast<DeviceBuffer&>(dUnits_).as<ogs_path_unit>(),
                          int32_t(nUnits_), flags_, &o[0], &o[1], stream),
           "ogs_ksp2_paths");
}

void Ksp2Batch::fetch() {
  if (!nUnits_) return;
  for (int k = 0; k < 2; ++k) {
    count_[k].resize(nUnits_);
    len_[k].resize(nUnits_ * maxPaths_);
    edges_[k].resize(nUnits_ * maxEdges_);
    dCount_[k].download(count_[k].data(), nUnits_);
    dLen_[k].download(len_[k].data(), len_[k].size());
    dEdges2_[k].download(edges_[k].data(), edges_[k].size());
  }
  ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
  for (int k = 0; k < 2; ++k) {
    for (uint32_t c : count_[k]) {
      if (c >> 31) throw std::runtime_error("Ksp2Batch: path buffer overflow");
    }
  }
}

std::vector<std::vector<uint32_t>> Ksp2Batch::edgePaths(size_t i, int k) const {
  std::vector<std::vector<uint32_t>> out;
  if (k < 1 || k > 2) throw std::invalid_argument("Ksp2Batch: k must be 1 or 2");
  const int64_t u = unitOf_.at(i);
  if (u < 0) return out;
  if (count_[k - 1].empty()) throw std::logic_error("Ksp2Batch: fetch() first");
  const uint32_t n = count_[k - 1][u];
  const uint32_t* len = len_[k - 1].data() + size_t(u) * maxPaths_;
  const uint32_t* e = edges_[k - 1].data() + size_t(u) * maxEdges_;
  for (uint32_t p = 0; p < n; ++p) {
    out.emplace_back(e, e + len[p]);
    e += len[p];
  }
  return out;
}

std::vector<LinkState::Path> Ksp2Batch::paths(size_t i, int k) const {
  const LinkState& ls = *ls_.at(destArea_.at(i));
  const FlatTopology& f = ls.flat();
  std::vector<LinkState::Path> out;
  for (const auto& ep : edgePaths(i, k)) {
    LinkState::Path p;
    for (uint32_t e : ep) p.push_back(ls.linkByKey(f.edgeLink[e]->key()));
    out.push_back(std::move(p));
  }
  return out;
}

uint64_t Ksp2Batch::totalPathEdges(int k) const {
  uint64_t t = 0;
  for (size_t u = 0; u < nUnits_ && !count_[k - 1].empty(); ++u) {
    const uint32_t* len = len_[k - 1].data() + u * maxPaths_;
    for (uint32_t p = 0; p < count_[k - 1][u]; ++p) t += len[p];
  }
  return t;
}

void LinkState::prefetchKthPaths(const std::string& src,
                                 const std::vector<std::string>& dests) const {
  std::vector<std::string> todo;
  for (const auto& d : dests) {
    if (!kthMemo_.count({src, d, 1}) || !kthMemo_.count({src, d, 2})) {
      todo.push_back(d);
    }
  }
  if (todo.empty()) return;
  Ksp2Batch b(*this, src, todo);
  b.launch();
  b.fetch();
  if (b.numUnits()) {
    noteSpf(src);  // k = 1: getSpfResult(src)
    noteSpfRuns(b.numUnits());  // k = 2: one masked runSpf per destination
  }
  for (size_t i = 0; i < todo.size(); ++i) {
    kthMemo_[{src, todo[i], 1}] = b.paths(i, 1);
    kthMemo_[{src, todo[i], 2}] = b.paths(i, 2);
  }
}

}  // namespace openr_amd
