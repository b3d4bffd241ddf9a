// link_state.cpp — ingestion, change detection and CSR flattening for the
// GPU LinkState (reference: openr/decision/LinkState.cpp:50-715).
#include <algorithm>
#include <cstring>
#include <unordered_map>

#include "decision.h"
#include "slot_order.h"

namespace openr_amd {

// ------------------------------------------------------------------ Link --
Link::Link(const std::string& area, const std::string& n1,
           const std::string& if1, const std::string& n2,
           const std::string& if2, bool usable)
    : area_(area), usable_(usable) {
  node_[0] = n1;
  node_[1] = n2;
  if_[0] = if1;
  if_[1] = if2;
  auto a = std::make_pair(n1, if1), b = std::make_pair(n2, if2);
  key_ = a < b ? Key{a, b} : Key{b, a};  // unordered pair of (node, if)
}

Link::Link(const std::string& area, const std::string& n1, const Adjacency& a1,
           const std::string& n2, const Adjacency& a2, bool usable)
    : Link(area, n1, a1.ifName, n2, a2.ifName, usable) {
  const Adjacency* a[2] = {&a1, &a2};
  for (int i = 0; i < 2; ++i) {
    // thrift i32 -> LinkStateMetric (LinkState.cpp:77-78)
    metric_[i] = static_cast<LinkStateMetric>(static_cast<int64_t>(a[i]->metric));
    overload_[i] = a[i]->isOverloaded;
    label_[i] = a[i]->adjLabel;
    weight_[i] = a[i]->weight;
    v4_[i] = a[i]->nextHopV4;
    v6_[i] = a[i]->nextHopV6;
  }
}

bool Link::setOverloadFromNode(const std::string& n, bool ov) {
  const bool wasUp = isUp();  // only up<->down is a topology change
  overload_[side(n)] = ov;
  return wasUp != isUp();
}

bool Link::setLinkUsability(const Link& newLink) {
  if (!(*this == newLink)) throw std::logic_error("setLinkUsability: other link");
  const bool wasUp = isUp();
  usable_ = newLink.usable_;
  return wasUp != isUp();
}

// ------------------------------------------------------------- LinkState --
LinkState::LinkState(const std::string& area, const std::string& me)
    : area_(area), myNodeName_(me) {}
LinkState::LinkState(LinkState&&) noexcept = default;
LinkState::~LinkState() = default;

LinkPtr LinkState::makeLink(const std::string& node, const Adjacency& adj) const {
  // bidirectional only (LinkState.cpp:406-423); usability judged by the
  // LinkState owner (LinkState.h:18-40, 469-473)
  auto it = adjDbs_.find(adj.otherNodeName);
  if (it == adjDbs_.end()) return nullptr;
  for (const auto& rev : it->second.adjacencies) {
    if (rev.otherNodeName != node || rev.ifName != adj.otherIfName ||
        rev.otherIfName != adj.ifName) {
      continue;
    }
    auto usableBy = [&](const Adjacency& a) {
      return !a.adjOnlyUsedByOtherNode || a.otherNodeName == myNodeName_;
    };
    return std::make_shared<Link>(area_, node, adj, adj.otherNodeName, rev,
                                  usableBy(adj) && usableBy(rev));
  }
  return nullptr;
}

void LinkState::clearSpfMemos() const {  // LinkState.cpp:635-638
  spfMemo_.clear();
  spfCounted_.clear();
  kthMemo_.clear();
  deviceSpf_.clear();
  deviceSpfBytes_ = 0;
}

void LinkState::invalidate(bool topologyChanged) {
  ++mutation_;
  flatStale_ = true;
  if (topologyChanged) clearSpfMemos();
}

// device SPF rows memo ------------------------------------------------------
namespace {
// bytes of device SPF rows kept per LinkState before the memo starts over
// (C3: 2,080 sources x 2,080 nodes x (4 + 4 x 3) B = 69 MB)
size_t g_deviceSpfBudget = size_t(1) << 30;
size_t al256(size_t x) { return (x + 255) & ~size_t(255); }
}  // namespace

LinkState::DeviceSpf* LinkState::findDeviceSpf(uint32_t s, bool useLinkMetric, uint32_t N,
                                               int W, size_t db, bool exact) const {
  auto it = deviceSpf_.find(uint64_t(s) << 1 | (useLinkMetric ? 1u : 0u));
  if (it == deviceSpf_.end()) return nullptr;
  DeviceSpf& d = it->second;
  if (!d.valid || d.N != N || d.W != W || d.db != db || d.exact != exact) return nullptr;
  return &d;
}

LinkState::DeviceSpf& LinkState::newDeviceSpf(uint32_t s, bool useLinkMetric, uint32_t N, int W,
                                              size_t db, bool exact) const {
  const uint64_t key = uint64_t(s) << 1 | (useLinkMetric ? 1u : 0u);
  const size_t nhOff = al256(size_t(N) * db);
  const size_t reachOff = nhOff + al256(size_t(N) * W * 4);
  const size_t bytes = reachOff + al256((size_t(N) + 31) / 32 * 4 + 4);
  if (auto it = deviceSpf_.find(key); it != deviceSpf_.end()) {
    deviceSpfBytes_ -= it->second.rows.capacity();
    deviceSpf_.erase(it);
  }
  if (deviceSpfBytes_ + bytes > g_deviceSpfBudget) {  // over budget: start over
    deviceSpf_.clear();
    deviceSpfBytes_ = 0;
  }
  DeviceSpf& d = deviceSpf_[key];
  d.rows.resize(bytes);
  deviceSpfBytes_ += d.rows.capacity();
  d.N = N;
  d.W = W;
  d.db = db;
  d.nhOff = nhOff;
  d.reachOff = reachOff;
  d.exact = exact;
  d.valid = false;
  return d;
}

void LinkState::commitDeviceSpf(DeviceSpf& slot, const std::string& node,
                                bool useLinkMetric) const {
  slot.valid = true;
  ++deviceSpfLaunches_;
  addStatValue("decision.gpu.spf_launches", 1, StatType::COUNT);
  noteSpf(node, useLinkMetric);
}

LinkState::LinkStateChange LinkState::updateAdjacencyDatabase(
    const AdjacencyDatabase& db, const std::string& /*area*/,
    bool /*inInitialization*/) {
  LinkStateChange ch;
  const std::string name = db.thisNodeName;
  AdjacencyDatabase prior;
  // §8(f) f3: a known node whose link set is unchanged only moves link /
  // node attributes -> patch the CSR in place (patchFlat)
  bool structural = true;
  if (auto it = adjDbs_.find(name); it != adjDbs_.end()) {
    prior = it->second;
    structural = false;
  }
  std::vector<const Link*> touched;
  bool nodeFlagsChanged = false;
  adjDbs_[name] = db;

  std::map<Link::Key, LinkPtr> fresh;
  for (const auto& adj : db.adjacencies) {
    if (auto l = makeLink(name, adj)) fresh.emplace(l->key(), l);
  }

  // node hard-drain: a change (not a first sighting) moves the topology
  {
    auto it = overloaded_.find(name);
    if (it == overloaded_.end()) {
      overloaded_[name] = db.isOverloaded;
    } else if (it->second != db.isOverloaded) {
      it->second = db.isOverloaded;
      ch.topologyChanged = true;
      nodeFlagsChanged = true;
    }
  }
  nodeFlagsChanged |= prior.nodeMetricIncrementVal != db.nodeMetricIncrementVal;
  ch.topologyChanged |= prior.nodeMetricIncrementVal != db.nodeMetricIncrementVal;
  metricInc_[name] =
      static_cast<uint64_t>(static_cast<int64_t>(db.nodeMetricIncrementVal));
  ch.nodeLabelChanged = prior.nodeLabel != db.nodeLabel;

  // merge old vs new link sets, both in key order
  std::vector<Link::Key> oldKeys;
  if (auto it = byNode_.find(name); it != byNode_.end()) {
    oldKeys.reserve(it->second.size());
    for (const auto& [k, _] : it->second) oldKeys.push_back(k);
  }
  auto ni = fresh.begin();
  size_t oi = 0;
  while (ni != fresh.end() || oi < oldKeys.size()) {
    if (ni != fresh.end() && (oi == oldKeys.size() || ni->first < oldKeys[oi])) {
      const LinkPtr& l = ni->second;
      ch.topologyChanged |= l->isUp();
      links_[l->key()] = l;
      byNode_[l->firstNodeName()].emplace(l->key(), l);
      byNode_[l->secondNodeName()].emplace(l->key(), l);
      ch.addedLinks.push_back(l);
      structural = true;
      ++ni;
      continue;
    }
    if (oi < oldKeys.size() && (ni == fresh.end() || oldKeys[oi] < ni->first)) {
      const LinkPtr l = links_.at(oldKeys[oi]);
      ch.topologyChanged |= l->isUp();
      byNode_.at(l->firstNodeName()).erase(l->key());
      byNode_.at(l->secondNodeName()).erase(l->key());
      links_.erase(l->key());
      structural = true;
      ++oi;
      continue;
    }
    Link& nl = *ni->second;
    Link& ol = *links_.at(oldKeys[oi]);
    if (nl.getMetricFromNode(name) != ol.getMetricFromNode(name) ||
        nl.isUp() != ol.isUp() ||
        nl.getOverloadFromNode(name) != ol.getOverloadFromNode(name)) {
      touched.push_back(&ol);
    }
    if (nl.getMetricFromNode(name) != ol.getMetricFromNode(name)) {
      ch.topologyChanged |= ol.setMetricFromNode(name, nl.getMetricFromNode(name));
    }
    if (nl.isUp() != ol.isUp()) ch.topologyChanged |= ol.setLinkUsability(nl);
    if (nl.getOverloadFromNode(name) != ol.getOverloadFromNode(name)) {
      ch.topologyChanged |=
          ol.setOverloadFromNode(name, nl.getOverloadFromNode(name));
    }
    if (nl.getAdjLabelFromNode(name) != ol.getAdjLabelFromNode(name)) {
      ch.linkAttributesChanged = true;
      ol.setAdjLabelFromNode(name, nl.getAdjLabelFromNode(name));
    }
    if (nl.getWeightFromNode(name) != ol.getWeightFromNode(name)) {
      ch.linkAttributesChanged = true;
      ol.setWeightFromNode(name, nl.getWeightFromNode(name));
    }
    if (nl.getNhV4FromNode(name) != ol.getNhV4FromNode(name)) {
      ch.linkAttributesChanged = true;
      ol.setNhV4FromNode(name, nl.getNhV4FromNode(name));
    }
    if (nl.getNhV6FromNode(name) != ol.getNhV6FromNode(name)) {
      ch.linkAttributesChanged = true;
      ol.setNhV6FromNode(name, nl.getNhV6FromNode(name));
    }
    ++ni;
    ++oi;
  }
  if (!structural && incrementalFlatten_ && flat_ && !flatStale_) {
    patchFlat(name, touched, nodeFlagsChanged);
    if (ch.topologyChanged) clearSpfMemos();  // LinkState.cpp:635-638
  } else {
    invalidate(ch.topologyChanged);
  }
  return ch;
}

void LinkState::patchFlat(const std::string& node, const std::vector<const Link*>& touched,
                          bool nodeFlagsChanged) {
  FlatTopology& f = *flat_;
  ++mutation_;
  f.version = nextVersionStamp();  // version-keyed caches (prefix tables, policies) rebuild
  ++flatPatches_;
  const uint32_t u = f.id.at(node);
  std::vector<uint32_t> dirty;
  // same encoding as flat(): keep dst + rslot, recompute the rest
  auto reencode = [&](uint32_t e) {
    const Link* l = f.edgeLink[e];
    const uint64_t old = f.edges[e];
    const uint32_t keep = OGS_EDGE_DST_MASK | (OGS_EDGE_RSLOT_MASK << OGS_EDGE_RSLOT_SHIFT);
    uint32_t lo = uint32_t(old) & keep;
    if (isNodeOverloaded(f.names[lo & OGS_EDGE_DST_MASK])) lo |= OGS_EDGE_DST_OVERLOADED;
    if (!l->isUp()) lo |= OGS_EDGE_DOWN;
    const uint64_t w = uint64_t(lo) | (uint64_t(uint32_t(l->getMaxMetric())) << 32);
    if (w != old) {
      f.edges[e] = w;
      dirty.push_back(e);
    }
  };
  auto reverseOf = [&](uint32_t e) {
    const uint32_t lo = uint32_t(f.edges[e]);
    const uint32_t slot = f.rslotExt.empty() ? (lo >> OGS_EDGE_RSLOT_SHIFT) & OGS_EDGE_RSLOT_MASK
                                             : f.rslotExt[e];
    return f.rowPtr[lo & OGS_EDGE_DST_MASK] + slot;
  };
  for (uint32_t e = f.rowPtr[u]; e < f.rowPtr[u + 1]; ++e) {
    const bool linkTouched =
        std::find(touched.begin(), touched.end(), f.edgeLink[e]) != touched.end();
    // an overload flip of `node` changes DST_OVERLOADED on every edge into it
    if (linkTouched || nodeFlagsChanged) {
      reencode(e);
      reencode(reverseOf(e));
    }
  }
  bool flagsDirty = false;
  if (nodeFlagsChanged) {
    uint8_t fl = 0;
    if (isNodeOverloaded(node)) fl |= OGS_NODE_OVERLOADED;
    const uint64_t inc = getNodeMetricIncrement(node);
    if (static_cast<int>(inc) > 0) fl |= OGS_NODE_SOFTDRAIN;
    if (inc != 0) fl |= OGS_NODE_METRICINC;
    flagsDirty = fl != f.nodeFlags[u];
    f.nodeFlags[u] = fl;
  }
  if (!dirty.empty()) {  // the domain checks of flat() over the up links
    f.maxMetric = 0;
    f.hasZeroMetric = f.hasWideMetric = false;
    for (const Link* l : f.edgeLink) {
      if (!l->isUp()) continue;
      const LinkStateMetric m = l->getMaxMetric();
      f.maxMetric = std::max(f.maxMetric, m);
      if (m == 0) f.hasZeroMetric = true;
      if (m > 0xFFFFFFFFull) f.hasWideMetric = true;
    }
  }
  edgesPatched_ += dirty.size();
  if (deviceStale_) return;  // the next flatOnDevice() uploads everything
  if (!dirty.empty()) {
    std::vector<uint64_t> val(dirty.size());
    for (size_t i = 0; i < dirty.size(); ++i) val[i] = f.edges[dirty[i]];
    f.dPatchIdx.upload(dirty.data(), dirty.size());
    f.dPatchVal.upload(val.data(), val.size());
    ogsCheck(ogs_csr_patch(f.dEdges.as<uint64_t>(), f.dPatchIdx.as<uint32_t>(),
                           f.dPatchVal.as<uint64_t>(), int32_t(dirty.size()), nullptr),
             "ogs_csr_patch");
  }
  if (flagsDirty) f.dFlags.upload(f.nodeFlags.data(), f.nodeFlags.size());
  if (!dirty.empty() && f.slotStride) uploadSlotImages(f);
}

LinkState::LinkStateChange LinkState::deleteAdjacencyDatabase(
    const std::string& name) {  // LinkState.cpp:642-659
  LinkStateChange ch;
  auto it = adjDbs_.find(name);
  if (it == adjDbs_.end()) return ch;
  if (auto bn = byNode_.find(name); bn != byNode_.end()) {
    std::vector<Link::Key> keys;
    for (const auto& [k, _] : bn->second) keys.push_back(k);
    for (const auto& key : keys) {
      const LinkPtr l = links_.at(key);
      byNode_.at(l->getOtherNodeName(name)).erase(key);
      links_.erase(key);
    }
    byNode_.erase(name);
    overloaded_.erase(name);
  }
  adjDbs_.erase(it);
  ch.topologyChanged = true;
  invalidate(true);
  return ch;
}

std::vector<LinkPtr> LinkState::linksFromNode(const std::string& n) const {
  std::vector<LinkPtr> out;
  if (auto it = byNode_.find(n); it != byNode_.end()) {
    for (const auto& [_, l] : it->second) out.push_back(l);
  }
  return out;
}

size_t LinkState::numNodes() const { return byNode_.size(); }

bool LinkState::isNodeOverloaded(const std::string& n) const {
  auto it = overloaded_.find(n);
  return it != overloaded_.end() && it->second;
}

uint64_t LinkState::getNodeMetricIncrement(const std::string& n) const {
  auto it = metricInc_.find(n);
  return it == metricInc_.end() ? 0 : it->second;
}

bool LinkState::pathAInPathB(const Path& a, const Path& b) {
  if (a.size() > b.size()) return false;  // LinkState.h:488-503
  for (size_t i = 0; i + a.size() <= b.size(); ++i) {
    size_t k = 0;
    while (k < a.size() && *a[k] == *b[i + k]) ++k;
    if (k == a.size()) return true;
  }
  return false;
}

// ------------------------------------------------------------ flattening --
const FlatTopology& LinkState::flat() const {
  if (flat_ && !flatStale_) return *flat_;
  // node ids are ranks of the current names: rows of the device SPF memo
  // are indexed by the old ones
  deviceSpf_.clear();
  deviceSpfBytes_ = 0;
  auto f = std::make_unique<FlatTopology>();
  f->version = nextVersionStamp();
  f->names.reserve(adjDbs_.size());
  f->id.reserve(adjDbs_.size());
  f->nodeFlags.reserve(adjDbs_.size());
  for (const auto& [n, db] : adjDbs_) {  // byte-wise name order == id order
    f->id.emplace(n, uint32_t(f->names.size()));
    f->names.push_back(n);
    // the node's flags straight from its adjacency database (overloaded_ /
    // metricInc_ mirror these fields, set by updateAdjacencyDatabase)
    uint8_t fl = db.isOverloaded ? OGS_NODE_OVERLOADED : 0;
    const int64_t inc = db.nodeMetricIncrementVal;
    if (static_cast<int>(static_cast<uint64_t>(inc)) > 0) fl |= OGS_NODE_SOFTDRAIN;
    if (inc != 0) fl |= OGS_NODE_METRICINC;
    f->nodeFlags.push_back(fl);
  }
  const uint32_t N = uint32_t(f->names.size());
  if (N > OGS_MAX_NODES_PER_TOPO) throw std::domain_error("too many nodes");
  // Rows in canonical link order straight from links_ (key order): every
  // link is appended to both endpoint rows, so each row is a subsequence of
  // the sorted link sequence (the order of byNode_'s key-ordered sets), and
  // a link's two directed edges are placed together -- the reverse of every
  // edge is known without a sort or a string-keyed lookup per edge.
  f->rowPtr.assign(N + 1, 0);
  // links_ is ordered by (first node, ...) and names by name: the first
  // endpoint's id follows a cursor; only the second is looked up
  struct End {
    const Link* l;
    uint32_t a, b;
  };
  std::vector<End> ends;
  ends.reserve(links_.size());
  uint32_t cur = 0;
  for (const auto& [_, lp] : links_) {
    const std::string& n1 = lp->firstNodeName();
    while (cur < N && f->names[cur] < n1) ++cur;
    const auto b = f->id.find(lp->secondNodeName());
    if (cur == N || f->names[cur] != n1 || b == f->id.end() || b->second == cur) {
      throw std::logic_error("LinkState::flat: link with one endpoint");
    }
    ends.push_back(End{lp.get(), cur, b->second});
    ++f->rowPtr[cur + 1];
    ++f->rowPtr[b->second + 1];
  }
  for (uint32_t u = 0; u < N; ++u) {
    f->maxDegree = std::max<int>(f->maxDegree, int(f->rowPtr[u + 1]));
    f->rowPtr[u + 1] += f->rowPtr[u];
  }
  // rows of 512+ edges (a hub / route reflector): the edge word's reverse
  // slot saturates at 511 and the exact slots go to rslotExt (LinkState.cpp:
  // 760-813 iterates links of any count)
  const bool extSlots = f->maxDegree >= OGS_MAX_DEGREE;
  const uint32_t E = f->rowPtr[N];
  if (extSlots) f->rslotExt.assign(E, 0u);
  f->edgeLink.assign(E, nullptr);
  std::vector<uint32_t> owner(E), rev(E);
  {
    std::vector<uint32_t> pos(f->rowPtr.begin(), f->rowPtr.end() - 1);
    for (const End& x : ends) {
      const uint32_t a = x.a, b = x.b;
      const uint32_t ea = pos[a]++, eb = pos[b]++;
      f->edgeLink[ea] = f->edgeLink[eb] = const_cast<Link*>(x.l);
      owner[ea] = a;
      owner[eb] = b;
      rev[ea] = eb;
      rev[eb] = ea;
    }
  }
  f->edges.resize(E);
  for (uint32_t e = 0; e < E; ++e) {
    const Link* l = f->edgeLink[e];
    const uint32_t r = rev[e];
    const uint32_t v = owner[r];
    const uint32_t rslot = r - f->rowPtr[v];
    if (extSlots) f->rslotExt[e] = rslot;
    const LinkStateMetric m = l->getMaxMetric();
    uint32_t lo = v | (std::min<uint32_t>(rslot, OGS_EDGE_RSLOT_MASK) << OGS_EDGE_RSLOT_SHIFT);
    if (f->nodeFlags[v] & OGS_NODE_OVERLOADED) lo |= OGS_EDGE_DST_OVERLOADED;
    const bool up = l->isUp();
    if (!up) lo |= OGS_EDGE_DOWN;
    if (up) {
      f->maxMetric = std::max(f->maxMetric, m);
      if (m == 0) f->hasZeroMetric = true;
      if (m > 0xFFFFFFFFull) f->hasWideMetric = true;
    }
    f->edges[e] = uint64_t(lo) | (uint64_t(uint32_t(m)) << 32);
  }
  flat_ = std::move(f);
  flatStale_ = false;
  deviceStale_ = true;
  ++flatBuilds_;
  return *flat_;
}

const FlatTopology& LinkState::flatOnDevice() const {
  const FlatTopology& f = flat();
  if (!deviceStale_) return f;
  FlatTopology& m = *flat_;
  // every device image of the CSR packed into one block: one H2D
  const uint32_t N = uint32_t(m.names.size());
  const size_t E = m.edges.size();
  const uint32_t nodeBase[2] = {0, N};
  std::vector<uint32_t> esrc;
  esrc.reserve(E);
  for (uint32_t v = 0; v < N; ++v) esrc.insert(esrc.end(), m.rowPtr[v + 1] - m.rowPtr[v], v);
  std::vector<uint16_t> slots;
  std::vector<uint32_t> img;
  slotImages(m, slots, img);
  struct Span {
    const void* src;
    size_t bytes;
    DeviceBuffer* dst;
  };
  const Span spans[] = {{nodeBase, sizeof nodeBase, &m.dNodeBase},
                        {m.rowPtr.data(), m.rowPtr.size() * 4, &m.dRow},
                        {m.edges.data(), E * 8, &m.dEdges},
                        {m.nodeFlags.data(), m.nodeFlags.size(), &m.dFlags},
                        {esrc.data(), esrc.size() * 4, &m.dEdgeSrc},
                        {slots.data(), slots.size() * 2, &m.dSlot},
                        {img.data(), img.size() * 4, &m.dSlotEdges},
                        {m.rslotExt.data(), m.rslotExt.size() * 4, &m.dRslotExt}};
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  size_t total = 0;
  for (const Span& sp : spans) total += al(std::max<size_t>(sp.bytes, 16));
  std::vector<char> host(total);
  size_t off = 0;
  for (const Span& sp : spans) {
    if (sp.bytes) std::memcpy(host.data() + off, sp.src, sp.bytes);
    off += al(std::max<size_t>(sp.bytes, 16));
  }
  m.dBlock.resize(total);
  ogsCheck(ogs_memcpy_h2d(m.dBlock.get(), host.data(), total, nullptr), "ogs_memcpy_h2d");
  off = 0;
  for (const Span& sp : spans) {
    sp.dst->view(static_cast<char*>(m.dBlock.get()) + off, std::max<size_t>(sp.bytes, 16));
    off += al(std::max<size_t>(sp.bytes, 16));
  }
  deviceStale_ = false;
  return f;
}

// host images of the wave-kernel relaxation order and per-slot edges
// (slot_order.h); sets m.slotStride / m.slotDegree (0: none)
void LinkState::slotImages(FlatTopology& m, std::vector<uint16_t>& slots,
                           std::vector<uint32_t>& img) const {
  slots.clear();
  img.clear();
  m.slotStride = slotStrideFor(int(m.names.size()));
  m.slotDegree = 0;
  if (!m.slotStride) return;
  slots.resize(m.slotStride);
  placeSlots(colorNodes(m.rowPtr.data(), m.edges.data(), uint32_t(m.names.size())),
             m.slotStride, slots.data());
  m.slotDegree = slotDegreeFor(m.maxDegree, m.maxMetric, m.slotStride);
  if (m.slotDegree) {
    img.resize(size_t(m.slotDegree) * m.slotStride);
    placeSlotEdges(slots.data(), m.slotStride, m.rowPtr.data(), m.edges.data(),
                   uint32_t(m.names.size()), m.slotDegree, img.data());
  }
}

// wave-kernel relaxation order + per-slot edge image (slot_order.h); the
// image carries edge weights, so a patched CSR re-derives it
void LinkState::uploadSlotImages(FlatTopology& m) const {
  std::vector<uint16_t> slots;
  std::vector<uint32_t> img;
  slotImages(m, slots, img);
  if (m.slotStride) m.dSlot.upload(slots.data(), slots.size());
  if (m.slotDegree) m.dSlotEdges.upload(img.data(), img.size());
}

// ------------------------------------------------------------------- SPF --
namespace {
// Shared scratch for single-source launches made through the API surface.
struct SpfScratch {
  DeviceBuffer unit;
};
SpfScratch& scratch() {
  static SpfScratch s;
  return s;
}

bool needsWide(const FlatTopology& f, bool useLinkMetric) {
  if (!useLinkMetric) return false;
  const uint64_t n = f.names.empty() ? 0 : f.names.size() - 1;
  return f.maxMetric != 0 && n != 0 &&
      f.maxMetric > (0x7FFFFFFEull / n);
}
}  // namespace

const LinkState::SpfResult& LinkState::getSpfResult(const std::string& node,
                                                    bool useLinkMetric) const {
  auto key = std::make_pair(node, useLinkMetric);
  if (auto it = spfMemo_.find(key); it != spfMemo_.end()) return it->second;

  SpfResult res;
  const auto t0 = std::chrono::steady_clock::now();  // decision.spf_ms (LinkState.cpp:818)
  const FlatTopology& f = flatOnDevice();
  auto idIt = f.id.find(node);
  noteSpf(node, useLinkMetric);
  if (idIt == f.id.end()) {
    res.emplace(node, NodeSpfResult(0));  // unknown source settles only itself
    addStatValue("decision.spf_ms", msSince(t0), StatType::AVG);
    return spfMemo_.emplace(key, std::move(res)).first->second;
  }
  // zero / negative link metrics: the reference's extraction order replayed
  // on the device (spf_exact.hip, OGS_F_EXACT_ORDER), 64-bit distances
  const bool exact = useLinkMetric && (f.hasZeroMetric || f.hasWideMetric);
  const uint32_t s = idIt->second;
  const uint32_t N = uint32_t(f.names.size());
  const int degree = int(f.rowPtr[s + 1] - f.rowPtr[s]);
  const int W = std::max(1, ogs_nh_words_for_degree(degree));
  const bool wide = exact || needsWide(f, useLinkMetric);
  const size_t db = wide ? 8 : 4;

  // the device rows memo (shared with buildRouteDb): D2H of rows already on
  // the device, else ONE SPF launch into a new slot
  DeviceSpf* memo = findDeviceSpf(s, useLinkMetric, N, W, db, exact);
  if (!memo) {
    auto& sc = scratch();
    const ogs_unit u{0, s};
    sc.unit.upload(&u, 1);
    DeviceSpf& slot = newDeviceSpf(s, useLinkMetric, N, W, db, exact);
    ogs_graph g{};
    g.num_topos = 1;
    g.max_nodes = int32_t(N);
    g.max_edges = int32_t(f.edges.size());
    g.max_degree = f.maxDegree;
    g.node_base = f.dNodeBase.as<uint32_t>();
    g.row_ptr = f.dRow.as<uint32_t>();
    g.edges = f.dEdges.as<uint64_t>();
    g.node_flags = f.dFlags.as<uint8_t>();
    g.slot_node = f.slotStride ? f.dSlot.as<uint16_t>() : nullptr;
    g.slot_stride = f.slotStride;
    g.slot_edges = f.slotDegree ? f.dSlotEdges.as<uint32_t>() : nullptr;
    g.slot_degree = f.slotDegree;
    g.edge_src = f.dEdgeSrc.as<uint32_t>();
    ogs_spf_out out{};
    out.dist = slot.dist();
    out.nh = slot.nh();
    out.reached = exact ? slot.reach() : nullptr;
    uint32_t flags = (useLinkMetric ? 0u : OGS_F_HOP_METRIC) |
        (wide ? OGS_F_WIDE_METRIC : 0u) | (exact ? OGS_F_EXACT_ORDER : 0u);
    ogsCheck(ogs_spf_routes(&g, nullptr, sc.unit.as<ogs_unit>(), 1, flags, W,
                            &out, nullptr),
             "ogs_spf_routes");
    commitDeviceSpf(slot, node, useLinkMetric);
    memo = &slot;
  }
  std::vector<uint64_t> dist(N);
  std::vector<uint32_t> nh(size_t(N) * W);
  if (wide) {
    ogsCheck(ogs_memcpy_d2h(dist.data(), memo->dist(), size_t(N) * 8, nullptr), "ogs_memcpy_d2h");
  } else {
    std::vector<uint32_t> d32(N);
    ogsCheck(ogs_memcpy_d2h(d32.data(), memo->dist(), size_t(N) * 4, nullptr), "ogs_memcpy_d2h");
    ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");
    for (uint32_t v = 0; v < N; ++v) {
      dist[v] = d32[v] == 0xFFFFFFFFu ? ~0ull : d32[v];
    }
  }
  ogsCheck(ogs_memcpy_d2h(nh.data(), memo->nh(), nh.size() * 4, nullptr), "ogs_memcpy_d2h");
  // exact order: the settled bitset decides reachability (a wrapped u64
  // distance of a settled node may be all ones, kept by the reference)
  std::vector<uint32_t> reach(exact ? (size_t(N) + 31) / 32 : 0);
  if (exact) {
    ogsCheck(ogs_memcpy_d2h(reach.data(), memo->reach(), reach.size() * 4, nullptr),
             "ogs_memcpy_d2h");
  }
  ogsCheck(ogs_stream_sync(nullptr), "ogs_stream_sync");

  const uint32_t rb = f.rowPtr[s];
  for (uint32_t v = 0; v < N; ++v) {
    if (exact ? !bitAt(reach.data(), v) : dist[v] == ~0ull) continue;
    NodeSpfResult r(dist[v]);
    for (int w = 0; w < W; ++w) {
      uint32_t bits = nh[size_t(w) * N + v];
      while (bits) {
        const int b = __builtin_ctz(bits);
        bits &= bits - 1;
        const Link* l = f.edgeLink[rb + w * 32 + b];
        r.addNextHop(l->getOtherNodeName(node));
      }
    }
    res.emplace(f.names[v], std::move(r));
  }
  addStatValue("decision.spf_ms", msSince(t0), StatType::AVG);
  return spfMemo_.emplace(key, std::move(res)).first->second;
}

std::optional<LinkStateMetric> LinkState::getMetricFromAToB(
    const std::string& a, const std::string& b, bool useLinkMetric) const {
  if (a == b) return 0;  // LinkState.cpp:661-672
  const auto& r = getSpfResult(a, useLinkMetric);
  auto it = r.find(b);
  if (it == r.end()) return std::nullopt;
  return it->second.metric();
}

}  // namespace openr_amd
