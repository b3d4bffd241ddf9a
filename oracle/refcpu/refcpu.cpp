// refcpu — CPU ORACLE (test infrastructure only; see refcpu.h header).
#include "refcpu.h"

#include <arpa/inet.h>

#include <algorithm>
#include <stdexcept>

namespace refcpu {

// ===================== Link (LinkState.cpp:50-188) ==========================
Link::Link(const std::string& area, const std::string& n1,
           const std::string& if1, const std::string& n2,
           const std::string& if2, bool usable)
    : area_(area), n1_(n1), n2_(n2), if1_(if1), if2_(if2), usable_(usable) {
  auto a = std::make_pair(n1, if1);
  auto b = std::make_pair(n2, if2);
  ordered_ = a < b ? std::make_pair(a, b) : std::make_pair(b, a);
}

Link::Link(const std::string& area, const std::string& n1, const Adjacency& a1,
           const std::string& n2, const Adjacency& a2, bool usable)
    : Link(area, n1, a1.ifName, n2, a2.ifName, usable) {
  // i32 metric -> uint64 (LinkState.cpp:77-78): negative sign-extends
  metric1_ = static_cast<Metric>(static_cast<int64_t>(a1.metric));
  metric2_ = static_cast<Metric>(static_cast<int64_t>(a2.metric));
  overload1_ = a1.isOverloaded;
  overload2_ = a2.isOverloaded;
  adjLabel1_ = a1.adjLabel;
  adjLabel2_ = a2.adjLabel;
  nhV41_ = a1.nextHopV4;
  nhV42_ = a2.nextHopV4;
  nhV61_ = a1.nextHopV6;
  nhV62_ = a2.nextHopV6;
  weight1_ = a1.weight;
  weight2_ = a2.weight;
}

#define REFCPU_SIDE(n, a, b)            \
  if (n1_ == (n)) return a;             \
  if (n2_ == (n)) return b;             \
  throw std::invalid_argument(n);

const std::string& Link::getOtherNodeName(const std::string& n) const {
  REFCPU_SIDE(n, n2_, n1_)
}
const std::string& Link::getIfaceFromNode(const std::string& n) const {
  REFCPU_SIDE(n, if1_, if2_)
}
Metric Link::getMetricFromNode(const std::string& n) const {
  REFCPU_SIDE(n, metric1_, metric2_)
}
int32_t Link::getAdjLabelFromNode(const std::string& n) const {
  REFCPU_SIDE(n, adjLabel1_, adjLabel2_)
}
int64_t Link::getWeightFromNode(const std::string& n) const {
  REFCPU_SIDE(n, weight1_, weight2_)
}
bool Link::getOverloadFromNode(const std::string& n) const {
  REFCPU_SIDE(n, overload1_, overload2_)
}
const std::string& Link::getNhV4FromNode(const std::string& n) const {
  REFCPU_SIDE(n, nhV41_, nhV42_)
}
const std::string& Link::getNhV6FromNode(const std::string& n) const {
  REFCPU_SIDE(n, nhV61_, nhV62_)
}
#undef REFCPU_SIDE

#define REFCPU_SET(n, a, b, v) \
  if (n1_ == (n)) {            \
    a = v;                     \
  } else if (n2_ == (n)) {     \
    b = v;                     \
  } else {                     \
    throw std::invalid_argument(n); \
  }

void Link::setNhV4FromNode(const std::string& n, const std::string& v) {
  REFCPU_SET(n, nhV41_, nhV42_, v)
}
void Link::setNhV6FromNode(const std::string& n, const std::string& v) {
  REFCPU_SET(n, nhV61_, nhV62_, v)
}
bool Link::setMetricFromNode(const std::string& n, Metric d) {
  REFCPU_SET(n, metric1_, metric2_, d)
  return true;
}
void Link::setAdjLabelFromNode(const std::string& n, int32_t l) {
  REFCPU_SET(n, adjLabel1_, adjLabel2_, l)
}
void Link::setWeightFromNode(const std::string& n, int64_t w) {
  REFCPU_SET(n, weight1_, weight2_, w)
}
bool Link::setOverloadFromNode(const std::string& n, bool ov) {
  // LinkState.cpp:149-162: only an up/down transition is a topology change
  const bool wasUp = isUp();
  REFCPU_SET(n, overload1_, overload2_, ov)
  return wasUp != isUp();
}
#undef REFCPU_SET

bool Link::setLinkUsability(const Link& newLink) {  // LinkState.cpp:164-172
  if (!(*this == newLink)) throw std::logic_error("setLinkUsability");
  const bool wasUp = isUp();
  usable_ = newLink.usable_;
  return wasUp != isUp();
}

// ===================== LinkState ============================================
bool LinkState::linkUsable(const Adjacency& a1, const Adjacency& a2) const {
  // LinkState.h:18-40 adjUsable, 469-473 linkUsable: judged by the OWNER
  auto usable = [&](const Adjacency& a) {
    return !(a.adjOnlyUsedByOtherNode && a.otherNodeName != myNodeName_);
  };
  return usable(a1) && usable(a2);
}

std::optional<LinkState::Path> LinkState::traceOnePath(
    const std::string& src, const std::string& dest, const SpfResult& result,
    LinkSet& linksToIgnore) const {
  // LinkState.cpp:226-247 greedy DFS; links stay marked once visited
  if (src == dest) return Path{};
  const auto& nodeResult = result.at(dest);
  for (const auto& pl : nodeResult.pathLinks()) {
    if (linksToIgnore.insert(pl.link).second) {
      auto path = traceOnePath(src, pl.prevNode, result, linksToIgnore);
      if (path) {
        path->push_back(pl.link);
        return path;
      }
    }
  }
  return std::nullopt;
}

void LinkState::addLink(const LinkPtr& l) {  // LinkState.cpp:249-254
  if (!linkMap_[l->firstNodeName()].insert(l).second ||
      !linkMap_[l->secondNodeName()].insert(l).second ||
      !allLinks_.insert(l).second) {
    throw std::logic_error("addLink: duplicate");
  }
}

void LinkState::removeLink(const LinkPtr& l) {  // LinkState.cpp:257-262
  if (!linkMap_.at(l->firstNodeName()).erase(l) ||
      !linkMap_.at(l->secondNodeName()).erase(l) || !allLinks_.erase(l)) {
    throw std::logic_error("removeLink: missing");
  }
}

void LinkState::removeNode(const std::string& n) {  // LinkState.cpp:264-283
  auto it = linkMap_.find(n);
  if (it == linkMap_.end()) return;
  for (const auto& l : it->second) {
    linkMap_.at(l->getOtherNodeName(n)).erase(l);
    allLinks_.erase(l);
  }
  linkMap_.erase(it);
  nodeOverloads_.erase(n);
}

const LinkSet& LinkState::linksFromNode(const std::string& n) const {
  static const LinkSet kEmpty;
  auto it = linkMap_.find(n);
  return it == linkMap_.end() ? kEmpty : it->second;
}

std::vector<LinkPtr> LinkState::orderedLinksFromNode(
    const std::string& n) const {
  const auto& s = linksFromNode(n);
  return std::vector<LinkPtr>(s.begin(), s.end());  // already ordered
}

bool LinkState::updateNodeOverloaded(const std::string& n, bool ov) {
  // LinkState.cpp:308-333: no change reported for a new node or a duplicate
  auto it = nodeOverloads_.find(n);
  if (it != nodeOverloads_.end() && it->second == ov) return false;
  const bool inserted = (it == nodeOverloads_.end());
  nodeOverloads_[n] = ov;
  return !inserted;
}

bool LinkState::isNodeOverloaded(const std::string& n) const {
  auto it = nodeOverloads_.find(n);
  return it != nodeOverloads_.end() && it->second;
}

uint64_t LinkState::getNodeMetricIncrement(const std::string& n) const {
  auto it = nodeMetricIncrementVals_.find(n);
  return it == nodeMetricIncrementVals_.end() ? 0 : it->second;
}

LinkPtr LinkState::maybeMakeLink(const std::string& node,
                                 const Adjacency& adj) const {
  // LinkState.cpp:406-423: bidirectional iff the reverse adjacency exists
  auto it = adjacencyDatabases_.find(adj.otherNodeName);
  if (it == adjacencyDatabases_.end()) return nullptr;
  for (const auto& other : it->second.adjacencies) {
    if (node == other.otherNodeName && adj.otherIfName == other.ifName &&
        adj.ifName == other.otherIfName) {
      return std::make_shared<Link>(area_, node, adj, adj.otherNodeName, other,
                                    linkUsable(adj, other));
    }
  }
  return nullptr;
}

std::vector<LinkPtr> LinkState::getOrderedLinkSet(
    const AdjacencyDatabase& db) const {  // LinkState.cpp:425-438
  std::vector<LinkPtr> links;
  for (const auto& adj : db.adjacencies) {
    if (auto l = maybeMakeLink(db.thisNodeName, adj)) links.push_back(l);
  }
  std::sort(links.begin(), links.end(), LinkPtrLess{});
  return links;
}

LinkState::LinkStateChange LinkState::updateAdjacencyDatabase(
    const AdjacencyDatabase& newDb, const std::string& /*area*/,
    bool /*inInitialization*/) {
  // LinkState.cpp:440-640
  LinkStateChange change;
  const std::string nodeName = newDb.thisNodeName;
  AdjacencyDatabase prior = std::move(adjacencyDatabases_[nodeName]);
  adjacencyDatabases_[nodeName] = newDb;

  auto oldLinks = orderedLinksFromNode(nodeName);
  auto newLinks = getOrderedLinkSet(newDb);

  change.topologyChanged |= updateNodeOverloaded(nodeName, newDb.isOverloaded);
  change.topologyChanged |=
      prior.nodeMetricIncrementVal != newDb.nodeMetricIncrementVal;
  nodeMetricIncrementVals_[nodeName] =
      static_cast<uint64_t>(static_cast<int64_t>(newDb.nodeMetricIncrementVal));
  change.nodeLabelChanged = prior.nodeLabel != newDb.nodeLabel;

  size_t ni = 0, oi = 0;
  while (ni < newLinks.size() || oi < oldLinks.size()) {
    if (ni < newLinks.size() &&
        (oi == oldLinks.size() || *newLinks[ni] < *oldLinks[oi])) {
      change.topologyChanged |= newLinks[ni]->isUp();
      addLink(newLinks[ni]);
      change.addedLinks.push_back(newLinks[ni]);
      ++ni;
      continue;
    }
    if (oi < oldLinks.size() &&
        (ni == newLinks.size() || *oldLinks[oi] < *newLinks[ni])) {
      change.topologyChanged |= oldLinks[oi]->isUp();
      removeLink(oldLinks[oi]);
      ++oi;
      continue;
    }
    Link& nl = *newLinks[ni];
    Link& ol = *oldLinks[oi];
    if (nl.getMetricFromNode(nodeName) != ol.getMetricFromNode(nodeName)) {
      change.topologyChanged |=
          ol.setMetricFromNode(nodeName, nl.getMetricFromNode(nodeName));
    }
    if (nl.isUp() != ol.isUp()) {
      change.topologyChanged |= ol.setLinkUsability(nl);
    }
    if (nl.getOverloadFromNode(nodeName) != ol.getOverloadFromNode(nodeName)) {
      change.topologyChanged |=
          ol.setOverloadFromNode(nodeName, nl.getOverloadFromNode(nodeName));
    }
    if (nl.getAdjLabelFromNode(nodeName) != ol.getAdjLabelFromNode(nodeName)) {
      change.linkAttributesChanged = true;
      ol.setAdjLabelFromNode(nodeName, nl.getAdjLabelFromNode(nodeName));
    }
    if (nl.getWeightFromNode(nodeName) != ol.getWeightFromNode(nodeName)) {
      change.linkAttributesChanged = true;
      ol.setWeightFromNode(nodeName, nl.getWeightFromNode(nodeName));
    }
    if (nl.getNhV4FromNode(nodeName) != ol.getNhV4FromNode(nodeName)) {
      change.linkAttributesChanged = true;
      ol.setNhV4FromNode(nodeName, nl.getNhV4FromNode(nodeName));
    }
    if (nl.getNhV6FromNode(nodeName) != ol.getNhV6FromNode(nodeName)) {
      change.linkAttributesChanged = true;
      ol.setNhV6FromNode(nodeName, nl.getNhV6FromNode(nodeName));
    }
    ++ni;
    ++oi;
  }
  if (change.topologyChanged) {  // LinkState.cpp:635-638
    spfResults_.clear();
    kthPathResults_.clear();
  }
  return change;
}

LinkState::LinkStateChange LinkState::deleteAdjacencyDatabase(
    const std::string& n) {  // LinkState.cpp:642-659
  LinkStateChange change;
  auto it = adjacencyDatabases_.find(n);
  if (it != adjacencyDatabases_.end()) {
    removeNode(n);
    adjacencyDatabases_.erase(it);
    spfResults_.clear();
    kthPathResults_.clear();
    change.topologyChanged = true;
  }
  return change;
}

std::optional<Metric> LinkState::getMetricFromAToB(const std::string& a,
                                                   const std::string& b,
                                                   bool useLinkMetric) const {
  if (a == b) return 0;  // LinkState.cpp:661-672
  const auto& r = getSpfResult(a, useLinkMetric);
  auto it = r.find(b);
  if (it == r.end()) return std::nullopt;
  return it->second.metric();
}

const std::vector<LinkState::Path>& LinkState::getKthPaths(
    const std::string& src, const std::string& dest, size_t k) const {
  // LinkState.cpp:674-703
  if (k < 1) throw std::invalid_argument("k >= 1");
  auto key = std::make_tuple(src, dest, k);
  auto it = kthPathResults_.find(key);
  if (it != kthPathResults_.end()) return it->second;
  LinkSet ignore;
  for (size_t i = 1; i < k; ++i) {
    for (const auto& p : getKthPaths(src, dest, i)) {
      for (const auto& l : p) ignore.insert(l);
    }
  }
  std::vector<Path> paths;
  SpfResult masked;
  const SpfResult* res;
  if (ignore.empty()) {
    res = &getSpfResult(src, true);
  } else {
    masked = runSpf(src, true, ignore);
    res = &masked;
  }
  if (res->count(dest)) {
    LinkSet visited;
    auto path = traceOnePath(src, dest, *res, visited);
    while (path && !path->empty()) {
      paths.push_back(std::move(*path));
      path = traceOnePath(src, dest, *res, visited);
    }
  }
  return kthPathResults_.emplace(key, std::move(paths)).first->second;
}

const LinkState::SpfResult& LinkState::getSpfResult(const std::string& node,
                                                    bool useLinkMetric) const {
  auto key = std::make_pair(node, useLinkMetric);  // LinkState.cpp:705-715
  auto it = spfResults_.find(key);
  if (it == spfResults_.end()) {
    it = spfResults_.emplace(key, runSpf(node, useLinkMetric)).first;
  }
  return it->second;
}

namespace {
// DijkstraQ (LinkState.h:612-663): binary heap ordered by (metric, nodeName),
// name->node index, O(n) re-heapify after a decrease.
struct QNode {
  QNode(const std::string& n, Metric m) : name(n), result(m) {}
  std::string name;
  LinkState::NodeSpfResult result;
};
using QNodePtr = std::shared_ptr<QNode>;
struct QGreater {
  bool operator()(const QNodePtr& a, const QNodePtr& b) const {
    if (a->result.metric() != b->result.metric()) {
      return a->result.metric() > b->result.metric();
    }
    return a->name > b->name;
  }
};
class DijkstraQ {
 public:
  void insert(const std::string& n, Metric d) {
    heap_.push_back(std::make_shared<QNode>(n, d));
    byName_[n] = heap_.back();
    std::push_heap(heap_.begin(), heap_.end(), QGreater{});
  }
  QNodePtr get(const std::string& n) {
    auto it = byName_.find(n);
    return it == byName_.end() ? nullptr : it->second;
  }
  QNodePtr extractMin() {
    if (heap_.empty()) return nullptr;
    auto m = heap_.front();
    byName_.erase(m->name);
    std::pop_heap(heap_.begin(), heap_.end(), QGreater{});
    heap_.pop_back();
    return m;
  }
  void reMake() { std::make_heap(heap_.begin(), heap_.end(), QGreater{}); }

 private:
  std::vector<QNodePtr> heap_;
  std::unordered_map<std::string, QNodePtr> byName_;
};
}  // namespace

LinkState::SpfResult LinkState::runSpf(const std::string& src,
                                       bool useLinkMetric,
                                       const LinkSet& ignore) const {
  // LinkState.cpp:720-820
  ++spfRuns_;
  SpfResult result;
  DijkstraQ q;
  q.insert(src, 0);
  while (auto node = q.extractMin()) {
    auto rc = result.emplace(node->name, std::move(node->result));
    if (!rc.second) throw std::logic_error("runSpf: settled twice");
    const std::string& u = rc.first->first;
    const Metric du = rc.first->second.metric();
    const auto nhU = rc.first->second.nextHops();  // copy: map may rehash
    if (isNodeOverloaded(u) && u != src) continue;  // hard-drained transit
    for (const auto& link : linksFromNode(u)) {
      const std::string& v = link->getOtherNodeName(u);
      if (!link->isUp() || result.count(v) || ignore.count(link)) continue;
      const Metric w = useLinkMetric ? link->getMaxMetric() : 1;
      auto other = q.get(v);
      if (!other) {
        q.insert(v, du + w);
        other = q.get(v);
      }
      if (other->result.metric() >= du + w) {
        if (other->result.metric() > du + w) {
          other->result.reset(du + w);
          q.reMake();
        }
        other->result.addPath(link, u);
        other->result.addNextHops(nhU);
        if (other->result.nextHops().empty()) other->result.addNextHop(v);
      }
    }
  }
  return result;
}

bool LinkState::pathAInPathB(const Path& a, const Path& b) {
  // LinkState.h:488-503
  if (a.size() > b.size()) return false;
  for (size_t i = 0; i < b.size() - a.size() + 1; ++i) {
    size_t ai = 0, bi = i;
    while (ai < a.size() && *a[ai] == *b[bi]) {
      ++ai;
      ++bi;
    }
    if (ai == a.size()) return true;
  }
  return false;
}

// ===================== PrefixState (PrefixState.cpp:15-57) =================
// toIPNetwork(prefix, applyMask) (NetworkUtil.h:196-208) printed as
// folly::IPAddress::networkToString ("<addr>/<len>", addr = inet_ntop text).
std::string networkOf(const std::string& text, bool applyMask) {
  const auto slash = text.rfind('/');
  if (slash == std::string::npos || slash + 1 == text.size())
    throw std::invalid_argument("Invalid IPAddress: " + text);
  const std::string addr = text.substr(0, slash), len = text.substr(slash + 1);
  if (len.size() > 3 || len.find_first_not_of("0123456789") != std::string::npos)
    throw std::invalid_argument("Invalid IPAddress: " + text);
  const int fam = addr.find(':') != std::string::npos ? AF_INET6 : AF_INET;
  unsigned char b[16];
  if (inet_pton(fam, addr.c_str(), b) != 1) throw std::invalid_argument("Invalid IPAddress: " + text);
  const int bits = fam == AF_INET6 ? 128 : 32, n = std::stoi(len);
  if (n > bits) throw std::invalid_argument("Invalid IPAddress: " + text);
  if (applyMask)
    for (int i = n; i < bits; ++i) b[i / 8] &= static_cast<unsigned char>(~(0x80u >> (i % 8)));
  char out[INET6_ADDRSTRLEN];
  inet_ntop(fam, b, out, sizeof out);
  return std::string(out) + "/" + std::to_string(n);
}

// The key is PrefixKey(node, toIPNetwork(*entry.prefix()), area), as every
// caller builds it (Decision.cpp:772-773); the entry is kept as advertised.
std::set<std::string> PrefixState::updatePrefix(const std::string& node,
                                                const std::string& area,
                                                const PrefixEntry& entry) {
  std::set<std::string> changed;
  const std::string network = networkOf(entry.prefix, true);
  auto& entries = prefixes_[network];
  auto key = std::make_pair(node, area);
  auto it = entries.find(key);
  if (it != entries.end() && *it->second == entry) return changed;
  entries[key] = std::make_shared<PrefixEntry>(entry);
  changed.insert(network);
  return changed;
}

// `prefix` is the key's CIDRNetwork as given (not masked), compared by value
std::set<std::string> PrefixState::deletePrefix(const std::string& node,
                                                const std::string& area,
                                                const std::string& prefix) {
  std::set<std::string> changed;
  const std::string network = networkOf(prefix, false);
  auto it = prefixes_.find(network);
  if (it != prefixes_.end() && it->second.erase(std::make_pair(node, area))) {
    changed.insert(network);
    if (it->second.empty()) prefixes_.erase(it);
  }
  return changed;
}

// ===================== DecisionRouteDb (SpfSolver.cpp:21-72) ===============
DecisionRouteUpdate DecisionRouteDb::calculateUpdate(
    const DecisionRouteDb& newDb) const {
  DecisionRouteUpdate d;
  for (const auto& [p, e] : newDb.unicastRoutes) {
    auto it = unicastRoutes.find(p);
    if (it == unicastRoutes.end() || it->second != e) {
      d.unicastRoutesToUpdate[p] = e;
    }
  }
  for (const auto& [p, _] : unicastRoutes) {
    if (!newDb.unicastRoutes.count(p)) d.unicastRoutesToDelete.push_back(p);
  }
  for (const auto& [l, e] : newDb.mplsRoutes) {
    auto it = mplsRoutes.find(l);
    if (it == mplsRoutes.end() || it->second != e) {
      d.mplsRoutesToUpdate[l] = e;
    }
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

// ===================== LsdbUtil selection ===================================
NodeAndArea selectBestNodeArea(const std::set<NodeAndArea>& all,
                               const std::string& me) {
  // LsdbUtil.cpp:700-711: self if selected, else the smallest key
  for (const auto& na : all) {
    if (na.first == me) return na;
  }
  return *all.begin();
}

namespace {
std::set<NodeAndArea> selectShortestDistance(const PrefixEntries& entries,
                                             const std::set<NodeAndArea>& in) {
  // LsdbUtil.cpp:715-736
  std::set<NodeAndArea> ret;
  int32_t best = std::numeric_limits<int32_t>::max();
  for (const auto& na : in) {
    auto it = entries.find(na);
    if (it == entries.end()) continue;
    const int32_t d = it->second->metrics.distance;
    if (d > best) continue;
    if (d < best) {
      best = d;
      ret.clear();
    }
    ret.insert(na);
  }
  return ret;
}
}  // namespace

std::set<NodeAndArea> selectRoutes(
    const PrefixEntries& entries, bool perArea,
    const std::unordered_set<NodeAndArea, NodeAndAreaHash>& drained) {
  // LsdbUtil.cpp:760-823: max (-(drained), path_pref, source_pref) then
  // shortest distance (globally or per area)
  std::tuple<int32_t, int32_t, int32_t> best{
      std::numeric_limits<int32_t>::min(), std::numeric_limits<int32_t>::min(),
      std::numeric_limits<int32_t>::min()};
  std::set<NodeAndArea> set;
  for (const auto& [key, e] : entries) {
    const auto& m = e->metrics;
    const int32_t isDrained =
        (m.drain_metric != 0 || drained.count(key) != 0) ? 1 : 0;
    std::tuple<int32_t, int32_t, int32_t> t{-isDrained, m.path_preference,
                                            m.source_preference};
    if (t < best) continue;
    if (t > best) {
      best = t;
      set.clear();
    }
    set.insert(key);
  }
  if (!perArea) return selectShortestDistance(entries, set);
  std::map<std::string, std::set<NodeAndArea>> byArea;
  for (const auto& na : set) byArea[na.second].insert(na);
  std::set<NodeAndArea> ret;
  for (const auto& [_, s] : byArea) {
    for (const auto& na : selectShortestDistance(entries, s)) ret.insert(na);
  }
  return ret;
}

bool hasBestRoutesInArea(const std::string& area, const PrefixEntries& entries,
                         const std::set<NodeAndArea>& best) {
  // LsdbUtil.cpp:373-389
  for (const auto& [na, _] : entries) {
    if (best.count(na) && na.second == area) return true;
  }
  return false;
}

// ===================== SpfSolver ============================================
void SpfSolver::updateStaticUnicastRoutes(
    const std::map<std::string, RibUnicastEntry>& toUpdate,
    const std::vector<std::string>& toDelete) {  // SpfSolver.cpp:109-137
  for (const auto& [p, e] : toUpdate) staticUnicastRoutes_[p] = e;
  for (const auto& p : toDelete) staticUnicastRoutes_.erase(p);
}

std::optional<RibUnicastEntry> SpfSolver::createRouteForPrefixOrGetStaticRoute(
    const std::string& me, const AreaLinkStates& ls, const PrefixState& ps,
    const std::string& prefix) {  // SpfSolver.cpp:139-158
  if (auto r = createRouteForPrefix(me, ls, ps, prefix)) return r;
  auto it = staticUnicastRoutes_.find(prefix);
  if (it != staticUnicastRoutes_.end()) return it->second;
  return std::nullopt;
}

std::optional<RibUnicastEntry> SpfSolver::createRouteForPrefix(
    const std::string& me, const AreaLinkStates& areaLinkStates,
    const PrefixState& ps, const std::string& prefix) {
  // SpfSolver.cpp:160-311
  const bool isV4 = prefixIsV4(prefix);
  if (isV4 && !enableV4_ && !v4OverV6Nexthop_) return std::nullopt;
  auto search = ps.prefixes().find(prefix);
  if (search == ps.prefixes().end()) return std::nullopt;
  bestRoutesCache_.erase(prefix);

  PrefixEntries entries = search->second;  // copy (SpfSolver.cpp:192)
  bool localPrefixConsidered = false;
  for (const auto& [area, linkState] : areaLinkStates) {
    const auto& mySpf = linkState.getSpfResult(me);
    for (auto it = entries.begin(); it != entries.end();) {
      const auto& [node, pArea] = it->first;
      if (me == node) localPrefixConsidered = true;
      if (area != pArea || mySpf.count(node)) {
        ++it;
      } else {
        it = entries.erase(it);
      }
    }
  }
  if (entries.empty()) return std::nullopt;

  auto sel = selectBestRoutes(me, entries, areaLinkStates);
  if (sel.allNodeAreas.empty()) return std::nullopt;
  bestRoutesCache_[prefix] = sel;
  if (sel.hasNode(me)) return std::nullopt;

  std::set<std::string> areasWithBest;
  for (const auto& [areaId, _] : areaLinkStates) {
    if (hasBestRoutesInArea(areaId, entries, sel.allNodeAreas)) {
      areasWithBest.insert(areaId);
    }
  }

  NextHopSet total;
  Metric shortest = std::numeric_limits<Metric>::max();
  for (const auto& area : areasWithBest) {
    auto lsIt = areaLinkStates.find(area);
    if (lsIt == areaLinkStates.end()) continue;
    auto r = selectBestPathsSpf(me, prefix, sel, area, lsIt->second);
    if (shortest >= r.bestMetric) {
      if (shortest > r.bestMetric) {
        shortest = r.bestMetric;
        total.clear();
      }
      total.insert(r.nextHops.begin(), r.nextHops.end());
    }
  }
  return addBestPaths(me, prefix, sel, entries, std::move(total), shortest,
                      localPrefixConsidered);
}

std::optional<DecisionRouteDb> SpfSolver::buildRouteDb(
    const std::string& me, const AreaLinkStates& areaLinkStates,
    const PrefixState& ps) {
  // SpfSolver.cpp:313-453
  bool exists = false;
  for (const auto& [_, l] : areaLinkStates) exists |= l.hasNode(me);
  if (!exists) return std::nullopt;

  DecisionRouteDb db;
  bestRoutesCache_.clear();
  for (const auto& [prefix, _] : ps.prefixes()) {
    if (auto r = createRouteForPrefix(me, areaLinkStates, ps, prefix)) {
      db.unicastRoutes.emplace(prefix, std::move(*r));
    }
  }
  for (const auto& [prefix, e] : staticUnicastRoutes_) {
    if (!db.unicastRoutes.count(prefix)) db.unicastRoutes.emplace(prefix, e);
  }

  if (enableNodeSegmentLabel_) {
    std::map<int32_t, std::pair<std::string, RibMplsEntry>> labelToNode;
    for (const auto& [area, linkState] : areaLinkStates) {
      for (const auto& [_, adjDb] : linkState.getAdjacencyDatabases()) {
        const int32_t label = adjDb.nodeLabel;
        const std::string& node = adjDb.thisNodeName;
        if (label == 0 || !isMplsLabelValid(label)) continue;
        auto it = labelToNode.find(label);
        if (it != labelToNode.end() && it->second.first < node) continue;
        if (node == me) {
          NextHop nh;
          nh.addr = "::";
          nh.area = area;
          nh.mplsAction = MplsAction{POP_AND_LOOKUP, std::nullopt, std::nullopt};
          labelToNode.erase(label);
          labelToNode.emplace(
              label, std::make_pair(me, RibMplsEntry{label, NextHopSet{nh}}));
          continue;
        }
        auto bnm = getNextHopsWithMetric(me, {{node, area}}, linkState);
        if (bnm.second.empty()) continue;
        labelToNode.erase(label);
        labelToNode.emplace(
            label,
            std::make_pair(
                node,
                RibMplsEntry{label,
                             getNextHopsThrift(me, {{node, area}}, false, bnm,
                                               label, area, linkState)}));
      }
    }
    for (auto& [_, ne] : labelToNode) {
      db.mplsRoutes.emplace(ne.second.label, std::move(ne.second));
    }
  }
  return db;
}

RouteSelectionResult SpfSolver::selectBestRoutes(
    const std::string& me, PrefixEntries& entries,
    const AreaLinkStates& ls) {  // SpfSolver.cpp:455-494
  RouteSelectionResult ret;
  auto filtered = filterHardDrainedNodes(entries, ls);
  auto soft = getSoftDrainedNodes(entries, ls);
  if (enableBestRouteSelection_) {
    ret.allNodeAreas = selectRoutes(filtered, /*perArea=*/false, soft);
    ret.bestNodeArea = selectBestNodeArea(ret.allNodeAreas, me);
  } else {
    for (const auto& [na, _] : filtered) ret.allNodeAreas.insert(na);
    ret.bestNodeArea = *ret.allNodeAreas.begin();
  }
  if (isNodeDrained(ret.bestNodeArea, ls)) ret.isBestNodeDrained = true;
  return ret;
}

std::optional<int64_t> SpfSolver::getMinNextHopThreshold(
    const RouteSelectionResult& sel, const PrefixEntries& entries) {
  // SpfSolver.cpp:496-509: max over selected of minNexthop
  std::optional<int64_t> r;
  for (const auto& na : sel.allNodeAreas) {
    const auto& e = entries.at(na);
    if (e->minNexthop && (!r || *e->minNexthop > *r)) r = e->minNexthop;
  }
  return r;
}

std::unordered_set<NodeAndArea, NodeAndAreaHash> SpfSolver::getSoftDrainedNodes(
    PrefixEntries& p, const AreaLinkStates& ls) const {  // SpfSolver.cpp:511-524
  std::unordered_set<NodeAndArea, NodeAndAreaHash> r;
  for (const auto& [na, _] : p) {
    // `int softDrainValue = uint64` then `> 0` (SpfSolver.cpp:518-519)
    const int v = static_cast<int>(ls.at(na.second).getNodeMetricIncrement(na.first));
    if (v > 0) r.insert(na);
  }
  return r;
}

PrefixEntries SpfSolver::filterHardDrainedNodes(
    PrefixEntries& p, const AreaLinkStates& ls) const {  // SpfSolver.cpp:526-541
  PrefixEntries f = p;
  for (auto it = f.begin(); it != f.end();) {
    if (ls.at(it->first.second).isNodeOverloaded(it->first.first)) {
      it = f.erase(it);
    } else {
      ++it;
    }
  }
  return f.empty() ? p : f;
}

bool SpfSolver::isNodeDrained(const NodeAndArea& na,
                              const AreaLinkStates& ls) const {
  const auto& l = ls.at(na.second);  // SpfSolver.cpp:543-551
  return l.isNodeOverloaded(na.first) || l.getNodeMetricIncrement(na.first) != 0;
}

SpfSolver::SpfAreaResults SpfSolver::selectBestPathsSpf(
    const std::string& me, const std::string& prefix,
    const RouteSelectionResult& sel, const std::string& area,
    const LinkState& linkState) {  // SpfSolver.cpp:553-593
  SpfAreaResults r;
  auto bnm = getNextHopsWithMetric(me, sel.allNodeAreas, linkState);
  r.bestMetric = bnm.first;
  if (bnm.second.empty()) return r;
  r.nextHops = getNextHopsThrift(me, sel.allNodeAreas, prefixIsV4(prefix), bnm,
                                 std::nullopt, area, linkState);
  return r;
}

std::optional<RibUnicastEntry> SpfSolver::addBestPaths(
    const std::string& /*me*/, const std::string& prefix,
    const RouteSelectionResult& sel, const PrefixEntries& entries,
    NextHopSet&& nextHops, Metric shortest, bool localPrefixConsidered) {
  // SpfSolver.cpp:595-639
  if (nextHops.empty()) return std::nullopt;
  auto minNh = getMinNextHopThreshold(sel, entries);
  // `int64 > size_t` compares as unsigned (SpfSolver.cpp:612): a negative
  // minNexthop always drops the route.
  if (minNh && static_cast<uint64_t>(*minNh) > nextHops.size()) {
    return std::nullopt;
  }
  PrefixEntry best = *entries.at(sel.bestNodeArea);
  if (sel.isBestNodeDrained) best.metrics.drain_metric = 1;
  RibUnicastEntry e;
  e.prefix = prefix;
  e.nexthops = std::move(nextHops);
  e.bestPrefixEntry = std::move(best);
  e.bestPrefixEntry.weight = std::nullopt;  // RibEntry.h:77 from_optional
  e.bestArea = sel.bestNodeArea.second;
  e.doNotInstall = false;
  e.igpCost = static_cast<unsigned int>(shortest);
  e.localRouteConsidered = localPrefixConsidered;
  return e;
}

SpfSolver::BestNextHopMetrics SpfSolver::getNextHopsWithMetric(
    const std::string& me, const std::set<NodeAndArea>& dsts,
    const LinkState& linkState) {  // SpfSolver.cpp:648-688
  std::unordered_map<std::string, Metric> nhNodes;
  Metric shortest = std::numeric_limits<Metric>::max();
  const auto& spf = linkState.getSpfResult(me);
  std::set<std::string> minCost;
  for (const auto& [dst, _] : dsts) {  // area ignored (SpfSolver.cpp:664-665)
    auto it = spf.find(dst);
    if (it == spf.end()) continue;
    const Metric d = it->second.metric();
    if (shortest >= d) {
      if (shortest > d) {
        shortest = d;
        minCost.clear();
      }
      minCost.insert(dst);
    }
  }
  for (const auto& dst : minCost) {
    for (const auto& nh : spf.at(dst).nextHops()) {
      nhNodes[nh] = shortest - *linkState.getMetricFromAToB(me, nh);
    }
  }
  return {shortest, nhNodes};
}

NextHopSet SpfSolver::getNextHopsThrift(
    const std::string& me, const std::set<NodeAndArea>& dsts, bool isV4,
    const BestNextHopMetrics& bnm, std::optional<int32_t> swapLabel,
    const std::string& area, const LinkState& linkState) const {
  // SpfSolver.cpp:690-767
  const auto& nhNodes = bnm.second;
  const Metric minMetric = bnm.first;
  NextHopSet out;
  for (const auto& link : linkState.linksFromNode(me)) {
    const std::string nbr = link->getOtherNodeName(me);
    auto s = nhNodes.find(nbr);
    if (s == nhNodes.end() || !link->isUp()) continue;
    const Metric distOverLink = link->getMaxMetric() + s->second;
    if (distOverLink != minMetric) continue;
    std::optional<MplsAction> act;
    if (swapLabel) {
      const bool php = dsts.count({nbr, area}) != 0;
      act = php ? MplsAction{PHP, std::nullopt, std::nullopt}
                : MplsAction{SWAP, swapLabel, std::nullopt};
    }
    NextHop nh;
    nh.addr = (isV4 && !v4OverV6Nexthop_) ? link->getNhV4FromNode(me)
                                          : link->getNhV6FromNode(me);
    nh.ifName = link->getIfaceFromNode(me);
    nh.metric = static_cast<int32_t>(distOverLink);
    nh.mplsAction = act;
    nh.area = link->getArea();
    nh.neighborNodeName = link->getOtherNodeName(me);
    nh.weight = 0;
    out.insert(nh);
  }
  return out;
}

// ===================== RibPolicy (RibPolicy.cpp:20-249) ====================
RibPolicyStatement::RibPolicyStatement(const RibPolicyStatementSpec& s)
    : name_(s.name), counterID_(s.counterID) {
  if (!s.set_weight) {
    throw std::invalid_argument(
        "Missing policy_statement.action.set_weight attribute");
  }
  if (!s.prefixes && !s.tags) {
    throw std::invalid_argument(
        "Missing policy_statement.matcher.prefixes or "
        "policy_statement.matcher.tags attribute");
  }
  weight_ = *s.set_weight;
  if (s.prefixes) prefixSet_.insert(s.prefixes->begin(), s.prefixes->end());
  if (s.tags) tagSet_.insert(s.tags->begin(), s.tags->end());
}

bool RibPolicyStatement::match(const RibUnicastEntry& r) const {
  if (tagSet_.empty() && prefixSet_.empty()) return false;
  bool tagMatch = tagSet_.empty();
  for (const auto& t : tagSet_) {
    if (r.bestPrefixEntry.tags.count(t)) {
      tagMatch = true;
      break;
    }
  }
  const bool prefixMatch = prefixSet_.empty() || prefixSet_.count(r.prefix);
  return tagMatch && prefixMatch;
}

bool RibPolicyStatement::applyAction(RibUnicastEntry& r) const {
  if (!match(r)) return false;
  r.counterID = counterID_;
  NextHopSet out;
  for (const auto& nh : r.nexthops) {
    int32_t w = weight_.default_weight;  // neighbor > area > default
    if (nh.area) {
      auto it = weight_.area_to_weight.find(*nh.area);
      if (it != weight_.area_to_weight.end()) w = it->second;
    }
    if (nh.neighborNodeName) {
      auto it = weight_.neighbor_to_weight.find(*nh.neighborNodeName);
      if (it != weight_.neighbor_to_weight.end()) w = it->second;
    }
    if (w > 0) {
      NextHop n2 = nh;
      n2.weight = w;
      out.insert(n2);
    }
  }
  if (out.empty()) return false;  // keep old next-hops
  r.nexthops = std::move(out);
  return true;
}

RibPolicy::RibPolicy(const std::vector<RibPolicyStatementSpec>& stmts,
                     int64_t ttlSecs)
    : validUntil_(std::chrono::steady_clock::now() + std::chrono::seconds(ttlSecs)) {
  if (stmts.empty()) {
    throw std::invalid_argument("Missing policy.statements attribute");
  }
  for (const auto& s : stmts) statements_.emplace_back(s);
}

bool RibPolicy::match(const RibUnicastEntry& r) const {
  for (const auto& s : statements_) {
    if (s.match(r)) return true;
  }
  return false;
}

bool RibPolicy::applyAction(RibUnicastEntry& r) const {
  for (const auto& s : statements_) {
    if (s.applyAction(r)) return true;
  }
  return false;
}

std::vector<std::string> RibPolicy::applyPolicy(
    std::map<std::string, RibUnicastEntry>& entries) const {
  std::vector<std::string> updated;
  if (!isActive()) return updated;
  for (auto& [p, e] : entries) {
    if (applyAction(e)) updated.push_back(p);
  }
  return updated;
}

}  // namespace refcpu
