// decision.h — MI355X drop-in for Open/R Decision's route computation.
//
// Same classes and method signatures as the reference (openr/decision):
//   Link / LinkState        LinkState.h:64-583
//   PrefixState             PrefixState.h:18-57
//   SpfSolver               SpfSolver.h:112-277
//   DecisionRouteDb         SpfSolver.h:68-109
//   RibUnicastEntry / RibMplsEntry   RibEntry.h:22-196
//   RibPolicy               RibPolicy.h:70-124
// with plain structs in place of the thrift types. All SPF and route
// computation runs on the GPU through the C-ABI in include/openr_gpu.h; this
// layer owns ingestion (link formation and change detection, which define
// LinkStateChange), flattening to the HBM CSR, and materialisation of the
// compact GPU results back into API objects. There is no CPU route path: a
// missing device or an input outside the GPU engine's domain throws.
#pragma once

#include <atomic>
#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstdint>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "device.h"

namespace openr_amd {

using LinkStateMetric = uint64_t;  // LinkState.h:16

enum MplsActionCode : int32_t {
  PUSH = 0,
  SWAP = 1,
  PHP = 2,
  POP_AND_LOOKUP = 3,
  NOOP = 4
};

struct MplsAction {
  int32_t action{SWAP};
  std::optional<int32_t> swapLabel;
  std::optional<std::vector<int32_t>> pushLabels;
  auto tie() const { return std::tie(action, swapLabel, pushLabels); }
  bool operator==(const MplsAction& o) const { return tie() == o.tie(); }
  bool operator<(const MplsAction& o) const { return tie() < o.tie(); }
};

struct NextHopThrift {  // Network.thrift:61-92
  std::string address;
  std::optional<std::string> ifName;
  int32_t weight{0};
  std::optional<MplsAction> mplsAction;
  int32_t metric{0};
  std::optional<std::string> area;
  std::optional<std::string> neighborNodeName;
  auto tie() const {
    return std::tie(address, ifName, weight, mplsAction, metric, area,
                    neighborNodeName);
  }
  bool operator==(const NextHopThrift& o) const { return tie() == o.tie(); }
  bool operator<(const NextHopThrift& o) const { return tie() < o.tie(); }
};
using NextHops = std::set<NextHopThrift>;

struct Adjacency {  // Types.thrift:145-215
  std::string otherNodeName, ifName, nextHopV6, nextHopV4;
  int32_t metric{0};
  int32_t adjLabel{0};
  bool isOverloaded{false};
  int32_t rtt{0};
  int64_t timestamp{0};
  int64_t weight{1};
  std::string otherIfName;
  bool adjOnlyUsedByOtherNode{false};
};

struct PerfEvent {  // Types.thrift:80-84
  std::string nodeName, eventDescr;
  int64_t unixTs{0};
};
using PerfEvents = std::vector<PerfEvent>;  // thrift::PerfEvents.events (Types.thrift:86-95)

struct AdjacencyDatabase {  // Types.thrift:223-270
  std::string thisNodeName;
  bool isOverloaded{false};
  std::vector<Adjacency> adjacencies;
  int32_t nodeLabel{0};
  std::optional<PerfEvents> perfEvents;
  std::string area;
  int32_t nodeMetricIncrementVal{0};
};

struct PrefixMetrics {
  int32_t version{1}, drain_metric{0}, path_preference{0},
      source_preference{0}, distance{0};
  auto tie() const {
    return std::tie(version, drain_metric, path_preference, source_preference,
                    distance);
  }
  bool operator==(const PrefixMetrics& o) const { return tie() == o.tie(); }
};

struct PrefixEntry {  // Types.thrift:349-408
  std::string prefix;
  int32_t type{0}, forwardingType{0}, forwardingAlgorithm{0};
  std::optional<int64_t> minNexthop;
  PrefixMetrics metrics;
  std::set<std::string> tags;
  std::vector<std::string> area_stack;
  std::optional<int64_t> weight;
  auto tie() const {
    return std::tie(prefix, type, forwardingType, forwardingAlgorithm,
                    minNexthop, metrics, tags, area_stack, weight);
  }
  bool operator==(const PrefixEntry& o) const { return tie() == o.tie(); }
};

inline bool isV4Prefix(const std::string& p) {
  return p.find(':') == std::string::npos;
}

// "<addr>/<len>" -> the network folly::IPAddress::createNetwork(addr, len,
// applyMask) prints (toIPNetwork, NetworkUtil.h:196-208); throws
// std::invalid_argument on text toIPNetwork rejects. Defined in lsdb_codec.cpp.
std::string prefixNetworkKey(const std::string& text, bool applyMask = true);

using NodeAndArea = std::pair<std::string, std::string>;

// ------------------------------------------------------------------ Link --
class Link {
 public:
  using Key = std::pair<std::pair<std::string, std::string>,
                        std::pair<std::string, std::string>>;
  Link(const std::string& area, const std::string& n1, const std::string& if1,
       const std::string& n2, const std::string& if2, bool usable = true);
  Link(const std::string& area, const std::string& n1, const Adjacency& a1,
       const std::string& n2, const Adjacency& a2, bool usable = true);

  bool isUp() const { return !overload_[0] && !overload_[1] && usable_; }
  const std::string& getArea() const { return area_; }
  const std::string& getOtherNodeName(const std::string& n) const {
    return node_[1 - side(n)];
  }
  const std::string& firstNodeName() const { return key_.first.first; }
  const std::string& secondNodeName() const { return key_.second.first; }
  const std::string& getIfaceFromNode(const std::string& n) const {
    return if_[side(n)];
  }
  LinkStateMetric getMetricFromNode(const std::string& n) const {
    return metric_[side(n)];
  }
  LinkStateMetric getMaxMetric() const {
    return std::max(metric_[0], metric_[1]);
  }
  int32_t getAdjLabelFromNode(const std::string& n) const {
    return label_[side(n)];
  }
  int64_t getWeightFromNode(const std::string& n) const {
    return weight_[side(n)];
  }
  bool getOverloadFromNode(const std::string& n) const {
    return overload_[side(n)];
  }
  const std::string& getNhV4FromNode(const std::string& n) const {
    return v4_[side(n)];
  }
  const std::string& getNhV6FromNode(const std::string& n) const {
    return v6_[side(n)];
  }
  bool getUsability() const { return usable_; }

  void setNhV4FromNode(const std::string& n, const std::string& v) {
    v4_[side(n)] = v;
  }
  void setNhV6FromNode(const std::string& n, const std::string& v) {
    v6_[side(n)] = v;
  }
  bool setMetricFromNode(const std::string& n, LinkStateMetric d) {
    metric_[side(n)] = d;
    return true;
  }
  void setAdjLabelFromNode(const std::string& n, int32_t l) {
    label_[side(n)] = l;
  }
  void setWeightFromNode(const std::string& n, int64_t w) {
    weight_[side(n)] = w;
  }
  bool setOverloadFromNode(const std::string& n, bool ov);
  bool setLinkUsability(const Link& newLink);

  const Key& key() const { return key_; }
  bool operator<(const Link& o) const { return key_ < o.key_; }
  bool operator==(const Link& o) const { return key_ == o.key_; }

 private:
  int side(const std::string& n) const {  // throws like LinkState.h:136
    if (node_[0] == n) return 0;
    if (node_[1] == n) return 1;
    throw std::invalid_argument(n);
  }
  std::string area_;
  std::string node_[2], if_[2], v4_[2], v6_[2];
  LinkStateMetric metric_[2]{1, 1};
  bool overload_[2]{false, false};
  int32_t label_[2]{0, 0};
  int64_t weight_[2]{1, 1};
  bool usable_{true};
  Key key_;
};
using LinkPtr = std::shared_ptr<Link>;

// ---------------------------------------------------------------- stats --
// fb303-style Decision counters (stats.cpp): the reference's
// fb303::fbData->addStatValue keys (decision.spf_runs / spf_ms,
// route_build_runs / route_build_ms, get_route_for_prefix,
// no_route_to_prefix) plus the engine's split of a single-area build:
// decision.gpu.prepare_ms (CSR flatten / uploads when stale), launch_ms
// (kernels + D2H to stream sync) and materialize_ms (host RouteDb).
// getDecisionCounters exports COUNT keys as "<key>.count" (the sum) and AVG
// keys as "<key>.avg" / ".sum" / ".count" (samples); times in ms.
enum class StatType { COUNT, AVG };
void addStatValue(const std::string& key, double value, StatType type);
std::map<std::string, double> getDecisionCounters();
void resetDecisionCounters();
inline double msSince(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
      .count();
}

// Process-wide version stamps of FlatTopology / PrefixState contents: a
// (pointer, stamp) cache key never matches a different object that reuses
// the address.
uint64_t nextVersionStamp();

// ---------------------------------------------------- flattened topology --
// Host image of one LinkState in the C-ABI's CSR encoding + the device copy.
struct FlatTopology {
  std::vector<std::string> names;               // id -> node name (sorted)
  std::unordered_map<std::string, uint32_t> id;  // node name -> id
  std::vector<uint32_t> rowPtr;                  // [N+1]
  std::vector<uint64_t> edges;                   // [E] packed
  std::vector<uint8_t> nodeFlags;                // [N]
  std::vector<Link*> edgeLink;                   // [E] link of each edge
  // [E] exact reverse slot of every edge when a row has 512+ edges (the
  // edge word's 9-bit field saturates at 511; ogs_graph.rslot_ext), else empty
  std::vector<uint32_t> rslotExt;
  uint64_t maxMetric{0};
  int maxDegree{0};
  bool hasZeroMetric{false};
  bool hasWideMetric{false};  // metric >= 2^32 (negative i32)
  uint64_t version{0};
  int slotStride{0};  // ogs_graph.slot_stride of dSlot (0: none)
  int slotDegree{0};  // ogs_graph.slot_degree of dSlotEdges (0: none)
  // views into dBlock (one H2D per full upload); patches write in place
  DeviceBuffer dBlock;
  DeviceBuffer dRow, dEdges, dFlags, dNodeBase, dSlot, dSlotEdges, dEdgeSrc, dRslotExt;
  const uint32_t* rslotExtDev() const {
    return rslotExt.empty() ? nullptr : dRslotExt.as<uint32_t>();
  }
  DeviceBuffer dPatchIdx, dPatchVal;  // ogs_csr_patch staging (§8(f) f3)
};

// ------------------------------------------------------------- LinkState --
class LinkState {
 public:
  LinkState(const std::string& area, const std::string& myNodeName);
  LinkState(LinkState&&) noexcept;
  ~LinkState();

  class NodeSpfResult {  // LinkState.h:290-344 (pathLinks: via getKthPaths)
   public:
    explicit NodeSpfResult(LinkStateMetric m) : metric_(m) {}
    LinkStateMetric metric() const { return metric_; }
    const std::set<std::string>& nextHops() const { return nextHops_; }
    void addNextHop(const std::string& n) { nextHops_.insert(n); }

   private:
    LinkStateMetric metric_;
    std::set<std::string> nextHops_;
  };
  using SpfResult = std::unordered_map<std::string, NodeSpfResult>;
  using Path = std::vector<LinkPtr>;

  struct LinkStateChange {  // LinkState.h:396-421
    bool topologyChanged{false};
    std::vector<LinkPtr> addedLinks;
    bool linkAttributesChanged{false};
    bool nodeLabelChanged{false};
  };

  const SpfResult& getSpfResult(const std::string& nodeName,
                                bool useLinkMetric = true) const;
  const std::vector<Path>& getKthPaths(const std::string& src,
                                       const std::string& dest,
                                       size_t k) const;
  // Fills getKthPaths(src, d, 1) and (src, d, 2) for every d of `dests` in
  // one batched GPU call (Ksp2Batch); later getKthPaths calls hit the memo.
  void prefetchKthPaths(const std::string& src,
                        const std::vector<std::string>& dests) const;
  LinkStateChange updateAdjacencyDatabase(const AdjacencyDatabase& db,
                                          const std::string& area,
                                          bool inInitialization = false);
  LinkStateChange deleteAdjacencyDatabase(const std::string& nodeName);
  std::optional<LinkStateMetric> getMetricFromAToB(
      const std::string& a, const std::string& b,
      bool useLinkMetric = true) const;

  const std::string& getArea() const { return area_; }
  bool hasNode(const std::string& n) const { return adjDbs_.count(n) != 0; }
  std::vector<LinkPtr> linksFromNode(const std::string& n) const;
  bool isNodeOverloaded(const std::string& n) const;
  uint64_t getNodeMetricIncrement(const std::string& n) const;
  size_t numLinks() const { return links_.size(); }
  size_t numNodes() const;
  const std::map<std::string, AdjacencyDatabase>& getAdjacencyDatabases()
      const {
    return adjDbs_;
  }
  static bool pathAInPathB(const Path& a, const Path& b);
  uint64_t spfRuns() const { return spfRuns_; }

  // GPU plumbing (used by SpfSolver and the batch builders)
  const FlatTopology& flat() const;          // re-flattens when stale
  const FlatTopology& flatOnDevice() const;  // + uploads when stale
  LinkPtr linkByKey(const Link::Key& k) const { return links_.at(k); }
  // runSpf calls the reference would make (decision.spf_runs,
  // LinkState.cpp:727): noteSpfRuns for SPFs it never memoises (the masked
  // getKthPaths runs, LinkState.cpp:692), noteSpf for the memoised
  // getSpfResult(node, useLinkMetric) (LinkState.cpp:705-715) -- counted
  // once per key until the topology changes, however many device launches
  // or memo layers this engine uses for it
  void noteSpfRuns(uint64_t n) const {
    spfRuns_ += n;
    addStatValue("decision.spf_runs", double(n), StatType::COUNT);  // LinkState.cpp:727
  }
  void noteSpf(const std::string& node, bool useLinkMetric = true) const {
    if (spfCounted_.emplace(node, useLinkMetric).second) noteSpfRuns(1);
  }
  // Device half of the getSpfResult memo (LinkState.cpp:705-715,
  // LinkState.h:369-372): the SPF rows of (source id, useLinkMetric) kept on
  // the device while the host memo's key stays valid (cleared on a topology
  // change) and node ids are stable (no re-flatten). buildRouteDb of any
  // source routes against them (ogs_routes_from_spf) instead of relaunching
  // the SPF; every SPF launched into a slot counts decision.gpu.spf_launches.
  // Rows: dist [N] (db bytes each) | nh [W][N] | reach [ceil(N/32)].
  struct DeviceSpf {
    DeviceBuffer rows;
    uint32_t N{0};
    int W{0};
    size_t db{0}, nhOff{0}, reachOff{0};
    bool exact{false}, valid{false};
    void* dist() const { return rows.get(); }
    uint32_t* nh() const { return reinterpret_cast<uint32_t*>(rows.as<char>() + nhOff); }
    uint32_t* reach() const { return reinterpret_cast<uint32_t*>(rows.as<char>() + reachOff); }
  };
  // the rows of source id s, or nullptr (not computed, or of another shape)
  DeviceSpf* findDeviceSpf(uint32_t s, bool useLinkMetric, uint32_t N, int W, size_t db,
                           bool exact) const;
  // an empty slot for s sized for (N, W, db); the caller launches the SPF
  // into it and then calls commitDeviceSpf
  DeviceSpf& newDeviceSpf(uint32_t s, bool useLinkMetric, uint32_t N, int W, size_t db,
                          bool exact) const;
  void commitDeviceSpf(DeviceSpf& slot, const std::string& node, bool useLinkMetric) const;
  uint64_t deviceSpfLaunches() const { return deviceSpfLaunches_; }
  size_t deviceSpfSlots() const { return deviceSpf_.size(); }
  // attribute-only updates patch the CSR in place (default) or, off,
  // re-flatten + re-upload it (A/B measurements)
  void setIncrementalFlatten(bool on) { incrementalFlatten_ = on; }
  // full CSR builds vs in-place patches (§8(f) f3) so far
  uint64_t flatBuilds() const { return flatBuilds_; }
  uint64_t flatPatches() const { return flatPatches_; }
  uint64_t edgesPatched() const { return edgesPatched_; }

 private:
  LinkPtr makeLink(const std::string& node, const Adjacency& adj) const;
  void invalidate(bool topologyChanged);
  // attribute-only change of `node` (no link / node added or removed):
  // re-encode the touched edges in the current CSR image and scatter them
  // into the device copy (ogs_csr_patch) instead of re-flattening
  void patchFlat(const std::string& node, const std::vector<const Link*>& touched,
                 bool nodeFlagsChanged);
  void uploadSlotImages(FlatTopology& m) const;
  void slotImages(FlatTopology& m, std::vector<uint16_t>& slots,
                  std::vector<uint32_t>& img) const;

  std::string area_, myNodeName_;
  std::map<std::string, AdjacencyDatabase> adjDbs_;
  std::map<Link::Key, LinkPtr> links_;                      // all links
  // per node its links in key order (LinkState.h linkMap_), with the link
  // itself: the flatten walks rows without a links_ lookup per edge
  std::unordered_map<std::string, std::map<Link::Key, LinkPtr>> byNode_;
  std::unordered_map<std::string, bool> overloaded_;
  std::unordered_map<std::string, uint64_t> metricInc_;
  mutable std::map<std::pair<std::string, bool>, SpfResult> spfMemo_;
  mutable std::set<std::pair<std::string, bool>> spfCounted_;  // noteSpf
  mutable std::unordered_map<uint64_t, DeviceSpf> deviceSpf_;  // key s << 1 | useLinkMetric
  mutable size_t deviceSpfBytes_{0};
  mutable uint64_t deviceSpfLaunches_{0};
  void clearSpfMemos() const;
  mutable std::map<std::tuple<std::string, std::string, size_t>,
                   std::vector<Path>>
      kthMemo_;
  mutable std::unique_ptr<FlatTopology> flat_;
  mutable bool flatStale_{true};
  mutable bool deviceStale_{true};
  mutable uint64_t spfRuns_{0};
  uint64_t mutation_{0};
  mutable uint64_t flatBuilds_{0};
  uint64_t flatPatches_{0}, edgesPatched_{0};
  bool incrementalFlatten_{true};
};

// ----------------------------------------------------------- PrefixState --
// Grow a node-based hash table (unordered_map / unordered_set) 8x instead of
// the library's 2x while it is under 1M entries: every rehash relinks each
// node through a cache miss, and a bulk ingest (the C3 publication: 208k
// prefix keys, no count known up front) then pays ~1.1 relinks per entry
// instead of ~2. Past 1M entries the library's policy applies, and one
// reserve never asks for more than 2M buckets (16 MB of bucket pointers), so
// a table just under 1M entries holds at most twice the library's buckets.
// setHashGrowthFactor(k) sets the factor process-wide (<= 2: the library's
// policy; for A/B runs).
inline std::atomic<int>& hashGrowthFactorRef() {
  static std::atomic<int> k{8};
  return k;
}
inline void setHashGrowthFactor(int k) { hashGrowthFactorRef().store(k); }
inline int hashGrowthFactor() { return hashGrowthFactorRef().load(std::memory_order_relaxed); }
template <typename Table>
inline void growHashTable(Table& t) {
  const int k = hashGrowthFactor();
  constexpr size_t kMaxEntries = size_t(1) << 20, kMaxBuckets = size_t(1) << 21;
  if (k > 2 && t.size() + 1 > size_t(double(t.bucket_count()) * t.max_load_factor()) &&
      t.size() < kMaxEntries) {
    const size_t want = std::max<size_t>(64, t.size() * size_t(k));
    t.reserve(std::max(std::min(want, kMaxBuckets), 2 * t.size()));
  }
}

// PrefixState.h:55: a hashed map keyed by the prefix network (the reference's
// unordered_map<CIDRNetwork, PrefixEntries>): ingestion is one hash insert
// per key. Nothing downstream depends on its iteration order -- the device
// prefix table lists prefixes in that order and maps results back by index,
// RouteDbs are keyed by prefix, route digests are XOR-combined.
// A prefix's advertisements keyed by (node, area), in key order: a sorted
// vector (one allocation for the one or few advertisers a prefix has, where
// a node-based map allocates per entry). Iterates as pairs, like a map.
class PrefixEntryList {
  // sorted by (node, area); most prefixes have ONE advertisement, kept inline
  // (no heap block per prefix: the C3 publication's 208k keys), more move to
  // a vector
 public:
  using value_type = std::pair<NodeAndArea, std::shared_ptr<PrefixEntry>>;
  using const_iterator = const value_type*;
  using iterator = value_type*;
  PrefixEntryList() = default;
  PrefixEntryList(const PrefixEntryList& o) { *this = o; }
  PrefixEntryList(PrefixEntryList&& o) noexcept { *this = std::move(o); }
  PrefixEntryList& operator=(const PrefixEntryList& o) {
    if (this != &o) {
      one_ = o.one_;
      many_ = o.many_;
      n_ = o.n_;
      heap_ = o.heap_;
    }
    return *this;
  }
  PrefixEntryList& operator=(PrefixEntryList&& o) noexcept {
    if (this == &o) return *this;
    one_ = std::move(o.one_);
    many_ = std::move(o.many_);
    n_ = o.n_;
    heap_ = o.heap_;
    o.n_ = 0;
    o.heap_ = false;
    return *this;
  }
  const_iterator begin() const { return data(); }
  const_iterator end() const { return data() + n_; }
  iterator begin() { return data(); }
  iterator end() { return data() + n_; }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  // the entry of `k` (inserted empty when absent) and whether it was new
  std::pair<iterator, bool> try_emplace(const NodeAndArea& k) {
    iterator it = find(k);
    if (it != end() && it->first == k) return {it, false};
    if (!heap_ && n_ == 0) {
      one_ = value_type(k, nullptr);
      n_ = 1;
      return {&one_, true};
    }
    const size_t at = size_t(it - begin());  // before the storage moves
    if (!heap_) {  // the second advertisement: both to the vector
      many_.reserve(4);
      many_.push_back(std::move(one_));
      one_ = value_type();
      heap_ = true;
    }
    many_.insert(many_.begin() + at, value_type(k, nullptr));
    ++n_;
    return {many_.data() + at, true};
  }
  size_t erase(const NodeAndArea& k) {
    iterator it = find(k);
    if (it == end() || it->first != k) return 0;
    if (!heap_) {
      one_ = value_type();
      n_ = 0;
      return 1;
    }
    many_.erase(many_.begin() + (it - many_.data()));
    --n_;
    return 1;
  }

 private:
  value_type* data() { return heap_ ? many_.data() : &one_; }
  const value_type* data() const { return heap_ ? many_.data() : &one_; }
  iterator find(const NodeAndArea& k) {
    return std::lower_bound(begin(), end(), k,
                            [](const value_type& a, const NodeAndArea& b) { return a.first < b; });
  }
  value_type one_;
  std::vector<value_type> many_;
  uint32_t n_{0};
  bool heap_{false};
};

class PrefixState {
 public:
  using Entries = PrefixEntryList;
  using Map = std::unordered_map<std::string, Entries>;
  const Map& prefixes() const { return prefixes_; }
  std::set<std::string> updatePrefix(const std::string& node,
                                     const std::string& area,
                                     const PrefixEntry& entry);
  std::set<std::string> updatePrefix(const std::string& node,
                                     const std::string& area, PrefixEntry&& entry);
  // PrefixState::updatePrefix(PrefixKey, entry) (PrefixState.cpp:15-38) with
  // the key's network given: `network` = toIPNetwork(entry.prefix) as
  // Decision.cpp:772-773 builds it. The overloads above derive it from the
  // entry; the entry itself is stored as advertised (host bits kept).
  std::set<std::string> updatePrefixKeyed(const std::string& node, const std::string& area,
                                          const std::string& network, PrefixEntry entry);
  // the same update without the changed-set allocation (the ingestion hot
  // path): the table's key of `network` when it changed, else nullptr;
  // `network` is moved into the table on first sight
  const std::string* updatePrefixInPlace(const std::string& node, const std::string& area,
                                         std::string&& network, PrefixEntry&& entry);
  // true when (node, area)'s entry of `prefix` existed and was removed
  bool deletePrefixInPlace(const std::string& node, const std::string& area,
                           const std::string& prefix, std::string* network = nullptr);
  void reserve(size_t prefixes) { prefixes_.reserve(prefixes); }
  // `prefix` is the key's network as given (PrefixKey does not mask);
  // compared by value, so the text is normalised first
  std::set<std::string> deletePrefix(const std::string& node,
                                     const std::string& area,
                                     const std::string& prefix);
  uint64_t version() const { return version_; }
  // Every changed network in change order -- what Decision collects as
  // DecisionPendingUpdates::updatedPrefixes (Decision.cpp:35-60) and loops
  // over in the incremental branch of rebuildRoutes (Decision.cpp:929-951).
  // Entry i of changeLog() has the absolute position changeLogBase() + i;
  // the oldest half is dropped past kChangeLogCap entries (a reader behind
  // changeLogBase() has lost its place and must not rely on it).
  // The log is kept once a reader asked for it (trackChanges: the
  // SpfSolver's first build / incremental call), so bulk ingestion before
  // the first build records nothing.
  const std::vector<std::string>& changeLog() const { return changeLog_; }
  uint64_t changeLogBase() const { return changeLogBase_; }
  uint64_t changeLogEnd() const { return changeLogBase_ + changeLog_.size(); }
  void trackChanges() const { tracking_ = true; }
  static constexpr size_t kChangeLogCap = size_t(1) << 20;

 private:
  void logChange(const std::string& network);
  Map prefixes_;
  uint64_t version_{0};
  std::vector<std::string> changeLog_;
  uint64_t changeLogBase_{0};
  mutable bool tracking_{false};
};

// ------------------------------------------------------------ RIB types --
struct RibUnicastEntry {  // RibEntry.h:45-113
  std::string prefix;
  NextHops nexthops;
  unsigned int igpCost{0};
  PrefixEntry bestPrefixEntry;
  std::string bestArea;
  bool doNotInstall{false};
  std::optional<std::string> counterID;
  bool localRouteConsidered{false};
  bool operator==(const RibUnicastEntry& o) const {  // RibEntry.h:81-87
    return prefix == o.prefix && bestPrefixEntry == o.bestPrefixEntry &&
        doNotInstall == o.doNotInstall && counterID == o.counterID &&
        localRouteConsidered == o.localRouteConsidered &&
        nexthops == o.nexthops;
  }
  bool operator!=(const RibUnicastEntry& o) const { return !(*this == o); }
};

struct RibMplsEntry {  // RibEntry.h:115-197
  int32_t label{0};
  NextHops nexthops;
  bool operator==(const RibMplsEntry& o) const {
    return label == o.label && nexthops == o.nexthops;
  }
  bool operator!=(const RibMplsEntry& o) const { return !(*this == o); }
};

struct DecisionRouteUpdate {  // RouteUpdate.h:28-110
  std::map<std::string, RibUnicastEntry> unicastRoutesToUpdate;
  std::vector<std::string> unicastRoutesToDelete;
  std::map<int32_t, RibMplsEntry> mplsRoutesToUpdate;
  std::vector<int32_t> mplsRoutesToDelete;
  std::optional<PerfEvents> perfEvents;  // the batch's (Decision.cpp:954-955)
};

// thrift::UnicastRoute / MplsRoute / RouteDatabase (Network.thrift,
// OpenrCtrl's getRouteDbComputed payload) as plain structs; the prefix stays
// in its CIDR text form (toIpPrefix is the thrift adapter's job)
struct UnicastRoute {
  std::string dest;
  std::vector<NextHopThrift> nextHops;
  std::optional<std::string> counterID;
};
struct MplsRoute {
  int32_t topLabel{0};
  std::vector<NextHopThrift> nextHops;
};
struct RouteDatabase {
  std::string thisNodeName;
  std::vector<UnicastRoute> unicastRoutes;
  std::vector<MplsRoute> mplsRoutes;
};

struct DecisionRouteDb {  // SpfSolver.h:68-109
  std::map<std::string, RibUnicastEntry> unicastRoutes;
  std::map<int32_t, RibMplsEntry> mplsRoutes;
  // SpfSolver.h:82-94 + RibEntry.h:95-103 (unicast) / MplsRoute of RibMplsEntry
  RouteDatabase toThrift() const;
  DecisionRouteUpdate calculateUpdate(const DecisionRouteDb& newDb) const;
  void update(const DecisionRouteUpdate& u);
};

struct RouteSelectionResult {  // SpfSolver.h:37-66
  std::set<NodeAndArea> allNodeAreas;
  NodeAndArea bestNodeArea;
  bool isBestNodeDrained{false};
  bool hasNode(const std::string& n) const {
    for (const auto& na : allNodeAreas) {
      if (na.first == n) return true;
    }
    return false;
  }
};

using AreaLinkStates = std::map<std::string, LinkState>;

class RibPolicy;

// ------------------------------------------------------------- Ksp2Batch --
// getKthPaths(src, d, 1) and (src, d, 2) for many destinations d of one
// LinkState, on the GPU (ogs_ksp2_paths): one unmasked SPF of src, then per
// destination the k = 1 trace, the masked rerun and the k = 2 trace. The
// device buffers stay resident; launch() may be repeated (benchmarks).
class Ksp2Batch {
 public:
  Ksp2Batch(const LinkState& ls, const std::string& src,
            const std::vector<std::string>& dests);
  // several topologies (e.g. the areas of a multi-area source) in ONE pair
  // of launches: destinations[i] is searched in areas[i]
  Ksp2Batch(const std::vector<const LinkState*>& areas, const std::string& src,
            const std::vector<std::vector<std::string>>& destinations);
  void launch(void* stream = nullptr) const;  // asynchronous
  void fetch();                               // D2H of both path sets (sync)
  size_t size() const { return dests_.size(); }
  const std::vector<std::string>& dests() const { return dests_; }
  // topology index (position in `areas`) of destination i
  size_t areaOf(size_t i) const { return destArea_.at(i); }
  // unit i's k-th (1 or 2) paths as topology-local directed edge ids
  std::vector<std::vector<uint32_t>> edgePaths(size_t i, int k) const;
  std::vector<LinkState::Path> paths(size_t i, int k) const;
  size_t numUnits() const { return nUnits_; }
  uint64_t totalPathEdges(int k) const;

 private:
  void init(const std::string& src,
            const std::vector<std::vector<std::string>>& destinations);
  std::vector<const LinkState*> ls_;
  std::vector<std::string> dests_;
  std::vector<size_t> destArea_;
  std::vector<int64_t> unitOf_;  // dest index -> unit (-1: unknown dest)
  size_t nUnits_{0}, nSources_{0};
  uint32_t flags_{0}, maxPaths_{0}, maxEdges_{0};
  ogs_graph g_{};
  DeviceBuffer dNodeBase_, dRow_, dEdges_, dFlags_, dRslot_;  // multi-topology batch
  DeviceBuffer dSrc_, dUnits_, dCount_[2], dLen_[2], dEdges2_[2];
  std::vector<uint32_t> count_[2], len_[2], edges_[2];
};

// ------------------------------------------------------------- SpfSolver --
class SpfSolver {
 public:
  SpfSolver(const std::string& myNodeName, bool enableV4,
            bool enableNodeSegmentLabel, bool enableBestRouteSelection = false,
            bool v4OverV6Nexthop = false);
  ~SpfSolver();

  void updateStaticUnicastRoutes(
      const std::map<std::string, RibUnicastEntry>& toUpdate,
      const std::vector<std::string>& toDelete);
  std::optional<DecisionRouteDb> buildRouteDb(
      const std::string& myNodeName, const AreaLinkStates& areaLinkStates,
      const PrefixState& prefixState);
  std::optional<RibUnicastEntry> createRouteForPrefixOrGetStaticRoute(
      const std::string& myNodeName, const AreaLinkStates& areaLinkStates,
      const PrefixState& prefixState, const std::string& prefix);
  // The incremental branch of Decision::rebuildRoutes (Decision.cpp:929-951)
  // calls the above once per changed prefix; this answers a whole changed
  // set (DecisionPendingUpdates::updatedPrefixes) with ONE build over a
  // sub-table of those prefixes. Same per-prefix result (nullopt = delete).
  std::map<std::string, std::optional<RibUnicastEntry>> createRoutesForPrefixes(
      const std::string& myNodeName, const AreaLinkStates& areaLinkStates,
      const PrefixState& prefixState, const std::set<std::string>& prefixes);
  // Device-only buildRouteDb over the multi-area kernels (any number of
  // areas): the source's SPF in every area, the RouteDb and the RibPolicy
  // are enqueued on `stream` and left in device memory -- no download, no
  // DecisionRouteDb. Returns false when myNodeName is in no area.
  bool enqueueRouteDb(const std::string& myNodeName,
                      const AreaLinkStates& areaLinkStates,
                      const PrefixState& prefixState, void* stream);
  // The DecisionRouteDb of the last enqueueRouteDb(myNodeName, ...) (syncs
  // `stream`, downloads and materialises those device results; the
  // AreaLinkStates / PrefixState must be unchanged since).
  std::optional<DecisionRouteDb> collectRouteDb(const std::string& myNodeName,
                                                const AreaLinkStates& areaLinkStates,
                                                void* stream = nullptr);
  const std::map<std::string, RouteSelectionResult>& getBestRoutesCache()
      const {
    return bestRoutesCache_;
  }
  // per-prefix calls answered from one batch (createRouteForPrefixOr-
  // GetStaticRoute): launches made / prefixes they computed (tests, bench)
  uint64_t incrementalBatches() const { return incBatches_; }
  uint64_t incrementalBatchPrefixes() const { return incBatchPrefixes_; }
  // GPU-side RibPolicy (UCMP weights): when set and active, buildRouteDb
  // returns the routes RibPolicy::applyPolicy would leave (the reference's
  // buildRouteDb + Decision's applyPolicy on the result, Decision.cpp:
  // 912-925), computed on the device before materialisation. nullptr: off.
  void setRibPolicy(const RibPolicy* policy) { ribPolicy_ = policy; }

 private:
  // several areas (SpfSolver.cpp:160-311 across LinkStates)
  struct MultiAreaResult;
  void enqueueMultiArea(const std::string& myNodeName,
                        const AreaLinkStates& areaLinkStates,
                        const PrefixState& prefixState, void* stream,
                        MultiAreaResult& r);
  std::optional<DecisionRouteDb> buildRouteDbMultiArea(
      const std::string& myNodeName, const AreaLinkStates& areaLinkStates,
      const PrefixState& prefixState);
  std::optional<DecisionRouteDb> buildRouteDbSingleArea(
      const std::string& myNodeName, const AreaLinkStates& areaLinkStates,
      const PrefixState& prefixState);
  // single-area prefix table (packed, one H2D) cached on (ps, f) versions
  void prepareSingleArea(const FlatTopology& f, const PrefixState& ps,
                         const std::string& area);
  void routesFromSpfMemo(const std::string& me, const LinkState& ls,
                         const std::string& area, const PrefixState& ps,
                         const PrefixState& sub,
                         std::map<std::string, std::optional<RibUnicastEntry>>& out);
  // createRoutesForPrefixes without the counters or the static fallback
  std::map<std::string, std::optional<RibUnicastEntry>> computeRoutes(
      const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
      const std::set<std::string>& prefixes);
  void prepareMultiArea(const AreaLinkStates& areaLinkStates,
                        const PrefixState& prefixState);
  struct MultiAreaResult {  // host copies of one source's GPU results
    std::vector<uint32_t> row;  // [A] SPF row of each area or OGS_NODE_NONE
    std::vector<uint64_t> dist, metric;  // widened, all-ones = unreachable
    std::vector<uint32_t> nh, meta, mask, sel;
    std::vector<uint32_t> reach;  // exact-order settled bitsets per SPF row
    bool wide{false};  // device buffers hold 64-bit distances
    std::vector<uint16_t> applied, counter;  // RibPolicy (empty: none)
    int W{1};
    size_t Sn{0}, P{0};
  };
  DecisionRouteDb materializeMultiArea(const std::string& myNodeName,
                                       const AreaLinkStates& areaLinkStates,
                                       const MultiAreaResult& r);
  DecisionRouteDb downloadMultiArea(const std::string& myNodeName,
                                    const AreaLinkStates& areaLinkStates,
                                    MultiAreaResult& r);
  friend class RouteDbBatch;
  struct Impl;
  std::unique_ptr<Impl> impl_;
  std::map<std::string, RibUnicastEntry> staticUnicastRoutes_;
  std::map<std::string, RouteSelectionResult> bestRoutesCache_;
  // Per-prefix calls of Decision's incremental loop: the first call after a
  // PrefixState / topology change computes every prefix changed since the
  // last build or batch (PrefixState::changeLog) in ONE batch; the rest of
  // the loop is served from incCache_, valid for (me, PrefixState version --
  // a process-unique stamp --, the areas' topology versions). Each entry
  // keeps the prefix's best-route selection too: the selection cache
  // (getBestRoutesCache) changes only when the prefix itself is asked, as
  // with the reference's per-prefix calls.
  struct IncEntry {
    std::optional<RibUnicastEntry> route;
    std::optional<RouteSelectionResult> sel;  // nullopt: no cache entry
    bool touched{false};  // a known, ungated prefix: its cache entry is reset
  };
  std::unordered_map<std::string, IncEntry> incCache_;
  const PrefixState* incPs_{nullptr};
  uint64_t incPsVersion_{~0ull}, incLogCursor_{0};
  std::string incMe_;
  std::vector<std::pair<const FlatTopology*, uint64_t>> incTopo_;
  uint64_t incBatches_{0}, incBatchPrefixes_{0};
  std::unique_ptr<SpfSolver> probe_;  // multi-area sub-table builds
  bool quietStats_{false};             // probe_: no route-build counters
  const RibPolicy* ribPolicy_{nullptr};
  std::string myNodeName_;
  bool enableV4_, enableNodeSegmentLabel_, enableBestRouteSelection_,
      v4OverV6Nexthop_;
};

// ------------------------------------------------------------- RibPolicy --
struct RibRouteActionWeight {
  int32_t default_weight{0};
  std::map<std::string, int32_t> area_to_weight;
  std::map<std::string, int32_t> neighbor_to_weight;
};
struct RibPolicyStatementSpec {
  std::string name;
  std::optional<std::vector<std::string>> prefixes;
  std::optional<std::vector<std::string>> tags;
  std::optional<RibRouteActionWeight> set_weight;
  std::optional<std::string> counterID;
};

class RibPolicy {  // RibPolicy.h:70-124
 public:
  RibPolicy(const std::vector<RibPolicyStatementSpec>& statements,
            int64_t ttlSecs);
  // RibPolicy.cpp:167-171,199-208: valid until ctor time + ttl_secs
  bool isActive() const { return std::chrono::steady_clock::now() < validUntil_; }
  int64_t getTtlDurationMs() const {
    return std::chrono::duration_cast<std::chrono::milliseconds>(
               validUntil_ - std::chrono::steady_clock::now())
        .count();
  }
  bool match(const RibUnicastEntry& route) const;
  bool applyAction(RibUnicastEntry& route) const;
  std::vector<std::string> applyPolicy(
      std::map<std::string, RibUnicastEntry>& unicastEntries) const;

  // compiled form for the GPU (ogs_rib_policy, SpfSolver::setRibPolicy)
  size_t numStatements() const { return stmts_.size(); }
  bool hasMatcher(size_t k) const {
    return !stmts_[k].prefixes.empty() || !stmts_[k].tags.empty();
  }
  bool matchesPrefix(size_t k, const std::string& prefix) const {
    return stmts_[k].prefixes.empty() || stmts_[k].prefixes.count(prefix) != 0;
  }
  bool matchesTags(size_t k, const std::set<std::string>& tags) const;
  int32_t weightOf(size_t k, const NextHopThrift& nh) const;  // RibPolicy.cpp:122-137
  const std::optional<std::string>& counterIDOf(size_t k) const {
    return stmts_[k].counterID;
  }

 private:
  struct Stmt {
    std::string name;
    std::set<std::string> prefixes, tags;
    RibRouteActionWeight weight;
    std::optional<std::string> counterID;
  };
  bool matchStmt(const Stmt& s, const RibUnicastEntry& r) const;
  std::vector<Stmt> stmts_;
  std::chrono::steady_clock::time_point validUntil_;

 public:
  uint64_t uid() const { return uid_; }  // compiled-policy cache key

 private:
  uint64_t uid_;
};

// ---------------------------------------------------- batch flattening --
// T independent single-area LSDBs flattened into one C-ABI graph batch +
// prefix table (the bench and the batched parity tests use this).
struct HostBatch {
  std::vector<uint32_t> nodeBase{0}, rowPtr{0};
  std::vector<uint32_t> topoDesc;  // [T*8], see ogs_graph.topo_desc
  std::vector<uint64_t> edges;
  std::vector<uint8_t> nodeFlags;
  std::vector<uint32_t> pfxBase{0}, advOff{0}, advNode;
  std::vector<int32_t> advMetrics;
  std::vector<int64_t> advMinNh;
  std::vector<uint8_t> pfxFlags;
  std::vector<uint8_t> color;  // [N_total] BFS 2-colouring (slot_order.h)
  std::vector<uint32_t> edgeSrc;  // [E_total] topology-local row of each edge
  int maxNodes{0}, maxEdges{0}, maxPrefixes{0}, maxDegree{0}, maxAdvs{0};
  uint64_t maxMetric{0};
  bool hasZeroMetric{false};
  void append(const FlatTopology& t, const PrefixState& ps,
              const std::string& area);
  // only the prefix-table half of append (no CSR, colouring or topoDesc);
  // returns the number of prefixes appended
  uint32_t appendPrefixes(const FlatTopology& t, const PrefixState& ps,
                          const std::string& area);
  // ogs_graph.slot_node image ([T*stride]); returns the stride, 0 if none.
  // With `edgesOut`, also the slot_edges image and its degree (0 if the
  // batch does not qualify).
  int slotOrder(std::vector<uint16_t>& out,
                std::vector<uint32_t>* edgesOut = nullptr,
                int* degreeOut = nullptr) const;
};

// ---------------------------------------------------- materialisation --
// One unit's compact GPU results (host copies, distances widened to 64-bit,
// all-ones = unreachable) and the host side of the prefix table.
// host threads of materializeRouteDb (0 / 1: the caller's thread only)
extern int g_materializeThreads;

struct UnitView {
  int W{1};
  uint32_t N{0}, P{0};
  const uint64_t* dist{nullptr};
  const uint32_t* nh{nullptr};
  size_t nhStride{0};  // nh[w * nhStride + v]
  const uint32_t* meta{nullptr};
  const uint64_t* metric{nullptr};
  const uint32_t* mask{nullptr};
  size_t maskStride{0};  // mask[w * maskStride + p]
  const uint32_t* sel{nullptr};
  // settled bitset of an exact-order SPF (nullptr: all-ones dist =
  // unreachable); a wrapped u64 distance of a reached node may be all ones
  const uint32_t* reach{nullptr};
  // device-applied RibPolicy (SpfSolver::setRibPolicy): statement whose
  // weights / counterID each route took, OGS_POLICY_NONE = none
  const RibPolicy* policy{nullptr};
  const uint16_t* applied{nullptr};
  const uint16_t* counter{nullptr};
};

struct PrefixHostTable {
  std::vector<std::string> prefixes;
  std::vector<const PrefixEntry*> advEntry;
  std::vector<NodeAndArea> advKey;
  std::vector<uint32_t> advOff;
  uint64_t generation{0};  // bumped by every build (compiled-policy cache key)
  void build(const PrefixState& ps);
  // prefix indices in prefix order (PrefixState is a hashed map): computed
  // on first use per build, for the outputs that list routes sorted (the
  // direct thrift build of getRouteDbComputed, merged with the statics)
  const std::vector<uint32_t>& sortedOrder() const;

 private:
  mutable std::mutex sortedMutex_;
  mutable std::vector<uint32_t> sorted_;
  mutable uint64_t sortedGen_{0};
};

bool wideDistancesNeeded(const FlatTopology& f);

// label -> (owner node, route), the reference's labelToNode
// (SpfSolver.cpp:356-358, duplicate labels: smallest owner name wins)
using LabelRoutes = std::map<int32_t, std::pair<std::string, RibMplsEntry>>;
// Node-label routes of one area from the source's SPF there (dist/nh as in
// UnitView; dist == nullptr when the source has no SPF in that area).
void addNodeLabelRoutes(const LinkState& ls, const FlatTopology& f,
                        const std::string& area, const std::string& me,
                        const uint64_t* dist, const uint32_t* nhWords,
                        size_t nhStride, int W, LabelRoutes& labelToNode,
                        const uint32_t* reach = nullptr);

// Next-hop words of a source in an all-sources batch (RouteDbBatch, the C3
// launches): the smallest kernel width, except that sources of 65..96 links
// on large topologies (the fused frontier + route stream's domain) keep three
// words instead of rounding up to four -- one mask word per route less
// (C3's FSWs, 84 links: 0.21 GB less per whole-node build).
inline int batchNhWords(int degree, size_t nodes, bool wideMetric) {
  const int w = std::max(1, ogs_nh_words_for_degree(degree));
  if (w == 4 && degree <= 96 && nodes > 256 && nodes <= 30000 && !wideMetric) return 3;
  return w;
}

// bit v of a settled bitset (exact-order SPF rows)
inline bool bitAt(const uint32_t* bits, uint32_t v) { return (bits[v >> 5] >> (v & 31u)) & 1u; }

std::optional<RibUnicastEntry> materializeRoute(
    const FlatTopology& f, const std::string& me, const PrefixHostTable& pt,
    uint32_t p, uint32_t meta, uint64_t metric, const uint32_t* mask,
    size_t maskStride, int W, bool v4OverV6Nexthop, const RibPolicy* policy,
    uint16_t applied, uint16_t counter);
// the same with the source's CSR row start `rb` (= f.rowPtr[f.id.at(me)])
// looked up once by the caller: loops over many routes of one source
std::optional<RibUnicastEntry> materializeRouteAt(
    const FlatTopology& f, uint32_t rb, const std::string& me, const PrefixHostTable& pt,
    uint32_t p, uint32_t meta, uint64_t metric, const uint32_t* mask,
    size_t maskStride, int W, bool v4OverV6Nexthop, const RibPolicy* policy,
    uint16_t applied, uint16_t counter);

// Changed records of many variants in the ogs_route_changes layout: variant
// v owns records [offsets[v], offsets[v + 1]), record i = prefix index,
// meta, metric and mask word w at mask[w * total + i].
struct ChangeRecords {
  const uint32_t* offsets{nullptr};  // [variants + 1]
  size_t variants{0};
  const uint32_t* prefix{nullptr};
  const uint32_t* meta{nullptr};
  const uint32_t* metric{nullptr};
  const uint32_t* mask{nullptr};
  size_t total{0};
  int W{1};
};
// One DecisionRouteUpdate per variant (calculateUpdate, SpfSolver.cpp:21-56:
// records without VALID are deletions, the rest materialised routes), built
// on `threads` host threads (0: up to 16 / the hardware's).
std::vector<DecisionRouteUpdate> materializeUpdates(const FlatTopology& f, const std::string& me,
                                                    const PrefixHostTable& pt,
                                                    const ChangeRecords& c, bool v4OverV6Nexthop,
                                                    int threads);

DecisionRouteDb materializeRouteDb(
    const LinkState& ls, const FlatTopology& f, const std::string& area,
    const std::string& me, const UnitView& r, const PrefixHostTable& pt,
    bool v4OverV6Nexthop, bool enableNodeSegmentLabel,
    const std::map<std::string, RibUnicastEntry>& statics,
    std::map<std::string, RouteSelectionResult>* bestRoutesCache);

// ------------------------------------------------------ LinkFailureSweep --
// SURVEY.md §8(f) f1 over config C4: the route updates Decision would hand
// Fib (Decision::rebuildRoutes incremental branch, Decision.cpp:929-951 =
// buildRouteDb + DecisionRouteDb::calculateUpdate, SpfSolver.cpp:21-56) for
// many what-if variants of ONE area, a variant being a set of <= 2 links taken
// down (adjacency withdrawn at both ends, LinkState.cpp:406-659). All variants
// run in one launch (ogs_spf_routes_variants, route diff fused in); only the
// changed records are gathered on the device (ogs_route_changes_gather) and
// materialised. Areas with zero / negative link metrics or path sums past 32
// bits, and sources of degree > 128, run each variant as its own topology
// (exact extraction order, 64-bit distances), in ogs_spf_routes launches of
// up to kExactChunk (256) topologies each, rebuilt from the live `ls` / `ps`
// at launch time, and diff on the host with calculateUpdate. Node-segment
// labels are not part of the sweep (off in the DecisionBenchmark config,
// SURVEY.md A.8). `ls` and `ps` must outlive the sweep unchanged.
class LinkFailureSweep {
 public:
  struct LinkDown {  // one end of the link: (node, its interface)
    std::string node, ifName;
  };
  LinkFailureSweep(const std::string& myNodeName, const LinkState& ls,
                   const PrefixState& ps,
                   const std::vector<std::vector<LinkDown>>& variants,
                   bool enableV4, bool enableBestRouteSelection = false,
                   bool v4OverV6Nexthop = false);
  // base RouteDb records (the diff's reference); launch() runs it when needed
  void runBase(void* stream = nullptr);
  // every variant + diff, one launch; records = false keeps only the diff
  // (bitmap + counts) -- fetchUpdates() then needs records, so it re-runs
  void launch(void* stream = nullptr, bool records = true);
  // how launch() computes a variant: kFull re-runs its SPF from scratch,
  // kRepair repairs the base SPF below the failed tight links
  // (OGS_F_INCREMENTAL, every record written), kChangedOnly repairs and
  // writes only changed records and no per-variant SPF state
  // (OGS_F_CHANGED_ONLY: routeUpdate / counts / changedPrefixes only)
  enum Mode { kFull = 0, kRepair = 1, kChangedOnly = 2 };
  void setMode(Mode m) { mode_ = m; }
  Mode mode() const { return mode_; }
  // counts -> offsets -> device gather of the changed records -> host
  void fetchUpdates(void* stream = nullptr);
  // bitmap + counts, and every variant's full records when the launch wrote
  // them (parity tests)
  void fetchRecords(void* stream = nullptr);

  size_t numVariants() const { return dead_.size() / kDeadMax; }
  const DecisionRouteDb& baseRouteDb() const;             // after a launch
  DecisionRouteUpdate routeUpdate(size_t v) const;        // after fetchUpdates
  // every variant's update, materialised on `threads` host threads (0: up to
  // 16 / the hardware's); variants are independent, so the batch splits
  std::vector<DecisionRouteUpdate> routeUpdates(int threads = 0) const;
  ChangeRecords changeRecords() const;  // the fetched compact records
  DecisionRouteDb routeDb(size_t v) const;                // after fetchRecords
  std::vector<std::string> changedPrefixes(size_t v) const;  // after either
  std::pair<uint32_t, uint32_t> counts(size_t v) const;   // {update, delete}
  uint64_t totalChanges() const { return offsets_.empty() ? 0 : offsets_.back(); }
  int nhWords() const { return W_; }
  const HostBatch& batch() const { return hb_; }
  uint32_t flags() const;

 private:
  static constexpr int kDeadMax = 4;  // <= 2 links x 2 directions
  static constexpr size_t kDescMaxNodes = 16384;  // ogs_route_diff.base_desc bound
  ogs_graph graph() const;
  ogs_prefix_table table() const;
  void exactLaunch(void* stream);
  void exactFetch(void* stream);
  const LinkState& ls_;
  const PrefixState& ps_;
  std::string me_, area_;
  bool enableV4_, brs_, v4OverV6_;
  PrefixHostTable table_;
  HostBatch hb_;
  int W_{1};
  size_t words_{1}, Sp_{1};
  bool baseRun_{false}, recordsRun_{false}, changedOnlyRun_{false};
  bool descValid_{false};  // bDesc_ holds the base's descendant rows
  DeviceBuffer bDesc_;
  Mode mode_{kRepair};
  std::vector<uint32_t> dead_;
  DeviceBuffer dNodeBase_, dDesc_, dRow_, dEdges_, dEdgeSrc_, dFlags_, dPfxBase_,
      dAdvOff_, dAdvNode_, dAdvMetrics_, dAdvMinNh_, dPfxFlags_, dUnits_,
      dBaseUnit_, dDead_, dAdvClass_;
  DeviceBuffer bDist_, bNh_, bMeta_, bMetric_, bMask_, bSel_;
  DeviceBuffer dDist_, dNh_, dMeta_, dMetric_, dMask_, dSel_, dChanged_, dCounts_;
  DeviceBuffer dOffsets_, cPrefix_, cMeta_, cMetric_, cMask_;
  mutable std::optional<DecisionRouteDb> base_;
  std::vector<uint32_t> baseMeta_, baseMetric_, baseMask_;
  std::vector<uint32_t> counts_, changed_, offsets_;
  std::vector<uint32_t> cPrefixH_, cMetaH_, cMetricH_, cMaskH_;  // compact
  std::vector<uint32_t> meta_, metric_, mask_;                   // full
  // zero / negative metrics or 64-bit path sums: one topology per variant
  // through ogs_spf_routes (exactLaunch), updates by calculateUpdate
  bool exact_{false}, exactOrder_{false};
  // the exact domain runs in chunks of kExactChunk topologies (device and
  // host memory O(chunk x (E + P)) instead of O(variants x (E + P)));
  // records of every topology (0 = base, v + 1 = variant v) on the host
  static constexpr size_t kExactChunk = 256;
  std::vector<uint32_t> xMeta_, xMask_;
  std::vector<uint64_t> xMetric_;
  std::vector<DecisionRouteDb> xDb_;
  std::vector<DecisionRouteUpdate> xUpd_;
};

// ----------------------------------------------------------- RouteDbBatch --
// the RouteDbs of MANY sources of one area computed in
// one launch per next-hop width group and kept in HBM, then served per node
// the way Decision::getDecisionRouteDb (Decision.cpp:341-360, behind
// OpenrCtrl getRouteDbComputed, OpenrCtrlHandler.cpp:640-643) serves one:
// SpfSolver::buildRouteDb(node) (incl. the solver's static routes and node
// labels) -> DecisionRouteDb::toThrift with thisNodeName. Only the requested
// node's records cross PCIe. No RibPolicy (getDecisionRouteDb applies none).
// `solver`, the LinkStates and `ps` must outlive the batch unchanged.
// Over a multi-area domain the build is LAZY: launch() records nothing and
// each routeDb(node) runs that node's multi-area buildRouteDb on a private
// solver (serialised by a mutex, so concurrent routeDb calls are safe) from
// the live LinkStates / PrefixState -- which is why they must stay unchanged.
class RouteDbBatch {
 public:
  RouteDbBatch(const SpfSolver& solver, const AreaLinkStates& areaLinkStates,
               const PrefixState& ps, const std::vector<std::string>& sources);
  void launch(void* stream = nullptr);  // asynchronous
  // nullopt when `node` has no adjacency database (SpfSolver.cpp:318-324);
  // std::out_of_range when `node` is not one of the batch's sources
  std::optional<DecisionRouteDb> routeDb(const std::string& node, void* stream = nullptr) const;
  // getDecisionRouteDb: empty routes when there is no RouteDb
  RouteDatabase getRouteDbComputed(const std::string& node, void* stream = nullptr) const;
  size_t numSources() const { return sources_.size(); }
  size_t numGroups() const { return groups_.size(); }

 private:
  struct UnitRecords;
  bool fetchUnit(const std::string& node, void* stream, UnitRecords& r) const;

 public:

 private:
  struct Group {
    int W{1};
    std::vector<uint32_t> members;  // source index per unit of this group
    DeviceBuffer units, dist, nh, meta, metric, mask, sel, reach;
  };
  ogs_graph graph() const;
  ogs_prefix_table table() const;
  const SpfSolver& solver_;
  const LinkState* ls_{nullptr};
  std::string area_;
  PrefixHostTable table_;
  HostBatch hb_;
  bool wide_{false}, exact_{false};
  std::vector<std::string> sources_;
  std::map<std::string, size_t> index_;
  std::vector<std::pair<size_t, size_t>> units_;  // source -> (group, unit)
  std::vector<Group> groups_;
  DeviceBuffer dDesc_, dPfxBase_, dAdvOff_, dAdvNode_, dAdvMetrics_, dAdvMinNh_,
      dPfxFlags_;
  bool launched_{false};
  // multi-area domain: served node by node through a private solver's
  // multi-area buildRouteDb (areaLinkStates / prefixState must outlive it)
  bool multiArea_{false};
  const AreaLinkStates* als_{nullptr};
  const PrefixState* ps_{nullptr};
  std::unique_ptr<SpfSolver> multi_;
  mutable std::mutex multiMu_;  // routeDb() mutates multi_'s memo
};

}  // namespace openr_amd
