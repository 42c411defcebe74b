// link_state.h — host-side mirror of OpenR's LinkState whose SPF runs on the
// MI355X engine (libopenr_spf_hip, include/openr_spf.h).
//
// Public surface and semantics follow openr/decision/LinkState.h:339-452:
// links exist only when both ends advertise each other with matching
// interface names, are kept once per undirected link in per-node hash sets
// keyed by the folly hash of the ordered (node, ifName) pairs (so iteration
// order — which fixes pathLinks and KSP2 order — matches the reference), and
// SPF / KSP results are memoised until a topology change.
//
// What differs is where runSpf happens: the graph is snapshotted into a CSR
// (node id = rank of the node name in byte order, rows sorted by neighbour
// id, link_rank = position in linksFromNode iteration) and handed to the
// engine, which returns per-root distances and next-hop bitsets. SpfResult
// objects (names, next-hop name sets, ordered pathLinks) are rebuilt from
// those arrays on demand.
#pragma once

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdint>
#include <exception>
#include <functional>
#include <iterator>
#include <memory>
#include <mutex>
#include <thread>
#include <optional>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../../include/openr_adjdb.h"
#include "../engine/host_pool.h"
#include "../../../include/openr_spf.h"

namespace odl {

using Metric = uint64_t;

// Run f(lo, hi) over [0, n) in chunks handed out to up to 16 host threads
// (rows differ in length by 1000x: spines vs racks). The first exception a
// chunk throws is rethrown on the calling thread after every thread joined.
template <class F>
void parallelFor(uint32_t n, F&& f, uint32_t chunk = 64) {
  const uint32_t hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const uint32_t nt = std::max(1u, std::min(hw, n / (4 * chunk)));
  if (nt == 1) {
    f(0u, n);
    return;
  }
  // the persistent pool (host_pool.h); threads of its own when it is busy
  if (host_pool::Pool::get().run(n, chunk, nt, [&](uint32_t lo, uint32_t hi) { f(lo, hi); }))
    return;
  std::atomic<uint32_t> next{0};
  std::exception_ptr err;
  std::atomic<bool> failed{false};
  auto work = [&] {
    for (;;) {
      const uint32_t lo = next.fetch_add(chunk);
      if (lo >= n || failed.load()) return;
      try {
        f(lo, std::min(n, lo + chunk));
      } catch (...) {
        if (!failed.exchange(true)) err = std::current_exception();
        return;
      }
    }
  };
  std::vector<std::thread> th;
  th.reserve(nt - 1);
  for (uint32_t t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
  if (err) std::rethrow_exception(err);
}

// std::sort of v on up to 16 host threads: sorted slices merged pairwise
template <class T>
void parallelSort(std::vector<T>& v) {
  const size_t n = v.size();
  uint32_t C = 1;
  const uint32_t hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  while (C * 2 <= hw && n / (C * 2) >= 4096) C *= 2;
  if (C == 1) {
    std::sort(v.begin(), v.end());
    return;
  }
  std::vector<size_t> b(C + 1);
  for (uint32_t k = 0; k <= C; ++k) b[k] = n * k / C;
  // fn(k) for k < m, one thread each (the calling thread runs k = 0)
  auto each = [](uint32_t m, const std::function<void(uint32_t)>& fn) {
    if (host_pool::Pool::get().run(m, 1, m, [&](uint32_t lo, uint32_t hi) {
          for (uint32_t k = lo; k < hi; ++k) fn(k);
        }))
      return;
    std::vector<std::thread> th;
    for (uint32_t k = 1; k < m; ++k) {
      try {
        th.emplace_back(fn, k);
      } catch (const std::system_error&) {
        fn(k);
      }
    }
    fn(0);
    for (auto& t : th) t.join();
  };
  each(C, [&](uint32_t k) { std::sort(v.begin() + b[k], v.begin() + b[k + 1]); });
  for (uint32_t w = 1; w < C; w *= 2)
    each(C / (2 * w), [&](uint32_t q) {
      std::inplace_merge(v.begin() + b[2 * q * w], v.begin() + b[2 * q * w + w],
                         v.begin() + b[2 * q * w + 2 * w]);
    });
}

struct Adjacency {
  std::string otherNodeName, ifName, otherIfName;
  int32_t metric = 1;
  int32_t adjLabel = 0;
  bool isOverloaded = false;
  int64_t weight = 1;
  bool adjOnlyUsedByOtherNode = false;  // read by Decision's filter only
};

struct AdjacencyDatabase {
  std::string thisNodeName;
  bool isOverloaded = false;
  int32_t nodeLabel = 0;
  std::vector<Adjacency> adjacencies;
};

// A value whose change can be held back for a number of decrementHolds()
// calls (HoldableValue, LinkState.h:26-62 / LinkState.cpp:48-117): ordered
// FIB programming. A change "bringing up" (overload true -> false, a metric
// decrease) is held holdUpTtl calls, any other holdDownTtl; value() is the
// held value meanwhile. A second change while a hold is on drops the hold.
template <class T>
class HoldableValue {
 public:
  explicit HoldableValue(T v) : val_(v) {}
  void operator=(T v) {
    val_ = v;
    held_.reset();
    ttl_ = 0;
  }
  const T& value() const { return held_ ? *held_ : val_; }
  bool hasHold() const { return held_.has_value(); }
  // true when a hold expired (the value changed)
  bool decrementTtl() {
    if (held_ && --ttl_ == 0) {
      held_.reset();
      return true;
    }
    return false;
  }
  // true when the change is effective now (no hold taken)
  bool updateValue(T v, Metric holdUpTtl, Metric holdDownTtl) {
    if (v == val_) return false;
    if (hasHold()) {  // a change on top of a hold: the fast update
      held_.reset();
      ttl_ = 0;
    } else {
      ttl_ = bringsUp(v) ? holdUpTtl : holdDownTtl;
      if (ttl_ != 0) held_ = val_;
    }
    val_ = v;
    return !hasHold();
  }

 private:
  bool bringsUp(T v) const {
    if constexpr (std::is_same_v<T, bool>) return val_ && !v;  // overload cleared
    else return v < val_;                                       // metric decreased
  }
  T val_;
  std::optional<T> held_;
  Metric ttl_ = 0;
};

// One undirected link (LinkState.h:80-182).
class Link {
 public:
  Link(const std::string& n1, const Adjacency& a1, const std::string& n2, const Adjacency& a2);

  const std::string& otherNode(const std::string& n) const;
  const std::string& ifaceFrom(const std::string& n) const;
  Metric metricFrom(const std::string& n) const;
  bool overloadFrom(const std::string& n) const;
  int32_t adjLabelFrom(const std::string& n) const;
  int64_t weightFrom(const std::string& n) const;
  bool isUp() const {
    return holdUpTtl_ == 0 && !end_[0].overload.value() && !end_[1].overload.value();
  }

  // attribute updates from node n; return value per LinkState.cpp:284-330
  // (hold TTLs: LinkState.cpp:313-360)
  bool setMetricFrom(const std::string& n, Metric m, Metric holdUpTtl = 0, Metric holdDownTtl = 0);
  // true iff isUp() flipped
  bool setOverloadFrom(const std::string& n, bool ov, Metric holdUpTtl = 0, Metric holdDownTtl = 0);
  // a new link is held down for holdUpTtl decrementHolds() calls
  // (LinkState.cpp:237-263)
  void setHoldUpTtl(Metric ttl) { holdUpTtl_ = ttl; }
  bool decrementHolds();  // true when a hold expired
  bool hasHolds() const;
  void setAdjLabelFrom(const std::string& n, int32_t l);
  void setWeightFrom(const std::string& n, int64_t w);

  const std::string& lowNode() const { return end_[lo_].node; }
  const std::string& highNode() const { return end_[lo_ ^ 1].node; }
  bool sameLink(const Link& o) const;
  bool orderedBefore(const Link& o) const;  // Link::operator< (hash, names)
  std::string key() const;                  // "n1%if1|n2%if2" (ordered)

  const size_t hash;
  // id of this link in the CSR snapshot that last listed it (LinkState::linkIdOf
  // checks it still does)
  mutable uint32_t snapLid = 0xFFFFFFFFu;
  mutable uint32_t snapEnd[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};  // snapshot node ids of the ends
  int endIndex(const std::string& n) const { return end_[0].node == n ? 0 : 1; }
  int lowIndex() const { return lo_; }
  bool selfLoop() const { return end_[0].node == end_[1].node; }
  Metric metricOfEnd(int i) const { return end_[i].metric.value(); }

 private:
  struct End {
    std::string node, iface;
    HoldableValue<Metric> metric{1};
    HoldableValue<bool> overload{false};
    int32_t adjLabel = 0;
    int64_t weight = 0;
  };
  End& endOf(const std::string& n);
  const End& endOf(const std::string& n) const;
  End end_[2];
  Metric holdUpTtl_ = 0;
  uint8_t lo_ = 0;  // end_[lo_] is the lower (node, iface) pair, end_[lo_ ^ 1] the higher
  static size_t hashOf(const End& lo, const End& hi);
};

using LinkPtr = std::shared_ptr<Link>;
struct LinkPtrHash {
  size_t operator()(const LinkPtr& l) const { return l->hash; }
};
struct LinkPtrEq {
  bool operator()(const LinkPtr& a, const LinkPtr& b) const { return a->sameLink(*b); }
};
using LinkSet = std::unordered_set<LinkPtr, LinkPtrHash, LinkPtrEq>;

struct PathLink {
  LinkPtr link;
  std::string prevNode;
};

// The CSR snapshot the engine sees: node id = rank of the name in byte order,
// rows sorted by (neighbour id, linkRank), linkRank = position of the link in
// linksFromNode(row node), link ids handed out on first sight in node order
// (later: an added link takes a retired id or a new one). Shared with the
// engine-backed SpfResults made on it (they index its rows).
struct CsrSnapshot {
  std::vector<std::string> names;                 // id -> name (sorted)
  std::unordered_map<std::string, uint32_t> ids;  // name -> id
  std::vector<uint32_t> rowPtr, col, metric, linkId, twin, linkRank;
  std::vector<uint8_t> edgeUp, noTransit;
  std::vector<LinkPtr> links;      // link id -> link (null: a retired id)
  std::vector<uint32_t> freeLids;  // retired ids, taken again by added links
  std::vector<uint64_t> rowMax;    // largest in-contract out-metric per node
};

// One engine run (or KSP2 masked rerun): distance and next-hop rows of the
// root, kept with the snapshot they index; SpfResult entries are rebuilt from
// them on first access.
struct SpfRows {
  std::shared_ptr<const CsrSnapshot> csr;
  uint32_t root = 0;
  uint32_t W = 1;                 // next-hop words per node
  bool useLinkMetric = true;
  std::vector<uint32_t> dist;     // [V], OSPF_DIST_INF = unreached
  std::vector<uint32_t> nh;       // [V][W] (empty: next hops not kept)
  std::vector<uint32_t> nbrs;     // the root's distinct neighbours = next-hop bit order
  std::vector<uint32_t> ignored;  // sorted link ids the run ignored
  // pathLinks of v: every usable tight in-link (l, u), u transit or the root,
  // in (u's pop order (dist, name), l's position in linksFromNode(u)) order
  // (LinkState.cpp:885-901)
  std::vector<PathLink> pathLinksOf(uint32_t v) const;
  std::unordered_set<std::string> nextHopsOf(uint32_t v) const;
};

// LinkState::NodeSpfResult (LinkState.h:211-268). A result of the engine
// keeps only its metric eagerly; nextHops and pathLinks are rebuilt from the
// run's rows on first access (thread-safe: the route build reads results on
// host threads), so getSpfResult costs O(V) words, not O(V) hash sets.
class NodeSpfResult {
 public:
  explicit NodeSpfResult(Metric m) : metric_(m) {}
  NodeSpfResult(NodeSpfResult&& o) noexcept
      : metric_(o.metric_), pathLinks_(std::move(o.pathLinks_)), nextHops_(std::move(o.nextHops_)),
        rows_(o.rows_), node_(o.node_) {}
  NodeSpfResult& operator=(NodeSpfResult&& o) noexcept {
    metric_ = o.metric_;
    pathLinks_ = std::move(o.pathLinks_);
    nextHops_ = std::move(o.nextHops_);
    rows_ = o.rows_;
    node_ = o.node_;
    return *this;
  }
  // a copy is a materialised one
  NodeSpfResult(const NodeSpfResult& o)
      : metric_(o.metric_), pathLinks_(o.pathLinks()), nextHops_(o.nextHops()) {}
  Metric metric() const { return metric_; }
  const std::vector<PathLink>& pathLinks() const {
    if (rows_) std::call_once(plOnce_, [this] { pathLinks_ = rows_->pathLinksOf(node_); });
    return pathLinks_;
  }
  const std::unordered_set<std::string>& nextHops() const {
    if (rows_) std::call_once(nhOnce_, [this] { nextHops_ = rows_->nextHopsOf(node_); });
    return nextHops_;
  }

 private:
  friend class LinkState;
  friend class SpfResult;
  NodeSpfResult(Metric m, const SpfRows* rows, uint32_t node) : metric_(m), rows_(rows), node_(node) {}
  Metric metric_;
  mutable std::vector<PathLink> pathLinks_;
  mutable std::unordered_set<std::string> nextHops_;
  const SpfRows* rows_ = nullptr;  // lazy: the run's rows (owned by the SpfResult)
  uint32_t node_ = 0;
  mutable std::once_flag plOnce_, nhOnce_;
};

// LinkState::SpfResult (LinkState.h:267-268: unordered_map<string,
// NodeSpfResult>) with the map's read interface -- find / count / at / size /
// iteration over (name, NodeSpfResult) pairs. A host-path result is a map; an
// engine result holds the run's rows and makes an entry the first time it is
// looked up or iterated over (iteration in node id = name order).
class SpfResult {
 public:
  using value_type = std::pair<const std::string, NodeSpfResult>;
  using Map = std::unordered_map<std::string, NodeSpfResult>;
  class const_iterator {
   public:
    using iterator_category = std::forward_iterator_tag;
    using value_type = SpfResult::value_type;
    using difference_type = std::ptrdiff_t;
    using pointer = const value_type*;
    using reference = const value_type&;
    const_iterator() = default;
    reference operator*() const { return r_->rows_ ? r_->entry(k_) : *m_; }
    pointer operator->() const { return &**this; }
    const_iterator& operator++() {
      if (r_->rows_) ++k_;
      else ++m_;
      return *this;
    }
    const_iterator operator++(int) {
      const_iterator t = *this;
      ++*this;
      return t;
    }
    bool operator==(const const_iterator& o) const { return r_ == o.r_ && k_ == o.k_ && m_ == o.m_; }
    bool operator!=(const const_iterator& o) const { return !(*this == o); }

   private:
    friend class SpfResult;
    const SpfResult* r_ = nullptr;
    Map::const_iterator m_{};
    size_t k_ = 0;
  };
  using iterator = const_iterator;

  SpfResult() = default;
  explicit SpfResult(Map&& m) : map_(std::move(m)) {}
  explicit SpfResult(std::shared_ptr<const SpfRows> rows);
  SpfResult(SpfResult&& o) noexcept;
  SpfResult& operator=(SpfResult&& o) noexcept;
  SpfResult(const SpfResult&) = delete;
  SpfResult& operator=(const SpfResult&) = delete;
  ~SpfResult() { release(); }

  size_t size() const { return rows_ ? reached_.size() : map_.size(); }
  bool empty() const { return size() == 0; }
  const_iterator begin() const;
  const_iterator end() const;
  const_iterator find(const std::string& node) const;
  size_t count(const std::string& node) const { return find(node) != end() ? 1 : 0; }
  const NodeSpfResult& at(const std::string& node) const;
  // the engine run behind the result (null for a host-path result)
  const std::shared_ptr<const SpfRows>& rows() const { return rows_; }

 private:
  const value_type& entry(size_t k) const;  // reached_[k]'s entry, made on first use
  void release();
  Map map_;
  std::shared_ptr<const SpfRows> rows_;
  std::vector<uint32_t> reached_;  // reached node ids, ascending
  std::unique_ptr<std::atomic<value_type*>[]> slot_;  // [reached_.size()]
};

using Path = std::vector<LinkPtr>;

// thrift::PrefixForwardingAlgorithm values of the two UCMP algorithms
enum class UcmpAlgo : int { kAdjWeightPropagation = 2, kPrefixWeightPropagation = 3 };

// LinkState::NodeUcmpResult (LinkState.h:275-333)
class NodeUcmpResult {
 public:
  struct NextHopLink {
    LinkPtr link;
    std::string nextHopNode;
    int64_t weight = 0;
  };
  const std::unordered_map<std::string, NextHopLink>& nextHopLinks() const {
    return nextHopLinks_;
  }
  std::optional<int64_t> weight() const { return weight_; }
  void setWeight(int64_t w) { weight_ = w; }
  void addNextHopLink(const std::string& localIface, const LinkPtr& link,
                      const std::string& nextHopNode, int64_t weight) {
    nextHopLinks_.emplace(localIface, NextHopLink{link, nextHopNode, weight});
  }
  void normalizeNextHopWeights();

 private:
  std::unordered_map<std::string, NextHopLink> nextHopLinks_;
  std::optional<int64_t> weight_;
};
using UcmpResult = std::unordered_map<std::string, NodeUcmpResult>;

struct LinkStateChange {
  bool topologyChanged = false;
  bool linkAttributesChanged = false;
  bool nodeLabelChanged = false;
  std::vector<LinkPtr> addedLinks;
  // applyKvs: the key's value did not decode; the key was skipped, as
  // Decision::updateKeyInLsdb catches, logs and skips it (Decision.cpp:803-806)
  bool decodeError = false;
};

// Raised for engine failures (no device, engine error). Graphs outside the
// engine's metric contract (a metric 0 or negative i32 adjacency, or
// distances that may not fit u32) are not an error: their link-metric runs
// take LinkState's host path (runSpfHost), the reference's own algorithm.
struct EngineError : std::runtime_error {
  int code;
  EngineError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

struct MemoReaper;

class LinkState {
 public:
  LinkState(std::string area, int device);
  // several devices of the node (SURVEY.md §8(b) n_gpus): the graph is
  // replicated, all-sources sweeps run one root partition part per device
  LinkState(std::string area, std::vector<int> devices);
  ~LinkState();
  LinkState(const LinkState&) = delete;
  LinkState& operator=(const LinkState&) = delete;

  const std::string& area() const { return area_; }
  // holdUpTtl / holdDownTtl: LinkState::updateAdjacencyDatabase's hold TTLs
  // (LinkState.cpp:585-700; Decision passes 0, Decision.cpp:756)
  LinkStateChange updateAdjacencyDatabase(const AdjacencyDatabase& db, Metric holdUpTtl = 0,
                                          Metric holdDownTtl = 0);
  // one step of every hold (LinkState.cpp:520-548): topologyChanged when one
  // expired (the memo is dropped then); hasHolds: any hold left
  LinkStateChange decrementHolds();
  bool hasHolds() const;
  LinkStateChange deleteAdjacencyDatabase(const std::string& node);
  // A batch of databases in order (Decision's debounced batch,
  // Decision.cpp:731-765; the initial sync delivers the whole area): the same
  // state and change records as updateAdjacencyDatabase on each in turn. A
  // batch of nodes not yet known (no name twice) is built with host threads.
  // The databases are moved from.
  std::vector<LinkStateChange> updateAdjacencyDatabases(std::vector<AdjacencyDatabase>& dbs,
                                                        Metric holdUpTtl = 0,
                                                        Metric holdDownTtl = 0);
  // Decision::processPublication's LinkState part (Decision.cpp:846-870):
  // every key-value in order -- an "adj:" key with a value decoded from
  // compact thrift (on host threads) and applied (updateKeyInLsdb,
  // :743-765), TTL-only values and other keys skipped -- then every expired
  // "adj:" key deleted (deleteKeyFromLsdb, :812-826). myNodeName (may be
  // null) turns on filterUnuseableAdjacency (:568-600). One change record
  // per key-value, then per expired key (empty for skipped ones). A value
  // that fails to decode skips only its own key (decodeError set, the reason
  // in lastDecodeError()); the rest of the publication is applied.
  struct KvIn {
    std::string_view key, value;
    bool hasValue = false;
  };
  std::vector<LinkStateChange> applyKvs(const std::vector<KvIn>& kvs,
                                        const std::vector<std::string_view>& expired,
                                        const std::string* myNodeName);
  // the last decode failure of applyKvs ("" when none) and how many so far
  const std::string& lastDecodeError() const { return lastDecodeError_; }
  uint64_t decodeErrors() const { return decodeErrors_; }

  const LinkSet& linksFromNode(const std::string& node) const;
  bool isNodeOverloaded(const std::string& node) const;
  size_t numLinks() const {
    size_t k = 0;
    for (const auto& s : allLinks_) k += s.size();
    return k;
  }
  size_t numNodes() const { return adjDbs_.size(); }
  const std::unordered_map<std::string, AdjacencyDatabase>& getAdjacencyDatabases() const {
    return adjDbs_;
  }

  const SpfResult& getSpfResult(const std::string& node, bool useLinkMetric = true);
  std::optional<Metric> getMetricFromAToB(const std::string& a, const std::string& b,
                                          bool useLinkMetric = true);
  const std::vector<Path>& getKthPaths(const std::string& src, const std::string& dst, size_t k);
  static bool pathAInPathB(const Path& a, const Path& b);
  // LinkState::resolveUcmpWeights (LinkState.cpp:913-1033): host walk of the
  // SPF DAG (computed on the engine) from equally distant weighted leaves.
  UcmpResult resolveUcmpWeights(const SpfResult& spfGraph,
                                const std::unordered_map<std::string, int64_t>& leafNodeToWeights,
                                UcmpAlgo algo, bool useLinkMetric = true) const;

  // ---- batched entry points (no reference counterpart) ----
  void prefetchSpf(const std::vector<std::string>& roots, bool useLinkMetric);
  std::vector<ospf_digest> spfDigests(const std::vector<std::string>& roots, bool useLinkMetric);
  void prefetchKsp2(const std::string& src, const std::vector<std::string>& dsts);
  // All-sources: runSpf for every node in one engine sweep (ospf_sweep_*,
  // one part per device), rows kept resident on the devices; getSpfResult /
  // prefetchSpf of any node then copies its rows instead of running again
  // (decision.spf_runs counts the V runs of the sweep once). The reference's
  // all-sources use is getDecisionRouteDb(node) for every node
  // (Decision.cpp:309).
  void prefetchAllSources(bool useLinkMetric = true);
  // digests of every node (node-id order = snapshot().names) from one sweep
  std::vector<ospf_digest> allSourcesDigests(bool useLinkMetric = true);
  bool isMemoised(const std::string& root, bool useLinkMetric) const {
    return (useLinkMetric ? memoMetric_ : memoHops_).count(root) > 0;
  }
  // drop memoised results (bounded host memory for all-nodes route builds)
  void evictSpf(const std::vector<std::string>& roots, bool useLinkMetric);
  // prefetchSpf takes the sweep when it is asked for at least this many
  // roots not yet memoised (and at least half of the nodes)
  static constexpr size_t kSweepMinRoots = 256;
  struct SweepStats {
    uint64_t sweeps = 0, rows_copied = 0;
    uint32_t mode = 0, devices = 0, hip_graph = 0;
  };
  const SweepStats& sweepStats() const { return sweepStats_; }

  uint64_t spfRuns() const { return spfRuns_; }

  // ---- device errors (degrade, never abort Decision) ----
  // An engine call that fails (any OSPF_E_* other than an out-of-contract
  // input, which the host path already takes) does not escape: the LinkState
  // records it, releases the engine and switches to its host path
  // (runSpfHost, the reference algorithm -- product code, not the oracle) for
  // every later SPF / KSP2 / digest, and the failed call is answered there.
  // setHostSpf(false) re-enables the engine. The reference instead ends in
  // XLOG(FATAL) when an exception leaves the Decision fiber
  // (Decision.cpp:240-250).
  // fb303 counters of the path (LinkState.cpp:843,909,926,1029;
  // SpfSolver.cpp:640-644): decision.spf_runs COUNT, decision.spf_ms /
  // ucmp_ms / route_build_ms AVG -- kept as sums and sample counts (AVG =
  // sum / samples). A batched engine call is charged to its logical runs.
  struct Counters {
    uint64_t spf_runs = 0, spf_ms_samples = 0;
    double spf_ms_sum = 0;
    uint64_t ucmp_runs = 0;
    double ucmp_ms_sum = 0;
    uint64_t route_build_runs = 0;
    double route_build_ms_sum = 0;
  };
  Counters counters() const {
    Counters c = counters_;
    c.spf_runs = spfRuns_;
    return c;
  }
  void addRouteBuild(double ms) {
    ++counters_.route_build_runs;
    counters_.route_build_ms_sum += ms;
  }
  uint64_t engineErrors() const { return engineErrors_; }
  const std::string& lastEngineError() const { return lastEngineError_; }
  // test hook: the after-th engine call from now fails with OSPF_E_DEVICE
  // (ospf_inject_error; applied when the engine opens)
  void injectEngineError(uint32_t after);
  // degrade on device errors (default on; off: the EngineError escapes, as
  // before). A LinkState whose engine never opened (no device) always
  // throws: there is no silent CPU path for a box without a GPU. The
  // environment variable ODL_STRICT_ENGINE turns it off at construction (the
  // test suite sets it, so a GPU test cannot pass on the host path).
  void setDegradeOnError(bool on) { degradeOnError_ = on; }

  // ---- incremental mode (off by default) ----
  // The reference drops every memoised SPF on a topology change
  // (LinkState.cpp:751-754). With incremental mode on, an update that only
  // changes link metrics, link up state or node overload bits (no link or
  // node added or removed) keeps the result of every root the change cannot
  // affect -- no changed link was on its shortest-path DAG before, none
  // reaches or ties a distance after, no re-flagged reached node can relax
  // (the rule of ospf_affected_roots, on the memoised SpfResults) -- and
  // patches the CSR and the device graph in place instead of re-snapshotting.
  // Results are identical; decision.spf_runs then counts only the re-runs.
  void setIncremental(bool on) { incremental_ = on; }
  struct IncrementalStats {
    uint64_t patches = 0, kept = 0, dropped = 0;
  };
  const IncrementalStats& incrementalStats() const { return incStats_; }

  // ---- CSR snapshot (what the engine sees) ----
  using Csr = CsrSnapshot;
  const Csr& snapshot();
  uint32_t linkIdOf(const Link& l) const;  // id in the current snapshot
  // true when the current snapshot is outside the engine's metric contract:
  // link-metric SPF / KSP2 then run on the host (hop-count runs stay on the
  // engine)
  bool hostMetricMode() {
    snapshot();
    return hostMetric_;
  }
  // Every SPF / KSP2 / digest on the host (runSpfHost, the reference
  // algorithm), the engine never opened: a GPU-free run of the whole ingest /
  // patch / memo logic (sanitizer builds, link-event sequences on the CPU).
  // Also set by the environment variable ODL_HOST_SPF at construction.
  void setHostSpf(bool on) {
    hostOnly_ = on;
    if (!on) degraded_ = false;
  }
  bool degraded() const { return degraded_; }
  bool hostSpf() const { return hostOnly_; }
  // Links added or removed between known nodes ([LINK UP] / [LINK DOWN],
  // LinkState.cpp:632-657) patch the snapshot and the device graph in place
  // (ospf_update_rows) instead of a new snapshot and device load.
  struct TopologyStats {
    uint64_t snapshots = 0;     // whole CSR snapshots taken
    uint64_t loads = 0;         // whole device graph loads
    uint64_t link_patches = 0;  // updates patched in place with links added / removed
    uint64_t rows_patched = 0;  // CSR rows rebuilt by them
    uint64_t node_patches = 0;  // nodes added / removed in place (ids renumbered)
  };
  const TopologyStats& topologyStats() const { return topoStats_; }

  // Root batches (prefetchSpf outside a sweep: a KSP2 source, LFA-style
  // neighbour batches) and KSP2 destinations split across the device slots
  // of a multi-device LinkState; one host thread per slot, the
  // records land in the caller's host arrays (Decision consumes them there).
  struct ShardStats {
    uint64_t spf_batches = 0;   // batches split across slots
    uint64_t spf_launches = 0;  // per-slot launches of them
    uint64_t ksp2_runs = 0;     // KSP2 prefetches split across slots
    uint64_t ksp2_launches = 0; // per-slot ospf_ksp2_run calls of them
  };
  const ShardStats& shardStats() const { return shardStats_; }

 private:
  LinkPtr makeLink(const std::string& node, const Adjacency& adj) const;
  void addLink(const LinkPtr& l);
  void removeLink(const LinkPtr& l);
  std::vector<LinkPtr> sortedLinksOf(const std::string& node) const;
  void invalidate();
  void clearMemo();
  void ensureEngine();
  void dropSweep();
  bool sweepHas(bool useLinkMetric) const;
  // copy rows of roots (all owned by the current sweep) into dist / nh (W words)
  void sweepRows(const std::vector<uint32_t>& roots, uint32_t W, std::vector<uint32_t>& dist,
                 std::vector<uint32_t>& nh);
  uint32_t nhWordsFor(uint32_t root) const;
  std::vector<uint32_t> nbrsOf(uint32_t root) const;  // distinct neighbours (bit order)
  void runBatch(const std::vector<uint32_t>& roots, const std::vector<std::vector<uint32_t>>* ign,
                bool useLinkMetric, uint32_t flags, uint32_t W, std::vector<uint32_t>* dist,
                std::vector<uint32_t>* nh, std::vector<ospf_digest>* dig);
  // the engine's device slots (slot 0 = engine_; after ensureEngine)
  std::vector<ospf_ctx*> slots() const;
  // runBatch's launch on one slot into dist / nh rows at the given offsets
  int batchOn(ospf_ctx* c, const uint32_t* roots, uint32_t n, bool useLinkMetric, uint32_t flags,
              uint32_t W, uint32_t* dist, uint32_t* nh) const;
  std::optional<Path> trace(const SpfRows& run, uint32_t src, uint32_t x,
                            std::unordered_set<const Link*>& seen) const;
  std::vector<Path> tracePaths(const SpfRows& run, uint32_t src, uint32_t dst) const;
  // the engine rows of getSpfResult(node, true) (the memo's, or a re-run
  // when the memoised result came from another snapshot)
  std::shared_ptr<const SpfRows> rawSpf(const std::string& node);
  // LinkState::runSpf (LinkState.cpp:836-911) on the host, u64 metrics with
  // the reference's wrap-around, for graphs outside the engine contract
  SpfResult runSpfHost(const std::string& root, bool useLinkMetric,
                       const std::unordered_set<const Link*>& ignore) const;
  // traceOnePath (LinkState.cpp:418-439) over a host result's pathLinks
  std::vector<Path> tracePathsHost(const SpfResult& res, const std::string& src,
                                   const std::string& dst) const;
  ospf_digest digestHost(const std::string& root, const SpfResult& res) const;
  struct LinkDelta {  // a kept link whose metric or up state changed
    LinkPtr link;
    bool up0;
    Metric mlo0, mhi0;  // metric advertised by lowNode / highNode before
  };
  // links added / removed between known nodes: the rows of their ends
  // rebuilt in the snapshot (same node ids), then ospf_update_rows
  void patchStructure(const std::vector<LinkPtr>& added, const std::vector<LinkPtr>& removed);
  void applyIncremental(const std::vector<LinkDelta>& links,
                        const std::vector<std::string>& nodes);
  void patchGraph(const std::vector<LinkDelta>& links, const std::vector<std::string>& nodes);
  // links of the rows in `rows` to the engine (ospf_update_rows), or a reload
  void patchEngineRows(const std::vector<uint32_t>& rows);
  // a node enters / leaves the snapshot in place (node id = name rank: ids
  // from k on move by one); its row is empty (links: patchStructure). The
  // device graph reloads on its next use (the node count changed).
  void csrInsertNode(uint32_t k, const std::string& name, bool overloaded);
  void csrEraseNode(uint32_t k);
  Csr& csrForWrite();  // copy-on-write when a kept memoised result reads it

  std::string area_;
  std::string lastDecodeError_;
  uint64_t decodeErrors_ = 0;
  int device_;
  std::vector<int> devices_;
  ospf_multi* multi_ = nullptr;  // devices_.size() > 1: owns engine_ (its slot 0)
  ospf_ctx* engine_ = nullptr;
  ospf_sweep* sweep_ = nullptr;     // single device
  ospf_msweep* msweep_ = nullptr;   // several devices
  uint64_t sweepVersion_ = 0;       // snapshot version the sweep's rows describe
  bool sweepMetric_ = true;
  SweepStats sweepStats_;
  uint64_t engineVersion_ = 0;  // snapshot version loaded into the engine
  uint64_t version_ = 1;        // bumped on every ingest call
  uint64_t snapVersion_ = 0;
  std::shared_ptr<Csr> csr_ = std::make_shared<Csr>();
  TopologyStats topoStats_;
  ShardStats shardStats_;
  bool hostMetric_ = false;   // snapshot outside the engine's metric contract
  bool hostOnly_ = false;     // setHostSpf: no engine at all
  bool degraded_ = false;     // hostOnly_ set by a device error
  bool degradeOnError_ = true;
  bool engineOpened_ = false;  // an engine context was opened once
  int guardDepth_ = 0;        // nesting of the public entry points (guarded)
  uint64_t engineErrors_ = 0;
  std::string lastEngineError_;
  uint32_t injectAfter_ = 0;  // test hook, handed to the engine when it opens
  mutable Counters counters_;  // spf_runs lives in spfRuns_
  // run f; an EngineError escaping the outermost public entry point degrades
  // the LinkState to its host path and runs f again there
  template <class F>
  decltype(auto) guarded(F&& f);
  void onEngineError(const std::exception& e);
  const SpfResult& getSpfResultImpl(const std::string& node, bool useLinkMetric);
  void prefetchSpfImpl(const std::vector<std::string>& roots, bool useLinkMetric);
  std::vector<ospf_digest> spfDigestsImpl(const std::vector<std::string>& roots, bool useLinkMetric);
  void prefetchAllSourcesImpl(bool useLinkMetric);
  std::vector<ospf_digest> allSourcesDigestsImpl(bool useLinkMetric);
  const std::vector<Path>& getKthPathsImpl(const std::string& src, const std::string& dst, size_t k);
  void prefetchKsp2Impl(const std::string& src, const std::vector<std::string>& dsts);
  bool hostRun(bool useLinkMetric) const { return hostOnly_ || (useLinkMetric && hostMetric_); }
  uint64_t distBound_ = 0;    // >= every simple-path metric sum of the snapshot
  uint64_t spfRuns_ = 0;
  bool incremental_ = false;
  IncrementalStats incStats_;

  std::unordered_map<std::string, LinkSet> linkMap_;
  // every link, in shards by hash (only membership and the count are read;
  // the bulk path fills the shards on separate threads)
  static constexpr uint32_t kLinkShards = 16;
  std::array<LinkSet, kLinkShards> allLinks_;
  LinkSet& shardOf(const Link& l) { return allLinks_[(l.hash >> 7) % kLinkShards]; }
  std::unordered_map<std::string, HoldableValue<bool>> nodeOverloads_;
  std::unordered_map<std::string, AdjacencyDatabase> adjDbs_;
  // per node: (otherNodeName, ifName, otherIfName) -> adjacency position; the
  // views point into adjDbs_[node]'s own strings and are rebuilt with it
  struct AdjKey {
    std::string_view other, ifn, oifn;
    bool operator==(const AdjKey& o) const { return other == o.other && ifn == o.ifn && oifn == o.oifn; }
  };
  struct AdjKeyHash {
    size_t operator()(const AdjKey& k) const;
  };
  std::unordered_map<std::string, std::unordered_map<AdjKey, uint32_t, AdjKeyHash>> adjIndex_;

  std::unordered_map<std::string, SpfResult> memoMetric_, memoHops_;
  std::unordered_map<std::string, std::vector<Path>> memoKsp_;
  // frees dropped memos on one background thread (clearMemo); joined by the
  // destructor
  std::unique_ptr<struct MemoReaper> reaper_;
  // the engine opened on a host thread beside a bulk ingest (Decision opens
  // its device at start; here the first bulk ingest does):
  // the HIP runtime's start and the kernels' code objects are loaded by a
  // tiny warm-up run, off the first getSpfResult's path. ensureEngine joins.
  std::thread opener_;
  ospf_ctx* openerCtx_ = nullptr;
  void startOpen(size_t nodes);  // nodes: the warm-up graph's size
  void joinOpen();
};

}  // namespace odl
