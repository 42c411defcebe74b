// link_state.cpp — LinkState mirror (see link_state.h); SPF on the engine.
#include "link_state.h"

#include <cstdlib>
#include <cstring>
#include <numeric>
#include <set>
#include <algorithm>
#include <unordered_set>
#include <system_error>
#include <thread>
#include <functional>
#include <map>
#include <stdexcept>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <cstdio>
#include <thread>
#include <tuple>

namespace odl {

namespace {

// folly::hash::hash_128_to_64 (folly rev 04c2275157a3e44c1d1fa1df75835fe4ec8a7b1e,
// folly/hash/Hash.h), used by folly's std::hash<std::pair> specialisation that
// the reference's Link hash relies on (LinkState.cpp:134-138).
inline uint64_t fold(uint64_t hi, uint64_t lo) {
  constexpr uint64_t kMul = 0x9ddfea08eb382d69ULL;
  uint64_t a = (lo ^ hi) * kMul;
  a ^= a >> 47;
  uint64_t b = (hi ^ a) * kMul;
  b ^= b >> 47;
  return b * kMul;
}

inline uint64_t hashEnd(const std::string& node, const std::string& iface) {
  const std::hash<std::string> h;
  return fold(h(node), h(iface));  // std::hash<std::pair<string, string>>
}

constexpr uint32_t kInf = OSPF_DIST_INF;

}  // namespace

// ---------------------------------------------------------------- Link
// One thread per LinkState frees dropped memos, in the order they were
// dropped; the LinkState's destructor drains the queue and joins it, so no
// release outlives the object (r04 had a detached thread per event). Only
// memory unreachable from the LinkState is handed over: the SpfResults own
// their rows and entries, and the Links / snapshots they share are
// reference-counted (std::shared_ptr, atomic counts).
struct MemoReaper {
  using Memo = std::unordered_map<std::string, SpfResult>;
  struct Dead {
    Memo a, b;
    std::unordered_map<std::string, std::vector<Path>> k;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::unique_ptr<Dead>> q;
  bool stop = false;
  std::thread th;
  MemoReaper() : th([this] { loop(); }) {}
  ~MemoReaper() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_one();
    th.join();
  }
  void push(std::unique_ptr<Dead> d) {
    {
      std::lock_guard<std::mutex> g(mu);
      q.push_back(std::move(d));
    }
    cv.notify_one();
  }
  void loop() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [this] { return stop || !q.empty(); });
      if (q.empty()) return;  // stop, and everything freed
      std::unique_ptr<Dead> d = std::move(q.front());
      q.pop_front();
      lk.unlock();
      d.reset();
      lk.lock();
    }
  }
};

size_t Link::hashOf(const End& lo, const End& hi) {
  return fold(hashEnd(lo.node, lo.iface), hashEnd(hi.node, hi.iface));
}

size_t LinkState::AdjKeyHash::operator()(const AdjKey& k) const {
  const std::hash<std::string_view> h;
  return fold(h(k.other), fold(h(k.ifn), h(k.oifn)));
}

static bool endLess(const std::string& n1, const std::string& i1, const std::string& n2,
                    const std::string& i2) {
  const int c = n1.compare(n2);
  return c < 0 || (c == 0 && i1 < i2);
}

// The ends are stored once, end_[lo_] holding the smaller (node, iface) pair
// -- the reference's n1/if1 after its ordering (LinkState.cpp:95-110).
Link::Link(const std::string& n1, const Adjacency& a1, const std::string& n2, const Adjacency& a2)
    : hash([&] {
        return endLess(n2, a2.ifName, n1, a1.ifName)
                   ? fold(hashEnd(n2, a2.ifName), hashEnd(n1, a1.ifName))
                   : fold(hashEnd(n1, a1.ifName), hashEnd(n2, a2.ifName));
      }()) {
  lo_ = endLess(n2, a2.ifName, n1, a1.ifName) ? 1 : 0;
  const Adjacency* adj[2] = {&a1, &a2};
  const std::string* nn[2] = {&n1, &n2};
  for (int i = 0; i < 2; ++i) {
    end_[i].node = *nn[i];
    end_[i].iface = adj[i]->ifName;
    end_[i].metric = (Metric)(int64_t)adj[i]->metric;  // i32 -> u64 as the reference
    end_[i].overload = (bool)adj[i]->isOverloaded;
    end_[i].adjLabel = adj[i]->adjLabel;
    end_[i].weight = adj[i]->weight;
  }
}

Link::End& Link::endOf(const std::string& n) {
  if (end_[0].node == n) return end_[0];
  if (end_[1].node == n) return end_[1];
  throw std::invalid_argument(n);
}
const Link::End& Link::endOf(const std::string& n) const {
  return const_cast<Link*>(this)->endOf(n);
}
const std::string& Link::otherNode(const std::string& n) const {
  if (end_[0].node == n) return end_[1].node;
  if (end_[1].node == n) return end_[0].node;
  throw std::invalid_argument(n);
}
const std::string& Link::ifaceFrom(const std::string& n) const { return endOf(n).iface; }
Metric Link::metricFrom(const std::string& n) const { return endOf(n).metric.value(); }
bool Link::overloadFrom(const std::string& n) const { return endOf(n).overload.value(); }
int32_t Link::adjLabelFrom(const std::string& n) const { return endOf(n).adjLabel; }
int64_t Link::weightFrom(const std::string& n) const { return endOf(n).weight; }

bool Link::setMetricFrom(const std::string& n, Metric m, Metric holdUpTtl, Metric holdDownTtl) {
  return endOf(n).metric.updateValue(m, holdUpTtl, holdDownTtl);
}
bool Link::setOverloadFrom(const std::string& n, bool ov, Metric holdUpTtl, Metric holdDownTtl) {
  const bool wasUp = isUp();
  endOf(n).overload.updateValue(ov, holdUpTtl, holdDownTtl);
  return wasUp != isUp();
}
bool Link::decrementHolds() {
  bool expired = false;
  if (holdUpTtl_ != 0) expired |= --holdUpTtl_ == 0;
  for (End& e : end_) {
    expired |= e.metric.decrementTtl();
    expired |= e.overload.decrementTtl();
  }
  return expired;
}
bool Link::hasHolds() const {
  return holdUpTtl_ != 0 || end_[0].metric.hasHold() || end_[1].metric.hasHold() ||
         end_[0].overload.hasHold() || end_[1].overload.hasHold();
}
void Link::setAdjLabelFrom(const std::string& n, int32_t l) { endOf(n).adjLabel = l; }
void Link::setWeightFrom(const std::string& n, int64_t w) { endOf(n).weight = w; }

bool Link::sameLink(const Link& o) const {
  const End &a = end_[lo_], &b = end_[lo_ ^ 1], &c = o.end_[o.lo_], &d = o.end_[o.lo_ ^ 1];
  return hash == o.hash && a.node == c.node && a.iface == c.iface && b.node == d.node &&
         b.iface == d.iface;
}
bool Link::orderedBefore(const Link& o) const {
  if (hash != o.hash) return hash < o.hash;
  const End &a = end_[lo_], &b = end_[lo_ ^ 1], &c = o.end_[o.lo_], &d = o.end_[o.lo_ ^ 1];
  return std::tie(a.node, a.iface, b.node, b.iface) < std::tie(c.node, c.iface, d.node, d.iface);
}
std::string Link::key() const {
  const End &a = end_[lo_], &b = end_[lo_ ^ 1];
  return a.node + "%" + a.iface + "|" + b.node + "%" + b.iface;
}

// ---------------------------------------------------------------- LinkState
LinkState::LinkState(std::string area, int device)
    : area_(std::move(area)), device_(device), devices_{device} {
  hostOnly_ = getenv("ODL_HOST_SPF") != nullptr;
  degradeOnError_ = getenv("ODL_STRICT_ENGINE") == nullptr;
}

LinkState::LinkState(std::string area, std::vector<int> devices)
    : area_(std::move(area)), device_(devices.empty() ? 0 : devices[0]), devices_(std::move(devices)) {
  if (devices_.empty()) throw std::invalid_argument("LinkState: no device");
  hostOnly_ = getenv("ODL_HOST_SPF") != nullptr;
  degradeOnError_ = getenv("ODL_STRICT_ENGINE") == nullptr;
}

LinkState::~LinkState() {
  joinOpen();
  reaper_.reset();  // drains the dropped memos, joins the thread
  dropSweep();
  if (multi_) ospf_multi_close(multi_);
  else if (engine_) ospf_close(engine_);
}

const LinkSet& LinkState::linksFromNode(const std::string& node) const {
  static const LinkSet kEmpty;
  auto it = linkMap_.find(node);
  return it == linkMap_.end() ? kEmpty : it->second;
}

bool LinkState::isNodeOverloaded(const std::string& node) const {
  auto it = nodeOverloads_.find(node);
  return it != nodeOverloads_.end() && it->second.value();
}

LinkStateChange LinkState::decrementHolds() {
  LinkStateChange ch;
  for (auto& shard : allLinks_)
    for (const auto& l : shard) ch.topologyChanged |= l->decrementHolds();
  for (auto& kv : nodeOverloads_) ch.topologyChanged |= kv.second.decrementTtl();
  // an expired hold changes what the snapshot holds (metrics, up state, node
  // overload): the memo is dropped (LinkState.cpp:530-533) and the CSR taken
  // again
  if (ch.topologyChanged) invalidate();
  return ch;
}

bool LinkState::hasHolds() const {
  for (const auto& shard : allLinks_)
    for (const auto& l : shard)
      if (l->hasHolds()) return true;
  for (const auto& kv : nodeOverloads_)
    if (kv.second.hasHold()) return true;
  return false;
}

LinkPtr LinkState::makeLink(const std::string& node, const Adjacency& adj) const {
  auto other = adjDbs_.find(adj.otherNodeName);
  if (other == adjDbs_.end()) return nullptr;
  auto idx = adjIndex_.find(adj.otherNodeName);
  if (idx == adjIndex_.end()) return nullptr;
  auto hit = idx->second.find(AdjKey{node, adj.otherIfName, adj.ifName});
  if (hit == idx->second.end()) return nullptr;
  return std::make_shared<Link>(node, adj, adj.otherNodeName,
                                other->second.adjacencies[hit->second]);
}

void LinkState::addLink(const LinkPtr& l) {
  if (!linkMap_[l->lowNode()].insert(l).second || !linkMap_[l->highNode()].insert(l).second ||
      !shardOf(*l).insert(l).second)
    throw std::logic_error("duplicate link " + l->key());
}

void LinkState::removeLink(const LinkPtr& l) {
  if (!linkMap_.at(l->lowNode()).erase(l) || !linkMap_.at(l->highNode()).erase(l) ||
      !shardOf(*l).erase(l))
    throw std::logic_error("missing link " + l->key());
}

std::vector<LinkPtr> LinkState::sortedLinksOf(const std::string& node) const {
  const LinkSet& s = linksFromNode(node);
  std::vector<LinkPtr> v(s.begin(), s.end());
  std::sort(v.begin(), v.end(), [](const LinkPtr& a, const LinkPtr& b) {
    return a->orderedBefore(*b);
  });
  return v;
}

static size_t V_of(const LinkState::Csr& c) { return c.names.size(); }

void LinkState::clearMemo() {
  if (memoMetric_.empty() && memoHops_.empty() && memoKsp_.empty()) return;
  // A route build materialises every entry of its results (~100k node
  // results with next-hop sets and path links at F100k): freeing them took
  // most of an event's apply time, so the reaper thread frees them.
  auto dead = std::make_unique<MemoReaper::Dead>();
  dead->a.swap(memoMetric_);
  dead->b.swap(memoHops_);
  dead->k.swap(memoKsp_);
  if (!reaper_) {
    try {
      reaper_ = std::make_unique<MemoReaper>();
    } catch (const std::system_error&) {  // no thread to spare: free here
      return;
    }
  }
  reaper_->push(std::move(dead));
}

void LinkState::invalidate() {
  ++version_;
  dropSweep();
  clearMemo();
}

LinkStateChange LinkState::updateAdjacencyDatabase(const AdjacencyDatabase& db, Metric holdUpTtl,
                                                   Metric holdDownTtl) {
  LinkStateChange ch;
  const std::string me = db.thisNodeName;
  const bool known = adjDbs_.count(me) > 0;
  const int32_t priorLabel = known ? adjDbs_.at(me).nodeLabel : 0;
  bool structural = !known;  // a link or node added / removed (incremental mode)
  std::vector<LinkDelta> deltas;
  std::vector<std::string> nodeDeltas;
  std::vector<LinkPtr> removedLinks;
  auto& idx = adjIndex_[me];
  idx.clear();  // (its views point into the database replaced here)
  const AdjacencyDatabase& kept = adjDbs_[me] = db;
  for (uint32_t i = 0; i < kept.adjacencies.size(); ++i) {
    const auto& a = kept.adjacencies[i];
    idx.emplace(AdjKey{a.otherNodeName, a.ifName, a.otherIfName}, i);
  }

  std::vector<LinkPtr> before = sortedLinksOf(me);
  std::vector<LinkPtr> after;
  after.reserve(db.adjacencies.size());
  for (const auto& a : db.adjacencies)
    if (LinkPtr l = makeLink(me, a)) after.push_back(std::move(l));
  std::sort(after.begin(), after.end(),
            [](const LinkPtr& a, const LinkPtr& b) { return a->orderedBefore(*b); });

  auto ov = nodeOverloads_.find(me);
  if (ov == nodeOverloads_.end()) {
    nodeOverloads_.emplace(me, db.isOverloaded);  // a new node is not a change
  } else {
    const bool was = ov->second.value();
    ch.topologyChanged |= ov->second.updateValue(db.isOverloaded, holdUpTtl, holdDownTtl);
    if (ov->second.value() != was) nodeDeltas.push_back(me);
  }
  ch.nodeLabelChanged = priorLabel != db.nodeLabel;

  // two-pointer merge of old vs new link sets (both in Link::operator< order)
  size_t i = 0, j = 0;
  while (i < after.size() || j < before.size()) {
    const bool takeNew = i < after.size() && (j == before.size() || after[i]->orderedBefore(*before[j]));
    const bool takeOld = !takeNew && j < before.size() &&
                         (i == after.size() || before[j]->orderedBefore(*after[i]));
    if (takeNew) {
      structural = true;
      after[i]->setHoldUpTtl(holdUpTtl);
      ch.topologyChanged |= after[i]->isUp();
      addLink(after[i]);
      ch.addedLinks.push_back(after[i]);
      ++i;
    } else if (takeOld) {
      structural = true;
      ch.topologyChanged |= before[j]->isUp();
      removeLink(before[j]);
      removedLinks.push_back(before[j]);
      ++j;
    } else {
      const Link& fresh = *after[i];
      Link& kept = *before[j];
      if (fresh.metricFrom(me) != kept.metricFrom(me) ||
          fresh.overloadFrom(me) != kept.overloadFrom(me))
        deltas.push_back(LinkDelta{before[j], kept.isUp(), kept.metricFrom(kept.lowNode()),
                                   kept.metricFrom(kept.highNode())});
      if (fresh.metricFrom(me) != kept.metricFrom(me))
        ch.topologyChanged |= kept.setMetricFrom(me, fresh.metricFrom(me), holdUpTtl, holdDownTtl);
      if (fresh.overloadFrom(me) != kept.overloadFrom(me))
        ch.topologyChanged |=
            kept.setOverloadFrom(me, fresh.overloadFrom(me), holdUpTtl, holdDownTtl);
      if (fresh.adjLabelFrom(me) != kept.adjLabelFrom(me)) {
        kept.setAdjLabelFrom(me, fresh.adjLabelFrom(me));
        ch.linkAttributesChanged = true;
      }
      if (fresh.weightFrom(me) != kept.weightFrom(me)) {
        kept.setWeightFrom(me, fresh.weightFrom(me));
        ch.linkAttributesChanged = true;
      }
      ++i;
      ++j;
    }
  }
  // Incremental mode: same nodes and links, CSR current -> patch in place
  // (not in host-metric mode, and only while the patched metrics keep the
  // engine contract: an in-range increase raises the distance bound by at
  // most the new metric)
  bool keepsContract = !hostMetric_;
  uint64_t bound = distBound_;
  for (const auto& d : deltas) {
    for (const Metric m : {d.link->metricFrom(d.link->lowNode()), d.link->metricFrom(d.link->highNode())}) {
      keepsContract &= m >= 1 && m <= 0xFFFFFFFFull;
      bound += keepsContract ? m : 0;
    }
  }
  // links added between known nodes: their metrics join the bound
  for (const auto& l : ch.addedLinks)
    for (const Metric m : {l->metricFrom(l->lowNode()), l->metricFrom(l->highNode())}) {
      keepsContract &= m >= 1 && m <= 0xFFFFFFFFull;
      bound += keepsContract ? m : 0;
    }
  keepsContract &= bound < 0xFFFFFFFFull;
  // [LINK UP] / [LINK DOWN] between known nodes (LinkState.cpp:632-657): the
  // snapshot and the device graph are patched in place; the memo is dropped on
  // a topology change as in the reference (:751-754) -- in incremental mode
  // too (its kept-root rule covers metric / up / overload changes only)
  if (known && structural && snapVersion_ == version_ && keepsContract &&
      !getenv("ODL_NO_LINK_PATCH")) {
    if (ch.topologyChanged || incremental_) {
      if (incremental_) incStats_.dropped += memoMetric_.size() + memoHops_.size();
      clearMemo();
    }
    // kept links' metric / up changes first (on the rows as they are), so the
    // rebuilt rows and their partners agree when the structure is patched
    if (!deltas.empty() || !nodeDeltas.empty()) patchGraph(deltas, nodeDeltas);
    patchStructure(ch.addedLinks, removedLinks);
    return ch;
  }
  if (incremental_ && !structural && snapVersion_ == version_ && keepsContract) {
    distBound_ = bound;
    if (ch.topologyChanged) applyIncremental(deltas, nodeDeltas);
    return ch;
  }
  // The same nodes and links: the snapshot stays (node ids are name ranks,
  // unchanged). Metric / up / overload changes are patched into the CSR and
  // the device graph in place; the memo is dropped on a topology change,
  // exactly as in the reference (LinkState.cpp:751-754), and survives
  // attribute-only updates (:721-724: labels, weights).
  if (!structural && snapVersion_ == version_ && keepsContract) {
    distBound_ = bound;
    if (ch.topologyChanged) clearMemo();
    if (!deltas.empty() || !nodeDeltas.empty()) patchGraph(deltas, nodeDeltas);
    return ch;
  }
  // a node added while the snapshot is current: its (empty) row enters in
  // place, then the links it formed (peers that already advertised it)
  // patch their rows; the device graph reloads on its next use
  if (!known && snapVersion_ == version_ && keepsContract && !getenv("ODL_NO_LINK_PATCH")) {
    if (ch.topologyChanged) clearMemo();
    engineVersion_ = 0;
    const auto& nm = csr_->names;
    const uint32_t k = (uint32_t)(std::lower_bound(nm.begin(), nm.end(), me) - nm.begin());
    csrInsertNode(k, me, db.isOverloaded);
    patchStructure(ch.addedLinks, {});
    return ch;
  }
  // a metric leaving the engine contract, or a change without a current
  // snapshot: the CSR is snapshotted again
  if (ch.topologyChanged) {
    invalidate();
  } else {
    ++version_;
  }
  return ch;
}

// Bulk path: every database is a node not yet known. Such a node has no
// links before its own update (a link needs both databases), and its update
// creates the links to the nodes known by then -- before the batch, earlier
// in it, or itself -- in Link order, inserted into the low then the high
// node's LinkSet and into allLinks_. Built here: databases and adjacency
// indexes per node in parallel, each node's created links in parallel (the
// indexes are only read), then every node's LinkSet filled in parallel with
// its links in the sequential insertion order (creation order), so each
// unordered_set ends up with the same buckets and iteration order.
std::vector<LinkStateChange> LinkState::updateAdjacencyDatabases(std::vector<AdjacencyDatabase>& dbs,
                                                                Metric holdUpTtl,
                                                                Metric holdDownTtl) {
  const auto tIn = std::chrono::steady_clock::now();
  const uint32_t n = (uint32_t)dbs.size();
  std::vector<LinkStateChange> out(n);
  // (the bulk path makes links without holds)
  bool bulk = n >= 64 && holdUpTtl == 0 && !getenv("ODL_NO_BULK_INGEST");
  std::unordered_map<std::string, uint32_t> posOf;
  if (bulk) {
    posOf.reserve(n);
    for (uint32_t i = 0; i < n && bulk; ++i)
      bulk = !adjDbs_.count(dbs[i].thisNodeName) && posOf.emplace(dbs[i].thisNodeName, i).second;
  }
  if (!bulk) {
    for (uint32_t i = 0; i < n; ++i) out[i] = updateAdjacencyDatabase(dbs[i], holdUpTtl, holdDownTtl);
    return out;
  }

  using Clock = std::chrono::steady_clock;
  const bool timing = getenv("ODL_SPF_TIMING") != nullptr;
  Clock::time_point tp[6];
  tp[0] = Clock::now();
  std::vector<AdjacencyDatabase*> dbp(n);
  std::vector<std::unordered_map<AdjKey, uint32_t, AdjKeyHash>*> idxp(n);
  // (no order of these maps or of allLinks_ is observed: node ids are name
  // ranks; only the per-node LinkSets' iteration order is, and those are not
  // reserved)
  adjDbs_.reserve(adjDbs_.size() + n);
  adjIndex_.reserve(adjIndex_.size() + n);
  nodeOverloads_.reserve(nodeOverloads_.size() + n);
  linkMap_.reserve(linkMap_.size() + n);
  for (uint32_t i = 0; i < n; ++i) {
    const std::string me = dbs[i].thisNodeName;
    nodeOverloads_.emplace(me, dbs[i].isOverloaded);  // a new node is not a change
    out[i].nodeLabelChanged = dbs[i].nodeLabel != 0;
    AdjacencyDatabase& slot = adjDbs_[me];
    slot = std::move(dbs[i]);
    dbp[i] = &slot;
    idxp[i] = &adjIndex_[me];
  }
  parallelFor(n, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) {
      auto& idx = *idxp[i];
      idx.clear();
      const auto& adj = dbp[i]->adjacencies;
      idx.reserve(adj.size());
      for (uint32_t k = 0; k < adj.size(); ++k)
        idx.emplace(AdjKey{adj[k].otherNodeName, adj[k].ifName, adj[k].otherIfName}, k);
    }
  }, 256);
  // links each update creates, in Link order
  tp[1] = Clock::now();
  // (link, batch position of its other end or kNone) per update
  std::vector<std::vector<std::pair<LinkPtr, uint32_t>>> created(n);
  parallelFor(n, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) {
      const AdjacencyDatabase& db = *dbp[i];
      auto& v = created[i];
      for (const auto& a : db.adjacencies) {
        auto p = posOf.find(a.otherNodeName);
        if (p != posOf.end() && p->second > i) continue;  // created by that node's update
        if (LinkPtr l = makeLink(db.thisNodeName, a))
          v.emplace_back(std::move(l), p != posOf.end() ? p->second : kInf);
      }
      std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) {
        return a.first->orderedBefore(*b.first);
      });
    }
  }, 256);
  tp[2] = Clock::now();
  // every touched node's insertions in creation order (low end, then high)
  std::unordered_map<std::string, uint32_t> other;  // nodes known before the batch
  // (pointers into out[i].addedLinks, reserved up front: no reallocation)
  std::vector<std::vector<const LinkPtr*>> ins(n);
  std::array<std::vector<const LinkPtr*>, kLinkShards> shardIns;
  bool anyTopo = false;
  for (uint32_t i = 0; i < n; ++i) {
    out[i].addedLinks.reserve(created[i].size());
    for (auto& c : created[i]) {
      out[i].addedLinks.push_back(std::move(c.first));
      const LinkPtr* l = &out[i].addedLinks.back();
      if (c.second == i) throw std::logic_error("duplicate link " + (*l)->key());  // a self-link
      uint32_t o = c.second;
      if (o == kInf) {
        auto q = other.emplace((*l)->otherNode(dbp[i]->thisNodeName), (uint32_t)ins.size());
        if (q.second) ins.emplace_back();
        o = q.first->second;
      }
      const bool meLow = (*l)->lowNode() == dbp[i]->thisNodeName;
      ins[meLow ? i : o].push_back(l);
      ins[meLow ? o : i].push_back(l);
      out[i].topologyChanged |= (*l)->isUp();
      shardIns[((*l)->hash >> 7) % kLinkShards].push_back(l);
    }
    anyTopo |= out[i].topologyChanged;
  }
  created = {};
  tp[3] = Clock::now();
  std::vector<LinkSet*> setp(ins.size());
  for (uint32_t i = 0; i < n; ++i) setp[i] = &linkMap_[dbp[i]->thisNodeName];
  for (const auto& o : other) setp[o.second] = &linkMap_[o.first];
  std::atomic<bool> dup{false};
  parallelFor((uint32_t)ins.size(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t u = lo; u < hi; ++u)
      for (const LinkPtr* l : ins[u])
        if (!setp[u]->insert(*l).second) dup = true;
  }, 256);
  parallelFor(kLinkShards, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t s = lo; s < hi; ++s) {
      allLinks_[s].reserve(allLinks_[s].size() + shardIns[s].size());
      for (const LinkPtr* l : shardIns[s])
        if (!allLinks_[s].insert(*l).second) dup = true;
    }
  }, 1);
  tp[4] = Clock::now();
  if (timing) {
    auto ms = [&](int a) { return std::chrono::duration<double, std::milli>(tp[a + 1] - tp[a]).count(); };
    std::fprintf(stderr, "ODL_INGEST dbs=%u check_ms=%.1f index_ms=%.1f links_ms=%.1f order_ms=%.1f sets_ms=%.1f\n",
                 n, std::chrono::duration<double, std::milli>(tp[0] - tIn).count(), ms(0), ms(1), ms(2), ms(3));
  }
  if (dup) throw std::logic_error("duplicate link in an adjacency database batch");
  // one version step per database, as in turn (a new node is structural)
  version_ += n - (anyTopo ? 1u : 0u);
  if (anyTopo) invalidate();
  // (after the ingest, not beside it: the HIP runtime's start beside the
  // ingest's page-fault-heavy host work slowed the ingest by ~150-290 ms
  // at F100k, more than it saved the first getSpfResult, c9 vs c5)
  startOpen(adjDbs_.size());
  return out;
}

LinkStateChange LinkState::deleteAdjacencyDatabase(const std::string& node) {
  LinkStateChange ch;
  auto db = adjDbs_.find(node);
  if (db == adjDbs_.end()) return ch;
  // in place when the snapshot is current: the node's links leave their
  // rows (patchStructure), then its empty row leaves (ids above it move)
  const bool inPlace = snapVersion_ == version_ && !hostMetric_ && csr_->ids.count(node) &&
                       !getenv("ODL_NO_LINK_PATCH");
  std::vector<LinkPtr> removed;
  auto lm = linkMap_.find(node);
  if (lm != linkMap_.end()) {
    for (const auto& l : lm->second) {
      if (!linkMap_.at(l->otherNode(node)).erase(l) || !shardOf(*l).erase(l))
        throw std::logic_error("inconsistent link map");
      removed.push_back(l);
    }
    linkMap_.erase(lm);
    nodeOverloads_.erase(node);
  }
  adjDbs_.erase(db);
  adjIndex_.erase(node);
  ch.topologyChanged = true;
  if (!inPlace) {
    invalidate();
    return ch;
  }
  clearMemo();  // LinkState.cpp:751-754
  engineVersion_ = 0;  // the node count changes: the device graph reloads
  const uint32_t k = csr_->ids.at(node);
  patchStructure({}, removed);
  csrEraseNode(k);
  ++version_;
  snapVersion_ = version_;
  return ch;
}

// ---------------------------------------------------------------- snapshot

// Rows in parallel (threads over node ranges; the link sets are only read):
// 1. each row gathers its links (neighbour id, linksFromNode position, metric
//    from this end) and counts the links it sees first (smaller end id),
//    recording its own id on its end of each Link;
// 2. prefix sums give row offsets and link ids -- the same ids a sequential
//    sweep in (node id, linksFromNode order) hands out on first sight;
// 3. the lower end writes the link id into the Link, the upper end reads it;
// 4. rows are sorted by (neighbour id, rank) and written, then twins.
const LinkState::Csr& LinkState::snapshot() {
  if (snapVersion_ == version_) return *csr_;
  const bool tm = getenv("ODL_SNAP_TIMING") != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!tm) return;
    auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "snapshot %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
    t0 = t;
  };
  ++topoStats_.snapshots;
  Csr c;
  {
    // sorted by (first 8 bytes big-endian, then the whole name): 16-B keys
    // move and compare as integers (the string sort's merges had moved and
    // compared strings); the order is the names' byte-wise order either way
    struct NameKey {
      uint64_t k;
      const std::string* s;
      bool operator<(const NameKey& o) const { return k != o.k ? k < o.k : *s < *o.s; }
    };
    // the map's buckets walked on threads (its nodes are scattered on the
    // heap: a serial walk was ~14 ms of cache misses at 100k nodes)
    constexpr uint32_t kParts = 64;
    const size_t nbk = adjDbs_.bucket_count();
    std::vector<std::vector<NameKey>> part(kParts);
    parallelFor(kParts, [&](uint32_t lo, uint32_t hi) {
      for (uint32_t p = lo; p < hi; ++p) {
        auto& out = part[p];
        for (size_t b = nbk * p / kParts; b < nbk * (p + 1) / kParts; ++b)
          for (auto it = adjDbs_.begin(b); it != adjDbs_.end(b); ++it) {
            const std::string& n = it->first;
            uint64_t k = 0;
            for (size_t i = 0; i < std::min<size_t>(8, n.size()); ++i)
              k |= (uint64_t)(uint8_t)n[i] << (56 - 8 * i);
            out.push_back({k, &n});
          }
      }
    }, 1);
    std::vector<NameKey> keyed;
    keyed.reserve(adjDbs_.size());
    for (auto& v : part) keyed.insert(keyed.end(), v.begin(), v.end());
    parallelSort(keyed);
    c.names.reserve(keyed.size());
    for (const auto& x : keyed) c.names.push_back(*x.s);
  }
  lap("names sorted");
  c.ids.reserve(c.names.size() * 2);
  for (uint32_t i = 0; i < c.names.size(); ++i) c.ids.emplace(c.names[i], i);
  lap("names");
  const uint32_t V = (uint32_t)c.names.size();
  c.rowPtr.assign(V + 1, 0);
  c.noTransit.assign(V, 0);
  struct Ent {
    uint32_t v, rank, metric;
    uint8_t up, low, end;
    const LinkPtr* link;
  };
  std::vector<std::vector<Ent>> rows(V);
  std::vector<uint32_t> nfirst(V + 1, 0);
  std::vector<uint8_t> rowBad(V, 0);
  std::vector<uint64_t> rowMax(V, 0);
  parallelFor(V, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t u = lo; u < hi; ++u) {
      const std::string& un = c.names[u];
      c.noTransit[u] = isNodeOverloaded(un) ? 1 : 0;
      const LinkSet& ls = linksFromNode(un);
      auto& row = rows[u];
      row.reserve(ls.size());
      uint32_t rank = 0, nf = 0;
      for (const auto& l : ls) {
        Ent e;
        e.end = (uint8_t)l->endIndex(un);
        l->snapEnd[e.end] = u;
        if (e.end == 0 && l->selfLoop()) l->snapEnd[1] = u;
        const Metric m = l->metricOfEnd(e.end);
        e.v = kInf;  // the other end's id: written by its own row
        e.rank = rank++;
        // a metric outside [1, 2^32) (0, or a negative i32 wrapped to u64) is
        // outside the engine contract: the snapshot goes to host mode and the
        // engine (hop-count runs only) sees 1
        const bool inRange = m >= 1 && m <= 0xFFFFFFFFull;
        e.metric = inRange ? (uint32_t)m : 1u;
        if (!inRange) rowBad[u] = 1;
        rowMax[u] = std::max<uint64_t>(rowMax[u], inRange ? m : 0);
        e.up = l->isUp() ? 1 : 0;
        // the lower end by name = by id sees the link first in id order
        e.low = (e.end == l->lowIndex() || l->selfLoop()) ? 1 : 0;
        e.link = &l;
        nf += e.low;
        row.push_back(e);
      }
      nfirst[u + 1] = nf;
      c.rowPtr[u + 1] = (uint32_t)row.size();
    }
  });
  for (uint32_t u = 0; u < V; ++u) {
    nfirst[u + 1] += nfirst[u];
    c.rowPtr[u + 1] += c.rowPtr[u];
  }
  // A simple path leaves each node at most once, so sum_u max_out(u) bounds
  // every shortest distance: below 2^32 - 1 (the engine's unreached value)
  // the engine's u32 distances cannot overflow.
  uint64_t bound = 0;
  bool bad = false;
  for (uint32_t u = 0; u < V; ++u) {
    bad |= rowBad[u] != 0;
    bound = std::min<uint64_t>(bound + rowMax[u], ~0ull >> 1);
  }
  distBound_ = bound;
  hostMetric_ = bad || bound >= 0xFFFFFFFFull;
  lap("gather");
  const size_t E = c.rowPtr[V];
  c.links.resize(nfirst[V]);
  parallelFor(V, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t u = lo; u < hi; ++u) {
      uint32_t lid = nfirst[u];
      for (auto& e : rows[u]) {
        e.v = (*e.link)->snapEnd[e.end ^ 1];
        if (!e.low) continue;
        (*e.link)->snapLid = lid;
        c.links[lid++] = *e.link;
      }
    }
  });
  lap("link ids");
  // room for the links patchStructure may add in place
  for (auto* v : {&c.col, &c.metric, &c.linkId, &c.twin, &c.linkRank}) v->reserve(E + 4096 + E / 64);
  c.edgeUp.reserve(E + 4096 + E / 64);
  c.col.resize(E);
  c.metric.resize(E);
  c.linkId.resize(E);
  c.twin.resize(E);
  c.linkRank.resize(E);
  c.edgeUp.resize(E);
  std::vector<uint32_t> side(c.links.size() * 2, kInf);
  parallelFor(V, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t u = lo; u < hi; ++u) {
      auto& row = rows[u];
      std::sort(row.begin(), row.end(), [](const Ent& a, const Ent& b) {
        return a.v != b.v ? a.v < b.v : a.rank < b.rank;
      });
      size_t e = c.rowPtr[u];
      for (const auto& x : row) {
        const uint32_t lid = (*x.link)->snapLid;
        c.col[e] = x.v;
        c.metric[e] = x.metric;
        c.linkId[e] = lid;
        c.linkRank[e] = x.rank;
        c.edgeUp[e] = x.up;
        side[lid * 2ull + (x.low ? 0 : 1)] = (uint32_t)e;  // each (link, end) once
        ++e;
      }
    }
  });
  lap("rows sorted");
  parallelFor(V, [&](uint32_t lo, uint32_t hi) {
    for (size_t e = c.rowPtr[lo]; e < c.rowPtr[hi]; ++e) {
      const uint32_t lid = c.linkId[e];
      const uint32_t mine = side[lid * 2ull] == e ? 0u : 1u;
      c.twin[e] = side[lid * 2ull + (1u - mine)];
    }
  });
  lap("rows");
  c.rowMax = std::move(rowMax);
  csr_ = std::make_shared<Csr>(std::move(c));
  lap("move");
  snapVersion_ = version_;
  return *csr_;
}

uint32_t LinkState::linkIdOf(const Link& l) const {
  const uint32_t lid = l.snapLid;
  if (lid >= csr_->links.size() || csr_->links[lid].get() != &l)
    throw std::out_of_range("link not in the CSR snapshot");
  return lid;
}

// ---- device errors: degrade to the host path
template <class F>
decltype(auto) LinkState::guarded(F&& f) {
  if (guardDepth_) return f();  // an inner entry point: the outermost one handles it
  struct Depth {
    int& d;
    explicit Depth(int& x) : d(x) { ++d; }
    ~Depth() { --d; }
  };
  const uint64_t runs0 = spfRuns_;
  const size_t memo0 = memoMetric_.size() + memoHops_.size();
  // decision.spf_ms (LinkState.cpp:844,906-909): the call's time, charged to
  // the logical runs it made
  struct Timer {
    LinkState& ls;
    uint64_t runs0;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~Timer() {
      if (ls.spfRuns_ <= runs0) return;
      ls.counters_.spf_ms_samples += ls.spfRuns_ - runs0;
      ls.counters_.spf_ms_sum +=
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
  } timer{*this, runs0};
  try {
    Depth dp(guardDepth_);
    return f();
  } catch (const EngineError& e) {
    if (!degradeOnError_ || !engineOpened_) throw;
    onEngineError(e);
  }
  // runs memoised before the failure were made (and stay); the retry counts
  // its own
  spfRuns_ = runs0 + (memoMetric_.size() + memoHops_.size() - memo0);
  Depth dp(guardDepth_);
  return f();
}

void LinkState::onEngineError(const std::exception& e) {
  ++engineErrors_;
  lastEngineError_ = e.what();
  fprintf(stderr, "odl::LinkState(%s): engine error, continuing on the host path: %s\n",
          area_.c_str(), e.what());
  dropSweep();
  if (multi_) ospf_multi_close(multi_);
  else if (engine_) ospf_close(engine_);
  multi_ = nullptr;
  engine_ = nullptr;
  engineVersion_ = 0;
  hostOnly_ = true;
  degraded_ = true;
}

void LinkState::injectEngineError(uint32_t after) {
  injectAfter_ = after;
  if (engine_) {
    ospf_inject_error(engine_, after);
    injectAfter_ = 0;
  }
}

const SpfResult& LinkState::getSpfResult(const std::string& node, bool useLinkMetric) {
  return guarded([&]() -> const SpfResult& { return getSpfResultImpl(node, useLinkMetric); });
}
void LinkState::prefetchSpf(const std::vector<std::string>& roots, bool useLinkMetric) {
  guarded([&] { prefetchSpfImpl(roots, useLinkMetric); });
}
std::vector<ospf_digest> LinkState::spfDigests(const std::vector<std::string>& roots,
                                               bool useLinkMetric) {
  return guarded([&] { return spfDigestsImpl(roots, useLinkMetric); });
}
void LinkState::prefetchAllSources(bool useLinkMetric) {
  guarded([&] { prefetchAllSourcesImpl(useLinkMetric); });
}
std::vector<ospf_digest> LinkState::allSourcesDigests(bool useLinkMetric) {
  return guarded([&] { return allSourcesDigestsImpl(useLinkMetric); });
}
const std::vector<Path>& LinkState::getKthPaths(const std::string& src, const std::string& dst,
                                                size_t k) {
  return guarded([&]() -> const std::vector<Path>& { return getKthPathsImpl(src, dst, k); });
}
void LinkState::prefetchKsp2(const std::string& src, const std::vector<std::string>& dsts) {
  guarded([&] { prefetchKsp2Impl(src, dsts); });
}

void LinkState::startOpen(size_t nodes) {
  if (hostOnly_ || engine_ || opener_.joinable() || devices_.size() != 1 ||
      getenv("ODL_NO_PREOPEN"))
    return;
  // the warm-up: one link, one root (a warm-up graph as large as the
  // ingested one -- a hypercube, to size the batch path's buffers too -- cost
  // more on the first getSpfResult's path than the ~14 ms it saved there)
  (void)nodes;
  constexpr uint32_t V = 2;
  try {
    opener_ = std::thread([this, dev = device_] {
      ospf_ctx* c = nullptr;
      if (ospf_open(dev, &c) != OSPF_OK) return;
      const std::vector<uint32_t> rp{0, 1, 2}, col{1, 0}, one{1, 1}, lid{0, 0}, twin{1, 0};
      const std::vector<uint8_t> up{1, 1};
      const uint32_t E = 2;
      ospf_csr g{};
      g.n_nodes = V;
      g.n_edges = E;
      g.row_ptr = rp.data();
      g.col = col.data();
      g.metric = one.data();
      g.link_id = lid.data();
      g.twin = twin.data();
      g.edge_up = up.data();
      uint32_t root = 0;
      std::vector<uint32_t> dist(V), nh(V);
      if (ospf_load_graph(c, &g, 0) != OSPF_OK ||
          ospf_sssp_batch(c, &root, 1, nullptr, OSPF_WANT_DIST | OSPF_WANT_NH, 1, dist.data(),
                          nh.data(), nullptr) != OSPF_OK) {
        ospf_close(c);
        return;
      }
      openerCtx_ = c;
    });
  } catch (const std::system_error&) {  // no thread: the engine opens on first use
  }
}

void LinkState::joinOpen() {
  if (!opener_.joinable()) return;
  opener_.join();
  if (!openerCtx_) return;  // failed: ensureEngine opens (and reports) as before
  if (engine_ || hostOnly_) {
    ospf_close(openerCtx_);
  } else {
    engine_ = openerCtx_;
    engineOpened_ = true;
    engineVersion_ = 0;  // the warm-up graph: the snapshot loads on first use
  }
  openerCtx_ = nullptr;
}

void LinkState::ensureEngine() {
  snapshot();
  joinOpen();
  const auto t0 = std::chrono::steady_clock::now();
  const bool opening = !engine_, loading = engineVersion_ != snapVersion_;
  if (!engine_) {
    int rc = OSPF_OK;
    if (devices_.size() > 1) {
      rc = ospf_multi_open(devices_.data(), (uint32_t)devices_.size(), &multi_);
      if (rc == OSPF_OK) engine_ = ospf_multi_ctx(multi_, 0);
    } else {
      rc = ospf_open(device_, &engine_);
    }
    if (rc != OSPF_OK) {
      engine_ = nullptr;
      multi_ = nullptr;
      throw EngineError(rc, "ospf_open failed (no MI355X device / HIP runtime?)");
    }
    engineOpened_ = true;
  }
  if (injectAfter_) {
    ospf_inject_error(engine_, injectAfter_);
    injectAfter_ = 0;
  }
  const auto tOpen = std::chrono::steady_clock::now();
  if (engineVersion_ != snapVersion_) {
    dropSweep();
    ospf_csr g{};
    g.n_nodes = (uint32_t)csr_->names.size();
    g.n_edges = (uint32_t)csr_->col.size();
    g.row_ptr = csr_->rowPtr.data();
    g.col = csr_->col.data();
    g.metric = csr_->metric.data();
    g.link_id = csr_->linkId.data();
    g.twin = csr_->twin.data();
    g.edge_up = csr_->edgeUp.data();
    g.no_transit = csr_->noTransit.data();
    g.link_rank = csr_->linkRank.data();
    int rc = multi_ ? ospf_multi_load_graph(multi_, &g, snapVersion_)
                    : ospf_load_graph(engine_, &g, snapVersion_);
    if (rc != OSPF_OK)
      throw EngineError(rc, multi_ ? ospf_multi_last_error(multi_) : ospf_last_error(engine_));
    ++topoStats_.loads;
    engineVersion_ = snapVersion_;
  }
  if ((opening || loading) && getenv("ODL_SPF_TIMING"))
    fprintf(stderr, "ensure_engine open=%d load=%d open_ms=%.3f load_ms=%.3f\n", opening, loading,
            std::chrono::duration<double, std::milli>(tOpen - t0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tOpen).count());
}

void LinkState::dropSweep() {
  if (sweep_) ospf_sweep_destroy(sweep_);
  if (msweep_) ospf_msweep_destroy(msweep_);
  sweep_ = nullptr;
  msweep_ = nullptr;
  sweepVersion_ = 0;
}

bool LinkState::sweepHas(bool useLinkMetric) const {
  return (sweep_ || msweep_) && sweepVersion_ == snapVersion_ && sweepMetric_ == useLinkMetric &&
         snapVersion_ == version_;
}

void LinkState::prefetchAllSourcesImpl(bool useLinkMetric) {
  snapshot();
  if (sweepHas(useLinkMetric)) return;
  if (hostRun(useLinkMetric)) {  // outside the engine contract: the reference algorithm
    prefetchSpf(csr_->names, useLinkMetric);
    return;
  }
  ensureEngine();
  dropSweep();
  ospf_sweep_opts o{};
  // one run per snapshot: nothing to replay, and the create makes no run of
  // its own (OSPF_SWEEP_DEFER): the run below is the only one
  o.flags = (useLinkMetric ? 0u : OSPF_HOP_COUNT) | OSPF_SWEEP_DEFER;
  o.mode = OSPF_SWEEP_AUTO;
  o.hip_graph = 0;
  int rc;
  ospf_sweep_info info{};
  if (multi_) {
    rc = ospf_msweep_create(multi_, &o, &msweep_);
    if (rc == OSPF_OK) rc = ospf_msweep_run(msweep_);
    if (rc != OSPF_OK) {
      const std::string m = ospf_multi_last_error(multi_);
      dropSweep();
      throw EngineError(rc, m);
    }
    ospf_sweep_get_info(ospf_msweep_part(msweep_, 0), &info);
    sweepStats_.devices = ospf_multi_size(multi_);
  } else {
    // the serial prefix of the run starts while the plan is still built
    o.flags |= OSPF_SWEEP_EARLY_START;
    rc = ospf_sweep_create(engine_, &o, &sweep_);
    bool runErr = false;  // ospf_sweep_run reports through the sweep's own error
    if (rc == OSPF_OK) runErr = (rc = ospf_sweep_run(sweep_, nullptr)) != OSPF_OK;
    if (rc == OSPF_OK) rc = ospf_sync(engine_, nullptr);
    if (rc != OSPF_OK) {
      const std::string m = runErr ? ospf_sweep_last_error(sweep_) : ospf_last_error(engine_);
      dropSweep();
      throw EngineError(rc, m);
    }
    ospf_sweep_get_info(sweep_, &info);
    sweepStats_.devices = 1;
  }
  sweepVersion_ = snapVersion_;
  sweepMetric_ = useLinkMetric;
  spfRuns_ += csr_->names.size();  // every node's runSpf, once
  ++sweepStats_.sweeps;
  sweepStats_.mode = info.mode;
  sweepStats_.hip_graph = info.hip_graph;
}

void LinkState::sweepRows(const std::vector<uint32_t>& roots, uint32_t W,
                          std::vector<uint32_t>& dist, std::vector<uint32_t>& nh) {
  const size_t V = csr_->names.size();
  dist.assign(roots.size() * V, kInf);
  nh.assign(roots.size() * V * W, 0);
  if (sweep_) {
    const int rc = ospf_sweep_copy_rows(sweep_, roots.data(), (uint32_t)roots.size(), W,
                                        dist.data(), nh.data());
    if (rc != OSPF_OK) throw EngineError(rc, ospf_sweep_last_error(sweep_));
  } else {
    for (size_t i = 0; i < roots.size(); ++i) {
      uint32_t slot = 0;
      int rc = ospf_msweep_owner(msweep_, roots[i], &slot);
      if (rc != OSPF_OK)
        throw EngineError(rc, "all-sources sweep: no part owns node " + csr_->names[roots[i]]);
      ospf_sweep* part = ospf_msweep_part(msweep_, slot);
      rc = ospf_sweep_copy_rows(part, &roots[i], 1, W, dist.data() + i * V, nh.data() + i * V * W);
      if (rc != OSPF_OK) throw EngineError(rc, ospf_sweep_last_error(part));
    }
  }
  sweepStats_.rows_copied += roots.size();
}

std::vector<ospf_digest> LinkState::allSourcesDigestsImpl(bool useLinkMetric) {
  snapshot();
  const size_t V = csr_->names.size();
  if (hostRun(useLinkMetric)) return spfDigests(csr_->names, useLinkMetric);
  prefetchAllSources(useLinkMetric);
  std::vector<ospf_digest> out(V);
  if (msweep_) {
    const int rc = ospf_msweep_digests(msweep_, out.data());
    if (rc != OSPF_OK) throw EngineError(rc, ospf_multi_last_error(multi_));
    return out;
  }
  ospf_sweep_info info{};
  ospf_sweep_get_info(sweep_, &info);
  std::vector<uint32_t> roots(info.n_roots);
  ospf_sweep_roots(sweep_, roots.data());
  std::vector<ospf_digest> tmp(roots.size());
  const int rc = ospf_sweep_digests_host(sweep_, tmp.data());
  if (rc != OSPF_OK) throw EngineError(rc, ospf_sweep_last_error(sweep_));
  for (size_t i = 0; i < roots.size(); ++i) out[roots[i]] = tmp[i];
  return out;
}

void LinkState::evictSpf(const std::vector<std::string>& roots, bool useLinkMetric) {
  auto& memo = useLinkMetric ? memoMetric_ : memoHops_;
  for (const auto& r : roots) memo.erase(r);
}

uint32_t LinkState::nhWordsFor(uint32_t root) const {
  uint32_t n = 0;
  for (uint32_t e = csr_->rowPtr[root]; e < csr_->rowPtr[root + 1]; ++e)
    if (csr_->col[e] != root && (e == csr_->rowPtr[root] || csr_->col[e - 1] != csr_->col[e])) ++n;
  return std::max<uint32_t>(1, (n + 31) / 32);
}

std::vector<ospf_ctx*> LinkState::slots() const {
  std::vector<ospf_ctx*> out;
  if (multi_) {
    for (uint32_t i = 0, n = ospf_multi_size(multi_); i < n; ++i) out.push_back(ospf_multi_ctx(multi_, i));
  } else if (engine_) {
    out.push_back(engine_);
  }
  return out;
}

int LinkState::batchOn(ospf_ctx* c, const uint32_t* roots, uint32_t n, bool useLinkMetric,
                       uint32_t flags, uint32_t W, uint32_t* dist, uint32_t* nh) const {
  if (!useLinkMetric) flags |= OSPF_HOP_COUNT;
  return ospf_sssp_batch(c, roots, n, nullptr, flags, W, dist, nh, nullptr);
}

// Run fn(slot, ctx) for every slot, slot 0 on the calling thread; the first
// failure (rc, slot) is returned after every thread joined. A slot whose
// thread cannot be created runs on the calling thread too.
static std::pair<int, size_t> onSlots(const std::vector<ospf_ctx*>& cs,
                                      const std::function<int(size_t, ospf_ctx*)>& fn) {
  std::vector<int> rc(cs.size(), OSPF_OK);
  std::vector<std::thread> th;
  std::vector<size_t> here{0};
  for (size_t i = 1; i < cs.size(); ++i) {
    try {
      th.emplace_back([&, i] { rc[i] = fn(i, cs[i]); });
    } catch (const std::system_error&) {
      here.push_back(i);
    }
  }
  for (size_t i : here) rc[i] = fn(i, cs[i]);
  for (auto& t : th) t.join();
  for (size_t i = 0; i < cs.size(); ++i)
    if (rc[i] != OSPF_OK) return {rc[i], i};
  return {OSPF_OK, 0};
}

void LinkState::runBatch(const std::vector<uint32_t>& roots,
                         const std::vector<std::vector<uint32_t>>* ign, bool useLinkMetric,
                         uint32_t flags, uint32_t W, std::vector<uint32_t>* dist,
                         std::vector<uint32_t>* nh, std::vector<ospf_digest>* dig) {
  ensureEngine();
  const size_t V = csr_->names.size(), n = roots.size();
  if (!useLinkMetric) flags |= OSPF_HOP_COUNT;
  if (dist) dist->assign(n * V, kInf);
  if (nh) nh->assign(n * V * W, 0);
  if (dig) dig->assign(n, ospf_digest{0, 0, 0});
  std::vector<uint32_t> off, ids;
  ospf_ignore ig{};
  if (ign) {
    off.reserve(n + 1);
    off.push_back(0);
    for (const auto& l : *ign) {
      ids.insert(ids.end(), l.begin(), l.end());
      off.push_back((uint32_t)ids.size());
    }
    ig.offsets = off.data();
    ig.link_ids = ids.data();
  }
  int rc = ospf_sssp_batch(engine_, roots.data(), (uint32_t)n, ign ? &ig : nullptr, flags, W,
                           dist ? dist->data() : nullptr, nh ? nh->data() : nullptr,
                           dig ? dig->data() : nullptr);
  if (rc != OSPF_OK) throw EngineError(rc, ospf_last_error(engine_));
}

// ---------------------------------------------------------------- results
std::vector<PathLink> SpfRows::pathLinksOf(uint32_t v) const {
  std::vector<PathLink> out;
  const CsrSnapshot& c = *csr;
  const uint32_t dv = dist[v];
  if (v == root || dv == kInf) return out;
  struct Cand {
    uint32_t du, u, rank, lid;
  };
  std::vector<Cand> cands;
  for (uint32_t e = c.rowPtr[v]; e < c.rowPtr[v + 1]; ++e) {
    if (!c.edgeUp[e]) continue;
    const uint32_t lid = c.linkId[e];
    if (!ignored.empty() && std::binary_search(ignored.begin(), ignored.end(), lid)) continue;
    const uint32_t u = c.col[e];
    const uint32_t du = dist[u];
    if (du == kInf) continue;
    const uint32_t t = c.twin[e];  // entry u -> v: metric advertised by u
    const uint64_t w = useLinkMetric ? c.metric[t] : 1u;
    if ((uint64_t)du + w != dv) continue;
    if (u != root && c.noTransit[u]) continue;
    cands.push_back({du, u, c.linkRank[t], lid});
  }
  // reference order: predecessor pop order (dist, name) then the link's
  // position in linksFromNode(predecessor)
  std::sort(cands.begin(), cands.end(), [](const Cand& a, const Cand& b) {
    return std::tie(a.du, a.u, a.rank) < std::tie(b.du, b.u, b.rank);
  });
  out.reserve(cands.size());
  for (const auto& x : cands) out.push_back(PathLink{c.links[x.lid], c.names[x.u]});
  return out;
}

std::unordered_set<std::string> SpfRows::nextHopsOf(uint32_t v) const {
  std::unordered_set<std::string> out;
  if (nh.empty()) return out;
  const uint32_t* bits = nh.data() + (size_t)v * W;
  for (uint32_t w = 0; w < W; ++w)
    for (uint32_t b = bits[w]; b; b &= b - 1) {
      const uint32_t i = w * 32 + (uint32_t)__builtin_ctz(b);
      out.insert(csr->names[nbrs.at(i)]);
    }
  return out;
}

SpfResult::SpfResult(std::shared_ptr<const SpfRows> rows) : rows_(std::move(rows)) {
  const auto& d = rows_->dist;
  size_t n = 0;
  for (const uint32_t x : d) n += x != kInf;
  reached_.reserve(n);
  for (uint32_t v = 0; v < (uint32_t)d.size(); ++v)
    if (d[v] != kInf) reached_.push_back(v);
  slot_ = std::make_unique<std::atomic<value_type*>[]>(n);  // value-initialised: null
}

SpfResult::SpfResult(SpfResult&& o) noexcept
    : map_(std::move(o.map_)), rows_(std::move(o.rows_)), reached_(std::move(o.reached_)),
      slot_(std::move(o.slot_)) {
  o.reached_.clear();
}

SpfResult& SpfResult::operator=(SpfResult&& o) noexcept {
  if (this != &o) {
    release();
    map_ = std::move(o.map_);
    rows_ = std::move(o.rows_);
    reached_ = std::move(o.reached_);
    slot_ = std::move(o.slot_);
    o.reached_.clear();
  }
  return *this;
}

void SpfResult::release() {
  if (slot_)
    for (size_t k = 0; k < reached_.size(); ++k) delete slot_[k].load(std::memory_order_relaxed);
  slot_.reset();
}

const SpfResult::value_type& SpfResult::entry(size_t k) const {
  value_type* p = slot_[k].load(std::memory_order_acquire);
  if (p) return *p;
  const uint32_t v = reached_[k];
  auto* fresh = new value_type(std::piecewise_construct, std::forward_as_tuple(rows_->csr->names[v]),
                               std::forward_as_tuple(NodeSpfResult(rows_->dist[v], rows_.get(), v)));
  if (slot_[k].compare_exchange_strong(p, fresh, std::memory_order_acq_rel)) return *fresh;
  delete fresh;  // another thread made it first
  return *p;
}

SpfResult::const_iterator SpfResult::begin() const {
  const_iterator it;
  it.r_ = this;
  if (!rows_) it.m_ = map_.begin();
  return it;
}

SpfResult::const_iterator SpfResult::end() const {
  const_iterator it;
  it.r_ = this;
  if (rows_) it.k_ = reached_.size();
  else it.m_ = map_.end();
  return it;
}

SpfResult::const_iterator SpfResult::find(const std::string& node) const {
  if (!rows_) {
    const_iterator it;
    it.r_ = this;
    it.m_ = map_.find(node);
    return it;
  }
  const auto& ids = rows_->csr->ids;
  auto id = ids.find(node);
  if (id == ids.end() || rows_->dist[id->second] == kInf) return end();
  const_iterator it;
  it.r_ = this;
  it.k_ = (size_t)(std::lower_bound(reached_.begin(), reached_.end(), id->second) - reached_.begin());
  return it;
}

const NodeSpfResult& SpfResult::at(const std::string& node) const {
  auto it = find(node);
  if (it == end()) throw std::out_of_range("SpfResult::at: " + node);
  return it->second;
}

std::vector<uint32_t> LinkState::nbrsOf(uint32_t root) const {
  std::vector<uint32_t> out;
  for (uint32_t e = csr_->rowPtr[root]; e < csr_->rowPtr[root + 1]; ++e) {
    const uint32_t v = csr_->col[e];
    if (v != root && (out.empty() || out.back() != v)) out.push_back(v);
  }
  return out;
}

const SpfResult& LinkState::getSpfResultImpl(const std::string& node, bool useLinkMetric) {
  auto& memo = useLinkMetric ? memoMetric_ : memoHops_;
  auto it = memo.find(node);
  if (it != memo.end()) return it->second;
  prefetchSpf({node}, useLinkMetric);
  return memo.at(node);
}

void LinkState::prefetchSpfImpl(const std::vector<std::string>& roots, bool useLinkMetric) {
  auto& memo = useLinkMetric ? memoMetric_ : memoHops_;
  snapshot();
  std::unordered_map<uint32_t, std::vector<uint32_t>> byW;  // W -> roots
  std::unordered_set<std::string> queued;
  size_t pending = 0;
  for (const auto& r : roots) {
    if (memo.count(r) || !queued.insert(r).second) continue;
    auto id = csr_->ids.find(r);
    if (id == csr_->ids.end()) {  // no adjacency DB: only the root itself
      ++spfRuns_;
      SpfResult::Map res;
      res.emplace(r, NodeSpfResult(0));
      memo.emplace(r, SpfResult(std::move(res)));
      continue;
    }
    if (hostRun(useLinkMetric)) {
      ++spfRuns_;
      memo.emplace(r, runSpfHost(r, useLinkMetric, {}));
      continue;
    }
    byW[nhWordsFor(id->second)].push_back(id->second);
    ++pending;
  }
  const size_t V = csr_->names.size();
  // most of the nodes asked for: one all-sources sweep, rows copied from it
  if (!sweepHas(useLinkMetric) && pending >= kSweepMinRoots && 2 * pending >= V)
    prefetchAllSources(useLinkMetric);
  const bool fromSweep = sweepHas(useLinkMetric);
  if (!fromSweep) spfRuns_ += pending;  // a sweep counted every node's run
  for (auto& [W, ids] : byW) {
    const size_t chunk = std::max<size_t>(1, std::min<size_t>(ids.size(), (256ull << 20) / (V * 4 * (1 + W))));
    for (size_t c0 = 0; c0 < ids.size(); c0 += chunk) {
      std::vector<uint32_t> part(ids.begin() + c0, ids.begin() + std::min(ids.size(), c0 + chunk));
      std::vector<uint32_t> dist, nh;
      const auto t0 = std::chrono::steady_clock::now();
      const std::vector<ospf_ctx*> cs = fromSweep ? std::vector<ospf_ctx*>{} : (ensureEngine(), slots());
      if (fromSweep) {
        sweepRows(part, W, dist, nh);
      } else if (cs.size() > 1 && part.size() >= cs.size()) {
        // split across the device slots: contiguous slices, rows in place
        const size_t m = part.size(), ns = cs.size();
        dist.assign(m * V, kInf);
        nh.assign(m * V * W, 0);
        const auto [rc, bad] = onSlots(cs, [&](size_t i, ospf_ctx* c) {
          const size_t a = m * i / ns, b = m * (i + 1) / ns;
          return b > a ? batchOn(c, part.data() + a, (uint32_t)(b - a), useLinkMetric,
                                 OSPF_WANT_DIST | OSPF_WANT_NH, W, dist.data() + a * V,
                                 nh.data() + a * V * W)
                       : OSPF_OK;
        });
        if (rc != OSPF_OK) throw EngineError(rc, ospf_last_error(cs[bad]));
        ++shardStats_.spf_batches;
        shardStats_.spf_launches += ns;
      } else {
        runBatch(part, nullptr, useLinkMetric, OSPF_WANT_DIST | OSPF_WANT_NH, W, &dist, &nh, nullptr);
      }
      const auto t1 = std::chrono::steady_clock::now();
      for (size_t i = 0; i < part.size(); ++i) {
        auto rows = std::make_shared<SpfRows>();
        rows->csr = csr_;
        rows->root = part[i];
        rows->W = W;
        rows->useLinkMetric = useLinkMetric;
        rows->dist.assign(dist.begin() + i * V, dist.begin() + (i + 1) * V);
        rows->nh.assign(nh.begin() + i * V * W, nh.begin() + (i + 1) * V * W);
        rows->nbrs = nbrsOf(part[i]);
        memo.emplace(csr_->names[part[i]], SpfResult(std::move(rows)));
      }
      if (getenv("ODL_SPF_TIMING")) {
        const auto t2 = std::chrono::steady_clock::now();
        fprintf(stderr, "spf_timing roots=%zu W=%u engine_ms=%.3f build_result_ms=%.3f\n",
                part.size(), W, std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(t2 - t1).count());
      }
    }
  }
}

std::vector<ospf_digest> LinkState::spfDigestsImpl(const std::vector<std::string>& roots,
                                                   bool useLinkMetric) {
  snapshot();
  std::vector<ospf_digest> out(roots.size(), ospf_digest{0, 0, 0});
  std::vector<uint32_t> ids;
  std::vector<size_t> pos;
  uint32_t W = 1;
  for (size_t i = 0; i < roots.size(); ++i) {
    ++spfRuns_;
    auto id = csr_->ids.find(roots[i]);
    if (id == csr_->ids.end()) {
      // root without a database: result {root: 0}; node_term(0xFFFFFFFF, 0)
      uint64_t x = (0xFFFFFFFFull << 32);
      x ^= x >> 30;
      x *= 0xbf58476d1ce4e5b9ULL;
      x ^= x >> 27;
      x *= 0x94d049bb133111ebULL;
      x ^= x >> 31;
      out[i] = ospf_digest{1, 0, x};
      continue;
    }
    if (hostRun(useLinkMetric)) {
      out[i] = digestHost(roots[i], runSpfHost(roots[i], useLinkMetric, {}));
      continue;
    }
    ids.push_back(id->second);
    pos.push_back(i);
    W = std::max(W, nhWordsFor(id->second));
  }
  if (!ids.empty()) {
    std::vector<ospf_digest> d;
    runBatch(ids, nullptr, useLinkMetric, OSPF_WANT_DIGEST, W, nullptr, nullptr, &d);
    for (size_t k = 0; k < ids.size(); ++k) out[pos[k]] = d[k];
  }
  return out;
}

std::optional<Metric> LinkState::getMetricFromAToB(const std::string& a, const std::string& b,
                                                   bool useLinkMetric) {
  if (a == b) return 0;
  const SpfResult& r = getSpfResult(a, useLinkMetric);
  auto it = r.find(b);
  if (it == r.end()) return std::nullopt;
  return it->second.metric();
}

std::shared_ptr<const SpfRows> LinkState::rawSpf(const std::string& node) {
  const SpfResult& r = getSpfResult(node, true);
  if (r.rows()) return r.rows();
  // a memoised result without engine rows: re-derive the distances (not a
  // new logical runSpf)
  snapshot();
  const uint32_t s = csr_->ids.at(node);
  auto rows = std::make_shared<SpfRows>();
  rows->csr = csr_;
  rows->root = s;
  runBatch({s}, nullptr, true, OSPF_WANT_DIST, nhWordsFor(s), &rows->dist, nullptr, nullptr);
  return rows;
}

std::optional<Path> LinkState::trace(const SpfRows& run, uint32_t src, uint32_t x,
                                     std::unordered_set<const Link*>& seen) const {
  if (x == src) return Path{};
  for (const auto& pl : run.pathLinksOf(x)) {
    if (!seen.insert(pl.link.get()).second) continue;
    auto p = trace(run, src, run.csr->ids.at(pl.prevNode), seen);
    if (p) {
      p->push_back(pl.link);
      return p;
    }
  }
  return std::nullopt;
}

std::vector<Path> LinkState::tracePaths(const SpfRows& run, uint32_t src, uint32_t dst) const {
  std::vector<Path> out;
  if (run.dist[dst] == kInf) return out;
  std::unordered_set<const Link*> seen;
  for (auto p = trace(run, src, dst, seen); p && !p->empty(); p = trace(run, src, dst, seen))
    out.push_back(std::move(*p));
  return out;
}

static std::string kspKey(const std::string& s, const std::string& d, size_t k) {
  std::string key = s;
  key += '\x01';
  key += d;
  key += '\x01';
  key += std::to_string(k);
  return key;
}

const std::vector<Path>& LinkState::getKthPathsImpl(const std::string& src, const std::string& dst,
                                                    size_t k) {
  if (k < 1) throw std::invalid_argument("k must be >= 1");
  const std::string key = kspKey(src, dst, k);
  auto it = memoKsp_.find(key);
  if (it != memoKsp_.end()) return it->second;
  std::unordered_set<const Link*> skipSet;
  std::vector<LinkPtr> skip;
  for (size_t i = 1; i < k; ++i)
    for (const auto& p : getKthPaths(src, dst, i))
      for (const auto& l : p)
        if (skipSet.insert(l.get()).second) skip.push_back(l);
  std::vector<Path> paths;
  snapshot();
  if (hostRun(true)) {
    if (skip.empty()) {
      paths = tracePathsHost(getSpfResult(src, true), src, dst);
    } else {
      ++spfRuns_;
      paths = tracePathsHost(runSpfHost(src, true, skipSet), src, dst);
    }
  } else if (skip.empty()) {
    const SpfResult& r = getSpfResult(src, true);
    if (r.count(dst) && csr_->ids.count(src)) {
      const auto run = rawSpf(src);
      paths = tracePaths(*run, run->csr->ids.at(src), run->csr->ids.at(dst));
    }
  } else {
    ++spfRuns_;
    snapshot();
    const uint32_t s = csr_->ids.at(src);
    std::vector<uint32_t> ign;
    for (const auto& l : skip) ign.push_back(linkIdOf(*l));
    std::sort(ign.begin(), ign.end());
    std::vector<uint32_t> dist;
    if (ign.size() <= OSPF_MAX_IGNORED_PER_RUN) {
      std::vector<std::vector<uint32_t>> igns{ign};
      runBatch({s}, &igns, true, OSPF_WANT_DIST, nhWordsFor(s), &dist, nullptr, nullptr);
    } else {
      // more ignored links than a run's list holds (e.g. the host side of a
      // KSP2 destination whose k = 1 paths overflowed the device record):
      // take them down on the device graph for this one run, then restore
      // (ospf_links_mask / unmask: the device graph and the engine's bounds
      // come back exactly as they were; on any failure the engine is marked
      // stale and reloaded by the next ensureEngine)
      ensureEngine();
      int rc = ospf_links_mask(engine_, ign.data(), (uint32_t)ign.size(), ~snapVersion_);
      if (rc != OSPF_OK) {
        const std::string m = ospf_last_error(engine_);
        ospf_links_unmask(engine_);
        engineVersion_ = 0;
        throw EngineError(rc, m);
      }
      dist.assign(V_of(*csr_), kInf);
      rc = ospf_sssp_batch(engine_, &s, 1, nullptr, OSPF_WANT_DIST, nhWordsFor(s), dist.data(),
                           nullptr, nullptr);
      const std::string m = rc != OSPF_OK ? ospf_last_error(engine_) : "";
      const int rc2 = ospf_links_unmask(engine_);
      if (rc != OSPF_OK || rc2 != OSPF_OK) {
        engineVersion_ = 0;
        throw EngineError(rc != OSPF_OK ? rc : rc2, rc != OSPF_OK ? m : ospf_last_error(engine_));
      }
    }
    SpfRows run;
    run.csr = csr_;
    run.root = s;
    run.dist = std::move(dist);
    run.ignored = std::move(ign);
    auto d = csr_->ids.find(dst);
    if (d != csr_->ids.end()) paths = tracePaths(run, s, d->second);
  }
  return memoKsp_.emplace(key, std::move(paths)).first->second;
}

void LinkState::prefetchKsp2Impl(const std::string& src, const std::vector<std::string>& dsts) {
  snapshot();
  if (hostRun(true)) {
    for (const auto& d : dsts) getKthPaths(src, d, 2);
    return;
  }
  auto sid = csr_->ids.find(src);
  std::vector<uint32_t> ids;
  std::vector<const std::string*> names;
  std::unordered_set<std::string> queued;
  for (const auto& d : dsts) {
    if (memoKsp_.count(kspKey(src, d, 2)) || !queued.insert(d).second) continue;
    auto did = csr_->ids.find(d);
    if (sid == csr_->ids.end() || did == csr_->ids.end()) {
      getKthPaths(src, d, 2);  // a side without an adjacency DB: no paths, host
      continue;
    }
    ids.push_back(did->second);
    names.push_back(&did->first);
  }
  if (ids.empty()) return;
  // k = 1 traces the memoised SPF of src (LinkState.cpp:804-805): one run
  getSpfResult(src, true);
  ensureEngine();
  // Device KSP2: SPF of src, k = 1 traces, masked reruns and k = 2 traces all
  // on the engine; records hold link ids. A destination over the engine's
  // budgets is computed by the host path below (same results, slower).
  uint32_t kCap = 1024;  // record words per destination and k
  if (const char* x = getenv("ODL_KSP_CAP")) kCap = std::max(2, std::min(2048, atoi(x)));
  const size_t n = ids.size();
  std::vector<uint32_t> k1(n * kCap), k2(n * kCap), status(n);
  auto runOn = [&](ospf_ctx* c, size_t a0, size_t a1) {
    ospf_ksp2 a{};
    a.src = sid->second;
    a.dsts = ids.data() + a0;
    a.n = (uint32_t)(a1 - a0);
    a.path_cap = kCap;
    a.k1 = k1.data() + a0 * kCap;
    a.k2 = k2.data() + a0 * kCap;
    a.status = status.data() + a0;
    return a1 > a0 ? ospf_ksp2_run(c, &a) : OSPF_OK;
  };
  const std::vector<ospf_ctx*> cs = slots();
  if (cs.size() > 1 && n >= cs.size()) {
    // destinations of one source split across the device slots (SURVEY
    // §8(e)): each slot runs the source's SPF, its k = 1 traces and its
    // destinations' reruns; records land in place in k1 / k2 / status
    const size_t ns = cs.size();
    const auto [rc, bad] = onSlots(cs, [&](size_t i, ospf_ctx* c) {
      return runOn(c, n * i / ns, n * (i + 1) / ns);
    });
    if (rc != OSPF_OK) throw EngineError(rc, ospf_last_error(cs[bad]));
    ++shardStats_.ksp2_runs;
    shardStats_.ksp2_launches += ns;
  } else {
    const int rc = runOn(engine_, 0, n);
    if (rc != OSPF_OK) throw EngineError(rc, ospf_last_error(engine_));
  }
  auto decode = [&](const uint32_t* rec) {
    std::vector<Path> paths(rec[0]);
    for (uint32_t p = 0, q = 1; p < rec[0]; ++p) {
      const uint32_t len = rec[q];
      paths[p].reserve(len);
      for (uint32_t j = 0; j < len; ++j) paths[p].push_back(csr_->links.at(rec[q + 1 + j]));
      q += 1 + len;
    }
    return paths;
  };
  for (size_t i = 0; i < n; ++i) {
    const std::string& d = *names[i];
    if (!(status[i] & OSPF_KSP_OVF1)) memoKsp_.emplace(kspKey(src, d, 1), decode(&k1[i * kCap]));
    if (status[i] & (OSPF_KSP_OVF1 | OSPF_KSP_OVF2)) {
      getKthPaths(src, d, 2);
      continue;
    }
    if (status[i] & OSPF_KSP_RERUN) ++spfRuns_;  // runSpf(src, true, linksToIgnore)
    memoKsp_.emplace(kspKey(src, d, 2), decode(&k2[i * kCap]));
  }
}

// ---------------------------------------------------------------- incremental
void LinkState::applyIncremental(const std::vector<LinkDelta>& links,
                                 const std::vector<std::string>& nodes) {
  ++incStats_.patches;
  constexpr uint64_t kInf64 = ~0ull;
  auto distOf = [](const SpfResult& r, const std::string& n) -> uint64_t {
    auto it = r.find(n);
    return it == r.end() ? kInf64 : it->second.metric();
  };
  // the rule of ospf_affected_roots (include/openr_spf.h), on a memoised result
  auto affected = [&](const std::string& root, const SpfResult& r, bool hop) {
    for (const auto& d : links) {
      const Link& l = *d.link;
      const uint64_t da = distOf(r, l.lowNode()), db = distOf(r, l.highNode());
      const uint64_t w0ab = hop ? 1 : d.mlo0, w0ba = hop ? 1 : d.mhi0;
      const uint64_t w1ab = hop ? 1 : l.metricFrom(l.lowNode()),
                     w1ba = hop ? 1 : l.metricFrom(l.highNode());
      if (d.up0 && da != kInf64 && da + w0ab == db) return true;
      if (d.up0 && db != kInf64 && db + w0ba == da) return true;
      if (l.isUp() && da != kInf64 && da + w1ab <= db) return true;
      if (l.isUp() && db != kInf64 && db + w1ba <= da) return true;
    }
    for (const auto& x : nodes) {
      const uint64_t dx = distOf(r, x);
      if (dx == kInf64 || x == root) continue;
      for (const auto& l : linksFromNode(x)) {
        if (!l->isUp()) continue;
        if (dx + (hop ? 1 : l->metricFrom(x)) <= distOf(r, l->otherNode(x))) return true;
      }
    }
    return false;
  };
  // the dropped results go to the reaper thread, as clearMemo's do (a
  // route build's result holds ~100k materialised entries at F100k)
  auto dead = std::make_unique<MemoReaper::Dead>();
  for (int mode = 0; mode < 2; ++mode) {
    auto& memo = mode == 0 ? memoMetric_ : memoHops_;
    auto& to = mode == 0 ? dead->a : dead->b;
    for (auto it = memo.begin(); it != memo.end();) {
      if (affected(it->first, it->second, mode == 1)) {
        to.insert(memo.extract(it++));
        ++incStats_.dropped;
      } else {
        ++it;
        ++incStats_.kept;
      }
    }
  }
  dead->k.swap(memoKsp_);  // KSP2 masked reruns are not tracked
  if (!reaper_) {
    try {
      reaper_ = std::make_unique<MemoReaper>();
    } catch (const std::system_error&) {  // no thread to spare: freed here
    }
  }
  if (reaper_) reaper_->push(std::move(dead));
  patchGraph(links, nodes);
}

// The CSR and the device graph, patched in place (same node ids, same
// links): metrics, up state, overload bits.
void LinkState::patchGraph(const std::vector<LinkDelta>& links,
                           const std::vector<std::string>& nodes) {
  std::vector<ospf_link_update> ups;
  for (const auto& d : links) {
    const Link& l = *d.link;
    const uint32_t lid = linkIdOf(l);
    const uint32_t lo = csr_->ids.at(l.lowNode());
    auto clamp = [](Metric m) { return (m >= 1 && m <= 0xFFFFFFFFull) ? (uint32_t)m : 0u; };
    const uint32_t mlo = clamp(l.metricFrom(l.lowNode())), mhi = clamp(l.metricFrom(l.highNode()));
    for (uint32_t e = csr_->rowPtr[lo]; e < csr_->rowPtr[lo + 1]; ++e) {
      if (csr_->linkId[e] != lid) continue;
      const uint32_t t = csr_->twin[e];
      csr_->metric[e] = mlo;
      csr_->metric[t] = mhi;
      csr_->edgeUp[e] = csr_->edgeUp[t] = l.isUp() ? 1 : 0;
      break;
    }
    ups.push_back(ospf_link_update{lid, l.isUp() ? 1u : 0u, mlo, mhi});
    for (const std::string* n : {&l.lowNode(), &l.highNode()}) {  // largest in-range out-metric
      const uint32_t u = csr_->ids.at(*n);
      uint64_t mx = 0;
      for (const auto& x : linksFromNode(*n)) {
        const Metric m = x->metricFrom(*n);
        if (m >= 1 && m <= 0xFFFFFFFFull) mx = std::max<uint64_t>(mx, m);
      }
      csr_->rowMax[u] = mx;
    }
  }
  std::vector<uint32_t> nids;
  std::vector<uint8_t> nts;
  for (const auto& x : nodes) {
    const uint32_t id = csr_->ids.at(x);
    csr_->noTransit[id] = isNodeOverloaded(x) ? 1 : 0;
    nids.push_back(id);
    nts.push_back(csr_->noTransit[id]);
  }
  const bool inSync = engine_ && engineVersion_ == snapVersion_;
  ++version_;
  snapVersion_ = version_;
  dropSweep();  // its rows describe the graph before the patch
  if (inSync) {
    const uint32_t nctx = multi_ ? ospf_multi_size(multi_) : 1u;
    for (uint32_t i = 0; i < nctx; ++i) {
      ospf_ctx* c = multi_ ? ospf_multi_ctx(multi_, i) : engine_;
      int rc = ospf_update_links(c, ups.data(), (uint32_t)ups.size(), snapVersion_);
      if (rc == OSPF_OK) rc = ospf_update_nodes(c, nids.data(), nts.data(), (uint32_t)nids.size(),
                                                snapVersion_);
      if (rc != OSPF_OK) {
        engineVersion_ = 0;  // reload every device on the next use
        throw EngineError(rc, ospf_last_error(c));
      }
    }
    engineVersion_ = snapVersion_;
  }
}

// Links added / removed between known nodes, in place (LinkState.cpp:632-657
// [LINK UP] / [LINK DOWN]; node ids stay). The rows of the links' ends are
// rebuilt from their LinkSets (a set's iteration order -- the link ranks --
// may change on an insert), the arrays between them move as blocks, twins are
// remapped, and the engine patches the same rows (ospf_update_rows). O(E)
// block moves on host threads, no re-snapshot, no device reload.
void LinkState::patchStructure(const std::vector<LinkPtr>& added,
                               const std::vector<LinkPtr>& removed) {
  dropSweep();  // its rows describe the graph before the patch
  Csr& c = csrForWrite();
  const uint32_t V = (uint32_t)c.names.size();
  std::vector<uint32_t> rows;
  for (const auto* set : {&added, &removed})
    for (const auto& l : *set) {
      rows.push_back(c.ids.at(l->lowNode()));
      rows.push_back(c.ids.at(l->highNode()));
    }
  std::sort(rows.begin(), rows.end());
  rows.erase(std::unique(rows.begin(), rows.end()), rows.end());
  for (const auto& l : removed) {
    const uint32_t lid = linkIdOf(*l);
    c.links[lid] = nullptr;
    c.freeLids.push_back(lid);
  }
  std::sort(c.freeLids.begin(), c.freeLids.end(), std::greater<uint32_t>());
  for (const auto& l : added) {
    uint32_t lid;
    if (!c.freeLids.empty()) {  // the smallest retired id
      lid = c.freeLids.back();
      c.freeLids.pop_back();
    } else {
      lid = (uint32_t)c.links.size();
      c.links.emplace_back();
    }
    c.links[lid] = l;
    l->snapLid = lid;
  }
  // the new rows, (neighbour id, rank) order
  struct Ent {
    uint32_t v, rank, metric, lid;
    uint8_t up;
  };
  const size_t K = rows.size();
  std::vector<std::vector<Ent>> nrow(K);
  for (size_t k = 0; k < K; ++k) {
    const uint32_t u = rows[k];
    const std::string& un = c.names[u];
    uint32_t rank = 0;
    uint64_t mx = 0;
    for (const auto& l : linksFromNode(un)) {
      const Metric m = l->metricOfEnd(l->endIndex(un));
      const bool inRange = m >= 1 && m <= 0xFFFFFFFFull;
      mx = std::max<uint64_t>(mx, inRange ? m : 0);
      nrow[k].push_back(Ent{c.ids.at(l->otherNode(un)), rank++, inRange ? (uint32_t)m : 1u,
                            l->snapLid, (uint8_t)(l->isUp() ? 1 : 0)});
    }
    std::sort(nrow[k].begin(), nrow[k].end(), [](const Ent& a, const Ent& b) {
      return a.v != b.v ? a.v < b.v : a.rank < b.rank;
    });
    c.rowMax[u] = mx;
  }
  // offsets: segment s (0..K) = the unchanged rows between changed rows
  // s - 1 and s, moved by shift[s]
  const std::vector<uint32_t> old = c.rowPtr;
  const size_t E0 = old[V];
  std::vector<int64_t> shift(K + 1, 0);
  for (size_t k = 0; k < K; ++k)
    shift[k + 1] = shift[k] + (int64_t)nrow[k].size() - (int64_t)(old[rows[k] + 1] - old[rows[k]]);
  const size_t E1 = (size_t)((int64_t)E0 + shift[K]);
  for (uint32_t u = 0, k = 0; u < V; ++u) {
    const bool ch = k < K && rows[k] == u;
    c.rowPtr[u + 1] = c.rowPtr[u] + (ch ? (uint32_t)nrow[k++].size() : old[u + 1] - old[u]);
  }
  auto segLo = [&](size_t s) { return s == 0 ? (size_t)0 : (size_t)old[rows[s - 1] + 1]; };
  auto segHi = [&](size_t s) { return s == K ? E0 : (size_t)old[rows[s]]; };
  auto move = [&](auto& a) {
    using T = typename std::decay_t<decltype(a)>::value_type;
    if (E1 > E0) a.resize(E1);
    for (size_t s = 1; s <= K; ++s)  // leftwards first, in order
      if (shift[s] < 0 && segHi(s) > segLo(s))
        std::memmove(a.data() + (int64_t)segLo(s) + shift[s], a.data() + segLo(s),
                     (segHi(s) - segLo(s)) * sizeof(T));
    for (size_t s = K; s >= 1; --s)  // then rightwards, from the end
      if (shift[s] > 0 && segHi(s) > segLo(s))
        std::memmove(a.data() + (int64_t)segLo(s) + shift[s], a.data() + segLo(s),
                     (segHi(s) - segLo(s)) * sizeof(T));
    if (E1 < E0) a.resize(E1);
  };
  std::vector<std::function<void()>> jobs = {[&] { move(c.col); }, [&] { move(c.metric); },
                                            [&] { move(c.linkId); }, [&] { move(c.twin); },
                                            [&] { move(c.linkRank); }, [&] { move(c.edgeUp); }};
  parallelFor((uint32_t)jobs.size(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t j = lo; j < hi; ++j) jobs[j]();
  }, 1);
  // the rebuilt rows
  for (size_t k = 0; k < K; ++k) {
    size_t e = c.rowPtr[rows[k]];
    for (const Ent& x : nrow[k]) {
      c.col[e] = x.v;
      c.metric[e] = x.metric;
      c.linkId[e] = x.lid;
      c.linkRank[e] = x.rank;
      c.edgeUp[e] = x.up;
      c.twin[e] = kInf;
      ++e;
    }
  }
  // twins of unchanged entries: an old position in a segment moves with it;
  // one inside a changed row is set from that row below
  std::vector<uint32_t> starts(K);
  for (size_t k = 0; k < K; ++k) starts[k] = old[rows[k]];
  auto remap = [&](uint32_t t) -> uint32_t {
    const size_t i = (size_t)(std::upper_bound(starts.begin(), starts.end(), t) - starts.begin());
    if (i > 0 && t < old[rows[i - 1] + 1]) return kInf;  // inside changed row i - 1
    return (uint32_t)((int64_t)t + shift[i]);
  };
  for (size_t s = 0; s <= K; ++s) {
    const size_t lo = (size_t)((int64_t)segLo(s) + shift[s]), hi = (size_t)((int64_t)segHi(s) + shift[s]);
    if (hi <= lo) continue;
    parallelFor((uint32_t)(hi - lo), [&](uint32_t a, uint32_t b) {
      for (size_t e = lo + a; e < lo + b; ++e) c.twin[e] = remap(c.twin[e]);
    }, 1u << 16);
  }
  for (size_t k = 0; k < K; ++k) {
    const uint32_t u = rows[k];
    for (size_t e = c.rowPtr[u]; e < c.rowPtr[u + 1]; ++e) {
      if (c.twin[e] != kInf) continue;  // set from the partner row already
      const uint32_t x = c.col[e], lid = c.linkId[e];
      size_t q = c.rowPtr[x];
      while (q < c.rowPtr[x + 1] && !(c.linkId[q] == lid && q != e)) ++q;
      if (q == c.rowPtr[x + 1]) throw std::logic_error("patchStructure: link without a twin");
      c.twin[e] = (uint32_t)q;
      c.twin[q] = (uint32_t)e;
    }
  }
  uint64_t bound = 0;
  for (uint32_t u = 0; u < V; ++u) bound = std::min<uint64_t>(bound + c.rowMax[u], ~0ull >> 1);
  distBound_ = bound;
  ++topoStats_.link_patches;
  topoStats_.rows_patched += K;
  const bool inSync = engine_ && engineVersion_ == snapVersion_;
  ++version_;
  snapVersion_ = version_;
  if (inSync) patchEngineRows(rows);
}

LinkState::Csr& LinkState::csrForWrite() {
  // a kept memoised result reads this snapshot's ranks lazily: give it its own
  // (results handed to the reaper are no readers; only the live memo is)
  bool kept = false;
  for (const auto* m : {&memoMetric_, &memoHops_})
    for (const auto& kv : *m) kept |= kv.second.rows() && kv.second.rows()->csr == csr_;
  if (kept) csr_ = std::make_shared<Csr>(*csr_);
  return *csr_;
}

void LinkState::csrInsertNode(uint32_t k, const std::string& name, bool overloaded) {
  Csr& c = csrForWrite();
  const uint32_t V = (uint32_t)c.names.size();
  if (k > V) throw std::logic_error("csrInsertNode: position");
  c.names.insert(c.names.begin() + k, name);
  for (auto& kv : c.ids)
    if (kv.second >= k) ++kv.second;
  c.ids.emplace(name, k);
  c.rowPtr.insert(c.rowPtr.begin() + k + 1, c.rowPtr[k]);  // an empty row k
  parallelFor((uint32_t)c.col.size(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t e = lo; e < hi; ++e)
      if (c.col[e] >= k && c.col[e] != kInf) ++c.col[e];
  }, 1u << 16);
  c.noTransit.insert(c.noTransit.begin() + k, overloaded ? 1 : 0);
  c.rowMax.insert(c.rowMax.begin() + k, 0);
  ++topoStats_.node_patches;
}

void LinkState::csrEraseNode(uint32_t k) {
  Csr& c = csrForWrite();
  if (k >= c.names.size() || c.rowPtr[k] != c.rowPtr[k + 1])
    throw std::logic_error("csrEraseNode: row not empty");
  c.ids.erase(c.names[k]);
  for (auto& kv : c.ids)
    if (kv.second > k) --kv.second;
  c.names.erase(c.names.begin() + k);
  c.rowPtr.erase(c.rowPtr.begin() + k + 1);
  parallelFor((uint32_t)c.col.size(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t e = lo; e < hi; ++e)
      if (c.col[e] > k && c.col[e] != kInf) --c.col[e];
  }, 1u << 16);
  c.noTransit.erase(c.noTransit.begin() + k);
  c.rowMax.erase(c.rowMax.begin() + k);
  ++topoStats_.node_patches;
}

void LinkState::patchEngineRows(const std::vector<uint32_t>& rows) {
  const Csr& c = *csr_;
  ospf_csr g{};
  g.n_nodes = (uint32_t)c.names.size();
  g.n_edges = (uint32_t)c.col.size();
  g.row_ptr = c.rowPtr.data();
  g.col = c.col.data();
  g.metric = c.metric.data();
  g.link_id = c.linkId.data();
  g.twin = c.twin.data();
  g.edge_up = c.edgeUp.data();
  g.no_transit = c.noTransit.data();
  g.link_rank = c.linkRank.data();
  const uint32_t nctx = multi_ ? ospf_multi_size(multi_) : 1u;
  for (uint32_t i = 0; i < nctx; ++i) {
    ospf_ctx* x = multi_ ? ospf_multi_ctx(multi_, i) : engine_;
    const int rc = ospf_update_rows(x, &g, rows.data(), (uint32_t)rows.size(), snapVersion_);
    if (rc == OSPF_E_RANGE) {  // the device layout's reserve is spent: reload
      engineVersion_ = 0;
      return;
    }
    if (rc != OSPF_OK) {
      engineVersion_ = 0;  // reload every device on the next use
      throw EngineError(rc, ospf_last_error(x));
    }
  }
  engineVersion_ = snapVersion_;
}

void NodeUcmpResult::normalizeNextHopWeights() {
  int64_t g = 0;
  for (const auto& kv : nextHopLinks_) g = std::gcd(g, kv.second.weight);
  if (g > 1)
    for (auto& kv : nextHopLinks_) kv.second.weight /= g;
}

UcmpResult LinkState::resolveUcmpWeights(
    const SpfResult& spfGraph, const std::unordered_map<std::string, int64_t>& leafNodeToWeights,
    UcmpAlgo algo, bool useLinkMetric) const {
  // decision.ucmp_runs / ucmp_ms (LinkState.cpp:926,1025-1029)
  struct Timer {
    Counters& c;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~Timer() {
      ++c.ucmp_runs;
      c.ucmp_ms_sum +=
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
  } timer{counters_};
  UcmpResult out;
  // DijkstraQ<DijkstraQUcmpNode> (LinkState.h:573-645): entries still queued,
  // by name; pop order (metric, name). A popped node leaves the map, so a later
  // path link to it queues it again, as in the reference.
  struct Item {
    Metric metric;
    NodeUcmpResult result;
  };
  std::unordered_map<std::string, Item> queued;
  std::set<std::pair<Metric, std::string>> order;
  auto insert = [&](const std::string& n, Metric m) {
    queued[n] = Item{m, NodeUcmpResult{}};
    order.emplace(m, n);
  };
  // leaves present in the SPF graph, all at the same distance from the root
  // (LinkState.cpp:937-959)
  std::optional<Metric> spfMetric;
  for (const auto& [leaf, weight] : leafNodeToWeights) {
    auto it = spfGraph.find(leaf);
    if (it == spfGraph.end()) continue;
    const Metric m = it->second.metric();
    if (!spfMetric) {
      spfMetric = m;
    } else if (*spfMetric != m) {
      return UcmpResult{};  // "Skipping resolveUcmpWeights"
    }
    insert(leaf, 0);
    queued.at(leaf).result.setWeight(weight);
  }
  // walk from the leaves towards the root (LinkState.cpp:961-1023)
  while (!order.empty()) {
    const auto [metric, name] = *order.begin();
    order.erase(order.begin());
    NodeUcmpResult cur = std::move(queued.at(name).result);
    queued.erase(name);
    if (!cur.weight()) {
      int64_t advertised = 0;
      for (const auto& [iface, nh] : cur.nextHopLinks())
        advertised += algo == UcmpAlgo::kAdjWeightPropagation ? nh.link->weightFrom(name)
                                                              : nh.weight;
      cur.setWeight(advertised);
    }
    auto sit = spfGraph.find(name);
    if (sit == spfGraph.end()) throw std::logic_error("UCMP node not in the SPF graph");
    for (const auto& pl : sit->second.pathLinks()) {
      const Metric lm = useLinkMetric ? pl.link->metricFrom(pl.prevNode) : 1;
      auto q = queued.find(pl.prevNode);
      if (q == queued.end()) {
        insert(pl.prevNode, metric + lm);
        q = queued.find(pl.prevNode);
      }
      q->second.result.addNextHopLink(pl.link->ifaceFrom(pl.prevNode), pl.link, name,
                                      *cur.weight());
    }
    cur.normalizeNextHopWeights();
    out.emplace(name, std::move(cur));
  }
  return out;
}

// ---------------------------------------------------------------- host path
SpfResult LinkState::runSpfHost(const std::string& root, bool useLinkMetric,
                                const std::unordered_set<const Link*>& ignore) const {
  // Dijkstra with the reference's queue order -- (metric, name), keys only
  // ever lowered by a strictly better path -- and its u64 arithmetic, so a
  // wrapped negative metric behaves exactly as there.
  SpfResult::Map done;
  std::unordered_map<std::string, NodeSpfResult> open;
  std::set<std::pair<Metric, std::string>> order;
  open.emplace(root, NodeSpfResult(0));
  order.emplace(0, root);
  while (!order.empty()) {
    const std::string name = order.begin()->second;
    order.erase(order.begin());
    auto node = open.find(name);
    auto& rec = done.emplace(name, std::move(node->second)).first->second;
    open.erase(node);
    if (name != root && isNodeOverloaded(name)) continue;  // no transit
    for (const auto& link : linksFromNode(name)) {
      const std::string& other = link->otherNode(name);
      if (!link->isUp() || done.count(other) || ignore.count(link.get())) continue;
      const Metric cand = rec.metric() + (useLinkMetric ? link->metricFrom(name) : 1);
      auto it = open.find(other);
      if (it == open.end()) {
        it = open.emplace(other, NodeSpfResult(cand)).first;
        order.emplace(cand, other);
      }
      NodeSpfResult& o = it->second;
      if (o.metric() < cand) continue;
      if (o.metric() > cand) {  // strictly better: forget the other paths
        order.erase({o.metric(), other});
        o = NodeSpfResult(cand);
        order.emplace(cand, other);
      }
      o.pathLinks_.push_back(PathLink{link, name});
      o.nextHops_.insert(rec.nextHops_.begin(), rec.nextHops_.end());
      if (o.nextHops_.empty()) o.nextHops_.insert(other);  // a neighbour of the root
    }
  }
  return SpfResult(std::move(done));
}

std::vector<Path> LinkState::tracePathsHost(const SpfResult& res, const std::string& src,
                                            const std::string& dst) const {
  std::vector<Path> out;
  if (!res.count(dst)) return out;
  std::unordered_set<const Link*> seen;
  std::function<std::optional<Path>(const std::string&)> one =
      [&](const std::string& x) -> std::optional<Path> {
    if (x == src) return Path{};
    for (const auto& pl : res.at(x).pathLinks()) {
      if (!seen.insert(pl.link.get()).second) continue;
      auto p = one(pl.prevNode);
      if (p) {
        p->push_back(pl.link);
        return p;
      }
    }
    return std::nullopt;
  };
  for (auto p = one(dst); p && !p->empty(); p = one(dst)) out.push_back(std::move(*p));
  return out;
}

ospf_digest LinkState::digestHost(const std::string& root, const SpfResult& res) const {
  // the engine's digest with u64 distances: node ids and the
  // root's neighbour bit positions of the current snapshot
  auto mix = [](uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebULL;
    x ^= x >> 31;
    return x;
  };
  const uint32_t r = csr_->ids.at(root);
  std::unordered_map<std::string, uint32_t> bit;
  for (uint32_t e = csr_->rowPtr[r]; e < csr_->rowPtr[r + 1]; ++e) {
    const uint32_t v = csr_->col[e];
    if (v != r && !bit.count(csr_->names[v])) {
      const uint32_t i = (uint32_t)bit.size();
      bit.emplace(csr_->names[v], i);
    }
  }
  ospf_digest d{0, 0, 0};
  for (const auto& [name, nr] : res) {
    const uint32_t v = csr_->ids.at(name);
    const uint64_t kd = mix((uint64_t)v ^ 0x2545F4914F6CDD1DULL) | 1ull;
    const uint64_t kn = mix((uint64_t)v ^ 0xD6E8FEB86659FD93ULL) | 1ull;
    std::map<uint32_t, uint32_t> words;
    for (const auto& h : nr.nextHops()) {
      const uint32_t i = bit.at(h);
      words[i / 32] |= 1u << (i % 32);
    }
    uint64_t ws = 0;
    for (const auto& [w, word] : words)
      if (word) ws += mix((((uint64_t)w << 32) | word) ^ 0x9E3779B97F4A7C15ULL);
    d.reached += 1;
    d.sum_dist += nr.metric();
    d.hash += kd * (nr.metric() + 1) + kn * ws;
  }
  return d;
}

bool LinkState::pathAInPathB(const Path& a, const Path& b) {
  if (a.size() > b.size()) return false;
  for (size_t i = 0; i + a.size() <= b.size(); ++i) {
    size_t k = 0;
    while (k < a.size() && a[k]->sameLink(*b[i + k])) ++k;
    if (k == a.size()) return true;
  }
  return false;
}

}  // namespace odl
