// ============================================================================
// linkstate_oracle.cpp — CPU ORACLE for the OpenR SPF hot path.
//
// TEST INFRASTRUCTURE ONLY. Nothing under openr_amd/ links, loads or calls
// this file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may use it, and only as the checker / the timed CPU baseline.
//
// What it is: a reference-shaped restatement of OpenR's LinkState SPF path
// (dgrnbrg-meta/openr @ 2025-02-28), written from the published behaviour:
//   * Link identity + hash       LinkState.cpp:122-140, 344-357 (orderedNames_,
//                                folly std::hash<pair> = hash_128_to_64 fold;
//                                folly rev 04c2275157a3e44c1d1fa1df75835fe4ec8a7b1e,
//                                folly/hash/Hash.h hash_combine_generic)
//   * ingest                     LinkState.cpp:551-756 (maybeMakeLink,
//                                getOrderedLinkSet, updateAdjacencyDatabase,
//                                deleteAdjacencyDatabase, removeNode)
//   * runSpf                     LinkState.cpp:836-911 (Dijkstra, ECMP
//                                next-hop name sets, pathLinks, overload)
//   * DijkstraQ                  LinkState.h:594-645 ((metric,name) heap,
//                                make_heap on strict improvement)
//   * getSpfResult / memo        LinkState.cpp:821-831
//   * getKthPaths/traceOnePath   LinkState.cpp:418-439, 790-819
//   * getMetricFromAToB          LinkState.cpp:777-788
//   * resolveUcmpWeights         LinkState.cpp:913-1033 (+ NodeUcmpResult,
//                                LinkState.h:275-333; DijkstraQUcmpNode :573-586)
// It keeps the reference's data-structure style (string keys, hash sets of
// shared_ptr<Link>, heap + reMake) on purpose: that cost shape is what the
// bench's cpu_baseline measures.
//
// Holds (hold-up / hold-down TTLs) are not modelled: Decision always ingests
// with TTL 0 (openr/decision/Decision.cpp:756), for which HoldableValue is a
// plain value.
//
// Parity pinning: the reference cannot be built here (it needs folly, fbthrift
// and fb303, none of which exist in this image), so this restatement is pinned
// by the reference's own known-answer tests transcribed under tests/golden/
// (see tests/golden/make_golden.py and DESIGN.md §Oracle).
// ============================================================================
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <optional>
#include <queue>
#include <sstream>
#include <string>
#include <thread>
#include <tuple>
#include <map>
#include <numeric>
#include <set>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../include/openr_adjdb.h"

namespace orc {

using Metric = uint64_t;

// folly::hash::hash_128_to_64 (Murmur-inspired fold), restated.
static inline uint64_t fold128(uint64_t upper, uint64_t lower) {
  const uint64_t k = 0x9ddfea08eb382d69ULL;
  uint64_t a = (lower ^ upper) * k;
  a ^= (a >> 47);
  uint64_t b = (upper ^ a) * k;
  b ^= (b >> 47);
  return b * k;
}

// folly's std::hash<std::pair<A,B>> = hash_128_to_64(hash(A), hash(B)),
// with std::hash<std::string> from libstdc++ for the leaves.
static inline uint64_t pairHash(const std::string& a, const std::string& b) {
  std::hash<std::string> h;
  return fold128(h(a), h(b));
}

struct Edge {  // one undirected Link of the reference
  std::string nA, nB, ifA, ifB;  // as constructed (node1 = the advertiser)
  Metric mA = 1, mB = 1;
  bool ovA = false, ovB = false;
  int32_t lblA = 0, lblB = 0;
  int64_t wA = 0, wB = 0;
  // orderedNames_: min/max of (node, if) pairs
  std::pair<std::string, std::string> lo, hi;
  size_t hash = 0;

  Edge(const std::string& n1, const std::string& if1, const std::string& n2,
       const std::string& if2)
      : nA(n1), nB(n2), ifA(if1), ifB(if2) {
    auto p1 = std::make_pair(n1, if1), p2 = std::make_pair(n2, if2);
    if (p2 < p1) std::swap(p1, p2);
    lo = p1;
    hi = p2;
    hash = fold128(pairHash(lo.first, lo.second), pairHash(hi.first, hi.second));
  }
  bool up() const { return !ovA && !ovB; }
  const std::string& peer(const std::string& n) const {
    if (nA == n) return nB;
    if (nB == n) return nA;
    throw std::invalid_argument(n);
  }
  Metric metricFrom(const std::string& n) const {
    if (nA == n) return mA;
    if (nB == n) return mB;
    throw std::invalid_argument(n);
  }
  const std::string& ifFrom(const std::string& n) const {
    if (nA == n) return ifA;
    if (nB == n) return ifB;
    throw std::invalid_argument(n);
  }
  int64_t weightFrom(const std::string& n) const {  // Link::getWeightFromNode
    if (nA == n) return wA;
    if (nB == n) return wB;
    throw std::invalid_argument(n);
  }
  bool sameAs(const Edge& o) const {
    return hash == o.hash && lo == o.lo && hi == o.hi;
  }
  bool before(const Edge& o) const {  // Link::operator<
    if (hash != o.hash) return hash < o.hash;
    return std::tie(lo, hi) < std::tie(o.lo, o.hi);
  }
  std::string key() const {
    return lo.first + "%" + lo.second + "|" + hi.first + "%" + hi.second;
  }
};
using EdgeP = std::shared_ptr<Edge>;

struct EdgeHash {
  size_t operator()(const EdgeP& e) const { return e->hash; }
};
struct EdgeEq {
  bool operator()(const EdgeP& a, const EdgeP& b) const { return a->sameAs(*b); }
};
using EdgeSet = std::unordered_set<EdgeP, EdgeHash, EdgeEq>;

struct Adj {
  std::string other, ifName, otherIf;
  int32_t metric = 1, label = 0;
  bool overloaded = false;
  int64_t weight = 1;
};
struct AdjDb {
  std::string name;
  bool overloaded = false;
  int32_t nodeLabel = 0;
  std::vector<Adj> adjs;
  // (otherNodeName, ifName, otherIfName) -> first adjacency with that triple;
  // lets tryLink find the reverse adjacency without the reference's linear
  // scan while returning the same (first) match.
  std::unordered_map<std::string, uint32_t> byTriple;
  static std::string triple(const std::string& o, const std::string& i,
                            const std::string& oi) {
    std::string k;
    k.reserve(o.size() + i.size() + oi.size() + 2);
    k.append(o).push_back('\0');
    k.append(i).push_back('\0');
    k.append(oi);
    return k;
  }
  void index() {
    byTriple.clear();
    for (uint32_t i = 0; i < adjs.size(); ++i)
      byTriple.emplace(triple(adjs[i].other, adjs[i].ifName, adjs[i].otherIf), i);
  }
};

struct NodeResult {
  Metric metric;
  std::vector<std::pair<EdgeP, std::string>> pathLinks;
  std::unordered_set<std::string> nextHops;
  explicit NodeResult(Metric m) : metric(m) {}
};
using SpfResult = std::unordered_map<std::string, NodeResult>;
using Path = std::vector<EdgeP>;

// (metric, name) binary heap with a name index; reMake == std::make_heap.
class HeapQ {
 public:
  struct Item {
    std::string name;
    NodeResult res;
    Item(const std::string& n, Metric m) : name(n), res(m) {}
  };
  using ItemP = std::shared_ptr<Item>;

  void push(const std::string& n, Metric m) {
    heap_.push_back(std::make_shared<Item>(n, m));
    index_[n] = heap_.back();
    std::push_heap(heap_.begin(), heap_.end(), greater_);
  }
  ItemP find(const std::string& n) {
    auto it = index_.find(n);
    return it == index_.end() ? nullptr : it->second;
  }
  ItemP popMin() {
    if (heap_.empty()) return nullptr;
    ItemP top = heap_.front();
    index_.erase(top->name);
    std::pop_heap(heap_.begin(), heap_.end(), greater_);
    heap_.pop_back();
    return top;
  }
  void rebuild() { std::make_heap(heap_.begin(), heap_.end(), greater_); }

 private:
  struct Greater {
    bool operator()(const ItemP& a, const ItemP& b) const {
      if (a->res.metric != b->res.metric) return a->res.metric > b->res.metric;
      return a->name > b->name;
    }
  } greater_;
  std::vector<ItemP> heap_;
  std::unordered_map<std::string, ItemP> index_;
};

class Graph {
 public:
  std::unordered_map<std::string, EdgeSet> byNode;
  EdgeSet all;
  std::unordered_map<std::string, bool> nodeOverload;
  std::unordered_map<std::string, AdjDb> dbs;
  mutable std::unordered_map<std::string, SpfResult> memoMetric, memoHops;
  mutable std::unordered_map<std::string, std::vector<Path>> memoKsp;
  mutable std::atomic<uint64_t> spfRuns{0};

  const EdgeSet& linksOf(const std::string& n) const {
    static const EdgeSet empty;
    auto it = byNode.find(n);
    return it == byNode.end() ? empty : it->second;
  }
  bool overloaded(const std::string& n) const {
    auto it = nodeOverload.find(n);
    return it != nodeOverload.end() && it->second;
  }
  void clearMemo() {
    memoMetric.clear();
    memoHops.clear();
    memoKsp.clear();
  }

  EdgeP tryLink(const std::string& self, const Adj& a) const {
    auto it = dbs.find(a.other);
    if (it == dbs.end()) return nullptr;
    auto hit = it->second.byTriple.find(AdjDb::triple(self, a.otherIf, a.ifName));
    if (hit != it->second.byTriple.end()) {
      const Adj& b = it->second.adjs[hit->second];
      {
        auto e = std::make_shared<Edge>(self, a.ifName, a.other, b.ifName);
        e->mA = (Metric)(int64_t)a.metric;  // i32 -> u64 as in the reference
        e->mB = (Metric)(int64_t)b.metric;
        e->ovA = a.overloaded;
        e->ovB = b.overloaded;
        e->lblA = a.label;
        e->lblB = b.label;
        e->wA = a.weight;
        e->wB = b.weight;
        return e;
      }
    }
    return nullptr;
  }

  static void sortLinks(std::vector<EdgeP>& v) {
    std::sort(v.begin(), v.end(),
              [](const EdgeP& x, const EdgeP& y) { return x->before(*y); });
  }

  void insertLink(const EdgeP& e) {
    if (!byNode[e->lo.first].insert(e).second) abort();
    if (!byNode[e->hi.first].insert(e).second) abort();
    if (!all.insert(e).second) abort();
  }
  void eraseLink(const EdgeP& e) {
    if (!byNode.at(e->lo.first).erase(e)) abort();
    if (!byNode.at(e->hi.first).erase(e)) abort();
    if (!all.erase(e)) abort();
  }

  oadj_change update(const AdjDb& db) {
    oadj_change ch{0, 0, 0, 0, 0};
    const std::string& me = db.name;
    AdjDb prior = std::move(dbs[me]);
    dbs[me] = db;

    std::vector<EdgeP> oldL;
    if (byNode.count(me)) {
      oldL.assign(byNode.at(me).begin(), byNode.at(me).end());
      sortLinks(oldL);
    }
    std::vector<EdgeP> newL;
    for (const auto& a : db.adjs) {
      if (auto e = tryLink(me, a)) newL.push_back(e);
    }
    sortLinks(newL);

    // node overload (HoldableValue with TTL 0: plain value)
    auto ov = nodeOverload.find(me);
    if (ov == nodeOverload.end()) {
      nodeOverload.emplace(me, db.overloaded);
    } else if (ov->second != db.overloaded) {
      ov->second = db.overloaded;
      ch.topology_changed = 1;
    }
    ch.node_label_changed = prior.nodeLabel != db.nodeLabel;

    size_t i = 0, j = 0;
    while (i < newL.size() || j < oldL.size()) {
      if (i < newL.size() && (j == oldL.size() || newL[i]->before(*oldL[j]))) {
        ch.topology_changed |= newL[i]->up();
        insertLink(newL[i]);
        ch.n_added_links++;
        ++i;
      } else if (j < oldL.size() &&
                 (i == newL.size() || oldL[j]->before(*newL[i]))) {
        ch.topology_changed |= oldL[j]->up();
        eraseLink(oldL[j]);
        ++j;
      } else {
        Edge& nw = *newL[i];
        Edge& od = *oldL[j];
        bool meIsA = (od.nA == me);
        Metric nm = nw.metricFrom(me);
        Metric& om = meIsA ? od.mA : od.mB;
        if (nm != om) {
          om = nm;
          ch.topology_changed = 1;
        }
        bool nov = (nw.nA == me) ? nw.ovA : nw.ovB;
        bool& oov = meIsA ? od.ovA : od.ovB;
        if (nov != oov) {
          bool wasUp = od.up();
          oov = nov;
          ch.topology_changed |= (wasUp != od.up());
        }
        int32_t nl = (nw.nA == me) ? nw.lblA : nw.lblB;
        int32_t& ol = meIsA ? od.lblA : od.lblB;
        if (nl != ol) {
          ol = nl;
          ch.link_attributes_changed = 1;
        }
        int64_t nwt = (nw.nA == me) ? nw.wA : nw.wB;
        int64_t& owt = meIsA ? od.wA : od.wB;
        if (nwt != owt) {
          owt = nwt;
          ch.link_attributes_changed = 1;
        }
        ++i;
        ++j;
      }
    }
    if (ch.topology_changed) clearMemo();
    return ch;
  }

  oadj_change remove(const std::string& me) {
    oadj_change ch{0, 0, 0, 0, 0};
    auto it = dbs.find(me);
    if (it == dbs.end()) return ch;
    auto bn = byNode.find(me);
    if (bn != byNode.end()) {
      for (const auto& e : bn->second) {
        if (!byNode.at(e->peer(me)).erase(e)) abort();
        if (!all.erase(e)) abort();
      }
      byNode.erase(bn);
      nodeOverload.erase(me);
    }
    dbs.erase(it);
    clearMemo();
    ch.topology_changed = 1;
    return ch;
  }

  // runSpf restated: Dijkstra over up links, ECMP next-hop name sets,
  // pathLinks in (pop order, linksOf iteration order).
  SpfResult dijkstra(const std::string& src, bool useMetric,
                     const EdgeSet* skip) const {
    spfRuns.fetch_add(1, std::memory_order_relaxed);
    SpfResult out;
    HeapQ q;
    q.push(src, 0);
    while (auto cur = q.popMin()) {
      auto ins = out.emplace(cur->name, std::move(cur->res));
      if (!ins.second) abort();
      const std::string& u = ins.first->first;
      const Metric du = ins.first->second.metric;
      const auto& nhU = ins.first->second.nextHops;
      if (u != src && overloaded(u)) continue;  // no transit
      for (const auto& e : linksOf(u)) {
        const std::string& v = e->peer(u);
        if (!e->up() || out.count(v) || (skip && skip->count(e))) continue;
        Metric w = useMetric ? e->metricFrom(u) : 1;
        auto item = q.find(v);
        if (!item) {
          q.push(v, du + w);
          item = q.find(v);
        }
        if (item->res.metric < du + w) continue;
        if (item->res.metric > du + w) {
          item->res.metric = du + w;
          item->res.pathLinks.clear();
          item->res.nextHops.clear();
          q.rebuild();
        }
        item->res.pathLinks.emplace_back(e, u);
        item->res.nextHops.insert(nhU.begin(), nhU.end());
        if (item->res.nextHops.empty()) item->res.nextHops.insert(v);
      }
    }
    return out;
  }

  const SpfResult& spf(const std::string& n, bool useMetric) const {
    auto& memo = useMetric ? memoMetric : memoHops;
    auto it = memo.find(n);
    if (it == memo.end()) it = memo.emplace(n, dijkstra(n, useMetric, nullptr)).first;
    return it->second;
  }

  std::optional<Path> trace(const std::string& src, const std::string& dst,
                            const SpfResult& r, EdgeSet& seen) const {
    if (src == dst) return Path{};
    for (const auto& pl : r.at(dst).pathLinks) {
      if (seen.insert(pl.first).second) {
        auto p = trace(src, pl.second, r, seen);
        if (p) {
          p->push_back(pl.first);
          return p;
        }
      }
    }
    return std::nullopt;
  }

  const std::vector<Path>& kthPaths(const std::string& s, const std::string& d,
                                    size_t k) const {
    if (k < 1) abort();
    std::string key = s + '\x01' + d + '\x01' + std::to_string(k);
    auto it = memoKsp.find(key);
    if (it != memoKsp.end()) return it->second;
    EdgeSet skip;
    for (size_t i = 1; i < k; ++i)
      for (const auto& p : kthPaths(s, d, i))
        for (const auto& e : p) skip.insert(e);
    std::vector<Path> paths;
    SpfResult tmp;
    const SpfResult* r;
    if (skip.empty()) {
      r = &spf(s, true);
    } else {
      tmp = dijkstra(s, true, &skip);
      r = &tmp;
    }
    if (r->count(d)) {
      EdgeSet seen;
      auto p = trace(s, d, *r, seen);
      while (p && !p->empty()) {
        paths.push_back(std::move(*p));
        p = trace(s, d, *r, seen);
      }
    }
    return memoKsp.emplace(key, std::move(paths)).first->second;
  }
};

// ---------------------------------------------------------------------------
// resolveUcmpWeights (LinkState.cpp:913-1033): walk the SPF DAG from equally
// distant weighted leaves towards the root in (metric, name) order; a node's
// advertised weight is the sum over its next-hop links of the link weight
// (ADJ propagation, algo 2) or of the next hop's advertised weight (PREFIX
// propagation, algo 3); next-hop weights are then divided by their gcd.
struct UcmpHop {
  EdgeP link;
  std::string nextHopNode;
  int64_t weight;
};
struct NodeUcmp {
  std::optional<int64_t> weight;
  std::unordered_map<std::string, UcmpHop> hops;  // local interface -> hop
};
using UcmpResult = std::unordered_map<std::string, NodeUcmp>;

static UcmpResult resolveUcmp(const SpfResult& spf,
                              const std::vector<std::pair<std::string, int64_t>>& leaves,
                              int algo, bool useMetric) {
  UcmpResult out;
  // DijkstraQ<DijkstraQUcmpNode>: live entries by name, pop order (metric, name)
  struct Item {
    Metric metric;
    NodeUcmp res;
  };
  std::unordered_map<std::string, Item> live;
  std::set<std::pair<Metric, std::string>> order;
  auto insert = [&](const std::string& n, Metric m) {
    live[n] = Item{m, NodeUcmp{}};
    order.emplace(m, n);
  };
  std::optional<Metric> spfMetric;
  for (const auto& [leaf, w] : leaves) {
    auto it = spf.find(leaf);
    if (it == spf.end()) continue;
    const Metric m = it->second.metric;
    if (!spfMetric) {
      spfMetric = m;
    } else if (*spfMetric != m) {
      return UcmpResult{};  // leaves at different distances: skipped
    }
    insert(leaf, 0);
    live[leaf].res.weight = w;
  }
  while (!order.empty()) {
    const auto [m, name] = *order.begin();
    order.erase(order.begin());
    NodeUcmp cur = std::move(live.at(name).res);
    live.erase(name);
    if (!cur.weight) {
      int64_t w = 0;
      for (const auto& [iface, hop] : cur.hops)
        w += algo == 2 ? hop.link->weightFrom(name) : hop.weight;
      cur.weight = w;
    }
    auto sit = spf.find(name);
    if (sit == spf.end()) abort();  // CHECK in the reference
    for (const auto& [link, prev] : sit->second.pathLinks) {
      const Metric lm = useMetric ? link->metricFrom(prev) : 1;
      if (!live.count(prev)) insert(prev, m + lm);
      live.at(prev).res.hops.emplace(link->ifFrom(prev), UcmpHop{link, name, *cur.weight});
    }
    int64_t g = 0;  // normalizeNextHopWeights
    for (const auto& [iface, hop] : cur.hops) g = std::gcd(g, hop.weight);
    if (g > 1)
      for (auto& [iface, hop] : cur.hops) hop.weight /= g;
    out.emplace(name, std::move(cur));
  }
  return out;
}

// ---------------------------------------------------------------------------
// digest (layout-independent; identical definition in DESIGN.md §Digest)
static inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

struct Digest {
  uint64_t reached = 0, sumDist = 0, hash = 0;
};

// sum over reached nodes v of dist_key(v) * (dist + 1) plus,
// for every non-zero next-hop word g of v, node_key(v) * word_key(g, word)
// (mod 2^64). Word g holds the bits of the root's distinct neighbours
// 32g .. 32g+31 in ascending id order (ids = name ranks; neighbours over
// every link of the root, up or down). Unknown names get id 0xFFFFFFFF.
static inline uint64_t nodeTerm(uint64_t v, uint64_t dist) {
  const uint64_t distKey = mix64((v & 0xFFFFFFFFull) ^ 0x2545F4914F6CDD1DULL) | 1ull;
  return distKey * (dist + 1);
}
static inline uint64_t wordTerm(uint64_t v, uint64_t g, uint32_t word) {
  if (!word) return 0;
  const uint64_t nodeKey = mix64((v & 0xFFFFFFFFull) ^ 0xD6E8FEB86659FD93ULL) | 1ull;
  const uint64_t wordKey = mix64(((g << 32) | word) ^ 0x9E3779B97F4A7C15ULL);
  return nodeKey * wordKey;
}

static Digest digestOf(const Graph& g, const std::string& root, const SpfResult& r,
                       const std::unordered_map<std::string, uint32_t>& ids) {
  Digest d;
  auto idOf = [&](const std::string& n) -> uint64_t {
    auto it = ids.find(n);
    return it == ids.end() ? 0xFFFFFFFFull : it->second;
  };
  std::vector<uint64_t> nbr;  // the root's distinct neighbours, ascending id
  for (const auto& e : g.linksOf(root)) {
    const std::string& p = e->peer(root);
    if (p != root) nbr.push_back(idOf(p));
  }
  std::sort(nbr.begin(), nbr.end());
  nbr.erase(std::unique(nbr.begin(), nbr.end()), nbr.end());
  std::map<uint64_t, uint32_t> words;
  for (const auto& [name, nr] : r) {
    const uint64_t id = idOf(name);
    d.reached++;
    d.sumDist += nr.metric;
    d.hash += nodeTerm(id, nr.metric);
    words.clear();
    for (const auto& nh : nr.nextHops) {
      const uint64_t i = std::lower_bound(nbr.begin(), nbr.end(), idOf(nh)) - nbr.begin();
      words[i / 32] |= 1u << (i % 32);
    }
    for (const auto& [w, bits] : words) d.hash += wordTerm(id, w, bits);
  }
  return d;
}

static std::string str(const oadj_stream* s, uint32_t i) {
  return std::string(s->str_data + s->str_off[i], s->str_data + s->str_off[i + 1]);
}

}  // namespace orc

// ============================================================================
// C API (ctypes) — test infrastructure only
// ============================================================================
using namespace orc;

namespace {
// CSR view of the oracle's own link sets (built from Graph, never from the
// product's snapshot) for the CSR-Dijkstra restatement below.
struct FastCsr {
  uint32_t V = 0;
  std::vector<uint32_t> rowPtr, col, wOut, wIn, nbrOff, nbr;
  std::vector<uint8_t> up, noTransit;
};

struct Oracle {
  Graph g;
  std::unordered_map<std::string, uint32_t> ids;  // name -> rank (byte-lex)
  bool idsDirty = true;
  FastCsr csr;
  bool csrDirty = true;
  void refreshCsr() {
    refreshIds();
    if (!csrDirty) return;
    std::vector<std::string> names(ids.size());
    for (const auto& kv : ids) names[kv.second] = kv.first;
    FastCsr c;
    c.V = (uint32_t)names.size();
    c.rowPtr.assign(c.V + 1, 0);
    c.nbrOff.assign(c.V + 1, 0);
    c.noTransit.assign(c.V, 0);
    for (uint32_t u = 0; u < c.V; ++u) {
      c.noTransit[u] = g.overloaded(names[u]) ? 1 : 0;
      std::vector<uint32_t> nb;
      for (const auto& e : g.linksOf(names[u])) {
        const std::string& p = e->peer(names[u]);
        auto it = ids.find(p);
        if (it == ids.end()) continue;
        c.col.push_back(it->second);
        c.wOut.push_back((uint32_t)e->metricFrom(names[u]));
        c.wIn.push_back((uint32_t)e->metricFrom(p));
        c.up.push_back(e->up() ? 1 : 0);
        if (p != names[u]) nb.push_back(it->second);
      }
      std::sort(nb.begin(), nb.end());
      nb.erase(std::unique(nb.begin(), nb.end()), nb.end());
      c.nbr.insert(c.nbr.end(), nb.begin(), nb.end());
      c.rowPtr[u + 1] = (uint32_t)c.col.size();
      c.nbrOff[u + 1] = (uint32_t)c.nbr.size();
    }
    csr = std::move(c);
    csrDirty = false;
  }
  void refreshIds() {
    if (!idsDirty) return;
    std::vector<std::string> names;
    names.reserve(g.dbs.size());
    for (const auto& kv : g.dbs) names.push_back(kv.first);
    std::sort(names.begin(), names.end());
    ids.clear();
    for (uint32_t i = 0; i < names.size(); ++i) ids.emplace(names[i], i);
    idsDirty = false;
  }
};

char* dupString(const std::string& s) {
  char* p = (char*)malloc(s.size() + 1);
  memcpy(p, s.data(), s.size() + 1);
  return p;
}

std::string ucmpText(const UcmpResult& r) {
  std::vector<std::string> names;
  for (const auto& kv : r) names.push_back(kv.first);
  std::sort(names.begin(), names.end());
  std::ostringstream os;
  for (const auto& n : names) {
    const NodeUcmp& u = r.at(n);
    os << n << '\t' << (u.weight ? *u.weight : 0) << '\t';
    std::vector<std::string> ifs;
    for (const auto& kv : u.hops) ifs.push_back(kv.first);
    std::sort(ifs.begin(), ifs.end());
    for (size_t i = 0; i < ifs.size(); ++i) {
      const UcmpHop& hp = u.hops.at(ifs[i]);
      os << (i ? "," : "") << ifs[i] << '=' << hp.nextHopNode << ':' << hp.weight;
    }
    os << '\n';
  }
  return os.str();
}

std::string spfText(const SpfResult& r) {
  std::vector<const std::string*> names;
  for (const auto& kv : r) names.push_back(&kv.first);
  std::sort(names.begin(), names.end(),
            [](const std::string* a, const std::string* b) { return *a < *b; });
  std::ostringstream os;
  for (const auto* n : names) {
    const NodeResult& nr = r.at(*n);
    std::vector<std::string> nh(nr.nextHops.begin(), nr.nextHops.end());
    std::sort(nh.begin(), nh.end());
    os << *n << '\t' << nr.metric << '\t';
    for (size_t i = 0; i < nh.size(); ++i) os << (i ? "," : "") << nh[i];
    os << '\t';
    for (size_t i = 0; i < nr.pathLinks.size(); ++i)
      os << (i ? ";" : "") << nr.pathLinks[i].first->key() << '@'
         << nr.pathLinks[i].second;
    os << '\n';
  }
  return os.str();
}
}  // namespace

extern "C" {

void* orc_create() { return new Oracle(); }
void orc_destroy(void* h) { delete (Oracle*)h; }
void orc_free(char* p) { free(p); }

int orc_apply(void* h, const oadj_stream* s, uint32_t first, uint32_t count,
              oadj_change* changes) {
  Oracle* o = (Oracle*)h;
  for (uint32_t k = 0; k < count; ++k) {
    uint32_t i = first + k;
    if (i >= s->n_dbs) return -1;
    std::string name = str(s, s->db_name[i]);
    oadj_change ch;
    if (s->db_delete && s->db_delete[i]) {
      ch = o->g.remove(name);
    } else {
      AdjDb db;
      db.name = name;
      db.overloaded = s->db_overloaded[i] != 0;
      db.nodeLabel = s->db_node_label[i];
      for (uint64_t a = s->db_adj_off[i]; a < s->db_adj_off[i + 1]; ++a) {
        Adj x;
        x.other = str(s, s->adj_other[a]);
        x.ifName = str(s, s->adj_if[a]);
        x.otherIf = str(s, s->adj_other_if[a]);
        x.metric = s->adj_metric[a];
        x.label = s->adj_label[a];
        x.overloaded = s->adj_overloaded[a] != 0;
        x.weight = s->adj_weight[a];
        db.adjs.push_back(std::move(x));
      }
      db.index();
      ch = o->g.update(db);
    }
    o->idsDirty = true;
    o->csrDirty = true;
    if (changes) changes[k] = ch;
  }
  return 0;
}

char* orc_spf_text(void* h, const char* root, int useMetric) {
  Oracle* o = (Oracle*)h;
  return dupString(spfText(o->g.spf(root, useMetric != 0)));
}

char* orc_kth_paths_text(void* h, const char* src, const char* dst, int k) {
  Oracle* o = (Oracle*)h;
  std::ostringstream os;
  for (const auto& p : o->g.kthPaths(src, dst, (size_t)k)) {
    for (size_t i = 0; i < p.size(); ++i) os << (i ? "," : "") << p[i]->key();
    os << '\n';
  }
  return dupString(os.str());
}

// resolveUcmpWeights over getSpfResult(root): leaves = "name\tweight\n"...,
// algo 2 (ADJ weight propagation) or 3 (PREFIX weight propagation). Text: one
// line per node, sorted: node \t weight \t iface=nextHop:weight,... (sorted)
char* orc_ucmp_text(void* h, const char* root, const char* leavesNl, uint32_t n, int algo,
                    int useMetric) {
  Oracle* o = (Oracle*)h;
  std::vector<std::pair<std::string, int64_t>> leaves;
  const char* p = leavesNl;
  for (uint32_t i = 0; i < n; ++i) {
    const char* q = strchr(p, '\n');
    if (!q) q = p + strlen(p);
    const std::string ln(p, q);
    const size_t t = ln.find('\t');
    leaves.emplace_back(ln.substr(0, t), std::stoll(ln.substr(t + 1)));
    p = *q ? q + 1 : q;
  }
  return dupString(ucmpText(resolveUcmp(o->g.spf(root, useMetric != 0), leaves, algo,
                                        useMetric != 0)));
}

char* orc_links_text(void* h, const char* node) {
  Oracle* o = (Oracle*)h;
  std::ostringstream os;
  for (const auto& e : o->g.linksOf(node))
    os << e->key() << '\t' << e->metricFrom(node) << '\t' << e->up() << '\n';
  return dupString(os.str());
}

int64_t orc_metric_a_to_b(void* h, const char* a, const char* b, int useMetric) {
  Oracle* o = (Oracle*)h;
  if (std::string(a) == b) return 0;
  const auto& r = o->g.spf(a, useMetric != 0);
  auto it = r.find(b);
  return it == r.end() ? -1 : (int64_t)it->second.metric;
}

uint64_t orc_spf_runs(void* h) { return ((Oracle*)h)->g.spfRuns.load(); }
uint32_t orc_num_nodes(void* h) { return (uint32_t)((Oracle*)h)->g.dbs.size(); }
uint32_t orc_num_links(void* h) { return (uint32_t)((Oracle*)h)->g.all.size(); }
int orc_is_overloaded(void* h, const char* n) { return ((Oracle*)h)->g.overloaded(n); }

// Un-memoized runSpf for `n` roots on `threads` host threads (the bench's CPU
// baseline and the at-scale digest checker). roots = '\n'-separated names.
// out: 3 u64 per root {reached, sumDist, digest}.
int orc_digest_roots(void* h, const char* rootsNl, uint32_t n, int useMetric,
                     int threads, uint64_t* out) {
  Oracle* o = (Oracle*)h;
  o->refreshIds();
  std::vector<std::string> roots;
  const char* p = rootsNl;
  for (uint32_t i = 0; i < n; ++i) {
    const char* q = strchr(p, '\n');
    if (!q) q = p + strlen(p);
    roots.emplace_back(p, q);
    p = *q ? q + 1 : q;
  }
  if (threads < 1) threads = 1;
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    for (uint32_t i; (i = next.fetch_add(1)) < n;) {
      SpfResult r = o->g.dijkstra(roots[i], useMetric != 0, nullptr);
      Digest d = digestOf(o->g, roots[i], r, o->ids);
      out[3 * i] = d.reached;
      out[3 * i + 1] = d.sumDist;
      out[3 * i + 2] = d.hash;
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  return 0;
}

// CSR-Dijkstra restatement of runSpf: the same
// result as Graph::dijkstra -- distances, and next-hop sets as the OR over
// tight usable in-links from settled transit tails (LinkState.cpp:869-901),
// a directly connected node contributing itself -- on integer node ids with a
// lazy-deletion binary heap, so weighted 100k..1M-node graphs take
// milliseconds..seconds per root instead of the reference-shaped heap's
// O(V) make_heap per strict improvement (LinkState.cpp:893). Metrics must be
// >= 1 (then dist and next-hop sets do not depend on pop order within a
// distance). Digests as orc_digest_roots. The test suite pins it against the
// reference-shaped Graph::dijkstra on random graphs. Roots unknown to the
// graph fall back to Graph::dijkstra.
int orc_fast_digest_roots(void* h, const char* rootsNl, uint32_t n, int useMetric,
                          int threads, uint64_t* out) {
  Oracle* o = (Oracle*)h;
  o->refreshCsr();
  const FastCsr& c = o->csr;
  std::vector<std::string> roots;
  const char* p = rootsNl;
  for (uint32_t i = 0; i < n; ++i) {
    const char* q = strchr(p, '\n');
    if (!q) q = p + strlen(p);
    roots.emplace_back(p, q);
    p = *q ? q + 1 : q;
  }
  if (threads < 1) threads = 1;
  std::atomic<uint32_t> next{0};
  const uint32_t INF = 0xFFFFFFFFu;
  auto work = [&]() {
    std::vector<uint32_t> dist(c.V), nh;
    std::vector<uint8_t> done(c.V);
    for (uint32_t i; (i = next.fetch_add(1)) < n;) {
      auto it = o->ids.find(roots[i]);
      if (it == o->ids.end()) {
        SpfResult r = o->g.dijkstra(roots[i], useMetric != 0, nullptr);
        Digest d = digestOf(o->g, roots[i], r, o->ids);
        out[3 * i] = d.reached;
        out[3 * i + 1] = d.sumDist;
        out[3 * i + 2] = d.hash;
        continue;
      }
      const uint32_t s = it->second;
      const uint32_t nb0 = c.nbrOff[s], nnb = c.nbrOff[s + 1] - nb0;
      const uint32_t W = std::max<uint32_t>(1, (nnb + 31) / 32);
      std::fill(dist.begin(), dist.end(), INF);
      std::fill(done.begin(), done.end(), 0);
      nh.assign((size_t)c.V * W, 0u);
      using QE = std::pair<uint64_t, uint32_t>;
      std::priority_queue<QE, std::vector<QE>, std::greater<QE>> q;
      dist[s] = 0;
      q.push({0, s});
      Digest dg;
      while (!q.empty()) {
        const auto [d, v] = q.top();
        q.pop();
        if (done[v] || d != dist[v]) continue;
        done[v] = 1;
        uint32_t* row = &nh[(size_t)v * W];
        if (v != s) {
          for (uint32_t e = c.rowPtr[v]; e < c.rowPtr[v + 1]; ++e) {
            const uint32_t u = c.col[e];
            if (!c.up[e] || u == v || !done[u]) continue;
            const uint64_t w = useMetric ? c.wIn[e] : 1;
            if ((uint64_t)dist[u] + w != d) continue;
            if (u == s) {
              const uint32_t b = (uint32_t)(std::lower_bound(c.nbr.begin() + nb0,
                                                             c.nbr.begin() + nb0 + nnb, v) -
                                            (c.nbr.begin() + nb0));
              row[b / 32] |= 1u << (b % 32);
            } else if (!c.noTransit[u]) {
              const uint32_t* src = &nh[(size_t)u * W];
              for (uint32_t k = 0; k < W; ++k) row[k] |= src[k];
            }
          }
        }
        dg.reached++;
        dg.sumDist += d;
        dg.hash += nodeTerm(v, d);
        for (uint32_t k = 0; k < W; ++k) dg.hash += wordTerm(v, k, row[k]);
        if (v != s && c.noTransit[v]) continue;
        for (uint32_t e = c.rowPtr[v]; e < c.rowPtr[v + 1]; ++e) {
          const uint32_t y = c.col[e];
          if (!c.up[e] || y == v || done[y]) continue;
          const uint64_t nd = d + (useMetric ? c.wOut[e] : 1);
          if (nd < dist[y]) {
            dist[y] = (uint32_t)nd;
            q.push({nd, y});
          }
        }
      }
      out[3 * i] = dg.reached;
      out[3 * i + 1] = dg.sumDist;
      out[3 * i + 2] = dg.hash;
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  return 0;
}

// Masked KSP2 reruns for every destination of `src` (getKthPaths(src, d, 2)
// for d in dsts), k=2 paths as text blocks separated by a line "=".
char* orc_ksp2_text(void* h, const char* src, const char* dstsNl, uint32_t n) {
  Oracle* o = (Oracle*)h;
  std::ostringstream os;
  const char* p = dstsNl;
  for (uint32_t i = 0; i < n; ++i) {
    const char* q = strchr(p, '\n');
    if (!q) q = p + strlen(p);
    std::string d(p, q);
    p = *q ? q + 1 : q;
    for (const auto& path : o->g.kthPaths(src, d, 2)) {
      for (size_t j = 0; j < path.size(); ++j)
        os << (j ? "," : "") << path[j]->key();
      os << '\n';
    }
    os << "=\n";
  }
  return dupString(os.str());
}

// orc_ksp2_text on `threads` host threads (the KSP2 bench's CPU baseline):
// the memoised SPF of src is made once, then every destination's
// getKthPaths(src, d, 1) trace, its masked rerun runSpf(src, true, k = 1
// links) and the k = 2 trace run on the threads (LinkState.cpp:790-819,
// kthPaths above without the shared memo). Same text as orc_ksp2_text.
char* orc_ksp2_text_threads(void* h, const char* src, const char* dstsNl, uint32_t n,
                            int threads) {
  Oracle* o = (Oracle*)h;
  std::vector<std::string> dsts;
  const char* p = dstsNl;
  for (uint32_t i = 0; i < n; ++i) {
    const char* q = strchr(p, '\n');
    if (!q) q = p + strlen(p);
    dsts.emplace_back(p, q);
    p = *q ? q + 1 : q;
  }
  const std::string s(src);
  const SpfResult& base = o->g.spf(s, true);  // serial: the memo is not shared below
  auto tracesOf = [&](const SpfResult& r, const std::string& d) {
    std::vector<Path> paths;
    if (!r.count(d)) return paths;
    EdgeSet seen;
    auto pth = o->g.trace(s, d, r, seen);
    while (pth && !pth->empty()) {
      paths.push_back(std::move(*pth));
      pth = o->g.trace(s, d, r, seen);
    }
    return paths;
  };
  std::vector<std::string> out(n);
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    for (uint32_t i; (i = next.fetch_add(1)) < n;) {
      const std::vector<Path> k1 = tracesOf(base, dsts[i]);
      EdgeSet skip;
      for (const auto& path : k1)
        for (const auto& e : path) skip.insert(e);
      std::vector<Path> k2;
      if (skip.empty()) {
        k2 = k1;
      } else {
        const SpfResult r = o->g.dijkstra(s, true, &skip);
        k2 = tracesOf(r, dsts[i]);
      }
      std::ostringstream os;
      for (const auto& path : k2) {
        for (size_t j = 0; j < path.size(); ++j) os << (j ? "," : "") << path[j]->key();
        os << '\n';
      }
      os << "=\n";
      out[i] = os.str();
    }
  };
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  std::string all;
  for (const auto& x : out) all += x;
  return dupString(all);
}

}  // extern "C"

// Iteration order of std::unordered_map<int, T> built from an initializer
// list of `keys` (the order DecisionTestUtils.cpp:20 getLinkState ingests
// its adjacency map in). Same libstdc++ => same order.
extern "C" int orc_intmap_order(const int32_t* keys, uint32_t n, int32_t* out) {
  std::vector<std::pair<const int, int>> init;
  for (uint32_t i = 0; i < n; ++i) init.emplace_back(keys[i], (int)i);
  std::unordered_map<int, int> m(init.begin(), init.end());
  uint32_t k = 0;
  for (const auto& kv : m) out[k++] = kv.first;
  return (int)k;
}
