// spf_solver.cpp — see spf_solver.h.
#include "spf_solver.h"

#include <algorithm>
#include <limits>
#include <set>
#include <stdexcept>
#include <tuple>

namespace odl {

bool NextHop::operator<(const NextHop& o) const {
  return std::tie(ifName, neighbor, metric, op, labels, weight) <
         std::tie(o.ifName, o.neighbor, o.metric, o.op, o.labels, o.weight);
}
bool NextHop::operator==(const NextHop& o) const {
  return std::tie(ifName, neighbor, metric, op, labels, weight) ==
         std::tie(o.ifName, o.neighbor, o.metric, o.op, o.labels, o.weight);
}

namespace {
void sortUnique(std::vector<NextHop>& v) {
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
}
}  // namespace

int32_t SpfSolver::nodeLabel(const std::string& node) const {
  const auto& dbs = ls_.getAdjacencyDatabases();
  auto it = dbs.find(node);
  return it == dbs.end() ? 0 : it->second.nodeLabel;
}

MinCostNextHops SpfSolver::nextHopsWithMetric(const std::string& me,
                                              const std::vector<std::string>& dsts,
                                              bool perDestination) {
  return nextHopsWithMetric(ls_.getSpfResult(me), dsts, perDestination);
}

MinCostNextHops SpfSolver::nextHopsWithMetric(const SpfResult& spf,
                                              const std::vector<std::string>& dsts,
                                              bool perDestination) {
  // the closest destinations (:1062-1077)
  MinCostNextHops out;
  out.shortest = std::numeric_limits<Metric>::max();
  std::vector<std::string> closest;
  for (const auto& d : dsts) {
    auto it = spf.find(d);
    if (it == spf.end()) continue;
    const Metric m = it->second.metric();
    if (m < out.shortest) {
      out.shortest = m;
      closest.clear();
    }
    if (m == out.shortest) closest.push_back(d);
  }
  // their next-hop neighbours with the remaining distance (:1079-1086)
  for (const auto& d : closest)
    for (const auto& nh : spf.at(d).nextHops())
      // getMetricFromAToB(me, nh): nh is a reached neighbour of me
      out.viaNode[{nh, perDestination ? d : std::string()}] = out.shortest - spf.at(nh).metric();
  return out;
}

std::vector<NextHop> SpfSolver::nextHopsThrift(
    const std::string& me, const std::vector<std::string>& dsts, bool perDestination,
    const MinCostNextHops& m, std::optional<int32_t> swapLabel,
    const std::map<std::string, const PrefixEntry*>& entries, const NodeUcmpResult* ucmp) {
  std::set<std::string> dstSet(dsts.begin(), dsts.end());
  const std::vector<std::string> loop =
      perDestination ? std::vector<std::string>(dstSet.begin(), dstSet.end())
                     : std::vector<std::string>{std::string()};
  std::vector<NextHop> out;
  for (const auto& link : ls_.linksFromNode(me)) {
    const std::string& nbr = link->otherNode(me);
    for (const auto& dst : loop) {
      auto it = m.viaNode.find({nbr, dst});
      // overloaded links and non-next-hop neighbours drop out
      if (it == m.viaNode.end() || !link->isUp()) continue;
      // do not reach one destination through another
      if (!dst.empty() && dstSet.count(nbr) && nbr != dst) continue;
      const Metric over = link->metricFrom(me) + it->second;
      if (over != m.shortest) continue;  // a longer parallel link
      NextHop nh;
      nh.ifName = link->ifaceFrom(me);
      nh.neighbor = nbr;
      nh.metric = toThriftMetric(over);
      if (swapLabel) {
        if (dstSet.count(nbr)) {
          nh.op = MplsOp::kPhp;
        } else {
          nh.op = MplsOp::kSwap;
          nh.labels = {*swapLabel};
        }
      }
      if (!dst.empty()) {
        // SR_MPLS towards dst: prepend label, then dst's node label unless
        // dst is the neighbour (:1231-1261); an invalid label drops the hop
        std::vector<int32_t> push;
        const PrefixEntry* e = entries.at(dst);
        if (e->prependLabel) {
          push.push_back(*e->prependLabel);
          if (!isMplsLabelValid(push.back())) continue;
        }
        if (dst != nbr) {
          push.push_back(nodeLabel(dst));
          if (!isMplsLabelValid(push.back())) continue;
        }
        if (!push.empty()) {
          nh.op = MplsOp::kPush;
          nh.labels = std::move(push);
        }
      }
      if (ucmp) {
        auto w = ucmp->nextHopLinks().find(nh.ifName);
        if (w != ucmp->nextHopLinks().end()) nh.weight = (int32_t)w->second.weight;
      }
      out.push_back(std::move(nh));
    }
  }
  sortUnique(out);
  return out;
}

std::vector<NextHop> SpfSolver::ecmpRoute(const std::string& me,
                                          const std::vector<std::string>& announcers) {
  if (std::find(announcers.begin(), announcers.end(), me) != announcers.end())
    return {};  // self-originated: no route
  auto m = nextHopsWithMetric(me, announcers, false);
  if (m.viaNode.empty()) return {};
  return nextHopsThrift(me, announcers, false, m, std::nullopt, {}, nullptr);
}

std::vector<NextHop> SpfSolver::nodeLabelRoute(const std::string& me, const std::string& dst) {
  return nodeLabelRoute(me, dst, ls_.getSpfResult(me));
}

std::vector<NextHop> SpfSolver::nodeLabelRoute(const std::string& me, const std::string& dst,
                                               const SpfResult& mine) {
  if (dst == me) return {};  // POP_AND_LOOKUP, not an SPF product
  auto m = nextHopsWithMetric(mine, {dst}, false);
  if (m.viaNode.empty()) return {};
  return nextHopsThrift(me, {dst}, false, m, nodeLabel(dst), {}, nullptr);
}

std::vector<NextHop> SpfSolver::ksp2Route(const std::string& me,
                                          const std::vector<std::string>& announcers) {
  return ksp2Paths(me, announcers, {});
}

std::vector<NextHop> SpfSolver::ksp2Paths(const std::string& me,
                                          const std::vector<std::string>& announcers,
                                          const std::map<std::string, const PrefixEntry*>& entries) {
  // selectBestPathsKsp2 (SpfSolver.cpp:847-973), one area
  std::vector<Path> paths;
  for (const auto& node : announcers) {
    if (node == me) continue;
    for (const auto& p : ls_.getKthPaths(me, node, 1)) paths.push_back(p);
  }
  const size_t firstPaths = paths.size();
  for (const auto& node : announcers) {
    for (const auto& p : ls_.getKthPaths(me, node, 2)) {
      bool covered = false;
      for (size_t i = 0; i < firstPaths && !covered; ++i)
        covered = LinkState::pathAInPathB(paths[i], p);
      if (!covered) paths.push_back(p);
    }
  }
  std::vector<NextHop> out;
  for (const auto& p : paths) {
    Metric cost = 0;
    std::vector<int32_t> stack;  // built front-first like the reference's list
    std::string at = me;
    bool valid = true;           // a node without a valid label voids the path
    for (const auto& l : p) {
      cost += l->metricFrom(at);
      at = l->otherNode(at);
      const int32_t lbl = nodeLabel(at);
      stack.insert(stack.begin(), lbl);
      valid &= isMplsLabelValid(lbl);
    }
    if (!valid) continue;
    stack.pop_back();  // PHP: the first hop's label
    auto e = entries.find(at);
    if (e != entries.end() && e->second->prependLabel)
      stack.insert(stack.begin(), *e->second->prependLabel);  // bottom of stack
    NextHop nh;
    nh.ifName = p.front()->ifaceFrom(me);
    nh.neighbor = p.front()->otherNode(me);
    nh.metric = toThriftMetric(cost);
    if (!stack.empty()) {
      nh.op = MplsOp::kPush;
      nh.labels = std::move(stack);
    }
    out.push_back(std::move(nh));
  }
  sortUnique(out);
  return out;
}

std::optional<UnicastRoute> SpfSolver::prefixRoute(const std::string& me, const PrefixRoute& pr,
                                                   const RouteOptions& opt) {
  return prefixRoute(me, pr, opt, ls_.getSpfResult(me));
}

std::optional<UnicastRoute> SpfSolver::prefixRoute(const std::string& me, const PrefixRoute& pr,
                                                   const RouteOptions& opt, const SpfResult& mine) {
  // entries of reachable announcers only (:225-253)
  std::map<std::string, const PrefixEntry*> entries;
  for (const auto& e : pr.entries)
    if (mine.count(e.node)) entries.emplace(e.node, &e);
  if (entries.empty()) return std::nullopt;
  bool selfPrepend = true;
  if (auto s = entries.find(me); s != entries.end()) selfPrepend = s->second->prependLabel.has_value();
  // every reachable announcer is a best route; drained (overloaded)
  // announcers drop out unless all are drained (maybeFilterDrainedNodes :709-731)
  std::vector<std::string> best;
  for (const auto& kv : entries)
    if (!ls_.isNodeOverloaded(kv.first)) best.push_back(kv.first);
  if (best.empty())
    for (const auto& kv : entries) best.push_back(kv.first);
  const bool hasMe = std::find(best.begin(), best.end(), me) != best.end();
  if (hasMe && !selfPrepend) return std::nullopt;  // :333-337
  // forwarding type and algorithm: the minimum over the best entries
  // (getPrefixForwardingTypeAndAlgorithm, LsdbUtil.cpp:379-413)
  int fwdType = 1, algo = 3;
  for (const auto& n : best) {
    fwdType = std::min(fwdType, entries.at(n)->fwdType);
    algo = std::min(algo, entries.at(n)->algo);
  }
  UnicastRoute route;
  Metric shortest = std::numeric_limits<Metric>::max();
  if (algo == 1) {
    // KSP2_ED_ECMP needs SR_MPLS (:860-870)
    if (fwdType == 1) route.nextHops = ksp2Paths(me, best, entries);
  } else {
    // selectBestPathsSpf (:772-845)
    const bool perDestination = fwdType == 1;
    std::vector<std::string> filtered = best;
    if (hasMe && perDestination && entries.at(me)->prependLabel)
      filtered.erase(std::find(filtered.begin(), filtered.end(), me));
    const MinCostNextHops m = nextHopsWithMetric(mine, filtered, perDestination);
    shortest = m.shortest;
    if (!m.viaNode.empty()) {
      // getNodeUcmpResult (:1091-1161): weights of the best announcers at the
      // best metric; one without a weight turns UCMP off
      std::optional<NodeUcmpResult> ucmp;
      if (opt.ucmp && (algo == 2 || algo == 3)) {
        std::unordered_map<std::string, int64_t> weights;
        bool ok = true;
        for (const auto& n : best) {
          auto it = mine.find(n);
          if (it == mine.end() || it->second.metric() != m.shortest) continue;
          if (entries.at(n)->weight == 0) {
            ok = false;
            break;
          }
          weights.emplace(n, entries.at(n)->weight);
        }
        if (ok) {
          auto res = ls_.resolveUcmpWeights(mine, weights, (UcmpAlgo)algo);
          auto it = res.find(me);
          if (it != res.end()) ucmp = std::move(it->second);
        }
      }
      if (ucmp) route.weight = ucmp->weight();
      route.nextHops = nextHopsThrift(me, best, perDestination, m, std::nullopt, entries,
                                      ucmp ? &*ucmp : nullptr);
    }
  }
  // addBestPaths (:976-1041): no next hop, no route
  if (route.nextHops.empty()) return std::nullopt;
  route.igpCost = (uint32_t)shortest;
  return route;
}

std::optional<RouteDb> SpfSolver::buildRouteDb(const std::string& me,
                                               const std::vector<PrefixRoute>& prefixes,
                                               const RouteOptions& opt) {
  const auto& dbs = ls_.getAdjacencyDatabases();
  if (!dbs.count(me)) return std::nullopt;
  RouteDb db;
  // The SP prefixes read only the memoised SPF of `me` (and const link
  // state): they are built on host threads. A prefix with a KSP2 entry runs
  // getKthPaths, which fills a memo, so those are built on this thread.
  // `mine` is looked up (and memoised) here, on the calling thread; the
  // host threads below only read it
  const SpfResult& mine = ls_.getSpfResult(me);
  std::vector<std::optional<UnicastRoute>> routes(prefixes.size());
  std::vector<uint32_t> sp, ksp;
  for (uint32_t i = 0; i < prefixes.size(); ++i) {
    bool k = false;
    for (const auto& e : prefixes[i].entries) k |= e.algo == 1;
    (k ? ksp : sp).push_back(i);
  }
  parallelFor((uint32_t)sp.size(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t j = lo; j < hi; ++j) routes[sp[j]] = prefixRoute(me, prefixes[sp[j]], opt, mine);
  }, 256);
  for (const uint32_t i : ksp) routes[i] = prefixRoute(me, prefixes[i], opt);
  for (uint32_t i = 0; i < prefixes.size(); ++i) {
    if (!routes[i]) continue;
    if (!db.unicast.emplace(prefixes[i].prefix, std::move(*routes[i])).second)
      throw std::invalid_argument("duplicate prefix " + prefixes[i].prefix);
  }
  // node-label routes (:501-598): on a label collision the smallest node name
  // keeps it (the reference's `iter->second.first < nodeName` rule, in any
  // order); an unreachable node leaves no route and takes nothing over
  if (opt.nodeSegmentLabels) {
    std::vector<std::string> names;
    names.reserve(dbs.size());
    for (const auto& kv : dbs) names.push_back(kv.first);
    std::sort(names.begin(), names.end());
    // candidate routes of every labelled node, on host threads
    std::vector<std::vector<NextHop>> cand(names.size());
    parallelFor((uint32_t)names.size(), [&](uint32_t lo, uint32_t hi) {
      for (uint32_t j = lo; j < hi; ++j) {
        const int32_t top = dbs.at(names[j]).nodeLabel;
        if (top != 0 && isMplsLabelValid(top) && names[j] != me)
          cand[j] = nodeLabelRoute(me, names[j], mine);
      }
    }, 256);
    std::map<int32_t, std::pair<std::string, std::vector<NextHop>>> labelToNode;
    for (size_t j = 0; j < names.size(); ++j) {
      const std::string& node = names[j];
      const int32_t top = dbs.at(node).nodeLabel;
      if (top == 0 || !isMplsLabelValid(top)) continue;
      auto it = labelToNode.find(top);
      if (it != labelToNode.end() && it->second.first < node) continue;
      if (node == me) {
        NextHop pop;
        pop.op = MplsOp::kPopAndLookup;
        labelToNode[top] = {me, {pop}};
        continue;
      }
      if (cand[j].empty()) continue;
      labelToNode[top] = {node, std::move(cand[j])};
    }
    for (auto& kv : labelToNode) db.mpls.emplace(kv.first, std::move(kv.second.second));
  }
  // adjacency-label routes (:603-631): PHP over each of our links (up or not)
  if (opt.adjacencyLabels) {
    for (const auto& link : ls_.linksFromNode(me)) {
      const int32_t top = link->adjLabelFrom(me);
      if (top == 0 || !isMplsLabelValid(top)) continue;
      NextHop nh;
      nh.ifName = link->ifaceFrom(me);
      nh.neighbor = link->otherNode(me);
      nh.metric = toThriftMetric(link->metricFrom(me));
      nh.op = MplsOp::kPhp;
      if (!db.mpls.emplace(top, std::vector<NextHop>{nh}).second)
        throw std::invalid_argument("duplicate MPLS label " + std::to_string(top));
    }
  }
  return db;
}

std::vector<std::optional<RouteDb>> SpfSolver::buildRouteDbs(
    const std::vector<std::string>& mes, const std::vector<PrefixRoute>& prefixes,
    const RouteOptions& opt) {
  std::vector<std::string> roots;
  for (const auto& me : mes)
    if (ls_.getAdjacencyDatabases().count(me)) roots.push_back(me);
  std::vector<std::optional<RouteDb>> out;
  out.reserve(mes.size());
  const size_t V = ls_.numNodes();
  if (roots.size() < LinkState::kSweepMinRoots || 2 * roots.size() < V) {
    ls_.prefetchSpf(roots, true);
    for (const auto& me : mes) out.push_back(buildRouteDb(me, prefixes, opt));
    return out;
  }
  // Most of the nodes (Decision::getDecisionRouteDb for every node,
  // Decision.cpp:309): one all-sources sweep on the devices, then chunks of
  // nodes whose SpfResults are rebuilt from the resident rows, used and
  // dropped again (results memoised before the call stay).
  ls_.prefetchAllSources(true);
  constexpr size_t kChunk = 512;
  for (size_t c0 = 0; c0 < mes.size(); c0 += kChunk) {
    const size_t c1 = std::min(mes.size(), c0 + kChunk);
    std::vector<std::string> fresh;
    for (size_t i = c0; i < c1; ++i)
      if (ls_.getAdjacencyDatabases().count(mes[i]) && !ls_.isMemoised(mes[i], true))
        fresh.push_back(mes[i]);
    ls_.prefetchSpf(fresh, true);
    for (size_t i = c0; i < c1; ++i) out.push_back(buildRouteDb(mes[i], prefixes, opt));
    ls_.evictSpf(fresh, true);
  }
  return out;
}

}  // namespace odl
