// spf_solver.cpp — see spf_solver.h.
#include "spf_solver.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <set>
#include <stdexcept>
#include <tuple>

namespace odl {

bool NextHop::operator<(const NextHop& o) const {
  return std::tie(ifName, neighbor, metric, op, labels, weight, area) <
         std::tie(o.ifName, o.neighbor, o.metric, o.op, o.labels, o.weight, o.area);
}
bool NextHop::operator==(const NextHop& o) const {
  return std::tie(ifName, neighbor, metric, op, labels, weight, area) ==
         std::tie(o.ifName, o.neighbor, o.metric, o.op, o.labels, o.weight, o.area);
}

namespace {
LinkState& firstArea(const std::vector<LinkState*>& areas) {
  if (areas.empty()) throw std::invalid_argument("SpfSolver: no area");
  return **std::min_element(areas.begin(), areas.end(),
                            [](const LinkState* a, const LinkState* b) { return a->area() < b->area(); });
}
}  // namespace

SpfSolver::SpfSolver(const std::vector<LinkState*>& areas) : ls_(firstArea(areas)) {
  for (LinkState* a : areas) areas_.emplace_back(a->area(), a);
  std::sort(areas_.begin(), areas_.end());
  for (size_t i = 1; i < areas_.size(); ++i)
    if (areas_[i].first == areas_[i - 1].first)
      throw std::invalid_argument("SpfSolver: area " + areas_[i].first + " twice");
}

namespace {
void sortUnique(std::vector<NextHop>& v) {
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
}
}  // namespace

int32_t SpfSolver::nodeLabel(const LinkState& ls, const std::string& node) {
  const auto& dbs = ls.getAdjacencyDatabases();
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
    size_t ai, const std::string& me, const std::vector<NodeArea>& dsts, bool perDestination,
    const MinCostNextHops& m, std::optional<int32_t> swapLabel, const Entries& entries,
    const NodeUcmpResult* ucmp) {
  const std::string& area = areas_[ai].first;
  const LinkState& ls = *areas_[ai].second;
  std::set<std::string> dstSet;  // every destination node, any area
  for (const auto& d : dsts) dstSet.insert(d.first);
  // perDestination: the (node, area) pairs of this area (:1189-1194)
  std::vector<std::string> loop;
  if (perDestination) {
    std::set<std::string> mine;
    for (const auto& d : dsts)
      if (d.second.empty() || d.second == area) mine.insert(d.first);
    loop.assign(mine.begin(), mine.end());
  } else {
    loop.push_back(std::string());
  }
  std::vector<NextHop> out;
  for (const auto& link : ls.linksFromNode(me)) {
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
      nh.area = area;
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
        const PrefixEntry* e = entries.at({dst, area});
        if (e->prependLabel) {
          push.push_back(*e->prependLabel);
          if (!isMplsLabelValid(push.back())) continue;
        }
        if (dst != nbr) {
          push.push_back(nodeLabel(ls, dst));
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
  std::vector<NodeArea> d;
  for (const auto& n : announcers) d.emplace_back(n, ls_.area());
  return nextHopsThrift(lsIndex(), me, d, false, m, std::nullopt, {}, nullptr);
}

std::vector<NextHop> SpfSolver::nodeLabelRoute(const std::string& me, const std::string& dst) {
  return nodeLabelRoute(me, dst, ls_.getSpfResult(me));
}

std::vector<NextHop> SpfSolver::nodeLabelRoute(const std::string& me, const std::string& dst,
                                               const SpfResult& mine) {
  if (dst == me) return {};  // POP_AND_LOOKUP, not an SPF product
  auto m = nextHopsWithMetric(mine, {dst}, false);
  if (m.viaNode.empty()) return {};
  return nextHopsThrift(lsIndex(), me, {{dst, ls_.area()}}, false, m, nodeLabel(dst), {}, nullptr);
}

std::vector<NextHop> SpfSolver::ksp2Route(const std::string& me,
                                          const std::vector<std::string>& announcers) {
  std::set<NodeArea> best;
  for (const auto& n : announcers) best.emplace(n, ls_.area());
  return ksp2Paths(lsIndex(), me, best, {});
}

std::vector<NextHop> SpfSolver::ksp2Paths(size_t ai, const std::string& me,
                                          const std::set<NodeArea>& best, const Entries& entries) {
  // selectBestPathsKsp2 (SpfSolver.cpp:847-973) in area ai: k = 1 paths to
  // every best node (any area's entry, but not ourselves in this area),
  // k = 2 paths to the best nodes of this area not covering a k = 1 path
  const std::string& area = areas_[ai].first;
  LinkState& ls = *areas_[ai].second;
  std::vector<Path> paths;
  for (const auto& [node, a] : best) {
    if (node == me && a == area) continue;
    for (const auto& p : ls.getKthPaths(me, node, 1)) paths.push_back(p);
  }
  const size_t firstPaths = paths.size();
  for (const auto& [node, a] : best) {
    if (a != area) continue;
    for (const auto& p : ls.getKthPaths(me, node, 2)) {
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
      const int32_t lbl = nodeLabel(ls, at);
      stack.insert(stack.begin(), lbl);
      valid &= isMplsLabelValid(lbl);
    }
    if (!valid) continue;
    stack.pop_back();  // PHP: the first hop's label
    // the last node's entry in this area (the reference's
    // prefixEntries.at({lastNode, area}); absent: no prepend label)
    auto e = entries.find({at, area});
    if (e != entries.end() && e->second->prependLabel)
      stack.insert(stack.begin(), *e->second->prependLabel);  // bottom of stack
    NextHop nh;
    nh.ifName = p.front()->ifaceFrom(me);
    nh.neighbor = p.front()->otherNode(me);
    nh.metric = toThriftMetric(cost);
    nh.area = area;
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
  const bool tm = getenv("ODL_ROUTE_TIMING") != nullptr;
  auto tl = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!tm) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "route_build %s %.2f ms\n", what, std::chrono::duration<double, std::milli>(t - tl).count());
    tl = t;
  };
  std::vector<const SpfResult*> mines;
  for (auto& a : areas_) mines.push_back(&a.second->getSpfResult(me));
  lap("spf results");
  return prefixRoute(me, pr, opt, mines);
}

std::optional<UnicastRoute> SpfSolver::prefixRoute(const std::string& me, const PrefixRoute& pr,
                                                   const RouteOptions& opt,
                                                   const std::vector<const SpfResult*>& mines) {
  auto areaIx = [&](const std::string& a) -> size_t {
    for (size_t i = 0; i < areas_.size(); ++i)
      if (areas_[i].first == a) return i;
    // the reference reads areaLinkStates.at(area) (maybeFilterDrainedNodes)
    throw std::invalid_argument("prefix entry of unknown area " + a);
  };
  // (node, area) entries of reachable announcers only: an entry is dropped
  // when its node is not reached in its own area (:225-253)
  Entries entries;
  for (const auto& e : pr.entries) {
    const std::string& a = e.area.empty() ? areas_[0].first : e.area;
    if (mines[areaIx(a)]->count(e.node)) entries.emplace(NodeArea{e.node, a}, &e);
  }
  if (entries.empty()) return std::nullopt;
  bool selfPrepend = true, hasBgp = false, hasNonBgp = false, missingMv = false;
  for (const auto& [na, e] : entries) {
    if (na.first == me) selfPrepend &= e->prependLabel.has_value();
    hasBgp |= e->bgp;
    hasNonBgp |= !e->bgp;
    missingMv |= e->bgp && !e->hasMv;
  }
  // selectBestRoutes (:650-674)
  std::set<NodeArea> all;
  NodeArea bestNa;
  if (opt.bestRouteSelection) {
    all = selectShortestDistanceRoutes(entries);
    bestNa = *all.begin();  // selectBestNodeArea (LsdbUtil.cpp:758-769): me if selected
    for (const auto& na : all)
      if (na.first == me) {
        bestNa = na;
        break;
      }
  } else {
    // mixed BGP / other types, or a BGP entry without a metric vector: the
    // prefix is skipped (decision.skipped_unicast_route, :282-300)
    if (hasBgp && (hasNonBgp || missingMv)) return std::nullopt;
    if (hasBgp)
      throw std::invalid_argument("prefix " + pr.prefix + ": BGP metric-vector best-path "
                                  "selection (runBestPathSelectionBgp) is not restated");
    for (const auto& kv : entries) all.insert(kv.first);  // every announcer (:666-672)
    bestNa = *all.begin();
  }
  // maybeFilterDrainedNodes (:709-731): drained announcers drop out unless
  // all are drained; the reference's bestNodeArea update there compares the
  // filtered copy with itself (:723-727), so the best entry stays as selected
  std::set<NodeArea> best;
  for (const auto& na : all)
    if (!areas_[areaIx(na.second)].second->isNodeOverloaded(na.first)) best.insert(na);
  if (best.empty()) best = all;
  auto hasNode = [&](const std::string& n) {
    for (const auto& na : best)
      if (na.first == n) return true;
    return false;
  };
  const bool hasMe = hasNode(me);
  if (hasMe && !selfPrepend) return std::nullopt;  // :333-337
  // per area (default route computation rules, :1288-1317): forwarding type
  // and algorithm = the minimum over the area's best entries
  // (getPrefixForwardingTypeAndAlgorithm, LsdbUtil.cpp:379-413)
  std::set<NextHop> total, ksp;
  std::optional<int64_t> ucmpWeight;
  Metric shortest = std::numeric_limits<Metric>::max();
  for (size_t ai = 0; ai < areas_.size(); ++ai) {
    const std::string& area = areas_[ai].first;
    const SpfResult& mine = *mines[ai];
    bool any = false;
    int fwdType = 1, algo = 3;
    for (const auto& na : best) {
      if (na.second != area) continue;
      const PrefixEntry* e = entries.at(na);
      fwdType = any ? std::min(fwdType, e->fwdType) : e->fwdType;
      algo = any ? std::min(algo, e->algo) : e->algo;
      any = true;
    }
    if (!any) continue;
    if (algo == 1) {
      // KSP2_ED_ECMP needs SR_MPLS (:860-870)
      if (fwdType == 1) {
        auto nhs = ksp2Paths(ai, me, best, entries);
        ksp.insert(nhs.begin(), nhs.end());
      }
    } else {
      // selectBestPathsSpf (:772-845): destinations = the best nodes of every
      // area, looked up in this area's SPF
      const bool perDestination = fwdType == 1;
      std::set<NodeArea> filtered = best;
      if (hasMe && perDestination)
        for (const auto& [na, e] : entries)
          if (na.first == me && e->prependLabel) {
            filtered.erase(na);
            break;
          }
      std::vector<std::string> dsts;
      for (const auto& na : filtered) dsts.push_back(na.first);
      const MinCostNextHops m = nextHopsWithMetric(mine, dsts, perDestination);
      std::vector<NextHop> nhs;
      std::optional<int64_t> weight;
      if (!m.viaNode.empty()) {
        // getNodeUcmpResult (:1091-1161): weights of this area's best
        // announcers at the best metric; one without a weight turns UCMP off
        std::optional<NodeUcmpResult> ucmp;
        if (opt.ucmp && (algo == 2 || algo == 3)) {
          std::unordered_map<std::string, int64_t> weights;
          bool ok = true;
          for (const auto& na : best) {
            if (na.second != area) continue;
            auto it = mine.find(na.first);
            if (it == mine.end() || it->second.metric() != m.shortest) continue;
            if (entries.at(na)->weight == 0) {
              ok = false;
              break;
            }
            weights.emplace(na.first, entries.at(na)->weight);
          }
          if (ok) {
            auto res = areas_[ai].second->resolveUcmpWeights(mine, weights, (UcmpAlgo)algo);
            auto it = res.find(me);
            if (it != res.end()) ucmp = std::move(it->second);
          }
        }
        if (ucmp) weight = ucmp->weight();
        std::vector<NodeArea> bestv(best.begin(), best.end());
        nhs = nextHopsThrift(ai, me, bestv, perDestination, m, std::nullopt, entries,
                             ucmp ? &*ucmp : nullptr);
      }
      // only the areas at the shortest IGP metric contribute (:392-407)
      if (shortest >= m.shortest) {
        if (shortest > m.shortest) {
          shortest = m.shortest;
          total.clear();
          ucmpWeight.reset();
        }
        total.insert(nhs.begin(), nhs.end());
        if (!ucmpWeight) ucmpWeight = weight;
        else if (weight) *ucmpWeight += *weight;
      }
    }
    total.insert(ksp.begin(), ksp.end());  // KSP2 next hops merged (:436-437)
  }
  // addBestPaths (:976-1041): no next hop, no route; minNexthop = the largest
  // over the best entries (getMinNextHopThreshold :694-710)
  if (total.empty()) return std::nullopt;
  std::optional<int64_t> minNh;
  for (const auto& na : best) {
    const auto& mn = entries.at(na)->minNexthop;
    if (mn && (!minNh || *mn > *minNh)) minNh = mn;
  }
  if (minNh && *minNh > (int64_t)total.size()) return std::nullopt;
  UnicastRoute route;
  route.nextHops.assign(total.begin(), total.end());
  route.igpCost = (uint32_t)shortest;
  route.weight = ucmpWeight;
  route.selected = best;
  route.best = bestNa;
  return route;
}

// selectRoutes(prefixEntries, SHORTEST_DISTANCE) (LsdbUtil.cpp:837-880 +
// selectShortestDistance :772-793): the entries with the highest
// (path_preference, source_preference), then the smallest distance among them
std::set<SpfSolver::NodeArea> SpfSolver::selectShortestDistanceRoutes(const Entries& entries) {
  std::pair<int32_t, int32_t> top{std::numeric_limits<int32_t>::min(),
                                  std::numeric_limits<int32_t>::min()};
  std::set<NodeArea> tied;
  for (const auto& [na, e] : entries) {
    const std::pair<int32_t, int32_t> t{e->pathPreference, e->sourcePreference};
    if (t < top) continue;
    if (t > top) {
      top = t;
      tied.clear();
    }
    tied.insert(na);
  }
  std::set<NodeArea> out;
  int32_t shortest = std::numeric_limits<int32_t>::max();
  for (const auto& na : tied) {
    const int32_t d = entries.at(na)->distance;
    if (d > shortest) continue;
    if (d < shortest) {
      shortest = d;
      out.clear();
    }
    out.insert(na);
  }
  return out;
}

std::optional<RouteDb> SpfSolver::buildRouteDb(const std::string& me,
                                               const std::vector<PrefixRoute>& prefixes,
                                               const RouteOptions& opt) {
  // decision.route_build_ms (SpfSolver.cpp:460-462,640-644), on this
  // solver's own LinkState
  struct Timer {
    LinkState& ls;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    bool on = false;
    ~Timer() {
      if (on)
        ls.addRouteBuild(
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
  } timer{ls_};
  bool exists = false;  // :463-471: `me` in some area's link state
  for (const auto& a : areas_) exists |= a.second->getAdjacencyDatabases().count(me) > 0;
  if (!exists) return std::nullopt;
  timer.on = true;
  RouteDb db;
  // The SP prefixes read only the memoised SPF of `me` in each area (and
  // const link state): they are built on host threads. A prefix with a KSP2
  // entry runs getKthPaths, which fills a memo, so those are built on this
  // thread. The results are looked up (and memoised) here, on the calling
  // thread; the host threads below only read them
  const bool tm = getenv("ODL_ROUTE_TIMING") != nullptr;
  auto tl = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!tm) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "route_build %s %.2f ms\n", what, std::chrono::duration<double, std::milli>(t - tl).count());
    tl = t;
  };
  std::vector<const SpfResult*> mines;
  for (auto& a : areas_) mines.push_back(&a.second->getSpfResult(me));
  lap("spf results");
  std::vector<std::optional<UnicastRoute>> routes(prefixes.size());
  std::vector<uint32_t> sp, ksp;
  for (uint32_t i = 0; i < prefixes.size(); ++i) {
    bool k = false;
    for (const auto& e : prefixes[i].entries) k |= e.algo == 1;
    (k ? ksp : sp).push_back(i);
  }
  parallelFor((uint32_t)sp.size(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t j = lo; j < hi; ++j) routes[sp[j]] = prefixRoute(me, prefixes[sp[j]], opt, mines);
  }, 256);
  for (const uint32_t i : ksp) routes[i] = prefixRoute(me, prefixes[i], opt, mines);
  lap("prefix routes");
  // into the ordered map in key order: each insert at the end (a hint), not
  // a tree search per prefix
  std::vector<uint32_t> byKey;
  byKey.reserve(prefixes.size());
  for (uint32_t i = 0; i < prefixes.size(); ++i)
    if (routes[i]) byKey.push_back(i);
  bool ascending = true;
  for (size_t j = 1; j < byKey.size() && ascending; ++j)
    ascending = prefixes[byKey[j - 1]].prefix < prefixes[byKey[j]].prefix;
  if (!ascending)
    std::stable_sort(byKey.begin(), byKey.end(), [&](uint32_t a, uint32_t b) {
      return prefixes[a].prefix < prefixes[b].prefix;
    });
  for (size_t j = 0; j < byKey.size(); ++j) {
    const uint32_t i = byKey[j];
    if (j && prefixes[byKey[j - 1]].prefix == prefixes[i].prefix)
      throw std::invalid_argument("duplicate prefix " + prefixes[i].prefix);
    db.unicast.emplace_hint(db.unicast.end(), prefixes[i].prefix, std::move(*routes[i]));
  }
  lap("unicast map");
  // node-label routes (:501-598), every area's databases in area order: on a
  // label collision the smallest node name keeps it (the reference's
  // `iter->second.first < nodeName` rule, in any order; the same node in two
  // areas: the later area); an unreachable node leaves no route and takes
  // nothing over
  if (opt.nodeSegmentLabels) {
    std::map<int32_t, std::pair<std::string, std::vector<NextHop>>> labelToNode;
    for (size_t ai = 0; ai < areas_.size(); ++ai) {
      const LinkState& ls = *areas_[ai].second;
      const auto& dbs = ls.getAdjacencyDatabases();
      std::vector<std::string> names;
      names.reserve(dbs.size());
      for (const auto& kv : dbs) names.push_back(kv.first);
      parallelSort(names);
      std::vector<int32_t> tops(names.size());
      parallelFor((uint32_t)names.size(), [&](uint32_t lo, uint32_t hi) {
        for (uint32_t j = lo; j < hi; ++j) tops[j] = dbs.at(names[j]).nodeLabel;
      }, 1024);
      lap("labels: names");
      // candidate routes of every labelled node, on host threads
      std::vector<std::vector<NextHop>> cand(names.size());
      parallelFor((uint32_t)names.size(), [&](uint32_t lo, uint32_t hi) {
        for (uint32_t j = lo; j < hi; ++j) {
          const int32_t top = tops[j];
          if (top == 0 || !isMplsLabelValid(top) || names[j] == me) continue;
          auto m = nextHopsWithMetric(*mines[ai], {names[j]}, false);
          if (!m.viaNode.empty())
            cand[j] = nextHopsThrift(ai, me, {{names[j], areas_[ai].first}}, false, m, top, {}, nullptr);
        }
      }, 256);
      lap("labels: candidates");
      // the area's labelled nodes that can take their label (a route, or me)
      // by (label, name): the smallest name of each label first
      std::vector<std::pair<int32_t, uint32_t>> lab;
      lab.reserve(names.size());
      for (size_t j = 0; j < names.size(); ++j) {
        const int32_t top = tops[j];
        if (top == 0 || !isMplsLabelValid(top)) continue;
        if (names[j] != me && cand[j].empty()) continue;  // unreachable: takes nothing over
        lab.emplace_back(top, (uint32_t)j);
      }
      std::sort(lab.begin(), lab.end());
      for (size_t q = 0; q < lab.size(); ++q) {
        if (q && lab[q - 1].first == lab[q].first) continue;  // a larger name of this label
        const int32_t top = lab[q].first;
        const std::string& node = names[lab[q].second];
        auto it = labelToNode.lower_bound(top);
        const bool have = it != labelToNode.end() && it->first == top;
        // an earlier area's holder keeps it when its name is smaller (the same
        // node in two areas: the later area)
        if (have && it->second.first < node) continue;
        std::vector<NextHop> nhs;
        if (node == me) {
          NextHop pop;
          pop.op = MplsOp::kPopAndLookup;
          pop.area = areas_[ai].first;
          nhs.push_back(std::move(pop));
        } else {
          nhs = std::move(cand[lab[q].second]);
        }
        if (areas_.size() == 1) {  // one area: no holder to compare with later
          db.mpls.emplace_hint(db.mpls.end(), top, std::move(nhs));
          continue;
        }
        if (have) it->second = {node, std::move(nhs)};
        else labelToNode.emplace_hint(it, top, std::make_pair(node, std::move(nhs)));
      }
    }
    lap("labels: collisions");
    for (auto& kv : labelToNode) db.mpls.emplace_hint(db.mpls.end(), kv.first, std::move(kv.second.second));
  }
  lap("node labels");
  // adjacency-label routes (:603-631): PHP over each of our links (up or
  // not), every area
  if (opt.adjacencyLabels) {
    for (const auto& [area, ls] : areas_) {
      for (const auto& link : ls->linksFromNode(me)) {
        const int32_t top = link->adjLabelFrom(me);
        if (top == 0 || !isMplsLabelValid(top)) continue;
        NextHop nh;
        nh.ifName = link->ifaceFrom(me);
        nh.neighbor = link->otherNode(me);
        nh.metric = toThriftMetric(link->metricFrom(me));
        nh.op = MplsOp::kPhp;
        nh.area = area;
        if (!db.mpls.emplace(top, std::vector<NextHop>{nh}).second)
          throw std::invalid_argument("duplicate MPLS label " + std::to_string(top));
      }
    }
  }
  return db;
}

std::vector<std::optional<RouteDb>> SpfSolver::buildRouteDbs(
    const std::vector<std::string>& mes, const std::vector<PrefixRoute>& prefixes,
    const RouteOptions& opt) {
  std::vector<std::optional<RouteDb>> out;
  out.reserve(mes.size());
  if (areas_.size() > 1) {  // one batched launch per area, then the builds
    for (auto& a : areas_) {
      std::vector<std::string> roots;
      for (const auto& me : mes)
        if (a.second->getAdjacencyDatabases().count(me)) roots.push_back(me);
      a.second->prefetchSpf(roots, true);
    }
    for (const auto& me : mes) out.push_back(buildRouteDb(me, prefixes, opt));
    return out;
  }
  std::vector<std::string> roots;
  for (const auto& me : mes)
    if (ls_.getAdjacencyDatabases().count(me)) roots.push_back(me);
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
