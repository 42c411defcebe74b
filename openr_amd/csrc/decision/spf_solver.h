// spf_solver.h — route-building consumers of the SPF results (SURVEY.md §8
// rows a8-a10), host C++ over odl::LinkState (whose SPF runs on the MI355X
// engine). Restates, for a prefix announced by a set of nodes in one area:
//   getNextHopsWithMetric   openr/decision/SpfSolver.cpp:1043-1089
//   getNextHopsThrift       openr/decision/SpfSolver.cpp:1163-1285
//   selectBestPathsSpf      openr/decision/SpfSolver.cpp:772-845 (UCMP too)
//   selectBestPathsKsp2     openr/decision/SpfSolver.cpp:847-973
//   createRouteForPrefix / buildRouteDb  SpfSolver.cpp:197-646
// Several areas (one LinkState each): createRouteForPrefix's per-area loop
// (:229-250, :360-442: the shortest areas' next hops merged, UCMP weights
// summed, KSP2 next hops added), the node-label loop over every area's
// databases (:490-598) and the adjacency labels of every area (:603-631);
// addBestPaths' minNexthop threshold (:976-1000 with
// getMinNextHopThreshold :694-710). Best-route selection: with
// enableBestRouteSelection the announcers are picked by their prefix metrics
// (selectRoutes(SHORTEST_DISTANCE) + selectBestNodeArea, LsdbUtil.cpp:758-880;
// SpfSolver.cpp:658-663), otherwise every reachable announcer is best
// (:666-672) and a prefix announced as BGP together with another type, or by
// a BGP entry without a metric vector, gets no route (:272-300). RIB policy
// beyond that (BGP metric-vector comparison, SR policies, static routes) is
// outside the SPF path and not restated here.
#pragma once

#include <cstdint>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "link_state.h"

namespace odl {

enum class MplsOp : int { kNone = 0, kPhp = 1, kSwap = 2, kPush = 3, kPopAndLookup = 4 };

// thrift::NextHopThrift (openr/if/Network.thrift:54-70), SPF-relevant fields.
// `metric` is the thrift i32: createNextHop(..., int32_t metric, ...)
// (openr/common/LsdbUtil.cpp:658-675) narrows the u64 LinkState metric, which
// keeps its low 32 bits (two's complement), as toThriftMetric does.
struct NextHop {
  std::string ifName;
  std::string neighbor;
  int32_t metric = 0;
  MplsOp op = MplsOp::kNone;
  std::vector<int32_t> labels;  // SWAP: {label}; PUSH: stack, bottom first
  int32_t weight = 0;           // UCMP next-hop weight, 0 = ECMP
  std::string area;             // the area whose link the next hop leaves on
  bool operator<(const NextHop& o) const;
  bool operator==(const NextHop& o) const;
};
inline int32_t toThriftMetric(Metric m) { return (int32_t)(uint32_t)m; }

// isMplsLabelValid (openr/common/MplsUtil.h:19-22): 20-bit, non-zero
inline bool isMplsLabelValid(int32_t l) { return (l & 0xfff00000) == 0 && l != 0; }

// thrift::PrefixEntry (openr/if/Types.thrift), the fields the route build
// reads: forwarding type (0 IP, 1 SR_MPLS) and algorithm (0 SP_ECMP,
// 1 KSP2_ED_ECMP, 2 SP_UCMP_ADJ_WEIGHT_PROPAGATION, 3
// SP_UCMP_PREFIX_WEIGHT_PROPAGATION; OpenrConfig.thrift:18-50), UCMP weight
// (0 = unset), prepend label, the prefix metrics best-route selection reads
// (PrefixMetrics, Types.thrift:328-370: path_preference and
// source_preference prefer-higher, distance prefer-lower; IDL defaults 0) and
// the origin type as far as selectBestRoutes reads it (BGP or not, and
// whether a BGP entry carries a metric vector).
struct PrefixEntry {
  std::string node;
  int fwdType = 0;
  int algo = 0;
  int64_t weight = 0;
  std::optional<int32_t> prependLabel;
  std::string area;                  // "" = the solver's first area
  std::optional<int64_t> minNexthop;  // PrefixEntry.minNexthop (Types.thrift)
  int32_t pathPreference = 0, sourcePreference = 0, distance = 0;
  bool bgp = false;   // PrefixType::BGP
  bool hasMv = false; // a BGP entry's metric vector (mv) is set
};
struct PrefixRoute {
  std::string prefix;
  std::vector<PrefixEntry> entries;
};

// RibUnicastEntry (RibEntry.h:60-77): next hops, igpCost (unsigned int) and
// the UCMP weight that replaces bestPrefixEntry.weight.
struct UnicastRoute {
  std::vector<NextHop> nextHops;
  uint32_t igpCost = 0;
  std::optional<int64_t> weight;
  // RouteSelectionResult (bestRoutesCache_, SpfSolver.cpp:315): every
  // selected announcer and the best one (whose entry the RibUnicastEntry
  // carries, :1032-1041)
  std::set<std::pair<std::string, std::string>> selected;
  std::pair<std::string, std::string> best;
};

// DecisionRouteDb (SpfSolver.h:80-98): routes by prefix and by MPLS label,
// next hops sorted
struct RouteDb {
  std::map<std::string, UnicastRoute> unicast;
  std::map<int32_t, std::vector<NextHop>> mpls;
};

// SpfSolver constructor switches (SpfSolver.h:108-118) that shape the build
struct RouteOptions {
  bool nodeSegmentLabels = true;
  bool adjacencyLabels = true;
  bool ucmp = false;
  bool bestRouteSelection = false;  // enableBestRouteSelection (SpfSolver.h:113)
};

struct MinCostNextHops {
  Metric shortest = 0;
  // (next-hop node, destination or "" unless perDestination) -> distance
  // from the next hop to the closest announcer
  std::map<std::pair<std::string, std::string>, Metric> viaNode;
};

class SpfSolver {
 public:
  explicit SpfSolver(LinkState& ls) : ls_(ls), areas_{{ls.area(), &ls}} {}
  // one LinkState per area (LinkState::area() names it); ls_ = the first by
  // name (the single-area helpers below use it)
  explicit SpfSolver(const std::vector<LinkState*>& areas);

  // getNextHopsWithMetric (SpfSolver.cpp:1043-1089)
  MinCostNextHops nextHopsWithMetric(const std::string& me, const std::vector<std::string>& dsts,
                                     bool perDestination);
  // the same over `me`'s SPF result, read-only (safe on the route build's
  // host threads: no memo lookup, no insertion)
  static MinCostNextHops nextHopsWithMetric(const SpfResult& mine,
                                            const std::vector<std::string>& dsts,
                                            bool perDestination);
  // SP_ECMP unicast route from single-node IP announcers (empty: no route)
  std::vector<NextHop> ecmpRoute(const std::string& me, const std::vector<std::string>& announcers);
  // MPLS node-label route towards `dst` with its node label (PHP / SWAP)
  std::vector<NextHop> nodeLabelRoute(const std::string& me, const std::string& dst);
  std::vector<NextHop> nodeLabelRoute(const std::string& me, const std::string& dst,
                                      const SpfResult& mine);
  // KSP2_ED_ECMP route (SR-MPLS label stacks) over `announcers` (entries
  // without prepend labels)
  std::vector<NextHop> ksp2Route(const std::string& me, const std::vector<std::string>& announcers);
  // createRouteForPrefix (SpfSolver.cpp:197-458), every area, non-BGP
  std::optional<UnicastRoute> prefixRoute(const std::string& me, const PrefixRoute& pr,
                                          const RouteOptions& opt);
  // over `me`'s SPF result in each area (`mines`, areas_ order): what
  // buildRouteDb runs on host threads
  std::optional<UnicastRoute> prefixRoute(const std::string& me, const PrefixRoute& pr,
                                          const RouteOptions& opt,
                                          const std::vector<const SpfResult*>& mines);
  // SpfSolver::buildRouteDb (SpfSolver.cpp:460-646), one area: unicast routes
  // of `prefixes`, MPLS node-label routes of every node (POP_AND_LOOKUP for
  // our own label, PHP / SWAP towards the others, :501-598) and
  // adjacency-label routes (PHP, :603-631). nullopt when `me` is not in the
  // link state (:465-471). A duplicate MPLS label throws (the reference
  // CHECK-fails, SpfSolver.h:92-97).
  std::optional<RouteDb> buildRouteDb(const std::string& me, const std::vector<PrefixRoute>& prefixes,
                                      const RouteOptions& opt = RouteOptions{});
  // buildRouteDb for many nodes: one batched engine launch computes every
  // SPF result the builds read (each `me` and, for node-label routes, the
  // same roots), then the per-node builds run on the host.
  std::vector<std::optional<RouteDb>> buildRouteDbs(const std::vector<std::string>& mes,
                                                    const std::vector<PrefixRoute>& prefixes,
                                                    const RouteOptions& opt = RouteOptions{});

 private:
  using NodeArea = std::pair<std::string, std::string>;
  using Entries = std::map<NodeArea, const PrefixEntry*>;
  // getNextHopsThrift (SpfSolver.cpp:1163-1285) over area `ai`'s links;
  // dsts = (node, area) pairs, perDestination reads those of this area
  std::vector<NextHop> nextHopsThrift(size_t ai, const std::string& me,
                                      const std::vector<NodeArea>& dsts, bool perDestination,
                                      const MinCostNextHops& m, std::optional<int32_t> swapLabel,
                                      const Entries& entries, const NodeUcmpResult* ucmp);
  // selectBestPathsKsp2 (SpfSolver.cpp:847-973) in area `ai`
  std::vector<NextHop> ksp2Paths(size_t ai, const std::string& me, const std::set<NodeArea>& best,
                                 const Entries& entries);
  static int32_t nodeLabel(const LinkState& ls, const std::string& node);
  static std::set<NodeArea> selectShortestDistanceRoutes(const Entries& entries);
  size_t lsIndex() const {
    for (size_t i = 0; i < areas_.size(); ++i)
      if (areas_[i].second == &ls_) return i;
    return 0;
  }
  int32_t nodeLabel(const std::string& node) const { return nodeLabel(ls_, node); }
  LinkState& ls_;
  std::vector<std::pair<std::string, LinkState*>> areas_;  // by area name
};

}  // namespace odl
