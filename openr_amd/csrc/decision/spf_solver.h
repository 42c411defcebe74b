// spf_solver.h — route-building consumers of the SPF results (SURVEY.md §8
// rows a8-a10), host C++ over odl::LinkState (whose SPF runs on the MI355X
// engine). Restates, for a prefix announced by a set of nodes in one area:
//   getNextHopsWithMetric   openr/decision/SpfSolver.cpp:1043-1089
//   getNextHopsThrift       openr/decision/SpfSolver.cpp:1163-1285
//                           (perDestination = false: SP_ECMP unicast and
//                            MPLS node-label routes)
//   selectBestPathsKsp2     openr/decision/SpfSolver.cpp:847-973
// Prefix-state policy (RIB selection, BGP metrics, minNexthop, UCMP weights)
// is outside the SPF path and not restated here.
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

#include "link_state.h"

namespace odl {

enum class MplsOp : int { kNone = 0, kPhp = 1, kSwap = 2, kPush = 3 };

// thrift::NextHopThrift (openr/if/Network.thrift:54-70), SPF-relevant fields.
// `metric` is kept 64-bit; the reference stores it as i32.
struct NextHop {
  std::string ifName;
  std::string neighbor;
  Metric metric = 0;
  MplsOp op = MplsOp::kNone;
  std::vector<int32_t> labels;  // SWAP: {label}; PUSH: stack, bottom first
  bool operator<(const NextHop& o) const;
  bool operator==(const NextHop& o) const;
};

struct MinCostNextHops {
  Metric shortest = 0;
  // next-hop node -> distance from it to the closest announcer
  std::unordered_map<std::string, Metric> viaNode;
};

class SpfSolver {
 public:
  explicit SpfSolver(LinkState& ls) : ls_(ls) {}

  // getNextHopsWithMetric(me, announcers, perDestination=false)
  std::optional<MinCostNextHops> nextHopsWithMetric(const std::string& me,
                                                    const std::vector<std::string>& announcers);
  // SP_ECMP unicast route (empty: no route)
  std::vector<NextHop> ecmpRoute(const std::string& me, const std::vector<std::string>& announcers);
  // MPLS node-label route towards `dst` with its node label (PHP / SWAP)
  std::vector<NextHop> nodeLabelRoute(const std::string& me, const std::string& dst);
  // KSP2_ED_ECMP route (SR-MPLS label stacks)
  std::vector<NextHop> ksp2Route(const std::string& me, const std::vector<std::string>& announcers);

 private:
  std::vector<NextHop> expand(const std::string& me, const MinCostNextHops& m,
                              const std::vector<std::string>& announcers,
                              std::optional<int32_t> swapLabel);
  int32_t nodeLabel(const std::string& node) const;
  LinkState& ls_;
};

}  // namespace odl
