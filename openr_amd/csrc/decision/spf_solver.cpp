// spf_solver.cpp — see spf_solver.h.
#include "spf_solver.h"

#include <algorithm>
#include <limits>
#include <set>
#include <tuple>

namespace odl {

bool NextHop::operator<(const NextHop& o) const {
  return std::tie(ifName, neighbor, metric, op, labels) <
         std::tie(o.ifName, o.neighbor, o.metric, o.op, o.labels);
}
bool NextHop::operator==(const NextHop& o) const {
  return std::tie(ifName, neighbor, metric, op, labels) ==
         std::tie(o.ifName, o.neighbor, o.metric, o.op, o.labels);
}

int32_t SpfSolver::nodeLabel(const std::string& node) const {
  const auto& dbs = ls_.getAdjacencyDatabases();
  auto it = dbs.find(node);
  return it == dbs.end() ? 0 : it->second.nodeLabel;
}

std::optional<MinCostNextHops> SpfSolver::nextHopsWithMetric(
    const std::string& me, const std::vector<std::string>& announcers) {
  const SpfResult& spf = ls_.getSpfResult(me);
  // closest announcers (SpfSolver.cpp:1060-1073)
  Metric shortest = std::numeric_limits<Metric>::max();
  std::vector<std::string> closest;
  for (const auto& d : announcers) {
    auto it = spf.find(d);
    if (it == spf.end()) continue;
    const Metric m = it->second.metric();
    if (m < shortest) {
      shortest = m;
      closest.clear();
    }
    if (m == shortest) closest.push_back(d);
  }
  if (closest.empty()) return std::nullopt;
  MinCostNextHops out;
  out.shortest = shortest;
  for (const auto& d : closest)
    for (const auto& nh : spf.at(d).nextHops())
      out.viaNode[nh] = shortest - *ls_.getMetricFromAToB(me, nh);
  return out;
}

std::vector<NextHop> SpfSolver::expand(const std::string& me, const MinCostNextHops& m,
                                       const std::vector<std::string>& announcers,
                                       std::optional<int32_t> swapLabel) {
  // getNextHopsThrift, perDestination = false (SpfSolver.cpp:1176-1283)
  std::set<std::string> dsts(announcers.begin(), announcers.end());
  std::vector<NextHop> out;
  for (const auto& link : ls_.linksFromNode(me)) {
    const std::string& nbr = link->otherNode(me);
    auto it = m.viaNode.find(nbr);
    if (it == m.viaNode.end() || !link->isUp()) continue;
    const Metric over = link->metricFrom(me) + it->second;
    if (over != m.shortest) continue;  // a longer parallel link drops out
    NextHop nh;
    nh.ifName = link->ifaceFrom(me);
    nh.neighbor = nbr;
    nh.metric = over;
    if (swapLabel) {
      if (dsts.count(nbr)) {
        nh.op = MplsOp::kPhp;
      } else {
        nh.op = MplsOp::kSwap;
        nh.labels = {*swapLabel};
      }
    }
    out.push_back(std::move(nh));
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return out;
}

std::vector<NextHop> SpfSolver::ecmpRoute(const std::string& me,
                                          const std::vector<std::string>& announcers) {
  std::vector<std::string> others;
  for (const auto& a : announcers)
    if (a != me) others.push_back(a);
  if (others.size() != announcers.size()) return {};  // self-originated: no route
  auto m = nextHopsWithMetric(me, others);
  if (!m || m->viaNode.empty()) return {};
  return expand(me, *m, others, std::nullopt);
}

std::vector<NextHop> SpfSolver::nodeLabelRoute(const std::string& me, const std::string& dst) {
  if (dst == me) return {};  // POP_AND_LOOKUP, not an SPF product
  auto m = nextHopsWithMetric(me, {dst});
  if (!m || m->viaNode.empty()) return {};
  return expand(me, *m, {dst}, nodeLabel(dst));
}

std::vector<NextHop> SpfSolver::ksp2Route(const std::string& me,
                                          const std::vector<std::string>& announcers) {
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
    for (const auto& l : p) {
      cost += l->metricFrom(at);
      at = l->otherNode(at);
      stack.insert(stack.begin(), nodeLabel(at));
    }
    if (!stack.empty()) stack.pop_back();  // PHP: the first hop's label
    NextHop nh;
    nh.ifName = p.front()->ifaceFrom(me);
    nh.neighbor = p.front()->otherNode(me);
    nh.metric = cost;
    if (!stack.empty()) {
      nh.op = MplsOp::kPush;
      nh.labels = std::move(stack);
    }
    out.push_back(std::move(nh));
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return out;
}

}  // namespace odl
