// decision_capi.cpp — C ABI over odl::LinkState (include/openr_decision.h).
// Exceptions never cross the ABI: they become an error code + odl_last_error.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/openr_decision.h"
#include "link_state.h"
#include "spf_solver.h"
#include "adjdb_thrift.h"

struct odl_ls {
  odl::LinkState ls;
  std::string err;
  odl_ls(const char* area, int device) : ls(area ? area : "0", device) {}
  odl_ls(const char* area, std::vector<int> devices) : ls(area ? area : "0", std::move(devices)) {}
};

namespace {

char* dup(const std::string& s) {
  char* p = (char*)std::malloc(s.size() + 1);
  if (p) std::memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

std::string at(const oadj_stream* s, uint32_t i) {
  return std::string(s->str_data + s->str_off[i], s->str_data + s->str_off[i + 1]);
}

std::vector<std::string> splitNl(const char* p, uint32_t n) {
  std::vector<std::string> out;
  out.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    const char* q = std::strchr(p, '\n');
    if (!q) q = p + std::strlen(p);
    out.emplace_back(p, q);
    p = *q ? q + 1 : q;
  }
  return out;
}

// DESIGN.md §Result text: one line per reached node, sorted by name:
// name \t metric \t nexthops(sorted, ',') \t pathLinks(key@prev, ';')
std::string spfText(const odl::SpfResult& r) {
  std::vector<const std::string*> names;
  names.reserve(r.size());
  for (const auto& kv : r) names.push_back(&kv.first);
  std::sort(names.begin(), names.end(),
            [](const std::string* a, const std::string* b) { return *a < *b; });
  std::ostringstream os;
  for (const std::string* n : names) {
    const auto& nr = r.at(*n);
    std::vector<std::string> nh(nr.nextHops().begin(), nr.nextHops().end());
    std::sort(nh.begin(), nh.end());
    os << *n << '\t' << nr.metric() << '\t';
    for (size_t i = 0; i < nh.size(); ++i) os << (i ? "," : "") << nh[i];
    os << '\t';
    const auto& pl = nr.pathLinks();
    for (size_t i = 0; i < pl.size(); ++i)
      os << (i ? ";" : "") << pl[i].link->key() << '@' << pl[i].prevNode;
    os << '\n';
  }
  return os.str();
}

void pathsText(std::ostringstream& os, const std::vector<odl::Path>& paths) {
  for (const auto& p : paths) {
    for (size_t i = 0; i < p.size(); ++i) os << (i ? "," : "") << p[i]->key();
    os << '\n';
  }
}

oadj_change changeRecord(const odl::LinkStateChange& c) {
  return oadj_change{c.topologyChanged, c.linkAttributesChanged, c.nodeLabelChanged,
                     (int32_t)c.addedLinks.size(), c.decodeError};
}

template <class F>
auto guard(odl_ls* h, F&& f, decltype(f()) bad) -> decltype(f()) {
  if (!h) return bad;
  try {
    return f();
  } catch (const odl::EngineError& e) {
    h->err = std::string("engine: ") + e.what();
  } catch (const std::exception& e) {
    h->err = e.what();
  }
  return bad;
}

}  // namespace

extern "C" {

int odl_create(const char* area, int device, odl_ls** out) {
  if (!out) return -1;
  try {
    *out = new odl_ls(area, device);
    return 0;
  } catch (...) {
    *out = nullptr;
    return -1;
  }
}

int odl_create_multi(const char* area, const int* devices, uint32_t n, odl_ls** out) {
  if (!out || !devices || !n) return -1;
  try {
    *out = new odl_ls(area, std::vector<int>(devices, devices + n));
    return 0;
  } catch (...) {
    *out = nullptr;
    return -1;
  }
}

void odl_destroy(odl_ls* h) { delete h; }
const char* odl_last_error(const odl_ls* h) { return h ? h->err.c_str() : "null handle"; }
void odl_free(char* p) { std::free(p); }

int odl_apply(odl_ls* h, const oadj_stream* s, uint32_t first, uint32_t count,
              oadj_change* changes) {
  return odl_apply_hold(h, s, first, count, changes, 0, 0);
}

int odl_apply_hold(odl_ls* h, const oadj_stream* s, uint32_t first, uint32_t count,
                   oadj_change* changes, uint64_t hold_up_ttl, uint64_t hold_down_ttl) {
  return guard(h, [&]() -> int {
    if (!s) throw std::invalid_argument("null stream");
    bool deletes = false;
    for (uint32_t k = 0; k < count && s->db_delete; ++k)
      deletes |= first + k < s->n_dbs && s->db_delete[first + k];
    if (!deletes && count >= 64 && first + count <= s->n_dbs) {
      // a batch of updates: databases built on host threads, then applied in
      // order (LinkState::updateAdjacencyDatabases: in parallel when every
      // database is a new node)
      const auto t0 = std::chrono::steady_clock::now();
      std::vector<odl::AdjacencyDatabase> dbs(count);
      odl::parallelFor(count, [&](uint32_t lo, uint32_t hi) {
        for (uint32_t k = lo; k < hi; ++k) {
          const uint32_t i = first + k;
          odl::AdjacencyDatabase& db = dbs[k];
          db.thisNodeName = at(s, s->db_name[i]);
          db.isOverloaded = s->db_overloaded[i] != 0;
          db.nodeLabel = s->db_node_label[i];
          db.adjacencies.resize(s->db_adj_off[i + 1] - s->db_adj_off[i]);
          for (uint64_t a = s->db_adj_off[i]; a < s->db_adj_off[i + 1]; ++a) {
            odl::Adjacency& x = db.adjacencies[a - s->db_adj_off[i]];
            x.otherNodeName = at(s, s->adj_other[a]);
            x.ifName = at(s, s->adj_if[a]);
            x.otherIfName = at(s, s->adj_other_if[a]);
            x.metric = s->adj_metric[a];
            x.adjLabel = s->adj_label[a];
            x.isOverloaded = s->adj_overloaded[a] != 0;
            x.weight = s->adj_weight[a];
          }
        }
      }, 256);
      if (getenv("ODL_SPF_TIMING"))
        std::fprintf(stderr, "ODL_INGEST build_dbs_ms=%.1f\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      const auto chs = h->ls.updateAdjacencyDatabases(dbs, hold_up_ttl, hold_down_ttl);
      for (uint32_t k = 0; changes && k < count; ++k)
        changes[k] = changeRecord(chs[k]);
      return 0;
    }
    for (uint32_t k = 0; k < count; ++k) {
      const uint32_t i = first + k;
      if (i >= s->n_dbs) throw std::out_of_range("stream index");
      const std::string name = at(s, s->db_name[i]);
      odl::LinkStateChange ch;
      if (s->db_delete && s->db_delete[i]) {
        ch = h->ls.deleteAdjacencyDatabase(name);
      } else {
        odl::AdjacencyDatabase db;
        db.thisNodeName = name;
        db.isOverloaded = s->db_overloaded[i] != 0;
        db.nodeLabel = s->db_node_label[i];
        for (uint64_t a = s->db_adj_off[i]; a < s->db_adj_off[i + 1]; ++a) {
          odl::Adjacency x;
          x.otherNodeName = at(s, s->adj_other[a]);
          x.ifName = at(s, s->adj_if[a]);
          x.otherIfName = at(s, s->adj_other_if[a]);
          x.metric = s->adj_metric[a];
          x.adjLabel = s->adj_label[a];
          x.isOverloaded = s->adj_overloaded[a] != 0;
          x.weight = s->adj_weight[a];
          db.adjacencies.push_back(std::move(x));
        }
        ch = h->ls.updateAdjacencyDatabase(db, hold_up_ttl, hold_down_ttl);
      }
      if (changes)
        changes[k] = changeRecord(ch);
    }
    return 0;
  }, -1);
}

char* odl_spf_text(odl_ls* h, const char* root, int use_link_metric) {
  return guard(h, [&]() -> char* {
    return dup(spfText(h->ls.getSpfResult(root, use_link_metric != 0)));
  }, (char*)nullptr);
}

char* odl_kth_paths_text(odl_ls* h, const char* src, const char* dst, int k) {
  return guard(h, [&]() -> char* {
    std::ostringstream os;
    pathsText(os, h->ls.getKthPaths(src, dst, (size_t)k));
    return dup(os.str());
  }, (char*)nullptr);
}

char* odl_links_text(odl_ls* h, const char* node) {
  return guard(h, [&]() -> char* {
    std::ostringstream os;
    for (const auto& l : h->ls.linksFromNode(node))
      os << l->key() << '\t' << l->metricFrom(node) << '\t' << (l->isUp() ? 1 : 0) << '\n';
    return dup(os.str());
  }, (char*)nullptr);
}

char* odl_link_keys_text(odl_ls* h) {
  return guard(h, [&]() -> char* {
    std::ostringstream os;
    for (const auto& l : h->ls.snapshot().links) os << (l ? l->key() : std::string()) << '\n';
    return dup(os.str());
  }, (char*)nullptr);
}

int64_t odl_metric_a_to_b(odl_ls* h, const char* a, const char* b, int use_link_metric) {
  return guard(h, [&]() -> int64_t {
    auto m = h->ls.getMetricFromAToB(a, b, use_link_metric != 0);
    return m ? (int64_t)*m : -1;
  }, (int64_t)-2);
}

int odl_decrement_holds(odl_ls* h) {
  return guard(h, [&]() -> int { return h->ls.decrementHolds().topologyChanged ? 1 : 0; }, -1);
}
int odl_has_holds(const odl_ls* h) { return h ? (h->ls.hasHolds() ? 1 : 0) : -1; }

int odl_is_overloaded(odl_ls* h, const char* node) {
  return h ? (h->ls.isNodeOverloaded(node) ? 1 : 0) : -1;
}
uint64_t odl_spf_runs(const odl_ls* h) { return h ? h->ls.spfRuns() : 0; }
void odl_get_counters(const odl_ls* h, odl_counters* out) {
  if (!h || !out) return;
  const auto c = h->ls.counters();
  *out = odl_counters{c.spf_runs, c.spf_ms_samples, c.spf_ms_sum, c.ucmp_runs, c.ucmp_ms_sum,
                      c.route_build_runs, c.route_build_ms_sum, h->ls.engineErrors(),
                      h->ls.degraded() ? 1u : 0u};
}
const char* odl_last_engine_error(const odl_ls* h) {
  return h ? h->ls.lastEngineError().c_str() : "";
}
void odl_set_degrade(odl_ls* h, int on) {
  if (h) h->ls.setDegradeOnError(on != 0);
}
int odl_inject_engine_error(odl_ls* h, uint32_t after) {
  return guard(h, [&]() -> int {
    h->ls.injectEngineError(after);
    return 0;
  }, -1);
}
void odl_set_incremental(odl_ls* h, int on) {
  if (h) h->ls.setIncremental(on != 0);
}
int odl_apply_kvs(odl_ls* h, uint32_t n, const char* const* keys, const uint8_t* const* values,
                  const uint64_t* value_lens, uint32_t n_expired, const char* const* expired,
                  const char* my_node, oadj_change* changes) {
  return guard(h, [&]() -> int {
    if ((n && (!keys || !values || !value_lens)) || (n_expired && !expired))
      throw std::invalid_argument("null key-value arrays");
    std::vector<odl::LinkState::KvIn> kvs(n);
    for (uint32_t i = 0; i < n; ++i) {
      kvs[i].key = keys[i];
      kvs[i].hasValue = values[i] != nullptr;
      if (values[i]) kvs[i].value = std::string_view((const char*)values[i], (size_t)value_lens[i]);
    }
    std::vector<std::string_view> exp(expired, expired + n_expired);
    const std::string me = my_node ? my_node : "";
    const auto chs = h->ls.applyKvs(kvs, exp, my_node ? &me : nullptr);
    for (size_t k = 0; changes && k < chs.size(); ++k) changes[k] = changeRecord(chs[k]);
    return 0;
  }, -1);
}

int odl_apply_publication(odl_ls* h, const uint8_t* buf, uint64_t len, const char* my_node,
                          oadj_change* changes, uint32_t max_changes, uint32_t* n_changes_out) {
  return guard(h, [&]() -> int {
    if (!buf && len) throw std::invalid_argument("null publication buffer");
    odl::PublicationView pv;
    odl::thrift_compact::parsePublication(buf, (size_t)len, pv);
    if (!pv.area.empty() && pv.area != h->ls.area())
      throw std::invalid_argument("publication of area '" + std::string(pv.area) +
                                  "' given to the LinkState of area '" + h->ls.area() + "'");
    const size_t nrec = pv.keyVals.size() + pv.expiredKeys.size();
    if (n_changes_out) *n_changes_out = (uint32_t)nrec;
    if (changes && nrec > max_changes) return ODL_E_SMALL;  // nothing applied
    std::vector<odl::LinkState::KvIn> kvs(pv.keyVals.size());
    for (size_t i = 0; i < kvs.size(); ++i)
      kvs[i] = odl::LinkState::KvIn{pv.keyVals[i].key, pv.keyVals[i].value, pv.keyVals[i].hasValue};
    const std::string me = my_node ? my_node : "";
    const auto chs = h->ls.applyKvs(kvs, pv.expiredKeys, my_node ? &me : nullptr);
    for (size_t k = 0; changes && k < chs.size(); ++k) changes[k] = changeRecord(chs[k]);
    return 0;
  }, -1);
}

const char* odl_last_decode_error(const odl_ls* h, uint64_t* n_errors) {
  if (n_errors) *n_errors = h ? h->ls.decodeErrors() : 0;
  return h ? h->ls.lastDecodeError().c_str() : "";
}

void odl_set_host_spf(odl_ls* h, int on) {
  if (h) h->ls.setHostSpf(on != 0);
}
void odl_incremental_stats(const odl_ls* h, uint64_t* out) {
  if (!h || !out) return;
  const auto& st = h->ls.incrementalStats();
  out[0] = st.patches;
  out[1] = st.kept;
  out[2] = st.dropped;
}
void odl_topology_stats(const odl_ls* h, uint64_t* out4) {
  if (!h || !out4) return;
  const auto& st = h->ls.topologyStats();
  out4[0] = st.snapshots;
  out4[1] = st.loads;
  out4[2] = st.link_patches;
  out4[3] = st.rows_patched;
}
uint64_t odl_node_patches(const odl_ls* h) { return h ? h->ls.topologyStats().node_patches : 0; }
void odl_shard_stats(const odl_ls* h, uint64_t* out4) {
  if (!h || !out4) return;
  const auto& st = h->ls.shardStats();
  out4[0] = st.spf_batches;
  out4[1] = st.spf_launches;
  out4[2] = st.ksp2_runs;
  out4[3] = st.ksp2_launches;
}
uint32_t odl_num_nodes(const odl_ls* h) { return h ? (uint32_t)h->ls.numNodes() : 0; }
uint32_t odl_num_links(const odl_ls* h) { return h ? (uint32_t)h->ls.numLinks() : 0; }

int odl_spf_digests(odl_ls* h, const char* roots_nl, uint32_t n, int use_link_metric,
                    uint64_t* out) {
  return guard(h, [&]() -> int {
    auto d = h->ls.spfDigests(splitNl(roots_nl, n), use_link_metric != 0);
    for (uint32_t i = 0; i < n; ++i) {
      out[3 * i] = d[i].reached;
      out[3 * i + 1] = d[i].sum_dist;
      out[3 * i + 2] = d[i].hash;
    }
    return 0;
  }, -1);
}

int odl_all_sources_digests(odl_ls* h, int use_link_metric, uint64_t* out) {
  return guard(h, [&]() -> int {
    auto d = h->ls.allSourcesDigests(use_link_metric != 0);
    for (size_t i = 0; i < d.size(); ++i) {
      out[3 * i] = d[i].reached;
      out[3 * i + 1] = d[i].sum_dist;
      out[3 * i + 2] = d[i].hash;
    }
    return 0;
  }, -1);
}

int odl_all_sources_prefetch(odl_ls* h, int use_link_metric) {
  return guard(h, [&]() -> int {
    h->ls.prefetchAllSources(use_link_metric != 0);
    return 0;
  }, -1);
}

void odl_sweep_stats(const odl_ls* h, uint64_t* out5) {
  if (!h || !out5) return;
  const auto& st = h->ls.sweepStats();
  out5[0] = st.sweeps;
  out5[1] = st.rows_copied;
  out5[2] = st.mode;
  out5[3] = st.devices;
  out5[4] = st.hip_graph;
}

int odl_spf_prefetch(odl_ls* h, const char* roots_nl, uint32_t n, int use_link_metric) {
  return guard(h, [&]() -> int {
    h->ls.prefetchSpf(splitNl(roots_nl, n), use_link_metric != 0);
    return 0;
  }, -1);
}

char* odl_ksp2_text(odl_ls* h, const char* src, const char* dsts_nl, uint32_t n) {
  return guard(h, [&]() -> char* {
    auto dsts = splitNl(dsts_nl, n);
    h->ls.prefetchKsp2(src, dsts);
    std::ostringstream os;
    for (const auto& d : dsts) {
      pathsText(os, h->ls.getKthPaths(src, d, 2));
      os << "=\n";
    }
    return dup(os.str());
  }, (char*)nullptr);
}

char* odl_route_text(odl_ls* h, const char* me, const char* announcers_nl, uint32_t n,
                     int algo) {
  return guard(h, [&]() -> char* {
    odl::SpfSolver solver(h->ls);
    const auto ann = splitNl(announcers_nl, n);
    std::vector<odl::NextHop> nhs;
    if (algo == 0) nhs = solver.ecmpRoute(me, ann);
    else if (algo == 1) nhs = solver.ksp2Route(me, ann);
    else if (algo == 2 && n == 1) nhs = solver.nodeLabelRoute(me, ann[0]);
    else throw std::invalid_argument("algo must be 0, 1 or 2 (2 needs one announcer)");
    std::ostringstream os;
    for (const auto& x : nhs) {
      os << x.ifName << '\t' << x.neighbor << '\t' << x.metric << '\t' << (int)x.op << '\t';
      for (size_t i = 0; i < x.labels.size(); ++i) os << (i ? "," : "") << x.labels[i];
      os << '\n';
    }
    return dup(os.str());
  }, (char*)nullptr);
}

int odl_path_a_in_b(const char* a_nl, uint32_t na, const char* b_nl, uint32_t nb) {
  try {
    auto parse = [](const char* nl, uint32_t n) {
      odl::Path p;
      for (const auto& key : splitNl(nl, n)) {
        const size_t bar = key.find('|'), p1 = key.find('%'), p2 = key.find('%', bar);
        if (bar == std::string::npos || p1 > bar || p2 == std::string::npos)
          throw std::invalid_argument("link key must be n1%if1|n2%if2: " + key);
        odl::Adjacency a1, a2;
        const std::string n1 = key.substr(0, p1), n2 = key.substr(bar + 1, p2 - bar - 1);
        a1.otherNodeName = n2;
        a1.ifName = key.substr(p1 + 1, bar - p1 - 1);
        a2.otherNodeName = n1;
        a2.ifName = key.substr(p2 + 1);
        a1.otherIfName = a2.ifName;
        a2.otherIfName = a1.ifName;
        p.push_back(std::make_shared<odl::Link>(n1, a1, n2, a2));
      }
      return p;
    };
    return odl::LinkState::pathAInPathB(parse(a_nl, na), parse(b_nl, nb)) ? 1 : 0;
  } catch (...) {
    return -1;
  }
}

namespace {
// the prefix lines of odl_route_db_text / _bin -> PrefixRoutes, then the build
// (over `areas` when given, else h's LinkState alone)
std::vector<std::optional<odl::RouteDb>> buildDbs(odl_ls* h, const std::vector<std::string>& mes,
                                                  const char* prefixes_nl, uint32_t n, int flags,
                                                  const std::vector<odl::LinkState*>* areas = nullptr) {
    auto field = [](const std::string& s, size_t& pos, char sep) {
      const size_t e = s.find(sep, pos);
      std::string out = s.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
      pos = e == std::string::npos ? s.size() + 1 : e + 1;
      return out;
    };
    std::vector<odl::PrefixRoute> prefixes;
    for (const auto& ln : splitNl(prefixes_nl, n)) {
      const size_t t = ln.find('\t');
      if (t == std::string::npos) throw std::invalid_argument("prefix line needs prefix\\tentries");
      odl::PrefixRoute pr;
      pr.prefix = ln.substr(0, t);
      std::stringstream es(ln.substr(t + 1));
      for (std::string x; std::getline(es, x, ',');) {
        if (x.empty()) continue;
        // optional suffixes, in this order: "%pp/sp/d" (PrefixMetrics),
        // "!bgp" / "!bgpmv" (PrefixType::BGP without / with a metric
        // vector), "@area", "#minNexthop"
        std::optional<int64_t> minNh;
        std::string area, type;
        int32_t met[3] = {0, 0, 0};
        if (const size_t hsh = x.rfind('#'); hsh != std::string::npos) {
          minNh = std::stoll(x.substr(hsh + 1));
          x.resize(hsh);
        }
        if (const size_t at = x.rfind('@'); at != std::string::npos) {
          area = x.substr(at + 1);
          x.resize(at);
        }
        if (const size_t bang = x.rfind('!'); bang != std::string::npos) {
          type = x.substr(bang + 1);
          x.resize(bang);
          if (type != "bgp" && type != "bgpmv")
            throw std::invalid_argument("prefix entry type must be bgp or bgpmv: " + type);
        }
        if (const size_t pc = x.rfind('%'); pc != std::string::npos) {
          size_t q = pc + 1;
          for (int k = 0; k < 3; ++k) met[k] = std::stoi(field(x, q, '/'));
          x.resize(pc);
        }
        // node:fwd:algo:weight[:prepend] -- a node name holding ':' or ','
        // would shift the fields: this text ABI rejects it (the C++ API
        // takes any name)
        const size_t colons = (size_t)std::count(x.begin(), x.end(), ':');
        if (colons < 3 || colons > 4)
          throw std::invalid_argument("prefix entry needs node:fwd:algo:weight[:prepend] "
                                      "(node names with ':' or ',' are not supported here): " + x);
        size_t pos = 0;
        odl::PrefixEntry e;
        e.node = field(x, pos, ':');
        const std::string fwd = field(x, pos, ':'), algo = field(x, pos, ':'),
                          w = field(x, pos, ':'), pl = field(x, pos, ':');
        if (e.node.empty() || fwd.empty() || algo.empty() || w.empty())
          throw std::invalid_argument("prefix entry needs node:fwd:algo:weight[:prepend]");
        e.fwdType = std::stoi(fwd);
        e.algo = std::stoi(algo);
        e.weight = std::stoll(w);
        if (e.fwdType < 0 || e.fwdType > 1 || e.algo < 0 || e.algo > 3 || e.weight < 0)
          throw std::invalid_argument("prefix entry out of range: " + x);
        if (!pl.empty()) e.prependLabel = std::stoi(pl);
        e.area = area;
        e.minNexthop = minNh;
        e.pathPreference = met[0];
        e.sourcePreference = met[1];
        e.distance = met[2];
        e.bgp = !type.empty();
        e.hasMv = type == "bgpmv";
        pr.entries.push_back(std::move(e));
      }
      prefixes.push_back(std::move(pr));
    }
    odl::RouteOptions opt;
    opt.nodeSegmentLabels = flags & 1;
    opt.adjacencyLabels = flags & 2;
    opt.ucmp = flags & 4;
    opt.bestRouteSelection = flags & 8;
    odl::SpfSolver solver = areas ? odl::SpfSolver(*areas) : odl::SpfSolver(h->ls);
    const auto t0 = std::chrono::steady_clock::now();
    auto dbs = solver.buildRouteDbs(mes, prefixes, opt);
    if (getenv("ODL_SPF_TIMING"))
      fprintf(stderr, "route_timing mes=%zu prefixes=%zu build_route_db_ms=%.3f\n", mes.size(),
              prefixes.size(),
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    return dbs;
}
}  // namespace

namespace {
std::string routeDbText(const std::vector<std::string>& mes,
                        const std::vector<std::optional<odl::RouteDb>>& dbs, bool withArea,
                        bool withBest = false) {
  std::ostringstream os;
  for (size_t i = 0; i < mes.size(); ++i) {
    const auto& me = mes[i];
    if (!dbs[i]) {
      os << me << "\tNONE\n";
      continue;
    }
    // fields are tab-separated, records newline-separated: names holding
    // either cannot be written unambiguously by this text ABI
    auto plain = [](const std::string& f) {
      if (f.find_first_of("\t\n") != std::string::npos)
        throw std::invalid_argument("name with a tab or newline in the route text: " + f);
    };
    plain(me);
    auto put = [&](const char* kind, const std::string& key, const std::vector<odl::NextHop>& nhs) {
      for (const auto& x : nhs) {
        plain(x.ifName);
        plain(x.neighbor);
        os << me << '\t' << kind << '\t' << key << '\t' << x.ifName << '\t' << x.neighbor << '\t'
           << x.metric << '\t' << (int)x.op << '\t';
        for (size_t j = 0; j < x.labels.size(); ++j) os << (j ? "," : "") << x.labels[j];
        os << '\t' << x.weight;
        if (withArea) os << '\t' << x.area;
        os << '\n';
      }
    };
    for (const auto& kv : dbs[i]->unicast) {
      os << me << "\tR\t" << kv.first << '\t' << kv.second.igpCost << '\t';
      if (kv.second.weight) os << *kv.second.weight; else os << '-';
      if (withBest) {  // the best-route selection: best node@area, then every selected one
        os << '\t' << kv.second.best.first << '@' << kv.second.best.second << '\t';
        size_t j = 0;
        for (const auto& na : kv.second.selected) os << (j++ ? "," : "") << na.first << '@' << na.second;
      }
      os << '\n';
      put("U", kv.first, kv.second.nextHops);
    }
    for (const auto& kv : dbs[i]->mpls) put("M", std::to_string(kv.first), kv.second);
  }
  return os.str();
}
}  // namespace

char* odl_route_db_text(odl_ls* h, const char* mes_nl, uint32_t n_mes, const char* prefixes_nl,
                        uint32_t n, int flags) {
  return guard(h, [&]() -> char* {
    const auto mes = splitNl(mes_nl, n_mes);
    return dup(routeDbText(mes, buildDbs(h, mes, prefixes_nl, n, flags), false, flags & 8));
  }, (char*)nullptr);
}

char* odl_route_db_multi_text(odl_ls* const* areas, uint32_t n_areas, const char* mes_nl,
                              uint32_t n_mes, const char* prefixes_nl, uint32_t n, int flags) {
  if (!areas || n_areas == 0 || !areas[0]) return nullptr;
  return guard(areas[0], [&]() -> char* {
    std::vector<odl::LinkState*> ls;
    for (uint32_t i = 0; i < n_areas; ++i) {
      if (!areas[i]) throw std::invalid_argument("null area handle");
      ls.push_back(&areas[i]->ls);
    }
    const auto mes = splitNl(mes_nl, n_mes);
    return dup(routeDbText(mes, buildDbs(areas[0], mes, prefixes_nl, n, flags, &ls), true, flags & 8));
  }, (char*)nullptr);
}

int odl_route_db_bin(odl_ls* h, const char* mes_nl, uint32_t n_mes, const char* prefixes_nl,
                     uint32_t n, int flags, void** out, uint64_t* bytes) {
  return guard(h, [&]() -> int {
    if (!out) throw std::invalid_argument("null output pointer");
    *out = nullptr;
    const auto mes = splitNl(mes_nl, n_mes);
    const auto dbs = buildDbs(h, mes, prefixes_nl, n, flags);
    std::vector<odl_rdb_node> nodes(mes.size());
    std::vector<odl_rdb_route> routes;
    std::vector<odl_rdb_nh> nhs;
    std::vector<int32_t> labels;
    std::string strs;
    // every string once (names, interfaces, prefixes): offset into strs
    std::unordered_map<std::string, uint32_t> ids;
    auto sid = [&](const std::string& x) -> uint32_t {
      auto it = ids.find(x);
      if (it != ids.end()) return it->second;
      const uint32_t o = (uint32_t)strs.size();
      strs.append(x);
      strs.push_back('\0');
      ids.emplace(x, o);
      return o;
    };
    auto put = [&](odl_rdb_route& r, const std::vector<odl::NextHop>& v) {
      r.first_nh = (uint32_t)nhs.size();
      r.n_nh = (uint32_t)v.size();
      for (const auto& x : v) {
        odl_rdb_nh e{};
        e.if_name = sid(x.ifName);
        e.neighbor = sid(x.neighbor);
        e.metric = x.metric;
        e.weight = x.weight;
        e.op = (uint32_t)x.op;
        e.first_label = (uint32_t)labels.size();
        e.n_labels = (uint32_t)x.labels.size();
        labels.insert(labels.end(), x.labels.begin(), x.labels.end());
        nhs.push_back(e);
      }
    };
    for (size_t i = 0; i < mes.size(); ++i) {
      odl_rdb_node& nd = nodes[i];
      nd.name = sid(mes[i]);
      nd.first_route = (uint32_t)routes.size();
      if (!dbs[i]) continue;
      nd.found = 1;
      nd.n_unicast = (uint32_t)dbs[i]->unicast.size();
      nd.n_mpls = (uint32_t)dbs[i]->mpls.size();
      for (const auto& kv : dbs[i]->unicast) {
        odl_rdb_route r{};
        r.kind = 0;
        r.key = sid(kv.first);
        r.igp_cost = kv.second.igpCost;
        r.has_weight = kv.second.weight.has_value();
        r.ucmp_weight = kv.second.weight.value_or(0);
        put(r, kv.second.nextHops);
        routes.push_back(r);
      }
      for (const auto& kv : dbs[i]->mpls) {
        odl_rdb_route r{};
        r.kind = 1;
        r.key = (uint32_t)kv.first;
        put(r, kv.second);
        routes.push_back(r);
      }
    }
    auto al = [](uint64_t x) { return (x + 7) & ~7ull; };
    odl_rdb_header hd{};
    hd.magic = ODL_RDB_MAGIC;
    hd.version = 1;
    hd.n_nodes = (uint32_t)nodes.size();
    hd.n_routes = (uint32_t)routes.size();
    hd.n_nhs = (uint32_t)nhs.size();
    hd.n_labels = (uint32_t)labels.size();
    hd.off_nodes = al(sizeof(hd));
    hd.off_routes = al(hd.off_nodes + nodes.size() * sizeof(odl_rdb_node));
    hd.off_nhs = al(hd.off_routes + routes.size() * sizeof(odl_rdb_route));
    hd.off_labels = al(hd.off_nhs + nhs.size() * sizeof(odl_rdb_nh));
    hd.off_strings = al(hd.off_labels + labels.size() * sizeof(int32_t));
    hd.str_bytes = strs.size();
    hd.bytes = al(hd.off_strings + strs.size());
    char* b = (char*)std::calloc(1, hd.bytes);
    if (!b) throw std::bad_alloc();
    std::memcpy(b, &hd, sizeof(hd));
    auto cp = [&](uint64_t off, const void* src, size_t nb) { if (nb) std::memcpy(b + off, src, nb); };
    cp(hd.off_nodes, nodes.data(), nodes.size() * sizeof(odl_rdb_node));
    cp(hd.off_routes, routes.data(), routes.size() * sizeof(odl_rdb_route));
    cp(hd.off_nhs, nhs.data(), nhs.size() * sizeof(odl_rdb_nh));
    cp(hd.off_labels, labels.data(), labels.size() * sizeof(int32_t));
    cp(hd.off_strings, strs.data(), strs.size());
    *out = b;
    if (bytes) *bytes = hd.bytes;
    return 0;
  }, -1);
}

void odl_free_buf(void* p) { std::free(p); }

char* odl_ucmp_text(odl_ls* h, const char* root, const char* leaves_nl, uint32_t n, int algo,
                    int use_link_metric) {
  return guard(h, [&]() -> char* {
    if (algo != 2 && algo != 3) throw std::invalid_argument("algo must be 2 or 3");
    std::unordered_map<std::string, int64_t> leaves;
    for (const auto& ln : splitNl(leaves_nl, n)) {
      const size_t t = ln.find('\t');
      if (t == std::string::npos) throw std::invalid_argument("leaf line needs name\tweight");
      leaves.emplace(ln.substr(0, t), std::stoll(ln.substr(t + 1)));
    }
    const bool um = use_link_metric != 0;
    const auto res = h->ls.resolveUcmpWeights(h->ls.getSpfResult(root, um), leaves,
                                              (odl::UcmpAlgo)algo, um);
    std::vector<std::string> names;
    for (const auto& kv : res) names.push_back(kv.first);
    std::sort(names.begin(), names.end());
    std::ostringstream os;
    for (const auto& nm : names) {
      const auto& u = res.at(nm);
      os << nm << '\t' << (u.weight() ? *u.weight() : 0) << '\t';
      std::vector<std::string> ifs;
      for (const auto& kv : u.nextHopLinks()) ifs.push_back(kv.first);
      std::sort(ifs.begin(), ifs.end());
      for (size_t i = 0; i < ifs.size(); ++i) {
        const auto& hop = u.nextHopLinks().at(ifs[i]);
        os << (i ? "," : "") << ifs[i] << '=' << hop.nextHopNode << ':' << hop.weight;
      }
      os << '\n';
    }
    return dup(os.str());
  }, (char*)nullptr);
}

int odl_csr_size(odl_ls* h, uint32_t* n_nodes, uint32_t* n_edges) {
  return guard(h, [&]() -> int {
    const auto& c = h->ls.snapshot();
    if (n_nodes) *n_nodes = (uint32_t)c.names.size();
    if (n_edges) *n_edges = (uint32_t)c.col.size();
    return 0;
  }, -1);
}

int odl_csr_export(odl_ls* h, uint32_t* row_ptr, uint32_t* col, uint32_t* metric,
                   uint32_t* link_id, uint32_t* twin, uint8_t* edge_up, uint8_t* no_transit,
                   uint32_t* link_rank) {
  return guard(h, [&]() -> int {
    const auto& c = h->ls.snapshot();
    auto cp = [](auto* dst, const auto& v) {
      if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(v[0]));
    };
    cp(row_ptr, c.rowPtr);
    cp(col, c.col);
    cp(metric, c.metric);
    cp(link_id, c.linkId);
    cp(twin, c.twin);
    cp(edge_up, c.edgeUp);
    cp(no_transit, c.noTransit);
    cp(link_rank, c.linkRank);
    return 0;
  }, -1);
}

const char* odl_node_name(odl_ls* h, uint32_t id) {
  return guard(h, [&]() -> const char* {
    const auto& c = h->ls.snapshot();
    return id < c.names.size() ? c.names[id].c_str() : nullptr;
  }, (const char*)nullptr);
}

int64_t odl_node_id(odl_ls* h, const char* name) {
  return guard(h, [&]() -> int64_t {
    const auto& c = h->ls.snapshot();
    auto it = c.ids.find(name);
    return it == c.ids.end() ? -1 : (int64_t)it->second;
  }, (int64_t)-2);
}

struct odl_adjdbs {
  odl::AdjDbColumns cols;
};
static thread_local std::string g_adjdbs_err;
odl_adjdbs* odl_adjdbs_decode(const uint8_t* const* values, const uint64_t* lens, uint32_t n) {
  try {
    if (n && (!values || !lens)) throw std::invalid_argument("null value arrays");
    auto* d = new odl_adjdbs;
    try {
      d->cols.decode(values, lens, n);
    } catch (...) {
      delete d;
      throw;
    }
    return d;
  } catch (const std::exception& e) {
    g_adjdbs_err = e.what();
  } catch (...) {
    g_adjdbs_err = "unknown error";
  }
  return nullptr;
}
const oadj_stream* odl_adjdbs_stream(const odl_adjdbs* d) { return d ? &d->cols.stream : nullptr; }
const char* odl_adjdbs_error(void) { return g_adjdbs_err.c_str(); }
void odl_adjdbs_free(odl_adjdbs* d) { delete d; }

}  // extern "C"
