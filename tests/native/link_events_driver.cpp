// link_events_driver.cpp — a native driver of the link-event sequence of
// tests/link_events.py, for address-sanitized runs of the host code on a
// GPU box (scripts/asan_gpu.sh): libopenr_decision (odl::LinkState,
// patchStructure's CSR splice, the memo reaper), the host side of
// libopenr_spf_hip (ospf_update_rows' host shadows, plans, sweeps; built
// with -Xarch_host -fsanitize=address, device code uninstrumented) and the
// oracle, all driven from one instrumented executable so the sanitizer
// runtime is loaded first. Test infrastructure: every result is compared
// with the oracle (liboracle), and any mismatch or sanitizer report fails.
//
// Sequence per (seed, unit): a random link-state graph (parallel links,
// overloaded nodes, down adjacencies); withdraw / restore random adjacencies
// ([LINK DOWN] / [LINK UP], LinkState.cpp:632-657), KSP2 across events,
// brand-new links between known nodes (two one-sided advertisements),
// metric / overload changes; after every event the full SpfResult text of
// sampled roots (link metric and hop count) and decision.spf_runs; at the end
// every root's text and all-sources digests.
//
//   link_events_driver [n_seeds] [device] [host]   (host = 1: odl_set_host_spf)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "../../include/openr_adjdb.h"
#include "../../include/openr_decision.h"

extern "C" {
void* orc_create();
void orc_destroy(void*);
void orc_free(char*);
int orc_apply(void*, const oadj_stream*, uint32_t, uint32_t, oadj_change*);
char* orc_spf_text(void*, const char*, int);
char* orc_kth_paths_text(void*, const char*, const char*, int);
uint64_t orc_spf_runs(void*);
}

namespace {

struct Adj {
  std::string other, ifn, oifn;
  int32_t metric = 1;
  bool overloaded = false;
};
struct Db {
  std::string name;
  bool overloaded = false;
  int32_t label = 0;
  std::vector<Adj> adjs;
};

// Columnar stream of databases (include/openr_adjdb.h), owning its columns.
struct Stream {
  std::string data;
  std::vector<uint64_t> off{0};
  std::map<std::string, uint32_t> ids;
  std::vector<uint32_t> name, aother, aif, aoif;
  std::vector<uint8_t> ov, aov;
  std::vector<int32_t> label, metric, alabel;
  std::vector<int64_t> weight;
  std::vector<uint64_t> adjOff{0};
  oadj_stream s{};
  uint32_t str(const std::string& x) {
    auto it = ids.find(x);
    if (it != ids.end()) return it->second;
    data += x;
    off.push_back(data.size());
    return ids[x] = (uint32_t)off.size() - 2;
  }
  explicit Stream(const std::vector<const Db*>& dbs) {
    for (const Db* d : dbs) {
      name.push_back(str(d->name));
      ov.push_back(d->overloaded);
      label.push_back(d->label);
      for (const Adj& a : d->adjs) {
        aother.push_back(str(a.other));
        aif.push_back(str(a.ifn));
        aoif.push_back(str(a.oifn));
        metric.push_back(a.metric);
        alabel.push_back(0);
        aov.push_back(a.overloaded);
        weight.push_back(1);
      }
      adjOff.push_back(aother.size());
    }
    s.str_data = data.data();
    s.str_off = off.data();
    s.n_str = (uint32_t)off.size() - 1;
    s.n_dbs = (uint32_t)dbs.size();
    s.db_name = name.data();
    s.db_overloaded = ov.data();
    s.db_node_label = label.data();
    s.db_delete = nullptr;
    s.db_adj_off = adjOff.data();
    s.adj_other = aother.data();
    s.adj_if = aif.data();
    s.adj_other_if = aoif.data();
    s.adj_metric = metric.data();
    s.adj_label = alabel.data();
    s.adj_overloaded = aov.data();
    s.adj_weight = weight.data();
    s.adj_only_used_by_other = nullptr;
  }
};

int g_fail = 0;
#define EXPECT(c, ...)                                         \
  do {                                                         \
    if (!(c)) {                                                \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);     \
      fprintf(stderr, __VA_ARGS__);                            \
      fprintf(stderr, "\n");                                   \
      ++g_fail;                                                \
      return false;                                            \
    }                                                          \
  } while (0)

std::string take_odl(char* p) {
  std::string s = p ? p : "<null>";
  if (p) odl_free(p);
  return s;
}
std::string take_orc(char* p) {
  std::string s = p ? p : "<null>";
  if (p) orc_free(p);
  return s;
}

struct Pair {
  odl_ls* p = nullptr;
  void* o = nullptr;
  bool apply(const std::vector<const Db*>& dbs) {
    Stream st(dbs);
    std::vector<oadj_change> a(dbs.size()), b(dbs.size());
    EXPECT(odl_apply(p, &st.s, 0, (uint32_t)dbs.size(), a.data()) == 0, "odl_apply: %s",
           odl_last_error(p));
    EXPECT(orc_apply(o, &st.s, 0, (uint32_t)dbs.size(), b.data()) == 0, "orc_apply");
    for (size_t i = 0; i < dbs.size(); ++i)
      EXPECT(!memcmp(&a[i], &b[i], sizeof(oadj_change)), "change record of %s differs",
             dbs[i]->name.c_str());
    return true;
  }
  bool spf(const std::string& r) {
    for (int m = 0; m < 2; ++m) {
      const std::string x = take_odl(odl_spf_text(p, r.c_str(), m)), y = take_orc(orc_spf_text(o, r.c_str(), m));
      EXPECT(x == y, "spf text of %s (metric %d) differs", r.c_str(), m);
    }
    return true;
  }
  bool ksp(const std::string& s, const std::string& d) {
    for (int k = 1; k <= 2; ++k) {
      const std::string x = take_odl(odl_kth_paths_text(p, s.c_str(), d.c_str(), k)),
                        y = take_orc(orc_kth_paths_text(o, s.c_str(), d.c_str(), k));
      EXPECT(x == y, "kth paths %s -> %s k=%d differ", s.c_str(), d.c_str(), k);
    }
    return true;
  }
  bool runs(const char* what) {
    EXPECT(odl_spf_runs(p) == orc_spf_runs(o), "spf_runs %llu vs %llu after %s",
           (unsigned long long)odl_spf_runs(p), (unsigned long long)orc_spf_runs(o), what);
    return true;
  }
};

bool run_seed(int seed, bool unit, int device, bool host) {
  std::mt19937_64 rng(0x5eed0000ull + (uint64_t)seed * 2 + unit);
  auto U = [&](uint64_t n) { return (uint64_t)(rng() % n); };
  auto P = [&](double p) { return (double)(rng() >> 11) / 9007199254740992.0 < p; };
  const int n = 40 + (int)U(30);
  std::vector<Db> dbs(n);
  std::vector<std::string> names(n);
  for (int i = 0; i < n; ++i) {
    names[i] = "r" + std::to_string(U(100000));
    names[i] += "_" + std::to_string(i);
    dbs[i].name = names[i];
    dbs[i].label = i + 1;
    dbs[i].overloaded = P(0.1);
  }
  int k = 0;
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      if (!P(0.15)) continue;
      for (int par = P(0.2) ? 2 : 1; par > 0; --par, ++k) {
        const std::string ia = names[i] + "-" + names[j] + "-" + std::to_string(k),
                          ib = names[j] + "-" + names[i] + "-" + std::to_string(k);
        Adj a{names[j], ia, ib, unit ? 1 : (int32_t)(1 + U(20)), P(0.1)};
        Adj b{names[i], ib, ia, unit ? 1 : (int32_t)(1 + U(20)), false};
        dbs[i].adjs.push_back(a);
        dbs[j].adjs.push_back(b);
      }
    }
  Pair x;
  if (odl_create("0", device, &x.p) != 0) {
    fprintf(stderr, "odl_create failed\n");
    return false;
  }
  if (host) odl_set_host_spf(x.p, 1);
  x.o = orc_create();
  bool ok = true;
  auto check = [&](int kk) {
    for (int i = 0; i < kk && ok; ++i) ok = x.spf(names[U(n)]);
  };
  {
    std::vector<const Db*> all;
    for (const Db& d : dbs) all.push_back(&d);
    ok = x.apply(all);
  }
  check(6);
  for (int step = 0; step < 12 && ok; ++step) {
    Db& d = dbs[U(n)];
    if (d.adjs.empty()) continue;
    const size_t i = U(d.adjs.size());
    const Adj gone = d.adjs[i];
    d.adjs.erase(d.adjs.begin() + i);  // [LINK DOWN]
    ok = ok && x.apply({&d});
    check(6);
    ok = ok && x.runs("withdraw");
    if (ok && step % 3 == 0) ok = x.ksp(names[U(n)], names[U(n)]) && x.runs("ksp2");
    d.adjs.insert(d.adjs.begin() + i, gone);  // [LINK UP]
    ok = ok && x.apply({&d});
    check(6);
    ok = ok && x.runs("restore");
    if (ok && step % 4 == 1 && d.adjs.size() >= 2) {  // metric + overload bits in one update
      d.adjs[0].metric = unit ? 1 : (int32_t)(1 + U(40));
      d.adjs[1].overloaded = !d.adjs[1].overloaded;
      ok = x.apply({&d});
      check(4);
      d.overloaded = !d.overloaded;
      ok = ok && x.apply({&d});
      check(4);
      ok = ok && x.runs("metric / overload");
    }
  }
  for (int step = 0; step < 5 && ok; ++step) {  // new links between known nodes
    const int a = (int)U(n);
    int b = (int)U(n);
    if (b == a) b = (a + 1) % n;
    const std::string ia = names[a] + "-" + names[b] + "-new" + std::to_string(step),
                      ib = names[b] + "-" + names[a] + "-new" + std::to_string(step);
    dbs[a].adjs.push_back(Adj{names[b], ia, ib, unit ? 1 : (int32_t)(1 + U(20)), false});
    ok = x.apply({&dbs[a]});
    dbs[b].adjs.push_back(Adj{names[a], ib, ia, unit ? 1 : (int32_t)(1 + U(20)), false});
    ok = ok && x.apply({&dbs[b]});
    check(6);
    ok = ok && x.runs("new link");
  }
  if (ok) {  // every root, then the all-sources sweep's digests exist for every node
    for (int i = 0; i < n && ok; ++i) ok = x.spf(names[i]);
    std::vector<uint64_t> dg(3ull * n);
    if (ok && odl_all_sources_digests(x.p, 1, dg.data()) != 0) {
      fprintf(stderr, "FAIL all-sources digests: %s\n", odl_last_error(x.p));
      ++g_fail;
      ok = false;
    }
    for (int i = 0; ok && i < n; ++i)
      if (dg[3ull * i] == 0) {
        fprintf(stderr, "FAIL all-sources digest of node %d empty\n", i);
        ++g_fail;
        ok = false;
      }
  }
  odl_destroy(x.p);
  orc_destroy(x.o);
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  const int seeds = argc > 1 ? atoi(argv[1]) : 6;
  const int device = argc > 2 ? atoi(argv[2]) : 0;
  const bool host = argc > 3 && atoi(argv[3]) != 0;
  int passed = 0;
  for (int s = 0; s < seeds; ++s)
    for (int unit = 0; unit < 2; ++unit) {
      const bool ok = run_seed(s, unit != 0, device, host);
      printf("seed %d unit %d: %s\n", s, unit, ok ? "ok" : "FAIL");
      fflush(stdout);
      passed += ok;
    }
  printf("%d/%d sequences equal the oracle, %d failures\n", passed, 2 * seeds, g_fail);
  return g_fail ? 1 : 0;
}
