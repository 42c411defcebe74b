// spf_sweep.hip — all-sources sweeps and the multi-device context
// (include/openr_spf.h, "sweeps" / "devices").
//
// A sweep is runSpf (openr/decision/LinkState.cpp:836-911) for every node of
// the graph, or for one part of a root partition: the reference's
// all-sources use is Decision::getDecisionRouteDb(node) per node
// (openr/decision/Decision.cpp:309) and `breeze decision routes --nodes all`
// (openr/py/openr/cli/commands/decision.py:26-48). The sweep owns what a
// caller would otherwise orchestrate: the path (derive / weighted cover /
// weighted derive / batch), root order and width classes, the row buffers,
// one HIP stream per concurrent launch and the HIP graph a run replays.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <memory>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <new>
#include <numeric>
#include <string>
#include <atomic>
#include <system_error>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "spf_internal.h"

using namespace ospf_int;

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

__global__ void gather_digest_kernel(const ospf_digest* __restrict__ src,
                                     const uint32_t* __restrict__ idx, uint32_t n,
                                     ospf_digest* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[idx[i]];
}

// Empty dispatch queued before each launch unit by ospf_sweep_profile: in a
// rocprofv3 kernel trace or counter collection its dispatches cut the
// profile phase into units (scripts/sweep_unit_stats.py).
__global__ void sweep_unit_mark_kernel(uint32_t unit) { (void)unit; }

__global__ void scatter_digest_kernel(const ospf_digest* __restrict__ src,
                                      const uint32_t* __restrict__ roots, uint32_t n,
                                      ospf_digest* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && roots[i] != kNone) out[roots[i]] = src[i];
}

// ---------------------------------------------------------------- host graph facts
// distinct neighbours (ascending id, links of any state) come from the
// context's host copy (ospf_load_graph: dn_off / dn)
struct Facts {
  uint32_t V = 0;
  const std::vector<uint32_t>* dn_off = nullptr;
  const std::vector<uint32_t>* dn = nullptr;
  uint32_t nbrs(uint32_t v) const { return (*dn_off)[v + 1] - (*dn_off)[v]; }
  // smallest / largest neighbour id (V / 0 for an isolated node)
  uint64_t first(uint32_t v) const { return nbrs(v) ? (*dn)[(*dn_off)[v]] : V; }
  uint64_t last(uint32_t v) const { return nbrs(v) ? (*dn)[(*dn_off)[v + 1] - 1] : 0; }
  // launch class: 8, 16 or 32 x next-hop words (distinct neighbours)
  uint32_t cap(uint32_t v) const {
    const uint32_t k = nbrs(v);
    return k <= 8 ? 8u : k <= 16 ? 16u : 32u * std::max(1u, (k + 31) / 32);
  }
  uint32_t words(uint32_t v) const { return std::max(1u, (nbrs(v) + 31) / 32); }
};

// stable sort on host threads: chunks stable-sorted in parallel, then merged
// pairwise (left run first: stable)
using ospf_int::par_for;

template <class T, class Less>
void par_stable_sort(std::vector<T>& v, Less less) {
  const uint32_t n = (uint32_t)v.size();
  const uint32_t hw = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  uint32_t C = 1;
  while (C * 2 <= hw && n / (C * 2) >= 4096u) C *= 2;
  if (C == 1) {
    std::stable_sort(v.begin(), v.end(), less);
    return;
  }
  std::vector<uint32_t> b(C + 1);
  for (uint32_t k = 0; k <= C; ++k) b[k] = (uint32_t)((uint64_t)n * k / C);
  par_for(C, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t k = lo; k < hi; ++k) std::stable_sort(v.begin() + b[k], v.begin() + b[k + 1], less);
  }, 1);
  std::vector<T> tmp(n);
  for (uint32_t w = 1; w < C; w *= 2) {
    const uint32_t pairs = C / (2 * w);
    par_for(pairs, [&](uint32_t lo, uint32_t hi) {
      for (uint32_t q = lo; q < hi; ++q) {
        const uint32_t a0 = b[2 * q * w], a1 = b[2 * q * w + w], a2 = b[2 * q * w + 2 * w];
        std::merge(v.begin() + a0, v.begin() + a1, v.begin() + a1, v.begin() + a2, tmp.begin() + a0, less);
      }
    }, 1);
    v.swap(tmp);
  }
}

// OSPF_SWEEP_TIMING: sub-phases of a plan phase on stderr
struct SubLaps {
  const char* phase;
  bool on = getenv("OSPF_SWEEP_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  explicit SubLaps(const char* p) : phase(p) {}
  void operator()(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "sweep_create plan/%s/%s %.2f ms\n", phase, what,
            std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

// stable order of `v` by key(v)
template <class K>
void locality_order(std::vector<uint32_t>& v, K key) {
  std::stable_sort(v.begin(), v.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
}

// sorted ids of `roots` and all their neighbours
std::vector<uint32_t> closure(const Facts& f, const std::vector<uint32_t>& roots) {
  std::vector<uint8_t> mark(f.V, 0);
  // (serial: on host threads the marks of shared neighbours -- a pod's
  // fabric switches, marked by all its racks -- contended, 0.8 -> 2.4 ms)
  for (uint32_t r : roots) {
    mark[r] = 1;
    for (uint32_t k = (*f.dn_off)[r]; k < (*f.dn_off)[r + 1]; ++k) mark[(*f.dn)[k]] = 1;
  }
  std::vector<uint32_t> out;
  for (uint32_t v = 0; v < f.V; ++v)
    if (mark[v]) out.push_back(v);
  return out;
}

// [lo, hi) of part p's contiguous share of m items (sizes differ by <= 1)
std::pair<size_t, size_t> part_slice(size_t m, uint32_t parts, uint32_t p) {
  const size_t q = m / parts, r = m % parts;
  const size_t lo = p * q + std::min<size_t>(p, r);
  return {lo, lo + q + (p < r ? 1 : 0)};
}

// The roots of part p: every width class ordered by the node's largest
// neighbour (stable in id order), cut into contiguous slices. On a fabric
// the racks and fabric switches of a pod share their largest neighbour (a
// fabric switch / a rack of the same pod), the spines of a plane too (the
// plane's fabric switch in the last pod by name), so parts are pod and plane
// blocks and a part's closure adds little. Returns the class-major order.
std::vector<uint32_t> partition(const Facts& f, uint32_t parts, uint32_t p) {
  std::vector<uint32_t> all(f.V);
  std::iota(all.begin(), all.end(), 0u);
  if (parts <= 1) return all;
  std::vector<uint32_t> caps;
  for (uint32_t v = 0; v < f.V; ++v) caps.push_back(f.cap(v));
  std::vector<uint32_t> uc = caps;
  std::sort(uc.begin(), uc.end());
  uc.erase(std::unique(uc.begin(), uc.end()), uc.end());
  std::vector<uint32_t> out;
  for (uint32_t cap : uc) {
    std::vector<uint32_t> cls;
    for (uint32_t v = 0; v < f.V; ++v)
      if (caps[v] == cap) cls.push_back(v);
    locality_order(cls, [&](uint32_t v) { return f.last(v); });
    const auto sl = part_slice(cls.size(), parts, p);
    out.insert(out.end(), cls.begin() + sl.first, cls.begin() + sl.second);
  }
  return out;
}

// Independent set of nodes with <= 32 distinct neighbours, greedy in
// (distinct neighbours, id) order: the lexicographically first maximal
// independent set of the candidates under that priority (what Luby rounds
// with a fixed priority also produce). Links of any state count.
std::vector<uint8_t> leaf_set(const Facts& f, uint32_t max_nbrs = 32) {
  // candidates in (distinct neighbours, id) order: a counting sort
  std::vector<uint32_t> cnt(max_nbrs + 2, 0u);
  for (uint32_t v = 0; v < f.V; ++v)
    if (f.nbrs(v) <= max_nbrs) ++cnt[f.nbrs(v) + 1];
  for (uint32_t k = 1; k < cnt.size(); ++k) cnt[k] += cnt[k - 1];
  std::vector<uint32_t> cand(cnt.back());
  for (uint32_t v = 0; v < f.V; ++v)
    if (f.nbrs(v) <= max_nbrs) cand[cnt[f.nbrs(v)]++] = v;
  std::vector<uint8_t> leaf(f.V, 0), blocked(f.V, 0);
  for (uint32_t v : cand) {
    if (blocked[v]) continue;
    leaf[v] = 1;
    for (uint32_t k = (*f.dn_off)[v]; k < (*f.dn_off)[v + 1]; ++k) blocked[(*f.dn)[k]] = 1;
  }
  return leaf;
}

}  // namespace

// ---------------------------------------------------------------- the sweep
struct ospf_sweep {
  ospf_ctx* c = nullptr;
  ospf_sweep_opts opts{};
  uint32_t mode = 0;
  uint64_t gen = 0;
  std::string err;
  uint32_t V = 0;
  std::vector<uint32_t> roots;          // owned roots, digest order
  std::vector<uint32_t> own_slot;       // digest slot of roots[i] in dig_all
  // row of each owned root: device pointers, by node id (null: not owned)
  std::vector<const uint32_t*> row_dist, row_nh;
  std::vector<uint32_t> row_w;
  std::vector<void*> allocs;            // device allocations
  std::vector<size_t> alloc_bytes;      // their sizes (returned to the ctx's pool)
  uint64_t device_bytes = 0;
  ospf_digest* dig_all = nullptr;       // every digest a run writes
  uint32_t n_dig = 0;
  std::vector<std::pair<ospf_digest*, size_t>> dig_aux;  // intermediate digests (poisoned too)
  uint32_t* d_own_slot = nullptr;
  uint32_t n_rows = 0;
  uint64_t trav_edges = 0;  // edges scanned by the run's traversal kernels (TEPS)
  uint64_t step_comp = 0;
  // launches
  struct Unit {
    std::string name, kernel;
    int stream = 0;            // index into streams (0 = main)
    std::vector<int> wait;     // events waited for before the launch
    int record = -1;           // event recorded after it
    std::function<int(hipStream_t)> fn;
    uint32_t n_roots = 0, W = 0;
    uint64_t comp = 0;
  };
  std::vector<Unit> units;
  std::vector<hipStream_t> streams;     // [0] = main
  std::vector<hipEvent_t> events;       // [0] = run start
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  std::vector<hipEvent_t> ev_done;      // per non-main stream
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  bool ran = false;
  // OSPF_SWEEP_EARLY_START: units [0, started) of the first run already
  // queued by the plan (after ev_in on the null stream and events[0])
  bool early = false, early_on = false;
  size_t started = 0;
  // block order of the leaf launch (0 chunk-major, 1 group-major): picked at
  // create by timing both -- which order stores faster depends on where the
  // allocation's rows fall in the memory channels (the probe's two patterns
  // swap places from one allocation to the next)
  int leaf_order = 0;
  // the seed BFS's deepest level in the first run (device word), and the
  // level launches the HIP graph captures (0: the graph's transit-depth bound)
  uint32_t* d_lv_maxd = nullptr;
  uint32_t lv_cap = 0;
};

namespace {

int sfail(ospf_sweep* s, int code, const std::string& m) {
  s->err = m;
  if (s->c) s->c->err = m;
  return code;
}

int start_early(ospf_sweep* s);  // (below: OSPF_SWEEP_EARLY_START)

#define SCHK(sw, call)                                                               \
  do {                                                                               \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess)                                                            \
      return sfail(sw, OSPF_E_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

template <class T>
int dalloc(ospf_sweep* s, T** p, size_t count) {
  void* q = nullptr;
  const size_t want = std::max<size_t>(count, 1) * sizeof(T);
  // a block of a destroyed sweep, at most 1/8 larger (+ 1 MB), else new
  ospf_ctx* c = s->c;
  size_t bytes = (want + 255) & ~(size_t)255;
  auto it = c->sweep_pool.lower_bound(bytes);
  if (it != c->sweep_pool.end() && it->first <= bytes + bytes / 8 + (1u << 20)) {
    q = it->second;
    bytes = it->first;
    c->sweep_pool_bytes -= bytes;
    c->sweep_pool.erase(it);
  } else {
    const hipError_t e = ospf_int::dev_malloc(c, &q, bytes);  // frees the pool on failure
    if (e != hipSuccess)
      return sfail(s, OSPF_E_NOMEM, "sweep: hipMalloc " + std::to_string(bytes) + " B: " +
                                        hipGetErrorString(e));
  }
  s->allocs.push_back(q);
  s->alloc_bytes.push_back(bytes);
  s->device_bytes += bytes;
  *p = (T*)q;
  return OSPF_OK;
}

// dalloc without an error message (a caller that retries smaller)
template <class T>
int dalloc_try(ospf_sweep* s, T** p, size_t count) {
  const std::string keep = s->err, keep_c = s->c ? s->c->err : std::string();
  const int rc = dalloc(s, p, count);
  if (rc) {
    s->err = keep;
    if (s->c) s->c->err = keep_c;
  }
  return rc;
}

template <class T>
int upload(ospf_sweep* s, T** p, const std::vector<T>& h) {
  int rc = dalloc(s, p, h.size());
  if (rc) return rc;
  if (!h.empty()) SCHK(s, hipMemcpy(*p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return OSPF_OK;
}

int new_stream(ospf_sweep* s) {
  hipStream_t st;
  if (!s->c->stream_pool.empty()) {
    st = s->c->stream_pool.back();
    s->c->stream_pool.pop_back();
  } else {
    SCHK(s, hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  }
  s->streams.push_back(st);
  return (int)s->streams.size() - 1;
}

int new_event(ospf_sweep* s) {
  hipEvent_t e;
  if (!s->c->event_pool.empty()) {
    e = s->c->event_pool.back();
    s->c->event_pool.pop_back();
  } else {
    SCHK(s, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  s->events.push_back(e);
  return (int)s->events.size() - 1;
}

// Row pitch (u32 words) of the sweep's dist / one-word next-hop rows: V
// rounded up to 32 words (128-B aligned rows) when V is a multiple of 4 (the
// 16-B store path); OSPF_SWEEP_ROW_PITCH=V keeps the packed pitch (A/B knob)
uint32_t row_pitch(uint32_t V) {
  if (V & 3u) return V;
  if (const char* e = getenv("OSPF_SWEEP_ROW_PITCH"))
    if (e[0] == 'V') return V;
  return (V + 31u) / 32u * 32u;
}

// CSR bytes one distance-only scan reads: neighbour ids + row offsets
uint64_t scan_bytes(const ospf_ctx* c, bool weighted) {
  return (uint64_t)(weighted ? 8 : 4) * c->info.n_edges + 4ull * (c->info.n_nodes + 1);
}

// owned root r's digest is slot `slot` of dig_all; its rows are (d, nh, W)
void own(ospf_sweep* s, uint32_t r, uint32_t slot, const uint32_t* d, const uint32_t* nh,
         uint32_t W) {
  s->roots.push_back(r);
  s->own_slot.push_back(slot);
  s->row_dist[r] = d;
  s->row_nh[r] = nh;
  s->row_w[r] = W;
}

// ---------------------------------------------------------------- plans
// Usable-slot signature of a leaf root (bit k: an up link to its k-th
// distinct neighbour), from the context's padded host shadows.
uint32_t usable_slots(const ospf_ctx* c, uint32_t r) {
  uint32_t use = 0;
  const uint32_t* dn = c->h_dn.data() + c->h_dn_off[r];
  const uint32_t K = c->h_dn_off[r + 1] - c->h_dn_off[r];
  for (uint32_t e = c->h_prow[r]; e < c->h_prow[r + 1]; ++e) {
    const uint32_t cx = c->h_pcolx[e];
    if ((cx & 0x80000000u) || cx == r) continue;
    const uint32_t k = (uint32_t)(std::lower_bound(dn, dn + K, cx) - dn);
    if (k < 32u) use |= 1u << k;
  }
  return use;
}

// Leaf roots ordered so that roots with the same slot table (distinct
// neighbours + usable links: the racks of a pod) are adjacent, cut into
// groups of <= kLeafMaxG; returns the group offsets.
std::vector<uint32_t> leaf_groups(const ospf_ctx* c, const Facts& f, std::vector<uint32_t>& roots) {
  SubLaps lap("leaf groups");
  std::vector<uint32_t> use(roots.size());
  par_for((uint32_t)roots.size(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) use[i] = usable_slots(c, roots[i]);
  });
  std::vector<uint32_t> ord(roots.size());
  std::iota(ord.begin(), ord.end(), 0u);
  auto same_nbrs = [&](uint32_t a, uint32_t b) {
    return f.nbrs(a) == f.nbrs(b) &&
           std::equal(f.dn->begin() + (*f.dn_off)[a], f.dn->begin() + (*f.dn_off)[a + 1],
                      f.dn->begin() + (*f.dn_off)[b]);
  };
  par_stable_sort(ord, [&](uint32_t x, uint32_t y) {
    const uint32_t a = roots[x], b = roots[y];
    if (f.nbrs(a) != f.nbrs(b)) return f.first(a) != f.first(b) ? f.first(a) < f.first(b)
                                                                 : f.nbrs(a) < f.nbrs(b);
    const int cmp = std::lexicographical_compare(
                        f.dn->begin() + (*f.dn_off)[a], f.dn->begin() + (*f.dn_off)[a + 1],
                        f.dn->begin() + (*f.dn_off)[b], f.dn->begin() + (*f.dn_off)[b + 1])
                        ? -1
                        : (same_nbrs(a, b) ? 0 : 1);
    if (cmp) return cmp < 0;
    return use[x] < use[y];
  });
  lap("sort");
  std::vector<uint32_t> out(roots.size()), uo(roots.size());
  for (size_t i = 0; i < ord.size(); ++i) {
    out[i] = roots[ord[i]];
    uo[i] = use[ord[i]];
  }
  roots.swap(out);
  std::vector<uint32_t> grp{0u};
  for (uint32_t i = 1; i <= roots.size(); ++i) {
    const uint32_t g0 = grp.back();
    if (i == roots.size() || i - g0 >= ospf::kLeafMaxG || uo[i] != uo[g0] ||
        !same_nbrs(roots[i], roots[g0]))
      grp.push_back(i);
  }
  return grp;
}

// Twin classes (spf_twin.hip): nodes with the same usable distinct
// neighbours and the same transit bit. cls[v] = class id, rep / sec = the
// smallest two members of each class (sec = kNone for a class of one).
struct Twins {
  std::vector<uint32_t> cls, rep, sec;
};
Twins twin_classes(const ospf_ctx* c) {
  SubLaps lap("twin classes");
  const uint32_t V = c->info.n_nodes;
  std::vector<uint32_t> off(V + 1, 0);
  std::vector<uint64_t> key(V);
  // each node's usable distinct neighbours (sorted, unique): counted, then
  // written and hashed, both on host threads
  auto nbrs_of = [&](uint32_t u, uint32_t* out) {  // -> count (out may be null)
    uint32_t m = 0, prev = 0xFFFFFFFFu;
    bool sorted = true;
    for (uint32_t e = c->h_prow[u]; e < c->h_prow[u + 1]; ++e) {
      const uint32_t x = c->h_pcolx[e];
      if ((x & 0x80000000u) || x == u || x == prev) continue;
      sorted &= prev == 0xFFFFFFFFu || x > prev;
      if (out) out[m] = x;
      prev = x;
      ++m;
    }
    if (out && !sorted) {  // (rows are sorted by neighbour id; kept exact either way)
      std::sort(out, out + m);
      m = (uint32_t)(std::unique(out, out + m) - out);
    }
    return m;
  };
  std::vector<uint32_t> cnt(V);
  ospf_int::par_for_rows(V, c->h_prow.data(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t u = lo; u < hi; ++u) cnt[u] = nbrs_of(u, nullptr);
  });
  for (uint32_t u = 0; u < V; ++u) off[u + 1] = off[u] + cnt[u];
  // (uninitialized: every slot is written below; a zero fill of ~10 MB of
  // fresh pages cost more than the pass)
  std::unique_ptr<uint32_t[]> lst_buf(new uint32_t[std::max<uint32_t>(off[V], 1)]);
  uint32_t* const lst = lst_buf.get();
  ospf_int::par_for_rows(V, c->h_prow.data(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t u = lo; u < hi; ++u) {
      const uint32_t m = nbrs_of(u, lst + off[u]);
      for (uint32_t i = m; i < cnt[u]; ++i) lst[off[u] + i] = 0xFFFFFFFFu;  // (dups of an unsorted row)
      cnt[u] = m;
      const bool tr = !((c->h_nt[u >> 5] >> (u & 31)) & 1u);
      // (independent mixes, summed: no dependent chain through a spine's row;
      // a hash only -- classes are split by exact equality below)
      uint64_t h = tr ? 0x9E3779B97F4A7C15ull : 0xC2B2AE3D27D4EB4Full;
      for (uint32_t i = 0; i < m; ++i) h += ospf::digest_mix(lst[off[u] + i] ^ (i * 0x9E3779B97F4A7C15ull));
      key[u] = h;
    }
  });
  lap("lists + keys");
  auto same = [&](uint32_t a, uint32_t b) {
    const bool ta = !((c->h_nt[a >> 5] >> (a & 31)) & 1u), tb = !((c->h_nt[b >> 5] >> (b & 31)) & 1u);
    return ta == tb && cnt[a] == cnt[b] &&
           std::equal(lst + off[a], lst + off[a] + cnt[a], lst + off[b]);
  };
  // nodes by (key, id): the stable order by key
  std::vector<std::pair<uint64_t, uint32_t>> kv(V);
  for (uint32_t u = 0; u < V; ++u) kv[u] = {key[u], u};
  par_stable_sort(kv, [](const std::pair<uint64_t, uint32_t>& x, const std::pair<uint64_t, uint32_t>& y) {
    return x < y;
  });
  std::vector<uint32_t> ord(V);
  for (uint32_t u = 0; u < V; ++u) ord[u] = kv[u].second;
  lap("key sort");
  Twins t;
  t.cls.assign(V, kNone);
  for (size_t i = 0; i < V;) {
    size_t j = i;
    while (j < V && key[ord[j]] == key[ord[i]]) ++j;
    // within a hash run, split by exact equality (collisions are rare)
    for (size_t p = i; p < j; ++p) {
      const uint32_t u = ord[p];
      if (t.cls[u] != kNone) continue;
      const uint32_t id = (uint32_t)t.rep.size();
      t.rep.push_back(u);
      t.sec.push_back(kNone);
      t.cls[u] = id;
      for (size_t q = p + 1; q < j; ++q) {
        const uint32_t w = ord[q];
        if (t.cls[w] != kNone || !same(u, w)) continue;
        t.cls[w] = id;
      }
    }
    i = j;
  }
  lap("classes");
  // representative = smallest member, second = the next one
  for (uint32_t u = 0; u < V; ++u) {
    const uint32_t id = t.cls[u];
    if (u < t.rep[id]) {
      t.sec[id] = t.rep[id];
      t.rep[id] = u;
    } else if (u != t.rep[id] && (t.sec[id] == kNone || u < t.sec[id])) {
      t.sec[id] = u;
    }
  }
  return t;
}

// Host plan of the wide next-hop kernel (nh_wide_plan_kernel) for a class
// of roots (in order): runs of <= kWideG roots with the same distinct
// neighbours, each run's slot table over level-row positions, each root's
// usable-slot words.
struct WideHost {
  std::vector<uint32_t> run, soff, slots, keep, own;
};
int wide_plan_build(ospf_ctx* c, const Facts& f, const std::vector<uint32_t>& roots, uint32_t W,
                    const std::vector<uint32_t>& pos, WideHost& h) {
  const uint32_t n = (uint32_t)roots.size();
  h = WideHost{};
  h.keep.assign((size_t)n * W, 0u);
  auto same = [&](uint32_t a, uint32_t b) {
    return f.nbrs(a) == f.nbrs(b) &&
           std::equal(f.dn->begin() + (*f.dn_off)[a], f.dn->begin() + (*f.dn_off)[a + 1],
                      f.dn->begin() + (*f.dn_off)[b]);
  };
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t r = roots[i];
    if (pos[r] == kNone) return fail(c, OSPF_E_RANGE, "wide plan: a root without a level row");
    if (f.nbrs(r) > 32u * W || f.nbrs(r) > 2048u) return fail(c, OSPF_E_RANGE, "wide plan: too many neighbours");
    h.own.push_back(pos[r]);
  }
  // each root's usable slots, on host threads (rows ascend by neighbour id:
  // a cursor over the distinct neighbours, a search only if one is missed)
  par_for(n, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) {
      const uint32_t r = roots[i];
      const uint32_t* dn = f.dn->data() + (*f.dn_off)[r];
      const uint32_t K = f.nbrs(r);
      uint32_t k = 0;
      for (uint32_t e = c->h_prow[r]; e < c->h_prow[r + 1]; ++e) {
        const uint32_t x = c->h_pcolx[e];
        if ((x & 0x80000000u) || x == r) continue;
        while (k < K && dn[k] < x) ++k;
        if (k >= K || dn[k] != x) k = (uint32_t)(std::lower_bound(dn, dn + K, x) - dn);
        h.keep[(size_t)i * W + (k >> 5)] |= 1u << (k & 31u);
      }
    }
  }, 16);
  for (uint32_t i = 0; i < n; ++i)
    if (i == 0 || i - h.run.back() >= 64u || !same(roots[h.run.back()], roots[i])) h.run.push_back(i);
  h.run.push_back(n);
  h.soff.push_back(0u);
  for (size_t q = 0; q + 1 < h.run.size(); ++q) {
    const uint32_t r0 = roots[h.run[q]], K = f.nbrs(r0);
    const uint32_t* dn = f.dn->data() + (*f.dn_off)[r0];
    for (uint32_t k = 0; k < K; ++k) {
      bool used = false;
      for (uint32_t i = h.run[q]; i < h.run[q + 1] && !used; ++i)
        used = (h.keep[(size_t)i * W + (k >> 5)] >> (k & 31u)) & 1u;
      uint32_t v = kNone;
      if (used) {
        const uint32_t x = dn[k];
        if ((c->h_nt[x >> 5] >> (x & 31)) & 1u) {
          v = 0x80000000u | x;
        } else {
          v = pos[x];
          if (v == kNone) return fail(c, OSPF_E_RANGE, "wide plan: a neighbour without a level row");
        }
      }
      h.slots.push_back(v);
    }
    h.soff.push_back((uint32_t)h.slots.size());
  }
  return OSPF_OK;
}

// Host plan of the weighted run kernel (wnh_runs_kernel) for wide cover
// roots (in order): runs of <= kWrRun roots with the same distinct
// neighbours; per run its slot table over dist-row positions (padded to 32 W),
// per root the smallest metric of its up links per slot.
struct WRunsHost {
  std::vector<uint4> run;
  std::vector<uint32_t> slots, wt, own, rootid;
};
int wruns_build(ospf_ctx* c, const Facts& f, const std::vector<uint32_t>& roots, uint32_t W,
                const std::vector<uint32_t>& pos, WRunsHost& h) {
  const uint32_t n = (uint32_t)roots.size(), KW = 32u * W;
  h = WRunsHost{};
  h.wt.assign((size_t)n * KW, kNone);
  auto same = [&](uint32_t a, uint32_t b) {
    return f.nbrs(a) == f.nbrs(b) &&
           std::equal(f.dn->begin() + (*f.dn_off)[a], f.dn->begin() + (*f.dn_off)[a + 1],
                      f.dn->begin() + (*f.dn_off)[b]);
  };
  std::vector<uint32_t> first;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t r = roots[i];
    if (pos[r] == kNone) return fail(c, OSPF_E_RANGE, "wruns plan: a root without a row");
    h.own.push_back(pos[r]);
    h.rootid.push_back(r);
    const uint32_t* dn = f.dn->data() + (*f.dn_off)[r];
    const uint32_t K = f.nbrs(r);
    if (K > KW) return fail(c, OSPF_E_RANGE, "wruns plan: too many neighbours");
    for (uint32_t e = c->h_prow[r]; e < c->h_prow[r + 1]; ++e) {
      const uint32_t x = c->h_pcolx[e];
      if ((x & 0x80000000u) || x == r) continue;
      const uint32_t k = (uint32_t)(std::lower_bound(dn, dn + K, x) - dn);
      uint32_t& m = h.wt[(size_t)i * KW + k];
      m = std::min(m, c->h_pw[e]);
    }
    if (i == 0 || i - first.back() >= ospf::kWrRun || !same(roots[first.back()], r)) first.push_back(i);
  }
  first.push_back(n);
  for (size_t q = 0; q + 1 < first.size(); ++q) {
    const uint32_t r0 = roots[first[q]], K = f.nbrs(r0);
    const uint32_t* dn = f.dn->data() + (*f.dn_off)[r0];
    const uint32_t off = (uint32_t)h.slots.size();
    for (uint32_t k = 0; k < KW; ++k) {
      bool used = false;
      for (uint32_t i = first[q]; i < first[q + 1] && k < K && !used; ++i)
        used = h.wt[(size_t)i * KW + k] != kNone;
      uint32_t v = kNone;
      if (used) {
        const uint32_t x = dn[k];
        if ((c->h_nt[x >> 5] >> (x & 31)) & 1u) {
          v = 0x80000000u | x;
        } else {
          v = pos[x];
          if (v == kNone) return fail(c, OSPF_E_RANGE, "wruns plan: a neighbour without a row");
        }
      }
      h.slots.push_back(v);
    }
    h.run.push_back(make_uint4(first[q], first[q + 1] - first[q], off, 0u));
  }
  return OSPF_OK;
}

// Host plan of the weighted hub kernel (wnh_hub_kernel) for narrow cover
// roots (W <= 4, in order): hub rows = the transit neighbours most roots read
// (>= 16 roots, at most kHubMax, most-read first); groups = runs of <= 16
// consecutive roots whose own rows plus non-hub transit neighbours' rows
// number <= kHubLoc. OSPF_E_RANGE when a root alone needs more group rows.
struct HubHost {
  std::vector<uint32_t> hub, loc, ref, wt, ownl, rootid;
  std::vector<uint4> grp;
};
int hub_build(ospf_ctx* c, const Facts& f, const std::vector<uint32_t>& roots, uint32_t W,
              const std::vector<uint32_t>& pos, HubHost& h) {
  const uint32_t n = (uint32_t)roots.size(), KW = 32u * W, V = f.V;
  h = HubHost{};
  h.wt.assign((size_t)n * KW, kNone);
  auto nt = [&](uint32_t x) { return (c->h_nt[x >> 5] >> (x & 31)) & 1u; };
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t r = roots[i];
    const uint32_t* dn = f.dn->data() + (*f.dn_off)[r];
    const uint32_t K = f.nbrs(r);
    if (K > KW) return fail(c, OSPF_E_RANGE, "hub plan: too many neighbours");
    for (uint32_t e = c->h_prow[r]; e < c->h_prow[r + 1]; ++e) {
      const uint32_t x = c->h_pcolx[e];
      if ((x & 0x80000000u) || x == r) continue;
      const uint32_t k = (uint32_t)(std::lower_bound(dn, dn + K, x) - dn);
      uint32_t& m = h.wt[(size_t)i * KW + k];
      m = std::min(m, c->h_pw[e]);
    }
  }
  std::vector<uint32_t> cnt(V, 0u);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t r = roots[i];
    const uint32_t* dn = f.dn->data() + (*f.dn_off)[r];
    for (uint32_t k = 0; k < f.nbrs(r); ++k)
      if (h.wt[(size_t)i * KW + k] != kNone && !nt(dn[k])) ++cnt[dn[k]];
  }
  std::vector<uint32_t> cand;
  for (uint32_t v = 0; v < V; ++v)
    if (cnt[v] >= 16u) cand.push_back(v);
  std::stable_sort(cand.begin(), cand.end(), [&](uint32_t a, uint32_t b) { return cnt[a] > cnt[b]; });
  if (cand.size() > ospf::kHubMax) cand.resize(ospf::kHubMax);
  std::vector<uint32_t> hub_of(V, kNone);
  for (uint32_t j = 0; j < cand.size(); ++j) {
    hub_of[cand[j]] = j;
    if (pos[cand[j]] == kNone) return fail(c, OSPF_E_RANGE, "hub plan: a neighbour without a row");
    h.hub.push_back(pos[cand[j]]);
  }
  std::vector<uint32_t> locs;  // the open group's row nodes
  auto need = [&](uint32_t i, std::vector<uint32_t>& out) {
    const uint32_t r = roots[i];
    const uint32_t* dn = f.dn->data() + (*f.dn_off)[r];
    out.assign(1, r);
    for (uint32_t k = 0; k < f.nbrs(r); ++k)
      if (h.wt[(size_t)i * KW + k] != kNone && (nt(dn[k]) || hub_of[dn[k]] == kNone))
        out.push_back(nt(dn[k]) && dn[k] != r ? (0x80000000u | dn[k]) : dn[k]);
  };
  auto close = [&](uint32_t first, uint32_t end) {
    h.grp.push_back(make_uint4(first, end - first, (uint32_t)h.loc.size(), (uint32_t)locs.size()));
    for (uint32_t x : locs) {
      if (x & 0x80000000u) {
        h.loc.push_back(x);
        continue;
      }
      if (pos[x] == kNone) return false;
      h.loc.push_back(pos[x]);
    }
    return true;
  };
  std::vector<uint32_t> nd;
  uint32_t gfirst = 0;
  for (uint32_t i = 0; i < n; ++i) {
    need(i, nd);
    std::vector<uint32_t> merged = locs;
    for (uint32_t x : nd)
      if (std::find(merged.begin(), merged.end(), x) == merged.end()) merged.push_back(x);
    if (i > gfirst && (merged.size() > ospf::kHubLoc || i - gfirst >= ospf::kHubGrpRoots)) {
      if (!close(gfirst, i)) return fail(c, OSPF_E_RANGE, "hub plan: a row is missing");
      gfirst = i;
      locs.clear();
      merged.clear();
      for (uint32_t x : nd)
        if (std::find(merged.begin(), merged.end(), x) == merged.end()) merged.push_back(x);
    }
    if (merged.size() > ospf::kHubLoc) return fail(c, OSPF_E_RANGE, "hub plan: a root needs > 64 group rows");
    locs = merged;
  }
  if (n && !close(gfirst, n)) return fail(c, OSPF_E_RANGE, "hub plan: a row is missing");
  // slot refs and own rows per root
  h.ref.assign((size_t)n * KW, kNone);
  for (const uint4& gr : h.grp) {
    const uint32_t* L = h.loc.data() + gr.z;
    const uint32_t nhub = (uint32_t)h.hub.size();
    for (uint32_t i = gr.x; i < gr.x + gr.y; ++i) {
      const uint32_t r = roots[i];
      const uint32_t* dn = f.dn->data() + (*f.dn_off)[r];
      auto lidx = [&](uint32_t tag) {  // src row or 0x80000000 | node
        for (uint32_t l = 0; l < gr.w; ++l)
          if (L[l] == tag) return nhub + l;
        return kNone;
      };
      h.ownl.push_back(lidx(pos[r]));
      h.rootid.push_back(r);
      for (uint32_t k = 0; k < KW; ++k) {
        uint32_t& rf = h.ref[(size_t)i * KW + k];
        rf = nhub + ospf::kHubLoc;  // the unreached row
        if (k >= f.nbrs(r) || h.wt[(size_t)i * KW + k] == kNone) continue;
        const uint32_t x = dn[k];
        if (nt(x) && x != r) rf = lidx(0x80000000u | x);
        else if (hub_of[x] != kNone) rf = hub_of[x];
        else rf = lidx(pos[x]);
        if (rf == kNone) return fail(c, OSPF_E_RANGE, "hub plan: a slot row is missing");
      }
    }
  }
  return OSPF_OK;
}

// DERIVE (spf_levels.hip, spf_twin.hip, spf_leaf.hip, spf_msbfs.hip derive
// kernels), unit metric / hop count. The part's roots split into leaves (an
// independent set of nodes with <= 32 distinct neighbours: a fabric's racks)
// and the cover.
// (A) levels: the distance-only 128-root BFS for the seed rows -- the cover
//     rows the part needs (its cover roots, their neighbours, the leaves'
//     neighbours) that no twin class derives, plus the leaf representatives
//     of the classes the derived rows and the twin next-hop launches read --
//     ordered by each node's smallest neighbour so a traversal shares frontiers;
// (A') twin levels: the other cover rows from the representative rows of
//     their neighbours' twin classes (ospf_twin_levels_dev: a fabric switch
//     from one rack row of its pod and one spine row of its plane), no
//     traversal; without twins every cover row is a BFS row and the leaf
//     representatives come first in (B) instead;
// (B) the leaves' level, dist and next-hop rows from their neighbours' level
//     rows (next-hop rows only for BFS'd representatives), groups of leaves
//     with one slot table reading each tile once;
// (C) one next-hop launch per width class of cover roots, roots ordered by
//     their largest neighbour (their neighbours' level rows stay in L2 / MALL),
//     on their own streams beside (B).
// OSPF_SWEEP_TIMING: host phases of a plan on stderr
struct PlanLaps {
  bool on = getenv("OSPF_SWEEP_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void operator()(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "sweep_create plan/%s %.2f ms\n", what,
            std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

int plan_derive(ospf_sweep* s, const Facts& f, const std::vector<uint32_t>& mine) {
  ospf_ctx* c = s->c;
  const uint32_t V = s->V;
  const uint32_t hop = s->opts.flags & OSPF_HOP_COUNT;
  PlanLaps lap;
  double leaf_tail = 0.0;
  if (const char* x = getenv("OSPF_SWEEP_LEAF_TAIL")) leaf_tail = std::max(0.0, std::min(0.9, atof(x)));
  std::vector<uint8_t> leaf;
  if (!getenv("OSPF_SWEEP_NOLEAF")) leaf = leaf_set(f);
  else leaf.assign(V, 0);
  lap("leaf set");
  std::vector<uint32_t> own_l, own_c;
  for (uint32_t r : mine) (leaf[r] ? own_l : own_c).push_back(r);
  // leaves whose rows the cover roots' next hops read
  const std::vector<uint32_t> nb_c = closure(f, own_c);
  std::vector<uint8_t> in_l(V, 0);
  for (uint32_t r : own_l) in_l[r] = 1;
  std::vector<uint32_t> extra_l;
  for (uint32_t v : nb_c)
    if (leaf[v] && !in_l[v]) extra_l.push_back(v);
  lap("closure");
  // cover classes by capacity, roots by largest neighbour
  std::vector<uint32_t> caps;
  for (uint32_t r : own_c) caps.push_back(f.cap(r));
  std::sort(caps.begin(), caps.end());
  caps.erase(std::unique(caps.begin(), caps.end()), caps.end());
  struct Cls {
    uint32_t cap, W;
    std::vector<uint32_t> roots;
    bool twin = false, reads_leaf = false;
  };
  std::vector<Cls> cls;
  for (uint32_t cap : caps) {
    Cls k{cap, cap > 16 ? cap / 32 : 1u, {}};
    for (uint32_t r : own_c)
      if (f.cap(r) == cap) k.roots.push_back(r);
    locality_order(k.roots, [&](uint32_t v) { return f.last(v); });
    for (uint32_t r : k.roots)
      for (uint32_t q = (*f.dn_off)[r]; q < (*f.dn_off)[r + 1] && !k.reads_leaf; ++q)
        k.reads_leaf = leaf[(*f.dn)[q]] != 0;
    cls.push_back(std::move(k));
  }
  // twin classes: a class of <= 4-word roots whose usable transit
  // neighbours span few classes reads one row per class (spf_twin.hip), and
  // so can a cover row (twin levels)
  lap("width classes");
  Twins tw;
  if (!getenv("OSPF_SWEEP_NOTWIN")) tw = twin_classes(c);
  lap("twin classes");
  // classes of r's usable transit neighbours (sorted, unique); false past
  // kTwinMaxC. Every node's, once, on host threads: [V][kTwinMaxC + 1] slots
  // and a count (kTwinMaxC + 1: more)
  constexpr uint32_t kCS = ospf::kTwinMaxC + 1;
  std::vector<uint32_t> ccls, ccnt;
  if (!tw.cls.empty()) {
    ccls.resize((size_t)V * kCS);
    ccnt.resize(V);
    ospf_int::par_for_rows(V, c->h_prow.data(), [&](uint32_t lo, uint32_t hi) {
      std::vector<uint32_t> b;
      for (uint32_t r = lo; r < hi; ++r) {
        // distinct classes, sorted; stops at kCS of them (more is "too many")
        b.clear();
        for (uint32_t e = c->h_prow[r]; e < c->h_prow[r + 1] && b.size() < kCS; ++e) {
          const uint32_t x = c->h_pcolx[e];
          if ((x & 0x80000000u) || x == r || ((c->h_nt[x >> 5] >> (x & 31)) & 1u)) continue;
          const uint32_t k = tw.cls[x];
          const auto it = std::lower_bound(b.begin(), b.end(), k);
          if (it == b.end() || *it != k) b.insert(it, k);
        }
        const uint32_t m = std::min<uint32_t>((uint32_t)b.size(), kCS);
        std::copy(b.begin(), b.begin() + m, ccls.begin() + (size_t)r * kCS);
        ccnt[r] = m;
      }
    });
  }
  std::vector<uint32_t> cs;
  auto classes_of = [&](uint32_t r) {
    cs.assign(ccls.begin() + (size_t)r * kCS, ccls.begin() + (size_t)r * kCS + ccnt[r]);
    return cs.size() <= ospf::kTwinMaxC;
  };
  auto twin_ok = [&](const std::vector<uint32_t>& roots) {
    uint64_t slots = 0, classes = 0;
    for (uint32_t r : roots) {
      if (!classes_of(r)) return false;
      slots += f.nbrs(r);
      classes += cs.size();
    }
    // worth it when a class covers several slots (OSPF_SWEEP_TWIN=1: always)
    return getenv("OSPF_SWEEP_TWIN") || slots >= 3 * std::max<uint64_t>(1, classes);
  };
  bool all_leaf_rows = false;  // a class reads every neighbour's row (not twins)
  for (auto& k : cls) {
    k.twin = k.W <= 4 && !tw.cls.empty() && twin_ok(k.roots);
    if (k.reads_leaf && !k.twin) all_leaf_rows = true;
  }
  all_leaf_rows |= tw.cls.empty() || getenv("OSPF_SWEEP_ALL_LEAF_ROWS") != nullptr;
  lap("twin width classes");
  std::vector<uint32_t> need_l = own_l;
  need_l.insert(need_l.end(), extra_l.begin(), extra_l.end());
  // cover rows: own cover roots + every non-leaf neighbour of a needed root
  std::vector<uint8_t> in_a(V, 0);
  for (uint32_t v : own_c) in_a[v] = 1;
  for (uint32_t v : closure(f, need_l))
    if (!leaf[v]) in_a[v] = 1;
  for (uint32_t v : nb_c)
    if (!leaf[v]) in_a[v] = 1;
  uint32_t n_cover = 0;
  for (uint32_t v = 0; v < V; ++v) n_cover += in_a[v];
  // (A') cover rows derived from twin classes; their classes' representatives
  // are BFS rows (a derived representative leaves the set: repeat until
  // stable), and so are the leaf representatives the twin next hops read
  std::vector<uint8_t> in_d(V, 0), seed(V, 0);
  bool twin_lv = !tw.cls.empty() && !getenv("OSPF_SWEEP_NOTWINLV");
  if (twin_lv) {
    for (uint32_t v = 0; v < V; ++v)
      if (in_a[v] && f.nbrs(v) <= 128 && classes_of(v)) in_d[v] = 1;
    for (bool changed = true; changed;) {
      changed = false;
      for (uint32_t v = 0; v < V; ++v) {
        if (!in_d[v]) continue;
        classes_of(v);
        for (uint32_t k : cs)
          if (in_d[tw.rep[k]]) {
            in_d[tw.rep[k]] = 0;
            changed = true;
          }
      }
    }
    auto seed_reps = [&](uint32_t v) {
      classes_of(v);
      for (uint32_t k : cs)
        if (leaf[tw.rep[k]]) seed[tw.rep[k]] = 1;
    };
    for (uint32_t v = 0; v < V; ++v)
      if (in_d[v]) seed_reps(v);
    for (auto& k : cls)
      if (k.twin)
        for (uint32_t r : k.roots) seed_reps(r);
    uint32_t nbfs = 0;
    for (uint32_t v = 0; v < V; ++v) nbfs += (in_a[v] && !in_d[v]) || seed[v];
    // worth it when the traversal shrinks to half (OSPF_SWEEP_TWINLV=1: always)
    if (!getenv("OSPF_SWEEP_TWINLV") && 2ull * nbfs > n_cover) twin_lv = false;
    if (!twin_lv) {
      std::fill(in_d.begin(), in_d.end(), 0);
      std::fill(seed.begin(), seed.end(), 0);
    }
  }
  // leaves: with twin levels, BFS'd representatives first (next-hop rows
  // only), then the others; without, when only twin representatives' level
  // rows are read, the representatives go first in a launch of their own,
  // so the next hops of the cover roots start while the other leaves' rows
  // are written
  lap("cover rows + twin levels set");
  // (OSPF_SWEEP_MERGE_REPS: the BFS'd leaf representatives' next hops in
  // their groups' leaf launch -- rows re-derived there, identical -- instead
  // of a launch of their own that reads each one's neighbour rows alone)
  const bool merge_reps = twin_lv && getenv("OSPF_SWEEP_MERGE_REPS") != nullptr;
  std::vector<uint32_t> reps, rest;
  for (uint32_t x : need_l) {
    const bool first = twin_lv ? (seed[x] != 0 && !merge_reps)
                               : (!all_leaf_rows && tw.rep[tw.cls[x]] == x);
    (first ? reps : rest).push_back(x);
  }
  std::vector<uint32_t> grp_r = leaf_groups(c, f, reps);
  std::vector<uint32_t> grp = leaf_groups(c, f, rest);
  lap("leaf groups");
  need_l = reps;
  need_l.insert(need_l.end(), rest.begin(), rest.end());
  const uint32_t nR = (uint32_t)reps.size(), nL = (uint32_t)need_l.size();
  // rows: BFS rows (cover rows not derived + seed leaves), derived cover
  // rows, then the leaves that are not BFS rows
  std::vector<uint32_t> clo, drv;
  for (uint32_t v = 0; v < V; ++v) {
    if ((in_a[v] && !in_d[v]) || seed[v]) clo.push_back(v);
    else if (in_d[v]) drv.push_back(v);
  }
  locality_order(clo, [&](uint32_t v) { return f.first(v); });
  locality_order(drv, [&](uint32_t v) { return f.last(v); });
  const uint32_t nc = (uint32_t)clo.size(), nd = (uint32_t)drv.size();
  std::vector<uint32_t> pos(V, kNone);
  for (uint32_t i = 0; i < nc; ++i) pos[clo[i]] = i;
  for (uint32_t i = 0; i < nd; ++i) pos[drv[i]] = nc + i;
  // twin-levels groups: <= 8 consecutive derived rows (a pod's fabric
  // switches) reading <= kTwinMaxC class rows together (OSPF_TWIN_LV_G=4:
  // <= 4 rows, the launch's 4-root kernel with half the per-root registers)
  std::vector<uint32_t> dgo{0u};
  const char* tge = getenv("OSPF_TWIN_LV_G");
  const uint32_t tlg = tge && atoi(tge) == 4 ? 4u : ospf::kTwinLvG;
  if (nd) {
    std::vector<uint32_t> cl;
    for (uint32_t i = 0; i < nd; ++i) {
      classes_of(drv[i]);
      std::vector<uint32_t> u = cl;
      u.insert(u.end(), cs.begin(), cs.end());
      std::sort(u.begin(), u.end());
      u.erase(std::unique(u.begin(), u.end()), u.end());
      if (i > dgo.back() && (i - dgo.back() >= tlg || u.size() > ospf::kTwinMaxC)) {
        dgo.push_back(i);
        u = cs;
      }
      cl.swap(u);
    }
    dgo.push_back(nd);
  }
  const uint32_t n_dgrp = (uint32_t)dgo.size() - 1;
  // pipeline stages: the derived rows in S stages of whole groups (blocks of
  // pods on a fabric); a leaf group or a twin next-hop root waits only for
  // the stage of the derived rows it reads, so the leaves' row stores run
  // beside the later stages (OSPF_SWEEP_STAGES; default 1: F100k measured
  // 24.2 ms per sweep with one stage, 26.3 with 4, 28.1 with 8 -- the later
  // phase is HBM-bound and the staged twin-level launches lose efficiency)
  uint32_t S = 0;
  if (nd) {
    S = 1;
    if (const char* e = getenv("OSPF_SWEEP_STAGES")) S = (uint32_t)std::max(1, atoi(e));
    S = std::min(S, n_dgrp);
  }
  std::vector<uint32_t> sg(S + 1, 0u);  // first group of each stage
  std::vector<int> stage_of(V, -1);     // stage of a node's derived row
  for (uint32_t k = 0; k <= S; ++k) sg[k] = (uint32_t)((uint64_t)k * n_dgrp / std::max(1u, S));
  for (uint32_t k = 0; k < S; ++k)
    for (uint32_t i = dgo[sg[k]]; i < dgo[sg[k + 1]]; ++i) stage_of[drv[i]] = (int)k;
  auto dep_of = [&](uint32_t r, bool self) {  // latest stage r's rows need (0 if none)
    int d = self ? stage_of[r] : -1;
    for (uint32_t q = (*f.dn_off)[r]; q < (*f.dn_off)[r + 1]; ++q) d = std::max(d, stage_of[(*f.dn)[q]]);
    return std::max(d, 0);
  };
  std::vector<uint32_t> lsg(S + 1, 0u);  // first leaf group of each stage (rest)
  if (S > 1 && nL > nR) {
    const uint32_t ngr0 = (uint32_t)grp.size() - 1;
    std::vector<uint32_t> gi(ngr0), gdep(ngr0);
    for (uint32_t x = 0; x < ngr0; ++x) {
      gi[x] = x;
      gdep[x] = (uint32_t)dep_of(rest[grp[x]], false);
    }
    std::stable_sort(gi.begin(), gi.end(), [&](uint32_t a, uint32_t b) { return gdep[a] < gdep[b]; });
    std::vector<uint32_t> r2, g2{0u};
    for (uint32_t x : gi) {
      r2.insert(r2.end(), rest.begin() + grp[x], rest.begin() + grp[x + 1]);
      g2.push_back((uint32_t)r2.size());
    }
    rest.swap(r2);
    grp.swap(g2);
    need_l.resize(nR);
    need_l.insert(need_l.end(), rest.begin(), rest.end());
    for (uint32_t k = 0, x = 0; k <= S; ++k) {
      while (x < ngr0 && gdep[gi[x]] < k) ++x;
      lsg[k] = k == S ? ngr0 : x;
    }
  }
  lap("rows + stages");
  uint32_t rows = nc + nd;
  for (uint32_t i = 0; i < nL; ++i)
    if (pos[need_l[i]] == kNone) pos[need_l[i]] = rows++;
  // level rows (bytes), dist and leaf next-hop rows 128-B aligned (pitch a multiple of 32
  // words): every 1-KB wave store of the row writers then covers whole lines
  // (ospf_probe_store, leaf-shaped rows at V = 100,024: 7.0 TB/s aligned
  // against 5.8 TB/s at the 400,096-B pitch; profiles/r06/a3_*)
  const uint32_t DP = row_pitch(V);
  const uint32_t pitch = DP == V ? (V + 15) / 16 * 16 : (V + 127) / 128 * 128;
  uint32_t *d_clo = nullptr, *d_pos, *dist, *d_l = nullptr, *lnh = nullptr;
  uint32_t *d_grp_r = nullptr, *d_grp = nullptr, *d_lout = nullptr;
  uint8_t* lev;
  ospf_digest* ldg;
  int rc;
  if ((rc = upload(s, &d_pos, pos)) || (rc = dalloc(s, &lev, (size_t)rows * pitch)) ||
      (rc = dalloc(s, &dist, (size_t)rows * DP)) || (rc = dalloc(s, &ldg, std::max(1u, nc + nd))))
    return rc;
  if (nc && (rc = upload(s, &d_clo, clo))) return rc;
  if (nL && ((rc = upload(s, &d_l, need_l)) || (rc = dalloc(s, &lnh, (size_t)nL * DP))))
    return rc;
  if (nR && (rc = upload(s, &d_grp_r, grp_r))) return rc;
  if (nL > nR && (rc = upload(s, &d_grp, grp))) return rc;
  // level bytes not kept: BFS'd representatives (their BFS rows stay), and
  // the other leaves unless a non-twin class reads every leaf row
  const bool drop_rest = !all_leaf_rows && nL > nR;
  if (drop_rest || (twin_lv && nR)) {
    std::vector<uint32_t> lout(std::max(drop_rest ? nL - nR : 0u, twin_lv ? nR : 0u), kNone);
    if ((rc = upload(s, &d_lout, lout))) return rc;
  }
  lap("allocations + uploads");
  uint32_t *d_tcls = nullptr, *d_trep = nullptr, *d_tsec = nullptr;
  bool any_twin = nd > 0;
  for (auto& k : cls) any_twin |= k.twin;
  if (any_twin && ((rc = upload(s, &d_tcls, tw.cls)) || (rc = upload(s, &d_trep, tw.rep)) ||
                   (rc = upload(s, &d_tsec, tw.sec))))
    return rc;
  s->dig_aux.push_back({ldg, std::max(1u, nc + nd)});
  s->n_rows = rows;
  s->trav_edges = (uint64_t)nc * c->info.n_edges;  // the seed BFS rows; the rest is derived
  const uint32_t ndig = (uint32_t)own_c.size() + nL;
  if ((rc = dalloc(s, &s->dig_all, ndig))) return rc;
  s->n_dig = ndig;
  // events: levels done, cover rows done (= levels without twin levels),
  // representative leaves done, every leaf done
  const int ev_a = new_event(s), ev_t = new_event(s), ev_r = new_event(s), ev_b = new_event(s);
  if (ev_a < 0 || ev_t < 0 || ev_r < 0 || ev_b < 0) return std::min({ev_a, ev_t, ev_r, ev_b});
  std::vector<int> ev_s(S);  // stage k of the derived rows done (the last = ev_t)
  for (uint32_t k = 0; k < S; ++k) {
    ev_s[k] = k + 1 == S ? ev_t : new_event(s);
    if (ev_s[k] < 0) return ev_s[k];
  }
  if (nc) {
    ospf_sweep::Unit lv;
    lv.name = "levels";
    lv.kernel = "ospf_levels_dev (lv_init + lv_level/lv_settle per level + lv_rows: "
                "distance-only 128-root BFS, dist + level rows)";
    lv.stream = 0;
    lv.record = ev_a;
    lv.n_roots = nc;
    lv.comp = (uint64_t)nc * 4ull * V + ((nc + 127) / 128) * scan_bytes(c, false);
    if ((rc = upload(s, &s->d_lv_maxd, std::vector<uint32_t>{0u}))) return rc;
    lv.fn = [=](hipStream_t st) {
      return ospf_int::levels_dev(c, d_clo, nc, hop, dist, DP, lev, pitch, ldg, st, s->lv_cap,
                                  s->d_lv_maxd);
    };
    s->step_comp += lv.comp;
    s->units.push_back(lv);
  }
  // the twin next-hop launches write their roots' dist rows (from the level
  // rows they read anyway), off the serial prefix (OSPF_TWIN_DIST_IN_LEVELS:
  // the twin levels write them, as before)
  const bool nh_dist = twin_lv && !getenv("OSPF_TWIN_DIST_IN_LEVELS");
  std::vector<uint8_t> twin_nh(V, 0);
  for (const auto& k : cls)
    if (k.twin)
      for (uint32_t r : k.roots) twin_nh[r] = 1;
  for (uint32_t k = 0; k < S; ++k) {
    const uint32_t i0 = dgo[sg[k]], n = dgo[sg[k + 1]] - i0;
    std::vector<uint32_t> gk, rk(drv.begin() + i0, drv.begin() + i0 + n);
    for (uint32_t g = sg[k]; g <= sg[k + 1]; ++g) gk.push_back(dgo[g] - i0);
    // the stage's plan, built once on the host (spf_twin.hip twin_levels_kernel)
    ospf_int::TwinLvHost h;
    if ((rc = ospf_int::twin_lv_build(c, rk, gk, pos, tw.cls, tw.rep, h))) return sfail(s, rc, c->err);
    // roots whose twin next-hop launch writes their dist rows: level rows only here
    if (nh_dist)
      for (auto& ri : h.rinfo)
        if (twin_nh[ri.x]) ri.z |= 0x80000000u;
    ospf::TwinLvPlan plan{};
    uint32_t *d_grp2, *d_grow, *d_nbo, *d_nbl;
    uint4* d_rinfo;
    if ((rc = upload(s, &d_grp2, h.grp)) || (rc = upload(s, &d_grow, h.grow)) ||
        (rc = upload(s, &d_nbo, h.nbo)) || (rc = upload(s, &d_nbl, h.nbl)) ||
        (rc = upload(s, &d_rinfo, h.rinfo)))
      return rc;
    plan.n = n;
    plan.ngroups = (uint32_t)h.grp.size() - 1;
    plan.gsz = h.gmax;
    plan.grp = d_grp2;
    plan.grow = d_grow;
    plan.rinfo = d_rinfo;
    plan.nbo = d_nbo;
    plan.nbl = d_nbl;
    plan.lev = lev;
    plan.pitch = pitch;
    plan.dist = dist;
    plan.dpitch = DP;
    plan.lev_digest = ldg;
    ospf_sweep::Unit u;
    u.name = S > 1 ? "twin_levels_s" + std::to_string(k) : std::string("twin_levels");
    u.kernel = "ospf_twin_levels_dev (twin_levels_kernel: level + dist rows from the neighbour "
               "classes' representative rows)";
    u.stream = 0;
    u.record = ev_s[k];
    u.n_roots = n;
    // the unit: the dist rows it writes + its level rows (read by the
    // leaves); the step counts only the dist rows (level rows are
    // intermediate)
    uint64_t nd_rows = 0;
    for (const auto& ri : h.rinfo) nd_rows += (ri.z >> 31) ? 0u : 1u;
    u.comp = nd_rows * 4ull * V + (uint64_t)n * V;
    u.fn = [=](hipStream_t st) { return ospf_int::twin_lv_launch(c, plan, st); };
    s->step_comp += nd_rows * 4ull * V;
    s->units.push_back(u);
  }
  const int ev_cov = nd ? ev_t : ev_a;
  // (C) cover classes: digest slots 0 .. |own_c|
  uint32_t slot = 0;
  // OSPF_SWEEP_EARLY_START: the serial prefix starts now, the host plans on
  if ((rc = start_early(s))) return rc;
  lap("twin levels units");
  std::vector<ospf_sweep::Unit> side, after;
  for (size_t i = 0; i < cls.size(); ++i) {
    Cls& k = cls[i];
    if (k.twin && twin_lv && S > 1)
      std::stable_sort(k.roots.begin(), k.roots.end(), [&](uint32_t a, uint32_t b) {
        return dep_of(a, true) < dep_of(b, true);
      });
    const uint32_t n = (uint32_t)k.roots.size(), W = k.W, cap = std::min(k.cap, 2048u);
    uint32_t *d_roots, *nh;
    // twin classes' next-hop rows 128-B aligned too (nh_derive_twin_kernel
    // stores each 1,024-node tile's W words as one run)
    const uint32_t NPW = k.twin ? row_pitch(V * W) : V * W;
    if ((rc = upload(s, &d_roots, k.roots)) || (rc = dalloc(s, &nh, (size_t)n * NPW))) return rc;
    ospf_digest* dg = s->dig_all + slot;
    for (uint32_t j = 0; j < n; ++j)
      own(s, k.roots[j], slot + j, dist + (size_t)pos[k.roots[j]] * DP, nh + (size_t)j * NPW, W);
    slot += n;
    const int st = new_stream(s);
    if (st < 0) return st;
    if (k.twin && twin_lv && S > 1) {
      // one launch per stage of the roots' own rows (roots were ordered by
      // stage above), beside the later stages
      for (uint32_t q = 0, a0 = 0; q < S; ++q) {
        uint32_t a1 = a0;
        while (a1 < n && (uint32_t)dep_of(k.roots[a1], true) <= q) ++a1;
        if (a1 == a0) continue;
        ospf_sweep::Unit u;
        u.name = "derive_cap" + std::to_string(k.cap) + "_s" + std::to_string(q);
        u.kernel = "ospf_nh_derive_twin_dev (nh_derive_twin_kernel, " + std::to_string(W) +
                   " next-hop word" + (W > 1 ? "s)" : ")");
        u.stream = st;
        u.wait = {ev_s[q]};
        u.n_roots = a1 - a0;
        u.W = W;
        u.comp = (uint64_t)(a1 - a0) * 4ull * V * (W + (nh_dist ? 1u : 0u));
        const uint32_t *tc = d_tcls, *tr = d_trep, *ts = d_tsec, *rr = d_roots + a0;
        const uint32_t m = a1 - a0;
        uint32_t* nhq = nh + (size_t)a0 * NPW;
        ospf_digest* dq = dg + a0;
        uint32_t* dd = nh_dist ? dist : nullptr;
        u.fn = [=](hipStream_t strm) {
          return ospf_int::nh_derive_twin_launch(c, rr, m, W, cap, lev, pitch, d_pos, ldg, tc, tr, ts,
                                                 nhq, dq, dd, strm, DP, NPW);
        };
        s->step_comp += u.comp;
        side.push_back(std::move(u));
        a0 = a1;
      }
      continue;
    }
    if (!k.twin && W > 4 && W <= 64 && !getenv("OSPF_DERIVE_WIDE1")) {
      // spines: the planned tile-staged kernel (host-built runs and slot tables)
      WideHost wh;
      if ((rc = wide_plan_build(c, f, k.roots, W, pos, wh))) return sfail(s, rc, c->err);
      ospf::WidePlan plan{};
      uint32_t *d_run, *d_soff, *d_slots, *d_keep, *d_own;
      if ((rc = upload(s, &d_run, wh.run)) || (rc = upload(s, &d_soff, wh.soff)) ||
          (rc = upload(s, &d_slots, wh.slots)) || (rc = upload(s, &d_keep, wh.keep)) ||
          (rc = upload(s, &d_own, wh.own)))
        return rc;
      plan.n = n;
      plan.W = W;
      plan.nruns = (uint32_t)wh.run.size() - 1;
      plan.run = d_run;
      plan.soff = d_soff;
      plan.slots = d_slots;
      plan.keep = d_keep;
      plan.own = d_own;
      plan.lev = lev;
      plan.pitch = pitch;
      plan.lev_digest = ldg;
      plan.nh = nh;
      plan.digest = dg;
      ospf_sweep::Unit u;
      u.name = "derive_cap" + std::to_string(k.cap);
      u.kernel = "nh_wide_plan_kernel (" + std::to_string(W) + " next-hop words: host-planned runs, "
                 "16-node tiles staged in LDS)";
      u.stream = st;
      u.wait = {!k.reads_leaf ? ev_cov : ev_b};
      if (u.wait[0] == ev_b && nd) u.wait.push_back(ev_cov);
      u.n_roots = n;
      u.W = W;
      u.comp = (uint64_t)n * 4ull * V * W;
      u.fn = [=](hipStream_t strm) {
        const hipError_t e = ospf::launch_wide_plan(c->g, plan, strm);
        if (e != hipSuccess) return hip_fail(c, e, "launch_wide_plan");
        return (int)OSPF_OK;
      };
      s->step_comp += u.comp;
      (u.wait[0] == ev_b ? after : side).push_back(std::move(u));
      continue;
    }
    ospf_sweep::Unit u;
    u.name = "derive_cap" + std::to_string(k.cap);
    u.kernel = std::string(k.twin ? "ospf_nh_derive_twin_dev (" : "ospf_nh_derive_dev (") +
               (k.twin ? "nh_derive_twin_kernel" : W <= 4 ? "nh_derive16_kernel"
                                                          : "nh_derive_wide_kernel") +
               ", " + std::to_string(W) + " next-hop word" + (W > 1 ? "s)" : ")");
    u.stream = st;
    // twin classes read the representatives' rows (BFS'd with twin levels);
    // the others every neighbour's row
    u.wait = {!k.reads_leaf ? ev_cov : k.twin ? (twin_lv ? ev_cov : ev_r) : ev_b};
    // every leaf row (ev_b) does not imply every derived cover row when the
    // last leaf stage precedes the last twin-levels stage
    if (u.wait[0] == ev_b && nd) u.wait.push_back(ev_cov);
    u.n_roots = n;
    u.W = W;
    u.comp = (uint64_t)n * 4ull * V * (W + (k.twin && nh_dist ? 1u : 0u));
    if (k.twin) {
      const uint32_t *tc = d_tcls, *tr = d_trep, *ts = d_tsec;
      uint32_t* dd = nh_dist ? dist : nullptr;
      u.fn = [=](hipStream_t strm) {
        return ospf_int::nh_derive_twin_launch(c, d_roots, n, W, cap, lev, pitch, d_pos, ldg, tc, tr,
                                               ts, nh, dg, dd, strm, DP, NPW);
      };
    } else {
      u.fn = [=](hipStream_t strm) {
        return ospf_nh_derive_dev(c, d_roots, n, W, cap, lev, pitch, d_pos, ldg, nh, dg, strm);
      };
    }
    s->step_comp += u.comp;
    (u.wait[0] == ev_b || u.wait[0] == ev_r ? after : side).push_back(std::move(u));
  }
  for (auto& x : side) s->units.push_back(std::move(x));
  lap("cover next-hop units");
  // (B) leaves: digest slots after the cover roots'; representatives first
  if (nL) {
    uint32_t kmax = 1;
    for (uint32_t r : need_l) kmax = std::max(kmax, f.nbrs(r));
    for (uint32_t j = 0; j < nL; ++j)
      if (in_l[need_l[j]])
        own(s, need_l[j], slot + j, dist + (size_t)pos[need_l[j]] * DP, lnh + (size_t)j * DP, 1);
    ospf_digest* dg = s->dig_all + slot;
    const uint32_t ngr_r = nR ? (uint32_t)grp_r.size() - 1 : 0u;
    const uint32_t ngr = nL > nR ? (uint32_t)grp.size() - 1 : 0u;
    if (nR) {
      ospf_sweep::Unit u;
      u.name = twin_lv ? "leaf_seeds" : "leaf_reps";
      u.kernel = twin_lv ? "ospf_leaf_derive2_dev (leaf_derive_kernel: next-hop rows of BFS'd "
                           "leaf representatives)"
                         : "ospf_leaf_derive2_dev (leaf_derive_kernel: twin representatives' level "
                           "+ dist + next-hop rows)";
      if (twin_lv) {  // beside the other leaves, after the cover rows
        const int st = new_stream(s);
        if (st < 0) return st;
        u.stream = st;
        u.wait = {ev_cov};
      } else {
        u.stream = 0;
      }
      u.record = ev_r;
      u.n_roots = nR;
      u.W = 1;
      u.comp = (uint64_t)nR * (twin_lv ? 4ull : 8ull) * V;
      const uint32_t* lo = twin_lv ? d_lout : nullptr;
      uint32_t* dd = twin_lv ? nullptr : dist;
      u.fn = [=](hipStream_t strm) {
        return ospf_int::leaf_derive(c, d_l, nR, d_grp_r, ngr_r, kmax, lev, pitch, d_pos, lo, dd, DP,
                                     lnh, DP, dg, strm);
      };
      s->step_comp += u.comp;
      s->units.push_back(std::move(u));
    }
    if (nL > nR && twin_lv && S > 1) {
      const int lst = new_stream(s);
      if (lst < 0) return lst;
      for (uint32_t q = 0; q < S; ++q) {
        const uint32_t g0 = lsg[q], g1 = lsg[q + 1];
        if (g1 == g0) continue;
        const uint32_t i0 = grp[g0], n = grp[g1] - i0;
        std::vector<uint32_t> gq;
        for (uint32_t g = g0; g <= g1; ++g) gq.push_back(grp[g] - i0);
        uint32_t* d_gq;
        if ((rc = upload(s, &d_gq, gq))) return rc;
        ospf_sweep::Unit u;
        u.name = "leaf_s" + std::to_string(q);
        u.kernel = "ospf_leaf_derive2_dev (leaf_derive_kernel: level + dist + next-hop rows of leaf "
                   "roots from their neighbours' level rows)";
        u.stream = lst;
        u.wait = {ev_s[q]};
        if (g1 == (uint32_t)grp.size() - 1) u.record = ev_b;
        u.n_roots = n;
        u.W = 1;
        u.comp = (uint64_t)n * 8ull * V;
        const uint32_t* dl = d_l + nR + i0;
        uint32_t* nh = lnh + (size_t)(nR + i0) * DP;
        ospf_digest* dg2 = dg + nR + i0;
        const uint32_t* lo = drop_rest ? d_lout : nullptr;
        const uint32_t ngq = g1 - g0;
        u.fn = [=](hipStream_t strm) {
          return ospf_int::leaf_derive(c, dl, n, d_gq, ngq, kmax, lev, pitch, d_pos, lo, dist, DP, nh,
                                       DP, dg2, strm);
        };
        s->step_comp += u.comp;
        s->units.push_back(std::move(u));
      }
    } else if (nL > nR && leaf_tail > 0.0 && twin_lv && ngr >= 2) {
      // the leaves in two launches on the main stream: the second waits for
      // the largest cover next-hop launch, which so gets the GPU's share
      // before it and no longer finishes alone after the leaves
      // (OSPF_SWEEP_LEAF_TAIL = the second launch's share of the groups)
      int big = -1;
      for (size_t x = 0; x < s->units.size(); ++x)
        if (s->units[x].name.rfind("derive_cap", 0) == 0 && s->units[x].record < 0 &&
            (big < 0 || s->units[x].comp > s->units[big].comp))
          big = (int)x;
      const uint32_t gs = std::min(ngr - 1, std::max(1u, ngr - (uint32_t)(ngr * leaf_tail)));
      int ev_tn = -1;
      if (big >= 0) {
        ev_tn = new_event(s);
        if (ev_tn < 0) return ev_tn;
        s->units[big].record = ev_tn;
      }
      std::vector<uint32_t> gq;
      for (uint32_t g = gs; g <= ngr; ++g) gq.push_back(grp[g] - grp[gs]);
      uint32_t* d_gq;
      if ((rc = upload(s, &d_gq, gq))) return rc;
      const uint32_t* lo = drop_rest ? d_lout : nullptr;
      for (int part = 0; part < 2; ++part) {
        ospf_sweep::Unit u;
        u.name = part ? "leaf_tail" : "leaf";
        u.kernel = "ospf_leaf_derive2_dev (leaf_derive_kernel: level + dist + next-hop rows of leaf "
                   "roots from their neighbours' level rows)";
        u.stream = 0;
        const uint32_t i0 = part ? grp[gs] : 0u, i1 = part ? grp[ngr] : grp[gs];
        const uint32_t n = i1 - i0, ngq = part ? ngr - gs : gs;
        if (part) {
          if (ev_tn >= 0) u.wait = {ev_tn};
          u.record = ev_b;
        }
        u.n_roots = n;
        u.W = 1;
        u.comp = (uint64_t)n * 8ull * V;
        const uint32_t* dl = d_l + nR + i0;
        uint32_t* nh = lnh + (size_t)(nR + i0) * DP;
        ospf_digest* dg2 = dg + nR + i0;
        const uint32_t* lo2 = lo ? lo + i0 : nullptr;
        const uint32_t* gp = part ? d_gq : d_grp;
        u.fn = [=](hipStream_t strm) {
          return ospf_int::leaf_derive(c, dl, n, gp, ngq, kmax, lev, pitch, d_pos, lo2, dist, DP, nh,
                                       DP, dg2, strm);
        };
        s->step_comp += u.comp;
        s->units.push_back(std::move(u));
      }
    } else if (nL > nR) {
      ospf_sweep::Unit u;
      u.name = "leaf";
      u.kernel = "ospf_leaf_derive2_dev (leaf_derive_kernel: level + dist + next-hop rows of leaf "
                 "roots from their neighbours' level rows)";
      const uint32_t n = nL - nR;
      if (nR && !twin_lv) {  // beside the cover roots' next hops, on a stream of its own
        const int st = new_stream(s);
        if (st < 0) return st;
        u.stream = st;
        u.wait = {ev_a};
      } else {
        u.stream = 0;
      }
      u.record = ev_b;
      u.n_roots = n;
      u.W = 1;
      u.comp = (uint64_t)n * 8ull * V;
      const uint32_t* dl = d_l + nR;
      uint32_t* nh = lnh + (size_t)nR * DP;
      ospf_digest* dg2 = dg + nR;
      const uint32_t* lo = drop_rest ? d_lout : nullptr;
      ospf_sweep* sw = s;
      u.fn = [=](hipStream_t strm) {
        return ospf_int::leaf_derive(c, dl, n, d_grp, ngr, kmax, lev, pitch, d_pos, lo, dist, DP, nh, DP,
                                     dg2, strm, sw->leaf_order);
      };
      s->step_comp += u.comp;
      s->units.push_back(std::move(u));
    }
  }
  lap("next-hop + leaf units");
  // an event no launch records stands for the one before it
  auto alias = [&](int from, int to) {
    for (auto& u : after)
      for (int& e : u.wait)
        if (e == from) e = to;
  };
  if (!(nL > nR)) alias(ev_b, nR ? ev_r : ev_cov);
  if (!nR) alias(ev_r, ev_cov);
  for (auto& x : after) s->units.push_back(std::move(x));
  return OSPF_OK;
}

// BATCH: one engine batch per width class of the part, each on its own
// stream from the run's start (ospf_run_batch_dev picks the kernel).
int plan_batch(ospf_sweep* s, const Facts& f, const std::vector<uint32_t>& mine,
               bool weighted) {
  ospf_ctx* c = s->c;
  const uint32_t V = s->V;
  std::vector<uint32_t> caps;
  for (uint32_t r : mine) caps.push_back(f.cap(r));
  std::sort(caps.begin(), caps.end());
  caps.erase(std::unique(caps.begin(), caps.end()), caps.end());
  int rc;
  if ((rc = dalloc(s, &s->dig_all, mine.size()))) return rc;
  s->n_dig = (uint32_t)mine.size();
  s->n_rows = (uint32_t)mine.size();
  s->trav_edges = (uint64_t)mine.size() * c->info.n_edges;
  uint32_t slot = 0;
  const uint32_t flags = (s->opts.flags & OSPF_HOP_COUNT) | OSPF_WANT_DIST | OSPF_WANT_NH |
                         OSPF_WANT_DIGEST;
  for (uint32_t cap : caps) {
    std::vector<uint32_t> roots;
    uint32_t mx = 1;
    for (uint32_t r : mine)
      if (f.cap(r) == cap) {
        roots.push_back(r);
        mx = std::max(mx, f.nbrs(r));
      }
    locality_order(roots, [&](uint32_t v) { return f.first(v); });
    const uint32_t n = (uint32_t)roots.size(), W = std::max(1u, (cap + 31) / 32);
    uint32_t *d_roots, *dist, *nh;
    if ((rc = upload(s, &d_roots, roots)) || (rc = dalloc(s, &dist, (size_t)n * V)) ||
        (rc = dalloc(s, &nh, (size_t)n * V * W)))
      return rc;
    ospf_digest* dg = s->dig_all + slot;
    for (uint32_t j = 0; j < n; ++j)
      own(s, roots[j], slot + j, dist + (size_t)j * V, nh + (size_t)j * V * W, W);
    slot += n;
    ospf_plan_info pi{};
    ospf_plan_n(c, flags, W, 0, n, mx, &pi);
    ospf_sweep::Unit u;
    u.name = "batch_cap" + std::to_string(cap);
    u.kernel = "ospf_run_batch_dev (variant " + std::to_string(pi.variant) + ", " +
               std::to_string(W) + " next-hop word" + (W > 1 ? "s)" : ")");
    const int st = new_stream(s);
    if (st < 0) return st;
    u.stream = st;
    u.wait = {0};
    u.n_roots = n;
    u.W = W;
    const uint64_t scans = pi.variant == 5 ? (uint64_t)((n + 63) / 64) * pi.slices
                                           : (uint64_t)n;
    u.comp = (uint64_t)n * 4ull * V * (1 + W) + scans * scan_bytes(c, weighted && pi.variant != 5);
    u.fn = [=](hipStream_t strm) {
      ospf_batch b{};
      b.d_roots = d_roots;
      b.n_roots = n;
      b.flags = flags;
      b.nh_words = W;
      b.max_root_neighbors = mx;
      b.d_dist = dist;
      b.d_nh = nh;
      b.d_digest = dg;
      return ospf_run_batch_dev(c, &b, strm);
    };
    s->step_comp += u.comp;
    s->units.push_back(std::move(u));
  }
  return OSPF_OK;
}

// LDS (spf_small.hip): small graphs, one launch per next-hop width (W <= 4)
// -- a wave per root with the graph in LDS; the widest class on the main
// stream, the others beside it.
int plan_lds(ospf_sweep* s, const Facts& f, const std::vector<uint32_t>& mine) {
  ospf_ctx* c = s->c;
  const uint32_t V = s->V;
  const uint32_t hop = s->opts.flags & OSPF_HOP_COUNT;
  std::vector<uint32_t> ws;
  for (uint32_t r : mine) ws.push_back(f.words(r));
  std::sort(ws.begin(), ws.end());
  ws.erase(std::unique(ws.begin(), ws.end()), ws.end());
  int rc;
  if ((rc = dalloc(s, &s->dig_all, mine.size()))) return rc;
  s->n_dig = (uint32_t)mine.size();
  s->n_rows = (uint32_t)mine.size();
  s->trav_edges = (uint64_t)mine.size() * c->info.n_edges;
  uint32_t slot = 0;
  bool first = true;
  for (auto it = ws.rbegin(); it != ws.rend(); ++it) {
    const uint32_t W = *it;
    std::vector<uint32_t> roots;
    for (uint32_t r : mine)
      if (f.words(r) == W) roots.push_back(r);
    const uint32_t n = (uint32_t)roots.size();
    uint32_t *d_roots, *dist, *nh;
    if ((rc = upload(s, &d_roots, roots)) || (rc = dalloc(s, &dist, (size_t)n * V)) ||
        (rc = dalloc(s, &nh, (size_t)n * V * W)))
      return rc;
    ospf_digest* dg = s->dig_all + slot;
    for (uint32_t j = 0; j < n; ++j)
      own(s, roots[j], slot + j, dist + (size_t)j * V, nh + (size_t)j * V * W, W);
    slot += n;
    ospf_sweep::Unit u;
    u.name = "lds_w" + std::to_string(W);
    u.kernel = "ospf_lds_sweep_dev (lds_sweep_kernel<" + std::to_string(W) +
               ">: a wave per root, graph + BFS state in LDS)";
    if (first) {
      u.stream = 0;
    } else {
      const int st = new_stream(s);
      if (st < 0) return st;
      u.stream = st;
      u.wait = {0};
    }
    first = false;
    u.n_roots = n;
    u.W = W;
    // rows written + the padded CSR each block copies in (read once from HBM)
    u.comp = (uint64_t)n * 4ull * V * (1 + W) + scan_bytes(c, false);
    u.fn = [=](hipStream_t strm) {
      return ospf_lds_sweep_dev(c, d_roots, n, hop, W, dist, nh, dg, strm);
    };
    s->step_comp += u.comp;
    s->units.push_back(std::move(u));
  }
  return OSPF_OK;
}

// Node tiles for the closure rows (launch_closure_rows): consecutive nodes, a
// tile closed at kLtNodes nodes or when its union of cover indices (a cover
// node's own, a leaf's in-links') would pass kLtU. False when a leaf has
// more than kLtE in-links.
struct NodeTiles {
  std::vector<uint4> tile;
  std::vector<uint32_t> le, u;
};
bool node_tiles(const ospf_ctx* c, NodeTiles& t) {
  const std::vector<uint32_t>& cix = c->h_cix;
  const uint32_t V = (uint32_t)cix.size(), nS = (uint32_t)c->h_ccv.size();
  std::vector<uint32_t> slot(nS, kNone), ul;
  uint32_t first = 0;
  auto close = [&](uint32_t end) {
    if (end == first) return;
    t.tile.push_back(make_uint4(first, end - first, (uint32_t)t.u.size(), (uint32_t)ul.size()));
    for (uint32_t ci : ul) {
      t.u.push_back(ci);
      slot[ci] = kNone;
    }
    ul.clear();
    first = end;
  };
  t.le.assign((size_t)V * ospf::kLtE, 0xFFFFFFFFu);
  for (uint32_t v = 0, l = 0; v < V; ++v) {
    uint32_t ent[ospf::kLtE], ne = 0, fresh = 0;
    if (cix[v] & 0x80000000u) {
      for (uint32_t x = c->h_lrow[l]; x < c->h_lrow[l + 1]; ++x) {
        const uint32_t w = c->h_ladj[x], ci = w & 0xFFFFu;
        if (ci >= nS) continue;  // padding
        if (ne == ospf::kLtE) return false;
        ent[ne++] = w;
        if (slot[ci] == kNone) ++fresh;  // (a repeat counts twice: a bound)
      }
      ++l;
    } else {
      ent[ne++] = cix[v];
      if (slot[cix[v]] == kNone) ++fresh;
    }
    if (v - first == ospf::kLtNodes || ul.size() + fresh > ospf::kLtU) close(v);
    for (uint32_t q = 0; q < ne; ++q) {
      const uint32_t ci = ent[q] & 0xFFFFu;
      if (slot[ci] == kNone) {
        slot[ci] = (uint32_t)ul.size();
        ul.push_back(ci);
      }
      t.le[(size_t)v * ospf::kLtE + q] =
          (cix[v] & 0x80000000u) ? (slot[ci] | (ent[q] & 0xFFFF0000u)) : (slot[ci] | 0x100u);
    }
  }
  close(V);
  return true;
}

// WCOVER (spf_cover.hip + spf_wderive.hip): an independent set of leaves
// (<= 32 distinct neighbours; on a fabric the racks), the cover = the rest.
// (A) distance rows of the cover nodes the part needs by the contracted-graph
// SPF; (B) the leaves' dist + next-hop rows from their neighbours' rows;
// (C) next hops of cover roots (<= 2048 neighbours) from their own and their
// neighbours' rows, one launch per word count (> 4 words beside B). Cover
// roots beyond 2048 neighbours run their own batch from the start.
int plan_wcover(ospf_sweep* s, const Facts& f, const std::vector<uint32_t>& mine,
                const std::vector<uint8_t>& leaf) {
  ospf_ctx* c = s->c;
  const uint32_t V = s->V;
  std::vector<uint32_t> own_l, own_c, c_der, c_wide;
  for (uint32_t r : mine) (leaf[r] ? own_l : own_c).push_back(r);
  for (uint32_t r : own_c) (f.nbrs(r) <= 2048 ? c_der : c_wide).push_back(r);
  locality_order(own_l, [&](uint32_t v) { return f.first(v); });
  std::sort(own_c.begin(), own_c.end());
  const std::vector<uint32_t> nb_c = closure(f, c_der);
  std::vector<uint8_t> in_l(V, 0);
  for (uint32_t r : own_l) in_l[r] = 1;
  std::vector<uint32_t> extra_l;  // leaves the cover next hops read, not owned
  for (uint32_t v : nb_c)
    if (leaf[v] && !in_l[v]) extra_l.push_back(v);
  locality_order(extra_l, [&](uint32_t v) { return f.first(v); });
  std::vector<uint32_t> need_l = own_l;
  need_l.insert(need_l.end(), extra_l.begin(), extra_l.end());
  const std::vector<uint32_t> cl = closure(f, need_l);
  std::vector<uint8_t> in_a(V, 0);
  for (uint32_t v : own_c) in_a[v] = 1;
  for (uint32_t v : cl)
    if (!leaf[v]) in_a[v] = 1;
  for (uint32_t v : nb_c)
    if (!leaf[v]) in_a[v] = 1;
  std::vector<uint32_t> cover_a;
  for (uint32_t v = 0; v < V; ++v)
    if (in_a[v]) cover_a.push_back(v);
  const uint32_t nA = (uint32_t)cover_a.size(), nL = (uint32_t)need_l.size();
  std::vector<uint32_t> pos(V, kNone);
  for (uint32_t i = 0; i < nA; ++i) pos[cover_a[i]] = i;
  for (uint32_t i = 0; i < nL; ++i) pos[need_l[i]] = nA + i;
  uint32_t *slab, *d_pos, *d_a, *d_l, *lnh;
  int rc;
  if ((rc = dalloc(s, &slab, (size_t)(nA + nL) * V)) || (rc = upload(s, &d_pos, pos)) ||
      (rc = upload(s, &d_a, cover_a)) || (rc = upload(s, &d_l, need_l)) ||
      (rc = dalloc(s, &lnh, (size_t)nL * V)))
    return rc;
  uint32_t kmax = 1;
  for (uint32_t r : need_l) kmax = std::max(kmax, f.nbrs(r));
  // (A) plan: cover rows by the closure when the cover splits into seeds and
  // small components (the seeds' Dial, the closure's cover columns, then the
  // full rows), else every row by the Dial. With one word count <= 4 over
  // the closure roots, the closure also carries their next hops (masks of
  // first hops per seed term): their next-hop rows then come out of the
  // rows unit and no neighbour-row derivation runs for them.
  std::vector<uint32_t> seeds, clos;
  ospf_int::ClosureHost ch;
  bool closure = !c->cl_seed.empty() && !getenv("OSPF_COVER_NOCLOSURE");
  uint32_t NW = 0;
  if (closure) {
    const uint32_t nS = (uint32_t)c->h_ccv.size();
    std::vector<uint32_t> seed_row(nS, kNone);
    for (uint32_t j = 0; j < c->cl_seed.size(); ++j) {
      seed_row[c->cl_seed[j]] = j;
      seeds.push_back(c->h_ccv[c->cl_seed[j]]);
    }
    std::vector<uint8_t> is_seed(V, 0);
    for (uint32_t v : seeds) is_seed[v] = 1;
    for (uint32_t v : cover_a)
      if (!is_seed[v]) clos.push_back(v);
    const std::string err0 = c->err;  // a plan that does not apply is no error of the sweep
    NW = clos.empty() ? 0u : f.words(clos[0]);
    for (uint32_t r : clos)
      if (f.words(r) != NW) NW = 0;
    if (NW > ospf::kClMaxNW || getenv("OSPF_CLOSURE_NONH")) NW = 0;
    closure = clos.size() >= seeds.size() && ospf_int::closure_build(c, clos, seed_row, ch, NW) == OSPF_OK;
    if (!closure && NW) {  // the masks do not apply: distances only
      NW = 0;
      closure = ospf_int::closure_build(c, clos, seed_row, ch, 0) == OSPF_OK;
    }
    if (!closure) {
      c->err = err0;
      NW = 0;
    }
  }
  const bool cl_nh = closure && NW > 0;
  std::vector<uint8_t> nh_by_closure(V, 0);
  if (cl_nh)
    for (uint32_t r : clos) nh_by_closure[r] = 1;
  // the part's seeds (<= 64 next-hop words): next-hop masks during their
  // Dial, rows + digests after it (cover_spf_kernel seed mode)
  std::vector<uint32_t> sd_nh;
  uint32_t NWs = 0;
  if (closure && !getenv("OSPF_SEED_NONH")) {
    std::vector<uint8_t> in_d(V, 0);
    for (uint32_t r : c_der) in_d[r] = 1;
    for (uint32_t r : seeds)
      if (in_d[r]) {
        sd_nh.push_back(r);
        NWs = std::max(NWs, f.words(r));
      }
    if (NWs > ospf::kSeedMaxNW) {
      sd_nh.clear();
      NWs = 0;
    }
    for (uint32_t r : sd_nh) nh_by_closure[r] = 1;
  }
  {
    std::vector<uint32_t> keep;
    for (uint32_t r : c_der)
      if (!nh_by_closure[r]) keep.push_back(r);
    c_der.swap(keep);
  }
  // digests: cover classes (owned), then need_l (owned leaves first), then
  // the closure roots (next hops by the closure)
  std::vector<uint32_t> wset;
  for (uint32_t r : c_der) wset.push_back(f.words(r));
  std::sort(wset.begin(), wset.end());
  wset.erase(std::unique(wset.begin(), wset.end()), wset.end());
  const uint32_t ncl_dig = cl_nh ? (uint32_t)clos.size() : 0u;
  const uint32_t nsn = (uint32_t)sd_nh.size();
  const uint32_t ndig = (uint32_t)(c_der.size() + c_wide.size() + nL) + ncl_dig + nsn;
  const uint32_t cl_dig0 = ndig - nsn - ncl_dig, sn_dig0 = ndig - nsn;
  if ((rc = dalloc(s, &s->dig_all, ndig))) return rc;
  s->n_dig = ndig;
  s->n_rows = nA + nL;
  const uint32_t flags = OSPF_WANT_DIST | OSPF_WANT_NH | OSPF_WANT_DIGEST;
  uint32_t slot = 0;
  int ev_a = new_event(s);  // cover rows done
  if (ev_a < 0) return ev_a;
  // wide cover roots: their own batch, from the start
  if (!c_wide.empty()) {
    std::vector<uint32_t> roots = c_wide;
    locality_order(roots, [&](uint32_t v) { return f.first(v); });
    uint32_t W = 1, mx = 1;
    for (uint32_t r : roots) {
      W = std::max(W, f.words(r));
      mx = std::max(mx, f.nbrs(r));
    }
    const uint32_t n = (uint32_t)roots.size();
    uint32_t *d_roots, *dist, *nh;
    if ((rc = upload(s, &d_roots, roots)) || (rc = dalloc(s, &dist, (size_t)n * V)) ||
        (rc = dalloc(s, &nh, (size_t)n * V * W)))
      return rc;
    ospf_digest* dg = s->dig_all + slot;
    for (uint32_t j = 0; j < n; ++j)
      own(s, roots[j], slot + j, dist + (size_t)j * V, nh + (size_t)j * V * W, W);
    slot += n;
    ospf_sweep::Unit u;
    u.name = "cover_batch_w" + std::to_string(W);
    u.kernel = "ospf_run_batch_dev (" + std::to_string(W) + " next-hop words)";
    const int st = new_stream(s);
    if (st < 0) return st;
    u.stream = st;
    u.wait = {0};
    u.n_roots = n;
    u.W = W;
    u.comp = (uint64_t)n * 4ull * V * (1 + W) + (uint64_t)n * scan_bytes(c, true);
    u.fn = [=](hipStream_t strm) {
      ospf_batch b{};
      b.d_roots = d_roots;
      b.n_roots = n;
      b.flags = flags;
      b.nh_words = W;
      b.max_root_neighbors = mx;
      b.d_dist = dist;
      b.d_nh = nh;
      b.d_digest = dg;
      return ospf_run_batch_dev(c, &b, strm);
    };
    s->step_comp += u.comp;
    s->units.push_back(std::move(u));
  }
  // the Dial over the contracted cover graph: the seeds' rows (closure) or
  // every cover row
  s->trav_edges = (uint64_t)(closure ? seeds.size() : nA) * c->h_cedge.size();
  if (getenv("OSPF_SWEEP_DEBUG"))
    fprintf(stderr, "plan_wcover: cover %u seeds %zu comps %zu closure roots %zu -> %s (%s)\n", nA,
            c->cl_seed.size(), c->cl_comp_off.size() - 1, clos.size(), closure ? "closure" : "dial",
            c->err.c_str());
  int seed_rows_ev = -1;  // the seeds' rows, when on a stream of their own
  std::vector<uint32_t> row_chunk(V, kNone);  // closure root -> its rows chunk
  std::vector<int> rows_ev;                   // events of the rows chunks
  if (closure) {
    const uint32_t nS = (uint32_t)c->h_ccv.size(), nsd = (uint32_t)seeds.size();
    const uint32_t ncl = (uint32_t)clos.size();
    std::vector<uint32_t> seed_rp(nsd), clos_rp(ncl);
    for (uint32_t j = 0; j < nsd; ++j) seed_rp[j] = pos[seeds[j]];  // kNone: not a row here
    for (uint32_t j = 0; j < ncl; ++j) clos_rp[j] = pos[clos[j]];
    uint32_t *d_sd, *d_srp, *d_cl, *d_crp, *seedC, *dc, *d_jl, *d_cst, *d_mem, *d_dloc, *d_out;
    uint2* d_comp;
    if ((rc = upload(s, &d_sd, seeds)) || (rc = upload(s, &d_srp, seed_rp)) ||
        (rc = upload(s, &d_cl, clos)) || (rc = upload(s, &d_crp, clos_rp)) ||
        (rc = dalloc(s, &seedC, (size_t)nsd * nS)) || (rc = dalloc(s, &dc, (size_t)ncl * nS)) ||
        (rc = upload(s, &d_comp, ch.comp)) || (rc = upload(s, &d_jl, ch.jl)) ||
        (rc = upload(s, &d_cst, ch.cst)) || (rc = upload(s, &d_mem, ch.mem)) ||
        (rc = upload(s, &d_dloc, ch.dloc)) || (rc = upload(s, &d_out, ch.out)))
      return rc;
    ospf::ClosurePlan cp{};
    cp.ncomp = (uint32_t)ch.comp.size();
    cp.nS = nS;
    cp.chunks = (nS + 255u) / 256u;
    cp.comp = d_comp;
    cp.jl = d_jl;
    cp.cst = d_cst;
    cp.mem = d_mem;
    cp.dloc = d_dloc;
    cp.out = d_out;
    cp.seedC = seedC;
    cp.dc = dc;
    const uint32_t KW = ch.KW;
    // next hops of the closure roots: masks in, the cover columns' masks out
    // of the closure, rows + digests out of the rows unit
    uint32_t *d_fh = nullptr, *d_fhl = nullptr, *dcm = nullptr, *cnh = nullptr;
    ospf_digest* cdg = nullptr;
    if (cl_nh) {
      if ((rc = upload(s, &d_fh, ch.fh)) || (rc = upload(s, &d_fhl, ch.fhloc)) ||
          (rc = dalloc(s, &dcm, (size_t)ncl * nS * NW)) || (rc = dalloc(s, &cnh, (size_t)ncl * V * NW)))
        return rc;
      cp.NW = NW;
      cp.fh = d_fh;
      cp.fhloc = d_fhl;
      cp.dcm = dcm;
      cdg = s->dig_all + cl_dig0;
      std::vector<uint8_t> mine_m(V, 0);
      for (uint32_t r : mine) mine_m[r] = 1;
      for (uint32_t j = 0; j < ncl; ++j)
        if (mine_m[clos[j]])
          own(s, clos[j], cl_dig0 + j, slab + (size_t)clos_rp[j] * V, cnh + (size_t)j * V * NW, NW);
    }
    // next hops of the part's seeds out of their Dial
    uint32_t *d_snp = nullptr, *snm = nullptr, *snh = nullptr, *sdf = nullptr, *d_sroots = nullptr,
             *d_srp2 = nullptr;
    ospf_digest* sdg = nullptr;
    // the seeds' rows on a stream of their own, beside the closure and its
    // rows (OSPF_SEED_ROWS_INLINE: inside the Dial's launch)
    const bool seed_side = nsn && !getenv("OSPF_SEED_ROWS_INLINE");
    if (nsn) {
      std::vector<uint32_t> snp(nsd, kNone), at(V, kNone), srp2(nsn);
      for (uint32_t k = 0; k < nsn; ++k) {
        at[sd_nh[k]] = k;
        srp2[k] = pos[sd_nh[k]];
      }
      for (uint32_t j = 0; j < nsd; ++j) snp[j] = at[seeds[j]];
      if ((rc = upload(s, &d_snp, snp)) || (rc = dalloc(s, &snm, (size_t)nsn * nS * NWs)) ||
          (rc = dalloc(s, &snh, (size_t)nsn * V * NWs)) ||
          (seed_side && ((rc = dalloc(s, &sdf, (size_t)nsn * nS)) || (rc = upload(s, &d_sroots, sd_nh)) ||
                         (rc = upload(s, &d_srp2, srp2)))))
        return rc;
      sdg = s->dig_all + sn_dig0;
      for (uint32_t k = 0; k < nsn; ++k)
        own(s, sd_nh[k], sn_dig0 + k, slab + (size_t)pos[sd_nh[k]] * V, snh + (size_t)k * V * NWs, NWs);
    }
    {
      ospf_sweep::Unit u;
      u.name = "cover_seeds";
      u.kernel = nsn ? "cover_spf_kernel (seeds' Dial, next-hop masks at settle; cover columns, "
                       "dist + next-hop rows, digests)"
                     : "cover_spf_kernel (contracted-graph Dial of the closure's seeds, LDS-resident "
                       "distances; their cover columns out)";
      u.stream = 0;
      u.n_roots = nsd;
      u.W = NWs;
      u.comp = (uint64_t)nsd * 4ull * V + scan_bytes(c, true) +
               (uint64_t)nsn * 4ull * NWs * (V + 2ull * nS);
      u.fn = [=](hipStream_t strm) {
        if (sdg && !seed_side &&
            ospf::zero_async(sdg, (size_t)nsn * sizeof(ospf_digest), strm) != hipSuccess)
          return ospf_int::fail(c, OSPF_E_DEVICE, "zero seed digests");
        ospf::CoverArgs a{};
        a.roots = d_sd;
        a.n = nsd;
        a.dist = slab;
        a.err = c->d_err;
        a.rowpos = d_srp;
        a.dcomp = seedC;
        if (nsn) {
          a.nhpos = d_snp;
          a.nhm = snm;
          a.nh = snh;
          a.NW = NWs;
          a.digest = sdg;
          a.dfull = sdf;  // null: rows inside this launch
        }
        const hipError_t e = ospf::launch_cover_spf(c->g, c->cover, a, (uint32_t)c->n_cu, strm);
        return e == hipSuccess ? OSPF_OK : ospf_int::hip_fail(c, e, "launch_cover_spf");
      };
      s->step_comp += u.comp;
      if (seed_side) {
        u.record = new_event(s);
        if (u.record < 0) return u.record;
      }
      s->units.push_back(std::move(u));
    }
    if (seed_side) {  // the seeds' rows beside the closure
      const int ev_seeds = s->units.back().record;
      ospf_sweep::Unit u;
      u.name = "seed_rows";
      u.kernel = "seed_rows_kernel (the seeds' dist + next-hop rows and digests from their columns "
                 "and masks)";
      const int st = new_stream(s);
      if (st < 0) return st;
      u.stream = st;
      u.wait = {ev_seeds};
      seed_rows_ev = new_event(s);
      if (seed_rows_ev < 0) return seed_rows_ev;
      u.record = seed_rows_ev;
      u.n_roots = nsn;
      u.W = NWs;
      u.comp = (uint64_t)nsn * 4ull * V * (1 + NWs);
      s->units.back().comp -= u.comp;  // counted once
      u.fn = [=](hipStream_t strm) {
        if (sdg && ospf::zero_async(sdg, (size_t)nsn * sizeof(ospf_digest), strm) != hipSuccess)
          return ospf_int::fail(c, OSPF_E_DEVICE, "zero seed digests");
        const hipError_t e = ospf::launch_seed_rows(c->g, c->cover, d_sroots, nsn, sdf, snm, NWs, slab,
                                                    d_srp2, snh, sdg, c->d_err, (uint32_t)c->n_cu, strm);
        return e == hipSuccess ? OSPF_OK : ospf_int::hip_fail(c, e, "launch_seed_rows");
      };
      s->units.push_back(std::move(u));
    }
    {
      ospf_sweep::Unit u;
      u.name = "cover_closure";
      u.kernel = cl_nh ? "closure_nh_kernel<" + std::to_string(NW) +
                             "> (cover columns + their next-hop masks of the components' roots "
                             "from the seeds' columns)"
                       : "closure_kernel<" + std::to_string(KW) +
                             "> (cover columns of the components' roots from the seeds' columns)";
      u.stream = 0;
      u.n_roots = ncl;
      u.comp = (uint64_t)ncl * 4ull * nS * (1 + NW);
      u.fn = [=](hipStream_t strm) {
        const hipError_t e = ospf::launch_closure(cp, KW, strm);
        return e == hipSuccess ? OSPF_OK : ospf_int::hip_fail(c, e, "launch_closure");
      };
      s->step_comp += u.comp;
      s->units.push_back(std::move(u));
    }
    // opt-in (OSPF_WCOVER_STAGE): the closure roots' rows in K chunks (in
    // closure order: a fabric's pods), each recording an event, so the leaf
    // rows of the chunks done run beside the next chunk. Measured slower on
    // the weighted F100k (58.5 vs 54.9 ms, a22): the bandwidth-bound leaf
    // launch takes the CUs the latency-bound rows launch needs.
    const uint32_t K = (nL && ncl >= 64 && getenv("OSPF_WCOVER_STAGE")) ? 4u : 1u;
    // opt-in (OSPF_COVER_ROWS_TILED): with next hops, the rows by node tiles x
    // root chunks (closure_tile_rows_kernel) instead of a node-order pass per
    // root; exact, but measured 2x slower on the weighted F100k (35.3 vs
    // 16.9 ms, a27 / a28)
    bool tiled = false;
    ospf::ClosureRowsPlan rp{};
    if (cl_nh && K == 1 && getenv("OSPF_COVER_ROWS_TILED")) {
      NodeTiles nt;
      tiled = node_tiles(c, nt) && !nt.tile.empty();
      if (tiled) {
        std::vector<uint32_t> rcov(ncl);
        for (uint32_t j = 0; j < ncl; ++j) rcov[j] = c->h_cix[clos[j]];
        uint32_t *d_rcov, *d_tle, *d_tu;
        uint4* d_tile;
        if ((rc = upload(s, &d_rcov, rcov)) || (rc = upload(s, &d_tile, nt.tile)) ||
            (rc = upload(s, &d_tle, nt.le)) || (rc = upload(s, &d_tu, nt.u)))
          return rc;
        rp.nroots = ncl;
        rp.nS = nS;
        rp.NW = NW;
        rp.ntiles = (uint32_t)nt.tile.size();
        rp.roots = d_cl;
        rp.rcov = d_rcov;
        rp.rowpos = d_crp;
        rp.dc = dc;
        rp.dcm = dcm;
        rp.dist = slab;
        rp.nh = cnh;
        rp.digest = cdg;
        rp.tile = d_tile;
        rp.tle = d_tle;
        rp.tu = d_tu;
      }
    }
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t lo = (uint32_t)((uint64_t)ncl * k / K), hi = (uint32_t)((uint64_t)ncl * (k + 1) / K);
      for (uint32_t j = lo; j < hi; ++j) row_chunk[clos[j]] = k;
      ospf_sweep::Unit u;
      u.name = K > 1 ? "cover_rows_s" + std::to_string(k) : std::string("cover_rows");
      u.kernel = tiled ? "closure_tile_rows_kernel (the closure roots' dist + next-hop rows and "
                         "digests by node tiles: cover columns given, leaves by their last hops)"
                 : cl_nh ? "cover_rows_kernel (full dist + next-hop rows and digests of the closure's "
                         "roots: cover columns given, leaves by their last hop)"
                       : "cover_spf_kernel (full rows of the closure's roots: cover columns "
                         "given, leaves by their last hop)";
      u.stream = 0;
      if (k + 1 == K) {
        u.record = ev_a;
      } else {
        u.record = new_event(s);
        if (u.record < 0) return u.record;
      }
      rows_ev.push_back(u.record);
      u.n_roots = hi - lo;
      u.W = NW;
      u.comp = (uint64_t)(hi - lo) * 4ull * V * (1 + NW);
      u.fn = [=](hipStream_t strm) {
        if (hi == lo) return OSPF_OK;
        if (cdg && ospf::zero_async(cdg + lo, (size_t)(hi - lo) * sizeof(ospf_digest), strm) != hipSuccess)
          return ospf_int::fail(c, OSPF_E_DEVICE, "zero closure digests");
        if (tiled) {
          const hipError_t e = ospf::launch_closure_rows(c->g, c->cover, rp, strm);
          return e == hipSuccess ? OSPF_OK : ospf_int::hip_fail(c, e, "launch_closure_rows");
        }
        ospf::CoverArgs a{};
        a.roots = d_cl + lo;
        a.n = hi - lo;
        a.dist = slab;
        a.err = c->d_err;
        a.rowpos = d_crp + lo;
        a.dload = dc + (size_t)lo * nS;
        a.nhload = dcm ? dcm + (size_t)lo * nS * NW : nullptr;
        a.nh = cnh ? cnh + (size_t)lo * V * NW : nullptr;
        a.NW = NW;
        a.digest = cdg ? cdg + lo : nullptr;
        const hipError_t e = ospf::launch_cover_spf(c->g, c->cover, a, (uint32_t)c->n_cu, strm);
        return e == hipSuccess ? OSPF_OK : ospf_int::hip_fail(c, e, "launch_cover_spf");
      };
      s->step_comp += u.comp;
      s->units.push_back(std::move(u));
    }
  } else {
    ospf_sweep::Unit u;
    u.name = "cover_spf";
    u.kernel = "ospf_cover_dist_dev (cover_spf_kernel: contracted-graph Dial, LDS-resident "
               "distances)";
    u.stream = 0;
    u.record = ev_a;
    u.n_roots = nA;
    u.comp = (uint64_t)nA * 4ull * V + scan_bytes(c, true);
    u.fn = [=](hipStream_t strm) { return ospf_cover_dist_dev(c, d_a, nA, slab, strm); };
    s->step_comp += u.comp;
    s->units.push_back(std::move(u));
  }
  // (C) classes of cover roots by word count
  std::vector<ospf_sweep::Unit> narrow;
  for (uint32_t W : wset) {
    std::vector<uint32_t> roots;
    for (uint32_t r : c_der)
      if (f.words(r) == W) roots.push_back(r);
    locality_order(roots, [&](uint32_t v) { return f.last(v); });
    const uint32_t n = (uint32_t)roots.size();
    uint32_t *d_roots, *nh;
    if ((rc = upload(s, &d_roots, roots)) || (rc = dalloc(s, &nh, (size_t)n * V * W))) return rc;
    ospf_digest* dg = s->dig_all + slot;
    for (uint32_t j = 0; j < n; ++j)
      own(s, roots[j], slot + j, slab + (size_t)pos[roots[j]] * V, nh + (size_t)j * V * W, W);
    slot += n;
    ospf_sweep::Unit u;
    u.name = "wderive_wide_w" + std::to_string(W);
    u.kernel = std::string("ospf_wderive_wide_dev (") +
               (W <= 4 ? "wderive_wide_kernel<" + std::to_string(W) + ">"
                       : std::string("wderive_lanes_kernel")) + ")";
    u.n_roots = n;
    u.W = W;
    u.comp = (uint64_t)n * 4ull * V * W;
    // W > 4 (beside the leaves): 32-tile chunks, fewer blocks -- F100k-w step
    // 136 -> 126 ms though the launch alone takes 71 instead of 56 ms
    const uint32_t ct = W > 4 ? 32u : 0u;
    u.fn = [=](hipStream_t strm) {
      return ospf_int::wderive_wide(c, d_roots, n, 0, W, slab, V, d_pos, nh, dg, strm, ct);
    };
    HubHost hh;
    const std::string err0 = c->err;
    const bool hub = W <= 4 && getenv("OSPF_WNH_HUB") && hub_build(c, f, roots, W, pos, hh) == OSPF_OK;
    if (!hub) c->err = err0;  // not applicable: the lanes / wide kernels run
    if (hub) {
      uint4* d_grp;
      uint32_t *d_hub, *d_loc, *d_ref, *d_wt, *d_ownl, *d_rid;
      if ((rc = upload(s, &d_grp, hh.grp)) || (rc = upload(s, &d_hub, hh.hub.empty() ? std::vector<uint32_t>{0u} : hh.hub)) ||
          (rc = upload(s, &d_loc, hh.loc)) || (rc = upload(s, &d_ref, hh.ref)) ||
          (rc = upload(s, &d_wt, hh.wt)) || (rc = upload(s, &d_ownl, hh.ownl)) ||
          (rc = upload(s, &d_rid, hh.rootid)))
        return rc;
      ospf::HubPlan hp{};
      hp.nhub = (uint32_t)hh.hub.size();
      hp.ngroups = (uint32_t)hh.grp.size();
      hp.tiles = (V + ospf::kHubTile - 1) / ospf::kHubTile;
      hp.tchunk = std::min<uint32_t>(8u, hp.tiles);
      // groups per block: <= 32 (512 roots), fewer while the grid is small
      hp.gchunk = 32u;
      while (hp.gchunk > 1u &&
             ((hp.ngroups + hp.gchunk - 1) / hp.gchunk) * ((hp.tiles + hp.tchunk - 1) / hp.tchunk) <
                 8u * (uint32_t)c->n_cu)
        hp.gchunk /= 2u;
      hp.W = W;
      hp.nroots = n;
      hp.hub = d_hub;
      hp.grp = d_grp;
      hp.loc = d_loc;
      hp.ref = d_ref;
      hp.wt = d_wt;
      hp.ownl = d_ownl;
      hp.rootid = d_rid;
      hp.src = slab;
      hp.pitch = V;
      hp.nh = nh;
      hp.digest = dg;
      u.kernel = "wnh_hub_kernel<" + std::to_string(W) + "> (hub rows per tile in LDS, a group's "
                 "rows per group, wave = root, lane = node)";
      u.fn = [=](hipStream_t strm) {
        const hipError_t e = ospf::launch_wnh_hub(c->g, hp, strm);
        return e == hipSuccess ? OSPF_OK : ospf_int::hip_fail(c, e, "launch_wnh_hub");
      };
    }
    WRunsHost wh;
    const std::string err1 = c->err;
    const bool runs = W > 4 && getenv("OSPF_WNH_RUNS") && wruns_build(c, f, roots, W, pos, wh) == OSPF_OK;
    if (!runs) c->err = err1;
    if (runs) {  // runs of roots with one neighbour list
      uint4* d_run;
      uint32_t *d_sl, *d_wt, *d_own, *d_rid;
      if ((rc = upload(s, &d_run, wh.run)) || (rc = upload(s, &d_sl, wh.slots)) ||
          (rc = upload(s, &d_wt, wh.wt)) || (rc = upload(s, &d_own, wh.own)) ||
          (rc = upload(s, &d_rid, wh.rootid)))
        return rc;
      ospf::WRunsPlan wp{};
      wp.nruns = (uint32_t)wh.run.size();
      wp.nroots = n;
      wp.W = W;
      wp.tiles = (V + ospf::kWrTile - 1) / ospf::kWrTile;
      wp.run = d_run;
      wp.slots = d_sl;
      wp.wt = d_wt;
      wp.own = d_own;
      wp.rootid = d_rid;
      wp.src = slab;
      wp.pitch = V;
      wp.nh = nh;
      wp.digest = dg;
      u.kernel = "wnh_runs_kernel (runs of roots with one neighbour list, lane = node, a wave "
                 "per next-hop word)";
      u.fn = [=](hipStream_t strm) {
        const hipError_t e = ospf::launch_wnh_runs(c->g, wp, strm);
        return e == hipSuccess ? OSPF_OK : ospf_int::hip_fail(c, e, "launch_wnh_runs");
      };
    }
    s->step_comp += u.comp;
    bool reads_leaf = false;  // a neighbour's row comes from (B)
    for (uint32_t r : roots)
      for (uint32_t k = (*f.dn_off)[r]; k < (*f.dn_off)[r + 1] && !reads_leaf; ++k)
        reads_leaf = leaf[(*f.dn)[k]] != 0;
    if (W > 4 && !reads_leaf) {  // needs only the cover rows: beside the leaves
      const int st = new_stream(s);
      if (st < 0) return st;
      u.stream = st;
      u.wait = {ev_a};
      if (seed_rows_ev >= 0) u.wait.push_back(seed_rows_ev);  // may read a seed's row
      s->units.push_back(std::move(u));
    } else {
      u.stream = 0;
      if (seed_rows_ev >= 0) u.wait.push_back(seed_rows_ev);
      narrow.push_back(std::move(u));
    }
  }
  // (B) leaves, then the narrow cover classes (they read leaf rows)
  if (rows_ev.size() > 1 && nL) {  // leaf chunks beside the closure rows' chunks
    ospf_digest* dg = s->dig_all + slot;
    for (uint32_t j = 0; j < own_l.size(); ++j)
      own(s, own_l[j], slot + j, slab + (size_t)(nA + j) * V, lnh + (size_t)j * V, 1);
    slot += nL;
    std::vector<uint8_t> is_sn(V, 0);
    for (uint32_t r : sd_nh) is_sn[r] = 1;
    const int lst = new_stream(s);
    if (lst < 0) return lst;
    const uint32_t KL = 4;
    int last = -1;
    for (uint32_t k = 0; k < KL; ++k) {
      const uint32_t lo = (uint32_t)((uint64_t)nL * k / KL), hi = (uint32_t)((uint64_t)nL * (k + 1) / KL);
      uint32_t dep = 0;
      bool seedn = false;
      for (uint32_t j = lo; j < hi; ++j)
        for (uint32_t e = (*f.dn_off)[need_l[j]]; e < (*f.dn_off)[need_l[j] + 1]; ++e) {
          const uint32_t x = (*f.dn)[e];
          if (row_chunk[x] != kNone) dep = std::max(dep, row_chunk[x]);
          else if (is_sn[x]) seedn = true;
        }
      ospf_sweep::Unit u;
      u.name = "wderive_s" + std::to_string(k);
      u.kernel = "ospf_wderive_dev (wderive_kernel: leaf rows from the cover rows, a chunk)";
      u.stream = lst;
      u.wait = {rows_ev[dep]};
      if (seedn && seed_rows_ev >= 0) u.wait.push_back(seed_rows_ev);
      u.record = new_event(s);
      if (u.record < 0) return u.record;
      last = u.record;
      u.n_roots = hi - lo;
      u.W = 1;
      u.comp = (uint64_t)(hi - lo) * 8ull * V;
      uint32_t* ldist = slab + (size_t)(nA + lo) * V;
      uint32_t* lnh_k = lnh + (size_t)lo * V;
      const uint32_t* d_lk = d_l + lo;
      ospf_digest* dgk = dg + lo;
      u.fn = [=](hipStream_t strm) {
        if (hi == lo) return OSPF_OK;
        return ospf_wderive_dev(c, d_lk, hi - lo, 0, kmax, slab, V, d_pos, ldist, lnh_k, dgk, strm);
      };
      s->step_comp += u.comp;
      s->units.push_back(std::move(u));
    }
    for (auto& u : narrow) {
      u.wait.push_back(last);
      s->units.push_back(std::move(u));
    }
    return OSPF_OK;
  }
  {
    ospf_digest* dg = s->dig_all + slot;
    for (uint32_t j = 0; j < own_l.size(); ++j)
      own(s, own_l[j], slot + j, slab + (size_t)(nA + j) * V, lnh + (size_t)j * V, 1);
    slot += nL;
    ospf_sweep::Unit u;
    u.name = "wderive";
    u.kernel = "ospf_wderive_dev (wderive_kernel: leaf rows from the cover rows)";
    u.stream = 0;
    u.n_roots = nL;
    u.W = 1;
    u.comp = (uint64_t)nL * 8ull * V +
             (uint64_t)(cl.size() - std::min(cl.size(), (size_t)nL)) * 4ull * V;
    uint32_t* ldist = slab + (size_t)nA * V;
    if (seed_rows_ev >= 0) {  // a leaf next to a seed reads the seed's row
      std::vector<uint8_t> is_sn(V, 0);
      for (uint32_t r : sd_nh) is_sn[r] = 1;
      bool near = false;
      for (uint32_t r : need_l)
        for (uint32_t k = (*f.dn_off)[r]; k < (*f.dn_off)[r + 1] && !near; ++k) near = is_sn[(*f.dn)[k]] != 0;
      if (near) u.wait.push_back(seed_rows_ev);
    }
    u.fn = [=](hipStream_t strm) {
      if (!nL) return OSPF_OK;
      return ospf_wderive_dev(c, d_l, nL, 0, kmax, slab, V, d_pos, ldist, lnh, dg, strm);
    };
    s->step_comp += u.comp;
    s->units.push_back(std::move(u));
  }
  for (auto& u : narrow) s->units.push_back(std::move(u));
  return OSPF_OK;
}

// WMULTI: the distance rows the part needs -- its non-leaf roots and every
// neighbour of its roots that is not one of its leaves -- from the multi-root
// traversal (spf_msdist.hip: groups of 32 roots adjacent in id order share a
// wavefront), then the leaves' rows derived from their neighbours' rows
// (ospf_wderive_dev), then the non-leaf roots' next hops from their own and
// their neighbours' rows (ospf_wderive_wide_dev). For large graphs where the
// cover does not fit the contracted-graph kernel (a mesh).
int plan_wmulti(ospf_sweep* s, const Facts& f, const std::vector<uint32_t>& mine,
                const std::vector<uint8_t>& leaf) {
  ospf_ctx* c = s->c;
  const uint32_t V = s->V;
  const uint32_t hop = s->opts.flags & OSPF_HOP_COUNT;
  std::vector<uint8_t> own_m(V, 0), in_s(V, 0);
  std::vector<uint32_t> own_l, own_c;
  for (uint32_t r : mine) own_m[r] = 1;
  for (uint32_t r : mine) {
    (leaf[r] ? own_l : own_c).push_back(r);
    if (f.nbrs(r) > 2048) return fail(c, OSPF_E_RANGE, "wmulti: a root with > 2048 neighbours");
    if (!leaf[r]) in_s[r] = 1;
    for (uint32_t k = (*f.dn_off)[r]; k < (*f.dn_off)[r + 1]; ++k) {
      const uint32_t n = (*f.dn)[k];
      if (!(leaf[n] && own_m[n])) in_s[n] = 1;
    }
  }
  std::vector<uint32_t> srows;  // ascending ids: neighbours share a group
  for (uint32_t v = 0; v < V; ++v)
    if (in_s[v]) srows.push_back(v);
  const uint32_t nS = (uint32_t)srows.size(), nL = (uint32_t)own_l.size();
  std::vector<uint32_t> pos(V, kNone);
  for (uint32_t i = 0; i < nS; ++i) pos[srows[i]] = i;
  for (uint32_t j = 0; j < nL; ++j) pos[own_l[j]] = nS + j;
  // concurrent groups: two per CU, within a scratch budget (OSPF_MSD_MB, 64 GB)
  const uint32_t ngroups = (nS + 31u) / 32u;
  size_t budget = 65536ull << 20;
  if (const char* e = getenv("OSPF_MSD_MB")) budget = (size_t)std::max(64, atoi(e)) << 20;
  const size_t per = ospf::msdist_scratch_bytes(V, 1);
  uint32_t delta = hop ? 1u : std::max<uint32_t>(1, c->info.max_metric);
  if (const char* e = getenv("OSPF_MSD_DELTA")) delta = (uint32_t)std::max(1, atoi(e));
  uint32_t *slab, *d_pos, *d_s, *d_l, *lnh, *scratch = nullptr;
  int rc;
  if ((rc = dalloc(s, &slab, (size_t)(nS + nL) * V)) || (rc = upload(s, &d_pos, pos)) ||
      (rc = upload(s, &d_s, srows.empty() ? std::vector<uint32_t>{0u} : srows)) ||
      (rc = upload(s, &d_l, own_l.empty() ? std::vector<uint32_t>{0u} : own_l)) ||
      (rc = dalloc(s, &lnh, (size_t)std::max(1u, nL) * V)))
    return rc;
  // the scratch also fits what the device has left (other parts' sweeps,
  // smaller devices), with a 1 GB margin; fewer blocks when an allocation
  // still fails
  // (destroyed sweeps' pooled blocks count as free: the allocation takes
  // from the pool or frees it)
  {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
      fr += c->sweep_pool_bytes;
      budget = std::min<size_t>(budget, fr > (1ull << 30) ? fr - (1ull << 30) : per);
    }
  }
  uint32_t blocks = std::min<uint32_t>(std::max(1u, ngroups), 2u * (uint32_t)c->n_cu);
  blocks = std::max<uint32_t>(1, std::min<uint32_t>(blocks, (uint32_t)(budget / per)));
  if (const char* e = getenv("OSPF_MSD_BLOCKS")) blocks = std::max(1, std::min((int)blocks, atoi(e)));
  for (;;) {
    if (dalloc_try(s, &scratch, per * blocks / sizeof(uint32_t)) == OSPF_OK) break;
    if (blocks == 1) return sfail(s, OSPF_E_NOMEM, "wmulti: no room for one traversal's scratch");
    blocks = std::max(1u, blocks / 2);
  }
  std::vector<uint32_t> wset;
  for (uint32_t r : own_c) wset.push_back(f.words(r));
  std::sort(wset.begin(), wset.end());
  wset.erase(std::unique(wset.begin(), wset.end()), wset.end());
  const uint32_t ndig = (uint32_t)(own_c.size() + nL);
  if ((rc = dalloc(s, &s->dig_all, std::max(1u, ndig)))) return rc;
  s->n_dig = ndig;
  s->n_rows = nS + nL;
  s->trav_edges = (uint64_t)nS * c->info.n_edges;
  {
    ospf_sweep::Unit u;
    u.name = "msdist";
    u.kernel = "msdist_kernel (groups of 32 roots, [node][root] distances, label-correcting "
               "Delta-stepping)";
    u.stream = 0;
    u.n_roots = nS;
    u.comp = (uint64_t)nS * 4ull * V + (uint64_t)ngroups * scan_bytes(c, !hop);
    u.fn = [=](hipStream_t strm) {
      ospf::MsDistArgs a{};
      a.roots = d_s;
      a.n = nS;
      a.ngroups = ngroups;
      a.blocks = std::min(blocks, ngroups);
      a.delta = delta;
      a.hop = hop ? 1u : 0u;
      a.dist = slab;
      a.pitch = V;
      a.scratch = scratch;
      const bool dbg = getenv("OSPF_MSD_STATS") != nullptr;
      unsigned long long* st = nullptr;
      if (dbg && (hipMalloc(&st, 32) != hipSuccess || hipMemset(st, 0, 32) != hipSuccess))
        return ospf_int::fail(c, OSPF_E_DEVICE, "msdist stats");
      a.stats = st;
      const hipError_t e = ospf::launch_msdist(c->g, a, strm);
      if (e != hipSuccess) return ospf_int::hip_fail(c, e, "launch_msdist");
      if (dbg) {  // debug only (never inside a capture: OSPF_MSD_STATS runs eager sweeps)
        unsigned long long h[4];
        hipStreamSynchronize(strm);
        hipMemcpy(h, st, 32, hipMemcpyDeviceToHost);
        hipFree(st);
        fprintf(stderr, "msdist: %u rows, %u groups: phases %llu (%.1f per group), frontier "
                "nodes %llu (%.2f per node per group), candidates %llu (%.2f per node per group)\n",
                nS, ngroups, h[0], (double)h[0] / ngroups, h[1],
                (double)h[1] / ((double)ngroups * V), h[2], (double)h[2] / ((double)ngroups * V));
      }
      c->spf_runs += nS;
      return OSPF_OK;
    };
    s->step_comp += u.comp;
    s->units.push_back(std::move(u));
  }
  uint32_t slot = 0;
  {  // leaves from their neighbours' rows
    ospf_digest* dg = s->dig_all + slot;
    for (uint32_t j = 0; j < nL; ++j)
      own(s, own_l[j], slot + j, slab + (size_t)(nS + j) * V, lnh + (size_t)j * V, 1);
    slot += nL;
    uint32_t kmax = 1;
    for (uint32_t r : own_l) kmax = std::max(kmax, f.nbrs(r));
    ospf_sweep::Unit u;
    u.name = "wderive";
    u.kernel = "ospf_wderive_dev (wderive_kernel: leaf rows from neighbours' dist rows)";
    u.stream = 0;
    u.n_roots = nL;
    u.W = 1;
    u.comp = (uint64_t)nL * 8ull * V;
    uint32_t* ldist = slab + (size_t)nS * V;
    u.fn = [=](hipStream_t strm) {
      if (!nL) return OSPF_OK;
      return ospf_wderive_dev(c, d_l, nL, hop, kmax, slab, V, d_pos, ldist, lnh, dg, strm);
    };
    s->step_comp += u.comp;
    s->units.push_back(std::move(u));
  }
  for (uint32_t W : wset) {  // next hops of the non-leaf roots
    std::vector<uint32_t> roots;
    for (uint32_t r : own_c)
      if (f.words(r) == W) roots.push_back(r);
    const uint32_t n = (uint32_t)roots.size();
    uint32_t *d_roots, *nh;
    if ((rc = upload(s, &d_roots, roots)) || (rc = dalloc(s, &nh, (size_t)n * V * W))) return rc;
    ospf_digest* dg = s->dig_all + slot;
    for (uint32_t j = 0; j < n; ++j)
      own(s, roots[j], slot + j, slab + (size_t)pos[roots[j]] * V, nh + (size_t)j * V * W, W);
    slot += n;
    ospf_sweep::Unit u;
    u.name = "wderive_wide_w" + std::to_string(W);
    u.kernel = std::string("ospf_wderive_wide_dev (") +
               (W <= 4 ? "wderive_wide_kernel<" + std::to_string(W) + ">"
                       : std::string("wderive_lanes_kernel")) + ")";
    u.stream = 0;
    u.n_roots = n;
    u.W = W;
    u.comp = (uint64_t)n * 4ull * V * W;
    u.fn = [=](hipStream_t strm) {
      return ospf_int::wderive_wide(c, d_roots, n, hop, W, slab, V, d_pos, nh, dg, strm, 0);
    };
    s->step_comp += u.comp;
    s->units.push_back(std::move(u));
  }
  return OSPF_OK;
}

// WDERIVE: cover roots (the part's non-leaves plus every neighbour of its
// leaves) on the per-root batch path, one launch per class on its own
// stream; then the leaves derived from those rows.
int plan_wderive(ospf_sweep* s, const Facts& f, const std::vector<uint32_t>& mine,
                 const std::vector<uint8_t>& leaf) {
  ospf_ctx* c = s->c;
  const uint32_t V = s->V;
  const uint32_t hop = s->opts.flags & OSPF_HOP_COUNT;
  std::vector<uint32_t> lr, cov;
  std::vector<uint8_t> own_m(V, 0);
  for (uint32_t r : mine) {
    own_m[r] = 1;
    if (leaf[r]) lr.push_back(r);
  }
  std::vector<uint8_t> in_c(V, 0);
  for (uint32_t r : mine)
    if (!leaf[r]) in_c[r] = 1;
  for (uint32_t v : closure(f, lr))
    if (!leaf[v]) in_c[v] = 1;
  for (uint32_t v = 0; v < V; ++v)
    if (in_c[v]) cov.push_back(v);
  locality_order(lr, [&](uint32_t v) { return f.first(v); });
  std::vector<uint32_t> caps;
  for (uint32_t r : cov) caps.push_back(f.cap(r));
  std::sort(caps.begin(), caps.end());
  caps.erase(std::unique(caps.begin(), caps.end()), caps.end());
  const uint32_t nC = (uint32_t)cov.size(), nl = (uint32_t)lr.size();
  uint32_t *cdist, *d_pos, *d_lr, *ldist, *lnh;
  int rc;
  if ((rc = dalloc(s, &cdist, (size_t)nC * V)) || (rc = upload(s, &d_lr, lr)) ||
      (rc = dalloc(s, &ldist, (size_t)nl * V)) || (rc = dalloc(s, &lnh, (size_t)nl * V)) ||
      (rc = dalloc(s, &s->dig_all, nC + nl)))
    return rc;
  s->n_dig = nC + nl;
  s->n_rows = nC + nl;
  s->trav_edges = (uint64_t)nC * c->info.n_edges;  // cover rows on the batch path
  std::vector<uint32_t> pos(V, kNone);
  uint32_t off = 0;
  const uint32_t flags = hop | OSPF_WANT_DIST | OSPF_WANT_NH | OSPF_WANT_DIGEST;
  std::vector<int> done;
  for (uint32_t cap : caps) {
    std::vector<uint32_t> roots;
    uint32_t mx = 1;
    for (uint32_t r : cov)
      if (f.cap(r) == cap) {
        roots.push_back(r);
        mx = std::max(mx, f.nbrs(r));
      }
    locality_order(roots, [&](uint32_t v) { return f.first(v); });
    const uint32_t n = (uint32_t)roots.size(), W = std::max(1u, (cap + 31) / 32);
    uint32_t *d_roots, *nh;
    if ((rc = upload(s, &d_roots, roots)) || (rc = dalloc(s, &nh, (size_t)n * V * W))) return rc;
    uint32_t* dist = cdist + (size_t)off * V;
    ospf_digest* dg = s->dig_all + off;
    for (uint32_t j = 0; j < n; ++j) {
      pos[roots[j]] = off + j;
      if (own_m[roots[j]])
        own(s, roots[j], off + j, dist + (size_t)j * V, nh + (size_t)j * V * W, W);
    }
    off += n;
    ospf_plan_info pi{};
    ospf_plan_n(c, flags, W, 0, n, mx, &pi);
    ospf_sweep::Unit u;
    u.name = "cover_cap" + std::to_string(cap);
    u.kernel = "ospf_run_batch_dev (variant " + std::to_string(pi.variant) + ", " +
               std::to_string(W) + " next-hop word" + (W > 1 ? "s)" : ")");
    const int st = new_stream(s);
    if (st < 0) return st;
    const int ev = new_event(s);
    if (ev < 0) return ev;
    u.stream = st;
    u.wait = {0};
    u.record = ev;
    done.push_back(ev);
    u.n_roots = n;
    u.W = W;
    const uint64_t scans = pi.variant == 5 ? (uint64_t)((n + 63) / 64) * pi.slices : n;
    u.comp = (uint64_t)n * 4ull * V * (1 + W) + scans * scan_bytes(c, !hop && pi.variant != 5);
    u.fn = [=](hipStream_t strm) {
      ospf_batch b{};
      b.d_roots = d_roots;
      b.n_roots = n;
      b.flags = flags;
      b.nh_words = W;
      b.max_root_neighbors = mx;
      b.d_dist = dist;
      b.d_nh = nh;
      b.d_digest = dg;
      return ospf_run_batch_dev(c, &b, strm);
    };
    s->step_comp += u.comp;
    s->units.push_back(std::move(u));
  }
  if ((rc = upload(s, &d_pos, pos))) return rc;
  // owned leaves: digests after the cover rows
  for (uint32_t j = 0; j < nl; ++j)
    own(s, lr[j], nC + j, ldist + (size_t)j * V, lnh + (size_t)j * V, 1);
  uint32_t kmax = 1;
  for (uint32_t r : lr) kmax = std::max(kmax, f.nbrs(r));
  ospf_sweep::Unit u;
  u.name = "wderive";
  u.kernel = "ospf_wderive_dev (wderive_kernel: leaf rows from neighbours' dist rows)";
  u.stream = 0;
  u.wait = done;
  u.n_roots = nl;
  u.W = 1;
  u.comp = (uint64_t)nl * 8ull * V + (uint64_t)nC * 4ull * V;
  ospf_digest* dg = s->dig_all + nC;
  u.fn = [=](hipStream_t strm) {
    if (!nl) return OSPF_OK;
    return ospf_wderive_dev(c, d_lr, nl, hop, kmax, cdist, V, d_pos, ldist, lnh, dg, strm);
  };
  s->step_comp += u.comp;
  s->units.push_back(std::move(u));
  return OSPF_OK;
}

// queue one run's launches; the run starts when `origin` (the main stream)
// reaches this point and ends when main has waited for every other stream
// one unit of a run on its stream: its waits, the launch, its event
int launch_unit(ospf_sweep* s, ospf_sweep::Unit& u) {
  hipStream_t st = s->streams[u.stream];
  for (int e : u.wait)
    if (!(e == 0 && u.stream == 0)) SCHK(s, hipStreamWaitEvent(st, s->events[e], 0));
  const int rc = u.fn(st);
  if (rc != OSPF_OK) return sfail(s, rc, std::string(u.name) + ": " + ospf_last_error(s->c));
  if (u.record >= 0) SCHK(s, hipEventRecord(s->events[u.record], st));
  return OSPF_OK;
}

// OSPF_SWEEP_EARLY_START: queue the units planned so far (the first run's
// start: after the null stream's prior work, as run_eager orders it)
int start_early(ospf_sweep* s) {
  if (!s->early) return OSPF_OK;
  if (!s->early_on) {
    SCHK(s, hipEventRecord(s->ev_in, nullptr));
    SCHK(s, hipStreamWaitEvent(s->streams[0], s->ev_in, 0));
    SCHK(s, hipEventRecord(s->events[0], s->streams[0]));
    s->early_on = true;
  }
  for (; s->started < s->units.size(); ++s->started) {
    const int rc = launch_unit(s, s->units[s->started]);
    if (rc) return rc;
  }
  return OSPF_OK;
}

int enqueue(ospf_sweep* s) {
  hipStream_t main = s->streams[0];
  // (units an early start queued are skipped, once)
  const size_t first = s->early_on ? s->started : 0;
  if (!s->early_on) SCHK(s, hipEventRecord(s->events[0], main));
  s->early_on = false;
  s->started = 0;
  for (size_t i = first; i < s->units.size(); ++i) {
    const int rc = launch_unit(s, s->units[i]);
    if (rc) return rc;
  }
  for (size_t i = 1; i < s->streams.size(); ++i) {
    SCHK(s, hipEventRecord(s->ev_done[i], s->streams[i]));
    SCHK(s, hipStreamWaitEvent(main, s->ev_done[i], 0));
  }
  return OSPF_OK;
}

int run_eager(ospf_sweep* s, hipStream_t caller) {
  if (!s->early_on) {  // (an early start ordered it after the null stream)
    SCHK(s, hipEventRecord(s->ev_in, caller));
    SCHK(s, hipStreamWaitEvent(s->streams[0], s->ev_in, 0));
  }
  const int rc = enqueue(s);
  if (rc) return rc;
  SCHK(s, hipEventRecord(s->ev_out, s->streams[0]));
  SCHK(s, hipStreamWaitEvent(caller, s->ev_out, 0));
  return OSPF_OK;
}

// The leaf launch (derive mode) timed in both block orders on the rows of
// the eager run (its own digests are zeroed by the launch, rows rewritten
// identically), the faster kept for the HIP graph and every later run.
// OSPF_LEAF_GROUP_MAJOR fixes the order; OSPF_LEAF_NO_AUTO keeps chunk-major.
int pick_leaf_order(ospf_sweep* s) {
  if (getenv("OSPF_LEAF_GROUP_MAJOR") || getenv("OSPF_LEAF_NO_AUTO")) return OSPF_OK;
  ospf_sweep::Unit* u = nullptr;
  for (auto& x : s->units)
    if (x.name == "leaf") u = &x;
  if (!u || u->n_roots < 4096) return OSPF_OK;
  hipStream_t st = s->streams[u->stream];
  hipEvent_t a, b;
  SCHK(s, hipEventCreate(&a));
  SCHK(s, hipEventCreate(&b));
  float best[2] = {1e30f, 1e30f};
  int rc = OSPF_OK;
  for (int rep = 0; rep < 2 && rc == OSPF_OK; ++rep)
    for (int ord = 0; ord < 2 && rc == OSPF_OK; ++ord) {
      s->leaf_order = ord;
      if (hipEventRecord(a, st) != hipSuccess) rc = OSPF_E_DEVICE;
      if (rc == OSPF_OK) rc = u->fn(st);
      if (rc == OSPF_OK && (hipEventRecord(b, st) != hipSuccess || hipEventSynchronize(b) != hipSuccess))
        rc = OSPF_E_DEVICE;
      float t = 0;
      if (rc == OSPF_OK && hipEventElapsedTime(&t, a, b) == hipSuccess) best[ord] = std::min(best[ord], t);
    }
  hipEventDestroy(a);
  hipEventDestroy(b);
  if (rc) return sfail(s, rc, "sweep: leaf order probe: " + std::string(ospf_last_error(s->c)));
  s->leaf_order = best[1] < best[0] ? 1 : 0;
  if (getenv("OSPF_SWEEP_TIMING"))
    fprintf(stderr, "sweep_create leaf order %s (chunk-major %.3f ms, group-major %.3f ms)\n",
            s->leaf_order ? "group-major" : "chunk-major", best[0], best[1]);
  return ospf_sync(s->c, st);
}

void release(ospf_sweep* s) {
  if (s->c) hipSetDevice(s->c->device);
  for (hipStream_t st : s->streams)
    if (st) hipStreamSynchronize(st);
  if (s->exec) hipGraphExecDestroy(s->exec);
  if (s->graph) hipGraphDestroy(s->graph);
  // blocks, streams (with their scratch) and events go to the ctx's pools
  // for the next sweep (ospf_close frees them)
  constexpr size_t kPoolCap = 160ull << 30;
  for (size_t i = 0; i < s->allocs.size(); ++i) {
    if (s->c && i < s->alloc_bytes.size() && s->c->sweep_pool_bytes + s->alloc_bytes[i] <= kPoolCap) {
      s->c->sweep_pool.emplace(s->alloc_bytes[i], s->allocs[i]);
      s->c->sweep_pool_bytes += s->alloc_bytes[i];
    } else {
      hipFree(s->allocs[i]);
    }
  }
  for (hipEvent_t e : s->events)
    if (e) (s->c ? (void)s->c->event_pool.push_back(e) : (void)hipEventDestroy(e));
  for (hipEvent_t e : s->ev_done)
    if (e) hipEventDestroy(e);
  if (s->ev_in) hipEventDestroy(s->ev_in);
  if (s->ev_out) hipEventDestroy(s->ev_out);
  for (hipStream_t st : s->streams) {
    if (!st) continue;
    if (s->c) {
      s->c->stream_pool.push_back(st);
    } else {
      hipStreamDestroy(st);
    }
  }
  // idempotent: a sweep released by ospf_close is released again (a no-op)
  // by its own destroy
  s->allocs.clear();
  s->alloc_bytes.clear();
  s->streams.clear();
  s->events.clear();
  s->ev_done.clear();
  s->ev_in = s->ev_out = nullptr;
  s->exec = nullptr;
  s->graph = nullptr;
}

}  // namespace

extern "C" {

int ospf_sweep_create(ospf_ctx* c, const ospf_sweep_opts* o, ospf_sweep** out) {
  if (!c || !o || !out) return OSPF_E_INVAL;
  *out = nullptr;
  if (ospf_int::injected(c)) return OSPF_E_DEVICE;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (c->mask.on) return fail(c, OSPF_E_INVAL, "sweep: links are masked (ospf_links_unmask)");
  const uint32_t parts = std::max(1u, o->n_parts);
  if (o->part >= parts) return fail(c, OSPF_E_INVAL, "sweep: part >= n_parts");
  if (o->mode > OSPF_SWEEP_WMULTI) return fail(c, OSPF_E_INVAL, "sweep: unknown mode");
  if (o->flags & ~(OSPF_HOP_COUNT | OSPF_SWEEP_DEFER | OSPF_SWEEP_EARLY_START))
    return fail(c, OSPF_E_INVAL,
                "sweep: flags = 0 or OSPF_HOP_COUNT, | OSPF_SWEEP_DEFER (| OSPF_SWEEP_EARLY_START)");
  const bool defer = (o->flags & OSPF_SWEEP_DEFER) != 0;
  if ((o->flags & OSPF_SWEEP_EARLY_START) && !defer)
    return fail(c, OSPF_E_INVAL, "sweep: OSPF_SWEEP_EARLY_START needs OSPF_SWEEP_DEFER");
  if (defer && o->hip_graph)
    return fail(c, OSPF_E_INVAL, "sweep: OSPF_SWEEP_DEFER needs hip_graph = 0 (the capture "
                                 "follows the first run)");
  const bool hop = o->flags & OSPF_HOP_COUNT;
  if (!hop && c->dist_bound >= 0xFFFFFFFFull)
    return fail(c, OSPF_E_RANGE, "u32 distance overflow possible (sum of per-node max metrics)");
  ospf_sweep* s = new (std::nothrow) ospf_sweep();
  if (!s) return OSPF_E_NOMEM;
  s->c = c;
  c->live_sweeps.push_back(s);
  c->release_sweep = [](ospf_sweep* x) {  // ospf_close: release now, detach
    release(x);
    x->c = nullptr;
  };
  s->opts = *o;
  s->early = (o->flags & OSPF_SWEEP_EARLY_START) && !getenv("OSPF_SWEEP_NO_EARLY");
  s->gen = c->graph_gen;
  s->V = c->info.n_nodes;
  const uint32_t V = s->V;
  s->row_dist.assign(V, nullptr);
  s->row_nh.assign(V, nullptr);
  s->row_w.assign(V, 0);
  auto bail = [&](int rc) {
    const std::string m = s->err.empty() ? std::string(ospf_last_error(c)) : s->err;
    auto& lsw = c->live_sweeps;
    lsw.erase(std::remove(lsw.begin(), lsw.end(), s), lsw.end());
    release(s);
    delete s;
    c->err = m;
    return rc;
  };
  const bool tm = getenv("OSPF_SWEEP_TIMING") != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!tm) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "sweep_create %s %.2f ms\n", what,
            std::chrono::duration<double, std::milli>(t - t0).count());
    t0 = t;
  };
  if (hipSetDevice(c->device) != hipSuccess) return bail(fail(c, OSPF_E_DEVICE, "hipSetDevice"));
  if (new_stream(s) < 0 || new_event(s) < 0) return bail(OSPF_E_DEVICE);
  if (hipEventCreateWithFlags(&s->ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_out, hipEventDisableTiming) != hipSuccess)
    return bail(fail(c, OSPF_E_DEVICE, "hipEventCreate"));
  Facts f;
  f.V = V;
  f.dn_off = &c->h_dn_off;
  f.dn = &c->h_dn;
  const std::vector<uint32_t> mine = partition(f, parts, o->part);
  // path
  const bool unit = hop || c->info.unit_metric;
  const bool derive_ok = unit && c->max_dn <= 2048 && c->depth_bound <= 123;
  // small graphs: every root's next hops in <= 4 words and the graph in LDS
  const uint32_t max_w = std::max(1u, (c->max_dn + 31) / 32);
  const bool lds_ok = unit && max_w <= 4 && ospf_lds_sweep_fits(c, o->flags & OSPF_HOP_COUNT, max_w) &&
                      !getenv("OSPF_SWEEP_NOLDS");
  std::vector<uint8_t> leaf;
  bool any_leaf = false;
  uint32_t mode = o->mode;
  if (mode == OSPF_SWEEP_AUTO || mode == OSPF_SWEEP_WCOVER || mode == OSPF_SWEEP_WDERIVE ||
      mode == OSPF_SWEEP_WMULTI) {
    if (!(mode == OSPF_SWEEP_AUTO && derive_ok)) {
      leaf = leaf_set(f);
      for (uint8_t x : leaf) any_leaf |= x != 0;
    }
  }
  if (mode == OSPF_SWEEP_AUTO) {
    if (lds_ok) {
      mode = OSPF_SWEEP_LDS;
    } else if (derive_ok) {
      mode = OSPF_SWEEP_DERIVE;
    } else if (!hop && any_leaf && ospf_cover_prepare(c, leaf.data()) == OSPF_OK) {
      mode = OSPF_SWEEP_WCOVER;
    } else if (any_leaf) {
      mode = OSPF_SWEEP_WDERIVE;
    } else {
      mode = OSPF_SWEEP_BATCH;
    }
  } else if (mode == OSPF_SWEEP_DERIVE && !derive_ok) {
    return bail(fail(c, OSPF_E_RANGE, "sweep: derive needs unit metric or hop count, a depth "
                                      "bound <= 123 and <= 2048 distinct neighbours per node"));
  } else if (mode == OSPF_SWEEP_LDS && !lds_ok) {
    return bail(fail(c, OSPF_E_RANGE, "sweep: lds needs unit metric or hop count, <= 128 "
                                      "distinct neighbours per node and the graph in LDS"));
  } else if (mode == OSPF_SWEEP_WCOVER) {
    if (hop) return bail(fail(c, OSPF_E_INVAL, "sweep: the cover path runs link metrics"));
    const int rc = ospf_cover_prepare(c, leaf.data());
    if (rc) return bail(rc);
  }
  s->mode = mode;
  lap("partition + leaf set + cover prepare");
  int rc = OSPF_OK;
  switch (mode) {
    case OSPF_SWEEP_DERIVE: rc = plan_derive(s, f, mine); break;
    case OSPF_SWEEP_WCOVER: rc = plan_wcover(s, f, mine, leaf); break;
    case OSPF_SWEEP_WDERIVE: rc = plan_wderive(s, f, mine, leaf); break;
    case OSPF_SWEEP_WMULTI: rc = plan_wmulti(s, f, mine, leaf); break;
    case OSPF_SWEEP_LDS: rc = plan_lds(s, f, mine); break;
    default: rc = plan_batch(s, f, mine, !unit); break;
  }
  if (rc) return bail(rc);
  lap("plan");
  if (upload(s, &s->d_own_slot, s->own_slot)) return bail(OSPF_E_NOMEM);
  s->ev_done.assign(s->streams.size(), nullptr);
  for (size_t i = 1; i < s->streams.size(); ++i)
    if (hipEventCreateWithFlags(&s->ev_done[i], hipEventDisableTiming) != hipSuccess)
      return bail(fail(c, OSPF_E_DEVICE, "hipEventCreate"));
  lap("slots + events");
  if (defer) {  // the caller's first ospf_sweep_run is the first run
    *out = s;
    return OSPF_OK;
  }
  // one eager run: sizes every stream's scratch (nothing may allocate inside
  // a capture) and surfaces launch errors here
  const uint64_t runs0 = c->spf_runs;
  if ((rc = run_eager(s, s->streams[0]))) return bail(rc);
  if (hipStreamSynchronize(s->streams[0]) != hipSuccess)
    return bail(fail(c, OSPF_E_DEVICE, "sweep: first run failed"));
  if ((rc = ospf_sync(c, s->streams[0]))) return bail(rc);
  s->ran = true;
  if ((rc = pick_leaf_order(s))) return bail(rc);
  // the graph's seed BFS launches levels 1 .. the depth the eager run reached
  // (deterministic for this graph version; a deeper level would set error
  // bit 8 in the rows kernel) instead of the transit-depth bound (10 at
  // F100k, where the seeds' BFS ends at 4: 14 empty level launches).
  // OSPF_SWEEP_FULL_DEPTH keeps the bound.
  if (s->d_lv_maxd && !getenv("OSPF_SWEEP_FULL_DEPTH")) {
    uint32_t dm = 0;
    if (hipMemcpy(&dm, s->d_lv_maxd, 4, hipMemcpyDeviceToHost) != hipSuccess)
      return bail(fail(c, OSPF_E_DEVICE, "sweep: seed BFS depth readback"));
    if (dm >= 1 && dm < c->depth_bound) s->lv_cap = dm;
  }
  if (o->hip_graph) {
    hipStream_t m = s->streams[0];
    hipGraph_t g = nullptr;
    hipGraphExec_t ex = nullptr;
    bool ok = hipStreamBeginCapture(m, hipStreamCaptureModeRelaxed) == hipSuccess;
    if (ok) {
      const int erc = enqueue(s);
      ok = hipStreamEndCapture(m, &g) == hipSuccess && erc == OSPF_OK && g;
    }
    ok = ok && hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) == hipSuccess;
    if (ok) {
      s->graph = g;
      s->exec = ex;
    } else {
      if (ex) hipGraphExecDestroy(ex);
      if (g) hipGraphDestroy(g);
      (void)hipGetLastError();
      s->err.clear();
    }
  }
  c->spf_runs = runs0;
  *out = s;
  return OSPF_OK;
}

int ospf_sweep_destroy(ospf_sweep* s) {
  if (!s) return OSPF_E_INVAL;
  if (s->c) {
    auto& ls = s->c->live_sweeps;
    ls.erase(std::remove(ls.begin(), ls.end(), s), ls.end());
  }
  release(s);
  delete s;
  return OSPF_OK;
}

const char* ospf_sweep_last_error(const ospf_sweep* s) {
  return s ? s->err.c_str() : "null sweep";
}

int ospf_sweep_get_info(const ospf_sweep* s, ospf_sweep_info* info) {
  if (!s || !info) return OSPF_E_INVAL;
  info->mode = s->mode;
  info->n_roots = (uint32_t)s->roots.size();
  info->n_rows = s->n_rows;
  info->n_launches = (uint32_t)s->units.size();
  info->hip_graph = s->exec ? 1u : 0u;
  uint32_t mw = 0;
  for (uint32_t r : s->roots) mw = std::max(mw, s->row_w[r]);
  info->max_nh_words = mw;
  info->device_bytes = s->device_bytes;
  info->step_compulsory_bytes = s->step_comp;
  info->step_traversed_edges = s->trav_edges;
  return OSPF_OK;
}

int ospf_sweep_roots(const ospf_sweep* s, uint32_t* roots) {
  if (!s || (!roots && !s->roots.empty())) return OSPF_E_INVAL;
  std::copy(s->roots.begin(), s->roots.end(), roots);
  return OSPF_OK;
}

int ospf_sweep_run(ospf_sweep* s, void* stream) {
  if (!s) return OSPF_E_INVAL;
  ospf_ctx* c = s->c;
  if (ospf_int::injected(c)) return sfail(s, OSPF_E_DEVICE, c->err);
  if (c->graph_gen != s->gen || c->mask.on)
    return sfail(s, OSPF_E_NOGRAPH, "sweep: the graph changed since the sweep was created");
  SCHK(s, hipSetDevice(c->device));
  const uint64_t runs0 = c->spf_runs;
  if (s->exec) {
    SCHK(s, hipGraphLaunch(s->exec, (hipStream_t)stream));
  } else {
    const int rc = run_eager(s, (hipStream_t)stream);
    if (rc) return rc;
  }
  s->ran = true;
  c->spf_runs = runs0 + s->roots.size();
  return OSPF_OK;
}

int ospf_sweep_digests(ospf_sweep* s, ospf_digest* d_out, void* stream) {
  if (!s || (!d_out && !s->roots.empty())) return OSPF_E_INVAL;
  const uint32_t n = (uint32_t)s->roots.size();
  if (!n) return OSPF_OK;
  // a deferred sweep (OSPF_SWEEP_DEFER) has no rows or digests before its run
  if (!s->ran) return sfail(s, OSPF_E_INVAL, "sweep: digests before the first run");
  SCHK(s, hipSetDevice(s->c->device));
  hipLaunchKernelGGL(gather_digest_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, s->dig_all, s->d_own_slot, n, d_out);
  SCHK(s, hipGetLastError());
  return OSPF_OK;
}

int ospf_sweep_digests_host(ospf_sweep* s, ospf_digest* out) {
  if (!s || (!out && !s->roots.empty())) return OSPF_E_INVAL;
  const size_t n = s->roots.size();
  if (!n) return OSPF_OK;
  SCHK(s, hipSetDevice(s->c->device));
  ospf_digest* d = nullptr;
  SCHK(s, hipMalloc(&d, n * sizeof(ospf_digest)));
  int rc = ospf_sweep_digests(s, d, nullptr);
  hipError_t e = hipSuccess;
  if (rc == OSPF_OK) e = hipMemcpy(out, d, n * sizeof(ospf_digest), hipMemcpyDeviceToHost);
  hipFree(d);
  if (e != hipSuccess) return sfail(s, OSPF_E_DEVICE, std::string("hipMemcpy: ") + hipGetErrorString(e));
  return rc;
}

int ospf_sweep_poison(ospf_sweep* s, void* stream) {
  if (!s) return OSPF_E_INVAL;
  SCHK(s, hipSetDevice(s->c->device));
  // a kernel, not hipMemsetAsync: see ospf::zero_async
  auto fill = [&](void* p, size_t words) {
    return ospf::zero_by_memset() ? hipMemsetAsync(p, 0xFF, words * 4u, (hipStream_t)stream)
                                  : ospf::launch_fill32((uint32_t*)p, words, 0xFFFFFFFFu,
                                                        (hipStream_t)stream);
  };
  SCHK(s, fill(s->dig_all, (size_t)std::max(1u, s->n_dig) * 6u));
  for (auto& a : s->dig_aux) SCHK(s, fill(a.first, std::max<size_t>(1, a.second) * 6u));
  return OSPF_OK;
}

int ospf_sweep_graph_memsets(const ospf_sweep* s, uint32_t* n_memset, uint32_t* n_dead,
                             uint32_t* n_own) {
  if (!s || !n_memset || !n_dead || !n_own) return OSPF_E_INVAL;
  *n_memset = *n_dead = *n_own = 0;
  if (!s->graph) return OSPF_OK;
  size_t nn = 0;
  if (hipGraphGetNodes(s->graph, nullptr, &nn) != hipSuccess) return OSPF_E_DEVICE;
  std::vector<hipGraphNode_t> nodes(nn);
  if (nn && hipGraphGetNodes(s->graph, nodes.data(), &nn) != hipSuccess) return OSPF_E_DEVICE;
  for (hipGraphNode_t g : nodes) {
    hipGraphNodeType ty;
    if (hipGraphNodeGetType(g, &ty) != hipSuccess) return OSPF_E_DEVICE;
    if (ty != hipGraphNodeTypeMemset) continue;
    hipMemsetParams p{};
    if (hipGraphMemsetNodeGetParams(g, &p) != hipSuccess) return OSPF_E_DEVICE;
    ++*n_memset;
    const char* dst = static_cast<const char*>(p.dst);
    const size_t bytes = (size_t)p.elementSize * p.width * std::max<size_t>(1, p.height);
    // live allocation around [dst, dst + bytes)?
    hipDeviceptr_t base = nullptr;
    size_t sz = 0;
    if (hipMemGetAddressRange(&base, &sz, (hipDeviceptr_t)dst) != hipSuccess ||
        dst + bytes > static_cast<const char*>(base) + sz) {
      ++*n_dead;
      (void)hipGetLastError();
    }
    for (size_t i = 0; i < s->allocs.size() && i < s->alloc_bytes.size(); ++i) {
      const char* a = static_cast<const char*>(s->allocs[i]);
      if (dst >= a && dst + bytes <= a + s->alloc_bytes[i]) {
        ++*n_own;
        break;
      }
    }
  }
  return OSPF_OK;
}

int ospf_sweep_row(const ospf_sweep* s, uint32_t root, const uint32_t** d_dist,
                   const uint32_t** d_nh, uint32_t* nh_words) {
  if (!s || root >= s->V || !s->ran) return OSPF_E_INVAL;  // no rows before the first run
  if (!s->row_dist[root]) return OSPF_E_RANGE;
  if (d_dist) *d_dist = s->row_dist[root];
  if (d_nh) *d_nh = s->row_nh[root];
  if (nh_words) *nh_words = s->row_w[root];
  return OSPF_OK;
}

int ospf_sweep_copy_rows(ospf_sweep* s, const uint32_t* roots, uint32_t n, uint32_t nh_words,
                         uint32_t* dist_out, uint32_t* nh_out) {
  if (!s || (n && !roots)) return OSPF_E_INVAL;
  if (ospf_int::injected(s->c)) return sfail(s, OSPF_E_DEVICE, s->c->err);
  if (!s->ran) return sfail(s, OSPF_E_INVAL, "sweep: rows before the first run");
  const uint32_t V = s->V;
  for (uint32_t i = 0; i < n; ++i) {
    if (roots[i] >= V || !s->row_dist[roots[i]])
      return sfail(s, OSPF_E_RANGE, "sweep: root " + std::to_string(roots[i]) + " not owned");
    if (nh_out && s->row_w[roots[i]] > nh_words)
      return sfail(s, OSPF_E_INVAL, "sweep: nh_words below a root's next-hop words");
  }
  SCHK(s, hipSetDevice(s->c->device));
  SCHK(s, hipDeviceSynchronize());
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t r = roots[i], W = s->row_w[r];
    if (dist_out)
      SCHK(s, hipMemcpy(dist_out + (size_t)i * V, s->row_dist[r], (size_t)V * 4,
                        hipMemcpyDeviceToHost));
    if (nh_out) {
      uint32_t* dst = nh_out + (size_t)i * V * nh_words;
      if (W == nh_words) {
        SCHK(s, hipMemcpy(dst, s->row_nh[r], (size_t)V * W * 4, hipMemcpyDeviceToHost));
      } else {
        std::memset(dst, 0, (size_t)V * nh_words * 4);
        SCHK(s, hipMemcpy2D(dst, (size_t)nh_words * 4, s->row_nh[r], (size_t)W * 4, (size_t)W * 4,
                            V, hipMemcpyDeviceToHost));
      }
    }
  }
  return OSPF_OK;
}

int ospf_sweep_profile(ospf_sweep* s, uint32_t reps, ospf_sweep_launch* out, uint32_t cap) {
  if (!s || (cap && !out)) return OSPF_E_INVAL;
  if (!s->ran) return sfail(s, OSPF_E_INVAL, "sweep: profile needs one run first");
  ospf_ctx* c = s->c;
  if (c->graph_gen != s->gen) return sfail(s, OSPF_E_NOGRAPH, "sweep: the graph changed");
  reps = std::max(1u, reps);
  SCHK(s, hipSetDevice(c->device));
  SCHK(s, hipDeviceSynchronize());
  const uint64_t runs0 = c->spf_runs;
  hipEvent_t a, b;
  SCHK(s, hipEventCreate(&a));
  SCHK(s, hipEventCreate(&b));
  for (size_t i = 0; i < s->units.size() && i < cap; ++i) {
    auto& u = s->units[i];
    hipStream_t st = s->streams[u.stream];
    std::vector<double> ms;
    hipLaunchKernelGGL(sweep_unit_mark_kernel, dim3(1), dim3(64), 0, st, (uint32_t)i);
    SCHK(s, hipGetLastError());
    for (uint32_t k = 0; k <= reps; ++k) {
      SCHK(s, hipEventRecord(a, st));
      const int rc = u.fn(st);
      if (rc) return sfail(s, rc, u.name + ": " + ospf_last_error(c));
      SCHK(s, hipEventRecord(b, st));
      SCHK(s, hipEventSynchronize(b));
      float t = 0;
      SCHK(s, hipEventElapsedTime(&t, a, b));
      if (k) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    ospf_sweep_launch& L = out[i];
    std::memset(&L, 0, sizeof(L));
    std::snprintf(L.name, sizeof(L.name), "%s", u.name.c_str());
    std::snprintf(L.kernel, sizeof(L.kernel), "%s", u.kernel.c_str());
    L.n_roots = u.n_roots;
    L.nh_words = u.W;
    L.compulsory_bytes = u.comp;
    L.ms_median = ms[ms.size() / 2];
    L.ms_min = ms.front();
  }
  hipLaunchKernelGGL(sweep_unit_mark_kernel, dim3(1), dim3(64), 0, s->streams[0],
                     (uint32_t)s->units.size());
  SCHK(s, hipStreamSynchronize(s->streams[0]));
  hipEventDestroy(a);
  hipEventDestroy(b);
  c->spf_runs = runs0;
  return ospf_sync(c, nullptr);
}

}  // extern "C"

// ---------------------------------------------------------------- devices
struct ospf_multi {
  std::vector<ospf_ctx*> ctx;
  std::string err;
  // RCCL communicators, one per device slot (ncclCommInitAll in this
  // process): the digest gather of a sweep is one ncclAllGather over xGMI.
  // 0 = not tried, 1 = live, -1 = unavailable (duplicate devices -- RCCL
  // takes one rank per GPU -- or init failed: peer copies instead)
  int rccl = 0;
  std::vector<ncclComm_t> comms;
};

struct ospf_msweep {
  ospf_multi* m = nullptr;
  std::vector<ospf_sweep*> parts;
  std::vector<uint32_t> owner;          // slot owning each node (kNone: none)
  uint32_t V = 0;
  ospf_digest* d_all = nullptr;         // device 0: [total owned] part digests, part order
  uint32_t* d_roots = nullptr;          // device 0: their root ids
  ospf_digest* d_by_node = nullptr;     // device 0: [V]
  std::vector<ospf_digest*> d_part;     // per slot (on its device): [slot] (padded)
  uint32_t total = 0;
  // RCCL gather: every part's digests padded to `slot` entries, all-gathered
  // into d_recv on every device; d_roots_pad (device 0) = the root of each
  // gathered entry (kNone: padding)
  uint32_t slot = 0;
  std::vector<ospf_digest*> d_recv;     // per slot (on its device): [n_parts * slot]
  uint32_t* d_roots_pad = nullptr;
};

namespace {
// RCCL communicators for the multi context, once: distinct devices only
// (OSPF_RCCL=1 also takes a single device -- a one-rank communicator, which
// exercises the path on a one-GPU box; OSPF_RCCL=0 keeps peer copies)
bool multi_rccl(ospf_multi* m) {
  if (m->rccl) return m->rccl > 0;
  m->rccl = -1;
  const char* e = getenv("OSPF_RCCL");
  if (e && e[0] == '0') return false;
  const size_t n = m->ctx.size();
  std::vector<int> devs;
  for (ospf_ctx* c : m->ctx) devs.push_back(c->device);
  std::vector<int> u = devs;
  std::sort(u.begin(), u.end());
  if (std::unique(u.begin(), u.end()) != u.end()) return false;  // a device twice
  if (n < 2 && !(e && e[0] == '1')) return false;
  m->comms.assign(n, nullptr);
  if (ncclCommInitAll(m->comms.data(), (int)n, devs.data()) != ncclSuccess) {
    m->comms.clear();
    return false;
  }
  m->rccl = 1;
  return true;
}
}  // namespace

extern "C" {

int ospf_multi_open(const int* devices, uint32_t n, ospf_multi** out) {
  if (!devices || !n || !out) return OSPF_E_INVAL;
  *out = nullptr;
  ospf_multi* m = new (std::nothrow) ospf_multi();
  if (!m) return OSPF_E_NOMEM;
  for (uint32_t i = 0; i < n; ++i) {
    ospf_ctx* c = nullptr;
    const int rc = ospf_open(devices[i], &c);
    if (rc) {
      for (ospf_ctx* x : m->ctx) ospf_close(x);
      delete m;
      return rc;
    }
    m->ctx.push_back(c);
  }
  // peer access between distinct devices (xGMI); same-device slots need none
  for (uint32_t i = 0; i < n; ++i)
    for (uint32_t j = 0; j < n; ++j) {
      if (devices[i] == devices[j]) continue;
      int can = 0;
      hipDeviceCanAccessPeer(&can, devices[i], devices[j]);
      if (can) {
        hipSetDevice(devices[i]);
        hipDeviceEnablePeerAccess(devices[j], 0);
        (void)hipGetLastError();  // already enabled
      }
    }
  *out = m;
  return OSPF_OK;
}

int ospf_multi_close(ospf_multi* m) {
  if (!m) return OSPF_E_INVAL;
  for (ncclComm_t cm : m->comms)
    if (cm) ncclCommDestroy(cm);
  for (ospf_ctx* c : m->ctx) ospf_close(c);
  delete m;
  return OSPF_OK;
}

const char* ospf_multi_last_error(const ospf_multi* m) { return m ? m->err.c_str() : "null"; }

uint32_t ospf_multi_size(const ospf_multi* m) { return m ? (uint32_t)m->ctx.size() : 0u; }

ospf_ctx* ospf_multi_ctx(ospf_multi* m, uint32_t i) {
  return (m && i < m->ctx.size()) ? m->ctx[i] : nullptr;
}

int ospf_multi_load_graph(ospf_multi* m, const ospf_csr* csr, uint64_t version) {
  if (!m) return OSPF_E_INVAL;
  for (ospf_ctx* c : m->ctx) {
    const int rc = ospf_load_graph(c, csr, version);
    if (rc) {
      m->err = ospf_last_error(c);
      return rc;
    }
  }
  return OSPF_OK;
}

int ospf_msweep_destroy(ospf_msweep* ms) {
  if (!ms) return OSPF_E_INVAL;
  for (size_t i = 0; i < ms->parts.size(); ++i) {
    hipSetDevice(ms->m->ctx[i]->device);
    if (i < ms->d_part.size() && ms->d_part[i]) hipFree(ms->d_part[i]);
    if (i < ms->d_recv.size() && ms->d_recv[i]) hipFree(ms->d_recv[i]);
    ospf_sweep_destroy(ms->parts[i]);
  }
  if (!ms->m->ctx.empty()) hipSetDevice(ms->m->ctx[0]->device);
  if (ms->d_roots_pad) hipFree(ms->d_roots_pad);
  if (!ms->m->ctx.empty()) hipSetDevice(ms->m->ctx[0]->device);
  if (ms->d_all) hipFree(ms->d_all);
  if (ms->d_roots) hipFree(ms->d_roots);
  if (ms->d_by_node) hipFree(ms->d_by_node);
  delete ms;
  return OSPF_OK;
}

int ospf_msweep_create(ospf_multi* m, const ospf_sweep_opts* o, ospf_msweep** out) {
  if (!m || !o || !out || m->ctx.empty()) return OSPF_E_INVAL;
  *out = nullptr;
  ospf_msweep* ms = new (std::nothrow) ospf_msweep();
  if (!ms) return OSPF_E_NOMEM;
  ms->m = m;
  const uint32_t n = (uint32_t)m->ctx.size();
  auto bail = [&](int rc, const std::string& msg) {
    m->err = msg;
    ospf_msweep_destroy(ms);
    return rc;
  };
  ms->V = m->ctx[0]->info.n_nodes;
  ms->owner.assign(ms->V, kNone);
  std::vector<uint32_t> all_roots;
  for (uint32_t i = 0; i < n; ++i) {
    ospf_sweep_opts oi = *o;
    oi.part = i;
    oi.n_parts = n;
    // without HIP graphs no part runs at create: ospf_msweep_run starts every
    // device's first run together (a capture needs its part's eager run)
    if (!o->hip_graph) oi.flags |= OSPF_SWEEP_DEFER;
    ospf_sweep* s = nullptr;
    const int rc = ospf_sweep_create(m->ctx[i], &oi, &s);
    if (rc) return bail(rc, ospf_last_error(m->ctx[i]));
    ms->parts.push_back(s);
    for (uint32_t r : s->roots) ms->owner[r] = i;
    all_roots.insert(all_roots.end(), s->roots.begin(), s->roots.end());
    ms->slot = std::max<uint32_t>(ms->slot, (uint32_t)s->roots.size());
  }
  ms->slot = std::max(ms->slot, 1u);
  for (uint32_t i = 0; i < n; ++i) {  // digests padded to the widest part
    ospf_digest* dp = nullptr;
    hipSetDevice(m->ctx[i]->device);
    if (hipMalloc(&dp, (size_t)ms->slot * sizeof(ospf_digest)) != hipSuccess)
      return bail(OSPF_E_NOMEM, "msweep: hipMalloc");
    ms->d_part.push_back(dp);
    if (hipMemset(dp, 0, (size_t)ms->slot * sizeof(ospf_digest)) != hipSuccess)
      return bail(OSPF_E_DEVICE, "msweep: hipMemset");
  }
  if (multi_rccl(m)) {
    for (uint32_t i = 0; i < n; ++i) {
      ospf_digest* dr = nullptr;
      hipSetDevice(m->ctx[i]->device);
      if (hipMalloc(&dr, (size_t)n * ms->slot * sizeof(ospf_digest)) != hipSuccess)
        return bail(OSPF_E_NOMEM, "msweep: hipMalloc");
      ms->d_recv.push_back(dr);
    }
    std::vector<uint32_t> pad((size_t)n * ms->slot, kNone);
    for (uint32_t i = 0; i < n; ++i)
      std::copy(ms->parts[i]->roots.begin(), ms->parts[i]->roots.end(), pad.begin() + (size_t)i * ms->slot);
    hipSetDevice(m->ctx[0]->device);
    if (hipMalloc(&ms->d_roots_pad, pad.size() * 4) != hipSuccess ||
        hipMemcpy(ms->d_roots_pad, pad.data(), pad.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
      return bail(OSPF_E_NOMEM, "msweep: root table");
  }
  ms->total = (uint32_t)all_roots.size();
  hipSetDevice(m->ctx[0]->device);
  if (hipMalloc(&ms->d_all, std::max<size_t>(1, ms->total) * sizeof(ospf_digest)) != hipSuccess ||
      hipMalloc(&ms->d_roots, std::max<size_t>(1, ms->total) * 4) != hipSuccess ||
      hipMalloc(&ms->d_by_node, (size_t)ms->V * sizeof(ospf_digest)) != hipSuccess)
    return bail(OSPF_E_NOMEM, "msweep: hipMalloc");
  if (hipMemcpy(ms->d_roots, all_roots.data(), all_roots.size() * 4, hipMemcpyHostToDevice) !=
      hipSuccess)
    return bail(OSPF_E_DEVICE, "msweep: hipMemcpy");
  *out = ms;
  return OSPF_OK;
}

int ospf_msweep_run(ospf_msweep* ms) {
  if (!ms) return OSPF_E_INVAL;
  // queue every device's run first, then wait: the devices run concurrently
  for (size_t i = 0; i < ms->parts.size(); ++i) {
    const int rc = ospf_sweep_run(ms->parts[i], nullptr);
    if (rc) {
      ms->m->err = ospf_sweep_last_error(ms->parts[i]);
      return rc;
    }
  }
  for (size_t i = 0; i < ms->parts.size(); ++i) {
    const int rc = ospf_sync(ms->m->ctx[i], nullptr);
    if (rc) {
      ms->m->err = ospf_last_error(ms->m->ctx[i]);
      return rc;
    }
  }
  return OSPF_OK;
}

int ospf_msweep_digests(ospf_msweep* ms, ospf_digest* out) {
  if (!ms || !out) return OSPF_E_INVAL;
  ospf_ctx* c0 = ms->m->ctx[0];
  if (!ms->d_recv.empty()) {
    // every part's digests (queued on its device's stream), then ONE
    // ncclAllGather of the padded records; device 0 scatters them by root
    const size_t n = ms->parts.size();
    for (size_t i = 0; i < n; ++i) {
      const int rc = ospf_sweep_digests(ms->parts[i], ms->d_part[i], nullptr);
      if (rc) {
        ms->m->err = ms->parts[i]->err;
        return rc;
      }
    }
    ncclResult_t nr = ncclGroupStart();
    for (size_t i = 0; i < n && nr == ncclSuccess; ++i) {
      hipSetDevice(ms->m->ctx[i]->device);
      nr = ncclAllGather(ms->d_part[i], ms->d_recv[i], (size_t)ms->slot * 3, ncclUint64,
                         ms->m->comms[i], (hipStream_t)0);
    }
    const ncclResult_t ne = ncclGroupEnd();
    if (nr != ncclSuccess || ne != ncclSuccess) {
      ms->m->err = std::string("msweep: ncclAllGather: ") + ncclGetErrorString(nr != ncclSuccess ? nr : ne);
      return OSPF_E_DEVICE;
    }
    hipSetDevice(c0->device);
    hipMemset(ms->d_by_node, 0, (size_t)ms->V * sizeof(ospf_digest));
    const uint32_t tot = (uint32_t)(n * ms->slot);
    hipLaunchKernelGGL(scatter_digest_kernel, dim3((tot + 255) / 256), dim3(256), 0, 0,
                       ms->d_recv[0], ms->d_roots_pad, tot, ms->d_by_node);
    if (hipMemcpy(out, ms->d_by_node, (size_t)ms->V * sizeof(ospf_digest), hipMemcpyDeviceToHost) !=
        hipSuccess) {
      ms->m->err = "msweep: hipMemcpy";
      return OSPF_E_DEVICE;
    }
    return OSPF_OK;
  }
  size_t off = 0;
  for (size_t i = 0; i < ms->parts.size(); ++i) {
    ospf_sweep* s = ms->parts[i];
    const size_t n = s->roots.size();
    int rc = ospf_sweep_digests(s, ms->d_part[i], nullptr);
    if (rc) {
      ms->m->err = s->err;
      return rc;
    }
    hipSetDevice(ms->m->ctx[i]->device);
    if (hipDeviceSynchronize() != hipSuccess) return OSPF_E_DEVICE;
    if (n && hipMemcpyPeer(ms->d_all + off, c0->device, ms->d_part[i], ms->m->ctx[i]->device,
                           n * sizeof(ospf_digest)) != hipSuccess) {
      ms->m->err = "msweep: hipMemcpyPeer";
      return OSPF_E_DEVICE;
    }
    off += n;
  }
  hipSetDevice(c0->device);
  hipMemset(ms->d_by_node, 0, (size_t)ms->V * sizeof(ospf_digest));
  if (ms->total)
    hipLaunchKernelGGL(scatter_digest_kernel, dim3((ms->total + 255) / 256), dim3(256), 0, 0,
                       ms->d_all, ms->d_roots, ms->total, ms->d_by_node);
  if (hipMemcpy(out, ms->d_by_node, (size_t)ms->V * sizeof(ospf_digest), hipMemcpyDeviceToHost) !=
      hipSuccess) {
    ms->m->err = "msweep: hipMemcpy";
    return OSPF_E_DEVICE;
  }
  return OSPF_OK;
}

ospf_sweep* ospf_msweep_part(ospf_msweep* ms, uint32_t slot) {
  return (ms && slot < ms->parts.size()) ? ms->parts[slot] : nullptr;
}

uint32_t ospf_msweep_gather_backend(const ospf_msweep* ms) {
  return (ms && !ms->d_recv.empty()) ? 1u : 0u;
}

int ospf_msweep_owner(const ospf_msweep* ms, uint32_t root, uint32_t* slot) {
  if (!ms || !slot || root >= ms->V) return OSPF_E_INVAL;
  if (ms->owner[root] == kNone) return OSPF_E_RANGE;
  *slot = ms->owner[root];
  return OSPF_OK;
}

}  // extern "C"
