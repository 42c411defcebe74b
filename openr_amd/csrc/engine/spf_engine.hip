// spf_engine.hip — C ABI of libopenr_spf_hip (include/openr_spf.h).
//
// Owns the device-resident CSR snapshot of one LinkState (area), picks the
// kernel variant for a batch (LDS-resident vs HBM-streamed state) and launches
// one workgroup per SPF run. No CPU fallback: a missing device or an
// out-of-contract graph is an error code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <mutex>
#include <functional>
#include <cstdio>
#include <map>
#include <unordered_map>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "spf_internal.h"

namespace ospf_int {

int fail(ospf_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hip_fail(ospf_ctx* c, hipError_t e, const char* what) {
  return fail(c, OSPF_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

bool injected(ospf_ctx* c) {
  if (!c || !c->inject_after || --c->inject_after) return false;
  fail(c, OSPF_E_DEVICE, "injected device error (ospf_inject_error)");
  return true;
}

void pool_release(ospf_ctx* c) {
  for (auto& kv : c->sweep_pool) (void)hipFree(kv.second);
  c->sweep_pool.clear();
  c->sweep_pool_bytes = 0;
}

hipError_t dev_malloc(ospf_ctx* c, void** p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess && c && !c->sweep_pool.empty()) {  // the pooled blocks back first
    (void)hipGetLastError();
    // a rare, slow path (hipFree of pooled row blocks): said on stderr, so a
    // stall in a caller's timing can be traced to it
    const auto t0 = std::chrono::steady_clock::now();
    const size_t nb = c->sweep_pool.size(), pb = c->sweep_pool_bytes;
    pool_release(c);
    e = hipMalloc(p, bytes);
    fprintf(stderr, "ospf: hipMalloc of %zu B failed: released %zu pooled sweep blocks (%.2f GB) in %.1f ms, retry %s\n",
            bytes, nb, pb / 1e9,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
            e == hipSuccess ? "ok" : "failed");
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *p = nullptr;
  }
  return e;
}

static int ensure(ospf_ctx* c, void** p, size_t* have, size_t need) {
  if (*have >= need) return OSPF_OK;
  const size_t want = std::max(need, *have * 3 / 2);
  if (*p) hipFree(*p);
  *p = nullptr;
  *have = 0;
  hipError_t e = dev_malloc(c, p, want);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(c, OSPF_E_NOMEM, std::string("hipMalloc scratch: ") + hipGetErrorString(e));
  }
  *have = want;
  return OSPF_OK;
}

char* stream_scratch(ospf_ctx* c, void* stream, size_t need, int* rc, int slot) {
  ospf_ctx::Scratch& sc = c->scratch[(char*)stream + slot];
  *rc = OSPF_OK;
  if (sc.bytes >= need) return (char*)sc.p;
  if (sc.p) hipStreamSynchronize((hipStream_t)stream);
  *rc = ensure(c, &sc.p, &sc.bytes, need);
  return (char*)sc.p;
}

void release_stream_scratch(ospf_ctx* c, void* stream) {
  for (int slot = 0; slot < 5; ++slot) {
    auto it = c->scratch.find((char*)stream + slot);
    if (it == c->scratch.end()) continue;
    if (it->second.p) hipFree(it->second.p);
    c->scratch.erase(it);
  }
}

}  // namespace ospf_int

using namespace ospf_int;

namespace {


struct Plan {
  int variant;
  uint32_t block;
  size_t lds;
  uint32_t nbr_cap, ign_cap;
};

// multi-source BFS (variant 5) pays a fixed per-level cost for a whole
// 64-root batch; below this many roots the per-root kernels win
constexpr uint32_t kMsMinRoots = 32;

Plan make_plan(const ospf_ctx* c, uint32_t W, uint32_t ign_cap, bool unit, uint32_t n_roots) {
  Plan p{};
  const size_t V = c->info.n_nodes;
  p.nbr_cap = (uint32_t)align_up(std::max<uint32_t>(c->max_dn, 1), 4);
  p.ign_cap = (uint32_t)align_up(ign_cap, 4);
  const size_t head = (32 + p.nbr_cap + p.ign_cap) * 4;
  const size_t full = head + V * 4 + V * W * 4;   // variant 0
  const size_t half = head + V * 4;               // variant 1
  const size_t bw = (((V + 31) / 32) + 1) & ~(size_t)1;
  const size_t bfs = head + 3 * bw * 4;            // variant 4
  const size_t bfs_nh = bfs + ((V + 3) / 4) * 4;   // variant 3
  const size_t lim = c->lds_limit;
  auto fits = [&](int v) {
    switch (v) {
      case 0: return full <= lim;
      case 1: return half <= lim;
      case 2: return true;
      case 3: return unit && bfs_nh <= lim;
      case 4: return unit && bfs <= lim;
      case 5: return unit && ign_cap == 0;
      case 6: return !unit && c->info.max_metric + 1 <= ospf::kMaxDialRing;
      case 7: return true;
    }
    return false;
  };
  // wide roots (many next-hop words) go multi-source even in small batches:
  // the per-root kernel re-runs the traversal per 4-word slice
  if (unit && fits(5) && (n_roots >= kMsMinRoots || (W >= 8 && n_roots >= 4))) {
    p.variant = 5;
  } else if (unit) {
    p.variant = (W == 1 && fits(3)) ? 3 : fits(4) ? 4 : 7;
  } else {
    // beyond LDS: a wave per root over frontier lists (variant 7), any metric
    p.variant = fits(0) ? 0 : fits(1) ? 1 : 7;
  }
  // test/benchmark knob: OSPF_FORCE_VARIANT=0..4 forces a kernel variant when
  // its state fits (e.g. the HBM-state Dial kernel on a small graph).
  if (const char* f = getenv("OSPF_FORCE_VARIANT")) {
    const int want = atoi(f);
    if (want >= 0 && want <= 7 && fits(want)) p.variant = want;
  }
  const size_t ldsz[8] = {full, half, head, bfs_nh, bfs, 0, head, 0};
  p.lds = ldsz[p.variant];
  if (p.variant >= 5)
    p.block = 256;
  else if (p.variant >= 3)
    p.block = p.lds > 80 * 1024 ? 1024 : (V >= 4096 ? 512 : 256);
  else
    p.block = V >= 4096 ? 512 : 256;
  if (const char* b = getenv("OSPF_BLOCK")) {  // experiment knob: 256/512/1024
    const int want = atoi(b);
    if (want == 256 || want == 512 || want == 1024) p.block = (uint32_t)want;
  }
  return p;
}

// Upper bound on the number of BFS levels (max hop distance) from any root.
// A shortest path r = x0, x1, ..., xk = v has transit interior nodes
// x1..x(k-1) (overloaded nodes never relax, LinkState.cpp:859-866), and its
// interior is a shortest path of the transit subgraph G' (usable links
// between transit nodes), so k <= diam(component) + 2 <= 2 * ecc(seed) + 2.
// O(V + E) on the host at load time; lets the multi-source BFS launch a
// fixed number of level kernels with no device -> host round trip.
uint32_t transit_depth_bound(uint32_t V, const uint32_t* row_ptr, const uint32_t* colx,
                             const std::vector<uint32_t>& nt) {
  auto transit = [&](uint32_t u) { return !((nt[u >> 5] >> (u & 31)) & 1u); };
  std::vector<uint32_t> lvl(V, 0xFFFFFFFFu), q;
  q.reserve(V);
  uint32_t ecc_max = 0;
  for (uint32_t s = 0; s < V; ++s) {
    if (!transit(s) || lvl[s] != 0xFFFFFFFFu) continue;
    q.clear();
    q.push_back(s);
    lvl[s] = 0;
    uint32_t ecc = 0;
    for (size_t i = 0; i < q.size(); ++i) {
      const uint32_t u = q[i];
      for (uint32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
        const uint32_t cx = colx[e];
        if (cx & 0x80000000u) continue;
        if (!transit(cx) || lvl[cx] != 0xFFFFFFFFu) continue;
        lvl[cx] = lvl[u] + 1;
        ecc = std::max(ecc, lvl[cx]);
        q.push_back(cx);
      }
    }
    ecc_max = std::max(ecc_max, ecc);
  }
  return 2u * ecc_max + 2u;
}

// Batch shape of the multi-source BFS for n roots with at most kcap distinct
// neighbours: R roots per traversal, PP planes per 64-bit plane word, KP
// plane words per node, OW next-hop words per pass, npass passes per batch.
struct MsShape {
  uint32_t R = 64, PP = 1, KP = 32, OW = 1, npass = 1;
};

// Packing (R < 64) trades launch parallelism for fewer traversals: measured
// slower for a 12-spine batch on F100k (fewer, denser passes; the plane-presence
// skip is per root), so it is opt-in (OSPF_MS_PACK=1 or OSPF_MS_R) for now.
MsShape ms_shape(uint32_t n, uint32_t kcap, bool pack) {
  MsShape m;
  if (kcap <= 32) {  // one pass, one word: 64 roots, as few planes as will do
    m.KP = kcap <= 8 ? 8 : kcap <= 16 ? 16 : 32;
    return m;
  }
  // wide roots: KP = 32 words; pick R minimising the traversals
  // ceil(n / R) * ceil(kcap / (32 * PP)) (ties: more roots per traversal)
  m.KP = 32;
  m.npass = (kcap + 31) / 32;
  if (!pack) return m;
  const uint64_t t64 = (uint64_t)((n + 63) / 64) * m.npass;
  uint64_t best = ~0ull;
  for (uint32_t R = 64; R >= 1; --R) {
    const uint32_t PP = 64 / R;
    const uint64_t t = (uint64_t)((n + R - 1) / R) * ((kcap + 32 * PP - 1) / (32 * PP));
    if (t < best) {
      best = t;
      m.R = R;
      m.PP = PP;
    }
  }
  if (4 * best > 3 * t64) {  // packing must save a quarter of the traversals
    m.R = 64;
    m.PP = 1;
    return m;
  }
  m.OW = m.PP;
  m.npass = (kcap + 32 * m.OW - 1) / (32 * m.OW);
  return m;
}

// Variant 5: multi-source bit-parallel BFS (spf_msbfs.hip). Roots go in
// R-root batches; each batch runs npass passes (OW next-hop words each); a
// round runs up to `nb` (batch, pass) pairs side by side. All launches are
// queued on `s`; nothing waits on the host.
int run_msbfs(ospf_ctx* c, const ospf_batch* b, hipStream_t s) {
  const uint32_t V = c->info.n_nodes, W = b->nh_words, flags = b->flags;
  const uint32_t kcap = b->max_root_neighbors ? std::min(b->max_root_neighbors, 32u * W) : 32u * W;
  const bool dig = flags & OSPF_WANT_DIGEST;
  const uint32_t lmax = c->depth_bound + 2;
  // levels are recorded as dist + 1 in a byte per (node, root): rows are then
  // written once, whole, by msbfs_rows (needs depth + 2 <= 255: the check
  // level past the bound is recorded too), which also folds
  // the digest in (no row re-read, no row scratch); packed planes need it
  const bool defer = c->depth_bound <= 253 && !getenv("OSPF_MS_NODEFER");
  MsShape sh = ms_shape(b->n_roots, kcap, defer && getenv("OSPF_MS_PACK"));
  if (const char* e = getenv("OSPF_MS_R")) {  // test knob: force R (packs when defer)
    const uint32_t R = std::min(64, std::max(1, atoi(e)));
    if (defer && kcap > 32) {
      sh.R = R;
      sh.PP = sh.OW = 64 / R;
      sh.npass = (kcap + 32 * sh.OW - 1) / (32 * sh.OW);
    }
  }
  if (!(flags & (OSPF_WANT_NH | OSPF_WANT_DIGEST))) {  // distances only: one pass, no planes used
    sh.R = 64;
    sh.PP = sh.OW = sh.npass = 1;
    sh.KP = 8;
  }
  const int kp = (int)sh.KP;
  const uint32_t npass = sh.npass;
  uint64_t rep = 0;
  for (uint32_t j = 0; j < sh.PP; ++j) rep |= 1ull << (j * sh.R);
  const bool dist_scr = dig && !defer && !(flags & OSPF_WANT_DIST);
  const bool nh_scr = dig && !defer && !(flags & OSPF_WANT_NH);
  // seen, accb, 2 frontier records (16 B), planes (u64 per node each) + lev
  // (64 B per node) + found, mass
  const size_t per_vb = align_up((size_t)V * 8ull * (6 + kp) + (defer ? V * 64ull : 0) + lmax * 8ull, 256);
  uint32_t push_div = 8;  // push a level when its frontier's edge mass * push_div < E
  if (const char* e = getenv("OSPF_MS_PUSH_DIV")) push_div = (uint32_t)std::max(0, atoi(e));
  uint32_t nb_cap = 96;
  if (const char* e = getenv("OSPF_MS_NB")) nb_cap = std::max(1, atoi(e));
  nb_cap = (uint32_t)std::max<size_t>(1, std::min<size_t>(nb_cap, (6ull << 30) / per_vb));
  // roots per chunk: bounded when digest rows live in scratch
  const size_t row_bytes = (dist_scr ? V * 4ull : 0) + (nh_scr ? (size_t)V * W * 4ull : 0);
  uint32_t chunk = b->n_roots;
  if (row_bytes)
    chunk = (uint32_t)std::max<size_t>(64, std::min<size_t>(chunk, (2ull << 30) / row_bytes) / 64 * 64);
  // wide rows: the rows kernels stage each pass's words word-major
  // ([root][W][V], whole-line stores) and one interleave pass writes the
  // [V][W] rows; the passes' scattered word stores otherwise write a 4-B word
  // per W-word row entry. Measured on F100k: W = 56 class 4.55 -> 3.98 ms;
  // W = 3 slower (11.1 -> 12.2 ms: the rows kernel there is not store-bound and
  // the extra pass costs 1.3 ms), hence the threshold. OSPF_MS_ILV=0/1 forces.
  bool ilv = defer && W >= 8 && W <= 64 && (flags & OSPF_WANT_NH) && !nh_scr;
  if (const char* e = getenv("OSPF_MS_ILV"))
    ilv = atoi(e) && defer && W > 1 && W <= 64 && (flags & OSPF_WANT_NH) && !nh_scr;
  if (ilv) {
    const size_t cap = 8ull << 30, per_root = (size_t)V * W * 4ull;
    if ((size_t)chunk * per_root > cap)
      chunk = (uint32_t)std::max<size_t>(64, cap / per_root / 64 * 64);
  }
  // merged rows (2..7 words, one per pass): every pass of a batch in the same
  // round, all of a batch's passes on one XCD (nb a multiple of 8 * npass)
  bool merged = defer && !ilv && npass > 1 && sh.PP == 1 && sh.OW == 1 && W <= 7 &&
                (flags & (OSPF_WANT_NH | OSPF_WANT_DIGEST)) && !getenv("OSPF_MS_NOMERGE");
  uint32_t nb_max =
      std::min<uint32_t>(nb_cap, ((std::min(chunk, b->n_roots) + sh.R - 1) / sh.R) * npass);
  if (merged) {
    const uint32_t unit = nb_max >= 8 * npass ? 8 * npass : npass;
    nb_max = std::max(unit, nb_max / unit * unit);
    merged = nb_max <= nb_cap || nb_max == npass;
  }
  const size_t state_bytes = per_vb * nb_max;
  const size_t dist_bytes = dist_scr ? align_up((size_t)chunk * V * 4ull, 256) : 0;
  const size_t nh_bytes = (nh_scr || ilv) ? align_up((size_t)chunk * V * W * 4ull, 256) : 0;
  int rc = OSPF_OK;
  char* sp = stream_scratch(c, s, state_bytes + dist_bytes + nh_bytes, &rc);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  for (uint32_t r0 = 0; r0 < b->n_roots; r0 += chunk) {
    const uint32_t n = std::min(chunk, b->n_roots - r0);
    ospf::MsArgs a{};
    a.roots = b->d_roots + r0;
    a.n = n;
    a.W = W;
    a.npass = npass;
    a.R = sh.R;
    a.PP = sh.PP;
    a.OW = sh.OW;
    a.rep = rep;
    a.lmax = lmax;
    a.dbound = c->depth_bound;
    a.kcap = kcap;
    a.push_div = push_div;
    a.defer = defer ? 1u : 0u;
    a.merged = merged ? 1u : 0u;
    a.digest = (defer && dig) ? b->d_digest + r0 : nullptr;
    if (a.digest) HIPCHK(c, ospf::zero_async(a.digest, (size_t)n * sizeof(ospf_digest), s));
    a.err = c->d_err;
    a.dist = dist_scr ? (uint32_t*)(sp + state_bytes)
                      : ((flags & OSPF_WANT_DIST) ? b->d_dist + (size_t)r0 * V : nullptr);
    a.nh = nh_scr ? (uint32_t*)(sp + state_bytes + dist_bytes)
                  : ((flags & OSPF_WANT_NH) ? b->d_nh + (size_t)r0 * V * W : nullptr);
    a.nhs = ilv ? (uint32_t*)(sp + state_bytes + dist_bytes) : nullptr;
    const uint32_t total_vb = ((n + sh.R - 1) / sh.R) * npass;
    for (uint32_t vb0 = 0; vb0 < total_vb; vb0 += nb_max) {
      a.vb0 = vb0;
      a.nb = std::min(nb_max, total_vb - vb0);

      a.front = (uint64_t*)sp;  // 16-B records: first, for alignment
      a.seen = a.front + 4ull * a.nb * V;
      a.accb = a.seen + (size_t)a.nb * V;
      a.planes = a.accb + (size_t)a.nb * V;
      a.lev = (uint8_t*)(a.planes + (size_t)a.nb * V * kp);  // 16-B aligned (uint4 access)
      a.found = (uint32_t*)(a.lev + (defer ? (size_t)a.nb * V * 64ull : 0));
      a.mass = a.found + (size_t)a.nb * lmax;
      HIPCHK(c, ospf::zero_async(sp, (size_t)a.nb * V * 8ull * (6 + kp) +
                                          (defer ? (size_t)a.nb * V * 64ull : 0) +
                                          (size_t)a.nb * lmax * 8ull, s));
      hipError_t e = ospf::launch_msbfs_round(kp, c->g, a, c->depth_bound, s);
      if (e != hipSuccess) return hip_fail(c, e, "launch_msbfs_round");
    }
    if (ilv) {
      hipError_t e = ospf::launch_nh_interleave(a.nhs, a.nh, n, V, W,
                                                std::min(W, npass * sh.OW), s);
      if (e != hipSuccess) return hip_fail(c, e, "launch_nh_interleave");
    }
    if (dig && !defer) {
      hipError_t e = ospf::launch_row_digest(c->g, n, a.dist, a.nh, W, b->d_digest + r0, s);
      if (e != hipSuccess) return hip_fail(c, e, "launch_row_digest");
    }
  }
  c->spf_runs += b->n_roots;
  return OSPF_OK;
}


// Variant 7: group-per-root bucketed Dial (spf_wdial.hip). Persistent
// workgroups of G waves (OSPF_WD_GROUP, default from the graph: see below),
// 16 / G of them per CU, each own a ring of frontier lists; the ring covers
// every tentative distance ahead of the current one: NB = max metric + 1
// lists of one distance each, or, past kWDialMaxNB, buckets of delta
// distances with tagged entries. List capacity comes from a memory budget
// (OSPF_WD_LIST_MB, default 4096); an overflowing list falls back to node
// scans for its rounds (correct, slower).
int run_wdial(ospf_ctx* c, const ospf_batch* b, bool hop, hipStream_t s) {
  const uint32_t V = c->info.n_nodes, W = b->nh_words, n = b->n_roots;
  const uint32_t maxw = hop ? 1u : std::max<uint32_t>(c->info.max_metric, 1);
  uint32_t NB, delta;
  if (maxw + 1 <= ospf::kWDialMaxNB) {
    NB = maxw + 1;
    delta = 1;
  } else {
    NB = ospf::kWDialMaxNB;
    delta = (maxw + NB - 2) / (NB - 1);
  }
  if (const char* e = getenv("OSPF_WD_DELTA")) {  // test knob: force tagged buckets
    const uint32_t dl = (uint32_t)std::max(1, atoi(e));
    if (dl > 1) {
      delta = std::max(delta, dl);
      NB = std::min<uint32_t>(ospf::kWDialMaxNB, (maxw + delta - 1) / delta + 1);
      NB = std::max<uint32_t>(NB, 2);
    }
  }
  // Waves per root: a round's work is about E / (distinct distances); graphs
  // with many edges per distance value (low hop diameter, e.g. fabrics) get a
  // whole CU per root, thin-frontier graphs (meshes) a wave per root.
  const double rounds = (double)maxw * std::max<uint32_t>(2, c->depth_bound);
  const double per_round = (double)c->info.n_edges / std::max(1.0, rounds);
  uint32_t G = per_round > 2048 ? 8 : per_round > 128 ? 2 : 1;
  // fewer roots than groups: wider groups (more lanes per round) until every
  // group has a root
  while (G < 16 && n < (uint64_t)c->n_cu * (16 / G)) G *= 2;
  if (const char* e = getenv("OSPF_WD_GROUP")) G = (uint32_t)std::max(1, std::min(16, atoi(e)));
  while (16 % G) --G;
  uint32_t ngroups =
      std::max<uint32_t>(1, std::min<uint32_t>(n, (uint32_t)c->n_cu * (16 / G)));
  // knob: fewer roots in flight (their frontiers' state lines stay cached)
  if (const char* e = getenv("OSPF_WD_NGROUPS"))
    ngroups = std::max<uint32_t>(1, std::min<uint32_t>(ngroups, (uint32_t)atoi(e)));
  size_t budget = 4096ull << 20;
  if (const char* e = getenv("OSPF_WD_LIST_MB")) budget = (size_t)std::max(1, atoi(e)) << 20;
  const size_t eb = delta > 1 ? 8 : 4;
  uint64_t bcap = budget / ((uint64_t)ngroups * NB * eb);
  bcap = std::max<uint64_t>(64, std::min<uint64_t>(bcap, V));
  if (const char* e = getenv("OSPF_WD_BCAP")) bcap = (uint64_t)std::max(1, atoi(e));  // test knob
  // packed state (spf_wdial.hip PACK): one word per node for roots with at
  // most 16 distinct neighbours (the caller's max_root_neighbors hint)
  const uint32_t kcap = b->max_root_neighbors ? b->max_root_neighbors : 32u * W;
  uint32_t pk_bits = (W == 1 && kcap <= 16) ? (kcap <= 8 ? 8u : 16u) : 0u;
  if (const char* e = getenv("OSPF_WD_PACK")) {  // knob: 0 = off, 8 / 16 = field width
    const int v = atoi(e);
    pk_bits = (v == 0 || W != 1 || kcap > (uint32_t)v || (v != 8 && v != 16)) ? 0u : (uint32_t)v;
  }
  const bool want_dist = b->flags & OSPF_WANT_DIST, want_nh = b->flags & OSPF_WANT_NH;
  const size_t sz_lists = align_up((size_t)ngroups * NB * bcap * eb, 256);
  const size_t sz_dist = want_dist ? 0 : align_up((size_t)n * V * 4ull, 256);
  const size_t sz_nh = want_nh ? 0 : align_up((size_t)n * V * W * 4ull, 256);
  const size_t sz_pk = pk_bits ? align_up((size_t)ngroups * V * 4ull, 256) : 0;
  int rc = OSPF_OK;
  char* sp = stream_scratch(c, s, sz_lists + sz_dist + sz_nh + sz_pk, &rc);
  if (rc) return rc;
  ospf::WDialArgs a{};
  a.roots = b->d_roots;
  a.n = n;
  a.ign_off = b->d_ign_offsets;
  a.ign_ids = b->d_ign_ids;
  a.hop = hop ? 1u : 0u;
  a.W = W;
  a.lists = (uint32_t*)sp;
  a.dist = want_dist ? b->d_dist : (uint32_t*)(sp + sz_lists);
  a.nh = want_nh ? b->d_nh : (uint32_t*)(sp + sz_lists + sz_dist);
  a.digest = (b->flags & OSPF_WANT_DIGEST) ? b->d_digest : nullptr;
  a.err = c->d_err;
  a.NB = NB;
  a.bcap = (uint32_t)bcap;
  a.delta = delta;
  a.group_waves = G;
  a.ngroups = ngroups;
  a.pk_bits = pk_bits;
  a.pk = pk_bits ? (uint32_t*)(sp + sz_lists + sz_dist + sz_nh) : nullptr;
  a.wg_scope = getenv("OSPF_WD_WGSCOPE") ? 1u : 0u;
  HIPCHK(c, hipSetDevice(c->device));
  hipError_t e = ospf::launch_wdial(c->g, a, s);
  if (e != hipSuccess) return hip_fail(c, e, "launch_wdial");
  c->spf_runs += n;
  return OSPF_OK;
}

// ---------------------------------------------------------------- KSP2
// getKthPaths(src, dst, 1 and 2) for many destinations (LinkState.cpp:790-819):
//  1. the link-metric SPF of src (one run, any variant) -> dist row;
//  2. trace k = 1 per destination over that row -> records + sorted link sets;
//  3. the masked reruns (run i ignores destination i's k = 1 links) and the
//     k = 2 trace over each. Unit-metric graphs run the reruns as the
//     multi-source BFS in distance-only mode (64 runs per traversal, per-run
//     ignore masks) and trace straight from its level bytes; other graphs run
//     per-run kernels into dist rows, in chunks.
int run_ksp2(ospf_ctx* c, const ospf_ksp2* k, hipStream_t s) {
  const uint32_t V = c->info.n_nodes, n = k->n, cap = k->path_cap;
  const uint32_t src = k->src;
  const bool unit = c->info.unit_metric != 0;
  const uint32_t nn = c->h_dn_off[src + 1] - c->h_dn_off[src];
  const uint32_t W = std::max<uint32_t>(1, (nn + 31) / 32);
  const bool ms = unit && c->g.n_lid && c->depth_bound <= 253 && !getenv("OSPF_KSP_ROWS");
  constexpr uint32_t lmax = 256;
  const uint32_t dw = (V + 31) / 32;
  const size_t sz_ign = align_up((size_t)n * cap * 4ull, 256), sz_cnt = align_up(n * 4ull, 256),
               sz_one = align_up(V * 4ull, 256) + 256;
  // multi-source reruns: shared traversal state + igm, and a ring of `slots`
  // (lev bytes, dead bitmaps) so round r's trace (engine stream) overlaps
  // the reruns of rounds r+1 .. r+slots-1
  const size_t igw = ((size_t)c->g.E + 31) / 32;
  const size_t st_zero = (size_t)V * 8ull * 6 + lmax * 8ull + igw * 4ull;
  const size_t per_vb = align_up(st_zero, 256) + align_up((size_t)c->g.E * 8ull, 256);
  const size_t per_vb_slot = (size_t)V * 64ull + 64ull * dw * 4ull;
  uint32_t nb_cap = 96;
  if (const char* e = getenv("OSPF_MS_NB")) nb_cap = std::max(1, atoi(e));
  nb_cap = (uint32_t)std::max<size_t>(1, std::min<size_t>(nb_cap, (6ull << 30) / (per_vb + per_vb_slot)));
  const uint32_t total_vb = (n + 63) / 64, nb_max = std::min(nb_cap, total_vb);
  const uint32_t rounds = (total_vb + nb_max - 1) / nb_max;
  uint32_t slots = (uint32_t)std::max<size_t>(
      1, std::min<size_t>({(size_t)16, (size_t)rounds, (12ull << 30) / (per_vb_slot * nb_max)}));
  if (const char* e = getenv("OSPF_KSP_SLOTS")) slots = std::max(1, std::min((int)slots, atoi(e)));
  const size_t sz_lev = align_up((size_t)nb_max * V * 64ull, 256),
               sz_sdead = align_up((size_t)nb_max * 64ull * dw * 4ull, 256) +
                          align_up((nb_max * 64ull + 2) * 4ull, 256);
  // per-run rows path (and k = 1 traces): dead bitmaps per trace launch
  uint32_t chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(n, (2ull << 30) / (V * 4ull)));
  uint32_t tchunk = (uint32_t)std::max<size_t>(64, std::min<size_t>(n, (1ull << 30) / (dw * 4ull)));
  chunk = std::min(chunk, tchunk);
  const size_t sz_dead = align_up((size_t)tchunk * dw * 4ull, 256) + align_up((tchunk + 2) * 4ull, 256);
  const size_t sz_roots = align_up((size_t)(ms ? n : chunk) * 4ull, 256);
  const size_t sz_state = ms ? per_vb * nb_max + slots * (sz_lev + sz_sdead)
                             : align_up((size_t)chunk * V * 4ull, 256) + align_up((chunk + 1) * 4ull, 256);
  int rc = OSPF_OK;
  char* sp = stream_scratch(c, s, sz_ign + sz_cnt + sz_one + sz_roots + sz_dead + sz_state, &rc, 1);
  if (rc) return rc;
  uint32_t* d_ign = (uint32_t*)sp;
  uint32_t* d_cnt = (uint32_t*)(sp + sz_ign);
  uint32_t* d_dist1 = (uint32_t*)(sp + sz_ign + sz_cnt);
  uint32_t* d_src = (uint32_t*)(sp + sz_ign + sz_cnt + align_up(V * 4ull, 256));
  uint32_t* d_roots = (uint32_t*)(sp + sz_ign + sz_cnt + sz_one);
  uint32_t* d_dead = (uint32_t*)(sp + sz_ign + sz_cnt + sz_one + sz_roots);
  char* st = sp + sz_ign + sz_cnt + sz_one + sz_roots + sz_dead;
  HIPCHK(c, hipSetDevice(c->device));

  // 1-2: SPF of src (the multi-source BFS for one root beats a one-workgroup
  // BFS on a large graph), k = 1 traces
  HIPCHK(c, hipMemsetD32Async(d_src, (int)src, 1, s));
  ospf_batch b1{};
  b1.d_roots = d_src;
  b1.n_roots = 1;
  b1.flags = OSPF_WANT_DIST;
  b1.nh_words = W;
  b1.max_root_neighbors = nn;
  b1.d_dist = d_dist1;
  rc = (unit && c->depth_bound <= 253 && V >= 4096) ? run_msbfs(c, &b1, s)
                                                     : ospf_run_batch_dev(c, &b1, s);
  if (rc) return rc;
  ospf::TraceArgs t{};
  t.src = src;
  t.dsts = k->dsts;
  t.n = n;
  t.rows = d_dist1;
  t.row_stride = 0;
  t.stride = cap;
  t.out = k->k1;
  t.ign_out = d_ign;
  t.cnt_out = d_cnt;
  t.status = k->status;
  t.k = 1;
  t.unit = unit ? 1u : 0u;
  t.dead = d_dead;
  t.dead_words = dw;
  // unit metric: runs past kTraceBudget DFS steps finish on the 16-wave kernel
  constexpr uint32_t kTraceBudget = 256;
  t.budget = unit && !getenv("OSPF_KSP_NOHEAVY") ? kTraceBudget : 0u;
  if (const char* x = getenv("OSPF_KSP_BUDGET"))  // test knob: send runs to the heavy kernel
    if (t.budget) t.budget = (uint32_t)std::max(1, atoi(x));
  t.look = 16;  // (OSPF_KSP_LOOK: A/B knob, 0 = no lookahead)
  if (const char* x = getenv("OSPF_KSP_LOOK")) t.look = (uint32_t)std::max(0, atoi(x));
  t.heavy = (uint32_t*)((char*)d_dead + align_up((size_t)tchunk * dw * 4ull, 256));
  t.heavy_ctr = t.heavy + tchunk;
  hipError_t e = hipSuccess;
  for (uint32_t c0 = 0; c0 < n; c0 += tchunk) {
    ospf::TraceArgs tc = t;
    tc.n = std::min(tchunk, n - c0);
    tc.dsts = k->dsts + c0;
    tc.out = k->k1 + (size_t)c0 * cap;
    tc.ign_out = d_ign + (size_t)c0 * cap;
    tc.cnt_out = d_cnt + c0;
    tc.status = k->status + c0;
    HIPCHK(c, ospf::zero_async(d_dead, (size_t)tc.n * dw * 4ull, s));
    HIPCHK(c, ospf::zero_async(t.heavy_ctr, 8, s));
    e = ospf::launch_ksp_trace(false, c->g, tc, s);
    if (e != hipSuccess) return hip_fail(c, e, "launch_ksp_trace k1");
  }
  const ospf::TraceArgs t_k1 = t;

  // 3: masked reruns + k = 2 over a set of runs (all of them, or the ones the
  // decremental kernel left): the multi-source BFS with per-run ignore masks
  // (unit metric) or per-run rows
  // the stream of the full reruns: the caller's, or a high-priority one
  // while the decremental kernels run beside them (run_ksp2's presplit)
  hipStream_t fs = s;
  // after_first: called once the first round's traversal is done on fs (the
  // host waits for it anyway): the presplit runs' first round gets the GPU
  // alone, the decremental kernels are launched beside the later rounds
  // before_last(R_n): called once before the last round is queued; it may
  // append runs to the R_* arrays (their capacity) and raise R_n
  auto full_reruns = [&](const uint32_t* R_dsts, uint32_t R_n, const uint32_t* R_ign,
                         const uint32_t* R_cnt, uint32_t* R_status, uint32_t* R_k2,
                         const std::function<int()>& after_first = nullptr,
                         const std::function<int(uint32_t&)>& before_last = nullptr) -> int {
    ospf::TraceArgs t = t_k1;
    uint32_t total_vb = (R_n + 63) / 64;  // this set's virtual batches (<= the carve'fs)
    HIPCHK(c, hipMemsetD32Async(d_roots, (int)src, ms ? (before_last ? n : R_n) : chunk, fs));
    if (ms) {
      if (!c->aux) HIPCHK(c, hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
      while (c->ev.size() < 2 * (size_t)slots + 1) {
        hipEvent_t x;
        HIPCHK(c, hipEventCreateWithFlags(&x, hipEventDisableTiming));
        c->ev.push_back(x);
      }
      hipEvent_t* ev_bfs = c->ev.data();
      hipEvent_t* ev_tr = c->ev.data() + slots;
      hipEvent_t ev_end = c->ev[2 * slots];
      char* ring = st + per_vb * nb_max;
      std::vector<uint32_t> found;
      bool last_called = false;
      for (uint32_t r = 0, vb0 = 0; vb0 < total_vb; ++r, vb0 += nb_max) {
        if (before_last && !last_called && vb0 + nb_max >= total_vb) {
          last_called = true;
          const int rc3 = before_last(R_n);
          if (rc3) return rc3;
          total_vb = (R_n + 63) / 64;
        }
        const uint32_t slot = r % slots;
        uint8_t* lev = (uint8_t*)(ring + (size_t)slot * (sz_lev + sz_sdead));
        uint32_t* dead = (uint32_t*)(ring + (size_t)slot * (sz_lev + sz_sdead) + sz_lev);
        ospf::MsArgs a{};
        a.roots = d_roots;
        a.n = R_n;
        a.W = W;
        a.npass = 1;
        a.R = 64;
        a.PP = 1;
        a.OW = 1;
        a.rep = 1;
        a.vb0 = vb0;
        a.nb = std::min(nb_max, total_vb - vb0);
        a.lmax = lmax;
        a.kcap = nn;
        a.push_div = 8;
        if (const char* x = getenv("OSPF_MS_PUSH_DIV")) a.push_div = (uint32_t)std::max(0, atoi(x));
        a.defer = 1;
        a.err = c->d_err;
        a.front = (uint64_t*)st;
        a.seen = a.front + 4ull * a.nb * V;
        a.accb = a.seen + (size_t)a.nb * V;
        a.planes = a.accb + (size_t)a.nb * V;
        a.found = (uint32_t*)a.planes;
        a.mass = a.found + (size_t)a.nb * lmax;
        a.igw = (uint32_t)igw;
        a.igb = a.mass + (size_t)a.nb * lmax;
        const size_t zero = (char*)(a.igb + (size_t)a.nb * igw) - st;
        a.igm = (uint64_t*)(st + align_up(zero, 256));
        a.lev = lev;
        // a batch stops once all its destinations are reached
        // (OSPF_KSP_FULL_DEPTH: every level, as before)
        a.kdst = getenv("OSPF_KSP_FULL_DEPTH") ? nullptr : R_dsts;
        HIPCHK(c, ospf::zero_async(st, zero, fs));
        if (r >= slots) HIPCHK(c, hipStreamWaitEvent(fs, ev_tr[slot], 0));  // slot's trace done
        HIPCHK(c, ospf::zero_async(lev, (size_t)a.nb * V * 64ull, fs));
        e = ospf::launch_ksp_masks(c->g, a, R_ign, R_cnt, cap, fs);
        if (e != hipSuccess) return hip_fail(c, e, "launch_ksp_masks");
        uint32_t d = std::max<uint32_t>(2, c->depth_bound);
        // test knob: start with fewer levels (exercises the continuation below)
        if (const char* x = getenv("OSPF_KSP_D0")) d = std::max(2, std::min((int)d, atoi(x)));
        e = ospf::launch_msbfs_ksp(c->g, a, 1, d, fs);
        if (e != hipSuccess) return hip_fail(c, e, "launch_msbfs_ksp");
        // masked runs may be deeper than the graph's bound: continue while any
        // batch still has a frontier (levels up to 253: lev bytes hold dist + 1)
        std::vector<uint32_t> deep;
        for (;;) {
          found.resize((size_t)a.nb * lmax);
          HIPCHK(c, hipMemcpyAsync(found.data(), a.found, found.size() * 4ull, hipMemcpyDeviceToHost, fs));
          HIPCHK(c, hipStreamSynchronize(fs));
          deep.clear();
          for (uint32_t j = 0; j < a.nb; ++j)
            if (found[(size_t)j * lmax + d]) deep.push_back(j);
          if (deep.empty()) break;
          if (d >= 254) {  // these runs keep OVF2: their levels stop at 254
            for (uint32_t j : deep) {
              const uint32_t r0 = (vb0 + j) * 64u;
              e = ospf::launch_or_bits(R_status + r0, std::min(64u, R_n - r0), OSPF_KSP_OVF2, fs);
              if (e != hipSuccess) return hip_fail(c, e, "launch_or_bits");
            }
            break;
          }
          const uint32_t d1 = std::min<uint32_t>(d + 8, 254);
          e = ospf::launch_msbfs_ksp(c->g, a, d, d1, fs);
          if (e != hipSuccess) return hip_fail(c, e, "launch_msbfs_ksp");
          d = d1;
        }
        HIPCHK(c, hipEventRecord(ev_bfs[slot], fs));
        HIPCHK(c, hipStreamWaitEvent(c->aux, ev_bfs[slot], 0));
        if (r == 0 && after_first) {
          const int rc3 = after_first();
          if (rc3) return rc3;
        }
        const uint32_t r0 = vb0 * 64u;
        ospf::TraceArgs t2 = t;
        t2.dsts = R_dsts + r0;
        t2.n = std::min<uint32_t>(a.nb * 64u, R_n - r0);
        t2.rows = nullptr;
        t2.lev = lev;
        t2.ign = R_ign + (size_t)r0 * cap;
        t2.ign_cnt = R_cnt + r0;
        t2.out = R_k2 + (size_t)r0 * cap;
        t2.ign_out = nullptr;
        t2.cnt_out = nullptr;
        t2.status = R_status + r0;
        t2.k = 2;
        t2.dead = dead;
        t2.heavy = (uint32_t*)((char*)dead + align_up((size_t)nb_max * 64ull * dw * 4ull, 256));
        t2.heavy_ctr = t2.heavy + nb_max * 64u;
        HIPCHK(c, ospf::zero_async(dead, (size_t)t2.n * dw * 4ull, c->aux));
        HIPCHK(c, ospf::zero_async(t2.heavy_ctr, 8, c->aux));
        e = ospf::launch_ksp_trace(true, c->g, t2, c->aux);
        if (e != hipSuccess) return hip_fail(c, e, "launch_ksp_trace k2");
        HIPCHK(c, hipEventRecord(ev_tr[slot], c->aux));
      }
      HIPCHK(c, hipEventRecord(ev_end, c->aux));
      HIPCHK(c, hipStreamWaitEvent(fs, ev_end, 0));
      c->spf_runs += R_n;
    } else {
      uint32_t* d_rows = (uint32_t*)st;
      uint32_t* d_off = (uint32_t*)(st + align_up((size_t)chunk * V * 4ull, 256));
      e = ospf::launch_iota(d_off, chunk, cap, fs);
      if (e != hipSuccess) return hip_fail(c, e, "launch_iota");
      for (uint32_t r0 = 0; r0 < R_n; r0 += chunk) {
        const uint32_t nc = std::min(chunk, R_n - r0);
        ospf_batch b{};
        b.d_roots = d_roots;
        b.n_roots = nc;
        b.d_ign_offsets = d_off;
        b.d_ign_ids = R_ign + (size_t)r0 * cap;
        b.max_ignored = cap;
        b.flags = OSPF_WANT_DIST;
        b.nh_words = W;
        b.max_root_neighbors = nn;
        b.d_dist = d_rows;
        rc = ospf_run_batch_dev(c, &b, fs);
        if (rc) return rc;
        ospf::TraceArgs t2 = t;
        t2.dsts = R_dsts + r0;
        t2.n = nc;
        t2.rows = d_rows;
        t2.row_stride = V;
        t2.ign = R_ign + (size_t)r0 * cap;
        t2.ign_cnt = R_cnt + r0;
        t2.out = R_k2 + (size_t)r0 * cap;
        t2.ign_out = nullptr;
        t2.cnt_out = nullptr;
        t2.status = R_status + r0;
        t2.k = 2;
        HIPCHK(c, ospf::zero_async(d_dead, (size_t)t2.n * dw * 4ull, fs));
        HIPCHK(c, ospf::zero_async(t2.heavy_ctr, 8, fs));
        e = ospf::launch_ksp_trace(false, c->g, t2, fs);
        if (e != hipSuccess) return hip_fail(c, e, "launch_ksp_trace k2");
      }
    }
    return OSPF_OK;
  };
  if (getenv("OSPF_KSP_NODECR")) return full_reruns(k->dsts, n, d_ign, d_cnt, k->status, k->k2);
  // decremental reruns (spf_ksp2.hip): the source's row + per-run lost
  // supports. Runs whose ignore list is past its budget are known before it
  // starts (presplit): their full reruns go on `s` while the decremental
  // kernels run on ksp_aux; the runs it gives up on follow them, compacted.
  {
    const size_t dwb = align_up((size_t)dw * 4ull, 256);
    uint32_t bpc = ospf::ksp_decr_blocks_per_cu();
    if (const char* x = getenv("OSPF_KSP_DECR_BPC")) bpc = std::max(1u, std::min(bpc, (uint32_t)atoi(x)));
    // (OSPF_KSP_DECR_R: runs per block instead of persistent blocks)
    uint32_t decr_r = 0;
    if (const char* x = getenv("OSPF_KSP_DECR_R")) decr_r = (uint32_t)std::max(0, atoi(x));
    const uint32_t nblk = decr_r ? std::max(1u, (n + decr_r - 1) / decr_r)
                                 : std::max<uint32_t>(1, bpc * (uint32_t)c->n_cu);
    const uint32_t hblk = 2u * (uint32_t)c->n_cu;  // ksp_decr_heavy_kernel: 2 per CU
    const size_t sz_tc = align_up(V * 4ull, 256), sz_fb = align_up(n * 4ull, 256), sz_ctr = 256,
                 sz_dd = dwb * std::max(nblk, hblk);
    // heavy runs' pruning (unit metric): level order + per-block good bits
    const bool prune = t_k1.budget && !getenv("OSPF_KSP_NOPRUNE");
    const size_t sz_ord = prune ? align_up(V * 4ull, 256) + align_up(2 * 257 * 4ull, 256) : 0,
                 sz_good = prune ? dwb * hblk + (size_t)hblk * ospf::kGoodBig * 4ull : 0;
    const size_t sz_pb = align_up((n + 31) / 32 * 4ull, 256);
    char* dp = stream_scratch(c, s, sz_tc + 3 * sz_fb + sz_ctr + sz_dd + sz_ord + sz_good + sz_pb, &rc, 2);
    if (rc) return rc;
    uint32_t* d_tc = (uint32_t*)dp;
    uint32_t* d_fb = (uint32_t*)(dp + sz_tc);
    uint32_t* d_hq = (uint32_t*)(dp + sz_tc + sz_fb);
    uint32_t* d_pre = (uint32_t*)(dp + sz_tc + 2 * sz_fb);
    uint32_t* d_ctr = (uint32_t*)(dp + sz_tc + 3 * sz_fb);
    uint32_t* d_dd = (uint32_t*)(dp + sz_tc + 3 * sz_fb + sz_ctr);
    HIPCHK(c, ospf::zero_async(d_ctr, 128, s));
    e = ospf::launch_ksp_hint(c->g, src, d_dist1, d_tc, s);
    if (e != hipSuccess) return hip_fail(c, e, "launch_ksp_hint");
    ospf::TraceArgs td = t_k1;
    td.rows = d_dist1;
    td.row_stride = 0;
    td.lev = nullptr;
    td.ign = d_ign;
    td.ign_cnt = d_cnt;
    td.out = k->k2;
    td.ign_out = nullptr;
    td.cnt_out = nullptr;
    td.status = k->status;
    td.k = 2;
    td.dead = d_dd;
    td.dead_words = (uint32_t)(dwb / 4);
    td.tc = d_tc;
    td.fb = d_fb;
    td.ctr = d_ctr;
    td.heavy = d_hq;
    td.heavy_ctr = d_ctr + 4;
    td.err = c->d_err;
    td.decr_runs = decr_r;
    // a run past the map budget goes to the full reruns (with presplit runs
    // it joins their last round) instead of the 16-wave kernel, whose
    // single slow run (F100k: 10.8 ms) had ended the launch: 20.17 -> 20.04
    // ms (profiles/r06/h1_ksp2_order_ab.txt; OSPF_KSP_MAP_FB=0 restores it)
    td.map_fb = 1u;
    if (const char* x = getenv("OSPF_KSP_MAP_FB")) td.map_fb = atoi(x) ? 1u : 0u;
    if (prune) {
      char* q = dp + sz_tc + 3 * sz_fb + sz_ctr + sz_dd;
      uint32_t* d_ord = (uint32_t*)q;
      uint32_t* d_off = (uint32_t*)(q + align_up(V * 4ull, 256));
      e = ospf::launch_ksp_levels(d_dist1, V, d_ord, d_off, d_off + 257, s);
      if (e != hipSuccess) return hip_fail(c, e, "launch_ksp_levels");
      td.ord = d_ord;
      td.lvl_off = d_off;
      td.nlvl = 256;
      td.good = (uint32_t*)(q + sz_ord);
      td.big = (uint32_t*)(q + sz_ord + dwb * hblk);
    }
    // (presplit count in ctr[12])
    uint32_t npre = 0;
    const bool split = getenv("OSPF_KSP_NOSPLIT") == nullptr;
    if (split) {
      td.src_cut = 16;  // (OSPF_KSP_SRCCUT: A/B knob, 0 = off)
      if (const char* x = getenv("OSPF_KSP_SRCCUT")) td.src_cut = (uint32_t)std::max(0, atoi(x));
      td.pre_bits = (uint32_t*)(dp + sz_tc + 3 * sz_fb + sz_ctr + sz_dd + sz_ord + sz_good);
      HIPCHK(c, ospf::zero_async(td.pre_bits, (n + 31) / 32 * 4ull, s));
      e = ospf::launch_ksp_presplit(c->g, td, d_pre, d_ctr + 12, s);
      if (e != hipSuccess) return hip_fail(c, e, "launch_ksp_presplit");
      HIPCHK(c, hipMemcpyAsync(&npre, d_ctr + 12, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(c, hipStreamSynchronize(s));
    }
    hipStream_t ks = s;
    // with presplit runs: the decremental kernels on a low-priority stream,
    // the full reruns (the launch's critical path) on a high-priority one
    // (OSPF_KSP_NOPRIO: the caller's stream for them)
    const bool prio = getenv("OSPF_KSP_NOPRIO") == nullptr;
    if (npre) {
      if (!c->ksp_aux || !c->ksp_hi) {
        int lo = 0, hi = 0;
        HIPCHK(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
        if (!c->ksp_aux) HIPCHK(c, hipStreamCreateWithPriority(&c->ksp_aux, hipStreamNonBlocking, lo));
        if (!c->ksp_hi) HIPCHK(c, hipStreamCreateWithPriority(&c->ksp_hi, hipStreamNonBlocking, hi));
      }
      for (hipEvent_t& x : c->ksp_ev)
        if (!x) HIPCHK(c, hipEventCreateWithFlags(&x, hipEventDisableTiming));
      HIPCHK(c, hipEventRecord(c->ksp_ev[0], s));
      HIPCHK(c, hipStreamWaitEvent(c->ksp_aux, c->ksp_ev[0], 0));
      ks = c->ksp_aux;
      if (prio) {
        HIPCHK(c, hipStreamWaitEvent(c->ksp_hi, c->ksp_ev[0], 0));
        fs = c->ksp_hi;
      }
    }
    // OSPF_KSP_DEBUG=2: a log of the heavy runs (run, start, traced, end)
    unsigned long long* d_hlog = nullptr;
    const char* kdbg = getenv("OSPF_KSP_DEBUG");
    if (kdbg && atoi(kdbg) >= 2 && td.budget) {
      HIPCHK(c, dev_malloc(c, (void**)&d_hlog, 4ull * 65536 * 8));
      td.hlog = d_hlog;
    }
    // the decremental kernels: queued before the presplit runs, beside them
    // (OSPF_KSP_DECR_AFTER=1: after their first traversal round -- measured
    // slower, 22.9 vs 20.4 ms per F100k launch: the presplit chain is not
    // the longer one once it shares the chip)
    bool decr_queued = false;
    auto launch_decr = [&]() -> int {
      if (decr_queued) return OSPF_OK;
      decr_queued = true;
      if (ks != s) {  // (the first round's traversal done: ordered on fs)
        HIPCHK(c, hipEventRecord(c->ksp_ev[0], fs));
        HIPCHK(c, hipStreamWaitEvent(ks, c->ksp_ev[0], 0));
      }
      hipError_t e3 = ospf::launch_ksp_decr(c->g, td, nblk, ks);
      if (e3 != hipSuccess) return hip_fail(c, e3, "launch_ksp_decr");
      if (npre) {  // the decremental kernel's fallback count (ctr[13]), then its event
        HIPCHK(c, hipMemcpyAsync(d_ctr + 13, d_ctr + 1, 4, hipMemcpyDeviceToDevice, ks));
        HIPCHK(c, hipEventRecord(c->ksp_ev[3], ks));
      }
      if (td.budget) {
        e3 = ospf::launch_ksp_decr_heavy(c->g, td, hblk, ks);
        if (e3 != hipSuccess) return hip_fail(c, e3, "launch_ksp_decr_heavy");
      }
      return OSPF_OK;
    };
    const bool decr_first = !npre || getenv("OSPF_KSP_DECR_AFTER") == nullptr;
    if (decr_first && (rc = launch_decr())) return rc;
    // a list of runs through full_reruns on s: compacted (dsts, status,
    // ignore sets, counts) into scratch slot `slot`, records scattered back
    // fold: before the last round, runs of a second list (the decremental
    // kernel's fallbacks) join it -- fold(d_list2, n2) returns the list and
    // how many (<= extra); they are gathered behind the first list's and
    // scattered back with it
    const uint32_t* fold_list = nullptr;
    uint32_t folded = 0;
    auto rerun_list = [&](const uint32_t* d_list, uint32_t nl, int slot,
                          const std::function<int()>& after_first = nullptr, uint32_t extra = 0,
                          const std::function<int(const uint32_t**, uint32_t*)>& fold = nullptr) -> int {
      const uint32_t cap_n = nl + extra;
      const size_t sz_fd = align_up(cap_n * 4ull, 256), sz_fr = align_up((size_t)cap_n * cap * 4ull, 256);
      int rc2 = OSPF_OK;
      char* fp = stream_scratch(c, s, 3 * sz_fd + 2 * sz_fr, &rc2, slot);
      if (rc2) return rc2;
      uint32_t* f_dsts = (uint32_t*)fp;
      uint32_t* f_status = (uint32_t*)(fp + sz_fd);
      uint32_t* f_cnt = (uint32_t*)(fp + 2 * sz_fd);
      uint32_t* f_ign = (uint32_t*)(fp + 3 * sz_fd);
      uint32_t* f_k2 = (uint32_t*)(fp + 3 * sz_fd + sz_fr);
      auto gather = [&](uint32_t at, const uint32_t* list, uint32_t m) -> int {
        hipError_t e2;
        if ((e2 = ospf::launch_rows_gather(f_dsts + at, k->dsts, list, m, 1, true, fs)) != hipSuccess ||
            (e2 = ospf::launch_rows_gather(f_status + at, k->status, list, m, 1, true, fs)) != hipSuccess ||
            (e2 = ospf::launch_rows_gather(f_cnt + at, d_cnt, list, m, 1, true, fs)) != hipSuccess ||
            (e2 = ospf::launch_rows_gather(f_ign + (size_t)at * cap, d_ign, list, m, cap, true, fs)) !=
                hipSuccess)
          return hip_fail(c, e2, "launch_rows_gather");
        return OSPF_OK;
      };
      auto scatter = [&](uint32_t at, const uint32_t* list, uint32_t m) -> int {
        hipError_t e2;
        if ((e2 = ospf::launch_rows_gather(k->status, f_status + at, list, m, 1, false, fs)) != hipSuccess ||
            (e2 = ospf::launch_rows_gather(k->k2, f_k2 + (size_t)at * cap, list, m, cap, false, fs)) !=
                hipSuccess)
          return hip_fail(c, e2, "launch_rows_gather");
        return OSPF_OK;
      };
      if ((rc2 = gather(0, d_list, nl))) return rc2;
      const uint32_t* l2 = nullptr;
      uint32_t n2 = 0;
      std::function<int(uint32_t&)> before_last;
      if (fold)
        before_last = [&](uint32_t& Rn) -> int {
          int rc4 = fold(&l2, &n2);
          if (rc4) return rc4;
          n2 = std::min(n2, extra);
          if (n2 && (rc4 = gather(Rn, l2, n2))) return rc4;
          Rn += n2;
          return OSPF_OK;
        };
      rc2 = full_reruns(f_dsts, nl, f_ign, f_cnt, f_status, f_k2, after_first, before_last);
      if (rc2) return rc2;
      if ((rc2 = scatter(0, d_list, nl))) return rc2;
      if (n2 && (rc2 = scatter(nl, l2, n2))) return rc2;
      fold_list = l2;
      folded = n2;
      return OSPF_OK;
    };
    if (npre) {  // beside the decremental kernels
      // OSPF_KSP_PRESORT=1: longest ignore lists (most k = 1 paths) first
      // (measured 21.3 vs 21.1 ms as found: off)
      const char* ps = getenv("OSPF_KSP_PRESORT");
      if (ps && atoi(ps) != 0) {
        std::vector<uint32_t> pre(npre), cnt(n);
        HIPCHK(c, hipMemcpyAsync(pre.data(), d_pre, npre * 4ull, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(cnt.data(), d_cnt, n * 4ull, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        std::stable_sort(pre.begin(), pre.end(), [&](uint32_t a, uint32_t b) {
          return cnt[a] != cnt[b] ? cnt[a] > cnt[b] : a < b;
        });
        HIPCHK(c, hipMemcpyAsync(d_pre, pre.data(), npre * 4ull, hipMemcpyHostToDevice, fs));
        HIPCHK(c, hipStreamSynchronize(fs));
      }
      // the decremental kernel's fallbacks join the last presplit round when
      // that kernel is done by then (OSPF_KSP_NOFOLD: a round of their own
      // after it, as before)
      const bool fold_on = !getenv("OSPF_KSP_NOFOLD");
      auto fold = [&](const uint32_t** l, uint32_t* m) -> int {
        *l = d_fb;
        *m = 0;
        if (!decr_queued || hipEventQuery(c->ksp_ev[3]) != hipSuccess) return OSPF_OK;
        uint32_t cnt = 0;
        HIPCHK(c, hipMemcpy(&cnt, d_ctr + 13, 4, hipMemcpyDeviceToHost));
        *m = cnt;
        return OSPF_OK;
      };
      constexpr uint32_t kFold = 256;  // fallbacks a presplit round takes
      rc = fold_on ? rerun_list(d_pre, npre, 3, launch_decr, kFold, fold)
                   : rerun_list(d_pre, npre, 3, launch_decr);
      if (rc) return rc;
    }
    if ((rc = launch_decr())) return rc;  // (no round called it)
    uint32_t ctr[32] = {};
    HIPCHK(c, hipMemcpyAsync(ctr, d_ctr, 128, hipMemcpyDeviceToHost, ks));
    HIPCHK(c, hipStreamSynchronize(ks));
    if (ks != s) {
      HIPCHK(c, hipEventRecord(c->ksp_ev[1], ks));
      HIPCHK(c, hipStreamWaitEvent(fs, c->ksp_ev[1], 0));
    }
    if (d_hlog) {
      const uint32_t nh = std::min(ctr[11], 65536u);
      std::vector<unsigned long long> hl(4ull * nh);
      HIPCHK(c, hipMemcpy(hl.data(), d_hlog, hl.size() * 8, hipMemcpyDeviceToHost));
      (void)hipFree(d_hlog);
      unsigned long long t0 = ~0ull;
      for (uint32_t q = 0; q < nh; ++q) t0 = std::min(t0, hl[4 * q + 1]);
      std::vector<uint32_t> ord(nh);
      for (uint32_t q = 0; q < nh; ++q) ord[q] = q;
      std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
        return hl[4 * a + 3] - hl[4 * a + 1] > hl[4 * b + 3] - hl[4 * b + 1];
      });
      for (uint32_t x = 0; x < std::min(nh, 12u); ++x) {
        const unsigned long long* l = &hl[4ull * ord[x]];
        fprintf(stderr, "ksp2 heavy run %llu (dst %u): start +%.3f ms, prep %.3f, trace %.3f ms\n", l[0],
                k->dsts ? 0u : 0u, (l[1] - t0) / 1e5, (l[2] - l[1]) / 1e5, (l[3] - l[2]) / 1e5);
      }
    }
    if (getenv("OSPF_KSP_DEBUG")) {
      uint64_t clk[8];
      memcpy(clk, ctr + 16, sizeof(clk));
      // wave-ms: wall-clock ms (100 MHz) summed over the waves / blocks
      auto wm = [](uint64_t x) { return (double)x / 1e5; };
      fprintf(stderr,
              "ksp2 decr: runs %u presplit %u decided %u fallbacks %u (A %u, map %u, ign %u, hash %u, edges %u) "
              "heavy %u affected %u; wave-ms prep %.1f step3 %.1f trace %.1f fb-prep %.1f; heavy "
              "block-ms prep %.1f trace %.1f; longest heavy run %.2f ms (run %u), %llu over 1 ms\n",
              n, npre, ctr[2], ctr[1], ctr[6], ctr[7], ctr[8], ctr[9], ctr[10], ctr[4], ctr[3], wm(clk[0]),
              wm(clk[1]), wm(clk[2]), wm(clk[3]), wm(clk[4]), wm(clk[5]), wm(clk[6] >> 24),
              (uint32_t)(clk[6] & 0xFFFFFFu), (unsigned long long)clk[7]);
    }
    c->ksp_decr_stats[0] += ctr[2];
    c->ksp_decr_stats[1] += ctr[1] + npre;
    c->ksp_decr_stats[2] += ctr[3];
    const uint32_t nfb = ctr[1];
    c->spf_runs += n - nfb - npre;  // (full_reruns counts its own)
    const uint32_t nfold = fold_list == d_fb ? std::min(folded, nfb) : 0u;
    if (nfb > nfold) {  // the fallbacks no presplit round took
      rc = rerun_list(d_fb + nfold, nfb - nfold, 4);
      if (rc) return rc;
    }
    if (fs != s) {  // the caller's stream after the full reruns (and, through them, ks)
      HIPCHK(c, hipEventRecord(c->ksp_ev[2], fs));
      HIPCHK(c, hipStreamWaitEvent(s, c->ksp_ev[2], 0));
    }
  }
  return OSPF_OK;
}

}  // namespace

namespace ospf_int {

int twin_lv_build(ospf_ctx* c, const std::vector<uint32_t>& roots, const std::vector<uint32_t>& groups,
                  const std::vector<uint32_t>& pos, const std::vector<uint32_t>& cls,
                  const std::vector<uint32_t>& rep, TwinLvHost& out) {
  const uint32_t V = c->info.n_nodes, n = (uint32_t)roots.size();
  constexpr uint32_t kNo = 0xFFFFFFFFu;
  out = TwinLvHost{};
  out.grp = groups;
  if (out.grp.empty())
    for (uint32_t i = 0; i <= n; ++i) out.grp.push_back(i);
  if (out.grp.front() != 0 || out.grp.back() != n)
    return fail(c, OSPF_E_INVAL, "twin levels: group offsets must run 0 .. n");
  const uint32_t ng = (uint32_t)out.grp.size() - 1;
  for (uint32_t gi = 0; gi < ng; ++gi) {
    if (out.grp[gi + 1] < out.grp[gi] || out.grp[gi + 1] - out.grp[gi] > ospf::kTwinLvG)
      return fail(c, OSPF_E_RANGE, "twin levels: a group of more than 8 roots");
    out.gmax = std::max(out.gmax, out.grp[gi + 1] - out.grp[gi]);
  }
  // two passes on host threads: each root's neighbour-list length, then per
  // group the lists, class rows and masks at their offsets
  std::atomic<int> bad{0};  // 1 no row, 2 no class row, 3 > 128 neighbours, 4 > 16 class rows
  auto flag = [&](int e) {
    int z = 0;
    bad.compare_exchange_strong(z, e);
  };
  std::vector<uint32_t> nn(n);
  par_for(n, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) {
      const uint32_t r = roots[i];
      if (r >= V || pos[r] == kNo) {
        flag(1);
        nn[i] = 0;
        continue;
      }
      uint32_t m = 0, prev = kNo;
      for (uint32_t e = c->h_prow[r]; e < c->h_prow[r + 1]; ++e) {
        const uint32_t x = c->h_pcolx[e];
        if ((x & 0x80000000u) || x == r || x == prev) continue;  // rows ascend
        prev = x;
        ++m;
      }
      if (m > 128) flag(3);
      nn[i] = m;
    }
  });
  out.nbo.assign(n + 1, 0u);
  for (uint32_t i = 0; i < n; ++i) out.nbo[i + 1] = out.nbo[i] + nn[i];
  out.nbl.resize(out.nbo[n]);
  out.rinfo.resize(n);
  out.grow.assign((size_t)ng * ospf::kTwinMaxC, kNo);
  if (!bad.load())
    par_for(ng, [&](uint32_t glo, uint32_t ghi) {
      std::vector<uint32_t> rows;  // a root's class rows
      for (uint32_t gi = glo; gi < ghi; ++gi) {
        uint32_t* urow = out.grow.data() + (size_t)gi * ospf::kTwinMaxC;
        uint32_t nu = 0;
        for (uint32_t i = out.grp[gi]; i < out.grp[gi + 1]; ++i) {
          const uint32_t r = roots[i];
          rows.clear();
          uint32_t w = out.nbo[i], prev = kNo;
          for (uint32_t e = c->h_prow[r]; e < c->h_prow[r + 1]; ++e) {
            const uint32_t x = c->h_pcolx[e];
            if ((x & 0x80000000u) || x == r) continue;
            if (x != prev) out.nbl[w++] = x;
            prev = x;
            if ((c->h_nt[x >> 5] >> (x & 31)) & 1u) continue;  // overloaded: reaches only itself
            const uint32_t k = cls[x];
            const uint32_t row = k < rep.size() && rep[k] < V ? pos[rep[k]] : kNo;
            if (row == kNo) flag(2);
            rows.push_back(row);
          }
          uint32_t mask = 0;
          for (uint32_t row : rows) {
            uint32_t u = 0;
            while (u < nu && urow[u] != row) ++u;
            if (u == nu) {
              if (u == ospf::kTwinMaxC) {
                flag(4);
                break;
              }
              urow[nu++] = row;
            }
            mask |= 1u << u;
          }
          out.rinfo[i] = make_uint4(r, pos[r], mask, out.nbo[i]);
        }
      }
    }, 64);
  switch (bad.load()) {
    case 1: return fail(c, OSPF_E_RANGE, "twin levels: a root without a row");
    case 2: return fail(c, OSPF_E_RANGE, "twin levels: a class row is missing");
    case 3: return fail(c, OSPF_E_RANGE, "twin levels: more than 128 usable neighbours");
    case 4: return fail(c, OSPF_E_RANGE, "twin levels: more than 16 class rows in a group");
    default: break;
  }
  return OSPF_OK;
}

int twin_lv_launch(ospf_ctx* c, const ospf::TwinLvPlan& p, void* stream) {
  HIPCHK(c, hipSetDevice(c->device));
  const hipError_t e = ospf::launch_twin_levels(c->g, p, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(c, e, "launch_twin_levels");
  c->spf_runs += p.n;
  return OSPF_OK;
}

}  // namespace ospf_int

// Closure split of the contracted graph C (host copy in c->h_cc*): seeds =
// the cover nodes of degree >= tau for the largest of C's few largest
// degrees tau at which every component of C minus the seeds has at most
// kClosureMaxK nodes and the seeds are at most max(64, nS / 8) (F100k: the
// 288 spines; components = the pods' 8 fabric switches). No split: empty.
static void cover_closure_split(ospf_ctx* c) {
  const uint32_t nS = (uint32_t)c->h_ccv.size();
  c->cl_seed.clear();
  c->cl_comp_of.assign(nS, ~0u);
  c->cl_comp_off.assign(1, 0u);
  c->cl_comp_mem.clear();
  if (getenv("OSPF_COVER_NOCLOSURE") || nS < 2) return;
  const auto& crow = c->h_ccrow;
  const auto& ced = c->h_cedge;
  std::vector<uint32_t> deg(nS), dd;
  for (uint32_t i = 0; i < nS; ++i) deg[i] = crow[i + 1] - crow[i];
  dd = deg;
  std::sort(dd.begin(), dd.end(), std::greater<uint32_t>());
  dd.erase(std::unique(dd.begin(), dd.end()), dd.end());
  const uint32_t max_seeds = std::max<uint32_t>(64u, nS / 8u);
  std::vector<uint32_t> par(nS), sz(nS);
  auto find = [&](uint32_t x) {
    while (par[x] != x) x = par[x] = par[par[x]];
    return x;
  };
  for (size_t t = 0; t < std::min<size_t>(dd.size(), 8); ++t) {
    const uint32_t tau = dd[t];
    uint32_t ns = 0;
    for (uint32_t i = 0; i < nS; ++i) ns += deg[i] >= tau;
    if (ns > max_seeds || ns == nS) break;
    for (uint32_t i = 0; i < nS; ++i) {
      par[i] = i;
      sz[i] = 1;
    }
    for (uint32_t i = 0; i < nS; ++i) {
      if (deg[i] >= tau) continue;
      for (uint32_t e = crow[i]; e < crow[i + 1]; ++e) {
        const uint32_t j = ced[e].x;
        if (deg[j] >= tau) continue;
        uint32_t a = find(i), b = find(j);
        if (a == b) continue;
        if (sz[a] < sz[b]) std::swap(a, b);
        par[b] = a;
        sz[a] += sz[b];
      }
    }
    bool fits = true;
    for (uint32_t i = 0; i < nS && fits; ++i)
      if (deg[i] < tau && sz[find(i)] > ospf::kClosureMaxK) fits = false;
    if (getenv("OSPF_SWEEP_DEBUG"))
      fprintf(stderr, "cover split: nS %u tau %u seeds %u fits %d\n", nS, tau, ns, (int)fits);
    if (!fits) continue;
    std::vector<uint32_t> id(nS, ~0u), cnt;
    for (uint32_t i = 0; i < nS; ++i) {
      if (deg[i] >= tau) {
        c->cl_seed.push_back(i);
        continue;
      }
      const uint32_t rt = find(i);
      if (id[rt] == ~0u) {
        id[rt] = (uint32_t)cnt.size();
        cnt.push_back(0);
      }
      c->cl_comp_of[i] = id[rt];
      ++cnt[id[rt]];
    }
    c->cl_comp_off.assign(cnt.size() + 1, 0u);
    for (size_t k = 0; k < cnt.size(); ++k) c->cl_comp_off[k + 1] = c->cl_comp_off[k] + cnt[k];
    c->cl_comp_mem.assign(c->cl_comp_off.back(), 0u);
    std::vector<uint32_t> fill(c->cl_comp_off.begin(), c->cl_comp_off.end() - 1);
    for (uint32_t i = 0; i < nS; ++i)
      if (c->cl_comp_of[i] != ~0u) c->cl_comp_mem[fill[c->cl_comp_of[i]]++] = i;
    return;
  }
}

namespace ospf_int {
int closure_build(ospf_ctx* c, const std::vector<uint32_t>& roots,
                  const std::vector<uint32_t>& seed_row, ClosureHost& h, uint32_t NW) {
  constexpr uint32_t kN = ~0u;
  const uint32_t nS = (uint32_t)c->h_ccv.size();
  if (c->cl_seed.empty()) return fail(c, OSPF_E_INVAL, "closure: no seed split of the cover");
  if (c->dist_bound >= ospf::kClInf) return fail(c, OSPF_E_RANGE, "closure: distances may reach 2^30");
  if (NW > ospf::kClMaxNW) return fail(c, OSPF_E_RANGE, "closure: next-hop masks of more than 4 words");
  std::vector<uint32_t> cidx(c->info.n_nodes, kN);
  for (uint32_t i = 0; i < nS; ++i) cidx[c->h_ccv[i]] = i;
  const uint32_t ncomp_all = (uint32_t)c->cl_comp_off.size() - 1;
  std::vector<uint32_t> slot(ncomp_all, kN), comps;
  uint32_t kmax = 1;
  for (uint32_t r : roots) {
    const uint32_t ci = r < cidx.size() ? cidx[r] : kN;
    if (ci == kN || c->cl_comp_of[ci] == kN)
      return fail(c, OSPF_E_INVAL, "closure: a root is not a non-seed cover node");
    const uint32_t k = c->cl_comp_of[ci];
    if (slot[k] == kN) {
      slot[k] = (uint32_t)comps.size();
      comps.push_back(k);
      kmax = std::max(kmax, c->cl_comp_off[k + 1] - c->cl_comp_off[k]);
    }
  }
  const uint32_t KW = kmax <= 8 ? 8u : 16u;
  if (NW && KW != 8) return fail(c, OSPF_E_RANGE, "closure: next-hop masks need components of <= 8");
  const uint32_t nq = (uint32_t)comps.size();
  h.KW = KW;
  h.NW = NW;
  h.comp.assign(nq, make_uint2(0, 0));
  h.jl.clear();
  h.cst.clear();
  h.fh.clear();
  h.mem.assign((size_t)nq * KW, kN);
  h.dloc.assign((size_t)nq * KW * KW, kN);
  h.fhloc.assign((size_t)nq * KW * KW * NW, 0u);
  h.out.assign((size_t)nq * KW, kN);
  auto transit = [&](uint32_t i) { return (c->h_cctr[i >> 5] >> (i & 31u)) & 1u; };
  auto node_transit = [&](uint32_t v) { return !((c->h_nt[v >> 5] >> (v & 31u)) & 1u); };
  const auto& crow = c->h_ccrow;
  const auto& ced = c->h_cedge;
  std::vector<uint32_t> jof(nS, kN);  // seed -> term of the current component
  std::vector<uint64_t> d(KW);
  // next-hop masks (NW words) per member: first hops of f's shortest paths
  // to it inside the component
  std::vector<uint32_t> Mk((size_t)KW * ospf::kClMaxNW);
  // f's contracted out-edges with the next-hop bits achieving each one's
  // weight: the direct link (bit of the neighbour) and every transit leaf
  // detour f -> x -> b (bit of x), LinkState.cpp:885-901 with f the root
  struct EM {
    uint64_t w;
    uint32_t m[ospf::kClMaxNW];
  };
  std::unordered_map<uint32_t, EM> em;
  for (uint32_t i = 0; i < (uint32_t)roots.size(); ++i) {
    const uint32_t ci = cidx[roots[i]], k = c->cl_comp_of[ci];
    const uint32_t* M = c->cl_comp_mem.data() + c->cl_comp_off[k];
    const uint32_t kk = c->cl_comp_off[k + 1] - c->cl_comp_off[k];
    const uint32_t m = (uint32_t)(std::find(M, M + kk, ci) - M);
    h.out[(size_t)slot[k] * KW + m] = i;
  }
  for (uint32_t q = 0; q < nq; ++q) {
    const uint32_t k = comps[q];
    const uint32_t* M = c->cl_comp_mem.data() + c->cl_comp_off[k];
    const uint32_t kk = c->cl_comp_off[k + 1] - c->cl_comp_off[k];
    auto local = [&](uint32_t x) {
      for (uint32_t m = 0; m < kk; ++m)
        if (M[m] == x) return m;
      return kN;
    };
    for (uint32_t m = 0; m < kk; ++m) h.mem[(size_t)q * KW + m] = M[m];
    const uint32_t joff = (uint32_t)h.jl.size();
    std::vector<uint32_t> used;  // seeds given a term (jof reset after)
    for (uint32_t f = 0; f < kk; ++f) {
      if (NW) {  // f's out-edge masks from its CSR row
        em.clear();
        const uint32_t fn = c->h_ccv[M[f]];
        const uint32_t* dn = c->h_dn.data() + c->h_dn_off[fn];
        const uint32_t K = c->h_dn_off[fn + 1] - c->h_dn_off[fn];
        if (K > 32u * NW) return fail(c, OSPF_E_RANGE, "closure: a root with more neighbours than masks");
        auto cand = [&](uint32_t cb, uint64_t w, uint32_t bit) {
          auto it = em.find(cb);
          if (it == em.end()) {
            EM x{w, {0u, 0u, 0u, 0u}};
            x.m[bit >> 5] = 1u << (bit & 31u);
            em.emplace(cb, x);
          } else if (w < it->second.w) {
            it->second = EM{w, {0u, 0u, 0u, 0u}};
            it->second.m[bit >> 5] = 1u << (bit & 31u);
          } else if (w == it->second.w) {
            it->second.m[bit >> 5] |= 1u << (bit & 31u);
          }
        };
        for (uint32_t e = c->h_prow[fn]; e < c->h_prow[fn + 1]; ++e) {
          const uint32_t y = c->h_pcolx[e];
          if ((y & 0x80000000u) || y == fn) continue;  // down / padding, self-loop
          const uint32_t bit = (uint32_t)(std::lower_bound(dn, dn + K, y) - dn);
          if (cidx[y] != kN) {
            cand(cidx[y], c->h_pw[e], bit);
          } else if (node_transit(y)) {  // a leaf detour
            for (uint32_t e2 = c->h_prow[y]; e2 < c->h_prow[y + 1]; ++e2) {
              const uint32_t b = c->h_pcolx[e2];
              if ((b & 0x80000000u) || b == y || b == fn || cidx[b] == kN) continue;
              cand(cidx[b], (uint64_t)c->h_pw[e] + c->h_pw[e2], bit);
            }
          }
        }
      }
      // the mask an edge u -> (cover index x, weight w) hands on: f's own edge
      // masks from f, the tail's mask otherwise
      auto emask = [&](uint32_t u, uint32_t x, uint64_t w, const uint32_t*& m) {
        if (u != f) {
          m = Mk.data() + (size_t)u * ospf::kClMaxNW;
          return true;
        }
        auto it = em.find(x);
        if (it == em.end() || it->second.w != w) return false;  // inconsistent contraction
        m = it->second.m;
        return true;
      };
      // distances (and masks) inside the component from f: members relay when
      // transit (f itself always: the root), Bellman-Ford over <= 16 nodes
      std::fill(d.begin(), d.end(), UINT64_MAX);
      std::fill(Mk.begin(), Mk.end(), 0u);
      d[f] = 0;
      for (uint32_t it = 0; it <= kk; ++it) {
        bool ch = false;
        for (uint32_t u = 0; u < kk; ++u) {
          if (d[u] == UINT64_MAX || (u != f && !transit(M[u]))) continue;
          for (uint32_t e = crow[M[u]]; e < crow[M[u] + 1]; ++e) {
            const uint32_t x = local(ced[e].x);
            if (x == kN) continue;
            const uint64_t nd = d[u] + ced[e].y;
            const uint32_t* m = nullptr;
            if (NW && !emask(u, ced[e].x, ced[e].y, m))
              return fail(c, OSPF_E_RANGE, "closure: contracted edge without its next hops");
            uint32_t* mx = Mk.data() + (size_t)x * ospf::kClMaxNW;
            if (nd < d[x]) {
              d[x] = nd;
              for (uint32_t w = 0; w < NW; ++w) mx[w] = m[w];
              ch = true;
            } else if (NW && nd == d[x]) {
              for (uint32_t w = 0; w < NW; ++w) {
                ch |= (mx[w] | m[w]) != mx[w];
                mx[w] |= m[w];
              }
            }
          }
        }
        if (!ch) break;
      }
      for (uint32_t m = 0; m < kk; ++m) {
        h.dloc[((size_t)q * KW + f) * KW + m] = d[m] >= ospf::kClInf ? ospf::kClInf : (uint32_t)d[m];
        for (uint32_t w = 0; w < NW; ++w)
          h.fhloc[(((size_t)q * KW + f) * KW + m) * NW + w] =
              d[m] >= ospf::kClInf ? 0u : Mk[(size_t)m * ospf::kClMaxNW + w];
      }
      for (uint32_t g = 0; g < kk; ++g) {
        if (d[g] == UINT64_MAX || (g != f && !transit(M[g]))) continue;
        for (uint32_t e = crow[M[g]]; e < crow[M[g] + 1]; ++e) {
          const uint32_t x = ced[e].x;
          if (c->cl_comp_of[x] != kN) continue;  // not a seed
          if (jof[x] == kN) {
            if (seed_row[x] == kN) return fail(c, OSPF_E_INVAL, "closure: a seed row is missing");
            jof[x] = (uint32_t)h.jl.size() - joff;
            h.jl.push_back(seed_row[x]);
            h.cst.resize(h.jl.size() * KW, ospf::kClInf);
            h.fh.resize(h.jl.size() * KW * NW, 0u);
            used.push_back(x);
          }
          const uint64_t cc = d[g] + ced[e].y;
          const size_t ti = (size_t)(joff + jof[x]) * KW + f;
          uint32_t& dst = h.cst[ti];
          const uint32_t* m = nullptr;
          if (NW && !emask(g, x, ced[e].y, m))
            return fail(c, OSPF_E_RANGE, "closure: contracted edge without its next hops");
          if (cc < dst) {  // (dst <= kClInf)
            dst = (uint32_t)cc;
            for (uint32_t w = 0; w < NW; ++w) h.fh[ti * NW + w] = m[w];
          } else if (NW && cc == dst) {
            for (uint32_t w = 0; w < NW; ++w) h.fh[ti * NW + w] |= m[w];
          }
        }
      }
    }
    // terms in ascending order of their smallest constant: a column's best
    // value tends to come early, so later terms rarely tie or beat it and the
    // kernel's mask updates (taken only when some lane does) are mostly skipped
    {
      const uint32_t nt = (uint32_t)h.jl.size() - joff;
      std::vector<uint32_t> ord(nt), key(nt, ospf::kClInf);
      for (uint32_t t = 0; t < nt; ++t) {
        ord[t] = t;
        for (uint32_t f = 0; f < KW; ++f) key[t] = std::min(key[t], h.cst[(size_t)(joff + t) * KW + f]);
      }
      std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
      std::vector<uint32_t> jl2(nt), cst2((size_t)nt * KW), fh2((size_t)nt * KW * NW);
      for (uint32_t t = 0; t < nt; ++t) {
        const uint32_t o = ord[t];
        jl2[t] = h.jl[joff + o];
        std::copy_n(h.cst.begin() + (size_t)(joff + o) * KW, KW, cst2.begin() + (size_t)t * KW);
        if (NW)
          std::copy_n(h.fh.begin() + (size_t)(joff + o) * KW * NW, (size_t)KW * NW,
                      fh2.begin() + (size_t)t * KW * NW);
      }
      std::copy(jl2.begin(), jl2.end(), h.jl.begin() + joff);
      std::copy(cst2.begin(), cst2.end(), h.cst.begin() + (size_t)joff * KW);
      if (NW) std::copy(fh2.begin(), fh2.end(), h.fh.begin() + (size_t)joff * KW * NW);
    }
    h.comp[q] = make_uint2(joff, (uint32_t)h.jl.size() - joff);
    for (uint32_t x : used) jof[x] = kN;
  }
  if (h.jl.empty()) {  // no seed terms at all: one unused row keeps the arrays non-empty
    h.jl.push_back(0);
    h.cst.assign(KW, ospf::kClInf);
    h.fh.assign((size_t)KW * std::max(NW, 1u), 0u);
  }
  if (h.fh.empty()) h.fh.assign(1, 0u);
  if (h.fhloc.empty()) h.fhloc.assign(1, 0u);
  return OSPF_OK;
}
}  // namespace ospf_int

extern "C" {

int ospf_open(int device, ospf_ctx** out) {
  if (!out) return OSPF_E_INVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return OSPF_E_DEVICE;
  if (device < 0 || device >= n) return OSPF_E_INVAL;
  ospf_ctx* c = new (std::nothrow) ospf_ctx();
  if (!c) return OSPF_E_NOMEM;
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) {
    delete c;
    return OSPF_E_DEVICE;
  }
  int lds = 0, cu = 0;
  hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device);
  hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device);
  // keep 1 KiB for the kernels' static LDS (digest reduction)
  if (lds > 2048) c->lds_limit = (size_t)lds - 1024;
  c->lds_attr = lds;
  if (cu > 0) c->n_cu = cu;
  if (hipMalloc((void**)&c->d_err, sizeof(uint32_t)) != hipSuccess ||
      hipMemset(c->d_err, 0, sizeof(uint32_t)) != hipSuccess) {
    delete c;
    return OSPF_E_DEVICE;
  }
  *out = c;
  return OSPF_OK;
}

int ospf_close(ospf_ctx* c) {
  if (!c) return OSPF_E_INVAL;
  hipSetDevice(c->device);
  // sweeps still alive: their resources back (to the pools freed below) and
  // detached from this context
  for (ospf_sweep* s : std::vector<ospf_sweep*>(c->live_sweeps))
    if (c->release_sweep) c->release_sweep(s);
  c->live_sweeps.clear();
  if (c->d_graph) hipFree(c->d_graph);
  for (auto& kv : c->scratch)
    if (kv.second.p) hipFree(kv.second.p);
  if (c->d_stage) hipFree(c->d_stage);
  if (c->d_err) hipFree(c->d_err);
  for (hipEvent_t e : c->ev) hipEventDestroy(e);
  if (c->aux) hipStreamDestroy(c->aux);
  if (c->ksp_aux) hipStreamDestroy(c->ksp_aux);
  if (c->ksp_hi) hipStreamDestroy(c->ksp_hi);
  for (hipEvent_t e : c->ksp_ev)
    if (e) hipEventDestroy(e);
  for (hipEvent_t e : c->lv_ev)
    if (e) hipEventDestroy(e);
  if (c->d_cover) hipFree(c->d_cover);
  if (c->lv_aux) hipStreamDestroy(c->lv_aux);
  pool_release(c);
  for (hipStream_t st : c->stream_pool) hipStreamDestroy(st);
  for (hipEvent_t e : c->event_pool) hipEventDestroy(e);
  delete c;
  return OSPF_OK;
}

const char* ospf_last_error(const ospf_ctx* c) { return c ? c->err.c_str() : "null context"; }

int ospf_inject_error(ospf_ctx* c, uint32_t after_calls) {
  if (!c) return OSPF_E_INVAL;
  c->inject_after = after_calls;
  return OSPF_OK;
}

uint64_t ospf_spf_runs(const ospf_ctx* c) { return c ? c->spf_runs : 0; }

int ospf_load_graph(ospf_ctx* c, const ospf_csr* csr, uint64_t version) {
  if (!c || !csr) return OSPF_E_INVAL;
  if (injected(c)) return OSPF_E_DEVICE;
  // OSPF_SWEEP_TIMING: host phases of the load on stderr
  const bool tm = getenv("OSPF_SWEEP_TIMING") != nullptr;
  auto tl = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!tm) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "sweep_create load/%s %.2f ms\n", what,
            std::chrono::duration<double, std::milli>(now - tl).count());
    tl = now;
  };
  const uint32_t V = csr->n_nodes, E = csr->n_edges;
  if (V == 0 || V >= 0x80000000u) return fail(c, OSPF_E_INVAL, "n_nodes out of range");
  if (!csr->row_ptr || (E && (!csr->col || !csr->metric || !csr->link_id || !csr->twin ||
                              !csr->edge_up)))
    return fail(c, OSPF_E_INVAL, "null CSR array");
  if (csr->row_ptr[0] != 0 || csr->row_ptr[V] != E)
    return fail(c, OSPF_E_INVAL, "row_ptr must start at 0 and end at n_edges");

  // validation, flagged entries and distinct-neighbour counts per node on
  // host threads (chunks of 512 nodes: whole words of the no-transit bits)
  std::vector<uint32_t> colx(E), rw(E), nt((V + 31) / 32, 0u), dn_off(V + 1, 0u);
  uint32_t max_deg = 0, max_metric = 0, max_dn = 0, n_links = 0;
  uint64_t dist_bound = 0;
  bool unit = true;
  std::mutex red_mu;
  int bad_rc = OSPF_OK;
  const char* bad_msg = nullptr;
  // (chunks by entries, starting at multiples of 32 nodes: whole words of
  // the no-transit bits)
  ospf_int::par_for_rows(V, csr->row_ptr, [&](uint32_t lo, uint32_t hi) {
    uint32_t l_deg = 0, l_metric = 0, l_dn = 0, l_links = 0;
    uint64_t l_bound = 0;
    bool l_unit = true;
    int rc = OSPF_OK;
    const char* msg = nullptr;
    auto bad = [&](int code, const char* m) {
      rc = code;
      msg = m;
    };
    for (uint32_t u = lo; u < hi && rc == OSPF_OK; ++u) {
      const uint32_t b = csr->row_ptr[u], e1 = csr->row_ptr[u + 1];
      uint32_t row_max = 0, ndn = 0;
      if (e1 < b || e1 > E) {
        bad(OSPF_E_INVAL, "row_ptr not monotone");
        break;
      }
      l_deg = std::max(l_deg, e1 - b);
      for (uint32_t e = b; e < e1; ++e) {
        const uint32_t v = csr->col[e];
        if (v >= V) { bad(OSPF_E_INVAL, "col out of range"); break; }
        if (e > b && csr->col[e - 1] > v) { bad(OSPF_E_INVAL, "rows must be sorted by col"); break; }
        const uint32_t t = csr->twin[e];
        if (t >= E || csr->twin[t] != e || csr->col[t] != u || t < csr->row_ptr[v] ||
            t >= csr->row_ptr[v + 1] || csr->link_id[t] != csr->link_id[e]) {
          bad(OSPF_E_INVAL, "twin/link_id inconsistent");
          break;
        }
        if (csr->edge_up[e] != csr->edge_up[t]) {
          bad(OSPF_E_INVAL, "edge_up must match on both directions of a link");
          break;
        }
        const bool up = csr->edge_up[e] != 0;
        colx[e] = v | (up ? 0u : 0x80000000u);
        rw[e] = csr->metric[t];
        if (up) {
          if (csr->metric[e] == 0) {
            bad(OSPF_E_RANGE, "metric 0 on a usable link is outside the engine contract");
            break;
          }
          l_metric = std::max(l_metric, csr->metric[e]);
          row_max = std::max(row_max, csr->metric[e]);
          l_unit &= csr->metric[e] == 1;
        }
        if (e < t) ++l_links;
        if (v != u && (e == b || csr->col[e - 1] != v)) ++ndn;
      }
      dn_off[u + 1] = ndn;
      l_dn = std::max(l_dn, ndn);
      l_bound += row_max;
      if (csr->no_transit && csr->no_transit[u]) nt[u >> 5] |= 1u << (u & 31);
    }
    std::lock_guard<std::mutex> g(red_mu);
    max_deg = std::max(max_deg, l_deg);
    max_metric = std::max(max_metric, l_metric);
    max_dn = std::max(max_dn, l_dn);
    n_links += l_links;
    dist_bound += l_bound;
    unit &= l_unit;
    if (rc != OSPF_OK && bad_rc == OSPF_OK) {
      bad_rc = rc;
      bad_msg = msg;
    }
  }, 8192, 32);
  if (bad_rc != OSPF_OK) return fail(c, bad_rc, bad_msg);
  for (uint32_t u = 0; u < V; ++u) dn_off[u + 1] += dn_off[u];
  std::vector<uint32_t> dn(dn_off[V]);
  ospf_int::par_for_rows(V, csr->row_ptr, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t u = lo; u < hi; ++u) {
      uint32_t k = dn_off[u];
      for (uint32_t e = csr->row_ptr[u], b = e; e < csr->row_ptr[u + 1]; ++e) {
        const uint32_t v = csr->col[e];
        if (v != u && (e == b || csr->col[e - 1] != v)) dn[k++] = v;
      }
    }
  });
  lap("validate + distinct neighbours");
  if (max_dn > OSPF_MAX_ROOT_NEIGHBORS)
    return fail(c, OSPF_E_RANGE, "a node has more distinct neighbours than OSPF_MAX_ROOT_NEIGHBORS");

  // Device rows are padded to a multiple of 4 entries with down-marked
  // fillers (colx = 0x80000000, link id UINT32_MAX) so every row starts on a
  // 16-B boundary and the kernels read the CSR with uint4 loads.
  std::vector<uint32_t> prow(V + 1, 0u);
  for (uint32_t u = 0; u < V; ++u)
    prow[u + 1] = prow[u] + ((csr->row_ptr[u + 1] - csr->row_ptr[u] + 3u) & ~3u);
  const uint32_t Ep = prow[V];
  std::vector<uint32_t> pcolx(Ep, 0x80000000u), pw(Ep, 0u), prw(Ep, 0u), plink(Ep, 0xFFFFFFFFu);
  // link_rank given: a parallel group (same neighbour) is ordered by the
  // twin entry's rank = the link's position in linksFromNode(neighbour), the
  // order pathLinks lists links of one predecessor in (LinkState.cpp:885-901)
  uint32_t max_lid = 0;
  ospf_int::par_for_rows(V, csr->row_ptr, [&](uint32_t lo, uint32_t hi) {
    std::vector<uint32_t> ord;
    uint32_t l_lid = 0;
    for (uint32_t u = lo; u < hi; ++u) {
      const uint32_t b = csr->row_ptr[u], n = csr->row_ptr[u + 1] - b, pb = prow[u];
      ord.resize(n);
      for (uint32_t k = 0; k < n; ++k) ord[k] = b + k;
      // rows are sorted by neighbour: only a run of parallel links (equal
      // neighbours) is reordered, by its twins' ranks
      if (csr->link_rank)
        for (uint32_t k = 0; k < n;) {
          uint32_t k1 = k + 1;
          while (k1 < n && csr->col[b + k1] == csr->col[b + k]) ++k1;
          if (k1 - k > 1)
            std::stable_sort(ord.begin() + k, ord.begin() + k1, [&](uint32_t x, uint32_t y) {
              return csr->link_rank[csr->twin[x]] < csr->link_rank[csr->twin[y]];
            });
          k = k1;
        }
      for (uint32_t k = 0; k < n; ++k) {
        const uint32_t e = ord[k];
        pcolx[pb + k] = colx[e];
        pw[pb + k] = csr->metric[e];
        prw[pb + k] = rw[e];
        plink[pb + k] = csr->link_id[e];
        l_lid = std::max(l_lid, csr->link_id[e]);
      }
    }
    std::lock_guard<std::mutex> g(red_mu);
    max_lid = std::max(max_lid, l_lid);
  });
  lap("padded rows + parallel-link order");
  // entries of each link id (KSP2 ignore masks); ids above 2^28 disable them
  const uint32_t n_lid = (E && max_lid < (1u << 28)) ? max_lid + 1 : 0;
  // Reserves for structural patches (ospf_update_rows, links added / removed
  // in place): per-entry arrays, distinct neighbours and link ids get ~3 %
  // headroom past their current use; an update that outgrows one returns
  // OSPF_E_RANGE and the caller reloads.
  auto reserve = [](size_t used) { return used + std::max<size_t>(1024, used / 32); };
  const size_t cap_e = align_up(reserve(Ep), 4), cap_dn = reserve(dn.size()),
               cap_lid = n_lid ? reserve(n_lid) : 0;
  // [2 lid] = the link's first entry, [2 lid + 1] = its second (none: ~0):
  // the smallest and largest entry of each id, on host threads
  std::vector<uint32_t> link_e(std::max<size_t>(2ull * n_lid, 2), 0xFFFFFFFFu);
  if (n_lid) {
    for (size_t l = 0; l < n_lid; ++l) link_e[2 * l + 1] = 0u;
    ospf_int::par_for(Ep, [&](uint32_t lo, uint32_t hi) {
      for (uint32_t e = lo; e < hi; ++e) {
        if (plink[e] == 0xFFFFFFFFu) continue;
        uint32_t* le = &link_e[2ull * plink[e]];
        __atomic_fetch_min(le, e, __ATOMIC_RELAXED);
        __atomic_fetch_max(le + 1, e, __ATOMIC_RELAXED);
      }
    }, 1u << 14);
    for (size_t l = 0; l < n_lid; ++l)
      if (link_e[2 * l + 1] == link_e[2 * l] || link_e[2 * l] == 0xFFFFFFFFu)
        link_e[2 * l + 1] = 0xFFFFFFFFu;  // one entry (or none)
  }

  // device layout: one allocation, 256-B aligned sub-buffers
  std::vector<uint32_t> big;  // rows the multi-source BFS scans with a whole wave
  for (uint32_t u = 0; u < V; ++u)
    if (prow[u + 1] - prow[u] > ospf::kMsBigDeg) big.push_back(u);
  const size_t sz_row = (V + 1) * 4ull, sz_e = (size_t)Ep * 4ull, sz_nt = nt.size() * 4ull,
               sz_dnoff = (V + 1) * 4ull, sz_dn = std::max<size_t>(dn.size(), 1) * 4ull,
               sz_big = std::max<size_t>(big.size(), 1) * 4ull, sz_key = V * 16ull,
               sz_le = link_e.size() * 4ull;
  std::vector<uint64_t> dkey(2ull * V);  // digest key tables (row digest kernel)
  ospf_int::par_for(V, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t u = lo; u < hi; ++u) {
      dkey[2ull * u] = ospf::digest_dist_key(u);
      dkey[2ull * u + 1] = ospf::digest_node_key(u);
    }
  });
  // packed {colx, w | rw << 16} entries when every metric fits 16 bits
  bool ew_ok = true;
  for (uint32_t e = 0; e < Ep && ew_ok; ++e) ew_ok = pw[e] <= 0xFFFFu && prw[e] <= 0xFFFFu;
  std::vector<uint32_t> pew(ew_ok ? 2ull * Ep : 2, 0u);
  if (ew_ok)
    ospf_int::par_for(Ep, [&](uint32_t lo, uint32_t hi) {
      for (uint32_t e = lo; e < hi; ++e) {
        pew[2ull * e] = pcolx[e];
        pew[2ull * e + 1] = pw[e] | (prw[e] << 16);
      }
    }, 1u << 16);
  const size_t sz_ew = pew.size() * 4ull;
  // distinct-neighbour index per padded entry (rows are sorted by neighbour)
  std::vector<uint16_t> didx(std::max<uint32_t>(Ep, 1), 0xFFFFu);
  ospf_int::par_for_rows(V, prow.data(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t u = lo; u < hi; ++u) {
      uint32_t k = 0, prev = 0xFFFFFFFFu;
      for (uint32_t e = prow[u]; e < prow[u + 1]; ++e) {
        const uint32_t v = pcolx[e] & 0x7FFFFFFFu;
        if (plink[e] == 0xFFFFFFFFu || v == u) continue;  // padding, self-loop
        if (prev != 0xFFFFFFFFu && v != prev) ++k;
        prev = v;
        didx[e] = (uint16_t)k;
      }
    }
  });
  const size_t sz_didx = didx.size() * 2ull;
  // node keys alone, zero padded past V: a lane's 16 nodes in 8 loads, and
  // kernels that walk level rows to their pitch (V rounded up to 128 in the
  // sweeps) read up to 128 keys past V
  std::vector<uint64_t> dkn((V + 127) / 128 * 128 + 128, 0ull);
  for (uint32_t u = 0; u < V; ++u) dkn[u] = dkey[2ull * u + 1];
  const size_t sz_kn = dkn.size() * 8ull;
  lap("link entries, digest keys, packed entries, didx");
  size_t off[14], tot = 0;
  const size_t szs[14] = {sz_row, sz_e,     sz_e,  sz_e,   sz_e,  sz_nt,  sz_dnoff,
                          sz_dn,  sz_big,   sz_key, sz_le, sz_ew, sz_didx, sz_kn};
  // allocated: the per-entry arrays, dn and link_e with their reserves, big
  // for every node
  const size_t caps[14] = {sz_row, cap_e * 4, cap_e * 4, cap_e * 4, cap_e * 4, sz_nt, sz_dnoff,
                           cap_dn * 4, V * 4ull, sz_key, std::max<size_t>(2 * cap_lid, 2) * 4,
                           ew_ok ? cap_e * 8 : sz_ew, cap_e * 2, sz_kn};
  for (int i = 0; i < 14; ++i) {
    off[i] = tot;
    tot += align_up(std::max<size_t>(caps[i], 4), 256);
  }
  HIPCHK(c, hipSetDevice(c->device));
  if (c->d_graph) {
    hipFree(c->d_graph);
    c->d_graph = nullptr;
    c->loaded = false;
  }
  hipError_t he = dev_malloc(c, &c->d_graph, tot);
  if (he != hipSuccess) {
    c->d_graph = nullptr;
    return fail(c, OSPF_E_NOMEM, std::string("hipMalloc graph: ") + hipGetErrorString(he));
  }
  char* base = (char*)c->d_graph;
  const void* srcs[14] = {prow.data(), pcolx.data(), pw.data(), prw.data(), plink.data(),
                          nt.data(), dn_off.data(), dn.data(), big.data(), dkey.data(),
                          link_e.data(), pew.data(), didx.data(), dkn.data()};
  for (int i = 0; i < 14; ++i)
    if (szs[i] && srcs[i]) HIPCHK(c, hipMemcpy(base + off[i], srcs[i], szs[i], hipMemcpyHostToDevice));
  lap("device allocation + copies");
  c->g.V = V;
  c->g.E = Ep;
  c->g.row_ptr = (const uint32_t*)(base + off[0]);
  c->g.colx = (const uint32_t*)(base + off[1]);
  c->g.w = (const uint32_t*)(base + off[2]);
  c->g.rw = (const uint32_t*)(base + off[3]);
  c->g.link_id = (const uint32_t*)(base + off[4]);
  c->g.nt_bits = (const uint32_t*)(base + off[5]);
  c->g.dn_off = (const uint32_t*)(base + off[6]);
  c->g.dn = (const uint32_t*)(base + off[7]);
  c->g.nbig = (uint32_t)big.size();
  c->g.big = (const uint32_t*)(base + off[8]);
  c->g.dkey = (const uint64_t*)(base + off[9]);
  c->g.n_lid = n_lid;
  c->g.link_e = (const uint32_t*)(base + off[10]);
  c->g.ew = ew_ok ? (const uint2*)(base + off[11]) : nullptr;
  c->g.didx = (const uint16_t*)(base + off[12]);
  c->g.dkn = (const uint64_t*)(base + off[13]);
  c->ew_base = ew_ok ? (const uint32_t*)(base + off[11]) : nullptr;
  c->cap_e = cap_e;
  c->cap_dn = cap_dn;
  c->cap_lid = cap_lid;
  c->h_plink = std::move(plink);
  c->h_row_ptr.assign(csr->row_ptr, csr->row_ptr + V + 1);
  c->h_dn_off = std::move(dn_off);
  c->h_dn = std::move(dn);
  c->max_dn = max_dn;
  c->depth_bound = transit_depth_bound(V, csr->row_ptr, colx.data(), nt);
  c->exact_bound = c->depth_bound;
  c->h_prow = std::move(prow);
  c->h_pcolx = std::move(pcolx);
  c->h_pw = std::move(pw);
  c->h_prw = std::move(prw);
  c->h_nt = std::move(nt);
  c->h_link_e = std::move(link_e);
  c->non_unit = 0;
  {
    std::atomic<uint64_t> nu{0};
    ospf_int::par_for(Ep, [&](uint32_t lo, uint32_t hi) {
      uint64_t k = 0;
      for (uint32_t e = lo; e < hi; ++e) k += !(c->h_pcolx[e] & 0x80000000u) && c->h_pw[e] != 1;
      nu += k;
    }, 1u << 16);
    c->non_unit = nu.load();
  }
  c->info.n_nodes = V;
  c->info.n_edges = E;
  c->info.n_links = n_links;
  c->info.max_degree = max_deg;
  c->info.max_metric = max_metric;
  c->info.unit_metric = unit ? 1u : 0u;
  c->info.version = version;
  c->cover_ok = false;  // the contracted cover graph describes the old graph
  c->info.device_bytes = tot;
  c->dist_bound = dist_bound;
  c->h_rowmax.assign(V, 0u);
  ospf_int::par_for_rows(V, c->h_prow.data(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t u = lo; u < hi; ++u)
      for (uint32_t e = c->h_prow[u]; e < c->h_prow[u + 1]; ++e)
        if (!(c->h_pcolx[e] & 0x80000000u)) c->h_rowmax[u] = std::max(c->h_rowmax[u], c->h_pw[e]);
  });
  c->mask = ospf_ctx::Mask{};
  c->loaded = true;
  ++c->graph_gen;
  lap("depth bound + host shadows");
  return OSPF_OK;
}

int ospf_graph_info_get(const ospf_ctx* c, ospf_graph_info* info) {
  if (!c || !info) return OSPF_E_INVAL;
  if (!c->loaded) return OSPF_E_NOGRAPH;
  *info = c->info;
  return OSPF_OK;
}

int ospf_root_neighbors(const ospf_ctx* c, uint32_t root, uint32_t* ids, uint32_t cap,
                        uint32_t* n) {
  if (!c || !n) return OSPF_E_INVAL;
  if (!c->loaded) return OSPF_E_NOGRAPH;
  if (root >= c->info.n_nodes) return OSPF_E_INVAL;
  const uint32_t b = c->h_dn_off[root], e = c->h_dn_off[root + 1];
  *n = e - b;
  if (ids)
    for (uint32_t i = 0; i < std::min(cap, e - b); ++i) ids[i] = c->h_dn[b + i];
  return OSPF_OK;
}

int ospf_plan_variant(const ospf_ctx* c, uint32_t flags, uint32_t nh_words, int* variant) {
  if (!c || !variant) return OSPF_E_INVAL;
  if (!c->loaded) return OSPF_E_NOGRAPH;
  const bool unit = (flags & OSPF_HOP_COUNT) || c->info.unit_metric;
  *variant = make_plan(c, std::max<uint32_t>(nh_words, 1), 0, unit, 0xFFFFFFFFu).variant;
  return OSPF_OK;
}

int ospf_plan_n(const ospf_ctx* c, uint32_t flags, uint32_t nh_words, uint32_t max_ignored,
                uint32_t n_roots, uint32_t max_root_neighbors, ospf_plan_info* out) {
  if (!c || !out) return OSPF_E_INVAL;
  if (!c->loaded) return OSPF_E_NOGRAPH;
  const bool unit = (flags & OSPF_HOP_COUNT) || c->info.unit_metric;
  const uint32_t W = std::max<uint32_t>(nh_words, 1);
  const Plan p = make_plan(c, W, max_ignored, unit, n_roots);
  out->variant = p.variant;
  out->block = p.block;
  out->lds_bytes = (uint32_t)p.lds;
  if (p.variant == 5) {
    const uint32_t kcap = max_root_neighbors ? std::min(max_root_neighbors, 32u * W) : 32u * W;
    out->slices = ms_shape(n_roots, kcap, c->depth_bound <= 253 && getenv("OSPF_MS_PACK")).npass;
  } else {
    out->slices = (p.variant == 3 || p.variant == 4) ? ospf::bfs_slices(W) : 1u;
  }
  return OSPF_OK;
}

int ospf_plan(const ospf_ctx* c, uint32_t flags, uint32_t nh_words, uint32_t max_ignored,
              ospf_plan_info* out) {
  return ospf_plan_n(c, flags, nh_words, max_ignored, 0xFFFFFFFFu, 0, out);
}

int ospf_run_batch_dev(ospf_ctx* c, const ospf_batch* b, void* stream) {
  if (!c || !b) return OSPF_E_INVAL;
  const uint32_t* d_roots = b->d_roots;
  const uint32_t n_roots = b->n_roots;
  const uint32_t *d_ign_off = b->d_ign_offsets, *d_ign_ids = b->d_ign_ids;
  const uint32_t max_ignored = b->max_ignored, flags = b->flags, nh_words = b->nh_words;
  uint32_t* d_dist = b->d_dist;
  uint32_t* d_nh = b->d_nh;
  ospf_digest* d_digest = b->d_digest;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (n_roots == 0) return OSPF_OK;
  if (!d_roots) return fail(c, OSPF_E_INVAL, "null roots");
  if (nh_words == 0 || nh_words > OSPF_MAX_ROOT_NEIGHBORS / 32)
    return fail(c, OSPF_E_INVAL, "nh_words out of range");
  if ((flags & OSPF_WANT_DIST) && !d_dist) return fail(c, OSPF_E_INVAL, "WANT_DIST without buffer");
  if ((flags & OSPF_WANT_NH) && !d_nh) return fail(c, OSPF_E_INVAL, "WANT_NH without buffer");
  if ((flags & OSPF_WANT_DIGEST) && !d_digest)
    return fail(c, OSPF_E_INVAL, "WANT_DIGEST without buffer");
  const bool hop = flags & OSPF_HOP_COUNT;
  const bool ign = d_ign_off != nullptr;
  if (ign && (!d_ign_ids && max_ignored)) return fail(c, OSPF_E_INVAL, "null ignore ids");
  if (ign && max_ignored > OSPF_MAX_IGNORED_PER_RUN)
    return fail(c, OSPF_E_RANGE, "max_ignored above OSPF_MAX_IGNORED_PER_RUN");
  const uint64_t V = c->info.n_nodes;
  if (!hop && c->dist_bound >= 0xFFFFFFFFull)
    return fail(c, OSPF_E_RANGE, "u32 distance overflow possible (sum of per-node max metrics)");
  const bool unit = hop || c->info.unit_metric;

  const Plan p = make_plan(c, nh_words, ign ? std::max<uint32_t>(max_ignored, 1) : 0, unit, n_roots);
  if (p.variant == 5) return run_msbfs(c, b, (hipStream_t)stream);
  if (p.variant == 7) return run_wdial(c, b, hop, (hipStream_t)stream);
  // scratch for state the caller does not want back (HBM-state variants
  // keep dist / next-hops in the output rows while they run)
  size_t need = 0;
  const bool dist_scratch = (p.variant >= 2) && !(flags & OSPF_WANT_DIST);
  const bool nh_scratch = (p.variant >= 1) && !(flags & OSPF_WANT_NH);
  const uint32_t slices = (p.variant == 3 || p.variant == 4) ? ospf::bfs_slices(nh_words) : 1u;
  const size_t planes_bytes = slices > 1 ? align_up((size_t)n_roots * slices * V * 16ull, 256) : 0;
  if (dist_scratch) need += align_up(n_roots * V * 4, 256);
  if (nh_scratch) need += align_up(n_roots * V * nh_words * 4ull, 256);
  need += planes_bytes;
  // variant 6: per-root frontier lists
  const uint32_t nbk = c->info.max_metric + 1;
  const uint32_t bcap = (uint32_t)std::min<uint64_t>(V, 16384);
  const size_t bkt_bytes = p.variant == 6 ? align_up((size_t)n_roots * nbk * bcap * 4ull, 256) : 0;
  need += bkt_bytes;
  int src = OSPF_OK;
  char* sp = need ? stream_scratch(c, stream, need, &src) : nullptr;
  if (src) return src;
  ospf::RunArgs a{};
  a.roots = d_roots;
  a.ign_off = ign ? d_ign_off : nullptr;
  a.ign_ids = d_ign_ids;
  a.flags = flags;
  a.W = nh_words;
  a.nbr_cap = p.nbr_cap;
  a.ign_cap = p.ign_cap;
  a.dist = d_dist;
  a.nh = d_nh;
  a.digest = d_digest;
  a.err = c->d_err;
  a.slices = slices;
  a.planes = nullptr;
  if (planes_bytes) {
    a.planes = (uint32_t*)sp;
    sp += planes_bytes;
  }
  if (bkt_bytes) {
    a.bkt = (uint32_t*)sp;
    a.bcap = bcap;
    a.nbk = nbk;
    sp += bkt_bytes;
  }
  if (dist_scratch) {
    a.dist = (uint32_t*)sp;
    sp += align_up(n_roots * V * 4, 256);
  }
  if (nh_scratch) a.nh = (uint32_t*)sp;
  if (!(flags & OSPF_WANT_DIST) && p.variant < 2) a.dist = nullptr;
  if (!(flags & OSPF_WANT_NH) && p.variant == 0) a.nh = nullptr;

  HIPCHK(c, hipSetDevice(c->device));
  if (a.slices > 1 && (flags & OSPF_WANT_DIGEST))  // slices add into the records
    HIPCHK(c, ospf::zero_async(d_digest, n_roots * sizeof(ospf_digest), (hipStream_t)stream));
  hipError_t e = p.variant == 6
      ? ospf::launch_dial(ign, c->g, a, n_roots, p.lds, (hipStream_t)stream)
      : p.variant >= 3
      ? ospf::launch_bfs(p.variant == 3, ign, c->g, a, n_roots, p.block, p.lds, (hipStream_t)stream)
      : ospf::launch_spf(p.variant, unit, ign, c->g, a, n_roots, p.block, p.lds,
                         (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(c, e, "launch_spf");
  c->spf_runs += n_roots;
  return OSPF_OK;
}

int ospf_sssp_batch_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n_roots,
                        const uint32_t* d_ign_off, const uint32_t* d_ign_ids,
                        uint32_t max_ignored, uint32_t flags, uint32_t nh_words,
                        uint32_t* d_dist, uint32_t* d_nh, ospf_digest* d_digest,
                        void* stream) {
  ospf_batch b{};
  b.d_roots = d_roots;
  b.n_roots = n_roots;
  b.d_ign_offsets = d_ign_off;
  b.d_ign_ids = d_ign_ids;
  b.max_ignored = max_ignored;
  b.flags = flags;
  b.nh_words = nh_words;
  b.max_root_neighbors = 0;
  b.d_dist = d_dist;
  b.d_nh = d_nh;
  b.d_digest = d_digest;
  return ospf_run_batch_dev(c, &b, stream);
}

int ospf_sync(ospf_ctx* c, void* stream) {
  if (!c) return OSPF_E_INVAL;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
  uint32_t err = 0;
  HIPCHK(c, hipMemcpy(&err, c->d_err, 4, hipMemcpyDeviceToHost));
  if (err) {
    HIPCHK(c, hipMemset(c->d_err, 0, 4));
    return fail(c, OSPF_E_RANGE,
                (err & 1u) ? "a root has more distinct neighbours than 32*nh_words"
                : (err & 2u) ? "a run's ignore list exceeds max_ignored"
                : (err & 8u) ? "a BFS level past the graph's depth bound was reached"
                : (err & 16u) ? "derive: a root or a usable neighbour has no level row"
                : (err & 64u) ? "a device root id is out of range"
                : (err & 128u) ? "leaf derive: a group's roots do not share their slot table"
                : (err & 256u) ? "twin derive: a root's neighbours span more than 16 twin classes"
                : (err & 512u) ? "wderive: a metric above 65534 in a > 4-word next-hop derivation"
                : (err & 2048u) ? "internal: a heavy KSP2 run no longer fits the decremental budgets"
                             : "internal: a frontier entry out of range");
  }
  return OSPF_OK;
}

// ---------------------------------------------------------------- derive
// All-sources next hops in two phases (spf_msbfs.hip "derive"): distances of
// every root by the distance-only multi-source BFS (no bit-planes, one
// traversal per 64 roots whatever their width), written as dist rows and as
// byte level rows; then each root's next-hop words from its neighbours'
// level rows. Unit metric or hop count, depth bound <= 253.
int ospf_levels_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                    uint32_t* d_dist, uint8_t* d_lev, uint32_t lev_pitch,
                    ospf_digest* d_lev_digest, void* stream) {
  return ospf_int::levels_dev(c, d_roots, n, flags, d_dist, 0, d_lev, lev_pitch, d_lev_digest,
                              stream);
}
}  // extern "C"

namespace ospf_int {
int levels_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t flags,
               uint32_t* d_dist, uint32_t dist_pitch, uint8_t* d_lev, uint32_t lev_pitch,
               ospf_digest* d_lev_digest, void* stream, uint32_t depth_cap, uint32_t* d_maxd) {
  if (!c) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (n == 0) return OSPF_OK;
  if (!d_roots || !d_lev) return fail(c, OSPF_E_INVAL, "null roots / level rows");
  if (lev_pitch % 16u || lev_pitch < c->info.n_nodes)
    return fail(c, OSPF_E_INVAL, "lev_pitch: a multiple of 16 >= V");
  if (!(flags & OSPF_HOP_COUNT) && !c->info.unit_metric)
    return fail(c, OSPF_E_RANGE, "level rows need unit metric or hop count");
  if (c->depth_bound > 123)  // level bytes <= 125, below nh_derive's 0x7F marker
    return fail(c, OSPF_E_RANGE, "level rows need a depth bound <= 123");
  hipStream_t s = (hipStream_t)stream;
  const uint32_t V = c->info.n_nodes, lmax = c->depth_bound + 2;
  if (!getenv("OSPF_LV64")) {  // 128-root traversals (spf_levels.hip)
    // per wide batch: frontier slots 2 x 16 B, seen 16 B, accb 16 B, records 128 B;
    // two state buffers: the rows kernel of round k (on lv_aux) runs beside
    // the traversal of round k + 1 (on the caller's stream): the traversal is
    // latency-bound, the rows kernel store-bound
    const size_t per_wb = align_up((size_t)V * 16ull * 4 + V * 128ull + lmax * 8ull, 256);
    uint32_t nb_cap = 192;
    if (const char* e = getenv("OSPF_LV_NB")) nb_cap = std::max(1, atoi(e));
    const bool overlap = !getenv("OSPF_LV_SERIAL");
    const size_t nbuf = overlap ? 2 : 1;
    nb_cap = (uint32_t)std::max<size_t>(1, std::min<size_t>(nb_cap, (6ull << 30) / (per_wb * nbuf)));
    const uint32_t total = (n + 127) / 128, nb_max = std::min(nb_cap, total);
    int rc = OSPF_OK;
    char* sp = stream_scratch(c, s, per_wb * nb_max * nbuf, &rc);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    if (overlap && !c->lv_aux) {
      HIPCHK(c, hipStreamCreateWithFlags(&c->lv_aux, hipStreamNonBlocking));
      for (hipEvent_t& e : c->lv_ev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    ospf::LvArgs a{};
    a.roots = d_roots;
    a.n = n;
    a.lmax = lmax;
    a.dbound = depth_cap ? std::min(depth_cap, c->depth_bound) : c->depth_bound;
    a.maxd = d_maxd;
    a.push_div = 16;
    if (const char* e = getenv("OSPF_MS_PUSH_DIV")) a.push_div = (uint32_t)std::max(0, atoi(e));
    a.masked = 0;
    if (const char* e = getenv("OSPF_LV_MASKED")) a.masked = (uint32_t)atoi(e);
    a.dist = d_dist;
    a.dpitch = dist_pitch;
    a.levrow = d_lev;
    a.lev_pitch = lev_pitch;
    a.digest = d_lev_digest;
    a.err = c->d_err;
    if (d_lev_digest) HIPCHK(c, ospf::zero_async(d_lev_digest, (size_t)n * sizeof(ospf_digest), s));
    uint32_t k = 0;
    for (uint32_t vb0 = 0; vb0 < total; vb0 += nb_max, ++k) {
      const uint32_t buf = overlap ? (k & 1u) : 0u;
      char* base = sp + per_wb * nb_max * buf;
      a.vb0 = vb0;
      a.nb = std::min(nb_max, total - vb0);
      a.front = (uint4*)base;
      a.seen = a.front + 2ull * a.nb * V;
      a.accb = a.seen + (size_t)a.nb * V;
      a.lev = (uint8_t*)(a.accb + (size_t)a.nb * V);
      a.found = (uint32_t*)(a.lev + (size_t)a.nb * V * 128ull);
      a.mass = a.found + (size_t)a.nb * lmax;
      // the buffer's previous rows kernel (round k - 2) must be done with it
      if (overlap && k >= 2) HIPCHK(c, hipStreamWaitEvent(s, c->lv_ev[2 + buf], 0));
      // zero frontier slot 1, seen, accb (contiguous) and found / mass; slot 0
      // is written whole by every level before it is read; records are not
      // cleared (set once per (node, root), read masked by seen)
      HIPCHK(c, ospf::zero_async(a.front + (size_t)a.nb * V, (size_t)a.nb * V * 16ull * 3, s));
      HIPCHK(c, ospf::zero_async(a.found, (size_t)a.nb * lmax * 8ull, s));
      hipError_t e = ospf::launch_levels128_traverse(c->g, a, s);
      if (e != hipSuccess) return hip_fail(c, e, "launch_levels128_traverse");
      if (overlap) {
        HIPCHK(c, hipEventRecord(c->lv_ev[buf], s));
        HIPCHK(c, hipStreamWaitEvent(c->lv_aux, c->lv_ev[buf], 0));
        e = ospf::launch_levels128_rows(c->g, a, c->lv_aux);
        if (e != hipSuccess) return hip_fail(c, e, "launch_levels128_rows");
        HIPCHK(c, hipEventRecord(c->lv_ev[2 + buf], c->lv_aux));
      } else {
        e = ospf::launch_levels128_rows(c->g, a, s);
        if (e != hipSuccess) return hip_fail(c, e, "launch_levels128_rows");
      }
    }
    if (overlap) {  // the caller's stream sees every rows kernel done
      HIPCHK(c, hipEventRecord(c->lv_ev[2], c->lv_aux));
      HIPCHK(c, hipStreamWaitEvent(s, c->lv_ev[2], 0));
    }
    c->spf_runs += n;
    return OSPF_OK;
  }
  // per batch: frontier slots 2 x 8 B, seen 8 B, accb 8 B, level records 64 B
  const size_t per_vb = align_up((size_t)V * 8ull * 4 + V * 64ull + lmax * 8ull, 256);
  uint32_t nb_cap = 96;
  if (const char* e = getenv("OSPF_MS_NB")) nb_cap = std::max(1, atoi(e));
  nb_cap = (uint32_t)std::max<size_t>(1, std::min<size_t>(nb_cap, (6ull << 30) / per_vb));
  const uint32_t total_vb = (n + 63) / 64;
  const uint32_t nb_max = std::min(nb_cap, total_vb);
  int rc = OSPF_OK;
  char* sp = stream_scratch(c, s, per_vb * nb_max, &rc);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  uint32_t push_div = 8;
  if (const char* e = getenv("OSPF_MS_PUSH_DIV")) push_div = (uint32_t)std::max(0, atoi(e));
  if (dist_pitch && dist_pitch != V)
    return fail(c, OSPF_E_INVAL, "levels (OSPF_LV64): dist rows of pitch V only");
  ospf::MsArgs a{};
  a.roots = d_roots;
  a.n = n;
  a.W = 1u << 26;  // no next-hop words: every root width passes the init check
  a.npass = 1;
  a.R = 64;
  a.PP = a.OW = 1;
  a.rep = 1;
  a.lmax = lmax;
  a.dbound = c->depth_bound;
  a.kcap = 0xFFFFFFFFu;
  a.push_div = push_div;
  a.defer = 1;
  a.merged = 0;
  a.err = c->d_err;
  a.dist = d_dist;
  a.levrow = d_lev;
  a.lev_pitch = lev_pitch;
  a.digest = d_lev_digest;
  if (d_lev_digest) HIPCHK(c, ospf::zero_async(d_lev_digest, (size_t)n * sizeof(ospf_digest), s));
  for (uint32_t vb0 = 0; vb0 < total_vb; vb0 += nb_max) {
    a.vb0 = vb0;
    a.nb = std::min(nb_max, total_vb - vb0);
    a.front = (uint64_t*)sp;  // distances only: 8-B records, slots d & 1
    a.seen = a.front + 2ull * a.nb * V;
    a.accb = a.seen + (size_t)a.nb * V;
    a.planes = nullptr;
    a.lev = (uint8_t*)(a.accb + (size_t)a.nb * V);
    a.found = (uint32_t*)(a.lev + (size_t)a.nb * V * 64ull);
    a.mass = a.found + (size_t)a.nb * lmax;
    // zero: frontier slot 1 (the init kernel ORs level 1 into it; slot 0 is
    // written whole by every level before it is read), seen, accb, found /
    // mass. The level records are not cleared: their bytes are set once per
    // (node, root) and read masked by seen.
    HIPCHK(c, ospf::zero_async(a.front + (size_t)a.nb * V, (size_t)a.nb * V * 8ull * 3, s));
    HIPCHK(c, ospf::zero_async(a.found, (size_t)a.nb * lmax * 8ull, s));
    hipError_t e = ospf::launch_msbfs_levels(c->g, a, c->depth_bound, s);
    if (e != hipSuccess) return hip_fail(c, e, "launch_msbfs_levels");
  }
  c->spf_runs += n;
  return OSPF_OK;
}
}  // namespace ospf_int

extern "C" {

int ospf_nh_derive_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t nh_words,
                       uint32_t max_root_neighbors, const uint8_t* d_lev, uint32_t lev_pitch,
                       const uint32_t* d_lev_pos, const ospf_digest* d_lev_digest,
                       uint32_t* d_nh, ospf_digest* d_digest, void* stream) {
  if (!c) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (n == 0) return OSPF_OK;
  if (!d_roots || !d_lev || !d_lev_pos || !d_nh) return fail(c, OSPF_E_INVAL, "null argument");
  if (lev_pitch % 16u || lev_pitch < c->info.n_nodes)
    return fail(c, OSPF_E_INVAL, "lev_pitch: a multiple of 16 >= V");
  if (d_digest && !d_lev_digest)
    return fail(c, OSPF_E_INVAL, "derive: digests need the level rows' digests");
  if (nh_words == 0 || nh_words > 64) return fail(c, OSPF_E_RANGE, "derive: nh_words 1..64");
  const uint32_t cap = max_root_neighbors ? std::min(max_root_neighbors, 32u * nh_words)
                                          : 32u * nh_words;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(c, hipSetDevice(c->device));
  if (d_digest) HIPCHK(c, ospf::zero_async(d_digest, (size_t)n * sizeof(ospf_digest), s));
  ospf::DeriveArgs d{};
  d.roots = d_roots;
  d.n = n;
  d.W = nh_words;
  d.cap = std::min<uint32_t>(cap, 2048u);
  d.lev = d_lev;
  d.pitch = lev_pitch;
  d.pos = d_lev_pos;
  d.lev_digest = d_lev_digest;
  if (const char* e = getenv("OSPF_DERIVE_CTILES")) d.ctiles = (uint32_t)std::max(1, atoi(e));
  d.nh = d_nh;
  d.digest = d_digest;
  d.err = c->d_err;
  hipError_t e = ospf::launch_nh_derive(c->g, d, s);
  if (e != hipSuccess) return hip_fail(c, e, "launch_nh_derive");
  return OSPF_OK;
}

// Twin derive (spf_twin.hip): next-hop rows of roots whose usable transit
// neighbours fall into few twin classes (<= 16), from one representative
// level row per class.
int ospf_nh_derive_twin_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t nh_words,
                            uint32_t max_root_neighbors, const uint8_t* d_lev,
                            uint32_t lev_pitch, const uint32_t* d_lev_pos,
                            const ospf_digest* d_lev_digest, const uint32_t* d_twin_class,
                            const uint32_t* d_twin_rep, const uint32_t* d_twin_second,
                            uint32_t* d_nh, ospf_digest* d_digest, void* stream) {
  return ospf_int::nh_derive_twin_launch(c, d_roots, n, nh_words, max_root_neighbors, d_lev,
                                         lev_pitch, d_lev_pos, d_lev_digest, d_twin_class,
                                         d_twin_rep, d_twin_second, d_nh, d_digest, nullptr, stream);
}

}  // extern "C"

namespace ospf_int {
int nh_derive_twin_launch(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t nh_words,
                          uint32_t max_root_neighbors, const uint8_t* d_lev, uint32_t lev_pitch,
                          const uint32_t* d_lev_pos, const ospf_digest* d_lev_digest,
                          const uint32_t* d_twin_class, const uint32_t* d_twin_rep,
                          const uint32_t* d_twin_second, uint32_t* d_nh, ospf_digest* d_digest,
                          uint32_t* d_dist, void* stream, uint32_t dist_pitch,
                          uint32_t nh_pitch) {
  if (!c) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (n == 0) return OSPF_OK;
  if (!d_roots || !d_lev || !d_lev_pos || !d_nh || !d_twin_class || !d_twin_rep || !d_twin_second)
    return fail(c, OSPF_E_INVAL, "null argument");
  if (lev_pitch % 16u || lev_pitch < c->info.n_nodes)
    return fail(c, OSPF_E_INVAL, "lev_pitch: a multiple of 16 >= V");
  if (d_digest && !d_lev_digest)
    return fail(c, OSPF_E_INVAL, "derive: digests need the level rows' digests");
  if (nh_words == 0 || nh_words > 4) return fail(c, OSPF_E_RANGE, "twin derive: nh_words 1..4");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(c, hipSetDevice(c->device));
  if (d_digest) HIPCHK(c, ospf::zero_async(d_digest, (size_t)n * sizeof(ospf_digest), s));
  ospf::TwinArgs a{};
  a.roots = d_roots;
  a.n = n;
  a.W = nh_words;
  a.cap = max_root_neighbors ? std::min(max_root_neighbors, 32u * nh_words) : 32u * nh_words;
  a.lev = d_lev;
  a.pitch = lev_pitch;
  a.pos = d_lev_pos;
  a.lev_digest = d_lev_digest;
  a.tcls = d_twin_class;
  a.trep = d_twin_rep;
  a.tsec = d_twin_second;
  a.nh = d_nh;
  a.digest = d_digest;
  a.err = c->d_err;
  a.dist = d_dist;
  a.dpitch = dist_pitch;
  a.npitch = nh_pitch;
  // (a pitch that is not a multiple of 4 words takes the kernels' 4-B stores)
  if (nh_pitch && nh_pitch < c->info.n_nodes * nh_words)
    return fail(c, OSPF_E_INVAL, "twin derive: next-hop row pitch < V * nh_words");
  if (const char* e = getenv("OSPF_TWIN_CTILES")) a.ctiles = (uint32_t)std::max(1, atoi(e));
  hipError_t e = ospf::launch_nh_derive_twin(c->g, a, s);
  if (e != hipSuccess) return hip_fail(c, e, "launch_nh_derive_twin");
  return OSPF_OK;
}
}  // namespace ospf_int

extern "C" {

// Twin levels (spf_twin.hip): level + dist rows of roots from the
// representative rows of their neighbours' twin classes (no traversal).

// The public entry reads its (device) inputs back, plans on the host and
// waits for the launch (the sweep plans once and replays).
int ospf_twin_levels_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n,
                         const uint32_t* d_groups, uint32_t n_groups, uint8_t* d_lev,
                         uint32_t lev_pitch, const uint32_t* d_pos, const uint32_t* d_twin_class,
                         const uint32_t* d_twin_rep, uint32_t* d_dist, ospf_digest* d_lev_digest,
                         void* stream) {
  if (!c) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (n == 0) return OSPF_OK;
  if (!d_roots || !d_lev || !d_pos || !d_twin_class || !d_twin_rep)
    return fail(c, OSPF_E_INVAL, "null argument");
  if (lev_pitch % 16u || lev_pitch < c->info.n_nodes)
    return fail(c, OSPF_E_INVAL, "lev_pitch: a multiple of 16 >= V");
  if (c->depth_bound > 123) return fail(c, OSPF_E_RANGE, "level rows need a depth bound <= 123");
  if (d_groups && n_groups == 0) return fail(c, OSPF_E_INVAL, "twin levels: no groups");
  const uint32_t V = c->info.n_nodes;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(s));
  std::vector<uint32_t> roots(n), pos(V), cls(V), groups;
  HIPCHK(c, hipMemcpy(roots.data(), d_roots, n * 4ull, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(pos.data(), d_pos, V * 4ull, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(cls.data(), d_twin_class, V * 4ull, hipMemcpyDeviceToHost));
  uint32_t ncls = 0;
  for (uint32_t k : cls)
    if (k != 0xFFFFFFFFu) ncls = std::max(ncls, k + 1);
  std::vector<uint32_t> rep(ncls);
  if (ncls) HIPCHK(c, hipMemcpy(rep.data(), d_twin_rep, ncls * 4ull, hipMemcpyDeviceToHost));
  if (d_groups) {
    groups.resize(n_groups + 1);
    HIPCHK(c, hipMemcpy(groups.data(), d_groups, (n_groups + 1) * 4ull, hipMemcpyDeviceToHost));
  }
  ospf_int::TwinLvHost h;
  int rc = ospf_int::twin_lv_build(c, roots, groups, pos, cls, rep, h);
  if (rc) return rc;
  void* buf = nullptr;
  const size_t b0 = h.grp.size() * 4, b1 = h.grow.size() * 4, b2 = h.rinfo.size() * 16,
               b3 = h.nbo.size() * 4, b4 = std::max<size_t>(4, h.nbl.size() * 4);
  HIPCHK(c, dev_malloc(c, (void**)&buf, b0 + b1 + b2 + b3 + b4 + 64));
  char* p = (char*)buf;
  ospf::TwinLvPlan a{};
  a.n = n;
  a.ngroups = (uint32_t)h.grp.size() - 1;
  a.gsz = h.gmax;
  a.rinfo = (const uint4*)p;
  HIPCHK(c, hipMemcpy(p, h.rinfo.data(), b2, hipMemcpyHostToDevice));
  p += b2;
  a.grp = (const uint32_t*)p;
  HIPCHK(c, hipMemcpy(p, h.grp.data(), b0, hipMemcpyHostToDevice));
  p += b0;
  a.grow = (const uint32_t*)p;
  HIPCHK(c, hipMemcpy(p, h.grow.data(), b1, hipMemcpyHostToDevice));
  p += b1;
  a.nbo = (const uint32_t*)p;
  HIPCHK(c, hipMemcpy(p, h.nbo.data(), b3, hipMemcpyHostToDevice));
  p += b3;
  a.nbl = (const uint32_t*)p;
  if (!h.nbl.empty()) HIPCHK(c, hipMemcpy(p, h.nbl.data(), h.nbl.size() * 4, hipMemcpyHostToDevice));
  a.lev = d_lev;
  a.pitch = lev_pitch;
  a.dist = d_dist;
  a.lev_digest = d_lev_digest;
  rc = ospf_int::twin_lv_launch(c, a, s);
  const hipError_t e = hipStreamSynchronize(s);
  hipFree(buf);
  if (rc) return rc;
  if (e != hipSuccess) return hip_fail(c, e, "twin levels");
  return OSPF_OK;
}

// Leaf derive (spf_leaf.hip): level, dist and next-hop rows of leaf roots
// from their neighbours' level rows. Unit metric or hop count.
int ospf_leaf_derive_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n,
                         const uint32_t* d_groups, uint32_t n_groups, uint32_t max_root_neighbors,
                         uint8_t* d_lev, uint32_t lev_pitch, const uint32_t* d_pos,
                         uint32_t* d_dist, uint32_t* d_nh, ospf_digest* d_digest, void* stream) {
  return ospf_leaf_derive2_dev(c, d_roots, n, d_groups, n_groups, max_root_neighbors, d_lev,
                               lev_pitch, d_pos, nullptr, d_dist, d_nh, d_digest, stream);
}

int ospf_leaf_derive2_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n,
                          const uint32_t* d_groups, uint32_t n_groups,
                          uint32_t max_root_neighbors, uint8_t* d_lev, uint32_t lev_pitch,
                          const uint32_t* d_pos, const uint32_t* d_lev_out, uint32_t* d_dist,
                          uint32_t* d_nh, ospf_digest* d_digest, void* stream) {
  return ospf_int::leaf_derive(c, d_roots, n, d_groups, n_groups, max_root_neighbors, d_lev,
                               lev_pitch, d_pos, d_lev_out, d_dist, 0, d_nh, 0, d_digest, stream);
}
}  // extern "C"

namespace ospf_int {
int leaf_derive(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, const uint32_t* d_groups,
                uint32_t n_groups, uint32_t max_root_neighbors, uint8_t* d_lev,
                uint32_t lev_pitch, const uint32_t* d_pos, const uint32_t* d_lev_out,
                uint32_t* d_dist, uint32_t dist_pitch, uint32_t* d_nh, uint32_t nh_pitch,
                ospf_digest* d_digest, void* stream, int group_major) {
  if (!c) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (n == 0) return OSPF_OK;
  if (!d_roots || !d_lev || !d_pos || !d_nh) return fail(c, OSPF_E_INVAL, "null argument");
  if (lev_pitch % 16u || lev_pitch < c->info.n_nodes)
    return fail(c, OSPF_E_INVAL, "lev_pitch: a multiple of 16 >= V");
  if (d_groups && n_groups == 0) return fail(c, OSPF_E_INVAL, "leaf derive: no groups");
  if (max_root_neighbors > 32)
    return fail(c, OSPF_E_RANGE, "leaf derive: leaf roots have at most 32 distinct neighbours");
  if (c->depth_bound > 123) return fail(c, OSPF_E_RANGE, "level rows need a depth bound <= 123");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(c, hipSetDevice(c->device));
  if (d_digest) HIPCHK(c, ospf::zero_async(d_digest, (size_t)n * sizeof(ospf_digest), s));
  ospf::LeafArgs a{};
  a.roots = d_roots;
  a.n = n;
  a.grp = d_groups;
  a.ngroups = d_groups ? n_groups : n;
  a.lev = d_lev;
  a.pitch = lev_pitch;
  a.pos = d_pos;
  a.dist = d_dist;
  a.levrow = d_lev_out;
  a.nh = d_nh;
  a.digest = d_digest;
  a.err = c->d_err;
  if (const char* e = getenv("OSPF_LEAF_CTILES")) a.ctiles = (uint32_t)std::max(1, atoi(e));
  if (group_major >= 0) a.group_major = group_major ? 1u : 0u;  // the sweep's choice
  if (const char* e = getenv("OSPF_LEAF_GROUP_MAJOR")) a.group_major = atoi(e) ? 1u : 0u;
  a.dpitch = dist_pitch;
  a.npitch = nh_pitch;
  hipError_t e = ospf::launch_leaf_derive(c->g, a, max_root_neighbors ? max_root_neighbors : 32u, s);
  if (e != hipSuccess) return hip_fail(c, e, "launch_leaf_derive");
  c->spf_runs += n;
  return OSPF_OK;
}
}  // namespace ospf_int

extern "C" {

// Small-graph sweep (spf_small.hip): waves per block that fit the LDS (0 =
// the graph does not fit, or the run is outside the kernel's contract).
static uint32_t lds_sweep_waves(const ospf_ctx* c, uint32_t flags, uint32_t W) {
  if (!c->loaded || W == 0 || W > 4) return 0;
  if (!(flags & OSPF_HOP_COUNT) && !c->info.unit_metric) return 0;
  const uint32_t V = c->info.n_nodes;
  if (V == 0 || V > 65535u || c->h_prow.size() != (size_t)V + 1) return 0;
  const uint32_t Ep = c->h_prow[V];
  for (uint32_t w = 4; w >= 1; --w)
    if (ospf::small_lds_bytes(V, Ep, W, w) <= c->lds_limit) return w;
  return 0;
}

int ospf_lds_sweep_fits(const ospf_ctx* c, uint32_t flags, uint32_t nh_words) {
  return c && lds_sweep_waves(c, flags, nh_words) ? 1 : 0;
}

int ospf_lds_sweep_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                       uint32_t nh_words, uint32_t* d_dist, uint32_t* d_nh,
                       ospf_digest* d_digest, void* stream) {
  if (!c) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (n == 0) return OSPF_OK;
  if (!d_roots) return fail(c, OSPF_E_INVAL, "null roots");
  if (flags & ~(OSPF_HOP_COUNT | OSPF_WANT_DIST | OSPF_WANT_NH | OSPF_WANT_DIGEST))
    return fail(c, OSPF_E_INVAL, "lds sweep: flags");
  const uint32_t waves = lds_sweep_waves(c, flags, nh_words);
  if (!waves)
    return fail(c, OSPF_E_RANGE, "lds sweep: needs unit metric or hop count, nh_words 1..4, "
                                 "V <= 65535 and the graph in LDS");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(c, hipSetDevice(c->device));
  ospf::SmallArgs a{};
  a.roots = d_roots;
  a.n = n;
  a.Ep = c->h_prow[c->info.n_nodes];
  a.waves = waves;
  a.dist = d_dist;
  a.nh = d_nh;
  a.digest = d_digest;
  a.err = c->d_err;
  hipError_t e = ospf::launch_lds_sweep(c->g, a, nh_words, s);
  if (e != hipSuccess) return hip_fail(c, e, "launch_lds_sweep");
  c->spf_runs += n;
  return OSPF_OK;
}

// Weighted derive (spf_wderive.hip): the rows of leaf roots (<= 32 distinct
// neighbours, every transit one with a row in d_src) by Bellman's equation
// over their out-links. Any metric (or hop count); no ignored links.
int ospf_wderive_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                     uint32_t max_root_neighbors, const uint32_t* d_src, uint64_t src_pitch, const uint32_t* d_pos,
                     uint32_t* d_dist, uint32_t* d_nh, ospf_digest* d_digest, void* stream) {
  if (!c) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (n == 0) return OSPF_OK;
  if (!d_roots || !d_src || !d_pos || !d_dist) return fail(c, OSPF_E_INVAL, "null argument");
  const uint32_t V = c->info.n_nodes;
  if (src_pitch < V) return fail(c, OSPF_E_INVAL, "wderive: src_pitch >= V");
  if (!(flags & OSPF_HOP_COUNT) && c->dist_bound >= 0xFFFFFFFFull)
    return fail(c, OSPF_E_RANGE, "distances may reach 2^32 - 1");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(c, hipSetDevice(c->device));
  if (d_digest) HIPCHK(c, ospf::zero_async(d_digest, (size_t)n * sizeof(ospf_digest), s));
  ospf::WDeriveArgs a{};
  a.roots = d_roots;
  a.n = n;
  a.hop = (flags & OSPF_HOP_COUNT) ? 1u : 0u;
  a.src = d_src;
  a.src_pitch = src_pitch;
  a.pos = d_pos;
  a.dist = d_dist;
  a.nh = d_nh;
  a.digest = d_digest;
  a.err = c->d_err;
  const uintptr_t al = (uintptr_t)d_src | (uintptr_t)d_dist | (uintptr_t)d_nh;
  a.vec = (V % 4u == 0 && src_pitch % 4u == 0 && (al & 15u) == 0) ? 1u : 0u;
  if (const char* e = getenv("OSPF_WD_G")) a.G = (uint32_t)std::max(1, atoi(e));
  if (const char* e = getenv("OSPF_WD_CTILES")) a.ctiles = (uint32_t)std::max(1, atoi(e));
  // slot table width from the caller's bound (the roots' distinct neighbour
  // counts are checked on the device: a wider root raises error bit 1)
  if (max_root_neighbors > ospf::kWdMaxK)
    return fail(c, OSPF_E_RANGE, "wderive: leaf roots have at most 32 distinct neighbours");
  uint32_t kmax = max_root_neighbors ? max_root_neighbors : ospf::kWdMaxK;
  if (const char* e = getenv("OSPF_WD_KMAX")) kmax = (uint32_t)std::max(1, atoi(e));
  hipError_t e = ospf::launch_wderive(c->g, a, kmax, s);
  if (e != hipSuccess) return hip_fail(c, e, "launch_wderive");
  c->spf_runs += n;
  return OSPF_OK;
}

// Next hops of roots with up to 128 distinct neighbours (W <= 4 words) from
// their neighbours' dist rows and their own (spf_wderive.hip), any metric.
int ospf_wderive_wide_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                          uint32_t nh_words, const uint32_t* d_src, uint64_t src_pitch,
                          const uint32_t* d_pos, uint32_t* d_nh, ospf_digest* d_digest,
                          void* stream) {
  return ospf_int::wderive_wide(c, d_roots, n, flags, nh_words, d_src, src_pitch, d_pos, d_nh,
                                d_digest, stream, 0u);
}
}  // extern "C"

int ospf_int::wderive_wide(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                           uint32_t nh_words, const uint32_t* d_src, uint64_t src_pitch,
                           const uint32_t* d_pos, uint32_t* d_nh, ospf_digest* d_digest,
                           void* stream, uint32_t ctiles) {
  if (!c) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (n == 0) return OSPF_OK;
  if (!d_roots || !d_src || !d_pos || !d_nh) return fail(c, OSPF_E_INVAL, "null argument");
  const uint32_t V = c->info.n_nodes;
  if (src_pitch < V) return fail(c, OSPF_E_INVAL, "wderive: src_pitch >= V");
  if (nh_words == 0 || nh_words > 64)
    return fail(c, OSPF_E_RANGE, "wderive_wide: 1 .. 64 next-hop words (<= 2048 neighbours)");
  if (nh_words > 4 && !(flags & OSPF_HOP_COUNT) && c->info.max_metric > 0xFFFEu)
    return fail(c, OSPF_E_RANGE, "wderive_wide: metrics <= 65534 for more than 4 words");
  if (!(flags & OSPF_HOP_COUNT) && c->dist_bound >= 0xFFFFFFFFull)
    return fail(c, OSPF_E_RANGE, "distances may reach 2^32 - 1");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(c, hipSetDevice(c->device));
  if (d_digest) HIPCHK(c, ospf::zero_async(d_digest, (size_t)n * sizeof(ospf_digest), s));
  ospf::WDeriveArgs a{};
  a.roots = d_roots;
  a.n = n;
  a.hop = (flags & OSPF_HOP_COUNT) ? 1u : 0u;
  a.src = d_src;
  a.src_pitch = src_pitch;
  a.pos = d_pos;
  a.nh = d_nh;
  a.digest = d_digest;
  a.err = c->d_err;
  const uintptr_t al = (uintptr_t)d_src | (uintptr_t)d_nh;
  a.vec = (V % 4u == 0 && src_pitch % 4u == 0 && (al & 15u) == 0) ? 1u : 0u;
  a.ctiles = ctiles;
  if (const char* e = getenv("OSPF_WD_CTILES")) a.ctiles = (uint32_t)std::max(1, atoi(e));
  if (const char* e = getenv(nh_words > 4 ? "OSPF_WL_CTILES" : "OSPF_WW_CTILES"))
    a.ctiles = (uint32_t)std::max(1, atoi(e));
  if (const char* e = getenv("OSPF_WD_G")) a.G = (uint32_t)std::max(1, atoi(e));
  hipError_t e = ospf::launch_wderive_wide(c->g, a, nh_words, s);
  if (e != hipSuccess) return hip_fail(c, e, "launch_wderive_wide");
  return OSPF_OK;
}
extern "C" {

// ---------------------------------------------------------------- cover SPF
// Contracted graph for ospf_cover_dist_dev (spf_cover.hip), built on the host
// from the current (patched) shadows: cover = nodes with leaf_mask 0, each
// leaf's neighbours must all be cover nodes.
int ospf_cover_prepare(ospf_ctx* c, const uint8_t* leaf) {
  if (!c || !leaf) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  c->cover_ok = false;
  const uint32_t V = c->info.n_nodes;
  const auto& prow = c->h_prow;
  const auto& pcolx = c->h_pcolx;
  auto transit = [&](uint32_t u) { return !((c->h_nt[u >> 5] >> (u & 31)) & 1u); };
  std::vector<uint32_t> cix(V), cv;
  uint32_t nL = 0;
  for (uint32_t v = 0; v < V; ++v) {
    if (leaf[v]) {
      cix[v] = 0x80000000u | nL++;
    } else {
      cix[v] = (uint32_t)cv.size();
      cv.push_back(v);
    }
  }
  const uint32_t nS = (uint32_t)cv.size();
  if (nS == 0 || nS > ospf::kCoverMaxS)
    return fail(c, OSPF_E_RANGE, "cover: 1 .. 32768 cover nodes (LDS-resident distances)");
  std::vector<uint32_t> crow(nS + 1, 0), ctr((nS + 31) / 32, 0);
  std::vector<uint2> cedge;
  // per C edge the first hops from its source achieving its weight: the
  // head's own bit for a direct link, the leaf's for a detour (bit = the
  // position in the source's distinct neighbours): a seed root's next hops
  // start there (spf_cover.hip, seed next-hop masks)
  std::vector<uint32_t> cfh_off(1, 0u), cfh;
  std::vector<std::array<uint32_t, 3>> cand;  // {head, weight, first-hop bit}
  for (uint32_t i = 0; i < nS; ++i) {
    const uint32_t a = cv[i];
    if (transit(a)) ctr[i >> 5] |= 1u << (i & 31);
    cand.clear();
    const uint32_t* dn = c->h_dn.data() + c->h_dn_off[a];
    const uint32_t K = c->h_dn_off[a + 1] - c->h_dn_off[a];
    auto bit_of = [&](uint32_t y) { return (uint32_t)(std::lower_bound(dn, dn + K, y) - dn); };
    for (uint32_t e = prow[a]; e < prow[a + 1]; ++e) {
      const uint32_t b = pcolx[e];
      if ((b & 0x80000000u) || b == a) continue;  // down / padding / self
      const uint64_t w = c->h_pw[e];
      if (!(cix[b] & 0x80000000u)) {
        cand.push_back({cix[b], (uint32_t)w, bit_of(b)});
        continue;
      }
      if (!transit(b)) continue;  // an overloaded leaf relays nothing
      const uint32_t lb = bit_of(b);
      for (uint32_t e2 = prow[b]; e2 < prow[b + 1]; ++e2) {
        const uint32_t x = pcolx[e2];
        if ((x & 0x80000000u) || x == b || x == a) continue;
        if (cix[x] & 0x80000000u) return fail(c, OSPF_E_INVAL, "cover: two adjacent leaves");
        const uint64_t ws = w + c->h_pw[e2];
        if (ws >= 0xFFFFFFFFull) return fail(c, OSPF_E_RANGE, "cover: shortcut weight overflow");
        cand.push_back({cix[x], (uint32_t)ws, lb});
      }
    }
    std::sort(cand.begin(), cand.end());
    for (size_t k = 0; k < cand.size(); ++k) {
      const bool head = k == 0 || cand[k][0] != cand[k - 1][0];
      if (head) {
        cedge.push_back(make_uint2(cand[k][0], cand[k][1]));
        cfh_off.push_back((uint32_t)cfh.size());
      }
      // the minimum-weight entries of a head (sorted: they lead its group)
      if (cand[k][1] == cedge.back().y && (head || cand[k][2] != cand[k - 1][2]))
        cfh.push_back(cand[k][2]);
      cfh_off.back() = (uint32_t)cfh.size();
    }
    crow[i + 1] = (uint32_t)cedge.size();
  }
  // the reverse contracted graph (in-edges per node: source, weight, and the
  // edge's index for its first hops)
  std::vector<uint32_t> crin(nS + 1, 0u), ceix(cedge.size());
  std::vector<uint2> cein(cedge.size());
  for (const uint2& x : cedge) ++crin[x.x + 1];
  for (uint32_t i = 0; i < nS; ++i) crin[i + 1] += crin[i];
  {
    std::vector<uint32_t> fill(crin.begin(), crin.end() - 1);
    for (uint32_t i = 0; i < nS; ++i)
      for (uint32_t e = crow[i]; e < crow[i + 1]; ++e) {
        const uint32_t q = fill[cedge[e].x]++;
        cein[q] = make_uint2(i, cedge[e].y);
        ceix[q] = e;
      }
  }
  std::vector<uint32_t> lrow(nL + 1, 0), ladj;
  for (uint32_t v = 0, l = 0; v < V; ++v) {
    if (!leaf[v]) continue;
    for (uint32_t e = prow[v]; e < prow[v + 1]; ++e) {
      const uint32_t a = pcolx[e];
      if ((a & 0x80000000u) || a == v) continue;
      if (cix[a] & 0x80000000u) return fail(c, OSPF_E_INVAL, "cover: two adjacent leaves");
      if (c->h_prw[e] > 0xFFFFu) return fail(c, OSPF_E_RANGE, "cover: leaf in-link metric > 65535");
      ladj.push_back(cix[a] | (c->h_prw[e] << 16));
    }
    while (ladj.size() % 4) ladj.push_back(0xFFFFu);
    lrow[++l] = (uint32_t)ladj.size();
  }
  // a leaf's cix word: 0x80000000 | (its first in-link quad << 5) | quads, so
  // the kernel reaches the list in one dependent load
  for (uint32_t v = 0, l = 0; v < V; ++v) {
    if (!leaf[v]) continue;
    const uint32_t q0 = lrow[l] / 4u, nq = (lrow[l + 1] - lrow[l]) / 4u;
    if (q0 >= (1u << 26) || nq > 31u)
      return fail(c, OSPF_E_RANGE, "cover: a leaf with > 124 in-link entries");
    cix[v] = 0x80000000u | (q0 << 5) | nq;
    ++l;
  }
  c->h_ccv = cv;
  c->h_ccrow = crow;
  c->h_cctr = ctr;
  c->h_cedge = cedge;
  c->h_cix = cix;
  c->h_lrow = lrow;
  c->h_ladj = ladj;
  cover_closure_split(c);
  if (ladj.empty()) ladj.assign(4, 0xFFFFu);
  if (cedge.empty()) {
    cedge.push_back(make_uint2(0, 0));
    cein.push_back(make_uint2(0, 0));
    ceix.push_back(0);
  }
  if (cfh.empty()) cfh.push_back(0);
  // one allocation: cix | crow | ctr | lrow | ladj | cedge | cfh_off | cfh |
  // crin | cein | ceix (16-B aligned parts)
  const size_t o_cix = 0, o_crow = align_up(o_cix + V * 4ull, 16);
  const size_t o_ctr = align_up(o_crow + crow.size() * 4ull, 16);
  const size_t o_lrow = align_up(o_ctr + ctr.size() * 4ull, 16);
  const size_t o_ladj = align_up(o_lrow + lrow.size() * 4ull, 16);
  const size_t o_ced = align_up(o_ladj + ladj.size() * 4ull, 16);
  const size_t o_cfo = align_up(o_ced + cedge.size() * 8ull, 16);
  const size_t o_cfh = align_up(o_cfo + cfh_off.size() * 4ull, 16);
  const size_t o_crin = align_up(o_cfh + cfh.size() * 4ull, 16);
  const size_t o_cein = align_up(o_crin + crin.size() * 4ull, 16);
  const size_t o_ceix = align_up(o_cein + cein.size() * 8ull, 16);
  const size_t bytes = o_ceix + ceix.size() * 4ull;
  HIPCHK(c, hipSetDevice(c->device));
  if (c->d_cover) HIPCHK(c, hipFree(c->d_cover));
  c->d_cover = nullptr;
  HIPCHK(c, dev_malloc(c, &c->d_cover, bytes));
  char* base = (char*)c->d_cover;
  HIPCHK(c, hipMemcpy(base + o_cix, cix.data(), V * 4ull, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(base + o_crow, crow.data(), crow.size() * 4ull, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(base + o_ctr, ctr.data(), ctr.size() * 4ull, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(base + o_lrow, lrow.data(), lrow.size() * 4ull, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(base + o_ladj, ladj.data(), ladj.size() * 4ull, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(base + o_ced, cedge.data(), cedge.size() * 8ull, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(base + o_cfo, cfh_off.data(), cfh_off.size() * 4ull, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(base + o_cfh, cfh.data(), cfh.size() * 4ull, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(base + o_crin, crin.data(), crin.size() * 4ull, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(base + o_cein, cein.data(), cein.size() * 8ull, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(base + o_ceix, ceix.data(), ceix.size() * 4ull, hipMemcpyHostToDevice));
  ospf::CoverGraph& C = c->cover;
  C.cfh_off = (const uint32_t*)(base + o_cfo);
  C.cfh = (const uint32_t*)(base + o_cfh);
  C.crin = (const uint32_t*)(base + o_crin);
  C.cein = (const uint2*)(base + o_cein);
  C.ceix = (const uint32_t*)(base + o_ceix);
  C.nS = nS;
  C.nL = nL;
  C.cix = (const uint32_t*)(base + o_cix);
  C.crow = (const uint32_t*)(base + o_crow);
  C.ctr = (const uint32_t*)(base + o_ctr);
  C.lrow = (const uint32_t*)(base + o_lrow);
  C.ladj = (const uint32_t*)(base + o_ladj);
  C.cedge = (const uint2*)(base + o_ced);
  c->cover_ver = c->info.version;
  c->cover_ok = true;
  return OSPF_OK;
}

int ospf_cover_dist_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t* d_dist,
                        void* stream) {
  if (!c) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (!c->cover_ok || c->cover_ver != c->info.version)
    return fail(c, OSPF_E_INVAL, "cover: ospf_cover_prepare the current graph first");
  if (n == 0) return OSPF_OK;
  if (!d_roots || !d_dist) return fail(c, OSPF_E_INVAL, "null argument");
  if (c->dist_bound >= 0xFFFFFFFFull) return fail(c, OSPF_E_RANGE, "distances may reach 2^32 - 1");
  HIPCHK(c, hipSetDevice(c->device));
  ospf::CoverArgs a{};
  a.roots = d_roots;
  a.n = n;
  a.dist = d_dist;
  a.err = c->d_err;
  hipError_t e = ospf::launch_cover_spf(c->g, c->cover, a, (uint32_t)c->n_cu, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(c, e, "launch_cover_spf");
  c->spf_runs += n;
  return OSPF_OK;
}

int ospf_sssp_batch(ospf_ctx* c, const uint32_t* roots, uint32_t n_roots, const ospf_ignore* ig,
                    uint32_t flags, uint32_t nh_words, uint32_t* dist_out, uint32_t* nh_out,
                    ospf_digest* digest_out) {
  if (!c) return OSPF_E_INVAL;
  if (injected(c)) return OSPF_E_DEVICE;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (n_roots == 0) return OSPF_OK;
  if (!roots) return fail(c, OSPF_E_INVAL, "null roots");
  const uint64_t V = c->info.n_nodes;
  uint32_t max_ign = 0, max_nn = 1;
  for (uint32_t i = 0; i < n_roots; ++i) {
    if (roots[i] >= V) return fail(c, OSPF_E_INVAL, "root out of range");
    const uint32_t nn = c->h_dn_off[roots[i] + 1] - c->h_dn_off[roots[i]];
    max_nn = std::max(max_nn, nn);
    const uint32_t need = (nn + 31) / 32;
    if (need > nh_words) return fail(c, OSPF_E_INVAL, "nh_words smaller than a root needs");
    if (ig) {
      if (ig->offsets[i + 1] < ig->offsets[i]) return fail(c, OSPF_E_INVAL, "ignore offsets");
      max_ign = std::max(max_ign, ig->offsets[i + 1] - ig->offsets[i]);
    }
  }
  if (max_ign > OSPF_MAX_IGNORED_PER_RUN)
    return fail(c, OSPF_E_RANGE, "ignore list above OSPF_MAX_IGNORED_PER_RUN");
  const uint32_t n_ign = ig ? ig->offsets[n_roots] : 0;
  HIPCHK(c, hipSetDevice(c->device));

  // chunk so one chunk's device outputs stay under ~2 GiB
  const uint64_t per_root = V * 4ull * (1 + nh_words) + sizeof(ospf_digest);
  uint32_t chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_roots, (2ull << 30) / per_root));
  const size_t sz_roots = align_up(chunk * 4ull, 256), sz_off = align_up((chunk + 1) * 4ull, 256),
               sz_ids = align_up(std::max<uint32_t>(n_ign, 1) * 4ull, 256),
               sz_dist = align_up(chunk * V * 4, 256), sz_nh = align_up(chunk * V * nh_words * 4, 256),
               sz_dig = align_up(chunk * sizeof(ospf_digest), 256);
  int rc = ensure(c, &c->d_stage, &c->stage_bytes, sz_roots + sz_off + sz_ids + sz_dist + sz_nh + sz_dig);
  if (rc) return rc;
  char* s = (char*)c->d_stage;
  uint32_t* d_roots = (uint32_t*)s;
  uint32_t* d_off = (uint32_t*)(s + sz_roots);
  uint32_t* d_ids = (uint32_t*)(s + sz_roots + sz_off);
  uint32_t* d_dist = (uint32_t*)(s + sz_roots + sz_off + sz_ids);
  uint32_t* d_nh = (uint32_t*)(s + sz_roots + sz_off + sz_ids + sz_dist);
  ospf_digest* d_dig = (ospf_digest*)(s + sz_roots + sz_off + sz_ids + sz_dist + sz_nh);
  if (ig && n_ign) HIPCHK(c, hipMemcpy(d_ids, ig->link_ids, n_ign * 4ull, hipMemcpyHostToDevice));
  std::vector<uint32_t> off(chunk + 1);
  const uint32_t want = flags & (OSPF_WANT_DIST | OSPF_WANT_NH | OSPF_WANT_DIGEST);
  for (uint32_t r0 = 0; r0 < n_roots; r0 += chunk) {
    const uint32_t n = std::min(chunk, n_roots - r0);
    HIPCHK(c, hipMemcpy(d_roots, roots + r0, n * 4ull, hipMemcpyHostToDevice));
    if (ig) {
      for (uint32_t i = 0; i <= n; ++i) off[i] = ig->offsets[r0 + i];
      HIPCHK(c, hipMemcpy(d_off, off.data(), (n + 1) * 4ull, hipMemcpyHostToDevice));
    }
    ospf_batch bt{};
    bt.d_roots = d_roots;
    bt.n_roots = n;
    bt.d_ign_offsets = ig ? d_off : nullptr;
    bt.d_ign_ids = d_ids;
    bt.max_ignored = max_ign;
    bt.flags = flags;
    bt.nh_words = nh_words;
    bt.max_root_neighbors = max_nn;
    bt.d_dist = (want & OSPF_WANT_DIST) ? d_dist : nullptr;
    bt.d_nh = (want & OSPF_WANT_NH) ? d_nh : nullptr;
    bt.d_digest = (want & OSPF_WANT_DIGEST) ? d_dig : nullptr;
    rc = ospf_run_batch_dev(c, &bt, nullptr);
    if (rc) return rc;
    rc = ospf_sync(c, nullptr);
    if (rc) return rc;
    if (want & OSPF_WANT_DIST)
      HIPCHK(c, hipMemcpy(dist_out + (size_t)r0 * V, d_dist, n * V * 4, hipMemcpyDeviceToHost));
    if (want & OSPF_WANT_NH)
      HIPCHK(c, hipMemcpy(nh_out + (size_t)r0 * V * nh_words, d_nh, n * V * nh_words * 4ull,
                          hipMemcpyDeviceToHost));
    if (want & OSPF_WANT_DIGEST)
      HIPCHK(c, hipMemcpy(digest_out + r0, d_dig, n * sizeof(ospf_digest), hipMemcpyDeviceToHost));
  }
  return OSPF_OK;
}

int ospf_ksp2_dev(ospf_ctx* c, const ospf_ksp2* k, void* stream) {
  if (!c || !k) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (k->n == 0) return OSPF_OK;
  if (!k->dsts || !k->k1 || !k->k2 || !k->status) return fail(c, OSPF_E_INVAL, "null KSP2 buffer");
  if (k->src >= c->info.n_nodes) return fail(c, OSPF_E_INVAL, "src out of range");
  if (k->path_cap < 2 || k->path_cap > OSPF_MAX_IGNORED_PER_RUN)
    return fail(c, OSPF_E_INVAL, "path_cap out of range");
  const uint64_t V = c->info.n_nodes;
  if (c->dist_bound >= 0xFFFFFFFFull)
    return fail(c, OSPF_E_RANGE, "u32 distance overflow possible (sum of per-node max metrics)");
  return run_ksp2(c, k, (hipStream_t)stream);
}

int ospf_ksp2_stats(const ospf_ctx* c, uint64_t* out) {
  if (!c || !out) return OSPF_E_INVAL;
  for (int i = 0; i < 3; ++i) out[i] = c->ksp_decr_stats[i];
  return OSPF_OK;
}

int ospf_ksp2_run(ospf_ctx* c, const ospf_ksp2* k) {
  if (!c || !k) return OSPF_E_INVAL;
  if (injected(c)) return OSPF_E_DEVICE;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (k->n == 0) return OSPF_OK;
  if (!k->dsts || !k->k1 || !k->k2 || !k->status) return fail(c, OSPF_E_INVAL, "null KSP2 buffer");
  for (uint32_t i = 0; i < k->n; ++i)
    if (k->dsts[i] >= c->info.n_nodes) return fail(c, OSPF_E_INVAL, "dst out of range");
  const size_t n = k->n, rec = (size_t)k->path_cap * 4ull;
  const size_t sz_d = align_up(n * 4, 256), sz_r = align_up(n * rec, 256);
  int rc = ensure(c, &c->d_stage, &c->stage_bytes, 2 * sz_d + 2 * sz_r);
  if (rc) return rc;
  char* s = (char*)c->d_stage;
  ospf_ksp2 d = *k;
  d.dsts = (const uint32_t*)s;
  d.status = (uint32_t*)(s + sz_d);
  d.k1 = (uint32_t*)(s + 2 * sz_d);
  d.k2 = (uint32_t*)(s + 2 * sz_d + sz_r);
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMemcpy((void*)d.dsts, k->dsts, n * 4, hipMemcpyHostToDevice));
  rc = ospf_ksp2_dev(c, &d, nullptr);
  if (rc) return rc;
  rc = ospf_sync(c, nullptr);
  if (rc) return rc;
  HIPCHK(c, hipMemcpy(k->status, d.status, n * 4, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(k->k1, d.k1, n * rec, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(k->k2, d.k2, n * rec, hipMemcpyDeviceToHost));
  return OSPF_OK;
}

// ---------------------------------------------------------------- incremental
namespace {
// Planner facts after a patch. unit_metric is exact (a count of usable
// entries with metric != 1); max_metric may stay conservative (a larger
// ring / range check only); the BFS level bound is recomputed (O(V + E), host) only when a link
// went down or a node stopped being transit, the changes that can deepen it.
void refresh_graph_stats(ospf_ctx* c, uint32_t new_max, bool deeper) {
  c->info.max_metric = std::max(c->info.max_metric, new_max);
  c->info.unit_metric = c->non_unit == 0 ? 1u : 0u;
  if (deeper) {
    c->depth_bound =
        transit_depth_bound(c->info.n_nodes, c->h_prow.data(), c->h_pcolx.data(), c->h_nt);
    c->exact_bound = c->depth_bound;
  }
}

// Hops of a shortest a -> b path in the transit subgraph of the current
// shadows, or UINT32_MAX when none is found within `budget` scanned entries.
uint32_t transit_detour(ospf_ctx* c, uint32_t a, uint32_t b, size_t budget) {
  auto transit = [&](uint32_t u) { return !((c->h_nt[u >> 5] >> (u & 31)) & 1u); };
  std::vector<uint32_t>& lvl = c->h_lvl;
  if (lvl.size() != c->info.n_nodes) lvl.assign(c->info.n_nodes, 0xFFFFFFFFu);
  std::vector<uint32_t> q{a};
  lvl[a] = 0;
  uint32_t found = 0xFFFFFFFFu;
  size_t scanned = 0;
  for (size_t i = 0; i < q.size() && found == 0xFFFFFFFFu && scanned < budget; ++i) {
    const uint32_t u = q[i];
    for (uint32_t e = c->h_prow[u]; e < c->h_prow[u + 1]; ++e, ++scanned) {
      const uint32_t x = c->h_pcolx[e];
      if ((x & 0x80000000u) || !transit(x) || lvl[x] != 0xFFFFFFFFu) continue;
      lvl[x] = lvl[u] + 1;
      q.push_back(x);
      if (x == b) {
        found = lvl[x];
        break;
      }
    }
  }
  for (uint32_t x : q) lvl[x] = 0xFFFFFFFFu;
  return found;
}
}  // namespace

int ospf_update_links(ospf_ctx* c, const ospf_link_update* u, uint32_t n, uint64_t version) {
  if (!c || (n && !u)) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  std::vector<uint32_t> idx, val;
  idx.reserve(6ull * n);
  val.reserve(6ull * n);
  uint32_t* base = (uint32_t*)c->d_graph;
  const size_t o_colx = c->g.colx - (const uint32_t*)base, o_w = c->g.w - (const uint32_t*)base,
               o_rw = c->g.rw - (const uint32_t*)base;
  auto owner = [&](uint32_t e) {
    return (uint32_t)(std::upper_bound(c->h_prow.begin(), c->h_prow.end(), e) - c->h_prow.begin() - 1);
  };
  auto set = [&](std::vector<uint32_t>& shadow, size_t off, uint32_t e, uint32_t v) {
    shadow[e] = v;
    idx.push_back((uint32_t)(off + e));
    val.push_back(v);
  };
  // validate every update before touching any state: a rejected batch leaves
  // the host shadows, the planner counters and the device graph as they were
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t lid = u[i].link_id;
    if (lid >= c->g.n_lid) return fail(c, OSPF_E_INVAL, "unknown link id");
    if (c->h_link_e[2ull * lid] == 0xFFFFFFFFu || c->h_link_e[2ull * lid + 1] == 0xFFFFFFFFu)
      return fail(c, OSPF_E_INVAL, "unknown link id");
    if (u[i].up && (u[i].metric_lo == 0 || u[i].metric_hi == 0))
      return fail(c, OSPF_E_RANGE, "metric 0 on a usable link is outside the engine contract");
  }
  uint32_t new_max = 0;
  bool ups = false;  // a link came up: components may join, the level bound may grow
  std::vector<std::pair<uint32_t, uint32_t>> downs;  // links that went down (ends)
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t lid = u[i].link_id;
    const uint32_t e0 = c->h_link_e[2ull * lid], e1 = c->h_link_e[2ull * lid + 1];
    const bool lo0 = owner(e0) <= owner(e1);
    const uint32_t elo = lo0 ? e0 : e1, ehi = lo0 ? e1 : e0;
    const uint32_t down = u[i].up ? 0u : 0x80000000u;
    if (!u[i].up && !(c->h_pcolx[elo] & 0x80000000u)) downs.push_back({owner(elo), owner(ehi)});
    if (u[i].up && (c->h_pcolx[elo] & 0x80000000u)) ups = true;
    if (u[i].up) new_max = std::max({new_max, u[i].metric_lo, u[i].metric_hi});
    for (uint32_t e : {elo, ehi}) {  // usable non-unit entries, before -> after
      if (!(c->h_pcolx[e] & 0x80000000u) && c->h_pw[e] != 1) --c->non_unit;
      const uint32_t m = e == elo ? u[i].metric_lo : u[i].metric_hi;
      if (u[i].up && m != 1) ++c->non_unit;
    }
    set(c->h_pcolx, o_colx, elo, (c->h_pcolx[elo] & 0x7FFFFFFFu) | down);
    set(c->h_pcolx, o_colx, ehi, (c->h_pcolx[ehi] & 0x7FFFFFFFu) | down);
    set(c->h_pw, o_w, elo, u[i].metric_lo);
    set(c->h_pw, o_w, ehi, u[i].metric_hi);
    set(c->h_prw, o_rw, elo, u[i].metric_hi);
    set(c->h_prw, o_rw, ehi, u[i].metric_lo);
    if (c->g.ew) {  // packed entries: same change, or dropped past 16-bit metrics
      if (u[i].metric_lo > 0xFFFFu || u[i].metric_hi > 0xFFFFu) {
        c->g.ew = nullptr;
      } else {
        const size_t o_ew = c->ew_base - (const uint32_t*)base;
        for (uint32_t e : {elo, ehi}) {
          idx.push_back((uint32_t)(o_ew + 2ull * e));
          val.push_back(c->h_pcolx[e]);
          idx.push_back((uint32_t)(o_ew + 2ull * e + 1));
          val.push_back(c->h_pw[e] | (c->h_prw[e] << 16));
        }
      }
    }
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipDeviceSynchronize());  // no batch may be reading the graph
  if (!idx.empty()) {
    int rc = ensure(c, &c->d_stage, &c->stage_bytes, idx.size() * 8ull + 256);
    if (rc) return rc;
    uint32_t* d_idx = (uint32_t*)c->d_stage;
    uint32_t* d_val = d_idx + idx.size();
    HIPCHK(c, hipMemcpy(d_idx, idx.data(), idx.size() * 4ull, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(d_val, val.data(), val.size() * 4ull, hipMemcpyHostToDevice));
    hipError_t e = ospf::launch_scatter(base, d_idx, d_val, (uint32_t)idx.size(), nullptr);
    if (e != hipSuccess) return hip_fail(c, e, "launch_scatter");
    HIPCHK(c, hipDeviceSynchronize());
  }
  // Level bound after links went down. A shortest path uses a removed link at
  // most once, so replacing each removed link (a, b) of the transit subgraph
  // by a shortest a -> b detour of k hops in the patched graph lengthens any
  // distance by at most sum(k - 1): bound += sum(k - 1), found by a budgeted
  // local BFS instead of the O(V + E) recomputation. A link with an
  // overloaded end is not in the transit subgraph (only the first / last hop
  // of a path, covered by the + 2 of the bound). No detour within the budget
  // (a split component), or drift of more than 8 levels over the last exact
  // bound, recomputes it. A link coming up can join two components of the
  // transit subgraph (an eccentricity the old bound never saw): recompute.
  bool deeper = ups;
  uint32_t grow = 0;
  auto transit = [&](uint32_t x) { return !((c->h_nt[x >> 5] >> (x & 31)) & 1u); };
  for (const auto& ab : downs) {
    if (deeper) break;
    if (!transit(ab.first) || !transit(ab.second)) continue;
    const uint32_t k = transit_detour(c, ab.first, ab.second, 1u << 20);
    if (k == 0xFFFFFFFFu) deeper = true;
    else grow += k - 1;
  }
  if (!deeper && grow) {
    if (c->depth_bound + grow > c->exact_bound + 8) deeper = true;
    else c->depth_bound += grow;
  }
  refresh_graph_stats(c, new_max, deeper);
  // distance bound = sum of per-node largest usable out-metrics, kept exact
  // (a patch that restores a metric does not ratchet it up)
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t lid = u[i].link_id;
    for (int k = 0; k < 2; ++k) {
      const uint32_t x = owner(c->h_link_e[2ull * lid + k]);
      uint32_t m = 0;
      for (uint32_t e = c->h_prow[x]; e < c->h_prow[x + 1]; ++e)
        if (!(c->h_pcolx[e] & 0x80000000u)) m = std::max(m, c->h_pw[e]);
      c->dist_bound = c->dist_bound - c->h_rowmax[x] + m;
      c->h_rowmax[x] = m;
    }
  }
  c->info.version = version;
  c->cover_ok = false;  // the contracted cover graph describes the old graph
  ++c->graph_gen;
  return OSPF_OK;
}

// Take links down for a while (KSP2 ignore sets beyond one run's list) and
// put back exactly what was there: entries and the planner state (level /
// distance bounds, metric facts, cover graph), so a mask / unmask pair leaves
// no trace in later runs.
int ospf_links_mask(ospf_ctx* c, const uint32_t* lids, uint32_t n, uint64_t version) {
  if (!c || (n && !lids)) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (c->mask.on) return fail(c, OSPF_E_INVAL, "links already masked (unmask first)");
  ospf_ctx::Mask m{};
  m.depth_bound = c->depth_bound;
  m.exact_bound = c->exact_bound;
  m.max_metric = c->info.max_metric;
  m.unit_metric = c->info.unit_metric;
  m.dist_bound = c->dist_bound;
  m.non_unit = c->non_unit;
  m.version = c->info.version;
  m.cover_ok = c->cover_ok;
  std::vector<ospf_link_update> down(n);
  auto owner = [&](uint32_t e) {
    return (uint32_t)(std::upper_bound(c->h_prow.begin(), c->h_prow.end(), e) - c->h_prow.begin() - 1);
  };
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t lid = lids[i];
    if (lid >= c->g.n_lid || c->h_link_e[2ull * lid] == 0xFFFFFFFFu ||
        c->h_link_e[2ull * lid + 1] == 0xFFFFFFFFu)
      return fail(c, OSPF_E_INVAL, "unknown link id");
    const uint32_t e0 = c->h_link_e[2ull * lid], e1 = c->h_link_e[2ull * lid + 1];
    const bool lo0 = owner(e0) <= owner(e1);
    const uint32_t elo = lo0 ? e0 : e1, ehi = lo0 ? e1 : e0;
    m.lids.push_back(lid);
    m.up.push_back((c->h_pcolx[elo] & 0x80000000u) ? 0u : 1u);
    m.mlo.push_back(c->h_pw[elo]);
    m.mhi.push_back(c->h_pw[ehi]);
    down[i] = ospf_link_update{lid, 0u, c->h_pw[elo], c->h_pw[ehi]};
  }
  const int rc = ospf_update_links(c, down.data(), n, version);
  if (rc != OSPF_OK) return rc;
  m.on = true;
  c->mask = std::move(m);
  return OSPF_OK;
}

int ospf_links_unmask(ospf_ctx* c) {
  if (!c) return OSPF_E_INVAL;
  if (!c->mask.on) return OSPF_OK;
  ospf_ctx::Mask m = std::move(c->mask);
  c->mask = ospf_ctx::Mask{};
  std::vector<ospf_link_update> back(m.lids.size());
  for (size_t i = 0; i < m.lids.size(); ++i)
    back[i] = ospf_link_update{m.lids[i], m.up[i], m.mlo[i], m.mhi[i]};
  // metric 0 never appears on an up link of a loaded graph, so the restore
  // passes ospf_update_links' checks
  const int rc = ospf_update_links(c, back.data(), (uint32_t)back.size(), m.version);
  if (rc != OSPF_OK) return rc;
  c->depth_bound = m.depth_bound;
  c->exact_bound = m.exact_bound;
  c->info.max_metric = m.max_metric;
  c->info.unit_metric = m.unit_metric;
  c->dist_bound = m.dist_bound;
  c->non_unit = m.non_unit;
  c->cover_ok = m.cover_ok;
  return OSPF_OK;
}

int ospf_update_nodes(ospf_ctx* c, const uint32_t* nodes, const uint8_t* no_transit, uint32_t n,
                      uint64_t version) {
  if (!c || (n && (!nodes || !no_transit))) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  for (uint32_t i = 0; i < n; ++i)
    if (nodes[i] >= c->info.n_nodes) return fail(c, OSPF_E_INVAL, "node out of range");
  bool deeper = false;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t v = nodes[i];
    // either direction can deepen the level bound: an overloaded node splits
    // transit paths, a node that becomes transit can join two components
    if ((no_transit[i] != 0) != (((c->h_nt[v >> 5] >> (v & 31u)) & 1u) != 0)) deeper = true;
    if (no_transit[i]) c->h_nt[v >> 5] |= 1u << (v & 31u);
    else c->h_nt[v >> 5] &= ~(1u << (v & 31u));
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipDeviceSynchronize());
  HIPCHK(c, hipMemcpy((void*)c->g.nt_bits, c->h_nt.data(), c->h_nt.size() * 4ull,
                      hipMemcpyHostToDevice));
  refresh_graph_stats(c, 0, deeper);
  c->info.version = version;
  c->cover_ok = false;  // the contracted cover graph describes the old graph
  ++c->graph_gen;
  return OSPF_OK;
}

// Structural patch (include/openr_spf.h). Validation first -- a rejected
// call leaves the context as it was -- then, with the device idle: rows that
// outgrow their padded slots move the tail of every per-entry array (device
// copies through the stage buffer, host shadows by insertion, row offsets and
// link positions shifted), the rebuilt rows are written into their slots
// (one scatter launch for every changed word), the distinct-neighbour lists
// and the planner facts follow.
int ospf_update_rows(ospf_ctx* c, const ospf_csr* csr, const uint32_t* rows, uint32_t n,
                     uint64_t version) {
  if (!c || !csr || (n && !rows)) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  if (c->mask.on) return fail(c, OSPF_E_INVAL, "update_rows: links are masked (ospf_links_unmask)");
  const uint32_t V = c->info.n_nodes;
  if (csr->n_nodes != V) return fail(c, OSPF_E_RANGE, "update_rows: the node count changed (reload)");
  const uint32_t E = csr->n_edges;
  if (!csr->row_ptr || (E && (!csr->col || !csr->metric || !csr->link_id || !csr->twin ||
                              !csr->edge_up)))
    return fail(c, OSPF_E_INVAL, "null CSR array");
  if (csr->row_ptr[0] != 0 || csr->row_ptr[V] != E)
    return fail(c, OSPF_E_INVAL, "row_ptr must start at 0 and end at n_edges");
  constexpr uint32_t kNo = 0xFFFFFFFFu;
  const uint32_t* rp = csr->row_ptr;
  auto row_ok = [&](uint32_t u) { return rp[u] <= rp[u + 1] && rp[u + 1] <= E; };
  // rows to rebuild: the given ones, and every neighbour holding parallel
  // links to one of them (their order follows the given row's link ranks)
  std::vector<uint32_t> R;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t u = rows[i];
    if (u >= V) return fail(c, OSPF_E_INVAL, "update_rows: row out of range");
    if (!row_ok(u)) return fail(c, OSPF_E_INVAL, "row_ptr not monotone");
    R.push_back(u);
    for (uint32_t e = rp[u] + 1; e < rp[u + 1]; ++e)
      if (csr->col[e] == csr->col[e - 1] && csr->col[e] != u && csr->col[e] < V) R.push_back(csr->col[e]);
  }
  std::sort(R.begin(), R.end());
  R.erase(std::unique(R.begin(), R.end()), R.end());
  struct Row {
    uint32_t u, cap0, len, need, grow;
    std::vector<uint32_t> colx, w, rw, lid, dn;
    std::vector<uint16_t> didx;
  };
  std::vector<Row> nr(R.size());
  std::vector<uint8_t> inR(V, 0);
  for (uint32_t u : R) inR[u] = 1;
  std::vector<uint32_t> ord;
  uint32_t new_max = 0, max_deg = c->info.max_degree, max_dn = c->max_dn;
  size_t grow_tot = 0, dn_tot = c->h_dn.size();
  std::vector<uint32_t> old_lids, new_lids;
  for (size_t k = 0; k < R.size(); ++k) {
    const uint32_t u = R[k], b = rp[u], len = rp[u + 1] - b;
    if (!row_ok(u)) return fail(c, OSPF_E_INVAL, "row_ptr not monotone");
    Row& x = nr[k];
    x.u = u;
    x.len = len;
    x.cap0 = c->h_prow[u + 1] - c->h_prow[u];
    x.need = (len + 3u) & ~3u;
    x.grow = x.need > x.cap0 ? ((x.need - x.cap0 + 3u) & ~3u) + 8u : 0u;
    grow_tot += x.grow;
    max_deg = std::max(max_deg, len);
    ord.resize(len);
    for (uint32_t j = 0; j < len; ++j) {
      const uint32_t e = b + j, v = csr->col[e], t = csr->twin[e];
      if (v >= V) return fail(c, OSPF_E_INVAL, "col out of range");
      if (j && csr->col[e - 1] > v) return fail(c, OSPF_E_INVAL, "rows must be sorted by col");
      if (t >= E || csr->twin[t] != e || csr->col[t] != u || !row_ok(v) || t < rp[v] ||
          t >= rp[v + 1] || csr->link_id[t] != csr->link_id[e])
        return fail(c, OSPF_E_INVAL, "twin/link_id inconsistent");
      if (csr->edge_up[e] != csr->edge_up[t])
        return fail(c, OSPF_E_INVAL, "edge_up must match on both directions of a link");
      if (csr->edge_up[e] && (csr->metric[e] == 0 || csr->metric[t] == 0))
        return fail(c, OSPF_E_RANGE, "metric 0 on a usable link is outside the engine contract");
      if (csr->link_id[e] >= c->cap_lid)
        return fail(c, OSPF_E_RANGE, "update_rows: link id past the reserve (reload)");
      ord[j] = e;
    }
    if (csr->link_rank)
      std::stable_sort(ord.begin(), ord.end(), [&](uint32_t p, uint32_t q) {
        if (csr->col[p] != csr->col[q]) return csr->col[p] < csr->col[q];
        return csr->link_rank[csr->twin[p]] < csr->link_rank[csr->twin[q]];
      });
    x.colx.assign(x.need, 0x80000000u);
    x.w.assign(x.need, 0u);
    x.rw.assign(x.need, 0u);
    x.lid.assign(x.need, kNo);
    x.didx.assign(x.need, 0xFFFFu);
    uint32_t kk = 0, prev = kNo;
    for (uint32_t j = 0; j < len; ++j) {
      const uint32_t e = ord[j], v = csr->col[e];
      const bool up = csr->edge_up[e] != 0;
      x.colx[j] = v | (up ? 0u : 0x80000000u);
      x.w[j] = csr->metric[e];
      x.rw[j] = csr->metric[csr->twin[e]];
      x.lid[j] = csr->link_id[e];
      new_lids.push_back(x.lid[j]);
      if (up) new_max = std::max(new_max, x.w[j]);
      if (v == u) continue;  // self-loop: no next-hop bit
      if (prev != kNo && v != prev) ++kk;
      if (v != prev) x.dn.push_back(v);
      prev = v;
      x.didx[j] = (uint16_t)kk;
    }
    if (x.dn.size() > OSPF_MAX_ROOT_NEIGHBORS)
      return fail(c, OSPF_E_RANGE, "a node has more distinct neighbours than OSPF_MAX_ROOT_NEIGHBORS");
    max_dn = std::max<uint32_t>(max_dn, (uint32_t)x.dn.size());
    dn_tot += x.dn.size() - (c->h_dn_off[u + 1] - c->h_dn_off[u]);
    for (uint32_t e = c->h_prow[u]; e < c->h_prow[u + 1]; ++e)
      if (c->h_plink[e] != kNo) old_lids.push_back(c->h_plink[e]);
  }
  const size_t Ep0 = c->h_prow[V];
  if (Ep0 + grow_tot > c->cap_e)
    return fail(c, OSPF_E_RANGE, "update_rows: entry reserve exhausted (reload)");
  if (dn_tot > c->cap_dn) return fail(c, OSPF_E_RANGE, "update_rows: neighbour reserve exhausted (reload)");
  std::sort(old_lids.begin(), old_lids.end());
  std::sort(new_lids.begin(), new_lids.end());
  // a link id new to these rows must be free (retired) before the call
  for (size_t i = 0; i < new_lids.size(); ++i) {
    const uint32_t l = new_lids[i];
    if (i && new_lids[i - 1] == l) continue;
    if (std::binary_search(old_lids.begin(), old_lids.end(), l)) continue;
    if (l < c->g.n_lid && (c->h_link_e[2ull * l] != kNo || c->h_link_e[2ull * l + 1] != kNo))
      return fail(c, OSPF_E_INVAL, "update_rows: an added link's id is still in use");
  }
  // transit connectivity the rows gain or lose (level bound, below): a pair
  // joined by a usable link after but not before, both ends transit, keeps
  // the bound only when the old graph already connects it
  auto transit = [&](uint32_t x) { return !((c->h_nt[x >> 5] >> (x & 31)) & 1u); };
  bool deeper = false;
  std::vector<std::pair<uint32_t, uint32_t>> lost;
  for (const Row& x : nr) {
    if (!transit(x.u)) continue;
    std::vector<uint32_t> before, after;
    for (uint32_t e = c->h_prow[x.u]; e < c->h_prow[x.u + 1]; ++e)
      if (!(c->h_pcolx[e] & 0x80000000u) && transit(c->h_pcolx[e])) before.push_back(c->h_pcolx[e]);
    for (uint32_t j = 0; j < x.len; ++j)
      if (!(x.colx[j] & 0x80000000u) && transit(x.colx[j])) after.push_back(x.colx[j]);
    std::sort(before.begin(), before.end());
    before.erase(std::unique(before.begin(), before.end()), before.end());
    std::sort(after.begin(), after.end());
    after.erase(std::unique(after.begin(), after.end()), after.end());
    for (uint32_t v : after)
      if (v > x.u && !std::binary_search(before.begin(), before.end(), v) && !deeper)
        deeper = transit_detour(c, x.u, v, 1u << 20) == kNo;
    for (uint32_t v : before)
      if (v > x.u && !std::binary_search(after.begin(), after.end(), v)) lost.push_back({x.u, v});
  }

  // ---- commit
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipDeviceSynchronize());  // no batch may be reading the graph
  if (!new_lids.empty() && 2ull * (new_lids.back() + 1) > c->h_link_e.size())
    c->h_link_e.resize(2ull * (new_lids.back() + 1), kNo);  // ids past the last one in use
  uint32_t* base = (uint32_t*)c->d_graph;
  auto woff = [&](const void* p) { return (size_t)((const char*)p - (const char*)base) / 4; };
  // positions of the old lids inside rebuilt rows leave link_e (the other
  // end's position stays when that row is not rebuilt)
  std::vector<uint32_t> touched;  // link ids whose link_e words change
  for (const Row& x : nr)
    for (uint32_t e = c->h_prow[x.u]; e < c->h_prow[x.u + 1]; ++e) {
      const uint32_t l = c->h_plink[e];
      if (l == kNo) continue;
      for (int s = 0; s < 2; ++s)
        if (c->h_link_e[2ull * l + s] == e) c->h_link_e[2ull * l + s] = kNo;
      touched.push_back(l);
    }
  // grow rows (last first: earlier positions stay put)
  std::vector<size_t> grow_ix;
  for (size_t k = 0; k < nr.size(); ++k)
    if (nr[k].grow) grow_ix.push_back(k);
  struct Arr {
    char* p;
    size_t esz;
  };
  std::vector<Arr> arrs = {{(char*)c->g.colx, 4}, {(char*)c->g.w, 4}, {(char*)c->g.rw, 4},
                           {(char*)c->g.link_id, 4}, {(char*)c->g.didx, 2}};
  if (c->g.ew) arrs.push_back({(char*)c->ew_base, 8});
  size_t Ep = Ep0;
  for (auto it = grow_ix.rbegin(); it != grow_ix.rend(); ++it) {
    const Row& x = nr[*it];
    const uint32_t pos = c->h_prow[x.u + 1], d = x.grow;
    const size_t tail = Ep - pos;
    if (tail) {
      int rc = ensure(c, &c->d_stage, &c->stage_bytes, tail * 8);
      if (rc) return rc;
      for (const Arr& a : arrs) {
        HIPCHK(c, hipMemcpy(c->d_stage, a.p + pos * a.esz, tail * a.esz, hipMemcpyDeviceToDevice));
        HIPCHK(c, hipMemcpy(a.p + ((size_t)pos + d) * a.esz, c->d_stage, tail * a.esz,
                            hipMemcpyDeviceToDevice));
      }
    }
    c->h_pcolx.insert(c->h_pcolx.begin() + pos, d, 0x80000000u);
    c->h_pw.insert(c->h_pw.begin() + pos, d, 0u);
    c->h_prw.insert(c->h_prw.begin() + pos, d, 0u);
    c->h_plink.insert(c->h_plink.begin() + pos, d, kNo);
    for (uint32_t v = x.u + 1; v <= V; ++v) c->h_prow[v] += d;
    for (auto& p : c->h_link_e)
      if (p != kNo && p >= pos) p += d;
    hipError_t he = ospf::launch_shift_add(base + woff(c->g.row_ptr), V + 1, x.u + 1, 0u, d, nullptr);
    if (he == hipSuccess && c->g.n_lid)
      he = ospf::launch_shift_add(base + woff(c->g.link_e), 2 * c->g.n_lid, 0u, pos, d, nullptr);
    if (he != hipSuccess) return hip_fail(c, he, "launch_shift_add");
    Ep += d;
  }
  // rebuilt rows into their slots; every changed word through one scatter
  std::vector<uint32_t> idx, val;
  auto put = [&](size_t word, uint32_t v) {
    idx.push_back((uint32_t)word);
    val.push_back(v);
  };
  const size_t o_colx = woff(c->g.colx), o_w = woff(c->g.w), o_rw = woff(c->g.rw),
               o_lid = woff(c->g.link_id), o_didx = woff(c->g.didx), o_ew = woff(c->ew_base),
               o_le = woff(c->g.link_e);
  uint32_t lid_max = c->g.n_lid;
  bool big_change = false;
  for (Row& x : nr) {
    const uint32_t b = c->h_prow[x.u], cap = c->h_prow[x.u + 1] - b;
    big_change |= (x.cap0 > ospf::kMsBigDeg) != (cap > ospf::kMsBigDeg);
    uint32_t m = 0;
    for (uint32_t j = 0; j < cap; ++j) {
      const size_t e = (size_t)b + j;
      const bool inrow = j < x.need;
      const uint32_t cx = inrow ? x.colx[j] : 0x80000000u, w = inrow ? x.w[j] : 0u,
                     rw = inrow ? x.rw[j] : 0u, l = inrow ? x.lid[j] : kNo;
      if (!(c->h_pcolx[e] & 0x80000000u) && c->h_pw[e] != 1) --c->non_unit;
      if (!(cx & 0x80000000u) && w != 1) ++c->non_unit;
      if (!(cx & 0x80000000u)) m = std::max(m, w);
      c->h_pcolx[e] = cx;
      c->h_pw[e] = w;
      c->h_prw[e] = rw;
      c->h_plink[e] = l;
      put(o_colx + e, cx);
      put(o_w + e, w);
      put(o_rw + e, rw);
      put(o_lid + e, l);
      if (c->g.ew) {
        if (w > 0xFFFFu || rw > 0xFFFFu) {
          c->g.ew = nullptr;
        } else {
          put(o_ew + 2 * e, cx);
          put(o_ew + 2 * e + 1, w | (rw << 16));
        }
      }
      if (l != kNo) {
        uint32_t* le = &c->h_link_e[2ull * l];
        (le[0] == kNo ? le[0] : le[1]) = (uint32_t)e;
        touched.push_back(l);
        lid_max = std::max(lid_max, l + 1);
      }
    }
    for (uint32_t j = 0; j < cap; j += 2) {  // didx: two u16 per word (rows start 8-B aligned)
      const uint32_t lo = j < x.need ? x.didx[j] : 0xFFFFu, hi = j + 1 < x.need ? x.didx[j + 1] : 0xFFFFu;
      put(o_didx + ((size_t)b + j) / 2, lo | (hi << 16));
    }
    c->dist_bound = c->dist_bound - c->h_rowmax[x.u] + m;
    c->h_rowmax[x.u] = m;
  }
  c->g.n_lid = lid_max;
  std::sort(touched.begin(), touched.end());
  touched.erase(std::unique(touched.begin(), touched.end()), touched.end());
  for (uint32_t l : touched) {
    put(o_le + 2ull * l, c->h_link_e[2ull * l]);
    put(o_le + 2ull * l + 1, c->h_link_e[2ull * l + 1]);
  }
  // distinct neighbours: a row whose count changes moves the lists after it
  // (last first, like the entry arrays; dn_off shifted on both sides), then
  // every rebuilt row's list is written in place
  const size_t o_dn = woff(c->g.dn);
  for (auto it = nr.rbegin(); it != nr.rend(); ++it) {
    const Row& x = *it;
    const uint32_t lo = c->h_dn_off[x.u], hi = c->h_dn_off[x.u + 1];
    const int64_t delta = (int64_t)x.dn.size() - (int64_t)(hi - lo);
    if (!delta) continue;
    const size_t tail = c->h_dn.size() - hi;
    if (tail) {
      int rc = ensure(c, &c->d_stage, &c->stage_bytes, tail * 4);
      if (rc) return rc;
      HIPCHK(c, hipMemcpy(c->d_stage, c->g.dn + hi, tail * 4, hipMemcpyDeviceToDevice));
      HIPCHK(c, hipMemcpy((void*)(c->g.dn + (int64_t)hi + delta), c->d_stage, tail * 4,
                          hipMemcpyDeviceToDevice));
    }
    if (delta > 0) c->h_dn.insert(c->h_dn.begin() + hi, (size_t)delta, 0u);
    else c->h_dn.erase(c->h_dn.begin() + ((int64_t)hi + delta), c->h_dn.begin() + hi);
    for (uint32_t v = x.u + 1; v <= V; ++v) c->h_dn_off[v] += (uint32_t)delta;
    hipError_t he = ospf::launch_shift_add(base + woff(c->g.dn_off), V + 1, x.u + 1, 0u,
                                           (uint32_t)delta, nullptr);
    if (he != hipSuccess) return hip_fail(c, he, "launch_shift_add");
  }
  for (const Row& x : nr)
    for (size_t k = 0; k < x.dn.size(); ++k) {
      c->h_dn[c->h_dn_off[x.u] + k] = x.dn[k];
      put(o_dn + c->h_dn_off[x.u] + k, x.dn[k]);
    }
  if (!idx.empty()) {
    int rc = ensure(c, &c->d_stage, &c->stage_bytes, idx.size() * 8ull + 256);
    if (rc) return rc;
    uint32_t* d_idx = (uint32_t*)c->d_stage;
    uint32_t* d_val = d_idx + idx.size();
    HIPCHK(c, hipMemcpy(d_idx, idx.data(), idx.size() * 4ull, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(d_val, val.data(), val.size() * 4ull, hipMemcpyHostToDevice));
    hipError_t e = ospf::launch_scatter(base, d_idx, d_val, (uint32_t)idx.size(), nullptr);
    if (e != hipSuccess) return hip_fail(c, e, "launch_scatter");
  }
  if (big_change) {
    std::vector<uint32_t> big;
    for (uint32_t u = 0; u < V; ++u)
      if (c->h_prow[u + 1] - c->h_prow[u] > ospf::kMsBigDeg) big.push_back(u);
    if (!big.empty())
      HIPCHK(c, hipMemcpy((void*)c->g.big, big.data(), big.size() * 4ull, hipMemcpyHostToDevice));
    c->g.nbig = (uint32_t)big.size();
  }
  HIPCHK(c, hipDeviceSynchronize());
  c->g.E = (uint32_t)Ep;
  c->max_dn = max_dn;
  c->h_row_ptr.assign(rp, rp + V + 1);
  c->info.n_edges = E;
  c->info.n_links = E / 2;
  c->info.max_degree = max_deg;
  // level bound after transit links were lost: the detour rule of
  // ospf_update_links (a split component recomputes it)
  uint32_t grow = 0;
  for (const auto& ab : lost) {
    if (deeper) break;
    const uint32_t k = transit_detour(c, ab.first, ab.second, 1u << 20);
    if (k == kNo) deeper = true;
    else grow += k - 1;
  }
  if (!deeper && grow) {
    if (c->depth_bound + grow > c->exact_bound + 8) deeper = true;
    else c->depth_bound += grow;
  }
  refresh_graph_stats(c, new_max, deeper);
  c->info.version = version;
  c->cover_ok = false;  // the contracted cover graph describes the old graph
  ++c->graph_gen;
  return OSPF_OK;
}

int ospf_affected_roots(ospf_ctx* c, const uint32_t* d_dist, uint32_t n_roots, uint32_t flags,
                        const ospf_change* ch, uint32_t n_ch, uint8_t* d_affected, void* stream) {
  if (!c || (n_roots && (!d_dist || !d_affected)) || (n_ch && !ch)) return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  for (uint32_t k = 0; k < n_ch; ++k)
    if (ch[k].a >= c->info.n_nodes || (ch[k].kind == OSPF_CHANGE_LINK && ch[k].b >= c->info.n_nodes))
      return fail(c, OSPF_E_INVAL, "change names a node out of range");
  if (n_roots == 0) return OSPF_OK;
  HIPCHK(c, hipSetDevice(c->device));
  int rc = OSPF_OK;
  ospf_change* d_ch =
      (ospf_change*)stream_scratch(c, stream, std::max<size_t>(n_ch, 1) * sizeof(ospf_change), &rc, 2);
  if (rc) return rc;
  if (n_ch)
    HIPCHK(c, hipMemcpyAsync(d_ch, ch, n_ch * sizeof(ospf_change), hipMemcpyHostToDevice,
                             (hipStream_t)stream));
  hipError_t e = ospf::launch_affected(c->g, d_dist, n_roots, (flags & OSPF_HOP_COUNT) != 0, d_ch,
                                       n_ch, d_affected, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(c, e, "launch_affected");
  return OSPF_OK;
}

int ospf_repair_runs(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                     uint32_t nh_words, uint32_t* d_dist, uint32_t* d_nh, const ospf_change* ch,
                     uint32_t n_ch, uint32_t* d_status, void* stream) {
  if (!c || (n && (!d_roots || !d_dist || !d_nh || !d_status)) || (n_ch && !ch) || !nh_words)
    return OSPF_E_INVAL;
  if (!c->loaded) return fail(c, OSPF_E_NOGRAPH, "no graph loaded");
  for (uint32_t k = 0; k < n_ch; ++k)
    if (ch[k].a >= c->info.n_nodes || (ch[k].kind == OSPF_CHANGE_LINK && ch[k].b >= c->info.n_nodes))
      return fail(c, OSPF_E_INVAL, "change names a node out of range");
  if (n == 0) return OSPF_OK;
  HIPCHK(c, hipSetDevice(c->device));
  int rc = OSPF_OK;
  ospf_change* d_ch =
      (ospf_change*)stream_scratch(c, stream, std::max<size_t>(n_ch, 1) * sizeof(ospf_change), &rc, 2);
  if (rc) return rc;
  if (n_ch)
    HIPCHK(c, hipMemcpyAsync(d_ch, ch, n_ch * sizeof(ospf_change), hipMemcpyHostToDevice,
                             (hipStream_t)stream));
  ospf::RepairArgs a{};
  a.roots = d_roots;
  a.n = n;
  a.W = nh_words;
  a.hop = (flags & OSPF_HOP_COUNT) ? 1u : 0u;
  a.dist = d_dist;
  a.nh = d_nh;
  a.ch = d_ch;
  a.n_ch = n_ch;
  a.status = d_status;
  hipError_t e = ospf::launch_repair(c->g, a, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(c, e, "launch_repair");
  return OSPF_OK;
}

}  // extern "C"
