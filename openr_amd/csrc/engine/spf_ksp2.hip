// spf_ksp2.hip — KSP2 edge-disjoint path trace on the device (gfx950).
//
// LinkState::getKthPaths(src, dst, k) (openr/decision/LinkState.cpp:790-819)
// traces paths greedily over one SPF result with a visited-link set shared by
// every path of the (src, dst, k) entry: traceOnePath (:418-439) walks dst's
// pathLinks in order, claims each link the first time it is seen and recurses
// into the link's predecessor, so a path is found by depth-first search back
// to src. pathLinks(v) = the usable, not ignored links (u, v) with u reached,
// u == src or u not overloaded, and dist(u) + metric(u -> v) == dist(v), in
// u's pop order (dist, name), then the link's position in linksFromNode(u)
// (:885-901). The device CSR keeps rows sorted by (neighbour id, that rank),
// so the candidate order of v is (dist(u), row position).
//
// One wave per run: the DFS state (node, cursor, depth) is wave-uniform; a
// candidate search scans v's row with 64 lanes (ballot for the first tight
// entry after the cursor in unit-metric graphs, a min-reduction of
// (dist(u), position) keys otherwise). Distances come from dist rows (k = 1:
// the source's row; per-run reruns) or from the level bytes of the
// multi-source BFS (k = 2 reruns, spf_msbfs.hip).
//
// Exact shortcuts (same paths as the reference, far fewer steps):
//  * dead nodes. When the DFS below a node u fails, every pathLink of u has
//    been claimed and none leads to src over unclaimed links; claims only
//    grow, so u fails again at once whenever it is re-entered. The reference's
//    claims made inside failed branches therefore only ever block links into
//    such dead nodes. The kernel marks u dead (a bit per node, HBM) and skips
//    links into dead nodes instead of claiming them, so the visited set holds
//    just the links of the paths found (an LDS hash) and each node is
//    explored in failure at most once per (src, dst, k).
//  * lookahead. A candidate predecessor with a short row (<= t.look entries, 16 by default)
//    is entered only if it has an open pathLink itself (unclaimed, into a
//    node not dead, or src); otherwise it would fail at once, so it is marked
//    dead without the descent.
//  * source cut. A path ends with an unclaimed pathLink out of src; when none
//    is left the next traceOnePath must fail, so the loop stops without the
//    (side-effect free) failing search of the whole DAG.
// Budgets (256 links deep, 1536 path links, the record size, 2^22 steps) end a
// run with an overflow status; the host then computes that destination itself.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;
constexpr int kWave = 64;
constexpr uint32_t kBlock = 256;
constexpr uint32_t kWaves = kBlock / kWave;
constexpr uint32_t kStack = 256;      // links per path
constexpr uint32_t kHash = 2048;      // visited-set slots (power of 2)
constexpr uint32_t kSteps = 1u << 22; // DFS steps per run (termination guard)
constexpr uint32_t kIgLog = 13, kIgBits = 1u << kIgLog;  // ignore-list filter bits per wave

__device__ __forceinline__ bool in_sorted(const uint32_t* a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo < n && a[lo] == x;
}

__device__ __forceinline__ uint64_t wave_min64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)x, o, kWave);
    const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), o, kWave);
    const uint64_t y = ((uint64_t)hi << 32) | lo;
    x = y < x ? y : x;
  }
  return x;
}

// distance sources of a run's trace: the source's (or a run's) dist row, the
// level bytes of the multi-source BFS, or the decremental form (below)
struct DistRows {
  const uint32_t* row;
  __device__ uint32_t operator()(uint32_t u) const { return row[u]; }
};
struct DistLev {
  const uint8_t* lev;  // the run's byte at [u][64]
  __device__ uint32_t operator()(uint32_t u) const {
    const uint32_t l = lev[(size_t)u * 64u];
    return l ? l - 1u : kInf;
  }
};
template <bool LEV>
__device__ __forceinline__ auto dist_src(const DevGraph& g, const TraceArgs& t, uint32_t i) {
  if constexpr (LEV) {
    return DistLev{t.lev + (size_t)(i >> 6) * g.V * 64u + (i & 63u)};
  } else {
    return DistRows{t.rows + (size_t)i * t.row_stride};
  }
}

// the DFS of one run (one wave); see the file comment
template <class DS, uint32_t HS = kHash>
struct Tracer {
  static constexpr uint32_t kHS = HS, kHM = HS / 4u * 3u;  // claim slots, claims allowed
  const DevGraph& g;
  const TraceArgs& t;
  uint32_t i, lane, src, dst;
  const uint32_t* ign;
  uint32_t nign;
  volatile uint32_t* hs;  // claimed links (the paths found), kHash slots
  uint32_t* dead;
  DS ds;
  // LDS filter of the ignore list when it lives in global memory (kIgBits
  // bits: a clear bit answers "not ignored" without the list's binary search)
  uint32_t* igb = nullptr;

  __device__ bool ignored(uint32_t lid) const {
    if (!nign) return false;
    if (igb) {
      const uint32_t h = igbit(lid);
      if (!((((volatile uint32_t*)igb)[h >> 5] >> (h & 31u)) & 1u)) return false;
    }
    return in_sorted(ign, nign, lid);
  }
  __device__ static uint32_t igbit(uint32_t lid) { return (lid * 0x9E3779B1u) >> (32 - kIgLog); }
  // the filter of the current ignore list (every lane of the wave)
  __device__ void build_igb() const {
    if (!igb) return;
    for (uint32_t k = lane; k < kIgBits / 32u; k += kWave) igb[k] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    for (uint32_t k = lane; k < nign; k += kWave) {
      const uint32_t h = igbit(ign[k]);
      atomicOr(&igb[h >> 5], 1u << (h & 31u));
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }

  __device__ uint32_t dist(uint32_t u) const { return ds(u); }
  __device__ static uint32_t hslot(uint32_t lid) {
    return (uint32_t)(((uint64_t)lid * 0x9E3779B97F4A7C15ull) >> 40);
  }
  __device__ bool claimed(uint32_t lid) const {  // per lane
    for (uint32_t h = hslot(lid);; ++h) {
      const uint32_t x = hs[h & (kHS - 1u)];
      if (x == lid + 1u) return true;
      if (x == 0u) return false;
    }
  }
  __device__ void claim(uint32_t lid) const {  // wave-uniform lid, not yet claimed
    const uint32_t h = hslot(lid);
    for (uint32_t p0 = 0;; p0 += kWave) {
      const uint32_t slot = (h + p0 + lane) & (kHS - 1u);
      const uint64_t em = __ballot(hs[slot] == 0u);
      if (em) {
        if (lane == (uint32_t)(__ffsll((unsigned long long)em) - 1)) hs[slot] = lid + 1u;
        return;
      }
    }
  }
  __device__ bool is_dead(uint32_t u) const {
    const uint32_t w =
        __hip_atomic_load(&dead[u >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return (w >> (u & 31u)) & 1u;
  }
  __device__ void mark_dead(uint32_t u) const {
    __hip_atomic_fetch_or(&dead[u >> 5], 1u << (u & 31u), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  // pathLinks entry e of row v, not claimed, predecessor cx not dead? (no
  // lookahead: see alive)
  __device__ bool cand0(uint32_t v, uint32_t dv, uint32_t e, uint32_t& du, uint32_t& cx) const {
    cx = g.colx[e];
    if (cx & kDown) return false;
    if (cx == v) return false;
    du = dist(cx);
    if (du == kInf) return false;
    const uint32_t w = t.unit ? 1u : g.rw[e];
    if ((uint64_t)du + w != dv) return false;
    if (cx != src && ((g.nt_bits[cx >> 5] >> (cx & 31u)) & 1u)) return false;
    const uint32_t lid = g.link_id[e];
    if (ignored(lid)) return false;
    if (cx == src) return !claimed(lid);
    return !is_dead(cx) && !claimed(lid);
  }
  // one level of lookahead by the whole wave (wave-uniform x != src, du =
  // dist(x)): a predecessor whose short row (<= t.look entries) holds no
  // open pathLink of its own fails at once when entered, i.e. it is dead
  __device__ bool alive(uint32_t x, uint32_t du) const {
    const uint32_t b2 = g.row_ptr[x], e2end = g.row_ptr[x + 1];
    if (e2end - b2 > t.look) return true;
    bool ok = false;
    for (uint32_t e2 = b2 + lane; e2 < e2end; e2 += kWave) {
      const uint32_t c2 = g.colx[e2];
      if ((c2 & kDown) || c2 == x) continue;
      const uint32_t d2 = dist(c2);
      if (d2 == kInf || (uint64_t)d2 + (t.unit ? 1u : g.rw[e2]) != du) continue;
      if (c2 != src && ((g.nt_bits[c2 >> 5] >> (c2 & 31u)) & 1u)) continue;
      const uint32_t l2 = g.link_id[e2];
      if (ignored(l2)) continue;
      if (c2 != src && is_dead(c2)) continue;
      if (!claimed(l2)) ok = true;
    }
    if (__ballot(ok)) return true;
    if (lane == 0) mark_dead(x);
    return false;
  }
  // cand0 plus this lane's own sequential lookahead (the 16-wave kernel's
  // candidate gathering)
  __device__ bool cand(uint32_t v, uint32_t dv, uint32_t e, uint32_t& du) const {
    uint32_t cx = 0;
    if (!cand0(v, dv, e, du, cx)) return false;
    return cx == src || look_lane(cx, du);
  }
  // this lane's lookahead of its own predecessor cx != src (see alive)
  __device__ bool look_lane(uint32_t cx, uint32_t du) const {
    const uint32_t b2 = g.row_ptr[cx], e2end = g.row_ptr[cx + 1];
    if (e2end - b2 > t.look) return true;
    for (uint32_t e2 = b2; e2 < e2end; ++e2) {
      const uint32_t c2 = g.colx[e2];
      if ((c2 & kDown) || c2 == cx) continue;
      const uint32_t d2 = dist(c2);
      if (d2 == kInf || (uint64_t)d2 + (t.unit ? 1u : g.rw[e2]) != du) continue;
      if (c2 != src && ((g.nt_bits[c2 >> 5] >> (c2 & 31u)) & 1u)) continue;
      const uint32_t l2 = g.link_id[e2];
      if (ignored(l2)) continue;
      if (c2 != src && is_dead(c2)) continue;
      if (!claimed(l2)) return true;
    }
    mark_dead(cx);
    return false;
  }
  // smallest candidate key (du << 32 | e) >= lo among v's pathLinks, ~0 =
  // none. The cheap checks run on every lane; the lookahead (alive) only for
  // the candidates in order until one passes, by the whole wave.
  __device__ uint64_t next_cand(uint32_t v, uint32_t dv, uint64_t lo) const {
    const uint32_t beg = g.row_ptr[v], end = g.row_ptr[v + 1];
    if (t.unit) {  // every candidate has du = dv - 1: row order
      const uint32_t e0 = lo ? max(beg, (uint32_t)lo) : beg;
      for (uint32_t base = e0; base < end; base += kWave) {
        const uint32_t e = base + lane;
        uint32_t du = 0, cx = 0;
        const bool ok = e < end && cand0(v, dv, e, du, cx);
        uint64_t bal = __ballot(ok);
        if (!bal) continue;
        // the first candidate by the whole wave; when it is dead, the rest of
        // the chunk each by its own lane at once (a failing search's chunks
        // are mostly dead ends: all of them pruned in one pass)
        const int j = __ffsll((unsigned long long)bal) - 1;
        const uint32_t xj = (uint32_t)__shfl((int)cx, j, kWave);
        if (xj == src || alive(xj, dv - 1u)) return ((uint64_t)(dv - 1u) << 32) | (base + (uint32_t)j);
        const bool ok2 = ok && lane != (uint32_t)j && (cx == src || look_lane(cx, dv - 1u));
        bal = __ballot(ok2);
        if (bal) return ((uint64_t)(dv - 1u) << 32) | (base + (uint32_t)(__ffsll((unsigned long long)bal) - 1));
      }
      return ~0ull;
    }
    for (;;) {
      uint64_t best = ~0ull;
      for (uint32_t e = beg + lane; e < end; e += kWave) {
        uint32_t du = 0, cx = 0;
        if (!cand0(v, dv, e, du, cx)) continue;
        const uint64_t key = ((uint64_t)du << 32) | e;
        if (key >= lo && key < best) best = key;
      }
      best = wave_min64(best);
      if (best == ~0ull) return best;
      const uint32_t x = g.colx[(uint32_t)best];
      if (x == src || alive(x, (uint32_t)(best >> 32))) return best;
      lo = best + 1ull;  // x is dead now: the next key
    }
  }
  // an unclaimed pathLink out of src is left (a node x with dist(x) ==
  // metric(src -> x)); a path to src ends with one
  __device__ bool src_open() const {
    const uint32_t beg = g.row_ptr[src], end = g.row_ptr[src + 1];
    bool any = false;
    for (uint32_t e = beg + lane; e < end; e += kWave) {
      const uint32_t cx = g.colx[e];
      if ((cx & kDown) || cx == src) continue;
      const uint32_t w = t.unit ? 1u : g.w[e];
      if (dist(cx) != w) continue;
      const uint32_t lid = g.link_id[e];
      if (ignored(lid)) continue;
      if (!claimed(lid)) any = true;
    }
    return __ballot(any) != 0ull;
  }
  // depth-first search (traceOnePath, LinkState.cpp:418-439) continuing from
  // the `depth` links on the stack (dst -> ...), never popping below d0.
  // 1: reached src (path on the stack), 0: failed, -1: step budget, -2: too deep
  __device__ int dfs(volatile uint32_t* stk, uint32_t& depth, uint32_t d0, uint32_t& steps,
                     uint32_t budget) const {
    uint32_t v = depth ? g.colx[stk[depth - 1]] : dst;
    uint32_t dv = dist(v);
    uint64_t lo = 0;
    for (;;) {
      if (v == src) return 1;
      if (++steps > budget) return -1;
      const uint64_t key = next_cand(v, dv, lo);
      if (key == ~0ull) {  // v's pathLinks are exhausted: v is dead
        if (depth > 0 && lane == 0) mark_dead(v);
        if (depth == d0) return 0;
        const uint32_t pe = stk[--depth];
        v = depth ? g.colx[stk[depth - 1]] : dst;
        dv = dist(v);
        lo = (((uint64_t)dist(g.colx[pe])) << 32 | pe) + 1ull;
        continue;
      }
      if (depth == kStack) return -2;
      const uint32_t e = (uint32_t)key;
      stk[depth++] = e;
      v = g.colx[e];
      dv = (uint32_t)(key >> 32);
      lo = 0;
    }
  }
  // append the path on the stack to the record at word w, claim its links
  __device__ bool emit(uint32_t* out, volatile uint32_t* stk, uint32_t depth, uint32_t& w,
                       uint32_t& npaths, uint32_t& nclaim) const {
    if (w + 1u + depth > t.stride || nclaim + depth > kHM) return false;
    // path from src to dst: the stack bottom-up is dst -> src
    for (uint32_t k = lane; k < depth; k += kWave) out[w + 1u + k] = g.link_id[stk[depth - 1u - k]];
    if (lane == 0) out[w] = depth;
    for (uint32_t k = 0; k < depth; ++k) claim(g.link_id[stk[k]]);
    nclaim += depth;
    w += 1u + depth;
    ++npaths;
    if (lane == 0) out[0] = npaths;
    return true;
  }
  // record count, k = 2 status, or k = 1's sorted link set + status
  // (LinkState.cpp:797-803; edge-disjoint paths, so no duplicates); `scr` is
  // LDS scratch of >= stride words
  __device__ void finish(uint32_t* out, uint32_t npaths, bool ovf, volatile uint32_t* scr) const {
    if (lane == 0) out[0] = ovf ? 0u : npaths;
    if (t.k == 2) {
      if (ovf && lane == 0) t.status[i] |= OSPF_KSP_OVF2;
      return;
    }
    uint32_t* io = t.ign_out + (size_t)i * t.stride;
    uint32_t m = 0;
    if (!ovf) {
      __threadfence_block();  // the record's words, written by other lanes
      for (uint32_t p = 0, q = 1; p < npaths; ++p) {
        const uint32_t len = out[q];
        for (uint32_t k = lane; k < len; k += kWave) scr[m + k] = out[q + 1u + k];
        m += len;
        q += 1u + len;
      }
      for (uint32_t j = lane; j < m; j += kWave) {
        const uint32_t x = scr[j];
        uint32_t rank = 0;
        for (uint32_t k = 0; k < m; ++k) rank += scr[k] < x ? 1u : 0u;
        io[rank] = x;
      }
    }
    for (uint32_t k = m + lane; k < t.stride; k += kWave) io[k] = kInf;
    if (lane == 0) {
      t.cnt_out[i] = ovf ? 0u : m;
      t.status[i] = ovf ? OSPF_KSP_OVF1 : (m ? OSPF_KSP_RERUN : 0u);
    }
  }
};

// run setup shared by both kernels: false = nothing to trace (record and
// status already final)
template <class DS, uint32_t HS>
__device__ bool trace_setup(const DevGraph& g, const TraceArgs& t, uint32_t i, uint32_t lane,
                            Tracer<DS, HS>& tr) {
  uint32_t* out = t.out + (size_t)i * t.stride;
  tr.ign = nullptr;
  tr.nign = 0;
  if (t.k == 2) {
    const uint32_t st = t.status[i];
    if (st & OSPF_KSP_OVF1) {  // no k = 1 paths, so no ignore set: not computed
      if (lane == 0) t.status[i] = st | OSPF_KSP_OVF2;
      return false;
    }
    if (!(st & OSPF_KSP_RERUN)) {  // k = 1 found nothing: neither does k = 2
      if (lane == 0) out[0] = 0u;
      return false;
    }
    tr.ign = t.ign + (size_t)i * t.stride;
    tr.nign = min(t.ign_cnt[i], t.stride);
    tr.build_igb();
  }
  if (tr.dst == tr.src || tr.dist(tr.dst) == kInf) {  // LinkState.cpp:808-809: no paths
    if (lane == 0) out[0] = 0u;
    if (t.k == 1) {
      for (uint32_t k = lane; k < t.stride; k += kWave) t.ign_out[(size_t)i * t.stride + k] = kInf;
      if (lane == 0) {
        t.cnt_out[i] = 0u;
        t.status[i] = 0u;
      }
    }
    return false;
  }
  return true;
}

// one wave per run; a run that spends more than t.budget DFS steps (unit
// metric) without finding a path -- a long failing search -- is queued for
// ksp_heavy_kernel, which resumes it with 16 waves
// HS: claim-hash slots per wave. With the 16-wave kernel behind it (unit
// metric) a 1,024-slot hash (20 KB per block: 7 blocks per CU, VGPR-bound)
// and runs past its claims go there; otherwise kHash slots.
template <bool LEV, uint32_t HS>
__global__ void __launch_bounds__(256) ksp_trace_kernel(DevGraph g, TraceArgs t) {
  __shared__ uint32_t s_stack[kWaves][kStack];
  __shared__ uint32_t s_hash[kWaves][HS];
  __shared__ uint32_t s_igb[kWaves][kIgBits / 32u];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t i = blockIdx.x * kWaves + wv;
  if (i >= t.n) return;
  volatile uint32_t* stk = s_stack[wv];
  Tracer<decltype(dist_src<LEV>(g, t, i)), HS> tr{g, t, i, lane, t.src, t.dsts[i], nullptr, 0,
                                                  s_hash[wv], t.dead + (size_t)i * t.dead_words,
                                                  dist_src<LEV>(g, t, i), s_igb[wv]};
  if (!trace_setup(g, t, i, lane, tr)) return;
  for (uint32_t k = lane; k < HS; k += kWave) tr.hs[k] = 0u;
  uint32_t* out = t.out + (size_t)i * t.stride;
  uint32_t npaths = 0, w = 1, steps = 0, nclaim = 0;
  bool ovf = false;
  const uint32_t budget = t.budget ? t.budget : kSteps;
  if (lane == 0) out[0] = 0u;
  while (!ovf && tr.src_open()) {  // one traceOnePath per iteration, until it fails
    uint32_t depth = 0;
    const int r = tr.dfs(stk, depth, 0, steps, budget);
    if (r == 0) break;
    // heavy: a long failing search, or more claimed links than this hash
    // holds; the paths so far stay in the record
    if ((r == -1 && t.budget) ||
        (r == 1 && t.budget && HS < kHash && nclaim + depth > tr.kHM && w + 1u + depth <= t.stride)) {
      if (lane == 0) t.heavy[atomicAdd(&t.heavy_ctr[0], 1u)] = i;
      return;
    }
    if (r < 0 || !tr.emit(out, stk, depth, w, npaths, nclaim)) ovf = true;
    if (t.budget) steps = 0;  // the budget bounds the steps between two paths
  }
  tr.finish(out, npaths, ovf, tr.hs);
}

// Heavy runs (the DFS took more than the budget, e.g. a spine behind 1,780
// pods): a workgroup of 16 waves per run, resuming from the paths already in
// its record. Each traceOnePath takes dst's candidates 16 at a time in order;
// wave j searches below candidate j with the same claims and shared dead
// marks (facts: a node once dead stays dead), and the lowest candidate that
// reaches src is the reference's choice (every earlier one failed). Blocks
// take runs from the queue until it is empty.
constexpr uint32_t kHeavyWaves = 16;
struct HeavyLds {
  uint32_t stack[kHeavyWaves][kStack];
  uint64_t cand[kHeavyWaves];
  int32_t res[kHeavyWaves];
  uint32_t ctl[4];
  uint32_t nbig;
};
// heavy_trace's pruning hook (every thread of the block calls it): none
struct NoPrune {
  __device__ void operator()() const {}
};
// the 16-wave trace of run i, resuming from its record; `hs` = the block's
// claim hash (kHash slots), every wave of the block calls it
template <class DS, class Prune = NoPrune>
__device__ void heavy_trace(const DevGraph& g, const TraceArgs& t, uint32_t i, Tracer<DS, kHash>& tr,
                            uint32_t* hs, HeavyLds& H, const Prune& prune = Prune{}) {
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint32_t* out = t.out + (size_t)i * t.stride;
  for (uint32_t k = threadIdx.x; k < kHash; k += blockDim.x) hs[k] = 0u;
  __syncthreads();
  // resume: the paths the single-wave pass found
  uint32_t npaths = 0, w = 1, nclaim = 0;
  if (wv == 0) {
    npaths = out[0];
    for (uint32_t p = 0; p < npaths; ++p) {
      const uint32_t len = out[w];
      for (uint32_t k = 0; k < len; ++k) tr.claim(out[w + 1u + k]);
      nclaim += len;
      w += 1u + len;
    }
  }
  __syncthreads();
  prune();  // (the claims of the paths found so far)
  bool ovf = false;
  uint32_t steps = 0;
  for (;;) {  // one traceOnePath per iteration
    if (wv == 0) H.ctl[1] = tr.src_open() ? 1u : 0u;
    __syncthreads();
    if (!H.ctl[1]) break;
    uint64_t lo = 0;
    int winner = -1;
    bool stop = false;
    for (uint32_t round = 0;; ++round) {  // dst's candidates, 16 at a time
      // a long failing search: prune again with the claims of now (nodes
      // that lost their last way to src since the last pruning)
      if (round == 4) prune();
      if (wv == 0) {  // the next (up to) 16 candidates of dst in row order
        uint32_t m = 0;
        const uint32_t dv = tr.dist(tr.dst);
        const uint32_t beg = g.row_ptr[tr.dst], end = g.row_ptr[tr.dst + 1];
        uint32_t base = lo ? max(beg, (uint32_t)lo) : beg;
        for (; base < end && m < kHeavyWaves; base += kWave) {
          const uint32_t e = base + lane;
          uint32_t du = 0;
          const bool ok = e < end && tr.cand(tr.dst, dv, e, du);
          const uint64_t bal = __ballot(ok);
          const uint32_t rank = m + __popcll(bal & ((1ull << lane) - 1ull));
          if (ok && rank < kHeavyWaves) H.cand[rank] = ((uint64_t)(dv - 1u) << 32) | e;
          const uint32_t got = m + (uint32_t)__popcll(bal);
          if (got >= kHeavyWaves) {  // resume after the 16th
            uint64_t b2 = bal;
            for (uint32_t k = m; k < kHeavyWaves - 1u; ++k) b2 &= b2 - 1ull;
            base += (uint32_t)(__ffsll((unsigned long long)b2) - 1) + 1u - kWave;
            m = kHeavyWaves;
            base += kWave;
            break;
          }
          m = got;
        }
        lo = ((uint64_t)(dv - 1u) << 32) | min(base, end);
        H.ctl[2] = m;
      }
      __syncthreads();
      const uint32_t m = H.ctl[2];
      if (m == 0) {
        stop = true;
        break;
      }
      if (wv < m) {
        uint32_t depth = 1, st2 = 0;
        H.stack[wv][0] = (uint32_t)H.cand[wv];
        const int r = tr.dfs(H.stack[wv], depth, 1, st2, kSteps);
        if (lane == 0) H.res[wv] = r == 1 ? (int32_t)depth : (r < 0 ? -1 : 0);
      }
      __syncthreads();
      uint32_t k = 0;
      for (; k < m; ++k)
        if (H.res[k] != 0) break;
      if (k < m) {
        if (H.res[k] < 0) ovf = true;
        else winner = (int)k;
        break;
      }
    }
    __syncthreads();
    if (ovf || stop || winner < 0) break;
    if (wv == 0 && !tr.emit(out, H.stack[winner], (uint32_t)H.res[winner], w, npaths, nclaim))
      H.ctl[3] = 1u;
    else if (wv == 0)
      H.ctl[3] = 0u;
    __syncthreads();
    if (H.ctl[3]) {
      ovf = true;
      break;
    }
    if (++steps > kSteps) {
      ovf = true;
      break;
    }
  }
  __syncthreads();
  if (wv == 0) tr.finish(out, npaths, ovf, hs);
  __syncthreads();
}

// Heavy runs (the DFS took more than the budget, e.g. a spine behind 1,780
// pods): a workgroup of 16 waves per run, resuming from the paths already in
// its record. Each traceOnePath takes dst's candidates 16 at a time in order;
// wave j searches below candidate j with the same claims and shared dead
// marks (facts: a node once dead stays dead), and the lowest candidate that
// reaches src is the reference's choice (every earlier one failed). Blocks
// take runs from the queue until it is empty.
template <bool LEV>
__global__ void __launch_bounds__(1024) ksp_heavy_kernel(DevGraph g, TraceArgs t) {
  __shared__ uint32_t s_hash[kHash];
  __shared__ HeavyLds H;
  __shared__ uint32_t s_igb[kHeavyWaves][kIgBits / 32u];  // each wave's own filter
  const uint32_t lane = threadIdx.x & 63u;
  for (;;) {
    if (threadIdx.x == 0) {
      const uint32_t q = atomicAdd(&t.heavy_ctr[1], 1u);
      H.ctl[0] = q < __hip_atomic_load(&t.heavy_ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     ? t.heavy[q] : kInf;
    }
    __syncthreads();
    const uint32_t i = H.ctl[0];
    __syncthreads();
    if (i == kInf) return;
    Tracer<decltype(dist_src<LEV>(g, t, i))> tr{g, t, i, lane, t.src, t.dsts[i], nullptr, 0, s_hash,
                                                t.dead + (size_t)i * t.dead_words,
                                                dist_src<LEV>(g, t, i), s_igb[threadIdx.x >> 6]};
    trace_setup(g, t, i, lane, tr);  // (a queued run always has work)
    heavy_trace(g, t, i, tr, s_hash, H);
  }
}

// ---------------------------------------------------------------- decremental reruns
// The k = 2 rerun of destination d is runSpf(src, true, I_d) with I_d the
// links of d's k = 1 paths (LinkState.cpp:797-805). Removing links only
// lengthens paths, and a node keeps its distance iff one of its supports --
// tight in-links (u, v) of the source's SPF: u transit or src, dist(u) +
// w(u -> v) == dist(v) -- survives with u unaffected. The affected set A is
// the fixed point of lost supports: an ignored link loses its tight
// directions, an affected node loses its tight out-links. Each node has a
// hint, the link of its last support (ksp_hint_kernel); a lost support that
// is not a node's hint changes nothing while the hint stands, so a node gets
// an LDS entry only once its hint is lost: then its surviving supports are
// counted once (tails unaffected, or affected and not yet expanded -- those
// decrement it when they are), and it joins A when the count reaches zero.
// On the fabric a rack's run touches ~2 nodes (F100k) where the full rerun
// scans the whole graph. The masked distances of A: its boundary terms
// (unaffected transit in-neighbours over usable, unignored links), then
// Bellman-Ford rounds over links inside A; every other node keeps the
// source's distance (DistDecr). The k = 2 trace then runs over them. Runs
// past the LDS budgets (A, hash, ignore list, claimed links) go to the full
// masked reruns; traces past the step budget to the 16-wave kernel.
constexpr uint32_t kAffFlag = 0x80000000u;
__device__ __forceinline__ uint32_t dslot(uint32_t u) { return (u * 0x9E3779B1u) >> 20; }

template <uint32_t MAP, uint32_t AFF, uint32_t IGN, uint32_t HS, uint32_t EDGE>
struct DecrLdsT {
  static constexpr uint32_t kMap = MAP, kFill = MAP / 4u * 3u, kAff = AFF, kIgn = IGN, kHS = HS;
  // out-links the affected nodes' expansion may scan before the run is given
  // up (a run that cuts a plane off scans the plane's spine rows: the full
  // masked rerun, 64 runs per traversal, does that for less)
  static constexpr uint32_t kEdge = EDGE;
  uint32_t keys[MAP];  // node + 1 (0: empty)
  uint32_t vals[MAP];  // supports left (hint lost), or kAffFlag | index in aff
  uint32_t aff[AFF];
  uint32_t dp[AFF];    // masked distance of aff[k]
  uint32_t ign[IGN];
  uint32_t hash[HS];   // the trace's claimed links
  uint32_t stack[kStack];
  uint32_t pend[64];   // nodes whose hint was just lost (their supports to count)
  uint32_t nkeys, naff, ovf, run, npend;
  uint32_t why;        // a failed prepare: 0 an LDS budget, 1 the edge budget, 2 the ignore list
  uint64_t t3;         // wall clock at step (3) (phase timing, t.ctr[16..])
};
using DecrSmall = DecrLdsT<512, 192, 256, 512, 4096>;  // ~10 KB: ~16 runs per CU in flight
using DecrHeavy = DecrLdsT<4096, 1024, 1024, kHash, 1u << 30>;

template <class L_>
struct DistDecr {
  const uint32_t* D;  // the source's dist row
  const L_* L;
  __device__ uint32_t operator()(uint32_t u) const {
    const volatile uint32_t* keys = L->keys;
    uint32_t h = dslot(u);
    for (uint32_t p = 0; p < L_::kMap; ++p, ++h) {  // (the map never fills: kFill)
      const uint32_t k = keys[h & (L_::kMap - 1u)];
      if (k == u + 1u) {
        const uint32_t v = ((const volatile uint32_t*)L->vals)[h & (L_::kMap - 1u)];
        return (v & kAffFlag) ? ((const volatile uint32_t*)L->dp)[v & ~kAffFlag] : D[u];
      }
      if (k == 0u) break;
    }
    return D[u];
  }
};

// hint[v] = link id of v's last support in row order (kInf: none). The
// last, not the first: a k = 1 trace takes each node's first candidate in
// row order (traceOnePath's pathLinks order), so the first supports are the
// ones the ignored links cut -- with them as hints every plane-0 fabric
// switch of F100k would lose its hint to a rack's k = 1 path through spine
// 1-0-0, with the last ones none does.
__global__ void __launch_bounds__(256) ksp_hint_kernel(DevGraph g, uint32_t src,
                                                       const uint32_t* __restrict__ D,
                                                       uint32_t* __restrict__ hint) {
  // one wave per node: a spine's row (1,781 entries at F100k) takes 28
  // coalesced steps, not 1,781 dependent ones of a single lane
  const uint32_t v = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  if (v >= g.V) return;
  const uint32_t dv = D[v];
  uint32_t h = kInf;
  if (dv != kInf && v != src) {
    const uint32_t beg = g.row_ptr[v], end = g.row_ptr[v + 1];
    for (uint32_t b = beg; b < end; b += kWave) {
      const uint32_t e = b + lane;
      bool ok = false;
      if (e < end) {
        const uint32_t u = g.colx[e];
        if (!(u & kDown) && u != v) {
          const uint32_t du = D[u];
          ok = du != kInf && (uint64_t)du + g.rw[e] == dv &&
               (u == src || !((g.nt_bits[u >> 5] >> (u & 31u)) & 1u));
        }
      }
      const uint64_t bal = __ballot(ok);
      if (bal) h = g.link_id[b + 63u - (uint32_t)__clzll((long long)bal)];
    }
  }
  if (lane == 0) hint[v] = h;
}

template <class L_>
__device__ __forceinline__ uint32_t map_find(const L_& L, uint32_t u) {  // slot, kInf: absent
  const volatile uint32_t* keys = L.keys;
  uint32_t h = dslot(u);
  for (uint32_t p = 0; p < L_::kMap; ++p, ++h) {
    const uint32_t k = keys[h & (L_::kMap - 1u)];
    if (k == u + 1u) return h & (L_::kMap - 1u);
    if (k == 0u) return kInf;
  }
  return kInf;
}
// index of u in A, kInf: not affected
template <class L_>
__device__ __forceinline__ uint32_t aff_ix(const L_& L, uint32_t u) {
  const uint32_t sl = map_find(L, u);
  if (sl == kInf) return kInf;
  const uint32_t v = ((const volatile uint32_t*)L.vals)[sl];
  return (v & kAffFlag) ? (v & ~kAffFlag) : kInf;
}
// a new key (this lane's node u, not present): its slot, kInf on overflow
template <class L_>
__device__ __forceinline__ uint32_t map_insert(L_& L, uint32_t u) {
  volatile uint32_t* keys = L.keys;
  if (((volatile uint32_t&)L.ovf)) return kInf;  // past the budget: the run is abandoned
  uint32_t h = dslot(u);
  for (uint32_t p = 0; p < L_::kMap; ++p, ++h) {
    const uint32_t sl = h & (L_::kMap - 1u);
    if (keys[sl] != 0u) {
      if (keys[sl] == u + 1u) return sl;
      continue;
    }
    const uint32_t old = atomicCAS(&L.keys[sl], 0u, u + 1u);
    if (old == 0u) {
      if (atomicAdd(&L.nkeys, 1u) >= L_::kFill) L.ovf = 1u;  // <= kFill + 63 keys: empty slots stay
      return sl;
    }
    if (old == u + 1u) return sl;
  }
  L.ovf = 1u;
  return kInf;
}
template <class L_>
__device__ __forceinline__ void make_affected(L_& L, uint32_t slot, uint32_t v) {
  const uint32_t k = atomicAdd(&L.naff, 1u);
  if (k >= L_::kAff) {
    L.ovf = 1u;
    return;
  }
  L.aff[k] = v;
  L.vals[slot] = kAffFlag | k;
}

// Steps (0)-(3) of run i by one wave into L; false: past a budget (the full
// rerun). na = |A|, or kInf when the ignored links cut the source off.
template <class L_>
__device__ bool decr_prepare(L_& L, const DevGraph& g, const TraceArgs& t, uint32_t i,
                             uint32_t lane, uint32_t& nign, uint32_t& na) {
  const uint32_t* D = t.rows;
  const uint32_t* hint = t.tc;
  const uint32_t src = t.src;
  auto transit = [&](uint32_t u) { return u == src || !((g.nt_bits[u >> 5] >> (u & 31u)) & 1u); };
  auto ignored = [&](uint32_t lid) { return nign && in_sorted(L.ign, nign, lid); };
  const uint32_t* gign = t.ign + (size_t)i * t.stride;
  nign = min(t.ign_cnt[i], t.stride);
  if (nign > L_::kIgn) {
    if (lane == 0) {
      atomicAdd(&t.ctr[8], 1u);
      L.why = 2u;
    }
    return false;
  }
  if (lane == 0) L.why = 0u;
  for (uint32_t k = lane; k < L_::kMap; k += kWave) {
    L.keys[k] = 0u;
    L.vals[k] = 0u;
  }
  for (uint32_t k = lane; k < nign; k += kWave) L.ign[k] = gign[k];
  if (lane == 0) {
    L.nkeys = 0u;
    L.naff = 0u;
    L.ovf = 0u;
    L.npend = 0u;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  // (0) the ignored links may cut every usable link of the source: then the
  // rerun reaches nothing but src
  {
    bool open = false;
    for (uint32_t e = g.row_ptr[src] + lane; e < g.row_ptr[src + 1]; e += kWave) {
      const uint32_t x = g.colx[e];
      if (!(x & kDown) && x != src && !ignored(g.link_id[e])) open = true;
    }
    if (!__ballot(open)) {
      na = kInf;
      return true;
    }
  }
  volatile uint32_t* vpend = L.pend;
  // count the supports of the pending nodes (their hint just lost): tails
  // unaffected, or affected and not yet expanded (index >= qexp, the count
  // of expanded nodes); none -> A
  auto settle_pending = [&](uint32_t qexp) {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
    const uint32_t np = min(((volatile uint32_t&)L.npend), 64u);
    if (((volatile uint32_t&)L.npend) > 64u) L.ovf = 1u;
    for (uint32_t j = 0; j < np; ++j) {
      const uint32_t x = vpend[j];
      const uint32_t dx = D[x];
      uint32_t cnt = 0;
      for (uint32_t e = g.row_ptr[x] + lane; e < g.row_ptr[x + 1]; e += kWave) {
        const uint32_t u = g.colx[e];
        if ((u & kDown) || u == x) continue;
        const uint32_t du = D[u];
        if (du == kInf || (uint64_t)du + g.rw[e] != dx || !transit(u)) continue;
        if (ignored(g.link_id[e])) continue;
        const uint32_t ui = aff_ix(L, u);
        if (ui != kInf && ui < qexp) continue;  // lost already (expanded)
        ++cnt;
      }
      for (int o = 32; o > 0; o >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, o, kWave);
      if (lane == 0) {
        const uint32_t sl = map_find(L, x);
        if (cnt == 0u) make_affected(L, sl, x);
        else L.vals[sl] = cnt;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) L.npend = 0u;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
  };
  // the support (., x) over link lid is lost: the hint -> x pending; else a
  // counted support of a settled x -> one fewer. While x is pending, only
  // the node being expanded loses supports of x, and the settle does not
  // count them.
  constexpr uint32_t kPend = 0x7FFFFFFFu;
  auto lose = [&](uint32_t x, uint32_t lid, bool is_ign) {
    const bool is_hint = hint[x] == lid;
    const uint32_t sl = map_find(L, x);
    if (is_hint) {
      if (sl != kInf) return;  // (cannot happen: a hint is lost once)
      const uint32_t ns = map_insert(L, x);
      if (ns == kInf) return;
      L.vals[ns] = kPend;
      const uint32_t k = atomicAdd(&L.npend, 1u);
      if (k < 64u) L.pend[k] = x;
      return;
    }
    if (is_ign || sl == kInf) return;  // the hint stands, or ignored links were never counted
    const uint32_t v = ((volatile uint32_t*)L.vals)[sl];
    if ((v & kAffFlag) || v == kPend) return;
    if (atomicSub(&L.vals[sl], 1u) == 1u) make_affected(L, sl, x);
  };
  // (1) the ignored links' tight directions: 32 links per step, lane =
  // (link, direction), so a step leaves <= 64 nodes pending
  for (uint32_t k0 = 0; k0 < nign; k0 += 32u) {
    const uint32_t k = k0 + (lane & 31u);
    if (k < nign) {
      const uint32_t l = L.ign[k];
      const uint32_t e0 = l < g.n_lid ? g.link_e[2u * l] : kInf;
      const uint32_t e1 = l < g.n_lid ? g.link_e[2u * l + 1u] : kInf;
      if (e0 != kInf && e1 != kInf) {
        const uint32_t b = g.colx[e0], a = g.colx[e1];  // e0 in a's row, e1 in b's row
        if (!(b & kDown) && !(a & kDown) && a != b) {  // a down link supports nothing
          // this lane's direction: u -> x over entry e of u's row
          const bool fwd = lane < 32u;
          const uint32_t u = fwd ? a : b, x = fwd ? b : a, e = fwd ? e0 : e1;
          const uint32_t du = D[u];
          if (du != kInf && transit(u) && (uint64_t)du + g.w[e] == D[x]) lose(x, l, true);
        }
      }
    }
    settle_pending(0u);
  }
  // (2) affected nodes in order lose their tight out-links
  uint32_t scanned = 0;
  for (uint32_t q = 0;; ++q) {
    const uint32_t nq = ((volatile uint32_t&)L.naff);
    if (((volatile uint32_t&)L.ovf) || q >= min(nq, L_::kAff)) break;
    const uint32_t v = ((volatile uint32_t*)L.aff)[q];
    if (!transit(v)) continue;
    const uint32_t dv = D[v];
    const uint32_t beg = g.row_ptr[v], end = g.row_ptr[v + 1];
    scanned += end - beg;
    if (scanned > L_::kEdge) {
      if (lane == 0) {
        L.ovf = 1u;
        L.why = 1u;
        atomicAdd(&t.ctr[10], 1u);
      }
      break;
    }
    for (uint32_t e0 = beg; e0 < end; e0 += kWave) {
      const uint32_t e = e0 + lane;
      bool go = false;
      uint32_t x = 0, lid = 0;
      if (e < end) {
        x = g.colx[e];
        if (!(x & kDown) && x != v && (uint64_t)dv + g.w[e] == D[x]) {
          lid = g.link_id[e];
          go = !ignored(lid);
        }
      }
      if (go) lose(x, lid, false);
      settle_pending(q + 1u);  // (<= 64 pending per step)
    }
  }
  if (((volatile uint32_t&)L.ovf)) {
    if (lane == 0 && scanned <= L_::kEdge)
      atomicAdd(&t.ctr[((volatile uint32_t&)L.naff) > L_::kAff ? 6 : 7], 1u);
    return false;
  }
  na = ((volatile uint32_t&)L.naff);
  if (lane == 0) L.t3 = wall_clock64();
  // (3) masked distances of A: boundary terms, then rounds over A's own links
  bool inner = false;
  for (uint32_t q = 0; q < na; ++q) {
    const uint32_t a = ((volatile uint32_t*)L.aff)[q];
    uint32_t best = kInf;
    for (uint32_t e = g.row_ptr[a] + lane; e < g.row_ptr[a + 1]; e += kWave) {
      const uint32_t u = g.colx[e];
      if ((u & kDown) || u == a || !transit(u)) continue;
      if (ignored(g.link_id[e])) continue;
      if (aff_ix(L, u) != kInf) {
        inner = true;
        continue;
      }
      const uint32_t du = D[u];
      if (du == kInf) continue;
      best = min(best, du + g.rw[e]);
    }
    for (int o = 32; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, kWave));
    if (lane == 0) L.dp[q] = best;
  }
  if (__ballot(inner)) {
    for (uint32_t round = 0; round <= na; ++round) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      bool changed = false;
      for (uint32_t q = 0; q < na; ++q) {
        const uint32_t a = ((volatile uint32_t*)L.aff)[q];
        uint32_t best = ((volatile uint32_t*)L.dp)[q];
        const uint32_t b0 = best;
        for (uint32_t e = g.row_ptr[a] + lane; e < g.row_ptr[a + 1]; e += kWave) {
          const uint32_t u = g.colx[e];
          if ((u & kDown) || u == a || !transit(u)) continue;
          const uint32_t ui = aff_ix(L, u);
          if (ui == kInf || ignored(g.link_id[e])) continue;
          const uint32_t du = ((volatile uint32_t*)L.dp)[ui];
          if (du == kInf) continue;
          best = min(best, du + g.rw[e]);
        }
        for (int o = 32; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, kWave));
        if (best < b0) {
          changed = true;
          if (lane == 0) L.dp[q] = best;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        __builtin_amdgcn_wave_barrier();
      }
      if (!changed) break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
  return true;
}

// One wave per run (blocks of one wave, runs taken from t.ctr[0]).
__global__ void __launch_bounds__(64) ksp_decr_kernel(DevGraph g, TraceArgs t) {
  __shared__ DecrSmall L;
  const uint32_t lane = threadIdx.x;
  const uint32_t src = t.src;
  uint32_t* dead = t.dead + (size_t)blockIdx.x * t.dead_words;
  // persistent (decr_runs 0: until the runs are taken), or decr_runs runs per
  // block so a higher-priority stream's blocks get the CUs as blocks retire
  for (uint32_t it = 0; t.decr_runs == 0 || it < t.decr_runs; ++it) {
    if (lane == 0) L.run = atomicAdd(&t.ctr[0], 1u);
    __builtin_amdgcn_wave_barrier();
    const uint32_t i = ((volatile uint32_t&)L.run);
    if (i >= t.n) return;
    uint32_t* out = t.out + (size_t)i * t.stride;
    const uint32_t st = t.status[i];
    if (st & OSPF_KSP_OVF1) {  // no k = 1 paths, so no ignore set: not computed
      if (lane == 0) t.status[i] = st | OSPF_KSP_OVF2;
      continue;
    }
    if (!(st & OSPF_KSP_RERUN)) {  // k = 1 found nothing: neither does k = 2
      if (lane == 0) out[0] = 0u;
      continue;
    }
    if (t.pre_bits && ((t.pre_bits[i >> 5] >> (i & 31u)) & 1u)) continue;  // presplit: the full reruns'
    auto fallback = [&]() {
      if (lane == 0) t.fb[atomicAdd(&t.ctr[1], 1u)] = i;
    };
    uint32_t nign = 0, na = 0;
    const uint64_t c0 = wall_clock64();
    if (lane == 0) L.t3 = 0;
    const bool prep = decr_prepare(L, g, t, i, lane, nign, na);
    const uint64_t c1 = wall_clock64();
    if (lane == 0) {  // phase clocks: steps (0)-(2), step (3), trace; [19] the fallbacks' prepare
      uint64_t* clk = reinterpret_cast<uint64_t*>(t.ctr + 16);
      const uint64_t t3 = L.t3 ? L.t3 : c1;
      atomicAdd((unsigned long long*)&clk[prep ? 0 : 3], (unsigned long long)(t3 - c0));
      if (prep) atomicAdd((unsigned long long*)&clk[1], (unsigned long long)(c1 - t3));
    }
    if (!prep) {
      // past the map or pending-node budget: the 16-wave kernel redoes it
      // with 8x budgets and traces it from the start; past the affected-set,
      // edge or ignore-list budget (a large change, whose single-wave
      // prepare there would be slow: OSPF_KSP_SRCCUT=0 at F100k sends 7 such
      // runs and takes 58 ms): the full reruns
      if (t.budget && !t.map_fb && ((volatile uint32_t&)L.why) == 0u &&
          ((volatile uint32_t&)L.naff) <= DecrSmall::kAff) {
        if (lane == 0) {
          out[0] = 0u;
          atomicAdd(&t.ctr[2], 1u);  // (decided there; un-counted if it falls back)
          t.heavy[atomicAdd(&t.heavy_ctr[0], 1u)] = i;
        }
      } else {
        fallback();
      }
      continue;
    }
    const uint32_t dst = t.dsts[i];
    Tracer<DistDecr<DecrSmall>, DecrSmall::kHS> tr{g, t, i, lane, src, dst, L.ign, nign, L.hash, dead,
                                                   DistDecr<DecrSmall>{t.rows, &L}};
    // no paths (LinkState.cpp:808-809): src == dst, dst unreached, or the
    // source cut off by the ignored links
    if (na == kInf || dst == src || tr.dist(dst) == kInf) {
      if (lane == 0) {
        out[0] = 0u;
        atomicAdd(&t.ctr[2], 1u);
      }
      continue;
    }
    for (uint32_t k = lane; k < DecrSmall::kHS; k += kWave) tr.hs[k] = 0u;
    for (uint32_t k = lane; k < t.dead_words; k += kWave) dead[k] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    volatile uint32_t* stk = L.stack;
    uint32_t npaths = 0, w = 1, steps = 0, nclaim = 0;
    bool ovf = false, heavy = false, tier = false;
    const uint32_t budget = t.budget ? t.budget : kSteps;
    if (lane == 0) out[0] = 0u;
    while (!ovf && tr.src_open()) {
      uint32_t depth = 0;
      const int r = tr.dfs(stk, depth, 0, steps, budget);
      if (r == 0) break;
      if (r == -1 && t.budget) {  // a long failing search: resumed by 16 waves
        heavy = true;
        break;
      }
      if (r == 1 && nclaim + depth > tr.kHM && w + 1u + depth <= t.stride) {
        tier = true;  // more claimed links than this kernel's hash holds
        break;
      }
      if (r < 0 || !tr.emit(out, stk, depth, w, npaths, nclaim)) ovf = true;
      if (t.budget) steps = 0;
    }
    if (lane == 0)
      atomicAdd((unsigned long long*)(t.ctr + 16) + 2, (unsigned long long)(wall_clock64() - c1));
    if (tier) {
      if (lane == 0) atomicAdd(&t.ctr[9], 1u);
      fallback();
      continue;
    }
    if (lane == 0) {
      atomicAdd(&t.ctr[2], 1u);
      atomicAdd(&t.ctr[3], na);
    }
    if (heavy) {  // the paths so far stay in the record
      if (lane == 0) t.heavy[atomicAdd(&t.heavy_ctr[0], 1u)] = i;
      continue;
    }
    tr.finish(out, npaths, ovf, tr.hs);
  }
}

// The good set of a heavy decremental run: the nodes that still reach src
// over tight, unignored, unclaimed links through transit nodes -- the only
// predecessors a trace can complete through. Pulled level by level over the
// source's level order (the run's affected nodes at their masked levels),
// then every other node is marked dead: a failing search over a spine's
// thousands of fabric switches ends at once instead of visiting each. Dead
// marks are facts (claims only grow), so pruning never changes a path.
struct GoodPrune {
  const DevGraph& g;
  const TraceArgs& t;
  Tracer<DistDecr<DecrHeavy>, kHash>& tr;
  const DecrHeavy& L;
  HeavyLds& H;
  uint32_t* gb;   // V bits
  uint32_t* big;  // kGoodBig node ids
  __device__ bool good(uint32_t u) const {
    const uint32_t w = __hip_atomic_load(&gb[u >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return (w >> (u & 31u)) & 1u;
  }
  __device__ void set_good(uint32_t u) const {
    __hip_atomic_fetch_or(&gb[u >> 5], 1u << (u & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  // entry e of v's row: a usable pathLink from a good predecessor at level d - 1
  __device__ bool link_ok(uint32_t v, uint32_t d, uint32_t e) const {
    const uint32_t u = g.colx[e];
    if ((u & kDown) || u == v || !good(u)) return false;
    if (tr.dist(u) + 1u != d) return false;  // unit metric: tight
    const uint32_t lid = g.link_id[e];
    if (tr.ignored(lid)) return false;
    return !tr.claimed(lid);
  }
  __device__ void operator()() const {
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    const uint32_t wv = tid >> 6, lane = tid & 63u, nw = nthr >> 6;
    const uint32_t dmax = tr.dist(tr.dst);
    if (t.nlvl == 0 || dmax == kInf || dmax >= t.nlvl) return;
    const uint32_t words = (g.V + 31u) / 32u;
    const uint32_t na = ((volatile uint32_t&)L.naff) < DecrHeavy::kAff ? ((volatile uint32_t&)L.naff) : 0u;
    for (uint32_t w = tid; w < words; w += nthr) gb[w] = 0u;
    __syncthreads();
    if (tid == 0) set_good(tr.src);
    for (uint32_t d = 1; d < dmax; ++d) {
      if (tid == 0) H.nbig = 0u;
      __syncthreads();
      const uint32_t b0 = t.lvl_off[d], b1 = t.lvl_off[d + 1];
      for (uint32_t k = b0 + tid; k < b1 + na; k += nthr) {
        uint32_t v;
        if (k < b1) {
          v = t.ord[k];
          if (aff_ix(L, v) != kInf) continue;  // affected: at its masked level
        } else {
          const uint32_t q = k - b1;
          if (((const volatile uint32_t*)L.dp)[q] != d) continue;
          v = ((const volatile uint32_t*)L.aff)[q];
        }
        if ((g.nt_bits[v >> 5] >> (v & 31u)) & 1u) continue;  // never a predecessor
        const uint32_t beg = g.row_ptr[v], end = g.row_ptr[v + 1];
        if (end - beg > 256u) {  // a spine's row: one wave below
          const uint32_t j = atomicAdd(&H.nbig, 1u);
          if (j < kGoodBig) big[j] = v;
          else set_good(v);  // (no room: kept, i.e. not pruned)
          continue;
        }
        for (uint32_t e = beg; e < end; ++e)
          if (link_ok(v, d, e)) {
            set_good(v);
            break;
          }
      }
      __syncthreads();
      const uint32_t nb = min(((volatile uint32_t&)H.nbig), kGoodBig);
      for (uint32_t j = wv; j < nb; j += nw) {
        const uint32_t v = big[j];
        const uint32_t beg = g.row_ptr[v], end = g.row_ptr[v + 1];
        for (uint32_t e0 = beg; e0 < end; e0 += kWave) {
          const uint32_t e = e0 + lane;
          if (__ballot(e < end && link_ok(v, d, e))) {
            if (lane == 0) set_good(v);
            break;
          }
        }
      }
      __syncthreads();
    }
    for (uint32_t w = tid; w < words; w += nthr) {
      const uint32_t x = ~__hip_atomic_load(&gb[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (x) __hip_atomic_fetch_or(&tr.dead[w], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
  }
};

__global__ void __launch_bounds__(256) lvl_hist_kernel(const uint32_t* __restrict__ D, uint32_t V,
                                                       uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < V && D[v] < 256u) atomicAdd(&h[D[v]], 1u);
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], h[threadIdx.x]);
}
// one block: off[d] = sum of cnt[< d]; cnt becomes the scatter cursor
__global__ void __launch_bounds__(256) lvl_scan_kernel(uint32_t* cnt, uint32_t* off) {
  if (threadIdx.x == 0) {
    uint32_t a = 0;
    for (uint32_t d = 0; d < 256u; ++d) {
      off[d] = a;
      const uint32_t c = cnt[d];
      cnt[d] = a;
      a += c;
    }
    off[256] = a;
  }
}
__global__ void __launch_bounds__(256) lvl_scatter_kernel(const uint32_t* __restrict__ D, uint32_t V,
                                                          uint32_t* __restrict__ cur,
                                                          uint32_t* __restrict__ ord) {
  __shared__ uint32_t h[256], base[256];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t d = v < V ? D[v] : kInf;
  uint32_t r = 0;
  if (d < 256u) r = atomicAdd(&h[d], 1u);
  __syncthreads();
  if (h[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cur[threadIdx.x], h[threadIdx.x]);
  __syncthreads();
  if (d < 256u) ord[base[d] + r] = v;
}

// Heavy decremental runs: the block's first wave recomputes the run's
// affected set and distances (the wider budgets hold whatever the small
// kernel held), then 16 waves resume its trace (heavy_trace).
__global__ void __launch_bounds__(1024) ksp_decr_heavy_kernel(DevGraph g, TraceArgs t) {
  extern __shared__ uint4 s_raw[];
  DecrHeavy& L = *reinterpret_cast<DecrHeavy*>(s_raw);
  __shared__ HeavyLds H;
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint32_t* dead = t.dead + (size_t)blockIdx.x * t.dead_words;
  for (;;) {
    if (threadIdx.x == 0) {
      const uint32_t q = atomicAdd(&t.heavy_ctr[1], 1u);
      H.ctl[0] = q < __hip_atomic_load(&t.heavy_ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     ? t.heavy[q] : kInf;
    }
    __syncthreads();
    const uint32_t i = H.ctl[0];
    __syncthreads();
    if (i == kInf) return;
    uint32_t nign = 0, na = 0;
    const uint64_t c0 = wall_clock64();
    if (wv == 0) {
      const bool ok = decr_prepare(L, g, t, i, lane, nign, na);
      if (lane == 0) {
        H.ctl[3] = ok ? nign : kInf;
        if (!ok) {  // past these budgets too: the full reruns
          t.fb[atomicAdd(&t.ctr[1], 1u)] = i;
          atomicSub(&t.ctr[2], 1u);
        }
      }
    }
    for (uint32_t k = threadIdx.x; k < t.dead_words; k += blockDim.x) dead[k] = 0u;
    __syncthreads();
    nign = H.ctl[3];
    if (nign == kInf) continue;
    const uint64_t c1 = wall_clock64();
    Tracer<DistDecr<DecrHeavy>, kHash> tr{g, t, i, lane, t.src, t.dsts[i], L.ign, nign, L.hash, dead,
                                          DistDecr<DecrHeavy>{t.rows, &L}};
    if (t.good) {
      const GoodPrune pr{g, t, tr, L, H, t.good + (size_t)blockIdx.x * t.dead_words,
                         t.big + (size_t)blockIdx.x * kGoodBig};
      heavy_trace(g, t, i, tr, L.hash, H, pr);
    } else {
      heavy_trace(g, t, i, tr, L.hash, H);
    }
    if (threadIdx.x == 0) {  // [20] prepare, [21] trace of the heavy runs
      uint64_t* clk = reinterpret_cast<uint64_t*>(t.ctr + 16);
      const uint64_t c2 = wall_clock64();
      atomicAdd((unsigned long long*)&clk[4], (unsigned long long)(c1 - c0));
      atomicAdd((unsigned long long*)&clk[5], (unsigned long long)(c2 - c1));
      // [22] the longest heavy run (time << 24 | run), [23] runs over 1 ms
      atomicMax((unsigned long long*)&clk[6], (unsigned long long)(((c2 - c0) << 24) | (i & 0xFFFFFFu)));
      if (c2 - c0 > 100000ull) atomicAdd((unsigned long long*)&clk[7], 1ull);
      if (t.hlog) {
        unsigned long long* l = t.hlog + 4ull * (atomicAdd(&t.ctr[11], 1u) & 0xFFFFu);
        l[0] = i;
        l[1] = c0;
        l[2] = c1;
        l[3] = c2;
      }
    }
  }
}

// Runs for the full reruns from the start: ignore lists past the
// decremental kernel's, and ignore sets holding more than t.src_cut of the
// source's own links (a destination whose k = 1 paths leave through most of
// the source's links -- F100k: a plane-0 fabric switch from 2-0-0 -- cuts
// whole planes off: its affected set is the plane, past every budget)
__global__ void ksp_presplit_kernel(DevGraph g, TraceArgs t, uint32_t* list, uint32_t* count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.n) return;
  const uint32_t st = t.status[i];
  if (!(st & OSPF_KSP_RERUN) || (st & OSPF_KSP_OVF1)) return;
  const uint32_t nign = t.ign_cnt[i];
  bool split = nign > DecrSmall::kIgn;
  if (!split && t.src_cut) {
    const uint32_t* ign = t.ign + (size_t)i * t.stride;
    uint32_t at_src = 0;
    for (uint32_t k = 0; k < nign && at_src <= t.src_cut; ++k) {
      const uint32_t l = ign[k];
      if (l >= g.n_lid) continue;
      const uint32_t e0 = g.link_e[2u * l], e1 = g.link_e[2u * l + 1u];
      if (e0 == kInf || e1 == kInf) continue;
      if ((g.colx[e0] & ~kDown) == t.src || (g.colx[e1] & ~kDown) == t.src) ++at_src;
    }
    split = at_src > t.src_cut;
  }
  if (split) {
    list[atomicAdd(count, 1u)] = i;
    atomicOr(&t.pre_bits[i >> 5], 1u << (i & 31u));
  }
}

__global__ void rows_gather_kernel(uint32_t* a, const uint32_t* b, const uint32_t* idx, uint32_t n,
                                   uint32_t w, bool gather) {
  const uint32_t j = blockIdx.x;
  if (j >= n) return;
  const uint32_t r = idx[j];
  uint32_t* dst = a + (size_t)(gather ? j : r) * w;
  const uint32_t* from = b + (size_t)(gather ? r : j) * w;
  for (uint32_t k = threadIdx.x; k < w; k += blockDim.x) dst[k] = from[k];
}

__global__ void iota_kernel(uint32_t* out, uint32_t n, uint32_t stride) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= n) out[i] = i * stride;
}

__global__ void or_bits_kernel(uint32_t* st, uint32_t n, uint32_t bits) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) st[i] |= bits;
}

}  // namespace

hipError_t launch_or_bits(uint32_t* st, uint32_t n, uint32_t bits, hipStream_t s) {
  if (n) hipLaunchKernelGGL(or_bits_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, st, n, bits);
  return hipGetLastError();
}

hipError_t launch_ksp_trace(bool lev, const DevGraph& g, const TraceArgs& t, hipStream_t s) {
  if (t.n == 0) return hipSuccess;
  const dim3 grid((t.n + kWaves - 1) / kWaves);
  // the small hash when the 16-wave kernel takes the overflow and a k = 1
  // record's sort (finish: stride words of the hash) fits
  const bool small = t.budget && t.stride <= 1024u;
  if (lev && small)
    hipLaunchKernelGGL((ksp_trace_kernel<true, 1024>), grid, dim3(kBlock), 0, s, g, t);
  else if (lev)
    hipLaunchKernelGGL((ksp_trace_kernel<true, kHash>), grid, dim3(kBlock), 0, s, g, t);
  else if (small)
    hipLaunchKernelGGL((ksp_trace_kernel<false, 1024>), grid, dim3(kBlock), 0, s, g, t);
  else
    hipLaunchKernelGGL((ksp_trace_kernel<false, kHash>), grid, dim3(kBlock), 0, s, g, t);
  if (t.budget) {  // heavy runs queued by the pass above (counters zeroed by the caller)
    const dim3 hg(std::min<uint32_t>(512u, t.n));  // 2 per CU
    if (lev)
      hipLaunchKernelGGL(ksp_heavy_kernel<true>, hg, dim3(64 * kHeavyWaves), 0, s, g, t);
    else
      hipLaunchKernelGGL(ksp_heavy_kernel<false>, hg, dim3(64 * kHeavyWaves), 0, s, g, t);
  }
  return hipGetLastError();
}


hipError_t launch_ksp_hint(const DevGraph& g, uint32_t src, const uint32_t* dist, uint32_t* hint,
                           hipStream_t s) {
  hipLaunchKernelGGL(ksp_hint_kernel, dim3((g.V + 3) / 4), dim3(256), 0, s, g, src, dist, hint);
  return hipGetLastError();
}

uint32_t ksp_decr_blocks_per_cu() {
  return std::min<uint32_t>(16u, (160u * 1024u) / (uint32_t)sizeof(DecrSmall));
}

hipError_t launch_ksp_levels(const uint32_t* dist, uint32_t V, uint32_t* ord, uint32_t* off,
                             uint32_t* cnt, hipStream_t s) {
  const hipError_t e = launch_fill32(cnt, 257, 0u, s);
  if (e != hipSuccess) return e;
  const dim3 grid((V + 255) / 256);
  hipLaunchKernelGGL(lvl_hist_kernel, grid, dim3(256), 0, s, dist, V, cnt);
  hipLaunchKernelGGL(lvl_scan_kernel, dim3(1), dim3(256), 0, s, cnt, off);
  hipLaunchKernelGGL(lvl_scatter_kernel, grid, dim3(256), 0, s, dist, V, cnt, ord);
  return hipGetLastError();
}

hipError_t launch_ksp_presplit(const DevGraph& g, const TraceArgs& t, uint32_t* list, uint32_t* count,
                               hipStream_t s) {
  if (t.n == 0) return hipSuccess;
  hipLaunchKernelGGL(ksp_presplit_kernel, dim3((t.n + 255) / 256), dim3(256), 0, s, g, t, list, count);
  return hipGetLastError();
}

hipError_t launch_ksp_decr(const DevGraph& g, const TraceArgs& t, uint32_t blocks, hipStream_t s) {
  if (t.n == 0) return hipSuccess;
  hipLaunchKernelGGL(ksp_decr_kernel, dim3(blocks), dim3(kWave), 0, s, g, t);
  return hipGetLastError();
}

hipError_t launch_ksp_decr_heavy(const DevGraph& g, const TraceArgs& t, uint32_t blocks,
                                 hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)ksp_decr_heavy_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(DecrHeavy));
    attr = true;
  }
  hipLaunchKernelGGL(ksp_decr_heavy_kernel, dim3(blocks), dim3(64 * kHeavyWaves), sizeof(DecrHeavy), s,
                     g, t);
  return hipGetLastError();
}

hipError_t launch_rows_gather(uint32_t* a, const uint32_t* b, const uint32_t* idx, uint32_t n,
                              uint32_t w, bool gather, hipStream_t s) {
  if (n) hipLaunchKernelGGL(rows_gather_kernel, dim3(n), dim3(256), 0, s, a, b, idx, n, w, gather);
  return hipGetLastError();
}

hipError_t launch_iota(uint32_t* out, uint32_t n, uint32_t stride, hipStream_t s) {
  hipLaunchKernelGGL(iota_kernel, dim3(n / kBlock + 1), dim3(kBlock), 0, s, out, n, stride);
  return hipGetLastError();
}

}  // namespace ospf
