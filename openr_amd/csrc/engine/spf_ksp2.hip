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
//  * lookahead. A candidate predecessor with a short row (<= kLook entries)
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
constexpr uint32_t kHashMax = 1536;   // links of the paths of one (src, dst, k)
constexpr uint32_t kSteps = 1u << 22; // DFS steps per run (termination guard)
constexpr uint32_t kLook = 16;        // lookahead row length limit

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

template <bool LEV>
__device__ __forceinline__ uint32_t dist_of(const DevGraph& g, const TraceArgs& t, uint32_t i,
                                            uint32_t u) {
  if (LEV) {
    const uint32_t l = t.lev[((size_t)(i >> 6) * g.V + u) * 64u + (i & 63u)];
    return l ? l - 1u : kInf;
  }
  return t.rows[(size_t)i * t.row_stride + u];
}

// the DFS of one run (one wave); see the file comment
template <bool LEV>
struct Tracer {
  const DevGraph& g;
  const TraceArgs& t;
  uint32_t i, lane, src, dst;
  const uint32_t* ign;
  uint32_t nign;
  volatile uint32_t* hs;  // claimed links (the paths found), kHash slots
  uint32_t* dead;

  __device__ uint32_t dist(uint32_t u) const { return dist_of<LEV>(g, t, i, u); }
  __device__ static uint32_t hslot(uint32_t lid) {
    return (uint32_t)(((uint64_t)lid * 0x9E3779B97F4A7C15ull) >> 40);
  }
  __device__ bool claimed(uint32_t lid) const {  // per lane
    for (uint32_t h = hslot(lid);; ++h) {
      const uint32_t x = hs[h & (kHash - 1u)];
      if (x == lid + 1u) return true;
      if (x == 0u) return false;
    }
  }
  __device__ void claim(uint32_t lid) const {  // wave-uniform lid, not yet claimed
    const uint32_t h = hslot(lid);
    for (uint32_t p0 = 0;; p0 += kWave) {
      const uint32_t slot = (h + p0 + lane) & (kHash - 1u);
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
  // pathLinks entry e of row v, not claimed, predecessor not dead?
  __device__ bool cand(uint32_t v, uint32_t dv, uint32_t e, uint32_t& du) const {
    const uint32_t cx = g.colx[e];
    if (cx & kDown) return false;
    if (cx == v) return false;
    du = dist(cx);
    if (du == kInf) return false;
    const uint32_t w = t.unit ? 1u : g.rw[e];
    if ((uint64_t)du + w != dv) return false;
    if (cx != src && ((g.nt_bits[cx >> 5] >> (cx & 31u)) & 1u)) return false;
    const uint32_t lid = g.link_id[e];
    if (nign && in_sorted(ign, nign, lid)) return false;
    if (cx == src) return !claimed(lid);
    if (is_dead(cx) || claimed(lid)) return false;
    // one level of lookahead on short rows: a predecessor without an open
    // pathLink of its own fails at once when entered, i.e. it is dead
    const uint32_t b2 = g.row_ptr[cx], e2end = g.row_ptr[cx + 1];
    if (e2end - b2 > kLook) return true;
    for (uint32_t e2 = b2; e2 < e2end; ++e2) {
      const uint32_t c2 = g.colx[e2];
      if ((c2 & kDown) || c2 == cx) continue;
      const uint32_t d2 = dist(c2);
      if (d2 == kInf || (uint64_t)d2 + (t.unit ? 1u : g.rw[e2]) != du) continue;
      if (c2 != src && ((g.nt_bits[c2 >> 5] >> (c2 & 31u)) & 1u)) continue;
      const uint32_t l2 = g.link_id[e2];
      if (nign && in_sorted(ign, nign, l2)) continue;
      if (c2 != src && is_dead(c2)) continue;
      if (!claimed(l2)) return true;
    }
    mark_dead(cx);
    return false;
  }
  // smallest candidate key (du << 32 | e) >= lo among v's pathLinks, ~0 = none
  __device__ uint64_t next_cand(uint32_t v, uint32_t dv, uint64_t lo) const {
    const uint32_t beg = g.row_ptr[v], end = g.row_ptr[v + 1];
    if (t.unit) {  // every candidate has du = dv - 1: row order
      const uint32_t e0 = lo ? max(beg, (uint32_t)lo) : beg;
      for (uint32_t base = e0; base < end; base += kWave) {
        const uint32_t e = base + lane;
        uint32_t du = 0;
        const bool ok = e < end && cand(v, dv, e, du);
        const uint64_t bal = __ballot(ok);
        if (bal) {
          const uint32_t eb = base + (uint32_t)(__ffsll((unsigned long long)bal) - 1);
          return ((uint64_t)(dv - 1u) << 32) | eb;
        }
      }
      return ~0ull;
    }
    uint64_t best = ~0ull;
    for (uint32_t e = beg + lane; e < end; e += kWave) {
      uint32_t du = 0;
      if (!cand(v, dv, e, du)) continue;
      const uint64_t key = ((uint64_t)du << 32) | e;
      if (key >= lo && key < best) best = key;
    }
    return wave_min64(best);
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
      if (nign && in_sorted(ign, nign, lid)) continue;
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
    if (w + 1u + depth > t.stride || nclaim + depth > kHashMax) return false;
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
template <bool LEV>
__device__ bool trace_setup(const DevGraph& g, const TraceArgs& t, uint32_t i, uint32_t lane,
                            Tracer<LEV>& tr) {
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
template <bool LEV>
__global__ void __launch_bounds__(256) ksp_trace_kernel(DevGraph g, TraceArgs t) {
  __shared__ uint32_t s_stack[kWaves][kStack];
  __shared__ uint32_t s_hash[kWaves][kHash];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t i = blockIdx.x * kWaves + wv;
  if (i >= t.n) return;
  volatile uint32_t* stk = s_stack[wv];
  Tracer<LEV> tr{g, t, i, lane, t.src, t.dsts[i], nullptr, 0, s_hash[wv],
                 t.dead + (size_t)i * t.dead_words};
  if (!trace_setup<LEV>(g, t, i, lane, tr)) return;
  for (uint32_t k = lane; k < kHash; k += kWave) tr.hs[k] = 0u;
  uint32_t* out = t.out + (size_t)i * t.stride;
  uint32_t npaths = 0, w = 1, steps = 0, nclaim = 0;
  bool ovf = false;
  const uint32_t budget = t.budget ? t.budget : kSteps;
  if (lane == 0) out[0] = 0u;
  while (!ovf && tr.src_open()) {  // one traceOnePath per iteration, until it fails
    uint32_t depth = 0;
    const int r = tr.dfs(stk, depth, 0, steps, budget);
    if (r == 0) break;
    if (r == -1 && t.budget) {  // heavy: the paths so far stay in the record
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
template <bool LEV>
__global__ void __launch_bounds__(1024) ksp_heavy_kernel(DevGraph g, TraceArgs t) {
  __shared__ uint32_t s_hash[kHash];
  __shared__ uint32_t s_stack[kHeavyWaves][kStack];
  __shared__ uint64_t s_cand[kHeavyWaves];
  __shared__ int32_t s_res[kHeavyWaves];
  __shared__ uint32_t s_ctl[4];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  for (;;) {
    if (threadIdx.x == 0) {
      const uint32_t q = atomicAdd(&t.heavy_ctr[1], 1u);
      s_ctl[0] = q < __hip_atomic_load(&t.heavy_ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     ? t.heavy[q] : kInf;
    }
    __syncthreads();
    const uint32_t i = s_ctl[0];
    if (i == kInf) return;
    uint32_t* out = t.out + (size_t)i * t.stride;
    Tracer<LEV> tr{g, t, i, lane, t.src, t.dsts[i], nullptr, 0, s_hash,
                   t.dead + (size_t)i * t.dead_words};
    trace_setup<LEV>(g, t, i, lane, tr);  // (a queued run always has work)
    for (uint32_t k = threadIdx.x; k < kHash; k += blockDim.x) s_hash[k] = 0u;
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
    bool ovf = false;
    uint32_t steps = 0;
    for (;;) {  // one traceOnePath per iteration
      if (wv == 0) s_ctl[1] = tr.src_open() ? 1u : 0u;
      __syncthreads();
      if (!s_ctl[1]) break;
      uint64_t lo = 0;
      int winner = -1;
      bool stop = false;
      for (;;) {  // dst's candidates, 16 at a time
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
            if (ok && rank < kHeavyWaves) s_cand[rank] = ((uint64_t)(dv - 1u) << 32) | e;
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
          s_ctl[2] = m;
        }
        __syncthreads();
        const uint32_t m = s_ctl[2];
        if (m == 0) {
          stop = true;
          break;
        }
        if (wv < m) {
          uint32_t depth = 1, st2 = 0;
          s_stack[wv][0] = (uint32_t)s_cand[wv];
          const int r = tr.dfs(s_stack[wv], depth, 1, st2, kSteps);
          if (lane == 0) s_res[wv] = r == 1 ? (int32_t)depth : (r < 0 ? -1 : 0);
        }
        __syncthreads();
        uint32_t k = 0;
        for (; k < m; ++k)
          if (s_res[k] != 0) break;
        if (k < m) {
          if (s_res[k] < 0) ovf = true;
          else winner = (int)k;
          break;
        }
      }
      __syncthreads();
      if (ovf || stop || winner < 0) break;
      if (wv == 0 && !tr.emit(out, s_stack[winner], (uint32_t)s_res[winner], w, npaths, nclaim))
        s_ctl[3] = 1u;
      else if (wv == 0)
        s_ctl[3] = 0u;
      __syncthreads();
      if (s_ctl[3]) {
        ovf = true;
        break;
      }
      if (++steps > kSteps) {
        ovf = true;
        break;
      }
    }
    __syncthreads();
    if (wv == 0) tr.finish(out, npaths, ovf, s_hash);
    __syncthreads();
  }
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
  if (lev)
    hipLaunchKernelGGL(ksp_trace_kernel<true>, grid, dim3(kBlock), 0, s, g, t);
  else
    hipLaunchKernelGGL(ksp_trace_kernel<false>, grid, dim3(kBlock), 0, s, g, t);
  if (t.budget) {  // heavy runs queued by the pass above (counters zeroed by the caller)
    const dim3 hg(std::min<uint32_t>(512u, t.n));  // 2 per CU
    if (lev)
      hipLaunchKernelGGL(ksp_heavy_kernel<true>, hg, dim3(64 * kHeavyWaves), 0, s, g, t);
    else
      hipLaunchKernelGGL(ksp_heavy_kernel<false>, hg, dim3(64 * kHeavyWaves), 0, s, g, t);
  }
  return hipGetLastError();
}

hipError_t launch_iota(uint32_t* out, uint32_t n, uint32_t stride, hipStream_t s) {
  hipLaunchKernelGGL(iota_kernel, dim3(n / kBlock + 1), dim3(kBlock), 0, s, out, n, stride);
  return hipGetLastError();
}

}  // namespace ospf
