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
// (dist(u), position) keys otherwise); the path stack and the visited set (an
// open-addressing table probed 64 slots at a time) live in LDS. Distances
// come from dist rows (k = 1: the source's row; other masked reruns) or from
// the level bytes of the multi-source BFS (k = 2 reruns, spf_msbfs.hip).
// Budgets (256 links deep, 1536 links visited, the record size) end a run
// with an overflow status; the host then computes that destination itself.
#include <hip/hip_runtime.h>
#include <stdint.h>

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
constexpr uint32_t kHashMax = 1536;   // links visited per (src, dst, k)
constexpr uint32_t kSteps = 1u << 22; // DFS steps per run (termination guard)

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

template <bool LEV>
__global__ void __launch_bounds__(256) ksp_trace_kernel(DevGraph g, TraceArgs t) {
  __shared__ uint32_t s_stack[kWaves][kStack];
  __shared__ uint32_t s_hash[kWaves][kHash];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t i = blockIdx.x * kWaves + wv;
  if (i >= t.n) return;
  volatile uint32_t* stk = s_stack[wv];
  volatile uint32_t* hs = s_hash[wv];
  uint32_t* out = t.out + (size_t)i * t.stride;
  const uint32_t src = t.src, dst = t.dsts[i];

  const uint32_t* ign = nullptr;
  uint32_t nign = 0;
  if (t.k == 2) {
    const uint32_t st = t.status[i];
    if (st & OSPF_KSP_OVF1) {  // no k = 1 paths, so no ignore set: not computed
      if (lane == 0) t.status[i] = st | OSPF_KSP_OVF2;
      return;
    }
    if (!(st & OSPF_KSP_RERUN)) {  // k = 1 found nothing: neither does k = 2
      if (lane == 0) out[0] = 0u;
      return;
    }
    ign = t.ign + (size_t)i * t.stride;
    nign = min(t.ign_cnt[i], t.stride);
  }
  auto finish_k1 = [&](uint32_t npaths, uint32_t m, bool ovf) {
    if (t.k != 1) return;
    if (lane == 0) {
      t.cnt_out[i] = ovf ? 0u : m;
      t.status[i] = ovf ? OSPF_KSP_OVF1 : (m ? OSPF_KSP_RERUN : 0u);
    }
  };

  const uint32_t ddst = dist_of<LEV>(g, t, i, dst);
  if (dst == src || ddst == kInf) {  // LinkState.cpp:808-809: no paths
    if (lane == 0) out[0] = 0u;
    if (t.ign_out)
      for (uint32_t k = lane; k < t.stride; k += kWave) t.ign_out[(size_t)i * t.stride + k] = kInf;
    finish_k1(0, 0, false);
    return;
  }
  for (uint32_t k = lane; k < kHash; k += kWave) hs[k] = 0u;

  // pathLinks entry e of row v? (u = colx[e] its predecessor, du its dist)
  auto tight = [&](uint32_t v, uint32_t dv, uint32_t e, uint32_t& du) -> bool {
    const uint32_t cx = g.colx[e];
    if (cx & kDown) return false;
    if (cx == v) return false;
    du = dist_of<LEV>(g, t, i, cx);
    if (du == kInf) return false;
    const uint32_t w = t.unit ? 1u : g.rw[e];
    if ((uint64_t)du + w != dv) return false;
    if (cx != src && ((g.nt_bits[cx >> 5] >> (cx & 31u)) & 1u)) return false;
    if (nign && in_sorted(ign, nign, g.link_id[e])) return false;
    return true;
  };
  // smallest candidate key (du << 32 | e) >= lo among v's pathLinks, ~0 = none
  auto next_cand = [&](uint32_t v, uint32_t dv, uint64_t lo) -> uint64_t {
    const uint32_t beg = g.row_ptr[v], end = g.row_ptr[v + 1];
    if (t.unit) {  // every candidate has du = dv - 1: row order
      const uint32_t e0 = lo ? max(beg, (uint32_t)lo) : beg;
      for (uint32_t base = e0; base < end; base += kWave) {
        const uint32_t e = base + lane;
        uint32_t du = 0;
        const bool ok = e < end && tight(v, dv, e, du);
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
      if (!tight(v, dv, e, du)) continue;
      const uint64_t key = ((uint64_t)du << 32) | e;
      if (key >= lo && key < best) best = key;
    }
    return wave_min64(best);
  };
  uint32_t nvis = 0;
  // visited.insert(link).second (LinkState.cpp:430)
  auto claim = [&](uint32_t lid) -> bool {
    const uint32_t key = lid + 1u;
    const uint32_t h = (uint32_t)(((uint64_t)lid * 0x9E3779B97F4A7C15ull) >> 40);
    for (uint32_t p0 = 0;; p0 += kWave) {
      const uint32_t slot = (h + p0 + lane) & (kHash - 1u);
      const uint32_t x = hs[slot];
      if (__ballot(x == key)) return false;
      const uint64_t em = __ballot(x == 0u);
      if (em) {
        if (lane == (uint32_t)(__ffsll((unsigned long long)em) - 1)) hs[slot] = key;
        ++nvis;
        return true;
      }
    }
  };

  uint32_t npaths = 0, w = 1, steps = 0;
  bool ovf = false;
  for (;;) {  // one traceOnePath per iteration, until it fails
    uint32_t depth = 0, v = dst, dv = ddst;
    uint64_t lo = 0;
    bool found = false;
    while (!ovf) {
      if (v == src) {
        found = true;
        break;
      }
      if (++steps > kSteps) {
        ovf = true;
        break;
      }
      const uint64_t key = next_cand(v, dv, lo);
      if (key == ~0ull) {  // v's pathLinks are exhausted: back to its successor
        if (depth == 0) break;
        const uint32_t pe = stk[--depth];
        v = depth ? g.colx[stk[depth - 1]] : dst;
        dv = dist_of<LEV>(g, t, i, v);
        lo = (((uint64_t)dist_of<LEV>(g, t, i, g.colx[pe])) << 32 | pe) + 1ull;
        continue;
      }
      lo = key + 1ull;
      const uint32_t e = (uint32_t)key;
      if (!claim(g.link_id[e])) continue;
      if (nvis > kHashMax || depth == kStack) {
        ovf = true;
        break;
      }
      stk[depth++] = e;
      v = g.colx[e];
      dv = (uint32_t)(key >> 32);
      lo = 0;
    }
    if (ovf || !found) break;
    if (w + 1u + depth > t.stride) {
      ovf = true;
      break;
    }
    // path from src to dst: the stack bottom-up is dst -> src
    for (uint32_t k = lane; k < depth; k += kWave) out[w + 1u + k] = g.link_id[stk[depth - 1u - k]];
    if (lane == 0) out[w] = depth;
    w += 1u + depth;
    ++npaths;
  }
  if (lane == 0) out[0] = ovf ? 0u : npaths;
  if (t.k == 2) {
    if (ovf && lane == 0) t.status[i] |= OSPF_KSP_OVF2;
    return;
  }
  // k = 1: the links of the paths, sorted = the k = 2 rerun's ignore set
  // (LinkState.cpp:797-803); edge-disjoint paths, so no duplicates
  uint32_t m = 0;
  if (!ovf) {
    __threadfence_block();  // the record's words, written by other lanes
    for (uint32_t p = 0, q = 1; p < npaths; ++p) {
      const uint32_t len = out[q];
      for (uint32_t k = lane; k < len; k += kWave) hs[m + k] = out[q + 1u + k];
      m += len;
      q += 1u + len;
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t* io = t.ign_out + (size_t)i * t.stride;
    for (uint32_t j = lane; j < m; j += kWave) {
      const uint32_t x = hs[j];
      uint32_t rank = 0;
      for (uint32_t k = 0; k < m; ++k) rank += hs[k] < x ? 1u : 0u;
      io[rank] = x;
    }
    for (uint32_t k = m + lane; k < t.stride; k += kWave) io[k] = kInf;
  } else {
    for (uint32_t k = lane; k < t.stride; k += kWave) t.ign_out[(size_t)i * t.stride + k] = kInf;
  }
  finish_k1(npaths, m, ovf);
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
  return hipGetLastError();
}

hipError_t launch_iota(uint32_t* out, uint32_t n, uint32_t stride, hipStream_t s) {
  hipLaunchKernelGGL(iota_kernel, dim3(n / kBlock + 1), dim3(kBlock), 0, s, out, n, stride);
  return hipGetLastError();
}

}  // namespace ospf
