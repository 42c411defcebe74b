// spf_update.hip — incremental updates of the resident graph and the
// affected-run test (include/openr_spf.h: ospf_update_links,
// ospf_affected_roots).
//
// The reference recomputes every SPF after a topology change (LinkState
// clears spfResults_, openr/decision/LinkState.cpp:751-754; Decision rebuilds
// routes per debounced batch, Decision.cpp:918-996). A run of root r is
// unchanged by a batch that only changes link metrics / up state / overload
// bits when no changed link is on r's shortest-path DAG before the batch and
// none reaches or ties a shortest distance after it; runSpf's result (dist,
// nextHops, pathLinks, LinkState.cpp:836-911) is then bit-identical, so only
// the flagged runs need to be re-run.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdint.h>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;

__global__ void scatter_kernel(uint32_t* base, const uint32_t* idx, const uint32_t* val,
                               uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) base[idx[i]] = val[i];
}

__global__ void shift_add_kernel(uint32_t* a, uint32_t n, uint32_t from, uint32_t thresh,
                                 uint32_t d) {
  const uint32_t i = from + blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint32_t x = a[i];
    if (x != 0xFFFFFFFFu && x >= thresh) a[i] = x + d;
  }
}

// can `x`'s relaxations matter to the run whose distance row is `d`?
__device__ bool node_matters(const DevGraph& g, const uint32_t* d, uint32_t x, bool hop) {
  const uint32_t dx = d[x];
  if (dx == kInf || dx == 0) return false;  // unreached, or the root (always relaxes)
  for (uint32_t e = g.row_ptr[x]; e < g.row_ptr[x + 1]; ++e) {
    const uint32_t cx = g.colx[e];
    if (cx & kDown) continue;
    const uint64_t nd = (uint64_t)dx + (hop ? 1u : g.w[e]);
    if (nd <= d[cx]) return true;
  }
  return false;
}

__global__ void affected_kernel(DevGraph g, const uint32_t* dist, uint32_t n_roots, uint32_t hop,
                                const ospf_change* ch, uint32_t n_ch, uint8_t* out) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_roots) return;
  const uint32_t* d = dist + (size_t)r * g.V;
  uint8_t hit = 0;
  for (uint32_t k = 0; k < n_ch && !hit; ++k) {
    const ospf_change c = ch[k];
    if (c.kind == OSPF_CHANGE_NODE) {
      hit = node_matters(g, d, c.a, hop != 0);
      continue;
    }
    const uint64_t da = d[c.a], db = d[c.b];
    const uint64_t w0ab = hop ? 1 : c.w_ab0, w0ba = hop ? 1 : c.w_ba0;
    const uint64_t w1ab = hop ? 1 : c.w_ab1, w1ba = hop ? 1 : c.w_ba1;
    // tight before (its head's dist / next hops / pathLinks used it)
    if (c.up0 && da != kInf && da + w0ab == db) hit = 1;
    if (c.up0 && db != kInf && db + w0ba == da) hit = 1;
    // shortens or ties a distance after
    if (c.up1 && da != kInf && da + w1ab <= db) hit = 1;
    if (c.up1 && db != kInf && db + w1ba <= da) hit = 1;
  }
  out[r] = hit;
}

// ---------------------------------------------------------------- repair
// In-place repair of a finished run's rows after a patch when no shortest
// distance changes (the common case of a link event in an ECMP fabric: a
// rack's uplink fails, every remote root loses one next hop to that rack and
// nothing else). One wave per run:
//  1. every changed link direction u -> v whose tightness for this run
//     changes (was tight and is not, or became tight) re-derives v: the
//     minimum over v's usable in-edges from reached transit nodes must still
//     be dist(v) (else the run is flagged for a re-run), and v's next hops
//     are pulled again (LinkState.cpp:885-901);
//     an overload toggle of node x re-derives every tight successor of x;
//  2. a node whose next hops changed re-derives its tight successors, in
//     increasing distance order (an LDS min-heap), so every pull reads final
//     predecessor words.
// A dropped or shortened distance, more than kPops re-derivations, or a full
// heap flag the run (status 1).
// Any next-hop width: words are re-derived 8 at a time.
constexpr uint32_t kRWaves = 4;
constexpr uint32_t kHeapCap = 1024;
constexpr uint32_t kPops = 8192;

__device__ __forceinline__ uint32_t wmin(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o, 64));
  return x;
}
__device__ __forceinline__ uint32_t wor(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, 64);
  return x;
}

__global__ void __launch_bounds__(256) repair_kernel(DevGraph g, RepairArgs a) {
  __shared__ uint64_t s_heap[kRWaves][kHeapCap];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t i = blockIdx.x * kRWaves + wv;
  if (i >= a.n) return;
  volatile uint64_t* heap = s_heap[wv];
  const uint32_t root = a.roots[i], V = g.V, W = a.W;
  uint32_t* D = a.dist + (size_t)i * V;
  uint32_t* H = a.nh + (size_t)i * V * W;
  const uint32_t nb0 = g.dn_off[root], nbn = g.dn_off[root + 1] - nb0;
  auto transit = [&](uint32_t x) {
    return x == root || !((g.nt_bits[x >> 5] >> (x & 31u)) & 1u);
  };
  // re-derive y: 0 unchanged, 1 next hops changed, 2 its distance would
  // change. Words go 8 at a time (one in-edge scan per group of 8 words).
  auto rederive = [&](uint32_t y) -> int {
    if (y == root) return 0;
    const uint32_t dy = D[y];
    bool changed = false;
    for (uint32_t w0 = 0; w0 < W; w0 += 8) {
      uint32_t best = kInf, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (uint32_t e = g.row_ptr[y] + lane; e < g.row_ptr[y + 1]; e += 64) {
        const uint32_t x = g.colx[e];
        if ((x & kDown) || x == y) continue;
        const uint32_t dx = D[x];
        if (dx == kInf || !transit(x)) continue;
        const uint64_t c = (uint64_t)dx + (a.hop ? 1u : g.rw[e]);
        if (c < best) best = (uint32_t)min<uint64_t>(c, kInf - 1);
        if (c != dy) continue;
        if (x == root) {
          uint32_t lo = 0, hi = nbn;
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (g.dn[nb0 + mid] < y) lo = mid + 1; else hi = mid;
          }
#pragma unroll
          for (uint32_t j = 0; j < 8; ++j)
            if ((lo >> 5) == w0 + j) acc[j] |= 1u << (lo & 31u);
        } else {
#pragma unroll
          for (uint32_t j = 0; j < 8; ++j)
            if (w0 + j < W) acc[j] |= H[(size_t)x * W + w0 + j];
        }
      }
      if (w0 == 0 && wmin(best) != dy) return 2;
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        if (w0 + j >= W) break;
        const uint32_t v = wor(acc[j]);
        changed |= v != H[(size_t)y * W + w0 + j];
        if (lane == 0) H[(size_t)y * W + w0 + j] = v;
      }
    }
    __threadfence_block();
    return changed ? 1 : 0;
  };
  uint32_t hn = 0;
  bool bail = false;
  auto push = [&](uint32_t y) {  // lane 0 owns the heap; hn is wave-uniform
    if (hn == kHeapCap) {
      bail = true;
      return;
    }
    if (lane == 0) {
      const uint64_t key = ((uint64_t)D[y] << 32) | y;
      uint32_t k = hn;
      while (k > 0 && heap[(k - 1) / 2] > key) {
        heap[k] = heap[(k - 1) / 2];
        k = (k - 1) / 2;
      }
      heap[k] = key;
    }
    ++hn;
  };
  auto pop = [&]() -> uint32_t {
    uint32_t top = 0;
    if (lane == 0) {
      top = (uint32_t)heap[0];
      const uint64_t last = heap[hn - 1];
      uint32_t k = 0, n2 = hn - 1;
      for (;;) {
        uint32_t c = 2 * k + 1;
        if (c >= n2) break;
        if (c + 1 < n2 && heap[c + 1] < heap[c]) ++c;
        if (heap[c] >= last) break;
        heap[k] = heap[c];
        k = c;
      }
      if (n2) heap[k] = last;
    }
    --hn;
    return __shfl((int)top, 0, 64);
  };
  for (uint32_t k = 0; k < a.n_ch && !bail; ++k) {
    const ospf_change c = a.ch[k];
    if (c.kind == OSPF_CHANGE_NODE) {
      // an overload toggle of x changes the usable relaxations x -> y: a
      // transit x may now shorten a distance (flag) or add a tight in-edge,
      // a non-transit x may have dropped one; every tight successor of x is
      // re-derived (from the current transit bits, whatever x's old state)
      const uint32_t x = c.a;
      const uint32_t dx = D[x];
      if (x == root || dx == kInf) continue;
      const bool tr = transit(x);
      for (uint32_t e0 = g.row_ptr[x]; e0 < g.row_ptr[x + 1] && !bail; e0 += 64) {
        const uint32_t e = e0 + lane;
        bool tight = false, shorter = false;
        uint32_t y = 0;
        if (e < g.row_ptr[x + 1]) {
          y = g.colx[e];
          if (!(y & kDown) && y != x) {
            const uint64_t nd = (uint64_t)dx + (a.hop ? 1u : g.w[e]);
            shorter = tr && nd < D[y];
            tight = D[y] != kInf && nd == D[y];
          }
        }
        if (__ballot(shorter)) {
          bail = true;
          break;
        }
        uint64_t m = __ballot(tight);
        while (m && !bail) {
          const int l = __ffsll((unsigned long long)m) - 1;
          m &= m - 1;
          const uint32_t ys = __shfl((int)y, l, 64);
          const int r = rederive(ys);
          if (r == 2) bail = true;
          else if (r == 1) push(ys);
        }
      }
      continue;
    }
    for (int dir = 0; dir < 2 && !bail; ++dir) {
      const uint32_t u = dir ? c.b : c.a, v = dir ? c.a : c.b;
      const uint64_t w0 = a.hop ? 1 : (dir ? c.w_ba0 : c.w_ab0);
      const uint64_t w1 = a.hop ? 1 : (dir ? c.w_ba1 : c.w_ab1);
      const uint64_t du = D[u], dv = D[v];
      if (du == kInf || !transit(u)) continue;
      if (c.up1 && du + w1 < dv) {  // a shorter distance
        bail = true;
        break;
      }
      const bool t0 = c.up0 && du + w0 == dv, t1 = c.up1 && du + w1 == dv;
      if (t0 == t1) continue;
      const int r = rederive(v);
      if (r == 2) bail = true;
      else if (r == 1) push(v);
    }
  }
  for (uint32_t pops = 0; hn && !bail; ++pops) {
    if (pops == kPops) {
      bail = true;
      break;
    }
    const uint32_t x = pop();
    if (!transit(x)) continue;
    const uint32_t dx = D[x];
    for (uint32_t e0 = g.row_ptr[x]; e0 < g.row_ptr[x + 1] && !bail; e0 += 64) {
      const uint32_t e = e0 + lane;
      bool succ = false;
      uint32_t y = 0;
      if (e < g.row_ptr[x + 1]) {
        y = g.colx[e];
        succ = !(y & kDown) && y != x && D[y] != kInf &&
               (uint64_t)dx + (a.hop ? 1u : g.w[e]) == D[y];
      }
      uint64_t m = __ballot(succ);
      while (m && !bail) {  // successors one by one (wave-wide re-derivations)
        const int l = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const uint32_t ys = __shfl((int)y, l, 64);
        const int r = rederive(ys);
        if (r == 2) bail = true;
        else if (r == 1) push(ys);
      }
    }
  }
  if (lane == 0) a.status[i] = bail ? 1u : 0u;
}

}  // namespace

hipError_t launch_repair(const DevGraph& g, const RepairArgs& a, hipStream_t s) {
  if (a.n)
    hipLaunchKernelGGL(repair_kernel, dim3((a.n + kRWaves - 1) / kRWaves), dim3(64 * kRWaves), 0,
                       s, g, a);
  return hipGetLastError();
}

hipError_t launch_scatter(uint32_t* base, const uint32_t* idx, const uint32_t* val, uint32_t n,
                          hipStream_t s) {
  if (n) hipLaunchKernelGGL(scatter_kernel, dim3((n + 255) / 256), dim3(256), 0, s, base, idx, val, n);
  return hipGetLastError();
}

__global__ void fill32_kernel(uint32_t* a, size_t n, uint32_t v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = v;
}

hipError_t launch_fill32(uint32_t* a, size_t n, uint32_t v, hipStream_t s) {
  if (n) {
    const size_t blocks = std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(fill32_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a, n, v);
  }
  return hipGetLastError();
}

hipError_t launch_shift_add(uint32_t* a, uint32_t n, uint32_t from, uint32_t thresh, uint32_t d,
                            hipStream_t s) {
  if (n > from)
    hipLaunchKernelGGL(shift_add_kernel, dim3((n - from + 255) / 256), dim3(256), 0, s, a, n, from,
                       thresh, d);
  return hipGetLastError();
}

hipError_t launch_affected(const DevGraph& g, const uint32_t* dist, uint32_t n_roots, bool hop,
                           const ospf_change* ch, uint32_t n_ch, uint8_t* out, hipStream_t s) {
  if (n_roots)
    hipLaunchKernelGGL(affected_kernel, dim3((n_roots + 255) / 256), dim3(256), 0, s, g, dist,
                       n_roots, hop ? 1u : 0u, ch, n_ch, out);
  return hipGetLastError();
}

}  // namespace ospf
