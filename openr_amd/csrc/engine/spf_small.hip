// spf_small.hip — all-sources SPF of small graphs in ONE launch (gfx950):
// a wave per root, the graph and every root's BFS state resident in LDS.
//
// LinkState::runSpf (openr/decision/LinkState.cpp:836-911) with unit weights
// (every usable metric 1, or useLinkMetric = false): the (dist, name) settle
// order degenerates to BFS levels; a node at level d + 1 takes the next hops
// of its usable in-edges from transit nodes at level d (:885-901); overloaded
// nodes never relay, the root always does (:859-866); a direct neighbour n_k
// of the root is its own next hop (bit k = its rank among the root's
// distinct neighbours).
//
// Why a wave per root. A 1,000-node grid has diameter 60: a level-synchronous
// multi-root traversal pays ~120 dependent launches per sweep and a
// workgroup-per-root BFS two block barriers per level; the output (8 B per
// (root, node)) is a few MB. Here a block copies the padded CSR into LDS
// once and each of its waves sweeps its own roots: frontier queue, visited
// bitmap, u16 levels and next-hop words of the root in the wave's LDS slice,
// no barrier but the wave's own. Per level: a push over the frontier's quads
// claims unvisited heads with LDS atomics (ballot-compacted appends to the
// queue), then a pull over the claimed nodes ORs the next hops of their
// in-neighbours at level d (no atomics). The rows leave with one coalesced
// pass per root, the digest folded in.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int o) {
  const uint32_t lo = __shfl_xor((uint32_t)x, o, 64);
  const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), o, 64);
  return ((uint64_t)hi << 32) | lo;
}
// LDS accesses of this wave before the call are complete and visible to its
// later ones (the compiler may not move LDS operations across it)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ uint32_t below(uint64_t m, uint32_t lane) {
  return (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

template <int W>
__global__ void __launch_bounds__(256) lds_sweep_kernel(DevGraph g, SmallArgs a) {
  extern __shared__ uint32_t s_mem[];
  const uint32_t V = g.V, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const SmallLayout L = small_layout(V, a.Ep, W);
  uint32_t* rp = s_mem;
  uint32_t* cx = rp + L.rp_words;
  uint32_t* nt = cx + a.Ep;
  for (uint32_t x = tid; x <= V; x += blockDim.x) rp[x] = g.row_ptr[x];
  for (uint32_t x = tid; x < a.Ep / 4u; x += blockDim.x)
    reinterpret_cast<uint4*>(cx)[x] = reinterpret_cast<const uint4*>(g.colx)[x];
  for (uint32_t x = tid; x < L.nt_words; x += blockDim.x) nt[x] = x < (V + 31u) / 32u ? g.nt_bits[x] : 0u;
  __syncthreads();
  uint32_t* vis = s_mem + L.graph_words + wave * L.wave_words;
  uint16_t* lev = reinterpret_cast<uint16_t*>(vis + L.vis_words);
  uint16_t* q = reinterpret_cast<uint16_t*>(vis + L.vis_words + L.half_words);
  uint32_t* nh = vis + L.vis_words + 2u * L.half_words;
  auto transit = [&](uint32_t u) { return !((nt[u >> 5] >> (u & 31u)) & 1u); };
  auto seen = [&](uint32_t u) { return (vis[u >> 5] >> (u & 31u)) & 1u; };
  // claim u for this wave's root: true for exactly one claimant
  auto claim = [&](uint32_t u) {
    const uint32_t b = 1u << (u & 31u);
    return !(atomicOr(&vis[u >> 5], b) & b);
  };

  for (uint32_t i = blockIdx.x * a.waves + wave; i < a.n; i += gridDim.x * a.waves) {
    const uint32_t s = a.roots[i];
    if (s >= V) {
      if (lane == 0) atomicOr(a.err, 64u);
      continue;
    }
    for (uint32_t x = lane; x < L.vis_words; x += 64u) vis[x] = 0u;
    for (uint32_t x = lane; x < V * W; x += 64u) nh[x] = 0u;
    wave_sync();
    if (lane == 0) {
      vis[s >> 5] |= 1u << (s & 31u);
      lev[s] = 0;
      q[0] = (uint16_t)s;
    }
    wave_sync();
    uint32_t tail = 1;
    // level 1: the root's usable links, next hop = the neighbour's slot bit
    {
      const uint32_t b = rp[s], e = rp[s + 1];
      for (uint32_t base = b; base < e; base += 64u) {
        const uint32_t ei = base + lane;
        const uint32_t x = ei < e ? cx[ei] : kDown;
        const bool ok = !(x & kDown) && x != s;
        bool nw = false;
        if (ok) {
          const uint32_t k = g.didx[ei];
          if (k < 32u * W) atomicOr(&nh[x * W + (k >> 5)], 1u << (k & 31u));
          else atomicOr(a.err, 1u);
          nw = claim(x);
        }
        const uint64_t bal = __ballot(nw);
        if (nw) {
          q[tail + below(bal, lane)] = (uint16_t)x;
          lev[x] = 1;
        }
        tail += (uint32_t)__popcll(bal);
      }
    }
    wave_sync();
    uint32_t qb = 1, d = 1;
    while (qb < tail) {
      const uint32_t qe = tail;
      // push: the transit frontier claims its unvisited heads (level d + 1)
      for (uint32_t base = qb; base < qe; base += 64u) {
        const uint32_t j = base + lane;
        uint32_t b = 0, e = 0;
        if (j < qe) {
          const uint32_t u = q[j];
          if (transit(u)) {
            b = rp[u];
            e = rp[u + 1];
          }
        }
        while (__ballot(b < e)) {
          uint4 c = make_uint4(kDown, kDown, kDown, kDown);
          if (b < e) {
            c = *reinterpret_cast<const uint4*>(cx + b);
            b += 4u;
          }
          const uint32_t cs[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const uint32_t x = cs[t];
            const bool nw = !(x & kDown) && claim(x);
            const uint64_t bal = __ballot(nw);
            if (nw) {
              q[tail + below(bal, lane)] = (uint16_t)x;
              lev[x] = (uint16_t)(d + 1u);
            }
            tail += (uint32_t)__popcll(bal);
          }
        }
      }
      wave_sync();
      // pull: next hops of the claimed nodes from their in-neighbours at level d
      for (uint32_t base = qe; base < tail; base += 64u) {
        const uint32_t j = base + lane;
        if (j >= tail) continue;
        const uint32_t x = q[j];
        uint32_t acc[W];
#pragma unroll
        for (int w = 0; w < W; ++w) acc[w] = 0u;
        const uint32_t e = rp[x + 1];
        for (uint32_t b = rp[x]; b < e; b += 4u) {
          const uint4 c = *reinterpret_cast<const uint4*>(cx + b);
          const uint32_t cs[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const uint32_t y = cs[t];
            if ((y & kDown) || !seen(y) || lev[y] != d || !transit(y)) continue;
#pragma unroll
            for (int w = 0; w < W; ++w) acc[w] |= nh[y * W + w];
          }
        }
#pragma unroll
        for (int w = 0; w < W; ++w) nh[x * W + w] = acc[w];
      }
      wave_sync();
      qb = qe;
      ++d;
    }
    // rows + digest
    uint64_t reached = 0, sumd = 0, h = 0;
    uint32_t* drow = a.dist ? a.dist + (size_t)i * V : nullptr;
    for (uint32_t v = lane; v < V; v += 64u) {
      const bool r = seen(v);
      const uint32_t dv = r ? (uint32_t)lev[v] : kInf;
      if (drow) __builtin_nontemporal_store(dv, drow + v);
      if (r) {
        reached += 1u;
        sumd += dv;
        h += g.dkey[2ull * v] * (uint64_t)(dv + 1u);
      }
    }
    uint32_t* nrow = a.nh ? a.nh + (size_t)i * V * W : nullptr;
    for (uint32_t x = lane; x < V * W; x += 64u) {
      const uint32_t word = nh[x];
      if (nrow) __builtin_nontemporal_store(word, nrow + x);
      if (word) h += g.dkn[x / W] * digest_word_key(x % W, word);
    }
    if (a.digest) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        reached += shfl_xor64(reached, o);
        sumd += shfl_xor64(sumd, o);
        h += shfl_xor64(h, o);
      }
      if (lane == 0) {
        ospf_digest dg;
        dg.reached = reached;
        dg.sum_dist = sumd;
        dg.hash = h;
        a.digest[i] = dg;
      }
    }
    wave_sync();  // the slice is cleared for the next root
  }
}

}  // namespace

size_t small_lds_bytes(uint32_t V, uint32_t Ep, uint32_t W, uint32_t waves) {
  const SmallLayout L = small_layout(V, Ep, W);
  return 4ull * (L.graph_words + (size_t)waves * L.wave_words);
}

hipError_t launch_lds_sweep(const DevGraph& g, const SmallArgs& a, uint32_t W, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (W == 0 || W > 4 || a.waves == 0 || a.waves > 4 || (a.Ep & 3u)) return hipErrorInvalidValue;
  const size_t lds = small_lds_bytes(g.V, a.Ep, W, a.waves);
  const dim3 grid((a.n + a.waves - 1) / a.waves), block(64u * a.waves);
  const void* k = W == 1 ? (const void*)lds_sweep_kernel<1>
                : W == 2 ? (const void*)lds_sweep_kernel<2>
                : W == 3 ? (const void*)lds_sweep_kernel<3>
                         : (const void*)lds_sweep_kernel<4>;
  if (lds > 64u * 1024u) {
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  switch (W) {
    case 1: hipLaunchKernelGGL(lds_sweep_kernel<1>, grid, block, lds, s, g, a); break;
    case 2: hipLaunchKernelGGL(lds_sweep_kernel<2>, grid, block, lds, s, g, a); break;
    case 3: hipLaunchKernelGGL(lds_sweep_kernel<3>, grid, block, lds, s, g, a); break;
    default: hipLaunchKernelGGL(lds_sweep_kernel<4>, grid, block, lds, s, g, a); break;
  }
  return hipGetLastError();
}

}  // namespace ospf
