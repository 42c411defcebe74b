// spf_bfs.hip — unit-metric / hop-count SPF for large graphs (gfx950).
//
// One workgroup per SPF run. Same result as LinkState::runSpf
// (openr/decision/LinkState.cpp:836-911) when every usable weight is 1
// (fabric and grid topologies, or useLinkMetric=false): Dijkstra's settle
// order by (dist, name) degenerates to BFS levels, and the ECMP next-hop set of
// a node at level d+1 is the OR over its usable in-edges from transit nodes
// of level d (LinkState.cpp:885-901).
//
// State lives in LDS as three V-bit bitmaps (visited, current level, next
// level) — 37.5 KB at V = 100k — so the per-edge random accesses of the BFS
// hit LDS, not HBM. Each level picks its direction (Beamer-style):
//   push  (top-down):  frontier nodes scan out-edges, mark unvisited heads;
//   pull  (bottom-up): unvisited nodes scan in-edges for frontier tails.
// Next-hop sets:
//   NH_LDS (root has <= 8 distinct neighbours, e.g. every rack switch): one
//     byte per node in LDS; push ORs it forward with 32-bit LDS atomics, pull
//     ORs it in registers — one pass per level either way.
//   otherwise: next-hops live in the HBM output row; push only marks the next
//     level and a pull over the new level ORs the tails' words.
// dist / nh rows are written once per node (masked coalesced stores), the
// digest is accumulated in the same pass.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;
constexpr int kWave = 64;
constexpr uint32_t kCoopDeg = 32;

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t* a, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint32_t wor(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, kWave);
  return x;
}
__device__ __forceinline__ uint64_t wsum(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
  return x;
}

__device__ __forceinline__ bool bit(const uint32_t* bm, uint32_t v) {
  return (bm[v >> 5] >> (v & 31)) & 1u;
}

template <bool NH_LDS, bool IGN, int WF>
struct Bfs {
  const DevGraph& g;
  const RunArgs& a;
  uint32_t root, V, W, nwords;
  uint32_t *vis, *cur, *nxt;   // LDS bitmaps
  uint32_t* nhb;               // NH_LDS: one byte per node, packed in words
  uint32_t* nh_out;            // HBM next-hop row (W words per node)
  uint32_t* dist_out;          // HBM dist row
  const uint32_t* nbr;
  uint32_t nbr_n;
  const uint32_t* ign;
  uint32_t ign_n;
  uint32_t* cnt;               // LDS counters

  __device__ Bfs(const DevGraph& g_, const RunArgs& a_) : g(g_), a(a_) {}

  __device__ __forceinline__ bool transit(uint32_t u) const {
    return u == root || !bit(g.nt_bits, u);
  }
  __device__ __forceinline__ bool usable(uint32_t e, uint32_t cx) const {
    if (cx & kDown) return false;
    if constexpr (IGN) {
      if (ign_n) {
        const uint32_t l = g.link_id[e];
        const uint32_t i = lower_bound_u32(ign, ign_n, l);
        if (i < ign_n && ign[i] == l) return false;
      }
    }
    return true;
  }
  __device__ __forceinline__ uint32_t nh_byte(uint32_t v) const {
    return (nhb[v >> 2] >> (8 * (v & 3))) & 0xFFu;
  }
  __device__ __forceinline__ uint32_t root_bit(uint32_t v) const {
    return lower_bound_u32(nbr, nbr_n, v);
  }

  // ---------------- push: u (level d, transit) -> mark unvisited heads
  __device__ __forceinline__ void push_edge(uint32_t u, uint32_t e, uint32_t nbu) {
    const uint32_t cx = g.colx[e];
    if (!usable(e, cx)) return;
    const uint32_t x = cx;
    if (bit(vis, x)) return;
    atomicOr(&nxt[x >> 5], 1u << (x & 31));
    if constexpr (NH_LDS) {
      const uint32_t val = (u == root) ? (1u << root_bit(x)) : nbu;
      atomicOr(&nhb[x >> 2], val << (8 * (x & 3)));
    }
  }

  // ---------------- pull: v collects next-hops from level-d tails
  // returns true when v has at least one tight transit tail
  template <bool COOP>
  __device__ __forceinline__ bool pull_node(uint32_t v, uint32_t beg, uint32_t end, int lane,
                                            uint32_t* acc) {
    bool any = false;
    bool zeroed = COOP;  // the cooperative path zeroes before calling
    const uint32_t step = COOP ? kWave : 1;
    for (uint32_t e = beg + (COOP ? lane : 0); e < end; e += step) {
      const uint32_t cx = g.colx[e];
      if (!usable(e, cx)) continue;
      const uint32_t u = cx;
      if (!bit(cur, u) || !transit(u)) continue;
      any = true;
      if constexpr (!NH_LDS && WF == 0 && !COOP) {
        if (!zeroed) {
          for (uint32_t w = 0; w < W; ++w) nh_out[(size_t)v * W + w] = 0;
          zeroed = true;
        }
      }
      if (u == root) {
        const uint32_t b = root_bit(v);
        if constexpr (NH_LDS) {
          acc[0] |= 1u << b;
        } else if constexpr (WF > 0) {
#pragma unroll
          for (int w = 0; w < WF; ++w) acc[w] |= ((b >> 5) == (uint32_t)w) ? (1u << (b & 31)) : 0u;
        } else {
          atomicOr(&nh_out[(size_t)v * W + (b >> 5)], 1u << (b & 31));
        }
      } else {
        if constexpr (NH_LDS) {
          acc[0] |= nh_byte(u);
        } else if constexpr (WF > 0) {
          const uint32_t* s = nh_out + (size_t)u * W;
#pragma unroll
          for (int w = 0; w < WF; ++w) if ((uint32_t)w < W) acc[w] |= s[w];
        } else {
          const uint32_t* s = nh_out + (size_t)u * W;
          for (uint32_t w = 0; w < W; ++w) {
            const uint32_t x = s[w];
            if (x) atomicOr(&nh_out[(size_t)v * W + w], x);
          }
        }
      }
    }
    return any;
  }

  __device__ __forceinline__ void store_nh(uint32_t v, const uint32_t* acc) {
    if constexpr (NH_LDS) {
      atomicOr(&nhb[v >> 2], acc[0] << (8 * (v & 3)));
    } else if constexpr (WF > 0) {
#pragma unroll
      for (int w = 0; w < WF; ++w) if ((uint32_t)w < W) nh_out[(size_t)v * W + w] = acc[w];
    }
  }

  // bottom-up over unvisited nodes (PULL_ALL) or over the marked next level
  template <bool PULL_ALL>
  __device__ void pull_level(int lane, int wave, int nwaves) {
    const uint32_t nchunks = (V + 63) / 64;
    for (uint32_t c = wave; c < nchunks; c += nwaves) {
      const uint32_t v = c * 64 + lane;
      bool act = v < V;
      if (act) act = PULL_ALL ? !bit(vis, v) : bit(nxt, v);
      uint32_t beg = 0, end = 0;
      if (act) {
        beg = g.row_ptr[v];
        end = g.row_ptr[v + 1];
      }
      const bool big = act && (end - beg) > kCoopDeg;
      if (act && !big) {
        uint32_t acc[WF > 0 ? WF : 1] = {};
        const bool any = pull_node<false>(v, beg, end, lane, acc);
        if (any) {
          store_nh(v, acc);
          if (PULL_ALL) atomicOr(&nxt[v >> 5], 1u << (v & 31));
        }
      }
      uint64_t bm = __ballot(big);
      while (bm) {
        const int l = __ffsll((unsigned long long)bm) - 1;
        bm &= bm - 1;
        const uint32_t bv = __shfl(v, l, kWave), bb = __shfl(beg, l, kWave),
                       be = __shfl(end, l, kWave);
        uint32_t acc[WF > 0 ? WF : 1] = {};
        if constexpr (!NH_LDS && WF == 0) {
          // wide rows: only zero (then OR into HBM) when the node has a tail
          bool has = false;
          for (uint32_t e = bb + lane; e < be && !has; e += kWave) {
            const uint32_t cx = g.colx[e];
            has = usable(e, cx) && bit(cur, cx) && transit(cx);
          }
          if (__ballot(has) == 0) continue;
          for (uint32_t w = lane; w < W; w += kWave) nh_out[(size_t)bv * W + w] = 0;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        const bool any_l = pull_node<true>(bv, bb, be, lane, acc);
        const bool any = __ballot(any_l) != 0;
        if constexpr (NH_LDS || WF > 0) {
#pragma unroll
          for (int w = 0; w < (WF > 0 ? WF : 1); ++w) acc[w] = wor(acc[w]);
        }
        if (any && lane == 0) {
          store_nh(bv, acc);
          if (PULL_ALL) atomicOr(&nxt[bv >> 5], 1u << (bv & 31));
        }
      }
    }
  }

  // top-down: frontier nodes push to unvisited heads
  __device__ void push_level(int lane, int wave, int nwaves) {
    const uint32_t nchunks = (V + 63) / 64;
    for (uint32_t c = wave; c < nchunks; c += nwaves) {
      // skip empty chunks cheaply (two bitmap words)
      const uint32_t w0 = cur[c * 2], w1 = (c * 2 + 1 < nwords) ? cur[c * 2 + 1] : 0u;
      if ((w0 | w1) == 0) continue;
      const uint32_t v = c * 64 + lane;
      bool act = v < V && bit(cur, v) && transit(v);
      uint32_t beg = 0, end = 0, nbv = 0;
      if (act) {
        beg = g.row_ptr[v];
        end = g.row_ptr[v + 1];
        if constexpr (NH_LDS) nbv = nh_byte(v);
      }
      const bool big = act && (end - beg) > kCoopDeg;
      if (act && !big)
        for (uint32_t e = beg; e < end; ++e) push_edge(v, e, nbv);
      uint64_t bm = __ballot(big);
      while (bm) {
        const int l = __ffsll((unsigned long long)bm) - 1;
        bm &= bm - 1;
        const uint32_t bv = __shfl(v, l, kWave), bb = __shfl(beg, l, kWave),
                       be = __shfl(end, l, kWave), bn = __shfl(nbv, l, kWave);
        for (uint32_t e = bb + lane; e < be; e += kWave) push_edge(bv, e, bn);
      }
    }
  }
};

template <bool NH_LDS, bool IGN, int WF>
__device__ void bfs_run(const DevGraph& g, const RunArgs& a, uint32_t* lds) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
  const uint32_t rix = blockIdx.x;
  Bfs<NH_LDS, IGN, WF> b(g, a);
  const uint32_t V = g.V, W = a.W;
  b.root = a.roots[rix];
  b.V = V;
  b.W = W;
  b.nwords = (V + 31) / 32;
  const uint32_t bw = (b.nwords + 1) & ~1u;  // even: chunks of two words
  uint32_t* cnt = lds;                        // [0,32) counters / reductions
  uint32_t* s_nbr = lds + 32;
  uint32_t* s_ign = s_nbr + a.nbr_cap;
  b.vis = s_ign + a.ign_cap;
  b.cur = b.vis + bw;
  b.nxt = b.cur + bw;
  b.nhb = b.nxt + bw;  // NH_LDS: (V+3)/4 words
  b.cnt = cnt;
  b.nbr = s_nbr;
  b.ign = s_ign;
  b.dist_out = a.dist + (size_t)rix * V;
  b.nh_out = a.nh + (size_t)rix * V * W;

  const uint32_t nb0 = g.dn_off[b.root];
  b.nbr_n = g.dn_off[b.root + 1] - nb0;
  if (b.nbr_n > 32u * W || b.nbr_n > a.nbr_cap) {
    if (tid == 0) atomicOr(a.err, 1u);
    return;
  }
  for (uint32_t i = tid; i < b.nbr_n; i += blockDim.x) s_nbr[i] = g.dn[nb0 + i];
  b.ign_n = 0;
  if constexpr (IGN) {
    const uint32_t i0 = a.ign_off[rix], i1 = a.ign_off[rix + 1];
    b.ign_n = i1 - i0;
    if (b.ign_n > a.ign_cap) {
      if (tid == 0) atomicOr(a.err, 2u);
      return;
    }
    for (uint32_t i = tid; i < b.ign_n; i += blockDim.x) s_ign[i] = a.ign_ids[i0 + i];
  }
  for (uint32_t i = tid; i < bw; i += blockDim.x) {
    const uint32_t r = (i == (b.root >> 5)) ? (1u << (b.root & 31)) : 0u;
    b.vis[i] = r;
    b.cur[i] = r;
    b.nxt[i] = 0u;
  }
  if constexpr (NH_LDS) {
    for (uint32_t i = tid; i < (V + 3) / 4; i += blockDim.x) b.nhb[i] = 0u;
  }
  if (tid < 32) cnt[tid] = 0u;
  if (tid == 0) {
    b.dist_out[b.root] = 0u;
    cnt[4] = g.row_ptr[b.root + 1] - g.row_ptr[b.root];  // frontier edge mass
  }
  for (uint32_t w = tid; w < W; w += blockDim.x) b.nh_out[(size_t)b.root * W + w] = 0u;
  __syncthreads();

  const bool want_dig = a.flags & 8u;
  uint64_t reached = 0, sumd = 0, hsum = 0;
  if (want_dig && tid == 0) {  // the root itself: dist 0, no next-hops
    reached = 1;
    hsum = mix((uint64_t)b.root << 32);
  }
  const uint32_t E = g.E;
  uint32_t unvisited_mass = E - cnt[4];
  for (uint32_t d = 0;; ++d) {
    const uint32_t front_mass = cnt[4 + (d & 1) * 2];
    // direction: pull when the unvisited edge mass is not larger than what a
    // push + follow-up pull would scan
    const bool pull_all = NH_LDS ? (unvisited_mass < front_mass)
                                 : (unvisited_mass < 2u * front_mass);
    if (pull_all) b.template pull_level<true>(lane, wave, nwaves);
    else b.push_level(lane, wave, nwaves);
    __syncthreads();
    if (!NH_LDS && !pull_all) {
      b.template pull_level<false>(lane, wave, nwaves);
      __syncthreads();
    }
    // new level: write dist (+ digest), count its edge mass, roll bitmaps
    uint32_t mass = 0, found = 0;
    const uint32_t nchunks = (V + 63) / 64;
    for (uint32_t c = wave; c < nchunks; c += nwaves) {
      const uint32_t v = c * 64 + lane;
      const bool in = v < V && bit(b.nxt, v);
      if (in) {
        b.dist_out[v] = d + 1;
        mass += g.row_ptr[v + 1] - g.row_ptr[v];
        found = 1;
        if (want_dig) {
          uint64_t s = 0;
          if constexpr (NH_LDS) {
            uint32_t bits = b.nh_byte(v);
            while (bits) {
              s += mix((uint64_t)s_nbr[__ffs(bits) - 1] + 1ull);
              bits &= bits - 1;
            }
          } else {
            for (uint32_t w = 0; w < W; ++w) {
              uint32_t bits = b.nh_out[(size_t)v * W + w];
              while (bits) {
                s += mix((uint64_t)s_nbr[w * 32 + __ffs(bits) - 1] + 1ull);
                bits &= bits - 1;
              }
            }
          }
          reached += 1;
          sumd += d + 1;
          hsum += mix(((uint64_t)v << 32) ^ (uint64_t)(d + 1) ^ (s * 0x9E3779B97F4A7C15ULL));
        }
      }
    }
    // reduce mass/found per wave, then into LDS
    uint64_t m64 = wsum((uint64_t)mass);
    const bool any = __ballot(found != 0) != 0;
    if (lane == 0 && m64) atomicAdd(&cnt[4 + ((d + 1) & 1) * 2], (uint32_t)m64);
    if (lane == 0 && any) cnt[1 + (d % 3)] = 1u;
    __syncthreads();
    for (uint32_t i = tid; i < bw; i += blockDim.x) {
      const uint32_t n = b.nxt[i];
      b.vis[i] |= n;
      b.cur[i] = n;
      b.nxt[i] = 0u;
    }
    const bool more = cnt[1 + (d % 3)] != 0;
    const uint32_t nm = cnt[4 + ((d + 1) & 1) * 2];
    __syncthreads();
    if (tid == 0) {
      cnt[1 + ((d + 1) % 3)] = 0u;
      cnt[4 + (d & 1) * 2] = 0u;  // this level's mass slot is reused two levels on
    }
    if (!more) break;
    unvisited_mass -= nm;
  }
  // epilogue: unreached nodes (dist INF, nh 0); NH_LDS next-hop row
  for (uint32_t v = tid; v < V; v += blockDim.x) {
    const bool seen = bit(b.vis, v);
    if (!seen) b.dist_out[v] = kInf;
    if constexpr (NH_LDS) {
      if (a.flags & 4u) {
        b.nh_out[(size_t)v * W] = seen ? b.nh_byte(v) : 0u;
        for (uint32_t w = 1; w < W; ++w) b.nh_out[(size_t)v * W + w] = 0u;
      }
    } else {
      if (!seen)
        for (uint32_t w = 0; w < W; ++w) b.nh_out[(size_t)v * W + w] = 0u;
    }
  }
  if (want_dig) {
    __shared__ uint64_t s_dig[48];
    reached = wsum(reached);
    sumd = wsum(sumd);
    hsum = wsum(hsum);
    if (lane == 0) {
      s_dig[wave] = reached;
      s_dig[16 + wave] = sumd;
      s_dig[32 + wave] = hsum;
    }
    __syncthreads();
    if (tid == 0) {
      ospf_digest dg{0, 0, 0};
      for (int i = 0; i < nwaves; ++i) {
        dg.reached += s_dig[i];
        dg.sum_dist += s_dig[16 + i];
        dg.hash += s_dig[32 + i];
      }
      a.digest[rix] = dg;
    }
  }
}

// NHL: LDS holds the byte next-hop array; a block uses it when its root has
// <= 8 distinct neighbours, the HBM next-hop path otherwise.
template <bool NHL, bool IGN, int WF>
__global__ void __launch_bounds__(1024) spf_bfs_kernel(DevGraph g, RunArgs a) {
  extern __shared__ uint32_t lds[];
  if constexpr (NHL) {
    const uint32_t root = a.roots[blockIdx.x];
    if (g.dn_off[root + 1] - g.dn_off[root] <= 8) {
      bfs_run<true, IGN, 1>(g, a, lds);
      return;
    }
  }
  bfs_run<false, IGN, WF>(g, a, lds);
}

template <bool NH_LDS, bool IGN, int WF>
hipError_t launch_bfs_one(const DevGraph& g, const RunArgs& a, uint32_t n, uint32_t block,
                          size_t lds, hipStream_t s) {
  auto k = spf_bfs_kernel<NH_LDS, IGN, WF>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(n), dim3(block), lds, s, g, a);
  return hipGetLastError();
}

template <bool NH_LDS, bool IGN>
hipError_t launch_bfs_wf(const DevGraph& g, const RunArgs& a, uint32_t n, uint32_t block,
                         size_t lds, hipStream_t s) {
  if (NH_LDS || a.W == 1) return launch_bfs_one<NH_LDS, IGN, 1>(g, a, n, block, lds, s);
  if (a.W <= 4) return launch_bfs_one<NH_LDS, IGN, 4>(g, a, n, block, lds, s);
  return launch_bfs_one<NH_LDS, IGN, 0>(g, a, n, block, lds, s);
}

}  // namespace

hipError_t launch_bfs(bool nh_lds, bool ign, const DevGraph& g, const RunArgs& a, uint32_t n,
                      uint32_t block, size_t lds, hipStream_t s) {
  if (nh_lds) {
    return ign ? launch_bfs_wf<true, true>(g, a, n, block, lds, s)
               : launch_bfs_wf<true, false>(g, a, n, block, lds, s);
  }
  return ign ? launch_bfs_wf<false, true>(g, a, n, block, lds, s)
             : launch_bfs_wf<false, false>(g, a, n, block, lds, s);
}

}  // namespace ospf
