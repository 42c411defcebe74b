// spf_kernels.hip — CDNA4 (gfx950) kernels for batched OpenR SPF.
//
// One workgroup = one SPF run (root, optional ignored-link set). Each run is
// the reference's LinkState::runSpf (openr/decision/LinkState.cpp:836-911)
// restated as a distance-bucketed (Dial) sweep, which visits nodes in exactly
// the reference's settle order by distance:
//
//   round d: every node v with dist[v] == d is final;
//     * its ECMP next-hop set is the OR over tight, usable in-edges u->v whose
//       tail u may transit (u == root or !overloaded, LinkState.cpp:859-866) of
//       (u == root ? {bit(v)} : nh[u])          (LinkState.cpp:885-901)
//     * if v may transit, its usable out-edges relax dist[x] to d + w(v->x)
//       (w = metric advertised by v, LinkState.cpp:878; 1 in hop-count mode)
//   next round: the smallest tentative distance > d (unit metric: d + 1).
//
// Because metrics are >= 1, every predecessor of a node in bucket d is settled
// in an earlier round, so next-hop sets are order-independent bit ORs and the
// result is bit-identical to the reference's heap-ordered run.
//
// Variants (picked per batch by the host, spf_engine.hip):
//   LDS_DIST/LDS_NH : state resident in the CU's LDS (small graphs: G31, F10k
//                     RSW roots) or streamed in HBM (large graphs: F100k, M1M).
//   UNIT            : unit metric / hop count: no weight loads, one barrier per
//                     level, next-hops pushed with LDS atomics when resident.
//   IGN             : per-run ignored links (KSP2 masked reruns).
//   WF              : next-hop words held in registers (1 or 4); 0 = generic.
// Work inside a round is node-per-lane; nodes with degree > HYB_DEG are
// expanded cooperatively by the whole 64-lane wave (ballot + shuffles) so a
// 1,781-port spine does not serialise one lane.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spf_kernels.h"

namespace ospf {

constexpr uint32_t INF = 0xFFFFFFFFu;
constexpr uint32_t DOWN = 0x80000000u;
constexpr int WAVE = 64;
constexpr uint32_t HYB_DEG = 32;

// lower_bound over a sorted LDS array
__device__ __forceinline__ uint32_t lbound(const uint32_t* a, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ bool in_sorted(const uint32_t* a, uint32_t n, uint32_t key) {
  uint32_t i = lbound(a, n, key);
  return i < n && a[i] == key;
}

__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, WAVE);
  return x;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, WAVE));
  return x;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, WAVE);
  return x;
}

template <bool UNIT, bool LDS_DIST, bool LDS_NH, bool IGN, int WF>
struct Run {
  // PUSH_NH: next-hops ORed forward with LDS atomics while relaxing (unit
  // metric, LDS-resident next-hops); otherwise pulled when a node settles.
  static constexpr bool PUSH_NH = UNIT && LDS_NH;

  const DevGraph& g;
  const RunArgs& a;
  uint32_t root, V, W;
  uint32_t* dist;
  uint32_t* nh;
  const uint32_t* nbr;
  uint32_t nbr_n;
  const uint32_t* ign;
  uint32_t ign_n;
  uint32_t* flag;

  __device__ Run(const DevGraph& g_, const RunArgs& a_) : g(g_), a(a_) {}

  __device__ __forceinline__ bool transit(uint32_t v) const {
    return v == root || !((g.nt_bits[v >> 5] >> (v & 31)) & 1u);
  }
  __device__ __forceinline__ bool usable(uint32_t e, uint32_t cx) const {
    if (cx & DOWN) return false;
    if constexpr (IGN) {
      if (ign_n && in_sorted(ign, ign_n, g.link_id[e])) return false;
    }
    return true;
  }
  __device__ __forceinline__ uint32_t* nh_of(uint32_t v) const { return nh + (size_t)v * W; }

  // ---- pull: next-hop set of v (dist d), owned by one lane ----
  __device__ void pull_serial(uint32_t v, uint32_t beg, uint32_t end, uint32_t d) {
    uint32_t acc[WF ? WF : 1];
#pragma unroll
    for (int w = 0; w < (WF ? WF : 1); ++w) acc[w] = 0;
    uint32_t* dst = nh_of(v);
    if constexpr (WF == 0) {
      for (uint32_t w = 0; w < W; ++w) dst[w] = 0;
    }
    for (uint32_t e = beg; e < end; ++e) {
      uint32_t cx = g.colx[e];
      if (!usable(e, cx)) continue;
      uint32_t u = cx;
      uint32_t du = dist[u];
      if (du == INF) continue;
      uint32_t wu = UNIT ? 1u : g.rw[e];
      if (du + wu != d) continue;
      if (u == root) {
        uint32_t b = lbound(nbr, nbr_n, v);
        if constexpr (WF == 0) dst[b >> 5] |= 1u << (b & 31);
        else {
#pragma unroll
          for (int w = 0; w < WF; ++w) acc[w] |= ((b >> 5) == (uint32_t)w) ? (1u << (b & 31)) : 0u;
        }
      } else if (transit(u)) {
        const uint32_t* s = nh_of(u);
        if constexpr (WF == 0) {
          for (uint32_t w = 0; w < W; ++w) dst[w] |= s[w];
        } else {
#pragma unroll
          for (int w = 0; w < WF; ++w) if ((uint32_t)w < W) acc[w] |= s[w];
        }
      }
    }
    if constexpr (WF != 0) {
#pragma unroll
      for (int w = 0; w < WF; ++w) if ((uint32_t)w < W) dst[w] = acc[w];
    }
  }

  // ---- pull by the whole wave (high-degree v) ----
  __device__ void pull_wave(uint32_t v, uint32_t beg, uint32_t end, uint32_t d, int lane) {
    uint32_t acc[WF ? WF : 1];
#pragma unroll
    for (int w = 0; w < (WF ? WF : 1); ++w) acc[w] = 0;
    uint32_t* dst = nh_of(v);
    if constexpr (WF == 0) {
      for (uint32_t w = lane; w < W; w += WAVE) dst[w] = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    for (uint32_t e = beg + lane; e < end; e += WAVE) {
      uint32_t cx = g.colx[e];
      if (!usable(e, cx)) continue;
      uint32_t u = cx;
      uint32_t du = dist[u];
      if (du == INF) continue;
      uint32_t wu = UNIT ? 1u : g.rw[e];
      if (du + wu != d) continue;
      if (u == root) {
        uint32_t b = lbound(nbr, nbr_n, v);
        if constexpr (WF == 0) atomicOr(&dst[b >> 5], 1u << (b & 31));
        else {
#pragma unroll
          for (int w = 0; w < WF; ++w) acc[w] |= ((b >> 5) == (uint32_t)w) ? (1u << (b & 31)) : 0u;
        }
      } else if (transit(u)) {
        const uint32_t* s = nh_of(u);
        if constexpr (WF == 0) {
          for (uint32_t w = 0; w < W; ++w) if (s[w]) atomicOr(&dst[w], s[w]);
        } else {
#pragma unroll
          for (int w = 0; w < WF; ++w) if ((uint32_t)w < W) acc[w] |= s[w];
        }
      }
    }
    if constexpr (WF != 0) {
#pragma unroll
      for (int w = 0; w < WF; ++w) {
        uint32_t x = wave_or(acc[w]);
        if (lane == 0 && (uint32_t)w < W) dst[w] = x;
      }
    }
  }

  // ---- relax one out-edge of v (dist d) ----
  __device__ __forceinline__ void relax(uint32_t v, uint32_t e, uint32_t d, const uint32_t* nhv,
                                        uint32_t ring) {
    uint32_t cx = g.colx[e];
    if (!usable(e, cx)) return;
    uint32_t x = cx;
    if constexpr (UNIT) {
      uint32_t old = dist[x];
      if (old == INF) {
        dist[x] = d + 1;
        old = d + 1;
        flag[ring] = 1u;
      }
      if constexpr (PUSH_NH) {
        if (old == d + 1) {
          uint32_t* t = nh_of(x);
          if (v == root) {
            uint32_t b = lbound(nbr, nbr_n, x);
            atomicOr(&t[b >> 5], 1u << (b & 31));
          } else {
            for (uint32_t w = 0; w < W; ++w) {
              uint32_t s = nhv[w];
              if (s) atomicOr(&t[w], s);
            }
          }
        }
      }
    } else {
      atomicMin(&dist[x], d + g.w[e]);
    }
  }

  __device__ void settle_round(uint32_t d, uint32_t ring, int lane, int wave, int nwaves) {
    for (uint32_t base = (uint32_t)wave * WAVE; base < V; base += (uint32_t)nwaves * WAVE) {
      const uint32_t v = base + lane;
      bool act = v < V && dist[v] == d;
      uint32_t beg = 0, end = 0;
      if (act) {
        beg = g.row_ptr[v];
        end = g.row_ptr[v + 1];
      }
      const bool big = act && (end - beg) > HYB_DEG;
      if (act && !big) {
        if constexpr (!PUSH_NH) {
          if (v != root) pull_serial(v, beg, end, d);
        }
        if (transit(v)) {
          const uint32_t* nhv = nh_of(v);
          for (uint32_t e = beg; e < end; ++e) relax(v, e, d, nhv, ring);
        }
      }
      uint64_t bigm = __ballot(big);
      while (bigm) {
        const int l = __ffsll((unsigned long long)bigm) - 1;
        bigm &= bigm - 1;
        const uint32_t bv = __shfl(v, l, WAVE);
        const uint32_t bb = __shfl(beg, l, WAVE);
        const uint32_t be = __shfl(end, l, WAVE);
        if constexpr (!PUSH_NH) {
          if (bv != root) pull_wave(bv, bb, be, d, lane);
        }
        if (transit(bv)) {
          const uint32_t* nhv = nh_of(bv);
          for (uint32_t e = bb + lane; e < be; e += WAVE) relax(bv, e, d, nhv, ring);
        }
      }
    }
  }
};

template <bool UNIT, bool LDS_DIST, bool LDS_NH, bool IGN, int WF>
__global__ void __launch_bounds__(512) spf_run_kernel(DevGraph g, RunArgs a) {
  extern __shared__ uint32_t lds[];
  const int tid = threadIdx.x;
  const int lane = tid & (WAVE - 1);
  const int wave = tid / WAVE;
  const int nwaves = blockDim.x / WAVE;
  const uint32_t rix = blockIdx.x;

  Run<UNIT, LDS_DIST, LDS_NH, IGN, WF> r(g, a);
  r.root = a.roots[rix];
  r.V = g.V;
  r.W = a.W;
  const uint32_t V = g.V, W = a.W;

  // LDS layout (u32 words): [0,16) flags | [16,32) reduction | nbr | ign | dist | nh
  uint32_t* s_flag = lds;
  uint32_t* s_red = lds + 16;
  uint32_t* s_nbr = lds + 32;
  uint32_t* s_ign = s_nbr + a.nbr_cap;
  uint32_t* s_dist = s_ign + a.ign_cap;
  uint32_t* s_nh = s_dist + (LDS_DIST ? V : 0);
  r.flag = s_flag;
  r.dist = LDS_DIST ? s_dist : a.dist + (size_t)rix * V;
  r.nh = LDS_NH ? s_nh : a.nh + (size_t)rix * V * W;
  r.nbr = s_nbr;
  r.ign = s_ign;

  // root neighbour table (bit order) and ignore list
  const uint32_t nb0 = g.dn_off[r.root], nb1 = g.dn_off[r.root + 1];
  r.nbr_n = nb1 - nb0;
  if (r.nbr_n > 32u * W || r.nbr_n > a.nbr_cap) {  // caller under-sized nh words
    if (tid == 0) atomicOr(a.err, 1u);
    return;
  }
  for (uint32_t i = tid; i < r.nbr_n; i += blockDim.x) s_nbr[i] = g.dn[nb0 + i];
  r.ign_n = 0;
  if constexpr (IGN) {
    const uint32_t i0 = a.ign_off[rix], i1 = a.ign_off[rix + 1];
    r.ign_n = i1 - i0;
    if (r.ign_n > a.ign_cap) {
      if (tid == 0) atomicOr(a.err, 2u);
      return;
    }
    for (uint32_t i = tid; i < r.ign_n; i += blockDim.x) s_ign[i] = a.ign_ids[i0 + i];
  }
  // state init
  for (uint32_t v = tid; v < V; v += blockDim.x) r.dist[v] = (v == r.root) ? 0u : INF;
  if constexpr (LDS_NH) {
    for (uint32_t i = tid; i < V * W; i += blockDim.x) s_nh[i] = 0u;
  } else {
    for (uint32_t w = tid; w < W; w += blockDim.x) r.nh[(size_t)r.root * W + w] = 0u;
  }
  if (tid < 16) s_flag[tid] = 0u;
  __syncthreads();

  if constexpr (UNIT) {
    for (uint32_t d = 0;; ++d) {
      const uint32_t ring = d % 3u;
      if (tid == 0) s_flag[(d + 1) % 3u] = 0u;
      r.settle_round(d, ring, lane, wave, nwaves);
      __syncthreads();
      if (!s_flag[ring]) break;
    }
  } else {
    uint32_t d = 0;
    for (uint32_t round = 0;; ++round) {
      r.settle_round(d, 0, lane, wave, nwaves);
      __syncthreads();
      uint32_t m = INF;
      for (uint32_t v = tid; v < V; v += blockDim.x) {
        uint32_t x = r.dist[v];
        if (x > d && x < m) m = x;
      }
      m = wave_min(m);
      uint32_t* red = s_red + (round & 1u) * 8u;
      if (lane == 0) red[wave] = m;
      __syncthreads();
      m = INF;
      for (int i = 0; i < nwaves; ++i) m = min(m, red[i]);
      if (m == INF) break;
      d = m;
    }
  }

  // epilogue: outputs + digest
  const bool want_dist = a.flags & 2u, want_nh = a.flags & 4u, want_dig = a.flags & 8u;
  uint32_t* out_dist = a.dist ? a.dist + (size_t)rix * V : nullptr;
  uint32_t* out_nh = a.nh ? a.nh + (size_t)rix * V * W : nullptr;
  uint64_t reached = 0, sumd = 0, hsum = 0;
  for (uint32_t v = tid; v < V; v += blockDim.x) {
    const uint32_t dv = r.dist[v];
    if constexpr (LDS_DIST) {
      if (want_dist) out_dist[v] = dv;
    }
    if (dv == INF) {
      if constexpr (!LDS_NH) {
        if (want_nh || !LDS_NH) {
          for (uint32_t w = 0; w < W; ++w) r.nh[(size_t)v * W + w] = 0u;
        }
      }
      continue;
    }
    if (want_dig) {
      const uint32_t* hv = r.nh_of(v);
      for (uint32_t w = 0; w < W; ++w) hsum += digest_word_term(v, w, hv[w]);
      reached += 1;
      sumd += dv;
      hsum += digest_node_term(v, dv);
    }
  }
  if constexpr (LDS_NH) {
    if (want_nh) {
      for (uint32_t i = tid; i < V * W; i += blockDim.x) out_nh[i] = s_nh[i];
    }
  }
  if (want_dig) {
    __shared__ uint64_t s_dig[3][16];
    reached = wave_sum64(reached);
    sumd = wave_sum64(sumd);
    hsum = wave_sum64(hsum);
    if (lane == 0) {
      s_dig[0][wave] = reached;
      s_dig[1][wave] = sumd;
      s_dig[2][wave] = hsum;
    }
    __syncthreads();
    if (tid == 0) {
      ospf_digest dg{0, 0, 0};
      for (int i = 0; i < nwaves; ++i) {
        dg.reached += s_dig[0][i];
        dg.sum_dist += s_dig[1][i];
        dg.hash += s_dig[2][i];
      }
      a.digest[rix] = dg;
    }
  }
}

// ---------------------------------------------------------------------------
template <bool UNIT, bool LDS_DIST, bool LDS_NH, bool IGN, int WF>
static hipError_t launch_one(const DevGraph& g, const RunArgs& a, uint32_t n_roots,
                             uint32_t block, size_t lds_bytes, hipStream_t s) {
  auto k = spf_run_kernel<UNIT, LDS_DIST, LDS_NH, IGN, WF>;
  if (lds_bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds_bytes);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(n_roots), dim3(block), lds_bytes, s, g, a);
  return hipGetLastError();
}

template <bool UNIT, bool LDS_DIST, bool LDS_NH, bool IGN>
static hipError_t launch_wf(const DevGraph& g, const RunArgs& a, uint32_t n_roots,
                            uint32_t block, size_t lds, hipStream_t s) {
  if (a.W == 1) return launch_one<UNIT, LDS_DIST, LDS_NH, IGN, 1>(g, a, n_roots, block, lds, s);
  if (a.W <= 4) return launch_one<UNIT, LDS_DIST, LDS_NH, IGN, 4>(g, a, n_roots, block, lds, s);
  return launch_one<UNIT, LDS_DIST, LDS_NH, IGN, 0>(g, a, n_roots, block, lds, s);
}

template <bool UNIT, bool IGN>
static hipError_t launch_var(int variant, const DevGraph& g, const RunArgs& a, uint32_t n_roots,
                             uint32_t block, size_t lds, hipStream_t s) {
  switch (variant) {
    case 0: return launch_wf<UNIT, true, true, IGN>(g, a, n_roots, block, lds, s);
    case 1: return launch_wf<UNIT, true, false, IGN>(g, a, n_roots, block, lds, s);
    default: return launch_wf<UNIT, false, false, IGN>(g, a, n_roots, block, lds, s);
  }
}

hipError_t launch_spf(int variant, bool unit, bool ign, const DevGraph& g, const RunArgs& a,
                      uint32_t n_roots, uint32_t block, size_t lds_bytes, hipStream_t s) {
  if (unit) {
    return ign ? launch_var<true, true>(variant, g, a, n_roots, block, lds_bytes, s)
               : launch_var<true, false>(variant, g, a, n_roots, block, lds_bytes, s);
  }
  return ign ? launch_var<false, true>(variant, g, a, n_roots, block, lds_bytes, s)
             : launch_var<false, false>(variant, g, a, n_roots, block, lds_bytes, s);
}

}  // namespace ospf
