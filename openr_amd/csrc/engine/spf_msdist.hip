// spf_msdist.hip — distance rows of many roots at once on large weighted
// graphs (gfx950): groups of 32 roots share one traversal, state [node][root].
//
// Why: on a 1M-node mesh a per-root Dial (spf_wdial.hip) keeps 4,096 roots in
// flight, each with its own wavefront somewhere in a 4 MB state array; the
// wavefronts' cache lines do not survive between the rounds that touch them
// (measured: ~92 MB written and ~240 MB fetched per root against 8 MB of
// rows). Roots that are neighbours in the graph (consecutive ids of a
// Hilbert-ordered mesh, one part of an all-sources sweep) have nearly the same
// wavefront: with the 32 roots' distances of a node in one 128-B line, one
// visit of the node reads its CSR row once and relaxes its out-edges for all
// of its active roots with one coalesced 128-B atomic per edge.
//
// Algorithm: label-correcting Delta-stepping over the group. A node is on the
// phase's list when some root of the group has a tentative distance at it
// that was lowered since the node last relaxed for that root (its "dirty"
// bit). A phase takes every listed node, claims its dirty bits, and relaxes
// its out-edges for the claimed roots whose distance lies below the current
// bucket end `hi` (and whose root may transit the node: an overloaded node
// relays only its own root's paths, LinkState.cpp:859-866); claimed roots at
// or past `hi` give their bits back and the node stays listed. Every lowered
// distance sets the head's dirty bit and lists the head for the next phase
// (once per phase: a stamp per node). When nothing left on the next list lies
// below `hi`, the bucket advances past the smallest listed distance. The
// fixed point is the shortest-distance table whatever the order (metrics >=
// 1); the buckets only keep the work near the wavefront. Next hops and
// digests are not computed here: the sweep derives them from these rows
// (ospf_wderive_dev / ospf_wderive_wide_dev: the first hops of the shortest
// paths, LinkState.cpp:885-901).
//
// Shape: one workgroup (512 threads) per group, persistent over groups; a
// half-wave per listed node (lane = root), two nodes per half-wave in flight.
// The group's state lives in the block's scratch: dist [V][32], dirty bits,
// stamps and two lists [V]. The dirty bits and distances are updated with
// L2 atomics by the block's own threads only (one CU, one L2): coherent.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;
constexpr uint32_t kR = 32;        // roots per group (a half-wave)
constexpr uint32_t kBlock = 512;   // threads per group
constexpr uint32_t kHW = kBlock / kR;
constexpr uint32_t kU = 2;         // nodes per half-wave in flight
constexpr uint32_t kTiles = 8;     // 32-node tiles per transpose step (33.8 KB of LDS)

__device__ __forceinline__ uint32_t ld2(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the group's state is touched by its own workgroup only: workgroup-scope
// atomics (performed in the CU's L2, not at the memory side)
__device__ __forceinline__ uint32_t wmin(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void wor(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t wxchg(uint32_t* p, uint32_t v) {
  return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
constexpr uint32_t kE = 8;  // edges of a node relaxed with their atomics in flight together

struct MsdState {
  uint32_t* D;       // [V][32]
  uint32_t* dirty;   // [V]
  uint32_t* stampP;  // [V] phase that listed the node for the next phase
  uint32_t* stampN;  // [V] bucket that listed the node for the next bucket
  uint32_t* L;       // [3][V]: current, next phase, next bucket (rotating)
};

__device__ __forceinline__ MsdState state_of(const MsDistArgs& a, uint32_t b, uint32_t V) {
  const size_t per = (size_t)V * (kR + 6u);
  uint32_t* base = a.scratch + per * b;
  MsdState s;
  s.D = base;
  s.dirty = base + (size_t)V * kR;
  s.stampP = s.dirty + V;
  s.stampN = s.stampP + V;
  s.L = s.stampN + V;
  return s;
}

__global__ void __launch_bounds__(kBlock, 4) msdist_kernel(DevGraph g, MsDistArgs a) {
  // list fills (current, next phase, next bucket), their buffers, the bucket
  __shared__ uint32_t s_nC, s_nP, s_nN, s_minN, s_hi, s_kb, s_ci, s_pi, s_ni;
  __shared__ uint32_t s_t[kTiles][32][33];  // row transpose tiles
  const uint32_t tid = threadIdx.x, lane = tid & 31u, hw = tid >> 5;
  const uint32_t hbase = (tid & 63u) & 32u;  // this half's first lane in the wave
  const uint32_t V = g.V;
  const MsdState st = state_of(a, blockIdx.x, V);
  for (uint32_t grp = blockIdx.x; grp < a.ngroups; grp += gridDim.x) {
    const uint32_t r0 = grp * kR, nr = min(kR, a.n - r0);
    // fresh state: every distance unreached, no dirty bit, no stamp
    {
      uint4* d4 = reinterpret_cast<uint4*>(st.D);
      const size_t n4 = (size_t)V * kR / 4u;
      const uint4 inf4 = make_uint4(kInf, kInf, kInf, kInf);
      for (size_t x = tid; x < n4; x += kBlock) d4[x] = inf4;
      for (uint32_t x = tid; x < V; x += kBlock) {
        st.dirty[x] = 0u;
        st.stampP[x] = kInf;
        st.stampN[x] = kInf;
      }
    }
    if (tid == 0) {
      s_nC = s_nP = s_nN = 0u;
      s_minN = kInf;
      s_hi = a.delta;
      s_kb = 0u;
      s_ci = 0u;
      s_pi = 1u;
      s_ni = 2u;
    }
    __syncthreads();
    const uint32_t myroot = lane < nr ? a.roots[r0 + lane] : kInf;
    if (hw == 0 && lane < nr) {
      st.D[(size_t)myroot * kR + lane] = 0u;
      wor(&st.dirty[myroot], 1u << lane);
      if (wxchg(&st.stampP[myroot], 0u) != 0u) st.L[atomicAdd(&s_nC, 1u)] = myroot;
    }
    __syncthreads();
    uint32_t phase = 0;
    while (true) {
      const uint32_t n = s_nC, hi = s_hi, kb1 = s_kb + 1u;
      uint32_t* LC = st.L + (size_t)s_ci * V;
      uint32_t* LP = st.L + (size_t)s_pi * V;
      uint32_t* LN = st.L + (size_t)s_ni * V;
      if (n == 0) break;  // block-uniform: no list holds anything
      __syncthreads();    // every thread has read the shared words
      if (tid == 0) s_nP = 0u;
      __syncthreads();
      const uint32_t nph = phase + 1u;
      uint32_t minN = kInf;
      // a half-wave's lane 0: list y for the next phase / the next bucket
      auto pushP = [&](uint32_t y) {
        if (wxchg(&st.stampP[y], nph) != nph) LP[atomicAdd(&s_nP, 1u)] = y;
      };
      auto pushN = [&](uint32_t y) {
        if (wxchg(&st.stampN[y], kb1) != kb1) LN[atomicAdd(&s_nN, 1u)] = y;
      };
      for (uint32_t i0 = hw * kU; i0 < n; i0 += kHW * kU) {
        uint32_t v[kU], take[kU], beg[kU], deg[kU], d[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) v[u] = i0 + u < n ? ld2(LC + i0 + u) : kInf;
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          take[u] = 0u;
          beg[u] = deg[u] = 0u;
          if (v[u] == kInf) continue;
          if (lane == 0) take[u] = wxchg(&st.dirty[v[u]], 0u);
          beg[u] = g.row_ptr[v[u]];
          deg[u] = g.row_ptr[v[u] + 1] - beg[u];
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          take[u] = (uint32_t)__shfl((int)take[u], (int)hbase, 64);
          d[u] = (take[u] >> lane) & 1u ? ld2(&st.D[(size_t)v[u] * kR + lane]) : kInf;
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          if (v[u] == kInf) continue;
          const bool mine = (take[u] >> lane) & 1u;
          const bool relay = v[u] == myroot || !((g.nt_bits[v[u] >> 5] >> (v[u] & 31u)) & 1u);
          const bool act = mine && relay && d[u] < hi;
          const bool later = mine && relay && d[u] >= hi;
          // roots already past the bucket: their bits back, the node on the
          // next bucket's list (it is there already when they were lowered
          // from this bucket: the stamp keeps one entry)
          const uint32_t lm = (uint32_t)(__ballot(later) >> hbase);
          if (lm) {
            minN = min(minN, later ? d[u] : kInf);
            if (lane == 0) {
              wor(&st.dirty[v[u]], lm);
              pushN(v[u]);
            }
          }
          if (!(uint32_t)(__ballot(act) >> hbase)) continue;
          // the row's entries over the lanes, then one edge at a time
          for (uint32_t e0 = 0; e0 < deg[u]; e0 += kR) {
            uint32_t ycol = kDown, yw = 0u;
            if (e0 + lane < deg[u]) {
              const uint32_t e = beg[u] + e0 + lane;
              if (g.ew) {
                const uint2 x = g.ew[e];
                ycol = x.x;
                yw = x.y & 0xFFFFu;
              } else {
                ycol = g.colx[e];
                yw = g.w[e];
              }
              if (a.hop) yw = 1u;
            }
            const uint32_t cnt = min(kR, deg[u] - e0);
            for (uint32_t j0 = 0; j0 < cnt; j0 += kE) {
              // kE edges: every atomicMin issued before any result is used
              uint32_t yy[kE], nd[kE], old[kE];
#pragma unroll
              for (uint32_t k = 0; k < kE; ++k) {
                const uint32_t j = min(j0 + k, cnt - 1u);
                yy[k] = (uint32_t)__shfl((int)ycol, (int)(hbase + j), 64);
                const uint32_t w = (uint32_t)__shfl((int)yw, (int)(hbase + j), 64);
                if (j0 + k >= cnt) yy[k] = kDown;  // past the row (half-uniform)
                nd[k] = d[u] + w;
                old[k] = 0u;
                if (act && !(yy[k] & kDown)) old[k] = wmin(&st.D[(size_t)yy[k] * kR + lane], nd[k]);
              }
              uint32_t im[kE], ip[kE];
#pragma unroll
              for (uint32_t k = 0; k < kE; ++k) {
                const bool imp = act && !(yy[k] & kDown) && nd[k] < old[k];
                im[k] = (uint32_t)(__ballot(imp) >> hbase);
                ip[k] = (uint32_t)(__ballot(imp && nd[k] < hi) >> hbase);
                if (imp && nd[k] >= hi) minN = min(minN, nd[k]);
              }
              if (lane == 0) {
                uint32_t sp[kE], sn[kE];
#pragma unroll
                for (uint32_t k = 0; k < kE; ++k) {
                  sp[k] = sn[k] = 0u;
                  if (!im[k]) continue;
                  wor(&st.dirty[yy[k]], im[k]);
                  if (ip[k]) sp[k] = wxchg(&st.stampP[yy[k]], nph);
                  if (im[k] & ~ip[k]) sn[k] = wxchg(&st.stampN[yy[k]], kb1);
                }
#pragma unroll
                for (uint32_t k = 0; k < kE; ++k) {
                  if (!im[k]) continue;
                  if (ip[k] && sp[k] != nph) LP[atomicAdd(&s_nP, 1u)] = yy[k];
                  if ((im[k] & ~ip[k]) && sn[k] != kb1) LN[atomicAdd(&s_nN, 1u)] = yy[k];
                }
              }
            }
          }
        }
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) minN = min(minN, (uint32_t)__shfl_xor((int)minN, o, 64));
      if (lane == 0 && minN != kInf) atomicMin(&s_minN, minN);
      __syncthreads();
      if (tid == 0) {
        const uint32_t c = s_ci, p = s_pi, nx = s_ni;
        if (s_nP > 0) {  // more of this bucket
          s_ci = p;
          s_pi = c;
          s_nC = s_nP;
        } else {         // the bucket is settled: on to the next one
          s_ci = nx;
          s_pi = c;
          s_ni = p;
          s_nC = s_nN;
          s_nN = 0u;
          if (s_minN != kInf) s_hi = max(s_hi + a.delta, (s_minN / a.delta + 1u) * a.delta);
          s_minN = kInf;
          s_kb += 1u;
        }
      }
      phase = nph;
      __syncthreads();
    }
    // rows: [V][32] -> 32 rows of V through LDS, 8 tiles of 32 nodes per
    // step: half-waves read nodes (their 32 roots, 128 B each), then write
    // roots' 32 nodes of each tile (128 B per store)
    for (uint32_t v0 = 0; v0 < V; v0 += 32u * kTiles) {
#pragma unroll
      for (uint32_t k = 0; k < kTiles; ++k)
        for (uint32_t x = hw; x < 32u; x += kHW) {
          const uint32_t v = v0 + 32u * k + x;
          s_t[k][x][lane] = v < V ? ld2(&st.D[(size_t)v * kR + lane]) : kInf;
        }
      __syncthreads();
      for (uint32_t rr = hw; rr < nr; rr += kHW) {
        uint32_t* row = a.dist + (size_t)(a.rowpos ? a.rowpos[r0 + rr] : r0 + rr) * a.pitch;
#pragma unroll
        for (uint32_t k = 0; k < kTiles; ++k) {
          const uint32_t v = v0 + 32u * k + lane;
          if (v < V) __builtin_nontemporal_store(s_t[k][lane][rr], row + v);
        }
      }
      __syncthreads();
    }
    __syncthreads();
  }
}

}  // namespace

size_t msdist_scratch_bytes(uint32_t V, uint32_t blocks) {
  return (size_t)V * (kR + 6u) * 4u * blocks;
}

hipError_t launch_msdist(const DevGraph& g, const MsDistArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (a.ngroups != (a.n + kR - 1) / kR || a.blocks == 0 || !a.scratch || a.delta == 0)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(msdist_kernel, dim3(a.blocks), dim3(kBlock), 0, s, g, a);
  return hipGetLastError();
}

}  // namespace ospf
