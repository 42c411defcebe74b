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
// visit of a node serves all 32 roots.
//
// Algorithm: Bellman-Ford by pulls in Delta buckets, no per-root atomics. A
// phase has a frontier F: nodes whose distance for some root was lowered in
// the previous phase to a value below the bucket end `hi`. (1) Expand: every
// neighbour of F becomes a candidate (once per phase: a stamp). (2) Pull:
// each candidate y, owned by one half-wave (lane = root), takes
// min(D[y], D[u] + w(u -> y)) over its up in-links from nodes u that relay for
// that root (transit, or the root itself: LinkState.cpp:859-866) and whose
// value lies below `hi`; lowered roots put y on the next frontier (below `hi`)
// or on the deferred list (at or past `hi`, with its smallest such value).
// When a phase leaves no frontier, the bucket advances past the smallest
// deferred value and the deferred nodes below the new end form the frontier.
// At the end every value has been pulled by every neighbour after its last
// change: the shortest distances (metrics >= 1, any order). Writes are
// owner-only (a candidate once per phase), so the state needs no per-root
// atomics; readers see old or new values, both upper bounds, and a lowered
// value is always followed by its node's expansion. Next hops and digests
// come from the rows afterwards (ospf_wderive_dev / ospf_wderive_wide_dev:
// the first hops of the shortest paths, LinkState.cpp:885-901).
//
// Shape: one workgroup (512 threads, 16 half-waves) per group, persistent over
// groups; group state in the block's scratch: dist [V][32], two stamps, the
// pending value per node and five lists [V].
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
constexpr uint32_t kU = 4;         // candidates per half-wave pulled at once
constexpr uint32_t kE = 4;         // in-links per candidate per step, loads in flight together
constexpr uint32_t kTiles = 8;     // 32-node tiles per transpose step (33.8 KB of LDS)
constexpr uint32_t kWords = kR + 8u;  // scratch words per node

__device__ __forceinline__ uint32_t ld2(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t wxchg(uint32_t* p, uint32_t v) {
  return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t wamin(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct MsdState {
  uint32_t* D;     // [V][32]
  uint32_t* stC;   // [V] phase that made the node a candidate
  uint32_t* stF;   // [V] phase that put the node on a frontier
  uint32_t* pend;  // [V] smallest deferred value (kInf: not on the deferred list)
  uint32_t* L;     // [5][V]: lists, roles rotating (s_buf)
};

__device__ __forceinline__ MsdState state_of(const MsDistArgs& a, uint32_t b, uint32_t V) {
  uint32_t* base = a.scratch + (size_t)V * kWords * b;
  MsdState s;
  s.D = base;
  s.stC = base + (size_t)V * kR;
  s.stF = s.stC + V;
  s.pend = s.stF + V;
  s.L = s.pend + V;
  return s;
}

__global__ void __launch_bounds__(kBlock, 4) msdist_kernel(DevGraph g, MsDistArgs a) {
  // list roles: 0 frontier, 1 next frontier, 2 candidates, 3 deferred,
  // 4 deferred being rebuilt; s_buf[role] = its buffer, s_n[role] = its fill
  __shared__ uint32_t s_n[5], s_buf[5];
  __shared__ uint32_t s_hi, s_minD, s_minD2;
  __shared__ uint32_t s_t[kTiles][32][33];  // row transpose tiles
  const uint32_t tid = threadIdx.x, lane = tid & 31u, hw = tid >> 5;
  const uint32_t hbase = (tid & 63u) & 32u;  // this half's first lane in the wave
  const uint32_t V = g.V;
  const MsdState st = state_of(a, blockIdx.x, V);
  for (uint32_t grp = blockIdx.x; grp < a.ngroups; grp += gridDim.x) {
    const uint32_t r0 = grp * kR, nr = min(kR, a.n - r0);
    {
      uint4* d4 = reinterpret_cast<uint4*>(st.D);
      const size_t n4 = (size_t)V * kR / 4u;
      const uint4 inf4 = make_uint4(kInf, kInf, kInf, kInf);
      for (size_t x = tid; x < n4; x += kBlock) d4[x] = inf4;
      for (uint32_t x = tid; x < V; x += kBlock) {
        st.stC[x] = kInf;
        st.stF[x] = kInf;
        st.pend[x] = kInf;
      }
    }
    if (tid < 5) {
      s_n[tid] = 0u;
      s_buf[tid] = tid;
    }
    if (tid == 0) {
      s_hi = a.delta;
      s_minD = kInf;
    }
    __syncthreads();
    const uint32_t myroot = lane < nr ? a.roots[r0 + lane] : kInf;
    if (hw == 0 && lane < nr) {
      st.D[(size_t)myroot * kR + lane] = 0u;
      if (wxchg(&st.stF[myroot], 0u) != 0u) st.L[atomicAdd(&s_n[0], 1u)] = myroot;
    }
    __syncthreads();
    uint32_t phase = 1;
    while (true) {
      const uint32_t nF = s_n[0];
      if (nF == 0) {
        // the bucket is done: advance past the smallest deferred value; the
        // deferred nodes below the new end form the frontier
        const uint32_t nD = s_n[3];
        if (nD == 0) break;  // block-uniform: nothing left anywhere
        // in 64 bits, saturated at kInf: near 2^32 the u32 form wrapped to a
        // small end no deferred value passes, and the block never drained;
        // a saturated end lets every finite deferred value join
        const uint64_t hi64 = max((uint64_t)s_hi + a.delta,
                                  ((uint64_t)(s_minD / a.delta) + 1u) * a.delta);
        const uint32_t hi = hi64 >= (uint64_t)kInf ? kInf : (uint32_t)hi64;
        uint32_t* LDef = st.L + (size_t)s_buf[3] * V;
        uint32_t* LDef2 = st.L + (size_t)s_buf[4] * V;
        uint32_t* LF = st.L + (size_t)s_buf[0] * V;
        __syncthreads();  // every thread has read the fills
        if (tid == 0) s_minD2 = kInf;
        __syncthreads();
        // half-wave per deferred node (lane = root): below the new end it
        // joins the frontier; its roots still at or past the end (never
        // propagated: values past `hi` are never pulled) keep it deferred
        uint32_t mn = kInf;
        for (uint32_t i = hw; i < nD; i += kHW) {
          const uint32_t y = ld2(LDef + i);
          const uint32_t p = ld2(&st.pend[y]);
          uint32_t keep = p;
          if (p < hi) {
            const uint32_t d = ld2(&st.D[(size_t)y * kR + lane]);
            keep = d >= hi && d != kInf ? d : kInf;
            for (int o = 16; o > 0; o >>= 1) keep = min(keep, (uint32_t)__shfl_xor((int)keep, o, 64));
          }
          if (lane == 0) {
            if (p < hi) {
              st.pend[y] = keep;
              if (wxchg(&st.stF[y], phase) != phase) LF[atomicAdd(&s_n[0], 1u)] = y;
            }
            if (keep != kInf) {
              LDef2[atomicAdd(&s_n[4], 1u)] = y;
              mn = min(mn, keep);
            }
          }
        }
        for (int o = 32; o > 0; o >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
        if ((tid & 63u) == 0 && mn != kInf) atomicMin(&s_minD2, mn);
        __syncthreads();
        if (tid == 0) {
          s_hi = hi;
          s_n[3] = s_n[4];
          s_n[4] = 0u;
          const uint32_t t = s_buf[3];
          s_buf[3] = s_buf[4];
          s_buf[4] = t;
          s_minD = s_minD2;
        }
        phase += 1u;
        __syncthreads();
        continue;
      }
      const uint32_t hi = s_hi;
      uint32_t* LF = st.L + (size_t)s_buf[0] * V;
      uint32_t* LNF = st.L + (size_t)s_buf[1] * V;
      uint32_t* LC = st.L + (size_t)s_buf[2] * V;
      uint32_t* LDef = st.L + (size_t)s_buf[3] * V;
      if (a.stats && tid == 0) {
        atomicAdd(&a.stats[0], 1ull);
        atomicAdd(&a.stats[1], (unsigned long long)nF);
      }
      // (1) expand: the frontier's neighbours become candidates (lane = edge)
      for (uint32_t i = hw; i < nF; i += kHW) {
        const uint32_t f = ld2(LF + i);
        const uint32_t beg = g.row_ptr[f], deg = g.row_ptr[f + 1] - beg;
        for (uint32_t e0 = 0; e0 < deg; e0 += kR) {
          uint32_t y = kDown;
          if (e0 + lane < deg) y = g.ew ? g.ew[beg + e0 + lane].x : g.colx[beg + e0 + lane];
          const bool fresh = !(y & kDown) && wxchg(&st.stC[y], phase) != phase;
          const uint32_t m = (uint32_t)(__ballot(fresh) >> hbase);
          if (!m) continue;
          uint32_t pos = 0;
          if (lane == 0) pos = atomicAdd(&s_n[2], (uint32_t)__popc(m));
          pos = (uint32_t)__shfl((int)pos, (int)hbase, 64);
          if (fresh) LC[pos + __popc(m & ((1u << lane) - 1u))] = y;
        }
      }
      __syncthreads();
      const uint32_t nC = s_n[2];
      if (a.stats && tid == 0) atomicAdd(&a.stats[2], (unsigned long long)nC);
      // (2) pull: kU candidates per half-wave at once, lane = root; their
      // first 32 in-links' loads in flight together (kE per candidate per
      // step), the rest of a wider row after
      uint32_t mnD = kInf;
      for (uint32_t i0 = hw * kU; i0 < nC; i0 += kHW * kU) {
        uint32_t y[kU], beg[kU], deg[kU], dy[kU], best[kU], ucol[kU], uw[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) y[u] = i0 + u < nC ? ld2(LC + i0 + u) : kInf;
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          beg[u] = deg[u] = 0u;
          if (y[u] == kInf) continue;
          beg[u] = g.row_ptr[y[u]];
          deg[u] = g.row_ptr[y[u] + 1] - beg[u];
        }
        uint32_t dmax = 0;
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          dy[u] = y[u] == kInf ? 0u : ld2(&st.D[(size_t)y[u] * kR + lane]);
          best[u] = dy[u];
          ucol[u] = kDown;
          uw[u] = 0u;
          if (lane < deg[u]) {
            const uint32_t e = beg[u] + lane;
            if (g.ew) {
              const uint2 x = g.ew[e];
              ucol[u] = x.x;
              uw[u] = x.y >> 16;  // metric of the link u -> y
            } else {
              ucol[u] = g.colx[e];
              uw[u] = g.rw[e];
            }
            if (a.hop) uw[u] = 1u;
          }
          dmax = max(dmax, min(deg[u], kR));
        }
        for (uint32_t j0 = 0; j0 < dmax; j0 += kE) {
          uint32_t uu[kU][kE], du[kU][kE];
#pragma unroll
          for (uint32_t u = 0; u < kU; ++u)
#pragma unroll
            for (uint32_t k = 0; k < kE; ++k) {
              uu[u][k] = (uint32_t)__shfl((int)ucol[u], (int)(hbase + min(j0 + k, kR - 1u)), 64);
              if (j0 + k >= min(deg[u], kR)) uu[u][k] = kDown;
              du[u][k] = (uu[u][k] & kDown) ? kInf : ld2(&st.D[(size_t)uu[u][k] * kR + lane]);
            }
#pragma unroll
          for (uint32_t u = 0; u < kU; ++u)
#pragma unroll
            for (uint32_t k = 0; k < kE; ++k) {
              const uint32_t w = (uint32_t)__shfl((int)uw[u], (int)(hbase + min(j0 + k, kR - 1u)), 64);
              if (du[u][k] >= hi) continue;  // unreached, or not settled into the bucket yet
              const uint32_t x = uu[u][k];
              const bool relay = x == myroot || !((g.nt_bits[x >> 5] >> (x & 31u)) & 1u);
              if (relay) best[u] = min(best[u], du[u][k] + w);
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          for (uint32_t e = kR; e < deg[u]; ++e) {  // rows past 32 in-links (rare)
            uint32_t x, w;
            if (g.ew) {
              const uint2 q = g.ew[beg[u] + e];
              x = q.x;
              w = q.y >> 16;
            } else {
              x = g.colx[beg[u] + e];
              w = g.rw[beg[u] + e];
            }
            if (a.hop) w = 1u;
            if (x & kDown) continue;
            const uint32_t dx = ld2(&st.D[(size_t)x * kR + lane]);
            const bool relay = x == myroot || !((g.nt_bits[x >> 5] >> (x & 31u)) & 1u);
            if (dx < hi && relay) best[u] = min(best[u], dx + w);
          }
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          if (y[u] == kInf) continue;
          const bool ch = best[u] < dy[u];
          if (ch) st.D[(size_t)y[u] * kR + lane] = best[u];
          const uint32_t cm = (uint32_t)(__ballot(ch) >> hbase);
          if (!cm) continue;
          const uint32_t lt = (uint32_t)(__ballot(ch && best[u] < hi) >> hbase);
          uint32_t late = (ch && best[u] >= hi) ? best[u] : kInf;
          for (int o = 16; o > 0; o >>= 1) late = min(late, (uint32_t)__shfl_xor((int)late, o, 64));
          if (lane == 0) {
            if (lt && wxchg(&st.stF[y[u]], phase) != phase) LNF[atomicAdd(&s_n[1], 1u)] = y[u];
            if (late != kInf) {
              mnD = min(mnD, late);
              if (wamin(&st.pend[y[u]], late) == kInf) LDef[atomicAdd(&s_n[3], 1u)] = y[u];
            }
          }
        }
      }
      for (int o = 32; o > 0; o >>= 1) mnD = min(mnD, (uint32_t)__shfl_xor((int)mnD, o, 64));
      if ((tid & 63u) == 0 && mnD != kInf) atomicMin(&s_minD, mnD);
      __syncthreads();
      if (tid == 0) {  // next frontier -> frontier; candidates emptied
        s_n[0] = s_n[1];
        s_n[1] = 0u;
        s_n[2] = 0u;
        const uint32_t t = s_buf[0];
        s_buf[0] = s_buf[1];
        s_buf[1] = t;
      }
      phase += 1u;
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
  }
}

}  // namespace

size_t msdist_scratch_bytes(uint32_t V, uint32_t blocks) {
  return (size_t)V * kWords * 4u * blocks;
}

hipError_t launch_msdist(const DevGraph& g, const MsDistArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (a.ngroups != (a.n + kR - 1) / kR || a.blocks == 0 || !a.scratch || a.delta == 0)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(msdist_kernel, dim3(a.blocks), dim3(kBlock), 0, s, g, a);
  return hipGetLastError();
}

}  // namespace ospf
