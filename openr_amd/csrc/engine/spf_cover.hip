// spf_cover.hip — distance rows of cover roots by a contracted-graph SPF with
// LDS-resident distances (gfx950), any metric.
//
// Weighted all-sources sweeps split the nodes into an independent set of leaf
// roots (no two adjacent; the racks of a fabric) and the cover (the rest).
// Every shortest path between cover nodes visits leaves only as single-node
// detours a -> x -> b (a leaf's neighbours are all cover nodes), and only
// through transit leaves (overloaded nodes never relay, LinkState.cpp:
// 859-866). So the cover's distances are those of the contracted graph C:
// nodes = the cover, edges = the up links between cover nodes plus one
// shortcut a -> b per transit leaf x with up links a - x - b, weight w(a -> x)
// + w(x -> b), parallel ones collapsed to their minimum. A leaf's distance is
// then min over its up in-links a -> x of D(a) + w(a -> x), a transit or the
// root (Bellman's equation on the last hop) -- the reference's runSpf
// distances (LinkState.cpp:836-911) with metrics >= 1.
//
// Kernel: a workgroup per root (persistent), the root's distances over the
// cover in LDS (F100k: 14,536 cover nodes = 58 KB, two roots per CU). Dial
// rounds by distance value t: every wave scans its share of the cover for
// nodes at t (settled: metrics >= 1 never lower a value to t), queues the
// transit ones (and the root), and expands the queue flat -- one trip for the
// row bounds of up to 64 queued nodes, one for their edges -- with LDS
// atomicMin relaxations; the next t is the minimum of the scan's unsettled
// values and of this round's new values. The row is then written in node
// order: cover nodes from LDS, leaves by the last-hop minimum over their
// (padded, 16-B) in-link lists. Next hops are derived afterwards from the
// neighbours' rows (ospf_wderive_dev).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kLeaf = 0x80000000u;
constexpr int kWave = 64;
constexpr uint32_t kBlock = 512;  // 8 waves per root: shorter scans and expansions per round
constexpr uint32_t kWaves = kBlock / kWave;
constexpr uint32_t kQ = 256;  // per-wave frontier queue

__device__ __forceinline__ uint32_t wave_min32(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o, kWave));
  return x;
}
__device__ __forceinline__ uint32_t wave_max32(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, kWave));
  return x;
}
// Closure early exit (wave-uniform): the terms are sorted by their smallest
// constant over the members, and a seed column is >= 0, so once that constant
// exceeds every lane's accumulator of every member in use no later term can
// improve or tie any of them.
template <int KW>
__device__ __forceinline__ bool closure_done(const uint32_t* acc, const uint32_t* cst_j,
                                             uint32_t used, bool ok) {
  uint32_t mx = 0, cmin = kClInf;
#pragma unroll
  for (int f = 0; f < KW; ++f)
    if ((used >> f) & 1u) {
      mx = max(mx, acc[f]);
      cmin = min(cmin, cst_j[f]);
    }
  mx = wave_max32(ok ? mx : 0u);
  return cmin > mx;
}

// expand queued nodes q[0 .. cnt) (this wave's) at distance t: 64 nodes per
// pass, their edges flattened over the lanes
__device__ __forceinline__ void expand(const CoverGraph& C, uint32_t* s_D, uint32_t* s_next,
                                       const uint32_t* q, uint32_t cnt, uint32_t* s_pre,
                                       uint32_t t, uint32_t lane) {
  for (uint32_t b0 = 0; b0 < cnt; b0 += kWave) {
    const uint32_t j = b0 + lane;
    uint32_t beg = 0, deg = 0;
    if (j < cnt) {
      const uint32_t u = q[j];
      beg = C.crow[u];
      deg = C.crow[u + 1] - beg;
    }
    uint32_t inc = deg;  // inclusive prefix over the lanes
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, o, kWave);
      if (lane >= (uint32_t)o) inc += y;
    }
    s_pre[lane] = inc;
    s_pre[kWave + lane] = beg;
    __builtin_amdgcn_wave_barrier();
    const uint32_t total = (uint32_t)__shfl((int)inc, kWave - 1, kWave);
    // kU edges per lane per step, every load issued before any relaxation (a
    // 1,781-edge spine is 7 trips, not 28)
    constexpr uint32_t kU = 16;
    for (uint32_t f0 = 0; f0 < total; f0 += kWave * kU) {
      uint2 ed[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t f = f0 + u * kWave + lane;
        ed[u] = make_uint2(0u, kInf);
        if (f < total) {
          uint32_t lo = 0, hi = kWave - 1;  // first k with pre[k] > f
#pragma unroll
          for (int it = 0; it < 6; ++it) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_pre[mid] > f) hi = mid;
            else lo = mid + 1;
          }
          const uint32_t before = lo ? s_pre[lo - 1] : 0u;
          ed[u] = C.cedge[s_pre[kWave + lo] + (f - before)];
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        if (ed[u].y == kInf) continue;
        const uint32_t nd = t + ed[u].y;
        const uint32_t old = atomicMin(&s_D[ed[u].x], nd);
        if (nd < old) atomicMin(s_next, nd);
      }
    }
    __builtin_amdgcn_wave_barrier();  // s_pre is rewritten by the next pass
  }
}

// The root's row in node order: cover nodes from LDS, leaves by their last
// hop (min over their up in-links from transit cover nodes or the root);
// four nodes per thread per step, their first two in-link quads loaded before
// any is used (a rack's 8 entries).
__device__ __forceinline__ void write_row(const DevGraph& g, const CoverGraph& C, uint32_t* row,
                                          const uint32_t* s_D, const uint32_t* s_tr, uint32_t r,
                                          uint32_t tid, uint32_t nthreads) {
  const uint32_t nS = C.nS, V = g.V;
  const uint4* la4 = reinterpret_cast<const uint4*>(C.ladj);
  const uint4 pad = make_uint4(0xFFFFu, 0xFFFFu, 0xFFFFu, 0xFFFFu);
  auto fold = [&](uint4 e4, uint32_t out) {
    const uint32_t es[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t ci = es[b] & 0xFFFFu;
      if (ci >= nS) continue;  // padding
      if (!((s_tr[ci >> 5] >> (ci & 31u)) & 1u) && ci != r) continue;
      const uint32_t d = s_D[ci];
      if (d != kInf) out = min(out, d + (es[b] >> 16));
    }
    return out;
  };
  for (uint32_t v0 = tid; v0 < V; v0 += 4u * nthreads) {
    uint32_t c4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t v = v0 + (uint32_t)k * nthreads;
      c4[k] = v < V ? C.cix[v] : 0u;
    }
    uint4 e0[4], e1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e0[k] = e1[k] = pad;
      if (c4[k] & kLeaf) {
        const uint32_t q0 = (c4[k] >> 5) & 0x3FFFFFFu, nq = c4[k] & 31u;
        if (nq > 0) e0[k] = la4[q0];
        if (nq > 1) e1[k] = la4[q0 + 1];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t v = v0 + (uint32_t)k * nthreads;
      if (v >= V) continue;
      uint32_t out;
      if (!(c4[k] & kLeaf)) {
        out = s_D[c4[k]];
      } else {
        out = fold(e1[k], fold(e0[k], kInf));
        const uint32_t q0 = (c4[k] >> 5) & 0x3FFFFFFu, nq = c4[k] & 31u;
        for (uint32_t qq = 2; qq < nq; ++qq) out = fold(la4[q0 + qq], out);
      }
      __builtin_nontemporal_store(out, row + v);
    }
  }
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int o) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, o, kWave);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), o, kWave);
  return ((uint64_t)hi << 32) | lo;
}

// Load mode with next hops (closure roots): the dist row as write_row, the
// next-hop row [V][NW] -- cover columns from the closure's masks, a leaf by
// the OR of its tight last hops' masks (the root itself as a last hop: the
// leaf's own bit; LinkState.cpp:885-901) -- and the run's digest (DESIGN.md
// §4) summed into dg.
template <int NW>
__device__ __forceinline__ void write_row_nh(const DevGraph& g, const CoverGraph& C, uint32_t* row,
                             uint32_t* nhrow, const uint32_t* s_D, const uint32_t* s_tr,
                             uint32_t r, uint32_t rn, const uint32_t* cm, ospf_digest* dg,
                             unsigned long long* s_acc, uint32_t* s_st, uint32_t tid,
                             uint32_t nthreads) {
  const uint32_t nS = C.nS, V = g.V, lane = tid & 63u;
  const uint4* la4 = reinterpret_cast<const uint4*>(C.ladj);
  const uint32_t* dn = g.dn + g.dn_off[rn];
  const uint32_t K = g.dn_off[rn + 1] - g.dn_off[rn];
  auto usable = [&](uint32_t ci) {
    return ci < nS && (ci == r || ((s_tr[ci >> 5] >> (ci & 31u)) & 1u));
  };
  uint64_t h = 0, sum = 0;
  uint32_t reach = 0;
  // a block step = nthreads consecutive nodes; their next-hop words leave
  // through LDS as one contiguous run (lane-strided NW-word records would
  // write partial lines). Loads run ahead: the next step's first two in-link
  // quads and the step after's cover index are issued before this step's
  // nodes are folded.
  const uint4 pad = make_uint4(0xFFFFu, 0xFFFFu, 0xFFFFu, 0xFFFFu);
  auto quads = [&](uint32_t vv, uint32_t cx, uint4& a, uint4& b) {
    a = b = pad;
    if (vv < V && (cx & kLeaf)) {
      const uint32_t q0 = (cx >> 5) & 0x3FFFFFFu, nq = cx & 31u;
      if (nq > 0) a = la4[q0];
      if (nq > 1) b = la4[q0 + 1];
    }
  };
  uint32_t cxA = tid < V ? C.cix[tid] : 0u;
  uint32_t cxB = tid + nthreads < V ? C.cix[tid + nthreads] : 0u;
  uint4 qA0, qA1;
  quads(tid, cxA, qA0, qA1);
  for (uint32_t v0 = 0; v0 < V; v0 += nthreads) {
    const uint32_t v = v0 + tid;
    uint4 qB0, qB1;
    quads(v + nthreads, cxB, qB0, qB1);
    const uint32_t cxC = v + 2u * nthreads < V ? C.cix[v + 2u * nthreads] : 0u;
    uint32_t out = kInf, m[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) m[w] = 0u;
    if (v < V) {
      const uint32_t cx = cxA;
      if (!(cx & kLeaf)) {
        out = s_D[cx];
#pragma unroll
        for (int w = 0; w < NW; ++w) m[w] = cm[(size_t)cx * NW + w];
      } else {
        const uint32_t q0 = (cx >> 5) & 0x3FFFFFFu, nq = cx & 31u;
        const uint32_t es[8] = {qA0.x, qA0.y, qA0.z, qA0.w, qA1.x, qA1.y, qA1.z, qA1.w};
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const uint32_t ci = es[b] & 0xFFFFu;
          if (!usable(ci) || s_D[ci] == kInf) continue;
          out = min(out, s_D[ci] + (es[b] >> 16));
        }
        for (uint32_t qq = 2; qq < nq; ++qq) {
          const uint4 e4 = la4[q0 + qq];
          const uint32_t ex[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const uint32_t ci = ex[b] & 0xFFFFu;
            if (!usable(ci) || s_D[ci] == kInf) continue;
            out = min(out, s_D[ci] + (ex[b] >> 16));
          }
        }
        auto tight = [&](uint32_t e) {
          const uint32_t ci = e & 0xFFFFu;
          if (!usable(ci) || s_D[ci] == kInf || s_D[ci] + (e >> 16) != out) return;
          if (ci == r) {  // a neighbour of the root: its own bit
            uint32_t lo = 0, hi = K;
            while (lo < hi) {
              const uint32_t mid = (lo + hi) >> 1;
              if (dn[mid] < v) lo = mid + 1;
              else hi = mid;
            }
            if (lo < 32u * NW) m[lo >> 5] |= 1u << (lo & 31u);
          } else {
#pragma unroll
            for (int w = 0; w < NW; ++w) m[w] |= cm[(size_t)ci * NW + w];
          }
        };
        if (out != kInf) {
#pragma unroll
          for (int b = 0; b < 8; ++b) tight(es[b]);
          for (uint32_t qq = 2; qq < nq; ++qq) {
            const uint4 e4 = la4[q0 + qq];
            tight(e4.x);
            tight(e4.y);
            tight(e4.z);
            tight(e4.w);
          }
        }
      }
      if (v == rn || out == kInf) {
#pragma unroll
        for (int w = 0; w < NW; ++w) m[w] = 0u;
      }
      __builtin_nontemporal_store(out, row + v);
      if (out != kInf) {
        reach += 1u;
        sum += out;
        h += g.dkey[2ull * v] * ((uint64_t)out + 1ull);
        uint64_t ws = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w)
          if (m[w]) ws += digest_word_key((uint32_t)w, m[w]);
        if (ws) h += g.dkey[2ull * v + 1] * ws;
      }
    }
#pragma unroll
    for (int w = 0; w < NW; ++w) s_st[tid * NW + w] = m[w];
    __syncthreads();
    const size_t base = (size_t)v0 * NW, lim = (size_t)V * NW;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const size_t i = (size_t)w * nthreads + tid;
      if (base + i < lim) __builtin_nontemporal_store(s_st[i], nhrow + base + i);
    }
    __syncthreads();  // s_st is rewritten by the next step
    cxA = cxB;
    qA0 = qB0;
    qA1 = qB1;
    cxB = cxC;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    h += shfl_xor64(h, o);
    sum += shfl_xor64(sum, o);
    reach += (uint32_t)__shfl_xor((int)reach, o, kWave);
  }
  if (lane == 0 && reach) {
    atomicAdd(&s_acc[0], (unsigned long long)reach);
    atomicAdd(&s_acc[1], (unsigned long long)sum);
    atomicAdd(&s_acc[2], (unsigned long long)h);
  }
  __syncthreads();
  if (tid == 0 && dg) {
    atomicAdd((unsigned long long*)&dg->reached, s_acc[0]);
    atomicAdd((unsigned long long*)&dg->sum_dist, s_acc[1]);
    atomicAdd((unsigned long long*)&dg->hash, s_acc[2]);
  }
}

// write_row_nh over a TAGGED column array: s_D[k] | 0x80000000 where cover
// node k is non-transit and not the root (it relays for no leaf), s_D[nS] =
// kInf (the padding slot). A leaf's term is then one saturating add per
// in-link, tight where it equals the minimum; no transit-bit lookups.
template <int NW>
__device__ __forceinline__ void write_row_nh_tag(const DevGraph& g, const CoverGraph& C, uint32_t* row,
                             uint32_t* nhrow, const uint32_t* s_D, const uint32_t* s_tr,
                             uint32_t r, uint32_t rn, const uint32_t* cm, ospf_digest* dg,
                             unsigned long long* s_acc, uint32_t* s_st, uint32_t tid,
                             uint32_t nthreads) {
  const uint32_t nS = C.nS, V = g.V, lane = tid & 63u;
  const uint4* la4 = reinterpret_cast<const uint4*>(C.ladj);
  const uint32_t* dn = g.dn + g.dn_off[rn];
  const uint32_t K = g.dn_off[rn + 1] - g.dn_off[rn];
  uint64_t h = 0, sum = 0;
  uint32_t reach = 0;
  // a block step = nthreads consecutive nodes; their next-hop words leave
  // through LDS as one contiguous run (lane-strided NW-word records would
  // write partial lines). Loads run ahead: the next step's first two in-link
  // quads and the step after's cover index are issued before this step's
  // nodes are folded.
  const uint4 pad = make_uint4(0xFFFFu, 0xFFFFu, 0xFFFFu, 0xFFFFu);
  auto quads = [&](uint32_t vv, uint32_t cx, uint4& a, uint4& b) {
    a = b = pad;
    if (vv < V && (cx & kLeaf)) {
      const uint32_t q0 = (cx >> 5) & 0x3FFFFFFu, nq = cx & 31u;
      if (nq > 0) a = la4[q0];
      if (nq > 1) b = la4[q0 + 1];
    }
  };
  uint32_t cxA = tid < V ? C.cix[tid] : 0u;
  uint32_t cxB = tid + nthreads < V ? C.cix[tid + nthreads] : 0u;
  uint4 qA0, qA1;
  quads(tid, cxA, qA0, qA1);
  for (uint32_t v0 = 0; v0 < V; v0 += nthreads) {
    const uint32_t v = v0 + tid;
    uint4 qB0, qB1;
    quads(v + nthreads, cxB, qB0, qB1);
    const uint32_t cxC = v + 2u * nthreads < V ? C.cix[v + 2u * nthreads] : 0u;
    uint32_t out = kInf, m[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) m[w] = 0u;
    if (v < V) {
      const uint32_t cx = cxA;
      if (!(cx & kLeaf)) {
        out = s_D[cx];
        if (out != kInf) out &= 0x7FFFFFFFu;  // a non-transit cover node's own column
#pragma unroll
        for (int w = 0; w < NW; ++w) m[w] = cm[(size_t)cx * NW + w];
      } else {
        const uint32_t q0 = (cx >> 5) & 0x3FFFFFFu, nq = cx & 31u;
        const uint32_t es[8] = {qA0.x, qA0.y, qA0.z, qA0.w, qA1.x, qA1.y, qA1.z, qA1.w};
        // a term: the tagged column (bit 31: a non-transit last hop, kInf:
        // unreached or padding) + the in-link's metric, saturating
        auto term = [&](uint32_t e) {
          const uint32_t x = s_D[min(e & 0xFFFFu, nS)], c = x + (e >> 16);
          return c < x ? kInf : c;
        };
#pragma unroll
        for (int b = 0; b < 8; ++b) out = min(out, term(es[b]));
        for (uint32_t qq = 2; qq < nq; ++qq) {
          const uint4 e4 = la4[q0 + qq];
          out = min(out, min(min(term(e4.x), term(e4.y)), min(term(e4.z), term(e4.w))));
        }
        auto tight = [&](uint32_t e) {
          if ((e & 0xFFFFu) == r) {  // a neighbour of the root: its own bit
            uint32_t lo = 0, hi = K;
            while (lo < hi) {
              const uint32_t mid = (lo + hi) >> 1;
              if (dn[mid] < v) lo = mid + 1;
              else hi = mid;
            }
            if (lo < 32u * NW) m[lo >> 5] |= 1u << (lo & 31u);
          } else {
            const uint32_t ci = e & 0xFFFFu;
#pragma unroll
            for (int w = 0; w < NW; ++w) m[w] |= cm[(size_t)ci * NW + w];
          }
        };
        if (out >= 0x80000000u) {  // no usable last hop reaches v
          out = kInf;
        } else {
#pragma unroll
          for (int b = 0; b < 8; ++b)
            if (term(es[b]) == out) tight(es[b]);
          for (uint32_t qq = 2; qq < nq; ++qq) {
            const uint4 e4 = la4[q0 + qq];
            if (term(e4.x) == out) tight(e4.x);
            if (term(e4.y) == out) tight(e4.y);
            if (term(e4.z) == out) tight(e4.z);
            if (term(e4.w) == out) tight(e4.w);
          }
        }
      }
      if (v == rn || out == kInf) {
#pragma unroll
        for (int w = 0; w < NW; ++w) m[w] = 0u;
      }
      __builtin_nontemporal_store(out, row + v);
      if (out != kInf) {
        reach += 1u;
        sum += out;
        h += g.dkey[2ull * v] * ((uint64_t)out + 1ull);
        uint64_t ws = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w)
          if (m[w]) ws += digest_word_key((uint32_t)w, m[w]);
        if (ws) h += g.dkey[2ull * v + 1] * ws;
      }
    }
#pragma unroll
    for (int w = 0; w < NW; ++w) s_st[tid * NW + w] = m[w];
    __syncthreads();
    const size_t base = (size_t)v0 * NW, lim = (size_t)V * NW;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const size_t i = (size_t)w * nthreads + tid;
      if (base + i < lim) __builtin_nontemporal_store(s_st[i], nhrow + base + i);
    }
    __syncthreads();  // s_st is rewritten by the next step
    cxA = cxB;
    qA0 = qB0;
    qA1 = qB1;
    cxB = cxC;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    h += shfl_xor64(h, o);
    sum += shfl_xor64(sum, o);
    reach += (uint32_t)__shfl_xor((int)reach, o, kWave);
  }
  if (lane == 0 && reach) {
    atomicAdd(&s_acc[0], (unsigned long long)reach);
    atomicAdd(&s_acc[1], (unsigned long long)sum);
    atomicAdd(&s_acc[2], (unsigned long long)h);
  }
  __syncthreads();
  if (tid == 0 && dg) {
    atomicAdd((unsigned long long*)&dg->reached, s_acc[0]);
    atomicAdd((unsigned long long*)&dg->sum_dist, s_acc[1]);
    atomicAdd((unsigned long long*)&dg->hash, s_acc[2]);
  }
}

// Seed next hops, during the Dial: the cover nodes this wave scans that
// settled at t (metrics >= 1: their tight in-edges come from nodes settled
// before t, whose masks are written) get the OR over their tight in-edges
// a -> b (a transit or the root, D(a) + w == t) of a's mask, or, for the
// root's own edge, of its first-hop bits (cfh: the direct link's or the
// detour leaf's position in the root's distinct neighbours) -- the
// reference's next hops (LinkState.cpp:885-901: a path's next hop is its
// first hop). Lane = mask word; up to 8 predecessor masks loaded at once.
__device__ __forceinline__ void seed_masks(const CoverGraph& C, const uint32_t* s_D,
                                           const uint32_t* s_tr, uint32_t r, uint32_t t,
                                           uint32_t* __restrict__ cm, uint32_t NW, uint32_t* s_mw,
                                           uint32_t wave, uint32_t lane) {
  const uint32_t nS = C.nS;
  const bool wl = lane < NW;
  for (uint32_t x0 = wave * kWave; x0 < nS; x0 += kBlock) {
    const uint32_t x = x0 + lane;
    uint64_t ball = __ballot(x < nS && x != r && s_D[x] == t);
    while (ball) {
      const uint32_t b = x0 + (uint32_t)__builtin_ctzll(ball);
      ball &= ball - 1ull;
      const uint32_t beg = C.crin[b], end = C.crin[b + 1];
      uint32_t acc = 0u;
      for (uint32_t e0 = beg; e0 < end; e0 += kWave) {
        const uint32_t e = e0 + lane;
        uint32_t src = kInf;
        bool tight = false;
        if (e < end) {
          const uint2 ew = C.cein[e];
          src = ew.x;
          const bool ok = src == r || ((s_tr[src >> 5] >> (src & 31u)) & 1u);
          const uint32_t ds = s_D[src];
          tight = ok && ds != kInf && ds + ew.y == t;
        }
        const uint64_t br = __ballot(tight && src == r);
        if (br) {  // the root's own C edge to b: its first hops
          const uint32_t ce = C.ceix[e0 + (uint32_t)__builtin_ctzll(br)];
          const uint32_t fo = C.cfh_off[ce], fe = C.cfh_off[ce + 1];
          for (uint32_t k = fo + lane; k < fe; k += kWave) {
            const uint32_t bit = C.cfh[k];
            atomicOr(&s_mw[bit >> 5], 1u << (bit & 31u));
          }
          __builtin_amdgcn_wave_barrier();
          acc |= s_mw[lane];
          __builtin_amdgcn_wave_barrier();
          s_mw[lane] = 0u;
          __builtin_amdgcn_wave_barrier();
        }
        uint64_t bt = __ballot(tight && src != r);
        while (bt) {
          uint32_t m[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            m[u] = 0u;
            if (bt) {
              const int j = __builtin_ctzll(bt);
              bt &= bt - 1ull;
              const uint32_t a = (uint32_t)__shfl((int)src, j, kWave);
              if (wl) m[u] = cm[(size_t)a * NW + lane];
            }
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) acc |= m[u];
        }
      }
      if (wl) cm[(size_t)b * NW + lane] = acc;
    }
  }
}

// The seed root's dist row, next-hop row [V][NW] (NW <= 64) and digest:
// lane = node for the distances and the tight last hops of a leaf (its
// first two recorded, the root as a last hop by the leaf's bit), then lane
// = mask word over the 64 nodes, four at a time, their masks loaded before
// any is used (a cover column's mask as it is; a leaf's the OR over its
// tight last hops', LinkState.cpp:885-901).
__device__ __forceinline__ void write_row_nhw(const DevGraph& g, const CoverGraph& C, uint32_t* row,
                              uint32_t* __restrict__ nhrow, const uint32_t* s_D,
                              const uint32_t* s_tr, uint32_t r, uint32_t rn,
                              const uint32_t* __restrict__ cm, uint32_t NW, ospf_digest* dg,
                              unsigned long long* s_acc, uint32_t wave, uint32_t lane,
                              uint32_t vbeg, uint32_t vend) {
  // nodes [vbeg, vend) of the row (vbeg a multiple of 64); the digest parts
  // of several ranges add up
  const uint32_t nS = C.nS, V = vend;
  const uint4* la4 = reinterpret_cast<const uint4*>(C.ladj);
  const uint32_t* dn = g.dn + g.dn_off[rn];
  const uint32_t K = g.dn_off[rn + 1] - g.dn_off[rn];
  const bool wl = lane < NW;
  auto usable = [&](uint32_t ci) {
    return ci < nS && (ci == r || ((s_tr[ci >> 5] >> (ci & 31u)) & 1u));
  };
  auto fold = [&](uint4 e4, uint32_t out) {
    const uint32_t es[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t ci = es[b] & 0xFFFFu;
      if (!usable(ci)) continue;
      const uint32_t d = s_D[ci];
      if (d != kInf) out = min(out, d + (es[b] >> 16));
    }
    return out;
  };
  auto rootbit = [&](uint32_t v) {
    uint32_t lo = 0, hi = K;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (dn[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  const uint4 pad = make_uint4(0xFFFFu, 0xFFFFu, 0xFFFFu, 0xFFFFu);
  uint64_t h = 0, sum = 0;
  uint32_t reach = 0;
  for (uint32_t v0 = vbeg + wave * kWave; v0 < V; v0 += kBlock) {
    const uint32_t v = v0 + lane;
    // lane = node: distance, first two tight last hops (cover indices), the
    // root's bit, and whether more remain (then the word pass rescans)
    uint32_t out = kInf, t0 = kInf, t1 = kInf, rb = kInf, more = 0u;
    if (v < V) {
      const uint32_t cx = C.cix[v];
      if (!(cx & kLeaf)) {
        out = s_D[cx];
        if (cx != r) t0 = cx;
      } else {
        const uint32_t q0 = (cx >> 5) & 0x3FFFFFFu, nq = cx & 31u;
        const uint4 e0 = nq > 0 ? la4[q0] : pad, e1 = nq > 1 ? la4[q0 + 1] : pad;
        out = fold(e1, fold(e0, kInf));
        for (uint32_t qq = 2; qq < nq; ++qq) out = fold(la4[q0 + qq], out);
        if (out != kInf) {
          bool hit_r = false;
          auto tight = [&](uint32_t e) {
            const uint32_t ci = e & 0xFFFFu;
            if (!usable(ci) || s_D[ci] == kInf || s_D[ci] + (e >> 16) != out) return;
            if (ci == r) hit_r = true;
            else if (t0 == kInf) t0 = ci;
            else if (t1 == kInf) t1 = ci;
            else more = 1u;
          };
          tight(e0.x); tight(e0.y); tight(e0.z); tight(e0.w);
          tight(e1.x); tight(e1.y); tight(e1.z); tight(e1.w);
          if (hit_r) rb = rootbit(v);
          if (nq > 2) more = 1u;
        }
      }
      if (v == rn || out == kInf) t0 = t1 = rb = kInf, more = 0u;
      __builtin_nontemporal_store(out, row + v);
      if (out != kInf) {
        reach += 1u;
        sum += out;
        h += g.dkey[2ull * v] * ((uint64_t)out + 1ull);
      }
    }
    // lane = word: the 64 nodes' masks, four nodes per step
    const uint32_t cnt = min((uint32_t)kWave, V - v0);
    for (uint32_t j0 = 0; j0 < cnt; j0 += 4u) {
      uint32_t m[4][2], sv[4][2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = (int)min(j0 + (uint32_t)u, cnt - 1u);
        sv[u][0] = (uint32_t)__builtin_amdgcn_readlane((int)t0, j);
        sv[u][1] = (uint32_t)__builtin_amdgcn_readlane((int)t1, j);
        if (j0 + (uint32_t)u >= cnt) sv[u][0] = sv[u][1] = kInf;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int p = 0; p < 2; ++p)
          m[u][p] = (sv[u][p] != kInf && wl) ? cm[(size_t)sv[u][p] * NW + lane] : 0u;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t j = min(j0 + (uint32_t)u, cnt - 1u);
        if (j0 + (uint32_t)u >= cnt) continue;  // uniform
        const uint32_t vj = v0 + j;
        uint32_t acc = m[u][0] | m[u][1];
        const uint32_t rbj = (uint32_t)__builtin_amdgcn_readlane((int)rb, (int)j);
        if (rbj != kInf && (rbj >> 5) == lane) acc |= 1u << (rbj & 31u);
        if (__builtin_amdgcn_readlane((int)more, (int)j)) {  // rare: every last hop again
          const uint32_t cx = C.cix[vj], q0 = (cx >> 5) & 0x3FFFFFFu, nq = cx & 31u;
          const uint32_t outj = (uint32_t)__builtin_amdgcn_readlane((int)out, (int)j);
          bool hit_r = false;
          auto orm = [&](uint32_t e) {
            const uint32_t ci = e & 0xFFFFu;
            if (!usable(ci) || s_D[ci] == kInf || s_D[ci] + (e >> 16) != outj) return;
            if (ci == r) hit_r = true;
            else if (wl) acc |= cm[(size_t)ci * NW + lane];
          };
          for (uint32_t qq = 0; qq < nq; ++qq) {
            const uint4 e4 = la4[q0 + qq];
            orm(e4.x); orm(e4.y); orm(e4.z); orm(e4.w);
          }
          if (hit_r) {
            const uint32_t bit = rootbit(vj);
            if ((bit >> 5) == lane) acc |= 1u << (bit & 31u);
          }
        }
        if (wl) __builtin_nontemporal_store(acc, nhrow + (size_t)vj * NW + lane);
        if (acc && wl) h += g.dkey[2ull * vj + 1] * digest_word_key(lane, acc);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    h += shfl_xor64(h, o);
    sum += shfl_xor64(sum, o);
    reach += (uint32_t)__shfl_xor((int)reach, o, kWave);
  }
  if (lane == 0) {
    atomicAdd(&s_acc[0], (unsigned long long)reach);
    atomicAdd(&s_acc[1], (unsigned long long)sum);
    atomicAdd(&s_acc[2], (unsigned long long)h);
  }
  __syncthreads();
  if (wave == 0 && lane == 0 && dg) {
    atomicAdd((unsigned long long*)&dg->reached, s_acc[0]);
    atomicAdd((unsigned long long*)&dg->sum_dist, s_acc[1]);
    atomicAdd((unsigned long long*)&dg->hash, s_acc[2]);
  }
}

// Expansion of queued nodes each from its own current distance, for the
// delta-stepping variant: a relaxation that lowers a distance (LDS atomicMin)
// sets the node's dirty bit and the round's flag.
__device__ __forceinline__ void expand_bf(const CoverGraph& C, uint32_t* s_D, uint32_t* nxt,
                                          const uint32_t* q, uint32_t cnt, uint32_t* s_pre,
                                          uint32_t* s_any, uint32_t lane) {
  for (uint32_t b0 = 0; b0 < cnt; b0 += kWave) {
    const uint32_t j = b0 + lane;
    uint32_t beg = 0, deg = 0, du = kInf;
    if (j < cnt) {
      const uint32_t u = q[j];
      beg = C.crow[u];
      deg = C.crow[u + 1] - beg;
      du = s_D[u];
    }
    uint32_t inc = deg;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, o, kWave);
      if (lane >= (uint32_t)o) inc += y;
    }
    s_pre[lane] = inc;
    s_pre[kWave + lane] = beg;
    s_pre[2 * kWave + lane] = du;
    __builtin_amdgcn_wave_barrier();
    const uint32_t total = (uint32_t)__shfl((int)inc, kWave - 1, kWave);
    constexpr uint32_t kU = 16;
    bool any = false;
    for (uint32_t f0 = 0; f0 < total; f0 += kWave * kU) {
      uint2 ed[kU];
      uint32_t base[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t f = f0 + u * kWave + lane;
        ed[u] = make_uint2(0u, kInf);
        base[u] = kInf;
        if (f < total) {
          uint32_t lo = 0, hi = kWave - 1;  // first k with pre[k] > f
#pragma unroll
          for (int it = 0; it < 6; ++it) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_pre[mid] > f) hi = mid;
            else lo = mid + 1;
          }
          const uint32_t before = lo ? s_pre[lo - 1] : 0u;
          ed[u] = C.cedge[s_pre[kWave + lo] + (f - before)];
          base[u] = s_pre[2 * kWave + lo];
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        if (ed[u].y == kInf || base[u] == kInf) continue;
        const uint32_t nd = base[u] + ed[u].y;
        const uint32_t v = ed[u].x;
        if (nd < atomicMin(&s_D[v], nd)) {
          atomicOr(&nxt[v >> 5], 1u << (v & 31u));
          any = true;
        }
      }
    }
    if (__ballot(any) && lane == 0) *s_any = 1u;
    __builtin_amdgcn_wave_barrier();  // s_pre is rewritten by the next pass
  }
}

// Delta-stepping over the contracted graph (OSPF_COVER_DELTA=d; not the
// default): the distance axis in buckets of width d; a bucket's round
// expands the "dirty" transit cover nodes (distance lowered since their last
// expansion) whose distance lies below the bucket's end, and repeats until
// none is left there; the next bucket starts at the smallest dirty distance.
// Exact at the fixed point (metrics >= 1), and a round scans the dirty bitmap
// (nS / 32 words) instead of the distances. Measured on F100k-w: 162 / 257 /
// 318 ms at d = 8 / 32 / 64 against 82 ms for the Dial rounds (and 341 ms for
// plain frontier Bellman-Ford): every re-expansion of a spine relaxes all its
// 1,781 edges again; a light / heavy edge split would be the next step.
__global__ void __launch_bounds__(512) cover_delta_kernel(DevGraph g, CoverGraph C, CoverArgs a,
                                                          uint32_t delta) {
  extern __shared__ uint32_t s_D[];  // [nS] distances, [nw] transit bits, [nw] dirty bits
  __shared__ uint32_t s_q[kWaves][kQ];
  __shared__ uint32_t s_pre[kWaves][3 * kWave];
  __shared__ uint32_t s_any[2], s_min;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t nS = C.nS, V = g.V, nw = (nS + 31u) / 32u;
  uint32_t* s_tr = s_D + nS;
  uint32_t* s_dirty = s_tr + nw;
  for (uint32_t x = tid; x < nw; x += kBlock) s_tr[x] = C.ctr[x];
  for (uint32_t i = blockIdx.x; i < a.n; i += gridDim.x) {
    const uint32_t rn = a.roots[i];
    const uint32_t r = rn < V ? C.cix[rn] : kInf;
    if (r >= nS) {  // not a cover node (or a bad id): its row is left alone
      if (tid == 0) atomicOr(a.err, 64u);
      continue;
    }
    for (uint32_t x = tid; x < nS; x += kBlock) s_D[x] = x == r ? 0u : kInf;
    for (uint32_t x = tid; x < nw; x += kBlock) s_dirty[x] = x == (r >> 5) ? 1u << (r & 31u) : 0u;
    if (tid == 0) {
      s_any[0] = s_any[1] = 0u;
      s_min = kInf;
    }
    __syncthreads();
    uint32_t hi = delta, par = 0;
    while (true) {
      uint32_t* q = s_q[wave];
      uint32_t cnt = 0, m2 = kInf;
      bool popped = false;
      for (uint32_t w0 = wave * kWave; w0 < nw; w0 += kBlock) {
        const uint32_t w = w0 + lane;
        uint32_t bits = w < nw ? s_dirty[w] : 0u, take = 0u;
        for (uint32_t b = bits; b; b &= b - 1u) {
          const uint32_t u = 32u * w + (uint32_t)__builtin_ctz(b);
          const uint32_t d = s_D[u];
          if (d < hi) take |= b & (0u - b);
          else m2 = min(m2, d);
        }
        if (take) {
          atomicAnd(&s_dirty[w], ~take);  // a later improvement sets the bit again
          popped = true;
          take &= s_tr[w] | (w == (r >> 5) ? 1u << (r & 31u) : 0u);  // transit or the root
        }
        while (__ballot(take != 0u)) {
          const bool has = take != 0u;
          const uint32_t u = has ? 32u * w + (uint32_t)__builtin_ctz(take) : 0u;
          if (has) take &= take - 1u;
          const uint64_t bal = __ballot(has);
          if (has) q[cnt + __popcll(bal & ((1ull << lane) - 1ull))] = u;
          cnt += (uint32_t)__popcll(bal);
          if (cnt > kQ - kWave) {
            __builtin_amdgcn_wave_barrier();
            expand_bf(C, s_D, s_dirty, q, cnt, s_pre[wave], &s_any[par], lane);
            cnt = 0;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (cnt) expand_bf(C, s_D, s_dirty, q, cnt, s_pre[wave], &s_any[par], lane);
      if (__ballot(popped) && lane == 0) s_any[par] = 1u;
      m2 = wave_min32(m2);
      if (lane == 0 && m2 != kInf) atomicMin(&s_min, m2);
      __syncthreads();
      const bool again = s_any[par] != 0u;
      const uint32_t nxt = s_min;
      __syncthreads();  // every thread has read the flags
      if (tid == 0) {
        s_any[par] = 0u;
        s_min = kInf;
      }
      par ^= 1u;
      if (!again) {  // the bucket below hi is settled: on to the next dirty distance
        if (nxt == kInf) break;
        hi = nxt + delta;
      }
      __syncthreads();  // the flag resets are visible before their use
    }
    write_row(g, C, a.dist + (size_t)i * V, s_D, s_tr, r, tid, kBlock);
    __syncthreads();  // s_D is reused by the next root
  }
}

// Closure rows by node tiles: block = (chunk of kLtTiles node tiles, chunk of
// kLtRoots roots). A tile is <= 256 consecutive nodes whose own cover indices
// (cover nodes) and in-links' cover indices (leaves) form a union U of <= 256
// slots; thread = node, its entries (slot | 0x100 for its own cover column,
// else slot | metric << 16) in registers for every root of the chunk. Per
// root the values and masks of U are staged in LDS (loaded one root ahead),
// the node's dist and next-hop words computed (a leaf: LinkState.cpp:885-901
// over its tight last hops; the root as a last hop gives the leaf's own bit)
// and both rows stored as contiguous runs; per-root digests summed in LDS over
// the block's tiles, one global add each at the end.
template <int NW>
__global__ void __launch_bounds__(256) closure_tile_rows_kernel(DevGraph g, CoverGraph C,
                                                                ClosureRowsPlan p) {
  __shared__ uint32_t s_val[kLtRoots][kLtU], s_u[kLtU], s_tr[kLtU];
  __shared__ uint32_t s_m[kLtRoots][kLtU * NW];
  __shared__ uint32_t s_st[2][kLtNodes * NW];
  __shared__ unsigned long long s_acc[kLtRoots][3];
  const uint32_t tid = threadIdx.x, V = g.V, lane = tid & 63u;
  const uint32_t nch = (p.ntiles + kLtTiles - 1) / kLtTiles;
  const uint32_t tch = blockIdx.x % nch, rch = blockIdx.x / nch;
  const uint32_t i0 = rch * kLtRoots, i1 = min(p.nroots, i0 + kLtRoots), nr = i1 > i0 ? i1 - i0 : 0u;
  for (uint32_t x = tid; x < kLtRoots * 3u; x += 256u) (&s_acc[0][0])[x] = 0ull;
  const uint32_t ta = tch * kLtTiles, tb = min(p.ntiles, ta + kLtTiles);
  uint32_t buf = 0;
  for (uint32_t t = ta; t < tb; ++t) {
    const uint4 tl = p.tile[t];  // {first node, nodes, first U entry, U size}
    const bool ok = tid < tl.y;
    const uint32_t v = tl.x + (ok ? tid : 0u);
    uint32_t e[kLtE];
    {
      const uint4* src = reinterpret_cast<const uint4*>(p.tle + (size_t)v * kLtE);
#pragma unroll
      for (int q = 0; q < (int)kLtE / 4; ++q) {
        const uint4 x = src[q];
        e[4 * q] = ok ? x.x : kInf;
        e[4 * q + 1] = ok ? x.y : kInf;
        e[4 * q + 2] = ok ? x.z : kInf;
        e[4 * q + 3] = ok ? x.w : kInf;
      }
    }
    // every root's slot values and masks of the tile, all loads in flight
    // (<= kLtRoots x kLtU / 256 per thread)
    constexpr uint32_t kPer = kLtRoots * kLtU / 256u;
    uint32_t lv[kPer], lm[kPer][NW];
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
      const uint32_t x = tid + q * 256u, j = x / kLtU, k = x % kLtU;
      lv[q] = kInf;
#pragma unroll
      for (int w = 0; w < NW; ++w) lm[q][w] = 0u;
      if (k < tl.w && i0 + j < i1) {
        const size_t b = (size_t)(i0 + j) * p.nS + p.tu[tl.z + k];
        lv[q] = p.dc[b];
#pragma unroll
        for (int w = 0; w < NW; ++w) lm[q][w] = p.dcm[b * NW + w];
      }
    }
    __syncthreads();  // the previous tile's slots are consumed
    if (tid < tl.w) {
      const uint32_t ci = p.tu[tl.z + tid];
      s_u[tid] = ci;
      s_tr[tid] = (C.ctr[ci >> 5] >> (ci & 31u)) & 1u;
    }
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
      const uint32_t x = tid + q * 256u, j = x / kLtU, k = x % kLtU;
      s_val[j][k] = lv[q];
#pragma unroll
      for (int w = 0; w < NW; ++w) s_m[j][k * NW + w] = lm[q][w];
    }
    __syncthreads();
    for (uint32_t i = i0; i < i1; ++i, buf ^= 1u) {
      const uint32_t r = p.rcov[i], rn = p.roots[i];
      const uint32_t* sv = s_val[i - i0];
      const uint32_t* sm = s_m[i - i0];
      uint32_t out = kInf, m[NW];
#pragma unroll
      for (int w = 0; w < NW; ++w) m[w] = 0u;
      if ((e[0] & 0x100u) && e[0] != kInf) {  // a cover node: its own column
        const uint32_t sl = e[0] & 0xFFu;
        out = sv[sl];
        if (v != rn && out != kInf) {
#pragma unroll
          for (int w = 0; w < NW; ++w) m[w] = sm[sl * NW + w];
        }
      } else {
        auto usable = [&](uint32_t sl) { return s_tr[sl] != 0u || s_u[sl] == r; };
#pragma unroll
        for (int q = 0; q < (int)kLtE; ++q) {
          if (e[q] == kInf) continue;
          const uint32_t sl = e[q] & 0xFFu, x = sv[sl];
          if (x != kInf && usable(sl)) out = min(out, x + (e[q] >> 16));
        }
        if (out != kInf) {
#pragma unroll
          for (int q = 0; q < (int)kLtE; ++q) {
            if (e[q] == kInf) continue;
            const uint32_t sl = e[q] & 0xFFu, x = sv[sl];
            if (x == kInf || !usable(sl) || x + (e[q] >> 16) != out) continue;
            if (s_u[sl] == r) {  // a neighbour of the root: its own bit
              const uint32_t* dn = g.dn + g.dn_off[rn];
              uint32_t lo = 0, hi = g.dn_off[rn + 1] - g.dn_off[rn];
              while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (dn[mid] < v) lo = mid + 1;
                else hi = mid;
              }
              if (lo < 32u * NW) m[lo >> 5] |= 1u << (lo & 31u);
            } else {
#pragma unroll
              for (int w = 0; w < NW; ++w) m[w] |= sm[sl * NW + w];
            }
          }
        }
      }
      uint64_t h = 0, sum = 0;
      uint32_t reach = 0;
      if (ok) {
        __builtin_nontemporal_store(out, p.dist + (size_t)p.rowpos[i] * V + v);
        if (out != kInf) {
          reach = 1u;
          sum = out;
          h = g.dkey[2ull * v] * ((uint64_t)out + 1ull);
          uint64_t ws = 0;
#pragma unroll
          for (int w = 0; w < NW; ++w)
            if (m[w]) ws += digest_word_key((uint32_t)w, m[w]);
          if (ws) h += g.dkey[2ull * v + 1] * ws;
        }
      }
#pragma unroll
      for (int w = 0; w < NW; ++w) s_st[buf][tid * NW + w] = m[w];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        h += shfl_xor64(h, o);
        sum += shfl_xor64(sum, o);
        reach += (uint32_t)__shfl_xor((int)reach, o, kWave);
      }
      if (lane == 0 && reach) {
        atomicAdd(&s_acc[i - i0][0], (unsigned long long)reach);
        atomicAdd(&s_acc[i - i0][1], (unsigned long long)sum);
        atomicAdd(&s_acc[i - i0][2], (unsigned long long)h);
      }
      __syncthreads();
      uint32_t* nrow = p.nh + ((size_t)i * V + tl.x) * NW;
      for (uint32_t x = tid; x < tl.y * NW; x += 256u) __builtin_nontemporal_store(s_st[buf][x], nrow + x);
    }
  }
  __syncthreads();
  if (p.digest)
    for (uint32_t j = tid; j < nr; j += 256u)
      if (s_acc[j][0]) {
        atomicAdd((unsigned long long*)&p.digest[i0 + j].reached, s_acc[j][0]);
        atomicAdd((unsigned long long*)&p.digest[i0 + j].sum_dist, s_acc[j][1]);
        atomicAdd((unsigned long long*)&p.digest[i0 + j].hash, s_acc[j][2]);
      }
}

// Rows of the seeds whose next-hop masks the Dial kept: their full cover
// columns back into LDS, then write_row_nhw (dist + next-hop rows, digest).
__global__ void __launch_bounds__(512) seed_rows_kernel(DevGraph g, CoverGraph C,
                                                        const uint32_t* roots, uint32_t n,
                                                        const uint32_t* dfull, const uint32_t* nhm,
                                                        uint32_t NW, uint32_t* dist,
                                                        const uint32_t* rowpos, uint32_t* nh,
                                                        ospf_digest* digest, uint32_t* err,
                                                        uint32_t nch) {
  extern __shared__ uint32_t s_D[];  // [nS] columns, then [ctr words] transit bits
  __shared__ unsigned long long s_acc[3];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t nS = C.nS, V = g.V;
  uint32_t* s_tr = s_D + nS;
  for (uint32_t x = tid; x < (nS + 31u) / 32u; x += kBlock) s_tr[x] = C.ctr[x];
  // items = (root, node range): a root's row in nch ranges, so a few hundred
  // seeds still fill the chip (each item reloads the root's columns)
  const uint32_t span = ((V + nch - 1) / nch + kWave - 1) / kWave * kWave;
  for (uint32_t it = blockIdx.x; it < n * nch; it += gridDim.x) {
    const uint32_t k = it % n, c = it / n;
    const uint32_t rn = roots[k];
    const uint32_t r = rn < V ? C.cix[rn] : kInf;
    if (r >= nS) {
      if (tid == 0 && c == 0) atomicOr(err, 64u);
      continue;
    }
    const uint32_t vb = c * span, ve = min(V, vb + span);
    if (vb >= ve) continue;  // block-uniform
    const uint32_t* src = dfull + (size_t)k * nS;
    for (uint32_t x = tid; x < nS; x += kBlock) s_D[x] = src[x];
    if (tid < 3) s_acc[tid] = 0ull;
    __syncthreads();
    write_row_nhw(g, C, dist + (size_t)rowpos[k] * V, nh + (size_t)k * V * NW, s_D, s_tr, r, rn,
                  nhm + (size_t)k * nS * NW, NW, digest ? digest + k : nullptr, s_acc, wave, lane, vb,
                  ve);
    __syncthreads();
  }
}

// Closure rows with next hops (load mode + masks) in a kernel of their own:
// the Dial kernel's register budget (its widest path) capped it at two
// 512-thread roots per CU; here a root gets 1,024 threads at <= 64 VGPRs, two
// roots per CU (the cover columns' 58 KB of LDS each), twice the waves to
// hide the in-link and mask gathers.
constexpr uint32_t kRowsBlock = 1024;
template <int NW>
__global__ void __launch_bounds__(kRowsBlock, 8) cover_rows_kernel(DevGraph g, CoverGraph C,
                                                                   CoverArgs a) {
  extern __shared__ uint32_t s_D[];  // [nS + 1] tagged cover columns, then [ctr words] transit bits
  __shared__ uint32_t s_st[kRowsBlock * NW];
  __shared__ unsigned long long s_acc[3];
  const uint32_t tid = threadIdx.x, nS = C.nS, V = g.V;
  uint32_t* s_tr = s_D + nS + 1u;
  for (uint32_t x = tid; x < (nS + 31u) / 32u; x += kRowsBlock) s_tr[x] = C.ctr[x];
  if (tid == 0) s_D[nS] = kInf;
  for (uint32_t i = blockIdx.x; i < a.n; i += gridDim.x) {
    const uint32_t rn = a.roots[i];
    const uint32_t r = rn < V ? C.cix[rn] : kInf;
    if (r >= nS) {
      if (tid == 0) atomicOr(a.err, 64u);
      continue;
    }
    const uint32_t* src = a.dload + (size_t)i * nS;
    for (uint32_t x = tid; x < nS; x += kRowsBlock) {
      const uint32_t d = src[x];  // < 2^31 when reached (the Dial's bound)
      const bool relay = x == r || ((s_tr[x >> 5] >> (x & 31u)) & 1u);
      s_D[x] = (d == kInf || relay) ? d : (d | 0x80000000u);
    }
    if (tid < 3) s_acc[tid] = 0ull;
    __syncthreads();
    write_row_nh_tag<NW>(g, C, a.dist + (size_t)a.rowpos[i] * V, a.nh + (size_t)i * V * NW, s_D, s_tr,
                     r, rn, a.nhload + (size_t)i * nS * NW, a.digest ? a.digest + i : nullptr, s_acc,
                     s_st, tid, kRowsBlock);
    __syncthreads();
  }
}

__global__ void __launch_bounds__(512) cover_spf_kernel(DevGraph g, CoverGraph C, CoverArgs a) {
  extern __shared__ uint32_t s_D[];  // [nS] distances, then [ctr words] transit bits
  __shared__ uint32_t s_q[kWaves][kQ];
  __shared__ uint32_t s_pre[kWaves][2 * kWave];
  __shared__ uint32_t s_next[2];
  __shared__ unsigned long long s_acc[3];  // rows with next hops: digest sums
  __shared__ uint32_t s_mw[kWaves][kWave];   // seed masks: the root's first-hop bits
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t nS = C.nS, V = g.V;
  uint32_t* s_tr = s_D + nS;
  for (uint32_t x = tid; x < (nS + 31u) / 32u; x += kBlock) s_tr[x] = C.ctr[x];
  s_mw[wave][lane] = 0u;
  for (uint32_t i = blockIdx.x; i < a.n; i += gridDim.x) {
    const uint32_t rn = a.roots[i];
    const uint32_t r = rn < V ? C.cix[rn] : kInf;
    if (r >= nS) {  // not a cover node (or a bad id): its row is left alone
      if (tid == 0) atomicOr(a.err, 64u);
      continue;
    }
    if (a.dload) {  // cover columns given (closure rows): the full row only
      const uint32_t* src = a.dload + (size_t)i * nS;
      for (uint32_t x = tid; x < nS; x += kBlock) s_D[x] = src[x];
      if (tid < 3) s_acc[tid] = 0ull;
      __syncthreads();
      uint32_t* drow = a.dist + (size_t)a.rowpos[i] * V;
      if (a.nhload) {  // and the next-hop row + digest from the masks
        const uint32_t* cm = a.nhload + (size_t)i * nS * a.NW;
        uint32_t* nrow = a.nh + (size_t)i * V * a.NW;
        ospf_digest* dg = a.digest ? a.digest + i : nullptr;
        uint32_t* s_st = &s_q[0][0];  // kWaves * kQ = 2048 words >= kBlock * NW (NW <= 4)
        switch (a.NW) {
          case 1: write_row_nh<1>(g, C, drow, nrow, s_D, s_tr, r, rn, cm, dg, s_acc, s_st, tid, kBlock); break;
          case 2: write_row_nh<2>(g, C, drow, nrow, s_D, s_tr, r, rn, cm, dg, s_acc, s_st, tid, kBlock); break;
          case 3: write_row_nh<3>(g, C, drow, nrow, s_D, s_tr, r, rn, cm, dg, s_acc, s_st, tid, kBlock); break;
          default: write_row_nh<4>(g, C, drow, nrow, s_D, s_tr, r, rn, cm, dg, s_acc, s_st, tid, kBlock); break;
        }
      } else {
        write_row(g, C, drow, s_D, s_tr, r, tid, kBlock);
      }
      __syncthreads();
      continue;
    }
    const uint32_t np = a.nhpos ? a.nhpos[i] : kInf;
    uint32_t* cmk = np != kInf ? a.nhm + (size_t)np * nS * a.NW : nullptr;
    for (uint32_t x = tid; x < nS; x += kBlock) s_D[x] = x == r ? 0u : kInf;
    if (tid == 0) s_next[0] = s_next[1] = kInf;
    if (tid < 3) s_acc[tid] = 0ull;
    __syncthreads();
    uint32_t t = 0, par = 0;
    while (true) {
      uint32_t* q = s_q[wave];
      uint32_t cnt = 0, m2 = kInf;
      for (uint32_t x0 = wave * kWave; x0 < nS; x0 += kBlock) {
        const uint32_t x = x0 + lane;
        const uint32_t d = x < nS ? s_D[x] : kInf;
        if (d > t && d != kInf) m2 = min(m2, d);
        const bool tr = x < nS && ((s_tr[x >> 5] >> (x & 31u)) & 1u);
        const bool fr = d == t && (tr || x == r);
        const uint64_t bal = __ballot(fr);
        if (fr) q[cnt + __popcll(bal & ((1ull << lane) - 1ull))] = x;
        cnt += (uint32_t)__popcll(bal);
        if (cnt > kQ - kWave) {
          __builtin_amdgcn_wave_barrier();
          expand(C, s_D, &s_next[par], q, cnt, s_pre[wave], t, lane);
          cnt = 0;
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (cnt) expand(C, s_D, &s_next[par], q, cnt, s_pre[wave], t, lane);
      if (cmk) seed_masks(C, s_D, s_tr, r, t, cmk, a.NW, s_mw[wave], wave, lane);
      m2 = wave_min32(m2);
      if (lane == 0 && m2 != kInf) atomicMin(&s_next[par], m2);
      __syncthreads();
      t = s_next[par];
      if (tid == 0) s_next[par ^ 1u] = kInf;  // the next round's slot
      par ^= 1u;
      if (t == kInf) break;  // every reachable cover node settled
      __syncthreads();       // the slot reset is visible before its use
    }
    if (a.dcomp) {  // the cover columns as a seed of the closure
      const bool tr = (s_tr[r >> 5] >> (r & 31u)) & 1u;
      uint32_t* dst = a.dcomp + (size_t)i * nS;
      for (uint32_t x = tid; x < nS; x += kBlock) {
        const uint32_t d = tr ? s_D[x] : (x == r ? 0u : kInf);
        dst[x] = d == kInf ? kClInf : d;
      }
    }
    const uint32_t rp = a.rowpos ? a.rowpos[i] : i;
    if (cmk && a.dfull) {  // the rows follow on another stream (launch_seed_rows)
      uint32_t* dst = a.dfull + (size_t)np * nS;
      for (uint32_t x = tid; x < nS; x += kBlock) dst[x] = s_D[x];
    } else if (cmk && rp != kInf)
      write_row_nhw(g, C, a.dist + (size_t)rp * V, a.nh + (size_t)np * V * a.NW, s_D, s_tr, r, rn,
                    cmk, a.NW, a.digest ? a.digest + np : nullptr, s_acc, wave, lane, 0u, V);
    else if (rp != kInf)
      write_row(g, C, a.dist + (size_t)rp * V, s_D, s_tr, r, tid, kBlock);
    __syncthreads();  // s_D is reused by the next root
  }
}

// Cover closure: block = (component, 256 cover columns), lane = column; the
// component's members' accumulators stay in registers while the seeds'
// columns stream past (8 loads in flight), the per-member constants are
// block-uniform (scalar loads). Blocks are ordered column-chunk-major and
// spread so that one XCD's resident blocks share a chunk of the seed rows in
// its L2.
// With next-hop masks (NW words, KW = 8): per member the mask of its best
// terms (a strictly better term replaces it, an equal one is ORed in) -- the
// next hops of f towards v are the first hops of f's shortest paths to the
// first seed s on a shortest f -> v path (LinkState.cpp:885-901: a path's
// next hop is its first hop; the tail from s is s's own shortest path).
template <int NW>
__global__ void __launch_bounds__(256) closure_nh_kernel(ClosurePlan p) {
  constexpr int KW = 8;
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  const uint32_t full = nb / 8u * 8u;
  const uint32_t item = b < full ? (b % 8u) * (full / 8u) + b / 8u : b;
  const uint32_t chunk = item / p.ncomp, ci = item % p.ncomp;
  const uint32_t v = chunk * 256u + threadIdx.x;
  const bool ok = v < p.nS;
  const uint2 cm = p.comp[ci];
  uint32_t acc[KW], mk[KW][NW];
#pragma unroll
  for (int f = 0; f < KW; ++f) {
    acc[f] = kClInf;
#pragma unroll
    for (int w = 0; w < NW; ++w) mk[f][w] = 0u;
  }
  auto take = [&](int f, uint32_t c, const uint32_t* m) {
    const bool lt = c < acc[f], le = c <= acc[f];
    if (__ballot(le)) {  // wave-uniform: most terms improve no lane (terms sorted by constant)
#pragma unroll
      for (int w = 0; w < NW; ++w) mk[f][w] = (lt ? 0u : mk[f][w]) | (le ? m[w] : 0u);
    }
    acc[f] = min(acc[f], c);
  };
  const uint32_t* cst = p.cst + (size_t)cm.x * KW;
  const uint32_t* fh = p.fh + (size_t)cm.x * KW * NW;
  const uint32_t* jl = p.jl + cm.x;
  uint32_t used = 0;  // members with an output row
#pragma unroll
  for (int f = 0; f < KW; ++f) used |= (p.out[(size_t)ci * KW + f] != kInf ? 1u : 0u) << f;
  for (uint32_t j0 = 0; j0 < cm.y; j0 += 8u) {
    if (j0 && closure_done<KW>(acc, cst + (size_t)j0 * KW, used, ok)) break;
    uint32_t x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t j = j0 + (uint32_t)u;
      x[u] = (ok && j < cm.y) ? p.seedC[(size_t)jl[j] * p.nS + v] : kClInf;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t j = j0 + (uint32_t)u;
      if (j >= cm.y) break;  // uniform
#pragma unroll
      for (int f = 0; f < KW; ++f) take(f, cst[j * KW + f] + x[u], fh + ((size_t)j * KW + f) * NW);
    }
  }
  const uint32_t* mem = p.mem + (size_t)ci * KW;
  const uint32_t* dl = p.dloc + (size_t)ci * KW * KW;
  const uint32_t* fl = p.fhloc + (size_t)ci * KW * KW * NW;
#pragma unroll
  for (int m = 0; m < KW; ++m)
    if (mem[m] == v)
#pragma unroll
      for (int f = 0; f < KW; ++f) take(f, dl[f * KW + m], fl + ((size_t)f * KW + m) * NW);
  const uint32_t* out = p.out + (size_t)ci * KW;
#pragma unroll
  for (int f = 0; f < KW; ++f) {
    if (!ok || out[f] == kInf) continue;
    const bool un = acc[f] >= kClInf;
    p.dc[(size_t)out[f] * p.nS + v] = un ? kInf : acc[f];
    uint32_t* dm = p.dcm + ((size_t)out[f] * p.nS + v) * NW;
#pragma unroll
    for (int w = 0; w < NW; ++w) dm[w] = un ? 0u : mk[f][w];
  }
}

template <int KW>
__global__ void __launch_bounds__(256) closure_kernel(ClosurePlan p) {
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  const uint32_t full = nb / 8u * 8u;
  const uint32_t item = b < full ? (b % 8u) * (full / 8u) + b / 8u : b;
  const uint32_t chunk = item / p.ncomp, ci = item % p.ncomp;
  const uint32_t v = chunk * 256u + threadIdx.x;
  const bool ok = v < p.nS;
  const uint2 cm = p.comp[ci];
  uint32_t acc[KW];
#pragma unroll
  for (int f = 0; f < KW; ++f) acc[f] = kClInf;
  const uint32_t* cst = p.cst + (size_t)cm.x * KW;
  const uint32_t* jl = p.jl + cm.x;
  uint32_t used = 0;  // members with an output row
#pragma unroll
  for (int f = 0; f < KW; ++f) used |= (p.out[(size_t)ci * KW + f] != kInf ? 1u : 0u) << f;
  for (uint32_t j0 = 0; j0 < cm.y; j0 += 8u) {
    if (j0 && closure_done<KW>(acc, cst + (size_t)j0 * KW, used, ok)) break;
    uint32_t x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t j = j0 + (uint32_t)u;
      x[u] = (ok && j < cm.y) ? p.seedC[(size_t)jl[j] * p.nS + v] : kClInf;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t j = j0 + (uint32_t)u;
      if (j >= cm.y) break;  // uniform
#pragma unroll
      for (int f = 0; f < KW; ++f) acc[f] = min(acc[f], cst[j * KW + f] + x[u]);  // < 2^31: no wrap
    }
  }
  const uint32_t* mem = p.mem + (size_t)ci * KW;
  const uint32_t* dl = p.dloc + (size_t)ci * KW * KW;
#pragma unroll
  for (int m = 0; m < KW; ++m)
    if (mem[m] == v)
#pragma unroll
      for (int f = 0; f < KW; ++f) acc[f] = min(acc[f], dl[f * KW + m]);
  const uint32_t* out = p.out + (size_t)ci * KW;
#pragma unroll
  for (int f = 0; f < KW; ++f)
    if (ok && out[f] != kInf) p.dc[(size_t)out[f] * p.nS + v] = acc[f] >= kClInf ? kInf : acc[f];
}
}  // namespace

hipError_t launch_closure_rows(const DevGraph& g, const CoverGraph& C, const ClosureRowsPlan& p,
                               hipStream_t s) {
  if (p.nroots == 0 || p.ntiles == 0) return hipSuccess;
  if (p.NW == 0 || p.NW > kClMaxNW || !p.dc || !p.dcm || !p.dist || !p.nh || !p.tile || !p.tle ||
      !p.tu)
    return hipErrorInvalidValue;
  const dim3 grid(((p.ntiles + kLtTiles - 1) / kLtTiles) * ((p.nroots + kLtRoots - 1) / kLtRoots));
  switch (p.NW) {
    case 1: hipLaunchKernelGGL(closure_tile_rows_kernel<1>, grid, dim3(256), 0, s, g, C, p); break;
    case 2: hipLaunchKernelGGL(closure_tile_rows_kernel<2>, grid, dim3(256), 0, s, g, C, p); break;
    case 3: hipLaunchKernelGGL(closure_tile_rows_kernel<3>, grid, dim3(256), 0, s, g, C, p); break;
    default: hipLaunchKernelGGL(closure_tile_rows_kernel<4>, grid, dim3(256), 0, s, g, C, p); break;
  }
  return hipGetLastError();
}

hipError_t launch_seed_rows(const DevGraph& g, const CoverGraph& C, const uint32_t* roots,
                            uint32_t n, const uint32_t* dfull, const uint32_t* nhm, uint32_t NW,
                            uint32_t* dist, const uint32_t* rowpos, uint32_t* nh,
                            ospf_digest* digest, uint32_t* err, uint32_t n_cu, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (!roots || !dfull || !nhm || !dist || !rowpos || !nh || NW == 0 || NW > kSeedMaxNW)
    return hipErrorInvalidValue;
  const size_t lds = ((size_t)C.nS + (C.nS + 31u) / 32u) * 4u;
  if (lds > 48 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)seed_rows_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  // >= ~8 items per CU: ranges of >= 4,096 nodes
  const uint32_t nch = std::max(1u, std::min((8u * n_cu + n - 1) / n, (g.V + 4095u) / 4096u));
  const uint32_t grid = std::min<uint32_t>(n * nch, 2u * n_cu);
  hipLaunchKernelGGL(seed_rows_kernel, dim3(grid), dim3(kBlock), lds, s, g, C, roots, n, dfull, nhm,
                     NW, dist, rowpos, nh, digest, err, nch);
  return hipGetLastError();
}

hipError_t launch_closure(const ClosurePlan& p, uint32_t KW, hipStream_t s) {
  if (p.ncomp == 0) return hipSuccess;
  const dim3 grid(p.ncomp * p.chunks);
  if (p.NW) {
    if (KW != 8 || !p.fh || !p.fhloc || !p.dcm) return hipErrorInvalidValue;
    switch (p.NW) {
      case 1: hipLaunchKernelGGL(closure_nh_kernel<1>, grid, dim3(256), 0, s, p); break;
      case 2: hipLaunchKernelGGL(closure_nh_kernel<2>, grid, dim3(256), 0, s, p); break;
      case 3: hipLaunchKernelGGL(closure_nh_kernel<3>, grid, dim3(256), 0, s, p); break;
      case 4: hipLaunchKernelGGL(closure_nh_kernel<4>, grid, dim3(256), 0, s, p); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (KW <= 8) hipLaunchKernelGGL(closure_kernel<8>, grid, dim3(256), 0, s, p);
  else if (KW <= 16) hipLaunchKernelGGL(closure_kernel<16>, grid, dim3(256), 0, s, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_cover_spf(const DevGraph& g, const CoverGraph& C, const CoverArgs& a,
                            uint32_t n_cu, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (a.dload && !a.rowpos) return hipErrorInvalidValue;  // load mode writes rows by position
  if (a.nhload && (!a.dload || !a.nh || a.NW == 0 || a.NW > kClMaxNW)) return hipErrorInvalidValue;
  if (a.nhpos && (a.dload || !a.nhm || !a.nh || a.NW == 0 || a.NW > kSeedMaxNW))
    return hipErrorInvalidValue;
  const char* e = getenv("OSPF_COVER_DELTA");
  if (e && !a.rowpos && !a.dcomp && !a.dload) {  // delta-stepping (experiment)
    const uint32_t delta = (uint32_t)std::max(1, atoi(e));
    const size_t lds = ((size_t)C.nS + 2u * ((C.nS + 31u) / 32u)) * 4u;
    const uint32_t per_cu = std::max<uint32_t>(1, (uint32_t)((150u * 1024u) / (lds + 12u * 1024u)));
    const uint32_t grid = std::min<uint32_t>(a.n, n_cu * std::min<uint32_t>(per_cu, 4u));
    if (lds > 48 * 1024) {
      hipError_t e = hipFuncSetAttribute((const void*)cover_delta_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(cover_delta_kernel, dim3(grid), dim3(kBlock), lds, s, g, C, a, delta);
    return hipGetLastError();
  }
  const size_t lds = ((size_t)C.nS + (C.nS + 31u) / 32u) * 4u;
  if (a.nhload && !getenv("OSPF_COVER_ROWS_IN_DIAL")) {  // closure rows with next hops
    const uint32_t grid = std::min<uint32_t>(a.n, n_cu * 2u);
    const size_t lds = ((size_t)C.nS + 1u + (C.nS + 31u) / 32u) * 4u;  // + the padding slot
    auto go = [&](const void* k) -> hipError_t {
      if (lds > 48 * 1024) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
      }
      return hipSuccess;
    };
    hipError_t e = hipSuccess;
    switch (a.NW) {
      case 1: if ((e = go((const void*)cover_rows_kernel<1>)) == hipSuccess) hipLaunchKernelGGL(cover_rows_kernel<1>, dim3(grid), dim3(kRowsBlock), lds, s, g, C, a); break;
      case 2: if ((e = go((const void*)cover_rows_kernel<2>)) == hipSuccess) hipLaunchKernelGGL(cover_rows_kernel<2>, dim3(grid), dim3(kRowsBlock), lds, s, g, C, a); break;
      case 3: if ((e = go((const void*)cover_rows_kernel<3>)) == hipSuccess) hipLaunchKernelGGL(cover_rows_kernel<3>, dim3(grid), dim3(kRowsBlock), lds, s, g, C, a); break;
      default: if ((e = go((const void*)cover_rows_kernel<4>)) == hipSuccess) hipLaunchKernelGGL(cover_rows_kernel<4>, dim3(grid), dim3(kRowsBlock), lds, s, g, C, a); break;
    }
    return e != hipSuccess ? e : hipGetLastError();
  }
  const uint32_t per_cu = std::max<uint32_t>(1, (uint32_t)((150u * 1024u) / (lds + 14u * 1024u)));
  const uint32_t grid = std::min<uint32_t>(a.n, n_cu * std::min<uint32_t>(per_cu, 4u));
  if (lds > 48 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)cover_spf_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(cover_spf_kernel, dim3(grid), dim3(kBlock), lds, s, g, C, a);
  return hipGetLastError();
}

}  // namespace ospf
