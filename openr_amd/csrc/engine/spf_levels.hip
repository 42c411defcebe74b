// spf_levels.hip — derive phase 1 (ospf_levels_dev) on 128-root traversals
// (gfx950): distance-only multi-source BFS, unit metric / hop count.
//
// Same levels as msbfs_level_kernel<-1> (spf_msbfs.hip) and so as
// LinkState::runSpf (openr/decision/LinkState.cpp:836-911) with unit weights:
// a node at BFS level d + 1 of root r has a usable in-edge from a transit node
// at level d of r (overloaded nodes never relay, LinkState.cpp:859-866).
//
// Why 128 roots. At F100k the traversal is bound by its gathers: a pull
// level reads the frontier record of every in-neighbour of every node with
// unseen roots, one random L2 access per CSR entry whatever the record's
// width. A 16-B record {roots 0-63, roots 64-127} serves twice the roots per
// access and per CSR scan, so a whole all-sources sweep makes half the
// gathers and half the row scans of the 64-root form.
//
// State per 128-root batch ("wide batch"): frontier records of levels d and
// d + 1 (16 B per node, slot d & 1), seen (16 B), the push accumulator (16 B),
// and the level record lev[node][128] (dist + 1 per root, set once per (node,
// root) pair; bytes of roots not in seen are stale). A round runs nb wide
// batches side by side; the last kernel transposes each batch's records into
// level rows (u8) and dist rows (u32) plus the distance part of each digest.
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
constexpr uint32_t kRoots = 128;

struct R2 {  // a set of the batch's roots: bit r of lo (r < 64) / hi (r >= 64)
  uint64_t lo, hi;
  __device__ bool any() const { return (lo | hi) != 0ull; }
};
__device__ __forceinline__ R2 ld2(const uint4* p) {
  const uint4 x = *p;
  return {((uint64_t)x.y << 32) | x.x, ((uint64_t)x.w << 32) | x.z};
}
__device__ __forceinline__ void st2(uint4* p, R2 v) {
  *p = make_uint4((uint32_t)v.lo, (uint32_t)(v.lo >> 32), (uint32_t)v.hi, (uint32_t)(v.hi >> 32));
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int o) {
  const uint32_t lo = __shfl_xor((uint32_t)x, o, kWave);
  const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), o, kWave);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t wave_add32(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
  return x;
}
__device__ __forceinline__ bool transit(const DevGraph& g, uint32_t v) {
  return !((g.nt_bits[v >> 5] >> (v & 31)) & 1u);
}

struct WB {  // wide batch vbl of the round
  uint32_t vbl, rix0, V;
  R2 valid;
  uint4* seen;
  uint4* accb;
  __device__ WB(const LvArgs& a, uint32_t vbl_, uint32_t V_) : vbl(vbl_), V(V_) {
    rix0 = (a.vb0 + vbl) * kRoots;
    const uint32_t nv = min(kRoots, a.n - rix0);
    valid.lo = nv >= 64u ? ~0ull : ((1ull << nv) - 1ull);
    valid.hi = nv >= 128u ? ~0ull : nv > 64u ? ((1ull << (nv - 64u)) - 1ull) : 0ull;
    seen = a.seen + (size_t)vbl * V;
    accb = a.accb + (size_t)vbl * V;
  }
  __device__ uint4* front(const LvArgs& a, uint32_t d) const {
    return a.front + ((size_t)(d & 1u) * a.nb + vbl) * V;
  }
  __device__ uint8_t* rec(const LvArgs& a, uint32_t v) const {
    return a.lev + ((size_t)vbl * V + v) * kRoots;
  }
};

// level bytes of node v for the roots in acc := val; the owner thread of v is
// the only writer within a level (pull lane / settle thread)
__device__ __forceinline__ void set_lev(const LvArgs& a, const WB& b, uint32_t v, R2 acc,
                                        uint32_t val) {
  uint4* rec = reinterpret_cast<uint4*>(b.rec(a, v));
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint64_t word = c < 4 ? acc.lo : acc.hi;
    const uint32_t bits = (uint32_t)(word >> (16 * (c & 3))) & 0xFFFFu;
    if (!bits) continue;
    auto put = [&](uint32_t w, uint32_t nib) {  // bit i of the nibble -> byte i := val
      const uint32_t ones = (nib * 0x00204081u) & 0x01010101u;
      return (w & ~(ones * 0xFFu)) | ones * val;
    };
    uint4 w = rec[c];
    w.x = put(w.x, bits & 0xFu);
    w.y = put(w.y, (bits >> 4) & 0xFu);
    w.z = put(w.z, (bits >> 8) & 0xFu);
    w.w = put(w.w, (bits >> 12) & 0xFu);
    rec[c] = w;
  }
}

// ---------------------------------------------------------------- init
// One block per root: level 0 (the root) and level 1 (its usable
// neighbours), the row strided over the block (a spine's 1,781 entries in 7
// steps of returning atomics instead of a wave's 28: 0.12 ms at F100k for the
// launch, bound by its spine roots). Roots of a batch may share nodes: atomics.
__global__ void __launch_bounds__(256) lv_init_kernel(DevGraph g, LvArgs a) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t slot = blockIdx.x;
  const uint32_t vbl = slot / kRoots, bit = slot % kRoots;
  if (vbl >= a.nb) return;
  const WB b(a, vbl, g.V);
  const uint32_t rix = b.rix0 + bit;
  if (rix >= a.n) return;
  const uint32_t V = g.V, s = a.roots[rix];
  if (s >= V) {
    if (tid == 0) atomicOr(a.err, 64u);
    return;
  }
  const uint32_t wi = bit >> 6;
  const unsigned long long bm = 1ull << (bit & 63u);
  uint32_t* lev32 = reinterpret_cast<uint32_t*>(a.lev);
  auto lev_put = [&](uint32_t v, uint32_t val) {  // byte `bit` of v's record := val
    uint32_t* w = &lev32[(((size_t)vbl * V + v) * kRoots + bit) / 4u];
    atomicAnd(w, ~(0xFFu << (8u * (bit & 3u))));  // stale bytes: records are not cleared
    atomicOr(w, val << (8u * (bit & 3u)));
  };
  auto or_word = [&](uint4* p, uint32_t v) {
    return atomicOr(reinterpret_cast<unsigned long long*>(p + v) + wi, bm);
  };
  if (tid == 0) {
    or_word(b.seen, s);
    lev_put(s, 1u);
  }
  uint4* f1 = b.front(a, 1);
  bool any = false;
  uint32_t mass = 0;
  for (uint32_t e = g.row_ptr[s] + tid; e < g.row_ptr[s + 1]; e += kBlock) {
    const uint32_t cx = g.colx[e];
    if ((cx & kDown) || cx == s) continue;
    or_word(b.seen, cx);
    if (transit(g, cx) && !or_word(f1, cx)) mass += g.row_ptr[cx + 1] - g.row_ptr[cx];
    lev_put(cx, 2u);  // parallel links: the same byte again
    any = true;
  }
  mass = wave_add32(mass);
  if (lane == 0 && mass) atomicAdd(&a.mass[vbl * a.lmax + 1], mass);
  if (__ballot(any) && lane == 0) a.found[vbl * a.lmax + 1] = 1u;
}

// ---------------------------------------------------------------- pull / push
// in-edges [beg, end) of a node with unseen roots m (STEP 4: one lane; STEP
// 256: a wave, lane offset folded into beg); four row quads per step with
// every load in flight; stops once every unseen root is found
template <uint32_t STEP>
__device__ __forceinline__ R2 pull_scan(const DevGraph& g, const uint4* fcur, uint32_t beg,
                                        uint32_t end, R2 m, bool masked) {
  const uint4* q = reinterpret_cast<const uint4*>(g.colx);
  R2 acc{0ull, 0ull};
  if (!masked) {  // whole four-quad steps, then quad by quad
    for (; beg + 3u * STEP < end; beg += 4u * STEP) {
      uint4 c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = q[(beg + j * STEP) >> 2];
      uint4 f[16];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t cs[4] = {c[j].x, c[j].y, c[j].z, c[j].w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          f[4 * j + i] = (cs[i] & kDown) ? make_uint4(0u, 0u, 0u, 0u) : fcur[cs[i]];
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        acc.lo |= (((uint64_t)f[k].y << 32) | f[k].x);
        acc.hi |= (((uint64_t)f[k].w << 32) | f[k].z);
      }
      acc.lo &= m.lo;
      acc.hi &= m.hi;
      if (acc.lo == m.lo && acc.hi == m.hi) return acc;
    }
    for (; beg < end; beg += STEP) {
      const uint4 c = q[beg >> 2];
      const uint32_t cs[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (cs[i] & kDown) continue;
        const R2 f = ld2(fcur + cs[i]);
        acc.lo |= f.lo & m.lo;
        acc.hi |= f.hi & m.hi;
      }
    }
    return acc;
  }
  // a rack's 8-entry row is one trip for its quads and one for its gathers;
  // quads past the row end are masked (read as down entries, never loaded)
  for (; beg < end; beg += 4u * STEP) {
    uint4 c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      c[j] = beg + j * STEP < end ? q[(beg + j * STEP) >> 2] : make_uint4(kDown, kDown, kDown, kDown);
    uint4 f[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t cs[4] = {c[j].x, c[j].y, c[j].z, c[j].w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
        f[4 * j + i] = (cs[i] & kDown) ? make_uint4(0u, 0u, 0u, 0u) : fcur[cs[i]];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      acc.lo |= (((uint64_t)f[k].y << 32) | f[k].x);
      acc.hi |= (((uint64_t)f[k].w << 32) | f[k].z);
    }
    acc.lo &= m.lo;
    acc.hi &= m.hi;
    if (acc.lo == m.lo && acc.hi == m.hi) break;
  }
  return acc;
}

// out-edges [beg, end) of frontier node u with roots fu
template <uint32_t STEP>
__device__ __forceinline__ void push_scan(const DevGraph& g, const WB& b, uint32_t beg,
                                          uint32_t end, R2 fu) {
  const uint4* q = reinterpret_cast<const uint4*>(g.colx);
  for (uint32_t e = beg; e < end; e += STEP) {
    const uint4 c = q[e >> 2];
    const uint32_t cs[4] = {c.x, c.y, c.z, c.w};
    R2 ss[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ss[i] = (cs[i] & kDown) ? R2{~0ull, ~0ull} : ld2(b.seen + cs[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t lo = fu.lo & ~ss[i].lo, hi = fu.hi & ~ss[i].hi;
      unsigned long long* p = reinterpret_cast<unsigned long long*>(b.accb + cs[i]);
      if (lo) atomicOr(p, (unsigned long long)lo);
      if (hi) atomicOr(p + 1, (unsigned long long)hi);
    }
  }
}

__global__ void __launch_bounds__(256) lv_level_kernel(DevGraph g, LvArgs a, uint32_t d) {
  const uint32_t vbl = blockIdx.x % a.nb;
  if (!a.found[vbl * a.lmax + d]) return;  // level d is empty: this batch is done
  const bool push = (uint64_t)a.mass[vbl * a.lmax + d] * a.push_div < g.E;
  const WB b(a, vbl, g.V);
  const uint32_t V = g.V, lane = threadIdx.x & 63u;
  const uint4* fcur = b.front(a, d);
  uint4* fnext = b.front(a, d + 1);
  const uint32_t blk = blockIdx.x / a.nb, chunks = (V + kBlock - 1) / kBlock;

  if (blk >= chunks) {  // ------------------------- one long row per wave
    const uint32_t bi = (blk - chunks) * kWaves + (threadIdx.x >> 6);
    if (bi >= g.nbig) return;
    const uint32_t u = g.big[bi];
    const uint32_t beg = g.row_ptr[u], end = g.row_ptr[u + 1];
    if (push) {
      const R2 fu = ld2(fcur + u);
      if (fu.any()) push_scan<4u * kWave>(g, b, beg + 4u * lane, end, fu);
      return;
    }
    const R2 s0 = ld2(b.seen + u);
    const R2 m{~s0.lo & b.valid.lo, ~s0.hi & b.valid.hi};
    if (!m.any()) return;  // the node's own lane writes fnext[u] = 0
    R2 acc = pull_scan<4u * kWave>(g, fcur, beg + 4u * lane, end, m, a.masked);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      acc.lo |= shfl_xor64(acc.lo, o);
      acc.hi |= shfl_xor64(acc.hi, o);
    }
    if (lane == 0) {
      const bool tr = transit(g, u);
      st2(fnext + u, tr ? acc : R2{0ull, 0ull});
      if (acc.any()) {
        st2(b.seen + u, R2{s0.lo | acc.lo, s0.hi | acc.hi});
        a.found[vbl * a.lmax + d + 1] = 1u;
        if (tr) atomicAdd(&a.mass[vbl * a.lmax + d + 1], end - beg);
        set_lev(a, b, u, acc, d + 2u);
      }
    }
    return;
  }

  // ------------------------------------------------ one node per lane
  const uint32_t v = blk * kBlock + threadIdx.x;
  if (push) {
    if (v >= V) return;
    const R2 fu = ld2(fcur + v);
    if (!fu.any()) return;
    const uint32_t beg = g.row_ptr[v], end = g.row_ptr[v + 1];
    if (end - beg > kMsBigDeg) return;
    push_scan<4u>(g, b, beg, end, fu);
    return;
  }
  R2 s0{0ull, 0ull}, m{0ull, 0ull};
  uint32_t beg = 0, end = 0;
  if (v < V) {  // the row bounds load with seen (one trip), used or not
    s0 = ld2(b.seen + v);
    beg = g.row_ptr[v];
    end = g.row_ptr[v + 1];
    m = R2{~s0.lo & b.valid.lo, ~s0.hi & b.valid.hi};
  }
  const bool big = m.any() && (end - beg) > kMsBigDeg;
  R2 acc{0ull, 0ull};
  if (m.any() && !big) acc = pull_scan<4u>(g, fcur, beg, end, m, a.masked);
  uint32_t mass = 0;
  if (v < V && !big) {
    const bool tr = acc.any() && transit(g, v);
    st2(fnext + v, tr ? acc : R2{0ull, 0ull});
    if (acc.any()) {
      st2(b.seen + v, R2{s0.lo | acc.lo, s0.hi | acc.hi});
      set_lev(a, b, v, acc, d + 2u);
    }
    if (tr) mass = end - beg;
  }
  mass = wave_add32(mass);
  if (lane == 0 && mass) atomicAdd(&a.mass[vbl * a.lmax + d + 1], mass);
  if (__ballot(acc.any()) && lane == 0) a.found[vbl * a.lmax + d + 1] = 1u;
}

// settle a pushed level: fold the accumulator into seen / next frontier
__global__ void __launch_bounds__(256) lv_settle_kernel(DevGraph g, LvArgs a, uint32_t d) {
  const uint32_t vbl = blockIdx.x % a.nb;
  if (!a.found[vbl * a.lmax + d]) return;
  if (!((uint64_t)a.mass[vbl * a.lmax + d] * a.push_div < g.E)) return;
  const WB b(a, vbl, g.V);
  const uint32_t V = g.V, lane = threadIdx.x & 63u;
  uint4* fnext = b.front(a, d + 1);
  const uint32_t v = (blockIdx.x / a.nb) * kBlock + threadIdx.x;
  R2 acc{0ull, 0ull};
  uint32_t mass = 0;
  if (v < V) {
    acc = ld2(b.accb + v);
    const bool tr = acc.any() && transit(g, v);
    if (acc.any()) {
      st2(b.accb + v, R2{0ull, 0ull});
      const R2 s0 = ld2(b.seen + v);
      st2(b.seen + v, R2{s0.lo | acc.lo, s0.hi | acc.hi});
      set_lev(a, b, v, acc, d + 2u);
      if (tr) mass = g.row_ptr[v + 1] - g.row_ptr[v];
    }
    st2(fnext + v, tr ? acc : R2{0ull, 0ull});
  }
  mass = wave_add32(mass);
  if (lane == 0 && mass) atomicAdd(&a.mass[vbl * a.lmax + d + 1], mass);
  if (__ballot(acc.any()) && lane == 0) a.found[vbl * a.lmax + d + 1] = 1u;
}

// ---------------------------------------------------------------- rows
// Block = (wide batch, root half h: roots 64 h .. 64 h + 63, 512 nodes in two
// 256-node halves). Load: thread (quad q = tid % 64, root group rg = tid / 64:
// roots 16 rg .. + 15 of the half) reads the 16-root slices of its four
// nodes' records (bytes of roots not in seen are stale: masked), transposes
// the 4 x 4 byte blocks with byte permutes and parks [root][quad] words in LDS
// (row pitch 65 words: conflict-free both ways). Store: wave w takes roots
// 16 w .. + 15, lane = quad: each store instruction writes 1 KB of consecutive
// dist row and 256 B of level row (non-temporal: read by the next launch).
__device__ __forceinline__ uint32_t byte_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t nib_bytes(uint32_t nib) {
  return (nib * 0x00204081u) & 0x01010101u;
}
template <int N, typename T>
__device__ __forceinline__ void xreduce_step(T* v, uint32_t lane, int o) {
  const bool up = lane & (uint32_t)o;
#pragma unroll
  for (int i = 0; i < N / 2; ++i) {
    const T send = up ? v[i] : v[i + N / 2];
    const T keep = up ? v[i + N / 2] : v[i];
    T recv;
    if constexpr (sizeof(T) == 8) recv = shfl_xor64(send, o);
    else recv = (T)__shfl_xor((int)send, o);
    v[i] = keep + recv;
  }
}

__global__ void __launch_bounds__(256) lv_rows_kernel(DevGraph g, LvArgs a) {
  __shared__ uint32_t s_T[64 * 65];
  const uint32_t per = 2u * a.nb;
  const uint32_t vbl = (blockIdx.x % per) >> 1, h = blockIdx.x & 1u;
  const WB b(a, vbl, g.V);
  const uint32_t V = g.V, tid = threadIdx.x, q = tid & 63u, rg = tid >> 6;
  const uint32_t vb0 = (blockIdx.x / per) * 512u;
  if (vb0 == 0 && h == 0 && tid == 0) {
    if (a.found[vbl * a.lmax + a.dbound + 1]) atomicOr(a.err, 8u);
    if (a.maxd) {  // the deepest non-empty level (a sweep caps its captured launches there)
      uint32_t dm = 0;
      for (uint32_t d = 1; d <= a.dbound + 1; ++d)
        if (a.found[vbl * a.lmax + d]) dm = d;
      atomicMax(a.maxd, dm);
    }
  }
  const uint32_t base = b.rix0 + 64u * h;  // first root of this half
  if (base >= a.n) return;                  // block-uniform
  const uint32_t nr = min(64u, a.n - base);
  uint32_t pk[16];  // per root of this wave: reached | sum dist << 16
  uint64_t hh[16];  // per root: sum dist_key * (dist + 1)
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    pk[j] = 0u;
    hh[j] = 0ull;
  }
  for (uint32_t half = 0; half < 2u; ++half) {
    const uint32_t v0 = vb0 + 256u * half;
    if (v0 >= V) break;  // block-uniform
    const uint32_t vq = v0 + 4u * q;
    {
      uint32_t x[4][4];  // [node c][word m]: roots 16 rg + 4 m .. + 3 of node vq + c
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t v = vq + c;
        uint4 r4 = make_uint4(0u, 0u, 0u, 0u);
        uint32_t sn = 0;
        if (v < V) {
          r4 = *reinterpret_cast<const uint4*>(b.rec(a, v) + 64u * h + 16u * rg);
          const uint4 s4 = b.seen[v];
          const uint64_t sw = h ? (((uint64_t)s4.w << 32) | s4.z) : (((uint64_t)s4.y << 32) | s4.x);
          sn = (uint32_t)(sw >> (16u * rg)) & 0xFFFFu;
        }
        x[c][0] = r4.x & (nib_bytes(sn & 0xFu) * 0xFFu);
        x[c][1] = r4.y & (nib_bytes((sn >> 4) & 0xFu) * 0xFFu);
        x[c][2] = r4.z & (nib_bytes((sn >> 8) & 0xFu) * 0xFFu);
        x[c][3] = r4.w & (nib_bytes((sn >> 12) & 0xFu) * 0xFFu);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const uint32_t t0 = byte_perm(x[1][m], x[0][m], 0x05010400u);
        const uint32_t t1 = byte_perm(x[1][m], x[0][m], 0x07030602u);
        const uint32_t t2 = byte_perm(x[3][m], x[2][m], 0x05010400u);
        const uint32_t t3 = byte_perm(x[3][m], x[2][m], 0x07030602u);
        const uint32_t r0 = 16u * rg + 4u * m;
        s_T[(r0 + 0u) * 65u + q] = byte_perm(t2, t0, 0x05040100u);
        s_T[(r0 + 1u) * 65u + q] = byte_perm(t2, t0, 0x07060302u);
        s_T[(r0 + 2u) * 65u + q] = byte_perm(t3, t1, 0x05040100u);
        s_T[(r0 + 3u) * 65u + q] = byte_perm(t3, t1, 0x07060302u);
      }
    }
    uint64_t kd[4] = {0ull, 0ull, 0ull, 0ull};
    if (a.digest) {
#pragma unroll
      for (int c = 0; c < 4; ++c) kd[c] = vq + c < V ? g.dkey[2ull * (vq + c)] : 0ull;
    }
    __syncthreads();
    const bool vec = (V & 3u) == 0 && vq + 4u <= V;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t r = 16u * rg + j;  // rg = this wave
      const uint32_t u = s_T[r * 65u + q];
      if (r >= nr) continue;
      // level row: dist + 1, 0x7F for unreached and padding (bytes < 0x80)
      const uint32_t zm = ~((u | 0x80808080u) - 0x01010101u) & 0x80808080u;
      if (vq < a.lev_pitch)
        __builtin_nontemporal_store(
            u | (zm - (zm >> 7)),
            reinterpret_cast<uint32_t*>(a.levrow + (size_t)(base + r) * a.lev_pitch + vq));
      uint32_t dv[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t l = (u >> (8 * c)) & 0xFFu;
        dv[c] = l ? l - 1u : kInf;
        if (a.digest && l) {
          pk[j] += 1u + ((l - 1u) << 16);
          hh[j] += kd[c] * (uint64_t)l;
        }
      }
      if (a.dist) {
        uint32_t* row = a.dist + (size_t)(base + r) * (a.dpitch ? a.dpitch : V) + vq;
        if (vec) {
          store_row16(row, make_uint4(dv[0], dv[1], dv[2], dv[3]));
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (vq + c < V) row[c] = dv[c];
        }
      }
    }
    __syncthreads();  // s_T is rewritten by the next half
  }
  if (a.digest) {
    // 16 roots x 64 lanes -> lane (32 a + 16 b + 8 c + 4 d) holds root 8a+4b+2c+d
    xreduce_step<16>(pk, q, 32);
    xreduce_step<8>(pk, q, 16);
    xreduce_step<4>(pk, q, 8);
    xreduce_step<2>(pk, q, 4);
    xreduce_step<16>(hh, q, 32);
    xreduce_step<8>(hh, q, 16);
    xreduce_step<4>(hh, q, 8);
    xreduce_step<2>(hh, q, 4);
    uint32_t p = pk[0];
    uint64_t hsum = hh[0];
#pragma unroll
    for (int o = 2; o > 0; o >>= 1) {
      p += (uint32_t)__shfl_xor((int)p, o);
      hsum += shfl_xor64(hsum, o);
    }
    const uint32_t r = 16u * rg + ((q >> 5) & 1u) * 8u + ((q >> 4) & 1u) * 4u +
                       ((q >> 3) & 1u) * 2u + ((q >> 2) & 1u);
    if ((q & 3u) == 0 && r < nr && (p & 0xFFFFu)) {
      ospf_digest* dg = a.digest + base + r;
      atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)(p & 0xFFFFu));
      atomicAdd((unsigned long long*)&dg->sum_dist, (unsigned long long)(p >> 16));
      atomicAdd((unsigned long long*)&dg->hash, (unsigned long long)hsum);
    }
  }
}

}  // namespace

hipError_t launch_levels128_traverse(const DevGraph& g, const LvArgs& a, hipStream_t s) {
  const uint32_t init_blocks = a.nb * kRoots;
  hipLaunchKernelGGL(lv_init_kernel, dim3(init_blocks), dim3(kBlock), 0, s, g, a);
  const uint32_t chunks = (g.V + kBlock - 1) / kBlock;
  const uint32_t bigblocks = (g.nbig + kWaves - 1) / kWaves;
  for (uint32_t d = 1; d <= a.dbound; ++d) {
    hipLaunchKernelGGL(lv_level_kernel, dim3(a.nb * (chunks + bigblocks)), dim3(kBlock), 0, s, g,
                       a, d);
    hipLaunchKernelGGL(lv_settle_kernel, dim3(a.nb * chunks), dim3(kBlock), 0, s, g, a, d);
  }
  return hipGetLastError();
}

hipError_t launch_levels128_rows(const DevGraph& g, const LvArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(lv_rows_kernel, dim3(2u * a.nb * ((g.V + 511u) / 512u)), dim3(kBlock), 0, s,
                     g, a);
  return hipGetLastError();
}

}  // namespace ospf
