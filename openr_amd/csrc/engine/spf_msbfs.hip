// spf_msbfs.hip — multi-source bit-parallel BFS (gfx950), unit metric /
// hop count, no ignored links: the all-sources path.
//
// Same result as LinkState::runSpf (openr/decision/LinkState.cpp:836-911) for
// every root of a batch when every usable weight is 1: levels are BFS levels
// and the ECMP next-hop set of a node at level d+1 is the OR over its usable
// in-edges from transit level-d nodes (LinkState.cpp:885-901).
//
// 64 roots share one traversal: per node, one 64-bit word holds a bit per
// root ("seen", "frontier"), so one CSR scan serves 64 SPF runs and the
// per-edge work is a 64-bit AND/OR instead of 64 bitmap probes. Next-hop sets
// are bit-sliced the same way: plane k of node v (one u64) has bit r set when
// the k-th distinct neighbour of root r is a next hop of v. A pass computes
// one 32-bit next-hop word g (planes for neighbour indices [32g, 32g+32)); a
// root with K distinct neighbours needs ceil(K/32) passes, each re-running the
// traversal. Small batches of wide roots pack planes: a batch of R <= 64
// roots keeps PP = 64/R planes per word (bit j*R + r = plane j of root r), so
// a pass covers 32*PP neighbours (PP next-hop words) and a 12-root batch of
// 1,781-port spines needs 12 passes instead of 56 (the host picks R, PP).
// A "virtual batch" = (R-root batch, pass g); a round runs up to
// NB virtual batches side by side, and virtual batch i of a round is served by
// workgroups i, i+NB, ... so with NB a multiple of 8 its workgroups land on one
// XCD and its state stays in that XCD's L2.
//
// Level d -> d+1, chosen per virtual batch from the frontier's out-edge mass:
//  * pull (bottom-up): node v with unseen roots m scans its in-edges u:
//    f = frontier[u] & m; next |= f; plane_k(v) |= plane_k(u) & f. The owner
//    lane of v is the only writer of v's state: no atomics.
//  * push (top-down, small frontiers): frontier node u ORs f = frontier[u] &
//    ~seen[v] into an accumulator and planes of each head v (64-bit atomics);
//    a finalize pass then folds the accumulator into seen / next frontier.
// Rows longer than kMsBigDeg (spines) are scanned by a whole wave each, in
// extra workgroups after the per-node ones, so they never serialise a wave.
// dist / next-hop rows of newly reached (root, node) pairs are written when
// the level is settled (coalesced across the wave's 64 nodes, one store per
// root). Level 1 (the root's own neighbours) is expanded by the init kernel.
// The level count is bounded on the host (spf_engine.hip: 2 * eccentricity of
// the transit subgraph + 2), so the launches need no host round trip; a level
// whose predecessor found nothing returns at once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;
constexpr int kWave = 64;
constexpr uint32_t kBlock = 256;
constexpr uint32_t kWavesPerBlock = kBlock / kWave;

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int o) {
  const uint32_t lo = __shfl_xor((uint32_t)x, o, kWave);
  const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), o, kWave);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x |= shfl_xor64(x, o);
  return x;
}
__device__ __forceinline__ uint32_t wave_add32(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
  return x;
}
__device__ __forceinline__ bool transit(const DevGraph& g, uint32_t v) {
  return !((g.nt_bits[v >> 5] >> (v & 31)) & 1u);
}
__device__ __forceinline__ void or64(uint64_t* p, uint64_t x) {
  atomicOr((unsigned long long*)p, (unsigned long long)x);
}
// register arrays of KP plane words (KP = 0: KSP2 distance-only mode)
constexpr int kpa(int kp) { return kp > 0 ? kp : 1; }

// one (64-root batch, next-hop word) of the round, and its state arrays
struct VB {
  uint32_t vbl, g, rix0, V;
  uint64_t valid;  // bits of roots present (R bits at most)
  uint64_t* seen;
  uint64_t* accb;
  uint64_t* P;
  const uint32_t* igb;  // KSP2 mode: ignored-edge bitmap and root masks
  const uint64_t* igm;
  __device__ VB(const MsArgs& a, uint32_t vbl_, uint32_t V_, int kp, uint32_t E = 0)
      : vbl(vbl_), V(V_), fs(kp > 0 ? 2u : 1u) {
    // Multi-pass rounds: the passes of one batch write different next-hop
    // words of the same row entries, so they go to one XCD (workgroup i of a
    // launch runs on XCD i % 8 and serves state slot vbl = i % nb): slot vbl
    // takes round position (vbl % 8) * nb / 8 + vbl / 8, and a batch's passes
    // (consecutive positions) fill their lines in one L2 instead of writing
    // back partial lines from several.
    uint32_t t = vbl;
    if (a.npass > 1 && (a.nb & 7u) == 0) t = (vbl & 7u) * (a.nb >> 3) + (vbl >> 3);
    const uint32_t vb = a.vb0 + t;
    g = vb % a.npass;
    rix0 = (vb / a.npass) * a.R;
    const uint32_t nv = min(a.R, a.n - rix0);
    valid = nv == 64u ? ~0ull : ((1ull << nv) - 1ull);
    seen = a.seen + (size_t)vbl * V;
    accb = a.accb + (size_t)vbl * V;
    P = kp > 0 ? a.planes + (size_t)vbl * V * kp : nullptr;  // kp -1: distances only
    igb = kp == 0 ? a.igb + (size_t)vbl * a.igw : nullptr;
    igm = kp == 0 ? a.igm + (size_t)vbl * E : nullptr;
  }
  // roots (of the batch) that ignore the link of entry e (KSP2 mode)
  __device__ __forceinline__ uint64_t ignored(uint32_t e) const {
    return ((igb[e >> 5] >> (e & 31u)) & 1u) ? igm[e] : 0ull;
  }
  // same for the 4 entries e .. e+3 (e % 4 == 0): ~mask per entry
  __device__ __forceinline__ void keep4(uint32_t e, uint64_t* keep) const {
    const uint32_t ib = (igb[e >> 5] >> (e & 31u)) & 0xFu;
#pragma unroll
    for (int i = 0; i < 4; ++i) keep[i] = ((ib >> i) & 1u) ? ~igm[e + i] : ~0ull;
  }
  // frontier record of level d: {roots with v in the frontier, those of them
  // with a non-zero plane in this pass} (16 B per node)
  // (KP <= 0, distances only: the record is the frontier word alone, 8 B)
  uint32_t fs;  // u64 words per frontier record: 2 with planes, 1 without
  __device__ uint64_t* front(const MsArgs& a, uint32_t d) const {
    return a.front + ((size_t)(d & 1u) * a.nb + vbl) * V * fs;
  }
};

// next-hop word of root r from the KP planes (bit k = plane k, bit r)
template <int KP>
__device__ __forceinline__ uint32_t gather_word(const uint64_t* p, uint32_t r) {
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < KP; ++k) w |= (uint32_t)((p[k] >> r) & 1ull) << k;
  return w;
}

// lev bytes of node v for the roots in `acc` := val (a (node, root) pair is
// reached once; the other bytes are kept, stale or not: readers mask the
// record with seen[v]). Byte r of the 64-B record is root r.
__device__ __forceinline__ void set_lev(const MsArgs& a, const VB& b, uint32_t v, uint64_t acc,
                                        uint32_t val) {
  uint4* rec = reinterpret_cast<uint4*>(a.lev + ((size_t)b.vbl * b.V + v) * 64u);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint32_t bits = (uint32_t)(acc >> (16 * c)) & 0xFFFFu;
    if (!bits) continue;
    // nibble -> one 0x01 byte per set bit (bit i -> byte i); byte := val
    auto put = [&](uint32_t w, uint32_t nib) {
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

// dist / next-hop rows of the (root, v) pairs in `acc` (lane = node v): one
// coalesced store per root present anywhere in the wave; deferred runs only
// record dist + 1 in lev (msbfs_rows writes whole rows at the end)
template <int KP>
__device__ __forceinline__ void emit_rows(const MsArgs& a, const VB& b, uint32_t v, uint64_t acc,
                                          const uint64_t* pacc, uint32_t dist) {
  if (a.defer) {  // merged rows: the passes share the levels, pass 0 records them
    if (acc && (!a.merged || b.g == 0)) set_lev(a, b, v, acc, dist + 1u);
    return;
  }
  uint64_t un = wave_or64(acc);
  while (un) {
    const uint32_t r = (uint32_t)(__ffsll((unsigned long long)un) - 1);
    un &= un - 1;
    if ((acc >> r) & 1ull) {
      const size_t row = (size_t)(b.rix0 + r) * b.V + v;
      if (a.dist && b.g == 0) a.dist[row] = dist;
      if (a.nh) a.nh[row * a.W + b.g] = gather_word<KP>(pacc, r);
    }
  }
}

template <int KP>
__device__ __forceinline__ void load_planes(const uint64_t* P, uint32_t u, uint64_t* pu) {
  if constexpr (KP <= 0) return;
  const uint4* q = reinterpret_cast<const uint4*>(P + (size_t)u * KP);
#pragma unroll
  for (int k = 0; k < KP / 2; ++k) {
    const uint4 w = q[k];
    pu[2 * k] = ((uint64_t)w.y << 32) | w.x;
    pu[2 * k + 1] = ((uint64_t)w.w << 32) | w.z;
  }
}

// roots with a set bit in any of the KP packed plane words
template <int KP>
__device__ __forceinline__ uint64_t planes_roots(const MsArgs& a, const uint64_t* p) {
  uint64_t z = 0;
#pragma unroll
  for (int k = 0; k < KP; ++k) z |= p[k];
  uint64_t zz = z;
  for (uint32_t j = 1; j < a.PP; ++j) zz |= z >> (j * a.R);
  return a.PP == 1 ? zz : zz & ((1ull << a.R) - 1ull);
}

// next-hop word w (0 .. OW-1) of this pass for root r: planes 32w .. 32w+31
// of the pass (plane li = k * PP + j sits in word k, bit j * R + r)
template <int KP>
__device__ __forceinline__ uint32_t pass_word(const MsArgs& a, const uint64_t* p, uint32_t r,
                                              uint32_t w) {
  if (a.PP == 1) return gather_word<KP>(p, r);
  const uint32_t lo = 32u * w, hi = lo + 32u;
  uint32_t word = 0;
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const uint32_t l0 = (uint32_t)k * a.PP;
    if (l0 + a.PP <= lo || l0 >= hi) continue;
    const uint64_t x = p[k] >> r;
    for (uint32_t j = 0; j < a.PP; ++j) {
      const uint32_t li = l0 + j;
      if (li >= lo && li < hi) word |= (uint32_t)((x >> (j * a.R)) & 1ull) << (li - lo);
    }
  }
  return word;
}

// ---------------------------------------------------------------- init
// One wave per root: level 0 (the root) and level 1 (its usable neighbours,
// next hop = themselves). Atomics: several roots of a batch may share nodes.
template <int KP>
__global__ void __launch_bounds__(256) msbfs_init_kernel(DevGraph g, MsArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t slot = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const uint32_t vbl = slot / a.R, bit = slot % a.R;
  if (vbl >= a.nb) return;
  const VB b(a, vbl, g.V, KP, g.E);
  const uint32_t rix = b.rix0 + bit;
  if (rix >= a.n) return;
  const uint32_t V = g.V;
  const uint32_t s = a.roots[rix];
  if (s >= V) {  // device-side root list: never index past the graph
    if (lane == 0) atomicOr(a.err, 64u);
    return;
  }
  const uint32_t nb0 = g.dn_off[s], nn = g.dn_off[s + 1] - nb0;
  if (nn > a.kcap || nn > 32u * a.W) {
    if (lane == 0) atomicOr(a.err, 1u);
    return;
  }
  const uint64_t bm = 1ull << bit;
  uint64_t* f1 = b.front(a, 1);
  const size_t row = (size_t)rix * V;
  uint32_t* lev32 = reinterpret_cast<uint32_t*>(a.lev);
  auto lev_or = [&](uint32_t v, uint32_t val) {  // byte `bit` of node v's record := val
    uint32_t* w = &lev32[(((size_t)vbl * V + v) * 64u + bit) / 4u];
    atomicAnd(w, ~(0xFFu << (8u * (bit & 3u))));  // stale bytes: records are not cleared
    atomicOr(w, val << (8u * (bit & 3u)));
  };
  const bool rec = !a.merged || b.g == 0;  // merged rows: pass 0 records the levels
  if (lane == 0) {
    or64(&b.seen[s], bm);
    if (a.defer) {
      if (rec) lev_or(s, 1u);
    } else {
      if (a.dist && b.g == 0) a.dist[row + s] = 0u;
      if (a.nh) a.nh[(row + s) * a.W + b.g] = 0u;
    }
  }
  const uint32_t e0 = g.row_ptr[s], e1 = g.row_ptr[s + 1];
  bool any = false;
  uint32_t mass = 0;
  for (uint32_t e = e0 + lane; e < e1; e += kWave) {
    const uint32_t cx = g.colx[e];
    if ((cx & kDown) || cx == s) continue;
    if (KP == 0 && ((b.ignored(e) >> bit) & 1ull)) continue;
    const uint32_t v = cx;
    const uint32_t lo = g.didx[e];  // index of v among s's distinct neighbours
    // plane of v in this pass (>= KP * PP, wrapped, when outside it)
    const uint32_t li = lo - 32u * a.OW * b.g;
    const bool in = KP > 0 && li < (uint32_t)KP * a.PP;
    const uint32_t k = li / a.PP, pb = (li % a.PP) * a.R + bit;  // plane word, bit
    const uint32_t kw = lo - 32u * b.g;  // unpacked (PP == 1) next-hop word bit
    or64(&b.seen[v], bm);
    if (transit(g, v)) {
      const unsigned long long old =
          atomicOr((unsigned long long*)&f1[b.fs * v], (unsigned long long)bm);
      if (!old) mass += g.row_ptr[v + 1] - g.row_ptr[v];  // first root to reach v
      if (in) or64(&f1[b.fs * v + 1u], bm);
    }
    if (in) or64(&b.P[(size_t)v * KP + k], 1ull << pb);
    if (a.defer) {
      // parallel links: the same byte again, same value (an OR of 2 | 2 = 2)
      if (rec) lev_or(v, 2u);
    } else {
      if (a.dist && b.g == 0) a.dist[row + v] = 1u;
      if (a.nh) a.nh[(row + v) * a.W + b.g] = (kw < 32u) ? (1u << kw) : 0u;
    }
    any = true;
  }
  mass = wave_add32(mass);
  if (lane == 0 && mass) atomicAdd(&a.mass[vbl * a.lmax + 1], mass);
  if (__ballot(any) && lane == 0) a.found[vbl * a.lmax + 1] = 1u;
}

// ---------------------------------------------------------------- pull
// in-edges [beg, end) of a node with unseen roots m, one lane (STEP 4) or the
// wave (lane offset folded into beg, STEP 256); rows are padded to 4 entries
template <int KP, uint32_t STEP>
__device__ __forceinline__ void pull_scan(const DevGraph& g, const VB& b, const uint64_t* fcur,
                                          const uint64_t* P, uint32_t beg, uint32_t end,
                                          uint64_t m, uint64_t rep, uint64_t& acc,
                                          uint64_t* pacc) {
  const uint4* q = reinterpret_cast<const uint4*>(g.colx);
  const uint4* fr = reinterpret_cast<const uint4*>(fcur);
  if constexpr (KP <= 0) {
    // distances only: four row quads (16 entries) per step, every load of a
    // step issued before any is used (a fabric switch's 84-entry row is six
    // dependent trips instead of 21); stop once every unseen root is found
    for (; beg + 3u * STEP < end; beg += 4u * STEP) {
      uint4 c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = q[(beg + j * STEP) >> 2];
      uint64_t f[16];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t cs[4] = {c[j].x, c[j].y, c[j].z, c[j].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) f[4 * j + i] = (cs[i] & kDown) ? 0ull : fcur[cs[i]];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint64_t keep[4] = {~0ull, ~0ull, ~0ull, ~0ull};
        if (KP == 0) b.keep4(beg + j * STEP, keep);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc |= f[4 * j + i] & m & keep[i];
      }
      if (acc == m) return;
    }
  }
  for (uint32_t e = beg; e < end; e += STEP) {
    const uint4 c = q[e >> 2];
    const uint32_t cs[4] = {c.x, c.y, c.z, c.w};
    uint4 fs[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (KP > 0) {
        fs[i] = (cs[i] & kDown) ? make_uint4(0, 0, 0, 0) : fr[cs[i]];
      } else {  // 8-B records: the frontier word alone
        const uint64_t f = (cs[i] & kDown) ? 0ull : fcur[cs[i]];
        fs[i] = make_uint4((uint32_t)f, (uint32_t)(f >> 32), 0u, 0u);
      }
    }
    uint64_t keep[4] = {~0ull, ~0ull, ~0ull, ~0ull};
    if (KP == 0) b.keep4(e, keep);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t f = (((uint64_t)fs[i].y << 32) | fs[i].x) & m & keep[i];
      if (!f) continue;
      acc |= f;
      if (KP <= 0) continue;  // distances only (KSP2 reruns, derive mode)
      // roots whose tail has no plane bit in this pass add nothing to them
      const uint64_t fz = (((uint64_t)fs[i].w << 32) | fs[i].z) & f;
      if (!fz) continue;
      const uint64_t fx = fz * rep;  // the roots' bits in every packed plane slot
      uint64_t pu[kpa(KP)];
      load_planes<KP>(P, cs[i], pu);
#pragma unroll
      for (int k = 0; k < KP; ++k) pacc[k] |= pu[k] & fx;
    }
  }
}

// ---------------------------------------------------------------- push
// out-edges [beg, end) of frontier node u (roots fu, planes pu)
template <int KP, uint32_t STEP>
__device__ __forceinline__ void push_scan(const DevGraph& g, const VB& b, uint32_t beg,
                                          uint32_t end, uint64_t fu, uint64_t rep,
                                          const uint64_t* pu) {
  const uint4* q = reinterpret_cast<const uint4*>(g.colx);
  for (uint32_t e = beg; e < end; e += STEP) {
    const uint4 c = q[e >> 2];
    const uint32_t cs[4] = {c.x, c.y, c.z, c.w};
    uint64_t ss[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ss[i] = (cs[i] & kDown) ? ~0ull : b.seen[cs[i]];
    uint64_t keep[4] = {~0ull, ~0ull, ~0ull, ~0ull};
    if (KP == 0) b.keep4(e, keep);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t f = fu & ~ss[i] & keep[i];
      if (!f) continue;
      const uint32_t v = cs[i];
      or64(&b.accb[v], f);
      const uint64_t fx = f * rep;
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const uint64_t x = pu[k] & fx;
        if (x) or64(&b.P[(size_t)v * KP + k], x);
      }
    }
  }
}

template <int KP>
__device__ __forceinline__ uint64_t planes_or(const uint64_t* p) {
  uint64_t z = 0;
#pragma unroll
  for (int k = 0; k < KP; ++k) z |= p[k];
  return z;
}

template <int KP>
__global__ void __launch_bounds__(256) msbfs_level_kernel(DevGraph g, MsArgs a, uint32_t d) {
  const uint32_t vbl = blockIdx.x % a.nb;
  if (!a.found[vbl * a.lmax + d]) return;  // level d is empty: this batch is done
  const bool push = (uint64_t)a.mass[vbl * a.lmax + d] * a.push_div < g.E;
  const VB b(a, vbl, g.V, KP, g.E);
  const uint32_t V = g.V;
  const int lane = threadIdx.x & 63;
  const uint64_t* fcur = b.front(a, d);
  uint64_t* fnext = b.front(a, d + 1);
  const uint32_t blk = blockIdx.x / a.nb, chunks = (V + kBlock - 1) / kBlock;

  if (blk >= chunks) {  // ------------------------- one long row per wave
    const uint32_t bi = (blk - chunks) * kWavesPerBlock + (threadIdx.x >> 6);
    if (bi >= g.nbig) return;
    const uint32_t u = g.big[bi];
    const uint32_t beg = g.row_ptr[u], end = g.row_ptr[u + 1];
    if (push) {
      const uint64_t fu = fcur[b.fs * u];
      if (!fu) return;
      uint64_t pu[kpa(KP)];
      load_planes<KP>(b.P, u, pu);
      push_scan<KP, 4u * kWave>(g, b, beg + 4u * lane, end, fu, a.rep, pu);
      return;
    }
    const uint64_t m = ~b.seen[u] & b.valid;
    if (!m) return;  // the node's own lane writes fnext[u] = 0
    uint64_t acc = 0, pacc[kpa(KP)];
#pragma unroll
    for (int k = 0; k < kpa(KP); ++k) pacc[k] = 0;
    pull_scan<KP, 4u * kWave>(g, b, fcur, b.P, beg + 4u * lane, end, m, a.rep, acc, pacc);
    acc = wave_or64(acc);
#pragma unroll
    for (int k = 0; k < KP; ++k) pacc[k] = wave_or64(pacc[k]);
    const bool tr = transit(g, u);
    if (lane == 0) {
      fnext[b.fs * u] = tr ? acc : 0ull;
      if constexpr (KP > 0) fnext[2u * u + 1u] = tr ? planes_roots<KP>(a, pacc) & acc : 0ull;
      if (acc) {
        b.seen[u] = (~m & b.valid) | acc;
#pragma unroll
        for (int k = 0; k < KP; ++k) b.P[(size_t)u * KP + k] |= pacc[k];
        a.found[vbl * a.lmax + d + 1] = 1u;
        if (tr) atomicAdd(&a.mass[vbl * a.lmax + d + 1], end - beg);
      }
    }
    if (a.defer) {
      if (lane == 0 && acc && (!a.merged || b.g == 0)) set_lev(a, b, u, acc, d + 2u);
    } else if ((acc >> lane) & 1ull) {  // lane r writes root r's entries
      const size_t row = (size_t)(b.rix0 + lane) * V + u;
      if (a.dist && b.g == 0) a.dist[row] = d + 1;
      if (a.nh) a.nh[row * a.W + b.g] = gather_word<KP>(pacc, lane);
    }
    return;
  }

  // ------------------------------------------------ one node per lane
  const uint32_t v = blk * kBlock + threadIdx.x;
  if (push) {
    if (v >= V) return;
    const uint64_t fu = fcur[b.fs * v];
    if (!fu) return;
    const uint32_t beg = g.row_ptr[v], end = g.row_ptr[v + 1];
    if (end - beg > kMsBigDeg) return;
    uint64_t pu[kpa(KP)];
    load_planes<KP>(b.P, v, pu);
    push_scan<KP, 4u>(g, b, beg, end, fu, a.rep, pu);
    return;
  }
  uint64_t s0 = 0, m = 0;
  uint32_t beg = 0, end = 0;
  if (v < V) {
    s0 = b.seen[v];
    m = ~s0 & b.valid;
    if (m) {
      beg = g.row_ptr[v];
      end = g.row_ptr[v + 1];
    }
  }
  const bool big = m && (end - beg) > kMsBigDeg;
  uint64_t acc = 0, pacc[kpa(KP)];
#pragma unroll
  for (int k = 0; k < kpa(KP); ++k) pacc[k] = 0;
  if (m && !big) pull_scan<KP, 4u>(g, b, fcur, b.P, beg, end, m, a.rep, acc, pacc);
  uint32_t mass = 0;
  if (v < V && !big) {
    const bool tr = acc && transit(g, v);
    if (acc) {
      b.seen[v] = s0 | acc;
#pragma unroll
      for (int k = 0; k < KP; ++k)
        if (pacc[k]) b.P[(size_t)v * KP + k] |= pacc[k];
    }
    fnext[b.fs * v] = tr ? acc : 0ull;
    if constexpr (KP > 0) fnext[2u * v + 1u] = tr ? planes_roots<KP>(a, pacc) & acc : 0ull;
    if (tr) mass = end - beg;
  }
  emit_rows<KP>(a, b, v, acc, pacc, d + 1);
  mass = wave_add32(mass);
  if (lane == 0 && mass) atomicAdd(&a.mass[vbl * a.lmax + d + 1], mass);
  if (__ballot(acc != 0) && lane == 0) a.found[vbl * a.lmax + d + 1] = 1u;
}

// settle a pushed level: fold the accumulator into seen / next frontier and
// write the rows (pull levels return at once)
template <int KP>
__global__ void __launch_bounds__(256) msbfs_settle_kernel(DevGraph g, MsArgs a, uint32_t d) {
  const uint32_t vbl = blockIdx.x % a.nb;
  if (!a.found[vbl * a.lmax + d]) return;
  if (!((uint64_t)a.mass[vbl * a.lmax + d] * a.push_div < g.E)) return;
  const VB b(a, vbl, g.V, KP);
  const uint32_t V = g.V;
  const int lane = threadIdx.x & 63;
  uint64_t* fnext = b.front(a, d + 1);
  const uint32_t v = (blockIdx.x / a.nb) * kBlock + threadIdx.x;
  uint64_t acc = 0, pacc[kpa(KP)];
#pragma unroll
  for (int k = 0; k < kpa(KP); ++k) pacc[k] = 0;
  uint32_t mass = 0;
  if (v < V) {
    acc = b.accb[v];
    const bool tr = acc && transit(g, v);
    if (acc) {
      b.accb[v] = 0ull;
      b.seen[v] |= acc;
      load_planes<KP>(b.P, v, pacc);
      if (tr) mass = g.row_ptr[v + 1] - g.row_ptr[v];
    }
    fnext[b.fs * v] = tr ? acc : 0ull;
    if constexpr (KP > 0) fnext[2u * v + 1u] = tr ? planes_roots<KP>(a, pacc) & acc : 0ull;
  }
  emit_rows<KP>(a, b, v, acc, pacc, d + 1);
  mass = wave_add32(mass);
  if (lane == 0 && mass) atomicAdd(&a.mass[vbl * a.lmax + d + 1], mass);
  if (__ballot(acc != 0) && lane == 0) a.found[vbl * a.lmax + d + 1] = 1u;
}

// ---------------------------------------------------------------- final
// Unreached (root, node) pairs: dist INF, next-hop word 0; words past the
// computed passes (nh_words > passes needed) are zero for every node.
__global__ void __launch_bounds__(256) msbfs_final_kernel(DevGraph g, MsArgs a) {
  const uint32_t vbl = blockIdx.x % a.nb;
  const VB b(a, vbl, g.V, 0);
  const uint32_t V = g.V;
  const uint32_t v = (blockIdx.x / a.nb) * kBlock + threadIdx.x;
  if (v == 0 && a.found[vbl * a.lmax + a.dbound + 1]) atomicOr(a.err, 8u);
  const uint64_t un = v < V ? (~b.seen[v] & b.valid) : 0ull;
  uint64_t w = wave_or64(un);
  while (w) {
    const uint32_t r = (uint32_t)(__ffsll((unsigned long long)w) - 1);
    w &= w - 1;
    if ((un >> r) & 1ull) {
      const size_t row = (size_t)(b.rix0 + r) * V + v;
      if (a.dist && b.g == 0) a.dist[row] = kInf;
      if (a.nh) a.nh[row * a.W + b.g] = 0u;
    }
  }
  if (a.nh && b.g == a.npass - 1 && a.npass < a.W && v < V) {
    for (uint64_t x = b.valid; x; x &= x - 1) {
      const uint32_t r = (uint32_t)(__ffsll((unsigned long long)x) - 1);
      uint32_t* p = a.nh + ((size_t)(b.rix0 + r) * V + v) * a.W;
      for (uint32_t k = a.npass; k < a.W; ++k) p[k] = 0u;
    }
  }
}

// ---------------------------------------------------------------- rows
// Deferred output: one workgroup writes the rows of 64 nodes x the batch's
// roots for this pass. lev (dist + 1) and, word by word, the pass's next-hop
// words (bit-planes transposed per root) are staged in LDS and stored root by
// root: 16 lanes x 16 B cover one root's 64 consecutive dist values, so the
// dist rows (and nh rows when W == 1) go out as whole 16-B stores; wider nh
// rows store word g*OW + w of each node. The digest terms of the same values
// are added into the roots' records (passes add up).
template <int KP>
__global__ void __launch_bounds__(256) msbfs_rows_kernel(DevGraph g, MsArgs a) {
  __shared__ uint8_t s_lev[64 * 64];   // [node][root]
  __shared__ uint32_t s_nh[64 * 65];   // [root][node] (+1 pad: conflict-free columns)
  __shared__ uint64_t s_dk[64 * 2];    // [node] {dist_key, node_key}
  const uint32_t vbl = blockIdx.x % a.nb;
  const VB b(a, vbl, g.V, KP);
  const uint32_t V = g.V, tid = threadIdx.x;
  const uint32_t v0 = (blockIdx.x / a.nb) * 64u, nv = min(64u, V - v0);
  if (v0 == 0 && tid == 0 && a.found[vbl * a.lmax + a.dbound + 1]) atomicOr(a.err, 8u);
  const uint32_t nr = min(a.R, a.n - b.rix0);
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.lev + ((size_t)vbl * V + v0) * 64u);
    if (tid < nv * 4u) reinterpret_cast<uint4*>(s_lev)[tid] = src[tid];
  }
  if (a.digest && tid < 128u) s_dk[tid] = (v0 + tid / 2u < V) ? g.dkey[2ull * v0 + tid] : 0ull;
  // node n = tid / 4 computes the words of roots 16q .. 16q+15 (q = tid % 4)
  const uint32_t pn = tid >> 2, pq = tid & 3u;
  uint64_t p[KP];
  if (pn < nv) {
    load_planes<KP>(b.P, v0 + pn, p);
  } else {
#pragma unroll
    for (int k = 0; k < KP; ++k) p[k] = 0;
  }
  // digest: root dr = tid / 4 over nodes 16 * (tid % 4) .. + 15
  const uint32_t dr = tid >> 2, dn0 = 16u * (tid & 3u);
  uint64_t reached = 0, sumd = 0, h = 0;
  const bool vec = (V & 3u) == 0 && nv == 64u;
  // the pass's words of root r (stage: s_nh[r][node]); the first word is
  // staged before the barrier (nothing reads s_nh yet)
  auto stage_words = [&](uint32_t w) {
    for (uint32_t i = 0; i < 16u; ++i) {
      const uint32_t r = 16u * pq + i;
      if (r < nr) s_nh[r * 65u + pn] = pass_word<KP>(a, p, r, w);
    }
  };
  const uint32_t nw = b.g * a.OW < a.W ? min(a.OW, a.W - b.g * a.OW) : 0u;  // words of this pass
  if (nw) stage_words(0);
  __syncthreads();
  // stores first, then the digest terms of the same LDS values: no barrier
  // follows the last stores, so they drain under the digest work
  if (b.g == 0) {
    if (a.dist) {
      for (uint32_t i = tid; i < 64u * 16u; i += kBlock) {  // (root, node quad)
        const uint32_t r = i >> 4, q = i & 15u;
        if (r >= nr) break;
        uint32_t dv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t l = s_lev[(4u * q + j) * 64u + r];
          dv[j] = l ? l - 1u : kInf;
        }
        uint32_t* row = a.dist + (size_t)(b.rix0 + r) * V + v0 + 4u * q;
        if (vec) {
          *reinterpret_cast<uint4*>(row) = make_uint4(dv[0], dv[1], dv[2], dv[3]);
        } else {
          for (uint32_t j = 0; j < 4u; ++j)
            if (4u * q + j < nv) row[j] = dv[j];
        }
      }
    }
    if (a.digest && dr < nr) {
      for (uint32_t n = dn0; n < dn0 + 16u && n < nv; ++n) {
        const uint32_t l = s_lev[n * 64u + dr];
        if (!l) continue;
        reached += 1;
        sumd += l - 1u;
        h += s_dk[2u * n] * (uint64_t)l;
      }
    }
  }
  for (uint32_t w = 0; w < nw; ++w) {
    const uint32_t wg = b.g * a.OW + w;  // next-hop word of the output row
    if (w > 0) {
      stage_words(w);
      __syncthreads();
    }
    if (a.nh) {
      if (a.W == 1 || a.nhs) {  // word-major rows: 16 lanes x 16 B per root
        for (uint32_t i = tid; i < 64u * 16u; i += kBlock) {
          const uint32_t r = i >> 4, q = i & 15u;
          if (r >= nr) break;
          const uint32_t* src = &s_nh[r * 65u + 4u * q];
          uint32_t* row = (a.nhs ? a.nhs + ((size_t)(b.rix0 + r) * a.W + wg) * V
                                 : a.nh + (size_t)(b.rix0 + r) * V) + v0 + 4u * q;
          if (vec) {
            *reinterpret_cast<uint4*>(row) = make_uint4(src[0], src[1], src[2], src[3]);
          } else {
            for (uint32_t j = 0; j < 4u; ++j)
              if (4u * q + j < nv) row[j] = src[j];
          }
        }
      } else {
        for (uint32_t i = tid; i < 64u * 64u; i += kBlock) {  // (root, node)
          const uint32_t r = i >> 6, n = i & 63u;
          if (r >= nr) break;
          if (n < nv) a.nh[((size_t)(b.rix0 + r) * V + v0 + n) * a.W + wg] = s_nh[r * 65u + n];
        }
      }
    }
    if (a.digest && dr < nr) {
      for (uint32_t n = dn0; n < dn0 + 16u && n < nv; ++n) {
        const uint32_t word = s_nh[dr * 65u + n];
        if (word && s_lev[n * 64u + dr]) h += s_dk[2u * n + 1u] * digest_word_key(wg, word);
      }
    }
    if (w + 1 < nw) __syncthreads();  // s_nh is rewritten for the next word
  }
  // words past the computed passes are zero for every node
  if (a.nh && !a.nhs && b.g == a.npass - 1 && a.npass * a.OW < a.W) {
    for (uint32_t i = tid; i < 64u * 64u; i += kBlock) {
      const uint32_t r = i >> 6, n = i & 63u;
      if (r >= nr) break;
      if (n >= nv) continue;
      uint32_t* row = a.nh + ((size_t)(b.rix0 + r) * V + v0 + n) * a.W;
      for (uint32_t k = a.npass * a.OW; k < a.W; ++k) row[k] = 0u;
    }
  }
  if (a.digest) {
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) {
      reached += shfl_xor64(reached, o);
      sumd += shfl_xor64(sumd, o);
      h += shfl_xor64(h, o);
    }
    if ((tid & 3u) == 0 && dr < nr) {
      ospf_digest* dg = a.digest + b.rix0 + dr;
      if (reached) {
        atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)reached);
        atomicAdd((unsigned long long*)&dg->sum_dist, (unsigned long long)sumd);
      }
      if (h) atomicAdd((unsigned long long*)&dg->hash, (unsigned long long)h);
    }
  }
}

// Multi-pass batches (2..7 next-hop words, one word per pass): ONE rows
// kernel per round for all passes of a batch, instead of one per pass that
// writes its word into every W-word row entry (W partial writes per line,
// each pass's lines written back separately). A block = (batch of the
// round, 64 nodes): lev bytes once (the passes share the traversal; passes
// g > 0 do not record them), then per half of the roots every pass's words
// are assembled in LDS as [root][node][word] and each root's 64 x W words go
// out as contiguous 16-B stores; dist rows and digests once.
template <int KP>
__global__ void __launch_bounds__(256) msbfs_rows_multi_kernel(DevGraph g, MsArgs a,
                                                               uint32_t nbatch) {
  __shared__ uint8_t s_lev[64 * 64];  // [node][root]
  __shared__ uint64_t s_dk[64 * 2];
  extern __shared__ uint32_t s_row[];  // [32 roots of the half][node][W words]
  const uint32_t V = g.V, tid = threadIdx.x, W = a.W, np = a.npass;
  const uint32_t bl = blockIdx.x % nbatch;
  const uint32_t v0 = (blockIdx.x / nbatch) * 64u, nv = min(64u, V - v0);
  const uint32_t nb8 = a.nb >> 3;
  auto slot = [&](uint32_t t) {  // round position -> state slot (inverse of VB's map)
    return (a.nb & 7u) == 0 ? (t % nb8) * 8u + t / nb8 : t;
  };
  const uint32_t vbl0 = slot(bl * np);
  const uint32_t rix0 = (a.vb0 / np + bl) * a.R;
  const uint32_t nr = min(a.R, a.n - rix0);
  if (v0 == 0 && tid == 0 && a.found[vbl0 * a.lmax + a.dbound + 1]) atomicOr(a.err, 8u);
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.lev + ((size_t)vbl0 * V + v0) * 64u);
    if (tid < nv * 4u) reinterpret_cast<uint4*>(s_lev)[tid] = src[tid];
  }
  if (a.digest && tid < 128u) s_dk[tid] = (v0 + tid / 2u < V) ? g.dkey[2ull * v0 + tid] : 0ull;
  __syncthreads();
  const bool vec = (V & 3u) == 0 && nv == 64u;
  if (a.dist) {
    for (uint32_t i = tid; i < 64u * 16u; i += kBlock) {  // (root, node quad)
      const uint32_t r = i >> 4, q = i & 15u;
      if (r >= nr) break;
      uint32_t dv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t l = s_lev[(4u * q + j) * 64u + r];
        dv[j] = l ? l - 1u : kInf;
      }
      uint32_t* row = a.dist + (size_t)(rix0 + r) * V + v0 + 4u * q;
      if (vec) {
        *reinterpret_cast<uint4*>(row) = make_uint4(dv[0], dv[1], dv[2], dv[3]);
      } else {
        for (uint32_t j = 0; j < 4u; ++j)
          if (4u * q + j < nv) row[j] = dv[j];
      }
    }
  }
  // digest: root dr = tid / 4 over nodes 16 * (tid % 4) .. + 15
  const uint32_t dr = tid >> 2, dn0 = 16u * (tid & 3u);
  uint64_t reached = 0, sumd = 0, h = 0;
  if (a.digest && dr < nr) {
    for (uint32_t n = dn0; n < dn0 + 16u && n < nv; ++n) {
      const uint32_t l = s_lev[n * 64u + dr];
      if (!l) continue;
      reached += 1;
      sumd += l - 1u;
      h += s_dk[2u * n] * (uint64_t)l;
    }
  }
  const uint32_t pn = tid >> 2, pq = tid & 3u;  // node, 8-root group of the half
  const uint32_t span = nv * W;                 // words of one root's slice
  const bool vw = (((size_t)V * W) & 3u) == 0 && ((v0 * W) & 3u) == 0 && (span & 3u) == 0;
  for (uint32_t h0 = 0; h0 < nr; h0 += 32u) {
    for (uint32_t gp = 0; gp < W; ++gp) {
      uint64_t p[KP];
      const bool have = gp < np && pn < nv;
      if (have) {
        load_planes<KP>(a.planes + (size_t)slot(bl * np + gp) * V * KP, v0 + pn, p);
      }
#pragma unroll
      for (uint32_t i = 0; i < 8u; ++i) {
        const uint32_t rr = 8u * pq + i, r = h0 + rr;
        if (pn >= nv || r >= nr) continue;
        const uint32_t word = (have && s_lev[pn * 64u + r]) ? gather_word<KP>(p, r) : 0u;
        s_row[(rr * 64u + pn) * W + gp] = word;
      }
    }
    __syncthreads();
    if (a.nh) {  // each root's nv * W words: contiguous in its row
      const uint32_t nrh = min(32u, nr - h0);
      if (vw) {
        const uint32_t q4 = span / 4u;
        for (uint32_t i = tid; i < nrh * q4; i += kBlock) {
          const uint32_t rr = i / q4, k = i - rr * q4;
          const uint32_t* src = &s_row[rr * 64u * W + 4u * k];
          uint32_t* dst = a.nh + ((size_t)(rix0 + h0 + rr) * V + v0) * W + 4u * k;
          *reinterpret_cast<uint4*>(dst) = make_uint4(src[0], src[1], src[2], src[3]);
        }
      } else {
        for (uint32_t i = tid; i < nrh * span; i += kBlock) {
          const uint32_t rr = i / span, k = i - rr * span;
          a.nh[((size_t)(rix0 + h0 + rr) * V + v0) * W + k] = s_row[rr * 64u * W + k];
        }
      }
    }
    if (a.digest && dr >= h0 && dr < min(nr, h0 + 32u)) {
      for (uint32_t n = dn0; n < dn0 + 16u && n < nv; ++n)
        for (uint32_t gp = 0; gp < W; ++gp) {
          const uint32_t word = s_row[((dr - h0) * 64u + n) * W + gp];
          if (word) h += s_dk[2u * n + 1u] * digest_word_key(gp, word);
        }
    }
    __syncthreads();
  }
  if (a.digest) {
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) {
      reached += shfl_xor64(reached, o);
      sumd += shfl_xor64(sumd, o);
      h += shfl_xor64(h, o);
    }
    if ((tid & 3u) == 0 && dr < nr) {
      ospf_digest* dg = a.digest + rix0 + dr;
      if (reached) {
        atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)reached);
        atomicAdd((unsigned long long*)&dg->sum_dist, (unsigned long long)sumd);
      }
      if (h) atomicAdd((unsigned long long*)&dg->hash, (unsigned long long)h);
    }
  }
}

// ---------------------------------------------------------------- derive
// All-sources next hops from neighbour levels (unit metric / hop count).
// Phase 1 (distances only, KP = -1): msbfs_levrows writes each batch's levels
// as byte rows lev[run][node] = dist + 1 (0 = unreached) and the dist rows.
// Phase 2 (nh_derive): the next hops of root r towards v are the distinct
// neighbours n_k of r with an up link r-n_k, n_k transit or n_k == v, and
// dist(n_k, v) = dist(r, v) - 1 -- exactly the reference's nextHops
// (LinkState.cpp:885-901: a next hop n lies on a shortest r -> v path, whose
// tail from n is a shortest n -> v path with transit intermediates, and
// whose length is 1 + dist(n, v)). No bit-planes, one traversal per 64 roots
// whatever their width, and the next-hop words are written once, whole.
__device__ __forceinline__ uint32_t byte_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}
// 0x01 in byte i for bit i of a nibble
__device__ __forceinline__ uint32_t nib_bytes(uint32_t nib) {
  return (nib * 0x00204081u) & 0x01010101u;
}
// one step of a transposing wave reduction: N values per lane, lanes paired
// across offset o; afterwards value i (< N/2) of a lane is the pair's sum of
// value i + (lane & o ? N/2 : 0)
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

__global__ void __launch_bounds__(256) msbfs_levrows_kernel(DevGraph g, MsArgs a) {
  // Block = (virtual batch, 512 nodes in two 256-node halves). Load: thread
  // (quad q = tid % 64, root group rg = tid / 64: roots 16 rg .. 16 rg + 15)
  // reads the 16-root slices of its four nodes' [node][root] records (bytes
  // of roots not in seen[v] are stale: masked), transposes the 4 x 4 byte
  // blocks with byte permutes and parks [root][quad] words (four nodes of one
  // root) in LDS (row pitch 65 words: conflict-free both ways). Store: wave w
  // takes roots 16 w .. 16 w + 15, lane = quad, so each store instruction
  // writes 1 KB of consecutive dist row and 256 B of level row.
  __shared__ uint32_t s_T[64 * 65];
  const uint32_t vbl = blockIdx.x % a.nb;
  const VB b(a, vbl, g.V, -1);
  const uint32_t V = g.V, tid = threadIdx.x, q = tid & 63u, rg = tid >> 6;
  const uint32_t vb0 = (blockIdx.x / a.nb) * 512u;
  if (vb0 == 0 && tid == 0 && a.found[vbl * a.lmax + a.dbound + 1]) atomicOr(a.err, 8u);
  const uint32_t nr = min(a.R, a.n - b.rix0);
  uint32_t pk[16];        // per root of this wave: reached | sum dist << 16
  uint64_t hh[16];        // per root: sum dist_key * (dist + 1)
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
          r4 = *reinterpret_cast<const uint4*>(a.lev + ((size_t)vbl * V + v) * 64u + 16u * rg);
          sn = (uint32_t)(b.seen[v] >> (16u * rg)) & 0xFFFFu;
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
            reinterpret_cast<uint32_t*>(a.levrow + (size_t)(b.rix0 + r) * a.lev_pitch + vq));
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
        uint32_t* row = a.dist + (size_t)(b.rix0 + r) * V + vq;
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
    uint64_t h = hh[0];
#pragma unroll
    for (int o = 2; o > 0; o >>= 1) {
      p += (uint32_t)__shfl_xor((int)p, o);
      h += shfl_xor64(h, o);
    }
    const uint32_t r = 16u * rg + ((q >> 5) & 1u) * 8u + ((q >> 4) & 1u) * 4u +
                       ((q >> 3) & 1u) * 2u + ((q >> 2) & 1u);
    if ((q & 3u) == 0 && r < nr && (p & 0xFFFFu)) {
      ospf_digest* dg = a.digest + b.rix0 + r;
      atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)(p & 0xFFFFu));
      atomicAdd((unsigned long long*)&dg->sum_dist, (unsigned long long)(p >> 16));
      atomicAdd((unsigned long long*)&dg->hash, (unsigned long long)h);
    }
  }
}

// Phase 2: block = (group of G roots, chunk of C node tiles); a tile is
// T = 1024 / S nodes, S threads per node quad splitting a root's next-hop
// words. The group's neighbour tables (level row per usable transit
// neighbour) are staged once per block; per tile, the group's own level bytes
// and the node keys are staged once and reused by every root. A neighbour
// row read is one 4-B load of four level bytes, compared with the root's own
// four (minus one) by a SWAR zero-byte test; eight neighbours' flags gather
// in one register per quad before they are spread into the four words.
// A non-transit neighbour n is a next hop only towards n itself (dist 1 from
// the root over the up link): its bit is set directly, its row never read.
constexpr uint32_t kDeriveTab = 2048;  // LDS neighbour slots of a block's group
constexpr uint32_t kDeriveMaxG = 16;
template <int S>
__global__ void __launch_bounds__(256) nh_derive_kernel(DevGraph g, DeriveArgs d) {
  constexpr uint32_t T = 1024u / S;
  // [G][cap] per neighbour slot: its level row; 0x80000000 | id for a
  // non-transit usable neighbour; kInf: no up link (skip)
  __shared__ uint32_t s_pos[kDeriveTab];
  __shared__ uint32_t s_K[kDeriveMaxG], s_root[kDeriveMaxG], s_own[kDeriveMaxG];
  __shared__ uint32_t s_L[kDeriveMaxG * T / 4];  // own level bytes, [G][T] packed by quads
  __shared__ uint64_t s_kn[T];
  __shared__ unsigned long long s_h[kDeriveMaxG];
  extern __shared__ uint32_t s_out[];  // [T][W]
  const uint32_t V = g.V, W = d.W, tid = threadIdx.x, G = d.G, cap = d.cap;
  // chunk-major: the blocks in flight cover one node chunk for many groups,
  // so neighbour rows shared by several roots are read while in L2 / MALL;
  // within a chunk, runs of consecutive groups (similar neighbourhoods in a
  // locality-ordered root list) go to one XCD (workgroup b runs on XCD b % 8)
  const uint32_t ngroups = (d.n + G - 1) / G;
  const uint32_t ci = blockIdx.x / ngroups, rr = blockIdx.x % ngroups;
  const uint32_t full = ngroups / 8u * 8u;
  const uint32_t gi = rr < full ? (rr % 8u) * (full / 8u) + rr / 8u : rr;
  const uint32_t i0 = gi * G, ng = min(G, d.n - i0);
  // ---- neighbour tables of the group
  if (tid < ng) {
    const uint32_t r = d.roots[i0 + tid];
    s_root[tid] = r;
    s_h[tid] = 0ull;
    s_own[tid] = kInf;
    s_K[tid] = 0;
    if (r >= V) {
      atomicOr(d.err, 64u);
    } else {
      const uint32_t K = g.dn_off[r + 1] - g.dn_off[r];
      s_own[tid] = d.pos[r];
      if (K > cap || K > 32u * W || s_own[tid] == kInf)
        atomicOr(d.err, s_own[tid] == kInf ? 16u : 1u);
      if (s_own[tid] != kInf) s_K[tid] = min(K, cap);
    }
  }
  for (uint32_t x = tid; x < ng * cap; x += kBlock) s_pos[x] = kInf;
  __syncthreads();
  for (uint32_t j = 0; j < ng; ++j) {  // mark usable neighbours (an up link) per root
    const uint32_t r = s_root[j];
    if (r >= V) continue;
    for (uint32_t e = g.row_ptr[r] + tid; e < g.row_ptr[r + 1]; e += kBlock) {
      const uint32_t cx = g.colx[e];
      if ((cx & kDown) || cx == r) continue;
      const uint32_t k = g.didx[e];
      if (k < s_K[j]) s_pos[j * cap + k] = 0u;  // benign race: same value
    }
  }
  __syncthreads();
  for (uint32_t x = tid; x < ng * cap; x += kBlock) {
    const uint32_t j = x / cap, k = x - j * cap;
    if (k >= s_K[j] || s_pos[x] == kInf) continue;
    const uint32_t n = g.dn[g.dn_off[s_root[j]] + k];
    const uint32_t p = d.pos[n];
    if (transit(g, n)) {
      s_pos[x] = p;
      if (p == kInf) atomicOr(d.err, 16u);
    } else {
      s_pos[x] = 0x80000000u | n;  // next hop towards itself only
    }
  }
  __syncthreads();
  // ---- tiles
  const uint32_t q = tid / S, sub = tid % S, n0 = 4u * q;
  const uint32_t t0 = ci * d.ctiles, t1 = min(d.tiles, t0 + d.ctiles);
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t v0 = t * T, nv = min(T, V - v0);
    const bool vec = nv == T;  // rows are pitch-aligned (16 B): whole words
    for (uint32_t x = tid; x < ng * (T / 4u); x += kBlock) {
      const uint32_t j = x / (T / 4u), qq = x - j * (T / 4u);
      uint32_t w4 = 0;
      if (s_own[j] != kInf) {
        const uint8_t* orow = d.lev + (size_t)s_own[j] * d.pitch + v0 + 4u * qq;
        if (vec) {
          w4 = *reinterpret_cast<const uint32_t*>(orow);
        } else {
          for (uint32_t b = 0; b < 4u; ++b)
            if (4u * qq + b < nv) w4 |= (uint32_t)orow[b] << (8 * b);
        }
      }
      s_L[x] = w4;
    }
    if (d.digest)
      for (uint32_t n = tid; n < T; n += kBlock) s_kn[n] = n < nv ? g.dkey[2ull * (v0 + n) + 1] : 0ull;
    __syncthreads();
    for (uint32_t j = 0; j < ng; ++j) {
      const uint32_t K = s_K[j];
      const uint32_t L4 = s_L[j * (T / 4u) + q];
      // per byte: L - 1 where 2 <= L < 0x7F (reached, not the root), else
      // 0xFF (matches no level byte)
      uint32_t lm1 = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t l = (L4 >> (8 * b)) & 0xFFu;
        lm1 |= (l >= 2u && l < 0x7Fu ? l - 1u : 0xFFu) << (8 * b);
      }
      const uint32_t* tab = s_pos + j * cap;
      for (uint32_t w = sub; w < W; w += S) {
        uint32_t word[4] = {0u, 0u, 0u, 0u};
        const uint32_t k0 = 32u * w;
        if (lm1 != 0xFFFFFFFFu && k0 < K) {
          for (uint32_t k8 = 0; k8 < 32u; k8 += 8u) {
            const uint32_t kb = k0 + k8;
            if (kb >= K) break;
            uint32_t A = 0;
#pragma unroll
            for (uint32_t kk = 0; kk < 8u; ++kk) {
              const uint32_t p = (kb + kk < K) ? tab[kb + kk] : kInf;
              if (p >= 0x80000000u) {
                const uint32_t b = (p & 0x7FFFFFFFu) - (v0 + n0);
                if (p != kInf && b < 4u) A |= 1u << (8u * b + kk);
                continue;
              }
              const uint8_t* nrow = d.lev + (size_t)p * d.pitch + v0 + n0;
              uint32_t x4;
              if (vec) {
                x4 = *reinterpret_cast<const uint32_t*>(nrow);
              } else {
                x4 = 0;
                for (uint32_t b = 0; b < 4u; ++b)
                  if (n0 + b < nv) x4 |= (uint32_t)nrow[b] << (8 * b);
              }
              const uint32_t df = x4 ^ lm1;  // zero byte: level == L - 1
              const uint32_t z = ~(((df & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | df | 0x7F7F7F7Fu);
              A |= (z >> 7) << kk;  // byte b, bit kk
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) word[b] |= ((A >> (8 * b)) & 0xFFu) << k8;
          }
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) s_out[(n0 + b) * W + w] = word[b];
      }
      __syncthreads();
      const uint32_t i = i0 + j, span = nv * W;
      uint32_t* dst = d.nh + ((size_t)i * V + v0) * W;
      if (vec && (((size_t)i * V + v0) * W & 3u) == 0 && (span & 3u) == 0) {
        for (uint32_t x = tid; x < span / 4u; x += kBlock)
          reinterpret_cast<uint4*>(dst)[x] = reinterpret_cast<const uint4*>(s_out)[x];
      } else {
        for (uint32_t x = tid; x < span; x += kBlock) dst[x] = s_out[x];
      }
      if (d.digest) {
        uint64_t h = 0;
        for (uint32_t n = tid; n < nv; n += kBlock) {
          uint64_t ws = 0;
          for (uint32_t w = 0; w < W; ++w) {
            const uint32_t word = s_out[n * W + w];
            if (word) ws += digest_word_key(w, word);
          }
          h += s_kn[n] * ws;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) h += shfl_xor64(h, o);
        if ((tid & 63u) == 0 && h) atomicAdd(&s_h[j], (unsigned long long)h);
      }
      __syncthreads();  // s_out is rewritten by the next root
    }
  }
  if (d.digest && tid < ng) {
    const uint32_t i = i0 + tid;
    ospf_digest* dg = d.digest + i;
    unsigned long long h = s_h[tid];
    if (ci == 0) {  // the distance part from phase 1, once per root
      const uint32_t p = s_own[tid];
      if (p != kInf) {
        const ospf_digest ld = d.lev_digest[p];
        atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)ld.reached);
        atomicAdd((unsigned long long*)&dg->sum_dist, (unsigned long long)ld.sum_dist);
        h += ld.hash;
      }
    }
    if (h) atomicAdd((unsigned long long*)&dg->hash, h);
  }
}

// Narrow rows (W <= 4 words): a wave per (root, 1,024-node tile), each lane
// 16 consecutive nodes: one 16-B load per neighbour row per lane (a wave reads
// 1 KB of a row at once), SWAR compares on four words, the W words of the
// lane's 16 nodes in registers, stored as the lane's contiguous 64 W bytes.
// Block = group of G roots x chunk of tiles (chunk-major, XCD-grouped, as in
// nh_derive_kernel); its 4 waves take (tile, root) pairs.
// Uniform group (every root of the block's group has the same <= KM
// neighbour slots): each tile's neighbour rows are loaded once into registers
// and compared against every root's own levels in turn. KM is a compile-time
// bound (slots k >= K are masked, never branched on), so the register arrays
// stay in registers.
template <int KM>
__device__ __forceinline__ void derive_uniform_tiles(
    const DevGraph& g, const DeriveArgs& d, uint32_t t0, uint32_t t1, uint32_t ng, uint32_t i0,
    const uint32_t* s_pos, const uint32_t* s_own, uint32_t K, uint32_t* s_stage,
    const uint64_t* s_wk, unsigned long long* s_h, bool small, uint32_t lane, uint32_t wave) {
  const uint32_t V = g.V;
  for (uint32_t t = t0 + wave; t < t1; t += kWavesPerBlock) {
    const uint32_t vl = t * 1024u + 16u * lane;
    const bool live = vl < d.pitch;
    const uint32_t vs = live ? vl : 0u;
    uint4 xv[KM];
    uint32_t pp[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      pp[k] = (uint32_t)k < K ? s_pos[k] : kInf;
      const uint32_t row = pp[k] < 0x80000000u ? pp[k] : s_own[0];
      xv[k] = *reinterpret_cast<const uint4*>(d.lev + (size_t)row * d.pitch + vs);
    }
    uint64_t kn[16];
    if (d.digest) {
      const uint4* kp = reinterpret_cast<const uint4*>(g.dkn + vs);
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        const uint4 k2 = kp[x];
        kn[2 * x] = ((uint64_t)k2.y << 32) | k2.x;
        kn[2 * x + 1] = ((uint64_t)k2.w << 32) | k2.z;
      }
    }
    uint32_t* st = s_stage + wave * 1024u;
    const uint32_t tv0 = t * 1024u, tn = min(1024u, V - tv0);
    // The roots of a uniform group share their neighbour rows, so a root whose
    // own level bytes over the wave's 1,024 nodes equal the previous root's
    // has the same words there (the racks of a pod, everywhere outside their
    // pod): the staged words and the wave's digest sum are reused and only the
    // stores are issued again.
    uint4 Lp = make_uint4(kInf, kInf, kInf, kInf);  // level bytes are < 0x80
    uint64_t hw = 0;  // the previous root's wave digest sum of this tile
    uint4 sv[4];      // this lane's four staged store pieces (kept across reused roots)
    // the next root's own levels are loaded while this root's words are
    // stored (one load in flight across the loop)
    uint4 Ln = make_uint4(0, 0, 0, 0);
    if (live) Ln = *reinterpret_cast<const uint4*>(d.lev + (size_t)s_own[0] * d.pitch + vl);
    for (uint32_t j = 0; j < ng; ++j) {
      const uint4 L = Ln;
      if (live && j + 1 < ng)
        Ln = *reinterpret_cast<const uint4*>(d.lev + (size_t)s_own[j + 1] * d.pitch + vl);
      const bool same = L.x == Lp.x && L.y == Lp.y && L.z == Lp.z && L.w == Lp.w;
      Lp = L;
      if (__ballot(!same)) {  // some lane's levels differ: recompute the wave's words
      const uint32_t Lw[4] = {L.x, L.y, L.z, L.w};
      uint32_t lm1[4];  // as in nh_derive16_kernel: ((L - 1) | 0x80) per byte
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t l = (Lw[q] >> (8 * b)) & 0xFFu;
          m |= (l >= 2u && l < 0x7Fu ? l - 1u : 0u) << (8 * b);
        }
        lm1[q] = m | 0x80808080u;
      }
      uint32_t A0[4] = {0u, 0u, 0u, 0u}, A1[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const uint32_t keep = (pp[k] < 0x80000000u && live) ? 0xFFFFFFFFu : 0u;
        const uint32_t xw[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
        uint32_t zz[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) zz[q] = ((lm1[q] - xw[q]) & 0x80808080u & keep) >> 7;
        const uint32_t off = (pp[k] & 0x7FFFFFFFu) - vl;
        if (pp[k] >= 0x80000000u && pp[k] != kInf && off < 16u) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if ((off >> 2) == (uint32_t)q) zz[q] |= 1u << (8u * (off & 3u));
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (k < 8) A0[q] |= zz[q] << k;
          else A1[q] |= zz[q] << (k - 8);
        }
      }
      uint32_t word[16];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          word[4 * q + b] = ((A0[q] >> (8 * b)) & 0xFFu) | (((A1[q] >> (8 * b)) & 0xFFu) << 8);
      __builtin_amdgcn_wave_barrier();  // the previous root's stores have read the slice
#pragma unroll
      for (int x = 0; x < 4; ++x)
        reinterpret_cast<uint4*>(st + 16u * lane)[x] =
            make_uint4(word[4 * x], word[4 * x + 1], word[4 * x + 2], word[4 * x + 3]);
      __builtin_amdgcn_wave_barrier();
      hw = 0;
      if (d.digest) {
        if (live) {
#pragma unroll
          for (int n = 0; n < 16; ++n) {
            const uint32_t wd = word[n];
            const uint64_t ws = small ? s_wk[wd & 0xFFu] : (wd ? digest_word_key(0, wd) : 0ull);
            hw += kn[n] * ws;
          }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) hw += shfl_xor64(hw, o);
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) sv[x] = reinterpret_cast<const uint4*>(st)[x * 64 + lane];
      }  // recomputed
      const size_t i = i0 + j;
      uint32_t* dst = d.nh + (size_t)i * V + tv0;
      if (tn == 1024u && (((size_t)i * V + tv0) & 3u) == 0) {
#pragma unroll
        for (int x = 0; x < 4; ++x)
          store_row16(reinterpret_cast<uint4*>(dst) + x * 64 + lane, sv[x]);
      } else {
        for (uint32_t x = lane; x < tn; x += 64u) dst[x] = st[x];
      }
      if (lane == 0 && hw) atomicAdd(&s_h[j], (unsigned long long)hw);
    }
  }
}

template <int W>
__global__ void __launch_bounds__(256) nh_derive16_kernel(DevGraph g, DeriveArgs d) {
  __shared__ uint32_t s_pos[kDeriveTab];
  __shared__ uint32_t s_K[kDeriveMaxG], s_root[kDeriveMaxG], s_own[kDeriveMaxG];
  __shared__ unsigned long long s_h[kDeriveMaxG];
  extern __shared__ uint32_t s_stage[];  // [4 waves][1024 nodes][W]
  const uint32_t V = g.V, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t G = d.G, cap = d.cap;
  const uint32_t ngroups = (d.n + G - 1) / G;
  const uint32_t ci = blockIdx.x / ngroups, rr = blockIdx.x % ngroups;
  const uint32_t full = ngroups / 8u * 8u;
  const uint32_t gi = rr < full ? (rr % 8u) * (full / 8u) + rr / 8u : rr;
  const uint32_t i0 = gi * G, ng = min(G, d.n - i0);
  if (tid < ng) {
    const uint32_t r = d.roots[i0 + tid];
    s_root[tid] = r;
    s_h[tid] = 0ull;
    s_own[tid] = kInf;
    s_K[tid] = 0;
    if (r >= V) {
      atomicOr(d.err, 64u);
    } else {
      const uint32_t K = g.dn_off[r + 1] - g.dn_off[r];
      s_own[tid] = d.pos[r];
      if (K > cap || K > 32u * W || s_own[tid] == kInf)
        atomicOr(d.err, s_own[tid] == kInf ? 16u : 1u);
      if (s_own[tid] != kInf) s_K[tid] = min(K, cap);
    }
  }
  for (uint32_t x = tid; x < ng * cap; x += kBlock) s_pos[x] = kInf;
  __syncthreads();
  for (uint32_t j = 0; j < ng; ++j) {
    const uint32_t r = s_root[j];
    if (r >= V) continue;
    for (uint32_t e = g.row_ptr[r] + tid; e < g.row_ptr[r + 1]; e += kBlock) {
      const uint32_t cx = g.colx[e];
      if ((cx & kDown) || cx == r) continue;
      const uint32_t k = g.didx[e];
      if (k < s_K[j]) s_pos[j * cap + k] = 0u;
    }
  }
  __syncthreads();
  for (uint32_t x = tid; x < ng * cap; x += kBlock) {
    const uint32_t j = x / cap, k = x - j * cap;
    if (k >= s_K[j] || s_pos[x] == kInf) continue;
    const uint32_t n = g.dn[g.dn_off[s_root[j]] + k];
    const uint32_t p = d.pos[n];
    if (transit(g, n)) {
      s_pos[x] = p;
      if (p == kInf) atomicOr(d.err, 16u);
    } else {
      s_pos[x] = 0x80000000u | n;
    }
  }
  // a uniform group (every root with the same <= 8 neighbour slots: the
  // racks of one pod) loads each tile's neighbour rows once for all its roots;
  // one-word rows of <= 8 neighbours hash their words through a 256-entry table
  __shared__ uint32_t s_uni;
  __shared__ uint64_t s_wk[256];
  if (tid == 0) s_uni = (W == 1 && ng > 1 && s_K[0] <= 8u && s_own[0] != kInf) ? 1u : 0u;
  const bool small = W == 1 && cap <= 8u;
  if (small && d.digest) s_wk[tid] = tid ? digest_word_key(0, tid) : 0ull;
  __syncthreads();
  if (s_uni) {
    for (uint32_t x = tid; x < ng * cap; x += kBlock) {
      const uint32_t j = x / cap, k = x - j * cap;
      if (j && (s_K[j] != s_K[0] || s_own[j] == kInf || (k < s_K[0] && s_pos[x] != s_pos[k])))
        s_uni = 0u;  // benign race: every writer stores 0
    }
  }
  __syncthreads();
  const uint32_t t0 = ci * d.ctiles, t1 = min(d.tiles, t0 + d.ctiles), nt = t1 - t0;
  if (s_uni) {
    if constexpr (W == 1) {
      derive_uniform_tiles<8>(g, d, t0, t1, ng, i0, s_pos, s_own, s_K[0], s_stage, s_wk, s_h,
                              small, lane, wave);
    }
  } else
  for (uint32_t pr = wave; pr < nt * ng; pr += kWavesPerBlock) {
    const uint32_t t = t0 + pr / ng, j = pr % ng;
    const uint32_t own = s_own[j], K = s_K[j];
    if (own == kInf) continue;
    const uint32_t vl = t * 1024u + 16u * lane;  // this lane's first node
    const bool live = vl < d.pitch;             // inside the (16-aligned) rows
    uint4 L = make_uint4(0, 0, 0, 0);
    if (live) L = *reinterpret_cast<const uint4*>(d.lev + (size_t)own * d.pitch + vl);
    // per byte (L - 1) | 0x80 where 2 <= L < 0x7F, else 0x80. For a transit
    // neighbour with an up link, x >= L - 1 whenever x is reached (< 0x7F), so
    // x == L - 1 <=> L - 1 >= x: bit 7 of ((L - 1) | 0x80) - x, no borrow
    // between bytes (x in 1 .. 0x7F)
    uint32_t lm1[4];
    {
      const uint32_t Lw[4] = {L.x, L.y, L.z, L.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t l = (Lw[q] >> (8 * b)) & 0xFFu;
          m |= (l >= 2u && l < 0x7Fu ? l - 1u : 0u) << (8 * b);
        }
        lm1[q] = m | 0x80808080u;
      }
    }
    uint32_t word[W][16];
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int n = 0; n < 16; ++n) word[w][n] = 0u;
    const uint32_t* tab = s_pos + j * cap;
    const uint32_t vs = live ? vl : 0u;  // a valid address for lanes past the rows
#pragma unroll
    for (int w = 0; w < W; ++w) {
#pragma unroll
      for (int k8 = 0; k8 < 32; k8 += 8) {
        const uint32_t kb = 32u * w + k8;
        if (kb >= K) break;
        // branch-free: 8 table entries, then 8 loads in flight (skipped /
        // non-transit entries load the own row and are masked out)
        uint32_t pp[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) pp[kk] = (kb + kk < K) ? tab[kb + kk] : kInf;
        uint4 xv[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const uint32_t row = pp[kk] < 0x80000000u ? pp[kk] : own;
          xv[kk] = *reinterpret_cast<const uint4*>(d.lev + (size_t)row * d.pitch + vs);
        }
        uint32_t A[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const uint32_t keep = (pp[kk] < 0x80000000u && live) ? 0xFFFFFFFFu : 0u;
          const uint32_t xw[4] = {xv[kk].x, xv[kk].y, xv[kk].z, xv[kk].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t z = (lm1[q] - xw[q]) & 0x80808080u & keep;
            A[q] |= (z >> 7) << kk;
          }
          // a non-transit neighbour: a next hop towards itself only
          const uint32_t off = (pp[kk] & 0x7FFFFFFFu) - vl;
          if (pp[kk] >= 0x80000000u && pp[kk] != kInf && off < 16u)
            A[off >> 2] |= 1u << (8u * (off & 3u) + kk);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int b = 0; b < 4; ++b) word[w][4 * q + b] |= ((A[q] >> (8 * b)) & 0xFFu) << k8;
      }
    }
    // the tile's 1,024 nodes x W words are contiguous in the root's row:
    // staged through this wave's LDS slice so each store instruction writes
    // 1 KB of consecutive row (per-lane 64 W-byte runs would leave partial
    // lines: 5.6x the row bytes written at W = 3, measured)
    uint32_t* st = s_stage + wave * 1024u * W;
#pragma unroll
    for (int x = 0; x < 4 * W; ++x) {
      uint32_t v4[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 4 * x + c;  // flat index node * W + word within the lane
        v4[c] = word[f % W][f / W];
      }
      reinterpret_cast<uint4*>(st + 16u * W * lane)[x] = make_uint4(v4[0], v4[1], v4[2], v4[3]);
    }
    __builtin_amdgcn_wave_barrier();  // LDS ops of a wave complete in order
    const size_t i = i0 + j;
    const uint32_t tv0 = t * 1024u, tn = min(1024u, V - tv0);
    uint32_t* dst = d.nh + ((size_t)i * V + tv0) * W;
    if (tn == 1024u && ((((size_t)i * V + tv0) * W) & 3u) == 0) {
#pragma unroll
      for (int x = 0; x < 4 * W; ++x)
        store_row16(reinterpret_cast<uint4*>(dst) + x * 64 + lane,
                    reinterpret_cast<const uint4*>(st)[x * 64 + lane]);
    } else {
      for (uint32_t x = lane; x < tn * W; x += 64u) dst[x] = st[x];
    }
    __builtin_amdgcn_wave_barrier();  // the slice is rewritten by the next pair
    if (d.digest) {
      uint64_t h = 0;
      if (live) {
      uint64_t kn[16];
      const uint4* kp = reinterpret_cast<const uint4*>(g.dkn + vl);  // zero past V
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        const uint4 k2 = kp[x];
        kn[2 * x] = ((uint64_t)k2.y << 32) | k2.x;
        kn[2 * x + 1] = ((uint64_t)k2.w << 32) | k2.z;
      }
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        uint64_t ws = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          if (small) ws += s_wk[word[w][n] & 0xFFu];
          else if (word[w][n]) ws += digest_word_key(w, word[w][n]);
        }
        h += kn[n] * ws;
      }
      }  // live
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) h += shfl_xor64(h, o);  // every lane of the wave
      if (lane == 0 && h) atomicAdd(&s_h[j], (unsigned long long)h);
    }
  }
  __syncthreads();
  if (d.digest && tid < ng) {
    ospf_digest* dg = d.digest + i0 + tid;
    unsigned long long h = s_h[tid];
    if (ci == 0 && s_own[tid] != kInf) {
      const ospf_digest ld = d.lev_digest[s_own[tid]];
      atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)ld.reached);
      atomicAdd((unsigned long long*)&dg->sum_dist, (unsigned long long)ld.sum_dist);
      h += ld.hash;
    }
    if (h) atomicAdd((unsigned long long*)&dg->hash, h);
  }
}

// Wide rows (W > 4 words: spines, whose neighbours are one switch per pod).
// Lane = next-hop word w (its 32 neighbour slots), a wave walks 8-node chunks
// of the block's tile. Block = up to kWideG consecutive roots x a chunk of
// tiles; inside it, runs of roots with the same distinct-neighbour list (the
// spines of one plane) share the neighbour loads: each lane reads its 32
// slots' level bytes of 8 nodes once per chunk, and the word of 8 nodes is
// recomputed only when a root's own levels differ from the previous root's
// (all spines of a plane are equally far from nearly every node). Per root
// only the link-up mask, the stores (W consecutive words = one node's record
// per store instruction) and the digest terms remain.
constexpr uint32_t kWideG = 64;
constexpr uint32_t kWideTile = 256;
__global__ void __launch_bounds__(256) nh_derive_wide_kernel(DevGraph g, DeriveArgs d) {
  __shared__ uint32_t s_pos[kDeriveTab];           // slot table of the current run
  __shared__ uint32_t s_keep[kWideG * 64];         // [root][word]: slots with an up link
  __shared__ uint32_t s_L[kWideG * kWideTile / 4];  // own level bytes of the tile, [root][node]
  __shared__ uint32_t s_root[kWideG], s_own[kWideG], s_K[kWideG], s_same[kWideG];
  __shared__ unsigned long long s_h[kWideG];
  const uint32_t V = g.V, W = d.W, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t G = d.G, cap = d.cap;
  const uint32_t ngroups = (d.n + G - 1) / G;
  const uint32_t ci = blockIdx.x / ngroups, rr = blockIdx.x % ngroups;
  const uint32_t full = ngroups / 8u * 8u;
  const uint32_t gi = rr < full ? (rr % 8u) * (full / 8u) + rr / 8u : rr;
  const uint32_t i0 = gi * G, ng = min(G, d.n - i0);
  if (tid < ng) {
    const uint32_t r = d.roots[i0 + tid];
    s_root[tid] = r;
    s_h[tid] = 0ull;
    s_own[tid] = kInf;
    s_K[tid] = 0;
    if (r >= V) {
      atomicOr(d.err, 64u);
    } else {
      const uint32_t K = g.dn_off[r + 1] - g.dn_off[r];
      s_own[tid] = d.pos[r];
      if (K > cap || K > 32u * W || s_own[tid] == kInf)
        atomicOr(d.err, s_own[tid] == kInf ? 16u : 1u);
      if (s_own[tid] != kInf) s_K[tid] = min(K, cap);
    }
  }
  for (uint32_t x = tid; x < ng * 64u; x += kBlock) s_keep[x] = 0u;
  __syncthreads();
  // usable slots per root; s_same[j]: root j has root j-1's neighbour list
  if (tid < ng)
    s_same[tid] = tid > 0 && s_own[tid] != kInf && s_own[tid - 1] != kInf &&
                  s_K[tid] == s_K[tid - 1];
  for (uint32_t j = 0; j < ng; ++j) {
    const uint32_t r = s_root[j];
    if (r >= V || s_own[j] == kInf) continue;
    for (uint32_t e = g.row_ptr[r] + tid; e < g.row_ptr[r + 1]; e += kBlock) {
      const uint32_t cx = g.colx[e];
      if ((cx & kDown) || cx == r) continue;
      const uint32_t k = g.didx[e];
      if (k < s_K[j]) atomicOr(&s_keep[j * 64u + (k >> 5)], 1u << (k & 31u));
    }
  }
  __syncthreads();
  for (uint32_t j = 1; j < ng; ++j) {
    if (!s_same[j]) continue;
    const uint32_t* a0 = g.dn + g.dn_off[s_root[j - 1]];
    const uint32_t* a1 = g.dn + g.dn_off[s_root[j]];
    for (uint32_t k = tid; k < s_K[j]; k += kBlock)
      if (a0[k] != a1[k]) s_same[j] = 0u;  // benign race: every writer stores 0
  }
  __syncthreads();
  const uint32_t t0 = ci * d.ctiles, t1 = min(d.tiles, t0 + d.ctiles);
  for (uint32_t j0 = 0; j0 < ng;) {
    uint32_t j1 = j0 + 1;
    while (j1 < ng && s_same[j1]) ++j1;
    const uint32_t K = s_K[j0];
    if (s_own[j0] == kInf) {  // a bad root (error flagged): its own run
      j0 = j1;
      continue;
    }
    // slot table: the neighbour's level row; 0x80000000 | id for a non-transit
    // neighbour (a next hop towards itself only); kInf when no root of the run
    // has an up link to it
    for (uint32_t k = tid; k < K; k += kBlock) {
      bool used = false;
      for (uint32_t j = j0; j < j1 && !used; ++j) used = (s_keep[j * 64u + (k >> 5)] >> (k & 31u)) & 1u;
      uint32_t p = kInf;
      if (used) {
        const uint32_t n = g.dn[g.dn_off[s_root[j0]] + k];
        if (transit(g, n)) {
          p = d.pos[n];
          if (p == kInf) atomicOr(d.err, 16u);
        } else {
          p = 0x80000000u | n;
        }
      }
      s_pos[k] = p;
    }
    const uint32_t own0 = s_own[j0];
    for (uint32_t t = t0; t < t1; ++t) {
      const uint32_t v0 = t * kWideTile;
      __syncthreads();  // s_pos written / the previous tile's s_L consumed
      for (uint32_t x = tid; x < (j1 - j0) * (kWideTile / 16u); x += kBlock) {
        const uint32_t j = x / (kWideTile / 16u), c = x - j * (kWideTile / 16u);
        uint4 l4 = make_uint4(0x7F7F7F7Fu, 0x7F7F7F7Fu, 0x7F7F7F7Fu, 0x7F7F7F7Fu);
        if (v0 + 16u * c < d.pitch)
          l4 = *reinterpret_cast<const uint4*>(d.lev + (size_t)s_own[j0 + j] * d.pitch + v0 + 16u * c);
        reinterpret_cast<uint4*>(s_L + j * (kWideTile / 4u))[c] = l4;
      }
      __syncthreads();
      for (uint32_t c = wave; c < kWideTile / 8u; c += kWavesPerBlock) {
        const uint32_t vc = v0 + 8u * c;
        if (vc >= V) break;  // wave-uniform
        // this lane's 32 slots at the chunk's 8 nodes (vc + 8 <= pitch)
        uint2 xv[32];
        uint32_t selfw[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          const uint32_t k = 32u * lane + i;
          const uint32_t p = (lane < W && k < K) ? s_pos[k] : kInf;
          const uint32_t row = p < 0x80000000u ? p : own0;
          xv[i] = *reinterpret_cast<const uint2*>(d.lev + (size_t)row * d.pitch + vc);
          if (p >= 0x80000000u) {
            xv[i] = make_uint2(0x7F7F7F7Fu, 0x7F7F7F7Fu);  // never matches
            const uint32_t off = (p & 0x7FFFFFFFu) - vc;
            if (p != kInf && off < 8u) {
#pragma unroll
              for (int b = 0; b < 8; ++b)
                if (off == (uint32_t)b) selfw[b] |= 1u << i;
            }
          }
        }
        uint64_t kn[8];
        if (d.digest) {
#pragma unroll
          for (int b = 0; b < 8; ++b) kn[b] = g.dkn[vc + b];  // zero past V
        }
        uint32_t word[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        uint32_t plo = 0xFFFFFFFFu, phi = 0xFFFFFFFFu;  // lm1 of the last computed word set
        for (uint32_t j = j0; j < j1; ++j) {
          const uint2 L8 = reinterpret_cast<const uint2*>(s_L + (j - j0) * (kWideTile / 4u))[c];
          uint32_t lo = 0, hi = 0;  // ((L - 1) | 0x80) per byte, L - 1 := 0 outside 2 <= L < 0x7F
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const uint32_t l0 = (L8.x >> (8 * b)) & 0xFFu, l1 = (L8.y >> (8 * b)) & 0xFFu;
            lo |= (l0 >= 2u && l0 < 0x7Fu ? l0 - 1u : 0u) << (8 * b);
            hi |= (l1 >= 2u && l1 < 0x7Fu ? l1 - 1u : 0u) << (8 * b);
          }
          lo |= 0x80808080u;
          hi |= 0x80808080u;
          if (lo != plo || hi != phi) {  // wave-uniform (the root's own levels)
            plo = lo;
            phi = hi;
#pragma unroll
            for (int k8 = 0; k8 < 32; k8 += 8) {
              uint32_t A0 = 0, A1 = 0;
#pragma unroll
              for (int kk = 0; kk < 8; ++kk) {
                A0 |= (((lo - xv[k8 + kk].x) & 0x80808080u) >> 7) << kk;
                A1 |= (((hi - xv[k8 + kk].y) & 0x80808080u) >> 7) << kk;
              }
#pragma unroll
              for (int b = 0; b < 4; ++b) {
                const uint32_t m = k8 ? 0xFFFFFFFFu : 0u;  // first block overwrites
                word[b] = (word[b] & m) | (((A0 >> (8 * b)) & 0xFFu) << k8);
                word[4 + b] = (word[4 + b] & m) | (((A1 >> (8 * b)) & 0xFFu) << k8);
              }
            }
          }
          const uint32_t keep = lane < W ? s_keep[j * 64u + lane] : 0u;
          uint32_t* dst = d.nh + ((size_t)(i0 + j) * V + vc) * W + lane;
          uint64_t h = 0;
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            const uint32_t ow = (word[b] | selfw[b]) & keep;
            if (lane < W && vc + b < V) __builtin_nontemporal_store(ow, dst + (size_t)b * W);
            if (d.digest && ow) h += kn[b] * digest_word_key(lane, ow);
          }
          if (h) atomicAdd(&s_h[j], (unsigned long long)h);
        }
      }
    }
    j0 = j1;
    __syncthreads();  // s_pos is rewritten by the next run
  }
  __syncthreads();
  if (d.digest && tid < ng) {
    ospf_digest* dg = d.digest + i0 + tid;
    unsigned long long h = s_h[tid];
    if (ci == 0 && s_own[tid] != kInf) {
      const ospf_digest ld = d.lev_digest[s_own[tid]];
      atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)ld.reached);
      atomicAdd((unsigned long long*)&dg->sum_dist, (unsigned long long)ld.sum_dist);
      h += ld.hash;
    }
    if (h) atomicAdd((unsigned long long*)&dg->hash, h);
  }
}



// Wide rows, planned and tile-staged (W > 4 words: spines; the sweep's
// path). The host plans runs of roots with the same distinct-neighbour list
// (the spines of one plane, <= kWideG roots), each run's slot table (a
// neighbour's level row, 0x80000000 | node for a non-transit neighbour, kInf
// when no root of the run has an up link to it) and each root's usable-slot
// words, so a block's setup is a few coalesced loads. Block = (run, chunk of
// 16-node tiles), XCD-major over the chunks (an XCD's resident blocks hold
// consecutive tiles, so the 16-B pieces of each neighbour row's 128-B lines
// meet in its L2). Per tile the K rows' 16 level bytes are staged in LDS
// slot-major (one 16-B load per slot, all of a thread's in flight; a slot
// without a transit row holds 0xFF, a non-transit neighbour 0x01 at its own
// position: a next hop towards itself exactly when the root is one hop away);
// then wave q takes nodes 4q .. 4q + 3 of the tile, lane = next-hop word w:
// 32 LDS words per word, each byte compared with L - 1 for 4 nodes at once
// (SWAR). A root whose own levels at the 4 nodes equal the previous root's
// keeps the words (the spines of a plane differ only at their own
// positions); each root stores its 4 nodes' records (W consecutive words per
// store instruction) masked by its usable links.
constexpr uint32_t kW3Tile = 16, kW3Pitch = 20;
__global__ void __launch_bounds__(256) nh_wide_plan_kernel(DevGraph g, WidePlan d) {
  __shared__ uint32_t s_pos[kDeriveTab];  // the run's slot table
  __shared__ uint32_t s_own[kWideG];
  __shared__ unsigned long long s_h[kWideG];
  __shared__ uint4 s_rec[4][64];          // st16: a wave's 4 node records (4 W words)
  extern __shared__ uint32_t s_dyn[];     // keep [G][W], then the staged bytes [K][kW3Pitch]
  const uint32_t V = g.V, W = d.W, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t NB = d.nruns * d.chunks, NB8 = NB / 8u * 8u, bb = blockIdx.x;
  const uint32_t item = bb < NB8 ? (bb % 8u) * (NB8 / 8u) + bb / 8u : bb;
  // run-major items (an XCD's resident blocks serve one run, when there are
  // 8), and a block's tiles strided by the chunk count: the blocks of a run
  // move through the row together, so the 8 tiles whose 16-B pieces share each
  // neighbour row's 128-B lines are in flight on one XCD at once
  const uint32_t ri = item / d.chunks, ci = item % d.chunks;
  const uint32_t j0 = d.run[ri], ng = min(kWideG, d.run[ri + 1] - j0);
  const uint32_t s0 = d.soff[ri], K = min(kDeriveTab, d.soff[ri + 1] - s0);
  uint32_t* s_keep = s_dyn;
  uint8_t* B = reinterpret_cast<uint8_t*>(s_dyn + kWideG * W);
  for (uint32_t k = tid; k < K; k += kBlock) s_pos[k] = d.slots[s0 + k];
  for (uint32_t x = tid; x < ng * W; x += kBlock) s_keep[x] = d.keep[(size_t)j0 * W + x];
  if (tid < ng) {
    s_own[tid] = d.own[j0 + tid];
    s_h[tid] = 0ull;
  }
  __syncthreads();
  for (uint32_t t = ci; t < d.tiles; t += d.chunks) {
    const uint32_t v0 = t * kW3Tile;
    if (t > ci) __syncthreads();  // the previous tile's bytes are consumed
    // every slot load of the thread in flight at once (K <= 2048: <= 8 each)
    uint32_t pk[kDeriveTab / kBlock];
    uint4 xk[kDeriveTab / kBlock];
#pragma unroll
    for (uint32_t m = 0; m < kDeriveTab / kBlock; ++m) {
      const uint32_t k = tid + m * kBlock;
      pk[m] = k < K ? s_pos[k] : kInf;
    }
#pragma unroll
    for (uint32_t m = 0; m < kDeriveTab / kBlock; ++m) {
      const uint32_t row = pk[m] < 0x80000000u ? pk[m] : s_own[0];  // a valid row, masked below
      xk[m] = *reinterpret_cast<const uint4*>(d.lev + (size_t)row * d.pitch + v0);
    }
    // this wave's 4 nodes: their digest keys and every root's own levels,
    // issued with the slot loads (their latency was exposed after the barrier)
    const uint32_t nq = v0 + 4u * wave;
    uint64_t kn[4] = {0ull, 0ull, 0ull, 0ull};
    uint32_t Lmine = 0u;
    if (nq < V && !d.late_keys) {
#pragma unroll
      for (int b = 0; b < 4; ++b) kn[b] = d.digest ? g.dkn[nq + b] : 0ull;  // zero past V
      Lmine = lane < ng ? *reinterpret_cast<const uint32_t*>(d.lev + (size_t)s_own[lane] * d.pitch + nq) : 0u;
    }
#pragma unroll
    for (uint32_t m = 0; m < kDeriveTab / kBlock; ++m) {
      const uint32_t k = tid + m * kBlock, p = pk[m];
      if (k >= K) break;
      uint4 x = xk[m];
      if (p >= 0x80000000u) {
        x = make_uint4(~0u, ~0u, ~0u, ~0u);
        const uint32_t o = (p & 0x7FFFFFFFu) - v0;
        if (p != kInf && o < kW3Tile) {
          uint32_t w4[4] = {x.x, x.y, x.z, x.w};
          w4[o >> 2] = (w4[o >> 2] & ~(0xFFu << (8u * (o & 3u)))) | (1u << (8u * (o & 3u)));
          x = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
      }
      uint32_t* bw = reinterpret_cast<uint32_t*>(B + (size_t)k * kW3Pitch);
      bw[0] = x.x;
      bw[1] = x.y;
      bw[2] = x.z;
      bw[3] = x.w;
    }
    __syncthreads();
    if (nq >= V) continue;  // wave-uniform (the next barrier is reached by all)
    if (d.late_keys) {
#pragma unroll
      for (int b = 0; b < 4; ++b) kn[b] = d.digest ? g.dkn[nq + b] : 0ull;
      Lmine = lane < ng ? *reinterpret_cast<const uint32_t*>(d.lev + (size_t)s_own[lane] * d.pitch + nq) : 0u;
    }
    // (Lmine: lane j holds root j's own levels at the 4 nodes)
    // st16 (wave-uniform): the 4 records (4 W words, 7 whole 128-B lines at
    // W = 56) staged in LDS and stored as W 16-B pieces by one instruction,
    // instead of 4 stores of W words whose 128-B lines straddle them
    const bool st16 = d.st16 && (W & 3u) == 0 && nq + 4u <= V;
    uint32_t* rec = reinterpret_cast<uint32_t*>(s_rec[wave]);
    uint32_t word[4] = {0u, 0u, 0u, 0u}, Lp = 0xFFFFFFFFu;
    // the word key of each node's masked word, kept while the next root's
    // masked word is the same (the roots of a run mostly store equal words)
    uint32_t kw_word[4] = {0u, 0u, 0u, 0u};
    uint64_t kw_key[4] = {0ull, 0ull, 0ull, 0ull};
    for (uint32_t j = 0; j < ng; ++j) {
      const uint32_t L = (uint32_t)__shfl((int)Lmine, (int)j, 64);
      if (L != Lp) {  // wave-uniform: the root's own levels at the 4 nodes
        Lp = L;
        // L - 1 per byte where 2 <= L < 0x7F, else 0xFE (matches nothing)
        uint32_t lm1 = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t l = (L >> (8 * b)) & 0xFFu;
          lm1 |= (l >= 2u && l < 0x7Fu ? l - 1u : 0xFEu) << (8 * b);
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) word[b] = 0u;
        if (lane < W) {
#pragma unroll 8
          for (uint32_t i = 0; i < 32u; ++i) {
            const uint32_t k = 32u * lane + i;
            const uint32_t x = k < K ? *reinterpret_cast<const uint32_t*>(B + (size_t)k * kW3Pitch + 4u * wave)
                                     : ~0u;
            const uint32_t y = x ^ lm1;  // bit 7 of each byte of eq: that byte of y is zero
            const uint32_t eq = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
#pragma unroll
            for (int b = 0; b < 4; ++b) word[b] |= ((eq >> (8 * b + 7)) & 1u) << i;
          }
        }
      }
      const uint32_t keep = lane < W ? s_keep[j * W + lane] : 0u;
      uint32_t* dst = d.nh + ((size_t)(j0 + j) * V + nq) * W + lane;
      uint64_t h = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t ow = word[b] & keep;
        if (st16) {
          if (lane < W) rec[(size_t)b * W + lane] = ow;
        } else if (lane < W && nq + b < V) {
          __builtin_nontemporal_store(ow, dst + (size_t)b * W);
        }
        if (d.digest && ow) {
          if (ow != kw_word[b]) {
            kw_word[b] = ow;
            kw_key[b] = digest_word_key(lane, ow);
          }
          h += kn[b] * kw_key[b];
        }
      }
      if (st16) {
        __builtin_amdgcn_wave_barrier();
        if (lane < W) store_row16(reinterpret_cast<uint4*>(dst - lane) + lane, s_rec[wave][lane]);
        __builtin_amdgcn_wave_barrier();  // the records are rewritten by the next root
      }
      // few lanes hold a non-zero word: their terms go straight to the root's sum
      if (d.digest && h) atomicAdd(&s_h[j], (unsigned long long)h);
    }
  }
  __syncthreads();
  if (d.digest && tid < ng) {
    ospf_digest* dg = d.digest + j0 + tid;
    unsigned long long h = s_h[tid];
    if (ci == 0) {
      const ospf_digest ld = d.lev_digest[s_own[tid]];
      atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)ld.reached);
      atomicAdd((unsigned long long*)&dg->sum_dist, (unsigned long long)ld.sum_dist);
      h += ld.hash;
    }
    if (h) atomicAdd((unsigned long long*)&dg->hash, h);
  }
}

// ---------------------------------------------------------------- digest
// Digest of finished rows (runs whose rows are written per level): `segs`
// workgroups per root, each over a node range, adding into a zeroed record.
__global__ void __launch_bounds__(256) row_digest_kernel(DevGraph g, const uint32_t* dist,
                                                         const uint32_t* nh, uint32_t W,
                                                         uint32_t segs, ospf_digest* out) {
  const uint32_t rix = blockIdx.x / segs, seg = blockIdx.x % segs, V = g.V;
  const uint32_t* drow = dist + (size_t)rix * V;
  const uint32_t* nrow = nh + (size_t)rix * V * W;
  const uint32_t v0 = (uint32_t)((uint64_t)V / 4u * seg / segs) * 4u,
                 v1 = seg + 1 == segs ? V : (uint32_t)((uint64_t)V / 4u * (seg + 1) / segs) * 4u;
  uint64_t reached = 0, sumd = 0, h = 0;
  auto node = [&](uint32_t v, uint32_t d, uint64_t wsum) {
    if (d == kInf) return;
    const uint4 kk = reinterpret_cast<const uint4*>(g.dkey)[v];
    const uint64_t kd = ((uint64_t)kk.y << 32) | kk.x, kn = ((uint64_t)kk.w << 32) | kk.z;
    reached += 1;
    sumd += d;
    h += kd * ((uint64_t)d + 1) + kn * wsum;
  };
  auto wk = [](uint32_t w, uint32_t word) { return word ? digest_word_key(w, word) : 0ull; };
  if (W == 1 && (V & 3u) == 0) {
    // 4 nodes per lane per step (segment bounds are multiples of 4): one
    // 16-B load each of dist and next hops
    for (uint32_t v = v0 + threadIdx.x * 4u; v < v1; v += blockDim.x * 4u) {
      const uint4 d4 = *reinterpret_cast<const uint4*>(drow + v);
      const uint4 n4 = *reinterpret_cast<const uint4*>(nrow + v);
      node(v, d4.x, wk(0, n4.x));
      node(v + 1, d4.y, wk(0, n4.y));
      node(v + 2, d4.z, wk(0, n4.z));
      node(v + 3, d4.w, wk(0, n4.w));
    }
  } else {
    for (uint32_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
      uint64_t ws = 0;
      for (uint32_t w = 0; w < W; ++w) ws += wk(w, nrow[(size_t)v * W + w]);
      node(v, drow[v], ws);
    }
  }
  __shared__ uint64_t s_r[kWavesPerBlock], s_s[kWavesPerBlock], s_h[kWavesPerBlock];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    reached += shfl_xor64(reached, o);
    sumd += shfl_xor64(sumd, o);
    h += shfl_xor64(h, o);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_r[wave] = reached;
    s_s[wave] = sumd;
    s_h[wave] = h;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t r = 0, sd = 0, hh = 0;
    for (uint32_t i = 0; i < kWavesPerBlock; ++i) {
      r += s_r[i];
      sd += s_s[i];
      hh += s_h[i];
    }
    atomicAdd((unsigned long long*)&out[rix].reached, (unsigned long long)r);
    atomicAdd((unsigned long long*)&out[rix].sum_dist, (unsigned long long)sd);
    atomicAdd((unsigned long long*)&out[rix].hash, (unsigned long long)hh);
  }
}

template <int KP>
hipError_t launch_round_kp(const DevGraph& g, const MsArgs& a, uint32_t depth_bound,
                           hipStream_t s) {
  const uint32_t init_blocks = (a.nb * a.R + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(msbfs_init_kernel<KP>, dim3(init_blocks), dim3(kBlock), 0, s, g, a);
  const uint32_t chunks = (g.V + kBlock - 1) / kBlock;
  const uint32_t bigblocks = (g.nbig + kWavesPerBlock - 1) / kWavesPerBlock;
  // levels 2 .. depth_bound + 1: the last one must come out empty (a node
  // there means the host's bound was stale; the rows kernel raises bit 8)
  for (uint32_t d = 1; d <= depth_bound; ++d) {
    hipLaunchKernelGGL(msbfs_level_kernel<KP>, dim3(a.nb * (chunks + bigblocks)), dim3(kBlock), 0,
                       s, g, a, d);
    hipLaunchKernelGGL(msbfs_settle_kernel<KP>, dim3(a.nb * chunks), dim3(kBlock), 0, s, g, a, d);
  }
  if (a.defer && a.merged)
    hipLaunchKernelGGL(msbfs_rows_multi_kernel<KP>, dim3((a.nb / a.npass) * ((g.V + 63u) / 64u)),
                       dim3(kBlock), 32u * 64u * a.W * 4u, s, g, a, a.nb / a.npass);
  else if (a.defer)
    hipLaunchKernelGGL(msbfs_rows_kernel<KP>, dim3(a.nb * ((g.V + 63u) / 64u)), dim3(kBlock), 0, s,
                       g, a);
  else
    hipLaunchKernelGGL(msbfs_final_kernel, dim3(a.nb * chunks), dim3(kBlock), 0, s, g, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------- KSP2
// Ignore masks of a round's runs (every batch of 64 runs shares the source):
// pass 0 clears the mask words of the entries listed in the round, pass 1 ORs
// the run bits in and marks the entries in the batch's bitmap (the bitmap is
// zeroed with the round's state, so stale mask words are never read).
__global__ void __launch_bounds__(256) ksp_mask_kernel(DevGraph g, MsArgs a, const uint32_t* ign,
                                                       const uint32_t* cnt, uint32_t stride,
                                                       uint32_t pass) {
  const uint32_t j = blockIdx.x * (blockDim.x / 64u) + (threadIdx.x >> 6);  // run of the round
  const uint32_t vbl = j / 64u, r = j % 64u;
  if (vbl >= a.nb) return;
  const uint32_t rix = (a.vb0 + vbl) * 64u + r;
  if (rix >= a.n) return;
  const uint32_t n = min(cnt[rix], stride);
  for (uint32_t k = threadIdx.x & 63u; k < 2u * n; k += 64u) {  // one wave per run
    const uint32_t lid = ign[(size_t)rix * stride + k / 2u];
    if (lid >= g.n_lid) continue;
    const uint32_t e = g.link_e[2ull * lid + (k & 1u)];
    if (e == kInf) continue;
    uint64_t* m = a.igm + (size_t)vbl * g.E + e;
    if (pass == 0) {
      *m = 0ull;
    } else {
      or64(m, 1ull << r);
      atomicOr(&a.igb[(size_t)vbl * a.igw + (e >> 5)], 1u << (e & 31u));
    }
  }
}

// Word-major staging -> [V][W] rows: block = (root, run of nodes); the
// block's W words of each node are read word by word (coalesced along the
// nodes), transposed through LDS and stored as one contiguous span, so every
// row line is written whole, once.
constexpr uint32_t kIlvWords = 4096;  // LDS words per block (16 KB)
__global__ void __launch_bounds__(256) nh_interleave_kernel(const uint32_t* nhs, uint32_t* nh,
                                                            uint32_t V, uint32_t W, uint32_t wcomp,
                                                            uint32_t span, uint32_t runs) {
  __shared__ uint32_t s[kIlvWords];
  const uint32_t r = blockIdx.x / runs, v0 = (blockIdx.x % runs) * span;
  const uint32_t nv = min(span, V - v0), tot = nv * W;
  const uint32_t* src = nhs + (size_t)r * W * V + v0;
  for (uint32_t i = threadIdx.x; i < tot; i += kBlock) {
    const uint32_t w = i / nv, n = i - w * nv;
    s[n * W + w] = w < wcomp ? src[(size_t)w * V + n] : 0u;
  }
  __syncthreads();
  uint32_t* dst = nh + ((size_t)r * V + v0) * W;
  for (uint32_t i = threadIdx.x; i < tot; i += kBlock) dst[i] = s[i];
}

}  // namespace

hipError_t launch_nh_interleave(const uint32_t* nhs, uint32_t* nh, uint32_t n, uint32_t V,
                                uint32_t W, uint32_t wcomp, hipStream_t s) {
  if (W == 0 || W > kIlvWords / 64u) return hipErrorInvalidValue;
  const uint32_t span = std::min<uint32_t>(1024u, (kIlvWords / W) / 64u * 64u);
  const uint32_t runs = (V + span - 1) / span;
  if (n) hipLaunchKernelGGL(nh_interleave_kernel, dim3(n * runs), dim3(kBlock), 0, s, nhs, nh, V, W,
                            wcomp, span, runs);
  return hipGetLastError();
}

namespace {
// KSP2 reruns: a batch stops after level d once every run has reached its
// destination (found[d + 1] cleared: the next level kernels return at once)
__global__ void __launch_bounds__(64) ksp_done_kernel(MsArgs a, uint32_t V, uint32_t d) {
  const uint32_t vbl = blockIdx.x, r = threadIdx.x;
  if (!a.found[vbl * a.lmax + d + 1]) return;  // block-uniform
  const uint32_t run = (a.vb0 + vbl) * a.R + r;  // (npass 1)
  bool ok = true;
  if (run < a.n) {
    const uint32_t dst = a.kdst[run];
    ok = dst < V && ((a.seen[(size_t)vbl * V + dst] >> r) & 1ull);
  }
  if (__all(ok) && r == 0) a.found[vbl * a.lmax + d + 1] = 0u;
}
}  // namespace

hipError_t launch_msbfs_ksp(const DevGraph& g, const MsArgs& a, uint32_t d0, uint32_t d1,
                            hipStream_t s) {
  if (d0 <= 1) {
    const uint32_t init_blocks = (a.nb * a.R + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(msbfs_init_kernel<0>, dim3(init_blocks), dim3(kBlock), 0, s, g, a);
    d0 = 1;
  }
  const uint32_t chunks = (g.V + kBlock - 1) / kBlock;
  const uint32_t bigblocks = (g.nbig + kWavesPerBlock - 1) / kWavesPerBlock;
  for (uint32_t d = d0; d < d1; ++d) {
    hipLaunchKernelGGL(msbfs_level_kernel<0>, dim3(a.nb * (chunks + bigblocks)), dim3(kBlock), 0, s,
                       g, a, d);
    hipLaunchKernelGGL(msbfs_settle_kernel<0>, dim3(a.nb * chunks), dim3(kBlock), 0, s, g, a, d);
    if (a.kdst && a.npass == 1 && a.R == 64)
      hipLaunchKernelGGL(ksp_done_kernel, dim3(a.nb), dim3(64), 0, s, a, g.V, d);
  }
  return hipGetLastError();
}

hipError_t launch_ksp_masks(const DevGraph& g, const MsArgs& a, const uint32_t* ign,
                            const uint32_t* cnt, uint32_t stride, hipStream_t s) {
  for (uint32_t pass = 0; pass < 2; ++pass)
    hipLaunchKernelGGL(ksp_mask_kernel, dim3(a.nb * 64u / kWavesPerBlock), dim3(kBlock), 0, s, g,
                       a, ign, cnt, stride, pass);
  return hipGetLastError();
}

hipError_t launch_msbfs_round(int kp, const DevGraph& g, const MsArgs& a, uint32_t depth_bound,
                              hipStream_t s) {
  switch (kp) {
    case 8: return launch_round_kp<8>(g, a, depth_bound, s);
    case 16: return launch_round_kp<16>(g, a, depth_bound, s);
    default: return launch_round_kp<32>(g, a, depth_bound, s);
  }
}

hipError_t launch_msbfs_levels(const DevGraph& g, const MsArgs& a, uint32_t depth_bound,
                               hipStream_t s) {
  const uint32_t init_blocks = (a.nb * a.R + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(msbfs_init_kernel<-1>, dim3(init_blocks), dim3(kBlock), 0, s, g, a);
  const uint32_t chunks = (g.V + kBlock - 1) / kBlock;
  const uint32_t bigblocks = (g.nbig + kWavesPerBlock - 1) / kWavesPerBlock;
  for (uint32_t d = 1; d <= depth_bound; ++d) {
    hipLaunchKernelGGL(msbfs_level_kernel<-1>, dim3(a.nb * (chunks + bigblocks)), dim3(kBlock), 0,
                       s, g, a, d);
    hipLaunchKernelGGL(msbfs_settle_kernel<-1>, dim3(a.nb * chunks), dim3(kBlock), 0, s, g, a, d);
  }
  hipLaunchKernelGGL(msbfs_levrows_kernel, dim3(a.nb * ((g.V + 511u) / 512u)), dim3(kBlock), 0, s,
                     g, a);
  return hipGetLastError();
}

hipError_t launch_nh_derive(const DevGraph& g, const DeriveArgs& d0, hipStream_t s) {
  DeriveArgs d = d0;
  if (d.n == 0) return hipSuccess;
  if (d.W == 0 || d.W > kDeriveTab / 32u || d.cap == 0 || d.cap > kDeriveTab)
    return hipErrorInvalidValue;
  if (d.W <= 4 && !getenv("OSPF_DERIVE_QUAD")) {  // lane = 16 nodes, words in registers
    d.G = std::max<uint32_t>(1, std::min<uint32_t>(kDeriveMaxG, kDeriveTab / d.cap));
    d.tiles = (g.V + 1023u) / 1024u;
    // 16 tiles per block: measured at F100k, W = 1 10.98 -> 10.08 ms, W = 3
    // 14.0 -> 13.8 ms against 8 (32: W = 1 9.8, W = 3 14.2)
    d.ctiles = std::max<uint32_t>(1, std::min<uint32_t>(d.tiles, d.ctiles ? d.ctiles : 16));
    d.chunks = (d.tiles + d.ctiles - 1) / d.ctiles;
    const dim3 grid(((d.n + d.G - 1) / d.G) * d.chunks);
    const size_t lds = (size_t)kWavesPerBlock * 1024u * d.W * 4u;
    switch (d.W) {
      case 1: hipLaunchKernelGGL(nh_derive16_kernel<1>, grid, dim3(kBlock), lds, s, g, d); break;
      case 2: hipLaunchKernelGGL(nh_derive16_kernel<2>, grid, dim3(kBlock), lds, s, g, d); break;
      case 3: hipLaunchKernelGGL(nh_derive16_kernel<3>, grid, dim3(kBlock), lds, s, g, d); break;
      default: hipLaunchKernelGGL(nh_derive16_kernel<4>, grid, dim3(kBlock), lds, s, g, d); break;
    }
    return hipGetLastError();
  }
  if (d.W > 4 && !getenv("OSPF_DERIVE_GENERIC")) {  // runs of equal lists share the words
    d.G = kWideG;
    if (const char* e = getenv("OSPF_DERIVE_WIDE_G"))
      d.G = std::max<uint32_t>(1, std::min<uint32_t>(kWideG, (uint32_t)atoi(e)));
    d.tiles = (g.V + kWideTile - 1) / kWideTile;
    d.ctiles = std::max<uint32_t>(1, std::min<uint32_t>(d.tiles, d.ctiles ? d.ctiles : 2));
    d.chunks = (d.tiles + d.ctiles - 1) / d.ctiles;
    const dim3 grid(((d.n + d.G - 1) / d.G) * d.chunks);
    hipLaunchKernelGGL(nh_derive_wide_kernel, grid, dim3(kBlock), 0, s, g, d);
    return hipGetLastError();
  }
  // one thread per node quad does all the words up to 8; wider rows split a
  // quad's words over 4 threads (a spine: 14 words x 32 neighbours each)
  const int S = d.W <= 8 ? 1 : 4;
  const uint32_t T = 1024u / S;
  d.G = std::max<uint32_t>(1, std::min<uint32_t>(kDeriveMaxG, kDeriveTab / d.cap));
  d.tiles = (g.V + T - 1) / T;
  d.ctiles = std::max<uint32_t>(1, std::min<uint32_t>(d.tiles, d.ctiles ? d.ctiles : 8));
  d.chunks = (d.tiles + d.ctiles - 1) / d.ctiles;
  const size_t lds = (size_t)T * d.W * 4u;
  const dim3 grid(((d.n + d.G - 1) / d.G) * d.chunks);
  if (S == 1) hipLaunchKernelGGL(nh_derive_kernel<1>, grid, dim3(kBlock), lds, s, g, d);
  else hipLaunchKernelGGL(nh_derive_kernel<4>, grid, dim3(kBlock), lds, s, g, d);
  return hipGetLastError();
}

hipError_t launch_wide_plan(const DevGraph& g, const WidePlan& p0, hipStream_t s) {
  WidePlan p = p0;
  if (p.n == 0) return hipSuccess;
  // digest keys and own levels issued with the slot loads (OSPF_WIDE_LATE_KEYS:
  // after the tile's barrier, as before; read per launch for in-process A/B)
  p.late_keys = getenv("OSPF_WIDE_LATE_KEYS") ? 1u : 0u;
  // records staged in LDS, 16-B stores (OSPF_WIDE_ST16=0: 4 word stores per
  // wave and root, as before; read per launch): 19.74 -> 19.21 ms per F100k
  // sweep in one process, profiles/r06/l1_late_kernel_ab.txt (box 3)
  const char* se = getenv("OSPF_WIDE_ST16");
  p.st16 = (!se || atoi(se) != 0) ? 1u : 0u;
  if (p.W < 1 || p.W > 64 || p.pitch % kW3Tile) return hipErrorInvalidValue;
  p.tiles = (g.V + kW3Tile - 1) / kW3Tile;
  // ~4096 blocks; a chunk of >= 7 tiles covers a 128-B line of every row
  const char* we = getenv("OSPF_WIDE_BLOCKS");  // read per launch: in-process A/B
  const uint32_t want = we ? (uint32_t)std::max(1, atoi(we)) : 8192u;  // (4096: +0.05 ms at F100k)
  if (!p.ctiles) p.ctiles = std::max<uint32_t>(7, p.tiles / std::max<uint32_t>(1, want / p.nruns));
  p.ctiles = std::min(p.ctiles, p.tiles);
  p.chunks = (p.tiles + p.ctiles - 1) / p.ctiles;
  const size_t lds = 4ull * kWideG * p.W + (size_t)kDeriveTab * kW3Pitch;
  if (lds > 64u * 1024u) {
    const hipError_t e = hipFuncSetAttribute((const void*)nh_wide_plan_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (p.digest) {
    const hipError_t e = ospf::zero_async(p.digest, (size_t)p.n * sizeof(ospf_digest), s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(nh_wide_plan_kernel, dim3(p.nruns * p.chunks), dim3(kBlock), lds, s, g, p);
  return hipGetLastError();
}

hipError_t launch_row_digest(const DevGraph& g, uint32_t n, const uint32_t* dist,
                             const uint32_t* nh, uint32_t W, ospf_digest* out, hipStream_t s) {
  hipError_t e = ospf::zero_async(out, (size_t)n * sizeof(ospf_digest), s);
  if (e != hipSuccess) return e;
  // enough workgroups to fill the chip; segment bounds are multiples of 4
  // nodes so the 16-B loads stay aligned
  const uint32_t segs = max(1u, min((16384u + n - 1) / n, max(1u, g.V / 1024u)));
  hipLaunchKernelGGL(row_digest_kernel, dim3(n * segs), dim3(kBlock), 0, s, g, dist, nh, W, segs,
                     out);
  return hipGetLastError();
}

}  // namespace ospf
