// spf_twin.hip — next hops of roots with twin neighbours (gfx950), unit
// metric / hop count.
//
// The derive rule (LinkState::runSpf's nextHops, openr/decision/
// LinkState.cpp:885-901, with unit weights): the k-th distinct neighbour n_k
// of root r is a next hop towards v iff the link r-n_k is up, n_k is transit
// or n_k == v, and dist(n_k, v) + 1 == dist(r, v). nh_derive16_kernel reads
// one level row per neighbour: 84 rows per fabric switch (48 racks of its
// pod, 36 spines of its plane) for 3 next-hop words per node.
//
// Twins. Two nodes a, b with the same usable distinct neighbours and the
// same transit bit (never adjacent: each would be its own neighbour) have
// dist(a, v) == dist(b, v) for every v outside {a, b}: a shortest path from
// either leaves through the same first hops, and overloaded nodes relay for
// neither (:859-866). And dist(a, b) == dist(b, a) (unit weights, the same
// transit conditions both ways). So a class of twins has ONE level row R
// (its representative's), except that member m sits at level 1 at its own
// position and, at the representative's position, every other member sits
// at X = R(any other member). A pod's racks are one class, a plane's spines
// another: a fabric switch reads its own row and two class rows per tile.
//
// Per lane 16 nodes (one 16-B load per row), a class is tight where
// R == L - 1 (L = the root's own level bytes; the borrow-free SWAR test of
// nh_derive16_kernel) and contributes its usable slots' bits at once. The
// members' own positions are patched afterwards (a neighbour is a next hop
// towards itself; at the representative the class is re-tested against X),
// on the words staged in LDS for the coalesced row stores, and the digest
// terms are taken from the patched words.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;
constexpr uint32_t kBlock = 256;
constexpr uint32_t kWaves = kBlock / 64u;
constexpr uint32_t kMaxK = 128;  // W <= 4 words
constexpr uint32_t kComboC = 6;  // classes whose mask combinations are tabled

__device__ __forceinline__ bool transit(const DevGraph& g, uint32_t v) {
  return !((g.nt_bits[v >> 5] >> (v & 31)) & 1u);
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int o) {
  const uint32_t lo = __shfl_xor((uint32_t)x, o, 64);
  const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), o, 64);
  return ((uint64_t)hi << 32) | lo;
}

// LDS tables of one root's neighbour classes, shared by the twin kernels.
struct TwinTab {
  uint32_t nb[kMaxK];     // distinct neighbours (ascending)
  uint32_t slot[kMaxK];   // per slot: class id (0xFFFFFFFE non-transit, kInf unusable)
  uint32_t first[kMaxK];  // first slot of the same class
  uint32_t cid[kMaxK];    // per slot: class index, 0x100 non-transit, kInf unusable
  uint32_t use[4];
  uint32_t ccls[kTwinMaxC], crow[kTwinMaxC], crep[kTwinMaxC], cx[kTwinMaxC];
  uint32_t cmask[kTwinMaxC][4];
  uint32_t nc, K, own, root, bad;
};

// Block-wide: the classes of root a.roots[i]'s usable transit neighbours,
// each with its representative's level row (crow) and slot mask. False (for
// the whole block) when the root or a class row is missing (error bits set).
__device__ bool twin_setup(const DevGraph& g, const TwinArgs& a, uint32_t i, uint32_t words,
                           TwinTab& T) {
  const uint32_t V = g.V, tid = threadIdx.x;
  if (tid == 0) {
    const uint32_t r = a.roots[i];
    T.root = r;
    T.bad = 0u;
    T.nc = 0u;
    T.own = r < V ? a.pos[r] : kInf;
    T.K = r < V ? g.dn_off[r + 1] - g.dn_off[r] : 0u;
    if (r >= V) atomicOr(a.err, 64u);
    else if (T.own == kInf) atomicOr(a.err, 16u);
    else if (T.K > a.cap || T.K > 32u * words) atomicOr(a.err, 1u);
  }
  if (tid < 4) T.use[tid] = 0u;
  __syncthreads();
  const uint32_t r = T.root, K = min(T.K, 32u * words);
  if (r >= V || T.own == kInf) return false;
  for (uint32_t e = g.row_ptr[r] + tid; e < g.row_ptr[r + 1]; e += kBlock) {
    const uint32_t cx = g.colx[e];
    if ((cx & kDown) || cx == r) continue;
    const uint32_t k = g.didx[e];
    if (k < K) atomicOr(&T.use[k >> 5], 1u << (k & 31u));
  }
  if (tid < K) T.nb[tid] = g.dn[g.dn_off[r] + tid];
  __syncthreads();
  // class of every usable transit slot (loads in parallel), first slot of
  // each class, then one pass over the slot table in LDS
  if (tid < K) {
    const uint32_t n = T.nb[tid];
    uint32_t v = kInf;  // unusable
    if ((T.use[tid >> 5] >> (tid & 31u)) & 1u) v = transit(g, n) ? a.tcls[n] : 0xFFFFFFFEu;
    T.slot[tid] = v;
  }
  __syncthreads();
  if (tid < K) {
    const uint32_t v = T.slot[tid];
    uint32_t first = tid;
    if (v < 0xFFFFFFFEu)
      for (uint32_t k = 0; k < tid; ++k)
        if (T.slot[k] == v) {
          first = k;
          break;
        }
    T.first[tid] = first;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t nc = 0;
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t v = T.slot[k];
      if (v >= 0xFFFFFFFEu) {
        T.cid[k] = v == kInf ? kInf : 0x100u;
        continue;
      }
      uint32_t j;
      if (T.first[k] == k) {
        if (nc == kTwinMaxC) {
          T.bad = 1u;
          break;
        }
        j = nc++;
        T.ccls[j] = v;
        for (int w = 0; w < 4; ++w) T.cmask[j][w] = 0u;
      } else {
        j = T.cid[T.first[k]];
      }
      T.cmask[j][k >> 5] |= 1u << (k & 31u);
      T.cid[k] = j;
    }
    T.nc = nc;
    if (T.bad) atomicOr(a.err, 256u);
  }
  __syncthreads();
  if (T.bad) return false;
  const uint32_t nc = T.nc;
  if (tid < nc) {
    const uint32_t c = T.ccls[tid], rep = a.trep[c], sec = a.tsec ? a.tsec[c] : kInf;
    const uint32_t row = a.pos[rep];
    T.crep[tid] = rep;
    T.crow[tid] = row;
    if (row == kInf) atomicOr(a.err, 16u);
    // X: level of another member at the representative's position
    T.cx[tid] = (sec != kInf && row != kInf) ? a.lev[(size_t)row * a.pitch + sec] : 0x7Fu;
  }
  __syncthreads();
  for (uint32_t x = 0; x < nc; ++x)
    if (T.crow[x] == kInf) return false;
  return true;
}

template <int W>
__global__ void __launch_bounds__(kBlock) nh_derive_twin_kernel(DevGraph g, TwinArgs a) {
  __shared__ TwinTab T;
  __shared__ unsigned long long s_h;
  __shared__ uint64_t s_wk[1u << kComboC];
  __shared__ uint32_t s_Lb[kWaves][256];  // own level bytes of each wave's tile
  extern __shared__ uint32_t s_stage[];  // [4 waves][1024 nodes][W]
  const uint32_t V = g.V, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  // XCD-aware order: XCD x (blocks x, x + 8, ...) walks a contiguous range
  // of (root, chunk) items, so roots sharing class rows share its L2
  const uint32_t NT = a.n * a.chunks, T8 = NT / 8u * 8u, b = blockIdx.x;
  const uint32_t item = b < T8 ? (b % 8u) * (T8 / 8u) + b / 8u : b;
  const uint32_t i = item / a.chunks, ci = item % a.chunks;
  if (tid == 0) s_h = 0ull;
  if (!twin_setup(g, a, i, W, T)) return;
  const uint32_t K = min(T.K, (uint32_t)(32 * W)), own = T.own, nc = T.nc;
  // an unpatched word is the OR of the tight classes' masks: with <= 6
  // classes its digest key is one of 2^nc, tabled in LDS (one lookup per node
  // instead of W splitmix hashes)
  const bool ctab = a.digest && nc <= kComboC;
  if (ctab && tid < (1u << nc)) {
    uint64_t ws = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      uint32_t m = 0;
      for (uint32_t j = 0; j < nc; ++j)
        if ((tid >> j) & 1u) m |= T.cmask[j][w];
      if (m) ws += digest_word_key(w, m);
    }
    s_wk[tid] = ws;
  }
  __syncthreads();
  const uint32_t t0 = ci * a.ctiles, t1 = min(a.tiles, t0 + a.ctiles);
  uint32_t* st = s_stage + wave * 1024u * W;
  uint64_t h = 0;
  // the own and class rows of the wave's next tile are loaded before this
  // tile is computed and stored (up to 1 + 3 classes prefetched)
  constexpr uint32_t kPre = 3;
  auto load_t = [&](uint32_t t, uint4& L, uint4* R) {
    const uint32_t vl = t * 1024u + 16u * lane;
    const uint32_t vs = (t < t1 && vl < a.pitch) ? vl : 0u;
    L = *reinterpret_cast<const uint4*>(a.lev + (size_t)own * a.pitch + vs);
#pragma unroll
    for (uint32_t j = 0; j < kPre; ++j)
      if (j < nc) R[j] = *reinterpret_cast<const uint4*>(a.lev + (size_t)T.crow[j] * a.pitch + vs);
  };
  uint4 Ln, Rn[kPre];
  load_t(t0 + wave, Ln, Rn);
  for (uint32_t t = t0 + wave; t < t1; t += kWaves) {
    const uint32_t tv0 = t * 1024u, vl = tv0 + 16u * lane;
    const bool live = vl < a.pitch;
    const uint32_t vs = live ? vl : 0u;
    const uint4 L = Ln;
    uint4 Rp[kPre];
#pragma unroll
    for (uint32_t j = 0; j < kPre; ++j) Rp[j] = Rn[j];
    load_t(t + kWaves, Ln, Rn);
    uint32_t lm1[4];
    {
      const uint32_t Lw[4] = {L.x, L.y, L.z, L.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t m = 0;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
          const uint32_t l = (Lw[q] >> (8 * bb)) & 0xFFu;
          m |= (l >= 2u && l < 0x7Fu ? l - 1u : 0u) << (8 * bb);
        }
        lm1[q] = m | 0x80808080u;
      }
    }
    uint32_t word[W][16], cbp[4] = {0u, 0u, 0u, 0u};  // cbp: tight-class bits, a byte per node
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int n = 0; n < 16; ++n) word[w][n] = 0u;
    for (uint32_t j = 0; j < nc; ++j) {
      uint4 R;
      if (j < kPre) {
#pragma unroll
        for (uint32_t q = 0; q < kPre; ++q)
          if (q == j) R = Rp[q];
      } else {
        R = *reinterpret_cast<const uint4*>(a.lev + (size_t)T.crow[j] * a.pitch + vs);
      }
      const uint32_t Rw[4] = {R.x, R.y, R.z, R.w};
      uint32_t cm[W];
#pragma unroll
      for (int w = 0; w < W; ++w) cm[w] = T.cmask[j][w];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t z = live ? (lm1[q] - Rw[q]) & 0x80808080u : 0u;
        if (ctab) cbp[q] |= ((z >> 7) & 0x01010101u) << j;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
          const uint32_t sel = 0u - ((z >> (8 * bb + 7)) & 1u);
#pragma unroll
          for (int w = 0; w < W; ++w) word[w][4 * q + bb] |= sel & cm[w];
        }
      }
    }
    // stage [node][word] in this wave's LDS slice
#pragma unroll
    for (int x = 0; x < 4 * W; ++x) {
      uint32_t v4[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 4 * x + c;
        v4[c] = word[f % W][f / W];
      }
      reinterpret_cast<uint4*>(st + 16u * W * lane)[x] = make_uint4(v4[0], v4[1], v4[2], v4[3]);
    }
    reinterpret_cast<uint4*>(s_Lb[wave])[lane] = L;  // the root's own level bytes of the tile
    __builtin_amdgcn_wave_barrier();
    // members' own positions inside this tile (slots are sorted by node id),
    // a lane per neighbour: distinct neighbours patch distinct nodes
    {
      uint32_t lo = 0, hi = K;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (T.nb[mid] < tv0) lo = mid + 1; else hi = mid;
      }
      uint32_t end = lo;
      hi = K;
      while (end < hi) {
        const uint32_t mid = (end + hi) >> 1;
        if (T.nb[mid] < tv0 + 1024u) end = mid + 1; else hi = mid;
      }
      for (uint32_t k = lo + lane; k < end; k += 64u) {
        const uint32_t sk = T.cid[k];
        if (sk == kInf) continue;
        const uint32_t n = T.nb[k], o = n - tv0;
        const uint32_t Ln = (s_Lb[wave][o >> 2] >> (8u * (o & 3u))) & 0xFFu;
        uint32_t nw[W], ow[W];
#pragma unroll
        for (int w = 0; w < W; ++w) nw[w] = ow[w] = st[o * W + w];
        if (sk != 0x100u && n == T.crep[sk]) {  // re-test the class against X
          const bool tight = Ln >= 2u && Ln < 0x7Fu && T.cx[sk] + 1u == Ln;
#pragma unroll
          for (int w = 0; w < W; ++w) nw[w] = (nw[w] & ~T.cmask[sk][w]) | (tight ? T.cmask[sk][w] : 0u);
        }
        // n itself: level 1 of its own row, a next hop iff dist(r, n) == 1
#pragma unroll
        for (int w = 0; w < W; ++w)
          if ((uint32_t)w == (k >> 5)) {
            const uint32_t bit = 1u << (k & 31u);
            nw[w] = (nw[w] & ~bit) | (Ln == 2u ? bit : 0u);
          }
#pragma unroll
        for (int w = 0; w < W; ++w) st[o * W + w] = nw[w];
        if (a.digest && n < V) {  // the digest terms below are of the unpatched words
          uint64_t d = 0;
#pragma unroll
          for (int w = 0; w < W; ++w)
            d += (nw[w] ? digest_word_key(w, nw[w]) : 0ull) - (ow[w] ? digest_word_key(w, ow[w]) : 0ull);
          h += g.dkn[n] * d;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    const size_t dst0 = (size_t)i * (a.npitch ? a.npitch : (size_t)V * W) + (size_t)tv0 * W;
    const uint32_t tn = tv0 < V ? min(1024u, V - tv0) : 0u;
    if (a.dist && tn) {  // dist row = own level - 1 (0x7F: unreached), 1 KB per store
      uint32_t* drow = a.dist + (size_t)own * (a.dpitch ? a.dpitch : V) + tv0;
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const uint32_t Lw = s_Lb[wave][x * 64 + lane], n0 = (uint32_t)x * 256u + 4u * lane;
        uint32_t dv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t l = (Lw >> (8 * q)) & 0xFFu;
          dv[q] = l < 0x7Fu ? l - 1u : kInf;
        }
        if (n0 + 4u <= tn && (V & 3u) == 0) {
          store_row16(reinterpret_cast<uint4*>(drow + n0), make_uint4(dv[0], dv[1], dv[2], dv[3]));
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (n0 + q < tn) drow[n0 + q] = dv[q];
        }
      }
    }
    if (tn == 1024u && (dst0 & 3u) == 0) {
#pragma unroll
      for (int x = 0; x < 4 * W; ++x)
        store_row16(reinterpret_cast<uint4*>(a.nh + dst0) + x * 64 + lane,
                    reinterpret_cast<const uint4*>(st)[x * 64 + lane]);
    } else {
      for (uint32_t x = lane; x < tn * W; x += 64u) a.nh[dst0 + x] = st[x];
    }
    if (a.digest && live) {
      const uint4* kp = reinterpret_cast<const uint4*>(g.dkn + vl);  // zero past V
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        const uint4 k2 = kp[x];
        const uint64_t kn[2] = {((uint64_t)k2.y << 32) | k2.x, ((uint64_t)k2.w << 32) | k2.z};
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          const int n = 2 * x + y;
          uint64_t ws = 0;
          if (ctab) {
            ws = s_wk[(cbp[n >> 2] >> (8 * (n & 3))) & 0xFFu];
          } else {
#pragma unroll
            for (int w = 0; w < W; ++w)
              if (word[w][n]) ws += digest_word_key(w, word[w][n]);
          }
          h += kn[y] * ws;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the slice is rewritten by the next tile
  }
  if (a.digest) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) h += shfl_xor64(h, o);
    if (lane == 0 && h) atomicAdd(&s_h, (unsigned long long)h);
    __syncthreads();
    if (tid == 0) {
      ospf_digest* dg = a.digest + i;
      unsigned long long hh = s_h;
      if (ci == 0) {
        const ospf_digest ld = a.lev_digest[own];
        atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)ld.reached);
        atomicAdd((unsigned long long*)&dg->sum_dist, (unsigned long long)ld.sum_dist);
        hh += ld.hash;
      }
      if (hh) atomicAdd((unsigned long long*)&dg->hash, hh);
    }
  }
}


// The same derivation with lane = 4 nodes (wave = 256 nodes): a tile's
// words staged per wave in 1 KB x W of LDS (12 KB a block at W = 3, against
// 48 KB for 1,024-node wave tiles), 4 x W word registers instead of 16 x W,
// so LDS and registers no longer cap the waves per SIMD; loads are one 4-B
// piece of the own and each class row per lane (256 B per wave instruction),
// stores W 1-KB runs of next-hop words and one 1-KB run of dist per chunk.
template <int W, int PD, bool KD>
__global__ void __launch_bounds__(kBlock) nh_twin4_kernel(DevGraph g, TwinArgs a) {
  __shared__ TwinTab T;
  __shared__ unsigned long long s_h;
  __shared__ uint64_t s_wk[1u << kComboC];
  __shared__ uint32_t s_L[kWaves][64];           // own level bytes of each wave's chunk
  __shared__ uint32_t s_st[kWaves][256 * W];     // [node][word] of each wave's chunk
  const uint32_t V = g.V, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t NT = a.n * a.chunks, T8 = NT / 8u * 8u, b = blockIdx.x;
  const uint32_t item = b < T8 ? (b % 8u) * (T8 / 8u) + b / 8u : b;
  const uint32_t i = item / a.chunks, ci = item % a.chunks;
  if (tid == 0) s_h = 0ull;
  if (!twin_setup(g, a, i, W, T)) return;
  const uint32_t K = min(T.K, (uint32_t)(32 * W)), own = T.own, nc = T.nc;
  const bool ctab = a.digest && nc <= kComboC;
  if (ctab && tid < (1u << nc)) {
    uint64_t ws = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      uint32_t m = 0;
      for (uint32_t j = 0; j < nc; ++j)
        if ((tid >> j) & 1u) m |= T.cmask[j][w];
      if (m) ws += digest_word_key(w, m);
    }
    s_wk[tid] = ws;
  }
  __syncthreads();
  const uint32_t c_beg = ci * a.ctiles * 4u;
  const uint32_t c_end = min((a.pitch + 255u) / 256u, (ci * a.ctiles + a.ctiles) * 4u);
  uint32_t* st = s_st[wave];
  const uint32_t dpitch = a.dpitch ? a.dpitch : V;
  const size_t npitch = a.npitch ? a.npitch : (size_t)V * W;
  const bool vec = (V & 3u) == 0 && (dpitch & 3u) == 0 && (npitch & 3u) == 0;
  uint64_t h = 0;
  // members' positions: a cursor over the ascending neighbour list (the
  // wave's chunks ascend), its next position cached in a register
  uint32_t ncur = 0, nnx = K ? T.nb[0] : kInf;
  constexpr uint32_t kPre = 3;
  // KD: the 4 nodes' digest keys ride in the same ring (their L2 latency
  // was exposed at the digest terms of every chunk)
  auto load_c = [&](uint32_t c, uint32_t& L, uint32_t* R, uint4* K) {
    const uint32_t v0 = c * 256u + 4u * lane;
    const uint32_t vs = (c < c_end && v0 < a.pitch) ? v0 : 0u;
    L = *reinterpret_cast<const uint32_t*>(a.lev + (size_t)own * a.pitch + vs);
#pragma unroll
    for (uint32_t j = 0; j < kPre; ++j)
      R[j] = j < nc ? *reinterpret_cast<const uint32_t*>(a.lev + (size_t)T.crow[j] * a.pitch + vs)
                    : 0x7F7F7F7Fu;
    if constexpr (KD) {  // (zero padded past V up to the level pitch)
      if (a.digest) {
        K[0] = reinterpret_cast<const uint4*>(g.dkn + vs)[0];
        K[1] = reinterpret_cast<const uint4*>(g.dkn + vs)[1];
      }
    }
  };
  // PD chunks of loads in flight per wave (a ring of prefetched rows)
  uint32_t Ln[PD], Rn[PD][kPre];
  uint4 Kn[PD][KD ? 2 : 1];
#pragma unroll
  for (int d = 0; d < PD; ++d) load_c(c_beg + wave + d * kWaves, Ln[d], Rn[d], Kn[d]);
  for (uint32_t c = c_beg + wave; c < c_end; c += kWaves) {
    const uint32_t c0 = c * 256u, v0 = c0 + 4u * lane;
    const bool live = v0 < a.pitch;
    const uint32_t vs = live ? v0 : 0u;
    const uint32_t L = Ln[0];
    uint32_t Rp[kPre];
#pragma unroll
    for (uint32_t j = 0; j < kPre; ++j) Rp[j] = Rn[0][j];
    uint64_t kd4[4] = {0ull, 0ull, 0ull, 0ull};
    if constexpr (KD) {
      kd4[0] = ((uint64_t)Kn[0][0].y << 32) | Kn[0][0].x;
      kd4[1] = ((uint64_t)Kn[0][0].w << 32) | Kn[0][0].z;
      kd4[2] = ((uint64_t)Kn[0][1].y << 32) | Kn[0][1].x;
      kd4[3] = ((uint64_t)Kn[0][1].w << 32) | Kn[0][1].z;
    }
#pragma unroll
    for (int d = 0; d + 1 < PD; ++d) {
      Ln[d] = Ln[d + 1];
#pragma unroll
      for (uint32_t j = 0; j < kPre; ++j) Rn[d][j] = Rn[d + 1][j];
      if constexpr (KD) {
        Kn[d][0] = Kn[d + 1][0];
        Kn[d][1] = Kn[d + 1][1];
      }
    }
    load_c(c + PD * kWaves, Ln[PD - 1], Rn[PD - 1], Kn[PD - 1]);
    uint32_t lm1 = 0;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const uint32_t l = (L >> (8 * bb)) & 0xFFu;
      lm1 |= (l >= 2u && l < 0x7Fu ? l - 1u : 0u) << (8 * bb);
    }
    lm1 |= 0x80808080u;
    uint32_t word[W][4], cbp = 0u;  // cbp: tight-class bits, a byte per node
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int n = 0; n < 4; ++n) word[w][n] = 0u;
    for (uint32_t j = 0; j < nc; ++j) {
      uint32_t R = 0x7F7F7F7Fu;
      if (j < kPre) {
#pragma unroll
        for (uint32_t q = 0; q < kPre; ++q)
          if (q == j) R = Rp[q];
      } else {
        R = *reinterpret_cast<const uint32_t*>(a.lev + (size_t)T.crow[j] * a.pitch + vs);
      }
      const uint32_t z = live ? (lm1 - R) & 0x80808080u : 0u;
      if (ctab) cbp |= ((z >> 7) & 0x01010101u) << j;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const uint32_t sel = 0u - ((z >> (8 * bb + 7)) & 1u);
#pragma unroll
        for (int w = 0; w < W; ++w) word[w][bb] |= sel & T.cmask[j][w];
      }
    }
    // stage [node][word]: the lane's 4 nodes are 4 W consecutive words
#pragma unroll
    for (int x = 0; x < W; ++x) {
      uint32_t v4[4];
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const int f = 4 * x + cc;
        v4[cc] = word[f % W][f / W];
      }
      reinterpret_cast<uint4*>(st + 4u * W * lane)[x] = make_uint4(v4[0], v4[1], v4[2], v4[3]);
    }
    s_L[wave][lane] = L;
    // digest terms of the unpatched words (the patches below add their deltas)
    if (a.digest && live) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint64_t ws = 0;
        if (ctab) {
          ws = s_wk[(cbp >> (8 * q)) & 0xFFu];
        } else {
#pragma unroll
          for (int w = 0; w < W; ++w)
            if (word[w][q]) ws += digest_word_key(w, word[w][q]);
        }
        h += (KD ? kd4[q] : g.dkn[v0 + q]) * ws;  // zero past V
      }
    }
    __builtin_amdgcn_wave_barrier();
    // members' own positions in this chunk, a lane per neighbour
    {
      uint32_t lo, end;
      if (a.bsearch) {
        uint32_t hi = K;
        lo = 0;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (T.nb[mid] < c0) lo = mid + 1; else hi = mid;
        }
        end = lo;
        hi = K;
        while (end < hi) {
          const uint32_t mid = (end + hi) >> 1;
          if (T.nb[mid] < c0 + 256u) end = mid + 1; else hi = mid;
        }
      } else {
        while (nnx < c0) {
          ++ncur;
          nnx = ncur < K ? T.nb[ncur] : kInf;
        }
        lo = ncur;
        while (nnx < c0 + 256u) {
          ++ncur;
          nnx = ncur < K ? T.nb[ncur] : kInf;
        }
        end = ncur;
      }
      for (uint32_t k = lo + lane; k < end; k += 64u) {
        const uint32_t sk = T.cid[k];
        if (sk == kInf) continue;
        const uint32_t n = T.nb[k], o = n - c0;
        const uint32_t Lo = (s_L[wave][o >> 2] >> (8u * (o & 3u))) & 0xFFu;
        uint32_t nw[W], ow[W];
#pragma unroll
        for (int w = 0; w < W; ++w) nw[w] = ow[w] = st[o * W + w];
        if (sk != 0x100u && n == T.crep[sk]) {  // re-test the class against X
          const bool tight = Lo >= 2u && Lo < 0x7Fu && T.cx[sk] + 1u == Lo;
#pragma unroll
          for (int w = 0; w < W; ++w) nw[w] = (nw[w] & ~T.cmask[sk][w]) | (tight ? T.cmask[sk][w] : 0u);
        }
#pragma unroll
        for (int w = 0; w < W; ++w)
          if ((uint32_t)w == (k >> 5)) {
            const uint32_t bit = 1u << (k & 31u);
            nw[w] = (nw[w] & ~bit) | (Lo == 2u ? bit : 0u);
          }
#pragma unroll
        for (int w = 0; w < W; ++w) st[o * W + w] = nw[w];
        if (a.digest && n < V) {
          uint64_t d = 0;
#pragma unroll
          for (int w = 0; w < W; ++w)
            d += (nw[w] ? digest_word_key(w, nw[w]) : 0ull) - (ow[w] ? digest_word_key(w, ow[w]) : 0ull);
          h += g.dkn[n] * d;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t tn = c0 < V ? min(256u, V - c0) : 0u;
    if (a.dist && tn) {  // dist row = own level - 1 (0x7F: unreached)
      uint32_t dv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t l = (L >> (8 * q)) & 0xFFu;
        dv[q] = l < 0x7Fu ? l - 1u : kInf;
      }
      uint32_t* drow = a.dist + (size_t)own * dpitch + c0;
      const uint32_t n0 = 4u * lane;
      if (vec && n0 + 4u <= tn) {
        store_row16(drow + n0, make_uint4(dv[0], dv[1], dv[2], dv[3]));
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (n0 + q < tn) drow[n0 + q] = dv[q];
      }
    }
    const size_t dst0 = (size_t)i * npitch + (size_t)c0 * W;
    if (tn == 256u && vec) {
#pragma unroll
      for (int x = 0; x < W; ++x)
        store_row16(reinterpret_cast<uint4*>(a.nh + dst0) + x * 64 + lane,
                    reinterpret_cast<const uint4*>(st)[x * 64 + lane]);
    } else {
      for (uint32_t x = lane; x < tn * W; x += 64u) a.nh[dst0 + x] = st[x];
    }
    __builtin_amdgcn_wave_barrier();  // the slice is rewritten by the next chunk
  }
  if (a.digest) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) h += shfl_xor64(h, o);
    if (lane == 0 && h) atomicAdd(&s_h, (unsigned long long)h);
    __syncthreads();
    if (tid == 0) {
      ospf_digest* dg = a.digest + i;
      unsigned long long hh = s_h;
      if (ci == 0) {
        const ospf_digest ld = a.lev_digest[own];
        atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)ld.reached);
        atomicAdd((unsigned long long*)&dg->sum_dist, (unsigned long long)ld.sum_dist);
        hh += ld.hash;
      }
      if (hh) atomicAdd((unsigned long long*)&dg->hash, hh);
    }
  }
}

// byte-wise min of 7-bit bytes: bit 7 of (a | 0x80) - b is set iff a >= b
__device__ __forceinline__ uint32_t bmin7(uint32_t a, uint32_t b) {
  const uint32_t ge = ((a | 0x80808080u) - b) & 0x80808080u;
  const uint32_t m = (ge << 1) - (ge >> 7);  // 0xFF in the bytes where a >= b
  return (b & m) | (a & ~m);
}
// bit 7 of each byte: the 7-bit bytes of x and y are equal
__device__ __forceinline__ uint32_t beq7(uint32_t x, uint32_t y) {
  return ~((x ^ y) + 0x7F7F7F7Fu) & 0x80808080u;
}

// Level + dist rows of a root from its neighbour classes (twin Bellman).
// dist(r, v) = 1 + min over the classes of the representative's row R_j(v)
// for v outside r and its usable neighbours; 0 at r; 1 at every usable
// neighbour, transit or not -- LinkState::runSpf's Bellman equation over the
// root's out-links with unit weights (LinkState.cpp:836-911; overloaded
// neighbours reach only themselves, :859-866): twins' rows agree except at
// their members' positions, and every member of a neighbour's class is
// itself a usable neighbour of r (twins share their usable neighbours, r
// among them). So a fabric switch reads two class rows (its pod's racks,
// its plane's spines) instead of a traversal.
// Block = a group of up to kTwinLvG roots whose classes' rows number <= 16
// (a pod's fabric switches: one rack row + the 8 planes' spine rows): per
// 256-node chunk a wave loads each of the group's rows once (lane = 4
// nodes), then per root takes the min over its rows, patches its own and its
// neighbours' positions (each root's sorted neighbour list walked by a
// cursor) and stores 256 B of level row + 1 KB of dist row per instruction.
// The distance part of each root's digest is stored (not added).
// OPT bit 1 (CUR, the default): each root's next neighbour position cached
// in a register, so the cursor tests read LDS only when a neighbour is due
// (18.73 -> 18.53 ms per F100k sweep in one process, profiles/r06/
// l1_late_kernel_ab.txt); bit 2 (NOHASH): diagnostic only -- the level-hash
// terms and their key loads skipped (digests then differ): -0.3 ms, what the
// hash costs. (Its terms as v_dot2_u32_u16 of level bytes and 16-bit key
// pieces were exact but no faster: the launch waits on loads, not the VALU.)
// RW: each wave takes G / 4 of the group's roots over every chunk of the
// block's range (loading only its roots' class rows) instead of every root
// over a quarter of the chunks: a quarter of the per-root registers, so more
// waves per SIMD hide the row and key loads' latency.
template <bool PRE, int OPT = 1, uint32_t G = kTwinLvG, bool RW = false>
__global__ void __launch_bounds__(kBlock) twin_levels_kernel(DevGraph g, TwinLvPlan a) {
  constexpr bool CUR = (OPT & 1) != 0, NOHASH = (OPT & 2) != 0;
  constexpr uint32_t NR = RW ? G / kWaves : G;  // roots per wave
  __shared__ uint32_t s_nb[G][kMaxK];  // usable neighbours (ascending), per root
  __shared__ uint32_t s_nnb[G], s_root[G], s_own[G], s_umask[G];
  __shared__ unsigned long long s_d[kWaves][G][3];
  const uint32_t V = g.V, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  // block = (group, part of the chunk range); XCD-aware order over the items
  const uint32_t NB = a.ngroups * a.parts, B8 = NB / 8u * 8u, b = blockIdx.x;
  const uint32_t item = b < B8 ? (b % 8u) * (B8 / 8u) + b / 8u : b;
  const uint32_t gi = item / a.parts, part = item % a.parts;
  const uint32_t i0 = a.grp[gi];
  const uint32_t ng = min(G, a.grp[gi + 1] - i0);
  if (RW && tid < kWaves * G * 3) (&s_d[0][0][0])[tid] = 0ull;  // owners write theirs
  if (tid < ng) {
    const uint4 ri = a.rinfo[i0 + tid];
    s_root[tid] = ri.x;
    s_own[tid] = ri.y;
    s_umask[tid] = ri.z;
    s_nnb[tid] = min(kMaxK, a.nbo[i0 + tid + 1] - ri.w);
  }
  for (uint32_t x = tid; x < ng * kMaxK; x += kBlock) {
    const uint32_t j = x / kMaxK, k = x % kMaxK;
    const uint32_t o = a.nbo[i0 + j];
    if (o + k < a.nbo[i0 + j + 1]) s_nb[j][k] = a.nbl[o + k];
  }
  uint32_t urow[kTwinMaxC];
  uint32_t nu = 0;
#pragma unroll
  for (uint32_t u = 0; u < kTwinMaxC; ++u) {
    urow[u] = a.grow[(size_t)gi * kTwinMaxC + u];
    nu += urow[u] != kInf ? 1u : 0u;
  }
  __syncthreads();
  const uint32_t nchunks = (a.pitch + 255u) / 256u;
  const uint32_t cb = (uint32_t)((uint64_t)part * nchunks / a.parts);
  const uint32_t ce = (uint32_t)((uint64_t)(part + 1) * nchunks / a.parts);
  const uint32_t j0 = RW ? wave * NR : 0u;  // this wave's first root
  uint32_t lmask = ~0u;  // class rows this wave loads
  if constexpr (RW) {
    lmask = 0u;
#pragma unroll
    for (uint32_t jj = 0; jj < NR; ++jj)
      if (j0 + jj < ng) lmask |= s_umask[j0 + jj];
    lmask = __builtin_amdgcn_readfirstlane(lmask);
  }
  // the next chunk's rows and distance keys are loaded before this one is used
  auto load_x = [&](uint32_t c, uint32_t* x, uint64_t* kd) {
    const uint32_t v0 = c * 256u + 4u * lane;
    const bool ok = c < ce && v0 < a.pitch;
#pragma unroll
    for (uint32_t u = 0; u < kTwinMaxC; ++u)
      x[u] = (u < nu && ok && ((lmask >> u) & 1u))
                 ? *reinterpret_cast<const uint32_t*>(a.lev + (size_t)urow[u] * a.pitch + v0)
                 : 0x7F7F7F7Fu;
#pragma unroll
    for (int q = 0; q < 4; ++q) kd[q] = !NOHASH && ok && v0 + q < V ? g.dkey[2ull * (v0 + q)] : 0ull;
  };
  // distance part of each root's digest, per lane: reached, sum of dist
  // (u32: <= V / 64 nodes x 125 per lane), sum of dkey * level split in
  // sum(dkey_lo * level) (u64, one v_mad_u64_u32 a node) and
  // sum(dkey_hi * level) mod 2^32 (the hash is mod 2^64)
  uint32_t br[NR], cur[NR], bs[NR], bhh[NR];
  uint64_t bl[NR];
#pragma unroll
  for (uint32_t j = 0; j < NR; ++j) {
    br[j] = 0u;
    cur[j] = 0u;
    bs[j] = bhh[j] = 0u;
    bl[j] = 0ull;
  }
  uint32_t nx[CUR ? NR : 1];  // CUR: s_nb[j][cur[j]], kInf past the list
  if constexpr (CUR) {
#pragma unroll
    for (uint32_t j = 0; j < NR; ++j) nx[j] = (j0 + j < ng && s_nnb[j0 + j]) ? s_nb[j0 + j][0] : kInf;
  }
  const bool vec = (V & 3u) == 0;
  // PRE: the next chunk's rows loaded before this one is used (24 more
  // registers: 3 waves per SIMD instead of 4)
  uint32_t xn[PRE ? kTwinMaxC : 1];
  uint64_t kdn[4];
  constexpr uint32_t cstep = RW ? 1u : kWaves;
  const uint32_t cfirst = RW ? cb : cb + wave;
  if constexpr (PRE) load_x(cfirst, xn, kdn);
  for (uint32_t c = cfirst; c < ce; c += cstep) {
    const uint32_t c0 = c * 256u, v0 = c0 + 4u * lane;
    uint32_t x[kTwinMaxC];
    uint64_t kd[4];
    if constexpr (PRE) {
#pragma unroll
      for (uint32_t u = 0; u < kTwinMaxC; ++u) x[u] = xn[u];
#pragma unroll
      for (int q = 0; q < 4; ++q) kd[q] = kdn[q];
      load_x(c + cstep, xn, kdn);
    } else {
      load_x(c, x, kd);
    }
    if (v0 >= a.pitch) continue;  // no wave-level work below (cursors are per wave: see skip)
#pragma unroll
    for (uint32_t j = 0; j < NR; ++j) {
      const uint32_t jr = j0 + j;  // the root's index in the group
      if (jr >= ng) break;
      // the root's class rows (a scalar mask: untaken rows cost a branch)
      const uint32_t mask = __builtin_amdgcn_readfirstlane(s_umask[jr]);
      uint32_t m = 0x7F7F7F7Fu;
#pragma unroll
      for (uint32_t u = 0; u < kTwinMaxC; ++u)
        if ((mask >> u) & 1u) m = bmin7(m, x[u]);
      uint32_t L = (m + 0x01010101u) - (((m + 0x01010101u) & 0x80808080u) >> 7);
      // neighbours in this chunk: level 2 (the list is ascending; chunks of a
      // wave ascend, so the cursor skips the other waves' chunks)
      const uint32_t nn = s_nnb[jr];
      if constexpr (CUR) {
        while (nx[j] < c0) {
          ++cur[j];
          nx[j] = cur[j] < nn ? s_nb[jr][cur[j]] : kInf;
        }
        while (nx[j] < c0 + 256u) {
          const uint32_t o = nx[j] - v0;
          if (o < 4u) L = (L & ~(0xFFu << (8u * o))) | (2u << (8u * o));
          ++cur[j];
          nx[j] = cur[j] < nn ? s_nb[jr][cur[j]] : kInf;
        }
      } else {
        while (cur[j] < nn && s_nb[jr][cur[j]] < c0) ++cur[j];
        while (cur[j] < nn && s_nb[jr][cur[j]] < c0 + 256u) {
          const uint32_t n = s_nb[jr][cur[j]++], o = n - v0;
          if (o < 4u) L = (L & ~(0xFFu << (8u * o))) | (2u << (8u * o));
        }
      }
      const uint32_t off = s_root[jr] - v0;
      if (off < 4u) L = (L & ~(0xFFu << (8u * off))) | (1u << (8u * off));
      const uint32_t own = s_own[jr];
      __builtin_nontemporal_store(L, reinterpret_cast<uint32_t*>(a.lev + (size_t)own * a.pitch + v0));
      if (v0 >= V) continue;
      // SWAR over the 4 nodes: reached bytes (< 0x7F, node < V), their
      // levels summed, and the hash terms of the levels
      uint32_t vb = ~beq7(L, 0x7F7F7F7Fu) & 0x80808080u;
      if (V - v0 < 4u) vb &= (1u << (8u * (V - v0))) - 1u;
      const uint32_t Lv = L & ((vb >> 7) * 0xFFu);
      const uint32_t nv = (uint32_t)__builtin_popcount(vb);
      const uint32_t t2 = (Lv & 0x00FF00FFu) + ((Lv >> 8) & 0x00FF00FFu);
      br[j] += nv;
      bs[j] += (t2 & 0xFFFFu) + (t2 >> 16) - nv;
      if constexpr (!NOHASH) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t l = (Lv >> (8 * q)) & 0xFFu;
          bl[j] += (uint64_t)(uint32_t)kd[q] * l;
          bhh[j] += (uint32_t)(kd[q] >> 32) * l;
        }
      }
      if (a.dist && !(s_umask[jr] >> 31)) {  // bit 31: the root's next-hop launch writes it
        uint32_t dv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t l = (L >> (8 * q)) & 0xFFu;
          dv[q] = l < 0x7Fu ? l - 1u : kInf;
        }
        uint32_t* drow = a.dist + (size_t)own * (a.dpitch ? a.dpitch : V) + v0;
        if (vec) {
          store_row16(drow, make_uint4(dv[0], dv[1], dv[2], dv[3]));
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (v0 + q < V) drow[q] = dv[q];
        }
      }
    }
  }
  if (!a.lev_digest) return;
#pragma unroll
  for (uint32_t j = 0; j < NR; ++j) {
    uint64_t r64 = br[j], s64 = bs[j], h64 = bl[j] + ((uint64_t)bhh[j] << 32);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      r64 += shfl_xor64(r64, o);
      s64 += shfl_xor64(s64, o);
      h64 += shfl_xor64(h64, o);
    }
    if (lane == 0 && j0 + j < G) {
      s_d[wave][j0 + j][0] = r64;
      s_d[wave][j0 + j][1] = s64;
      s_d[wave][j0 + j][2] = h64;
    }
  }
  __syncthreads();
  if (tid < ng) {
    ospf_digest d{0ull, 0ull, 0ull};
    for (uint32_t w = 0; w < kWaves; ++w) {
      d.reached += s_d[w][tid][0];
      d.sum_dist += s_d[w][tid][1];
      d.hash += s_d[w][tid][2];
    }
    ospf_digest* o = a.lev_digest + s_own[tid];
    if (a.parts == 1) {  // the root's only block: stored (no zeroing launch before)
      *o = d;
    } else {  // zeroed by twin_zero_kernel
      atomicAdd((unsigned long long*)&o->reached, (unsigned long long)d.reached);
      atomicAdd((unsigned long long*)&o->sum_dist, (unsigned long long)d.sum_dist);
      atomicAdd((unsigned long long*)&o->hash, (unsigned long long)d.hash);
    }
  }
}

__global__ void twin_zero_kernel(const uint4* rinfo, uint32_t n, ospf_digest* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[rinfo[i].y] = ospf_digest{0ull, 0ull, 0ull};
}

}  // namespace

hipError_t launch_nh_derive_twin(const DevGraph& g, const TwinArgs& a0, hipStream_t s) {
  TwinArgs a = a0;
  if (a.n == 0) return hipSuccess;
  if (a.W == 0 || a.W > 4) return hipErrorInvalidValue;
  // members' positions by binary search per chunk (OSPF_TWIN4_BSEARCH; read per launch)
  a.bsearch = getenv("OSPF_TWIN4_BSEARCH") ? 1u : 0u;
  a.tiles = (g.V + 1023u) / 1024u;
  if (!a.ctiles) a.ctiles = a.tiles;  // one block per root: the slot setup once
  a.ctiles = std::max(1u, std::min(a.tiles, a.ctiles));
  a.chunks = (a.tiles + a.ctiles - 1) / a.ctiles;
  const dim3 grid(a.n * a.chunks);
  // lane = 4 nodes (nh_twin4_kernel) unless OSPF_TWIN_NH16=1 (lane = 16 nodes)
  const bool nh16 = getenv("OSPF_TWIN_NH16") != nullptr;  // read per launch: in-process A/B
  if (!nh16) {
    // prefetch depth (chunks of loads in flight per wave): OSPF_TWIN4_PD 1 / 2;
    // the digest keys prefetched with the rows (OSPF_TWIN4_KD=0: loaded at
    // the digest terms; 20.10 -> 19.82 ms per F100k sweep in one process,
    // profiles/r06/k2_twin4_key_prefetch_ab.txt)
    const char* pe = getenv("OSPF_TWIN4_PD");
    const bool pd2 = !pe || atoi(pe) >= 2;
    const char* ke = getenv("OSPF_TWIN4_KD");
    const bool kd = pd2 && (!ke || atoi(ke) != 0);
#define OSPF_TWIN4(WW)                                                                          \
  if (kd) hipLaunchKernelGGL((nh_twin4_kernel<WW, 2, true>), grid, dim3(kBlock), 0, s, g, a);  \
  else if (pd2) hipLaunchKernelGGL((nh_twin4_kernel<WW, 2, false>), grid, dim3(kBlock), 0, s, g, a); \
  else hipLaunchKernelGGL((nh_twin4_kernel<WW, 1, false>), grid, dim3(kBlock), 0, s, g, a);
    switch (a.W) {
      case 1: OSPF_TWIN4(1) break;
      case 2: OSPF_TWIN4(2) break;
      case 3: OSPF_TWIN4(3) break;
      default: OSPF_TWIN4(4) break;
    }
#undef OSPF_TWIN4
    return hipGetLastError();
  }
  const size_t lds = (size_t)kWaves * 1024u * a.W * 4u;
  switch (a.W) {
    case 1: hipLaunchKernelGGL(nh_derive_twin_kernel<1>, grid, dim3(kBlock), lds, s, g, a); break;
    case 2: hipLaunchKernelGGL(nh_derive_twin_kernel<2>, grid, dim3(kBlock), lds, s, g, a); break;
    case 3: hipLaunchKernelGGL(nh_derive_twin_kernel<3>, grid, dim3(kBlock), lds, s, g, a); break;
    default: hipLaunchKernelGGL(nh_derive_twin_kernel<4>, grid, dim3(kBlock), lds, s, g, a); break;
  }
  return hipGetLastError();
}

}  // namespace ospf

namespace ospf {
hipError_t launch_twin_levels(const DevGraph& g, const TwinLvPlan& a0, hipStream_t s) {
  if (a0.n == 0) return hipSuccess;
  TwinLvPlan a = a0;
  // parts of the chunk range per group: ~2048 blocks, >= 8 chunks each
  const uint32_t nchunks = (a.pitch + 255u) / 256u;
  const char* be = getenv("OSPF_TWIN_LV_BLOCKS");  // read per launch: in-process A/B
  const uint32_t want = be ? (uint32_t)std::max(1, atoi(be)) : 2048u;  // (4096: +0.05 ms at F100k)
  if (!a.parts)
    a.parts = std::max(1u, std::min(std::max(1u, nchunks / 8u), want / std::max(1u, a.ngroups)));
  // (one part per group: each root's digest is stored by its block, no zeroing)
  if (a.lev_digest && a.parts > 1)
    hipLaunchKernelGGL(twin_zero_kernel, dim3((a.n + 255u) / 256u), dim3(256), 0, s, a.rinfo, a.n,
                       a.lev_digest);
  // (OSPF_TWIN_PREFETCH=1: the software-pipelined variant, 3 waves per SIMD;
  // OSPF_TWIN_LV_OPT: the OPT bits above, default 1; both read per launch)
  const bool pre = getenv("OSPF_TWIN_PREFETCH") != nullptr;
  const char* oe = getenv("OSPF_TWIN_LV_OPT");
  const int opt = oe ? atoi(oe) & 3 : 1;
  const dim3 grid(a.ngroups * a.parts);
  // groups of <= 4 roots (OSPF_TWIN_LV_G=4 at plan time): the 4-root kernel
#define OSPF_TWIN_LV(GG)                                                                 \
  if (pre)                                                                               \
    hipLaunchKernelGGL((twin_levels_kernel<true, 1, GG>), grid, dim3(kBlock), 0, s, g, a);  \
  else if (opt == 0)                                                                     \
    hipLaunchKernelGGL((twin_levels_kernel<false, 0, GG>), grid, dim3(kBlock), 0, s, g, a); \
  else if (opt == 2)                                                                     \
    hipLaunchKernelGGL((twin_levels_kernel<false, 2, GG>), grid, dim3(kBlock), 0, s, g, a); \
  else if (opt == 3)                                                                     \
    hipLaunchKernelGGL((twin_levels_kernel<false, 3, GG>), grid, dim3(kBlock), 0, s, g, a); \
  else                                                                                   \
    hipLaunchKernelGGL((twin_levels_kernel<false, 1, GG>), grid, dim3(kBlock), 0, s, g, a);
  // OSPF_TWIN_LV_RW=1: two roots a wave over every chunk (RW above)
  const char* rwe = getenv("OSPF_TWIN_LV_RW");
  const int rw = rwe ? atoi(rwe) : 0;
  if (rw == 1 && !pre && opt == 1 && !(a.gsz && a.gsz <= 4u)) {
    hipLaunchKernelGGL((twin_levels_kernel<false, 1, kTwinLvG, true>), grid, dim3(kBlock), 0, s, g, a);
  } else if (rw == 2 && !(a.gsz && a.gsz <= 4u)) {
    hipLaunchKernelGGL((twin_levels_kernel<true, 1, kTwinLvG, true>), grid, dim3(kBlock), 0, s, g, a);
  } else if (a.gsz && a.gsz <= 4u) {
    OSPF_TWIN_LV(4u)
  } else {
    OSPF_TWIN_LV(kTwinLvG)
  }
#undef OSPF_TWIN_LV
  return hipGetLastError();
}
}  // namespace ospf
