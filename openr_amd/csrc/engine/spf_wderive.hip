// spf_wderive.hip — weighted all-sources rows of leaf roots from their
// neighbours' distance rows (gfx950).
//
// For a root r with distinct neighbours n_0 .. n_{K-1} (ascending id = next-hop
// bit order), w_k = the smallest metric r advertises on an up link to n_k
// (1 in hop-count mode) and D_k = n_k's distance row, the reference's runSpf
// (openr/decision/LinkState.cpp:836-911) gives, for v != r,
//
//   dist(r, v) = min over usable k of  w_k + D_k(v)        (n_k transit)
//                                      w_k if v == n_k     (n_k overloaded)
//   bit k of nh(r, v)  <=>  that term of k equals dist(r, v)
//
// A shortest r -> v path leaves r over one link to some n_k, and its tail is a
// path of n_k's own SPF (interior nodes transit, LinkState.cpp:859-866; the
// tail never needs r again: metrics are >= 1), so the first line is Bellman's
// equation over r's out-links; the next hops of v are exactly the first hops
// of its shortest paths (nextHops = union over tight predecessors, with the
// root's own neighbours as seeds, LinkState.cpp:885-901). An overloaded
// neighbour is reachable but never relays.
//
// The host runs a per-root SPF kernel for a vertex cover S of the graph and
// derives every other root (an independent set I: all neighbours of a leaf
// are in S) here. On the fabric, I = the 85,488 rack switches (8 fabric
// switches each) and S = the 14,536 fabric and spine switches.
//
// Shape. Block = a group of up to kWdG roots x a chunk of 256-node subtiles;
// lane = 4 consecutive nodes (16-B loads of each neighbour row, 16-B stores of
// dist and next-hop rows: a wave writes 1 KB of each row per instruction).
// Consecutive roots with the same neighbour slots (the racks of one pod, when
// the host orders roots by neighbourhood) form a run: the subtile's neighbour
// rows are loaded once into registers for the whole run, and each root adds
// only its own link metrics, the compares and the stores. Digests (DESIGN.md
// §4) are summed per (root, subtile) by a wave reduction into LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;
constexpr uint32_t kNt = 0x80000000u;  // slot tag: overloaded neighbour (| its id)
constexpr int kWave = 64;
constexpr uint32_t kBlock = 256;
constexpr uint32_t kWaves = kBlock / kWave;
constexpr uint32_t kSub = 256;  // nodes per wave pass (4 per lane)

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int o) {
  const uint32_t lo = __shfl_xor((uint32_t)x, o, kWave);
  const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), o, kWave);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ bool transit(const DevGraph& g, uint32_t v) {
  return !((g.nt_bits[v >> 5] >> (v & 31)) & 1u);
}
// w + D saturating at kInf (w = kInf: unusable slot; D = kInf: unreached)
__device__ __forceinline__ uint32_t sat_add(uint32_t w, uint32_t D) {
  const uint32_t c = w + D;
  return c < D ? kInf : c;
}

template <int KM>
__global__ void __launch_bounds__(256) wderive_kernel(DevGraph g, WDeriveArgs a) {
  __shared__ uint32_t s_root[kWdG], s_K[kWdG], s_same[kWdG];
  __shared__ uint32_t s_w[kWdG * KM];  // [root][slot] metric of the slot's link (kInf: none up)
  __shared__ uint32_t s_p[kWdG * KM];  // [root][slot] row of n_k | kNt | n_k, kInf: unusable
  __shared__ unsigned long long s_h[kWdG], s_sum[kWdG];
  __shared__ uint32_t s_reach[kWdG];
  __shared__ uint64_t s_wk[256];
  const uint32_t V = g.V, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t G = a.G;
  const uint32_t ngroups = (a.n + G - 1) / G;
  const uint32_t ci = blockIdx.x / ngroups, gi = blockIdx.x % ngroups;
  const uint32_t i0 = gi * G, ng = min(G, a.n - i0);
  // ---- slot tables of the group's roots
  if (tid < ng) {
    const uint32_t r = a.roots[i0 + tid];
    s_root[tid] = r;
    s_K[tid] = 0;
    s_h[tid] = 0ull;
    s_sum[tid] = 0ull;
    s_reach[tid] = 0u;
    if (r >= V) {
      atomicOr(a.err, 64u);
    } else {
      const uint32_t K = g.dn_off[r + 1] - g.dn_off[r];
      if (K > (uint32_t)KM) atomicOr(a.err, 1u);
      s_K[tid] = min(K, (uint32_t)KM);
    }
  }
  for (uint32_t x = tid; x < ng * KM; x += kBlock) s_w[x] = kInf;
  if (a.digest) s_wk[tid] = tid ? digest_word_key(0, tid) : 0ull;
  __syncthreads();
  for (uint32_t j = 0; j < ng; ++j) {  // the root's up links: smallest metric per slot
    const uint32_t r = s_root[j];
    if (r >= V) continue;
    for (uint32_t e = g.row_ptr[r] + tid; e < g.row_ptr[r + 1]; e += kBlock) {
      const uint32_t cx = g.colx[e];
      if ((cx & kDown) || cx == r) continue;
      const uint32_t k = g.didx[e];
      if (k < s_K[j]) atomicMin(&s_w[j * KM + k], a.hop ? 1u : g.w[e]);
    }
  }
  __syncthreads();
  for (uint32_t x = tid; x < ng * KM; x += kBlock) {
    const uint32_t j = x / KM, k = x - j * KM;
    uint32_t p = kInf;
    if (k < s_K[j] && s_w[x] != kInf) {
      const uint32_t nb = g.dn[g.dn_off[s_root[j]] + k];
      if (transit(g, nb)) {
        p = a.pos[nb];
        if (p == kInf) atomicOr(a.err, 16u);
      } else {
        p = kNt | nb;
      }
    }
    s_p[x] = p;
  }
  __syncthreads();
  if (tid < ng) {  // a run continues while the neighbour slots stay the same
    uint32_t same = tid > 0 && s_K[tid] == s_K[tid - 1];
    for (uint32_t k = 0; same && k < (uint32_t)KM; ++k)
      same = s_p[tid * KM + k] == s_p[(tid - 1) * KM + k];
    s_same[tid] = same;
  }
  __syncthreads();
  // ---- subtiles
  const bool vec = a.vec != 0;
  const uint32_t t0 = ci * a.ctiles, t1 = min(a.tiles, t0 + a.ctiles);
  for (uint32_t t = t0 + wave; t < t1; t += kWaves) {
    const uint32_t v0 = t * kSub + 4u * lane;
    const bool full = v0 + 4u <= V;
    uint64_t dk[4], nk[4];
    if (a.digest) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t v = min(v0 + b, V - 1u);
        dk[b] = g.dkey[2ull * v];
        nk[b] = g.dkey[2ull * v + 1];
      }
    }
    uint32_t D[KM][4];
    for (uint32_t j = 0; j < ng; ++j) {
      const uint32_t r = s_root[j];
      if (r >= V) continue;
      const uint32_t* sp = s_p + j * KM;
      const uint32_t* sw = s_w + j * KM;
      if (!s_same[j]) {  // a new run: load its neighbour rows for this subtile
#pragma unroll
        for (int k = 0; k < KM; ++k) {
          const uint32_t p = sp[k];  // uniform across the wave
          if (p < kNt) {
            const uint32_t* row = a.src + (size_t)p * a.src_pitch;
            if (vec && full) {
              const uint4 x = *reinterpret_cast<const uint4*>(row + v0);
              D[k][0] = x.x; D[k][1] = x.y; D[k][2] = x.z; D[k][3] = x.w;
            } else {
#pragma unroll
              for (int b = 0; b < 4; ++b) D[k][b] = v0 + b < V ? row[v0 + b] : kInf;
            }
          } else if (p != kInf) {  // overloaded neighbour: reachable, never relays
#pragma unroll
            for (int b = 0; b < 4; ++b) D[k][b] = (v0 + b == (p & ~kNt)) ? 0u : kInf;
          } else {
#pragma unroll
            for (int b = 0; b < 4; ++b) D[k][b] = kInf;
          }
        }
      }
      uint32_t m[4] = {kInf, kInf, kInf, kInf};
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const uint32_t w = sw[k];
#pragma unroll
        for (int b = 0; b < 4; ++b) m[b] = min(m[b], sat_add(w, D[k][b]));
      }
      uint32_t bits[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const uint32_t w = sw[k];
#pragma unroll
        for (int b = 0; b < 4; ++b) bits[b] |= (sat_add(w, D[k][b]) == m[b] ? 1u : 0u) << k;
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if (v0 + b == r) m[b] = 0u;  // the root itself: dist 0, no next hops
        if (m[b] == kInf || v0 + b == r) bits[b] = 0u;
      }
      const size_t i = i0 + j;
      uint32_t* drow = a.dist + i * V;
      uint32_t* nrow = a.nh ? a.nh + i * V : nullptr;
      if (vec && full) {
        store_row16(drow + v0, make_uint4(m[0], m[1], m[2], m[3]));
        if (nrow) store_row16(nrow + v0, make_uint4(bits[0], bits[1], bits[2], bits[3]));
      } else {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (v0 + b < V) {
            drow[v0 + b] = m[b];
            if (nrow) nrow[v0 + b] = bits[b];
          }
        }
      }
      if (a.digest) {
        // reached count in the top byte of the distance sum (a row of 16
        // lanes: <= 64 nodes, sum < 2^38), both summed per row by DPP and
        // added to the root's LDS sums by the row's first lane
        uint64_t h = 0, sr = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (v0 + b < V && m[b] != kInf) {
            sr += (uint64_t)m[b] + (1ull << 56);
            h += dk[b] * ((uint64_t)m[b] + 1ull);
            if (bits[b]) h += nk[b] * (KM <= 8 ? s_wk[bits[b]] : digest_word_key(0, bits[b]));
          }
        }
        h = row_sum64(h);
        sr = row_sum64(sr);
        if ((lane & 15u) == 0 && sr) {
          atomicAdd(&s_h[j], (unsigned long long)h);
          atomicAdd(&s_sum[j], (unsigned long long)(sr & ((1ull << 56) - 1ull)));
          atomicAdd(&s_reach[j], (uint32_t)(sr >> 56));
        }
      }
    }
  }
  if (a.digest) {
    __syncthreads();
    if (tid < ng && s_reach[tid]) {
      ospf_digest* dg = a.digest + i0 + tid;
      atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)s_reach[tid]);
      atomicAdd((unsigned long long*)&dg->sum_dist, s_sum[tid]);
      atomicAdd((unsigned long long*)&dg->hash, s_h[tid]);
    }
  }
}

// Cover roots (up to 128 distinct neighbours, W <= 4 next-hop words): the
// next hops from the neighbours' rows against the root's own row (every row,
// the root's included, in src at pos[]): bit k of v iff w_k + D_k(v) ==
// D_r(v) with n_k transit, or v == n_k and w_k == D_r(v). Block = up to
// kWdWideG roots x a chunk of 256-node subtiles, lane = 4 nodes; the W words
// of the lane's 4 nodes stay in registers and leave through a per-wave LDS
// slice so each store instruction writes 1 KB of consecutive row. The digest
// (dist part from the own row) is summed per (root, subtile).
constexpr uint32_t kWdWideG = 16;
constexpr uint32_t kWdWideK = 128;
// neighbour rows loaded per batch (all in flight before the compares); 16
// measured slower on F100k-w (75.7 vs 49.8 ms: 130 VGPRs, 3 waves per SIMD)
#ifndef OSPF_WIDE_BATCH
#define OSPF_WIDE_BATCH 8
#endif
constexpr uint32_t kWideBatch = OSPF_WIDE_BATCH;
template <int W>
__global__ void __launch_bounds__(256) wderive_wide_kernel(DevGraph g, WDeriveArgs a) {
  __shared__ uint32_t s_root[kWdWideG], s_K[kWdWideG], s_own[kWdWideG];
  __shared__ uint32_t s_w[kWdWideG * kWdWideK];
  __shared__ uint32_t s_p[kWdWideG * kWdWideK];
  __shared__ unsigned long long s_h[kWdWideG], s_sum[kWdWideG];
  __shared__ uint32_t s_reach[kWdWideG];
  __shared__ uint32_t s_st[kWaves][kSub * W];
  const uint32_t V = g.V, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t G = a.G;
  const uint32_t ngroups = (a.n + G - 1) / G;
  const uint32_t ci = blockIdx.x / ngroups, gi = blockIdx.x % ngroups;
  const uint32_t i0 = gi * G, ng = min(G, a.n - i0);
  if (tid < ng) {
    const uint32_t r = a.roots[i0 + tid];
    s_root[tid] = r;
    s_K[tid] = 0;
    s_own[tid] = kInf;
    s_h[tid] = 0ull;
    s_sum[tid] = 0ull;
    s_reach[tid] = 0u;
    if (r >= V) {
      atomicOr(a.err, 64u);
    } else {
      const uint32_t K = g.dn_off[r + 1] - g.dn_off[r];
      if (K > kWdWideK || K > 32u * W) atomicOr(a.err, 1u);
      s_K[tid] = min(K, min(kWdWideK, 32u * W));
      s_own[tid] = a.pos[r];
      if (s_own[tid] == kInf) atomicOr(a.err, 16u);
    }
  }
  for (uint32_t x = tid; x < ng * kWdWideK; x += kBlock) s_w[x] = kInf;
  __syncthreads();
  for (uint32_t j = 0; j < ng; ++j) {
    const uint32_t r = s_root[j];
    if (r >= V) continue;
    for (uint32_t e = g.row_ptr[r] + tid; e < g.row_ptr[r + 1]; e += kBlock) {
      const uint32_t cx = g.colx[e];
      if ((cx & kDown) || cx == r) continue;
      const uint32_t k = g.didx[e];
      if (k < s_K[j]) atomicMin(&s_w[j * kWdWideK + k], a.hop ? 1u : g.w[e]);
    }
  }
  __syncthreads();
  for (uint32_t x = tid; x < ng * kWdWideK; x += kBlock) {
    const uint32_t j = x / kWdWideK, k = x - j * kWdWideK;
    uint32_t p = kInf;
    if (k < s_K[j] && s_w[x] != kInf) {
      const uint32_t nb = g.dn[g.dn_off[s_root[j]] + k];
      if (transit(g, nb)) {
        p = a.pos[nb];
        if (p == kInf) atomicOr(a.err, 16u);
      } else {
        p = kNt | nb;
      }
    }
    s_p[x] = p;
  }
  __syncthreads();
  const bool vec = a.vec != 0;
  const uint32_t t0 = ci * a.ctiles, t1 = min(a.tiles, t0 + a.ctiles);
  uint32_t* st = s_st[wave];
  for (uint32_t pr = wave; pr < (t1 - t0) * ng; pr += kWaves) {
    const uint32_t t = t0 + pr / ng, j = pr % ng;
    const uint32_t r = s_root[j], own = s_own[j];
    if (r >= V || own == kInf) continue;
    const uint32_t v0 = t * kSub + 4u * lane;
    const bool full = v0 + 4u <= V;
    auto load4 = [&](uint32_t p, uint32_t* D) {
      const uint32_t* row = a.src + (size_t)p * a.src_pitch;
      if (vec && full) {
        const uint4 x = *reinterpret_cast<const uint4*>(row + v0);
        D[0] = x.x; D[1] = x.y; D[2] = x.z; D[3] = x.w;
      } else {
#pragma unroll
        for (int b = 0; b < 4; ++b) D[b] = v0 + b < V ? row[v0 + b] : kInf;
      }
    };
    uint32_t R[4];
    load4(own, R);
    uint32_t word[W][4];
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int b = 0; b < 4; ++b) word[w][b] = 0u;
    const uint32_t* sp = s_p + j * kWdWideK;
    const uint32_t* sw = s_w + j * kWdWideK;
    const uint32_t K = s_K[j];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      for (uint32_t k8 = 0; k8 < 32u; k8 += kWideBatch) {
        const uint32_t kb = 32u * w + k8;
        if (kb >= K) break;  // uniform
        uint32_t D[kWideBatch][4], pk[kWideBatch], wk[kWideBatch];
#pragma unroll
        for (int kk = 0; kk < (int)kWideBatch; ++kk) {  // kWideBatch rows in flight
          pk[kk] = kb + kk < K ? sp[kb + kk] : kInf;
          wk[kk] = kb + kk < K ? sw[kb + kk] : kInf;
          if (pk[kk] < kNt) load4(pk[kk], D[kk]);
          else {
#pragma unroll
            for (int b = 0; b < 4; ++b)
              D[kk][b] = (pk[kk] != kInf && v0 + b == (pk[kk] & ~kNt)) ? 0u : kInf;
          }
        }
#pragma unroll
        for (int kk = 0; kk < (int)kWideBatch; ++kk) {
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            // w + D == R without the saturating add: R >= D and R - D == w
            // (an unreached R clears the words below)
            word[w][b] |= (R[b] >= D[kk][b] && R[b] - D[kk][b] == wk[kk] ? 1u : 0u) << (k8 + kk);
          }
        }
      }
    }
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (v0 + b == r || R[b] == kInf)
#pragma unroll
        for (int w = 0; w < W; ++w) word[w][b] = 0u;  // the root / unreached: no next hops
    // stage [node][word] and store whole 1-KB pieces of the row
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int w = 0; w < W; ++w) st[(4u * lane + b) * W + w] = word[w][b];
    __builtin_amdgcn_wave_barrier();
    const size_t i = i0 + j;
    uint32_t* dst = a.nh + ((size_t)i * V + t * kSub) * W;
    const uint32_t tn = min(kSub, V - t * kSub);
    if (vec && tn == kSub) {
#pragma unroll
      for (int x = 0; x < W; ++x)
        store_row16(reinterpret_cast<uint4*>(dst) + x * 64 + lane,
                    reinterpret_cast<const uint4*>(st)[x * 64 + lane]);
    } else {
      for (uint32_t x = lane; x < tn * W; x += 64u) dst[x] = st[x];
    }
    __builtin_amdgcn_wave_barrier();
    if (a.digest) {
      uint64_t h = 0, sum = 0;
      uint32_t reach = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t v = v0 + b;
        if (v < V && R[b] != kInf) {
          reach += 1u;
          sum += R[b];
          h += g.dkey[2ull * v] * ((uint64_t)R[b] + 1ull);
          uint64_t ws = 0;
#pragma unroll
          for (int w = 0; w < W; ++w)
            if (word[w][b]) ws += digest_word_key(w, word[w][b]);
          if (ws) h += g.dkey[2ull * v + 1] * ws;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        h += shfl_xor64(h, o);
        sum += shfl_xor64(sum, o);
        reach += __shfl_xor(reach, o, kWave);
      }
      if (lane == 0 && reach) {
        atomicAdd(&s_h[j], (unsigned long long)h);
        atomicAdd(&s_sum[j], (unsigned long long)sum);
        atomicAdd(&s_reach[j], reach);
      }
    }
  }
  if (a.digest) {
    __syncthreads();
    if (tid < ng && s_reach[tid]) {
      ospf_digest* dg = a.digest + i0 + tid;
      atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)s_reach[tid]);
      atomicAdd((unsigned long long*)&dg->sum_dist, s_sum[tid]);
      atomicAdd((unsigned long long*)&dg->hash, s_h[tid]);
    }
  }
}

// Cover roots with more than 128 neighbours (W > 4 words: the spines of a
// fabric, whose neighbours are one switch per pod). Lane = next-hop word w
// (slots 32 w .. 32 w + 31), a wave walks 2-node chunks of the block's tile;
// a run of consecutive roots with the same neighbour list (the spines of one
// plane) loads each chunk's slot values once and every root of the run adds
// its own link metrics (u16 in LDS) and compares with its own row (staged per
// tile). Per-root digest sums stay in registers until the block ends.
constexpr uint32_t kWlG = 8;
constexpr uint32_t kWlK = 2048;
constexpr uint32_t kWlTile = 256;
// slot k of a root's metric table sits at (k % 32) * 64 + k / 32: lane w reads
// its slots 32 w + i at i * 64 + w, consecutive lanes consecutive u16s (the
// k-major table put every lane of a read on two banks)
__device__ __forceinline__ uint32_t widx(uint32_t k) { return (k & 31u) * 64u + (k >> 5); }
template <uint32_t NC>  // nodes per chunk: 2 (8-B loads) or 4 (16-B loads)
__global__ void __launch_bounds__(256) wderive_lanes_kernel(DevGraph g, WDeriveArgs a) {
  __shared__ uint32_t s_pos[kWlK];
  __shared__ uint16_t s_w[kWlG][kWlK];
  __shared__ uint32_t s_R[kWlG][kWlTile];
  __shared__ uint32_t s_root[kWlG], s_K[kWlG], s_own[kWlG], s_same[kWlG];
  __shared__ unsigned long long s_h[kWlG], s_sum[kWlG];
  __shared__ uint32_t s_reach[kWlG];
  const uint32_t V = g.V, W = a.W, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t G = kWlG;
  const uint32_t ngroups = (a.n + G - 1) / G;
  const uint32_t ci = blockIdx.x / ngroups, rr = blockIdx.x % ngroups;
  const uint32_t full = ngroups / 8u * 8u;  // runs of groups on one XCD (block b on XCD b % 8)
  const uint32_t gi = rr < full ? (rr % 8u) * (full / 8u) + rr / 8u : rr;
  const uint32_t i0 = gi * G, ng = min(G, a.n - i0);
  if (tid < ng) {
    const uint32_t r = a.roots[i0 + tid];
    s_root[tid] = r;
    s_own[tid] = kInf;
    s_K[tid] = 0;
    s_h[tid] = 0ull;
    s_sum[tid] = 0ull;
    s_reach[tid] = 0u;
    if (r >= V) {
      atomicOr(a.err, 64u);
    } else {
      const uint32_t K = g.dn_off[r + 1] - g.dn_off[r];
      if (K > kWlK || K > 32u * W) atomicOr(a.err, 1u);
      s_K[tid] = min(K, min(kWlK, 32u * W));
      s_own[tid] = a.pos[r];
      if (s_own[tid] == kInf) atomicOr(a.err, 16u);
    }
  }
  for (uint32_t x = tid; x < ng * kWlK; x += kBlock) s_w[x / kWlK][x % kWlK] = 0xFFFFu;
  __syncthreads();
  if (tid < ng)
    s_same[tid] = tid > 0 && s_own[tid] != kInf && s_own[tid - 1] != kInf &&
                  s_K[tid] == s_K[tid - 1];
  for (uint32_t j = 0; j < ng; ++j) {  // the root's up links: smallest metric per slot
    const uint32_t r = s_root[j];
    if (r >= V || s_own[j] == kInf) continue;
    for (uint32_t e = g.row_ptr[r] + tid; e < g.row_ptr[r + 1]; e += kBlock) {
      const uint32_t cx = g.colx[e];
      if ((cx & kDown) || cx == r) continue;
      const uint32_t k = g.didx[e];
      if (k >= s_K[j]) continue;
      // u16 slot table: a metric above 65534 cannot be represented, and is
      // reported (error bit 512) rather than clamped silently
      if (!a.hop && g.w[e] > 0xFFFEu) atomicOr(a.err, 512u);
      const uint32_t w = a.hop ? 1u : min(g.w[e], 0xFFFEu);
      // 16-bit min through the aligned 32-bit word
      const uint32_t ix = widx(k);
      uint32_t* wp = reinterpret_cast<uint32_t*>(&s_w[j][ix & ~1u]);
      const uint32_t sh = 16u * (ix & 1u);
      uint32_t cw = *wp;
      while (true) {
        if (w >= ((cw >> sh) & 0xFFFFu)) break;
        const uint32_t nw = (cw & ~(0xFFFFu << sh)) | (w << sh);
        const uint32_t prev = atomicCAS(wp, cw, nw);
        if (prev == cw) break;
        cw = prev;
      }
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
  uint64_t h[kWlG];
#pragma unroll
  for (int j = 0; j < (int)kWlG; ++j) h[j] = 0ull;
  const uint32_t t0 = ci * a.ctiles, t1 = min(a.tiles, t0 + a.ctiles);
  for (uint32_t j0 = 0; j0 < ng;) {
    uint32_t j1 = j0 + 1;
    while (j1 < ng && s_same[j1]) ++j1;
    const uint32_t K = s_K[j0];
    if (s_own[j0] == kInf) {
      j0 = j1;
      continue;
    }
    for (uint32_t k = tid; k < K; k += kBlock) {  // slot rows of the run
      bool used = false;
      for (uint32_t j = j0; j < j1 && !used; ++j) used = s_w[j][widx(k)] != 0xFFFFu;
      uint32_t p = kInf;
      if (used) {
        const uint32_t nb = g.dn[g.dn_off[s_root[j0]] + k];
        if (transit(g, nb)) {
          p = a.pos[nb];
          if (p == kInf) atomicOr(a.err, 16u);
        } else {
          p = kNt | nb;
        }
      }
      s_pos[k] = p;
    }
    for (uint32_t t = t0; t < t1; ++t) {
      const uint32_t v0 = t * kWlTile;
      __syncthreads();  // s_pos written / the previous tile's s_R consumed
      for (uint32_t x = tid; x < (j1 - j0) * kWlTile; x += kBlock) {
        const uint32_t j = x / kWlTile, v = v0 + (x % kWlTile);
        s_R[j][x % kWlTile] = v < V ? a.src[(size_t)s_own[j0 + j] * a.src_pitch + v] : kInf;
      }
      __syncthreads();
      for (uint32_t c = wave; c < kWlTile / NC; c += kWaves) {
        const uint32_t vc = v0 + NC * c;
        if (vc >= V) break;  // wave-uniform
        uint32_t D[NC][32];
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          const uint32_t k = 32u * lane + i;
          const uint32_t p = (lane < W && k < K) ? s_pos[k] : kInf;
          if (p < kNt) {
            const uint32_t* row = a.src + (size_t)p * a.src_pitch + vc;
            if (a.vec && vc + NC - 1u < V) {
              if constexpr (NC == 4) {
                const uint4 x = *reinterpret_cast<const uint4*>(row);
                D[0][i] = x.x;
                D[1][i] = x.y;
                D[2][i] = x.z;
                D[3][i] = x.w;
              } else {
                const uint2 x = *reinterpret_cast<const uint2*>(row);
                D[0][i] = x.x;
                D[1][i] = x.y;
              }
            } else {
#pragma unroll
              for (uint32_t n = 0; n < NC; ++n) D[n][i] = vc + n < V ? row[n] : kInf;
            }
          } else {
#pragma unroll
            for (uint32_t n = 0; n < NC; ++n)
              D[n][i] = (p != kInf && vc + n == (p & ~kNt)) ? 0u : kInf;
          }
        }
        uint64_t kn[NC], kd[NC];
#pragma unroll
        for (uint32_t n = 0; n < NC; ++n) {
          kn[n] = kd[n] = 0ull;
          if (a.digest && vc + n < V) {
            kd[n] = g.dkey[2ull * (vc + n)];
            kn[n] = g.dkey[2ull * (vc + n) + 1];
          }
        }
#pragma unroll
        for (int jj = 0; jj < (int)kWlG; ++jj) {
          const uint32_t j = (uint32_t)jj;
          if (j < j0 || j >= j1) continue;  // uniform
          uint32_t R[NC], wd[NC];
#pragma unroll
          for (uint32_t n = 0; n < NC; ++n) {
            R[n] = s_R[j - j0][NC * c + n];
            wd[n] = 0u;
          }
#pragma unroll
          for (int i = 0; i < 32; ++i) {
            const uint32_t k = 32u * lane + i;
            const uint32_t wk = (lane < W && k < K) ? (uint32_t)s_w[j][i * 64u + lane] : 0xFFFFu;
            const uint32_t wv = wk == 0xFFFFu ? kInf : wk;
#pragma unroll
            for (uint32_t n = 0; n < NC; ++n)
              wd[n] |= (R[n] >= D[n][i] && R[n] - D[n][i] == wv ? 1u : 0u) << i;
          }
          const uint32_t r = s_root[j];
#pragma unroll
          for (uint32_t n = 0; n < NC; ++n)
            if (R[n] == kInf || vc + n == r) wd[n] = 0u;
          uint32_t* dst = a.nh + ((size_t)(i0 + j) * V + vc) * W + lane;
          if (lane < W) {
#pragma unroll
            for (uint32_t n = 0; n < NC; ++n)
              if (vc + n < V) __builtin_nontemporal_store(wd[n], dst + (size_t)n * W);
          }
          if (a.digest) {
#pragma unroll
            for (uint32_t n = 0; n < NC; ++n)
              if (wd[n]) h[jj] += kn[n] * digest_word_key(lane, wd[n]);
            if (lane == 0) {
              uint64_t hx = 0, sx = 0;
              uint32_t rc = 0;
#pragma unroll
              for (uint32_t n = 0; n < NC; ++n)
                if (vc + n < V && R[n] != kInf) {
                  hx += kd[n] * ((uint64_t)R[n] + 1ull);
                  sx += R[n];
                  ++rc;
                }
              h[jj] += hx;
              if (rc) {
                atomicAdd(&s_sum[j], (unsigned long long)sx);
                atomicAdd(&s_reach[j], rc);
              }
            }
          }
        }
      }
    }
    j0 = j1;
    __syncthreads();  // s_pos is rewritten by the next run
  }
  if (a.digest) {
#pragma unroll
    for (int jj = 0; jj < (int)kWlG; ++jj) {
      uint64_t x = h[jj];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) x += shfl_xor64(x, o);
      if (lane == 0 && x) atomicAdd(&s_h[jj], (unsigned long long)x);
    }
    __syncthreads();
    if (tid < ng && s_reach[tid]) {
      ospf_digest* dg = a.digest + i0 + tid;
      atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)s_reach[tid]);
      atomicAdd((unsigned long long*)&dg->sum_dist, s_sum[tid]);
      atomicAdd((unsigned long long*)&dg->hash, s_h[tid]);
    }
  }
}

__global__ void __launch_bounds__(256) wnh_runs_kernel(DevGraph g, WRunsPlan p) {
  __shared__ uint32_t s_R[kWrRun][kWrTile];
  __shared__ unsigned long long s_h[kWrRun], s_sum[kWrRun];
  __shared__ uint32_t s_reach[kWrRun];
  const uint32_t V = g.V, W = p.W, tid = threadIdx.x, lane = tid & 63u;
  // wave-uniform (scalar loads of the slot and metric tables)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t b = blockIdx.x, nb = gridDim.x, full = nb / 8u * 8u;
  const uint32_t item = b < full ? (b % 8u) * (full / 8u) + b / 8u : b;
  const uint32_t ri = item % p.nruns, tile = item / p.nruns;
  const uint4 rn = p.run[ri];
  const uint32_t nr = rn.y, v0 = tile * kWrTile, v = v0 + lane;
  if (tid < nr) {
    s_h[tid] = 0ull;
    s_sum[tid] = 0ull;
    s_reach[tid] = 0u;
  }
  __syncthreads();
  for (uint32_t x = tid; x < nr * kWrTile; x += 256u) {
    const uint32_t j = x / kWrTile, vv = v0 + (x % kWrTile);
    const uint32_t R = vv < V ? p.src[(size_t)p.own[rn.x + j] * p.pitch + vv] : kInf;
    s_R[j][x % kWrTile] = R;
    if (p.digest && R != kInf) {
      atomicAdd(&s_reach[j], 1u);
      atomicAdd(&s_sum[j], (unsigned long long)R);
      atomicAdd(&s_h[j], (unsigned long long)(g.dkey[2ull * vv] * ((uint64_t)R + 1ull)));
    }
  }
  __syncthreads();
  const uint64_t nkey = (p.digest && v < V) ? g.dkey[2ull * v + 1] : 0ull;
  for (uint32_t w = wave; w < W; w += 4u) {
    const uint32_t slv = lane < 32u ? p.slots[rn.z + 32u * w + lane] : kInf;
    uint32_t D[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint32_t sv = (uint32_t)__builtin_amdgcn_readlane((int)slv, i);
      if (sv < kNt) D[i] = v < V ? p.src[(size_t)sv * p.pitch + v] : kInf;
      else D[i] = (sv != kInf && v == (sv & ~kNt)) ? 0u : kInf;
    }
    const uint32_t* wrow = p.wt + (size_t)rn.x * 32u * W + 32u * w + lane;
    uint32_t wnext = lane < 32u ? wrow[0] : 0u;  // root j + 1's metrics load while j computes
    for (uint32_t j = 0; j < nr; ++j) {
      const uint32_t R = s_R[j][lane];
      const uint32_t wtv = wnext;
      if (j + 1u < nr) wnext = lane < 32u ? wrow[(size_t)(j + 1u) * 32u * W] : 0u;
      uint32_t word = 0u;
#pragma unroll
      for (int i = 0; i < 32; ++i) {  // w + D == R without overflow: R >= D, R - D == w
        const uint32_t wk = (uint32_t)__builtin_amdgcn_readlane((int)wtv, i);
        word |= (R >= D[i] && R - D[i] == wk ? 1u : 0u) << i;
      }
      if (R == kInf || v == p.rootid[rn.x + j]) word = 0u;
      if (v < V) __builtin_nontemporal_store(word, p.nh + ((size_t)(rn.x + j) * V + v) * W + w);
      if (p.digest && __ballot(word != 0u)) {
        uint64_t h = word ? nkey * digest_word_key(w, word) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) h += shfl_xor64(h, o);
        if (lane == 0) atomicAdd(&s_h[j], (unsigned long long)h);
      }
    }
  }
  if (p.digest) {
    __syncthreads();
    if (tid < nr && s_reach[tid]) {
      ospf_digest* dg = p.digest + rn.x + tid;
      atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)s_reach[tid]);
      atomicAdd((unsigned long long*)&dg->sum_dist, s_sum[tid]);
      atomicAdd((unsigned long long*)&dg->hash, s_h[tid]);
    } else if (tid < nr && s_h[tid]) {
      atomicAdd((unsigned long long*)&p.digest[rn.x + tid].hash, s_h[tid]);
    }
  }
}

// Block = (chunk of tchunk 64-node tiles, chunk of gchunk groups), 512
// threads; blocks of one tile chunk are spread over the XCDs in order, so the
// hub rows of a tile are read from one XCD's L2 by its resident blocks. One
// LDS row array: the hub rows, the group's rows (an overloaded neighbour's
// row is 0 at itself only), one unreached row -- every slot a single LDS read,
// no branch on the slot kind.
template <int W>
__global__ void __launch_bounds__(512) wnh_hub_kernel(DevGraph g, HubPlan p) {
  extern __shared__ uint32_t s_rows[];  // [nhub + kHubLoc + 1][64]
  __shared__ unsigned long long s_h[512], s_sum[512];
  __shared__ uint32_t s_reach[512];
  const uint32_t V = g.V, tid = threadIdx.x, lane = tid & 63u;
  // wave-uniform: a root's slot table and metrics by scalar loads
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t b = blockIdx.x, nb = gridDim.x, full = nb / 8u * 8u;
  const uint32_t item = b < full ? (b % 8u) * (full / 8u) + b / 8u : b;
  const uint32_t ngc = (p.ngroups + p.gchunk - 1) / p.gchunk;
  const uint32_t tc = item / ngc, gc = item % ngc;
  const uint32_t g0 = gc * p.gchunk, g1 = min(p.ngroups, g0 + p.gchunk);
  const uint32_t r0 = p.grp[g0].x;
  const uint32_t nrb = p.grp[g1 - 1].x + p.grp[g1 - 1].y - r0;  // roots of the block (<= 512)
  uint32_t* s_loc = s_rows + (size_t)p.nhub * kHubTile;
  for (uint32_t x = tid; x < nrb; x += 512u) {
    s_h[x] = 0ull;
    s_sum[x] = 0ull;
    s_reach[x] = 0u;
  }
  if (tid < kHubTile) s_loc[kHubLoc * kHubTile + tid] = kInf;  // the unreached row
  const uint32_t t0 = tc * p.tchunk, t1 = min(p.tiles, t0 + p.tchunk);
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t v0 = t * kHubTile, v = v0 + lane;
    __syncthreads();  // the previous tile's hub rows are consumed
    for (uint32_t x = tid; x < p.nhub * kHubTile; x += 512u) {
      const uint32_t vv = v0 + (x % kHubTile);
      s_rows[x] = vv < V ? p.src[(size_t)p.hub[x / kHubTile] * p.pitch + vv] : kInf;
    }
    const uint64_t dk0 = v < V ? g.dkey[2ull * v] : 0ull, dk1 = v < V ? g.dkey[2ull * v + 1] : 0ull;
    for (uint32_t gi = g0; gi < g1; ++gi) {
      const uint4 gr = p.grp[gi];
      __syncthreads();  // the previous group's rows are consumed (and the hub staged)
      for (uint32_t x = tid; x < gr.w * kHubTile; x += 512u) {
        const uint32_t vv = v0 + (x % kHubTile), lr = p.loc[gr.z + x / kHubTile];
        uint32_t d = kInf;
        if (lr < kNt) d = vv < V ? p.src[(size_t)lr * p.pitch + vv] : kInf;
        else if (vv == (lr & ~kNt)) d = 0u;
        s_loc[x] = d;
      }
      __syncthreads();
      for (uint32_t j = wave; j < gr.y; j += 8u) {
        const uint32_t ri = gr.x + j;
        const uint32_t R = s_rows[p.ownl[ri] * kHubTile + lane];
        const uint32_t* rf = p.ref + (size_t)ri * 32u * W;
        const uint32_t* wt = p.wt + (size_t)ri * 32u * W;
        uint32_t word[W], rvs[W], wvs[W];
        // the words' 32 slot refs / metrics: coalesced loads, all in flight,
        // then read lane by lane into scalar registers
#pragma unroll
        for (int w = 0; w < W; ++w) {
          rvs[w] = lane < 32u ? rf[32 * w + lane] : 0u;
          wvs[w] = lane < 32u ? wt[32 * w + lane] : 0u;
        }
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const uint32_t rv = rvs[w], wv = wvs[w];
          uint32_t x = 0u;
#pragma unroll
          for (int i = 0; i < 32; ++i) {
            const uint32_t ri_ = (uint32_t)__builtin_amdgcn_readlane((int)rv, i);
            const uint32_t wk = (uint32_t)__builtin_amdgcn_readlane((int)wv, i);
            const uint32_t D = s_rows[ri_ * kHubTile + lane];
            x |= (R >= D && R - D == wk ? 1u : 0u) << i;
          }
          word[w] = x;
        }
        if (R == kInf || v == p.rootid[ri]) {
#pragma unroll
          for (int w = 0; w < W; ++w) word[w] = 0u;
        }
        if (v < V) {
          uint32_t* dst = p.nh + ((size_t)ri * V + v) * W;
#pragma unroll
          for (int w = 0; w < W; ++w) __builtin_nontemporal_store(word[w], dst + w);
        }
        if (p.digest) {
          uint64_t h = 0ull, sum = 0ull;
          uint32_t reach = 0u;
          if (v < V && R != kInf) {
            reach = 1u;
            sum = R;
            h = dk0 * ((uint64_t)R + 1ull);
            uint64_t ws = 0ull;
#pragma unroll
            for (int w = 0; w < W; ++w)
              if (word[w]) ws += digest_word_key((uint32_t)w, word[w]);
            h += dk1 * ws;
          }
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            h += shfl_xor64(h, o);
            sum += shfl_xor64(sum, o);
            reach += __shfl_xor(reach, o, kWave);
          }
          if (lane == 0 && reach) {
            s_h[ri - r0] += h;  // one wave per root at a time
            s_sum[ri - r0] += sum;
            s_reach[ri - r0] += reach;
          }
        }
      }
    }
  }
  if (p.digest) {
    __syncthreads();
    for (uint32_t x = tid; x < nrb; x += 512u) {
      if (!s_reach[x]) continue;
      ospf_digest* dg = p.digest + r0 + x;
      atomicAdd((unsigned long long*)&dg->reached, (unsigned long long)s_reach[x]);
      atomicAdd((unsigned long long*)&dg->sum_dist, s_sum[x]);
      atomicAdd((unsigned long long*)&dg->hash, s_h[x]);
    }
  }
}

}  // namespace

hipError_t launch_wnh_hub(const DevGraph& g, const HubPlan& p, hipStream_t s) {
  if (p.ngroups == 0) return hipSuccess;
  if (p.nhub > kHubMax || p.W == 0 || p.W > 4) return hipErrorInvalidValue;
  if (p.digest) {
    const hipError_t e = ospf::zero_async(p.digest, (size_t)p.nroots * sizeof(ospf_digest), s);
    if (e != hipSuccess) return e;
  }
  const size_t lds = (size_t)(p.nhub + kHubLoc + 1u) * kHubTile * 4u;
  const uint32_t ngc = (p.ngroups + p.gchunk - 1) / p.gchunk;
  const dim3 grid(ngc * ((p.tiles + p.tchunk - 1) / p.tchunk));
  const void* fn = p.W == 1 ? (const void*)wnh_hub_kernel<1>
                 : p.W == 2 ? (const void*)wnh_hub_kernel<2>
                 : p.W == 3 ? (const void*)wnh_hub_kernel<3>
                            : (const void*)wnh_hub_kernel<4>;
  if (lds > 48 * 1024) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  switch (p.W) {
    case 1: hipLaunchKernelGGL(wnh_hub_kernel<1>, grid, dim3(512), lds, s, g, p); break;
    case 2: hipLaunchKernelGGL(wnh_hub_kernel<2>, grid, dim3(512), lds, s, g, p); break;
    case 3: hipLaunchKernelGGL(wnh_hub_kernel<3>, grid, dim3(512), lds, s, g, p); break;
    default: hipLaunchKernelGGL(wnh_hub_kernel<4>, grid, dim3(512), lds, s, g, p); break;
  }
  return hipGetLastError();
}

hipError_t launch_wnh_runs(const DevGraph& g, const WRunsPlan& p, hipStream_t s) {
  if (p.nruns == 0) return hipSuccess;
  if (p.digest) {
    const hipError_t e = ospf::zero_async(p.digest, (size_t)p.nroots * sizeof(ospf_digest), s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(wnh_runs_kernel, dim3(p.nruns * p.tiles), dim3(256), 0, s, g, p);
  return hipGetLastError();
}

hipError_t launch_wderive(const DevGraph& g, WDeriveArgs a, uint32_t kmax, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (kmax > kWdMaxK) return hipErrorInvalidValue;
  a.tiles = (g.V + kSub - 1) / kSub;
  if (a.ctiles == 0) a.ctiles = 16;
  a.ctiles = std::min(a.ctiles, a.tiles);
  a.chunks = (a.tiles + a.ctiles - 1) / a.ctiles;
  if (a.G == 0 || a.G > kWdG) a.G = kWdG;
  const dim3 grid(((a.n + a.G - 1) / a.G) * a.chunks);
  if (kmax <= 8) hipLaunchKernelGGL(wderive_kernel<8>, grid, dim3(kBlock), 0, s, g, a);
  else if (kmax <= 16) hipLaunchKernelGGL(wderive_kernel<16>, grid, dim3(kBlock), 0, s, g, a);
  else hipLaunchKernelGGL(wderive_kernel<32>, grid, dim3(kBlock), 0, s, g, a);
  return hipGetLastError();
}

hipError_t launch_wderive_wide(const DevGraph& g, WDeriveArgs a, uint32_t W, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (W == 0 || W > kWlK / 32u) return hipErrorInvalidValue;
  if (W > 4) {  // lane = word, runs of roots with one neighbour list
    a.W = W;
    a.tiles = (g.V + kWlTile - 1) / kWlTile;
    if (a.ctiles == 0) a.ctiles = 4;
    a.ctiles = std::min(a.ctiles, a.tiles);
    a.chunks = (a.tiles + a.ctiles - 1) / a.ctiles;
    const dim3 grid(((a.n + kWlG - 1) / kWlG) * a.chunks);
    // 4 nodes per chunk (16-B loads of each slot row): F100k-w spines 71 -> 40
    // ms in the sweep (OSPF_WL_NC=2: the 8-B form)
    const char* nc = getenv("OSPF_WL_NC");
    if (nc && atoi(nc) == 2) hipLaunchKernelGGL(wderive_lanes_kernel<2>, grid, dim3(kBlock), 0, s, g, a);
    else hipLaunchKernelGGL(wderive_lanes_kernel<4>, grid, dim3(kBlock), 0, s, g, a);
    return hipGetLastError();
  }
  a.tiles = (g.V + kSub - 1) / kSub;
  if (a.ctiles == 0) a.ctiles = 16;
  a.ctiles = std::min(a.ctiles, a.tiles);
  a.chunks = (a.tiles + a.ctiles - 1) / a.ctiles;
  if (a.G == 0 || a.G > kWdWideG) a.G = kWdWideG;
  const dim3 grid(((a.n + a.G - 1) / a.G) * a.chunks);
  switch (W) {
    case 1: hipLaunchKernelGGL(wderive_wide_kernel<1>, grid, dim3(kBlock), 0, s, g, a); break;
    case 2: hipLaunchKernelGGL(wderive_wide_kernel<2>, grid, dim3(kBlock), 0, s, g, a); break;
    case 3: hipLaunchKernelGGL(wderive_wide_kernel<3>, grid, dim3(kBlock), 0, s, g, a); break;
    default: hipLaunchKernelGGL(wderive_wide_kernel<4>, grid, dim3(kBlock), 0, s, g, a); break;
  }
  return hipGetLastError();
}

}  // namespace ospf
