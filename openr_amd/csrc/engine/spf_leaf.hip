// spf_leaf.hip — leaf derive (gfx950): all-sources rows of leaf roots from
// their neighbours' level rows, unit metric / hop count.
//
// A leaf r (an independent set: no two leaves adjacent, <= 32 distinct
// neighbours n_k; on a fabric the racks) has, for every node v != r,
//   dist(r, v) = 1 + min_k dist(n_k, v)     over n_k with an up link r-n_k,
// where a non-transit (overloaded) n_k reaches only itself (dist(n_k, n_k) =
// 0) -- Bellman's equation of LinkState::runSpf over the root's out-links
// (openr/decision/LinkState.cpp:836-911: overloaded nodes never relax,
// :859-866). Its next hops towards v are the n_k whose term is tight
// (:885-901: a next hop lies on a shortest path whose tail from n_k is a
// shortest n_k -> v path; a direct neighbour gets {itself}). So the whole
// row -- level byte, dist, next-hop word -- follows from K level rows; no
// traversal of the leaf's own. One launch writes the three rows and the
// digest, the rows being the only compulsory traffic.
//
// Level bytes are dist + 1 (0x7F = unreached and padding; < 0x80 always),
// four nodes per u32: byte-wise min and equality by SWAR arithmetic with no
// borrow between bytes. Lane = 4 consecutive nodes, wave = 256 nodes (every
// load and store instruction of a wave covers a contiguous 256 B of a level
// row or 1 KB of a dist / next-hop row), block = 4 waves = one 1,024-node
// tile per step over a chunk of tiles, for one group of roots with the same
// slot table (the racks of a pod): the neighbour rows of a tile are read and
// reduced once, then only the rows of each root are stored (its own position
// patched: level 1, dist 0, no next hops).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;
constexpr uint32_t kBlock = 256;
constexpr uint32_t kNoRow = 0x7F7F7F7Fu;

__device__ __forceinline__ bool transit(const DevGraph& g, uint32_t v) {
  return !((g.nt_bits[v >> 5] >> (v & 31)) & 1u);
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int o) {
  const uint32_t lo = __shfl_xor((uint32_t)x, o, 64);
  const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), o, 64);
  return ((uint64_t)hi << 32) | lo;
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

template <int KM, int PD, bool KD = false>
__global__ void __launch_bounds__(kBlock) leaf_derive_kernel(DevGraph g, LeafArgs a) {
  __shared__ uint32_t s_root[kLeafMaxG], s_own[kLeafMaxG], s_use[kLeafMaxG], s_lrow[kLeafMaxG];
  __shared__ uint32_t s_rb[kLeafMaxG], s_re[kLeafMaxG];
  __shared__ uint32_t s_tab[32];
  __shared__ unsigned long long s_dr[kLeafMaxG], s_ds[kLeafMaxG], s_dh[kLeafMaxG];
  __shared__ unsigned long long s_br, s_bs, s_bh;
  __shared__ uint64_t s_wk[256];
  __shared__ uint32_t s_ok;
  const uint32_t V = g.V, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t gr = a.group_major ? blockIdx.x / a.chunks : blockIdx.x % a.ngroups;
  const uint32_t ci = a.group_major ? blockIdx.x % a.chunks : blockIdx.x / a.ngroups;
  const uint32_t i0 = a.grp ? a.grp[gr] : gr;
  const uint32_t ng = a.grp ? min(kLeafMaxG, a.grp[gr + 1] - i0) : 1u;
  if (tid < ng) {
    const uint32_t r = a.roots[i0 + tid];
    s_root[tid] = r;
    s_own[tid] = r < V ? a.pos[r] : kInf;
    s_lrow[tid] = a.levrow ? a.levrow[i0 + tid] : s_own[tid];
    s_use[tid] = 0u;
    s_dr[tid] = s_ds[tid] = s_dh[tid] = 0ull;
    if (r >= V) atomicOr(a.err, 64u);
    else if (s_own[tid] == kInf) atomicOr(a.err, 16u);
  }
  if (tid < 32) s_tab[tid] = kInf;
  if (tid == 0) {
    s_br = s_bs = s_bh = 0ull;
    s_ok = 1u;
  }
  const bool small = KM <= 8;
  if (small && a.digest) s_wk[tid] = tid ? digest_word_key(0, tid) : 0ull;
  __syncthreads();
  // usable slots of every root of the group (bit k: an up link to n_k):
  // (root, entry) pairs spread over the block, padded rows <= 64 entries per
  // root per pass
  if (tid < ng) s_rb[tid] = s_root[tid] < V ? g.row_ptr[s_root[tid]] : 0u;
  if (tid < ng) s_re[tid] = s_root[tid] < V ? g.row_ptr[s_root[tid] + 1] : 0u;
  __syncthreads();
  for (uint32_t x = tid; x < ng * 64u; x += kBlock) {
    const uint32_t j = x >> 6, r = s_root[j];
    for (uint32_t e = s_rb[j] + (x & 63u); e < s_re[j]; e += 64u) {
      const uint32_t cx = g.colx[e];
      if ((cx & kDown) || cx == r) continue;
      const uint32_t k = g.didx[e];
      if (k < 32u) atomicOr(&s_use[j], 1u << k);
    }
  }
  __syncthreads();
  const uint32_t r0 = s_root[0];
  const uint32_t K = r0 < V ? g.dn_off[r0 + 1] - g.dn_off[r0] : 0u;
  // the group must share the slot table: same distinct neighbours, same usable links
  for (uint32_t x = tid; x < ng * 32u; x += kBlock) {
    const uint32_t j = x >> 5, k = x & 31u, r = s_root[j];
    if (r >= V || s_own[j] == kInf) {
      s_ok = 0u;
      continue;
    }
    const uint32_t Kj = g.dn_off[r + 1] - g.dn_off[r];
    if (Kj != K || s_use[j] != s_use[0] ||
        (k < K && g.dn[g.dn_off[r] + k] != g.dn[g.dn_off[r0] + k]))
      s_ok = 0u;
  }
  if (tid < K && tid < 32u && ((s_use[0] >> tid) & 1u)) {
    const uint32_t n = g.dn[g.dn_off[r0] + tid];
    if (transit(g, n)) {
      s_tab[tid] = a.pos[n];
      if (a.pos[n] == kInf) atomicOr(a.err, 16u);
    } else {
      s_tab[tid] = 0x80000000u | n;
    }
  }
  __syncthreads();
  if (K > (uint32_t)KM || !s_ok) {
    if (tid == 0) atomicOr(a.err, K > (uint32_t)KM ? 1u : 128u);
    return;
  }
  uint32_t tab[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) tab[k] = s_tab[k];
  const uint32_t dpitch = a.dpitch ? a.dpitch : V, npitch = a.npitch ? a.npitch : V;
  const bool vec = (V & 3u) == 0 && (dpitch & 3u) == 0 && (npitch & 3u) == 0;
  uint32_t br = 0;
  uint64_t bs = 0, bh = 0;
  const uint32_t t0 = ci * a.ctiles, t1 = min(a.tiles, t0 + a.ctiles);
  // the neighbour words of the next PD tiles are loaded before this tile's
  // stores are issued (PD tiles of loads in flight per wave)
  auto load_x = [&](uint32_t t, uint32_t* x) {
    const uint32_t v0 = t * 1024u + wave * 256u + 4u * lane;
    const bool ok = t < t1 && v0 < a.pitch;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const bool rowk = ok && tab[k] < 0x80000000u;
      x[k] = rowk ? *reinterpret_cast<const uint32_t*>(a.lev + (size_t)tab[k] * a.pitch + v0)
                  : kNoRow;
    }
  };
  // KD: the tile's digest keys (dkey: {dist key, node key} per node, 64 B a
  // lane) one tile ahead, with the neighbour words
  auto load_k = [&](uint32_t t, uint4* k4) {
    const uint32_t v0 = t * 1024u + wave * 256u + 4u * lane;
    const bool ok = a.digest && t < t1 && v0 + 4u <= V;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      k4[q] = ok ? reinterpret_cast<const uint4*>(g.dkey + 2ull * v0)[q] : make_uint4(0u, 0u, 0u, 0u);
  };
  uint32_t xn[PD][KM];
  uint4 kn[KD ? 4 : 1];
#pragma unroll
  for (int d = 0; d < PD; ++d) load_x(t0 + d, xn[d]);
  if constexpr (KD) load_k(t0, kn);
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t v0 = t * 1024u + wave * 256u + 4u * lane;
    uint32_t x[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) x[k] = xn[0][k];
#pragma unroll
    for (int d = 0; d + 1 < PD; ++d)
#pragma unroll
      for (int k = 0; k < KM; ++k) xn[d][k] = xn[d + 1][k];
    load_x(t + PD, xn[PD - 1]);
    uint64_t kdist[4] = {0ull, 0ull, 0ull, 0ull}, knode[4] = {0ull, 0ull, 0ull, 0ull};
    bool kok = false;
    if constexpr (KD) {
      kok = v0 + 4u <= V;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        kdist[q] = ((uint64_t)kn[q].y << 32) | kn[q].x;
        knode[q] = ((uint64_t)kn[q].w << 32) | kn[q].z;
      }
      load_k(t + 1, kn);
    }
    if (v0 >= a.pitch) continue;
    uint32_t m = kNoRow;
#pragma unroll
    for (int k = 0; k < KM; ++k) m = bmin7(m, x[k]);
    // a non-transit neighbour is at level 1 of its own row only
    uint32_t ntb[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      ntb[k] = 0u;
      const uint32_t off = (tab[k] & 0x7FFFFFFFu) - v0;
      if (tab[k] != kInf && tab[k] >= 0x80000000u && off < 4u) {
        ntb[k] = 0x80u << (8u * off);
        m = bmin7(m, (m & ~(0xFFu << (8u * off))) | (1u << (8u * off)));
      }
    }
    const uint32_t reach = ((m ^ kNoRow) + 0x7F7F7F7Fu) & 0x80808080u;  // bit 7: reached
    // L = m + 1 where reached (<= 0x7E: the depth bound keeps levels <= 125)
    const uint32_t L = (m + 0x01010101u) - (((m + 0x01010101u) & 0x80808080u) >> 7);
    // next-hop bits: byte b of A[g] holds the bits of slots 8 g .. 8 g + 7
    uint32_t A[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const uint32_t e = tab[k] < 0x80000000u ? beq7(x[k], m) & reach : ntb[k];
      A[k >> 3] |= (e >> 7) << (k & 7);
    }
    uint32_t word[4], dv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      word[b] = ((A[0] >> (8 * b)) & 0xFFu) | (((A[1] >> (8 * b)) & 0xFFu) << 8) |
                (((A[2] >> (8 * b)) & 0xFFu) << 16) | (((A[3] >> (8 * b)) & 0xFFu) << 24);
      const uint32_t l = (L >> (8 * b)) & 0xFFu;
      dv[b] = l < 0x7Fu ? l - 1u : kInf;
    }
    // base digest terms of the 4 nodes (the same for every root of the group
    // except at the root itself, patched below)
    uint64_t hterm[4] = {0ull, 0ull, 0ull, 0ull};
    if (a.digest) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t v = v0 + b;
        if (v >= V || dv[b] == kInf) continue;
        const uint64_t wk = small ? s_wk[word[b] & 0xFFu]
                                  : (word[b] ? digest_word_key(0, word[b]) : 0ull);
        const uint64_t kdv = (KD && kok) ? kdist[b] : g.dkey[2ull * v];
        const uint64_t knv = (KD && kok) ? knode[b] : g.dkn[v];
        hterm[b] = kdv * (uint64_t)(dv[b] + 1u) + knv * wk;
        br += 1u;
        bs += dv[b];
        bh += hterm[b];
      }
    }
    for (uint32_t j = 0; j < ng; ++j) {
      const uint32_t r = s_root[j], own = s_own[j];
      uint32_t Lj = L, dj[4] = {dv[0], dv[1], dv[2], dv[3]}, wj[4] = {word[0], word[1], word[2], word[3]};
      const uint32_t off = r - v0;
      if (off < 4u) {  // the root itself: level 1, dist 0, no next hops
        Lj = (L & ~(0xFFu << (8u * off))) | (1u << (8u * off));
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if ((uint32_t)b == off) {
            if (a.digest) {
              const uint64_t own_h = g.dkey[2ull * r];
              atomicAdd(&s_dr[j], (unsigned long long)(1u - (dj[b] != kInf ? 1u : 0u)));
              atomicAdd(&s_ds[j], (unsigned long long)(0ull - (dj[b] != kInf ? (uint64_t)dj[b] : 0ull)));
              atomicAdd(&s_dh[j], (unsigned long long)(own_h - hterm[b]));
            }
            dj[b] = 0u;
            wj[b] = 0u;
          }
      }
      const uint32_t lrow = s_lrow[j];
      if (lrow != kInf)
        __builtin_nontemporal_store(Lj, reinterpret_cast<uint32_t*>(a.lev + (size_t)lrow * a.pitch + v0));
      if (v0 >= V) continue;
      uint32_t* nrow = a.nh + (size_t)(i0 + j) * npitch + v0;
      uint32_t* drow = a.dist ? a.dist + (size_t)own * dpitch + v0 : nullptr;
      if (vec) {
        store_row16(nrow, make_uint4(wj[0], wj[1], wj[2], wj[3]));
        if (drow) store_row16(drow, make_uint4(dj[0], dj[1], dj[2], dj[3]));
      } else {
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (v0 + b < V) {
            nrow[b] = wj[b];
            if (drow) drow[b] = dj[b];
          }
      }
    }
  }
  if (a.digest) {
    unsigned long long r64 = br;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      r64 += shfl_xor64(r64, o);
      bs += shfl_xor64(bs, o);
      bh += shfl_xor64(bh, o);
    }
    if (lane == 0) {
      atomicAdd(&s_br, r64);
      atomicAdd(&s_bs, (unsigned long long)bs);
      atomicAdd(&s_bh, (unsigned long long)bh);
    }
    __syncthreads();
    if (tid < ng) {
      ospf_digest* dg = a.digest + i0 + tid;
      atomicAdd((unsigned long long*)&dg->reached, s_br + s_dr[tid]);
      atomicAdd((unsigned long long*)&dg->sum_dist, s_bs + s_ds[tid]);
      atomicAdd((unsigned long long*)&dg->hash, s_bh + s_dh[tid]);
    }
  }
}

}  // namespace

hipError_t launch_leaf_derive(const DevGraph& g, const LeafArgs& a0, uint32_t kmax, hipStream_t s) {
  LeafArgs a = a0;
  a.tiles = (a.pitch + 1023u) / 1024u;
  if (!a.ctiles) {
    // enough blocks to fill the chip many times over: groups x chunks (F100k
    // headline: 8192 -> 32768 blocks took the sweep 22.5 -> 22.0 ms, the
    // shorter chunks even out the per-CU tail; profiles/r05/b20)
    const uint32_t want = 32768u;
    const uint32_t chunks = std::max(1u, std::min(a.tiles, (want + a.ngroups - 1) / a.ngroups));
    a.ctiles = (a.tiles + chunks - 1) / chunks;
  }
  const uint32_t chunks = (a.tiles + a.ctiles - 1) / a.ctiles;
  a.chunks = chunks;
  const dim3 grid(a.ngroups * chunks);
  // two tiles of neighbour loads in flight (OSPF_LEAF_PD=1: one; read per
  // launch for in-process A/B: 19.61 vs 19.71 ms per F100k sweep,
  // profiles/r06/i1_leaf_prefetch_ab.txt)
  const char* pe = getenv("OSPF_LEAF_PD");
  const bool pd2 = !pe || atoi(pe) >= 2;
  // the tile's digest keys one tile ahead with the neighbour words
  // (OSPF_LEAF_KD=0: loaded at the digest terms; 20.26 -> 19.48 ms per F100k
  // sweep in one process, profiles/r06/k3_leaf_key_prefetch_ab.txt)
  const char* ke = getenv("OSPF_LEAF_KD");
  const bool kd = !ke || atoi(ke) != 0;
  if (kmax <= 8) {
    if (pd2 && kd) hipLaunchKernelGGL((leaf_derive_kernel<8, 2, true>), grid, dim3(kBlock), 0, s, g, a);
    else if (pd2) hipLaunchKernelGGL((leaf_derive_kernel<8, 2>), grid, dim3(kBlock), 0, s, g, a);
    else hipLaunchKernelGGL((leaf_derive_kernel<8, 1>), grid, dim3(kBlock), 0, s, g, a);
  } else if (kmax <= 16) {
    hipLaunchKernelGGL((leaf_derive_kernel<16, 1>), grid, dim3(kBlock), 0, s, g, a);
  } else {
    hipLaunchKernelGGL((leaf_derive_kernel<32, 1>), grid, dim3(kBlock), 0, s, g, a);
  }
  return hipGetLastError();
}

}  // namespace ospf
