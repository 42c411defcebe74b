// spf_bfs.hip — unit-metric / hop-count SPF for large graphs (gfx950).
//
// One workgroup per (SPF run, next-hop slice). Same result as
// LinkState::runSpf (openr/decision/LinkState.cpp:836-911) when every usable
// weight is 1 (fabric and grid topologies, or useLinkMetric=false): the
// (dist, name) settle order degenerates to BFS levels, and the ECMP next-hop
// set of a node at level d+1 is the OR over its usable in-edges from transit
// nodes of level d (LinkState.cpp:885-901).
//
// State lives in LDS as three V-bit bitmaps (visited, current level, next
// level) — 37.5 KB at V = 100k — so the per-edge random accesses of the BFS
// hit LDS, not HBM. Each level picks its direction (Beamer-style) from exact
// edge masses:
//   push  (top-down):  frontier nodes scan out-edges, mark unvisited heads;
//   pull  (bottom-up): unvisited nodes scan in-edges for frontier tails.
// Next-hop sets:
//   NH_LDS (root has <= 8 distinct neighbours, e.g. every rack switch): one
//     byte per node in LDS (100 KB at V = 100k); push ORs it forward with
//     32-bit LDS atomics, pull ORs it in registers: one pass per level.
//   otherwise next-hops live in the HBM output row: push marks the next level
//     and a pull over it ORs the tails' words in registers. Rows wider than 4
//     words (a 1,781-port spine has 56) are cut into 4-word slices, one
//     workgroup each: OR is bitwise, so slices are independent runs that share
//     only the (recomputed) traversal. Slice 0 writes dist.
// dist / next-hop rows are written once per node (masked coalesced stores);
// the digest (a sum of per-node and per-(node, next-hop) terms, so slices add
// up) is folded into the same pass.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;
constexpr int kWave = 64;
constexpr uint32_t kCoopDeg = 32;
constexpr uint32_t kSliceWords = 4;

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

template <bool NH_LDS, bool IGN>
struct Bfs {
  const DevGraph& g;
  const RunArgs& a;
  uint32_t root, V, W, nwords;
  uint32_t w0, ws;              // slice: words [w0, w0 + ws) of each row
  bool slice0;
  uint32_t *vis, *cur, *nxt;    // LDS bitmaps
  uint32_t* nhb;                // NH_LDS: one byte per node, packed in words
  uint32_t* nh_out;             // HBM next-hop row base (W words per node)
  uint32_t* plane;              // sliced runs: this slice's [V][4] scratch plane
  uint32_t* dist_out;           // HBM dist row
  const uint32_t* nbr;
  uint32_t nbr_n;
  const uint32_t* ign;
  uint32_t ign_n;

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
  // where the propagation keeps v's next-hop words: the output row (W <= 4)
  // or, for sliced wide rows, a compact 16-B-per-node scratch plane so pulls
  // read whole lines of useful words (copied to the output rows at the end)
  __device__ __forceinline__ uint32_t* row(uint32_t v) const {
    return plane ? plane + (size_t)v * kSliceWords : nh_out + (size_t)v * W + w0;
  }
  __device__ __forceinline__ uint32_t* out_row(uint32_t v) const {
    return nh_out + (size_t)v * W + w0;
  }
  // bit of root-neighbour v inside this slice (>= 32*ws: not in slice)
  __device__ __forceinline__ uint32_t slice_bit(uint32_t v) const {
    return lower_bound_u32(nbr, nbr_n, v) - 32u * w0;
  }

  __device__ __forceinline__ void push_one(uint32_t u, uint32_t e, uint32_t cx, uint32_t nbu) {
    if (!usable(e, cx)) return;
    const uint32_t x = cx;
    if (bit(vis, x)) return;
    // non-returning LDS atomics are fire-and-forget: cheaper than testing
    // the bit first (measured: a read-before-atomic guard cost 14%)
    atomicOr(&nxt[x >> 5], 1u << (x & 31));
    if constexpr (NH_LDS) {
      const uint32_t val = (u == root) ? (1u << slice_bit(x)) : nbu;
      atomicOr(&nhb[x >> 2], val << (8 * (x & 3)));
    }
  }

  // edges [beg, end) of u (a padded row: beg, end multiples of 4), one lane
  // (LANES 1) or the whole wave (LANES 64, lane offset folded into beg),
  // read as uint4 so one load instruction fetches 4 CSR entries
  template <uint32_t LANES>
  __device__ __forceinline__ void push_edges(uint32_t u, uint32_t beg, uint32_t end,
                                             uint32_t nbu) {
    const uint4* q = reinterpret_cast<const uint4*>(g.colx);
    for (uint32_t e = beg; e < end; e += 4 * LANES * 2) {
      const uint4 a = q[e >> 2];
      const bool two = e + 4 * LANES < end;
      const uint4 b = two ? q[(e + 4 * LANES) >> 2] : make_uint4(kDown, kDown, kDown, kDown);
      push_one(u, e, a.x, nbu);
      push_one(u, e + 1, a.y, nbu);
      push_one(u, e + 2, a.z, nbu);
      push_one(u, e + 3, a.w, nbu);
      if (two) {
        const uint32_t f = e + 4 * LANES;
        push_one(u, f, b.x, nbu);
        push_one(u, f + 1, b.y, nbu);
        push_one(u, f + 2, b.z, nbu);
        push_one(u, f + 3, b.w, nbu);
      }
    }
  }

  // v collects next-hops from level-d tails (cur holds only transit nodes);
  // true when it has a tight tail
  __device__ __forceinline__ void pull_one(uint32_t v, uint32_t e, uint32_t cx, uint32_t* acc,
                                           bool& any) const {
    if (!usable(e, cx)) return;
    const uint32_t u = cx;
    if (!bit(cur, u)) return;
    any = true;
    if (u == root) {
      const uint32_t b = slice_bit(v);
      if constexpr (NH_LDS) {
        acc[0] |= 1u << b;
      } else {
#pragma unroll
        for (uint32_t w = 0; w < kSliceWords; ++w)
          acc[w] |= ((b >> 5) == w) ? (1u << (b & 31)) : 0u;
      }
    } else if constexpr (NH_LDS) {
      acc[0] |= nh_byte(u);
    } else {
      const uint32_t* s = row(u);
#pragma unroll
      for (uint32_t w = 0; w < kSliceWords; ++w)
        if (w < ws) acc[w] |= s[w];
    }
  }

  template <uint32_t LANES>
  __device__ __forceinline__ bool pull_edges(uint32_t v, uint32_t beg, uint32_t end,
                                             uint32_t* acc) const {
    bool any = false;
    const uint4* q = reinterpret_cast<const uint4*>(g.colx);
    for (uint32_t e = beg; e < end; e += 4 * LANES * 2) {
      const uint4 a = q[e >> 2];
      const bool two = e + 4 * LANES < end;
      const uint4 b = two ? q[(e + 4 * LANES) >> 2] : make_uint4(kDown, kDown, kDown, kDown);
      pull_one(v, e, a.x, acc, any);
      pull_one(v, e + 1, a.y, acc, any);
      pull_one(v, e + 2, a.z, acc, any);
      pull_one(v, e + 3, a.w, acc, any);
      if (two) {
        const uint32_t f = e + 4 * LANES;
        pull_one(v, f, b.x, acc, any);
        pull_one(v, f + 1, b.y, acc, any);
        pull_one(v, f + 2, b.z, acc, any);
        pull_one(v, f + 3, b.w, acc, any);
      }
    }
    return any;
  }

  __device__ __forceinline__ void store_nh(uint32_t v, const uint32_t* acc) {
    if constexpr (NH_LDS) {
      atomicOr(&nhb[v >> 2], acc[0] << (8 * (v & 3)));
    } else {
      uint32_t* r = row(v);
#pragma unroll
      for (uint32_t w = 0; w < kSliceWords; ++w)
        if (w < ws) r[w] = acc[w];
    }
  }

  // bottom-up over unvisited nodes (PULL_ALL) or over the marked next level
  template <bool PULL_ALL>
  __device__ void pull_level(int lane, int wave, int nwaves) {
    const uint32_t nchunks = (V + 63) / 64;
    for (uint32_t c = wave; c < nchunks; c += nwaves) {
      if (PULL_ALL) {  // skip chunks with every node already visited
        const uint32_t w1 = (c * 2 + 1 < nwords) ? vis[c * 2 + 1] : 0xFFFFFFFFu;
        if ((vis[c * 2] & w1) == 0xFFFFFFFFu) continue;
      } else {
        const uint32_t w1 = (c * 2 + 1 < nwords) ? nxt[c * 2 + 1] : 0u;
        if ((nxt[c * 2] | w1) == 0) continue;
      }
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
        uint32_t acc[kSliceWords] = {0u, 0u, 0u, 0u};
        if (pull_edges<1>(v, beg, end, acc)) {
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
        uint32_t acc[kSliceWords] = {0u, 0u, 0u, 0u};
        const bool any = __ballot(pull_edges<kWave>(bv, bb + 4 * lane, be, acc)) != 0;
#pragma unroll
        for (uint32_t w = 0; w < kSliceWords; ++w) acc[w] = wor(acc[w]);
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
      const uint32_t w1 = (c * 2 + 1 < nwords) ? cur[c * 2 + 1] : 0u;
      if ((cur[c * 2] | w1) == 0) continue;
      const uint32_t v = c * 64 + lane;
      const bool act = v < V && bit(cur, v);
      uint32_t beg = 0, end = 0, nbv = 0;
      if (act) {
        beg = g.row_ptr[v];
        end = g.row_ptr[v + 1];
        if constexpr (NH_LDS) nbv = nh_byte(v);
      }
      const bool big = act && (end - beg) > kCoopDeg;
      if (act && !big) push_edges<1>(v, beg, end, nbv);
      uint64_t bm = __ballot(big);
      while (bm) {
        const int l = __ffsll((unsigned long long)bm) - 1;
        bm &= bm - 1;
        const uint32_t bv = __shfl(v, l, kWave), bb = __shfl(beg, l, kWave),
                       be = __shfl(end, l, kWave), bn = __shfl(nbv, l, kWave);
        push_edges<kWave>(bv, bb + 4 * lane, be, bn);
      }
    }
  }

  // digest terms of the next-hop words of v held by this slice
  __device__ __forceinline__ uint64_t pair_terms(uint32_t v) const {
    if constexpr (NH_LDS) {
      return digest_word_term(v, 0, nh_byte(v));
    } else {
      const uint32_t* r = row(v);
      uint64_t h = 0;
      for (uint32_t w = 0; w < ws; ++w) h += digest_word_term(v, w0 + w, r[w]);
      return h;
    }
  }
};

template <bool NH_LDS, bool IGN>
__device__ void bfs_run(const DevGraph& g, const RunArgs& a, uint32_t* lds, uint32_t rix,
                        uint32_t slice) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
  Bfs<NH_LDS, IGN> b(g, a);
  const uint32_t V = g.V, W = a.W;
  b.root = a.roots[rix];
  b.V = V;
  b.W = W;
  b.nwords = (V + 31) / 32;
  b.w0 = slice * kSliceWords;
  b.ws = min(kSliceWords, W - b.w0);
  b.slice0 = slice == 0;
  const uint32_t bw = (b.nwords + 1) & ~1u;  // even: chunks of two words
  uint32_t* cnt = lds;                        // [0,32) counters
  uint32_t* s_nbr = lds + 32;
  uint32_t* s_ign = s_nbr + a.nbr_cap;
  b.vis = s_ign + a.ign_cap;
  b.cur = b.vis + bw;
  b.nxt = b.cur + bw;
  b.nhb = b.nxt + bw;  // NH_LDS: (V+3)/4 words
  b.nbr = s_nbr;
  b.ign = s_ign;
  b.dist_out = a.dist + (size_t)rix * V;
  b.nh_out = a.nh + (size_t)rix * V * W;
  b.plane = (!NH_LDS && a.slices > 1 && a.planes)
                ? a.planes + ((size_t)rix * a.slices + slice) * V * kSliceWords
                : nullptr;

  const uint32_t nb0 = g.dn_off[b.root];
  b.nbr_n = g.dn_off[b.root + 1] - nb0;
  if (b.nbr_n > 32u * W || b.nbr_n > a.nbr_cap) {
    if (tid == 0) atomicOr(a.err, 1u);
    return;
  }
  if (!b.slice0 && 32u * b.w0 >= b.nbr_n) {
    // slice past the root's last neighbour: its words are all zero
    for (uint32_t v = tid; v < V; v += blockDim.x)
      for (uint32_t w = 0; w < b.ws; ++w) b.out_row(v)[w] = 0u;
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
  } else {
    for (uint32_t w = tid; w < b.ws; w += blockDim.x) b.row(b.root)[w] = 0u;
  }
  if (tid < 32) cnt[tid] = 0u;
  if (tid == 0) {
    if (b.slice0) b.dist_out[b.root] = 0u;
    cnt[4] = g.row_ptr[b.root + 1] - g.row_ptr[b.root];  // level-0 edge mass
  }
  __syncthreads();

  const bool want_dig = a.flags & 8u;
  uint64_t reached = 0, sumd = 0, hsum = 0;
  if (want_dig && tid == 0 && b.slice0) {  // the root itself: dist 0, no next-hops
    reached = 1;
    hsum = digest_node_term(b.root, 0);
  }
  // cnt[1..3]: "level found" ring; cnt[4], cnt[6]: edge mass of levels d, d+1
  uint32_t unvisited_mass = g.E - cnt[4];
  for (uint32_t d = 0;; ++d) {
    const uint32_t front_mass = cnt[4 + (d & 1) * 2];
    // pull when the unvisited edge mass is below what push (+ the follow-up
    // pull when next-hops live in HBM) would scan
    const bool pull_all = NH_LDS ? (unvisited_mass < front_mass)
                                 : (unvisited_mass < 2u * front_mass);
    if (pull_all) {
      b.template pull_level<true>(lane, wave, nwaves);
      __syncthreads();
    } else {
      b.push_level(lane, wave, nwaves);
      __syncthreads();
      if constexpr (!NH_LDS) {
        b.template pull_level<false>(lane, wave, nwaves);
        __syncthreads();
      }
    }
    // new level: write dist (+ digest), count its edge mass
    uint32_t mass = 0;
    bool found = false;
    const uint32_t nchunks = (V + 63) / 64;
    for (uint32_t c = wave; c < nchunks; c += nwaves) {
      const uint32_t w1 = (c * 2 + 1 < b.nwords) ? b.nxt[c * 2 + 1] : 0u;
      if ((b.nxt[c * 2] | w1) == 0) continue;
      const uint32_t v = c * 64 + lane;
      if (v < V && bit(b.nxt, v)) {
        found = true;
        mass += g.row_ptr[v + 1] - g.row_ptr[v];
        if (b.slice0) b.dist_out[v] = d + 1;
        if (want_dig) {
          if (b.slice0) {
            reached += 1;
            sumd += d + 1;
            hsum += digest_node_term(v, d + 1);
          }
          hsum += b.pair_terms(v);
        }
      }
    }
    const uint64_t m64 = wsum((uint64_t)mass);
    const bool any = __ballot(found) != 0;
    if (lane == 0 && m64) atomicAdd(&cnt[4 + ((d + 1) & 1) * 2], (uint32_t)m64);
    if (lane == 0 && any) cnt[1 + (d % 3)] = 1u;
    __syncthreads();
    // roll bitmaps; the next frontier keeps only nodes that may transit
    // (overloaded nodes are reached but never relax, LinkState.cpp:859-866)
    for (uint32_t i = tid; i < bw; i += blockDim.x) {
      const uint32_t n = b.nxt[i];
      b.vis[i] |= n;
      b.cur[i] = (i < b.nwords) ? (n & ~g.nt_bits[i]) : 0u;
      b.nxt[i] = 0u;
    }
    const bool more = cnt[1 + (d % 3)] != 0;
    const uint32_t next_mass = cnt[4 + ((d + 1) & 1) * 2];
    __syncthreads();
    if (tid == 0) {
      cnt[1 + ((d + 1) % 3)] = 0u;
      cnt[4 + (d & 1) * 2] = 0u;  // level d's mass slot is reused by level d+2
    }
    if (!more) break;
    unvisited_mass -= next_mass;
  }
  // epilogue: unreached nodes (dist INF, zero next-hops); NH_LDS row write-out
  const bool want_nh = a.flags & 4u;
  for (uint32_t v = tid; v < V; v += blockDim.x) {
    const bool seen = bit(b.vis, v);
    if (!seen && b.slice0) b.dist_out[v] = kInf;
    if constexpr (NH_LDS) {
      if (want_nh) {
        uint32_t* r = b.row(v);
        r[0] = seen ? b.nh_byte(v) : 0u;
        for (uint32_t w = 1; w < b.ws; ++w) r[w] = 0u;
      }
    } else if (b.plane) {  // copy the compact plane into the output rows
      const uint4 q = seen ? *reinterpret_cast<const uint4*>(b.row(v)) : make_uint4(0, 0, 0, 0);
      uint32_t* r = b.out_row(v);
      const uint32_t qq[4] = {q.x, q.y, q.z, q.w};
      for (uint32_t w = 0; w < b.ws; ++w) r[w] = qq[w];
    } else if (!seen) {
      for (uint32_t w = 0; w < b.ws; ++w) b.row(v)[w] = 0u;
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
      if (a.slices == 1) {
        a.digest[rix] = dg;
      } else {  // slices add into a zeroed record
        atomicAdd((unsigned long long*)&a.digest[rix].reached, (unsigned long long)dg.reached);
        atomicAdd((unsigned long long*)&a.digest[rix].sum_dist, (unsigned long long)dg.sum_dist);
        atomicAdd((unsigned long long*)&a.digest[rix].hash, (unsigned long long)dg.hash);
      }
    }
  }
}

// NHL: LDS holds the byte next-hop array; a run uses it when its root has
// <= 8 distinct neighbours (then it is its own single slice).
template <bool NHL, bool IGN>
__global__ void __launch_bounds__(1024) spf_bfs_kernel(DevGraph g, RunArgs a) {
  extern __shared__ uint32_t lds[];
  const uint32_t rix = blockIdx.x / a.slices, slice = blockIdx.x % a.slices;
  if constexpr (NHL) {
    const uint32_t root = a.roots[rix];
    if (g.dn_off[root + 1] - g.dn_off[root] <= 8) {
      if (slice == 0) {
        bfs_run<true, IGN>(g, a, lds, rix, 0);
      } else {  // words beyond the first slice are zero for such a root
        uint32_t* base = a.nh + (size_t)rix * g.V * a.W;
        const uint32_t w0 = slice * kSliceWords, ws = min(kSliceWords, a.W - w0);
        for (uint32_t v = threadIdx.x; v < g.V; v += blockDim.x)
          for (uint32_t w = 0; w < ws; ++w) base[(size_t)v * a.W + w0 + w] = 0u;
      }
      return;
    }
  }
  bfs_run<false, IGN>(g, a, lds, rix, slice);
}

template <bool NHL, bool IGN>
hipError_t launch_bfs_one(const DevGraph& g, const RunArgs& a, uint32_t n, uint32_t block,
                          size_t lds, hipStream_t s) {
  auto k = spf_bfs_kernel<NHL, IGN>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(n * a.slices), dim3(block), lds, s, g, a);
  return hipGetLastError();
}

}  // namespace

uint32_t bfs_slices(uint32_t W) { return (W + kSliceWords - 1) / kSliceWords; }

hipError_t launch_bfs(bool nh_lds, bool ign, const DevGraph& g, const RunArgs& a, uint32_t n,
                      uint32_t block, size_t lds, hipStream_t s) {
  if (nh_lds) {
    return ign ? launch_bfs_one<true, true>(g, a, n, block, lds, s)
               : launch_bfs_one<true, false>(g, a, n, block, lds, s);
  }
  return ign ? launch_bfs_one<false, true>(g, a, n, block, lds, s)
             : launch_bfs_one<false, false>(g, a, n, block, lds, s);
}

}  // namespace ospf
