// spf_dial.hip — bucketed Dial SSSP (gfx950), variant 6: weighted graphs too
// large for LDS-resident state (M1M mesh, weighted fabric), small metrics.
//
// Same settle order and result as LinkState::runSpf
// (openr/decision/LinkState.cpp:836-911) for metrics >= 1: nodes become final in
// increasing distance; a node settled at distance d pulls its ECMP next-hop set
// from its tight in-edges (all tails settled earlier, LinkState.cpp:885-901) and,
// if it may transit (LinkState.cpp:859-866), relaxes its out-edges
// (LinkState.cpp:869-903).
//
// One workgroup per root. Instead of scanning all V nodes for each distance
// value (spf_kernels.hip variant 2: fine on a 100k fabric with a handful of
// distances, hopeless on a 1M-node mesh with ~5,000), tentative distances live
// in a ring of NB = max_metric + 1 frontier lists: a relaxation that lowers
// dist[y] to nd appends y to list nd % NB (every tentative distance is within
// max_metric of the current one, so a list only ever holds entries of one
// live distance; stale entries fail the dist[y] == d check). A round settles
// the current list; the next round is the nearest non-empty list. A list that
// overflows its capacity is marked and its round scans all nodes instead
// (correct, slower). A node is settled by a group of 4 lanes (its edges in
// parallel: the round's latency is a few dependent loads, not a serial walk
// of the row); rows longer than kBig entries are settled by a whole wave.
// dist / next-hop rows live in HBM (the caller's output rows or engine
// scratch); the digest is folded in as nodes settle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;
constexpr int kWave = 64;
constexpr uint32_t kBlock = 256;
constexpr uint32_t kWaves = kBlock / kWave;
constexpr uint32_t kBig = 64;       // rows settled by a whole wave
constexpr uint32_t kBigList = 256;  // big rows per round handed to waves (more: serial)
constexpr uint32_t kGroup = 4;      // lanes per node for rows <= kBig (1 < W <= 8)
constexpr uint32_t kVec = 32;       // W == 1: rows settled by one lane (uint4 reads)

__device__ __forceinline__ uint32_t lbound(const uint32_t* a, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, kWave);
  return x;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)x, o, kWave);
    const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), o, kWave);
    x += ((uint64_t)hi << 32) | lo;
  }
  return x;
}

template <bool IGN>
struct Dial {
  const DevGraph& g;
  const RunArgs& a;
  uint32_t root, V, W, NB, bcap;
  uint32_t* dist;
  uint32_t* nh;
  uint32_t* bkt;
  const uint32_t* nbr;
  uint32_t nbr_n;
  const uint32_t* ign;
  uint32_t ign_n;
  uint32_t* cnt;  // LDS [NB]
  uint32_t* ovf;  // LDS [NB]
  uint64_t reached = 0, sumd = 0, hsum = 0;

  __device__ bool transit(uint32_t v) const {
    return v == root || !((g.nt_bits[v >> 5] >> (v & 31u)) & 1u);
  }
  __device__ bool usable(uint32_t e, uint32_t cx) const {
    if (cx & kDown) return false;
    if (IGN && ign_n) {
      const uint32_t l = g.link_id[e];
      const uint32_t i = lbound(ign, ign_n, l);
      if (i < ign_n && ign[i] == l) return false;
    }
    return true;
  }
  __device__ void push(uint32_t y, uint32_t nd) {
    const uint32_t s = nd % NB;
    const uint32_t pos = atomicAdd(&cnt[s], 1u);
    if (pos < bcap) bkt[(size_t)s * bcap + pos] = y;
    else ovf[s] = 1u;
  }
  // tight in-edge e of x at distance d? -> its contribution to nh(x)
  __device__ void pull_edge(uint32_t x, uint32_t d, uint32_t e, uint32_t* acc) const {
    const uint32_t cx = g.colx[e];
    if (!usable(e, cx) || cx == x) return;
    const uint32_t du = dist[cx];
    if (du == kInf || (uint64_t)du + g.rw[e] != d) return;
    if (cx == root) {
      const uint32_t b = lbound(nbr, nbr_n, x);
      acc[b >> 5] |= 1u << (b & 31u);
    } else if (transit(cx)) {
      const uint32_t* s = nh + (size_t)cx * W;
      for (uint32_t w = 0; w < W; ++w) acc[w] |= s[w];
    }
  }
  __device__ void relax_edge(uint32_t x, uint32_t d, uint32_t e) {
    const uint32_t cx = g.colx[e];
    if (!usable(e, cx) || cx == x) return;
    const uint32_t nd = d + g.w[e];
    // a plain read first: most relaxations do not improve (settled or
    // already closer), and an atomic costs an L2 round trip each
    if (nd >= __hip_atomic_load(&dist[cx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return;
    const uint32_t old = atomicMin(&dist[cx], nd);
    if (nd < old) push(cx, nd);
  }
  __device__ void account(uint32_t x, uint32_t d, const uint32_t* words) {
    reached += 1;
    sumd += d;
    hsum += digest_node_term(x, d);
    for (uint32_t w = 0; w < W; ++w) hsum += digest_word_term(x, w, words[w]);
  }
  // settle x (dist d) in one lane; W <= 8 words in registers, else in the row
  __device__ void settle_lane(uint32_t x, uint32_t d, uint32_t beg, uint32_t end) {
    if (x != root) {
      if (W <= 8) {
        uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint32_t e = beg; e < end; ++e) pull_edge(x, d, e, acc);
        uint32_t* row = nh + (size_t)x * W;
        for (uint32_t w = 0; w < W; ++w) row[w] = acc[w];
        account(x, d, acc);
      } else {
        uint32_t* row = nh + (size_t)x * W;
        for (uint32_t e = beg; e < end; ++e) pull_edge(x, d, e, row);
        account(x, d, row);
      }
    } else {
      reached += 1;
      hsum += digest_node_term(x, 0);
    }
    if (transit(x))
      for (uint32_t e = beg; e < end; ++e) relax_edge(x, d, e);
  }
  // settle x in one lane, one next-hop word (W == 1), the row read 8 entries
  // at a time as uint4 loads with every neighbour's dist load in flight
  // together; the dist values read for the pull also pre-check the
  // relaxations
  __device__ void settle_vec(uint32_t x, uint32_t d, uint32_t beg, uint32_t end) {
    const bool tr = transit(x);
    const uint4* c4 = reinterpret_cast<const uint4*>(g.colx);
    const uint4* r4 = reinterpret_cast<const uint4*>(g.rw);
    const uint4* w4 = reinterpret_cast<const uint4*>(g.w);
    uint32_t acc = 0;
    for (uint32_t e0 = beg; e0 < end; e0 += 8) {
      const bool two = e0 + 4 < end;
      const uint4 ca = c4[e0 >> 2], ra = r4[e0 >> 2], wa = w4[e0 >> 2];
      const uint4 cb = two ? c4[(e0 >> 2) + 1] : make_uint4(kDown, kDown, kDown, kDown);
      const uint4 rb = two ? r4[(e0 >> 2) + 1] : make_uint4(0, 0, 0, 0);
      const uint4 wb = two ? w4[(e0 >> 2) + 1] : make_uint4(0, 0, 0, 0);
      const uint32_t cs[8] = {ca.x, ca.y, ca.z, ca.w, cb.x, cb.y, cb.z, cb.w};
      const uint32_t rs[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
      const uint32_t ws[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
      bool ok[8];
      uint32_t du[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        ok[i] = !(cs[i] & kDown) && cs[i] != x && (!IGN || usable(e0 + i, cs[i]));
        du[i] = ok[i] ? dist[cs[i]] : kInf;
      }
      if (x != root) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (du[i] == kInf || (uint64_t)du[i] + rs[i] != d) continue;
          if (cs[i] == root) {
            const uint32_t b = lbound(nbr, nbr_n, x);
            acc |= 1u << (b & 31u);
          } else if (transit(cs[i])) {
            acc |= nh[cs[i]];
          }
        }
      }
      if (tr) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (!ok[i]) continue;
          const uint32_t nd = d + ws[i];
          if (nd >= du[i]) continue;
          const uint32_t old = atomicMin(&dist[cs[i]], nd);
          if (nd < old) push(cs[i], nd);
        }
      }
    }
    if (x != root) {
      nh[x] = acc;
      account(x, d, &acc);
    } else {
      reached += 1;
      hsum += digest_node_term(x, 0);
    }
  }
  // settle x with a group of kGroup lanes (gl = lane in the group): the
  // row's edges are pulled / relaxed in parallel, next-hop words reduced with
  // shuffles; W <= 8
  __device__ void settle_group(uint32_t x, uint32_t d, uint32_t gl, bool act) {
    uint32_t beg = 0, end = 0;
    if (act) {
      beg = g.row_ptr[x];
      end = g.row_ptr[x + 1];
    }
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (act && x != root) {
      uint32_t e = beg + gl;
      for (; e + kGroup < end; e += 2 * kGroup) {  // two edges in flight per lane
        pull_edge(x, d, e, acc);
        pull_edge(x, d, e + kGroup, acc);
      }
      if (e < end) pull_edge(x, d, e, acc);
    }
#pragma unroll
    for (int o = 1; o < (int)kGroup; o <<= 1)
      for (uint32_t w = 0; w < W; ++w) acc[w] |= __shfl_xor(acc[w], o, kWave);
    if (!act) return;
    if (gl == 0) {
      if (x != root) {
        uint32_t* row = nh + (size_t)x * W;
        for (uint32_t w = 0; w < W; ++w) row[w] = acc[w];
        account(x, d, acc);
      } else {
        reached += 1;
        hsum += digest_node_term(x, 0);
      }
    }
    if (transit(x))
      for (uint32_t e = beg + gl; e < end; e += kGroup) relax_edge(x, d, e);
  }
  // settle x with the whole wave (long rows)
  __device__ void settle_wave(uint32_t x, uint32_t d, int lane) {
    const uint32_t beg = g.row_ptr[x], end = g.row_ptr[x + 1];
    if (x != root) {
      uint32_t* row = nh + (size_t)x * W;
      for (uint32_t w0 = 0; w0 < W; w0 += 8) {  // 8 next-hop words per sweep
        uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint32_t e = beg + lane; e < end; e += kWave) {
          const uint32_t cx = g.colx[e];
          if (!usable(e, cx) || cx == x) continue;
          const uint32_t du = dist[cx];
          if (du == kInf || (uint64_t)du + g.rw[e] != d) continue;
          if (cx == root) {
            const uint32_t b = lbound(nbr, nbr_n, x);
            if ((b >> 5) >= w0 && (b >> 5) < w0 + 8u) acc[(b >> 5) - w0] |= 1u << (b & 31u);
          } else if (transit(cx)) {
            const uint32_t* s = nh + (size_t)cx * W;
            for (uint32_t w = w0; w < min(W, w0 + 8u); ++w) acc[w - w0] |= s[w];
          }
        }
        for (uint32_t w = w0; w < min(W, w0 + 8u); ++w) {
          const uint32_t v = wave_or(acc[w - w0]);
          if (lane == 0) {
            row[w] = v;
            if (v) hsum += digest_word_term(x, w, v);
          }
        }
      }
      if (lane == 0) {
        reached += 1;
        sumd += d;
        hsum += digest_node_term(x, d);
      }
    } else if (lane == 0) {
      reached += 1;
      hsum += digest_node_term(x, 0);
    }
    if (transit(x))
      for (uint32_t e = beg + lane; e < end; e += kWave) relax_edge(x, d, e);
  }
};

template <bool IGN>
__global__ void __launch_bounds__(256) dial_bucket_kernel(DevGraph g, RunArgs a) {
  extern __shared__ uint32_t lds[];  // nbr (nbr_cap) | ign (ign_cap)
  __shared__ uint32_t s_cnt[kMaxDialRing], s_ovf[kMaxDialRing];
  __shared__ uint32_t s_big[kBigList];
  __shared__ uint32_t s_ctl[4];
  __shared__ uint64_t s_dig[3][kWaves];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t rix = blockIdx.x, V = g.V, W = a.W;
  Dial<IGN> r{g, a};
  r.root = a.roots[rix];
  r.V = V;
  r.W = W;
  r.NB = a.nbk;
  r.bcap = a.bcap;
  r.dist = a.dist + (size_t)rix * V;
  r.nh = a.nh + (size_t)rix * V * W;
  r.bkt = a.bkt + (size_t)rix * a.nbk * a.bcap;
  r.cnt = s_cnt;
  r.ovf = s_ovf;
  uint32_t* s_nbr = lds;
  uint32_t* s_ign = lds + a.nbr_cap;
  r.nbr = s_nbr;
  r.ign = s_ign;
  const uint32_t nb0 = g.dn_off[r.root];
  r.nbr_n = g.dn_off[r.root + 1] - nb0;
  if (r.nbr_n > 32u * W || r.nbr_n > a.nbr_cap) {
    if (tid == 0) atomicOr(a.err, 1u);
    return;
  }
  for (uint32_t i = tid; i < r.nbr_n; i += kBlock) s_nbr[i] = g.dn[nb0 + i];
  r.ign_n = 0;
  if (IGN) {
    const uint32_t i0 = a.ign_off[rix], i1 = a.ign_off[rix + 1];
    r.ign_n = i1 - i0;
    if (r.ign_n > a.ign_cap) {
      if (tid == 0) atomicOr(a.err, 2u);
      return;
    }
    for (uint32_t i = tid; i < r.ign_n; i += kBlock) s_ign[i] = a.ign_ids[i0 + i];
  }
  for (uint32_t i = tid; i < kMaxDialRing; i += kBlock) s_cnt[i] = s_ovf[i] = 0u;
  // state: dist INF, next hops 0 (16-B stores where aligned)
  for (uint32_t v = tid; v < V; v += kBlock) r.dist[v] = v == r.root ? 0u : kInf;
  for (size_t i = tid; i < (size_t)V * W; i += kBlock) r.nh[i] = 0u;
  if (tid == 0) {
    r.bkt[0] = r.root;
    s_cnt[0] = 1u;
    s_ctl[0] = 0u;
  }
  __syncthreads();

  const uint32_t NB = r.NB;
  for (uint32_t d = 0;;) {
    const uint32_t s = d % NB, n = s_cnt[s], full = s_ovf[s];
    auto settle = [&](uint32_t x) {
      if (r.dist[x] != d) return;  // stale entry (settled earlier at a smaller distance)
      const uint32_t beg = g.row_ptr[x], end = g.row_ptr[x + 1];
      if (end - beg > kBig) {
        const uint32_t k = atomicAdd(&s_ctl[0], 1u);
        if (k < kBigList) {
          s_big[k] = x;
          return;
        }
      }
      r.settle_lane(x, d, beg, end);
    };
    if (!full && W == 1) {
      // a lane per entry, rows read as uint4 (settle_vec); long rows go to
      // the waves below
      const uint32_t* list = r.bkt + (size_t)s * r.bcap;
      for (uint32_t i = tid; i < n; i += kBlock) {
        const uint32_t x = list[i];
        if (r.dist[x] != d) continue;  // stale entry
        const uint32_t beg = g.row_ptr[x], end = g.row_ptr[x + 1];
        if (end - beg > kVec) {
          const uint32_t k = atomicAdd(&s_ctl[0], 1u);
          if (k < kBigList) s_big[k] = x;
          else r.settle_lane(x, d, beg, end);
          continue;
        }
        r.settle_vec(x, d, beg, end);
      }
    } else if (!full && W <= 8) {
      // a group of kGroup lanes per entry; long rows go to the waves below
      const uint32_t* list = r.bkt + (size_t)s * r.bcap;
      const uint32_t gi = tid / kGroup, gl = tid % kGroup;
      for (uint32_t base = 0; base < n; base += kBlock / kGroup) {
        const uint32_t idx = base + gi;
        uint32_t x = idx < n ? list[idx] : kInf;
        bool act = x != kInf && r.dist[x] == d;
        if (act && g.row_ptr[x + 1] - g.row_ptr[x] > kBig) {
          if (gl == 0) {
            const uint32_t k = atomicAdd(&s_ctl[0], 1u);
            if (k < kBigList) s_big[k] = x;
            else r.settle_lane(x, d, g.row_ptr[x], g.row_ptr[x + 1]);
          }
          act = false;
        }
        r.settle_group(x, d, gl, act);
      }
    } else if (!full) {
      const uint32_t* list = r.bkt + (size_t)s * r.bcap;
      for (uint32_t i = tid; i < n; i += kBlock) settle(list[i]);
    } else {
      for (uint32_t v = tid; v < V; v += kBlock) settle(v);
    }
    __syncthreads();
    const uint32_t nbig = min(s_ctl[0], kBigList);
    if (nbig) {  // (block-uniform)
      for (uint32_t j = wave; j < nbig; j += kWaves) r.settle_wave(s_big[j], d, lane);
      __syncthreads();
    }
    if (tid == 0) {
      s_ctl[0] = 0u;
      s_cnt[s] = 0u;
      s_ovf[s] = 0u;
      uint32_t nx = kInf;
      for (uint32_t k = 1; k < NB; ++k) {
        const uint32_t q = (d + k) % NB;
        if (s_cnt[q] || s_ovf[q]) {
          nx = d + k;
          break;
        }
      }
      s_ctl[1] = nx;
    }
    __syncthreads();
    d = s_ctl[1];
    if (d == kInf) break;
  }

  if (a.digest) {
    const uint64_t rs = wave_sum64(r.reached), ss = wave_sum64(r.sumd), hs = wave_sum64(r.hsum);
    if (lane == 0) {
      s_dig[0][wave] = rs;
      s_dig[1][wave] = ss;
      s_dig[2][wave] = hs;
    }
    __syncthreads();
    if (tid == 0) {
      ospf_digest dg{0, 0, 0};
      for (uint32_t i = 0; i < kWaves; ++i) {
        dg.reached += s_dig[0][i];
        dg.sum_dist += s_dig[1][i];
        dg.hash += s_dig[2][i];
      }
      a.digest[rix] = dg;
    }
  }
}

}  // namespace

hipError_t launch_dial(bool ign, const DevGraph& g, const RunArgs& a, uint32_t n_roots,
                       size_t lds, hipStream_t s) {
  if (ign)
    hipLaunchKernelGGL(dial_bucket_kernel<true>, dim3(n_roots), dim3(kBlock), lds, s, g, a);
  else
    hipLaunchKernelGGL(dial_bucket_kernel<false>, dim3(n_roots), dim3(kBlock), lds, s, g, a);
  return hipGetLastError();
}

}  // namespace ospf
