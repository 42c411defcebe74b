// spf_wdial.hip — group-per-root bucketed Dial (gfx950), variant 7: weighted
// graphs whose per-root state does not fit LDS (weighted F100k fabric, M1M
// mesh), any metric >= 1, optional per-run ignored links.
//
// Same settle order and result as LinkState::runSpf
// (openr/decision/LinkState.cpp:836-911): nodes become final in increasing
// distance; a node settled at distance d takes its ECMP next-hop set from its
// tight in-edges (every tail is settled earlier since metrics are >= 1,
// LinkState.cpp:885-901) and, when it may transit (the root always may,
// LinkState.cpp:859-866), relaxes its out-edges (LinkState.cpp:869-903).
//
// Shape. A Dial sweep is a chain of distance rounds (about 250 on the
// weighted fabric, 5,000 on the 1M mesh), each a few dependent memory round
// trips. One workgroup of G waves runs one root at a time (G = 1 .. 16, the
// host picks it from the frontier size: a wave per root on the mesh, where a
// round settles ~200 nodes, a whole CU per root on the fabric, where a round
// expands ~10k edges); workgroups are persistent (group i runs roots i,
// i + ngroups, ...), so the frontier lists are allocated per group, and
// fewer roots in flight keep their rows in the Infinity Cache.
//
// A round. The nodes settled at distance d are gathered into an LDS queue;
// their rows are expanded as ONE flat edge range (prefix sum of the row
// lengths), 64·G lanes x kUnroll edges per step with every load / atomic of
// a step issued before any is waited for, so the round costs a handful of
// dependent memory trips whatever its degree mix (a 1,781-port spine,
// 84-entry fabric switches and 8-entry racks alike). Per tight edge the
// tail's next-hop words are ORed into the head's row with no-return L2
// atomics; per improving out-edge an atomicMin lowers the tentative distance
// and the head is appended to its frontier list. Digests are folded from the
// finished rows afterwards (row digest kernel), off the rounds' critical path.
//
// Frontier lists. Tentative distances live in a ring of NB lists, one per
// distance bucket of width delta: a relaxation that lowers dist[y] to nd
// appends y to list (nd / delta) % NB. delta = 1 when NB > max metric (every
// tentative distance then has its own list and an entry is live iff
// dist[y] == the list's distance); otherwise delta = ceil(max / (NB - 1)) and
// entries carry their distance (a bucket holds several distances; a round
// settles the smallest live one and compacts the list). A list that
// overflows its capacity is marked and its rounds scan every node instead
// (correct, slower).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;
constexpr int kWave = 64;
constexpr uint32_t kUnroll = 4;      // edges per lane per step, issued together
constexpr uint32_t kQPerWave = 256;  // queue entries per wave of the group

// per-group LDS control block (the queue arrays follow it, kQ = 256 G each)
struct Ctl {
  uint32_t cnt[kWDialMaxNB];       // entries appended to each list
  uint32_t ovf[kWDialMaxNB / 32];  // list overflowed: its rounds scan every node
  uint32_t nq;                     // queue fill
  uint32_t next;                   // next distance (kInf: done)
  uint32_t overflow;               // packed run: a distance outgrew its field
  uint32_t pad;
};

// every global store / atomic of this thread has been performed
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// state that L2 atomics update (distances, next-hop words): read past the L1
__device__ __forceinline__ uint32_t ld2(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void or2(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a run's state is touched by its own workgroup only: with `wg` (knob
// OSPF_WD_WGSCOPE) the state atomics are workgroup-scope
__device__ __forceinline__ void or2s(uint32_t* p, uint32_t v, bool wg) {
  if (wg) __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t amins(uint32_t* p, uint32_t v, bool wg) {
  return wg ? __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
            : atomicMin(p, v);
}
__device__ __forceinline__ uint32_t wmin(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor(x, o, kWave));
  return x;
}
__device__ __forceinline__ uint32_t lbound(const uint32_t* a, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint64_t lanes_below(uint32_t lane) {
  return lane ? (~0ull >> (64u - lane)) : 0ull;
}

// PACK: the run's state is one 32-bit word per node, (dist << K) | next-hop
// bits (K = 8 or 16 bits: roots with at most K distinct neighbours, one
// next-hop word), in the group's scratch instead of the dist and next-hop
// rows: half the bytes, and a tight predecessor's distance and next hops
// arrive in one load. Sound because a node's next-hop bits are only set once
// its distance is final (pull at settle), so atomicMin on the packed word of
// an unsettled node compares distances alone. The rows are expanded from the
// words when the run ends; a distance that would not fit the field aborts the
// packed run and the root is run again unpacked.
template <bool IGN, bool TAG, bool PACK>
struct GRun {
  const DevGraph& g;
  const WDialArgs& a;
  Ctl* ctl;
  uint32_t* q;   // [kQ] settled nodes of the round (a chunk of them)
  uint32_t* qb;  // [kQ] their row starts
  uint32_t* qp;  // [kQ + 1] exclusive prefix of their row lengths
  uint32_t kQ, nthr, tid, lane, wave;
  uint32_t root, V, W, NB, bcap, delta;
  uint32_t* dist;
  uint32_t* nh;
  uint32_t* pk;             // PACK: [V] packed words
  uint32_t K, infk, nhmask; // PACK: next-hop bits, the distance field's INF, K-bit mask
  uint32_t* lists;      // [NB][bcap] entries (TAG: {node, dist} pairs)
  const uint32_t* nbr;  // root's distinct neighbours (ascending) = next-hop bit order
  uint32_t nbr_n;
  const uint32_t* ign;  // run's ignored link ids (sorted)
  uint32_t ign_n;

  __device__ bool transit(uint32_t v) const {
    return v == root || !((g.nt_bits[v >> 5] >> (v & 31u)) & 1u);
  }
  __device__ bool ignored(uint32_t e) const {
    if (!IGN || !ign_n) return false;
    const uint32_t l = g.link_id[e];
    const uint32_t i = lbound(ign, ign_n, l);
    return i < ign_n && ign[i] == l;
  }
  __device__ uint32_t slot_of(uint32_t dd) const { return (dd / delta) % NB; }
  __device__ uint32_t* entry(uint32_t s, uint32_t i) const {
    return lists + ((size_t)s * bcap + i) * (TAG ? 2u : 1u);
  }
  __device__ void push(uint32_t y, uint32_t nd) {
    if (y >= V) {  // never: a guard that turns a bug into an error word, not a fault
      atomicOr(a.err, 4u);
      return;
    }
    const uint32_t s = slot_of(nd);
    const uint32_t pos = atomicAdd(&ctl->cnt[s], 1u);
    if (pos < bcap) {
      uint32_t* p = entry(s, pos);
      p[0] = y;
      if (TAG) p[1] = nd;
    } else {
      atomicOr(&ctl->ovf[s >> 5], 1u << (s & 31u));
    }
  }
  __device__ bool ovf(uint32_t s) const { return (ctl->ovf[s >> 5] >> (s & 31u)) & 1u; }
  __device__ uint32_t field(uint32_t w) const {  // PACK: distance of a packed word
    const uint32_t f = w >> K;
    return f == infk ? kInf : f;
  }
  __device__ uint32_t dist_of(uint32_t v) const {
    return PACK ? field(ld2(&pk[v])) : ld2(&dist[v]);
  }
  // all memory operations of the group performed and visible to it
  __device__ void sync() {
    drain();
    __syncthreads();
  }

  // Expand the rows of the nq queued nodes (all settled at d) as one flat
  // edge range. Entered and left with the group synchronised.
  __device__ void flush(uint32_t nq, uint32_t d) {
    if (wave == 0) {  // row starts and an exclusive prefix of the (padded) row lengths
      uint32_t carry = 0;
      for (uint32_t j0 = 0; j0 < nq; j0 += kWave) {
        const uint32_t j = j0 + lane;
        uint32_t len = 0;
        if (j < nq) {
          const uint32_t x = q[j];
          const uint32_t b = g.row_ptr[x];
          len = g.row_ptr[x + 1] - b;
          qb[j] = b;
        }
        uint32_t inc = len;  // inclusive wave scan
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
          const uint32_t y = __shfl_up(inc, o, kWave);
          if ((int)lane >= o) inc += y;
        }
        if (j < nq) qp[j] = carry + inc - len;
        carry += __shfl(inc, kWave - 1, kWave);
      }
      if (lane == 0) qp[nq] = carry;
    }
    __syncthreads();
    const uint32_t T = qp[nq];
    for (uint32_t t0 = 0; t0 < T; t0 += nthr * kUnroll) {
      uint32_t x[kUnroll], e[kUnroll], cx[kUnroll], du[kUnroll], pw[kUnroll], w[kUnroll],
          rw[kUnroll];
      bool ok[kUnroll];
#pragma unroll
      for (uint32_t u = 0; u < kUnroll; ++u) {
        const uint32_t t = t0 + u * nthr + tid;
        ok[u] = t < T;
        x[u] = 0;
        e[u] = 0;
        if (ok[u]) {
          // the queued node whose row holds flat edge t: last qp[j] <= t
          uint32_t lo = 0, hi = nq;
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (qp[mid] <= t) lo = mid; else hi = mid;
          }
          x[u] = q[lo];
          e[u] = qb[lo] + (t - qp[lo]);
        }
      }
      if (g.ew) {  // {colx, w | rw << 16}: one 8-B load per entry
#pragma unroll
        for (uint32_t u = 0; u < kUnroll; ++u) {
          const uint2 ce = ok[u] ? g.ew[e[u]] : make_uint2(kDown, 0u);
          cx[u] = ce.x;
          w[u] = a.hop ? 1u : (ce.y & 0xFFFFu);
          rw[u] = a.hop ? 1u : (ce.y >> 16);
        }
      } else {
#pragma unroll
        for (uint32_t u = 0; u < kUnroll; ++u) {
          cx[u] = ok[u] ? g.colx[e[u]] : kDown;
          w[u] = 1u;
          rw[u] = 1u;
          if (!a.hop && ok[u]) {
            w[u] = g.w[e[u]];
            rw[u] = g.rw[e[u]];
          }
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < kUnroll; ++u) {
        ok[u] = ok[u] && !(cx[u] & kDown) && cx[u] != x[u] && !ignored(e[u]);
        pw[u] = ok[u] ? ld2(PACK ? &pk[cx[u]] : &dist[cx[u]]) : kInf;
        du[u] = PACK ? (ok[u] ? field(pw[u]) : kInf) : pw[u];
      }
      // pull: tight in-edge cx -> x adds cx's next hops (or x itself when cx
      // is the root) to x's row; the loads of a step are issued together
      bool tight[kUnroll];
#pragma unroll
      for (uint32_t u = 0; u < kUnroll; ++u)
        tight[u] = ok[u] && x[u] != root && du[u] != kInf && (uint64_t)du[u] + rw[u] == d;
      if (PACK) {  // the tail's next hops came with its distance
        uint32_t v[kUnroll];
#pragma unroll
        for (uint32_t u = 0; u < kUnroll; ++u) {
          v[u] = 0u;
          if (!tight[u]) continue;
          if (cx[u] == root) v[u] = 1u << lbound(nbr, nbr_n, x[u]);
          else if (transit(cx[u])) v[u] = pw[u] & nhmask;
        }
#pragma unroll
        for (uint32_t u = 0; u < kUnroll; ++u)
          if (v[u]) or2s(pk + x[u], v[u], a.wg_scope);
      } else if (W == 1) {
        uint32_t v[kUnroll];
#pragma unroll
        for (uint32_t u = 0; u < kUnroll; ++u) {
          v[u] = 0u;
          if (!tight[u]) continue;
          if (cx[u] == root) v[u] = 1u << (lbound(nbr, nbr_n, x[u]) & 31u);
          else if (transit(cx[u])) v[u] = ld2(nh + cx[u]);
        }
#pragma unroll
        for (uint32_t u = 0; u < kUnroll; ++u)
          if (v[u]) or2s(nh + x[u], v[u], a.wg_scope);
      } else {
#pragma unroll
        for (uint32_t u = 0; u < kUnroll; ++u) {
          if (!tight[u]) continue;
          uint32_t* row = nh + (size_t)x[u] * W;
          if (cx[u] == root) {
            const uint32_t b = lbound(nbr, nbr_n, x[u]);
            or2s(row + (b >> 5), 1u << (b & 31u), a.wg_scope);
          } else if (transit(cx[u])) {
            const uint32_t* src = nh + (size_t)cx[u] * W;
            for (uint32_t w0 = 0; w0 < W; w0 += 8) {  // 8 loads in flight, then the ORs
              uint32_t v[8];
#pragma unroll
              for (uint32_t k = 0; k < 8; ++k) v[k] = w0 + k < W ? ld2(src + w0 + k) : 0u;
#pragma unroll
              for (uint32_t k = 0; k < 8; ++k)
                if (v[k]) or2s(row + w0 + k, v[k], a.wg_scope);
            }
          }
        }
      }
      // relax: improving out-edges lower the head's distance
      uint32_t nd[kUnroll], old[kUnroll];
#pragma unroll
      for (uint32_t u = 0; u < kUnroll; ++u) {
        nd[u] = d + w[u];
        old[u] = 0u;  // no relaxation: nothing to push
        if (!(ok[u] && nd[u] < du[u] && transit(x[u]))) continue;
        if (PACK) {
          if (nd[u] >= infk) {
            ctl->overflow = 1u;
            continue;
          }
          old[u] = field(amins(&pk[cx[u]], nd[u] << K, a.wg_scope));
        } else {
          old[u] = amins(&dist[cx[u]], nd[u], a.wg_scope);
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < kUnroll; ++u)
        if (nd[u] < old[u]) push(cx[u], nd[u]);
    }
    sync();  // atomics performed, queue free again
  }

  // settle every node at distance d: list entries (or, for an overflowed
  // list, every node), compacted into the queue in chunks. Entered and left
  // with the group synchronised.
  __device__ void settle_round(uint32_t s, uint32_t d) {
    const bool full = ovf(s);
    const uint32_t n = full ? V : min(ctl->cnt[s], bcap);
    for (uint32_t i0 = 0; i0 < n; i0 += nthr) {
      const uint32_t i = i0 + tid;
      uint32_t x = 0;
      bool live = false;
      if (i < n) {
        if (full) {
          x = i;
          live = dist_of(x) == d;
        } else {
          const uint32_t* p = entry(s, i);
          x = p[0];
          live = x < V && (!TAG || p[1] == d) && dist_of(x) == d;
        }
      }
      const uint64_t m = __ballot(live);
      uint32_t base = 0;
      if (lane == 0 && m) base = atomicAdd(&ctl->nq, (uint32_t)__popcll(m));
      base = __shfl(base, 0, kWave);
      if (live) q[base + (uint32_t)__popcll(m & lanes_below(lane))] = x;
      __syncthreads();
      const uint32_t nq = ctl->nq;
      // flush once another chunk might not fit (and after the last chunk)
      if (nq && (nq + nthr > kQ || i0 + nthr >= n)) {
        flush(nq, d);
        if (tid == 0) ctl->nq = 0;
      }
      __syncthreads();
    }
  }

  // (wave 0) smallest live distance of list s in [lo, hi) (INF: none).
  // Overflowed lists are incomplete: scan every node's distance instead.
  __device__ uint32_t list_min(uint32_t s, uint32_t lo, uint32_t hi) const {
    uint32_t m = kInf;
    if (ovf(s)) {
      for (uint32_t v = lane; v < V; v += kWave) {
        const uint32_t dv = dist_of(v);
        if (dv >= lo && dv < hi) m = min(m, dv);
      }
    } else {
      const uint32_t n = min(ctl->cnt[s], bcap);
      for (uint32_t i = lane; i < n; i += kWave) {
        const uint32_t* p = entry(s, i);
        const uint32_t ed = TAG ? p[1] : lo;
        if (ed >= lo && ed < hi && dist_of(p[0]) == ed) m = min(m, ed);
      }
    }
    return wmin(m);
  }
  // (wave 0) TAG: drop the entries of list s that are no longer live above d
  __device__ void compact(uint32_t s, uint32_t d) {
    const uint32_t n = min(ctl->cnt[s], bcap);
    uint32_t out = 0;
    for (uint32_t b = 0; b < n; b += kWave) {
      const uint32_t i = b + lane;
      uint32_t x = 0, ed = 0;
      bool live = false;
      if (i < n) {
        const uint32_t* p = entry(s, i);
        x = p[0];
        ed = p[1];
        live = ed > d && dist_of(x) == ed;
      }
      const uint64_t m = __ballot(live);
      if (live) {
        uint32_t* qq = entry(s, out + (uint32_t)__popcll(m & lanes_below(lane)));
        qq[0] = x;
        qq[1] = ed;
      }
      out += (uint32_t)__popcll(m);
    }
    drain();
    if (lane == 0) ctl->cnt[s] = out;
  }
  // (wave 0) the distance after d: ctl->next
  __device__ void next_distance(uint32_t d) {
    const uint32_t s = slot_of(d);
    const bool full = ovf(s);
    uint32_t nx = kInf;
    if (TAG) {  // the rest of this bucket first
      nx = list_min(s, d + 1, (d / delta + 1) * delta);
      if (nx != kInf) {
        if (!full) compact(s, d);
        if (lane == 0) ctl->next = nx;
        return;
      }
    }
    if (lane == 0) {
      ctl->cnt[s] = 0u;
      ctl->ovf[s >> 5] &= ~(1u << (s & 31u));
    }
    const uint32_t b0 = d / delta;  // current bucket
    for (;;) {
      // first non-empty list after slot s (offsets 1 .. NB-1)
      uint32_t k = 0;
      for (uint32_t l0 = 0; l0 + 1 < NB && !k; l0 += kWave) {
        const uint32_t off = l0 + lane + 1;
        const uint32_t qs = (s + off) % NB;
        const bool ne = off < NB && (ctl->cnt[qs] != 0u || ovf(qs));
        const uint64_t m = __ballot(ne);
        if (m) k = l0 + (uint32_t)__ffsll((unsigned long long)m);
      }
      if (!k) break;
      const uint32_t qs = (s + k) % NB, b = b0 + k;
      if (!TAG) {
        nx = b;  // delta == 1: the list's distance
        break;
      }
      nx = list_min(qs, b * delta, (b + 1) * delta);
      if (nx != kInf) break;
      if (lane == 0) {  // only stale entries: drop the list, keep looking
        ctl->cnt[qs] = 0u;
        ctl->ovf[qs >> 5] &= ~(1u << (qs & 31u));
      }
    }
    if (lane == 0) ctl->next = nx;
  }

  // false: a packed run overflowed its distance field (nothing valid written)
  __device__ bool run() {
    if (PACK) {  // state: one word per node, INF; the rows are written at the end
      for (uint32_t i = tid; i < V; i += nthr) pk[i] = 0xFFFFFFFFu;
    } else {     // rows: dist INF (root 0), next hops 0
      if ((V & 3u) == 0) {
        uint4* d4 = reinterpret_cast<uint4*>(dist);
        for (uint32_t i = tid; i < V / 4; i += nthr) d4[i] = make_uint4(kInf, kInf, kInf, kInf);
      } else {
        for (uint32_t i = tid; i < V; i += nthr) dist[i] = kInf;
      }
      const size_t nw = (size_t)V * W;
      if ((nw & 3u) == 0) {
        uint4* n4 = reinterpret_cast<uint4*>(nh);
        for (size_t i = tid; i < nw / 4; i += nthr) n4[i] = make_uint4(0, 0, 0, 0);
      } else {
        for (size_t i = tid; i < nw; i += nthr) nh[i] = 0u;
      }
    }
    for (uint32_t i = tid; i < NB; i += nthr) ctl->cnt[i] = 0u;
    if (tid < kWDialMaxNB / 32) ctl->ovf[tid] = 0u;
    if (tid == 0) {
      ctl->nq = 0u;
      ctl->overflow = 0u;
    }
    sync();
    if (tid == 0) {
      if (PACK) pk[root] = 0u;
      else dist[root] = 0u;
      uint32_t* p = entry(0, 0);
      p[0] = root;
      if (TAG) p[1] = 0u;
      ctl->cnt[0] = 1u;
    }
    sync();
    for (uint32_t d = 0;;) {
      settle_round(slot_of(d), d);
      if (wave == 0) next_distance(d);
      sync();
      if (PACK && ctl->overflow) return false;
      d = ctl->next;
      if (d == kInf) break;
    }
    if (PACK) {  // rows from the packed words
      for (uint32_t i = tid; i < V; i += nthr) {
        const uint32_t wd = ld2(&pk[i]);
        dist[i] = field(wd);
        nh[i] = wd & nhmask;
      }
    }
    return true;
  }
};

template <bool IGN, bool TAG, bool PACK>
__device__ bool run_root(const DevGraph& g, const WDialArgs& a, uint32_t* lds, uint32_t rix) {
  const uint32_t nthr = blockDim.x, kQ = kQPerWave * (nthr / kWave);
  uint32_t* qa = lds + sizeof(Ctl) / 4;
  GRun<IGN, TAG, PACK> r{g, a};
  r.ctl = reinterpret_cast<Ctl*>(lds);
  r.q = qa;
  r.qb = qa + kQ;
  r.qp = qa + 2 * kQ;
  r.kQ = kQ;
  r.nthr = nthr;
  r.tid = threadIdx.x;
  r.lane = threadIdx.x & 63u;
  r.wave = threadIdx.x >> 6;
  r.root = a.roots[rix];
  r.V = g.V;
  r.W = a.W;
  r.NB = a.NB;
  r.bcap = a.bcap;
  r.delta = a.delta;
  r.dist = a.dist + (size_t)rix * g.V;
  r.nh = a.nh + (size_t)rix * g.V * a.W;
  r.pk = PACK ? a.pk + (size_t)blockIdx.x * g.V : nullptr;
  r.K = a.pk_bits;
  r.infk = PACK ? 0xFFFFFFFFu >> a.pk_bits : 0u;
  r.nhmask = PACK ? (1u << a.pk_bits) - 1u : 0u;
  r.lists = a.lists + (size_t)blockIdx.x * a.NB * a.bcap * (TAG ? 2u : 1u);
  const uint32_t nb0 = g.dn_off[r.root];
  r.nbr = g.dn + nb0;
  r.nbr_n = g.dn_off[r.root + 1] - nb0;
  if (r.nbr_n > 32u * a.W || (PACK && r.nbr_n > a.pk_bits)) {
    if (threadIdx.x == 0) atomicOr(a.err, 1u);
    return true;
  }
  r.ign = nullptr;
  r.ign_n = 0;
  if (IGN) {
    const uint32_t i0 = a.ign_off[rix];
    r.ign = a.ign_ids + i0;
    r.ign_n = a.ign_off[rix + 1] - i0;
  }
  return r.run();
}

// Root order: callers sweep roots in locality order (roots hanging off the
// same switches adjacent), and workgroup b runs on XCD b % 8. The k-th root
// of group b is k * ngroups + (b % 8) * (ngroups / 8) + b / 8, so the groups
// of one XCD run consecutive roots at once: they read the same graph rows
// around the same rounds, and the XCD's L2 serves them to all of them.
__device__ __forceinline__ uint32_t root_slot(uint32_t b, uint32_t ngroups) {
  if (ngroups & 7u) return b;
  return (b & 7u) * (ngroups >> 3) + (b >> 3);
}

template <bool IGN, bool TAG, bool PACK>
__global__ void __launch_bounds__(1024) wdial_kernel(DevGraph g, WDialArgs a) {
  extern __shared__ uint32_t lds[];
  for (uint32_t rix = root_slot(blockIdx.x, gridDim.x); rix < a.n; rix += gridDim.x) {
    bool done = true;
    if (PACK) done = run_root<IGN, TAG, true>(g, a, lds, rix);
    __syncthreads();
    if (!PACK || !done) run_root<IGN, TAG, false>(g, a, lds, rix);
    __syncthreads();  // the group's LDS is reused by its next root
  }
}

}  // namespace

hipError_t launch_wdial(const DevGraph& g, const WDialArgs& a, hipStream_t s) {
  if (a.NB < 2 || a.NB > kWDialMaxNB || a.delta == 0 || a.bcap == 0 || a.group_waves == 0 ||
      a.group_waves > 16 || a.ngroups == 0 || (a.pk_bits && (a.pk_bits > 16 || a.W != 1 || !a.pk)))
    return hipErrorInvalidValue;
  const uint32_t nthr = 64u * a.group_waves;
  const size_t lds = sizeof(Ctl) + (3ull * kQPerWave * a.group_waves + 1) * 4ull;
  const bool ign = a.ign_off != nullptr, tag = a.delta > 1, pack = a.pk_bits != 0;
  const dim3 grid(a.ngroups), block(nthr);
#define OSPF_WD_LAUNCH(I, T, P) \
  hipLaunchKernelGGL((wdial_kernel<I, T, P>), grid, block, lds, s, g, a)
  if (ign && tag) {
    if (pack) OSPF_WD_LAUNCH(true, true, true); else OSPF_WD_LAUNCH(true, true, false);
  } else if (ign) {
    if (pack) OSPF_WD_LAUNCH(true, false, true); else OSPF_WD_LAUNCH(true, false, false);
  } else if (tag) {
    if (pack) OSPF_WD_LAUNCH(false, true, true); else OSPF_WD_LAUNCH(false, true, false);
  } else {
    if (pack) OSPF_WD_LAUNCH(false, false, true); else OSPF_WD_LAUNCH(false, false, false);
  }
#undef OSPF_WD_LAUNCH
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !a.digest) return e;
  return launch_row_digest(g, a.n, a.dist, a.nh, a.W, a.digest, s);
}

}  // namespace ospf
