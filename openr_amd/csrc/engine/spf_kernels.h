// spf_kernels.h — device-side graph layout and launch interface.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/openr_spf.h"

namespace ospf {

// Device-resident CSR snapshot (built once per ospf_load_graph). Rows are
// padded to a multiple of 4 entries (row_ptr[v] % 4 == 0) with down-marked
// fillers, so rows can be read as uint4; E counts the padded entries.
//   colx[e]    = neighbour id | 0x80000000 when the link is down (!isUp)
//   w[e]       = metric advertised by the row node (u -> colx[e])
//   rw[e]      = w[twin[e]]: metric of the reverse direction, i.e. of the
//                in-edge colx[e] -> u, read by the next-hop pull
//   link_id[e] = undirected link id (ignore sets)
//   nt_bits    = no-transit (overloaded) bitmap, 1 bit per node
//   dn_off/dn  = distinct neighbours per node, ascending (next-hop bit order)
struct DevGraph {
  uint32_t V, E;
  const uint32_t* row_ptr;
  const uint32_t* colx;
  const uint32_t* w;
  const uint32_t* rw;
  const uint32_t* link_id;
  const uint32_t* nt_bits;
  const uint32_t* dn_off;
  const uint32_t* dn;
};

struct RunArgs {
  const uint32_t* roots;
  const uint32_t* ign_off;  // [n_roots+1] or null
  const uint32_t* ign_ids;
  uint32_t flags;
  uint32_t W;               // next-hop words per node
  uint32_t nbr_cap;         // LDS words reserved for the root neighbour table
  uint32_t ign_cap;         // LDS words reserved for the ignore list
  uint32_t* dist;           // [n_roots][V] (required unless LDS variant w/o WANT_DIST)
  uint32_t* nh;             // [n_roots][V][W]
  ospf_digest* digest;      // [n_roots] when OSPF_WANT_DIGEST
  uint32_t* err;            // device error word (bit0: nh words, bit1: ignore cap)
  uint32_t slices;          // BFS kernel: workgroups per run (4-word next-hop slices)
  uint32_t* planes;         // BFS kernel, slices > 1: [n_roots][slices][V][4] scratch
};

// Digest: sum over reached nodes of node_term(v, dist) plus,
// for every next-hop n of v, pair_term(v, n) (mod 2^64). A sum of independent
// terms, so next-hop slices of one run add up.
__host__ __device__ inline uint64_t digest_mix(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}
__host__ __device__ inline uint64_t digest_node_term(uint32_t v, uint32_t dist) {
  return digest_mix(((uint64_t)v << 32) | dist);
}
__host__ __device__ inline uint64_t digest_pair_term(uint32_t v, uint32_t nh) {
  return digest_mix((((uint64_t)nh + 1) << 32) ^ (uint64_t)v ^ 0xD6E8FEB86659FD93ULL);
}

// Dial kernels (spf_kernels.hip), any metric:
//   variant 0 = LDS dist + LDS nh, 1 = LDS dist + HBM nh, 2 = HBM dist + HBM nh
hipError_t launch_spf(int variant, bool unit, bool ign, const DevGraph& g, const RunArgs& a,
                      uint32_t n_roots, uint32_t block, size_t lds_bytes, hipStream_t s);

// BFS kernel (spf_bfs.hip), unit metric / hop count, LDS bitmaps:
//   nh_lds = variant 3 (byte next-hops in LDS for roots with <= 8 neighbours),
//   otherwise variant 4 (next-hops in HBM).
uint32_t bfs_slices(uint32_t W);
hipError_t launch_bfs(bool nh_lds, bool ign, const DevGraph& g, const RunArgs& a, uint32_t n,
                      uint32_t block, size_t lds, hipStream_t s);

}  // namespace ospf
