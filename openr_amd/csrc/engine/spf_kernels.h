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
//   big        = nodes whose padded row is longer than kMsBigDeg (scanned by a
//                whole wave in the multi-source BFS)
//   link_e     = [n_lid][2] padded positions of the two entries of link id l
//                (UINT32_MAX when absent): ignore masks of the KSP2 reruns
// Parallel entries of a row (same neighbour) are ordered by the rank of the
// twin entry in the neighbour's linksFromNode when the caller gives link_rank,
// so row order = (neighbour id, rank) = the pathLinks order of a tight group.
constexpr uint32_t kMsBigDeg = 256;
struct DevGraph {
  uint32_t V, E;
  uint32_t nbig;
  const uint32_t* big;
  const uint64_t* dkey;  // [V][2] = {digest_dist_key(v), digest_node_key(v)}
  const uint32_t* row_ptr;
  const uint32_t* colx;
  const uint32_t* w;
  const uint32_t* rw;
  const uint32_t* link_id;
  const uint32_t* nt_bits;
  const uint32_t* dn_off;
  const uint32_t* dn;
  uint32_t n_lid;
  const uint32_t* link_e;
  // [E] {colx, w | rw << 16}: one 8-B load per entry for the weighted path
  // (null when a metric exceeds 0xFFFF: the separate arrays are read instead)
  const uint2* ew;
  // [E] index of the entry's neighbour among the row node's distinct
  // neighbours (= its next-hop bit when the row node is a root); 0xFFFF for
  // self-loops and padding
  const uint16_t* didx;
  const uint64_t* dkn;  // [V rounded up to 16] digest_node_key(v), zero padded
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
  uint32_t* bkt;            // bucketed Dial: [n_roots][nbk][bcap] frontier lists
  uint32_t bcap, nbk;       //   list capacity, ring size (max_metric + 1)
};
constexpr uint32_t kMaxDialRing = 64;  // bucketed Dial: metrics up to 63

// Digest, mod 2^64, a sum of independent terms:
//   sum over reached v of  dist_key(v) * (dist + 1)
//                        + sum over next-hop words g != 0 of v of
//                          node_key(v) * word_key(g, word)
// where word g holds the next-hop bits of the root's distinct neighbours
// 32g .. 32g+31 (ascending node id). Words and slices of one run add up, and
// a node costs one multiply plus one hash per non-zero next-hop word.
__host__ __device__ inline uint64_t digest_mix(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}
__host__ __device__ inline uint64_t digest_dist_key(uint32_t v) {
  return digest_mix((uint64_t)v ^ 0x2545F4914F6CDD1DULL) | 1ull;
}
__host__ __device__ inline uint64_t digest_node_key(uint32_t v) {
  return digest_mix((uint64_t)v ^ 0xD6E8FEB86659FD93ULL) | 1ull;
}
__host__ __device__ inline uint64_t digest_node_term(uint32_t v, uint32_t dist) {
  return digest_dist_key(v) * ((uint64_t)dist + 1);
}
__host__ __device__ inline uint64_t digest_word_key(uint32_t g, uint32_t word) {
  return digest_mix((((uint64_t)g << 32) | word) ^ 0x9E3779B97F4A7C15ULL);
}
__host__ __device__ inline uint64_t digest_word_term(uint32_t v, uint32_t g, uint32_t word) {
  return word ? digest_node_key(v) * digest_word_key(g, word) : 0ull;
}

// Sum over each 16-lane row of a wave, every lane of the row getting it:
// DPP quad permutes + row rotations (VALU only; no LDS permute round trips).
template <int kCtrl>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, kCtrl, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), kCtrl, 0xF, 0xF, true);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t row_sum64(uint64_t x) {
  x += dpp_u64<0xB1>(x);   // quad_perm [1, 0, 3, 2]
  x += dpp_u64<0x4E>(x);   // quad_perm [2, 3, 0, 1]
  x += dpp_u64<0x124>(x);  // row_ror:4
  x += dpp_u64<0x128>(x);  // row_ror:8
  return x;
}

// 16-B store of a row that this launch never reads back (dist / next-hop
// rows of finished runs): non-temporal, so the stream of output lines does not
// evict the L2 lines the traversal or derivation re-reads.
typedef uint32_t ospf_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_row16(void* p, uint4 v) {
  const ospf_u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<ospf_u32x4*>(p));
}

// Dial kernels (spf_kernels.hip), any metric:
//   variant 0 = LDS dist + LDS nh, 1 = LDS dist + HBM nh, 2 = HBM dist + HBM nh
hipError_t launch_spf(int variant, bool unit, bool ign, const DevGraph& g, const RunArgs& a,
                      uint32_t n_roots, uint32_t block, size_t lds_bytes, hipStream_t s);

// Bucketed Dial (spf_dial.hip), variant 6: any metric <= 63, HBM state,
// frontier lists instead of a per-distance scan of every node.
hipError_t launch_dial(bool ign, const DevGraph& g, const RunArgs& a, uint32_t n_roots,
                       size_t lds, hipStream_t s);

// Group-per-root bucketed Dial (spf_wdial.hip), variant 7: any metric >= 1,
// optional per-run ignored links; ngroups persistent workgroups of
// group_waves waves, group i runs roots i, i + ngroups, ... with its own ring
// of NB frontier lists of bcap entries (delta > 1: {node, dist} pairs).
// dist / nh are the output rows (required).
constexpr uint32_t kWDialMaxNB = 128;
struct WDialArgs {
  const uint32_t* roots;
  uint32_t n;
  const uint32_t* ign_off;  // [n + 1] or null
  const uint32_t* ign_ids;
  uint32_t hop;             // hop-count mode: every usable weight is 1
  uint32_t W;               // next-hop words per node
  uint32_t* dist;           // [n][V]
  uint32_t* nh;             // [n][V][W]
  ospf_digest* digest;      // [n] or null
  uint32_t* err;
  uint32_t* lists;          // [ngroups][NB][bcap][delta > 1 ? 2 : 1]
  uint32_t NB, bcap, delta;
  uint32_t group_waves;     // 1 .. 16 waves per root
  uint32_t ngroups;
  uint32_t pk_bits;         // 0, or 8 / 16: packed (dist << K | next hops) state
  uint32_t* pk;             // [ngroups][V] packed words (pk_bits != 0)
  uint32_t wg_scope = 0;    // 1: workgroup-scope state atomics (a run is one workgroup's)
};
hipError_t launch_wdial(const DevGraph& g, const WDialArgs& a, hipStream_t s);

// Multi-root distances (spf_msdist.hip): groups of 32 roots, one workgroup
// per group, Bellman-Ford by pulls in Delta buckets with [node][root] state in
// the block's scratch (msdist_scratch_bytes per `blocks` concurrent groups).
struct MsDistArgs {
  const uint32_t* roots;  // [n] node ids, neighbours adjacent (a group shares its wavefront)
  uint32_t n;
  uint32_t ngroups;       // ceil(n / 32)
  uint32_t blocks;        // concurrent groups (grid)
  uint32_t delta;         // bucket width (>= 1)
  uint32_t hop;           // hop-count mode
  uint32_t* dist;         // rows: dist + rowpos[i] * pitch (or i * pitch)
  uint64_t pitch;
  const uint32_t* rowpos;
  uint32_t* scratch;
  unsigned long long* stats = nullptr;  // debug: {phases, frontier nodes, candidates, -}
};
size_t msdist_scratch_bytes(uint32_t V, uint32_t blocks);
hipError_t launch_msdist(const DevGraph& g, const MsDistArgs& a, hipStream_t s);

// BFS kernel (spf_bfs.hip), unit metric / hop count, LDS bitmaps:
//   nh_lds = variant 3 (byte next-hops in LDS for roots with <= 8 neighbours),
//   otherwise variant 4 (next-hops in HBM).
uint32_t bfs_slices(uint32_t W);
hipError_t launch_bfs(bool nh_lds, bool ign, const DevGraph& g, const RunArgs& a, uint32_t n,
                      uint32_t block, size_t lds, hipStream_t s);

// Multi-source bit-parallel BFS (spf_msbfs.hip), variant 5: unit metric / hop
// count, no ignored links. One round = up to nb "virtual batches"
// (64-root batch, next-hop word g) sharing the launches.
struct MsArgs {
  const uint32_t* roots;  // every root of the call
  uint32_t n;             // roots in the call
  uint32_t W;             // nh words per node of the output rows
  uint32_t npass;         // passes per R-root batch (each computes OW next-hop words)
  uint32_t R;             // roots per batch (<= 64)
  uint32_t PP;            // planes per 64-bit plane word (PP * R <= 64)
  uint32_t OW;            // next-hop words per pass (32 * OW planes)
  uint64_t rep;           // sum over j < PP of 1 << (j * R): root bits -> every plane slot
  uint32_t vb0;           // first virtual batch of this round (vb = batch*npass + g)
  uint32_t nb;            // virtual batches in this round
  uint32_t lmax;          // stride of found[]
  uint32_t dbound;        // levels launched: 1 .. dbound + 1 (found[dbound + 1] set =
                          //   the host's depth bound was too small: error bit 8)
  uint32_t kcap;          // max distinct neighbours of a root (caller's bound)
  uint32_t push_div;      // level d pushes when frontier edge mass * push_div < E
  uint32_t* dist;         // [n][V] or null
  uint32_t* nh;           // [n][V][W] or null
  uint32_t* nhs;          // [n][W][V] word-major staging (defer, W > 1) or null:
                          //   msbfs_rows stores each pass's words as whole lines,
                          //   launch_nh_interleave then writes the [V][W] rows
  uint64_t* seen;         // [nb][V]
  uint64_t* front;        // [2][nb][V][2] {frontier, with-planes} of level d in front[d & 1]
  uint64_t* accb;         // [nb][V]      push accumulator (zero between levels)
  uint64_t* planes;       // [nb][V][KP]
  uint32_t* found;        // [nb][lmax]   level d non-empty
  uint32_t* mass;         // [nb][lmax]   out-edge mass of level d's frontier
  uint8_t* lev;           // [nb][V][64]  dist + 1 per (node, root), 0 = unreached
                          //              (defer: rows are written once, at the end)
  uint32_t defer;         // 1: levels fill lev, msbfs_rows writes the rows
  uint32_t merged;        // defer, 2..7 words, one per pass: one rows kernel for all
                          //   passes of a batch (msbfs_rows_multi); pass 0 records lev
  ospf_digest* digest;    // [n] (defer: msbfs_rows adds each pass's terms; zeroed first)
  uint32_t* err;
  // KSP2 reruns (kp = 0: distances only, every root of a batch is the same
  // source, run r ignores its own links): edge e is ignored by the roots in
  // igm[vb][e] when bit e of igb[vb] is set (both entries of a link marked)
  uint32_t* igb;          // [nb][igw]
  uint64_t* igm;          // [nb][E]
  uint32_t igw;
  // KSP2 reruns: destination of each run (by run index), or null. A batch
  // whose every run has reached its destination stops after that level (the
  // k = 2 trace reads only levels below the destination's)
  const uint32_t* kdst;
  uint8_t* levrow;        // derive phase 1 (kp -1): [n][lev_pitch] dist + 1 per (run, node)
  uint32_t lev_pitch;     //   bytes per level row (multiple of 16, >= V; padding zeroed)
};

// Derive phase 2 (nh_derive_kernel): next-hop words of n roots from the level
// rows of their neighbours. pos[v] = level row of node v (0xFFFFFFFF: none).
struct DeriveArgs {
  const uint32_t* roots;
  uint32_t n, W;
  uint32_t cap;            // max distinct neighbours of a root of the call (<= 2048)
  const uint8_t* lev;      // [rows][pitch]
  uint32_t pitch;          // bytes per level row (multiple of 16, >= V)
  const uint32_t* pos;     // [V]
  const ospf_digest* lev_digest;  // [rows] distance part of each row's digest (phase 1)
  uint32_t* nh;            // [n][V][W]
  ospf_digest* digest;     // [n] (zeroed by the caller) or null
  uint32_t* err;           // bit 1: K > cap / 32 W, 16: a neighbour has no level row, 64: bad root
  uint32_t ctiles;         // node tiles per block (0: default 8)
  uint32_t G, tiles, chunks;  // set by the launcher
};
// Wide next hops planned on the host (spf_msbfs.hip nh_wide_plan_kernel):
// runs of roots with the same distinct-neighbour list (<= 64 roots), each
// run's slot table and each root's usable-slot words.
struct WidePlan {
  uint32_t n, W, nruns;
  const uint32_t* run;    // [nruns + 1] root offsets
  const uint32_t* soff;   // [nruns + 1] offsets into slots (K <= 2048 per run)
  const uint32_t* slots;  // level row | 0x80000000 | node (non-transit) | 0xFFFFFFFF (unused)
  const uint32_t* keep;   // [n][W] usable-slot words
  const uint32_t* own;    // [n] each root's level row
  const uint8_t* lev;
  uint32_t pitch;
  const ospf_digest* lev_digest;  // [rows] distance parts of the level rows
  uint32_t* nh;           // [n][V][W]
  ospf_digest* digest;    // [n] (zeroed by the launcher) or null
  uint32_t tiles, ctiles, chunks;  // set by the launcher (ctiles 0: its choice)
  uint32_t late_keys;     // set by the launcher: OSPF_WIDE_LATE_KEYS (A/B)
  uint32_t st16;          // set by the launcher: records staged, 16-B stores (A/B)
};
hipError_t launch_wide_plan(const DevGraph& g, const WidePlan& p, hipStream_t s);

// Derive phase 1 on 128-root traversals (spf_levels.hip): distance-only
// multi-source BFS, 16-B root sets per node, then level / dist rows + the
// distance part of each digest. Wide batch i of a round = roots
// (vb0 + i) * 128 .. + 127 of the call.
struct LvArgs {
  const uint32_t* roots;
  uint32_t n;
  uint32_t vb0, nb;         // first wide batch of this round, wide batches in it
  uint32_t lmax, dbound;    // stride of found / mass; levels launched 1 .. dbound
  uint32_t push_div;        // level d pushes when frontier edge mass * push_div < E
  uint32_t masked;          // pull scans in masked four-quad steps (else whole steps + quads)
  uint4* front;             // [2][nb][V] frontier root sets of level d in slot d & 1
  uint4* seen;              // [nb][V]
  uint4* accb;              // [nb][V] push accumulator (zero between levels)
  uint8_t* lev;             // [nb][V][128] dist + 1 per (node, root)
  uint32_t* found;          // [nb][lmax]
  uint32_t* mass;           // [nb][lmax]
  uint32_t* dist;           // [n][dpitch] or null
  uint32_t dpitch;          // dist row pitch in words (0: V)
  uint8_t* levrow;          // [n][lev_pitch]
  uint32_t lev_pitch;
  ospf_digest* digest;      // [n] distance parts (zeroed by the caller) or null
  uint32_t* err;            // bit 8: depth bound too small, 64: bad root
  uint32_t* maxd;           // optional: max over batches of the deepest non-empty level
};
// a round = init + levels (traverse), then the rows kernel; rounds of
// different state buffers may overlap (rows of round k beside the levels of
// round k + 1)
hipError_t launch_levels128_traverse(const DevGraph& g, const LvArgs& a, hipStream_t s);
hipError_t launch_levels128_rows(const DevGraph& g, const LvArgs& a, hipStream_t s);

// Contracted-graph SPF of cover roots (spf_cover.hip): distances over the
// cover (the nodes outside an independent set of leaves) with shortcut edges
// through transit leaves, then full dist rows (leaves by their last hop).
constexpr uint32_t kCoverMaxS = 32768;  // cover nodes (LDS-resident distances)
struct CoverGraph {
  uint32_t nS, nL;
  const uint32_t* cix;   // [V] cover index, or 0x80000000 | first ladj quad << 5 | quads
  const uint32_t* crow;  // [nS + 1]
  const uint2* cedge;    // [crow[nS]] {target cover index, weight}
  const uint32_t* ctr;   // [(nS + 31) / 32] transit bits
  const uint32_t* lrow;  // [nL + 1] (multiples of 4)
  const uint32_t* ladj;  // [lrow[nL]] cover index | metric (cover -> leaf) << 16; 0xFFFF pads
  // first hops of each C edge from its source (bits of the source's distinct
  // neighbours achieving the edge's weight): cfh[cfh_off[e] .. cfh_off[e+1])
  const uint32_t* cfh_off;  // [crow[nS] + 1]
  const uint32_t* cfh;
  // reverse contracted graph: in-edges of cover node i at crin[i] ..
  // crin[i+1]: {source cover index, weight}, and the edge's index in cedge
  const uint32_t* crin;     // [nS + 1]
  const uint2* cein;
  const uint32_t* ceix;
};
struct CoverArgs {
  const uint32_t* roots;  // node ids (cover nodes)
  uint32_t n;
  uint32_t* dist;         // [n][V] (row i), or row rowpos[i] when rowpos is set
  uint32_t* err;          // bit 64: a root outside the cover
  const uint32_t* rowpos = nullptr;  // [n] row of root i in dist (0xFFFFFFFF: none)
  uint32_t* dcomp = nullptr;         // [n][nS] cover columns out, unreached = kClInf (a
                                     // non-transit root: 0 at itself only -- it relays nothing)
  const uint32_t* dload = nullptr;   // [n][nS] cover columns given: no Dial, rows only
  // load mode with next hops (closure roots): the cover columns' next-hop
  // masks [n][nS][NW] given; the root's next-hop row [V][NW] written at
  // nh + rowpos-independent i * V * NW (leaves: OR over their tight last
  // hops, the root's own leaves their bit) and its digest (zeroed by the
  // caller) accumulated
  const uint32_t* nhload = nullptr;
  uint32_t* nh = nullptr;
  uint32_t NW = 0;
  ospf_digest* digest = nullptr;
  // Dial mode with next hops (seed roots, NW <= kSeedMaxNW): for root i with
  // nhpos[i] != 0xFFFFFFFF the cover nodes' next-hop masks are built during
  // the Dial (a node settled at t ORs its tight in-edges' masks: the root's
  // own edges give their first-hop bits, cfh) into nhm + nhpos[i] * nS * NW,
  // then the next-hop row [V][NW] into nh + nhpos[i] * V * NW and the digest
  // (zeroed by the caller) into digest + nhpos[i]
  const uint32_t* nhpos = nullptr;
  uint32_t* nhm = nullptr;
  // with nhpos: the seeds' full cover columns out at dfull + nhpos[i] * nS
  // and their rows left to launch_seed_rows (another stream)
  uint32_t* dfull = nullptr;
};
// The rows of the seeds whose masks the Dial kept (dfull, nhm from
// cover_spf_kernel): dist + next-hop rows + digests, root k of roots[] at
// dist + rowpos[k] * V, nh + k * V * NW, digest + k.
hipError_t launch_seed_rows(const DevGraph& g, const CoverGraph& C, const uint32_t* roots,
                            uint32_t n, const uint32_t* dfull, const uint32_t* nhm, uint32_t NW,
                            uint32_t* dist, const uint32_t* rowpos, uint32_t* nh,
                            ospf_digest* digest, uint32_t* err, uint32_t n_cu, hipStream_t s);
constexpr uint32_t kSeedMaxNW = 64;
hipError_t launch_cover_spf(const DevGraph& g, const CoverGraph& C, const CoverArgs& a,
                            uint32_t n_cu, hipStream_t s);

// Cover closure (spf_cover.hip closure_kernel): the cover columns of the
// roots of small components of C minus a seed set, from the seeds' cover
// columns: D_f(v) = min( dloc_f(v) for v in f's component,
//                        min over seeds s of cst_f(s) + D_s(v) ),
// cst_f(s) = min over members g usable from f of dloc_f(g) + w(g -> s).
constexpr uint32_t kClosureMaxK = 16;
// unreached in the closure's seed columns, constants and local distances:
// 2^30 (the closure runs when every distance is below it), so a sum of two
// never wraps and any sum with an unreached part stays >= 2^30
constexpr uint32_t kClInf = 0x40000000u;
struct ClosurePlan {
  uint32_t ncomp, nS, chunks;
  const uint2* comp;       // [ncomp] {first seed term, seed terms}
  const uint32_t* jl;      // [terms] seed row in seedC
  const uint32_t* cst;     // [terms][KW] constants per member (unreached: kClInf)
  const uint32_t* mem;     // [ncomp][KW] member cover index (0xFFFFFFFF: none)
  const uint32_t* dloc;    // [ncomp][KW][KW] member f -> member m (unreached: kClInf)
  const uint32_t* out;     // [ncomp][KW] dc row of member f (0xFFFFFFFF: not needed)
  const uint32_t* seedC;   // [seeds][nS] (unreached: kClInf)
  uint32_t* dc;            // [rows][nS] (unreached: 0xFFFFFFFF)
  // next-hop masks (NW words, 0: none; KW = 8): fh [terms][KW][NW], fhloc
  // [ncomp][KW][KW][NW] first hops to the term's seed / to member m; dcm
  // [rows][nS][NW] the cover columns' next hops out (tight terms ORed)
  uint32_t NW = 0;
  const uint32_t* fh = nullptr;
  const uint32_t* fhloc = nullptr;
  uint32_t* dcm = nullptr;
};
constexpr uint32_t kClMaxNW = 4;

// Closure roots' full rows from their cover columns + masks (dc / dcm) by
// node tiles (closure_tile_rows_kernel): tiles of <= kLtNodes consecutive
// nodes whose own / in-link cover indices form a union U of <= kLtU slots,
// <= kLtE entries per node, kLtTiles tiles x kLtRoots roots per block.
constexpr uint32_t kLtNodes = 256, kLtU = 64, kLtE = 16, kLtRoots = 32, kLtTiles = 8;
struct ClosureRowsPlan {
  uint32_t nroots, nS, NW, ntiles;
  const uint32_t* roots;   // [nroots] node ids
  const uint32_t* rcov;    // [nroots] their cover indices
  const uint32_t* rowpos;  // [nroots] dist row positions
  const uint32_t* dc;      // [nroots][nS]
  const uint32_t* dcm;     // [nroots][nS][NW]
  uint32_t* dist;          // rows at dist + rowpos[i] * V
  uint32_t* nh;            // [nroots][V][NW]
  ospf_digest* digest;     // [nroots] (zeroed by the caller)
  const uint4* tile;       // [ntiles] {first node, nodes, first U entry, U size}
  const uint32_t* tle;     // [V][kLtE] slot | 0x100 (own column) or slot | metric << 16;
                           // 0xFFFFFFFF: none
  const uint32_t* tu;      // [U entries] cover indices
};
hipError_t launch_closure_rows(const DevGraph& g, const CoverGraph& C, const ClosureRowsPlan& p,
                               hipStream_t s);
hipError_t launch_closure(const ClosurePlan& p, uint32_t KW, hipStream_t s);

// Weighted derive (spf_wderive.hip): dist + next-hop rows (one word) of n
// leaf roots from the distance rows of their neighbours (src + pos[v] *
// src_pitch = row of node v, kInf: none).
constexpr uint32_t kWdG = 64;     // roots per block
constexpr uint32_t kWdMaxK = 32;  // distinct neighbours of a leaf root
struct WDeriveArgs {
  const uint32_t* roots;
  uint32_t n;
  uint32_t hop;             // hop-count mode: every usable weight is 1
  const uint32_t* src;      // neighbours' distance rows
  uint64_t src_pitch;       // words per src row
  const uint32_t* pos;      // [V]
  uint32_t* dist;           // [n][V]
  uint32_t* nh;             // [n][V] (one word per node) or null
  ospf_digest* digest;      // [n] (zeroed by the caller) or null
  uint32_t* err;            // bit 1: K > 32, 16: a transit neighbour has no row, 64: bad root
  uint32_t vec;             // 16-B aligned rows (V, src_pitch % 4 == 0): uint4 loads / stores
  uint32_t W;               // next-hop words (wide kernels)
  uint32_t G, ctiles;       // roots per block, 256-node subtiles per block (0: defaults)
  uint32_t tiles, chunks;   // set by the launcher
};
hipError_t launch_wderive(const DevGraph& g, WDeriveArgs a, uint32_t kmax, hipStream_t s);

// Weighted next hops of wide cover roots by runs (spf_wderive.hip
// wnh_runs_kernel): runs of <= kWrRun consecutive roots with the same distinct
// neighbours (a plane's spines); block = (run, 64-node tile), lane = node, a
// wave per next-hop word: the word's 32 slot values of the lane's node are
// loaded once (coalesced rows) and every root of the run compares them with
// its own row and metrics.
constexpr uint32_t kWrRun = 40;
constexpr uint32_t kWrTile = 64;
struct WRunsPlan {
  uint32_t nruns, W, tiles;
  const uint4* run;        // {first root, roots, slot offset, -}
  const uint32_t* slots;   // [runs][32 W]: row in src | 0x80000000 | node (relays nothing) | ~0u
  const uint32_t* wt;      // [roots][32 W] metric of the root's usable link per slot (~0u: none)
  const uint32_t* own;     // [roots] row of the root in src
  const uint32_t* rootid;  // [roots] node id
  const uint32_t* src;
  uint64_t pitch;
  uint32_t* nh;            // [roots][V][W]
  ospf_digest* digest;     // [roots] or null (zeroed by the launcher)
  uint32_t nroots;
};
hipError_t launch_wnh_runs(const DevGraph& g, const WRunsPlan& p, hipStream_t s);

// Weighted next hops of narrow cover roots (W <= 4) by hub rows
// (spf_wderive.hip wnh_hub_kernel): the rows many roots read (a fabric's
// spines) are staged per 64-node tile in LDS once per block, each group's own
// rows (a pod's racks and fabric switches) per group; wave = root, lane =
// node, the root's slot refs and metrics block-uniform (scalar loads).
constexpr uint32_t kHubMax = 320;   // hub rows (80 KB of LDS per 64-node tile)
constexpr uint32_t kHubLoc = 64;    // rows of a group
constexpr uint32_t kHubGrpRoots = 16;
constexpr uint32_t kHubTile = 64;
struct HubPlan {
  uint32_t nhub, ngroups, gchunk, tiles, tchunk, W, nroots;
  const uint32_t* hub;     // [nhub] rows in src
  const uint4* grp;        // [ngroups] {first root, roots, first local row, local rows}
  const uint32_t* loc;     // group rows: row in src | 0x80000000 | node (relays nothing)
  const uint32_t* ref;     // [roots][32 W] LDS row per slot: hub j, nhub + group row l, or
                           // nhub + kHubLoc (unreached: an unusable slot)
  const uint32_t* wt;      // [roots][32 W] metric per slot (~0u: unusable)
  const uint32_t* ownl;    // [roots] LDS row of the root's own row (nhub + l)
  const uint32_t* rootid;  // [roots]
  const uint32_t* src;
  uint64_t pitch;
  uint32_t* nh;            // [roots][V][W]
  ospf_digest* digest;     // [roots] or null (zeroed by the launcher)
};
hipError_t launch_wnh_hub(const DevGraph& g, const HubPlan& p, hipStream_t s);
// cover roots (<= 128 distinct neighbours): next-hop words [n][V][W] (W <= 4)
// + digests from the neighbours' rows and the root's own row (all in src)
hipError_t launch_wderive_wide(const DevGraph& g, WDeriveArgs a, uint32_t W, hipStream_t s);
// phase 1: distances only (kp -1) + msbfs_levrows; phase 2: nh_derive
hipError_t launch_msbfs_levels(const DevGraph& g, const MsArgs& a, uint32_t depth_bound,
                               hipStream_t s);
hipError_t launch_nh_derive(const DevGraph& g, const DeriveArgs& d, hipStream_t s);

// Twin derive (spf_twin.hip): next-hop words (W <= 4) of roots whose
// usable transit neighbours fall into few twin classes -- nodes with the
// same usable distinct neighbours and the same transit bit, whose level rows
// agree everywhere except at the members' own positions -- so a tile reads
// one representative row per class instead of one row per neighbour.
constexpr uint32_t kTwinMaxC = 16;
struct TwinArgs {
  const uint32_t* roots;
  uint32_t n, W, cap;
  const uint8_t* lev;
  uint32_t pitch;
  const uint32_t* pos;
  const ospf_digest* lev_digest;
  const uint32_t* tcls;   // [V] twin class of each node
  const uint32_t* trep;   // [classes] representative (smallest id)
  const uint32_t* tsec;   // [classes] second member (kInf: a class of one)
  uint32_t* nh;           // [n][V][W]
  ospf_digest* digest;    // [n] (zeroed by the caller) or null
  uint32_t* err;          // + bit 256: a root with more than kTwinMaxC classes
  uint32_t tiles, ctiles, chunks;
  // the roots' own dist rows at dist + pos[root] * dpitch from their own
  // level bytes, beside the next-hop rows (the sweep's twin levels then write
  // level rows only: their dist rows leave the serial prefix); null: not written
  uint32_t* dist;
  uint32_t dpitch;        // 0: V
  uint32_t npitch;        // next-hop row pitch in words (0: V * W)
  uint32_t bsearch;       // set by the launcher: OSPF_TWIN4_BSEARCH (A/B)
  // twin_levels_kernel: the roots' own rows at pos[root]
};
hipError_t launch_nh_derive_twin(const DevGraph& g, const TwinArgs& a, hipStream_t s);
// Twin levels (twin_levels_kernel): level + dist rows (+ the distance part of
// the digest) of roots from the level rows of their neighbours' twin classes'
// representatives; the caller plans the groups on the host (<= kTwinLvG
// roots, <= kTwinMaxC class rows per group).
constexpr uint32_t kTwinLvG = 8;
struct TwinLvPlan {
  uint32_t n, ngroups;
  uint32_t gsz;           // largest group (0: kTwinLvG); <= 4 takes the 4-root kernel
  const uint32_t* grp;    // [ngroups + 1] root offsets
  const uint32_t* grow;   // [ngroups][kTwinMaxC] class rows (level-row positions; kInf unused)
  const uint4* rinfo;     // [n] {root, own row, mask over the group's class rows, nbl offset}
  const uint32_t* nbo;    // [n + 1] offsets into nbl
  const uint32_t* nbl;    // usable distinct neighbours of each root, ascending (<= 128)
  uint8_t* lev;           // level rows: class rows read, the roots' own rows written
  uint32_t pitch;
  uint32_t* dist;         // [rows][dpitch] or null
  uint32_t dpitch;        // 0: V
  ospf_digest* lev_digest;  // [rows] distance parts (zeroed, then added) or null
  uint32_t parts;         // blocks per group over the node range (0: launcher's choice)
};
hipError_t launch_twin_levels(const DevGraph& g, const TwinLvPlan& a, hipStream_t s);

// Leaf derive (spf_leaf.hip), unit metric / hop count: the level, dist and
// one-word next-hop rows of leaf roots (<= 32 distinct neighbours, every
// usable transit neighbour's level row present) from their neighbours' level
// rows. Roots of a group share their slot table (same distinct neighbours,
// same usable links): each tile's neighbour rows are read once per group.
constexpr uint32_t kLeafMaxG = 64;
struct LeafArgs {
  const uint32_t* roots;  // [n] leaf node ids
  uint32_t n;
  const uint32_t* grp;    // [ngroups + 1] offsets into roots (null: one root per group)
  uint32_t ngroups;
  uint8_t* lev;           // [rows][pitch]: neighbours' rows read, the roots' rows written
  uint32_t pitch;
  const uint32_t* pos;    // [V] row of each node in lev / dist (kInf: none)
  uint32_t* dist;         // [rows][dpitch] (same row index as lev) or null
  const uint32_t* levrow; // [n] level row each root's bytes go to (kInf: not kept); null: pos
  uint32_t* nh;           // [n][npitch] one next-hop word per node, root order
  // row pitches in words (0: V). A pitch of a multiple of 32 words keeps
  // every row 128-B aligned: the 1-KB wave stores then cover whole lines
  // (measured with ospf_probe_store: 7.0 vs 5.8 TB/s for V = 100,024)
  uint32_t dpitch, npitch;
  ospf_digest* digest;    // [n] (zeroed by the caller) or null
  uint32_t* err;
  uint32_t tiles, ctiles; // 1,024-node tiles of the rows, tiles per block
  uint32_t chunks;        // blocks per group (set by the launcher)
  uint32_t group_major;   // block order: 0 = chunk-major (a chunk of every group), 1 = group-major
};
hipError_t launch_leaf_derive(const DevGraph& g, const LeafArgs& a, uint32_t kmax, hipStream_t s);

// Small-graph sweep (spf_small.hip), unit metric / hop count: one wave per
// root, the padded CSR (row offsets, entries, transit bits) copied into LDS
// once per block, each wave's BFS state in its LDS slice. LDS words: graph
// = row offsets (V + 1, rounded to 4) + Ep entries + transit words (rounded
// to 4); per wave = visited bits + u16 levels + u16 queue + V * W next-hop
// words (each rounded to 4 words).
struct SmallLayout {
  uint32_t rp_words, nt_words, graph_words;
  uint32_t vis_words, half_words, wave_words;
};
__host__ __device__ inline SmallLayout small_layout(uint32_t V, uint32_t Ep, uint32_t W) {
  auto r4 = [](uint32_t x) { return (x + 3u) & ~3u; };
  SmallLayout L;
  L.rp_words = r4(V + 1u);
  L.nt_words = r4((V + 31u) / 32u);
  L.graph_words = L.rp_words + r4(Ep) + L.nt_words;
  L.vis_words = L.nt_words;
  L.half_words = r4((V + 1u) / 2u);
  L.wave_words = L.vis_words + 2u * L.half_words + r4(V * W);
  return L;
}
struct SmallArgs {
  const uint32_t* roots;
  uint32_t n;
  uint32_t Ep;            // padded CSR entries (row_ptr[V], a multiple of 4)
  uint32_t waves;         // waves (roots in flight) per block, 1..4
  uint32_t* dist;         // [n][V] or null
  uint32_t* nh;           // [n][V][W] or null
  ospf_digest* digest;    // [n] or null (written, not added)
  uint32_t* err;          // bit 1: a root with more than 32 W distinct neighbours, 64: bad root
};
size_t small_lds_bytes(uint32_t V, uint32_t Ep, uint32_t W, uint32_t waves);
hipError_t launch_lds_sweep(const DevGraph& g, const SmallArgs& a, uint32_t W, hipStream_t s);
// kp = 8, 16 or 32 planes per node; depth_bound bounds the BFS level count
hipError_t launch_msbfs_round(int kp, const DevGraph& g, const MsArgs& a, uint32_t depth_bound,
                              hipStream_t s);
// nh[r][v][w] = w < wcomp ? nhs[r][w][v] : 0 for n rows (whole-line stores)
hipError_t launch_nh_interleave(const uint32_t* nhs, uint32_t* nh, uint32_t n, uint32_t V,
                                uint32_t W, uint32_t wcomp, hipStream_t s);
// KSP2 mode (kp = 0): init + levels [d0, d1) only; lev holds the distances
hipError_t launch_msbfs_ksp(const DevGraph& g, const MsArgs& a, uint32_t d0, uint32_t d1,
                            hipStream_t s);
// ignore masks of the runs of a round: run j of the round (root rix = vb0*64+j)
// ignores ign[rix][0 .. cnt[rix]) (sorted)
hipError_t launch_ksp_masks(const DevGraph& g, const MsArgs& a, const uint32_t* ign,
                            const uint32_t* cnt, uint32_t stride, hipStream_t s);

// KSP2 trace (spf_ksp2.hip): one wave per (source, destination) run walks
// traceOnePath (LinkState.cpp:418-439) over the run's distances; see TraceArgs.
struct TraceArgs {
  uint32_t src;
  const uint32_t* dsts;     // [n]
  uint32_t n;
  const uint32_t* rows;     // rows mode: dist of run i = rows + i * row_stride (0: shared)
  uint64_t row_stride;
  const uint8_t* lev;       // lev mode: [n/64][V][64] dist + 1 of run i at byte i % 64
  const uint32_t* ign;      // [n][stride] run's ignored links, sorted (null: none)
  const uint32_t* ign_cnt;  // [n]
  uint32_t stride;          // words per record (= path_cap)
  uint32_t* out;            // [n][stride] path record
  uint32_t* ign_out;        // k = 1: [n][stride] links of the paths, sorted, UINT32_MAX padded
  uint32_t* cnt_out;        // k = 1: [n]
  uint32_t* status;         // [n]
  uint32_t k;               // 1 or 2
  uint32_t unit;            // every usable metric is 1
  uint32_t* dead;           // [n][dead_words] dead-node bits, zeroed by the caller
  uint32_t dead_words;      // (V + 31) / 32
  uint32_t budget;          // DFS steps before a run goes to the heavy kernel (0 = none)
  uint32_t look;            // lookahead: predecessors with rows <= look entries are probed
  uint32_t src_cut;         // presplit: runs ignoring more of the source's links (0: off)
  uint32_t decr_runs;       // ksp_decr: runs per block (0: persistent blocks)
  uint32_t* pre_bits;       // [n / 32] runs the presplit sent to the full reruns (ksp_decr skips them)
  uint32_t* heavy;          // [n] queued run indices
  uint32_t* heavy_ctr;      // [2] {queued, taken}, zeroed by the caller
  unsigned long long* hlog; // debug (OSPF_KSP_DEBUG=2): [n][4] {run, start, traced, end} clocks of heavy runs
  uint32_t map_fb;          // runs past the decremental map budget: 1 = the full reruns, 0 = the heavy kernel
  // decremental reruns (launch_ksp_decr): rows = the source's dist row
  const uint32_t* tc;       // [V] hint: link of each node's last support (launch_ksp_hint)
  uint32_t* fb;             // [n] runs left to the full masked reruns
  uint32_t* ctr;            // [8] {next run, fallbacks, runs decided, affected nodes, heavy
                            //  queued / taken, A overflows, hash overflows}, zeroed
  uint32_t* err;            // the engine's device error word
  // heavy decremental runs: the source's nodes by level (unit metric,
  // levels < nlvl; launch_ksp_levels) and per-block scratch for the good set
  const uint32_t* ord;      // [V] node ids, level-major
  const uint32_t* lvl_off;  // [nlvl + 1]
  uint32_t nlvl;            // 0: no level order (no pruning)
  uint32_t* good;           // [blocks][dead_words]
  uint32_t* big;            // [blocks][kGoodBig] long-row nodes of a level
};
// the nodes of the source's dist row by level: ord[V], off[257] (levels
// 0..255; farther nodes are left out), cnt: 257 words of scratch
hipError_t launch_ksp_levels(const uint32_t* dist, uint32_t V, uint32_t* ord, uint32_t* off,
                             uint32_t* cnt, hipStream_t s);
constexpr uint32_t kGoodBig = 4096;
hipError_t launch_ksp_trace(bool lev, const DevGraph& g, const TraceArgs& t, hipStream_t s);
// KSP2 k = 2 by decremental SSSP (spf_ksp2.hip): hint[v] = the link id of
// v's last usable in-link (u, v) in row order with u transit (or the
// source) and dist(u) + w(u -> v) == dist(v) in the source's dist row
hipError_t launch_ksp_hint(const DevGraph& g, uint32_t src, const uint32_t* dist, uint32_t* hint,
                           hipStream_t s);
// each run's masked distances from the source's row by propagating the lost
// tight supports of its ignored links, then its k = 2 trace over them;
// runs beyond the kernel's LDS budgets are listed in t.fb (t.ctr[1] of them)
// for the full masked reruns. t.dead: [blocks][dead_words], zeroed.
hipError_t launch_ksp_decr(const DevGraph& g, const TraceArgs& t, uint32_t blocks, hipStream_t s);
uint32_t ksp_decr_blocks_per_cu();
// runs past the decremental kernel's ignore-list budget (the ones it would
// send to the full reruns at once): their indices into list, *count of them
hipError_t launch_ksp_presplit(const DevGraph& g, const TraceArgs& t, uint32_t* list, uint32_t* count,
                               hipStream_t s);
// the runs ksp_decr queued as heavy (t.heavy / t.heavy_ctr): 16 waves each;
// t.dead: [blocks][dead_words]; t.err: the engine's error word
hipError_t launch_ksp_decr_heavy(const DevGraph& g, const TraceArgs& t, uint32_t blocks,
                                 hipStream_t s);
// a[j][0 .. w) = b[idx[j]][0 .. w) (gather = true) or a[idx[j]] = b[j] (scatter), j < n
hipError_t launch_rows_gather(uint32_t* a, const uint32_t* b, const uint32_t* idx, uint32_t n,
                              uint32_t w, bool gather, hipStream_t s);
// st[i] |= bits, i < n
hipError_t launch_or_bits(uint32_t* st, uint32_t n, uint32_t bits, hipStream_t s);
// incremental updates (spf_update.hip): base[idx[i]] = val[i]; affected runs
hipError_t launch_scatter(uint32_t* base, const uint32_t* idx, const uint32_t* val, uint32_t n,
                          hipStream_t s);
// structural patches: a[i] += d for i in [from, n) where a[i] >= thresh and
// a[i] != UINT32_MAX (row offsets / entry positions past a grown row)
// a[0 .. n) = v (a kernel node, also inside captured graphs)
hipError_t launch_fill32(uint32_t* a, size_t n, uint32_t v, hipStream_t s);
// Zero / fill device memory with a kernel instead of hipMemsetAsync: memset
// nodes of a captured sweep graph replayed right after a caller's memset on
// the same stream were seen writing pointer-like values into digest slots
// (ROCm 7.2, gfx950; scripts/debug/replay_parity.py), kernel nodes never.
// OSPF_ZERO_MEMSET=1 restores hipMemsetAsync (the round-4 behaviour), for
// the A/B of scripts/debug/memset_nodes.py.
inline bool zero_by_memset() {
  static const bool m = getenv("OSPF_ZERO_MEMSET") != nullptr;
  return m;
}
inline hipError_t zero_async(void* p, size_t bytes, hipStream_t s) {
  if ((bytes & 3u) || zero_by_memset()) return hipMemsetAsync(p, 0, bytes, s);
  return launch_fill32(static_cast<uint32_t*>(p), bytes / 4u, 0u, s);
}
hipError_t launch_shift_add(uint32_t* a, uint32_t n, uint32_t from, uint32_t thresh, uint32_t d,
                            hipStream_t s);
hipError_t launch_affected(const DevGraph& g, const uint32_t* dist, uint32_t n_roots, bool hop,
                           const ospf_change* ch, uint32_t n_ch, uint8_t* out, hipStream_t s);
struct RepairArgs {
  const uint32_t* roots;
  uint32_t n, W, hop;
  uint32_t* dist;  // [n][V]
  uint32_t* nh;    // [n][V][W]
  const ospf_change* ch;
  uint32_t n_ch;
  uint32_t* status;  // [n] 0 repaired, 1 re-run
};
hipError_t launch_repair(const DevGraph& g, const RepairArgs& a, hipStream_t s);
// out[i] = i * stride, i <= n
hipError_t launch_iota(uint32_t* out, uint32_t n, uint32_t stride, hipStream_t s);

// digests of finished rows, one workgroup per root
hipError_t launch_row_digest(const DevGraph& g, uint32_t n, const uint32_t* dist,
                             const uint32_t* nh, uint32_t W, ospf_digest* out, hipStream_t s);

}  // namespace ospf
