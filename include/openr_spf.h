/*
 * openr_spf.h — C ABI of libopenr_spf_hip, the MI355X batched SPF engine.
 *
 * Drop-in boundary for OpenR's Decision SPF hot path. The reference has no
 * FFI or plugin hook for SPF (openr/plugin/Plugin.h:19-42 is queue-level), so
 * the surface this ABI replaces is the body of one private C++ method:
 *
 *   LinkState::runSpf(src, useLinkMetric, linksToIgnore)
 *                                  openr/decision/LinkState.cpp:836-911
 *                                  (declared openr/decision/LinkState.h:518-525)
 *
 * batched over many roots, plus the graph those calls read
 * (linkMap_/allLinks_/nodeOverloads_, LinkState.h:538-549). The C++ caller (our
 * LinkState mirror, include/openr_decision.h, or the reference's own LinkState
 * after the patch in INTEGRATION.md) keeps the memo, SpfResult reconstruction
 * and route building; this library only computes, per root:
 *   dist[v]   u32, LinkState metric (UINT32_MAX = not reached)
 *   nh[v][w]  next-hop set of v as a bitset over the root's distinct
 *             neighbours in ascending node-id order (bit i = i-th neighbour)
 *   digest    {reached, sum dist, 64-bit hash} (definition: DESIGN.md §Digest)
 *
 * Semantics = the reference's runSpf: edges usable iff
 * Link::isUp (LinkState.cpp:242-245) and not ignored; weight = metric
 * advertised by the relaxing node (Link::getMetricFromNode, LinkState.cpp:193)
 * or 1 in hop-count mode; overloaded nodes other than the root never relax
 * (LinkState.cpp:859-866); nextHops(v) = union over tight transit predecessors
 * u of (u == root ? {v} : nextHops(u)) (LinkState.cpp:885-901).
 *
 * Conventions: every function returns OSPF_OK (0) or a negative OSPF_E_*
 * code; nothing throws or aborts across the ABI; ospf_last_error() explains
 * the last failure. One context per LinkState (area); a context is not
 * thread-safe (the reference calls SPF from the single Decision thread,
 * openr/Main.cpp:515-527). Out-of-contract inputs (metric 0, possible u32
 * distance overflow, > OSPF_MAX_ROOT_NEIGHBORS distinct root neighbours)
 * return OSPF_E_RANGE; there is no CPU fallback.
 */
#ifndef OPENR_SPF_H
#define OPENR_SPF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OSPF_OK 0
#define OSPF_E_INVAL (-1)   /* bad argument */
#define OSPF_E_NOGRAPH (-2) /* no graph loaded */
#define OSPF_E_DEVICE (-3)  /* HIP runtime / device error */
#define OSPF_E_RANGE (-4)   /* input outside the engine's contract */
#define OSPF_E_NOMEM (-5)   /* device allocation failed */

#define OSPF_DIST_INF 0xFFFFFFFFu
#define OSPF_MAX_ROOT_NEIGHBORS 8192u /* nh words <= 256 */
#define OSPF_MAX_IGNORED_PER_RUN 2048u

/* flags for ospf_sssp_batch* */
#define OSPF_HOP_COUNT 0x1u   /* useLinkMetric = false (LinkState.cpp:878) */
#define OSPF_WANT_DIST 0x2u
#define OSPF_WANT_NH 0x4u
#define OSPF_WANT_DIGEST 0x8u

typedef struct ospf_ctx ospf_ctx;

/* Link-state graph snapshot in CSR form (caller-owned, copied on load).
 * Node ids are 0..n_nodes-1; each row lists the directed edges u->col[e] of
 * node u sorted by col ascending (parallel links adjacent). Every undirected
 * link appears twice (once per endpoint); twin[e] is the other entry. */
typedef struct ospf_csr {
  uint32_t n_nodes;
  uint32_t n_edges;            /* directed entries = 2 x links */
  const uint32_t* row_ptr;     /* [n_nodes + 1] */
  const uint32_t* col;         /* [n_edges] neighbour id */
  const uint32_t* metric;      /* [n_edges] metric advertised by the row node, >= 1 */
  const uint32_t* link_id;     /* [n_edges] undirected link id (same for twins) */
  const uint32_t* twin;        /* [n_edges] index of the reverse entry */
  const uint8_t* edge_up;      /* [n_edges] Link::isUp() */
  const uint8_t* no_transit;   /* [n_nodes] LinkState::isNodeOverloaded() */
  /* optional (NULL = keep the given order of parallel entries): position of
   * the entry's link in linksFromNode(row node) iteration
   * (LinkState.cpp:477-485). The engine orders each parallel group of a row
   * by the rank of the twin entry, i.e. by the link's position in the
   * neighbour's linksFromNode, which is the pathLinks order
   * (LinkState.cpp:885-901) the KSP2 trace walks. */
  const uint32_t* link_rank;   /* [n_edges] */
} ospf_csr;

/* Per-run ignored links (LinkState::runSpf linksToIgnore). Run i ignores
 * link_ids[offsets[i] .. offsets[i+1]) (sorted ascending). */
typedef struct ospf_ignore {
  const uint32_t* offsets;  /* [n_roots + 1] */
  const uint32_t* link_ids;
} ospf_ignore;

typedef struct ospf_digest {
  uint64_t reached;
  uint64_t sum_dist;
  uint64_t hash;
} ospf_digest;

typedef struct ospf_graph_info {
  uint32_t n_nodes;
  uint32_t n_edges;
  uint32_t n_links;
  uint32_t max_degree;
  uint32_t max_metric;
  uint32_t unit_metric;        /* every usable edge has metric 1 */
  uint64_t version;
  uint64_t device_bytes;       /* resident graph bytes on the device */
} ospf_graph_info;

/* Open a context on HIP device `device` (ordinal). */
int ospf_open(int device, ospf_ctx** out);
int ospf_close(ospf_ctx* ctx);
const char* ospf_last_error(const ospf_ctx* ctx);

/* Upload (replace) the graph. `version` is the caller's topology version;
 * it is echoed by ospf_graph_info. */
int ospf_load_graph(ospf_ctx* ctx, const ospf_csr* csr, uint64_t version);
int ospf_graph_info_get(const ospf_ctx* ctx, ospf_graph_info* info);

/* Distinct neighbours of `root` in ascending id order = the nh bit order.
 * Writes min(n, cap) ids; *n = total. nh words for root = ceil(n / 32). */
int ospf_root_neighbors(const ospf_ctx* ctx, uint32_t root, uint32_t* ids,
                        uint32_t cap, uint32_t* n);

/* Batched SPF, host buffers, synchronous.
 *   roots[n_roots]; ignore may be NULL (no run ignores anything);
 *   dist_out: [n_roots][n_nodes] when OSPF_WANT_DIST;
 *   nh_out:   [n_roots][n_nodes][nh_words] when OSPF_WANT_NH; nh_words must be
 *             >= ceil(distinct neighbours / 32) of every root in the batch;
 *   digest_out: [n_roots] when OSPF_WANT_DIGEST. */
int ospf_sssp_batch(ospf_ctx* ctx, const uint32_t* roots, uint32_t n_roots,
                    const ospf_ignore* ignore, uint32_t flags, uint32_t nh_words,
                    uint32_t* dist_out, uint32_t* nh_out, ospf_digest* digest_out);

/* Same, device-resident: every pointer is device memory, the work is queued
 * on `stream` (hipStream_t, NULL = default stream) and NOT synchronised.
 * d_dist / d_nh may be NULL when not wanted (the engine then uses its own
 * scratch). d_ign_offsets / d_ign_ids may be NULL; otherwise max_ignored
 * bounds every run's ignore-list length. A run whose root has more than
 * 32 * nh_words distinct neighbours, or whose ignore list exceeds
 * max_ignored, raises the context's device error word: check it with
 * ospf_sync(). */
int ospf_sssp_batch_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n_roots,
                        const uint32_t* d_ign_offsets, const uint32_t* d_ign_ids,
                        uint32_t max_ignored, uint32_t flags, uint32_t nh_words,
                        uint32_t* d_dist, uint32_t* d_nh, ospf_digest* d_digest,
                        void* stream);

/* Device-resident batch with every option in one descriptor. Same contract
 * as ospf_sssp_batch_dev, plus a hint: max_root_neighbors >= the distinct
 * neighbour count of every root in the batch (0 = unknown, 32 * nh_words).
 * It sizes the multi-source BFS (next-hop passes and planes); a root above
 * it raises the device error word like a too-small nh_words. */
typedef struct ospf_batch {
  const uint32_t* d_roots;
  uint32_t n_roots;
  const uint32_t* d_ign_offsets; /* NULL = no run ignores links */
  const uint32_t* d_ign_ids;
  uint32_t max_ignored;
  uint32_t flags;
  uint32_t nh_words;
  uint32_t max_root_neighbors;
  uint32_t* d_dist;
  uint32_t* d_nh;
  ospf_digest* d_digest;
} ospf_batch;
int ospf_run_batch_dev(ospf_ctx* ctx, const ospf_batch* batch, void* stream);

/* Wait for `stream`, then report (and clear) the device error word:
 * OSPF_OK or OSPF_E_RANGE. */
int ospf_sync(ospf_ctx* ctx, void* stream);

/* All-sources next hops in two phases ("derive", unit metric or hop count).
 * ospf_levels_dev: distances of the n device roots by the distance-only
 * multi-source BFS, written as d_dist [n][V] u32 rows (optional), byte level
 * rows d_lev [n][lev_pitch] (dist + 1; 0x7F = unreached and padding;
 * lev_pitch a multiple of 16 >= V; needs a depth bound <= 123, else
 * OSPF_E_RANGE) and, optional, the distance
 * part {reached, sum dist, sum dist_key * (dist + 1)} of each run's digest.
 * ospf_nh_derive_dev: next-hop words [n][V][nh_words] (+ complete digests) of
 * the n device roots from level rows: d_lev_pos[v] = row of node v in d_lev
 * (0xFFFFFFFF: none), d_lev_digest = the level rows' digest parts (needed for
 * d_digest). Every distinct transit neighbour of every root with an up link
 * must have a row (else error bit 16 at ospf_sync); max_root_neighbors (0 =
 * 32 nh_words, at most 2048) bounds the roots' distinct neighbours. Bit k of a
 * root's word k / 32 = its k-th distinct neighbour n is a next hop towards v:
 * an up link, n transit or n == v, and dist(n, v) + 1 == dist(root, v) (the
 * reference's nextHops, LinkState.cpp:885-901). Both queue on `stream`. */
int ospf_levels_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                    uint32_t* d_dist, uint8_t* d_lev, uint32_t lev_pitch,
                    ospf_digest* d_lev_digest, void* stream);
int ospf_nh_derive_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n, uint32_t nh_words,
                       uint32_t max_root_neighbors, const uint8_t* d_lev, uint32_t lev_pitch,
                       const uint32_t* d_lev_pos, const ospf_digest* d_lev_digest,
                       uint32_t* d_nh, ospf_digest* d_digest, void* stream);

/* Next hops (nh_words 1..4) from twin classes (spf_twin.hip), otherwise as
 * ospf_nh_derive_dev. Twins = nodes with the same usable distinct
 * neighbours and the same transit bit: their level rows agree except at the
 * members' own positions (dist(a, v) == dist(b, v) for v outside {a, b},
 * dist(a, b) == dist(b, a); LinkState.cpp:836-911 with unit weights), so a
 * root reads one row per class of its neighbours (a fabric switch: its
 * pod's racks, its plane's spines) instead of one per neighbour.
 * d_twin_class [V] = class of each node, d_twin_rep / d_twin_second
 * [classes] = its smallest member (whose level row is read) and another
 * member (0xFFFFFFFF for a class of one). A root whose usable transit
 * neighbours span more than 16 classes raises error bit 256. */
int ospf_nh_derive_twin_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n, uint32_t nh_words,
                            uint32_t max_root_neighbors, const uint8_t* d_lev,
                            uint32_t lev_pitch, const uint32_t* d_lev_pos,
                            const ospf_digest* d_lev_digest, const uint32_t* d_twin_class,
                            const uint32_t* d_twin_rep, const uint32_t* d_twin_second,
                            uint32_t* d_nh, ospf_digest* d_digest, void* stream);

/* Level + dist rows from twin classes, no traversal (spf_twin.hip; unit
 * metric or hop count, depth bound <= 123). For a root r whose usable transit
 * neighbours fall into <= 16 twin classes (d_twin_class / d_twin_rep as for
 * ospf_nh_derive_twin_dev), every class's representative having a level row
 * in d_lev at d_pos: dist(r, v) = 1 + min over the classes of the
 * representative's dist(rep, v), except 0 at r and 1 at every usable
 * neighbour -- Bellman's equation over r's out-links (LinkState.cpp:836-911,
 * overloaded neighbours reach only themselves, :859-866): twins' rows agree
 * outside their members, and every member of a neighbour class is a usable
 * neighbour of r. Writes r's level row (d_lev at d_pos[r]), its dist row
 * (d_dist + d_pos[r] * V; NULL = not wanted) and the distance part of its
 * digest (d_lev_digest[d_pos[r]], stored; NULL = not wanted). Error bits at
 * ospf_sync: 1 (> 128 distinct neighbours), 16 (a class row missing), 256
 * (> 16 classes, or > 16 distinct class rows in a group). d_groups
 * [n_groups + 1]: offsets into the roots, <= 8 roots per group, the roots of
 * a group reading <= 16 class rows together (each chunk's rows loaded once
 * for the group); NULL = one root per group. On a fabric the fabric
 * switches' rows come from one rack row of their pod and one spine row of
 * their plane (group = a pod's fabric switches). */
int ospf_twin_levels_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n,
                         const uint32_t* d_groups, uint32_t n_groups, uint8_t* d_lev,
                         uint32_t lev_pitch, const uint32_t* d_pos, const uint32_t* d_twin_class,
                         const uint32_t* d_twin_rep, uint32_t* d_dist, ospf_digest* d_lev_digest,
                         void* stream);

/* All-sources rows of leaf roots from level rows (unit metric or hop count;
 * spf_leaf.hip). A leaf r (no two leaves adjacent, <= 32 distinct
 * neighbours n_k) has dist(r, v) = 1 + min_k dist(n_k, v) over n_k with an
 * up link r-n_k (a non-transit n_k reaches only itself) and next hops = the
 * tight n_k -- LinkState::runSpf's Bellman equation over the root's
 * out-links (LinkState.cpp:836-911, :859-866, :885-901). Reads the level rows
 * of every usable transit neighbour (d_lev at d_pos[n], e.g. from
 * ospf_levels_dev) and writes the roots' own level rows and dist rows at
 * d_pos[root] (d_dist [rows][V], NULL = not wanted), one-word next-hop rows
 * d_nh [n][V] in root order and complete digests d_digest [n] (NULL = not
 * wanted). Groups: d_groups [n_groups + 1] offsets into the roots, <= 64
 * roots each, every root of a group with the same distinct neighbours and
 * usable links (the racks of a pod: a tile's neighbour rows are read once
 * per group; a group that is not uniform raises error bit 128); NULL = one
 * root per group. max_root_neighbors (0 = 32) bounds every root's distinct
 * neighbours. Needs a depth bound <= 123. Queued on `stream`. */
int ospf_leaf_derive_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n,
                         const uint32_t* d_groups, uint32_t n_groups, uint32_t max_root_neighbors,
                         uint8_t* d_lev, uint32_t lev_pitch, const uint32_t* d_pos,
                         uint32_t* d_dist, uint32_t* d_nh, ospf_digest* d_digest, void* stream);

/* Same, with d_lev_out [n] (device): the level row each root's level bytes
 * are written to, 0xFFFFFFFF = not kept (their dist and next-hop rows are
 * still written); NULL = d_pos[root] (ospf_leaf_derive_dev). A sweep keeps
 * only the rows its next-hop launches read: one per twin class. */
int ospf_leaf_derive2_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n,
                          const uint32_t* d_groups, uint32_t n_groups,
                          uint32_t max_root_neighbors, uint8_t* d_lev, uint32_t lev_pitch,
                          const uint32_t* d_pos, const uint32_t* d_lev_out, uint32_t* d_dist,
                          uint32_t* d_nh, ospf_digest* d_digest, void* stream);

/* All-sources rows of small graphs in one launch (spf_small.hip), unit
 * metric or OSPF_HOP_COUNT: a wave per root, the padded CSR and the root's
 * BFS state (visited bits, u16 levels, queue, next-hop words) in LDS --
 * LinkState::runSpf (LinkState.cpp:836-911) with unit weights, next hops as
 * :885-901 (the first hops of the shortest paths; overloaded nodes never
 * relay, :859-866). Writes d_dist [n][V], d_nh [n][V][nh_words] and
 * d_digest [n] (each NULL = not wanted); nh_words 1..4 must cover every
 * root's distinct neighbours (else error bit 1 at ospf_sync). flags may
 * carry OSPF_HOP_COUNT (the WANT bits are ignored: the buffers decide).
 * OSPF_E_RANGE when the graph is outside the kernel's contract (V > 65535,
 * or the CSR + one root's state does not fit in LDS): ospf_lds_sweep_fits
 * says beforehand. Queued on `stream`. Replaces the per-node
 * Decision::getDecisionRouteDb loop (Decision.cpp:309) for small areas. */
int ospf_lds_sweep_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                       uint32_t nh_words, uint32_t* d_dist, uint32_t* d_nh,
                       ospf_digest* d_digest, void* stream);
int ospf_lds_sweep_fits(const ospf_ctx* ctx, uint32_t flags, uint32_t nh_words);

/* Weighted all-sources rows of leaf roots (any metric, or OSPF_HOP_COUNT; no
 * ignored links). For a root r with distinct neighbours n_k, w_k = the
 * smallest metric r advertises on an up link to n_k and D_k = the distance row
 * of n_k (d_src + d_pos[n_k] * src_pitch, computed by any engine path with the
 * same flags): dist(r, v) = min_k w_k + D_k(v) over transit n_k (an overloaded
 * n_k only reaches itself, at w_k), and bit k of next-hop word 0 of v is set
 * iff n_k's term is tight -- the reference's runSpf (LinkState.cpp:836-911:
 * Bellman's equation over the root's out-links; nextHops = the first hops of
 * the shortest paths, :885-901). Writes d_dist [n][V], d_nh [n][V] (one word
 * per node; NULL = not wanted) and d_digest [n] (NULL = not wanted). Every
 * root must have <= max_root_neighbors (1..32, 0 = 32) distinct neighbours,
 * each transit one with an up link needing a row (else error bits 1 / 16 at
 * ospf_sync). The caller derives an independent set of roots (no two
 * adjacent: the racks of a fabric) from the rows of the others. */
int ospf_wderive_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                     uint32_t max_root_neighbors, const uint32_t* d_src, uint64_t src_pitch,
                     const uint32_t* d_pos, uint32_t* d_dist, uint32_t* d_nh,
                     ospf_digest* d_digest, void* stream);

/* Distance rows of cover roots on weighted graphs (the cover = the nodes
 * outside an independent set of leaves, e.g. the fabric and spine switches
 * when the racks are the leaves). ospf_cover_prepare builds the contracted
 * graph from the loaded graph: leaf_mask[V] (host) = 1 for leaves, no two of
 * them adjacent; cover nodes <= 32768, leaf in-link metrics <= 65535 (else
 * OSPF_E_RANGE). Shortest paths between cover nodes cross leaves only as
 * single-node detours through transit leaves, so the cover's distances are
 * those of the cover plus one shortcut edge per transit leaf detour, and a
 * leaf's distance is the minimum over its up in-links (LinkState.cpp:836-911
 * with metrics >= 1). ospf_cover_dist_dev writes d_dist [n][V] (link metrics;
 * no ignored links) for n cover roots (node ids; a leaf root raises error bit
 * 64). The prepared graph is tied to the graph version: prepare again after
 * ospf_load_graph / ospf_update_*. Next hops then come from ospf_wderive_dev
 * (leaves) and ospf_wderive_wide_dev (cover roots). */
int ospf_cover_prepare(ospf_ctx* ctx, const uint8_t* leaf_mask);
int ospf_cover_dist_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n, uint32_t* d_dist,
                        void* stream);

/* Next hops of roots with up to 128 distinct neighbours (nh_words 1..4), any
 * metric: every row -- the roots' own and their transit neighbours' -- is in
 * d_src at d_pos[] (computed with the same flags: ospf_cover_dist_dev for the
 * cover, ospf_wderive_dev for the leaves); bit k of v is set iff w_k + D_k(v)
 * == D_root(v) with n_k transit, or v == n_k and w_k == D_root(v) (the first
 * hops of the shortest paths, LinkState.cpp:885-901). Writes d_nh
 * [n][V][nh_words] and the complete digests (dist part from the own row). */
int ospf_wderive_wide_dev(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                          uint32_t nh_words, const uint32_t* d_src, uint64_t src_pitch,
                          const uint32_t* d_pos, uint32_t* d_nh, ospf_digest* d_digest,
                          void* stream);

/* Kernel variant the engine would use for a large batch (for reporting):
 * 0 = Dial, LDS-resident (dist+nh in LDS), 1 = Dial, LDS dist + HBM
 * next-hops, 2 = Dial, HBM state, 3 = per-root BFS with LDS bitmaps and LDS
 * byte next-hops, 4 = per-root BFS with HBM next-hops, 5 = multi-source
 * bit-parallel BFS (64 roots per traversal; unit metric, no ignored links). */
int ospf_plan_variant(const ospf_ctx* ctx, uint32_t flags, uint32_t nh_words,
                      int* variant);

/* Full launch plan the engine would use for a batch (reporting / profiling). */
typedef struct ospf_plan_info {
  int32_t variant;       /* as ospf_plan_variant */
  uint32_t block;        /* threads per workgroup */
  uint32_t lds_bytes;    /* dynamic LDS per workgroup */
  uint32_t slices;       /* workgroups per SPF run (next-hop slices); variant 5:
                            passes per 64-root batch */
} ospf_plan_info;
int ospf_plan(const ospf_ctx* ctx, uint32_t flags, uint32_t nh_words, uint32_t max_ignored,
              ospf_plan_info* out);
/* Same for a batch of n_roots roots with the given neighbour hint (variant 5:
 * slices = next-hop passes per 64-root batch). */
int ospf_plan_n(const ospf_ctx* ctx, uint32_t flags, uint32_t nh_words, uint32_t max_ignored,
                uint32_t n_roots, uint32_t max_root_neighbors, ospf_plan_info* out);

/* KSP2 edge-disjoint paths (LinkState::getKthPaths k = 1 and k = 2,
 * LinkState.cpp:790-819, with traceOnePath :418-439) from one source to many
 * destinations, computed on the device: the link-metric SPF of src; per
 * destination the greedy edge-disjoint trace over its pathLinks (k = 1);
 * the masked SPF rerun that ignores every link of the k = 1 paths and the
 * trace over it (k = 2). Records (u32, per destination and k, path_cap words):
 *   n_paths, then per path: len, link ids (ospf_csr link_id) from src to dst.
 * status[i] bits: OSPF_KSP_RERUN = destination i's k = 2 needed a masked SPF
 * (its k = 1 paths are not empty, LinkState.cpp:802-806); OSPF_KSP_OVF1 /
 * OSPF_KSP_OVF2 = the k = 1 / k = 2 record was not computed (record or trace
 * budget exceeded: path_cap, 256 links deep, 1536 links visited); the caller
 * computes those destinations itself. src == dst and unreached destinations
 * give empty records (no paths). The graph must be loaded with link_rank for
 * the reference's parallel-link order. */
#define OSPF_KSP_RERUN 0x1u
#define OSPF_KSP_OVF1 0x2u
#define OSPF_KSP_OVF2 0x4u
typedef struct ospf_ksp2 {
  uint32_t src;
  const uint32_t* dsts;  /* [n] node ids */
  uint32_t n;
  uint32_t path_cap;     /* words per record, 2 .. OSPF_MAX_IGNORED_PER_RUN */
  uint32_t* k1;          /* [n][path_cap] */
  uint32_t* k2;          /* [n][path_cap] */
  uint32_t* status;      /* [n] */
} ospf_ksp2;
/* host buffers, synchronous */
int ospf_ksp2_run(ospf_ctx* ctx, const ospf_ksp2* args);
/* device buffers, queued on `stream` (hipStream_t); the engine waits on the
 * stream itself between rounds only when a masked run is deeper than the
 * graph's static depth bound. */
int ospf_ksp2_dev(ospf_ctx* ctx, const ospf_ksp2* args, void* stream);
/* The k = 2 masked reruns run as decremental SSSP from the source's row (the
 * nodes whose every tight in-link the ignored links cut, directly or through
 * other such nodes, get new distances; the rest keep the source's) with the
 * trace fused in one launch; a run past that kernel's LDS budgets takes the
 * full masked rerun. Cumulative counts of this context since open: out3 =
 * {runs by the decremental kernel, runs sent to the full reruns, affected
 * nodes summed over the decremental runs}. OSPF_KSP_NODECR in the environment
 * sends every run to the full reruns. */
int ospf_ksp2_stats(const ospf_ctx* ctx, uint64_t* out3);

/* Incremental updates (Decision.cpp:918-996 re-runs SPF after
 * every debounced adjacency batch; LinkState clears every memoised result on
 * a topology change, LinkState.cpp:751-754). When a batch changes only link
 * metrics, link up/down state or node overload bits -- no link or node added
 * or removed -- the resident device CSR is patched in place instead of
 * reloaded, and ospf_affected_roots tells which of a set of finished runs can
 * differ under the new state; the others are bit-identical and need no rerun.
 *
 * Link update: the two CSR entries of link_id get Link::isUp() = up and the
 * metrics advertised by each endpoint (metric_lo: the endpoint with the lower
 * node id). Node update: LinkState::isNodeOverloaded. `version` is the
 * caller's new topology version. */
typedef struct ospf_link_update {
  uint32_t link_id;
  uint32_t up;
  uint32_t metric_lo;
  uint32_t metric_hi;
} ospf_link_update;
int ospf_update_links(ospf_ctx* ctx, const ospf_link_update* updates, uint32_t n,
                      uint64_t version);
int ospf_update_nodes(ospf_ctx* ctx, const uint32_t* nodes, const uint8_t* no_transit,
                      uint32_t n, uint64_t version);

/* Structural update in place: links added or removed between existing nodes
 * -- LinkState's [LINK UP] / [LINK DOWN] (LinkState.cpp:632-657; Decision
 * applies them per adjacency database, Decision.cpp:743-765). `csr` is the
 * caller's whole CSR after the change (same nodes and node ids, any link ids:
 * a removed link's id simply no longer appears, an added link may take a new
 * or a retired id), `rows` the nodes whose rows changed (both ends of every
 * added / removed link). The engine rebuilds those rows (and, when a row's
 * parallel links to a neighbour may have been reordered, that neighbour's
 * row) in their padded slots, moving the rows after a row that outgrows its
 * slots, and refreshes the distinct-neighbour lists, link positions and
 * planner bounds. O(changed rows) host work plus device copies; sweeps made
 * before the call return OSPF_E_NOGRAPH. OSPF_E_RANGE when the layout's
 * reserve (~3 % of entries, distinct neighbours, link ids) is exhausted, a
 * metric leaves the contract, or the node count differs: reload with
 * ospf_load_graph. On any error the context is unchanged except after a
 * device error (then reload). */
int ospf_update_rows(ospf_ctx* ctx, const ospf_csr* csr, const uint32_t* rows, uint32_t n,
                     uint64_t version);

/* One change of a batch, for ospf_affected_roots. LINK: endpoints a, b;
 * before / after: up, metric advertised by a (w_ab) and by b (w_ba). NODE:
 * node a changed its overload bit (either way). */
#define OSPF_CHANGE_LINK 0u
#define OSPF_CHANGE_NODE 1u
typedef struct ospf_change {
  uint32_t kind;
  uint32_t a, b;
  uint32_t up0, w_ab0, w_ba0;
  uint32_t up1, w_ab1, w_ba1;
} ospf_change;
/* Which finished runs can change: d_dist = their distance rows ([n_roots][V],
 * device, computed before the batch), flags as the runs were made (only
 * OSPF_HOP_COUNT is read); d_affected[i] = 1 if run i must be re-run, 0 if
 * its dist / next hops / pathLinks are unchanged. Run i is unaffected when no
 * changed link was tight for it before (dist(a) + w_ab0 == dist(b), or the
 * reverse) nor reaches or ties a distance after (dist(a) + w_ab1 <= dist(b),
 * or the reverse), and every re-flagged node either is unreached, is the root,
 * or has no up link (x, y) with dist(x) + w(x -> y) <= dist(y) (transit
 * conditions are ignored: the answer errs towards re-running). Graph state
 * read for node changes: the current (patched) one. Queued on `stream`. */
int ospf_affected_roots(ospf_ctx* ctx, const uint32_t* d_dist, uint32_t n_roots, uint32_t flags,
                        const ospf_change* changes, uint32_t n_changes, uint8_t* d_affected,
                        void* stream);

/* Repair finished runs in place after a patch (ospf_update_links /
 * ospf_update_nodes): d_dist / d_nh hold rows computed before the batch
 * ([n][V], [n][V][nh_words], device) for roots d_roots, made with `flags`
 * (OSPF_HOP_COUNT read). A run none of whose shortest distances the batch
 * changes -- only next-hop sets and ties move, the usual effect of a link
 * event in an ECMP fabric -- gets its next-hop words re-derived where they
 * change (d_status[i] = 0: the rows now equal a fresh run's). Link changes
 * and overload toggles (node changes: the current transit bit is read) are
 * both repaired. A run whose distances would change, or beyond the repair
 * budget (8192 re-derivations, 1024 queued nodes), gets d_status[i] = 1 and
 * must be re-run. Digests are not maintained. Queued on `stream`. */
int ospf_repair_runs(ospf_ctx* ctx, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                     uint32_t nh_words, uint32_t* d_dist, uint32_t* d_nh,
                     const ospf_change* changes, uint32_t n_changes, uint32_t* d_status,
                     void* stream);

/* Take links down for a while and put back exactly what was there. The
 * reference reruns runSpf(src, true, linksToIgnore) with every link of the
 * k = 1 paths ignored (LinkState.cpp:802-806); an ignore set beyond one
 * run's list (OSPF_MAX_IGNORED_PER_RUN) is applied to the device graph
 * instead. ospf_links_mask marks the links down (like ospf_update_links);
 * ospf_links_unmask restores their entries and the planner state (level and
 * distance bounds, metric facts, the prepared cover graph), so the pair
 * leaves no trace in later runs. One mask at a time. */
int ospf_links_mask(ospf_ctx* ctx, const uint32_t* link_ids, uint32_t n, uint64_t version);
int ospf_links_unmask(ospf_ctx* ctx);

/* ---------------------------------------------------------------- sweeps
 * All-sources sweeps: runSpf (LinkState.cpp:836-911) for every node of the
 * graph -- or for one part of a root partition (multi-GPU) -- with every
 * root's dist row and next-hop row written to device memory the sweep owns,
 * plus a digest per root. The reference's all-sources use is
 * Decision::getDecisionRouteDb(node) for every node (openr/decision/
 * Decision.cpp:309) and `breeze decision routes --nodes all` (openr/py/openr/
 * cli/commands/decision.py:26-48): one getSpfResult per node. A sweep owns
 * the whole orchestration -- the path, the root order, the width classes,
 * their streams and the HIP graph one run replays:
 *   OSPF_SWEEP_DERIVE  unit metric or hop count, depth bound <= 123, <= 2048
 *                      distinct neighbours per node: distance-only 128-root
 *                      BFS over the closure of the roots, then each root's
 *                      next hops from its neighbours' level rows
 *                      (ospf_levels_dev + ospf_nh_derive_dev);
 *   OSPF_SWEEP_WCOVER  link metrics: distance rows of a vertex cover by the
 *                      contracted-graph SPF, leaf rows and cover next hops
 *                      derived from them (ospf_cover_*, ospf_wderive*_dev);
 *   OSPF_SWEEP_WDERIVE cover rows on the per-root batch path, leaf rows
 *                      derived (any metric, or hop count);
 *   OSPF_SWEEP_BATCH   per width class batches (ospf_run_batch_dev);
 *   OSPF_SWEEP_LDS     small graphs, unit metric or hop count, <= 4 next-hop
 *                      words: one launch per width class, a wave per root
 *                      with the graph in LDS (ospf_lds_sweep_dev);
 *   OSPF_SWEEP_WMULTI  any metric (or hop count), large graphs without a
 *                      small cover (meshes): the rows the part needs by a
 *                      multi-root traversal (groups of 32 roots adjacent in
 *                      id order, [node][root] distances, Delta-stepping),
 *                      leaf rows and next hops derived from them.
 * OSPF_SWEEP_AUTO takes LDS when it applies, then the others in the order
 * above. Row layout:
 * dist u32[V] per root; next hops u32[V][W] with W = max(1, ceil(distinct
 * neighbours / 32)) words in the bit order of ospf_root_neighbors. A sweep
 * belongs to the graph it was created on: after ospf_load_graph,
 * ospf_update_* or ospf_links_mask, ospf_sweep_run returns OSPF_E_NOGRAPH
 * (rows already computed stay readable). Partition (n_parts > 1): each width
 * class, ordered by each node's largest neighbour id, is cut into n_parts
 * contiguous slices -- a fabric's racks and fabric switches by pod, its
 * spines by plane -- so a part's closure stays small. */
#define OSPF_SWEEP_AUTO 0u
#define OSPF_SWEEP_DERIVE 1u
#define OSPF_SWEEP_WCOVER 2u
#define OSPF_SWEEP_WDERIVE 3u
#define OSPF_SWEEP_BATCH 4u
#define OSPF_SWEEP_LDS 5u
#define OSPF_SWEEP_WMULTI 6u
/* opts.flags: create without the eager first run (hip_graph must be 0); the
 * first ospf_sweep_run is then the first run. A caller that runs the sweep
 * once per graph version (odl::LinkState; ospf_msweep_create, which starts
 * every device's first run together) pays one run instead of two. */
#define OSPF_SWEEP_DEFER 0x100u
/* opts.flags, with OSPF_SWEEP_DEFER: the first run starts inside
 * ospf_sweep_create -- each launch unit of the plan's serial prefix (derive
 * mode: the seed BFS and the twin levels) is queued as soon as it is planned,
 * ordered after the null stream's prior work, so the device works on it while
 * the host plans the rest; the first ospf_sweep_run queues the remaining
 * units and joins the caller's stream. For a caller that runs the sweep right
 * after creating it on an unchanged graph (odl::LinkState's re-sweep after a
 * topology change). */
#define OSPF_SWEEP_EARLY_START 0x200u

typedef struct ospf_sweep ospf_sweep;
typedef struct ospf_sweep_opts {
  uint32_t flags;      /* 0 (link metrics) or OSPF_HOP_COUNT, | OSPF_SWEEP_DEFER
                          (| OSPF_SWEEP_EARLY_START) */
  uint32_t mode;       /* OSPF_SWEEP_* */
  uint32_t part;       /* this part of the root partition ... */
  uint32_t n_parts;    /* ... over n_parts (0 or 1: every node) */
  uint32_t hip_graph;  /* 1: capture one run as a HIP graph, runs replay it
                          (eager launches if capture fails: see info) */
} ospf_sweep_opts;

typedef struct ospf_sweep_info {
  uint32_t mode;             /* the path taken (OSPF_SWEEP_*) */
  uint32_t n_roots;          /* roots this part owns */
  uint32_t n_rows;           /* distance rows computed per run (closure / cover rows) */
  uint32_t n_launches;       /* launch units (ospf_sweep_profile) */
  uint32_t hip_graph;        /* 1: runs replay a captured graph */
  uint32_t max_nh_words;     /* widest next-hop row of an owned root */
  uint64_t device_bytes;     /* rows, level rows, digests, tables */
  uint64_t step_compulsory_bytes;  /* rows written + CSR scans, per run */
  /* edges the run's traversal kernels relax: traversed rows x edges of the
   * graph they traverse (derive: seed BFS rows x E; weighted cover: seeds'
   * Dial rows x contracted-graph edges; batch / LDS: roots x E). Rows
   * derived from other rows relax no edge. TEPS = this / run time. */
  uint64_t step_traversed_edges;
} ospf_sweep_info;

/* One launch unit of a run, timed alone on its stream (HIP events). */
typedef struct ospf_sweep_launch {
  char name[32];
  char kernel[112];
  uint32_t n_roots;          /* runs the launch computes */
  uint32_t nh_words;         /* 0 = distance rows only */
  uint64_t compulsory_bytes; /* rows written + CSR / source rows read at least once */
  double ms_median;          /* isolated launch time, median of the reps */
  double ms_min;
} ospf_sweep_launch;

int ospf_sweep_create(ospf_ctx* ctx, const ospf_sweep_opts* opts, ospf_sweep** out);
int ospf_sweep_destroy(ospf_sweep* sw);
const char* ospf_sweep_last_error(const ospf_sweep* sw);
int ospf_sweep_get_info(const ospf_sweep* sw, ospf_sweep_info* info);
/* The owned roots, in digest order ([n_roots] host). */
int ospf_sweep_roots(const ospf_sweep* sw, uint32_t* roots);
/* One all-sources run queued on `stream` (hipStream_t; not synchronised;
 * ospf_sync(ctx, stream) reports device errors). */
int ospf_sweep_run(ospf_sweep* sw, void* stream);
/* Digests of the owned roots in ospf_sweep_roots order into device memory
 * d_out[n_roots], queued on `stream`. */
int ospf_sweep_digests(ospf_sweep* sw, ospf_digest* d_out, void* stream);
/* Same into host memory out[n_roots], synchronous. */
int ospf_sweep_digests_host(ospf_sweep* sw, ospf_digest* out);
/* Fill every digest the sweep keeps with 0xFF (a run rewrites them all; a
 * run that did nothing is then visible). */
int ospf_sweep_poison(ospf_sweep* sw, void* stream);
/* Device rows of an owned root (valid until ospf_sweep_destroy). */
int ospf_sweep_row(const ospf_sweep* sw, uint32_t root, const uint32_t** d_dist,
                   const uint32_t** d_nh, uint32_t* nh_words);
/* Host copies of owned roots' rows, synchronous (after the work queued on
 * every stream is done): dist_out [n][V] and nh_out [n][V][nh_words] (each
 * root's W words, zero padded; nh_words >= every root's W), either may be
 * NULL. */
int ospf_sweep_copy_rows(ospf_sweep* sw, const uint32_t* roots, uint32_t n, uint32_t nh_words,
                         uint32_t* dist_out, uint32_t* nh_out);
/* Time every launch unit alone on its stream: reps (>= 1) timed launches
 * after one untimed one; fills min(cap, n_launches) records. The sweep must
 * have run once. */
int ospf_sweep_profile(ospf_sweep* sw, uint32_t reps, ospf_sweep_launch* out, uint32_t cap);
/* Diagnostic: the memset nodes of the sweep's captured HIP graph (none
 * unless OSPF_ZERO_MEMSET=1 routes the engine's zeroing through
 * hipMemsetAsync): how many (n_memset), how many whose destination range is
 * not inside a live device allocation (n_dead), how many inside the
 * sweep's own blocks (n_own). */
int ospf_sweep_graph_memsets(const ospf_sweep* sw, uint32_t* n_memset, uint32_t* n_dead,
                             uint32_t* n_own);

/* ---------------------------------------------------------------- devices
 * Several devices of one node behind one handle (SURVEY.md §8(b) ospf_open
 * with n_gpus; Decision runs in one process on one thread,
 * openr/Main.cpp:515-527, so the drop-in reaches the node's GPUs from
 * there). The graph is replicated on every device; an all-sources sweep runs
 * part i of the root partition on device i (no data-path exchange: every
 * run is independent, rows stay device-local); the 24-B digests are gathered
 * onto the first device by peer copies. Devices may repeat (several
 * contexts on one device: a test of the partition on a one-GPU box). */
typedef struct ospf_multi ospf_multi;
typedef struct ospf_msweep ospf_msweep;
int ospf_multi_open(const int* devices, uint32_t n, ospf_multi** out);
int ospf_multi_close(ospf_multi* m);
const char* ospf_multi_last_error(const ospf_multi* m);
uint32_t ospf_multi_size(const ospf_multi* m);
/* the context of device slot i (owned by m) */
ospf_ctx* ospf_multi_ctx(ospf_multi* m, uint32_t i);
int ospf_multi_load_graph(ospf_multi* m, const ospf_csr* csr, uint64_t version);
/* One sweep per device slot (opts->part / n_parts are set per slot). */
int ospf_msweep_create(ospf_multi* m, const ospf_sweep_opts* opts, ospf_msweep** out);
int ospf_msweep_destroy(ospf_msweep* ms);
/* Queue one run on every device and wait for all of them. */
int ospf_msweep_run(ospf_msweep* ms);
/* Digests of every node by node id (host [V]). With distinct devices the
 * parts' 24-B records (padded to the largest part) are all-gathered by ONE
 * RCCL ncclAllGather over xGMI (communicators from ncclCommInitAll in this
 * process, made once per ospf_multi); with a device given twice (RCCL takes
 * one rank per GPU) or OSPF_RCCL=0, peer copies onto the first device. Then
 * one scatter by root id and one copy back. OSPF_RCCL=1 takes RCCL for a
 * single device too (a one-rank communicator). */
int ospf_msweep_digests(ospf_msweep* ms, ospf_digest* out_by_node);
/* 1: this sweep's digests are gathered by RCCL, 0: by peer copies. */
uint32_t ospf_msweep_gather_backend(const ospf_msweep* ms);
/* The slot's sweep (row access, info) and the slot owning `root`. */
ospf_sweep* ospf_msweep_part(ospf_msweep* ms, uint32_t slot);
int ospf_msweep_owner(const ospf_msweep* ms, uint32_t root, uint32_t* slot);

/* Runtime statistics. spf_runs counts logical runSpf executions (one per
 * root per batch), matching the reference's decision.spf_runs counter
 * (LinkState.cpp:843). */
uint64_t ospf_spf_runs(const ospf_ctx* ctx);

/* Test hook (fault injection): the after_calls-th call from now of
 * ospf_load_graph / ospf_sssp_batch / ospf_ksp2_run / ospf_sweep_create /
 * ospf_sweep_run / ospf_sweep_copy_rows on this context fails with
 * OSPF_E_DEVICE and does nothing (0 = off). Lets the caller's handling of a
 * device error be tested without a faulting GPU. */
int ospf_inject_error(ospf_ctx* ctx, uint32_t after_calls);

/* Box calibration (no reference counterpart: measurement).
 * The HBM store rate of this device, timed with HIP events: 2 * rows * V * 4
 * bytes written with 16-B non-temporal stores per launch, `reps` timed
 * launches after one untimed one, ms_out[reps]. pattern 0 = one buffer in
 * address order; 1 = two [rows][V] u32 arrays written the way the leaf
 * launch writes its dist and next-hop rows (blocks of `group` rows x
 * `ctiles` 1,024-node tiles, chunk-major); 2 = the same blocks group-major;
 * 3 = persistent blocks (`ctiles` per CU) taking (group, tile) items in
 * group-major order (the chip walks the rows in order).
 * Allocates (and frees) its own buffer: OSPF_E_NOMEM when it does not fit.
 * V must be a multiple of 4. */
#define OSPF_PROBE_STREAM 0u
#define OSPF_PROBE_ROWS_CHUNK 1u
#define OSPF_PROBE_ROWS_GROUP 2u
#define OSPF_PROBE_ROWS_WALK 3u
int ospf_probe_store(ospf_ctx* ctx, uint32_t pattern, uint32_t V, uint32_t rows, uint32_t group,
                     uint32_t ctiles, uint32_t reps, float* ms_out);

#ifdef __cplusplus
}
#endif

#endif /* OPENR_SPF_H */
