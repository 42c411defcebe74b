/*
 * openr_decision.h — C ABI of libopenr_decision, the host-side mirror of
 * OpenR's LinkState (openr/decision/LinkState.{h,cpp}) whose SPF runs on the
 * MI355X engine (include/openr_spf.h).
 *
 * The C++ class (openr_amd/csrc/decision/link_state.h, namespace odl) keeps
 * the reference's public surface and semantics:
 *   updateAdjacencyDatabase  LinkState.cpp:584-726 -> odl_apply (odl_apply_hold: TTLs)
 *   decrementHolds, hasHolds LinkState.cpp:520-548 -> odl_decrement_holds, odl_has_holds
 *   deleteAdjacencyDatabase  LinkState.cpp:728-746 -> odl_apply (db_delete=1)
 *   linksFromNode            LinkState.cpp:477-485 -> odl_links_text
 *   isNodeOverloaded         LinkState.cpp:515-518 -> odl_is_overloaded
 *   getSpfResult             LinkState.cpp:821-831 -> odl_spf_text
 *   getKthPaths              LinkState.cpp:790-819 -> odl_kth_paths_text
 *   getMetricFromAToB        LinkState.cpp:777-788 -> odl_metric_a_to_b
 *   decision.spf_runs        LinkState.cpp:843     -> odl_spf_runs
 *   resolveUcmpWeights       LinkState.cpp:913-1033 -> odl_ucmp_text
 * plus batched entry points the reference lacks (all-sources digests, KSP2
 * masked reruns for many destinations, per-neighbour reruns).
 *
 * This ABI exists for tests, benches and non-C++ callers; a C++ Decision
 * module links the class directly. Text results use the format documented
 * in DESIGN.md §Result text (same as the oracle's). Returned strings are
 * malloc'd; free them with odl_free(). NULL / negative return = error, see
 * odl_last_error().
 */
#ifndef OPENR_DECISION_H
#define OPENR_DECISION_H

#include <stdint.h>

#include "openr_adjdb.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct odl_ls odl_ls;

/* New LinkState for `area` whose SPF engine runs on HIP device `device`. */
int odl_create(const char* area, int device, odl_ls** out);
/* Same over several devices of the node (device ids, may repeat): the graph
 * is replicated, all-sources sweeps run one root partition part per device. */
int odl_create_multi(const char* area, const int* devices, uint32_t n, odl_ls** out);
void odl_destroy(odl_ls* ls);
const char* odl_last_error(const odl_ls* ls);
void odl_free(char* p);

/* Apply stream records [first, first+count) in order; changes[count] out. */
int odl_apply(odl_ls* ls, const oadj_stream* s, uint32_t first, uint32_t count,
              oadj_change* changes);
/* Same with updateAdjacencyDatabase's hold TTLs (LinkState.cpp:585-700,
 * HoldableValue LinkState.cpp:48-117): a new link stays down for hold_up_ttl
 * odl_decrement_holds calls; a metric / overload change is held back
 * hold_up_ttl calls when it brings the link up (metric decrease, overload
 * cleared), hold_down_ttl otherwise. Decision itself passes 0
 * (Decision.cpp:756), which is odl_apply. */
int odl_apply_hold(odl_ls* ls, const oadj_stream* s, uint32_t first, uint32_t count,
                   oadj_change* changes, uint64_t hold_up_ttl, uint64_t hold_down_ttl);
/* LinkState::decrementHolds (LinkState.cpp:520-535): 1 when a hold expired
 * (topology changed, memoised results dropped), 0 when none did, < 0 error.
 * odl_has_holds (:537-548): 1 while any hold is on. */
int odl_decrement_holds(odl_ls* ls);
int odl_has_holds(const odl_ls* ls);

char* odl_spf_text(odl_ls* ls, const char* root, int use_link_metric);
char* odl_kth_paths_text(odl_ls* ls, const char* src, const char* dst, int k);
char* odl_links_text(odl_ls* ls, const char* node);
/* Keys of the snapshot's links in link id order (the ids of odl_csr_export
 * and of the engine's KSP2 records), one per line. */
char* odl_link_keys_text(odl_ls* ls);
int64_t odl_metric_a_to_b(odl_ls* ls, const char* a, const char* b, int use_link_metric);
int odl_is_overloaded(odl_ls* ls, const char* node);
uint64_t odl_spf_runs(const odl_ls* ls);
/* The path's fb303 counters: decision.spf_runs COUNT
 * (LinkState.cpp:843); decision.spf_ms (:909), ucmp_ms (:1029) and
 * route_build_ms (SpfSolver.cpp:640-644) are AVG stats, kept here as a sum
 * and a sample count; ucmp_runs COUNT (:926). Plus the device errors the
 * LinkState survived (it then runs on its host path; degraded = 1). */
typedef struct odl_counters {
  uint64_t spf_runs;
  uint64_t spf_ms_samples;
  double spf_ms_sum;
  uint64_t ucmp_runs;
  double ucmp_ms_sum;
  uint64_t route_build_runs;
  double route_build_ms_sum;
  uint64_t engine_errors;
  uint32_t engine_degraded;
} odl_counters;
void odl_get_counters(const odl_ls* ls, odl_counters* out);
/* The last engine error the LinkState degraded on ("" when none). */
const char* odl_last_engine_error(const odl_ls* ls);
/* Test hook: the after-th engine call from now fails with OSPF_E_DEVICE
 * (ospf_inject_error); the LinkState must degrade to its host path. */
int odl_inject_engine_error(odl_ls* ls, uint32_t after);
/* Degrade to the host path on device errors (default 1; 0: the call fails
 * with the engine's error instead). A LinkState whose engine never opened
 * (no device) always fails: there is no silent CPU path. ODL_STRICT_ENGINE
 * in the environment sets 0 at creation. */
void odl_set_degrade(odl_ls* ls, int on);
/* Incremental mode (off by default; odl::LinkState::setIncremental): keep the
 * memoised SPF of roots a metric / up / overload-only update cannot affect.
 * Stats: {patches applied, results kept, results dropped}. */
/* KvStore publications (the step before LinkState in Decision): compact-
 * thrift values decoded on host threads (adjdb_thrift.cpp).
 *
 * odl_apply_kvs -- Decision::processPublication's LinkState part
 * (Decision.cpp:846-870): keys[i] / values[i] (value_lens[i] bytes,
 * values[i] == NULL: a TTL-only update) in the caller's keyVals iteration
 * order; an "adj:" key's value (a CompactSerializer thrift::AdjacencyDatabase,
 * Types.thrift:175-207) goes to updateAdjacencyDatabase (updateKeyInLsdb
 * :743-765), other keys are skipped; then each expired "adj:" key deletes
 * the node getNodeNameFromKey names (deleteKeyFromLsdb :812-826). my_node !=
 * NULL applies filterUnuseableAdjacency (:568-600). changes: n + n_expired
 * records (zero for skipped keys) or NULL. */
int odl_apply_kvs(odl_ls* ls, uint32_t n, const char* const* keys, const uint8_t* const* values,
                  const uint64_t* value_lens, uint32_t n_expired, const char* const* expired,
                  const char* my_node, oadj_change* changes);
/* Same from a whole compact-thrift thrift::Publication (KvStore.thrift:270-
 * 320) in `buf`: keyVals in wire order, then expiredKeys. n_changes_out (may
 * be NULL) = number of records. When `changes` is not NULL and the records
 * do not fit max_changes, nothing is applied and ODL_E_SMALL is returned with
 * *n_changes_out set (call again with room for them). A publication whose
 * area field is set and differs from this LinkState's area is rejected
 * (Decision::processPublication picks the LinkState by the area,
 * Decision.cpp:847-854; the caller routes it). */
#define ODL_E_SMALL (-2)
int odl_apply_publication(odl_ls* ls, const uint8_t* buf, uint64_t len, const char* my_node,
                          oadj_change* changes, uint32_t max_changes, uint32_t* n_changes_out);
/* The last value odl_apply_kvs / odl_apply_publication could not decode
 * ("" when none; owned by ls) and the number of such values so far. */
const char* odl_last_decode_error(const odl_ls* ls, uint64_t* n_errors);
/* Decode n compact-thrift AdjacencyDatabase values into a columnar stream
 * (include/openr_adjdb.h; adj_only_used_by_other filled, db_delete all 0),
 * owned by *out until odl_adjdbs_free. NULL on malformed input, with the
 * reason in odl_adjdbs_error. */
typedef struct odl_adjdbs odl_adjdbs;
odl_adjdbs* odl_adjdbs_decode(const uint8_t* const* values, const uint64_t* lens, uint32_t n);
const oadj_stream* odl_adjdbs_stream(const odl_adjdbs* d);
const char* odl_adjdbs_error(void);
void odl_adjdbs_free(odl_adjdbs* d);
void odl_set_incremental(odl_ls* ls, int on);
/* Every SPF / KSP2 / digest of this LinkState on the host with the
 * reference's algorithm (LinkState.cpp:836-911), the engine never opened: a
 * GPU-free run of the ingest / in-place patch / memo logic (sanitizer builds;
 * also the environment variable ODL_HOST_SPF at creation). Not a fallback:
 * off by default, and nothing switches it on by itself. */
void odl_set_host_spf(odl_ls* ls, int on);
void odl_incremental_stats(const odl_ls* ls, uint64_t* out3);
/* {whole CSR snapshots, whole device graph loads, updates whose added /
 * removed links were patched in place (ospf_update_rows), rows rebuilt by
 * them}: a [LINK UP] / [LINK DOWN] between known nodes (LinkState.cpp:632-657)
 * takes no snapshot and no load. */
void odl_topology_stats(const odl_ls* ls, uint64_t* out4);
/* nodes added or removed in place (their rows inserted / erased and the ids
 * above them renumbered, no whole snapshot; the device graph reloads) */
uint64_t odl_node_patches(const odl_ls* ls);
/* multi-device LinkState (odl_create_multi): out4 = {root batches split
 * across the device slots, their per-slot launches, KSP2 prefetches split
 * across the slots (destinations of one source), their per-slot runs} */
void odl_shard_stats(const odl_ls* ls, uint64_t* out4);
uint32_t odl_num_nodes(const odl_ls* ls);
uint32_t odl_num_links(const odl_ls* ls);

/* Batched runs. roots / dsts are '\n'-separated node names.
 * odl_spf_digests: one engine batch, out[3*i] = {reached, sum_dist, hash}. */
int odl_spf_digests(odl_ls* ls, const char* roots_nl, uint32_t n, int use_link_metric,
                    uint64_t* out);
/* All-sources: runSpf for every node in one engine sweep (ospf_sweep_*, one
 * partition part per device), rows resident on the devices; getSpfResult of
 * any node then copies its rows (Decision::getDecisionRouteDb for every
 * node, Decision.cpp:309). odl_all_sources_digests: out[3 * id] for every
 * node id (odl_node_name order). A prefetch / route build asking for at
 * least 256 roots and half of the nodes takes the sweep by itself.
 * odl_sweep_stats: {sweeps, rows copied, mode (OSPF_SWEEP_*), devices,
 * hip graph}. */
int odl_all_sources_prefetch(odl_ls* ls, int use_link_metric);
int odl_all_sources_digests(odl_ls* ls, int use_link_metric, uint64_t* out);
void odl_sweep_stats(const odl_ls* ls, uint64_t* out5);
/* Fill the getSpfResult memo for many roots with one engine batch. */
int odl_spf_prefetch(odl_ls* ls, const char* roots_nl, uint32_t n, int use_link_metric);
/* getKthPaths(src, d, 2) for every d, masked reruns batched on the engine;
 * text = paths of each d, then a line "=". */
char* odl_ksp2_text(odl_ls* ls, const char* src, const char* dsts_nl, uint32_t n);

/* Route building over the GPU SPF results (SpfSolver consumers, SURVEY.md §8
 * a8-a10) for a prefix announced by `announcers` ('\n'-separated):
 *   algo 0 = SP_ECMP unicast (getNextHopsWithMetric + getNextHopsThrift,
 *            SpfSolver.cpp:1043-1285), 1 = KSP2_ED_ECMP (selectBestPathsKsp2,
 *            SpfSolver.cpp:847-973), 2 = MPLS node-label route of the single
 *            announcer (PHP / SWAP, SpfSolver.cpp:501-598).
 * Text: one next-hop per line, sorted: ifName \t neighbor \t metric \t
 * mpls-op (0 none, 1 PHP, 2 SWAP, 3 PUSH) \t labels (',' separated). */
char* odl_route_text(odl_ls* ls, const char* me, const char* announcers_nl, uint32_t n,
                     int algo);

/* LinkState::pathAInPathB (LinkState.h:477-492): 1 if path a (n links, keys
 * "n1%if1|n2%if2" one per line) occurs contiguously in path b, else 0; -1 on
 * a malformed key. */
int odl_path_a_in_b(const char* a_nl, uint32_t na, const char* b_nl, uint32_t nb);

/* SpfSolver::buildRouteDb (SpfSolver.cpp:460-646), one area, for each of the
 * n_mes nodes in mes_nl (their SPF results come from one batched engine
 * launch). prefixes_nl = n lines "prefix \t entry,entry,..." with
 * entry = "node:fwd:algo:weight[:prepend]" (a thrift::PrefixEntry: fwd 0 IP /
 * 1 SR_MPLS; algo 0 SP_ECMP, 1 KSP2_ED_ECMP, 2 SP_UCMP_ADJ_WEIGHT_PROPAGATION,
 * 3 SP_UCMP_PREFIX_WEIGHT_PROPAGATION; weight 0 = unset; optional prepend
 * label; then optionally "%pp/sp/d" = PrefixMetrics path_preference /
 * source_preference / distance, and "!bgp" or "!bgpmv" = PrefixType::BGP
 * without / with a metric vector). flags: 1 node-segment labels, 2 adjacency
 * labels, 4 UCMP, 8 enableBestRouteSelection (the SpfSolver constructor
 * switches, SpfSolver.h:108-118). Text, one line each, next hops sorted:
 *   me \t NONE                       (`me` unknown: the reference's nullopt)
 *   me \t R \t prefix \t igpCost(u32) \t ucmpWeight | -
 *        [flag 8: \t best node@area \t selected node@area,...]
 *   me \t U \t prefix \t ifName \t neighbor \t metric(i32) \t op \t labels \t weight
 *   me \t M \t label  \t ifName \t neighbor \t metric(i32) \t op \t labels \t weight
 * op: 0 none, 1 PHP, 2 SWAP, 3 PUSH, 4 POP_AND_LOOKUP; labels comma-separated
 * (SWAP: the swap label; PUSH: bottom of stack first). */
char* odl_route_db_text(odl_ls* ls, const char* mes_nl, uint32_t n_mes, const char* prefixes_nl,
                        uint32_t n, int flags);
/* Prefix entries may end in "@area" (the entry's area; default: the first
 * area by name) and then "#n" (PrefixEntry.minNexthop = n: addBestPaths
 * drops a route with fewer next hops, SpfSolver.cpp:976-1000,
 * getMinNextHopThreshold :694-710).
 * odl_route_db_multi_text: the same over several areas, one LinkState each
 * (their area names, odl_create's `area`, distinct): createRouteForPrefix's
 * per-area loop (SpfSolver.cpp:229-250, 360-442: entries reachable in their
 * own area; per area the forwarding type / algorithm of its best entries;
 * the next hops of the areas at the shortest IGP metric, UCMP weights
 * summed, KSP2 next hops added), node labels of every area's databases
 * (:490-598) and adjacency labels of every area (:603-631). Next-hop lines
 * carry a last field: the next hop's area. Errors: odl_last_error(areas[0]). */
char* odl_route_db_multi_text(odl_ls* const* areas, uint32_t n_areas, const char* mes_nl,
                              uint32_t n_mes, const char* prefixes_nl, uint32_t n, int flags);

/* odl_route_db_text's databases as one binary buffer (no text formatting or
 * parsing on either side; every string stored once). *out is malloc'd (free
 * with odl_free_buf), *bytes its size. Layout (little-endian, sections 8-B
 * aligned, offsets from the buffer start; string fields are offsets into the
 * NUL-terminated string section):
 *   odl_rdb_header; odl_rdb_node[n_nodes] (one per requested node, in order);
 *   odl_rdb_route[n_routes] (per node: unicast by prefix, then MPLS by label);
 *   odl_rdb_nh[n_nhs] (per route, sorted as in the text); int32 labels[];
 *   strings.
 * Replaces the text hop of Decision's route publication
 * (Decision::getDecisionRouteDb -> DecisionRouteDb, SpfSolver.h:80-98). */
#define ODL_RDB_MAGIC 0x4244524Fu /* "ORDB" */
typedef struct {
  uint32_t magic, version;
  uint64_t bytes;
  uint32_t n_nodes, n_routes, n_nhs, n_labels;
  uint64_t off_nodes, off_routes, off_nhs, off_labels, off_strings, str_bytes;
} odl_rdb_header;
typedef struct {
  uint32_t name;    /* string */
  uint32_t found;   /* 0: unknown node (the reference's nullopt) */
  uint32_t first_route, n_unicast, n_mpls, pad;
} odl_rdb_node;
typedef struct {
  uint32_t kind;        /* 0 unicast, 1 MPLS */
  uint32_t key;         /* unicast: prefix string; MPLS: the label */
  uint32_t igp_cost;    /* unicast */
  uint32_t has_weight;  /* unicast: ucmp_weight set */
  int64_t ucmp_weight;
  uint32_t first_nh, n_nh;
} odl_rdb_route;
typedef struct {
  uint32_t if_name, neighbor; /* strings */
  int32_t metric, weight;
  uint32_t op;                /* 0 none, 1 PHP, 2 SWAP, 3 PUSH, 4 POP_AND_LOOKUP */
  uint32_t first_label, n_labels, pad;
} odl_rdb_nh;
int odl_route_db_bin(odl_ls* ls, const char* mes_nl, uint32_t n_mes, const char* prefixes_nl,
                     uint32_t n, int flags, void** out, uint64_t* bytes);
void odl_free_buf(void* p);

/* LinkState::resolveUcmpWeights (LinkState.cpp:913-1033) over
 * getSpfResult(root): leaves_nl = n lines "name\tweight"; algo 2 =
 * SP_UCMP_ADJ_WEIGHT_PROPAGATION, 3 = SP_UCMP_PREFIX_WEIGHT_PROPAGATION.
 * Text: one line per node of the result, sorted by name:
 *   node \t advertised weight \t iface=nextHopNode:weight,... (sorted by iface) */
char* odl_ucmp_text(odl_ls* ls, const char* root, const char* leaves_nl, uint32_t n, int algo,
                    int use_link_metric);

/* CSR snapshot the engine sees (node ids = rank of name, byte order).
 * Copies into caller arrays sized by odl_csr_size(); any pointer may be NULL. */
int odl_csr_size(odl_ls* ls, uint32_t* n_nodes, uint32_t* n_edges);
int odl_csr_export(odl_ls* ls, uint32_t* row_ptr, uint32_t* col, uint32_t* metric,
                   uint32_t* link_id, uint32_t* twin, uint8_t* edge_up, uint8_t* no_transit,
                   uint32_t* link_rank);
/* Node name of id (pointer valid until the next apply). */
const char* odl_node_name(odl_ls* ls, uint32_t id);
int64_t odl_node_id(odl_ls* ls, const char* name);

#ifdef __cplusplus
}
#endif

#endif /* OPENR_DECISION_H */
