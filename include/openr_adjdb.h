/*
 * openr_adjdb.h — columnar stream of AdjacencyDatabase updates.
 *
 * This is the *input data format* shared by the host LinkState mirror
 * (libopenr_decision) and the CPU oracle. It carries exactly the thrift
 * fields LinkState reads:
 *   thrift::AdjacencyDatabase  openr/if/Types.thrift:175-207
 *     thisNodeName, isOverloaded, adjacencies, nodeLabel
 *   thrift::Adjacency          openr/if/Types.thrift:98-168
 *     otherNodeName, ifName, otherIfName, metric (i32), adjLabel (i32),
 *     isOverloaded, weight (i64), adjOnlyUsedByOtherNode
 * One record = one LinkState::updateAdjacencyDatabase(db, area, 0, 0) call
 * (openr/decision/LinkState.cpp:584), or, with db_delete[i] = 1, one
 * LinkState::deleteAdjacencyDatabase(name) call (LinkState.cpp:730).
 *
 * Strings are interned in one table (str_data + str_off); every *_name / *_if
 * field is an index into it. All arrays are caller-owned and only read during
 * the call that receives the stream.
 */
#ifndef OPENR_ADJDB_H
#define OPENR_ADJDB_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oadj_stream {
  /* interned string table */
  const char* str_data;
  const uint64_t* str_off; /* n_str + 1 offsets into str_data */
  uint32_t n_str;

  /* one entry per adjacency-database record */
  uint32_t n_dbs;
  const uint32_t* db_name;        /* thisNodeName (string index) */
  const uint8_t* db_overloaded;   /* isOverloaded */
  const int32_t* db_node_label;   /* nodeLabel */
  const uint8_t* db_delete;       /* 1: delete this node's database; may be NULL */
  const uint64_t* db_adj_off;     /* n_dbs + 1 offsets into the adj_* columns */

  /* one entry per adjacency */
  const uint32_t* adj_other;      /* otherNodeName */
  const uint32_t* adj_if;         /* ifName */
  const uint32_t* adj_other_if;   /* otherIfName */
  const int32_t* adj_metric;      /* metric */
  const int32_t* adj_label;       /* adjLabel */
  const uint8_t* adj_overloaded;  /* isOverloaded */
  const int64_t* adj_weight;      /* weight */
  const uint8_t* adj_only_used_by_other; /* adjOnlyUsedByOtherNode; may be NULL */
} oadj_stream;

/* LinkState::LinkStateChange (openr/decision/LinkState.h:433-452), flattened. */
typedef struct oadj_change {
  int32_t topology_changed;
  int32_t link_attributes_changed;
  int32_t node_label_changed;
  int32_t n_added_links;
  /* odl_apply_kvs / odl_apply_publication: 1 when this key's value failed to
   * decode; the key was skipped and the rest applied (Decision::
   * updateKeyInLsdb catches and logs it, Decision.cpp:742-806) */
  int32_t decode_error;
} oadj_change;

#ifdef __cplusplus
}
#endif

#endif /* OPENR_ADJDB_H */
