// adjdb_thrift.h — compact-thrift KvStore publications -> adjacency
// databases (adjdb_thrift.cpp; Decision.cpp:743-765, 812-870).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "../../../include/openr_adjdb.h"

namespace odl {

struct AdjacencyDatabase;

namespace thrift_compact {
// thrift::AdjacencyDatabase (Types.thrift:175-207) from CompactSerializer
// bytes; throws std::runtime_error on malformed input
void decodeAdjacencyDatabase(const uint8_t* p, size_t n, AdjacencyDatabase& db);
}  // namespace thrift_compact

// thrift::Publication (KvStore.thrift:270-320) parsed without copies: views
// into the caller's buffer, keyVals in wire order
struct PublicationView {
  struct KeyVal {
    std::string_view key, value;
    bool hasValue = false;  // Value.value set (else a TTL-only update)
  };
  std::string_view area;
  std::vector<KeyVal> keyVals;
  std::vector<std::string_view> expiredKeys;
};
namespace thrift_compact {
void parsePublication(const uint8_t* p, size_t n, PublicationView& out);
}

// getNodeNameFromKey (openr/common/LsdbUtil.cpp:748-755)
std::string nodeNameFromKey(std::string_view key);

// Decoded databases as the columnar stream of include/openr_adjdb.h (owns
// the columns; strings not interned: one table entry per field)
struct AdjDbColumns {
  void decode(const uint8_t* const* values, const uint64_t* lens, uint32_t n);
  oadj_stream stream{};
  std::string str;
  std::vector<uint64_t> stroff, adjoff;
  std::vector<uint32_t> name, other, ifn, oifn;
  std::vector<uint8_t> overloaded, del, adjOverloaded, onlyOther;
  std::vector<int32_t> label, metric, adjLabel;
  std::vector<int64_t> weight;
};

}  // namespace odl
