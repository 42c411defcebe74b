// adjdb_thrift.cpp — the step before LinkState in Decision: KvStore
// publications of "adj:" keys, compact-protocol thrift, decoded on host
// threads into AdjacencyDatabases (odl::LinkState ingest) or into the
// columnar oadj_stream (include/openr_adjdb.h).
//
// Reference: Decision::processPublication (openr/decision/Decision.cpp:846-870)
// walks the publication's keyVals, then its expiredKeys; updateKeyInLsdb
// (:743-765) skips TTL-only values (no `value`), deserializes the value of
// an "adj:" key with apache::thrift::CompactSerializer
// (readThriftObjStr<thrift::AdjacencyDatabase>), drops the adjacencies with
// adjOnlyUsedByOtherNode set whose otherNodeName is not this node
// (filterUnuseableAdjacency :568-600, when ordered adjacency publication is
// enabled) and calls LinkState::updateAdjacencyDatabase; deleteKeyFromLsdb
// (:812-826) calls deleteAdjacencyDatabase(getNodeNameFromKey(key))
// (openr/common/LsdbUtil.cpp:748-755: the second ':'-separated field).
// Field ids: thrift::Adjacency / AdjacencyDatabase openr/if/Types.thrift:98-207,
// thrift::Value openr/if/KvStore.thrift:177-225, thrift::Publication :270-320.
//
// Compact protocol (Apache Thrift TCompactProtocol, as fbthrift's
// CompactSerializer writes it): a struct is a sequence of field headers --
// one byte, field-id delta (1..15) in the high nibble and the type in the low
// one, or delta 0 then the id as a zigzag varint i16 -- ended by a 0 byte;
// bools live in the header's type (1 true, 2 false; one byte of the same
// values inside lists); i16 / i32 / i64 are zigzag varints; binary / string
// = varint length + bytes; list / set = one byte (size < 15 in the high
// nibble, else 0xF and a varint size; element type low) + elements; map =
// varint size, then (if non-empty) one byte of key type << 4 | value type;
// double 8 bytes, float 4. Unknown fields are skipped by type.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "link_state.h"
#include "adjdb_thrift.h"

namespace odl {
namespace thrift_compact {
namespace {

enum : uint8_t {
  kStop = 0,
  kTrue = 1,
  kFalse = 2,
  kByte = 3,
  kI16 = 4,
  kI32 = 5,
  kI64 = 6,
  kDouble = 7,
  kBinary = 8,
  kList = 9,
  kSet = 10,
  kMap = 11,
  kStruct = 12,
  kFloat = 13,
};

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  int depth = 0;
  [[noreturn]] void bad(const char* what) const {
    throw std::runtime_error(std::string("compact thrift: ") + what);
  }
  // one level of struct / list / set / map nesting while skipping: bounded,
  // so a value of nested containers cannot run the decoding thread's stack out
  static constexpr int kMaxDepth = 64;
  struct Nest {
    Reader& r;
    explicit Nest(Reader& x) : r(x) {
      if (++r.depth > kMaxDepth) r.bad("nesting too deep");
    }
    ~Nest() { --r.depth; }
  };
  uint8_t byte() {
    if (p >= end) bad("truncated");
    return *p++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      const uint8_t b = byte();
      v |= (uint64_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) return v;
    }
    bad("varint too long");
  }
  int64_t zigzag() {
    const uint64_t v = varint();
    return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
  }
  std::string_view binary() {
    const uint64_t n = varint();
    if (n > (uint64_t)(end - p)) bad("string past the end");
    std::string_view s((const char*)p, (size_t)n);
    p += n;
    return s;
  }
  // field header: false at the stop byte; id relative to `last`
  bool field(int16_t& last, int16_t& id, uint8_t& type) {
    const uint8_t h = byte();
    if (h == kStop) return false;
    type = h & 0x0F;
    const uint8_t d = h >> 4;
    id = d ? (int16_t)(last + d) : (int16_t)zigzag();
    last = id;
    return true;
  }
  void list_header(uint8_t& et, uint64_t& n) {
    const uint8_t h = byte();
    et = h & 0x0F;
    n = h >> 4;
    if (n == 15) n = varint();
    if (n > (uint64_t)(end - p)) bad("list size past the end");  // >= 1 byte per element
  }
  bool boolean_field(uint8_t type) {
    if (type == kTrue) return true;
    if (type == kFalse) return false;
    bad("bool field of another type");
  }
  int64_t integer(uint8_t type) {
    if (type == kByte) return (int8_t)byte();
    if (type == kI16 || type == kI32 || type == kI64) return zigzag();
    bad("integer field of another type");
  }
  void skip(uint8_t type) {
    switch (type) {
      case kTrue:
      case kFalse:
        return;  // in a field header; inside containers see skip_elem
      case kByte:
        byte();
        return;
      case kI16:
      case kI32:
      case kI64:
        varint();
        return;
      case kDouble:
        advance(8);
        return;
      case kFloat:
        advance(4);
        return;
      case kBinary:
        binary();
        return;
      case kList:
      case kSet: {
        Nest nest(*this);
        uint8_t et;
        uint64_t n;
        list_header(et, n);
        for (uint64_t i = 0; i < n; ++i) skip_elem(et);
        return;
      }
      case kMap: {
        Nest nest(*this);
        const uint64_t n = varint();
        if (!n) return;
        const uint8_t kv = byte();
        if (n > (uint64_t)(end - p)) bad("map size past the end");  // >= 1 byte per entry
        for (uint64_t i = 0; i < n; ++i) {
          skip_elem(kv >> 4);
          skip_elem(kv & 0x0F);
        }
        return;
      }
      case kStruct: {
        Nest nest(*this);
        int16_t last = 0, id;
        uint8_t t;
        while (field(last, id, t)) skip(t);
        return;
      }
      default:
        bad("unknown type");
    }
  }
  void skip_elem(uint8_t type) {
    if (type == kTrue || type == kFalse) {
      byte();
      return;
    }
    skip(type);
  }
  void advance(size_t n) {
    if (n > (size_t)(end - p)) bad("truncated");
    p += n;
  }
};

void read_adjacency(Reader& r, Adjacency& a) {
  // defaults of Types.thrift:98-168 (metric has none: 0)
  a = Adjacency{};
  a.metric = 0;
  a.weight = 1;
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    switch (id) {
      case 1: if (t == kBinary) { a.otherNodeName = r.binary(); continue; } break;
      case 2: if (t == kBinary) { a.ifName = r.binary(); continue; } break;
      case 4: if (t == kI32) { a.metric = (int32_t)r.integer(t); continue; } break;
      case 6: if (t == kI32) { a.adjLabel = (int32_t)r.integer(t); continue; } break;
      case 7: if (t == kTrue || t == kFalse) { a.isOverloaded = r.boolean_field(t); continue; } break;
      case 10: if (t == kI64) { a.weight = r.integer(t); continue; } break;
      case 11: if (t == kBinary) { a.otherIfName = r.binary(); continue; } break;
      case 12:
        if (t == kTrue || t == kFalse) {
          a.adjOnlyUsedByOtherNode = r.boolean_field(t);
          continue;
        }
        break;
      default: break;
    }
    r.skip(t);  // nextHopV6 / V4, rtt, timestamp, unknown or mistyped fields
  }
}

}  // namespace

void decodeAdjacencyDatabase(const uint8_t* p, size_t n, AdjacencyDatabase& db) {
  Reader r{p, p + n};
  db = AdjacencyDatabase{};
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    if (id == 1 && t == kBinary) {
      db.thisNodeName = r.binary();
    } else if (id == 2 && (t == kTrue || t == kFalse)) {
      db.isOverloaded = r.boolean_field(t);
    } else if (id == 3 && t == kList) {
      uint8_t et;
      uint64_t cnt;
      r.list_header(et, cnt);
      if (et != kStruct) r.bad("adjacencies: not a list of structs");
      db.adjacencies.resize(cnt);
      for (uint64_t i = 0; i < cnt; ++i) read_adjacency(r, db.adjacencies[i]);
    } else if (id == 4 && t == kI32) {
      db.nodeLabel = (int32_t)r.integer(t);
    } else {
      r.skip(t);  // perfEvents, area, unknown fields
    }
  }
}

void parsePublication(const uint8_t* p, size_t n, PublicationView& out) {
  Reader r{p, p + n};
  out = PublicationView{};
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    if (id == 2 && t == kMap) {  // keyVals: map<string, Value>
      const uint64_t cnt = r.varint();
      if (!cnt) continue;
      const uint8_t kv = r.byte();
      if ((kv >> 4) != kBinary || (kv & 0x0F) != kStruct) r.bad("keyVals: not map<string, Value>");
      if (cnt > (uint64_t)(r.end - r.p)) r.bad("keyVals size past the end");
      out.keyVals.reserve(cnt);
      for (uint64_t i = 0; i < cnt; ++i) {
        PublicationView::KeyVal x;
        x.key = r.binary();
        int16_t vl = 0, vid;
        uint8_t vt;
        while (r.field(vl, vid, vt)) {
          if (vid == 2 && vt == kBinary) {  // optional binary value
            x.value = r.binary();
            x.hasValue = true;
          } else {
            r.skip(vt);  // version, originatorId, ttl, ttlVersion, hash
          }
        }
        out.keyVals.push_back(x);
      }
    } else if (id == 3 && t == kList) {  // expiredKeys: list<string>
      uint8_t et;
      uint64_t cnt;
      r.list_header(et, cnt);
      if (et != kBinary) r.bad("expiredKeys: not a list of strings");
      out.expiredKeys.reserve(cnt);
      for (uint64_t i = 0; i < cnt; ++i) out.expiredKeys.push_back(r.binary());
    } else if (id == 7 && t == kBinary) {
      out.area = r.binary();
    } else {
      r.skip(t);  // nodeIds, tobeUpdatedKeys, floodRootId, unknown fields
    }
  }
}

}  // namespace thrift_compact

std::string nodeNameFromKey(std::string_view key) {
  // LsdbUtil.cpp:748-755: folly::split(":", key)[1], "" when there is none
  const size_t a = key.find(':');
  if (a == std::string_view::npos) return "";
  const size_t b = key.find(':', a + 1);
  return std::string(key.substr(a + 1, b == std::string_view::npos ? std::string_view::npos : b - a - 1));
}

std::vector<LinkStateChange> LinkState::applyKvs(const std::vector<KvIn>& kvs,
                                                 const std::vector<std::string_view>& expired,
                                                 const std::string* myNodeName) {
  // decode every "adj:" value on host threads, then apply in order
  // (updateKeyInLsdb per key, deleteKeyFromLsdb per expired key)
  constexpr std::string_view kAdj = "adj:";
  std::vector<uint32_t> which;  // kvs index of each database
  for (uint32_t i = 0; i < kvs.size(); ++i)
    if (kvs[i].hasValue && kvs[i].key.substr(0, kAdj.size()) == kAdj) which.push_back(i);
  std::vector<AdjacencyDatabase> dbs(which.size());
  // a value that fails to decode skips its own key only (updateKeyInLsdb
  // catches the deserialization error, logs it and returns, Decision.cpp:742-806)
  std::vector<std::string> errs(which.size());
  parallelFor((uint32_t)which.size(), [&](uint32_t lo, uint32_t hi) {
    for (uint32_t k = lo; k < hi; ++k) {
      const KvIn& kv = kvs[which[k]];
      try {
        thrift_compact::decodeAdjacencyDatabase((const uint8_t*)kv.value.data(), kv.value.size(),
                                                dbs[k]);
      } catch (const std::exception& e) {
        errs[k] = "key " + std::string(kv.key) + ": " + e.what();
        continue;
      }
      if (myNodeName) {  // filterUnuseableAdjacency (Decision.cpp:568-600)
        auto& adjs = dbs[k].adjacencies;
        adjs.erase(std::remove_if(adjs.begin(), adjs.end(),
                                  [&](const Adjacency& a) {
                                    return a.adjOnlyUsedByOtherNode && a.otherNodeName != *myNodeName;
                                  }),
                   adjs.end());
      }
    }
  }, 64);
  std::vector<LinkStateChange> out(kvs.size() + expired.size());
  std::vector<AdjacencyDatabase> good;
  std::vector<uint32_t> goodAt;
  good.reserve(dbs.size());
  for (size_t k = 0; k < which.size(); ++k) {
    if (!errs[k].empty()) {
      out[which[k]].decodeError = true;
      lastDecodeError_ = errs[k];
      ++decodeErrors_;
      continue;
    }
    good.push_back(std::move(dbs[k]));
    goodAt.push_back(which[k]);
  }
  const auto chs = updateAdjacencyDatabases(good);
  for (size_t k = 0; k < goodAt.size(); ++k) out[goodAt[k]] = chs[k];
  for (size_t j = 0; j < expired.size(); ++j)
    if (expired[j].substr(0, kAdj.size()) == kAdj)
      out[kvs.size() + j] = deleteAdjacencyDatabase(nodeNameFromKey(expired[j]));
  return out;
}

// ---- columnar decode (oadj_stream)
void AdjDbColumns::decode(const uint8_t* const* values, const uint64_t* lens, uint32_t n) {
  std::vector<AdjacencyDatabase> dbs(n);
  parallelFor(n, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t k = lo; k < hi; ++k)
      thrift_compact::decodeAdjacencyDatabase(values[k], (size_t)lens[k], dbs[k]);
  }, 64);
  // per database: its strings (name, then other / if / otherIf per
  // adjacency) and bytes, prefix-summed so threads write disjoint ranges
  std::vector<uint64_t> soff(n + 1, 0), boff(n + 1, 0), aoff(n + 1, 0);
  for (uint32_t k = 0; k < n; ++k) {
    const auto& d = dbs[k];
    uint64_t b = d.thisNodeName.size();
    for (const auto& a : d.adjacencies) b += a.otherNodeName.size() + a.ifName.size() + a.otherIfName.size();
    soff[k + 1] = soff[k] + 1 + 3 * d.adjacencies.size();
    boff[k + 1] = boff[k] + b;
    aoff[k + 1] = aoff[k] + d.adjacencies.size();
  }
  const uint64_t ns = soff[n], na = aoff[n];
  if (ns >= 0xFFFFFFFFull) throw std::length_error("adjacency databases: more than 2^32 strings");
  str.resize(boff[n]);
  stroff.assign(ns + 1, 0);
  name.resize(n);
  overloaded.resize(n);
  label.resize(n);
  del.assign(n, 0);
  adjoff.assign(aoff.begin(), aoff.end());
  other.resize(na);
  ifn.resize(na);
  oifn.resize(na);
  metric.resize(na);
  adjLabel.resize(na);
  adjOverloaded.resize(na);
  weight.resize(na);
  onlyOther.resize(na);
  parallelFor(n, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t k = lo; k < hi; ++k) {
      const auto& d = dbs[k];
      uint64_t si = soff[k], bi = boff[k], ai = aoff[k];
      auto put = [&](const std::string& x) {
        std::memcpy(&str[bi], x.data(), x.size());
        bi += x.size();
        stroff[si + 1] = bi;
        return (uint32_t)si++;
      };
      name[k] = put(d.thisNodeName);
      overloaded[k] = d.isOverloaded;
      label[k] = d.nodeLabel;
      for (const auto& a : d.adjacencies) {
        other[ai] = put(a.otherNodeName);
        ifn[ai] = put(a.ifName);
        oifn[ai] = put(a.otherIfName);
        metric[ai] = a.metric;
        adjLabel[ai] = a.adjLabel;
        adjOverloaded[ai] = a.isOverloaded;
        weight[ai] = a.weight;
        onlyOther[ai] = a.adjOnlyUsedByOtherNode;
        ++ai;
      }
    }
  }, 256);
  stream = oadj_stream{};
  stream.str_data = str.data();
  stream.str_off = stroff.data();
  stream.n_str = (uint32_t)ns;
  stream.n_dbs = n;
  stream.db_name = name.data();
  stream.db_overloaded = overloaded.data();
  stream.db_node_label = label.data();
  stream.db_delete = del.data();
  stream.db_adj_off = adjoff.data();
  stream.adj_other = other.data();
  stream.adj_if = ifn.data();
  stream.adj_other_if = oifn.data();
  stream.adj_metric = metric.data();
  stream.adj_label = adjLabel.data();
  stream.adj_overloaded = adjOverloaded.data();
  stream.adj_weight = weight.data();
  stream.adj_only_used_by_other = onlyOther.data();
}

}  // namespace odl
