"""f4: KvStore publications of "adj:" keys, compact
thrift, decoded by libopenr_decision (adjdb_thrift.cpp) and applied the way
Decision::processPublication does (openr/decision/Decision.cpp:846-870:
keyVals in order -> updateKeyInLsdb :743-765, then expiredKeys ->
deleteKeyFromLsdb :812-826; filterUnuseableAdjacency :568-600). The bytes
come from tests/thrift_compact.py (an independent encoder written from the
Apache Thrift compact protocol) and from hand-worked known-answer vectors;
the resulting LinkState is checked against the same databases applied as a
columnar stream and against the oracle. GPU-free (odl_set_host_spf)."""
import numpy as np
import pytest

import thrift_compact as TC
from graphs import random_stream
from oracle import Oracle
from openr_amd.adjdb import AdjDb, AdjDbStream, create_adjacency, decode_adjdbs
from openr_amd.linkstate import LinkState, LinkStateError

# AdjacencyDatabase{1: "a", 2: false, 3: [Adjacency{1: "b", 2: "i", 4: 5,
# 11: "j"}], 4: 1} worked out by hand (short field headers: delta << 4 | type)
KAT_SHORT = bytes([0x18, 0x01, ord("a"),          # 1: string "a"
                   0x12,                          # 2: bool false
                   0x19, 0x1C,                    # 3: list, 1 x struct
                   0x18, 0x01, ord("b"),          #   1: "b"
                   0x18, 0x01, ord("i"),          #   2: "i"
                   0x25, 0x0A,                    #   4: i32 zigzag(5) = 10
                   0x78, 0x01, ord("j"),          #   11 (delta 7): "j"
                   0x00,                          #   stop
                   0x15, 0x02,                    # 4: i32 zigzag(1) = 2
                   0x00])                         # stop
def _kat_long():
    """Worked by hand: the adjacency's fields out of order (4 before 1: the
    long header form -- type byte, then the id as a zigzag varint), a
    negative metric (zigzag(-3) = 5), a skipped nested struct (3:
    nextHopV6), 0x41 (delta 4, type 1) = field 7 isOverloaded true, 0x36 0x0E
    = field 10 i64 zigzag(7) = 14, field 11 "z", 0x11 = field 12 true; then
    4: nodeLabel zigzag(-1) = 1."""
    return bytes([0x18, 0x01, ord("x"),
                  0x11,
                  0x19, 0x1C,
                  0x45, 0x05,
                  0x08, 0x02, 0x01, ord("y"),
                  0x18, 0x02, ord("p"), ord("q"),
                  0x1C, 0x18, 0x02, 0xFE, 0x80, 0x00,
                  0x41,
                  0x36, 0x0E,
                  0x18, 0x01, ord("z"),
                  0x11,
                  0x00,
                  0x15, 0x01,
                  0x00])


def host_ls():
    p = LinkState()
    p.set_host_spf(True)
    return p


def test_known_answer_vectors():
    s = decode_adjdbs([KAT_SHORT, _kat_long()]).to_dbs()
    a, b = s
    assert a.name == "a" and not a.overloaded and a.node_label == 1
    assert len(a.adjs) == 1
    x = a.adjs[0]
    assert (x.other, x.if_name, x.other_if, x.metric, x.label, x.overloaded, x.weight,
            x.only_used_by_other) == ("b", "i", "j", 5, 0, False, 1, False)  # IDL defaults
    assert b.name == "x" and b.overloaded and b.node_label == -1
    y = b.adjs[0]
    assert (y.other, y.if_name, y.other_if, y.metric, y.overloaded, y.weight,
            y.only_used_by_other) == ("y", "pq", "z", -3, True, 7, True)


def test_encoder_matches_known_answer():
    db = AdjDb("a", [create_adjacency("b", "i", "j", 5)], 1)
    w = TC.Writer()
    w.begin()
    w.string(1, "a")
    w.boolean(2, False)
    w.list_header(3, TC.T_STRUCT, 1)
    w.begin()
    w.string(1, "b")
    w.string(2, "i")
    w.i32(4, 5)
    w.string(11, "j")
    w.end()
    w.i32(4, 1)
    w.end()
    assert bytes(w.buf) == KAT_SHORT
    assert decode_adjdbs([TC.adjacency_database(db)]).to_dbs()[0].adjs[0].metric == 5


@pytest.mark.parametrize("seed", range(4))
def test_round_trip_random_databases(seed):
    st, _ = random_stream(seed, n=60, p=0.12)
    dbs = st.to_dbs()
    rng = np.random.default_rng(seed)
    for d in dbs:  # exercise every field
        for a in d.adjs:
            a.label = int(rng.integers(-5, 100000))
            a.weight = int(rng.integers(1, 1 << 40))
            a.only_used_by_other = bool(rng.random() < 0.2)
            a.metric = int(rng.integers(-(1 << 31), 1 << 31))
        d.node_label = int(rng.integers(-(1 << 31), 1 << 31))
    vals = [TC.adjacency_database(d, perf=bool(i % 2), extra=bool(i % 3)) for i, d in enumerate(dbs)]
    assert decode_adjdbs(vals).to_dbs() == dbs
    # long lists (>= 15 elements: the varint list size)
    big = AdjDb("hub", [create_adjacency(f"n{i}", f"i{i}", f"o{i}", i + 1) for i in range(300)], 9)
    assert decode_adjdbs([TC.adjacency_database(big)]).to_dbs()[0] == big


def test_malformed_values_raise():
    v = TC.adjacency_database(AdjDb("a", [create_adjacency("b", "i", "j", 5)], 1))
    for cut in (1, 3, 7, len(v) // 2, len(v) - 1):
        with pytest.raises(ValueError):
            decode_adjdbs([v[:cut]])
    with pytest.raises(ValueError):  # a string length past the end
        decode_adjdbs([bytes([0x18, 0x7F, ord("a"), 0x00])])
    with pytest.raises(ValueError):  # adjacencies not a list of structs
        decode_adjdbs([bytes([0x39, 0x15, 0x02, 0x00])])  # (field 3: delta 3)


def _kv_of(dbs):
    return [(f"adj:{d.name}", TC.adjacency_database(d)) for d in dbs]


@pytest.mark.parametrize("seed", range(3))
def test_apply_kvs_equals_stream_and_oracle(seed):
    """updateKeyInLsdb per key in iteration order: the same LinkState (link
    keys, every root's SpfResult text, change records) as the columnar stream
    of the same databases, and as the oracle."""
    st, names = random_stream(40 + seed, n=50, p=0.12)
    dbs = st.to_dbs()
    a, b, o = host_ls(), host_ls(), Oracle()
    got = a.apply_kvs(_kv_of(dbs))
    want = b.apply(st)
    assert got == want == o.apply(st)
    assert a.link_keys() == b.link_keys()
    for r in names:
        assert a.spf_text(r) == o.spf_text(r)
    # an update of one node, a TTL-only value, a prefix key (skipped), then
    # an expired adj: key (the node's database deleted)
    d0 = dbs[3]
    d0.adjs = d0.adjs[1:]
    kv = [(f"adj:{d0.name}", TC.adjacency_database(d0)), (f"adj:{dbs[5].name}", None),
          ("prefix:x:0:[10.0.0.0/8]", b"\x00")]
    ch = a.apply_kvs(kv, expired=[f"adj:{dbs[7].name}", "prefix:y:0:[::/0]"])
    upd = AdjDbStream.from_dbs([d0, AdjDb(dbs[7].name, delete=True)])
    och = o.apply(upd)
    assert ch[0] == och[0] and ch[3] == och[1]
    assert ch[1] == ch[2] == ch[4] == (False, False, False, 0)
    for r in names:
        assert a.spf_text(r) == o.spf_text(r), r


def test_publication_bytes_and_filter():
    """A whole thrift::Publication (keyVals in wire order, expiredKeys, nodeIds,
    area), and filterUnuseableAdjacency: adjacencies with
    adjOnlyUsedByOtherNode set are dropped unless they point at my_node."""
    st, names = random_stream(77, n=40, p=0.15)
    dbs = st.to_dbs()
    for d in dbs[:10]:
        for a in d.adjs[:2]:
            a.only_used_by_other = True
    me = names[0]
    kv = [(k, TC.value(v, originator=k[4:])) for k, v in _kv_of(dbs)]
    kv.append((f"adj:{names[1]}", TC.value(None)))  # TTL refresh
    pub = TC.publication(kv, expired=[f"adj:{names[2]}:ignored-suffix"], area="0")
    p = host_ls()
    ch = p.apply_publication(pub, my_node=me)
    assert len(ch) == len(kv) + 1
    # the oracle gets the filtered databases, then the delete
    # (getNodeNameFromKey: the second ':' field)
    filt = []
    for d in dbs:
        d2 = AdjDb(d.name, [a for a in d.adjs if not (a.only_used_by_other and a.other != me)],
                   d.node_label, d.overloaded)
        filt.append(d2)
    o = Oracle()
    och = o.apply(AdjDbStream.from_dbs(filt + [AdjDb(names[2], delete=True)]))
    assert ch[: len(dbs)] == och[: len(dbs)] and ch[-1] == och[-1]
    for r in names:
        assert p.spf_text(r) == o.spf_text(r), r
    with pytest.raises(LinkStateError):
        p.apply_publication(pub[: len(pub) // 3])


def test_large_publication_decodes_on_threads():
    """A 5k-node fabric's publication: every database decoded (host threads)
    and ingested in one call equals the stream ingest."""
    from openr_amd import topology as T
    st = T.fabric(pods=40, planes=4)
    dbs = st.to_dbs()
    pub = TC.publication([(f"adj:{d.name}", TC.value(TC.adjacency_database(d, extra=False)))
                          for d in dbs])
    a, b = host_ls(), host_ls()
    a.apply_publication(pub)
    b.apply(st)
    assert a.link_keys() == b.link_keys()
    assert a.num_nodes() == b.num_nodes() == len(dbs)
    assert a.spf_text("2-0-0") == b.spf_text("2-0-0")


def test_corrupt_value_skips_only_its_key():
    """updateKeyInLsdb catches a value that fails to deserialize, logs it and
    skips that key (Decision.cpp:742-806): the other keys of the publication
    are applied and its expired keys deleted."""
    st, names = random_stream(91, n=40, p=0.15)
    dbs = st.to_dbs()
    p = host_ls()
    p.apply(st)
    # an update of node 3, a truncated value for node 4, node 6 updated, node 8 expired
    d3, d6 = dbs[3], dbs[6]
    d3.adjs = d3.adjs[1:]
    d6.node_label = 4242
    bad = TC.adjacency_database(dbs[4])[:5]
    kv = [(f"adj:{d3.name}", TC.value(TC.adjacency_database(d3))),
          (f"adj:{dbs[4].name}", TC.value(bad)),
          (f"adj:{d6.name}", TC.value(TC.adjacency_database(d6)))]
    pub = TC.publication(kv, expired=[f"adj:{dbs[8].name}"], area="0")
    ch = p.apply_publication(pub)
    assert p.decode_errors == [1]
    msg, n = p.last_decode_error()
    assert n == 1 and dbs[4].name in msg
    o = Oracle()
    o.apply(st)
    och = o.apply(AdjDbStream.from_dbs([d3, d6, AdjDb(dbs[8].name, delete=True)]))
    assert ch[0] == och[0] and ch[2] == och[1] and ch[3] == och[2]
    assert ch[1] == (False, False, False, 0)
    assert p.num_nodes() == o_nodes(names, dbs[8].name)
    for r in names:
        if r != dbs[8].name:
            assert p.spf_text(r) == o.spf_text(r), r


def o_nodes(names, deleted):
    return len([n for n in names if n != deleted])


def test_deeply_nested_values_raise_not_crash():
    """skip() bounds the nesting of lists / sets / maps as well as structs: a
    long run of 0x19 bytes (a one-element list of lists ...) in an unknown
    field is a decode error, not a stack overflow."""
    head = bytes([0x18, 0x01, ord("a")])          # 1: "a"
    nested_lists = head + bytes([0x59]) + bytes([0x19]) * 200000 + bytes([0x00])  # 6: list
    nested_maps = head + bytes([0x5B]) + bytes([0x01, 0xBB]) * 100000 + bytes([0x00])  # 6: map
    nested_structs = head + bytes([0x5C]) + bytes([0x1C]) * 100000 + bytes([0x00])
    for v in (nested_lists, nested_maps, nested_structs):
        with pytest.raises(ValueError):
            decode_adjdbs([v])
    # through a publication: the key is skipped, the call succeeds
    p = host_ls()
    pub = TC.publication([("adj:a", TC.value(nested_lists))])
    assert p.apply_publication(pub) == [(False, False, False, 0)]
    assert p.decode_errors == [0]
    # moderate nesting (< 64 levels) in an unknown field still decodes
    ok = head + bytes([0x59]) + bytes([0x19]) * 30 + bytes([0x13, 0x05]) + bytes([0x00])
    assert decode_adjdbs([ok]).to_dbs()[0].name == "a"


def test_publication_area_and_record_count():
    """A publication of another area is refused (Decision routes it to that
    area's LinkState, Decision.cpp:847-854); more change records than the
    first buffer holds: the wrapper asks again (nothing applied the first
    time), so every record of a large publication comes back."""
    st, names = random_stream(5, n=120, p=0.05)
    p = host_ls()
    pub = TC.publication([(k, TC.value(v)) for k, v in _kv_of(st.to_dbs())], area="other")
    with pytest.raises(LinkStateError, match="area"):
        p.apply_publication(pub)
    assert p.num_nodes() == 0
    pub = TC.publication([(k, TC.value(v)) for k, v in _kv_of(st.to_dbs())], area="0")
    ch = p.apply_publication(pub)
    assert len(ch) == len(names) > 64
    assert p.num_nodes() == len(names)
