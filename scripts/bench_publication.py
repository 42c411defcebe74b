#!/usr/bin/env python3
"""f4 ingest from serialized publications: the F100k
fabric's 100,024 adjacency databases as one KvStore thrift::Publication
(compact protocol, written by the test-side encoder tests/thrift_compact.py),
then Decision's path into the engine's input: odl_apply_publication (decode on
host threads + LinkState ingest, Decision.cpp:743-765 / 846-870) and the CSR
snapshot the engine loads (odl::LinkState::snapshot). Host code only (no
GPU). Prints one JSON line: publication bytes, decode + apply ms, snapshot ms,
against the columnar stream ingest (AdjDbStream) of the same databases.

Usage: python scripts/bench_publication.py [--pods 1781] [--planes 8] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from openr_amd import topology as T  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402
import thrift_compact as TC  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=1781)
    ap.add_argument("--planes", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    st = T.fabric(pods=a.pods, planes=a.planes)
    dbs = st.to_dbs()
    t = time.perf_counter()
    pub = TC.publication([(f"adj:{d.name}", TC.value(TC.adjacency_database(d, extra=False)))
                          for d in dbs])
    enc_s = time.perf_counter() - t
    res = {"apply_publication_ms": [], "snapshot_ms": [], "stream_apply_ms": [],
           "stream_snapshot_ms": []}
    for _ in range(a.reps):
        p = LinkState()
        p.set_host_spf(True)  # (no engine: the snapshot is the last step measured)
        t = time.perf_counter()
        p.apply_publication(pub)
        res["apply_publication_ms"].append((time.perf_counter() - t) * 1e3)
        t = time.perf_counter()
        csr = p.csr()
        res["snapshot_ms"].append((time.perf_counter() - t) * 1e3)
        q = LinkState()
        q.set_host_spf(True)
        t = time.perf_counter()
        q.apply(st)
        res["stream_apply_ms"].append((time.perf_counter() - t) * 1e3)
        t = time.perf_counter()
        csr2 = q.csr()
        res["stream_snapshot_ms"].append((time.perf_counter() - t) * 1e3)
        assert all((csr[k] == csr2[k]).all() for k in csr), "publication and stream CSRs differ"
        del p, q
    med = {k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}
    print(json.dumps({
        "workload": f"F100k fabric pods={a.pods} planes={a.planes}: {len(dbs)} adjacency "
                    f"databases in one thrift::Publication (compact protocol)",
        "publication_bytes": len(pub), "adjacencies": int(sum(len(d.adjs) for d in dbs)),
        "host_threads": os.cpu_count(), **med,
        "publication_to_csr_ms": round(med["apply_publication_ms"] + med["snapshot_ms"], 1),
        "python_encode_s": round(enc_s, 1),
        "note": "apply_publication = compact-thrift decode of every Value on host threads + "
                "LinkState ingest (bulk path); snapshot = the CSR the engine loads; the stream "
                "rows are the columnar AdjDbStream ingest of the same databases; the CSRs are "
                "checked equal"}))


if __name__ == "__main__":
    main()
