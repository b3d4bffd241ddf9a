"""Generates tests/golden/f4_publications.json: compact-thrift vectors for
AdjacencyDatabase / PrefixDatabase from the oracle encoder
(oracle/thrift_compact.py), over the reference's own test values
(openr/decision/tests/Consts.h adjacencies, SpfSolverTest.cpp prefixes).
Byte layout is parity unpinned (no reference-serialized fixtures exist);
the file freezes it so both codecs are held to the same bytes.

    python tests/golden/make_f4.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "..", "oracle")]

import thrift_compact as tc  # noqa: E402
import lsdb  # noqa: E402


def main():
    adj_dbs = [
        lsdb.createAdjDb("1", [lsdb.adj12, lsdb.adj13], 1),
        lsdb.createAdjDb("2", [lsdb.adj21, lsdb.adj23, lsdb.adj24], 2, overLoadBit=True),
        lsdb.createAdjDb("3", [], 0, nodeMetricIncrementVal=-7),
        lsdb.createAdjDb("4", [dict(lsdb.adj12, weight=1 << 40, timestamp=-1, rtt=-(1 << 31),
                                    isOverloaded=True, adjOnlyUsedByOtherNode=True)] * 16, 1 << 19),
    ]
    e1 = lsdb.createPrefixEntry(lsdb.addr1)
    e2 = lsdb.createPrefixEntry(lsdb.addr1V4, minNexthop=2, weight=-3)
    e3 = lsdb.createPrefixEntryWithMetrics("fc00:0:0:1::/64", lsdb.BGP, lsdb.createMetrics(200, 100, 7))
    e3["tags"] = ["COMMODITY", "65000:%d" % 1]
    e3["area_stack"] = ["spine", "edge"]
    prefix_dbs = [
        dict(thisNodeName="1", prefixEntries=[e1], deletePrefix=False),
        dict(thisNodeName="2", prefixEntries=[e2], deletePrefix=True),
        dict(thisNodeName="3", prefixEntries=[e3, e1], deletePrefix=False,
             perfEvents=[("3", "PREFIX_DB_UPDATED", 1700000000123)]),
        dict(thisNodeName="4", prefixEntries=[], deletePrefix=False),
    ]
    out = {
        "generator": "tests/golden/make_f4.py (oracle/thrift_compact.py encoder)",
        "adj_dbs": [{"struct": tc.decode_adj_db(tc.encode_adj_db(d)), "hex": tc.encode_adj_db(d).hex()}
                    for d in adj_dbs],
        "prefix_dbs": [{"struct": tc.decode_prefix_db(tc.encode_prefix_db(d)),
                        "hex": tc.encode_prefix_db(d).hex()} for d in prefix_dbs],
    }
    with open(os.path.join(HERE, "f4_publications.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
