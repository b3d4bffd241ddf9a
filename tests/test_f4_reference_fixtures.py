"""KvStore publication decode (§8(f) f4) pinned by the REFERENCE's own
fbthrift CompactSerializer bytes: the breeze decision-CLI fixtures
(openr/py/openr/cli/tests/decision/fixtures.py:259-346 KVSTORE_KEYVALS_OK,
with the decoded AdjacencyDatabases at :53-118 and the received routes with
their bestKey / bestKeys at :120-257), transcribed as data into
tests/golden/f4_reference_fixtures.json.

The bytes exercise what self-generated vectors may miss: a long-form field
header (AdjacencyDatabase field 4 written after 5 and 6), perfEvents inside
an AdjacencyDatabase, PrefixDatabase fields the decoder must skip, and
BinaryAddress / IpPrefix conversions. Both codecs (the product's C++
LsdbIngest / decodeAdjDb and oracle/thrift_compact.py) must decode every
field; ingestion (Decision::updateKeyInLsdb, Decision.cpp:710-785) must build
the same LSDB; on the GPU the routes and the best-route selection must equal
the oracle's and the fixture's bestKey / bestKeys."""
import json
import os

import pytest

import thrift_compact as tc

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                  "f4_reference_fixtures.json")))
AREA = FIX["area"]
KV = {k: bytes.fromhex(v["value_hex"]) for k, v in FIX["keyVals"].items()}
ADJ = {d["thisNodeName"]: d for d in FIX["expected_adj_dbs"]}
ROUTES = {r["prefix"]: r for r in FIX["expected_received_routes"]}


def _adj_fields(db):
    """Fields of an AdjacencyDatabase the route path consumes (everything the
    fixture states except perfEvents: DECISION_ADJ_DBS_OK's perf events are
    Decision's own, recorded at another time than the KvStore value's)."""
    out = {k: db[k] for k in ("thisNodeName", "isOverloaded", "nodeLabel")}
    out["adjacencies"] = [
        {k: a[k] for k in ("otherNodeName", "ifName", "nextHopV6", "nextHopV4", "metric",
                           "adjLabel", "isOverloaded", "rtt", "timestamp", "weight",
                           "otherIfName")}
        for a in db["adjacencies"]]
    return out


def _entry_fields(e):
    m = e["metrics"]
    return dict(prefix=e["prefix"], type=e["type"], forwardingType=e["forwardingType"],
                forwardingAlgorithm=e["forwardingAlgorithm"],
                metrics={k: m[k] for k in ("version", "path_preference", "source_preference",
                                           "distance", "drain_metric")},
                tags=sorted(e["tags"]), area_stack=list(e["area_stack"]))


@pytest.mark.parametrize("key", sorted(k for k in KV if k.startswith("adj:")))
def test_reference_adj_bytes_decode(host_module, key):
    node = key[len("adj:"):]
    want = _adj_fields(ADJ[node])
    py = tc.decode_adj_db(KV[key])
    cc = host_module.decodeAdjDb(KV[key])
    assert _adj_fields(py) == want
    assert _adj_fields(cc) == want
    assert py["area"] == cc["area"] == AREA
    # perfEvents of the KvStore value (field 5, a nested PerfEvents struct)
    assert [e[:2] for e in py["perfEvents"]] == [(node, "ADJ_DB_UPDATED")]
    assert py["perfEvents"][0][2] > 1631213000000


@pytest.mark.parametrize("key", sorted(k for k in KV if k.startswith("prefix:")))
def test_reference_prefix_bytes_decode(host_module, key):
    py = tc.decode_prefix_db(KV[key])
    cc = host_module.decodePrefixDb(KV[key])
    for db in (py, cc):
        assert len(db["prefixEntries"]) == 1
        assert db["deletePrefix"] is False
        e = db["prefixEntries"][0]
        r = ROUTES[e["prefix"]]
        (node, area), want = r["routes"][0]
        assert db["thisNodeName"] == node and area == AREA
        assert _entry_fields(e) == want
    # the key's own (area-qualified, pre-V2) format is not what updates read:
    # Decision decodes the value (Decision.cpp:742-770) and keys by its fields
    assert key.endswith(f"[{py['prefixEntries'][0]['prefix']}]")


def _ingest(M, me, make_pending):
    als = M.AreaLinkStates()
    ps = M.PrefixState()
    g = M.LsdbIngest(me, {AREA})
    pending = make_pending(me)
    g.processPublicationKeyVals(AREA, als, ps, sorted(KV.items()), [], pending)
    return als, ps, pending


def test_reference_publication_ingest_matches_oracle(host_module, oracle):
    """processPublication over the fixture's keyVals: the product's LsdbIngest
    and the oracle restatement build the same LSDB (one bidirectional link,
    four prefixes each advertised by one (node, area))."""
    als, ps, pending = _ingest(host_module, "openr-center", host_module.DecisionPendingUpdates)
    oals = {}
    ops = oracle.PrefixState()
    opend = tc.PendingUpdates("openr-center")
    tc.process_publication("openr-center", oals, oracle.LinkState, ops, AREA,
                           sorted(KV.items()), [], opend)
    ls, ols = als[AREA], oals[AREA]
    assert ls.numLinks() == ols.numLinks() == 1
    assert ls.linksFromNode("openr-center") == ols.linksFromNode("openr-center")
    want = {p: [[r["routes"][0][0][0], AREA]] for p, r in ROUTES.items()}
    got = {p: [list(na) for na in v] for p, v in ps.prefixes().items()}
    ogot = {p: [list(na) for na in v] for p, v in ops.prefixes().items()}
    assert got == ogot == want
    assert pending.needsFullRebuild() and opend.full
    assert set(pending.updatedPrefixes()) == opend.prefixes == set(ROUTES)


@pytest.mark.gpu
@pytest.mark.parametrize("brs", [False, True])
@pytest.mark.parametrize("me", ["openr-center", "openr-right"])
def test_reference_publication_routes_and_best_keys(product, oracle, me, brs):
    """RouteDb built from the decoded fixture equals the oracle's, and the
    best-route selection cache equals the fixture's bestKey / bestKeys
    (RECEIVED_ROUTES_DB_OK) for every prefix, self-advertised ones included."""
    als, ps, _ = _ingest(product, me, product.DecisionPendingUpdates)
    solver = product.SpfSolver(me, True, False, brs)
    db = solver.buildRouteDb(me, als, ps)
    oals = {}
    ops = oracle.PrefixState()
    tc.process_publication(me, oals, oracle.LinkState, ops, AREA, sorted(KV.items()), [],
                           tc.PendingUpdates(me))
    oas = oracle.AreaLinkStates()
    ols = oas.add(AREA, me)
    for key, val in sorted(KV.items()):  # same LSDB into an AreaLinkStates
        tc.update_key_in_lsdb(me, {AREA}, AREA, ols, oracle.PrefixState(), key, val)
    osolver = oracle.SpfSolver(me, True, False, brs)
    odb = osolver.buildRouteDb(me, oas, ops)
    assert db.canonical() == odb.canonical()
    other = "openr-right" if me == "openr-center" else "openr-center"
    assert set(db.unicastRoutes()) == {p for p, r in ROUTES.items() if r["bestKey"][0] == other}
    cache = solver.getBestRoutesCache()
    assert cache == osolver.getBestRoutesCache()
    for p, r in ROUTES.items():
        assert list(cache[p]["bestNodeArea"]) == r["bestKey"]
        assert [list(x) for x in cache[p]["allNodeAreas"]] == r["bestKeys"]
