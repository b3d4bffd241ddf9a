"""The incremental branch of Decision::rebuildRoutes (Decision.cpp:929-951):
createRouteForPrefixOrGetStaticRoute per changed prefix (SpfSolver.cpp:139-
311). The engine answers a changed set with one route launch over the SPF
memo of its last build (ogs_routes_from_spf; SPF-only launch on a miss).
Checked against the oracle's per-prefix calls: routes, the static-route
fallback, the v4 gate, unknown / local prefixes, and the best-route
selection cache after each call, across topology / prefix / source changes
that must invalidate the memo."""
import pytest

import lsdb as L

pytestmark = pytest.mark.gpu

A = L.kTestingAreaName
N = 5


def _grid(M, metric=lambda i, j: 1):
    als = M.AreaLinkStates()
    ls = als.add(A, "12")
    for i in range(N):
        for j in range(N):
            ls.updateAdjacencyDatabase(_adjdb(i, j, metric), A)
    return als, ls


def _adjdb(i, j, metric):
    node = i * N + j
    adjs = []
    for (ii, jj, ifn, oifn) in ((i, j + 1, "0/1", "0/3"), (i - 1, j, "0/2", "0/4"),
                                (i, j - 1, "0/3", "0/1"), (i + 1, j, "0/4", "0/2")):
        if 0 <= ii < N and 0 <= jj < N:
            nb = ii * N + jj
            m = metric(min(node, nb), max(node, nb))
            adjs.append(L.createAdjacency(str(nb), ifn, oifn, f"fe80::{nb:x}",
                                          f"192.168.0.{nb}", m, 100001 + nb))
    return L.createAdjDb(str(node), adjs, node + 1)


def _prefixes(M):
    ps = M.PrefixState()
    for n in range(N * N):
        ents = [L.createPrefixEntry(f"fc00::{n:x}/128")]
        if n in (3, 7):
            ents.append(L.createPrefixEntry(f"10.0.{n}.0/24"))
        if n in (4, 20):
            ents.append(L.createPrefixEntry("fc00::aa/128"))
        if n in (0, 12):  # also advertised by the source: selected, no route
            ents.append(L.createPrefixEntry("fc00::10c/128"))
        L.updatePrefixDatabase(ps, L.createPrefixDb(str(n), ents))
    return ps


STATICS = {
    "fc00::dead/128": dict(prefix="fc00::dead/128",
                           nexthops=[L.createNextHop("fe80::99", "eth9", 0)]),
    "10.9.9.0/24": dict(prefix="10.9.9.0/24",
                        nexthops=[L.createNextHop("10.1.1.1", "eth8", 0)]),
    # has a computed route too: the computed one wins
    "fc00::3/128": dict(prefix="fc00::3/128",
                        nexthops=[L.createNextHop("fe80::77", "eth7", 0)]),
}
ASKED = ["fc00::3/128", "fc00::6/128", "fc00::aa/128", "fc00::10c/128", "fc00::c/128",
         "10.0.3.0/24", "10.0.7.0/24", "fc00::dead/128", "10.9.9.0/24", "fc00::beef/128"]


def _solvers(product, oracle, me, v4, brs, v4o=False):
    out = []
    for M in (product, oracle):
        s = M.SpfSolver(me, v4, False, brs, v4o)
        s.updateStaticUnicastRoutes(STATICS, [])
        out.append(s)
    return out


def _check(ps_, os_, me, pa, pp, oa, op, label):
    for pfx in ASKED:
        want = os_.createRouteForPrefixOrGetStaticRoute(me, oa, op, pfx)
        got = ps_.createRouteForPrefixOrGetStaticRoute(me, pa, pp, pfx)
        assert got == want, (label, pfx)
    assert ps_.getBestRoutesCache() == os_.getBestRoutesCache(), label
    if not hasattr(ps_, "createRoutesForPrefixes"):  # oracle-only dry run
        return
    batch = ps_.createRoutesForPrefixes(me, pa, pp, set(ASKED))
    for pfx in ASKED:
        assert batch[pfx] == os_.createRouteForPrefixOrGetStaticRoute(me, oa, op, pfx), \
            (label, "batch", pfx)
    assert ps_.getBestRoutesCache() == os_.getBestRoutesCache(), (label, "batch")


@pytest.mark.parametrize("v4,v4o", [(False, False), (True, False), (False, True)])
@pytest.mark.parametrize("brs", [False, True])
def test_static_fallback_v4_gate_and_cache(product, oracle, v4, v4o, brs):
    pa, pls = _grid(product)
    oa, ols = _grid(oracle)
    pp, op = _prefixes(product), _prefixes(oracle)
    ps_, os_ = _solvers(product, oracle, "12", v4, brs, v4o)
    _check(ps_, os_, "12", pa, pp, oa, op, "cold")  # memo miss: SPF-only launch
    # a full build fills the memo; the incremental calls then reuse it
    assert ps_.buildRouteDb("12", pa, pp).canonical() == \
        os_.buildRouteDb("12", oa, op).canonical()
    _check(ps_, os_, "12", pa, pp, oa, op, "after build")


def test_memo_invalidation(product, oracle):
    """Topology change (attribute-only, CSR patched in place), prefix change
    and a different source on the same solver: never a stale SPF."""
    pa, pls = _grid(product)
    oa, ols = _grid(oracle)
    pp, op = _prefixes(product), _prefixes(oracle)
    ps_, os_ = _solvers(product, oracle, "12", True, True)
    _check(ps_, os_, "12", pa, pp, oa, op, "base")
    heavy = lambda i, j: 9 if (i, j) in ((7, 12), (11, 12), (12, 13)) else 1
    for ls in (pls, ols):
        for n in (7, 11, 12, 13):
            ls.updateAdjacencyDatabase(_adjdb(n // N, n % N, heavy), A)
    _check(ps_, os_, "12", pa, pp, oa, op, "metric change")
    for ps in (pp, op):
        L.updatePrefixDatabase(ps, L.createPrefixDb("6", [L.createPrefixEntry("fc00::aa/128")]))
    _check(ps_, os_, "12", pa, pp, oa, op, "prefix change")
    for me in ("0", "24", "12"):
        _check(ps_, os_, me, pa, pp, oa, op, f"source {me}")
    # node removed (structural change: re-flattened CSR)
    for ls in (pls, ols):
        ls.deleteAdjacencyDatabase("6")
    _check(ps_, os_, "12", pa, pp, oa, op, "node removed")


def test_source_absent(product, oracle):
    """A source with no adjacency database: no computed routes, statics
    still answer, the cache of known prefixes is cleared."""
    pa, _ = _grid(product)
    oa, _ = _grid(oracle)
    pp, op = _prefixes(product), _prefixes(oracle)
    ps_, os_ = _solvers(product, oracle, "99", True, True)
    _check(ps_, os_, "99", pa, pp, oa, op, "absent")


@pytest.mark.parametrize("areas", [1, 2])
def test_incremental_loop_one_batch(product, oracle, areas):
    """Decision's incremental loop as the reference runs it
    (Decision.cpp:929-951): after a full build, publications change a set
    of prefixes, then createRouteForPrefixOrGetStaticRoute is called once per
    changed prefix. The engine answers the whole loop from ONE batch over the
    PrefixState change log; every answer and the best-route selection cache
    after every call equal the oracle's per-prefix calls; single area and a
    two-area domain (the second area holds the source too)."""
    doms = []
    for M in (product, oracle):
        als, ls = _grid(M)
        if areas == 2:
            ls2 = als.add("area2", "12")
            ls2.updateAdjacencyDatabase(L.createAdjDb("12", [L.createAdjacency(
                "x1", "e1", "f1", "fe80::e1", "10.7.0.1", 3, 200001)], 13), "area2")
            ls2.updateAdjacencyDatabase(L.createAdjDb("x1", [L.createAdjacency(
                "12", "f1", "e1", "fe80::c", "10.7.0.2", 3, 200002)], 300), "area2")
        ps = _prefixes(M)
        if areas == 2:
            L.updatePrefixDatabase(ps, L.createPrefixDb("x1", [L.createPrefixEntry("fc00::aa/128")]),
                                   "area2")
        doms.append((als, ps))
    ps_, os_ = _solvers(product, oracle, "12", True, True)
    (pa, pp), (oa, op) = doms
    assert ps_.buildRouteDb("12", pa, pp).canonical() == os_.buildRouteDb("12", oa, op).canonical()
    assert ps_.getBestRoutesCache() == os_.getBestRoutesCache()
    changed = set()
    for ps in (pp, op):
        for n, pfx in ((6, "fc00::aa/128"), (9, "fc00::3/128"), (17, "fc00::77/128"),
                       (2, "10.0.3.0/24")):
            changed |= set(L.updatePrefixDatabase(ps, L.createPrefixDb(
                str(n), [L.createPrefixEntry(f"fc00::{n:x}/128"), L.createPrefixEntry(pfx)])))
    changed = sorted(changed)
    assert len(changed) >= 4
    b0 = ps_.incrementalBatches()
    for pfx in changed:
        got = ps_.createRouteForPrefixOrGetStaticRoute("12", pa, pp, pfx)
        want = os_.createRouteForPrefixOrGetStaticRoute("12", oa, op, pfx)
        assert got == want, pfx
        assert ps_.getBestRoutesCache() == os_.getBestRoutesCache(), pfx
    assert ps_.incrementalBatches() == b0 + 1
    # a prefix outside the changed set: one more (single-prefix) batch
    for pfx in ("fc00::c/128", "fc00::beef/128"):
        assert ps_.createRouteForPrefixOrGetStaticRoute("12", pa, pp, pfx) == \
            os_.createRouteForPrefixOrGetStaticRoute("12", oa, op, pfx)
        assert ps_.getBestRoutesCache() == os_.getBestRoutesCache(), pfx
