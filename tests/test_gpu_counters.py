"""fb303-style Decision counters of the drop-in (stats.cpp): the reference's
keys (SpfSolver.cpp:86-104) with the reference's increments --
decision.route_build_runs once per buildRouteDb of a known node (:327),
decision.get_route_for_prefix once per prefix considered (:166, the build's
loop :334-339), decision.no_route_to_prefix per prefix whose advertisers are
all unreachable (:221), decision.spf_runs per SPF (LinkState.cpp:727) -- and
the AVG timers decision.spf_ms / route_build_ms plus the engine's
decision.gpu.prepare_ms / launch_ms / materialize_ms."""
import pytest

import lsdb as L

pytestmark = pytest.mark.gpu

A = L.kTestingAreaName


def _line(M):
    """1 - 2 - 3 plus an isolated 4 (adjacency database without links):
    prefixes of 1..3 route, the prefix of 4 has no reachable advertiser."""
    als = M.AreaLinkStates()
    ls = als.add(A, "1")
    nbrs = {1: [2], 2: [1, 3], 3: [2], 4: []}
    for n, ns in nbrs.items():
        adjs = [L.createAdjacency(str(m), f"if{n}{m}", f"if{m}{n}", f"fe80::{m}",
                                  f"10.0.0.{m}", 1, 100 + m) for m in ns]
        ls.updateAdjacencyDatabase(L.createAdjDb(str(n), adjs, n), A)
    ps = M.PrefixState()
    for n in nbrs:
        L.updatePrefixDatabase(ps, L.createPrefixDb(str(n), [L.createPrefixEntry(f"fc00::{n}/128")]))
    return als, ls, ps


def test_decision_counters(product):
    M = product
    als, ls, ps = _line(M)
    solver = M.SpfSolver("1", True, False, False, False)
    M.reset_decision_counters()
    for _ in range(3):
        db = solver.buildRouteDb("1", als, ps)
        assert db is not None
    assert solver.buildRouteDb("no-such-node", als, ps) is None  # not counted (:322-324)
    ls.getSpfResult("2")
    c = M.decision_counters()
    assert c["decision.route_build_runs.count"] == 3
    assert c["decision.get_route_for_prefix.count"] == 3 * 4
    assert c["decision.no_route_to_prefix.count"] == 3  # fc00::4 each build
    # the reference memoises getSpfResult per (node, useLinkMetric) until the
    # topology changes (LinkState.cpp:705-715): the 3 builds of "1" run ONE
    # SPF, getSpfResult("2") another
    assert c["decision.spf_runs.count"] == 2
    for key in ("decision.route_build_ms", "decision.spf_ms", "decision.gpu.prepare_ms",
                "decision.gpu.launch_ms", "decision.gpu.materialize_ms"):
        assert c[key + ".count"] >= 1 and c[key + ".avg"] >= 0.0, key
    assert c["decision.route_build_ms.count"] == 3
    M.reset_decision_counters()
    assert M.decision_counters() == {}


def test_spf_runs_ring_four_sources(product):
    """SpfSolverTest.cpp:1655-1667 SimpleRingTopologyFixture.ShortestPathTest:
    route maps of 4 sources with node segment labels run exactly 4 SPFs
    (decision.spf_runs.count == 4). Building them again, or asking
    getSpfResult / getKthPaths(k = 1) of those sources, runs none (the memo);
    a topology change invalidates it (LinkState.cpp:635-638)."""
    M = product
    als = M.AreaLinkStates()
    ls = als.add(A, "1")
    for db in (L.createAdjDb("1", [L.adj12, L.adj13], 1), L.createAdjDb("2", [L.adj21, L.adj24], 2),
               L.createAdjDb("3", [L.adj31, L.adj34], 3), L.createAdjDb("4", [L.adj42, L.adj43], 4)):
        ls.updateAdjacencyDatabase(db, A)
    ps = M.PrefixState()
    for p in (L.prefixDb1, L.prefixDb2, L.prefixDb3, L.prefixDb4):
        L.updatePrefixDatabase(ps, p)
    solver = M.SpfSolver("1", False, True)
    M.reset_decision_counters()
    rm = L.getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
    assert len(rm) == 28
    assert M.decision_counters()["decision.spf_runs.count"] == 4
    assert L.getRouteMap(solver, ["1", "2", "3", "4"], als, ps) == rm
    ls.getSpfResult("3")
    ls.getKthPaths("2", "4", 1)
    assert M.decision_counters()["decision.spf_runs.count"] == 4
    ls.getKthPaths("2", "4", 2)  # a masked runSpf (LinkState.cpp:690-692)
    assert M.decision_counters()["decision.spf_runs.count"] == 5
    adj12b = L.createAdjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 30, 100002)
    assert ls.updateAdjacencyDatabase(L.createAdjDb("1", [adj12b, L.adj13], 1), A)["topologyChanged"]
    rm2 = L.getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
    assert rm2 != rm
    assert M.decision_counters()["decision.spf_runs.count"] == 9


def test_no_route_counted_on_every_path(product):
    """decision.no_route_to_prefix (SpfSolver.cpp:221, 242, 579) is counted
    per unroutable prefix considered on every route path, not only the
    single-area full build: the incremental branch
    (createRoutesForPrefixes -> one createRouteForPrefix per asked prefix)
    and the multi-area build."""
    M = product
    als, ls, ps = _line(M)
    solver = M.SpfSolver("1", True, False, False, False)
    solver.buildRouteDb("1", als, ps)
    M.reset_decision_counters()
    out = solver.createRoutesForPrefixes("1", als, ps, {"fc00::4/128", "fc00::2/128"})
    assert out["fc00::4/128"] is None and out["fc00::2/128"] is not None
    c = M.decision_counters()
    assert c["decision.get_route_for_prefix.count"] == 2
    assert c["decision.no_route_to_prefix.count"] == 1
    # a second area holding only node 1: the multi-area build
    ls_b = als.add("area_b", "1")
    ls_b.updateAdjacencyDatabase(L.createAdjDb("1", [], 1, area="area_b"), "area_b")
    M.reset_decision_counters()
    db = M.SpfSolver("1", True, False, False, False).buildRouteDb("1", als, ps)
    assert db is not None
    assert M.decision_counters()["decision.no_route_to_prefix.count"] == 1


def test_spf_memo_every_source(product, oracle):
    """The getSpfResult memo holds every source's SPF until a topology change
    (LinkState.cpp:705-715, LinkState.h:369-372), and Decision builds
    RouteDbs for arbitrary nodes (getDecisionRouteDb, Decision.cpp:341-361):
    alternating buildRouteDb("1"), ("2"), ("1") launches TWO device SPFs --
    the engine's own launch counter equals decision.spf_runs -- and the
    RouteDbs equal the oracle's. getSpfResult of a built source reads the
    same device rows (no launch); a topology change starts over."""
    M = product
    als, ls, ps = _line(M)
    oals, ols, ops = _line(oracle)
    solver = M.SpfSolver("1", True, True, False, False)
    osolver = oracle.SpfSolver("1", True, True, False, False)
    M.reset_decision_counters()
    for node in ("1", "2", "1", "2", "3", "1"):
        got = solver.buildRouteDb(node, als, ps).canonical()
        assert got == osolver.buildRouteDb(node, oals, ops).canonical(), node
    c = M.decision_counters()
    assert c["decision.spf_runs.count"] == 3
    assert c["decision.gpu.spf_launches.count"] == 3
    want = {k: (v[0], sorted(v[1])) for k, v in ols.getSpfResult("2").items()}
    assert {k: (v[0], sorted(v[1])) for k, v in ls.getSpfResult("2").items()} == want
    c = M.decision_counters()
    assert c["decision.spf_runs.count"] == 3 and c["decision.gpu.spf_launches.count"] == 3
    # incremental routes of a memoised source: no SPF either
    out = solver.createRoutesForPrefixes("3", als, ps, {"fc00::1/128"})
    assert out["fc00::1/128"] is not None
    assert M.decision_counters()["decision.gpu.spf_launches.count"] == 3
    # a topology change (metric 1 -> 5 on 1-2) invalidates every source
    adjs = [L.createAdjacency("2", "if12", "if21", "fe80::2", "10.0.0.2", 5, 102)]
    assert ls.updateAdjacencyDatabase(L.createAdjDb("1", adjs, 1), A)["topologyChanged"]
    assert ols.updateAdjacencyDatabase(L.createAdjDb("1", adjs, 1), A)["topologyChanged"]
    for node in ("2", "1", "2"):
        assert (solver.buildRouteDb(node, als, ps).canonical() ==
                osolver.buildRouteDb(node, oals, ops).canonical()), node
    c = M.decision_counters()
    assert c["decision.spf_runs.count"] == 5
    assert c["decision.gpu.spf_launches.count"] == 5
