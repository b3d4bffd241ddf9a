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
    assert c["decision.spf_runs.count"] >= 4  # 3 builds (fused SPF) + getSpfResult("2")
    for key in ("decision.route_build_ms", "decision.spf_ms", "decision.gpu.prepare_ms",
                "decision.gpu.launch_ms", "decision.gpu.materialize_ms"):
        assert c[key + ".count"] >= 1 and c[key + ".avg"] >= 0.0, key
    assert c["decision.route_build_ms.count"] == 3
    M.reset_decision_counters()
    assert M.decision_counters() == {}
