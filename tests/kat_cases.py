"""Known-answer tests transcribed from the reference's own unit tests.

Every case takes the implementation module `M` (oracle/_refcpu or the GPU
product openr_amd._decision) and asserts the expectations the reference
tests assert. Source of each case is cited as file:line under
/root/reference (read-only; not needed at run time).
"""
from lsdb import *  # noqa: F401,F403
import lsdb as L


def _setup(M, nodeName):
    als = M.AreaLinkStates()
    ls = als.add(L.kTestingAreaName, nodeName)
    return als, ls, M.PrefixState()


def _change(t, l, n):
    return dict(topologyChanged=t, linkAttributesChanged=l, nodeLabelChanged=n)


def _chg(r):
    return {k: r[k] for k in ("topologyChanged", "linkAttributesChanged", "nodeLabelChanged")}


# ---------------------------------------------------------------- LinkState
def kat_linkstate_basic(M):
    """LinkStateTest.cpp:76-146 LinkStateTest.BasicOperation."""
    n1, n2, n3 = "node1", "node2", "node3"
    adj12 = createAdjacency(n2, "if2", "if1", "fe80::2", "10.0.0.2", 1, 1, 1)
    adj13 = createAdjacency(n3, "if3", "if1", "fe80::3", "10.0.0.3", 1, 1, 1)
    adj21 = createAdjacency(n1, "if1", "if2", "fe80::1", "10.0.0.1", 1, 1, 1)
    adj23 = createAdjacency(n3, "if3", "if2", "fe80::3", "10.0.0.3", 1, 1, 1)
    adj31 = createAdjacency(n1, "if1", "if3", "fe80::1", "10.0.0.1", 1, 1, 1)
    adj32 = createAdjacency(n2, "if2", "if3", "fe80::2", "10.0.0.2", 1, 1, 1)
    # Link(n1, adj12, n2, adj21) etc.: each side keeps its OWN ifName
    l1 = (n1, "if2", n2, "if1")
    l2 = (n2, "if3", n3, "if2")
    l3 = (n1, "if3", n3, "if1")
    adjDb1 = createAdjDb(n1, [adj12, adj13], 1)
    adjDb2 = createAdjDb(n2, [adj21, adj23], 2)
    adjDb3 = createAdjDb(n3, [adj31, adj32], 3)
    als = M.AreaLinkStates()
    state = als.add(kTestingAreaName, n1)
    assert state.getArea() == kTestingAreaName
    assert not state.updateAdjacencyDatabase(adjDb1, kTestingAreaName)["topologyChanged"]
    u = state.updateAdjacencyDatabase(adjDb2, kTestingAreaName)
    assert u["topologyChanged"] and u["addedLinks"] == 1
    u = state.updateAdjacencyDatabase(adjDb3, kTestingAreaName)
    assert u["topologyChanged"] and u["addedLinks"] == 2

    def ids(n):
        return sorted(link_id(x) for x in state.linksFromNode(n))
    assert ids(n1) == sorted([l1, l3])
    assert ids(n2) == sorted([l1, l2])
    assert ids(n3) == sorted([l2, l3])
    assert ids("node4") == []

    assert not state.isNodeOverloaded(n1)
    adjDb1["isOverloaded"] = True
    assert state.updateAdjacencyDatabase(adjDb1, kTestingAreaName)["topologyChanged"]
    assert state.isNodeOverloaded(n1)
    assert not state.updateAdjacencyDatabase(adjDb1, kTestingAreaName)["topologyChanged"]
    adjDb1["isOverloaded"] = False
    assert state.updateAdjacencyDatabase(adjDb1, kTestingAreaName)["topologyChanged"]
    assert not state.isNodeOverloaded(n1)

    adjDb1 = createAdjDb(n1, [adj13], 1)
    assert state.updateAdjacencyDatabase(adjDb1, kTestingAreaName)["topologyChanged"]
    assert ids(n1) == [l3]
    assert ids(n2) == [l2]
    assert ids(n3) == sorted([l2, l3])
    assert state.deleteAdjacencyDatabase(n1)["topologyChanged"]
    assert ids(n1) == []
    assert ids(n2) == [l2]
    assert ids(n3) == [l2]


def kat_linkstate_link_usable(M):
    """LinkStateTest.cpp:148-187 LinkStateTest.linkUsable."""
    n1, n2, n3 = "node1", "node2", "node3"
    adj12 = createAdjacency(n2, "if2", "if1", "fe80::2", "10.0.0.2", 1, 1, 1)
    adj21 = createAdjacency(n1, "if1", "if2", "fe80::1", "10.0.0.1", 1, 1, 1)
    adj21["adjOnlyUsedByOtherNode"] = True
    adj23 = createAdjacency(n3, "if3", "if2", "fe80::3", "10.0.0.3", 1, 1, 1)
    adj32 = createAdjacency(n2, "if2", "if3", "fe80::2", "10.0.0.2", 1, 1, 1)
    dbs = [createAdjDb(n1, [adj12], 1), createAdjDb(n2, [adj21, adj23], 2),
           createAdjDb(n3, [adj32], 3)]
    for node in (n1, n2, n3):
        als = M.AreaLinkStates()
        state = als.add(kTestingAreaName, node)
        for db in dbs:
            state.updateAdjacencyDatabase(db, kTestingAreaName)
        n1links = state.linksFromNode(n1)
        assert len(n1links) == 1
        assert n1links[0]["usable"] == (node == n1)
        n3links = state.linksFromNode(n3)
        assert len(n3links) == 1 and n3links[0]["usable"]


def kat_linkstate_kth_paths(M):
    """LinkStateTest.cpp:234-306 LinkStateTest.getKthPaths."""
    _, ls = getLinkState(M, {
        1: [(2, 10), (3, 5)],
        2: [(1, 10), (4, 15), (4, 35)],
        3: [(1, 5), (4, 20)],
        4: [(2, 15), (3, 20), (2, 35)],
    })
    first = ls.getKthPaths("2", "4", 1)
    assert len(first) == 1 and len(first[0]) == 1
    assert metric_from(first[0][0], "2") == 15
    second = ls.getKthPaths("2", "4", 2)
    assert sorted(len(p) for p in second) == [1, 3]
    for path in second:
        node, dist = "2", 0
        for link in path:
            dist += metric_from(link, node)
            node = other_node(link, node)
        assert dist == 35

    _, ls = getLinkState(M, {
        1: [2, 2, 3, 3, 4, 4],
        2: [1, 1, 3, 3, 4, 4],
        3: [1, 1, 2, 2, 4, 4],
        4: [1, 1, 2, 2, 3, 3],
    })
    first = ls.getKthPaths("2", "4", 1)
    assert len(first) == 2 and all(len(p) == 1 for p in first)
    second = ls.getKthPaths("2", "4", 2)
    assert len(second) == 4 and all(len(p) == 2 for p in second)
    seen = set()
    for path in first + second:
        for link in path:
            assert link_id(link) not in seen
            seen.add(link_id(link))


# ---------------------------------------------------------------- SpfSolver
def kat_unreachable_nodes(M):
    """SpfSolverTest.cpp:142-176 ShortestPathTest.UnreachableNodes."""
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True, True, False)
    assert not ls.updateAdjacencyDatabase(createAdjDb("1", [], 0), kTestingAreaName)["topologyChanged"]
    assert not ls.updateAdjacencyDatabase(createAdjDb("2", [], 0), kTestingAreaName)["topologyChanged"]
    assert updatePrefixDatabase(ps, prefixDb1)
    assert updatePrefixDatabase(ps, prefixDb2)
    for node in ("1", "2"):
        db = solver.buildRouteDb(node, als, ps)
        assert db is not None
        assert len(db.unicastRoutes()) == 0 and len(db.mplsRoutes()) == 0


def kat_drained_node_least_preferred(M):
    """SpfSolverTest.cpp:186-298 SpfSolver.DrainedNodeLeastPreferred."""
    adjacencyDb1 = createAdjDb("1", [adj12], 0)
    adjacencyDb2 = createAdjDb("2", [adj21, adj23], 0)
    adjacencyDb3 = createAdjDb("3", [adj32], 0)
    als, ls, ps = _setup(M, "2")
    solver = M.SpfSolver("2", False, True, True, True)
    for db in (adjacencyDb1, adjacencyDb2, adjacencyDb3):
        ls.updateAdjacencyDatabase(db, kTestingAreaName)
    prefix = createPrefixEntryWithMetrics(addr1, CONFIG, createMetrics(100, 100, 0))
    prefixHigh = createPrefixEntryWithMetrics(addr1, CONFIG, createMetrics(300, 300, 0))
    assert updatePrefixDatabase(ps, createPrefixDb("1", [prefix]))
    assert not updatePrefixDatabase(ps, createPrefixDb("2", []))
    assert updatePrefixDatabase(ps, createPrefixDb("3", [prefixHigh]))

    def check(adj, drain):
        db = solver.buildRouteDb("2", als, ps)
        routes = db.unicastRoutes()
        assert len(routes) == 1
        e = routes[addr1]
        assert e["nexthops"] == {createNextHopFromAdj(adj, False, adj["metric"])}
        assert e["bestPrefixEntry"]["metrics"]["drain_metric"] == drain

    check(adj23, 0)
    adjacencyDb3["nodeMetricIncrementVal"] = 100
    assert ls.updateAdjacencyDatabase(adjacencyDb3, kTestingAreaName)["topologyChanged"]
    check(adj21, 0)
    adjacencyDb3["nodeMetricIncrementVal"] = 0
    adjacencyDb3["isOverloaded"] = True
    assert ls.updateAdjacencyDatabase(adjacencyDb3, kTestingAreaName)["topologyChanged"]
    check(adj21, 0)
    adjacencyDb3["isOverloaded"] = False
    prefixHigh["metrics"]["drain_metric"] = 1
    updatePrefixDatabase(ps, createPrefixDb("3", [prefixHigh]))
    assert ls.updateAdjacencyDatabase(adjacencyDb3, kTestingAreaName)["topologyChanged"]
    check(adj21, 0)


def kat_missing_and_empty_neighbor_db(M):
    """SpfSolverTest.cpp:305-380 MissingNeighborAdjacencyDb +
    EmptyNeighborAdjacencyDb."""
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True, True, False)
    assert not ls.updateAdjacencyDatabase(createAdjDb("1", [adj12], 0), kTestingAreaName)["topologyChanged"]
    assert updatePrefixDatabase(ps, prefixDb1)
    assert updatePrefixDatabase(ps, prefixDb2)
    db = solver.buildRouteDb("1", als, ps)
    assert len(db.unicastRoutes()) == 0 and len(db.mplsRoutes()) == 0

    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True, True, False)
    assert not ls.updateAdjacencyDatabase(createAdjDb("1", [adj12], 0), kTestingAreaName)["topologyChanged"]
    assert not ls.updateAdjacencyDatabase(createAdjDb("2", [], 0), kTestingAreaName)["topologyChanged"]
    updatePrefixDatabase(ps, prefixDb1)
    updatePrefixDatabase(ps, prefixDb2)
    assert len(solver.buildRouteDb("1", als, ps).unicastRoutes()) == 0
    assert len(solver.buildRouteDb("2", als, ps).unicastRoutes()) == 0


def kat_unknown_node(M):
    """SpfSolverTest.cpp:386-408 ShortestPathTest.UnknownNode."""
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True, True, False)
    assert solver.buildRouteDb("1", als, ps) is None
    assert solver.buildRouteDb("2", als, ps) is None


def kat_node_soft_drained_choice(M):
    """SpfSolverTest.cpp:415-540 SpfSolver.NodeSoftDrainedChoice."""
    adjacencyDb1 = createAdjDb("1", [adj12], 0)
    adjacencyDb2 = createAdjDb("2", [adj21, adj23], 0)
    adjacencyDb3 = createAdjDb("3", [adj32], 0)
    als, ls, ps = _setup(M, "2")
    solver = M.SpfSolver("2", False, True, True, False)
    assert not ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(adjacencyDb2, kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(adjacencyDb3, kTestingAreaName)["topologyChanged"]
    p1 = createPrefixEntry(addr1, CONFIG)
    assert updatePrefixDatabase(ps, createPrefixDb("1", [p1]))
    assert not updatePrefixDatabase(ps, createPrefixDb("2", []))
    assert updatePrefixDatabase(ps, createPrefixDb("3", [p1]))

    def route():
        routes = solver.buildRouteDb("2", als, ps).unicastRoutes()
        assert len(routes) == 1
        return routes[addr1]

    adjacencyDb1["nodeMetricIncrementVal"] = 50
    assert ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    e = route()
    assert e["nexthops"] == {createNextHopFromAdj(adj23, False, 10)}
    assert e["bestPrefixEntry"]["metrics"]["drain_metric"] == 0
    adjacencyDb3["nodeMetricIncrementVal"] = 50
    assert ls.updateAdjacencyDatabase(adjacencyDb3, kTestingAreaName)["topologyChanged"]
    e = route()
    assert len(e["nexthops"]) == 2 and e["bestPrefixEntry"]["metrics"]["drain_metric"] == 1
    adjacencyDb1["nodeMetricIncrementVal"] = 100
    assert ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    e = route()
    assert len(e["nexthops"]) == 2 and e["bestPrefixEntry"]["metrics"]["drain_metric"] == 1
    adjacencyDb1["nodeMetricIncrementVal"] = 0
    assert ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    e = route()
    assert e["nexthops"] == {createNextHopFromAdj(adj21, False, 10)}
    assert e["bestPrefixEntry"]["metrics"]["drain_metric"] == 0


def kat_node_overload_route_choice(M):
    """SpfSolverTest.cpp:547-651 SpfSolver.NodeOverloadRouteChoice."""
    adjacencyDb1 = createAdjDb("1", [adj12], 1)
    adjacencyDb2 = createAdjDb("2", [adj21, adj23], 2)
    adjacencyDb3 = createAdjDb("3", [adj32], 3)
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True, True, False)
    r = ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)
    assert not r["topologyChanged"] and r["nodeLabelChanged"]
    r = ls.updateAdjacencyDatabase(adjacencyDb2, kTestingAreaName)
    assert r["topologyChanged"] and r["nodeLabelChanged"]
    r = ls.updateAdjacencyDatabase(adjacencyDb3, kTestingAreaName)
    assert r["topologyChanged"] and r["nodeLabelChanged"]
    prefix1 = createPrefixEntry(addr1, CONFIG)
    prefix3 = createPrefixEntry(addr1, VIP)
    assert updatePrefixDatabase(ps, createPrefixDb("1", [prefix1]))
    assert not updatePrefixDatabase(ps, createPrefixDb("2", []))
    assert updatePrefixDatabase(ps, createPrefixDb("3", [prefix3]))
    r2 = solver.buildRouteDb("2", als, ps).unicastRoutes()
    assert len(r2) == 1 and len(r2[addr1]["nexthops"]) == 2
    assert len(solver.buildRouteDb("1", als, ps).unicastRoutes()) == 0
    assert len(solver.buildRouteDb("3", als, ps).unicastRoutes()) == 0
    adjacencyDb1["isOverloaded"] = True
    r = ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)
    assert r["topologyChanged"] and not r["nodeLabelChanged"]
    r2 = solver.buildRouteDb("2", als, ps).unicastRoutes()
    assert len(r2) == 1 and len(r2[addr1]["nexthops"]) == 1
    r1 = solver.buildRouteDb("1", als, ps).unicastRoutes()
    assert len(r1) == 1
    assert r1[addr1]["bestPrefixEntry"] == prefix3
    assert r1[addr1]["localRouteConsidered"]
    assert len(solver.buildRouteDb("3", als, ps).unicastRoutes()) == 0


def kat_adjacency_update(M):
    """SpfSolverTest.cpp:657-784 SpfSolver.AdjacencyUpdate."""
    adjacencyDb1 = createAdjDb("1", [adj12], 1)
    adjacencyDb2 = createAdjDb("2", [adj21], 2)
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True, True, False)
    r = ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)
    assert not r["topologyChanged"] and r["nodeLabelChanged"]
    r = ls.updateAdjacencyDatabase(adjacencyDb2, kTestingAreaName)
    assert r["topologyChanged"] and r["nodeLabelChanged"]
    updatePrefixDatabase(ps, prefixDb1)
    updatePrefixDatabase(ps, prefixDb2)

    def counts():
        for n in ("1", "2"):
            db = solver.buildRouteDb(n, als, ps)
            assert len(db.unicastRoutes()) == 1 and len(db.mplsRoutes()) == 2
    counts()
    adjacencyDb1["adjacencies"][0]["nextHopV6"] = "fe80::1234:b00c"
    r = ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)
    assert not r["topologyChanged"] and r["linkAttributesChanged"]
    counts()
    # the new v6 next-hop address is what node 1 now programs toward node 2
    nhs = solver.buildRouteDb("1", als, ps).unicastRoutes()[addr2]["nexthops"]
    assert {nh[0] for nh in nhs} == {"fe80::1234:b00c"}
    adjacencyDb2["adjacencies"][0]["nextHopV6"] = "fe80::5678:b00c"
    r = ls.updateAdjacencyDatabase(adjacencyDb2, kTestingAreaName)
    assert not r["topologyChanged"] and r["linkAttributesChanged"]
    counts()
    adjacencyDb1["nodeLabel"] = 11
    assert _chg(ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)) == _change(False, False, True)
    adjacencyDb2["nodeLabel"] = 22
    assert _chg(ls.updateAdjacencyDatabase(adjacencyDb2, kTestingAreaName)) == _change(False, False, True)


def kat_mpls_basic(M):
    """SpfSolverTest.cpp:788-840 MplsRoutes.BasicTest."""
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True, False)
    adjacencyDb1 = createAdjDb("1", [adj12], 1)
    adjacencyDb2 = createAdjDb("2", [adj23], 0)
    adjacencyDb3 = createAdjDb("3", [adj32], 3)
    assert _chg(ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)) == _change(False, False, True)
    assert _chg(ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)) == _change(False, False, False)
    assert _chg(ls.updateAdjacencyDatabase(adjacencyDb2, kTestingAreaName)) == _change(False, False, False)
    assert _chg(ls.updateAdjacencyDatabase(adjacencyDb3, kTestingAreaName)) == _change(True, False, True)
    routeMap = getRouteMap(solver, ["1", "2", "3"], als, ps)
    assert len(routeMap) == 3
    assert routeMap[("1", "1")] == {labelPopNextHop}
    assert routeMap[("3", "3")] == {labelPopNextHop}


def kat_bgp_igp_metric(M):
    """SpfSolverTest.cpp:846-993 BGPRedistribution.IgpMetric."""
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True, True)
    bgp2 = createPrefixEntry(addr1, BGP, "data1", 0, 0)
    bgp3 = createPrefixEntry(addr1, BGP, "data1", 0, 0)
    adjacencyDb1 = createAdjDb("1", [adj12, adj13], 0)
    assert not ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(createAdjDb("2", [adj21], 0), kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(createAdjDb("3", [adj31], 0), kTestingAreaName)["topologyChanged"]
    assert updatePrefixDatabase(ps, createPrefixDb("2", [createPrefixEntry(addr2), bgp2]))
    assert updatePrefixDatabase(ps, createPrefixDb("3", [createPrefixEntry(addr3), bgp3]))

    def step(n_routes, expected):
        routes = solver.buildRouteDb("1", als, ps).unicastRoutes()
        assert len(routes) == n_routes
        assert routes[addr1]["nexthops"] == set(expected)

    step(3, [createNextHopFromAdj(adj12, False, 10), createNextHopFromAdj(adj13, False, 10)])
    adjacencyDb1["adjacencies"][1]["metric"] = 20
    assert ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    step(3, [createNextHopFromAdj(adj12, False, 10)])
    adjacencyDb1["adjacencies"][0]["isOverloaded"] = True
    assert ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    step(2, [createNextHopFromAdj(adj13, False, 20)])
    adjacencyDb1["adjacencies"][0]["metric"] = 20
    assert ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    step(2, [createNextHopFromAdj(adj13, False, 20)])
    adjacencyDb1["adjacencies"][0]["isOverloaded"] = False
    assert ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    step(3, [createNextHopFromAdj(adj12, False, 20), createNextHopFromAdj(adj13, False, 20)])


def kat_igp_cost(M):
    """SpfSolverTest.cpp:995-1056 Decision.IgpCost."""
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True, True)
    dbs = [createAdjDb("1", [adj12, adj13], 1), createAdjDb("2", [adj21, adj24], 2),
           createAdjDb("3", [adj31, adj34], 3), createAdjDb("4", [adj42, adj43], 4)]
    assert not ls.updateAdjacencyDatabase(dbs[0], kTestingAreaName)["topologyChanged"]
    for db in dbs[1:]:
        assert ls.updateAdjacencyDatabase(db, kTestingAreaName)["topologyChanged"]
    p2 = createPrefixEntryWithMetrics(addr1, DEFAULT, createMetrics(200, 0, 0))
    assert updatePrefixDatabase(ps, createPrefixDb("2", [p2]))
    assert solver.buildRouteDb("1", als, ps).unicastRoutes()[addr1]["igpCost"] == 10
    assert ls.updateAdjacencyDatabase(createAdjDb("2", [adj24], 4), kTestingAreaName)["topologyChanged"]
    assert solver.buildRouteDb("1", als, ps).unicastRoutes()[addr1]["igpCost"] == 30


def kat_best_route_selection(M):
    """SpfSolverTest.cpp:1058-1169 Decision.BestRouteSelection."""
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True, True)
    assert not ls.updateAdjacencyDatabase(createAdjDb("1", [adj12, adj13], 1), kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(createAdjDb("2", [adj21], 2), kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(createAdjDb("3", [adj31], 3), kTestingAreaName)["topologyChanged"]
    p2 = createPrefixEntryWithMetrics(addr1, DEFAULT, createMetrics(200, 0, 0))
    p3 = createPrefixEntryWithMetrics(addr1, BGP, createMetrics(200, 0, 0))
    assert updatePrefixDatabase(ps, createPrefixDb("2", [p2]))
    assert updatePrefixDatabase(ps, createPrefixDb("3", [p3]))
    assert len(solver.getBestRoutesCache()) == 0
    routes = solver.buildRouteDb("1", als, ps).unicastRoutes()
    assert len(routes) == 1
    assert routes[addr1]["nexthops"] == {createNextHopFromAdj(adj12, False, 10),
                                         createNextHopFromAdj(adj13, False, 10)}
    best = solver.getBestRoutesCache()[addr1]
    assert sorted(best["allNodeAreas"]) == [("2", kTestingAreaName), ("3", kTestingAreaName)]
    assert best["bestNodeArea"][0] == "2"
    p2b = createPrefixEntryWithMetrics(addr1, DEFAULT, createMetrics(200, 100, 0))
    assert updatePrefixDatabase(ps, createPrefixDb("2", [p2b]))
    routes = solver.buildRouteDb("1", als, ps).unicastRoutes()
    assert routes[addr1]["nexthops"] == {createNextHopFromAdj(adj12, False, 10)}
    best = solver.getBestRoutesCache()[addr1]
    assert list(best["allNodeAreas"]) == [("2", kTestingAreaName)]
    assert best["bestNodeArea"][0] == "2"


def kat_connectivity(M):
    """SpfSolverTest.cpp:1180-1238 ConnectivityTest.GraphConnectedOrPartitioned."""
    for partitioned in (False, True):
        adjacencyDb1 = createAdjDb("1", [] if partitioned else [adj12], 1)
        adjacencyDb2 = createAdjDb("2", [adj21, adj23], 2)
        adjacencyDb3 = createAdjDb("3", [] if partitioned else [adj32], 3)
        als, ls, ps = _setup(M, "1")
        solver = M.SpfSolver("1", False, True)
        assert _chg(ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)) == _change(False, False, True)
        assert _chg(ls.updateAdjacencyDatabase(adjacencyDb2, kTestingAreaName)) == _change(not partitioned, False, True)
        assert _chg(ls.updateAdjacencyDatabase(adjacencyDb3, kTestingAreaName)) == _change(not partitioned, False, True)
        for p in (prefixDb1, prefixDb2, prefixDb3):
            assert updatePrefixDatabase(ps, p)
        db = solver.buildRouteDb("1", als, ps)
        foundV6 = db is not None and addr3 in db.unicastRoutes()
        foundLabel = db is not None and 3 in db.mplsRoutes()
        assert partitioned == (not foundV6)
        assert partitioned == (not foundLabel)


def kat_node_hard_drain(M):
    """SpfSolverTest.cpp:1246-1330 ConnectivityTest.NodeHardDrainTest."""
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True)
    adjacencyDb1 = createAdjDb("1", [adj12], 1)
    adjacencyDb2 = createAdjDb("2", [adj21, adj23], 2, overLoadBit=True)
    adjacencyDb3 = createAdjDb("3", [adj32], 3)
    for p in (prefixDb1, prefixDb2, prefixDb3):
        assert updatePrefixDatabase(ps, p)
    assert not ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(adjacencyDb2, kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(adjacencyDb3, kTestingAreaName)["topologyChanged"]
    rm = getRouteMap(solver, ["1", "2", "3"], als, ps)
    assert len(rm) == 11
    assert rm[("1", addr2)] == {createNextHopFromAdj(adj12, False, 10)}
    assert rm[("1", "2")] == {createNextHopFromAdj(adj12, False, 10, labelPhpAction)}
    assert rm[("1", "1")] == {labelPopNextHop}
    assert rm[("2", addr3)] == {createNextHopFromAdj(adj23, False, 10)}
    assert rm[("2", addr1)] == {createNextHopFromAdj(adj21, False, 10)}
    assert rm[("2", "1")] == {createNextHopFromAdj(adj21, False, 10, labelPhpAction)}
    assert rm[("2", "3")] == {createNextHopFromAdj(adj23, False, 10, labelPhpAction)}
    assert rm[("2", "2")] == {labelPopNextHop}
    assert rm[("3", addr2)] == {createNextHopFromAdj(adj32, False, 10)}
    assert rm[("3", "2")] == {createNextHopFromAdj(adj32, False, 10, labelPhpAction)}
    assert rm[("3", "3")] == {labelPopNextHop}


def kat_interface_soft_drain(M):
    """SpfSolverTest.cpp:1346-1491 ConnectivityTest.InterfaceSoftDrainTest."""
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True)
    adjacencyDb1 = createAdjDb("1", [adj12_1], 1)
    adjacencyDb2 = createAdjDb("2", [adj21, adj23], 2)
    adjacencyDb3 = createAdjDb("3", [adj32, adj31_old], 3)
    for p in (prefixDb1, prefixDb2, prefixDb3):
        assert updatePrefixDatabase(ps, p)
    assert not ls.updateAdjacencyDatabase(adjacencyDb2, kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(adjacencyDb3, kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(adjacencyDb1, kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(createAdjDb("1", [adj12_1, adj13], 1), kTestingAreaName)["topologyChanged"]
    assert ls.updateAdjacencyDatabase(createAdjDb("1", [adj12_2, adj13], 1), kTestingAreaName)["topologyChanged"]
    rm = getRouteMap(solver, ["1", "2", "3"], als, ps)
    assert len(rm) == 15
    assert rm[("1", addr2)] == {createNextHopFromAdj(adj12_2, False, 20),
                                createNextHopFromAdj(adj13, False, 20)}
    assert rm[("1", addr3)] == {createNextHopFromAdj(adj13, False, 10)}
    assert rm[("1", "2")] == {createNextHopFromAdj(adj12_2, False, 20, labelPhpAction),
                              createNextHopFromAdj(adj13, False, 20, labelSwapAction(2))}
    assert rm[("1", "3")] == {createNextHopFromAdj(adj13, False, 10, labelPhpAction)}
    assert rm[("1", "1")] == {labelPopNextHop}
    assert rm[("2", addr3)] == {createNextHopFromAdj(adj23, False, 10)}
    assert rm[("2", addr1)] == {createNextHopFromAdj(adj21, False, 20),
                                createNextHopFromAdj(adj23, False, 20)}
    assert rm[("2", "1")] == {createNextHopFromAdj(adj21, False, 20, labelPhpAction),
                              createNextHopFromAdj(adj23, False, 20, labelSwapAction(1))}
    assert rm[("2", "3")] == {createNextHopFromAdj(adj23, False, 10, labelPhpAction)}
    assert rm[("3", addr2)] == {createNextHopFromAdj(adj32, False, 10)}
    assert rm[("3", addr1)] == {createNextHopFromAdj(adj31, False, 10)}
    assert rm[("3", "1")] == {createNextHopFromAdj(adj31, False, 10, labelPhpAction)}
    assert rm[("3", "2")] == {createNextHopFromAdj(adj32, False, 10, labelPhpAction)}
    assert rm[("3", "3")] == {labelPopNextHop}
    assert ls.updateAdjacencyDatabase(createAdjDb("1", [adj12_2], 0), kTestingAreaName)["topologyChanged"]
    assert not ls.updateAdjacencyDatabase(createAdjDb("3", [adj32], 0), kTestingAreaName)["topologyChanged"]
    assert not ls.updateAdjacencyDatabase(createAdjDb("1", [adj12_2, adj13], 0), kTestingAreaName)["topologyChanged"]


def kat_simple_ring(M):
    """SpfSolverTest.cpp:1572-1765 SimpleRingTopologyFixture.ShortestPathTest
    (v4 and v6 instances)."""
    for v4 in (True, False):
        als, ls, ps = _setup(M, "1")
        solver = M.SpfSolver("1", v4, True)
        dbs = [createAdjDb("1", [adj12, adj13], 1), createAdjDb("2", [adj21, adj24], 2),
               createAdjDb("3", [adj31, adj34], 3), createAdjDb("4", [adj42, adj43], 4)]
        assert _chg(ls.updateAdjacencyDatabase(dbs[0], kTestingAreaName)) == _change(False, False, True)
        for db in dbs[1:]:
            assert _chg(ls.updateAdjacencyDatabase(db, kTestingAreaName)) == _change(True, False, True)
        for p in ((prefixDb1V4, prefixDb2V4, prefixDb3V4, prefixDb4V4) if v4
                  else (prefixDb1, prefixDb2, prefixDb3, prefixDb4)):
            updatePrefixDatabase(ps, p)
        a1, a2, a3, a4 = (addr1V4, addr2V4, addr3V4, addr4V4) if v4 else (addr1, addr2, addr3, addr4)
        rm = getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
        assert len(rm) == 28
        nh = createNextHopFromAdj
        assert rm[("1", a4)] == {nh(adj12, v4, 20), nh(adj13, v4, 20)}
        assert rm[("1", "4")] == {nh(adj12, False, 20, labelSwapAction(4)), nh(adj13, False, 20, labelSwapAction(4))}
        assert rm[("1", a3)] == {nh(adj13, v4, 10)}
        assert rm[("1", "3")] == {nh(adj13, False, 10, labelPhpAction)}
        assert rm[("1", a2)] == {nh(adj12, v4, 10)}
        assert rm[("1", "2")] == {nh(adj12, False, 10, labelPhpAction)}
        assert rm[("1", "1")] == {labelPopNextHop}
        assert rm[("2", a4)] == {nh(adj24, v4, 10)}
        assert rm[("2", a3)] == {nh(adj21, v4, 20), nh(adj24, v4, 20)}
        assert rm[("2", "3")] == {nh(adj21, False, 20, labelSwapAction(3)), nh(adj24, False, 20, labelSwapAction(3))}
        assert rm[("2", a1)] == {nh(adj21, v4, 10)}
        assert rm[("3", a4)] == {nh(adj34, v4, 10)}
        assert rm[("3", a2)] == {nh(adj31, v4, 20), nh(adj34, v4, 20)}
        assert rm[("3", a1)] == {nh(adj31, v4, 10)}
        assert rm[("4", a3)] == {nh(adj43, v4, 10)}
        assert rm[("4", a2)] == {nh(adj42, v4, 10)}
        assert rm[("4", a1)] == {nh(adj42, v4, 20), nh(adj43, v4, 20)}
        assert rm[("4", "1")] == {nh(adj42, False, 20, labelSwapAction(1)), nh(adj43, False, 20, labelSwapAction(1))}
        assert rm[("4", "4")] == {labelPopNextHop}


def kat_parallel_adj_ring(M):
    """SpfSolverTest.cpp:2332-2530 ParallelAdjRingTopologyFixture.ShortestPathTest."""
    A = createAdjacency
    adj12_1 = A("2", "2/1", "1/1", "fe80::2:1", "192.168.2.1", 11, 201)
    adj12_2 = A("2", "2/2", "1/2", "fe80::2:2", "192.168.2.2", 11, 202)
    adj12_3 = A("2", "2/3", "1/3", "fe80::2:3", "192.168.2.3", 20, 203)
    adj13_1 = A("3", "3/1", "1/1", "fe80::3:1", "192.168.3.1", 11, 301)
    adj21_1 = A("1", "1/1", "2/1", "fe80::1:1", "192.168.1.1", 11, 101)
    adj21_2 = A("1", "1/2", "2/2", "fe80::1:2", "192.168.1.2", 11, 102)
    adj21_3 = A("1", "1/3", "2/3", "fe80::1:3", "192.168.1.3", 20, 103)
    adj24_1 = A("4", "4/1", "2/1", "fe80::4:1", "192.168.4.1", 11, 401)
    adj31_1 = A("1", "1/1", "3/1", "fe80::1:1", "192.168.1.1", 11, 101)
    adj34_1 = A("4", "4/1", "3/1", "fe80::4:1", "192.168.4.1", 11, 401)
    adj34_2 = A("4", "4/2", "3/2", "fe80::4:2", "192.168.4.2", 20, 402)
    adj34_3 = A("4", "4/3", "3/3", "fe80::4:3", "192.168.4.3", 20, 403)
    adj42_1 = A("2", "2/1", "4/1", "fe80::2:1", "192.168.2.1", 11, 201)
    adj43_1 = A("3", "3/1", "4/1", "fe80::3:1", "192.168.3.1", 11, 301)
    adj43_2 = A("3", "3/2", "4/2", "fe80::3:2", "192.168.3.2", 20, 302)
    adj43_3 = A("3", "3/3", "4/3", "fe80::3:3", "192.168.3.3", 20, 303)
    als, ls, ps = _setup(M, "1")
    solver = M.SpfSolver("1", False, True)
    dbs = [createAdjDb("1", [adj12_1, adj12_2, adj12_3, adj13_1], 1),
           createAdjDb("2", [adj21_1, adj21_2, adj21_3, adj24_1], 2),
           createAdjDb("3", [adj31_1, adj34_1, adj34_2, adj34_3], 3),
           createAdjDb("4", [adj42_1, adj43_1, adj43_2, adj43_3], 4)]
    assert not ls.updateAdjacencyDatabase(dbs[0], kTestingAreaName)["topologyChanged"]
    for db in dbs[1:]:
        assert ls.updateAdjacencyDatabase(db, kTestingAreaName)["topologyChanged"]
    for p in (prefixDb1, prefixDb2, prefixDb3, prefixDb4):
        updatePrefixDatabase(ps, p)
    rm = getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
    assert len(rm) == 28
    nh = createNextHopFromAdj
    assert rm[("1", addr4)] == {nh(adj12_2, False, 22), nh(adj13_1, False, 22), nh(adj12_1, False, 22)}
    assert rm[("1", "4")] == {nh(adj12_2, False, 22, labelSwapAction(4)),
                              nh(adj13_1, False, 22, labelSwapAction(4)),
                              nh(adj12_1, False, 22, labelSwapAction(4))}
    assert rm[("1", addr3)] == {nh(adj13_1, False, 11)}
    assert rm[("1", "3")] == {nh(adj13_1, False, 11, labelPhpAction)}
    assert rm[("1", addr2)] == {nh(adj12_2, False, 11), nh(adj12_1, False, 11)}
    assert rm[("1", "2")] == {nh(adj12_2, False, 11, labelPhpAction), nh(adj12_1, False, 11, labelPhpAction)}
    assert rm[("1", "1")] == {labelPopNextHop}
    assert rm[("2", addr4)] == {nh(adj24_1, False, 11)}
    assert rm[("2", addr3)] == {nh(adj21_2, False, 22), nh(adj21_1, False, 22), nh(adj24_1, False, 22)}
    assert rm[("2", "3")] == {nh(adj21_2, False, 22, labelSwapAction(3)),
                              nh(adj21_1, False, 22, labelSwapAction(3)),
                              nh(adj24_1, False, 22, labelSwapAction(3))}
    assert rm[("2", addr1)] == {nh(adj21_2, False, 11), nh(adj21_1, False, 11)}
    assert rm[("3", addr4)] == {nh(adj34_1, False, 11)}
    assert rm[("3", addr2)] == {nh(adj31_1, False, 22), nh(adj34_1, False, 22)}


def kat_grid(M, sizes=(2, 4, 6, 8)):
    """SpfSolverTest.cpp:2700-2855 GridTopologyFixture.ShortestPathTest:
    2n^4 - n^2 routes, every next-hop metric equals the Manhattan distance."""
    for n in sizes:
        als = M.AreaLinkStates()
        ls = als.add(kTestingAreaName, kTestingNodeName)
        ps = M.PrefixState()
        for i in range(n):
            for j in range(n):
                node = i * n + j
                adjs = []

                def add(ii, jj, ifn, oifn):
                    if 0 <= ii < n and 0 <= jj < n:
                        nb = ii * n + jj
                        a = createAdjacency(str(nb), ifn, oifn, f"fe80::{nb}",
                                            f"192.168.{nb // 256}.{nb % 256}", 1, 100001 + nb)
                        a["rtt"], a["timestamp"] = 100, 10000
                        adjs.append(a)
                add(i, j + 1, "0/1", "0/3")
                add(i - 1, j, "0/2", "0/4")
                add(i, j - 1, "0/3", "0/1")
                add(i + 1, j, "0/4", "0/2")
                ls.updateAdjacencyDatabase(createAdjDb(str(node), adjs, node + 1), kTestingAreaName)
                updatePrefixDatabase(ps, createPrefixDb(str(node), [createPrefixEntry(
                    f"::ffff:10.1.{node // 256}.{node % 256}/128")]))
        solver = M.SpfSolver("1", False, True, False)
        nodes = [str(i) for i in range(n * n)]
        rm = getRouteMap(solver, nodes, als, ps)
        assert len(rm) == 2 * n ** 4 - n ** 2
        for (src, key), nhs in rm.items():
            if "/" not in key:
                continue
            dst = int(key.split(".")[-1].split("/")[0]) + 256 * int(key.split(".")[-2])
            s = int(src)
            dist = abs(s % n - dst % n) + abs(s // n - dst // n)
            assert {x[4] for x in nhs} == {dist}


def kat_rib_policy(M):
    """RibPolicyTest.cpp:75-122 RibPolicyStatement.ApplyAction and the
    applyPolicy precedence (neighbor > area > default, weight 0 drops,
    all-dropped keeps the route; RibPolicy.cpp:109-161,231-249)."""
    pol = M.RibPolicy([dict(name="s", prefixes=["fc00::/64"],
                            set_weight=dict(default_weight=1,
                                            area_to_weight={"area1": 0, "area2": 2}),
                            counterID="COUNTER_0")], 3600)
    nhDefault = createNextHop("fe80::1", "iface-default", 0)
    nh1 = createNextHop("fe80::1", "iface1", 0, None, "area1")
    nh2 = createNextHop("fe80::1", "iface2", 0, None, "area2")
    base = dict(prefix="fd00::/64", nexthops=frozenset({nhDefault, nh1, nh2}),
                bestPrefixEntry=createPrefixEntry("fd00::/64"))
    ok, r = pol.applyAction(dict(base))
    assert not ok and r["nexthops"] == base["nexthops"] and r["counterID"] is None
    ok, r = pol.applyAction(dict(base, prefix="fc00::/64"))
    assert ok and r["counterID"] == "COUNTER_0"
    assert r["nexthops"] == {createNextHop("fe80::1", "iface-default", 0, weight=1),
                             createNextHop("fe80::1", "iface2", 0, None, "area2", weight=2)}
    # neighbor weight wins over area weight
    pol2 = M.RibPolicy([dict(name="t", tags=["T"],
                             set_weight=dict(default_weight=1, area_to_weight={"a": 3},
                                             neighbor_to_weight={"n1": 7, "n2": 0}))], 3600)
    e = createPrefixEntry("fc01::/64")
    e["tags"] = ["T"]
    r0 = dict(prefix="fc01::/64", bestPrefixEntry=e, nexthops=frozenset({
        createNextHop("fe80::a", "i1", 5, None, "a", "n1"),
        createNextHop("fe80::b", "i2", 5, None, "a", "n2"),
        createNextHop("fe80::c", "i3", 5, None, "a", "n3")}))
    ok, r = pol2.applyAction(r0)
    assert ok and {(x[1], x[2]) for x in r["nexthops"]} == {("i1", 7), ("i3", 3)}
    # every next-hop dropped -> route untouched
    pol3 = M.RibPolicy([dict(name="z", tags=["T"], set_weight=dict(default_weight=0))], 3600)
    ok, r = pol3.applyAction(r0)
    assert not ok and r["nexthops"] == r0["nexthops"]


ALL_KATS = [
    kat_linkstate_basic, kat_linkstate_link_usable, kat_linkstate_kth_paths,
    kat_unreachable_nodes, kat_drained_node_least_preferred,
    kat_missing_and_empty_neighbor_db, kat_unknown_node,
    kat_node_soft_drained_choice, kat_node_overload_route_choice,
    kat_adjacency_update, kat_mpls_basic, kat_bgp_igp_metric, kat_igp_cost,
    kat_best_route_selection, kat_connectivity, kat_node_hard_drain,
    kat_interface_soft_drain, kat_simple_ring, kat_parallel_adj_ring, kat_grid,
    kat_rib_policy,
]

# multi-area known-answer tests (tests/kat_multiarea.py)
from kat_multiarea import MULTI_AREA_KATS  # noqa: E402
ALL_KATS += MULTI_AREA_KATS

# further cases (tests/kat_more.py)
from kat_more import MORE_KATS  # noqa: E402
ALL_KATS += MORE_KATS
