"""More known-answer tests transcribed from the reference's unit tests
(SURVEY.md §8(c)): the SimpleRing / ParallelAdjRing fixture cases beyond
ShortestPathTest, grid sizes 10..16, RibPolicyTest's Match / ApplyAction /
ApplyPolicy, and the compute-side assertions of DecisionTest's ParallelLinks,
SelfReditributePrefixPublication and RibPolicy. Each case takes the
implementation module `M` (oracle/_refcpu or openr_amd._decision); file:line
citations are under /root/reference (not read at run time)."""
import time

import lsdb as L
import thrift_compact as tc
from lsdb import (adj12, adj13, adj21, adj24, adj31, adj34, adj42, adj43, addr1, addr2,
                  addr3, addr4, addr1V4, addr2V4, addr3V4, addr4V4, createAdjacency,
                  createAdjDb, createNextHop, createNextHopFromAdj, createPrefixDb,
                  createPrefixEntry, getRouteMap, kTestingAreaName, labelPhpAction,
                  labelPopNextHop, labelSwapAction, updatePrefixDatabase)

nh = createNextHopFromAdj


def _ring(M, v4):
    """SimpleRingTopologyFixture::CustomSetUp(true) (SpfSolverTest.cpp:1579-1619):
    ring 1-2-4-3-1, metric 10, node labels 1..4, one prefix per node."""
    als = M.AreaLinkStates()
    ls = als.add(kTestingAreaName, "1")
    ps = M.PrefixState()
    solver = M.SpfSolver("1", v4, True)
    dbs = {"1": createAdjDb("1", [adj12, adj13], 1), "2": createAdjDb("2", [adj21, adj24], 2),
           "3": createAdjDb("3", [adj31, adj34], 3), "4": createAdjDb("4", [adj42, adj43], 4)}
    for db in dbs.values():
        ls.updateAdjacencyDatabase(db, kTestingAreaName)
    for p in ((L.prefixDb1V4, L.prefixDb2V4, L.prefixDb3V4, L.prefixDb4V4) if v4
              else (L.prefixDb1, L.prefixDb2, L.prefixDb3, L.prefixDb4)):
        updatePrefixDatabase(ps, p)
    addrs = (addr1V4, addr2V4, addr3V4, addr4V4) if v4 else (addr1, addr2, addr3, addr4)
    return als, ls, ps, solver, dbs, dict(zip("1234", addrs))


def _pop(rm, node, label):
    """validatePopLabelRoute (SpfSolverTest.cpp:109-118)."""
    assert rm[(node, str(label))] == {labelPopNextHop}


def kat_ring_duplicate_mpls_routes(M):
    """SpfSolverTest.cpp:1790-1838 SimpleRingTopologyFixture.DuplicateMplsRoutes:
    two nodes announce label 2 -> one route for it at every node, no
    withdrawal; relabel node 1 -> label 2's route updated, never deleted
    (verifyRouteInUpdateNoDelete, :1625-1634). The fb303 duplicate counter is
    not part of the route path."""
    for v4 in (True, False):
        als, ls, ps, solver, dbs, _ = _ring(M, v4)
        dbs["1"]["nodeLabel"] = 2
        ls.updateAdjacencyDatabase(dbs["1"], kTestingAreaName)
        comp = {}
        for n in ("1", "2", "3"):
            db = solver.buildRouteDb(n, als, ps)
            d = M.DecisionRouteDb().calculateUpdate(db)
            assert 2 in d["mplsRoutesToUpdate"] and not d["mplsRoutesToDelete"]
            comp[n] = db
        dbs["1"]["nodeLabel"] = 1
        ls.updateAdjacencyDatabase(dbs["1"], kTestingAreaName)
        for n in ("1", "2", "3"):
            d = comp[n].calculateUpdate(solver.buildRouteDb(n, als, ps))
            assert 2 in d["mplsRoutesToUpdate"] and not d["mplsRoutesToDelete"]


def kat_ring_multipath(M):
    """SpfSolverTest.cpp:1843-1968 SimpleRingTopologyFixture.MultiPathTest."""
    for v4 in (True, False):
        als, ls, ps, solver, dbs, a = _ring(M, v4)
        rm = getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
        assert len(rm) == 28
        exp = {
            ("1", a["4"]): {nh(adj12, v4, 20), nh(adj13, v4, 20)},
            ("1", "4"): {nh(adj12, False, 20, labelSwapAction(4)),
                         nh(adj13, False, 20, labelSwapAction(4))},
            ("1", a["3"]): {nh(adj13, v4, 10)},
            ("1", "3"): {nh(adj13, False, 10, labelPhpAction)},
            ("1", a["2"]): {nh(adj12, v4, 10)},
            ("1", "2"): {nh(adj12, False, 10, labelPhpAction)},
            ("2", a["4"]): {nh(adj24, v4, 10)},
            ("2", "4"): {nh(adj24, False, 10, labelPhpAction)},
            ("2", a["3"]): {nh(adj21, v4, 20), nh(adj24, v4, 20)},
            ("2", "3"): {nh(adj21, False, 20, labelSwapAction(3)),
                         nh(adj24, False, 20, labelSwapAction(3))},
            ("2", a["1"]): {nh(adj21, v4, 10)},
            ("2", "1"): {nh(adj21, False, 10, labelPhpAction)},
            ("3", a["4"]): {nh(adj34, v4, 10)},
            ("3", "4"): {nh(adj34, False, 10, labelPhpAction)},
            ("3", a["2"]): {nh(adj31, v4, 20), nh(adj34, v4, 20)},
            ("3", "2"): {nh(adj31, False, 20, labelSwapAction(2)),
                         nh(adj34, False, 20, labelSwapAction(2))},
            ("3", a["1"]): {nh(adj31, v4, 10)},
            ("3", "1"): {nh(adj31, False, 10, labelPhpAction)},
            ("4", a["3"]): {nh(adj43, v4, 10)},
            ("4", "3"): {nh(adj43, False, 10, labelPhpAction)},
            ("4", a["2"]): {nh(adj42, v4, 10)},
            ("4", "2"): {nh(adj42, False, 10, labelPhpAction)},
            ("4", a["1"]): {nh(adj42, v4, 20), nh(adj43, v4, 20)},
            ("4", "1"): {nh(adj42, False, 20, labelSwapAction(1)),
                         nh(adj43, False, 20, labelSwapAction(1))},
        }
        for k, v in exp.items():
            assert rm[k] == v, k
        for n in "1234":
            _pop(rm, n, int(n))


def kat_ring_attached_nodes(M):
    """SpfSolverTest.cpp:1973-2019 SimpleRingTopologyFixture.AttachedNodesTest:
    default routes from nodes 1 and 4; 2 and 3 reach both, 1 and 4 (self
    selected) install none."""
    for v4 in (True, False):
        als, ls, ps, solver, dbs, a = _ring(M, v4)
        default = "0.0.0.0/0" if v4 else "::/0"
        assert updatePrefixDatabase(ps, createPrefixDb("1", [createPrefixEntry(addr1),
                                                             createPrefixEntry(default)]))
        assert updatePrefixDatabase(ps, createPrefixDb("4", [createPrefixEntry(addr4),
                                                             createPrefixEntry(default)]))
        rm = getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
        assert len(rm) == 30
        assert ("1", default) not in rm and ("4", default) not in rm
        assert rm[("2", default)] == {nh(adj21, v4, 10), nh(adj24, v4, 10)}
        assert rm[("3", default)] == {nh(adj31, v4, 10), nh(adj34, v4, 10)}


def kat_ring_overload_node(M):
    """SpfSolverTest.cpp:2025-2135 SimpleRingTopologyFixture.OverloadNodeTest:
    nodes 2 and 3 hard-drained -> 1 and 4 cannot transit to each other."""
    for v4 in (True, False):
        als, ls, ps, solver, dbs, a = _ring(M, v4)
        for n in ("2", "3"):
            dbs[n]["isOverloaded"] = True
            assert ls.updateAdjacencyDatabase(dbs[n], kTestingAreaName)["topologyChanged"]
        rm = getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
        assert len(rm) == 24
        exp = {
            ("1", a["3"]): {nh(adj13, v4, 10)},
            ("1", "3"): {nh(adj13, False, 10, labelPhpAction)},
            ("1", a["2"]): {nh(adj12, v4, 10)},
            ("1", "2"): {nh(adj12, False, 10, labelPhpAction)},
            ("2", a["4"]): {nh(adj24, v4, 10)},
            ("2", "4"): {nh(adj24, False, 10, labelPhpAction)},
            ("2", a["3"]): {nh(adj21, v4, 20), nh(adj24, v4, 20)},
            ("2", "3"): {nh(adj21, False, 20, labelSwapAction(3)),
                         nh(adj24, False, 20, labelSwapAction(3))},
            ("2", a["1"]): {nh(adj21, v4, 10)},
            ("2", "1"): {nh(adj21, False, 10, labelPhpAction)},
            ("3", a["4"]): {nh(adj34, v4, 10)},
            ("3", "4"): {nh(adj34, False, 10, labelPhpAction)},
            ("3", a["2"]): {nh(adj31, v4, 20), nh(adj34, v4, 20)},
            ("3", "2"): {nh(adj31, False, 20, labelSwapAction(2)),
                         nh(adj34, False, 20, labelSwapAction(2))},
            ("3", a["1"]): {nh(adj31, v4, 10)},
            ("3", "1"): {nh(adj31, False, 10, labelPhpAction)},
            ("4", a["3"]): {nh(adj43, v4, 10)},
            ("4", "3"): {nh(adj43, False, 10, labelPhpAction)},
            ("4", a["2"]): {nh(adj42, v4, 10)},
            ("4", "2"): {nh(adj42, False, 10, labelPhpAction)},
        }
        for k, v in exp.items():
            assert rm[k] == v, k
        for n in "1234":
            _pop(rm, n, int(n))


def kat_ring_overload_link(M):
    """SpfSolverTest.cpp:2141-2330 SimpleRingTopologyFixture.OverloadLinkTest:
    adj31 overloaded (3 reachable only via 4), then adj34 too (3 cut off)."""
    for v4 in (True, False):
        als, ls, ps, solver, dbs, a = _ring(M, v4)
        dbs["3"]["adjacencies"][0]["isOverloaded"] = True
        assert ls.updateAdjacencyDatabase(dbs["3"], kTestingAreaName)["topologyChanged"]
        rm = getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
        assert len(rm) == 28
        exp = {
            ("1", a["4"]): {nh(adj12, v4, 20)},
            ("1", "4"): {nh(adj12, False, 20, labelSwapAction(4))},
            ("1", a["3"]): {nh(adj12, v4, 30)},
            ("1", "3"): {nh(adj12, False, 30, labelSwapAction(3))},
            ("1", a["2"]): {nh(adj12, v4, 10)},
            ("1", "2"): {nh(adj12, False, 10, labelPhpAction)},
            ("2", a["4"]): {nh(adj24, v4, 10)},
            ("2", "4"): {nh(adj24, False, 10, labelPhpAction)},
            ("2", a["3"]): {nh(adj24, v4, 20)},
            ("2", "3"): {nh(adj24, False, 20, labelSwapAction(3))},
            ("2", a["1"]): {nh(adj21, v4, 10)},
            ("2", "1"): {nh(adj21, False, 10, labelPhpAction)},
            ("3", a["4"]): {nh(adj34, v4, 10)},
            ("3", "4"): {nh(adj34, False, 10, labelPhpAction)},
            ("3", a["2"]): {nh(adj34, v4, 20)},
            ("3", "2"): {nh(adj34, False, 20, labelSwapAction(2))},
            ("3", a["1"]): {nh(adj34, v4, 30)},
            ("3", "1"): {nh(adj34, False, 30, labelSwapAction(1))},
            ("4", a["3"]): {nh(adj43, v4, 10)},
            ("4", "3"): {nh(adj43, False, 10, labelPhpAction)},
            ("4", a["2"]): {nh(adj42, v4, 10)},
            ("4", "2"): {nh(adj42, False, 10, labelPhpAction)},
            ("4", a["1"]): {nh(adj42, v4, 20)},
            ("4", "1"): {nh(adj42, False, 20, labelSwapAction(1))},
        }
        for k, v in exp.items():
            assert rm[k] == v, k
        for n in "1234":
            _pop(rm, n, int(n))
        dbs["3"]["adjacencies"][1]["isOverloaded"] = True
        assert ls.updateAdjacencyDatabase(dbs["3"], kTestingAreaName)["topologyChanged"]
        rm = getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
        assert len(rm) == 16
        exp = {
            ("1", a["4"]): {nh(adj12, v4, 20)},
            ("1", "4"): {nh(adj12, False, 20, labelSwapAction(4))},
            ("1", a["2"]): {nh(adj12, v4, 10)},
            ("1", "2"): {nh(adj12, False, 10, labelPhpAction)},
            ("2", a["4"]): {nh(adj24, v4, 10)},
            ("2", "4"): {nh(adj24, False, 10, labelPhpAction)},
            ("2", a["1"]): {nh(adj21, v4, 10)},
            ("2", "1"): {nh(adj21, False, 10, labelPhpAction)},
            ("4", a["2"]): {nh(adj42, v4, 10)},
            ("4", "2"): {nh(adj42, False, 10, labelPhpAction)},
            ("4", a["1"]): {nh(adj42, v4, 20)},
            ("4", "1"): {nh(adj42, False, 20, labelSwapAction(1))},
        }
        for k, v in exp.items():
            assert rm[k] == v, k
        for n in "1234":
            _pop(rm, n, int(n))


def kat_parallel_adj_ring_multipath(M):
    """SpfSolverTest.cpp:2558-2695 ParallelAdjRingTopologyFixture.MultiPathTest
    (fixture :2332-2427): parallel 1-2 links of metric 11, 11, 20 etc."""
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
    als = M.AreaLinkStates()
    ls = als.add(kTestingAreaName, "1")
    ps = M.PrefixState()
    solver = M.SpfSolver("1", False, True)
    for db in (createAdjDb("1", [adj12_1, adj12_2, adj12_3, adj13_1], 1),
               createAdjDb("2", [adj21_1, adj21_2, adj21_3, adj24_1], 2),
               createAdjDb("3", [adj31_1, adj34_1, adj34_2, adj34_3], 3),
               createAdjDb("4", [adj42_1, adj43_1, adj43_2, adj43_3], 4)):
        ls.updateAdjacencyDatabase(db, kTestingAreaName)
    for p in (L.prefixDb1, L.prefixDb2, L.prefixDb3, L.prefixDb4):
        updatePrefixDatabase(ps, p)
    rm = getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
    assert len(rm) == 28
    sw = labelSwapAction
    exp = {
        ("1", addr4): {nh(adj12_1, False, 22), nh(adj12_2, False, 22), nh(adj13_1, False, 22)},
        ("1", "4"): {nh(adj12_1, False, 22, sw(4)), nh(adj12_2, False, 22, sw(4)),
                     nh(adj13_1, False, 22, sw(4))},
        ("1", addr3): {nh(adj13_1, False, 11)},
        ("1", "3"): {nh(adj13_1, False, 11, labelPhpAction)},
        ("1", addr2): {nh(adj12_1, False, 11), nh(adj12_2, False, 11)},
        ("1", "2"): {nh(adj12_1, False, 11, labelPhpAction), nh(adj12_2, False, 11, labelPhpAction)},
        ("2", addr4): {nh(adj24_1, False, 11)},
        ("2", "4"): {nh(adj24_1, False, 11, labelPhpAction)},
        ("2", addr3): {nh(adj21_1, False, 22), nh(adj21_2, False, 22), nh(adj24_1, False, 22)},
        ("2", "3"): {nh(adj21_1, False, 22, sw(3)), nh(adj21_2, False, 22, sw(3)),
                     nh(adj24_1, False, 22, sw(3))},
        ("2", addr1): {nh(adj21_1, False, 11), nh(adj21_2, False, 11)},
        ("2", "1"): {nh(adj21_1, False, 11, labelPhpAction), nh(adj21_2, False, 11, labelPhpAction)},
        ("3", addr4): {nh(adj34_1, False, 11)},
        ("3", "4"): {nh(adj34_1, False, 11, labelPhpAction)},
        ("3", addr2): {nh(adj31_1, False, 22), nh(adj34_1, False, 22)},
        ("3", "2"): {nh(adj31_1, False, 22, sw(2)), nh(adj34_1, False, 22, sw(2))},
        ("3", addr1): {nh(adj31_1, False, 11)},
        ("3", "1"): {nh(adj31_1, False, 11, labelPhpAction)},
        ("4", addr3): {nh(adj43_1, False, 11)},
        ("4", "3"): {nh(adj43_1, False, 11, labelPhpAction)},
        ("4", addr2): {nh(adj42_1, False, 11)},
        ("4", "2"): {nh(adj42_1, False, 11, labelPhpAction)},
        ("4", addr1): {nh(adj42_1, False, 22), nh(adj43_1, False, 22)},
        ("4", "1"): {nh(adj42_1, False, 22, sw(1)), nh(adj43_1, False, 22, sw(1))},
    }
    for k, v in exp.items():
        assert rm[k] == v, k
    for n in "1234":
        _pop(rm, n, int(n))


def kat_grid_large(M):
    """SpfSolverTest.cpp:2798-2799: GridTopologyFixture instantiated for
    n = 2..16 step 2; this covers 10, 12, 14, 16 (kat_cases.kat_grid the rest)."""
    from kat_cases import kat_grid
    kat_grid(M, sizes=(10, 12, 14, 16))


# ---------------------------------------------------------------- RibPolicy
def _stmt(prefixes=None, tags=None, default=1, area=None, nbr=None, counter=None):
    """createPolicyStatement (RibPolicyTest.cpp:23-52)."""
    d = dict(name="stmt", set_weight=dict(default_weight=default, area_to_weight=area or {},
                                          neighbor_to_weight=nbr or {}))
    if prefixes is not None:
        d["prefixes"] = prefixes
    if tags is not None:
        d["tags"] = tags
    if counter is not None:
        d["counterID"] = counter
    return d


def _entry(prefix, tags=(), nexthops=()):
    e = createPrefixEntry(prefix)
    e["tags"] = list(tags)
    return dict(prefix=prefix, nexthops=frozenset(nexthops), bestPrefixEntry=e)


def kat_rib_policy_statement_match(M):
    """RibPolicyTest.cpp:124-201 RibPolicyStatement.Match (one statement per
    policy: RibPolicy::match is the any-statement match)."""
    p = M.RibPolicy([_stmt(["10.0.0.0/8"], None, 1, {"test-area": 2})], 3600)
    assert p.match(_entry("10.0.0.0/8", ["COMMODITY:EGRESS"]))
    assert not p.match(_entry("11.0.0.0/8", ["COMMODITY:EGRESS"]))
    p = M.RibPolicy([_stmt(None, ["COMMODITY:EGRESS"], 1, {"test-area": 2})], 3600)
    assert p.match(_entry("11.0.0.0/8", ["COMMODITY:EGRESS"]))
    assert not p.match(_entry("11.0.0.0/8", ["COMMODITY:INGRESS:pod1"]))
    p = M.RibPolicy([_stmt(["10.0.0.0/8"], ["COMMODITY:EGRESS"], 1, {"test-area": 2})], 3600)
    assert p.match(_entry("10.0.0.0/8", ["COMMODITY:EGRESS"]))
    assert not p.match(_entry("11.0.0.0/8", ["COMMODITY:EGRESS"]))
    assert not p.match(_entry("10.0.0.0/8", ["COMMODITY:INGRESS:pod1"]))
    assert not p.match(_entry("11.0.0.0/8", ["COMMODITY:INGRES:pod1"]))
    p = M.RibPolicy([_stmt([], [], 1, {"test-area": 2})], 3600)
    assert not p.match(_entry("10.0.0.0/8", ["COMMODITY:EGRESS"]))


def kat_rib_policy_apply_action(M):
    """RibPolicyTest.cpp:268-329 RibPolicy.ApplyAction: only the first
    matching statement transforms the route."""
    p = M.RibPolicy([_stmt(["fc01::/64"], None, 1, {"area1": 99}),
                     _stmt(["fc00::/64", "fc02::/64"], None, 1, {"area2": 99})], 1)
    nh1 = createNextHop("fe80::1", "iface1", 0, None, "area1")
    nh2 = createNextHop("fe80::1", "iface2", 0, None, "area2")

    def w(n, weight):
        return n[:2] + (weight,) + n[3:]
    ok, r = p.applyAction(_entry("fc01::/64", (), (nh1, nh2)))
    assert ok and r["nexthops"] == {w(nh1, 99), w(nh2, 1)}
    ok, r = p.applyAction(_entry("fc02::/64", (), (nh1, nh2)))
    assert ok and r["nexthops"] == {w(nh1, 1), w(nh2, 99)}
    e = _entry("fc03::/64", (), (nh1, nh2))
    ok, r = p.applyAction(dict(e))
    assert not ok and r["nexthops"] == e["nexthops"] and r["counterID"] is None


def kat_rib_policy_apply_policy(M):
    """RibPolicyTest.cpp:331-394 RibPolicy.ApplyPolicy: neighbor weight over
    area weight; a route whose next hops would all drop keeps them and is
    not reported; an expired policy (ttl 1 s) changes nothing."""
    p = M.RibPolicy([_stmt(["fc01::/64"], None, 1, {"area1": 99}, {"nbr3": 98}),
                     _stmt(["fc00::/64", "fc02::/64"], None, 1, {"area2": 0})], 1)
    nh1 = createNextHop("fe80::1", "iface1", 0, None, "area1", "nbr1")
    nh2 = createNextHop("fe80::1", "iface2", 0, None, "area2", "nbr2")
    nh3 = createNextHop("fe80::1", "iface3", 0, None, "area1", "nbr3")

    def w(n, weight):
        return n[:2] + (weight,) + n[3:]

    # applyPolicy = applyAction over every route, reporting the transformed
    # ones (RibPolicy.cpp:231-249)
    e1 = _entry("fc01::/64", (), (nh1, nh2, nh3))
    e2 = _entry("fc02::/64", (), (nh2,))
    ok1, r1 = p.applyAction(dict(e1))
    ok2, r2 = p.applyAction(dict(e2))
    assert p.isActive()
    assert ok1 and r1["nexthops"] == {w(nh1, 99), w(nh2, 1), w(nh3, 98)}
    assert not ok2 and r2["nexthops"] == e2["nexthops"]
    time.sleep(1.05)  # let the 1 s ttl run out (RibPolicy.cpp:199-208)
    assert not p.isActive()


# -------------------------------------------------------- Decision (LSDB) --
class _Decision:
    """Decision's ingest + rebuild loop over one implementation: KvStore
    publications (compact-thrift values, oracle/thrift_compact.py encoders)
    applied per key (Decision::processPublication / updateKeyInLsdb,
    Decision.cpp:710-846), then a full rebuild (buildRouteDb + RibPolicy,
    Decision.cpp:888-960) diffed against the previous RouteDb
    (calculateUpdate)."""

    def __init__(self, M, me, areas):
        self.M, self.me, self.areas = M, me, set(areas)
        self.als = M.AreaLinkStates()
        self.ps = M.PrefixState()
        self.solver = M.SpfSolver(me, True, False)
        self.db = M.DecisionRouteDb()
        self.policy = None
        self.product = hasattr(M, "LsdbIngest")
        if self.product:
            self.ingest = M.LsdbIngest(me, self.areas)

    def publish(self, area, kv):
        """kv: key -> value dict (adj or prefix database) or None."""
        enc = []
        for k, v in sorted(kv.items()):
            if v is None:
                enc.append((k, None))
            elif k.startswith("adj:"):
                enc.append((k, tc.encode_adj_db(v)))
            else:
                enc.append((k, tc.encode_prefix_db(v)))
        if self.product:
            pend = self.M.DecisionPendingUpdates(self.me)
            self.ingest.processPublicationKeyVals(area, self.als, self.ps, enc, [], pend)
            return pend.getCount()
        if area not in self.als.areas():
            self.als.add(area, self.me)
        pend = tc.PendingUpdates(self.me)
        for k, v in enc:
            pend.apply(*tc.update_key_in_lsdb(self.me, self.areas, area, self.als[area],
                                              self.ps, k, v))
        return pend.count

    def set_policy(self, stmts, ttl):
        self.policy = self.M.RibPolicy(stmts, ttl)
        if self.product:
            self.solver.setRibPolicy(self.policy)

    def rebuild(self):
        db = self.solver.buildRouteDb(self.me, self.als, self.ps)
        if not self.product and self.policy is not None:
            self.policy.applyPolicy(db)
        upd = self.db.calculateUpdate(db)
        self.db = db
        return upd


def _adj_val(node, adjs, label, overloaded=False):
    return createAdjDb(node, adjs, label, overloaded)


def kat_decision_parallel_links(M):
    """DecisionTest.cpp:1780-1874 DecisionTestFixture.ParallelLinks: parallel
    1-2 links of metric 100 / 800; withdraw / restore / overload the cheap one."""
    A = createAdjacency
    a12_1 = A("2", "1/2-1", "2/1-1", "fe80::2", "192.168.0.2", 100, 0)
    a12_2 = A("2", "1/2-2", "2/1-2", "fe80::2", "192.168.0.2", 800, 0)
    a21_1 = A("1", "2/1-1", "1/2-1", "fe80::1", "192.168.0.1", 100, 0)
    a21_2 = A("1", "2/1-2", "1/2-2", "fe80::1", "192.168.0.1", 800, 0)
    d = _Decision(M, "1", [kTestingAreaName])
    d.publish(kTestingAreaName, {
        "adj:1": _adj_val("1", [a12_1, a12_2], 0), "adj:2": _adj_val("2", [a21_1, a21_2], 0),
        f"prefix:1:[{addr1}]": createPrefixDb("1", [createPrefixEntry(addr1)]),
        f"prefix:2:[{addr2}]": createPrefixDb("2", [createPrefixEntry(addr2)])})

    def step(adjs2, want):
        if adjs2 is not None:
            d.publish(kTestingAreaName, {"adj:2": _adj_val("2", adjs2, 0)})
        u = d.rebuild()
        assert len(u["unicastRoutesToUpdate"]) == 1
        assert d.db.unicastRoutes()[addr2]["nexthops"] == {want}
    step(None, nh(a12_1, False, 100))
    step([a21_2], nh(a12_2, False, 800))
    step([a21_1, a21_2], nh(a12_1, False, 100))
    a21_1o = dict(a21_1, isOverloaded=True)
    step([a21_1o, a21_2], nh(a12_2, False, 800))


def kat_decision_self_redistribute(M):
    """DecisionTest.cpp:1213-1276 SelfReditributePrefixPublication: node 1's
    own redistribution of addr2 into area B (area_stack ending in an area
    it knows) is ignored -- no prefix-state change, no route update."""
    B = "B"
    d = _Decision(M, "1", [kTestingAreaName, B])
    origin = createPrefixEntry(addr2)
    origin["area_stack"] = ["65000"]
    d.publish(kTestingAreaName, {
        "adj:1": _adj_val("1", [adj12], 1), "adj:2": _adj_val("2", [adj21], 2),
        f"prefix:2:[{addr2}]": createPrefixDb("2", [origin])})
    d.rebuild()
    d.publish(B, {"adj:1": _adj_val("1", [adj13], 1), "adj:3": _adj_val("3", [adj31], 3)})
    d.rebuild()
    before = {p: sorted(map(tuple, v)) for p, v in d.ps.prefixes().items()}
    redis = createPrefixEntry(addr2, type=L.BGP)
    redis["type"] = 10  # PrefixType.RIB (Network.thrift)
    redis["area_stack"] = ["65000", kTestingAreaName]
    n = d.publish(B, {f"prefix:1:[{addr2}]": createPrefixDb("1", [redis])})
    assert n == 0
    assert {p: sorted(map(tuple, v)) for p, v in d.ps.prefixes().items()} == before
    u = d.rebuild()
    assert not u["unicastRoutesToUpdate"] and not u["unicastRoutesToDelete"]


def kat_decision_rib_policy(M):
    """DecisionTest.cpp:1292-1404 DecisionTestFixture.RibPolicy (compute side):
    weight 0 (ECMP) -> policy sets neighbour weight 2 -> weight 0 for that
    neighbour keeps the route intact (weights 0) -> the expired policy leaves
    the RouteDb unchanged."""
    d = _Decision(M, "1", [kTestingAreaName])
    d.publish(kTestingAreaName, {
        "adj:1": _adj_val("1", [adj12], 1), "adj:2": _adj_val("2", [adj21], 2),
        f"prefix:1:[{addr1}]": createPrefixDb("1", [createPrefixEntry(addr1)]),
        f"prefix:2:[{addr2}]": createPrefixDb("2", [createPrefixEntry(addr2)])})
    u = d.rebuild()
    assert len(u["unicastRoutesToUpdate"]) == 1
    assert [x[2] for x in u["unicastRoutesToUpdate"][addr2]["nexthops"]] == [0]
    stmt = dict(name="p", prefixes=[addr2],
                set_weight=dict(default_weight=0, neighbor_to_weight={"2": 2}))
    d.set_policy([stmt], 1)
    u = d.rebuild()
    assert len(u["unicastRoutesToUpdate"]) == 1
    assert [x[2] for x in u["unicastRoutesToUpdate"][addr2]["nexthops"]] == [2]
    stmt["set_weight"]["neighbor_to_weight"]["2"] = 0
    d.set_policy([stmt], 1)
    u = d.rebuild()
    assert list(u["unicastRoutesToUpdate"]) == [addr2] and not u["unicastRoutesToDelete"]
    assert all(x[2] == 0 for x in u["unicastRoutesToUpdate"][addr2]["nexthops"])
    time.sleep(1.05)
    u = d.rebuild()
    assert not u["unicastRoutesToUpdate"]


MORE_KATS = [
    kat_ring_duplicate_mpls_routes, kat_ring_multipath, kat_ring_attached_nodes,
    kat_ring_overload_node, kat_ring_overload_link, kat_parallel_adj_ring_multipath,
    kat_grid_large, kat_rib_policy_statement_match, kat_rib_policy_apply_action,
    kat_rib_policy_apply_policy, kat_decision_parallel_links,
    kat_decision_self_redistribute, kat_decision_rib_policy,
]
