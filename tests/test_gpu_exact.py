"""Zero and negative link metrics (spf_exact.hip, OGS_F_EXACT_ORDER): the
reference settles nodes in DijkstraQ order (LinkState.cpp:720-820,
LinkState.h:612-663), and with a zero metric the next-hop sets depend on
which of two equal-distance nodes is settled first; negative i32 metrics
become huge u64 link metrics whose sums wrap (LinkState.cpp:77-78). The
engine replays that order on the device. Parity against the oracle (a
restatement of the same heap algorithm) on hand-built cases whose answer
differs from the order-free fixpoint, and on generated grids / WANs /
fabrics with zero and negative links, through every API that builds routes
(getSpfResult, buildRouteDb, the batched launch, RouteDbBatch, the
incremental createRoutesForPrefixes) -- previously these threw."""
import random

import pytest

import lsdb as L

pytestmark = pytest.mark.gpu


def _cmp(a, b, label):
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            xa, ya = x.decode().splitlines(), y.decode().splitlines()
            diff = [(p, q) for p, q in zip(xa, ya) if p != q][:5]
            pytest.fail(f"{label}[{i}] differs: {diff} (len {len(xa)} vs {len(ya)})")


def _triangle(M, ab_metric=0):
    """0 -(1)- 1, 0 -(1)- 2, 1 -(ab_metric)- 2; one prefix per node."""
    als = M.AreaLinkStates()
    ls = als.add(L.kTestingAreaName, "0")
    ps = M.PrefixState()
    A = L.createAdjacency
    dbs = {
        "0": [A("1", "0/1", "1/0", "fe80::1", "10.0.0.1", 1, 101),
              A("2", "0/2", "2/0", "fe80::2", "10.0.0.2", 1, 102)],
        "1": [A("0", "1/0", "0/1", "fe80::10", "10.0.0.10", 1, 100),
              A("2", "1/2", "2/1", "fe80::12", "10.0.0.12", ab_metric, 102)],
        "2": [A("0", "2/0", "0/2", "fe80::20", "10.0.0.20", 1, 100),
              A("1", "2/1", "1/2", "fe80::21", "10.0.0.21", ab_metric, 101)],
    }
    for n, adjs in dbs.items():
        ls.updateAdjacencyDatabase(L.createAdjDb(n, adjs, int(n) + 1), L.kTestingAreaName)
        L.updatePrefixDatabase(ps, L.createPrefixDb(n, [L.createPrefixEntry(f"fc00::{n}/128")]))
    return als, ls, ps


def test_zero_metric_extraction_order(product, oracle):
    """Node "1" is settled before "2" (equal distance, name order): "2" gets
    both next hops, "1" only itself -- the order-free fixpoint would give
    "1" both as well (2 is a tight predecessor of 1 over the zero link)."""
    for M in (product, oracle):
        als, ls, ps = _triangle(M)
        r = {k: (v[0], sorted(v[1])) for k, v in ls.getSpfResult("0").items()}
        assert r == {"0": (0, []), "1": (1, ["1"]), "2": (1, ["1", "2"])}, M
    pa, pls, pps = _triangle(product)
    oa, ols, ops = _triangle(oracle)
    a = product.SpfSolver("0", True, True).buildRouteDb("0", pa, pps)
    b = oracle.SpfSolver("0", True, True).buildRouteDb("0", oa, ops)
    assert a.canonical() == b.canonical()
    nh2 = a.unicastRoutes()["fc00::2/128"]["nexthops"]
    assert {x[1] for x in nh2} == {"0/1", "0/2"}
    assert {x[1] for x in a.unicastRoutes()["fc00::1/128"]["nexthops"]} == {"0/1"}


def test_negative_metric_wraps(product, oracle):
    """A negative adjacency metric makes the link's u64 max metric 2^64 - k:
    distances over it wrap (the reference's arithmetic, reproduced)."""
    for m in (-5, -1, -100):
        pa, pls, pps = _triangle(product, m)
        oa, ols, ops = _triangle(oracle, m)
        for src in ("0", "1", "2"):
            x = {k: (v[0], sorted(v[1])) for k, v in pls.getSpfResult(src).items()}
            y = {k: (v[0], sorted(v[1])) for k, v in ols.getSpfResult(src).items()}
            assert x == y, (m, src)
            a = product.SpfSolver(src, True, True).buildRouteDb(src, pa, pps)
            b = oracle.SpfSolver(src, True, True).buildRouteDb(src, oa, ops)
            assert a.canonical() == b.canonical(), (m, src)


MIX = dict(v4Permille=150, anycastPermille=120, minNhPermille=60, drainPermille=50)


@pytest.mark.parametrize("zero,neg", [(300, 0), (150, 40), (0, 60)])
@pytest.mark.parametrize("brs", [False, True])
def test_grid_special_metrics_all_sources(product, oracle, zero, neg, brs):
    opts = dict(n=7, metricSeed=0xE0 + zero + neg, metricMax=5, prefixSeed=3,
                zeroMetricPermille=zero, negMetricPermille=neg, adjOverloadPermille=20,
                nodeOverloadPermille=20, overloadSeed=0xE1, **MIX)
    srcs = [str(i) for i in range(49)]
    _cmp(product.gen_route_dbs("grid", opts, srcs, True, True, brs),
         oracle.gen_route_dbs("grid", opts, srcs, True, True, brs), f"grid z{zero} n{neg}")


def test_wan_and_fabric_zero_metrics(product, oracle):
    wan = dict(nodes=400, seed=0xE2, prefixesPerNode=2, zeroMetricPermille=200,
               negMetricPermille=10, **MIX)
    rng = random.Random(2)
    srcs = [str(rng.randrange(400)) for _ in range(8)]
    _cmp(product.gen_route_dbs("wan", wan, srcs, True, True, True),
         oracle.gen_route_dbs("wan", wan, srcs, True, True, True), "wan")
    fab = dict(pods=4, planes=4, sswPerPlane=8, rswPerPod=8, full=True, prefixesPerNode=1,
               zeroMetricPermille=250)
    names = ([f"1-{p}-{s}" for p in range(4) for s in range(8)] +
             [f"2-{p}-{f}" for p in range(4) for f in range(4)] +
             [f"3-{p}-{r}" for p in range(4) for r in range(8)])
    _cmp(product.gen_route_dbs("fabric", fab, names[::3], True, True, False),
         oracle.gen_route_dbs("fabric", fab, names[::3], True, True, False), "fabric")


def test_batch_and_route_db_batch_zero_metrics(product, oracle):
    """The batched launch (BatchRunner) and the resident RouteDbBatch take
    the exact path for zero-metric topologies too."""
    opts = dict(n=6, metricSeed=0xE3, metricMax=4, prefixSeed=4, zeroMetricPermille=250,
                negMetricPermille=20)
    srcs = [str(i) for i in range(36)]
    br = product.BatchRunner(True, False, True)
    br.add_generated("grid", opts, srcs)
    br.upload()
    br.run()
    br.download()
    _cmp([br.canonical(u) for u in range(len(srcs))],
         oracle.gen_route_dbs("grid", opts, srcs, True, False, True), "batch")
    got, _, _ = product.gen_route_db_batch("grid", opts, srcs, True, True, False)
    want = oracle.gen_route_dbs("grid", opts, srcs, True, True, False)
    _cmp(got, want, "route_db_batch")


def test_incremental_routes_zero_metric(product, oracle):
    """createRoutesForPrefixes (the incremental branch of rebuildRoutes,
    Decision.cpp:929-938) on a topology with a zero-metric adjacency equals
    the oracle's per-prefix createRouteForPrefixOrGetStaticRoute (ADVICE r1:
    it used to throw)."""
    pa, pls, pps = _triangle(product)
    oa, ols, ops = _triangle(oracle)
    ps_ = product.SpfSolver("0", True, False)
    os_ = oracle.SpfSolver("0", True, False)
    asked = {"fc00::1/128", "fc00::2/128", "fc00::0/128", "fc00::dead/128"}
    got = ps_.createRoutesForPrefixes("0", pa, pps, asked)
    for p in asked:
        want = os_.createRouteForPrefixOrGetStaticRoute("0", oa, ops, p)
        assert got[p] == want, p
        assert ps_.createRouteForPrefixOrGetStaticRoute("0", pa, pps, p) == want, p


def _line_minus_one(M, two_areas=False):
    """0 -(-1)- 1 (and, with two_areas, 0 -(1)- 2 in a second area): from
    "0" node "1" is reached at the u64 distance 2^64 - 1 -- the all-ones
    value, which the reference keeps as a reachable metric (LinkState.cpp:
    77-78, 789; getNextHopsWithMetric accepts shortestMetric >= distance)."""
    als = M.AreaLinkStates()
    ls = als.add(L.kTestingAreaName, "0")
    ps = M.PrefixState()
    A = L.createAdjacency
    for n, adjs in {"0": [A("1", "0/1", "1/0", "fe80::1", "10.0.0.1", -1, 101)],
                    "1": [A("0", "1/0", "0/1", "fe80::10", "10.0.0.10", -1, 100)]}.items():
        ls.updateAdjacencyDatabase(L.createAdjDb(n, adjs, int(n) + 1), L.kTestingAreaName)
        L.updatePrefixDatabase(ps, L.createPrefixDb(n, [L.createPrefixEntry(f"fc00::{n}/128")]))
    if two_areas:
        lb = als.add("B", "0")
        for n, adjs in {"0": [A("2", "0/2", "2/0", "fe80::2", "10.0.0.2", 1, 102)],
                        "2": [A("0", "2/0", "0/2", "fe80::20", "10.0.0.20", 1, 100)]}.items():
            lb.updateAdjacencyDatabase(L.createAdjDb(n, adjs, int(n) + 11, area="B"), "B")
        L.updatePrefixDatabase(ps, L.createPrefixDb("2", [L.createPrefixEntry("fc00::2/128")]),
                               area="B")
    return als, ls, ps


@pytest.mark.parametrize("two_areas", [False, True])
def test_all_ones_distance_is_reachable(product, oracle, two_areas):
    """A settled node whose wrapped distance is exactly all ones is reached:
    getSpfResult keeps it, its prefix gets a route (metric -1 as i32) and its
    node label an MPLS route -- on the GPU through the settled bitset of the
    exact-order SPF, not the all-ones sentinel."""
    pa, pls, pps = _line_minus_one(product, two_areas)
    oa, ols, ops = _line_minus_one(oracle, two_areas)
    x = {k: (v[0], sorted(v[1])) for k, v in pls.getSpfResult("0").items()}
    y = {k: (v[0], sorted(v[1])) for k, v in ols.getSpfResult("0").items()}
    assert x == y and x["1"][0] == (1 << 64) - 1
    a = product.SpfSolver("0", True, True).buildRouteDb("0", pa, pps)
    b = oracle.SpfSolver("0", True, True).buildRouteDb("0", oa, ops)
    assert a.canonical() == b.canonical()
    routes = a.unicastRoutes()
    assert "fc00::1/128" in routes
    if not two_areas:
        s = product.SpfSolver("0", True, True)
        s.buildRouteDb("0", pa, pps)
        got = s.createRoutesForPrefixes("0", pa, pps, {"fc00::1/128"})
        assert got["fc00::1/128"] == routes["fc00::1/128"]
