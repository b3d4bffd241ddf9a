"""Nodes of 512+ links (a hub / route reflector): the reference iterates
linksFromNode of any length (LinkState.cpp:760-813) and unions next hops over
any number of source links (SpfSolver.cpp:690-743). Previously the drop-in
threw std::domain_error("degree > 511") (the edge word's 9-bit reverse slot);
now the slot saturates and the exact slots ride in ogs_graph.rslot_ext, and
sources of more than 512 links use next-hop sets of ceil(deg / 32) words
(runtime-width HBM kernels). Parity against the oracle for getSpfResult,
buildRouteDb (hub source and leaf sources, SR labels, best-route selection),
a UCMP RibPolicy over the hub's links, multi-area, zero / negative metrics
(exact extraction order with rows staged in HBM), the incremental
createRoutesForPrefixes and getKthPaths / prefetchKthPaths through the hub."""
import random

import pytest

import lsdb as L

pytestmark = pytest.mark.gpu

HUB = "h"


def _hub(M, leaves=600, seed=1, metrics=(1, 2, 3), parallel=0, area=L.kTestingAreaName,
         als=None, prefixes=True):
    """A hub linked to every leaf (plus `parallel` extra hub links to the first
    leaves), leaves in a ring (metric 10), one prefix per node, some anycast."""
    rng = random.Random(seed)
    als = als if als is not None else M.AreaLinkStates()
    ls = als.add(area, HUB)
    ps = M.PrefixState() if prefixes else None
    adj = {HUB: []}
    names = [f"l{i:04d}" for i in range(leaves)]
    for n in names:
        adj[n] = []

    def link(a, b, ia, ib, m):
        adj[a].append(L.createAdjacency(b, ia, ib, f"fe80::{len(adj[a]) + 1:x}",
                                        f"10.{len(adj[a]) // 250}.{len(adj[a]) % 250}.1", m, 0))
        adj[b].append(L.createAdjacency(a, ib, ia, f"fe80::{len(adj[b]) + 1:x}",
                                        f"10.{len(adj[b]) // 250}.{len(adj[b]) % 250}.2", m, 0))

    for i, n in enumerate(names):
        link(HUB, n, f"h-{n}", f"{n}-h", rng.choice(metrics))
    for i in range(parallel):
        link(HUB, names[i], f"h-{names[i]}-p", f"{names[i]}-h-p", rng.choice(metrics))
    for i, n in enumerate(names):
        nb = names[(i + 1) % leaves]
        link(n, nb, f"{n}-r", f"{nb}-l", 10)
    for k, (n, adjs) in enumerate(sorted(adj.items())):
        ls.updateAdjacencyDatabase(L.createAdjDb(n, adjs, 1000 + k, area=area), area)
    if prefixes:
        for k, n in enumerate([HUB] + names):
            entries = [L.createPrefixEntry(f"fc00:{k:x}::/64")]
            if k % 7 == 3:  # anycast: also advertised by another leaf
                entries.append(L.createPrefixEntry("fd00::%x/128" % (k // 7)))
            L.updatePrefixDatabase(ps, L.createPrefixDb(n, entries), area=area)
    return als, ls, ps


def _spf(ls, s):
    return {k: (v[0], sorted(v[1])) for k, v in ls.getSpfResult(s).items()}


@pytest.mark.parametrize("leaves", [520, 700])
def test_hub_spf_and_routes(product, oracle, leaves):
    pa, pls, pps = _hub(product, leaves)
    oa, ols, ops = _hub(oracle, leaves)
    for s in (HUB, "l0000", f"l{leaves - 1:04d}", "l0300"):
        assert _spf(pls, s) == _spf(ols, s), s
    for brs in (False, True):
        for s in (HUB, "l0000", "l0511"):
            a = product.SpfSolver(s, True, True, brs).buildRouteDb(s, pa, pps)
            b = oracle.SpfSolver(s, True, True, brs).buildRouteDb(s, oa, ops)
            assert a.canonical() == b.canonical(), (s, brs)
    # the hub's routes use next hops past link slot 511
    routes = product.SpfSolver(HUB, True, False).buildRouteDb(HUB, pa, pps).unicastRoutes()
    assert any(int(nh[1].split("-l")[1][:4]) >= 512
               for r in routes.values() for nh in r["nexthops"] if "-l" in nh[1])


def test_hub_parallel_links_and_policy(product, oracle):
    """Parallel hub links (ECMP over more than 512 slots) and a UCMP policy
    whose weights cover the hub's high link slots."""
    pa, pls, pps = _hub(product, 560, seed=2, metrics=(1,), parallel=40)
    oa, ols, ops = _hub(oracle, 560, seed=2, metrics=(1,), parallel=40)
    pol = [dict(name="all", prefixes=["fd00::%x/128" % i for i in range(0, 90)],
                set_weight=dict(default_weight=1, area_to_weight={},
                                neighbor_to_weight={f"l{i:04d}": (i % 4) for i in range(0, 560, 3)}),
                counterID="ucmp")]
    ppol, opol = product.RibPolicy(pol), oracle.RibPolicy(pol)
    for s in (HUB, "l0100"):
        ps_ = product.SpfSolver(s, True, False)
        ps_.setRibPolicy(ppol)  # applied on the device (rib_policy.hip)
        a = ps_.buildRouteDb(s, pa, pps)
        b = oracle.SpfSolver(s, True, False).buildRouteDb(s, oa, ops)
        opol.applyPolicy(b)  # RibPolicy::applyPolicy over the oracle's RouteDb
        assert a.canonical() == b.canonical(), s
        assert "cid=ucmp" in a.canonical().decode()


@pytest.mark.parametrize("metrics", [(0, 1, 2), (1, -1, 3), (0, -2)])
def test_hub_exact_order(product, oracle, metrics):
    """Zero / negative metrics on a hub: the exact replay stages rows of 512+
    edges in HBM and unions next hops over sets of any width."""
    pa, pls, pps = _hub(product, 540, seed=3, metrics=metrics)
    oa, ols, ops = _hub(oracle, 540, seed=3, metrics=metrics)
    for s in (HUB, "l0007", "l0539"):
        assert _spf(pls, s) == _spf(ols, s), s
        a = product.SpfSolver(s, True, True).buildRouteDb(s, pa, pps)
        b = oracle.SpfSolver(s, True, True).buildRouteDb(s, oa, ops)
        assert a.canonical() == b.canonical(), s


def test_hub_incremental_routes(product, oracle):
    pa, pls, pps = _hub(product, 530, seed=4)
    oa, ols, ops = _hub(oracle, 530, seed=4)
    asked = {"fc00:1::/64", "fc00:200::/64", "fd00::3/128", "fc00:dead::/64"}
    s_ = product.SpfSolver(HUB, True, False)
    o_ = oracle.SpfSolver(HUB, True, False)
    got = s_.createRoutesForPrefixes(HUB, pa, pps, asked)
    for p in asked:
        assert got[p] == o_.createRouteForPrefixOrGetStaticRoute(HUB, oa, ops, p), p


def test_hub_multi_area(product, oracle):
    """The hub is an ABR: area A has its 600 leaves, area B a small ring."""
    pa, pls, pps = _hub(product, 600, seed=5, area="A")
    oa, ols, ops = _hub(oracle, 600, seed=5, area="A")
    for M, als, ps in ((product, pa, pps), (oracle, oa, ops)):
        lb = als.add("B", HUB)
        ring = [HUB, "b1", "b2", "b3"]
        adj = {n: [] for n in ring}
        for i, n in enumerate(ring):
            nb = ring[(i + 1) % 4]
            adj[n].append(L.createAdjacency(nb, f"{n}>{nb}", f"{nb}<{n}", f"fe80::b{i}", "", 2, 0))
            adj[nb].append(L.createAdjacency(n, f"{nb}<{n}", f"{n}>{nb}", f"fe80::c{i}", "", 2, 0))
        for k, n in enumerate(ring):
            lb.updateAdjacencyDatabase(L.createAdjDb(n, adj[n], 5000 + k, area="B"), "B")
            L.updatePrefixDatabase(ps, L.createPrefixDb(n, [L.createPrefixEntry(f"fe00:{k}::/64")]),
                                   area="B")
    for s in (HUB, "b2", "l0042"):
        for brs in (False, True):
            a = product.SpfSolver(s, True, True, brs).buildRouteDb(s, pa, pps)
            b = oracle.SpfSolver(s, True, True, brs).buildRouteDb(s, oa, ops)
            assert (a is None) == (b is None), s
            if a is not None:
                assert a.canonical() == b.canonical(), (s, brs)


def _paths(ls, s, d, k):
    return [[(x["n1"], x["if1"], x["n2"], x["if2"]) for x in p] for p in ls.getKthPaths(s, d, k)]


@pytest.mark.parametrize("metrics", [(1, 2), (0, 1)])
def test_hub_kth_paths(product, oracle, metrics):
    """getKthPaths through the hub: pathLinks of leaves are ordered by (dist,
    pred, slot) with slots of the hub's 512+ row, and k = 2 masks links by
    id (both need the exact reverse slots)."""
    _, pls, _ = _hub(product, 600, seed=6, metrics=metrics, parallel=20, prefixes=False)
    _, ols, _ = _hub(oracle, 600, seed=6, metrics=metrics, parallel=20, prefixes=False)
    rng = random.Random(7)
    pairs = [("l0000", "l0300"), (HUB, "l0599"), ("l0550", HUB)]
    pairs += [(f"l{rng.randrange(600):04d}", f"l{rng.randrange(600):04d}") for _ in range(6)]
    for s, d in pairs:
        for k in (1, 2):
            assert _paths(pls, s, d, k) == _paths(ols, s, d, k), (s, d, k)
    dests = [f"l{i:04d}" for i in range(0, 600, 7)] + [HUB]
    pls.prefetchKthPaths("l0010", dests)
    for d in dests:
        for k in (1, 2):
            assert _paths(pls, "l0010", d, k) == _paths(ols, "l0010", d, k), (d, k)
