"""Deep topologies through the chunk-queue SPF forms (spf_lds.hip general-
weight rounds, spf_frontier.hip packed chunk scan): their per-node round
stamps are u8, so past round 255 a stale stamp matches again. A reached node
re-pushing is a no-op for the monotone fixpoint; an UNREACHED node must never
push (kInf + w wraps to a small candidate and would give a disconnected
island finite distances -- an anycast prefix would then select the island's
unreachable advertiser). Reference: LinkState::runSpf (LinkState.cpp:720-820)
never relaxes from a node it has not reached; SpfSolver.cpp:160-311 selects
among reachable advertisers only.

The case: a line of 300 nodes with mixed metrics (shortest paths of up to
299 hops, so 300+ rounds), plus a two-node island that advertises its own
prefixes and one anycast prefix shared with the line's far end."""
import pytest

import lsdb as L
from test_gpu_parity import _cmp

pytestmark = pytest.mark.gpu

N_LINE = 300


def _name(i):
    return f"n{i:03d}"


def _build(M, uniform=False):
    als = M.AreaLinkStates()
    ls = als.add(L.kTestingAreaName, _name(0))
    ps = M.PrefixState()
    A = L.createAdjacency

    def metric(i):  # link n_i -- n_{i+1}
        return 1 if uniform else 1 + (i * 7) % 3

    for i in range(N_LINE):
        adjs = []
        if i > 0:
            adjs.append(A(_name(i - 1), f"{i}/l", f"{i - 1}/r", f"fe80::{i:x}:1",
                          f"10.{i // 250}.{i % 250}.1", metric(i - 1), 0))
        if i + 1 < N_LINE:
            adjs.append(A(_name(i + 1), f"{i}/r", f"{i + 1}/l", f"fe80::{i:x}:2",
                          f"10.{i // 250}.{i % 250}.2", metric(i), 0))
        ls.updateAdjacencyDatabase(L.createAdjDb(_name(i), adjs, 0), L.kTestingAreaName)
        entries = [L.createPrefixEntry(f"fc00::{i:x}/128")]
        if i == N_LINE - 1:
            entries.append(L.createPrefixEntry("fd00::/64"))
        L.updatePrefixDatabase(ps, L.createPrefixDb(_name(i), entries))
    island = {"z0": "z1", "z1": "z0"}
    for z, other in island.items():
        ls.updateAdjacencyDatabase(
            L.createAdjDb(z, [A(other, f"{z}/x", f"{other}/x", f"fe80::{z}", "10.9.9.9",
                                 1 if uniform else 2, 0)],
                          0), L.kTestingAreaName)
        entries = [L.createPrefixEntry(f"fc01::{z[1]}/128")]
        if z == "z0":
            entries.append(L.createPrefixEntry("fd00::/64"))  # anycast with the line's end
        L.updatePrefixDatabase(ps, L.createPrefixDb(z, entries))
    return als, ps


SOURCES = [_name(0), _name(1), _name(150), _name(N_LINE - 1), "z0"]


def _oracle(oracle, uniform=False):
    als, ps = _build(oracle, uniform)
    out = []
    for s in SOURCES:
        db = oracle.SpfSolver(s, True, False).buildRouteDb(s, als, ps)
        out.append(b"NONE" if db is None else db.canonical())
    return out


@pytest.mark.parametrize("uniform", [False, True])
@pytest.mark.parametrize("options", [dict(route_stream=5), dict(route_stream=4),
                                     dict(route_stream=5, lds_bfs_exit=0, lds_tail_parts=9),
                                     dict(route_stream=5, lds_parts=3, lds_lead=2),
                                     dict(route_stream=5, lds_pull=0), dict(route_stream=5, lds_pull=15),
                                     dict(route_stream=2, spf_queue=0),
                                     dict(route_stream=1, spf_queue=0)])
def test_deep_line_with_island_batch(product, oracle, options, uniform):
    """All sources in one RouteDbBatch launch under the LDS-resident one-launch
    form (5), the LDS SPF + split stream (4) and the frontier chunk scan (2,
    1), vs the oracle's buildRouteDb per source. uniform: every metric 1, so
    the LDS form runs BFS layers (300 of them) and, with the island never
    reached, must not take the all-reached exit."""
    import openr_amd.capi as capi
    lib = capi.load()
    als, ps = _build(product, uniform)
    try:
        for k, v in options.items():
            capi.check(lib, lib.ogs_set_option(k.encode(), v), k)
        solver = product.SpfSolver(SOURCES[0], True, False)
        batch = product.RouteDbBatch(solver, als, ps, SOURCES)
        batch.launch()
        got = []
        for s in SOURCES:
            db = batch.routeDb(s)
            got.append(b"NONE" if db is None else db.canonical())
    finally:
        lib.ogs_set_option(b"route_stream", 5)
        lib.ogs_set_option(b"spf_queue", -1)
        lib.ogs_set_option(b"lds_bfs_exit", 1)
        lib.ogs_set_option(b"lds_lead", 0)
        lib.ogs_set_option(b"lds_tail_parts", 0)
        lib.ogs_set_option(b"lds_pull", 6)
    want = _oracle(oracle, uniform)
    # the island's anycast member is unreachable from the line: the line's
    # end must be the prefix's only route source
    assert b"fd00::/64" in want[0]
    _cmp(got, want, f"deep line {options}")


def test_deep_line_with_island_single_builds(product, oracle):
    """The drop-in's own single-source buildRouteDb on the same topology."""
    als, ps = _build(product)
    got = []
    for s in SOURCES:
        db = product.SpfSolver(s, True, False).buildRouteDb(s, als, ps)
        got.append(b"NONE" if db is None else db.canonical())
    _cmp(got, _oracle(oracle), "deep line single")


@pytest.mark.parametrize("pull", [0, 4, 15])
@pytest.mark.parametrize("kind", ["fabric", "fabric3"])
def test_bfs_pull_rounds(product, oracle, pull, kind):
    """Unit-weight (BFS) rounds of the LDS form pull a layer when the
    unreached nodes' edges are few against the frontier's (lds_pull; 0 push
    only): fabrics with hard-drained nodes (never relay), overloaded
    adjacencies (down links) and the prefix mix, one- and three-word sources,
    vs the oracle. Reference: LinkState.cpp:720-820 (a drained node settles
    but does not relax its links; down links are not used)."""
    from test_gpu_parity import MIX, _batch_dbs
    if kind == "fabric":
        opts = dict(pods=8, planes=4, sswPerPlane=16, rswPerPod=32, full=True,
                    prefixesPerNode=2, nodeOverloadPermille=30, adjOverloadPermille=20, **MIX)
        names = ([f"1-{p}-{s}" for p in range(4) for s in range(16)] +
                 [f"2-{p}-{f}" for p in range(8) for f in range(4)] +
                 [f"3-{p}-{r}" for p in range(8) for r in range(32)])
        srcs = names[::3]
    else:
        opts = dict(pods=4, planes=2, sswPerPlane=36, rswPerPod=48, full=True,
                    prefixesPerNode=2, nodeOverloadPermille=30, adjOverloadPermille=20, **MIX)
        srcs = [f"2-{p}-{f}" for p in range(4) for f in range(2)]
    a = _batch_dbs(product, "fabric", opts, srcs, True, True, route_stream=5, lds_pull=pull)
    _cmp(a, oracle.gen_route_dbs("fabric", opts, srcs, True, False, True), f"pull {pull} {kind}")
