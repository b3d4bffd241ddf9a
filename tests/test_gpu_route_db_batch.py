"""§8(f) f2: RouteDbBatch -- many sources' RouteDbs computed in one launch per
next-hop width group, kept in HBM, and served per node like
Decision::getDecisionRouteDb (Decision.cpp:341-360: buildRouteDb(node) ->
DecisionRouteDb::toThrift, thisNodeName = node). Every served RouteDb must be
bit-exact with the oracle's SpfSolver::buildRouteDb(node)."""
import random

import pytest

from test_gpu_parity import _cmp

pytestmark = pytest.mark.gpu


def _check(product, oracle, kind, opts, srcs, sr, brs, groups=None):
    got, shapes, n_groups = product.gen_route_db_batch(kind, opts, srcs, True, sr, brs)
    want = oracle.gen_route_dbs(kind, opts, srcs, True, sr, brs)
    _cmp(got, want, f"{kind} batch")
    for s, canon, (name, n_uni, n_mpls, n_nh, same) in zip(srcs, want, shapes):
        assert name == s
        # getRouteDbComputed's direct thrift build == routeDb(s)->toThrift()
        assert same, s
        if canon == b"NONE":
            assert (n_uni, n_mpls, n_nh) == (0, 0, 0)  # empty RouteDatabase
        else:
            assert n_uni + n_mpls > 0 or not canon.strip()
    if groups is not None:
        assert n_groups == groups


def test_fabric_all_sources_two_width_groups(product, oracle):
    """FSW rows are wider than 32 links only with many SSWs: 40 SSW per plane
    -> FSW degree 40 + RSWs -> 2 next-hop words; the rest 1 word."""
    opts = dict(pods=2, planes=2, sswPerPlane=40, rswPerPod=4, full=True, prefixesPerNode=2)
    names = ([f"1-{p}-{s}" for p in range(2) for s in range(40)] +
             [f"2-{p}-{f}" for p in range(2) for f in range(2)] +
             [f"3-{p}-{r}" for p in range(2) for r in range(4)])
    _check(product, oracle, "fabric", opts, names, True, False, groups=2)


@pytest.mark.parametrize("brs", [False, True])
def test_wan_sources_with_ghost(product, oracle, brs):
    opts = dict(nodes=300, seed=0xC4, prefixesPerNode=2, anycastPermille=100,
                nodeOverloadPermille=20, adjOverloadPermille=20, minNhPermille=50,
                v4Permille=50, drainPermille=50)
    rng = random.Random(11)
    srcs = sorted({str(rng.randrange(300)) for _ in range(24)}) + ["no-such-node"]
    _check(product, oracle, "wan", opts, srcs, True, brs)


def test_grid_all_sources_small_kernel_path(product, oracle):
    opts = dict(n=8, metricSeed=0xC2000042, prefixesPerNode=2)
    _check(product, oracle, "grid", opts, [str(i) for i in range(64)], True, False, groups=1)


@pytest.mark.parametrize("brs", [False, True])
def test_fabric_width_groups_one_launch(product, oracle, brs):
    """A fabric past 256 nodes (72 SSW + 8 FSW + 192 RSW) with FSWs of 84
    links (three next-hop words) and one-word SSW / RSW sources: the batch's
    two width groups go through ogs_spf_routes_groups -- one prep and one
    persistent launch (route_stream 5) -- with drained nodes /
    links and the prefix mix; every served RouteDb equals the oracle's."""
    opts = dict(pods=4, planes=2, sswPerPlane=36, rswPerPod=48, full=True, prefixesPerNode=2,
                nodeOverloadPermille=20, adjOverloadPermille=10, v4Permille=150,
                anycastPermille=120, minNhPermille=60, drainPermille=50)
    names = ([f"1-{p}-{s}" for p in range(2) for s in range(36)] +
             [f"2-{p}-{f}" for p in range(4) for f in range(2)] +
             [f"3-{p}-{r}" for p in range(4) for r in range(48)])
    srcs = names[::5] + [f"2-{p}-{f}" for p in range(4) for f in range(2)]
    _check(product, oracle, "fabric", opts, sorted(set(srcs)), True, brs, groups=2)
