"""The global-state SPF path (spf_global.hip): topologies
whose per-unit SPF state does not fit LDS run with dist / next-hop sets /
frontier lists in HBM. Parity against the oracle on the reference's 99x99
GridTopology.StressTest (SpfSolverTest.cpp:2858-2873, source "523"), on
single-area WANs of 20k-30k nodes (past every LDS path), and -- with the
"spf_global" option forcing the path -- on the small grid / fabric / WAN
cases the LDS kernels are tested on."""
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


class _Global:
    """Forces (on=1) or leaves automatic (on=0) the global path."""

    def __init__(self, on):
        import openr_amd.capi as capi
        self.lib, self.on = capi.load(), on

    def __enter__(self):
        import openr_amd.capi as capi
        capi.check(self.lib, self.lib.ogs_set_option(b"spf_global", self.on), "spf_global")

    def __exit__(self, *a):
        self.lib.ogs_set_option(b"spf_global", 0)


MIX = dict(v4Permille=150, anycastPermille=120, minNhPermille=60, drainPermille=50)


class _Opt:
    """Sets an engine option for the block, then restores `reset`."""

    def __init__(self, name, value, reset):
        import openr_amd.capi as capi
        self.lib, self.name, self.value, self.reset = capi.load(), name, value, reset

    def __enter__(self):
        import openr_amd.capi as capi
        capi.check(self.lib, self.lib.ogs_set_option(self.name, self.value), self.name.decode())

    def __exit__(self, *a):
        self.lib.ogs_set_option(self.name, self.reset)


@pytest.mark.parametrize("lds", [0, 1, 2, 3])
def test_forced_global_both_state_forms(product, oracle, lds):
    """The global path's state forms -- one-phase packed {dist, nh} words in
    LDS (lds=1, default where they fit: one next-hop word, u32 distances),
    two-phase distances + next-hop words in LDS (3), distances only (2),
    everything in HBM (0) -- on a grid with overloads and the prefix mix
    (both metric widths) and a fabric with multi-word next-hop sets."""
    grid = dict(n=9, metricSeed=0xC2000099, prefixSeed=7, adjOverloadPermille=30,
                nodeOverloadPermille=20, overloadSeed=0x79, **MIX)
    wide = dict(grid, metricMax=20000000)
    fab = dict(pods=4, planes=4, sswPerPlane=8, rswPerPod=16, full=True, prefixesPerNode=2,
               nodeOverloadPermille=20, **MIX)
    fsrc = ["1-0-0", "2-1-2", "3-3-15", "2-0-0"]
    with _Global(1), _Opt(b"spf_global_lds", lds, 1):
        for opts, label in ((grid, "grid"), (wide, "wide")):
            srcs = [str(i) for i in range(0, 81, 4)]
            _cmp(product.gen_route_dbs("grid", opts, srcs, True, True, True),
                 oracle.gen_route_dbs("grid", opts, srcs, True, True, True), f"{label}{lds}")
        _cmp(product.gen_route_dbs("fabric", fab, fsrc, True, True, False),
             oracle.gen_route_dbs("fabric", fab, fsrc, True, True, False), f"fabric{lds}")


@pytest.mark.parametrize("brs", [False, True])
def test_forced_global_grid_all_sources(product, oracle, brs):
    opts = dict(n=7, metricSeed=0xC2000077, prefixSeed=5, adjOverloadPermille=30,
                nodeOverloadPermille=20, overloadSeed=0x77, **MIX)
    srcs = [str(i) for i in range(49)]
    with _Global(1):
        a = product.gen_route_dbs("grid", opts, srcs, True, True, brs)
    _cmp(a, oracle.gen_route_dbs("grid", opts, srcs, True, True, brs), "grid7")


@pytest.mark.parametrize("metric_max", [100, 20000000])
def test_forced_global_distance_widths(product, oracle, metric_max):
    """u32 and u64 (OGS_F_WIDE_METRIC) distances through the global path."""
    opts = dict(n=10, metricSeed=0xC2300000, prefixSeed=0xC1, metricMax=metric_max)
    srcs = ["1", "45", "99"]
    with _Global(1):
        a = product.gen_route_dbs("grid", opts, srcs, True, True, False)
    _cmp(a, oracle.gen_route_dbs("grid", opts, srcs, True, True, False), "gridw")


def test_forced_global_fabric_prefix_mix(product, oracle):
    """Fabric (FSW next-hop sets of 2 words), drains, anycast / v4 / minNexthop
    prefix mix, node labels on."""
    opts = dict(pods=8, planes=4, sswPerPlane=16, rswPerPod=32, full=True, prefixesPerNode=2,
                nodeOverloadPermille=20, adjOverloadPermille=10, **MIX)
    names = ([f"1-{p}-{s}" for p in range(4) for s in range(16)] +
             [f"2-{p}-{f}" for p in range(8) for f in range(4)] +
             [f"3-{p}-{r}" for p in range(8) for r in range(32)])
    srcs = names[::9] + ["2-5-1"]
    with _Global(1):
        a = product.gen_route_dbs("fabric", opts, srcs, True, True, False)
    _cmp(a, oracle.gen_route_dbs("fabric", opts, srcs, True, True, False), "fabric")


def test_forced_global_wan_spf_results(product, oracle):
    """getSpfResult (dist + next-hop node names) of a 700-node WAN with
    overloads, both metric modes, through the global path."""
    opts = dict(nodes=700, seed=0xC7, prefixesPerNode=1, nodeOverloadPermille=30,
                adjOverloadPermille=20)
    rng = random.Random(3)
    srcs = [str(rng.randrange(700)) for _ in range(6)]
    with _Global(1):
        a = product.gen_route_dbs("wan", opts, srcs, True, True, True)
    _cmp(a, oracle.gen_route_dbs("wan", opts, srcs, True, True, True), "wan700")


def _stress_grid(M, n):
    """SpfSolverTest.cpp GridTopologyFixture / createGrid wiring (as
    kat_cases.kat_grid): unit metrics, node labels, one /128 per node."""
    als = M.AreaLinkStates()
    ls = als.add(L.kTestingAreaName, L.kTestingNodeName)
    ps = M.PrefixState()
    for i in range(n):
        for j in range(n):
            node = i * n + j
            adjs = []
            for (ii, jj, ifn, oifn) in ((i, j + 1, "0/1", "0/3"), (i - 1, j, "0/2", "0/4"),
                                        (i, j - 1, "0/3", "0/1"), (i + 1, j, "0/4", "0/2")):
                if 0 <= ii < n and 0 <= jj < n:
                    nb = ii * n + jj
                    a = L.createAdjacency(str(nb), ifn, oifn, f"fe80::{nb:x}",
                                          f"192.168.{nb // 256}.{nb % 256}", 1, 100001 + nb)
                    adjs.append(a)
            ls.updateAdjacencyDatabase(L.createAdjDb(str(node), adjs, node + 1),
                                       L.kTestingAreaName)
            ps.updatePrefix(str(node), L.kTestingAreaName, L.createPrefixEntry(
                f"::ffff:10.{node // 65536}.{(node // 256) % 256}.{node % 256}/128"))
    return als, ps


@pytest.mark.parametrize("force", [0, 1])
def test_stress_grid_99(product, oracle, force):
    """GridTopology.StressTest (SpfSolverTest.cpp:2858-2873): 99x99 grid,
    SpfSolver("1", v4 off, node labels on, best-route selection on),
    buildRouteDb("523"); equals the oracle and every route's metric is the
    Manhattan distance."""
    n = 99
    pa, pp = _stress_grid(product, n)
    oa, op = _stress_grid(oracle, n)
    with _Global(force):
        got = product.SpfSolver("1", False, True, True).buildRouteDb("523", pa, pp)
    want = oracle.SpfSolver("1", False, True, True).buildRouteDb("523", oa, op)
    assert got.canonical() == want.canonical()
    routes = got.unicastRoutes()
    assert len(routes) == n * n - 1
    s = 523
    for p, r in list(routes.items())[::97]:
        d = int(p.split("/")[0].split(".")[-1]) + 256 * int(p.split(".")[-2]) + \
            65536 * int(p.split(".")[-3])
        dist = abs(s % n - d % n) + abs(s // n - d // n)
        assert {x[4] for x in r["nexthops"]} == {dist}


@pytest.mark.parametrize("nodes", [20000, 30000])
def test_large_wan_single_area(product, oracle, nodes):
    """Single-area WANs past every LDS path (no option set): the engine
    solves them (no 'unsupported') and equals the oracle, prefix mix and
    overloads included."""
    opts = dict(nodes=nodes, seed=0xC9 + nodes, prefixesPerNode=1, nodeOverloadPermille=10,
                adjOverloadPermille=10, **MIX)
    rng = random.Random(nodes)
    srcs = [str(rng.randrange(nodes)) for _ in range(3)]
    a = product.gen_route_dbs("wan", opts, srcs, True, False, True)
    _cmp(a, oracle.gen_route_dbs("wan", opts, srcs, True, False, True), f"wan{nodes}")


def test_large_wan_batch_all_sources_sample(product, oracle):
    """One batched launch over 64 sources of a 20k-node WAN (the all-sources
    form of the global path): every RouteDb equals the oracle's."""
    opts = dict(nodes=20000, seed=0xCA, prefixesPerNode=1)
    rng = random.Random(5)
    srcs = sorted({str(rng.randrange(20000)) for _ in range(64)})
    br = product.BatchRunner(True, False, False)
    br.add_generated("wan", opts, srcs)
    br.upload()
    br.run()
    br.download()
    a = [br.canonical(u) for u in range(len(srcs))]
    _cmp(a, oracle.gen_route_dbs("wan", opts, srcs, True, False, False), "wan20k_batch")


def test_large_multi_area(product, oracle):
    """Multi-area domain with 22k-node areas: per-area SPF through the global
    path, then the multi-area route kernel."""
    opts = dict(areas=2, nodesPerArea=22000, abrs=8, prefixesPerNode=1, anycastPermille=50)
    srcs = ["abr-0", "a1-21999"]
    _cmp(product.gen_route_dbs_multiarea(opts, srcs, True, False, True),
         oracle.gen_route_dbs_multiarea(opts, srcs, True, False, True), "ma22k")
