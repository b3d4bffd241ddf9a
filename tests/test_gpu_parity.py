"""Bit-exact parity of the GPU product against the CPU oracle on seeded
synthetic LSDBs (grid / fabric / WAN), including the full 4096-topology
config-C2 batch the bench measures."""
import random

import pytest

pytestmark = pytest.mark.gpu


def _cmp(a, b, label):
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            xa, ya = x.decode().splitlines(), y.decode().splitlines()
            diff = [(p, q) for p, q in zip(xa, ya) if p != q][:5]
            pytest.fail(f"{label}[{i}] differs: {diff} (len {len(xa)} vs {len(ya)})")


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("brs", [False, True])
def test_grid_random_metrics_all_sources(product, oracle, seed, brs):
    opts = dict(n=6, metricSeed=0xC2000000 + seed, prefixSeed=seed,
                adjOverloadPermille=20, nodeOverloadPermille=10,
                overloadSeed=0xABC + seed)
    srcs = [str(i) for i in range(36)]
    a = product.gen_route_dbs("grid", opts, srcs, True, True, brs)
    b = oracle.gen_route_dbs("grid", opts, srcs, True, True, brs)
    _cmp(a, b, "grid")


def test_grid_unit_metric_ecmp(product, oracle):
    opts = dict(n=10, prefixesPerNode=2)
    srcs = [str(i) for i in range(0, 100, 7)]
    _cmp(product.gen_route_dbs("grid", opts, srcs, True, True, False),
         oracle.gen_route_dbs("grid", opts, srcs, True, True, False), "grid10")


@pytest.mark.parametrize("full", [True, False])
def test_fabric_small_all_sources(product, oracle, full):
    opts = dict(pods=3, planes=2, sswPerPlane=3, rswPerPod=4, full=full)
    n = 2 * 3 + 3 * 2 + 3 * 4
    srcs = None
    names = ([f"1-{p}-{s}" for p in range(2) for s in range(3)] +
             [f"2-{p}-{f}" for p in range(3) for f in range(2)] +
             [f"3-{p}-{r}" for p in range(3) for r in range(4)])
    assert len(names) == n
    srcs = names
    _cmp(product.gen_route_dbs("fabric", opts, srcs, True, True, False),
         oracle.gen_route_dbs("fabric", opts, srcs, True, True, False), "fabric")


def test_wan_random_sources(product, oracle):
    opts = dict(nodes=300, seed=0xC4)
    rng = random.Random(7)
    srcs = [str(rng.randrange(300)) for _ in range(12)]
    _cmp(product.gen_route_dbs("wan", opts, srcs, True, True, True),
         oracle.gen_route_dbs("wan", opts, srcs, True, True, True), "wan")


def test_spf_result_matches_oracle(product, oracle):
    import lsdb as L
    rng = random.Random(11)
    n = 7
    for M in (product, oracle):
        pass
    def build(M):
        als = M.AreaLinkStates()
        ls = als.add(L.kTestingAreaName, "0")
        r = random.Random(5)
        for i in range(n):
            for j in range(n):
                node = i * n + j
                adjs = []
                for (ii, jj, a, b) in ((i, j + 1, "e", "w"), (i, j - 1, "w", "e"),
                                       (i - 1, j, "n", "s"), (i + 1, j, "s", "n")):
                    if 0 <= ii < n and 0 <= jj < n:
                        nb = ii * n + jj
                        adjs.append(L.createAdjacency(str(nb), f"{a}{node}", f"{b}{nb}",
                                                      f"fe80::{nb}", f"10.0.0.{nb}",
                                                      r.randint(1, 9), 100 + nb))
                ls.updateAdjacencyDatabase(L.createAdjDb(str(node), adjs, node + 1),
                                           L.kTestingAreaName)
        return ls
    pls, ols = build(product), build(oracle)
    for src in [str(rng.randrange(n * n)) for _ in range(10)] + ["unknown"]:
        for ulm in (True, False):
            a = {k: (v[0], sorted(v[1])) for k, v in pls.getSpfResult(src, ulm).items()}
            b = {k: (v[0], sorted(v[1])) for k, v in ols.getSpfResult(src, ulm).items()}
            assert a == b, src


def test_c2_full_batch_bit_exact(product, oracle):
    """Config C2 at bench size: 4096 random-metric 10x10 grids, source "1",
    one batched launch; every topology's RouteDb equals the oracle's."""
    T = 4096
    opts = dict(n=10, metricSeed=0xC2000000, prefixSeed=0xC1)
    br = product.BatchRunner(True, False, False)
    br.add_grid_batch(opts, 0, T, "1")
    br.upload()
    br.run()
    br.download()
    assert br.num_units() == T
    gpu = [br.canonical(u) for u in range(T)]
    cpu = oracle.grid_batch_route_dbs(opts, 0, T, "1")
    _cmp(gpu, cpu, "c2")
    assert all(c == 99 for c in br.route_counts())


def test_c2_parity_variant_overloads(product, oracle):
    """C2 parity variant: 2% adjacency overload + 1% node overload."""
    T = 512
    opts = dict(n=10, metricSeed=0xC2100000, prefixSeed=0xC1,
                adjOverloadPermille=20, nodeOverloadPermille=10, overloadSeed=0xC20F)
    br = product.BatchRunner(True, False, False)
    br.add_grid_batch(opts, 0, T, "1")
    br.upload()
    br.run()
    br.download()
    _cmp([br.canonical(u) for u in range(T)],
         oracle.grid_batch_route_dbs(opts, 0, T, "1"), "c2ovl")


def _grid_ls(M, n, seed, metric_max, parallel=False):
    import lsdb as L
    als = M.AreaLinkStates()
    ls = als.add(L.kTestingAreaName, "0")
    r = random.Random(seed)
    metric = {}
    for i in range(n):
        for j in range(n):
            node = i * n + j
            adjs = []
            for (ii, jj) in ((i, j + 1), (i, j - 1), (i - 1, j), (i + 1, j)):
                if 0 <= ii < n and 0 <= jj < n:
                    nb = ii * n + jj
                    for k in range(2 if parallel else 1):
                        key = (min(node, nb), max(node, nb), k)
                        metric.setdefault(key, r.randint(1, metric_max))
                        adjs.append(L.createAdjacency(
                            str(nb), f"if{node}-{nb}-{k}", f"if{nb}-{node}-{k}",
                            f"fe80::{nb}", f"10.0.0.{nb % 250}", metric[key], 100 + nb))
            ls.updateAdjacencyDatabase(L.createAdjDb(str(node), adjs, node + 1),
                                       L.kTestingAreaName)
    return ls


def _paths(ls, s, d, k):
    return [[(l["n1"], l["if1"], l["n2"], l["if2"]) for l in p] for p in ls.getKthPaths(s, d, k)]


@pytest.mark.parametrize("seed", [3, 4])
def test_ksp2_exact_on_simple_graphs(product, oracle, seed):
    """KSP2 path lists (order included) equal the oracle's on graphs without
    parallel links, where the reference order is fully pinned."""
    n = 6
    pls, ols = _grid_ls(product, n, seed, 3), _grid_ls(oracle, n, seed, 3)
    rng = random.Random(seed)
    for _ in range(25):
        s, d = str(rng.randrange(n * n)), str(rng.randrange(n * n))
        for k in (1, 2, 3):
            assert _paths(pls, s, d, k) == _paths(ols, s, d, k), (s, d, k)


def test_ksp2_batch_prefetch(product, oracle):
    """prefetchKthPaths' batched KSP2 (one k = 1 memo fill, then every
    destination's masked k = 2 SPF in one launch): the same paths as the
    oracle's getKthPaths for every destination."""
    n = 9
    pls, ols = _grid_ls(product, n, 21, 7), _grid_ls(oracle, n, 21, 7)
    dests = [str(d) for d in range(n * n)]
    pls.prefetchKthPaths("40", dests)
    for d in dests:
        for k in (1, 2):
            assert _paths(pls, "40", d, k) == _paths(ols, "40", d, k), (d, k)


def test_ksp2_on_multigraphs(product, oracle):
    """With parallel links the reference orders them by folly hash (parity
    against the reference itself is unpinned there); the engine and the
    oracle share the canonical link order, so they must agree exactly."""
    n = 5
    pls, ols = _grid_ls(product, n, 9, 2, True), _grid_ls(oracle, n, 9, 2, True)
    rng = random.Random(9)
    for _ in range(15):
        s, d = str(rng.randrange(n * n)), str(rng.randrange(n * n))
        for k in (1, 2):
            a, b = _paths(pls, s, d, k), _paths(ols, s, d, k)
            assert a == b, (s, d, k)
            links = [l for p in a for l in p]
            assert len(links) == len(set(links))


@pytest.mark.parametrize("brs", [False, True])
def test_c2_kernel_variants_identical(product, oracle, brs):
    """Every SPF+RouteDb kernel variant (generic workgroup, small, wave; with
    and without the 2-colour slot order) gives the oracle's RouteDbs."""
    import openr_amd.capi as capi
    lib = capi.load()
    T = 256
    opts = dict(n=10, metricSeed=0xC2200000, prefixSeed=0xC1,
                adjOverloadPermille=10, nodeOverloadPermille=20, overloadSeed=0xC22F)
    cpu = None
    try:
        for uw in (0, 1, 2, 3, 128):
            for order, image in ((True, True), (True, False), (False, False)):
                capi.check(lib, lib.ogs_set_option(b"unit_width", uw), "unit_width")
                br = product.BatchRunner(True, False, brs)
                br.set_slot_order(order)
                br.set_slot_edge_image(image)
                br.add_grid_batch(opts, 0, T, "1")
                br.upload()
                br.run()
                br.download()
                gpu = [br.canonical(u) for u in range(T)]
                if cpu is None:
                    cpu = oracle.grid_batch_route_dbs(opts, 0, T, "1", brs)
                _cmp(gpu, cpu, f"c2 uw={uw} order={order} image={image}")
    finally:
        lib.ogs_set_option(b"unit_width", -1)


@pytest.mark.parametrize("metric_max", [85000, 200000, 20000000])
def test_wave_kernel_distance_forms(product, oracle, metric_max):
    """The wave kernel relaxes in a 32-bit packed form when every path is
    < 2^23 and in 64-bit words otherwise (decided per unit from the largest
    usable weight); both forms and the boundary between them are exact.
    metric_max 85000 * 99 straddles 2^23 across topologies; 2e7 * 99 needs
    the host's wide (u64) path."""
    T = 128
    opts = dict(n=10, metricSeed=0xC2300000, prefixSeed=0xC1, metricMax=metric_max)
    br = product.BatchRunner(True, False, False)
    br.add_grid_batch(opts, 0, T, "1")
    br.upload()
    br.run()
    br.download()
    _cmp([br.canonical(u) for u in range(T)],
         oracle.grid_batch_route_dbs(opts, 0, T, "1"), f"c2 metricMax={metric_max}")


@pytest.mark.parametrize("nt", [0, 2])
def test_wave_store_flavours(product, oracle, nt):
    """The wave kernel's non-temporal (route_store_nt bit 2, default) and
    ordinary output stores write the same SPF outputs and RouteDbs."""
    import openr_amd.capi as capi
    lib = capi.load()
    opts = dict(n=10, metricSeed=0xC2400077, prefixSeed=0xC1, metricMax=64)
    cpu = oracle.grid_batch_route_dbs(opts, 0, 48, "3")
    try:
        capi.check(lib, lib.ogs_set_option(b"route_store_nt", nt), "route_store_nt")
        br = product.BatchRunner(True, False, False)
        br.add_grid_batch(opts, 0, 48, "3")
        br.upload()
        br.run()
        br.download()
        got = [br.canonical(u) for u in range(br.num_units())]
    finally:
        lib.ogs_set_option(b"route_store_nt", 2)
    _cmp(got, cpu, f"wave store nt={nt}")


def _tri_grid(M, n, seed):
    """n x n grid plus one diagonal per cell: odd cycles (not bipartite), so
    the 2-colour slot order leaves same-slot edges and the wave kernel must
    fall back to the full-round convergence test."""
    import lsdb as L
    als = M.AreaLinkStates()
    ls = als.add(L.kTestingAreaName, "0")
    ps = M.PrefixState()
    r = random.Random(seed)
    metric, nbrs = {}, {}
    for i in range(n):
        for j in range(n):
            for (di, dj) in ((0, 1), (1, 0), (1, 1)):
                ii, jj = i + di, j + dj
                if ii < n and jj < n:
                    a, b = i * n + j, ii * n + jj
                    metric[(a, b)] = metric[(b, a)] = r.randint(1, 20)
                    nbrs.setdefault(a, []).append(b)
                    nbrs.setdefault(b, []).append(a)
    for v in range(n * n):
        adjs = [L.createAdjacency(str(u), f"if{v}-{u}", f"if{u}-{v}", f"fe80::{u}",
                                  f"10.0.{u // 250}.{u % 250}", metric[(v, u)], 100 + u)
                for u in sorted(nbrs[v])]
        ls.updateAdjacencyDatabase(L.createAdjDb(str(v), adjs, v + 1), L.kTestingAreaName)
        L.updatePrefixDatabase(ps, L.createPrefixDb(
            str(v), [L.createPrefixEntry(f"fc00::{v:x}/128")]))
    return als, ps


@pytest.mark.parametrize("seed", [1, 2])
def test_non_bipartite_small_topology(product, oracle, seed):
    n = 10
    (pa, pp), (oa, op) = _tri_grid(product, n, seed), _tri_grid(oracle, n, seed)
    ps_ = product.SpfSolver("0", True, False)
    os_ = oracle.SpfSolver("0", True, False)
    for src in ("0", "37", "99"):
        a = ps_.buildRouteDb(src, pa, pp)
        b = os_.buildRouteDb(src, oa, op)
        assert a.canonical() == b.canonical(), src


@pytest.mark.parametrize("group", [0, 1, 2, 4])
def test_multi_source_kernel_fabric_all_sources(product, oracle, group):
    """Edge-parallel multi-source kernel (topologies > 256 nodes): a 352-node
    fabric with drained nodes/links, every third node a source in ONE batch
    (FSW degree 48 -> 2-word next-hop sets), bit-exact against the oracle for
    every sources-per-workgroup grouping."""
    import openr_amd.capi as capi
    lib = capi.load()
    opts = dict(pods=8, planes=4, sswPerPlane=16, rswPerPod=32, full=True,
                prefixesPerNode=2, nodeOverloadPermille=20, adjOverloadPermille=10)
    names = ([f"1-{p}-{s}" for p in range(4) for s in range(16)] +
             [f"2-{p}-{f}" for p in range(8) for f in range(4)] +
             [f"3-{p}-{r}" for p in range(8) for r in range(32)])
    srcs = names[::3] + ["2-5-1", "1-3-15"]
    try:
        capi.check(lib, lib.ogs_set_option(b"ms_group", group), "ms_group")
        br = product.BatchRunner(True, False, False)
        br.add_generated("fabric", opts, srcs)
        br.upload()
        br.run()
        br.download()
        a = [br.canonical(u) for u in range(len(srcs))]
    finally:
        lib.ogs_set_option(b"ms_group", 0)
    _cmp(a, oracle.gen_route_dbs("fabric", opts, srcs, True, False, False), "fabric352")


@pytest.mark.parametrize("seed", [0xC4, 0xC5])
def test_multi_source_kernel_wan_overloads(product, oracle, seed):
    """WAN (700 nodes, random metrics) with overloaded nodes/links through
    the multi-source kernel, best-route selection on."""
    opts = dict(nodes=700, seed=seed, prefixesPerNode=2, nodeOverloadPermille=30,
                adjOverloadPermille=20)
    rng = random.Random(seed)
    srcs = [str(rng.randrange(700)) for _ in range(9)]
    _cmp(product.gen_route_dbs("wan", opts, srcs, True, True, True),
         oracle.gen_route_dbs("wan", opts, srcs, True, True, True), "wan700")


def _batch_dbs(product, kind, opts, srcs, enable_v4, brs, **options):
    """All sources of one generated topology in ONE BatchRunner launch, with
    engine options set for the duration of the call."""
    import openr_amd.capi as capi
    lib = capi.load()
    try:
        for k, v in options.items():
            capi.check(lib, lib.ogs_set_option(k.encode(), v), k)
        br = product.BatchRunner(enable_v4, False, brs)
        br.add_generated(kind, opts, srcs)
        br.upload()
        br.run()
        br.download()
        return [br.canonical(u) for u in range(len(srcs))]
    finally:
        lib.ogs_set_option(b"route_stream", 5)
        lib.ogs_set_option(b"lds_parts", 0)
        lib.ogs_set_option(b"lds_grid", 0)
        lib.ogs_set_option(b"lds_key16", 1)
        lib.ogs_set_option(b"lds_tail", 1)
        lib.ogs_set_option(b"lds_lead", 0)
        lib.ogs_set_option(b"lds_bfs_exit", 1)
        lib.ogs_set_option(b"lds_tail_parts", 0)
        lib.ogs_set_option(b"lds_pull", 6)
        lib.ogs_set_option(b"frontier_parts", 0)
        lib.ogs_set_option(b"frontier_parts_wide", 0)
        lib.ogs_set_option(b"spf_frontier", 1)
        lib.ogs_set_option(b"ms_group", 0)
        lib.ogs_set_option(b"route_store_nt", 2)
        lib.ogs_set_option(b"spf_seed_row", 1)


MIX = dict(v4Permille=150, anycastPermille=120, minNhPermille=60, drainPermille=50)


@pytest.mark.parametrize("stream,frontier", [(1, 0), (1, 1), (2, 0), (2, 1), (4, 1), (5, 1)])
@pytest.mark.parametrize("enable_v4,brs", [(True, False), (False, True), (True, True)])
def test_route_stream_fabric_prefix_mix(product, oracle, stream, frontier, enable_v4, brs):
    """Split SPF / route-stream launches vs the fused multi-source kernel on a
    352-node fabric whose prefix table mixes v4 (gated when v4 is off),
    anycast (several advertisers, ghost advertisers), minNexthop and drained
    advertisements, plus drained nodes/links: bit-exact vs the oracle."""
    opts = dict(pods=8, planes=4, sswPerPlane=16, rswPerPod=32, full=True,
                prefixesPerNode=3, nodeOverloadPermille=20, adjOverloadPermille=10,
                **MIX)
    names = ([f"1-{p}-{s}" for p in range(4) for s in range(16)] +
             [f"2-{p}-{f}" for p in range(8) for f in range(4)] +
             [f"3-{p}-{r}" for p in range(8) for r in range(32)])
    srcs = names[::5] + ["2-5-1", "1-3-15"]
    a = _batch_dbs(product, "fabric", opts, srcs, enable_v4, brs, route_stream=stream,
                   spf_frontier=frontier)
    _cmp(a, oracle.gen_route_dbs("fabric", opts, srcs, enable_v4, False, brs), "fabricmix")


@pytest.mark.parametrize("nt", [0, 1, 3])
@pytest.mark.parametrize("stream", [1, 2, 4, 5])
def test_route_stream_store_flavours(product, oracle, nt, stream):
    """The RouteDb stream's ordinary (default) and non-temporal 16-B stores
    (route_store_nt bit 1) write the same records: fused and split forms on the
    fabric prefix mix, vs the oracle."""
    opts = dict(pods=8, planes=4, sswPerPlane=16, rswPerPod=32, full=True,
                prefixesPerNode=3, nodeOverloadPermille=20, adjOverloadPermille=10,
                **MIX)
    names = ([f"1-{p}-{s}" for p in range(4) for s in range(16)] +
             [f"3-{p}-{r}" for p in range(8) for r in range(32)])
    srcs = names[::7]
    a = _batch_dbs(product, "fabric", opts, srcs, True, True, route_stream=stream,
                   route_store_nt=nt)
    _cmp(a, oracle.gen_route_dbs("fabric", opts, srcs, True, False, True), "storeflavour")


@pytest.mark.parametrize("seed", [0, 1])
@pytest.mark.parametrize("wide", [False, True])
def test_frontier_seed_row(product, oracle, seed, wide):
    """Round 1 of the chunk-scan SPF relaxes the source's row directly
    (spf_seed_row 1, default) or scans every chunk record (0): one-word
    (packed one-phase) and three-word (two-phase) sources, with drained
    nodes / links and the prefix mix, vs the oracle."""
    if wide:
        opts = dict(pods=4, planes=2, sswPerPlane=36, rswPerPod=48, full=True,
                    prefixesPerNode=2, nodeOverloadPermille=20, adjOverloadPermille=10, **MIX)
        srcs = [f"2-{p}-{f}" for p in range(4) for f in range(2)] + ["1-0-3", "3-2-7"]
    else:
        opts = dict(pods=8, planes=4, sswPerPlane=16, rswPerPod=32, full=True,
                    prefixesPerNode=3, nodeOverloadPermille=20, adjOverloadPermille=10, **MIX)
        srcs = ["1-0-0", "1-3-15", "2-5-1", "3-0-0", "3-7-31"]
    a = _batch_dbs(product, "fabric", opts, srcs, True, True, route_stream=2,
                   spf_seed_row=seed)
    _cmp(a, oracle.gen_route_dbs("fabric", opts, srcs, True, False, True), "seedrow")


@pytest.mark.parametrize("stream,frontier", [(1, 0), (1, 1), (2, 0), (2, 1), (4, 1), (5, 1)])
def test_route_stream_wan_prefix_mix(product, oracle, stream, frontier):
    """700-node WAN, random metrics, overloads and the prefix mix, best-route
    selection on, through every large-topology SPF / RouteDb form."""
    opts = dict(nodes=700, seed=0xC5, prefixesPerNode=2, nodeOverloadPermille=30,
                adjOverloadPermille=20, **MIX)
    rng = random.Random(11)
    srcs = [str(rng.randrange(700)) for _ in range(10)]
    a = _batch_dbs(product, "wan", opts, srcs, True, True, route_stream=stream,
                   spf_frontier=frontier)
    _cmp(a, oracle.gen_route_dbs("wan", opts, srcs, True, False, True), "wanmix")


@pytest.mark.parametrize("stream,key16", [(1, 1), (2, 1), (4, 1), (5, 1), (5, 0)])
def test_route_stream_three_word_sources(product, oracle, stream, key16):
    """FSW sources of 84 links (36 SSW + 48 RSW, the C3 shape on 4 pods x 2
    planes) keep three next-hop words: the fused kernel, the HBM split and
    the LDS-resident split, vs the oracle."""
    opts = dict(pods=4, planes=2, sswPerPlane=36, rswPerPod=48, full=True,
                prefixesPerNode=3, nodeOverloadPermille=10, **MIX)
    srcs = [f"2-{p}-{f}" for p in range(4) for f in range(2)]
    a = _batch_dbs(product, "fabric", opts, srcs, True, False, route_stream=stream,
                   lds_key16=key16)
    _cmp(a, oracle.gen_route_dbs("fabric", opts, srcs, True, False, False), "fsw3")


@pytest.mark.parametrize("packed", [1, 0])
@pytest.mark.parametrize("kind", ["fabric", "wan"])
def test_frontier_packed_chunk_scan(product, oracle, packed, kind):
    """The chunk-scan frontier SPF in its one-phase packed {dist, nh} form
    (spf_packed_scan 1, default for one-word next-hop sets) and in two
    phases (0), fused with the route stream: fabric sources of every degree
    class with drained nodes / links, and a WAN forced onto the chunk scan
    (spf_queue 0) with overloads and the prefix mix, vs the oracle."""
    if kind == "fabric":
        opts = dict(pods=8, planes=4, sswPerPlane=16, rswPerPod=32, full=True,
                    prefixesPerNode=3, nodeOverloadPermille=20, adjOverloadPermille=10, **MIX)
        names = ([f"1-{p}-{s}" for p in range(4) for s in range(16)] +
                 [f"3-{p}-{r}" for p in range(8) for r in range(32)])
        srcs = names[::7]
        extra = {}
    else:
        opts = dict(nodes=900, seed=0xC6, prefixesPerNode=2, nodeOverloadPermille=30,
                    adjOverloadPermille=20, **MIX)
        rng = random.Random(13)
        srcs = [str(rng.randrange(900)) for _ in range(12)]
        extra = dict(spf_queue=0)
    try:
        a = _batch_dbs(product, kind, opts, srcs, True, True, spf_packed_scan=packed, **extra)
    finally:
        import openr_amd.capi as capi
        lib = capi.load()
        lib.ogs_set_option(b"spf_packed_scan", 1)
        lib.ogs_set_option(b"spf_queue", -1)
    _cmp(a, oracle.gen_route_dbs(kind, opts, srcs, True, False, True), f"{kind} packed={packed}")


def test_route_stream_unaligned_prefix_rows(product, oracle):
    """Prefix count not a multiple of 4 (scalar tail path of the stream)."""
    opts = dict(pods=4, planes=4, sswPerPlane=20, rswPerPod=60, full=True,
                prefixesPerNode=1, **MIX)
    names = ([f"1-{p}-{s}" for p in range(4) for s in range(20)] +
             [f"2-{p}-{f}" for p in range(4) for f in range(4)] +
             [f"3-{p}-{r}" for p in range(4) for r in range(60)])
    srcs = names[::7]
    a = _batch_dbs(product, "fabric", opts, srcs, True, False)
    _cmp(a, oracle.gen_route_dbs("fabric", opts, srcs, True, False, False), "fabric_tail")


MA = dict(areas=3, nodesPerArea=60, abrs=6, prefixesPerNode=2, anycastPermille=200)


@pytest.mark.parametrize("enable_v4,sr,brs", [(True, False, False), (True, True, True),
                                              (False, False, True)])
def test_multi_area_domain(product, oracle, enable_v4, sr, brs):
    """Multi-area domain (3 WAN areas + 6 ABRs in two areas each, anycast
    across areas, overloads, v4 / minNexthop / drain prefix mix): per-source
    RouteDbs through SPF-per-area + the multi-area route kernel, bit-exact
    vs the oracle (incl. node-label MPLS routes with SR on)."""
    opts = dict(MA, nodeOverloadPermille=20, adjOverloadPermille=20, v4Permille=100,
                minNhPermille=50, drainPermille=50)
    srcs = ["abr-0", "abr-3", "abr-5", "a0-7", "a1-33", "a2-59", "a2-0"]
    _cmp(product.gen_route_dbs_multiarea(opts, srcs, enable_v4, sr, brs),
         oracle.gen_route_dbs_multiarea(opts, srcs, enable_v4, sr, brs), "multiarea")


def test_multi_area_large_areas(product, oracle):
    """Areas above the wave kernel's size (frontier SPF per area)."""
    opts = dict(areas=2, nodesPerArea=400, abrs=4, prefixesPerNode=1, anycastPermille=100)
    srcs = ["abr-1", "a1-399", "a0-5"]
    _cmp(product.gen_route_dbs_multiarea(opts, srcs, True, False, True),
         oracle.gen_route_dbs_multiarea(opts, srcs, True, False, True), "multiarea400")


def _ucmp_policy(plain, zero_nbr, area):
    """UCMP statements over prefixes picked from a policy-free DB (so the
    prefix matcher hits): tag / prefix / area / neighbor weights incl. zero
    weights (next hop dropped, route removed when none is left) and
    overlapping statements (last matching counterID wins)."""
    pfx = [ln.split()[1] for ln in plain.decode().splitlines() if ln.startswith("U ")]
    return [
        dict(name="ucmp", tags=["ucmp"], counterID="cnt-ucmp",
             set_weight=dict(default_weight=3, area_to_weight={area: 5, "area2": 0},
                             neighbor_to_weight={zero_nbr: 0, "abr-1": 4})),
        dict(name="pfx", prefixes=pfx[::7], counterID="cnt-pfx",
             set_weight=dict(default_weight=0, neighbor_to_weight={zero_nbr: 6})),
        dict(name="c1", tags=["c1"], counterID="cnt-c1",
             set_weight=dict(default_weight=2, area_to_weight={"area0": 9})),
        dict(name="c3", tags=["c3", "nope"],  # no counterID: keeps the earlier one
             set_weight=dict(default_weight=1, neighbor_to_weight={zero_nbr: 8})),
    ]


@pytest.mark.parametrize("brs", [False, True])
def test_rib_policy_wan(product, oracle, brs):
    """RibPolicy (UCMP weights, counterIDs) applied on the GPU to every route
    of a 500-node WAN with the prefix mix: bit-exact vs the oracle's
    RibPolicy::applyPolicy over its RouteDb."""
    opts = dict(nodes=500, seed=0xC6, prefixesPerNode=2, tagPermille=500, **MIX)
    srcs = ["0", "17", "250", "499"]
    plain = oracle.gen_route_dbs("wan", opts, srcs[:1], True, False, brs)[0]
    pol = _ucmp_policy(plain, "1", "0")
    _cmp(product.gen_route_dbs("wan", opts, srcs, True, False, brs, pol),
         oracle.gen_route_dbs("wan", opts, srcs, True, False, brs, pol), "policy_wan")


def test_rib_policy_statement_without_action(product):
    """A statement without set_weight is rejected (RibPolicy.cpp:20-30)."""
    with pytest.raises(ValueError):
        product.RibPolicy([dict(name="bad", tags=["c1"])])


def test_rib_policy_grid_small(product, oracle):
    """Policy on the wave (small-topology) kernel path."""
    opts = dict(n=6, metricSeed=0xC2000001, prefixSeed=1, tagPermille=400)
    srcs = [str(i) for i in range(0, 36, 5)]
    plain = oracle.gen_route_dbs("grid", opts, srcs[:1], True, True, False)[0]
    pol = _ucmp_policy(plain, "1", "0")
    _cmp(product.gen_route_dbs("grid", opts, srcs, True, True, False, pol),
         oracle.gen_route_dbs("grid", opts, srcs, True, True, False, pol), "policy_grid")


@pytest.mark.parametrize("brs", [False, True])
def test_rib_policy_multi_area(product, oracle, brs):
    """Policy over multi-area RouteDbs (area weights per next-hop area)."""
    opts = dict(MA, v4Permille=100, drainPermille=50)
    srcs = ["abr-0", "abr-1", "a0-7", "a2-59"]
    plain = oracle.gen_route_dbs_multiarea(opts, srcs[:1], True, False, brs)[0]
    pol = _ucmp_policy(plain, "a0-3", "area1")
    _cmp(product.gen_route_dbs_multiarea(opts, srcs, True, False, brs, pol),
         oracle.gen_route_dbs_multiarea(opts, srcs, True, False, brs, pol),
         "policy_multiarea")


@pytest.mark.parametrize("parallel", [False, True])
def test_ksp2_batch_prefetch(product, oracle, parallel):
    """LinkState.prefetchKthPaths (one ogs_ksp2_paths call for every
    destination: shared source SPF, k = 1 trace, masked rerun, k = 2 trace)
    fills getKthPaths exactly as the oracle computes it one by one; the
    source itself and unknown nodes give no paths."""
    n = 7
    pls = _grid_ls(product, n, 21, 4, parallel)
    ols = _grid_ls(oracle, n, 21, 4, parallel)
    dests = [str(i) for i in range(n * n)] + ["nope"]
    for s in ("0", "24", "48"):
        pls.prefetchKthPaths(s, dests)
        for d in dests:
            for k in (1, 2):
                assert _paths(pls, s, d, k) == _paths(ols, s, d, k), (s, d, k)


C5_SMALL = dict(areas=3, nodesPerArea=150, abrs=8, prefixesPerNode=3, anycastPermille=80,
                nodeOverloadPermille=20, adjOverloadPermille=20, v4Permille=50)


def _c5_runner(product, rank=0, world=1):
    from openr_amd.workloads import c5_policy
    r = product.C5Runner()
    r.setup(C5_SMALL, "abr-0", [], True, rank, world)
    pol = c5_policy(r.area_names(), r.source_neighbors())
    r.set_policy(pol)
    return r, pol


def test_c5_runner_parity(product, oracle):
    """Config C5 job at reduced size (3 areas x 150 nodes + 8 ABRs, overloads,
    anycast, v4 mix): the device build (enqueueRouteDb + UCMP policy) then
    download equals the oracle's buildRouteDb + RibPolicy::applyPolicy, and
    the batched KSP2 of every destination of the source's areas equals the
    oracle's getKthPaths(src, d, 1 / 2)."""
    r, pol = _c5_runner(product)
    r.launch_routes(0)
    r.launch_ksp(0)
    r.fetch()
    _cmp([r.routes()], oracle.gen_route_dbs_multiarea(C5_SMALL, ["abr-0"], True, False, True,
                                                       pol), "c5routes")
    dests = r.ksp_dests()
    assert len(dests) == r.shape()["total_dests"] > 300
    got, want = r.ksp_text(), oracle.kth_paths_multiarea(C5_SMALL, "abr-0", dests)
    assert len(got) == len(want)
    bad = [(g, w) for g, w in zip(got, want) if g != w]
    assert not bad, bad[:3]
    # random metrics: mostly one shortest path each; k = 2 finds the detours
    assert sum(1 for line in got if " 2: " in line) > len(dests) // 2


def test_c5_runner_sharded(product):
    """Two ranks' blocks (prefix range + destination range) reassemble the
    single-rank job exactly: no exchange is needed between ranks."""
    full, _ = _c5_runner(product)
    full.launch_ksp(0)
    full.fetch()
    parts = [_c5_runner(product, rank, 2)[0] for rank in range(2)]
    for p in parts:
        p.launch_ksp(0)
        p.fetch()
    assert parts[0].ksp_text() + parts[1].ksp_text() == full.ksp_text()
    routes = [p.routes().decode() for p in parts]
    assert routes[0] + routes[1] == full.routes().decode()


# ---- edge cases: sizes at kernel boundaries, empty / degenerate inputs ------

@pytest.mark.parametrize("n", [1, 2, 8, 9, 16, 17])
def test_grid_sizes_at_kernel_boundaries(product, oracle, n):
    """Grids of 1, 4, 64, 81, 256 and 289 nodes: single node (no links),
    exactly one / two / four 64-lane slots of the wave kernel and the first
    sizes past them (workgroup kernels), every node a source."""
    opts = dict(n=n, metricSeed=0xB0 + n, prefixSeed=n, adjOverloadPermille=30,
                nodeOverloadPermille=20, overloadSeed=n)
    srcs = [str(i) for i in range(0, n * n, max(1, (n * n) // 9))]
    for brs in (False, True):
        _cmp(product.gen_route_dbs("grid", opts, srcs, True, True, brs),
             oracle.gen_route_dbs("grid", opts, srcs, True, True, brs), f"grid{n}")


def test_long_prefix_tables(product, oracle):
    """More prefixes per topology than the wave kernel stages in registers
    (P > 64 * (NPL + 1)): the plain staging loop, anycast mix included."""
    opts = dict(n=5, metricSeed=0xB7, prefixSeed=7, prefixesPerNode=40, **MIX)
    srcs = ["0", "12", "24"]
    _cmp(product.gen_route_dbs("grid", opts, srcs, True, False, True),
         oracle.gen_route_dbs("grid", opts, srcs, True, False, True), "longpfx")


def test_unknown_source_gives_no_route_db(product, oracle):
    """buildRouteDb for a node in no area returns nullopt (SpfSolver.cpp:318-324)."""
    opts = dict(n=4, metricSeed=1, prefixSeed=1)
    a = product.gen_route_dbs("grid", opts, ["nope", "3"], True, False, False)
    b = oracle.gen_route_dbs("grid", opts, ["nope", "3"], True, False, False)
    assert a[0] == b[0] == b"NONE"
    _cmp(a, b, "unknown")


def test_empty_batch_is_a_no_op(product):
    """n_units = 0 returns OGS_OK without touching the (NULL) buffers."""
    import ctypes
    import openr_amd.capi as capi
    lib = capi.load()
    g = capi.Graph(1, 4, 8, 2, None, None, None, None, None)
    out = capi.SpfOut(None, None, None, None, None, None)
    assert lib.ogs_spf_routes(ctypes.byref(g), None, None, 0, 0, 1, ctypes.byref(out),
                              None) == 0
