"""Config C4 path: link-failure variants solved in one launch with the route
diff fused in (ogs_spf_routes_variants), bit-exact against the oracle's
adjacency-DB update + buildRouteDb + calculateUpdate for every variant."""
import pytest

pytestmark = pytest.mark.gpu

CASES = [
    ("wan", dict(nodes=300, seed=0xC4, prefixesPerNode=2), "0", False),
    ("wan", dict(nodes=400, seed=0xC5, prefixesPerNode=1, nodeOverloadPermille=20,
                 adjOverloadPermille=20, anycastPermille=100, minNhPermille=50,
                 v4Permille=50, drainPermille=50), "7", True),
    ("fabric", dict(pods=4, planes=4, sswPerPlane=8, rswPerPod=16, prefixesPerNode=2),
     "3-1-5", False),
    ("grid", dict(n=8, metricSeed=0xC2000003, prefixesPerNode=2), "9", False),
]


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("kind,opts,source,brs", CASES, ids=lambda x: str(x)[:12])
def test_link_failure_variants(product, oracle, kind, opts, source, brs, mode):
    """Every variant's full RouteDb, by a full SPF per variant (mode 0) and
    by repairing the base SPF below the failed tight links (mode 1,
    OGS_F_INCREMENTAL)."""
    n = 48
    vr = product.VariantRunner(True, brs)
    vr.setup(kind, opts, source, n, 0xC4F, 500)
    vr.set_mode(mode)
    vr.run_base()
    vr.launch()
    vr.download()
    base, variants, links = oracle.variant_route_updates(kind, opts, source, n, 0xC4F,
                                                         500, True, brs)
    assert vr.num_variants() == len(variants) == n
    some_change = False
    for v, (canon, changed, nu, nd) in enumerate(variants):
        got = vr.canonical(v)
        if got != canon:
            a, b = got.decode().splitlines(), canon.decode().splitlines()
            pytest.fail(f"variant {v} {links[v]}: {[(x, y) for x, y in zip(a, b) if x != y][:4]}")
        assert vr.changed(v) == changed, f"variant {v} {links[v]}"
        assert vr.counts(v) == (nu, nd), f"variant {v} {links[v]}"
        some_change |= bool(changed)
    assert some_change  # the sample exercises real route changes


def test_variants_records_optional(product):
    """Diff-only launches (no route records written) give the same diff."""
    opts = dict(nodes=300, seed=0xC4, prefixesPerNode=2)
    vr = product.VariantRunner(True, False)
    vr.setup("wan", opts, "0", 32, 0xC4F, 500)
    vr.run_base()
    vr.launch(0, True)
    vr.download()
    full = [(vr.changed(v), vr.counts(v)) for v in range(32)]
    vr.launch(0, False)
    vr.download()
    assert [(vr.changed(v), vr.counts(v)) for v in range(32)] == full


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("kind,opts,source,brs", CASES, ids=lambda x: str(x)[:12])
def test_route_updates_from_changed_records(product, oracle, kind, opts, source, brs, mode):
    """§8(f) f1: the DecisionRouteUpdate of every variant, materialised from the
    device-gathered changed records only (ogs_route_changes_gather), is
    DecisionRouteDb::calculateUpdate(base, variant) (SpfSolver.cpp:21-56):
    its update keys + deletions are exactly the changed prefixes with the
    oracle's counts, and base.update(it) (SpfSolver.cpp:58-72) is the
    oracle's variant RouteDb."""
    n = 48
    vr = product.VariantRunner(True, brs)
    vr.setup(kind, opts, source, n, 0xC4F, 500)
    vr.set_mode(mode)  # 2: repair writing changed records only (OGS_F_CHANGED_ONLY)
    vr.launch(0, True)
    vr.fetch_updates(0)
    base, variants, links = oracle.variant_route_updates(kind, opts, source, n, 0xC4F,
                                                         500, True, brs)
    assert vr.base_canonical() == base
    assert vr.total_changes() == sum(nu + nd for _, _, nu, nd in variants)
    for v, (canon, changed, nu, nd) in enumerate(variants):
        upd, dele = vr.update(v)
        assert (len(upd), len(dele)) == (nu, nd), f"variant {v} {links[v]}"
        assert sorted(upd + dele) == changed, f"variant {v} {links[v]}"
        got = vr.updated_canonical(v)
        if got != canon:
            a, b = got.decode().splitlines(), canon.decode().splitlines()
            pytest.fail(f"variant {v} {links[v]}: {[(x, y) for x, y in zip(a, b) if x != y][:4]}")


@pytest.mark.parametrize("mode", [0, 2])
def test_route_updates_c4_sample(product, oracle, mode):
    """The C4 bench workload (2,000-node WAN, seed 0xC4, source '0'): the first
    64 of its 10,000 variants, route updates vs the oracle."""
    opts = dict(nodes=2000, seed=0xC4, prefixesPerNode=1)
    vr = product.VariantRunner(True, False)
    vr.setup("wan", opts, "0", 10000, 0xC4F, 500, 0, 64)
    vr.set_mode(mode)
    vr.launch(0, True)
    vr.fetch_updates(0)
    _, variants, links = oracle.variant_route_updates("wan", opts, "0", 64, 0xC4F, 500,
                                                      True, False)
    for v, (canon, changed, nu, nd) in enumerate(variants):
        upd, dele = vr.update(v)
        assert sorted(upd + dele) == changed and (len(upd), len(dele)) == (nu, nd), v
        assert vr.updated_canonical(v) == canon, f"variant {v} {links[v]}"
    # the batch materialisation on several host threads gives the same updates
    for threads in (1, 3, 8):
        assert vr.updated_canonicals_all(threads) == [c for c, _, _, _ in variants], threads


def test_route_updates_need_records(product):
    opts = dict(nodes=120, seed=0xC4, prefixesPerNode=1)
    vr = product.VariantRunner(True, False)
    vr.setup("wan", opts, "0", 8, 0xC4F, 500)
    vr.launch(0, False)
    with pytest.raises(Exception, match="records"):
        vr.fetch_updates(0)


@pytest.mark.parametrize("ninfo", [0, -1, 1])
def test_queue_forms_node_info_option(product, oracle, ninfo):
    """The queue SPF (packed one-phase {dist, nh} words for one-word next-hop
    sets, two phases otherwise) with node info in LDS (spf_ninfo 1) or read
    from the CSR (0; -1 = whenever it raises units per CU): same variant
    RouteDbs and diffs, and the same plain RouteDbs, as the oracle."""
    import openr_amd.capi as capi
    lib = capi.load()
    kind, opts = "wan", dict(nodes=400, seed=0xC5, prefixesPerNode=1, nodeOverloadPermille=20,
                             adjOverloadPermille=20, anycastPermille=100, minNhPermille=50,
                             drainPermille=50)
    try:
        capi.check(lib, lib.ogs_set_option(b"spf_ninfo", ninfo), "spf_ninfo")
        vr = product.VariantRunner(True, True)
        vr.setup(kind, opts, "7", 32, 0xC4F, 500)
        vr.launch(0, True)
        vr.download()
        base, variants, links = oracle.variant_route_updates(kind, opts, "7", 32, 0xC4F,
                                                             500, True, True)
        for v, (canon, changed, nu, nd) in enumerate(variants):
            assert vr.canonical(v) == canon, f"variant {v} {links[v]}"
            assert vr.changed(v) == changed and vr.counts(v) == (nu, nd), v
        srcs = [str(i) for i in range(0, 400, 37)]
        got, _, _ = product.gen_route_db_batch(kind, opts, srcs, True, True, True)
        assert got == oracle.gen_route_dbs(kind, opts, srcs, True, True, True)
    finally:
        lib.ogs_set_option(b"spf_ninfo", 1)


def test_route_updates_wide_source(product, oracle):
    """A source with more than 32 links (fabric FSW: 40 SSWs + 4 RSWs -> two
    next-hop words): the gathered records carry both mask words, and the
    variants include failures of the source's own links."""
    opts = dict(pods=2, planes=2, sswPerPlane=40, rswPerPod=4, full=True, prefixesPerNode=2)
    vr = product.VariantRunner(True, False)
    vr.setup("fabric", opts, "2-0-0", 40, 0xC4F, 500)
    assert vr.shape()["nh_words"] == 2
    vr.launch(0, True)
    vr.fetch_updates(0)
    base, variants, links = oracle.variant_route_updates("fabric", opts, "2-0-0", 40, 0xC4F,
                                                         500, True, False)
    assert vr.base_canonical() == base
    own = 0
    for v, (canon, changed, nu, nd) in enumerate(variants):
        own += any("2-0-0" in (t[0], t[2]) for t in links[v])
        upd, dele = vr.update(v)
        assert sorted(upd + dele) == changed and (len(upd), len(dele)) == (nu, nd), v
        assert vr.updated_canonical(v) == canon, f"variant {v} {links[v]}"
    assert own > 0  # some variants fail the source's own links


def test_route_updates_empty_sweep(product):
    vr = product.VariantRunner(True, False)
    vr.setup("wan", dict(nodes=50, seed=3, prefixesPerNode=1), "0", 10, 0xC4F, 500, 0, 0)
    assert vr.num_variants() == 0
    vr.launch(0, True)
    vr.fetch_updates(0)
    assert vr.total_changes() == 0


def test_changed_only_launch_has_no_full_records(product):
    """OGS_F_CHANGED_ONLY leaves unchanged records unwritten: the full
    per-variant RouteDb is not available from such a launch."""
    opts = dict(nodes=200, seed=0xC4, prefixesPerNode=1)
    vr = product.VariantRunner(True, False)
    vr.setup("wan", opts, "0", 8, 0xC4F, 500)
    vr.set_mode(2)
    vr.launch(0, True)
    vr.download()
    with pytest.raises(Exception, match="fetchRecords"):
        vr.canonical(0)


def test_repair_edge_cases(product, oracle):
    """Repair on topologies with overloaded nodes / links, drained
    advertisers, anycast and minNexthop prefixes, hop-free ECMP grids
    (many tight ties) and failures of the source's own links."""
    cases = [
        ("grid", dict(n=9, metricSeed=0xC2000011, metricMax=2, prefixesPerNode=1,
                      anycastPermille=200, minNhPermille=100), "40"),
        ("wan", dict(nodes=250, seed=0xD4, prefixesPerNode=2, nodeOverloadPermille=60,
                     adjOverloadPermille=60, drainPermille=80, anycastPermille=150), "3"),
    ]
    for kind, opts, src in cases:
        n = 96
        base, variants, links = oracle.variant_route_updates(kind, opts, src, n, 0xBEE, 700,
                                                             True, True)
        for mode in (1, 2):
            vr = product.VariantRunner(True, True)
            vr.setup(kind, opts, src, n, 0xBEE, 700)
            vr.set_mode(mode)
            vr.launch(0, True)
            vr.fetch_updates(0)
            for v, (canon, changed, nu, nd) in enumerate(variants):
                upd, dele = vr.update(v)
                assert sorted(upd + dele) == changed, (kind, mode, v, links[v])
                assert vr.updated_canonical(v) == canon, (kind, mode, v, links[v])


@pytest.mark.parametrize("desc", [1, 0])
@pytest.mark.parametrize("mode", [1, 2])
def test_repair_large_wan(product, oracle, mode, desc):
    """The base-SPF repair past 8,192 nodes: a 9,500-node WAN (the repair's
    packed words, stamps, lists and affected-set bitset in 153 kB of LDS),
    with the affected sets from the descendant rows of the base tight DAG
    (9,500 x 297 words, desc 1) or grown per variant (desc 0); full records
    (mode 1) and changed records -> route updates (mode 2) vs the oracle."""
    import openr_amd.capi as capi
    lib = capi.load()
    opts = dict(nodes=9500, seed=0xC9, prefixesPerNode=1)
    n = 24
    base, variants, links = oracle.variant_route_updates("wan", opts, "5", n, 0xC4F, 500,
                                                         True, False)
    capi.check(lib, lib.ogs_set_option(b"c4_desc", desc), "c4_desc")
    try:
        vr = product.VariantRunner(True, False)
        vr.setup("wan", opts, "5", n, 0xC4F, 500)
        assert vr.shape()["nodes"] == 9500
        vr.set_mode(mode)
        vr.launch(0, True)
        if mode == 1:
            vr.download()
            for v, (canon, changed, nu, nd) in enumerate(variants):
                assert vr.canonical(v) == canon, f"variant {v} {links[v]}"
                assert vr.changed(v) == changed and vr.counts(v) == (nu, nd), v
        else:
            vr.fetch_updates(0)
            for v, (canon, changed, nu, nd) in enumerate(variants):
                upd, dele = vr.update(v)
                assert sorted(upd + dele) == changed, f"variant {v} {links[v]}"
                assert vr.updated_canonical(v) == canon, f"variant {v} {links[v]}"
    finally:
        lib.ogs_set_option(b"c4_desc", 1)
    assert any(changed for _, changed, _, _ in variants)


@pytest.mark.parametrize("first,second", [(0, 1), (1, 0), (1, 1)])
def test_repair_desc_cache_across_launches(product, oracle, first, second):
    """Two launches on ONE sweep with the descendant-row option toggled in
    between: the library reports whether it wrote the rows into
    the sweep's cache (ogs_route_diff.base_desc_valid in / out, ABI 4), so a
    launch after a c4_desc=0 launch builds them instead of reading rows
    that were never written. Both launches' route updates vs the oracle."""
    import openr_amd.capi as capi
    lib = capi.load()
    opts = dict(nodes=400, seed=0xC7, prefixesPerNode=2)
    n = 32
    _, variants, links = oracle.variant_route_updates("wan", opts, "3", n, 0xC4F, 500,
                                                      True, False)
    vr = product.VariantRunner(True, False)
    vr.setup("wan", opts, "3", n, 0xC4F, 500)
    vr.set_mode(2)
    try:
        for desc in (first, second):
            capi.check(lib, lib.ogs_set_option(b"c4_desc", desc), "c4_desc")
            vr.launch(0, True)
            vr.fetch_updates(0)
            for v, (canon, changed, nu, nd) in enumerate(variants):
                upd, dele = vr.update(v)
                assert sorted(upd + dele) == changed, (desc, v, links[v])
                assert vr.updated_canonical(v) == canon, (desc, v, links[v])
    finally:
        lib.ogs_set_option(b"c4_desc", 1)
    assert any(changed for _, changed, _, _ in variants)
