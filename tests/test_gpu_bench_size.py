"""Parity at the EXACT bench sizes (BASELINE.json configs C2-C5), through the
same launch paths bench.py times, against oracle-generated golden digests
(tests/golden/bench_digests.json, make_bench_digests.py) and live oracle
runs where those finish in seconds. The digest spec is
openr_amd/csrc/host/route_digest.h (RouteDbs) and openr_amd/shard.py (C4
change lists, C5 path lines)."""
import json
import os
import random

import pytest

from openr_amd import shard
from openr_amd.workloads import (C2_OPTS, C2_SOURCE, C2_TOPOS, C3_OPTS, C4_OPTS, C4_SOURCE,
                                 C4_VARIANTS, C4_SEED, C4_DUAL_PERMILLE, C5_OPTS, C5_SOURCE,
                                 c3_source_names, c5_policy)

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "bench_digests.json")))
C3_SOURCES = os.path.join(HERE, "golden", "c3_source_digests.json")


def _h(x):
    return f"{x:016x}"


def test_c2_full_batch_digest_matches_oracle_golden(product):
    """C2: 4096 topologies, one launch; the records digest of every unit
    (fast path, bench.py's) XORs to the oracle's golden block digest, and
    equals the digest of the materialised DecisionRouteDb on a sample."""
    br = product.BatchRunner(True, False, False)
    br.add_grid_batch(C2_OPTS, 0, C2_TOPOS, C2_SOURCE)
    br.upload()
    br.run()
    br.download()
    import numpy as np
    W = br.nh_words()
    h = br.host_arrays()
    Sp = h["max_prefixes"]
    meta = br.meta().astype(np.uint32)
    metric = br.metric().astype(np.uint32)  # narrow distances (C2 is u32)
    assert not br.wide()
    mask = br.mask().astype(np.uint32)
    keys = [str(t) for t in range(C2_TOPOS)]
    d = br.records_digests(keys, meta, metric, mask, W, 16)
    assert _h(shard.combine_digests(d)) == GOLDEN["c2_blocks"][0]
    for u in random.Random(2).sample(range(C2_TOPOS), 24):
        assert br.unit_digest(u, keys[u]) == d[u], u
    assert meta.shape[0] == C2_TOPOS * Sp


def _c3(product, names, ppn=100):
    """bench.py's C3 path for `names`: width-group launches on two streams."""
    import torch
    import bench
    import openr_amd.capi as capi
    lib = capi.load()
    dev = torch.device("cuda", 0)
    launches, _ = bench.c3_launches(torch, product, capi, dev, names, ppn)
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    bench.c3_launch_all(lib, capi, launches, main, side)
    torch.cuda.synchronize(dev)
    return launches


@pytest.mark.parametrize("opts", [{}, dict(route_stream=2),
                                  dict(route_stream=2, frontier_block=1024, frontier_parts=1),
                                  dict(route_stream=2, frontier_block=512, frontier_parts=3,
                                       frontier_parts_wide=5),
                                  dict(route_stream=4), dict(route_stream=4, frontier_parts=3,
                                                             frontier_parts_wide=5),
                                  dict(route_stream=5), dict(route_stream=5, lds_parts=7,
                                                             lds_grid=100),
                                  dict(route_stream=5, lds_key16=0),
                                  dict(route_stream=5, lds_tail=0),
                                  dict(route_stream=5, lds_lead=0, lds_bfs_exit=0),
                                  dict(route_stream=5, lds_parts=8, lds_grid=300),
                                  dict(route_stream=5, lds_lead=100, lds_tail_parts=16),
                                  dict(route_stream=5, lds_tail_parts=3, lds_lead=7, lds_grid=64),
                                  dict(route_stream=5, lds_pull=0),
                                  dict(route_stream=5, lds_pull=15, lds_lead=-1)])
def test_c3_full_every_source_matches_oracle(product, opts):
    """C3-full at bench size (2,080 sources x 208k prefixes) through
    bench.py's two-stream width-group launches: every source's digest equals
    the oracle's (golden per-source digests), and the job digest equals the
    golden job digest bench.py asserts; with the default launch form and
    forced ones (fused: frontier_block threads per workgroup, frontier_parts
    workgroups per unit each streaming one prefix range; route_stream 4: the
    LDS-resident SPF then the split stream; route_stream 5: both in one
    persistent launch, at several item / grid shapes)."""
    if not os.path.exists(C3_SOURCES):
        pytest.skip("oracle C3 per-source digests not generated")
    want = json.load(open(C3_SOURCES))
    names = c3_source_names()
    if len(want) != len(names):
        pytest.skip("oracle C3 per-source digests incomplete")
    assert set(want) == set(names)
    import openr_amd.capi as capi
    lib = capi.load()
    defaults = dict(frontier_block=0, frontier_parts=0, frontier_parts_wide=0, route_stream=5,
                    lds_parts=0, lds_grid=0, lds_key16=1, lds_tail=1, lds_lead=0,
                    lds_bfs_exit=1, lds_tail_parts=0, lds_pull=6)
    for k, v in opts.items():
        capi.check(lib, lib.ogs_set_option(k.encode(), v), k)
    try:
        launches = _c3(product, names)
    finally:
        for k, v in defaults.items():
            lib.ogs_set_option(k.encode(), v)
    job = 0
    bad = []
    for L in launches:
        o = L["o"]
        d = L["br"].records_digests([], o["meta"].cpu().numpy(), o["metric"].cpu().numpy(),
                                    o["mask"].cpu().numpy(), L["W"], 16)
        for n, x in zip(L["names"], d):
            job ^= x
            if _h(x) != want[n]:
                bad.append(n)
    assert not bad, f"{len(bad)} sources differ from the oracle, e.g. {bad[:8]}"
    assert _h(job) == GOLDEN["c3"]
    assert {L["W"] for L in launches} == {1, 3}  # FSW (degree 84): three mask words


@pytest.mark.parametrize("world", [8])
def test_c3_rank_shards_xor_to_golden(product, world):
    """The north_star's multi-GPU split: each of `world` ranks
    runs its shard.interleave share of the 2,080 sources as its own
    launches (bench.py --as-rank / shard_projection: c3_subset of the
    width groups). Every shard's digest equals the XOR of its sources'
    golden digests, and the shards XOR to the golden whole-build c3."""
    if not os.path.exists(C3_SOURCES):
        pytest.skip("oracle C3 per-source digests not generated")
    import torch
    import bench
    import openr_amd.capi as capi
    lib = capi.load()
    names = c3_source_names()
    dev = torch.device("cuda", 0)
    launches, _ = bench.c3_launches(torch, product, capi, dev, names)
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    job = 0
    for r in range(world):
        mine = shard.interleave(names, r, world)
        subs = [x for x in (bench.c3_subset(L, mine) for L in launches) if x is not None]
        assert sum(x["U"] for x in subs) == len(mine)
        bench.c3_launch_all(lib, capi, subs, main, side)
        torch.cuda.synchronize(dev)
        d = shard.combine_digests(bench.c3_digest(x) for x in subs)
        assert _h(d) == bench.c3_golden_shard(mine), r
        job ^= d
    assert _h(job) == GOLDEN["c3"]


def test_c3_mixed_sources_live_oracle(product, oracle):
    """12 C3 sources mixing SSW, FSW (W = 3) and RSW through the bench path,
    against a LIVE oracle buildRouteDb of each (route digests)."""
    names = c3_source_names()
    pick = ["1-0-0", "1-3-17", "1-7-35", "2-0-0", "2-13-5", "2-31-7", "3-0-0", "3-4-40",
            "3-15-11", "3-22-30", "3-31-47", "3-9-0"]
    assert set(pick) <= set(names)
    launches = _c3(product, pick)
    got = {}
    for L in launches:
        o = L["o"]
        d = L["br"].records_digests([], o["meta"].cpu().numpy(), o["metric"].cpu().numpy(),
                                    o["mask"].cpu().numpy(), L["W"], 16)
        got.update(zip(L["names"], d))
    want = oracle.gen_route_digests("fabric", C3_OPTS, pick, True, False, False, 16)
    assert [got[n] for n in pick] == list(want)


def test_c3_companion_canonical_text(product, oracle):
    """The C3 fabric with one prefix per node (P = 2,080, SURVEY §8(d)'s
    companion) for 12 mixed sources: full canonical RouteDb text equals the
    oracle's (every next hop, address, interface, metric)."""
    pick = ["1-0-0", "1-5-20", "2-0-0", "2-7-3", "2-31-7", "3-0-0", "3-16-24", "3-31-47",
            "1-7-35", "2-16-0", "3-1-1", "3-30-46"]
    opts = dict(C3_OPTS, prefixesPerNode=1)
    br = product.BatchRunner(True, False, False)
    br.add_generated("fabric", opts, pick)
    br.upload()
    br.run()
    br.download()
    a = [br.canonical(u) for u in range(len(pick))]
    b = oracle.gen_route_dbs("fabric", opts, pick, True, False, False)
    for n, x, y in zip(pick, a, b):
        assert x == y, n


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_c4_full_sweep_matches_oracle(product, oracle, mode):
    """C4 at bench size: all 10,000 variants in one launch -- full SPF per
    variant (mode 0), base-SPF repair (1) and repair writing changed records
    only (2, what bench.py times); the change-list digest equals the
    oracle's golden one, the first 600 variants' change lists equal a live
    oracle run, and the total matches."""
    vr = product.VariantRunner(True, False)
    vr.setup("wan", C4_OPTS, C4_SOURCE, C4_VARIANTS, C4_SEED, C4_DUAL_PERMILLE, 0, -1)
    vr.set_mode(mode)
    vr.run_base(0)
    vr.launch(0, True)
    vr.download()
    U = vr.num_variants()
    assert U == C4_VARIANTS
    ch = [(*vr.counts(v), vr.changed(v)) for v in range(U)]
    assert sum(len(c[2]) for c in ch) == GOLDEN["c4_changes"]
    assert _h(shard.changes_digest(range(U), ch)) == GOLDEN["c4"]
    live = oracle.variant_changes("wan", C4_OPTS, C4_SOURCE, 600, C4_SEED, C4_DUAL_PERMILLE, 16)
    for v, (u, d, prefixes) in enumerate(live):
        assert (ch[v][0], ch[v][1], sorted(ch[v][2])) == (u, d, sorted(prefixes)), v


def _c5_runner(product, rank=0, world=1):
    r = product.C5Runner()
    r.setup(C5_OPTS, C5_SOURCE, [], True, rank, world)
    pol = c5_policy(r.area_names(), r.source_neighbors())
    r.set_policy(pol)
    return r, pol


def test_c5_full_job_matches_oracle(product, oracle):
    """C5 at bench size: abr-0's multi-area RouteDb + UCMP policy (the
    enqueued device results, collected) and KSP2 k = 1, 2 of all 2,530
    destinations, against the oracle: full canonical text of the RouteDb,
    every path line, and the golden digests bench.py asserts."""
    r, pol = _c5_runner(product)
    r.launch_routes(0)
    r.launch_ksp(0)
    d = r.routes_digest(0)
    assert _h(d) == GOLDEN["c5_routes"]
    assert d == oracle.gen_route_digest_multiarea(C5_OPTS, C5_SOURCE, True, False, True, pol)
    got = r.routes()
    want = oracle.gen_route_dbs_multiarea(C5_OPTS, [C5_SOURCE], True, False, True, pol)[0]
    assert got == want
    r.fetch()
    lines = r.ksp_text()
    assert len(lines) == GOLDEN["c5_ksp_lines"] == 2 * r.shape()["total_dests"]
    ref = oracle.kth_paths_all_multiarea(C5_OPTS, C5_SOURCE, 16)
    assert sorted(lines) == sorted(ref)
    assert _h(shard.lines_digest(lines)) == GOLDEN["c5_paths"]


def test_c5_digests_rank_invariant(product):
    """Two ranks' prefix / destination blocks XOR to the single-rank digests
    (what shard.reduce_xor combines in bench.py at N > 1)."""
    full, _ = _c5_runner(product)
    full.launch_routes(0)
    full.launch_ksp(0)
    rd = full.routes_digest(0)
    full.fetch()
    pd = shard.lines_digest(full.ksp_text())
    parts = [_c5_runner(product, k, 2)[0] for k in range(2)]
    rds, pds = 0, 0
    for p in parts:
        p.launch_routes(0)
        p.launch_ksp(0)
        rds ^= p.routes_digest(0)
        p.fetch()
        pds ^= shard.lines_digest(p.ksp_text())
    assert (rds, pds) == (rd, pd)


@pytest.mark.parametrize("sr", [False, True])
def test_c1_exact_workload_canonical_text(product, oracle, sr):
    """Config C1 exactly as bench.py runs it (createGrid(10) wiring, metric
    1, prefix seed 0xC1, source "1", v4 on, best-route selection off)
    through the drop-in SpfSolver::buildRouteDb: the full canonical RouteDb
    text equals the oracle's -- also for the second build of the same
    source, which routes over the SPF memo (LinkState.cpp:705-715) -- with
    and without node segment labels."""
    from openr_amd.workloads import C1_OPTS, C1_SOURCE
    got = product.gen_route_dbs("grid", C1_OPTS, [C1_SOURCE, C1_SOURCE, "57", C1_SOURCE],
                                True, sr, False)
    want = oracle.gen_route_dbs("grid", C1_OPTS, [C1_SOURCE, C1_SOURCE, "57", C1_SOURCE],
                                True, sr, False)
    assert got == want
    assert got[0] == got[1] == got[3] and got[0] != b"NONE"


def test_c3ref_reference_fabric_at_bench_size(product, oracle):
    """C3-ref: the reference benchmark's own fabric (RoutingBenchmarkUtils.cpp
    :298-473 with the quirk at :316-327 -- every SSW keeps only its pod-0 FSW,
    so pods 1..31 are islands cut off from the spine) at bench size (2,080
    nodes, 208k prefixes), through bench.py's default one-launch form: 64
    stratified sources' digests equal the oracle's golden per-source digests
    (tests/golden/c3ref_source_digests.json), and 12 more mixing spine,
    pod-0 and island sources equal a LIVE oracle run. Exercises the
    persistent kernel's unreachable nodes (BFS layers that never reach the
    islands, no all-reached exit) at the LDS form's size."""
    from openr_amd.workloads import C3REF_OPTS, c3ref_sample_names
    path = os.path.join(HERE, "golden", "c3ref_source_digests.json")
    want = json.load(open(path))
    names = c3ref_sample_names()
    assert set(names) == set(want)
    live = ["1-0-0", "1-6-30", "2-0-0", "2-0-7", "2-1-0", "2-17-4", "2-31-7", "3-0-0",
            "3-0-47", "3-1-0", "3-20-20", "3-31-47"]
    got = {}
    for pick in (names, live):
        launches = _c3_opts(product, pick, C3REF_OPTS)
        for L in launches:
            o = L["o"]
            d = L["br"].records_digests([], o["meta"].cpu().numpy(), o["metric"].cpu().numpy(),
                                        o["mask"].cpu().numpy(), L["W"], 16)
            got.update(zip(L["names"], d))
    bad = [n for n in names if _h(got[n]) != want[n]]
    assert not bad, f"{len(bad)} sampled sources differ from the oracle, e.g. {bad[:8]}"
    ref = oracle.gen_route_digests("fabric", C3REF_OPTS, live, True, False, False, 16)
    assert [got[n] for n in live] == list(ref)


def _c3_opts(product, names, opts):
    import torch
    import bench
    import openr_amd.capi as capi
    lib = capi.load()
    dev = torch.device("cuda", 0)
    launches, _ = bench.c3_launches(torch, product, capi, dev, names, opts=opts)
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    bench.c3_launch_all(lib, capi, launches, main, side)
    torch.cuda.synchronize(dev)
    return launches
