#!/usr/bin/env python3
"""bench.py — SPF+RouteDb builds/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], config C2): a batch of 4096 random-metric
10x10 grid topologies (reference grid wiring, RoutingBenchmarkUtils.cpp:
209-291; per-direction metric U[1,100] seeded 0xC2000000+i, one seeded /128
prefix per node), ECMP SPF from node "1" + full RouteDb for every topology.
One "step" = one launch of the fused SPF+RouteDb kernel over the whole
batch; one "build" = one (topology, source) SPF + RouteDb. Inputs are
HBM-resident (torch-owned device buffers) before timing starts.

Multi-GPU (--gpus N via torch.distributed.run): weak scaling, each rank owns
its own 4096-topology shard (topology indices rank*4096 ...), no data-path
collective; RCCL only all-gathers per-rank digests/counts and max-reduces
the elapsed time.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# torch first: its HIP runtime must be the one libopenr_gpu.so binds to (one
# HIP runtime per process); openr_amd's import loads the engine library
import torch  # noqa: E402,F401
import numpy as np  # noqa: E402

from openr_amd import shard  # noqa: E402

TOPOS_PER_GPU = 4096
GRID_N = 10
METRIC_SEED = 0xC2000000
PREFIX_SEED = 0xC1
C3_INC_SOURCE = "2-0-0"  # a fabric node (incremental-routes sub-line)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def algorithmic_bytes_per_unit(N, E, T, P, W, Wl, S=1):
    """bytes_inputs/S + 4N + 4*W*N + P*(4*Wl + 8),
    bytes_inputs = 4(N+1) + 8E + ceil(N/8) + 16T."""
    inputs = 4 * (N + 1) + 8 * E + (N + 7) // 8 + 16 * T
    return inputs / S + 4 * N + 4 * W * N + P * (4 * Wl + 8)


def cpu_baseline(units, reps=3):
    """The oracle (refcpu, a faithful port of LinkState/SpfSolver) timed on
    this host's cores over the same workload; ingestion excluded."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import _refcpu
    threads = max(1, min(16, os.cpu_count() or 1))  # the box's CPU share
    opts = dict(n=GRID_N, metricSeed=METRIC_SEED, prefixSeed=PREFIX_SEED)
    rates = []
    for _ in range(reps):
        secs, n, routes = _refcpu.cpu_baseline_grid_batch(opts, units, threads, "1")
        rates.append(n / secs)
    rates.sort()
    return {"value": round(rates[len(rates) // 2], 1), "unit": "builds/s",
            "cores": threads, "kind": "port",
            "sample": f"{units} C2 topologies x {reps} reps (median), "
                      f"refcpu buildRouteDb('1'), {threads} threads, ingestion excluded"}


def fabric_names(pods, planes, ssw, rsw):
    """Node names of topogen::fabric (RoutingBenchmarkUtils.cpp:421-473)."""
    return ([f"1-{p}-{s}" for p in range(planes) for s in range(ssw)],
            [f"2-{p}-{f}" for p in range(pods) for f in range(planes)],
            [f"3-{p}-{r}" for p in range(pods) for r in range(rsw)])


def c3_launches(torch, M, capi, dev, rank, world, ppn, with_sel=False):
    """Host build + device upload of this rank's C3 launches: sources grouped
    by next-hop bitset width (SSW+RSW: 1 word, FSW: 3 words -> 4) so each
    launch writes masks of its own width."""
    opts = dict(pods=32, planes=8, sswPerPlane=36, rswPerPod=48, full=True,
                prefixesPerNode=ppn)
    ssw, fsw, rsw = fabric_names(32, 8, 36, 48)
    N = len(ssw) + len(fsw) + len(rsw)
    launches = []
    for names in (ssw + rsw, fsw):
        mine = shard.interleave(names, rank, world)
        br = M.BatchRunner(True, False, False)
        br.add_generated("fabric", opts, mine)
        h = br.host_arrays()
        up = lambda key, dt: torch.from_numpy(h[key].view(dt)).to(dev)  # noqa: E731
        t = {k: up(k, dt) for k, dt in (
            ("node_base", "int32"), ("row_ptr", "int32"), ("edges", "int64"),
            ("node_flags", "uint8"), ("topo_desc", "int32"), ("pfx_base", "int32"),
            ("adv_off", "int32"), ("adv_node", "int32"), ("adv_metrics", "int32"),
            ("adv_min_nh", "int64"), ("pfx_flags", "uint8"), ("units", "int32"),
            ("edge_src", "int32"))}
        U = len(h["units"]) // 2
        Sn, Sp, W = h["max_nodes"], h["max_prefixes"], h["nh_words"]
        o = dict(dist=torch.empty(U * Sn, dtype=torch.int32, device=dev),
                 nh=torch.empty(U * W * Sn, dtype=torch.int32, device=dev),
                 meta=torch.empty(U * Sp, dtype=torch.int32, device=dev),
                 metric=torch.empty(U * Sp, dtype=torch.int32, device=dev),
                 mask=torch.empty(U * W * Sp, dtype=torch.int32, device=dev))
        if with_sel:
            o["sel"] = torch.empty(U * Sp, dtype=torch.int32, device=dev)
        g = capi.Graph(h["num_topos"], Sn, h["max_edges"], h["max_degree"],
                       t["node_base"].data_ptr(), t["row_ptr"].data_ptr(),
                       t["edges"].data_ptr(), t["node_flags"].data_ptr(),
                       t["topo_desc"].data_ptr())
        g.edge_src = t["edge_src"].data_ptr()
        pt = capi.PrefixTable(Sp, h["max_advertisements"], t["pfx_base"].data_ptr(),
                              t["adv_off"].data_ptr(), t["adv_node"].data_ptr(),
                              t["adv_metrics"].data_ptr(), t["adv_min_nh"].data_ptr(),
                              t["pfx_flags"].data_ptr())
        so = capi.SpfOut(o["dist"].data_ptr(), o["nh"].data_ptr(), o["meta"].data_ptr(),
                         o["metric"].data_ptr(), o["mask"].data_ptr(),
                         o["sel"].data_ptr() if with_sel else None)
        # algorithmic bytes, inputs shared by all N sources
        E = h["max_edges"]
        P = Sp
        T = h["max_advertisements"]
        inputs = 4 * (N + 1) + 8 * E + (N + 7) // 8 + 16 * T
        rp = h["row_ptr"]
        srcs = h["units"].reshape(-1, 2)[:, 1]
        deg = rp[srcs + 1] - rp[srcs]
        wl = (deg + 31) // 32
        bpu = float((inputs / N + 4 * N + 4 * wl * N + P * (4 * wl + 8)).sum())
        launches.append(dict(br=br, h=h, t=t, o=o, g=g, pt=pt, so=so, U=U, W=W,
                             flags=h["flags"], bytes=bpu, names=mine))
    return launches, N


def hash_list(xs):
    """63-bit hash of an int list (C4 changed-prefix lists inside the digest)."""
    import hashlib
    return int.from_bytes(hashlib.sha256(repr(list(xs)).encode()).digest()[:8],
                          "little") >> 1


def pmc_traffic(tag, match):
    """HBM bytes per launch of the kernels whose name contains `match`, from
    the newest committed PMC summary profiles/r*_pmc_<tag>.json
    (tools/gpu_pmc.sh: FETCH_SIZE and WRITE_SIZE passes, gfx950 FETCH_SIZE
    x2 correction). Returns (bytes summed over matching kernels, file) or
    (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{tag}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    hits = [v["hbm_bytes_per_launch"] for k, v in d.items()
            if match in k and v.get("hbm_bytes_per_launch") is not None]
    if not hits:
        return None, None
    return float(sum(hits)), os.path.relpath(files[-1], ROOT)


def run_c3(args, torch, dist, rank, world, local_rank):
    """Config C3-full: fabric pods=32 planes=8 ssw/plane=36 rsw/pod=48
    (N=2080, E=43,008), `--prefixes-per-node` prefixes per node, every node a
    source. One step = this rank's share of the 2080 sources; one build = the
    RouteDbs of all 2080 sources."""
    import openr_amd
    import openr_amd.capi as capi
    openr_amd.require_gpu()
    M = openr_amd.decision
    lib = capi.load()
    lib.ogs_set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    steps = args.steps if args.config == "c3" else args.c3_steps
    warmup = args.warmup if args.config == "c3" else 2
    launches, N = c3_launches(torch, M, capi, dev, rank, world, args.prefixes_per_node)
    if args.c3_order == "wide-first":
        # the wide (FSW, 4-word) group has the longest units: dispatch it
        # first so it is not the lone tail after the 1-word group
        launches = launches[::-1]
    # the width groups are independent: with --c3-streams 2 the second group
    # runs on its own HIP stream, overlapped with the first
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev) if args.c3_streams > 1 else main
    streams = [main, side] + [main] * max(0, len(launches) - 2)

    def step():
        fork = torch.cuda.Event()
        fork.record(main)
        side.wait_event(fork)
        for L, st in zip(launches, streams):
            rc = lib.ogs_spf_routes(ctypes.byref(L["g"]), ctypes.byref(L["pt"]),
                                    ctypes.c_void_p(L["t"]["units"].data_ptr()), L["U"],
                                    L["flags"], L["W"], ctypes.byref(L["so"]),
                                    ctypes.c_void_p(st.cuda_stream))
            if rc != 0:
                capi.check(lib, rc, "ogs_spf_routes")
        join = torch.cuda.Event()
        join.record(side)
        main.wait_event(join)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(main)
    for _ in range(steps):
        step()
    e1.record(main)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    # device time of one whole build on this rank (all launches of a step)
    kernel_ms = e0.elapsed_time(e1) / steps
    units = sum(L["U"] for L in launches)
    nbytes = sum(L["bytes"] for L in launches)
    routes = sum(int(((L["o"]["meta"] & 1) != 0).sum().item()) for L in launches)
    # keyed by source name: the same job digest at any rank count
    digest = shard.combine_digests(
        shard.unit_digest(L["names"], L["o"]["meta"].cpu().numpy(),
                          L["o"]["metric"].cpu().numpy())
        for L in launches)
    total_units, total_routes, job_digest, tmax, _ = shard.reduce_stats(
        dist, torch, dev, units, routes, digest, wall)
    if rank == 0:
        achieved = nbytes / (kernel_ms * 1e-3) / 1e9
        value = total_units * steps / tmax / N
        line = {
            "metric": "SPF+RouteDb builds/sec (whole node)",
            "value": round(value, 4), "unit": "builds/s",
            "n_gpus": world, "steps": steps, "warmup": warmup,
            "ms_per_step": round(tmax / steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u32", "data": "synthetic",
            "config": {"workload": f"C3-full: fabric all-sources (N=2080, E=43008, "
                                   f"{args.prefixes_per_node} prefixes/node), one build = "
                                   "RouteDb of every node",
                       "sources": N, "prefixes": N * args.prefixes_per_node,
                       "parallelism": f"shard-by-source x{world}"},
            "route_dbs_per_s": round(total_units * steps / tmax, 1),
            "routes_per_step": total_routes,
            "route_digest": f"{job_digest:016x}",
            "gteps": round(43008 * total_units * steps / tmax / 1e9, 3),
            "kernel_ms": round(kernel_ms, 4),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                         "bytes_alg_per_step_rank0": round(nbytes, 1)},
        }
        # §8(f) f2, outside the timed region: the same build as a resident
        # RouteDbBatch served per node (getRouteDbComputed: D2H of one node's
        # records + host materialisation + toThrift)
        import openr_amd
        launch_ms, serve_ms, routes, ns = openr_amd.decision.route_db_batch_serve_bench(
            "fabric", dict(pods=32, planes=8, sswPerPlane=36, rswPerPod=48, full=True,
                           prefixesPerNode=args.prefixes_per_node), 3)
        line["serve"] = {"sources": ns, "batch_launch_ms": round(launch_ms, 3),
                         "getRouteDbComputed_ms": round(serve_ms, 2),
                         "routes_per_node": round(routes, 1),
                         "note": "RouteDbBatch (C++ drop-in) over all 2,080 sources, then "
                                 "3 nodes served; rank 0, after the timed region"}
        # §8(f) f4, host only: the same fabric as one KvStore publication
        # (2,080 "adj:" + 208k "prefix:" keys, compact thrift) decoded and
        # ingested per key (Decision::updateKeyInLsdb) into a fresh LSDB
        pub = openr_amd.decision.publication_ingest_bench(
            "fabric", dict(pods=32, planes=8, sswPerPlane=36, rswPerPod=48, full=True,
                           prefixesPerNode=args.prefixes_per_node), 3)
        keys = pub["adj_dbs"] + pub["prefix_keys"]
        line["publication_ingest"] = {
            "keys": keys, "bytes": pub["bytes"], "ingest_ms": round(pub["ingest_ms"], 2),
            "decode_ms": round(pub["decode_ms"], 2),
            "keys_per_s": round(keys / pub["ingest_ms"] * 1e3, 1),
            "decode_MB_per_s": round(pub["bytes"] / pub["decode_ms"] / 1e3, 1),
            "note": "LsdbIngest (C++ drop-in), 1 host thread, median of 3; rank 0, "
                    "after the timed region"}
        # §8(f) f1 incremental branch: 100 changed prefixes of node "ssw-0-0"'s
        # RouteDb in one sub-table build vs the per-prefix loop
        b_ms, l_ms, same, n_chg = openr_amd.decision.incremental_routes_bench(
            "fabric", dict(pods=32, planes=8, sswPerPlane=36, rswPerPod=48, full=True,
                           prefixesPerNode=args.prefixes_per_node), C3_INC_SOURCE, 100)
        assert same, "createRoutesForPrefixes differs from the per-prefix loop"
        line["incremental_routes"] = {"changed_prefixes": n_chg, "batch_ms": round(b_ms, 3),
                                      "per_prefix_loop_ms": round(l_ms, 2)}
        traffic, src = pmc_traffic("c3", "spf_frontier_kernel")
        if traffic is not None and world == 1:
            line["roofline"]["traffic"] = round(traffic, 1)
            line["roofline"]["traffic_source"] = src
        return line
    return None


C4_VARIANTS = 10000
C4_OPTS = dict(nodes=2000, seed=0xC4, prefixesPerNode=1)


def run_c4(args, torch, dist, rank, world, local_rank):
    """Config C4: link-failure sweep. WAN N=2000 (seed 0xC4), one prefix per
    node, source "0"; 10,000 single/dual link-removal variants (seed 0xC4F,
    50 % dual). One step = this rank's block of variants in ONE launch:
    frontier SPF without the failed links + RouteDb + route diff against the
    base RouteDb (changed-prefix bitmap + update/delete counts); one build =
    one variant. Strong scaling: the 10,000 variants split over the ranks."""
    import openr_amd
    import openr_amd.capi as capi
    openr_amd.require_gpu()
    lib = capi.load()
    lib.ogs_set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    steps = args.steps if args.config == "c4" else args.c4_steps
    warmup = args.warmup if args.config == "c4" else 2
    lo, hi = shard.block_range(C4_VARIANTS, rank, world)
    vr = openr_amd.decision.VariantRunner(True, False)
    vr.setup("wan", C4_OPTS, "0", C4_VARIANTS, 0xC4F, 500, lo, hi)
    sh = vr.shape()
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    vr.run_base(sptr)
    for _ in range(warmup):
        vr.launch(sptr, True)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        vr.launch(sptr, True)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kernel_ms = e0.elapsed_time(e1) / steps
    vr.download()
    U = vr.num_variants()
    changed = sum(len(vr.changed(v)) for v in range(U))
    counts = [vr.counts(v) for v in range(U)]
    # keyed by global variant index: the same job digest at any rank count
    digest = shard.unit_digest(
        list(range(lo, lo + U)),
        np.array([[c[0], c[1], hash_list(vr.changed(v))]
                  for v, c in enumerate(counts)], dtype="int64"))
    # §8(f) f1, outside the timed region: the DecisionRouteUpdate of every
    # variant from the device-gathered changed records (ogs_route_changes_gather
    # + D2H of those records), then host materialisation of all of them
    t1 = time.perf_counter()
    vr.fetch_updates(sptr)
    fetch_ms = (time.perf_counter() - t1) * 1e3
    t1 = time.perf_counter()
    n_changes = vr.materialize_all()
    mat_ms = (time.perf_counter() - t1) * 1e3
    assert n_changes == changed == vr.total_changes()
    # §8(f) f3, outside the timed region: one link-metric flap made current on
    # the device -- in-place CSR patch (ogs_csr_patch) vs re-flatten + upload
    csr_update = None
    if rank == 0:
        M = openr_amd.decision
        csr_update = {}
        for tag, kind, opts in (
                ("c4_wan", "wan", C4_OPTS),
                ("c3_fabric", "fabric", dict(pods=32, planes=8, sswPerPlane=36,
                                             rswPerPod=48, full=True, prefixesPerNode=1))):
            patch_us, rebuild_us, edges, flaps = M.flap_update_bench(kind, opts, 200, 0xF3)
            pub_us, n_pub, d_dev, d_fresh = M.publication_flap_bench(kind, opts, 200, 0xF3)
            assert d_dev == d_fresh, "publication-driven CSR patch diverged from a fresh flatten"
            csr_update[tag] = {"directed_edges": edges, "flaps": flaps,
                               "patch_us": round(patch_us, 2),
                               "rebuild_us": round(rebuild_us, 2),
                               "via_publication_us": round(pub_us, 2)}
    total_units, total_changed, job_digest, tmax, _ = shard.reduce_stats(
        dist, torch, dev, U, changed, digest, wall)
    if rank != 0:
        return None
    N, E, P = sh["nodes"], sh["directed_edges"], sh["prefixes"]
    T, W = sh["advertisements"], sh["nh_words"]
    inputs = 4 * (N + 1) + 8 * E + (N + 7) // 8 + 16 * T
    bpu = inputs / C4_VARIANTS + 4 * N + 4 * W * N + P * (4 * W + 8) + 16 + P / 8
    achieved = bpu * U / (kernel_ms * 1e-3) / 1e9
    value = total_units * steps / tmax
    line = {
        "metric": "link-failure variant builds/sec (SPF + RouteDb + route diff)",
        "value": round(value, 1), "unit": "variants/s",
        "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(tmax / steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "C4: 10,000 single/dual link-failure variants of a "
                               "2,000-node WAN (seed 0xC4), source '0', 1 prefix/node, "
                               "masked SPF + RouteDb + diff vs base",
                   "nodes": N, "directed_edges": E, "prefixes": P,
                   "variants": C4_VARIANTS,
                   "parallelism": f"shard-by-variant x{world}"},
        "changed_routes_per_step": total_changed, "route_digest": f"{job_digest:016x}",
        "csr_update": csr_update,
        "route_update": {
            "changes": n_changes, "gather_fetch_ms": round(fetch_ms, 3),
            "materialize_ms": round(mat_ms, 3),
            "note": "rank 0, after the timed region: counts D2H + scan + "
                    "ogs_route_changes_gather + D2H of the changed records, then host "
                    "DecisionRouteUpdate materialisation of every variant"},
        "gteps": round(E * value / 1e9, 3), "kernel_ms": round(kernel_ms, 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None, "bytes_alg_per_unit": round(bpu, 1)},
    }
    # PMC HBM bytes of the variant launch (10k units; committed passes)
    traffic, src = pmc_traffic("c4", "spf_frontier_kernel<1, true, true, true")
    if traffic is not None and world == 1:
        line["roofline"]["traffic"] = round(traffic, 1)
        line["roofline"]["traffic_source"] = src
    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import _refcpu
        threads = max(1, min(16, os.cpu_count() or 1))
        sample = 32 * threads
        secs, n, _ = _refcpu.cpu_baseline_variants("wan", C4_OPTS, "0", sample, 0xC4F, 500,
                                                   threads)
        line["cpu_baseline"] = {
            "value": round(n / secs, 2), "unit": "variants/s", "cores": threads,
            "kind": "port",
            "sample": f"first {sample} of the C4 variants, refcpu incremental "
                      f"updateAdjacencyDatabase + buildRouteDb + calculateUpdate, "
                      f"{threads} threads, ingestion excluded"}
    return line


def run_c5(args, torch, dist, rank, world, local_rank):
    """Config C5: multi-area WAN (8 areas x 1,250 nodes + 64 ABRs, ~100k
    prefixes, 5 % anycast, best-route selection), source "abr-0". One step =
    one job: the source's multi-area RouteDb + UCMP RibPolicy (SPF per area,
    route kernel, policy kernel; results left in HBM) and KSP2 (k = 1 and 2)
    for every destination of the source's two areas. Strong scaling: rank r
    owns block r of the prefix table and of the destinations."""
    import openr_amd
    import openr_amd.capi as capi
    from openr_amd.workloads import C5_OPTS, C5_SOURCE, c5_policy
    openr_amd.require_gpu()
    lib = capi.load()
    lib.ogs_set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    steps = args.steps if args.config == "c5" else args.c5_steps
    warmup = args.warmup if args.config == "c5" else 2
    r = openr_amd.decision.C5Runner()
    r.setup(C5_OPTS, C5_SOURCE, [], True, rank, world)
    # every rank holds the whole topology: the policy is the same everywhere
    pol = c5_policy(r.area_names(), r.source_neighbors())
    r.set_policy(pol)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    # the RouteDb (+ policy) and the KSP2 batch are independent: with
    # --c5-streams 2 the KSP2 launches run on a second HIP stream, overlapped
    side = torch.cuda.Stream(dev) if args.c5_streams > 1 else stream

    def job():
        fork = torch.cuda.Event()
        fork.record(stream)
        side.wait_event(fork)
        r.launch_routes(sptr)
        r.launch_ksp(side.cuda_stream)
        join = torch.cuda.Event()
        join.record(side)
        stream.wait_event(join)

    for _ in range(warmup):
        job()
    torch.cuda.synchronize(dev)
    # per-part kernel time (events on the launch stream), outside the job clock
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record(stream)
    r.launch_routes(sptr)
    ev[1].record(stream)
    r.launch_ksp(sptr)
    ev[2].record(stream)
    torch.cuda.synchronize(dev)
    route_ms, ksp_ms = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        job()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    job_ms = e0.elapsed_time(e1) / steps
    r.fetch()
    sh = r.shape()
    U = sh["ksp_units"]
    digest = r.digest() >> 1
    total_units, total_prefixes, job_digest, tmax, _ = shard.reduce_stats(
        dist, torch, dev, U, sh["prefixes"], digest, wall)
    if rank != 0:
        return None
    # KSP2 unit (CSR + E/8 mask + 4N + path output): the
    # area's CSR staged once (4(N+1) + 8E), the source's distance row (4N),
    # both path sets (4 B per path edge, 4 B per path, 4 B count each)
    Na = sh["source_area_nodes"] / 2
    Ea = sh["source_area_edges"] / 2
    pe = sh["path_edges_k1"] + sh["path_edges_k2"]
    bpu = 4 * (Na + 1) + 8 * Ea + 4 * Na + (4 * pe + 8 * 2 * U) / max(U, 1) + 8
    achieved = bpu * U / (ksp_ms * 1e-3) / 1e9
    value = steps / tmax
    line = {
        "metric": "C5 jobs/sec (multi-area RouteDb + UCMP RibPolicy + KSP2 of every "
                  "destination)",
        "value": round(value, 2), "unit": "jobs/s",
        "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(tmax / steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "C5: 8 areas x 1,250-node WAN + 64 ABRs (seed 0xC5A0), "
                               "10 prefixes/node, 5% anycast, best-route selection, "
                               "source abr-0, UCMP policy by tag, KSP2 k=1,2 to every "
                               "destination of its areas",
                   "nodes": sh["nodes"], "areas": sh["areas"],
                   "prefixes": total_prefixes, "ksp2_destinations": sh["total_dests"],
                   "parallelism": f"shard-by-prefix+destination x{world}"},
        "ksp2_dests_per_s": round(total_units * steps / tmax, 1),
        "route_kernels_ms": round(route_ms, 4), "ksp2_kernels_ms": round(ksp_ms, 4),
        "job_kernel_ms": round(job_ms, 4),
        "path_digest": f"{job_digest:016x}",
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": None, "bytes_alg_per_unit": round(bpu, 1),
                     "kernel": "ksp_base_kernel + ksp2_kernel (one launch pair over the source's areas)"},
    }
    # PMC HBM bytes per launch of both KSP kernels x the job's per-area batches
    traffic, src = pmc_traffic("c5", "ksp")
    if traffic is not None and world == 1:
        line["roofline"]["traffic"] = round(traffic * sh["ksp_batches"], 1)
        line["roofline"]["traffic_source"] = src
    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import _refcpu
        threads = max(1, min(16, os.cpu_count() or 1))
        sample = 24 * threads
        rs, ks, n, total, routes = _refcpu.cpu_baseline_c5(C5_OPTS, C5_SOURCE, pol, True,
                                                           sample, threads)
        job_s = rs + ks * total / n
        line["cpu_baseline"] = {
            "value": round(1.0 / job_s, 4), "unit": "jobs/s", "cores": threads,
            "kind": "port",
            "sample": f"refcpu buildRouteDb + RibPolicy::applyPolicy ({rs:.3f} s, 1 thread, "
                      f"{routes} routes) + getKthPaths k=1,2 for {n} of {total} "
                      f"destinations on {threads} threads ({ks:.3f} s), extrapolated to "
                      f"all destinations; ingestion excluded"}
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--prefixes-per-node", type=int, default=100)
    ap.add_argument("--c3-streams", type=int, default=2, choices=[1, 2],
                    help="C3: HIP streams for the two source groups")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--topos", type=int, default=TOPOS_PER_GPU)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c3", action="store_true",
                    help="skip the C3 fabric all-sources line embedded in the C2 result")
    ap.add_argument("--c3-steps", type=int, default=10)
    ap.add_argument("--c3-order", default="wide-first", choices=["narrow-first", "wide-first"],
                    help="C3: which next-hop width group is dispatched first")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the C4 link-failure sweep line embedded in the C2 result")
    ap.add_argument("--c4-steps", type=int, default=5)
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the C5 multi-area KSP2 + UCMP line embedded in the C2 result")
    ap.add_argument("--c5-steps", type=int, default=5)
    ap.add_argument("--c5-streams", type=int, default=2, choices=[1, 2],
                    help="C5: HIP streams (RouteDb+policy || KSP2)")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option name=value (ogs_set_option), for A/B runs")
    args = ap.parse_args()

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # OGS_BENCH_SHARE_DEVICE=1: rehearsal of the N>1 path on a box with fewer
    # GPUs than ranks (ranks share devices round-robin; gloo carries the
    # per-rank records since RCCL refuses two ranks on one GPU). Never set by
    # the driver; the numbers of such a run are not scaling numbers.
    share = os.environ.get("OGS_BENCH_SHARE_DEVICE") == "1"
    if share:
        local_rank %= torch.cuda.device_count()
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import openr_amd
    import openr_amd.capi as capi
    for o in args.opt:
        name, val = o.split("=", 1)
        lib0 = capi.load()
        capi.check(lib0, lib0.ogs_set_option(name.encode(), int(val)), name)
    if args.config in ("c4", "c5"):
        run = run_c4 if args.config == "c4" else run_c5
        line = run(args, torch, dist, rank, world, local_rank)
        if line is not None:
            print(json.dumps(line), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    if args.config == "c3":
        line = run_c3(args, torch, dist, rank, world, local_rank)
        if line is not None:
            print(json.dumps(line), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    openr_amd.require_gpu()
    M = openr_amd.decision
    lib = capi.load()
    lib.ogs_set_device(local_rank)

    # ---- build this rank's shard on the host (outside the timed region) ----
    # weak scaling: the job is world x --topos topologies, rank r owns block r
    lo, hi = shard.block_range(world * args.topos, rank, world)
    br = M.BatchRunner(True, False, False)
    br.add_grid_batch(dict(n=GRID_N, metricSeed=METRIC_SEED, prefixSeed=PREFIX_SEED),
                      lo, hi, "1")
    h = br.host_arrays()
    dev = torch.device("cuda", local_rank)

    def up(key, dtype):
        return torch.from_numpy(h[key].view(dtype)).to(dev)

    topo_desc = up("topo_desc", "int32")
    node_base = up("node_base", "int32")
    row_ptr = up("row_ptr", "int32")
    edges = up("edges", "int64")
    node_flags = up("node_flags", "uint8")
    pfx_base = up("pfx_base", "int32")
    adv_off = up("adv_off", "int32")
    adv_node = up("adv_node", "int32")
    adv_metrics = up("adv_metrics", "int32")
    adv_min_nh = up("adv_min_nh", "int64")
    pfx_flags = up("pfx_flags", "uint8")
    slot_node = up("slot_node", "uint16")
    slot_edges = up("slot_edges", "uint32")
    units = up("units", "int32")
    U = len(h["units"]) // 2
    Sn, Sp, W = h["max_nodes"], h["max_prefixes"], h["nh_words"]
    flags = h["flags"]
    assert not (flags & capi.OGS_F_WIDE_METRIC)
    o_dist = torch.empty(U * Sn, dtype=torch.int32, device=dev)
    o_nh = torch.empty(U * W * Sn, dtype=torch.int32, device=dev)
    o_meta = torch.empty(U * Sp, dtype=torch.int32, device=dev)
    o_metric = torch.empty(U * Sp, dtype=torch.int32, device=dev)
    o_mask = torch.empty(U * W * Sp, dtype=torch.int32, device=dev)
    o_sel = torch.empty(U * Sp, dtype=torch.int32, device=dev)

    g = capi.Graph(h["num_topos"], Sn, h["max_edges"], h["max_degree"], node_base.data_ptr(),
                   row_ptr.data_ptr(), edges.data_ptr(), node_flags.data_ptr(), topo_desc.data_ptr(),
                   slot_node.data_ptr(), h["slot_stride"],
                   slot_edges.data_ptr() if h["slot_degree"] else None, h["slot_degree"])
    pt = capi.PrefixTable(Sp, h["max_advertisements"], pfx_base.data_ptr(), adv_off.data_ptr(),
                          adv_node.data_ptr(), adv_metrics.data_ptr(),
                          adv_min_nh.data_ptr(), pfx_flags.data_ptr())
    out = capi.SpfOut(o_dist.data_ptr(), o_nh.data_ptr(), o_meta.data_ptr(),
                      o_metric.data_ptr(), o_mask.data_ptr(), o_sel.data_ptr())
    stream = torch.cuda.current_stream(dev)
    sptr = ctypes.c_void_p(stream.cuda_stream)
    gref, pref, oref = ctypes.byref(g), ctypes.byref(pt), ctypes.byref(out)

    def step():
        rc = lib.ogs_spf_routes(gref, pref, ctypes.c_void_p(units.data_ptr()),
                                U, flags, W, oref, sptr)
        if rc != 0:
            capi.check(lib, rc, "ogs_spf_routes")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # one launch per step

    # ---- per-rank digest (result sanity) + cross-rank reduction -----------
    meta = o_meta.cpu().numpy()
    n_routes = int(((meta & 1) != 0).sum())
    digest = shard.unit_digest(list(range(lo, hi)), meta, o_metric.cpu().numpy(),
                               o_mask.cpu().numpy())
    total_units, total_routes, job_digest, tmax, _ = shard.reduce_stats(
        dist, torch, dev, U, n_routes, digest, wall)

    if rank == 0:
        N, E, P = GRID_N * GRID_N, 4 * GRID_N * (GRID_N - 1), GRID_N * GRID_N
        bpu = algorithmic_bytes_per_unit(N, E, P, P, W, W)
        achieved = bpu * U / (kernel_ms * 1e-3) / 1e9
        value = total_units * args.steps / tmax
        line = {
            "metric": "SPF+RouteDb builds/sec (whole node)",
            "value": round(value, 1),
            "unit": "builds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {
                "workload": "C2: batch of 4096 random-metric (U[1,100]) 10x10 grid "
                            "topologies per GPU, ECMP SPF from node '1' + RouteDb "
                            "(100 prefixes/topology)",
                "topologies_per_gpu": U,
                "nodes": N, "directed_edges": E, "prefixes_per_topology": P,
                "source": "1",
                "parallelism": f"shard-by-topology x{world}",
            },
            "gteps": round(E * value / 1e9, 3),
            "kernel_ms": round(kernel_ms, 5),
            "routes_per_step": total_routes,
            "route_digest": f"{job_digest:016x}",
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None,
                "bytes_alg_per_unit": round(bpu, 1),
            },
        }
        traffic, src = pmc_traffic("c2", "spf_route_wave_kernel")
        if traffic is not None:
            line["roofline"]["traffic"] = round(traffic, 1)
            line["roofline"]["traffic_source"] = src
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(U)
    if not args.no_c3:
        # the north-star headline config, sharded by source over the ranks
        c3 = run_c3(args, torch, dist, rank, world, local_rank)
        if rank == 0:
            line["c3_fabric_all_sources"] = {
                k: c3[k] for k in ("value", "unit", "ms_per_step", "kernel_ms",
                                   "route_dbs_per_s", "gteps", "routes_per_step",
                                   "route_digest", "serve", "publication_ingest",
                                   "incremental_routes", "roofline",
                                   "config") if k in c3}
            line["c3_fabric_all_sources"]["steps"] = c3["steps"]
    if not args.no_c4:
        c4 = run_c4(args, torch, dist, rank, world, local_rank)
        if rank == 0:
            line["c4_link_failure_sweep"] = {
                k: c4[k] for k in ("value", "unit", "ms_per_step", "kernel_ms", "gteps",
                                   "changed_routes_per_step", "route_digest", "route_update", "csr_update",
                                   "roofline",
                                   "config", "steps") if k in c4}
            if "cpu_baseline" in c4:
                line["c4_link_failure_sweep"]["cpu_baseline"] = c4["cpu_baseline"]
    if not args.no_c5:
        c5 = run_c5(args, torch, dist, rank, world, local_rank)
        if rank == 0:
            line["c5_multiarea_ksp2_ucmp"] = {
                k: c5[k] for k in ("value", "unit", "ms_per_step", "ksp2_dests_per_s",
                                   "route_kernels_ms", "ksp2_kernels_ms", "job_kernel_ms",
                                   "path_digest", "roofline", "config", "steps",
                                   "cpu_baseline") if k in c5}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
