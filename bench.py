#!/usr/bin/env python3
"""bench.py — SPF+RouteDb builds/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], config C2): a batch of 4096 random-metric
10x10 grid topologies (reference grid wiring, RoutingBenchmarkUtils.cpp:
209-291; per-direction metric U[1,100] seeded 0xC2000000+i, one seeded /128
prefix per node), ECMP SPF from node "1" + full RouteDb for every topology.
One "step" = one launch of the fused SPF+RouteDb kernel over the whole
batch; one "build" = one (topology, source) SPF + RouteDb. Inputs are
HBM-resident (torch-owned device buffers) before timing starts.

The same JSON line carries sub-lines for C1 (single-source drop-in latency),
C3 (fabric all-sources), C4 (link-failure sweep) and C5 (multi-area KSP2 +
UCMP). Every config's output digest (openr_amd/csrc/host/route_digest.h,
openr_amd/shard.py) is checked against the ORACLE's digest of the same
workload (tests/golden/bench_digests.json, tests/golden/make_bench_digests.py):
a mismatch prints the line and exits non-zero.

Multi-GPU (--gpus N via torch.distributed.run): each config shards its units
over the ranks with no data-path collective; RCCL only all-gathers per-rank
digests/counts and max-reduces the elapsed time.
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
from openr_amd.workloads import (C1_OPTS, C1_SOURCE, C2_OPTS, C2_SOURCE, C2_TOPOS, C3_OPTS, C4_OPTS,  # noqa: E402
                                 C4_SOURCE, C4_VARIANTS, C4_SEED, C4_DUAL_PERMILLE,
                                 c3_source_names)

GRID_N = C2_OPTS["n"]
C3_INC_SOURCE = "2-0-0"  # a fabric FSW (incremental-routes sub-line)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CPU_REPS = 5  # BASELINE.md timing rule: median of >= 5 repetitions

# oracle-generated digests of the exact bench workloads
# (tests/golden/make_bench_digests.py); a mismatch fails the run
GOLDEN_PATH = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
GOLDEN = json.load(open(GOLDEN_PATH)) if os.path.exists(GOLDEN_PATH) else {}
DIGEST_FAILURES = []


def golden_check(line, key, got, want):
    """Records got vs the oracle's golden digest in line["golden"]; a
    mismatch is remembered and fails the run once the line is printed."""
    g = line.setdefault("golden", {})
    if want is None:
        g[key] = "n/a (no golden value for this workload)"
        return
    ok = f"{got:016x}" == want
    g[key] = "match" if ok else f"MISMATCH got {got:016x} want {want}"
    if not ok:
        DIGEST_FAILURES.append(f"{key}: got {got:016x}, oracle golden {want}")


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"bench.py [{time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cgroup_cpus():
    """CPU quota of this process's cgroup (cgroup v2 cpu.max "quota period"),
    rounded up, or None when unlimited / unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota == "max":
            return None
        return max(1, -(-int(quota) // int(period)))
    except (OSError, ValueError):
        return None


def host_cores():
    """The cores this process can actually use: its CPU affinity, capped by
    the cgroup CPU quota and the lease's OMP_NUM_THREADS share (the GPU box
    grants 16 cores while affinity and os.cpu_count() show the machine's
    256; 256 threads on a 16-core share only thrash)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = cgroup_cpus()
    if q:
        n = min(n, q)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_threads():
    return max(1, host_cores())  # T = the cores actually available


def host_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"cores": host_cores(), "affinity": aff, "cgroup_cpus": cgroup_cpus(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "machine_cpus": os.cpu_count(), "model": model}


def median(xs):
    xs = sorted(xs)
    n = len(xs)
    return xs[n // 2] if n % 2 else 0.5 * (xs[n // 2 - 1] + xs[n // 2])


def oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import _refcpu
    return _refcpu


def algorithmic_bytes_per_unit(N, E, T, P, W, Wl, S=1):
    """bytes_inputs/S + 4N + 4*W*N + P*(4*Wl + 8),
    bytes_inputs = 4(N+1) + 8E + ceil(N/8) + 16T."""
    inputs = 4 * (N + 1) + 8 * E + (N + 7) // 8 + 16 * T
    return inputs / S + 4 * N + 4 * W * N + P * (4 * Wl + 8)


def pmc_traffic(tag, match):
    """HBM bytes per launch of the kernels whose name contains `match` (a
    substring or a tuple of them), from
    the newest committed PMC summary profiles/r*_pmc_<tag>.json
    (tools/gpu_pmc.sh: FETCH_SIZE and WRITE_SIZE passes, gfx950 FETCH_SIZE
    x2 correction). Returns (bytes summed over matching kernels, file) or
    (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{tag}.json")))
    if not files:
        return None, None, None
    with open(files[-1]) as f:
        d = json.load(f)
    matches = (match,) if isinstance(match, str) else tuple(match)
    hits = [v["hbm_bytes_per_launch"] for k, v in d.items()
            if not k.startswith("_") and any(m in k for m in matches)
            and v.get("hbm_bytes_per_launch") is not None]
    if not hits:
        return None, None, None
    meta = d.get("_meta", {})
    return float(sum(hits)), os.path.relpath(files[-1], ROOT), meta.get("commit")


def set_traffic(line, tag, match, scale=1.0):
    """roofline.traffic from the committed PMC summary (per launch of the
    matching kernels, summed), with the commit that summary measured."""
    traffic, src, commit = pmc_traffic(tag, match)
    if traffic is not None:
        line["roofline"]["traffic"] = round(traffic * scale, 1)
        line["roofline"]["traffic_source"] = src
        line["roofline"]["traffic_commit"] = commit


# ----------------------------------------------------------------- C2 ---
def cpu_baseline_c2(units):
    """refcpu (a faithful port of LinkState/SpfSolver) on this host's cores
    over the C2 workload, private replicas per thread, ingestion excluded:
    median of CPU_REPS repetitions at T threads (all `units` topologies) and
    at 1 thread (512 of them)."""
    R = oracle()
    T = cpu_threads()
    rate = {}
    for threads, n in ((T, units), (1, min(units, 512))):
        rs = []
        for _ in range(CPU_REPS):
            secs, k, _ = R.cpu_baseline_grid_batch(C2_OPTS, n, threads, C2_SOURCE)
            rs.append(k / secs)
        rate[threads] = median(rs)
    return {"value": round(rate[T], 1), "unit": "builds/s", "cores": T, "kind": "port",
            "value_1thread": round(rate[1], 1), "reps": CPU_REPS, "host": host_info(),
            "sample": f"{units} C2 topologies at {T} threads, 512 at 1 thread; median of "
                      f"{CPU_REPS} reps; refcpu buildRouteDb('1'), private replicas, "
                      "ingestion excluded"}


# ----------------------------------------------------------------- C1 ---
def run_c1(args, rank):
    """Config C1 (BASELINE.json configs[0]): one buildRouteDb("1") on the
    10x10 metric-1 grid through the C++ drop-in (SpfSolver::buildRouteDb:
    flatten + uploads, the fused kernel, D2H, DecisionRouteDb
    materialisation) next to refcpu's buildRouteDb on one host thread. A
    single-unit latency, not a throughput: no roofline (the kernel is C2's
    at one unit)."""
    if rank != 0:
        return None
    import openr_amd
    reps = 21
    cold, warm, routes, d_cold, d_warm, _, _ = openr_amd.decision.build_latency_bench(
        "grid", C1_OPTS, C1_SOURCE, reps)
    out = {"unit": "us/build", "gpu_cold_us": round(median(cold), 1),
           "gpu_warm_us": round(median(warm), 1), "routes": routes, "reps": reps,
           "route_digest": f"{d_cold:016x}",
           "note": "drop-in SpfSolver::buildRouteDb('1'): cold = fresh LinkState/PrefixState/"
                   "solver (CSR flatten + H2D + kernel + D2H + materialisation), warm = same "
                   "objects again (device tables cached); median of reps"}
    # the RouteDb of the cold and the warm build vs the oracle's golden
    golden_check(out, "c1", d_cold, GOLDEN.get("c1"))
    golden_check(out, "c1_warm", d_warm, GOLDEN.get("c1"))
    if not args.no_cpu_baseline:
        n = 2 * CPU_REPS + 1
        cpu = oracle().cpu_time_build("grid", C1_OPTS, C1_SOURCE, n)
        out["cpu_baseline"] = {
            "value": round(median(cpu), 1), "unit": "us/build", "cores": 1, "kind": "port",
            "reps": n, "host": host_info(),
            "sample": "refcpu buildRouteDb('1') on a fresh replica per rep (ingestion "
                      "untimed), 1 thread, median"}
    return out


# ----------------------------------------------------------------- G1 ---
def run_g1(args, rank):
    """Row g1: the global-state SPF path on a single-area WAN
    past every LDS path -- 20,000 nodes, one prefix per node, 64 sources in
    ONE batched launch (spf_global.hip: frontier rounds with dist /
    next-hop sets / queues in HBM, then one thread per (unit, prefix)).
    Digest of the 64 RouteDbs vs the oracle's golden; refcpu beside it."""
    if rank != 0:
        return None
    import openr_amd
    from openr_amd.workloads import G1_OPTS, G1_SOURCES
    M = openr_amd.decision
    br = M.BatchRunner(True, False, False)
    br.add_generated("wan", G1_OPTS, G1_SOURCES)
    br.set_sel_output(False)  # no selection cache read here: 12 B per route (§8(d))
    br.upload()
    br.run()  # warm-up (code objects, workspace)
    reps = 5
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        br.run()  # one launch + stream sync
        times.append(time.perf_counter() - t0)
    sec = median(times)
    br.download()
    digest = shard.combine_digests(br.unit_digest(u, G1_SOURCES[u])
                                   for u in range(len(G1_SOURCES)))
    U, N = len(G1_SOURCES), G1_OPTS["nodes"]
    out = {"unit": "RouteDbs/s", "value": round(U / sec, 2), "ms_per_launch": round(sec * 1e3, 3),
           "sources": U, "nodes": N, "prefixes": N, "reps": reps,
           "route_digest": f"{digest:016x}",
           "note": "one ogs_spf_routes launch (global-state path) for 64 sources incl. "
                   "the launch-to-sync latency; median of reps"}
    # roofline of the launch (spf_global_kernel + route_global_kernel): the
    # 64 units share one topology (S = 64), each writes dist / next-hop sets
    # and its RouteDb; time = the launch's wall time
    h = br.host_arrays()
    E, W = len(h["edges"]), br.nh_words()
    bpu = algorithmic_bytes_per_unit(N, E, N, N, W, W, S=U)
    achieved = bpu * U / sec / 1e9
    out["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                       "traffic": None, "bytes_alg_per_unit": round(bpu, 1),
                       "kernel": "spf_global_lds3_kernel with the route pass fused in (one "
                                 "launch; latency bound: frontier rounds of one workgroup per "
                                 "unit)"}
    set_traffic(out, "g1", ("spf_global", "route_global_kernel"))
    # Decision's own call on this area: ONE buildRouteDb(myNode) through the
    # drop-in (Decision.cpp:912-913 -> SpfSolver.cpp:313-453), cold (fresh
    # LinkState / PrefixState / solver: flatten + uploads + launch + D2H +
    # materialisation) and warm, beside refcpu's single-thread build
    src = G1_SOURCES[0]
    sreps = 5
    if args.no_extras:  # PMC passes: only the batch launches reach the counters
        return finish_g1(out, digest, args)
    cold, warm, routes, d_cold, d_warm, s_cold, s_warm = M.build_latency_bench(
        "wan", G1_OPTS, src, sreps)
    names = ("prepare", "launch", "materialize")

    def median_rep(times, splits):
        # the median build (sreps is odd) and the drop-in's own timers
        # (decision.gpu.*_ms) of THAT build: flatten / uploads, kernels + D2H
        # (warm: the route pass over the SPF memo), host materialisation
        i = sorted(range(len(times)), key=lambda j: times[j])[len(times) // 2]
        return times[i], {k: round(v, 3) for k, v in zip(names, splits[i])}

    t_cold, sp_cold = median_rep(cold, s_cold)
    t_warm, sp_warm = median_rep(warm, s_warm)
    single = {"source": src, "unit": "ms/build", "gpu_cold_ms": round(t_cold / 1e3, 3),
              "gpu_warm_ms": round(t_warm / 1e3, 3), "routes": routes, "reps": sreps,
              "route_digest": f"{d_cold:016x}",
              "split_ms_cold": sp_cold, "split_ms_warm": sp_warm,
              "split_note": "decision.gpu.*_ms of the median build itself (the split sums "
                            "to at most its total)"}
    golden_check(single, "g1_single", d_cold, GOLDEN.get("g1_single"))
    golden_check(single, "g1_single_warm", d_warm, GOLDEN.get("g1_single"))
    if not args.no_cpu_baseline:
        cpu = oracle().cpu_time_build("wan", G1_OPTS, src, 3)
        single["cpu_baseline"] = {
            "value": round(median(cpu) / 1e3, 2), "unit": "ms/build", "cores": 1,
            "kind": "port", "reps": 3,
            "sample": f"refcpu buildRouteDb('{src}') on a fresh replica per rep, 1 thread, "
                      "median (ingestion untimed)"}
    out["single_source"] = single
    return finish_g1(out, digest, args)


def finish_g1(out, digest, args):
    """G1's golden check and refcpu baseline (run_g1's tail)."""
    from openr_amd.workloads import G1_OPTS, G1_SOURCES
    want = GOLDEN.get("g1")
    out["golden"] = "n/a" if want is None else ("match" if f"{digest:016x}" == want
                                                 else "MISMATCH")
    if want is not None and out["golden"] != "match":
        DIGEST_FAILURES.append(f"g1: {digest:016x} != golden {want}")
    if not args.no_cpu_baseline:
        R = oracle()
        T = cpu_threads()
        sample = G1_SOURCES[:2 * T]
        rates = {}
        for threads, srcs in ((T, sample), (1, G1_SOURCES[:4])):
            secs, _ = R.cpu_baseline_sources("wan", G1_OPTS, srcs, threads, CPU_REPS)
            rates[threads] = len(srcs) / median(secs)
        out["cpu_baseline"] = {
            "value": round(rates[T], 2), "unit": "RouteDbs/s", "cores": T, "kind": "port",
            "value_1thread": round(rates[1], 2), "reps": CPU_REPS, "host": host_info(),
            "sample": f"refcpu buildRouteDb of the first {len(sample)} of the 64 sources on "
                      f"{T} threads (4 on 1 thread), ingestion untimed, median"}
    return out


# ----------------------------------------------------------------- C3 ---
def c3_launches(torch, M, capi, dev, names, ppn=100, with_sel=False, opts=None):
    """Host build + device upload of the C3 launches for the sources
    `names`: grouped by next-hop bitset width (SSW+RSW: 1 word, FSW: 3 words
    -> 4) so each launch writes masks of its own width. `opts`: another
    fabric of the same naming (C3-ref, tests/test_gpu_bench_size.py)."""
    opts = dict(opts or C3_OPTS, prefixesPerNode=ppn)
    N = len(c3_source_names())
    launches = []
    fsw = [n for n in names if n.startswith("2-")]
    rest = [n for n in names if not n.startswith("2-")]
    for mine in (rest, fsw):
        if not mine:
            continue
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
        unit_bytes = inputs / N + 4 * N + 4 * wl * N + P * (4 * wl + 8)
        launches.append(dict(br=br, h=h, t=t, o=o, g=g, pt=pt, so=so, U=U, W=W,
                             flags=h["flags"], bytes=float(unit_bytes.sum()),
                             unit_bytes=unit_bytes, names=mine, rows=None))
    # the width groups are built from the same fabric: one graph / prefix
    # table serves all of them (ogs_spf_routes_groups) iff the arrays agree
    same = ("node_base", "row_ptr", "edges", "node_flags", "pfx_base", "adv_off",
            "adv_node", "adv_metrics", "adv_min_nh", "pfx_flags")
    h0 = launches[0]["h"]
    shared = all(np.array_equal(L["h"][k], h0[k]) for L in launches for k in same) and \
        all(L["flags"] == launches[0]["flags"] for L in launches)
    for L in launches:
        L["shared"] = shared
    return launches, N


def c3_subset(L, names):
    """The launch L restricted to the units of `names` (a rank's shard of
    the sources): same device inputs, a units array of those rows, outputs
    in rows 0..U-1 of L's buffers; `rows` maps them back to L's units for
    the digest. None when no unit of L is in `names`."""
    pos = {n: i for i, n in enumerate(L["names"])}
    idx = [pos[n] for n in names if n in pos]
    if not idx:
        return None
    units = L["t"]["units"].view(-1, 2)[idx].contiguous().view(-1)
    sub = dict(L, U=len(idx), bytes=float(L["unit_bytes"][idx].sum()),
               names=[L["names"][i] for i in idx], rows=idx)
    sub["t"] = dict(L["t"], units=units)
    return sub


def c3_time(lib, capi, launches, main, side, steps, warmup):
    """Device ms of one step (every width-group launch of `launches`), from
    HIP events on the launch stream over `steps` steps after `warmup`."""
    for _ in range(warmup):
        c3_launch_all(lib, capi, launches, main, side)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for _ in range(steps):
        c3_launch_all(lib, capi, launches, main, side)
    e1.record(main)
    e1.synchronize()
    return e0.elapsed_time(e1) / steps


def c3_golden_shard(names):
    """The oracle's digest of the sources `names`: XOR of their golden
    per-source digests (tests/golden/c3_source_digests.json), or None."""
    path = os.path.join(ROOT, "tests", "golden", "c3_source_digests.json")
    if not os.path.exists(path):
        return None
    want = json.load(open(path))
    if not set(names) <= set(want):
        return None
    out = 0
    for n in names:
        out ^= int(want[n], 16)
    return f"{out:016x}"


def c3_shard_projection(lib, capi, launches, main, side, world_sizes=(2, 4, 8),
                        steps=10, warmup=2):
    """North_star reports C3 at 1/2/4/8 GPUs with sources interleaved over
    the ranks. On ONE GPU: every rank r of every N runs its exact
    shard alone (the launches restricted to shard.interleave(names, r, N)),
    timed like the headline; per N the slowest rank's ms and its fraction of
    ONE GPU's HBM peak (a rank's algorithmic bytes / its ms), and the XOR of
    all N shards' digests, which must equal the golden whole-build c3."""
    names = [n for L in launches for n in L["names"]]
    order = c3_source_names()
    names = [n for n in order if n in set(names)]
    out = {}
    for N in world_sizes:
        ranks, job = [], 0
        for r in range(N):
            mine = shard.interleave(names, r, N)
            subs = [x for x in (c3_subset(L, mine) for L in launches) if x is not None]
            ms = c3_time(lib, capi, subs, main, side, steps, warmup)
            nbytes = sum(x["bytes"] for x in subs)
            d = shard.combine_digests(c3_digest(x) for x in subs)
            job ^= d
            want = c3_golden_shard(mine)
            ranks.append({"rank": r, "sources": len(mine), "ms": round(ms, 4),
                          "frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "digest": f"{d:016x}",
                          "golden": None if want is None else
                          ("match" if want == f"{d:016x}" else f"MISMATCH want {want}")})
            if want is not None and want != f"{d:016x}":
                DIGEST_FAILURES.append(f"c3 shard {r}/{N}: got {d:016x}, oracle golden {want}")
        slow = max(ranks, key=lambda x: x["ms"])
        out[str(N)] = {"slowest_rank": slow["rank"], "ms": slow["ms"], "frac": slow["frac"],
                       "min_frac": min(x["frac"] for x in ranks),
                       "builds_per_s_projected": round(1e3 / slow["ms"], 2),
                       "xor_digest": f"{job:016x}", "ranks": ranks}
        log(f"c3 shards N={N}: slowest {slow['ms']:.4f} ms (frac {slow['frac']:.3f}), "
            f"xor {job:016x}")
    return out


# C3 steps through ogs_spf_routes_groups (one call for every width group,
# the engine's one-launch form under route_stream 5) when True, else one
# ogs_spf_routes per group on two streams (--c3-launch per-group)
C3_GROUPS = [True]


def c3_launch_all(lib, capi, launches, main, side):
    """One C3 step: every width group's RouteDbs -- one ogs_spf_routes_groups
    call on `main` (the groups share the graph and prefix table: checked in
    c3_launches), or per group, the second on its own HIP stream (`side`),
    joined back into `main`."""
    if C3_GROUPS[0] and all(L.get("shared") for L in launches):
        arr = (capi.RouteGroup * len(launches))()
        for i, L in enumerate(launches):
            arr[i].units = L["t"]["units"].data_ptr()
            arr[i].n_units = L["U"]
            arr[i].nh_words = L["W"]
            arr[i].out = L["so"]
        L0 = launches[0]
        rc = lib.ogs_spf_routes_groups(ctypes.byref(L0["g"]), ctypes.byref(L0["pt"]), arr,
                                       len(launches), L0["flags"],
                                       ctypes.c_void_p(main.cuda_stream))
        if rc != 0:
            capi.check(lib, rc, "ogs_spf_routes_groups")
        return
    streams = [main, side] + [main] * max(0, len(launches) - 2)
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


def c3_digest(L, threads=16):
    """route_digest.h unit digests of one launch's records (keys = source
    names), XOR-combined. A subset launch (c3_subset) digests its rows
    0..U-1 as the units they came from."""
    o = L["o"]
    Sp, W, U = L["h"]["max_prefixes"], L["W"], L["U"]
    rows = L.get("rows")
    d = L["br"].records_digests([], o["meta"][:U * Sp].cpu().numpy(),
                                o["metric"][:U * Sp].cpu().numpy(),
                                o["mask"][:U * W * Sp].cpu().numpy(), W, threads,
                                rows if rows is not None else [])
    return shard.combine_digests(d)


C3_CPU_REPS = 5


def cpu_baseline_c3(N):
    """refcpu buildRouteDb(s) for a stratified sample of the 2,080 sources
    (every 130th name: 3 SSW, 2 FSW, 11 RSW) on T threads with private
    replicas, and 2 sources (1 SSW, 1 RSW) on 1 thread; 5 reps each (about
    2 s per rep on T threads and 4 s on one); extrapolated to whole-node
    builds/s = 1 / (mean s per source x 2080 / threads)."""
    R = oracle()
    T = cpu_threads()
    names = c3_source_names()
    out = {}
    for threads, sample in ((T, names[::130][:16]), (1, [names[0], names[-1]])):
        secs, _ = R.cpu_baseline_sources("fabric", C3_OPTS, sample, threads, C3_CPU_REPS)
        # thread-seconds per source -> whole-node builds/s at `threads`
        out[threads] = median(1.0 / (s * min(threads, len(sample)) / len(sample) * N / threads)
                              for s in secs)
    return {"value": round(out[T], 6), "unit": "builds/s", "cores": T, "kind": "port",
            "value_1thread": round(out[1], 7), "reps": C3_CPU_REPS, "host": host_info(),
            "sample": f"refcpu buildRouteDb(s) of 16 stratified sources on {T} threads and "
                      "2 (1-0-0, 3-31-47) on 1 thread, private replicas, ingestion excluded, "
                      f"median of {C3_CPU_REPS} reps, extrapolated to all 2,080 sources",
            "note": "value and value_1thread come from different source samples (degree "
                    "mixes): their ratio is not a thread-scaling measurement"}


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
    steps, warmup = args.steps, args.warmup  # C3 is the headline (or --config c3)
    ppn = args.prefixes_per_node
    # sources interleaved over ranks (balances SSW/FSW/RSW degree classes)
    shard_of = (rank, world)
    if args.as_rank:
        # rank r's exact share of an N-rank run, alone on this one GPU
        if world != 1:
            raise SystemExit("bench.py: --as-rank runs one process (no --gpus)")
        shard_of = tuple(int(x) for x in args.as_rank.split("/"))
        if not 0 <= shard_of[0] < shard_of[1]:
            raise SystemExit(f"bench.py: --as-rank {args.as_rank}: need 0 <= r < N")
    mine = shard.interleave(c3_source_names(), *shard_of)
    launches, N = c3_launches(torch, M, capi, dev, mine, ppn)
    if args.c3_order == "wide-first":
        # the wide (FSW, 4-word) group has the longest units: dispatch it
        # first so it is not the lone tail after the 1-word group
        launches = launches[::-1]
    main = torch.cuda.current_stream(dev)
    side = side_stream(torch, dev) if args.c3_streams > 1 else main

    for _ in range(warmup):
        c3_launch_all(lib, capi, launches, main, side)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(main)
    for _ in range(steps):
        c3_launch_all(lib, capi, launches, main, side)
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
    digest = shard.combine_digests(c3_digest(L) for L in launches)
    total_units, total_routes, _, tmax, _ = shard.reduce_stats(
        dist, torch, dev, units, routes, 0, wall)
    job_digest = shard.reduce_xor(dist, torch, dev, [digest])[0]
    if rank != 0:
        return None
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
                               f"{ppn} prefixes/node), one build = RouteDb of every node",
                   "sources": N, "prefixes": N * ppn,
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
    log(f"c3 timed: {kernel_ms:.4f} ms/build, digest {job_digest:016x}")
    if args.as_rank:
        r, n = shard_of
        line["metric"] = "SPF+RouteDb shard time (one rank's share, alone on one GPU)"
        line["value"] = round(kernel_ms, 4)
        line["unit"] = "ms"
        line["higher_is_better"] = False
        line["config"]["parallelism"] = f"rank {r} of {n} (interleaved sources), 1 GPU"
        line["config"]["sources"] = len(mine)
        line["shard_builds_per_s_projected"] = round(1e3 / kernel_ms, 2)
        golden_check(line, f"c3_shard_{r}_of_{n}", job_digest,
                     c3_golden_shard(mine) if ppn == 100 else None)
        return line
    golden_check(line, "c3", job_digest, GOLDEN.get("c3") if ppn == 100 else None)
    if world == 1:
        set_traffic(line, "c3", ("spf_lds_route_kernel", "lds_prep_kernel"))
        if not args.no_shard_projection:
            # the 2/4/8-GPU shards, each rank's share timed alone on this GPU
            line["shard_projection"] = c3_shard_projection(lib, capi, launches, main, side)
    # §8(f) f2, outside the timed region: the same build as a resident
    # RouteDbBatch served per node (getRouteDbComputed: D2H of one node's
    # records + host materialisation + toThrift)
    fab = dict(C3_OPTS, prefixesPerNode=ppn)
    if args.no_extras:
        return line
    launch_ms, serve_ms, nroutes, ns = M.route_db_batch_serve_bench("fabric", fab, 3)
    line["serve"] = {"sources": ns, "batch_launch_ms": round(launch_ms, 3),
                     "getRouteDbComputed_ms": round(serve_ms, 2),
                     "routes_per_node": round(nroutes, 1),
                     "note": "RouteDbBatch (C++ drop-in) over all 2,080 sources, then "
                             "3 nodes served after one untimed serve (warm process); "
                             "rank 0, after the timed region"}
    # §8(f) f4, host only: the same fabric as one KvStore publication
    # (2,080 "adj:" + 208k "prefix:" keys, compact thrift) decoded and
    # ingested per key (Decision::updateKeyInLsdb) into a fresh LSDB
    pub = M.publication_ingest_bench("fabric", fab, 3)
    keys = pub["adj_dbs"] + pub["prefix_keys"]
    line["publication_ingest"] = {
        "keys": keys, "bytes": pub["bytes"], "ingest_ms": round(pub["ingest_ms"], 2),
        "decode_ms": round(pub["decode_ms"], 2),
        "prefix_keyed_decode_ms": round(pub["prefix_keyed_decode_ms"], 2),
        "prefix_insert_ms": round(pub["prefix_insert_ms"], 2),
        # the whole publication through processPublication (key order, the
        # pending update set and perf events included)
        "process_publication_ms": round(pub["publication_ms"], 2),
        "keys_per_s": round(keys / pub["ingest_ms"] * 1e3, 1),
        "decode_MB_per_s": round(pub["bytes"] / pub["decode_ms"] / 1e3, 1),
        "note": "LsdbIngest (C++ drop-in), 1 host thread, median of 3; rank 0, "
                "after the timed region"}
    # §8(f) f1 incremental branch: 100 changed prefixes of FSW "2-0-0"'s
    # RouteDb in one sub-table build, vs the engine's per-prefix loop and vs
    # refcpu's createRouteForPrefixOrGetStaticRoute loop (SPF memo warm, as
    # in the reference's Decision::rebuildRoutes, Decision.cpp:929-938)
    b_ms, l_ms, same, n_chg, *split = M.incremental_routes_bench("fabric", fab, C3_INC_SOURCE,
                                                                 100)
    assert same, "createRoutesForPrefixes differs from the per-prefix loop"
    line["incremental_routes"] = {
        "changed_prefixes": n_chg, "batch_ms": round(b_ms, 3),
        "per_prefix_loop_ms": round(l_ms, 2),
        "batch_split_ms": dict(zip(("spf_memo", "sub_table_h2d", "launch_d2h_sync",
                                    "materialize"), (round(x, 3) for x in split)))}
    if not args.no_cpu_baseline:
        ms = [oracle().cpu_incremental_routes("fabric", fab, C3_INC_SOURCE, 100)[0]
              for _ in range(CPU_REPS)]
        line["incremental_routes"]["cpu_baseline"] = {
            "value": round(median(ms), 2), "unit": "ms", "cores": 1, "kind": "port",
            "reps": CPU_REPS,
            "sample": "refcpu createRouteForPrefixOrGetStaticRoute over the same 100 "
                      "prefixes, SPF memo warm, 1 thread, median"}
        if world == 1 and ppn == 100:
            log("c3 cpu baseline ...")
            line["cpu_baseline"] = cpu_baseline_c3(N)
            # f2 beside the reference's serving path: getRouteDbComputed
            # runs buildRouteDb(node) on the Decision thread (Decision.cpp:
            # 341-360) -- refcpu's single-source time from the same run
            # (toThrift not included: a lower bound of the reference's cost)
            one = line["cpu_baseline"].get("value_1thread")
            if one:
                line["serve"]["cpu_baseline"] = {
                    "value": round(1e3 / (one * N), 1), "unit": "ms per node", "cores": 1,
                    "kind": "port", "sample": "refcpu buildRouteDb(node) on 1 thread, from "
                    "this line's cpu_baseline (1-thread sources); toThrift excluded"}
    return line


# ----------------------------------------------------------------- C4 ---
def cpu_baseline_c4():
    """refcpu per variant: updateAdjacencyDatabase of the failed links'
    endpoints, buildRouteDb, calculateUpdate, restore -- private replicas;
    first 32*T variants on T threads and 64 on 1 thread; median of
    CPU_REPS reps."""
    R = oracle()
    T = cpu_threads()
    rate = {}
    for threads, n in ((T, 32 * T), (1, 64)):
        rs = []
        for _ in range(CPU_REPS):
            secs, k, _ = R.cpu_baseline_variants("wan", C4_OPTS, C4_SOURCE, n, C4_SEED,
                                                 C4_DUAL_PERMILLE, threads)
            rs.append(k / secs)
        rate[threads] = median(rs)
    return {"value": round(rate[T], 2), "unit": "variants/s", "cores": T, "kind": "port",
            "value_1thread": round(rate[1], 2), "reps": CPU_REPS, "host": host_info(),
            "sample": f"first {32 * T} C4 variants on {T} threads, 64 on 1 thread; refcpu "
                      "incremental updateAdjacencyDatabase + buildRouteDb + calculateUpdate, "
                      f"ingestion excluded, median of {CPU_REPS} reps"}


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
    vr.setup("wan", C4_OPTS, C4_SOURCE, C4_VARIANTS, C4_SEED, C4_DUAL_PERMILLE, lo, hi)
    # repair the base SPF below the failed tight links, write changed records
    # only (OGS_F_INCREMENTAL | OGS_F_CHANGED_ONLY; --opt-free A/B: C4_MODE=0)
    vr.set_mode(int(os.environ.get("C4_MODE", "2")))
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
    ch = [(*vr.counts(v), vr.changed(v)) for v in range(U)]
    changed = sum(len(c[2]) for c in ch)
    digest = shard.changes_digest(range(lo, lo + U), ch)
    # §8(f) f1, outside the timed region: the DecisionRouteUpdate of every
    # variant from the device-gathered changed records (ogs_route_changes_gather
    # + D2H of those records), then host materialisation of all of them
    t1 = time.perf_counter()
    vr.fetch_updates(sptr)
    fetch_ms = (time.perf_counter() - t1) * 1e3
    # host materialisation on 1 thread and on the host's cores (the build of
    # the DecisionRouteUpdates; their destruction, the consumer's, untimed)
    n_changes, mat_ms = vr.materialize_all(1)
    mat_t = cpu_threads()
    mat_ms_t = median([vr.materialize_all(mat_t)[1] for _ in range(3)])
    assert n_changes == changed == vr.total_changes()
    # §8(f) f3, outside the timed region: one link-metric flap made current on
    # the device -- in-place CSR patch (ogs_csr_patch) vs re-flatten + upload
    csr_update = None
    if rank == 0:
        M = openr_amd.decision
        csr_update = {}
        for tag, kind, opts in (("c4_wan", "wan", C4_OPTS),
                                ("c3_fabric", "fabric", dict(C3_OPTS, prefixesPerNode=1))):
            patch_us, rebuild_us, edges, flaps = M.flap_update_bench(kind, opts, 200, 0xF3)
            pub_us, n_pub, d_dev, d_fresh = M.publication_flap_bench(kind, opts, 200, 0xF3)
            assert d_dev == d_fresh, "publication-driven CSR patch diverged from a fresh flatten"
            csr_update[tag] = {"directed_edges": edges, "flaps": flaps,
                               "patch_us": round(patch_us, 2),
                               "rebuild_us": round(rebuild_us, 2),
                               "via_publication_us": round(pub_us, 2)}
    total_units, total_changed, _, tmax, _ = shard.reduce_stats(
        dist, torch, dev, U, changed, 0, wall)
    job_digest = shard.reduce_xor(dist, torch, dev, [digest])[0]
    if rank != 0:
        return None
    N, E, P = sh["nodes"], sh["directed_edges"], sh["prefixes"]
    T, W = sh["advertisements"], sh["nh_words"]
    inputs = 4 * (N + 1) + 8 * E + (N + 7) // 8 + 16 * T
    mode = vr.mode()
    if mode == 2:
        # repair: per variant the failed-edge list (16 B),
        # the changed bitmap (P/8) and counts (8), its changed records
        # (prefix-indexed meta + metric + W mask words), and -- for variants
        # that change routes, i.e. whose failed links were tight -- the base
        # SPF words it starts from (8 B/node)
        repaired = sum(1 for c in ch if c[0] or c[1])
        bpu = (inputs / C4_VARIANTS + 16 + P / 8 + 8 + changed * (8 + 4 * W) / U +
               8 * N * repaired / U)
    else:
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
            "materialize_ms_threads": round(mat_ms_t, 3), "materialize_threads": mat_t,
            "note": "rank 0, after the timed region: counts D2H + scan + "
                    "ogs_route_changes_gather + D2H of the changed records, then host "
                    "DecisionRouteUpdate materialisation of every variant on 1 thread "
                    "(materialize_ms) and on the host's cores (materialize_ms_threads, "
                    "median of 3); destruction of the updates untimed"},
        "gteps": round(E * value / 1e9, 3), "kernel_ms": round(kernel_ms, 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None, "bytes_alg_per_unit": round(bpu, 1)},
    }
    log(f"c4 timed: {kernel_ms:.4f} ms/sweep, digest {job_digest:016x}")
    golden_check(line, "c4", job_digest, GOLDEN.get("c4"))
    line["config"]["mode"] = {0: "full SPF per variant", 1: "base-SPF repair",
                              2: "base-SPF repair, changed records only"}[mode]
    if world == 1:
        # the base DAG's descendant rows (tight_desc_kernel) are built once
        # per base SPF and cached (ogs_route_diff.base_desc): not per sweep
        set_traffic(line, "c4", "spf_variant_repair_kernel<true>"
                    if mode == 2 else "spf_frontier_kernel<1, true, true, true")
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline_c4()
            # f1 beside the reference: Decision::rebuildRoutes per variant =
            # updateAdjacencyDatabase + buildRouteDb + calculateUpdate (the
            # refcpu loop measured for cpu_baseline), for all variants
            one = line["cpu_baseline"]["value_1thread"]
            line["route_update"]["cpu_baseline"] = {
                "value": round(C4_VARIANTS / one * 1e3, 1), "unit": "ms for all variants",
                "cores": 1, "kind": "port",
                "sample": "refcpu per-variant update + buildRouteDb + calculateUpdate at 1 "
                          "thread (this line's cpu_baseline), scaled to every variant"}
    return line


# ----------------------------------------------------------------- C5 ---
def cpu_baseline_c5(pol):
    """refcpu per job: buildRouteDb + RibPolicy::applyPolicy on one thread
    (one source's build is sequential in the reference) + getKthPaths k=1,2
    for a strided destination sample on T threads (24 per thread) or 1
    thread (48), extrapolated to all destinations; median of CPU_REPS."""
    from openr_amd.workloads import C5_OPTS, C5_SOURCE
    R = oracle()
    T = cpu_threads()
    out = {}
    for threads, sample in ((T, 24 * T), (1, 48)):
        rs, detail = [], None
        for _ in range(CPU_REPS):
            rsec, ksec, n, total, routes = R.cpu_baseline_c5(C5_OPTS, C5_SOURCE, pol, True,
                                                             sample, threads)
            rs.append(1.0 / (rsec + ksec * total / n))
            detail = (rsec, ksec, n, total, routes)
        out[threads] = (median(rs), detail)
    rsec, ksec, n, total, routes = out[T][1]
    return {"value": round(out[T][0], 4), "unit": "jobs/s", "cores": T, "kind": "port",
            "value_1thread": round(out[1][0], 4), "reps": CPU_REPS, "host": host_info(),
            "sample": f"refcpu buildRouteDb + RibPolicy::applyPolicy ({rsec:.3f} s, 1 thread, "
                      f"{routes} routes) + getKthPaths k=1,2 for {n} of {total} destinations on "
                      f"{T} threads ({ksec:.3f} s; 48 on 1 thread), extrapolated to all "
                      f"destinations; ingestion excluded; median of {CPU_REPS} reps"}


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
    side = side_stream(torch, dev) if args.c5_streams > 1 else stream

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
    # digests of the last timed job's results: its RouteDb (device records
    # downloaded + materialised) and its KSP2 paths
    routes_digest = r.routes_digest(sptr)
    r.fetch()
    paths_digest = shard.lines_digest(r.ksp_text())
    sh = r.shape()
    U = sh["ksp_units"]
    total_units, total_prefixes, _, tmax, _ = shard.reduce_stats(
        dist, torch, dev, U, sh["prefixes"], 0, wall)
    routes_job, paths_job = shard.reduce_xor(dist, torch, dev, [routes_digest, paths_digest])
    if rank != 0:
        return None
    # KSP2 unit: the shared inputs counted once per batch
    # that shares them -- the source area's CSR (4(N+1) + 8E + N/8) / S with
    # S = the destinations of the job -- plus the unit's own E/8 link mask,
    # 4N distance row and path output (4 B per path edge, 4 B per path,
    # 4 B count, for k = 1 and k = 2)
    Na = sh["source_area_nodes"] / 2
    Ea = sh["source_area_edges"] / 2
    pe = sh["path_edges_k1"] + sh["path_edges_k2"]
    shared = 2 * (4 * (Na + 1) + 8 * Ea + Na / 8)  # both areas of the source
    bpu = (shared / max(U, 1) + Ea / 8 + 4 * Na + (4 * pe + 8 * 2 * U) / max(U, 1) + 8)
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
        # (route + KSP2 kernel time) / job time: 2.0 = perfect two-stream
        # overlap of equal parts, 1.0 = the parts run back to back
        "overlap": round((route_ms + ksp_ms) / job_ms, 3) if job_ms > 0 else None,
        "route_digest": f"{routes_job:016x}", "path_digest": f"{paths_job:016x}",
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": None, "bytes_alg_per_unit": round(bpu, 1),
                     "kernel": "ksp_base_kernel + ksp2_kernel (one launch pair over the "
                               "source's areas)"},
    }
    log(f"c5 timed: {job_ms:.4f} ms/job (route {route_ms:.4f} + ksp2 {ksp_ms:.4f} ms, "
        f"overlap {line['overlap']})")
    golden_check(line, "c5_routes", routes_job, GOLDEN.get("c5_routes"))
    golden_check(line, "c5_paths", paths_job, GOLDEN.get("c5_paths"))
    if world == 1:
        # PMC HBM bytes per launch of both KSP kernels x the job's per-area batches
        set_traffic(line, "c5", "ksp", sh["ksp_batches"])
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline_c5(pol)
    return line


# --------------------------------------------------------------- main ---
DIST_BACKEND = [None]  # the process group the per-rank records went through
# The second HIP stream of the C3 / C5 steps. A HIP stream is bound to one of
# the process's GPU_MAX_HW_QUEUES (4) hardware queues at its FIRST dispatch,
# and RCCL's communicator init dispatches on its own streams. When the
# launch stream and the side stream were first used after that, both landed
# on the same hardware queue (kernel trace: null stream and side stream on
# queue 4, RCCL's streams on 2 and 4; without the group queues 1 and 2) and
# the C5 job's two streams ran back to back: 0.69 vs 0.47 ms per job
# (profiles/r06_c5_queue_trace.log). main() therefore dispatches once on both
# streams BEFORE the process group exists (--early-streams 1).
SIDE = {}


def side_stream(torch, dev, priority=0):
    key = (dev.index, priority)
    if key not in SIDE:
        SIDE[key] = torch.cuda.Stream(dev, priority=priority)
    return SIDE[key]


PERF_FLOOR_PATH = os.path.join(ROOT, "tests", "golden", "perf_floor.json")


def _dig(d, path):
    for k in path:
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return d if isinstance(d, (int, float)) else None


def perf_summary(line):
    """Every sub-line figure as ONE compact stderr line (the driver's record
    keeps the stderr tail, not the sub-lines), then a PERF-REGRESSION line per
    figure past its committed floor (tests/golden/perf_floor.json: the best
    driver / builder figures with a tolerance). The result goes into
    line["perf_check"]; a regression is reported, it does not fail the run."""
    floor = {}
    if os.path.exists(PERF_FLOOR_PATH):
        with open(PERF_FLOOR_PATH) as f:
            floor = {k: v for k, v in json.load(f).items() if not k.startswith("_")}
    figs, bad = [], []
    for name, spec in floor.items():
        got = _dig(line, spec["path"])
        if got is None:
            continue
        figs.append(f"{name}={got:g}")
        lim, worse = (spec["max"], got > spec["max"]) if "max" in spec else \
            (spec["min"], got < spec["min"])
        if worse:
            bad.append((name, got, lim, "max" if "max" in spec else "min"))
    gold = line.get("golden", {})
    ok = sum(1 for v in gold.values() if v == "match")
    figs.append(f"golden={ok}/{len(gold)}")
    log("SUMMARY " + " ".join(figs))
    for name, got, lim, kind in bad:
        print(f"PERF-REGRESSION: {name} = {got:g} (floor {kind} {lim:g}, "
              f"tests/golden/perf_floor.json)", file=sys.stderr, flush=True)
    line["perf_check"] = {"floor": os.path.relpath(PERF_FLOOR_PATH, ROOT),
                          "checked": len(figs) - 1,
                          "regressions": [f"{n}={g:g} vs {k} {lim:g}" for n, g, lim, k in bad]}


def finish(line):
    line["collectives"] = {"backend": DIST_BACKEND[0], "use": "per-rank record all-gather + "
                           "MAX elapsed only (no data-path exchange)"}
    print(json.dumps(line), flush=True)
    if DIGEST_FAILURES:
        for f in DIGEST_FAILURES:
            print(f"bench.py: DIGEST MISMATCH vs oracle golden: {f}", file=sys.stderr,
                  flush=True)
        raise SystemExit(1)


# ----------------------------------------------------------------- C2 ---
def run_c2(args, torch, dist, rank, world, local_rank):
    """Config C2 (BASELINE.json configs[1]): a batch of 4096 random-metric
    10x10 grid topologies per GPU (weak scaling: rank r owns block r), ECMP
    SPF from node "1" + full RouteDb for each; one step = one launch of the
    fused wave kernel over the batch; one build = one (topology, source)
    SPF + RouteDb."""
    import openr_amd
    import openr_amd.capi as capi
    steps = args.steps if args.config == "c2" else args.c2_steps
    warmup = args.warmup if args.config == "c2" else args.c2_warmup
    openr_amd.require_gpu()
    M = openr_amd.decision
    lib = capi.load()
    lib.ogs_set_device(local_rank)

    # ---- build this rank's shard on the host (outside the timed region) ----
    # weak scaling: the job is world x --topos topologies, rank r owns block r
    lo, hi = shard.block_range(world * args.topos, rank, world)
    br = M.BatchRunner(True, False, False)
    br.add_grid_batch(C2_OPTS, lo, hi, C2_SOURCE)
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

    g = capi.Graph(h["num_topos"], Sn, h["max_edges"], h["max_degree"], node_base.data_ptr(),
                   row_ptr.data_ptr(), edges.data_ptr(), node_flags.data_ptr(), topo_desc.data_ptr(),
                   slot_node.data_ptr(), h["slot_stride"],
                   slot_edges.data_ptr() if h["slot_degree"] else None, h["slot_degree"])
    pt = capi.PrefixTable(Sp, h["max_advertisements"], pfx_base.data_ptr(), adv_off.data_ptr(),
                          adv_node.data_ptr(), adv_metrics.data_ptr(),
                          adv_min_nh.data_ptr(), pfx_flags.data_ptr())
    # no selection bits: BatchRunner-style consumers read them only for
    # bestRoutesCache (not part of the §8(d) output bytes)
    out = capi.SpfOut(o_dist.data_ptr(), o_nh.data_ptr(), o_meta.data_ptr(),
                      o_metric.data_ptr(), o_mask.data_ptr(), None)
    stream = torch.cuda.current_stream(dev)
    sptr = ctypes.c_void_p(stream.cuda_stream)
    gref, pref, oref = ctypes.byref(g), ctypes.byref(pt), ctypes.byref(out)

    def step():
        rc = lib.ogs_spf_routes(gref, pref, ctypes.c_void_p(units.data_ptr()),
                                U, flags, W, oref, sptr)
        if rc != 0:
            capi.check(lib, rc, "ogs_spf_routes")

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / steps  # one launch per step

    # ---- digest of the timed launches' records + cross-rank reduction -----
    meta = o_meta.cpu().numpy()
    n_routes = int(((meta & 1) != 0).sum())
    digest = shard.combine_digests(br.records_digests(
        [str(t) for t in range(lo, hi)], meta, o_metric.cpu().numpy(), o_mask.cpu().numpy(),
        W, 16))
    total_units, total_routes, _, tmax, _ = shard.reduce_stats(
        dist, torch, dev, U, n_routes, 0, wall)
    job_digest = shard.reduce_xor(dist, torch, dev, [digest])[0]

    line = None
    if rank == 0:
        N, E, P = GRID_N * GRID_N, 4 * GRID_N * (GRID_N - 1), GRID_N * GRID_N
        bpu = algorithmic_bytes_per_unit(N, E, P, P, W, W)
        achieved = bpu * U / (kernel_ms * 1e-3) / 1e9
        value = total_units * steps / tmax
        line = {
            "metric": "SPF+RouteDb (topology, source) builds/sec",
            "value": round(value, 1),
            "unit": "builds/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": round(tmax / steps * 1e3, 4),
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
                "source": C2_SOURCE,
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
        blocks = GOLDEN.get("c2_blocks", [])
        want = None
        if args.topos == GOLDEN.get("c2_block_size") and world <= len(blocks):
            want = f"{shard.combine_digests(int(b, 16) for b in blocks[:world]):016x}"
        log(f"c2 timed: {kernel_ms * 1e3:.2f} us/launch, digest {job_digest:016x}")
        golden_check(line, "c2", job_digest, want)
        set_traffic(line, "c2", "spf_route_wave_kernel")
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline_c2(U)
            log("c2 cpu baseline done")
    return line


SUB_KEYS = {
    "c2_topology_batch": ("metric", "value", "unit", "ms_per_step", "kernel_ms", "gteps",
                          "routes_per_step", "route_digest", "golden", "roofline",
                          "cpu_baseline", "config", "steps", "warmup"),
    "c4_link_failure_sweep": ("value", "unit", "ms_per_step", "kernel_ms", "gteps",
                              "changed_routes_per_step", "route_digest", "golden",
                              "route_update", "csr_update", "roofline", "cpu_baseline",
                              "config", "steps"),
    "c5_multiarea_ksp2_ucmp": ("value", "unit", "ms_per_step", "ksp2_dests_per_s",
                               "route_kernels_ms", "ksp2_kernels_ms", "job_kernel_ms",
                               "overlap",
                               "route_digest", "path_digest", "golden", "roofline",
                               "config", "steps", "cpu_baseline"),
}


def launch_ranks(args):
    """`--gpus N` without a torch.distributed launcher around us: start N
    ranks as CHILD processes (torch.distributed.run, 127.0.0.1) and exit with
    their status. Runs before anything touches the GPU; this process never
    initialises HIP and never execs."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"--gpus {args.gpus}: launching {args.gpus} ranks")
    return subprocess.call(cmd)


def check_world(args, world):
    """The rank count must be the --gpus count: never silently measure fewer
    GPUs than asked for."""
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        raise SystemExit(2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="all",
                    choices=["all", "c1", "c2", "c3", "c4", "c5", "g1"],
                    help="all (default): the C3 headline line with the C1/C2/G1/C4/C5 "
                         "sub-lines; cN: that config alone as the line")
    ap.add_argument("--prefixes-per-node", type=int, default=100)
    ap.add_argument("--c3-streams", type=int, default=2, choices=[1, 2],
                    help="C3: HIP streams for the two source groups")
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without a launcher bench.py starts them")
    ap.add_argument("--steps", type=int, default=20, help="timed steps of the headline line")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--topos", type=int, default=C2_TOPOS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the f1-f4 sub-lines run after the timed regions (PMC "
                         "passes: only the timed launches reach the counters)")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 single-source line")
    ap.add_argument("--no-g1", action="store_true",
                    help="skip the 20,000-node WAN sub-line (global-state SPF path)")
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 topology-batch sub-line")
    ap.add_argument("--host-lines-last", action="store_true",
                    help="run the C1 / G1 single-source host builds after the C3 line and its "
                         "host sub-lines (A/B of the heap state they leave; default: before)")
    ap.add_argument("--c2-steps", type=int, default=50)
    ap.add_argument("--c2-warmup", type=int, default=5)
    ap.add_argument("--as-rank", default=None, metavar="r/N",
                    help="C3: time rank r's interleaved share of an N-rank run alone "
                         "on this GPU (the line reports that shard)")
    ap.add_argument("--no-shard-projection", action="store_true",
                    help="C3 at N=1: skip the per-rank shard timings for N=2/4/8")
    ap.add_argument("--c3-launch", default="groups", choices=["groups", "per-group"],
                    help="C3 width groups through one ogs_spf_routes_groups call (default) "
                         "or one ogs_spf_routes per group on two streams")
    ap.add_argument("--c3-order", default="wide-first", choices=["narrow-first", "wide-first"],
                    help="C3: which next-hop width group is dispatched first")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 link-failure sub-line")
    ap.add_argument("--c4-steps", type=int, default=5)
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 multi-area sub-line")
    ap.add_argument("--c5-steps", type=int, default=5)
    ap.add_argument("--c5-streams", type=int, default=2, choices=[1, 2],
                    help="C5: HIP streams (RouteDb+policy || KSP2)")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option name=value (ogs_set_option), for A/B runs")
    ap.add_argument("--dist", default="auto", choices=["auto", "nccl", "none"],
                    help="process group: auto (default) RCCL ('nccl') at every world size, "
                         "so the N=1 line takes the N>1 collective path too (gloo when "
                         "ranks share a device); nccl the same; none only at N=1: no group")
    ap.add_argument("--early-streams", type=int, default=1, choices=[0, 1],
                    help="first dispatch on the launch and side streams before the process "
                         "group (1, default: their own hardware queues) or when first used "
                         "(0: after RCCL's streams; A/B)")
    ap.add_argument("--launch-check", action="store_true",
                    help="only join the process group and print the rank map (no GPU)")
    args = ap.parse_args()
    C3_GROUPS[0] = args.c3_launch == "groups"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    check_world(args, world)
    if args.launch_check:
        # CPU check of the launcher path: gloo group, all-gather of ranks
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group("gloo")
        t = torch.tensor([rank, local_rank], dtype=torch.int64)
        got = [torch.zeros_like(t) for _ in range(world)]
        if world > 1:
            dist.all_gather(got, t)
            dist.destroy_process_group()
        else:
            got = [t]
        if rank == 0:
            print(json.dumps({"world": world, "ranks": [g.tolist() for g in got]}), flush=True)
        return
    # OGS_BENCH_SHARE_DEVICE=1: rehearsal of the N>1 path on a box with fewer
    # GPUs than ranks (ranks share devices round-robin; gloo carries the
    # per-rank records since RCCL refuses two ranks on one GPU). Never set by
    # the driver; the numbers of such a run are not scaling numbers.
    share = os.environ.get("OGS_BENCH_SHARE_DEVICE") == "1"
    ndev = torch.cuda.device_count()
    if share:
        local_rank %= max(1, ndev)
    elif world > 1 and local_rank >= ndev:
        print(f"bench.py: rank {rank} needs GPU {local_rank}, {ndev} visible", file=sys.stderr)
        raise SystemExit(2)
    torch.cuda.set_device(local_rank)
    if args.early_streams:
        # the launch stream and the side stream take their hardware queues
        # (first dispatch) before RCCL's streams exist (see SIDE)
        d0 = torch.device("cuda", local_rank)
        for st in (torch.cuda.current_stream(d0), side_stream(torch, d0)):
            with torch.cuda.stream(st):
                torch.zeros(1, device=d0)
        torch.cuda.synchronize(d0)
    dist = None
    if world > 1 and args.dist == "none":
        print("bench.py: --dist none needs a single rank", file=sys.stderr)
        raise SystemExit(2)
    if world > 1 or args.dist != "none":
        # RCCL carries the per-rank records (shard.reduce_stats / reduce_xor)
        # at every world size: the N=1 line runs the same collective code as
        # N=8 (tests/test_gpu_rccl.py). A single rank without a launcher
        # rendezvous on 127.0.0.1 itself.
        import torch.distributed as dist
        init = {}
        if "MASTER_ADDR" not in os.environ:
            import socket
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                init = dict(init_method=f"tcp://127.0.0.1:{sk.getsockname()[1]}",
                            rank=rank, world_size=world)
        if share:
            dist.init_process_group("gloo", **init)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), **init)
        DIST_BACKEND[0] = dist.get_backend()

    import openr_amd
    import openr_amd.capi as capi
    openr_amd.require_gpu()
    for o in args.opt:
        name, val = o.split("=", 1)
        lib0 = capi.load()
        capi.check(lib0, lib0.ogs_set_option(name.encode(), int(val)), name)
    single = {"c2": run_c2, "c3": run_c3, "c4": run_c4, "c5": run_c5,
              "c1": lambda a, t, d, r, w, lr: run_c1(a, r),
              "g1": lambda a, t, d, r, w, lr: run_g1(a, r)}.get(args.config)
    if single is not None:
        line = single(args, torch, dist, rank, world, local_rank)
        if dist:
            dist.destroy_process_group()
        if line is not None:
            finish(line)
        elif DIGEST_FAILURES:
            raise SystemExit(1)
        return

    # the single-source host builds (C1, G1: the drop-in's materialisation of
    # std::map / std::string routes) run first by default: after the C3 host
    # sub-lines (hundreds of MB of route maps built and freed) the same G1
    # build measures 17-21 ms instead of 11 (heap state, not the build;
    # profiles/r05_g1_heap_ab.log, --host-lines-last)
    host = {}

    def host_lines():
        if rank != 0:
            return
        if not args.no_c1:
            host["c1_single_source"] = run_c1(args, rank)
        if not args.no_g1:
            log("g1 large WAN ...")
            host["g1_large_wan"] = run_g1(args, rank)

    if not args.host_lines_last:
        host_lines()
    # headline: the north-star config, C3 fabric all-sources (whole-node
    # builds/s), sources sharded over the ranks; sub-lines after it
    line = run_c3(args, torch, dist, rank, world, local_rank)
    if not args.no_c2:
        c2 = run_c2(args, torch, dist, rank, world, local_rank)
        if rank == 0:
            line["c2_topology_batch"] = {k: c2[k] for k in SUB_KEYS["c2_topology_batch"]
                                         if k in c2}
    if args.host_lines_last:
        host_lines()
    if rank == 0:
        line.update(host)
    if not args.no_c4:
        c4 = run_c4(args, torch, dist, rank, world, local_rank)
        if rank == 0:
            line["c4_link_failure_sweep"] = {k: c4[k] for k in SUB_KEYS["c4_link_failure_sweep"]
                                             if k in c4}
    if not args.no_c5:
        c5 = run_c5(args, torch, dist, rank, world, local_rank)
        if rank == 0:
            line["c5_multiarea_ksp2_ucmp"] = {k: c5[k] for k in SUB_KEYS["c5_multiarea_ksp2_ucmp"]
                                              if k in c5}
    if dist:
        dist.destroy_process_group()
    if rank == 0:
        # sub-line digest results roll up into the headline line's golden map
        for sub in ("c2_topology_batch", "c1_single_source", "g1_large_wan",
                    "c4_link_failure_sweep", "c5_multiarea_ksp2_ucmp"):
            g = (line.get(sub) or {}).get("golden", {})
            if isinstance(g, dict):
                for k, v in g.items():
                    line["golden"][k] = v
            elif sub == "g1_large_wan":
                line["golden"]["g1"] = g
        for k, v in ((line.get("g1_large_wan") or {}).get("single_source") or {}).get(
                "golden", {}).items():
            line["golden"][k] = v
        perf_summary(line)
        finish(line)
    elif DIGEST_FAILURES:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
