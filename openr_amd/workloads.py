"""Synthetic workload definitions shared by bench.py and the tests.

Config C5: a multi-area WAN of 8 areas x
1,250 nodes (the C4 WAN generator per area, seeds 0xC5A0 + a) plus 64 ABRs
present in two areas each, 10 prefixes per node (~100k), 5 % anycast,
prefix metrics pp/sp in {100, 200} and distance U[0, 10], best-route
selection on, source "abr-0". A job = the source's multi-area RouteDb with a
UCMP RibPolicy (SpfSolver.cpp:313-453 + RibPolicy.cpp:231-249) and
getKthPaths(src, d, 1) / (src, d, 2) for every destination d of the source's
areas (LinkState.cpp:674-703).
"""
import random

# C2 (BASELINE.json configs[1]): 4096 random-metric 10x10 grids per GPU
# (topology t: metric seed 0xC2000000 + t, prefix seed 0xC1 + t), source "1"
# C1: createGrid(10) wiring, metric 1, one seeded prefix per node, source "1"
C1_OPTS = dict(n=10, prefixSeed=0xC1)
C1_SOURCE = "1"
C2_OPTS = dict(n=10, metricSeed=0xC2000000, prefixSeed=0xC1)
C2_SOURCE = "1"
C2_TOPOS = 4096

# C3-full: DecisionBenchmark fabric (RoutingBenchmarkUtils.cpp:421-473) with
# every SSW wired to its plane's FSW in every pod, 100 prefixes per node,
# every node a source
C3_OPTS = dict(pods=32, planes=8, sswPerPlane=36, rswPerPod=48, full=True,
               prefixesPerNode=100)


# C3-ref: the reference benchmark's own fabric (RoutingBenchmarkUtils.cpp:
# 298-473), including its quirk at :316-327 -- each SSW keeps only its link
# to the pod-0 FSW of its plane, so pods 1..31 have no link to the spine
# (each is an island of 8 FSWs + 48 RSWs): the parity case for unreachable
# nodes at bench size (tests/test_gpu_bench_size.py)
C3REF_OPTS = dict(pods=32, planes=8, sswPerPlane=36, rswPerPod=48, full=False,
                  prefixesPerNode=100)


def c3ref_sample_names():
    """64 stratified C3-ref sources: every 33rd of the 2,080 names (SSWs,
    pod-0 and island FSWs, pod-0 and island RSWs)."""
    return c3_source_names()[::33][:64]


def c3_source_names(pods=32, planes=8, ssw=36, rsw=48):
    """Node names of topogen::fabric: SSW "1-plane-i", FSW "2-pod-plane",
    RSW "3-pod-i"."""
    return ([f"1-{p}-{s}" for p in range(planes) for s in range(ssw)] +
            [f"2-{p}-{f}" for p in range(pods) for f in range(planes)] +
            [f"3-{p}-{r}" for p in range(pods) for r in range(rsw)])


# C4: 2,000-node WAN (seed 0xC4), one prefix per node, source "0"; 10,000
# single/dual link-failure variants (seed 0xC4F, 50 % dual)
C4_OPTS = dict(nodes=2000, seed=0xC4, prefixesPerNode=1)
C4_SOURCE = "0"
C4_VARIANTS = 10000
C4_SEED = 0xC4F
C4_DUAL_PERMILLE = 500

C5_OPTS = dict(areas=8, nodesPerArea=1250, abrs=64, k=3, seed=0xC5A0,
               prefixesPerNode=10, anycastPermille=50)
C5_SOURCE = "abr-0"


def c5_policy(areas, neighbors, seed=0xC5):
    """The C5 UCMP policy: one statement matched by the prefix tag "ucmp"
    (the generator tags about half the prefixes), set_weight {default 1,
    area_to_weight U[1, 4] per area, neighbor_to_weight U[0, 8] for 16 of the
    source's neighbours (0 drops that next hop)}, counterID "c5-ucmp"."""
    rng = random.Random(seed)
    area_w = {a: rng.randint(1, 4) for a in sorted(areas)}
    nbrs = sorted(neighbors)
    picked = sorted(rng.sample(nbrs, min(16, len(nbrs))))
    nbr_w = {n: rng.randint(0, 8) for n in picked}
    return [dict(name="c5-ucmp", tags=["ucmp"], counterID="c5-ucmp",
                 set_weight=dict(default_weight=1, area_to_weight=area_w,
                                 neighbor_to_weight=nbr_w))]

# G1 (north_star "large WAN graphs"): a single-area WAN
# past every LDS path (20,000 nodes, one prefix per node), 64 sources spread
# over the node ids, solved in one batched launch through the global-state
# SPF path (spf_global.hip).
G1_OPTS = dict(nodes=20000, seed=0x61, prefixesPerNode=1)
G1_SOURCES = [str(i * 20000 // 64) for i in range(64)]

