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
