"""KSP2 (LinkState::getKthPaths, LinkState.cpp:674-703, and its greedy
traceOnePath, 226-247) in the domains the LDS-resident KSP kernels of
ksp.hip do not hold, through the HBM-state path:

* zero and negative link metrics -- pathLinks then follow the reference's
  extraction order (runSpf, LinkState.cpp:720-820: a link joins pathLinks(v)
  only if its other end was settled first), which the device replays
  (OGS_F_EXACT_ORDER);
* topologies past the LDS budget: the reference's 99x99 GridTopology stress
  grid (SpfSolverTest.cpp:2858-2873, source "523") and a 16k-node grid;
* every small case again with the "ksp_hbm" option forcing the HBM path.

Both the single getKthPaths call (k = 1, 2, 3: masked reruns) and the
batched prefetchKthPaths (Ksp2Batch: k = 1 and 2 in one launch pair) are
compared path for path with the oracle's getKthPaths. Before this path the
drop-in threw std::domain_error for all of these."""
import random

import pytest

import lsdb as L

pytestmark = pytest.mark.gpu


class _Hbm:
    """Forces (on=1) or leaves automatic (on=0) the HBM-state KSP path."""

    def __init__(self, on):
        import openr_amd.capi as capi
        self.lib, self.on = capi.load(), on

    def __enter__(self):
        import openr_amd.capi as capi
        capi.check(self.lib, self.lib.ogs_set_option(b"ksp_hbm", self.on), "ksp_hbm")

    def __exit__(self, *a):
        self.lib.ogs_set_option(b"ksp_hbm", 0)


def _grid(M, n, seed, metrics, parallel=False, overload=()):
    """n x n grid; each link's metric drawn from `metrics` (both directions
    may differ: the link's max metric counts, LinkState.h:171-174); optional
    parallel links and hard-drained nodes."""
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
                        key = (node, nb, k)
                        metric.setdefault(key, r.choice(metrics))
                        adjs.append(L.createAdjacency(
                            str(nb), f"if{node}-{nb}-{k}", f"if{nb}-{node}-{k}",
                            f"fe80::{nb}", f"10.0.0.{nb % 250}", metric[key], 100 + nb))
            ls.updateAdjacencyDatabase(
                L.createAdjDb(str(node), adjs, node + 1, node in overload),
                L.kTestingAreaName)
    return als, ls


def _paths(ls, s, d, k):
    return [[(l["n1"], l["if1"], l["n2"], l["if2"]) for l in p] for p in ls.getKthPaths(s, d, k)]


def _pairs(n, count, seed):
    rng = random.Random(seed)
    return [(str(rng.randrange(n * n)), str(rng.randrange(n * n))) for _ in range(count)]


def _check_single(pls, ols, pairs, ks=(1, 2, 3)):
    for s, d in pairs:
        for k in ks:
            assert _paths(pls, s, d, k) == _paths(ols, s, d, k), (s, d, k)


def _check_batch(pls, ols, src, dests):
    pls.prefetchKthPaths(src, dests)
    found = 0
    for d in dests:
        for k in (1, 2):
            got = _paths(pls, src, d, k)
            assert got == _paths(ols, src, d, k), (src, d, k)
            found += len(got)
    assert found > 0  # non-trivial: some destinations have paths


SPECIAL = [
    ("zero", [0, 0, 1, 2, 3]),
    ("zero_only", [0]),
    ("negative", [1, 2, 3, -1, -7]),
    ("mixed", [0, 1, 2, -2]),
]


@pytest.mark.parametrize("name,metrics", SPECIAL)
def test_special_metrics_single_calls(product, oracle, name, metrics):
    n = 6
    pa, pls = _grid(product, n, 11, metrics)
    oa, ols = _grid(oracle, n, 11, metrics)
    _check_single(pls, ols, _pairs(n, 20, 1))


@pytest.mark.parametrize("name,metrics", SPECIAL)
def test_special_metrics_batch(product, oracle, name, metrics):
    n = 6
    pa, pls = _grid(product, n, 12, metrics, overload={8, 20})
    oa, ols = _grid(oracle, n, 12, metrics, overload={8, 20})
    _check_batch(pls, ols, "14", [str(i) for i in range(n * n)])


def test_special_metrics_multigraph(product, oracle):
    """Parallel links: the engine and the oracle share the canonical link
    order (the reference's folly-hash order is unpinned)."""
    n = 5
    pa, pls = _grid(product, n, 13, [0, 1, 2], parallel=True)
    oa, ols = _grid(oracle, n, 13, [0, 1, 2], parallel=True)
    _check_single(pls, ols, _pairs(n, 12, 2), ks=(1, 2))
    _check_batch(pls, ols, "7", [str(i) for i in range(n * n)])


@pytest.mark.parametrize("parallel", [False, True])
def test_forced_hbm_path_matches_oracle(product, oracle, parallel):
    """Positive metrics through the HBM-state path (option ksp_hbm): single
    calls with masked reruns and the batch, overloads included."""
    n = 7
    with _Hbm(1):
        pa, pls = _grid(product, n, 14, [1, 2, 3, 5], parallel, overload={10, 30})
        oa, ols = _grid(oracle, n, 14, [1, 2, 3, 5], parallel, overload={10, 30})
        _check_single(pls, ols, _pairs(n, 15, 3))
        _check_batch(pls, ols, "24", [str(i) for i in range(n * n)])


def test_forced_hbm_wide_distances(product, oracle):
    """64-bit distances (path sums past 2^31: metric x (N - 1) decides the
    width, as for buildRouteDb) on the HBM path."""
    n = 12
    big = [21_000_000, 20_999_999, 15_000_000]
    with _Hbm(1):
        pa, pls = _grid(product, n, 15, big)
        oa, ols = _grid(oracle, n, 15, big)
        _check_single(pls, ols, _pairs(n, 10, 4))
        _check_batch(pls, ols, "0", [str(i) for i in range(n * n)])


def _stress_grid(M, n):
    """createGrid wiring of SpfSolverTest.cpp's GridTopologyFixture (unit
    metrics, ifNames 0/1..0/4)."""
    als = M.AreaLinkStates()
    ls = als.add(L.kTestingAreaName, L.kTestingNodeName)
    for i in range(n):
        for j in range(n):
            node = i * n + j
            adjs = []
            for (ii, jj, ifn, oifn) in ((i, j + 1, "0/1", "0/3"), (i - 1, j, "0/2", "0/4"),
                                        (i, j - 1, "0/3", "0/1"), (i + 1, j, "0/4", "0/2")):
                if 0 <= ii < n and 0 <= jj < n:
                    nb = ii * n + jj
                    adjs.append(L.createAdjacency(str(nb), ifn, oifn, f"fe80::{nb:x}",
                                                  f"192.168.{nb // 256}.{nb % 256}", 1,
                                                  100001 + nb))
            ls.updateAdjacencyDatabase(L.createAdjDb(str(node), adjs, node + 1),
                                       L.kTestingAreaName)
    return ls


@pytest.mark.parametrize("n", [99, 128])
def test_large_grid_past_lds(product, oracle, n):
    """99x99 (the reference's stress grid, source "523") and 128x128 (16,384
    nodes): KSP2 state no longer fits LDS; single calls k = 1..3 and a batch
    of destinations equal the oracle."""
    pls, ols = _stress_grid(product, n), _stress_grid(oracle, n)
    rng = random.Random(n)
    dests = sorted({str(rng.randrange(n * n)) for _ in range(24)} | {str(n * n - 1)})
    for d in dests[:6]:
        for k in (1, 2, 3):
            assert _paths(pls, "523", d, k) == _paths(ols, "523", d, k), (d, k)
    _check_batch(pls, ols, "523", dests)


def test_large_grid_zero_metrics(product, oracle):
    """Zero metrics on a grid past the LDS budget: exact order, HBM state."""
    n = 90
    pa, pls = _grid(product, n, 16, [0, 1, 1, 2])
    oa, ols = _grid(oracle, n, 16, [0, 1, 1, 2])
    rng = random.Random(16)
    dests = sorted({str(rng.randrange(n * n)) for _ in range(12)})
    _check_batch(pls, ols, "4000", dests)
