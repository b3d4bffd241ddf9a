"""Inputs that used to be refused with std::domain_error on the GPU path
(VERDICT r1 "throwing domains"), now computed and checked against the
oracle: more than 32 areas, RibPolicies of more than 32 statements (applied
in 32-statement chunks, first transforming statement wins across chunks,
RibPolicy.cpp:222-229), RibPolicy over 64-bit distances, and multi-area
domains with zero / negative link metrics (exact extraction order)."""
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


def test_more_than_32_areas(product, oracle):
    opts = dict(areas=40, nodesPerArea=25, abrs=60, prefixesPerNode=2, anycastPermille=150,
                nodeOverloadPermille=20, adjOverloadPermille=20, v4Permille=50)
    srcs = ["abr-0", "abr-17", "abr-59", "a0-3", "a39-24", "a20-0"]
    for brs in (False, True):
        _cmp(product.gen_route_dbs_multiarea(opts, srcs, True, True, brs),
             oracle.gen_route_dbs_multiarea(opts, srcs, True, True, brs), f"areas40 brs={brs}")


def _many_statements(n, seed, neighbors, areas):
    """n statements over the generator's tags ("ucmp", "c0".."c3") and some
    prefix-less matchers; weights from the neighbours / areas given, some
    all-zero (the route keeps its next hops and the next statement is
    tried), counterIDs on every other one."""
    rng = random.Random(seed)
    tags = ["ucmp", "c0", "c1", "c2", "c3", "none"]
    out = []
    for k in range(n):
        st = dict(name=f"s{k}", tags=rng.sample(tags, rng.randint(1, 2)),
                  set_weight=dict(default_weight=rng.choice([0, 0, 1, 2]),
                                  area_to_weight={a: rng.randint(0, 3) for a in
                                                  rng.sample(areas, min(2, len(areas)))},
                                  neighbor_to_weight={nb: rng.randint(0, 5) for nb in
                                                      rng.sample(neighbors, min(3, len(neighbors)))}))
        if k % 2:
            st["counterID"] = f"cnt{k}"
        out.append(st)
    return out


@pytest.mark.parametrize("n", [33, 70, 200])
def test_policy_more_than_32_statements_single_area(product, oracle, n):
    opts = dict(nodes=300, seed=0xD1, prefixesPerNode=3, tagPermille=500, anycastPermille=100)
    srcs = ["0", "150", "299"]
    nbrs = [str(i) for i in range(300)]
    pol = _many_statements(n, n, nbrs, ["test_area_name"])
    _cmp(product.gen_route_dbs("wan", opts, srcs, True, False, True, pol),
         oracle.gen_route_dbs("wan", opts, srcs, True, False, True, pol), f"pol{n}")


@pytest.mark.parametrize("n", [300, 700])
def test_policy_more_than_255_statements(product, oracle, n):
    """Statement ids past the former u8 range (applied / counter are u16):
    n - 40 statements that never match (tag "none"), then 40 random ones, so
    the statement each route takes and its counterID lie past index 255
    (RibPolicy.cpp:222-249 walks any number of statements)."""
    opts = dict(nodes=300, seed=0xD1, prefixesPerNode=3, tagPermille=500, anycastPermille=100)
    srcs = ["0", "150"]
    nbrs = [str(i) for i in range(300)]
    dead = [dict(name=f"d{k}", tags=["none"], counterID=f"dead{k}",
                 set_weight=dict(default_weight=1, area_to_weight={}, neighbor_to_weight={}))
            for k in range(n - 40)]
    live = _many_statements(40, n, nbrs, ["test_area_name"])
    for k, st in enumerate(live):
        st["counterID"] = f"live{k}"
    pol = dead + live
    got = product.gen_route_dbs("wan", opts, srcs, True, False, True, pol)
    _cmp(got, oracle.gen_route_dbs("wan", opts, srcs, True, False, True, pol), f"pol{n}")
    text = b"".join(got).decode()
    assert "cid=live" in text and "dead" not in text  # late counterIDs reached the routes


def test_policy_more_than_32_statements_multi_area(product, oracle):
    opts = dict(areas=3, nodesPerArea=60, abrs=6, prefixesPerNode=2, anycastPermille=200)
    srcs = ["abr-0", "abr-1", "a0-7"]
    nbrs = [f"a{a}-{i}" for a in range(3) for i in range(60)] + [f"abr-{i}" for i in range(6)]
    areas = [f"area{a}" for a in range(3)]
    pol = _many_statements(45, 7, nbrs, areas)
    _cmp(product.gen_route_dbs_multiarea(opts, srcs, True, False, True, pol),
         oracle.gen_route_dbs_multiarea(opts, srcs, True, False, True, pol), "ma_pol45")


def test_policy_over_wide_distances(product, oracle):
    """Metrics large enough that 32-bit path sums could overflow: the
    route path runs with 64-bit distances and the policy still applies."""
    opts = dict(n=8, metricSeed=0xD2, metricMax=300000000, prefixSeed=5, tagPermille=600)
    srcs = ["0", "27", "63"]
    pol = [dict(name="u", tags=["ucmp"], counterID="u",
                set_weight=dict(default_weight=2, neighbor_to_weight={"1": 0, "8": 7})),
           dict(name="c", tags=["c1", "c2"],
                set_weight=dict(default_weight=0, neighbor_to_weight={"9": 3}))]
    _cmp(product.gen_route_dbs("grid", opts, srcs, True, False, False, pol),
         oracle.gen_route_dbs("grid", opts, srcs, True, False, False, pol), "wide_pol")


def test_multi_area_zero_and_negative_metrics(product, oracle):
    """Multi-area domain whose areas carry zero and negative link metrics:
    every area's SPF replays the extraction order, the multi-area route
    kernel runs on 64-bit distances."""
    srcs = ["abr-0", "abr-3", "a1-9"]
    for zero, neg in ((250, 0), (100, 30)):
        opts = dict(areas=3, nodesPerArea=40, abrs=6, prefixesPerNode=2, anycastPermille=150,
                    zeroMetricPermille=zero, negMetricPermille=neg)
        _cmp(product.gen_route_dbs_multiarea(opts, srcs, True, True, True),
             oracle.gen_route_dbs_multiarea(opts, srcs, True, True, True), f"ma z{zero} n{neg}")
