"""Pin the CPU oracle: it must pass every known-answer test transcribed from
the reference's own unit tests. CPU only."""
import pytest

import kat_cases


@pytest.mark.parametrize("kat", kat_cases.ALL_KATS, ids=lambda f: f.__name__)
def test_oracle_kat(oracle, kat):
    kat(oracle)


def test_oracle_path_a_in_path_b(oracle):
    """LinkStateTest.cpp:189-232 LinkStateTest.pathAInPathB."""
    l1 = ("1", "1/2", "2", "2/1")
    l2 = ("2", "2/3", "3", "3/2")
    l3 = ("1", "1/3", "3", "3/1")
    f = oracle.pathAInPathB
    p1, p2 = [], []
    assert f(p1, p2) and f(p2, p1)
    p1 = [l1]
    assert not f(p1, p2) and f(p2, p1)
    p2 = [l1]
    assert f(p1, p2) and f(p2, p1)
    p1 = [l1, l2]
    assert not f(p1, p2) and f(p2, p1)
    p1 = [l1, l2, l3]
    p2 = [l1, l2]
    assert not f(p1, p2) and f(p2, p1)
    assert not f([l3, l2], [l1]) and not f([l1], [l3, l2])


def test_oracle_spf_runs_counter(oracle):
    """SpfSolverTest.cpp:1666-1667: one SPF per source per build."""
    import lsdb as L
    als = oracle.AreaLinkStates()
    ls = als.add(L.kTestingAreaName, "1")
    for db in (L.createAdjDb("1", [L.adj12, L.adj13], 1), L.createAdjDb("2", [L.adj21, L.adj24], 2),
               L.createAdjDb("3", [L.adj31, L.adj34], 3), L.createAdjDb("4", [L.adj42, L.adj43], 4)):
        ls.updateAdjacencyDatabase(db, L.kTestingAreaName)
    ps = oracle.PrefixState()
    for p in (L.prefixDb1, L.prefixDb2, L.prefixDb3, L.prefixDb4):
        L.updatePrefixDatabase(ps, p)
    solver = oracle.SpfSolver("1", False, True)
    L.getRouteMap(solver, ["1", "2", "3", "4"], als, ps)
    assert ls.spfRuns() == 4


def test_oracle_multi_area_generator(oracle):
    """The multi-area generator builds a connected domain: an ABR reaches
    prefixes in both of its areas, a plain node only its own area + anycast."""
    opts = dict(areas=3, nodesPerArea=40, abrs=6, prefixesPerNode=1, anycastPermille=0)
    abr, plain = oracle.gen_route_dbs_multiarea(opts, ["abr-0", "a2-3"], True, False, False)
    n_abr = abr.count(b"\nU ") + abr.startswith(b"U ")
    n_plain = plain.count(b"\nU ") + plain.startswith(b"U ")
    assert n_abr >= 2 * 40 - 2  # two areas' worth of routes
    assert 30 <= n_plain < n_abr


def test_oracle_variant_updates(oracle):
    """Removing a link changes routes only through it: the oracle's per-variant
    calculateUpdate lists exactly the prefixes whose route text changed."""
    base, variants, links = oracle.variant_route_updates(
        "wan", dict(nodes=120, seed=0xC4, prefixesPerNode=1), "0", 12, 0xC4F, 500)

    def routes(c):
        out, cur = {}, None
        for line in c.decode().splitlines():
            if line.startswith("U "):
                cur = line.split()[1]
                out[cur] = [line.split(" c=")[0]]
            elif cur:
                out[cur].append(line)
        return out
    b = routes(base)
    for canon, changed, nu, nd in variants:
        v = routes(canon)
        diff = sorted(p for p in set(b) | set(v) if b.get(p) != v.get(p))
        assert changed == diff
        assert nd == len(set(b) - set(v))


def _policy(prefixes=(), zero_nbr="", area="area1"):
    """UCMP RibPolicy statements (RibPolicy.h:40-90 semantics): tag matcher with
    area/neighbor weights (incl. zero = drop next hop), a prefix matcher, and a
    second tag statement whose counterID overrides the first's on overlap."""
    return [
        dict(name="ucmp", tags=["ucmp"], counterID="cnt-ucmp",
             set_weight=dict(default_weight=3, area_to_weight={area: 5, "area2": 0},
                             neighbor_to_weight={zero_nbr: 0} if zero_nbr else {})),
        dict(name="pfx", prefixes=list(prefixes), counterID="cnt-pfx",
             set_weight=dict(default_weight=0, neighbor_to_weight={})),
        dict(name="c1", tags=["c1"], counterID="cnt-c1",
             set_weight=dict(default_weight=2, area_to_weight={"area0": 9})),
    ]


def _weights(c):
    return [ln.split(" w=")[1].split()[0] for ln in c.decode().splitlines()
            if " w=" in ln]


def test_oracle_policy_changes_weights(oracle):
    """The generated-DB helper applies the policy: weights other than 0 appear,
    counterIDs are set, and an empty policy leaves the DB unchanged."""
    opts = dict(nodes=120, seed=0xC5, prefixesPerNode=2, tagPermille=500)
    [plain] = oracle.gen_route_dbs("wan", opts, ["3"], True, False, False)
    [same] = oracle.gen_route_dbs("wan", opts, ["3"], True, False, False, [])
    [pol] = oracle.gen_route_dbs("wan", opts, ["3"], True, False, False,
                                 _policy(area="0"))
    assert plain == same and plain != pol
    assert set(_weights(plain)) == {"0"}
    assert {"2", "3"} <= set(_weights(pol))
    assert b"cid=cnt-ucmp" in pol and b"cid=cnt-c1" in pol
