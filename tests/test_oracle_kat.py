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
