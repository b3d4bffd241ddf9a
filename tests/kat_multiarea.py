"""Multi-area known-answer tests, transcribed from
the reference's DecisionTest; each case takes the implementation module `M`
(oracle/_refcpu or the GPU product openr_amd._decision)."""
from lsdb import *  # noqa: F401,F403


def _route(db, prefix):
    return db.unicastRoutes().get(prefix)


def kat_multi_area_best_path(M):
    """DecisionTest.cpp:1070-1202 DecisionTestFixture.MultiAreaBestPathCalculation.

    area A (kTestingAreaName): 1 -- 2 -- 4 ; area B: 1 -- 3 -- 4 (metric 10).
    "1" and "4" are in both areas; prefixes addr1/addr2 in A, addr3/addr4 in
    B; then "1" also originates addr1 into B."""
    A, B = kTestingAreaName, "B"
    als = M.AreaLinkStates()
    lsA = als.add(A, "1")
    lsB = als.add(B, "1")
    for db in (createAdjDb("1", [adj12], 1, area=A), createAdjDb("2", [adj21, adj24], 2, area=A),
               createAdjDb("4", [adj42], 4, area=A)):
        lsA.updateAdjacencyDatabase(db, A)
    for db in (createAdjDb("1", [adj13], 1, area=B), createAdjDb("3", [adj31, adj34], 3, area=B),
               createAdjDb("4", [adj43], 4, area=B)):
        lsB.updateAdjacencyDatabase(db, B)
    ps = M.PrefixState()
    updatePrefixDatabase(ps, createPrefixDb("1", [createPrefixEntry(addr1)]), A)
    updatePrefixDatabase(ps, createPrefixDb("2", [createPrefixEntry(addr2)]), A)
    updatePrefixDatabase(ps, createPrefixDb("3", [createPrefixEntry(addr3)]), B)
    updatePrefixDatabase(ps, createPrefixDb("4", [createPrefixEntry(addr4)]), B)
    solver = M.SpfSolver("1", False, False, False, False)

    def nh(adj, metric, area):
        return createNextHopFromAdj(adj, False, metric, None, area)

    db1 = solver.buildRouteDb("1", als, ps)
    assert set(db1.unicastRoutes()) == {addr2, addr3, addr4}
    assert _route(db1, addr2)["nexthops"] == {nh(adj12, 10, A)}
    assert _route(db1, addr3)["nexthops"] == {nh(adj13, 10, B)}
    assert _route(db1, addr4)["nexthops"] == {nh(adj13, 20, B)}  # only in B

    db2 = solver.buildRouteDb("2", als, ps)  # sees addr1 in A only
    assert set(db2.unicastRoutes()) == {addr1}
    assert _route(db2, addr1)["nexthops"] == {nh(adj21, 10, A)}

    db3 = solver.buildRouteDb("3", als, ps)  # sees addr4 in B only
    assert set(db3.unicastRoutes()) == {addr4}
    assert _route(db3, addr4)["nexthops"] == {nh(adj34, 10, B)}

    db4 = solver.buildRouteDb("4", als, ps)
    assert set(db4.unicastRoutes()) == {addr1, addr2, addr3}
    assert _route(db4, addr2)["nexthops"] == {nh(adj42, 10, A)}
    assert _route(db4, addr3)["nexthops"] == {nh(adj43, 10, B)}
    assert _route(db4, addr1)["nexthops"] == {nh(adj42, 20, A)}  # only in A

    # "1" originates addr1 into B as well
    updatePrefixDatabase(ps, createPrefixDb("1", [createPrefixEntry(addr1)]), B)
    db3 = solver.buildRouteDb("3", als, ps)
    assert _route(db3, addr1)["nexthops"] == {nh(adj31, 10, B)}
    db4 = solver.buildRouteDb("4", als, ps)
    # reachable through A or B at the same metric: union of both areas
    assert _route(db4, addr1)["nexthops"] == {nh(adj43, 20, B), nh(adj42, 20, A)}


MULTI_AREA_KATS = [kat_multi_area_best_path]
