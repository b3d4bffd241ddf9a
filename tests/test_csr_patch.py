"""§8(f) f3: attribute-only adjacency-DB updates (LinkState::
updateAdjacencyDatabase, LinkState.cpp:440-640: metric, adjacency overload,
usability, node overload, node metric increment, labels) patch the CSR image
in place instead of re-flattening it. The patched image must equal a fresh
flatten of the same adjacency databases, and structural updates (links added
or removed, new nodes) must still rebuild. Host-only (no device calls): the
device scatter (ogs_csr_patch) is checked by the gpu-marked tests below."""
import copy
import random

import pytest

from lsdb import createAdjacency, createAdjDb, kTestingAreaName


def grid_dbs(n, seed, parallel=2):
    """n x n grid; every 7th pair of neighbours has a parallel second link."""
    rnd = random.Random(seed)
    adjs = {f"{i}": [] for i in range(n * n)}
    k = 0
    for r in range(n):
        for c in range(n):
            a = r * n + c
            for b in ([a + 1] if c + 1 < n else []) + ([a + n] if r + 1 < n else []):
                links = parallel if k % 7 == 0 else 1
                k += 1
                for j in range(links):
                    ia, ib = f"if_{a}_{b}_{j}", f"if_{b}_{a}_{j}"
                    adjs[f"{a}"].append(createAdjacency(f"{b}", ia, ib, f"fe80::{b}",
                                                        f"10.0.{b // 256}.{b % 256}",
                                                        rnd.randint(1, 20), 100000 + a))
                    adjs[f"{b}"].append(createAdjacency(f"{a}", ib, ia, f"fe80::{a}",
                                                        f"10.0.{a // 256}.{a % 256}",
                                                        rnd.randint(1, 20), 100000 + b))
    return {name: createAdjDb(name, a, 100 + int(name)) for name, a in adjs.items()}


def fresh_image(host, dbs, owner):
    ls = host.LinkState(kTestingAreaName, owner)
    for name in sorted(dbs):
        ls.updateAdjacencyDatabase(dbs[name], kTestingAreaName)
    return ls.flat_image()


def mutate(rnd, db):
    """One attribute-only change of an adjacency DB (no link added/removed)."""
    db = copy.deepcopy(db)
    kind = rnd.choice(["metric", "adj_overload", "node_overload", "metric_inc",
                       "only_other", "label", "noop"])
    adj = rnd.choice(db["adjacencies"])
    if kind == "metric":
        adj["metric"] = rnd.randint(1, 30)
    elif kind == "adj_overload":
        adj["isOverloaded"] = not adj["isOverloaded"]
    elif kind == "node_overload":
        db["isOverloaded"] = not db["isOverloaded"]
    elif kind == "metric_inc":
        db["nodeMetricIncrementVal"] = rnd.choice([0, 0, 5, 17])
    elif kind == "only_other":
        adj["adjOnlyUsedByOtherNode"] = not adj["adjOnlyUsedByOtherNode"]
    elif kind == "label":
        adj["adjLabel"] += 1
    return kind, db


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_attribute_updates_patch_in_place(host_module, seed):
    product = host_module
    rnd = random.Random(seed)
    dbs = grid_dbs(6, seed)
    owner = "7"
    ls = product.LinkState(kTestingAreaName, owner)
    for name in sorted(dbs):
        ls.updateAdjacencyDatabase(dbs[name], kTestingAreaName)
    assert ls.flat_image() == fresh_image(product, dbs, owner)
    builds = ls.flatBuilds()
    for step in range(60):
        name = rnd.choice(sorted(dbs))
        kind, db = mutate(rnd, dbs[name])
        dbs[name] = db
        ls.updateAdjacencyDatabase(db, kTestingAreaName)
        assert ls.flat_image() == fresh_image(product, dbs, owner), (step, kind, name)
    assert ls.flatBuilds() == builds  # every update above was patched
    assert ls.flatPatches() == 60
    assert ls.edgesPatched() > 0


def test_structural_updates_rebuild(host_module):
    product = host_module
    dbs = grid_dbs(4, 9)
    ls = product.LinkState(kTestingAreaName, "0")
    for name in sorted(dbs):
        ls.updateAdjacencyDatabase(dbs[name], kTestingAreaName)
    ls.flat_image()
    builds = ls.flatBuilds()
    db = copy.deepcopy(dbs["5"])
    db["adjacencies"].pop()  # link removed at one end -> link gone
    dbs["5"] = db
    ls.updateAdjacencyDatabase(db, kTestingAreaName)
    assert ls.flat_image() == fresh_image(product, dbs, "0")
    assert ls.flatBuilds() == builds + 1
    ls.deleteAdjacencyDatabase("3")
    del dbs["3"]
    assert ls.flat_image() == fresh_image(product, dbs, "0")
    assert ls.flatBuilds() == builds + 2


def _world(M, dbs, owner):
    from lsdb import createPrefixEntry, createPrefixDb, updatePrefixDatabase
    als = M.AreaLinkStates()
    ls = als.add(kTestingAreaName, owner)
    for name in sorted(dbs):
        ls.updateAdjacencyDatabase(dbs[name], kTestingAreaName)
    ps = M.PrefixState()
    for name in sorted(dbs):
        updatePrefixDatabase(ps, createPrefixDb(name, [createPrefixEntry(f"fc00::{name}/128")]))
    return als, ls, ps


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4, 5])
def test_patched_device_csr_parity(product, oracle, seed):
    """After every attribute-only update the device CSR (scattered by
    ogs_csr_patch) equals the host image, and SPF results and the RouteDb
    (node labels on) equal the oracle's, which replays the same updates."""
    rnd = random.Random(seed)
    dbs = grid_dbs(6, seed)
    owner = "14"
    world = {M: _world(M, dbs, owner) for M in (product, oracle)}
    solvers = {M: M.SpfSolver(owner, True, True, False, False) for M in (product, oracle)}
    for step in range(40):
        if step:
            name = rnd.choice(sorted(dbs))
            kind, db = mutate(rnd, dbs[name])
            dbs[name] = db
            for M in (product, oracle):
                world[M][1].updateAdjacencyDatabase(db, kTestingAreaName)
        else:
            kind = "initial"
        ls = world[product][1]
        edges, flags = ls.device_edges()
        img = ls.flat_image()
        assert edges == img["edges"] and list(flags) == list(img["node_flags"]), (step, kind)
        for src in (owner, "0", "35"):
            assert (world[product][1].getSpfResult(src) ==
                    world[oracle][1].getSpfResult(src)), (step, kind, src)
        got, want = (solvers[M].buildRouteDb(owner, world[M][0], world[M][2])
                     for M in (product, oracle))
        assert got.canonical() == want.canonical(), (step, kind)
    assert world[product][1].flatBuilds() == 1
    assert world[product][1].flatPatches() == 39
