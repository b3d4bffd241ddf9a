"""CPU checks of the HBM image the adapter hands the kernels
(BatchRunner.host_arrays): CSR/offset consistency and the wave kernel's
relaxation order (ogs_graph.slot_node, openr_amd/csrc/host/slot_order.h)."""
import ctypes

import numpy as np
import pytest


def _batch(kind="grid", **kw):
    import openr_amd
    M = openr_amd.decision
    br = M.BatchRunner(True, False, False)
    if kind == "grid":
        opts = dict(n=kw.get("n", 10), metricSeed=0xC2000000, prefixSeed=0xC1)
        if kw.get("ovl"):
            opts.update(adjOverloadPermille=50, nodeOverloadPermille=30, overloadSeed=7)
        br.add_grid_batch(opts, 0, kw.get("topos", 8), "1")
    else:
        br.add_generated(kind, kw["opts"], kw["sources"])
    return br.host_arrays()


def _check_slots(h):
    T, stride = h["num_topos"], h["slot_stride"]
    assert stride in (64, 128, 256) and stride >= h["max_nodes"]
    slots = h["slot_node"].reshape(T, stride)
    nb = h["node_base"]
    for t in range(T):
        n = int(nb[t + 1] - nb[t])
        ids = slots[t][slots[t] != 0xFFFF]
        assert sorted(ids.tolist()) == list(range(n)), "not a permutation"
    return slots


def test_grid_slot_order_is_two_coloured_permutation():
    h = _batch(n=10, topos=4)
    slots = _check_slots(h)
    assert h["slot_stride"] == 128
    rp, edges = h["row_ptr"], h["edges"]
    for t in range(4):
        pos = {int(v): i for i, v in enumerate(slots[t]) if v != 0xFFFF}
        base = int(h["node_base"][t])
        e0 = int(rp[base])
        # a grid is bipartite: every edge joins slot 0 and slot 1
        for v in range(100):
            for e in range(int(rp[base + v]), int(rp[base + v + 1])):
                u = int(edges[e]) & 0x1FFFFF
                assert (pos[v] // 64) != (pos[u] // 64), (t, v, u, e - e0)


@pytest.mark.parametrize("n", [3, 7, 8, 16])
def test_slot_order_small_and_large_grids(n):
    h = _batch(n=n, topos=2)
    _check_slots(h)


def test_fabric_slot_order():
    h = _batch("fabric", opts=dict(pods=2, planes=2, sswPerPlane=2, rswPerPod=4),
               sources=["3-0-0"])
    _check_slots(h)


def test_prefix_min_nexthop_flag():
    h = _batch(n=4, topos=1)
    # generated grids carry no minNexthop: bit1 clear everywhere
    assert not (h["pfx_flags"] & 0x2).any()
    assert (h["adv_min_nh"] == np.iinfo(np.int64).min).all()


def test_spf_routes_rejects_bad_slot_stride():
    import openr_amd.capi as capi
    lib = capi.load()
    out = capi.SpfOut()
    g = capi.Graph()
    g.max_nodes = 100
    buf = (ctypes.c_uint32 * 4)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    g.node_base = g.row_ptr = g.node_flags = p
    g.slot_node = p
    units = (ctypes.c_uint32 * 2)()
    for stride in (0, 96, 64, 512):
        g.slot_stride = stride
        rc = lib.ogs_spf_routes(ctypes.byref(g), None, units, 1, 0, 1,
                                ctypes.byref(out), None)
        assert rc == -1, stride


@pytest.mark.parametrize("n", [7, 10, 16])
def test_slot_edge_image_matches_csr(n):
    """ogs_graph.slot_edges restates each ordered node's CSR row: neighbour
    position, down / overloaded bits, reverse slot and metric."""
    h = _batch(n=n, topos=3, ovl=True)
    T, S, D = h["num_topos"], h["slot_stride"], h["slot_degree"]
    assert D in (4, 8)
    slots = h["slot_node"].reshape(T, S)
    img = h["slot_edges"].reshape(T, D, S)
    rp, edges, nb = h["row_ptr"], h["edges"], h["node_base"]
    for t in range(T):
        for p in range(S):
            v = int(slots[t, p])
            if v == 0xFFFF:
                assert (img[t, :, p] & 0x200).all()
                continue
            row = range(int(rp[nb[t] + v]), int(rp[nb[t] + v + 1]))
            for j in range(D):
                x = int(img[t, j, p])
                if j >= len(row):
                    assert x & 0x200
                    continue
                e = int(edges[row[j]])
                lo, w = e & 0xFFFFFFFF, e >> 32
                u = lo & 0x1FFFFF
                assert int(slots[t, x & 0x1FF]) == u
                assert bool(x & 0x200) == bool(lo >> 31)
                assert bool(x & 0x400) == bool(lo & (1 << 21))
                assert (x >> 11) & 7 == (lo >> 22) & 0x1FF
                assert x >> 16 == w


def test_prefix_state_many_advertisers_vs_oracle(host_module, oracle):
    """PrefixState (PrefixState.cpp:15-57) keeps each prefix's entries sorted
    by (node, area) -- one advertisement inline, more in a vector: random
    update / re-advertise / delete sequences with up to 6 advertisers per
    prefix over 2 areas, the product's change sets and final table equal the
    oracle's after every step (host only)."""
    import random
    import lsdb as L
    rng = random.Random(5)
    ps, ops = host_module.PrefixState(), oracle.PrefixState()
    nodes, areas = [f"n{i}" for i in range(6)], ["a", "b"]
    prefixes = [f"fc00::{i:x}/128" for i in range(5)] + ["10.0.0.0/8"]
    for step in range(600):
        node, area, pfx = rng.choice(nodes), rng.choice(areas), rng.choice(prefixes)
        if rng.random() < 0.3:
            got = ps.deletePrefix(node, area, pfx)
            want = ops.deletePrefix(node, area, pfx)
        else:
            e = L.createPrefixEntry(pfx)
            e["metrics"]["path_preference"] = rng.choice([100, 200])
            got = ps.updatePrefix(node, area, e)
            want = ops.updatePrefix(node, area, e)
        assert set(got) == set(want), step
        a, b = ps.prefixes(), ops.prefixes()
        assert set(a) == set(b), step
        for p in a:
            assert list(a[p]) == list(b[p]), (step, p)
