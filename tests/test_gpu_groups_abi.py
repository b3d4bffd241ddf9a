"""ogs_spf_routes_groups (include/openr_gpu.h, ABI 5) against one
ogs_spf_routes call per group, through the C-ABI with torch-owned device
buffers -- the way a C consumer drives it.

Three groups of different next-hop widths (W = 4, 2, 1) over one fabric
graph and prefix table; group 2 brings its own dist / nh buffers (the SPF
rows are then written straight into them with that group's W stride, while
the one-launch form's LDS state is laid out for Wmax). Every output array of
every group must equal the per-group call's, byte for byte. Reference
semantics: SpfSolver::buildRouteDb per source (SpfSolver.cpp:313-453); the
per-group calls themselves are pinned to the oracle elsewhere
(test_gpu_parity.py, test_gpu_bench_size.py)."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu

OPTS = dict(pods=4, planes=2, sswPerPlane=36, rswPerPod=48, full=True, prefixesPerNode=2,
            nodeOverloadPermille=20, adjOverloadPermille=10, v4Permille=150,
            anycastPermille=120, minNhPermille=60, drainPermille=50)


def _arrays(product, names):
    br = product.BatchRunner(True, False, False)
    br.add_generated("fabric", OPTS, names)
    return br.host_arrays()


@pytest.mark.parametrize("route_stream,lead", [(5, 0), (5, -1), (5, 3), (2, 0)])
def test_groups_match_per_group_calls(product, route_stream, lead):
    import torch

    import openr_amd.capi as capi
    lib = capi.load()
    dev = torch.device("cuda:0")
    fsw = [f"2-{p}-{f}" for p in range(4) for f in range(2)]
    ssw = [f"1-{p}-{s}" for p in range(2) for s in range(0, 36, 5)]
    rsw = [f"3-{p}-{r}" for p in range(4) for r in range(0, 48, 7)]
    # the graph / prefix table of one generated fabric serves all groups
    h = _arrays(product, fsw + ssw + rsw)
    up = lambda key, dt: torch.from_numpy(h[key].view(dt)).to(dev)  # noqa: E731
    t = {k: up(k, dt) for k, dt in (
        ("node_base", "int32"), ("row_ptr", "int32"), ("edges", "int64"),
        ("node_flags", "uint8"), ("topo_desc", "int32"), ("pfx_base", "int32"),
        ("adv_off", "int32"), ("adv_node", "int32"), ("adv_metrics", "int32"),
        ("adv_min_nh", "int64"), ("pfx_flags", "uint8"), ("edge_src", "int32"))}
    Sn, Sp = h["max_nodes"], h["max_prefixes"]
    assert Sn > 256  # the large-topology forms
    g = capi.Graph(h["num_topos"], Sn, h["max_edges"], h["max_degree"],
                   t["node_base"].data_ptr(), t["row_ptr"].data_ptr(), t["edges"].data_ptr(),
                   t["node_flags"].data_ptr(), t["topo_desc"].data_ptr())
    g.edge_src = t["edge_src"].data_ptr()
    pt = capi.PrefixTable(Sp, h["max_advertisements"], t["pfx_base"].data_ptr(),
                          t["adv_off"].data_ptr(), t["adv_node"].data_ptr(),
                          t["adv_metrics"].data_ptr(), t["adv_min_nh"].data_ptr(),
                          t["pfx_flags"].data_ptr())
    units_all = torch.from_numpy(h["units"].view("int32")).view(-1, 2)
    nf, ns = len(fsw), len(ssw)
    specs = [(units_all[:nf], 4, False), (units_all[nf:nf + ns], 2, True),
             (units_all[nf + ns:], 1, False)]

    def outs(U, W, rows):
        o = dict(meta=torch.full((U * Sp,), -7, dtype=torch.int32, device=dev),
                 metric=torch.full((U * Sp,), -7, dtype=torch.int32, device=dev),
                 mask=torch.full((U * W * Sp,), -7, dtype=torch.int32, device=dev))
        if rows:
            o["dist"] = torch.full((U * Sn,), -7, dtype=torch.int32, device=dev)
            o["nh"] = torch.full((U * W * Sn,), -7, dtype=torch.int32, device=dev)
        so = capi.SpfOut(o["dist"].data_ptr() if rows else None,
                         o["nh"].data_ptr() if rows else None, o["meta"].data_ptr(),
                         o["metric"].data_ptr(), o["mask"].data_ptr(), None)
        return o, so

    stream = torch.cuda.current_stream()
    try:
        capi.check(lib, lib.ogs_set_option(b"route_stream", route_stream), "route_stream")
        capi.check(lib, lib.ogs_set_option(b"lds_lead", lead), "lds_lead")
        units = [u.contiguous().view(-1).to(dev) for u, _, _ in specs]
        grouped = [outs(len(u) // 2, W, rows) for u, (_, W, rows) in zip(units, specs)]
        arr = (capi.RouteGroup * 3)()
        for i, (u, (_, W, _), (_, so)) in enumerate(zip(units, specs, grouped)):
            arr[i].units = u.data_ptr()
            arr[i].n_units = len(u) // 2
            arr[i].nh_words = W
            arr[i].out = so
        capi.check(lib, lib.ogs_spf_routes_groups(ctypes.byref(g), ctypes.byref(pt), arr, 3,
                                                  h["flags"],
                                                  ctypes.c_void_p(stream.cuda_stream)),
                   "ogs_spf_routes_groups")
        single = []
        for u, (_, W, rows) in zip(units, specs):
            o, so = outs(len(u) // 2, W, rows)
            capi.check(lib, lib.ogs_spf_routes(ctypes.byref(g), ctypes.byref(pt),
                                               ctypes.c_void_p(u.data_ptr()), len(u) // 2,
                                               h["flags"], W, ctypes.byref(so),
                                               ctypes.c_void_p(stream.cuda_stream)),
                       "ogs_spf_routes")
            single.append(o)
        torch.cuda.synchronize()
    finally:
        lib.ogs_set_option(b"route_stream", 5)
        lib.ogs_set_option(b"lds_tail_parts", 0)
    for i, ((o, _), s) in enumerate(zip(grouped, single)):
        for k in o:
            assert torch.equal(o[k], s[k]), f"group {i} (W={specs[i][1]}) array {k} differs"
        # the records were written (not left at the fill value)
        assert not torch.equal(o["meta"], torch.full_like(o["meta"], -7)), i
