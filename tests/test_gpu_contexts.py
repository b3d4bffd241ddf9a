"""Execution contexts of the C-ABI (ABI 6, include/openr_gpu.h): a context
owns a device, its own copy of the tuning knobs and its own launch scratch,
so host threads that each drive their own context never share a scratch
buffer or a setting ("explicit stream/device handle;
thread-compatible, one context per host thread").

Two host threads run concurrently, each with its own context and HIP stream:
  A: the C2 4096-topology batch (BASELINE configs[1]) -- the records digest
     equals the oracle's golden c2 block digest every time;
  B: a 352-node fabric's width groups through ogs_ctx_spf_routes_groups with
     its context set to route_stream 2 (the fused frontier form), while the
     default context stays on 5 -- the outputs equal a single-threaded run
     on the default context every time.
Reference semantics pinned elsewhere (test_gpu_bench_size.py, the oracle)."""
import ctypes
import json
import os
import threading

import pytest

from openr_amd.workloads import C2_OPTS, C2_SOURCE, C2_TOPOS

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "bench_digests.json")))
FABRIC = dict(pods=8, planes=4, sswPerPlane=16, rswPerPod=32, full=True, prefixesPerNode=3,
              nodeOverloadPermille=20, adjOverloadPermille=10, v4Permille=150,
              anycastPermille=120, minNhPermille=60, drainPermille=50)


def _device_arrays(torch, dev, h, keys):
    return {k: torch.from_numpy(h[k].view(dt)).to(dev) for k, dt in keys}


def _c2_job(product, capi, torch, dev):
    br = product.BatchRunner(True, False, False)
    br.add_grid_batch(C2_OPTS, 0, C2_TOPOS, C2_SOURCE)
    h = br.host_arrays()
    t = _device_arrays(torch, dev, h, (
        ("topo_desc", "int32"), ("node_base", "int32"), ("row_ptr", "int32"),
        ("edges", "int64"), ("node_flags", "uint8"), ("pfx_base", "int32"),
        ("adv_off", "int32"), ("adv_node", "int32"), ("adv_metrics", "int32"),
        ("adv_min_nh", "int64"), ("pfx_flags", "uint8"), ("slot_node", "uint16"),
        ("slot_edges", "uint32"), ("units", "int32")))
    U = len(h["units"]) // 2
    Sn, Sp, W = h["max_nodes"], h["max_prefixes"], h["nh_words"]
    o = {k: torch.empty(n, dtype=torch.int32, device=dev) for k, n in (
        ("dist", U * Sn), ("nh", U * W * Sn), ("meta", U * Sp), ("metric", U * Sp),
        ("mask", U * W * Sp))}
    g = capi.Graph(h["num_topos"], Sn, h["max_edges"], h["max_degree"],
                   t["node_base"].data_ptr(), t["row_ptr"].data_ptr(), t["edges"].data_ptr(),
                   t["node_flags"].data_ptr(), t["topo_desc"].data_ptr(),
                   t["slot_node"].data_ptr(), h["slot_stride"],
                   t["slot_edges"].data_ptr() if h["slot_degree"] else None, h["slot_degree"])
    pt = capi.PrefixTable(Sp, h["max_advertisements"], t["pfx_base"].data_ptr(),
                          t["adv_off"].data_ptr(), t["adv_node"].data_ptr(),
                          t["adv_metrics"].data_ptr(), t["adv_min_nh"].data_ptr(),
                          t["pfx_flags"].data_ptr())
    out = capi.SpfOut(o["dist"].data_ptr(), o["nh"].data_ptr(), o["meta"].data_ptr(),
                      o["metric"].data_ptr(), o["mask"].data_ptr(), None)
    keys = [str(u) for u in range(U)]

    def run(lib, ctx, stream):
        rc = lib.ogs_ctx_spf_routes(ctx, ctypes.byref(g), ctypes.byref(pt),
                                    ctypes.c_void_p(t["units"].data_ptr()), U, h["flags"], W,
                                    ctypes.byref(out), ctypes.c_void_p(stream.cuda_stream))
        capi.check(lib, rc, "ogs_ctx_spf_routes")
        stream.synchronize()
        from openr_amd import shard
        return shard.combine_digests(br.records_digests(
            keys, o["meta"].cpu().numpy(), o["metric"].cpu().numpy(), o["mask"].cpu().numpy(),
            W, 4))
    return run, (t, o)


def _fabric_job(product, capi, torch, dev):
    names = ([f"1-{p}-{s}" for p in range(4) for s in range(16)] +
             [f"2-{p}-{f}" for p in range(8) for f in range(4)] +
             [f"3-{p}-{r}" for p in range(8) for r in range(32)])
    fsw = [n for n in names if n.startswith("2-")][::2]
    rest = [n for n in names if not n.startswith("2-")][::3]
    br = product.BatchRunner(True, False, False)
    br.add_generated("fabric", FABRIC, fsw + rest)
    h = br.host_arrays()
    t = _device_arrays(torch, dev, h, (
        ("node_base", "int32"), ("row_ptr", "int32"), ("edges", "int64"),
        ("node_flags", "uint8"), ("topo_desc", "int32"), ("pfx_base", "int32"),
        ("adv_off", "int32"), ("adv_node", "int32"), ("adv_metrics", "int32"),
        ("adv_min_nh", "int64"), ("pfx_flags", "uint8"), ("edge_src", "int32")))
    Sn, Sp = h["max_nodes"], h["max_prefixes"]
    g = capi.Graph(h["num_topos"], Sn, h["max_edges"], h["max_degree"],
                   t["node_base"].data_ptr(), t["row_ptr"].data_ptr(), t["edges"].data_ptr(),
                   t["node_flags"].data_ptr(), t["topo_desc"].data_ptr())
    g.edge_src = t["edge_src"].data_ptr()
    pt = capi.PrefixTable(Sp, h["max_advertisements"], t["pfx_base"].data_ptr(),
                          t["adv_off"].data_ptr(), t["adv_node"].data_ptr(),
                          t["adv_metrics"].data_ptr(), t["adv_min_nh"].data_ptr(),
                          t["pfx_flags"].data_ptr())
    units = torch.from_numpy(h["units"].view("int32")).view(-1, 2)
    nf = len(fsw)
    specs = [(units[:nf].contiguous().view(-1).to(dev), 2), (units[nf:].contiguous().view(-1).to(dev), 1)]
    o = [{k: torch.zeros(n, dtype=torch.int32, device=dev) for k, n in (
        ("meta", (len(u) // 2) * Sp), ("metric", (len(u) // 2) * Sp),
        ("mask", (len(u) // 2) * W * Sp))} for u, W in specs]
    arr = (capi.RouteGroup * 2)()
    for i, ((u, W), oo) in enumerate(zip(specs, o)):
        arr[i].units = u.data_ptr()
        arr[i].n_units = len(u) // 2
        arr[i].nh_words = W
        arr[i].out = capi.SpfOut(None, None, oo["meta"].data_ptr(), oo["metric"].data_ptr(),
                                 oo["mask"].data_ptr(), None)

    def run(lib, ctx, stream):
        with torch.cuda.stream(stream):  # ordered before the launch on `stream`
            for oo in o:
                for v in oo.values():
                    v.zero_()
        if ctx is None:
            rc = lib.ogs_spf_routes_groups(ctypes.byref(g), ctypes.byref(pt), arr, 2, h["flags"],
                                           ctypes.c_void_p(stream.cuda_stream))
        else:
            rc = lib.ogs_ctx_spf_routes_groups(ctx, ctypes.byref(g), ctypes.byref(pt), arr, 2,
                                               h["flags"], ctypes.c_void_p(stream.cuda_stream))
        capi.check(lib, rc, "spf_routes_groups")
        stream.synchronize()
        return [{k: v.cpu() for k, v in oo.items()} for oo in o]
    return run, (t, o, specs)


def test_two_threads_own_contexts(product):
    import torch

    import openr_amd.capi as capi
    lib = capi.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c2_run, keep_a = _c2_job(product, capi, torch, dev)
    fab_run, keep_b = _fabric_job(product, capi, torch, dev)
    want_fabric = fab_run(lib, None, torch.cuda.current_stream(dev))  # default context, route_stream 5
    ctx_a, ctx_b = ctypes.c_void_p(), ctypes.c_void_p()
    capi.check(lib, lib.ogs_ctx_create(0, ctypes.byref(ctx_a)), "ogs_ctx_create")
    capi.check(lib, lib.ogs_ctx_create(0, ctypes.byref(ctx_b)), "ogs_ctx_create")
    try:
        capi.check(lib, lib.ogs_ctx_set_option(ctx_b, b"route_stream", 2), "ctx option")
        assert lib.ogs_ctx_set_option(ctx_b, b"no_such_option", 1) != 0
        golden = GOLDEN["c2_blocks"][0]
        errors, results = [], {"a": [], "b": []}
        reps = 12

        def thread_a():
            try:
                torch.cuda.set_device(dev)
                s = torch.cuda.Stream(dev)
                for _ in range(reps):
                    results["a"].append(f"{c2_run(lib, ctx_a, s):016x}")
            except Exception as e:  # noqa: BLE001
                errors.append(("a", repr(e)))

        def thread_b():
            try:
                torch.cuda.set_device(dev)
                s = torch.cuda.Stream(dev)
                for _ in range(reps):
                    results["b"].append(fab_run(lib, ctx_b, s))
            except Exception as e:  # noqa: BLE001
                errors.append(("b", repr(e)))

        ts = [threading.Thread(target=thread_a), threading.Thread(target=thread_b)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=240)
        assert not any(t.is_alive() for t in ts), "a context thread hung"
        assert not errors, errors
        assert results["a"] == [golden] * reps
        assert len(results["b"]) == reps
        for got in results["b"]:
            for g, w in zip(got, want_fabric):
                for k in w:
                    assert torch.equal(g[k], w[k]), k
        # the default context's knob was never touched by ctx_b's setting
        assert lib.ogs_set_option(b"route_stream", 5) == 0
    finally:
        lib.ogs_ctx_destroy(ctx_a)
        lib.ogs_ctx_destroy(ctx_b)


def _c3_shard_job(product, capi, torch, dev, rank=0, world=8):
    """The C3 fabric (2,080 nodes x 208k prefixes) restricted to the sources
    of one N-rank shard (bench.py's interleave), every width group through
    ONE ogs_ctx_spf_routes_groups call; the XOR of its per-source digests
    must equal the oracle's golden per-source digests of those sources."""
    import bench
    from openr_amd import shard
    from openr_amd.workloads import c3_source_names
    mine = shard.interleave(c3_source_names(), rank, world)
    launches, _ = bench.c3_launches(torch, product, capi, dev, mine)
    assert all(L["shared"] for L in launches)
    want = bench.c3_golden_shard(mine)
    arr = (capi.RouteGroup * len(launches))()
    for i, L in enumerate(launches):
        arr[i].units = L["t"]["units"].data_ptr()
        arr[i].n_units = L["U"]
        arr[i].nh_words = L["W"]
        arr[i].out = L["so"]
    L0 = launches[0]

    def run(lib, ctx, stream):
        with torch.cuda.stream(stream):  # ordered before the launch on `stream`
            for L in launches:
                for k in ("meta", "metric", "mask"):
                    L["o"][k].zero_()
        rc = lib.ogs_ctx_spf_routes_groups(ctx, ctypes.byref(L0["g"]), ctypes.byref(L0["pt"]),
                                           arr, len(launches), L0["flags"],
                                           ctypes.c_void_p(stream.cuda_stream))
        capi.check(lib, rc, "ogs_ctx_spf_routes_groups")
        stream.synchronize()
        return f"{shard.combine_digests(bench.c3_digest(L) for L in launches):016x}"
    return run, want, (launches, arr)


def test_two_threads_default_lds_form(product, oracle):
    """Both threads on the DEFAULT one-launch LDS form (route_stream 5: the
    persistent SPF + route-stream kernel with its device-wide item counter
    and release / acquire ready flags in per-context scratch), each on its
    own context and HIP stream, at the same time:
      A: the C3-size fabric's N=8 rank-0 shard (260 sources, 208k prefixes)
         -- equals the oracle's golden per-source digests every time;
      B: the 352-node fabric's two width groups -- every source's digest
         equals a live oracle buildRouteDb every time.
    Each context call leaves the calling thread's HIP device as it was."""
    import torch

    import openr_amd.capi as capi
    lib = capi.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c3_run, c3_want, keep_a = _c3_shard_job(product, capi, torch, dev)
    assert c3_want is not None, "golden C3 per-source digests missing"
    fab_run, keep_b = _fabric_job(product, capi, torch, dev)
    names = ([f"1-{p}-{s}" for p in range(4) for s in range(16)] +
             [f"2-{p}-{f}" for p in range(8) for f in range(4)] +
             [f"3-{p}-{r}" for p in range(8) for r in range(32)])
    fsw = [n for n in names if n.startswith("2-")][::2]
    rest = [n for n in names if not n.startswith("2-")][::3]
    fab_names = fsw + rest
    fab_want = list(oracle.gen_route_digests("fabric", FABRIC, fab_names, True, False, False, 8))
    _, o_b, specs = keep_b
    # one digest runner per width group (records_digests takes the runner's
    # own next-hop width): FSWs (W = 2), then SSW / RSW (W = 1)
    runners = []
    for grp, (u, W) in zip((fsw, rest), specs):
        r = product.BatchRunner(True, False, False)
        r.add_generated("fabric", FABRIC, grp)
        assert r.nh_words() == W
        runners.append(r)

    def fab_digests(got):
        out = []
        for g, (u, W), r in zip(got, specs, runners):
            out += list(r.records_digests([], g["meta"].numpy(), g["metric"].numpy(),
                                          g["mask"].numpy(), W, 4))
        return out

    ctx_a, ctx_b = ctypes.c_void_p(), ctypes.c_void_p()
    capi.check(lib, lib.ogs_ctx_create(0, ctypes.byref(ctx_a)), "ogs_ctx_create")
    capi.check(lib, lib.ogs_ctx_create(0, ctypes.byref(ctx_b)), "ogs_ctx_create")
    try:
        errors, results = [], {"a": [], "b": []}
        reps = 6

        def worker(key, run, ctx):
            try:
                torch.cuda.set_device(dev)
                s = torch.cuda.Stream(dev)
                for _ in range(reps):
                    before = torch.cuda.current_device()
                    results[key].append(run(lib, ctx, s))
                    assert torch.cuda.current_device() == before, "ctx call moved the device"
            except Exception as e:  # noqa: BLE001
                errors.append((key, repr(e)))

        ts = [threading.Thread(target=worker, args=("a", c3_run, ctx_a)),
              threading.Thread(target=worker, args=("b", fab_run, ctx_b))]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=240)
        assert not any(t.is_alive() for t in ts), "a context thread hung"
        assert not errors, errors
        assert results["a"] == [c3_want] * reps
        assert len(results["b"]) == reps
        for got in results["b"]:
            d = fab_digests(got)
            assert d == fab_want, [n for n, x, y in zip(fab_names, d, fab_want) if x != y][:8]
    finally:
        lib.ogs_ctx_destroy(ctx_a)
        lib.ogs_ctx_destroy(ctx_b)


def test_ctx_calls_restore_callers_device():
    """BoundContext / ogs_ctx_destroy restore the calling thread's HIP
    device: a thread on device 1 that destroys (or calls) a device-0
    context is still on device 1 afterwards. With one visible device the
    call on the same device must leave it unchanged."""
    import torch

    import openr_amd.capi as capi
    lib = capi.load()
    n = torch.cuda.device_count()
    cur = 1 if n >= 2 else 0
    torch.cuda.set_device(cur)
    ctx = ctypes.c_void_p()
    capi.check(lib, lib.ogs_ctx_create(0, ctypes.byref(ctx)), "ogs_ctx_create")
    capi.check(lib, lib.ogs_ctx_set_option(ctx, b"route_stream", 5), "ctx option")
    assert torch.cuda.current_device() == cur
    capi.check(lib, lib.ogs_ctx_destroy(ctx), "ogs_ctx_destroy")
    assert torch.cuda.current_device() == cur
    torch.cuda.set_device(0)
