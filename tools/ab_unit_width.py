"""A/B of the SPF+RouteDb kernel variants on the C2 batch, interleaved in ONE
process (cdna_hip_programming.md §5.4 rule 24): unit_width 0 (generic
kernel), 64, 128, 256. Prints median/min kernel ms per variant and checks
every variant's outputs are identical."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import openr_amd
    import openr_amd.capi as capi
    openr_amd.require_gpu()
    lib = capi.load()
    M = openr_amd.decision
    br = M.BatchRunner(True, False, False)
    br.add_grid_batch(dict(n=10, metricSeed=0xC2000000, prefixSeed=0xC1), 0, 4096, "1")
    h = br.host_arrays()
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(h[k]).to(dev) for k in
         ("topo_desc", "node_base", "row_ptr", "edges", "node_flags", "pfx_base", "adv_off",
          "adv_node", "adv_metrics", "adv_min_nh", "pfx_flags", "units")}
    U = len(h["units"]) // 2
    Sn, Sp, W = h["max_nodes"], h["max_prefixes"], h["nh_words"]
    g = capi.Graph(h["num_topos"], Sn, h["max_edges"], h["max_degree"], t["node_base"].data_ptr(),
                   t["row_ptr"].data_ptr(), t["edges"].data_ptr(), t["node_flags"].data_ptr(), t["topo_desc"].data_ptr())
    pt = capi.PrefixTable(Sp, h["max_advertisements"], t["pfx_base"].data_ptr(),
                          t["adv_off"].data_ptr(), t["adv_node"].data_ptr(),
                          t["adv_metrics"].data_ptr(), t["adv_min_nh"].data_ptr(),
                          t["pfx_flags"].data_ptr())
    outs = {}
    stream = torch.cuda.current_stream(dev)
    variants = [int(x) for x in os.environ.get("VARIANTS", "0,1,2,64").split(",")]
    times = {v: [] for v in variants}
    for v in variants:
        o = [torch.zeros(n, dtype=torch.int32, device=dev) for n in
             (U * Sn, U * W * Sn, U * Sp, U * Sp, U * W * Sp, U * Sp)]
        outs[v] = o
    for rnd in range(12):
        for v in variants:
            capi.check(lib, lib.ogs_set_option(b"unit_width", v), "set_option")
            o = outs[v]
            so = capi.SpfOut(*[x.data_ptr() for x in o])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                capi.check(lib, lib.ogs_spf_routes(ctypes.byref(g), ctypes.byref(pt),
                                                   ctypes.c_void_p(t["units"].data_ptr()), U,
                                                   h["flags"], W, ctypes.byref(so),
                                                   ctypes.c_void_p(stream.cuda_stream)),
                           "spf_routes")
            e1.record(stream)
            torch.cuda.synchronize()
            if rnd >= 2:
                times[v].append(e0.elapsed_time(e1) / 10)
    ref = outs[variants[0]]
    for v in variants:
        same = all(torch.equal(a, b) for a, b in zip(ref, outs[v]))
        ts = sorted(times[v])
        print(f"unit_width={v:4d} median={ts[len(ts)//2]*1e3:8.2f} us "
              f"min={ts[0]*1e3:8.2f} us identical={same}")


if __name__ == "__main__":
    main()
