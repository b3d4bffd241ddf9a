"""Phase breakdown of the small SPF+RouteDb kernel from a diagnostic
(-DOGS_STAMPS) build: cycles in staging / SPF rounds / routes per unit, and
the number of relaxation rounds. Run with OGS_LIB=<stamped lib>."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import openr_amd
    import openr_amd.capi as capi
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
    o = [torch.zeros(n, dtype=torch.int32, device=dev) for n in
         (U * Sn, U * W * Sn, U * Sp, U * Sp, U * W * Sp, U * Sp)]
    so = capi.SpfOut(*[x.data_ptr() for x in o])
    for uw in [int(x) for x in os.environ.get("VARIANTS", "1,64").split(",")]:
        capi.check(lib, lib.ogs_set_option(b"unit_width", uw), "opt")
        for _ in range(3):
            capi.check(lib, lib.ogs_spf_routes(ctypes.byref(g), ctypes.byref(pt),
                                               ctypes.c_void_p(t["units"].data_ptr()), U,
                                               h["flags"], W, ctypes.byref(so), None), "run")
        torch.cuda.synchronize()
        st = o[5].cpu().numpy().reshape(U, Sp)[:, :6].astype(np.float64)
        names = ["stage", "spf", "routes", "rounds", "desc", "evals"]
        print(f"unit_width={uw}: " + "  ".join(
            f"{n}: med={np.median(st[:, i]):.0f} p90={np.percentile(st[:, i], 90):.0f} "
            f"max={st[:, i].max():.0f}" for i, n in enumerate(names)))
        print(f"   spf cycles/round (median) = {np.median(st[:, 1] / st[:, 3]):.0f}")


if __name__ == "__main__":
    main()
