"""Phase breakdown of the C3 frontier SPF + RouteDb kernel from a diagnostic
(-DOGS_STAMPS) build: cycles per workgroup in setup / dist phase / next-hop
phase / routes, relaxation rounds, and workgroup lifetimes. Run with
OGS_LIB=openr_amd/lib/libopenr_gpu_stamps.so."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import openr_amd
    import openr_amd.capi as capi
    ppn = int(os.environ.get("PPN", "100"))
    lib = capi.load()
    dev = torch.device("cuda", 0)
    from openr_amd.workloads import c3_source_names
    launches, N = bench.c3_launches(torch, openr_amd.decision, capi, dev, c3_source_names(),
                                    ppn, with_sel=True)
    stream = torch.cuda.current_stream(dev)
    for _ in range(3):
        for L in launches:
            capi.check(lib, lib.ogs_spf_routes(
                ctypes.byref(L["g"]), ctypes.byref(L["pt"]),
                ctypes.c_void_p(L["t"]["units"].data_ptr()), L["U"], L["flags"], L["W"],
                ctypes.byref(L["so"]), ctypes.c_void_p(stream.cuda_stream)), "spf")
        torch.cuda.synchronize()
    for L in launches:
        Sp = L["h"]["max_prefixes"]
        raw = L["o"]["sel"].cpu().numpy().view(np.uint32).reshape(L["U"], Sp)[:, :8]
        st = raw[:, :6].astype(np.float64)
        rt0 = raw[:, 6].astype(np.int64) - int(raw[:, 6].min())
        rt1 = raw[:, 7].astype(np.int64) - int(raw[:, 6].min())
        print(f"W={L['W']} units={L['U']}: WG start med={np.median(rt0)/100:.1f}us "
              f"max={rt0.max()/100:.1f}us; end max={rt1.max()/100:.1f}us; "
              f"life med={np.median(rt1-rt0)/100:.1f}us")
        for i, n in enumerate(["setup", "dist", "nh", "routes", "rounds_d", "rounds_nh"]):
            print(f"   {n}: med={np.median(st[:, i]):.0f} p90={np.percentile(st[:, i], 90):.0f} "
                  f"max={st[:, i].max():.0f}")


if __name__ == "__main__":
    main()
