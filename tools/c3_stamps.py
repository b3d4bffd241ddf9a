"""Phase breakdown of the C3 fused frontier SPF + RouteDb launches from a
diagnostic (-DOGS_STAMPS, `make stamps`) build: per workgroup the cycles of
setup / dist phase / next-hop phase / routes, the relaxation rounds, and
start / end on the shader clock (100 MHz realtime), both width groups
launched as bench.py does (two streams). Run with
OGS_LIB=openr_amd/lib/libopenr_gpu_stamps.so; options: --as-rank r/N (one
rank's shard), --opt name=value (ogs_set_option)."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--as-rank", default=None)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--lds", action="store_true",
                    help="stamps of the LDS-resident SPF kernel (route_stream 4)")
    a = ap.parse_args()
    import torch
    import bench
    import openr_amd
    import openr_amd.capi as capi
    from openr_amd import shard
    from openr_amd.workloads import c3_source_names
    lib = capi.load()
    for o in a.opt:
        k, v = o.split("=")
        capi.check(lib, lib.ogs_set_option(k.encode(), int(v)), k)
    dev = torch.device("cuda", 0)
    names = c3_source_names()
    if a.as_rank:
        r, n = (int(x) for x in a.as_rank.split("/"))
        names = shard.interleave(names, r, n)
    launches, _ = bench.c3_launches(torch, openr_amd.decision, capi, dev, names)
    launches = launches[::-1]
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    for _ in range(3):
        bench.c3_launch_all(lib, capi, launches, main_s, side)
    torch.cuda.synchronize()
    if a.lds:
        raw = np.zeros(4 * 4096 * 32, dtype=np.uint32)
        lib.ogs_diag_lds_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        assert lib.ogs_diag_lds_stamps(raw.ctypes.data, raw.size) == 0
        raw = raw.reshape(4, 4096, 32)
        for L in launches:
            st = raw[L["W"] - 1]
            st = st[st[:, 4] != 0]
            print(f"W={L['W']} workgroups={len(st)}: stage med={np.median(st[:, 0]):.0f} "
                  f"first-unit(incl stage) med={np.median(st[:, 1]):.0f} "
                  f"rounds med={np.median(st[:, 2]):.0f} queued med={np.median(st[:, 5]):.0f} "
                  f"units med={np.median(st[:, 3]):.0f} "
                  f"kernel med={np.median(st[:, 4]):.0f} max={st[:, 4].max():.0f}")
            print("   round (queue / dist / nh) cycles (med): " + "  ".join(
                "/".join(f"{np.median(st[:, 8 + 3 * k + j]):.0f}" for j in range(3))
                for k in range(8) if np.median(st[:, 8 + 3 * k + 2]) > 0))
        return
    raw = np.zeros(65536 * 8, dtype=np.uint32)
    lib.ogs_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    assert lib.ogs_diag_stamps(raw.ctypes.data, raw.size) == 0
    raw = raw.reshape(-1, 8)
    rows = {}
    for L in launches:
        nwg = int(np.count_nonzero(raw[(L["W"] - 1) * 16384:(L["W"] - 1) * 16384 + 16384, 7]))
        rows[L["W"]] = raw[(L["W"] - 1) * 16384:(L["W"] - 1) * 16384 + nwg]
    t0 = min(int(x[:, 6].min()) for x in rows.values())
    for W, st in sorted(rows.items()):
        rt0 = st[:, 6].astype(np.int64) - t0
        rt1 = st[:, 7].astype(np.int64) - t0
        print(f"W={W} workgroups={len(st)}: start med={np.median(rt0)/100:.1f}us "
              f"max={rt0.max()/100:.1f}us; end med={np.median(rt1)/100:.1f}us "
              f"max={rt1.max()/100:.1f}us; life med={np.median(rt1-rt0)/100:.1f}us")
        for i, n in enumerate(["setup", "dist", "nh", "routes", "rounds_d", "rounds_nh"]):
            x = st[:, i].astype(np.float64)
            print(f"   {n}: med={np.median(x):.0f} p90={np.percentile(x, 90):.0f} "
                  f"max={x.max():.0f}")


if __name__ == "__main__":
    main()
