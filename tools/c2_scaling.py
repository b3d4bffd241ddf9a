#!/usr/bin/env python3
"""C2's kernel time against batch size, in ONE process (VERDICT r5 item 4:
replace the "one chain long" guess with a measured model). The 4096-topology
C2 batch is uploaded once; the wave kernel (spf_route_wave_kernel, the
default launch form) then runs on the first U units for U in --sizes, each
timed with HIP events over --steps launches after --warmup, the sizes
interleaved over --reps passes (median per size). Per size: us per launch,
ns per unit, and the HBM fraction of the algorithmic bytes (SURVEY §8(d),
bench.algorithmic_bytes_per_unit). The full-batch records digest is checked
against the golden c2 block after the last pass.
  python tools/c2_scaling.py [--sizes 1,64,256,1024,2048,4096]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import bench  # noqa: E402
from c2dev import C2  # noqa: E402
from openr_amd import shard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,64,256,512,1024,2048,4096")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--opt", action="append", default=[], help="name=value (ogs_set_option)")
    args = ap.parse_args()
    sizes = [int(x) for x in args.sizes.split(",")]
    c = C2()
    for o in args.opt:
        k, v = o.split("=", 1)
        c.capi.check(c.lib, c.lib.ogs_set_option(k.encode(), int(v)), k)
    assert max(sizes) <= c.U
    g, pt = c.graph(), c.table()
    o = c.outputs()
    so = c.capi.SpfOut(*[x.data_ptr() for x in o[:5]], None)
    s = torch.cuda.current_stream(c.dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    units = c.t["units"].view(torch.int32).data_ptr()

    def launch(U):
        rc = c.lib.ogs_spf_routes(ctypes.byref(g), ctypes.byref(pt), ctypes.c_void_p(units), U,
                                  c.flags, c.W, ctypes.byref(so), sp)
        c.capi.check(c.lib, rc, "ogs_spf_routes")

    N, E, P = 100, 4 * 10 * 9, 100
    bpu = bench.algorithmic_bytes_per_unit(N, E, P, P, c.W, c.W)
    times = {U: [] for U in sizes}
    for _ in range(args.reps):
        for U in sizes:
            for _ in range(args.warmup):
                launch(U)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.steps):
                launch(U)
            e1.record(s)
            e1.synchronize()
            times[U].append(e0.elapsed_time(e1) / args.steps * 1e3)
    launch(c.U)
    torch.cuda.synchronize()
    # golden check of the full batch (records of every unit)
    import openr_amd
    br = openr_amd.decision.BatchRunner(True, False, False)
    br.add_grid_batch(dict(n=10, metricSeed=0xC2000000, prefixSeed=0xC1), 0, c.U, "1")
    d = shard.combine_digests(br.records_digests(
        [str(t) for t in range(c.U)], o[2].cpu().numpy(), o[3].cpu().numpy(),
        o[4].cpu().numpy(), c.W, 16))
    want = bench.GOLDEN.get("c2_blocks", [None])[0]
    rows = []
    for U in sizes:
        us = bench.median(times[U])
        rows.append({"units": U, "us": round(us, 2), "ns_per_unit": round(us * 1e3 / U, 2),
                     "frac": round(bpu * U / (us * 1e-6) / 1e9 / bench.HBM_PEAK_GBS, 4),
                     "all_us": [round(x, 2) for x in times[U]]})
        print(f"U={U:5d}  {us:8.2f} us  {us * 1e3 / U:9.2f} ns/unit  frac {rows[-1]['frac']:.3f}",
              flush=True)
    print(json.dumps({"tool": "c2_scaling", "bytes_alg_per_unit": round(bpu, 1),
                      "opts": args.opt, "rows": rows,
                      "digest": f"{d:016x}", "golden": "match" if f"{d:016x}" == want else
                      f"MISMATCH want {want}"}), flush=True)


if __name__ == "__main__":
    main()
