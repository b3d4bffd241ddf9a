"""Experiment: the C2 batch as ONE launch of 4096 units vs two launches of
2048 units on two HIP streams (the second half's staging reads overlap the
first half's rounds, its rounds the first half's output writes). Same
outputs required; prints median step time of each form (events on stream A,
which joins stream B before the end event)."""
import ctypes
import os
import sys
from statistics import median

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c2dev import C2  # noqa: E402


def main():
    import torch
    c = C2()
    pt = c.table()
    g = c.graph("pi")
    o1, o2 = c.outputs(), c.outputs()
    h, t = c.h, c.t
    U, half = c.U, c.U // 2
    sa = torch.cuda.Stream(c.dev)
    sb = torch.cuda.Stream(c.dev)
    # second half: per-topology arrays and units rebased so unit i is topology i
    import numpy as np
    hu = h["units"].reshape(-1, 2)[half:].astype(np.int64)
    hu[:, 0] -= half
    u2 = torch.from_numpy(hu.astype(np.uint32).reshape(-1)).to(c.dev)
    g2 = c.capi.Graph(h["num_topos"] - half, c.Sn, h["max_edges"], h["max_degree"],
                      t["node_base"].data_ptr() + 4 * half, t["row_ptr"].data_ptr(),
                      t["edges"].data_ptr(), t["node_flags"].data_ptr(),
                      t["topo_desc"].data_ptr() + 32 * half)
    g2.slot_node = t["slot_node"].data_ptr() + 2 * half * h["slot_stride"]
    g2.slot_stride = h["slot_stride"]
    g2.slot_edges = t["slot_edges"].data_ptr() + 4 * half * h["slot_degree"] * h["slot_stride"]
    g2.slot_degree = h["slot_degree"]
    Sn, Sp, W = c.Sn, c.Sp, c.W
    rows = [Sn, W * Sn, Sp, Sp, W * Sp, Sp]

    def launch(gr, unit_ptr, n, outs, off, stream):
        so = c.capi.SpfOut(*[x.data_ptr() + 4 * off * r for x, r in zip(outs, rows)])
        rc = c.lib.ogs_spf_routes(ctypes.byref(gr), ctypes.byref(pt), ctypes.c_void_p(unit_ptr),
                                  n, c.flags, W, ctypes.byref(so),
                                  ctypes.c_void_p(stream.cuda_stream))
        c.capi.check(c.lib, rc, "ogs_spf_routes")

    def one():
        launch(g, t["units"].data_ptr(), U, o1, 0, sa)

    def split():
        ev = torch.cuda.Event()
        ev.record(sa)
        sb.wait_event(ev)
        launch(g, t["units"].data_ptr(), half, o2, 0, sa)
        launch(g2, u2.data_ptr(), U - half, o2, half, sb)
        ev2 = torch.cuda.Event()
        ev2.record(sb)
        sa.wait_event(ev2)

    times = {"one": [], "split": []}
    for rnd in range(30):
        for name, fn in (("one", one), ("split", split)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(sa)
            for _ in range(10):
                fn()
            e1.record(sa)
            torch.cuda.synchronize()
            if rnd >= 3:
                times[name].append(e0.elapsed_time(e1) / 10 * 1e3)
    same = all(torch.equal(a, b) for a, b in zip(o1, o2))
    for k, v in times.items():
        print(f"{k}: median {median(v):.2f} us/step min {min(v):.2f} identical={same}")


if __name__ == "__main__":
    main()
