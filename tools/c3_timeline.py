"""Item timeline of the C3 one-launch form (spf_lds_route_kernel) from the
diagnostic build (`make stamps`, OGS_LIB=openr_amd/lib/libopenr_gpu_stamps.so):
per workgroup every item {SPF | stream | join, unit, start, ready, end} on the
100 MHz realtime clock. Prints where one launch's time goes: the SPF head
(launch start -> a workgroup's first stream item), stream items' wait for
their SPF (the first one's too), busy stream time per width group, and each
workgroup's idle tail (its last item's end -> the launch's end). Usage:
  python tools/c3_timeline.py [--as-rank r/N] [--opt name=value ...]"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KINDS = {1: "spf", 2: "stream", 3: "join"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--as-rank", default=None)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--reps", type=int, default=3)
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
    lib.ogs_diag_item_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    for rep in range(a.reps):
        assert lib.ogs_diag_item_stamps_clear() == 0
        bench.c3_launch_all(lib, capi, launches, main_s, side)
        torch.cuda.synchronize()
        raw = np.zeros(1024 * 64 * 4, dtype=np.uint32)
        assert lib.ogs_diag_item_stamps(raw.ctypes.data, raw.size) == 0
        raw = raw.reshape(1024, 64, 4).astype(np.int64)
        wgs = [w for w in range(1024) if raw[w, 0, 3] != 0]
        t0 = min(raw[w, :, 1][raw[w, :, 3] != 0].min() for w in wgs)
        t1 = max(raw[w, :, 3].max() for w in wgs)
        us = lambda x: x / 100.0  # noqa: E731
        head, waits, busy, idle, spf_t, n_items = [], [], [], [], [], []
        first_wait = []
        item_us = {k: [] for k in KINDS.values()}
        uw = launches[0]["U"] if len(launches) > 1 else 0  # wide group first
        by_group = {"stream wide": [], "stream narrow": [], "spf wide": [], "spf narrow": []}
        for w in wgs:
            it = raw[w][raw[w, :, 3] != 0]
            kinds = it[:, 0] >> 28
            # SPF items: start..end; stream items: start..ready (wait), ready..end (busy)
            for row, k in zip(it, kinds):
                item_us[KINDS[int(k)]].append(us(row[3] - row[1]))
                unit = int(row[0]) & 0x0FFFFFFF
                grp = "wide" if unit < uw else "narrow"
                by_group[("spf " if int(k) == 1 else "stream ") + grp].append(
                    us(row[3] - (row[2] if int(k) != 1 else row[1])))
            sp = it[kinds == 1]
            spf_t.append(us((sp[:, 3] - sp[:, 1]).sum()) if len(sp) else 0.0)
            st = it[(kinds == 2) | (kinds == 3)]
            head.append(us(st[:, 1].min() - t0) if len(st) else us(t1 - t0))
            waits.append(us((st[:, 2] - st[:, 1]).sum()) if len(st) else 0.0)
            if len(st):
                first_wait.append(us(st[0, 2] - st[0, 1]))
            busy.append(us((st[:, 3] - st[:, 2]).sum()) if len(st) else 0.0)
            idle.append(us(t1 - it[:, 3].max()))
            n_items.append(len(it))
        pct = lambda x, q: float(np.percentile(x, q))  # noqa: E731
        print(f"rep {rep}: launch {us(t1 - t0):.1f} us over {len(wgs)} workgroups, "
              f"items/wg med {np.median(n_items):.0f} max {max(n_items)}")
        for name, x in [("spf time", spf_t), ("first stream start", head),
                        ("first item wait", first_wait),
                        ("stream wait", waits), ("stream busy", busy), ("tail idle", idle)]:
            print(f"   {name:18s} mean {np.mean(x):6.1f}  p10 {pct(x, 10):6.1f}  "
                  f"med {pct(x, 50):6.1f}  p90 {pct(x, 90):6.1f}  max {max(x):6.1f} us")
        for k, x in by_group.items():
            if x:
                print(f"   {k:14s} n={len(x):5d}  med {np.median(x):6.1f}  "
                      f"p90 {pct(x, 90):6.1f}  max {max(x):6.1f} us (busy part)")
        for k, x in item_us.items():
            if x:
                print(f"   item {k:6s} n={len(x):5d}  med {np.median(x):6.1f}  "
                      f"p90 {pct(x, 90):6.1f}  max {max(x):6.1f} us")


if __name__ == "__main__":
    main()
