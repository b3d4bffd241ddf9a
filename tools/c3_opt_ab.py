#!/usr/bin/env python3
"""In-process A/B of engine options on the C3 headline build (one box, one
process, launches built once): the variants alternate pair by pair, each
timed like bench.py's headline (HIP events over STEPS builds), digest checked
against the golden c3 after the last pair. Usage:
  python tools/c3_opt_ab.py [--pairs 5] [--steps 20] [--as-rank r/N] \\
      "route_stream=2" "route_stream=4" ...
Each variant is a comma-separated list of name=value (ogs_set_option);
"lib=base" runs that variant through openr_amd/lib/libopenr_gpu_base.so
(tools/build_ab_base.sh: kernels from another revision)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from openr_amd import shard  # noqa: E402
from openr_amd.workloads import c3_source_names  # noqa: E402


# engine defaults (capi.hip / the kernels' g_* globals) of the options A/B'd here
DEFAULTS = {"frontier_block": 0, "frontier_parts": 0, "route_stream": 5,
            "spf_packed_scan": 1, "spf_seed_row": 1, "frontier_parts_wide": 0,
            "route_store_nt": 2, "spf_lane_walk": -1, "spf_preload": 1,
            "lds_parts": 0, "lds_grid": 0, "lds_key16": 1, "lds_tail": 1,
            "lds_bfs_exit": 1, "lds_lead": 0, "lds_tail_parts": 0,
            "lds_pull": 6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--pairs", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--as-rank", default=None)
    a = ap.parse_args()
    import openr_amd
    import openr_amd.capi as capi
    openr_amd.require_gpu()
    lib = capi.load()
    dev = torch.device("cuda", 0)
    names = c3_source_names()
    if a.as_rank:
        r, n = (int(x) for x in a.as_rank.split("/"))
        names = shard.interleave(names, r, n)
    launches, _ = bench.c3_launches(torch, openr_amd.decision, capi, dev, names)
    launches = launches[::-1]  # wide-first, as bench.py
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    nbytes = sum(L["bytes"] for L in launches)

    # every option any variant names is reset to its default before each
    # variant (options are process-wide and would otherwise carry over)
    keys = {kv.split("=")[0] for v in a.variants for kv in filter(None, v.split(","))}
    keys.discard("lib")
    keys.discard("c3groups")  # bench.C3_GROUPS: 1 one groups call, 0 per-group streams
    libs = {"": lib}
    if any("lib=base" in v for v in a.variants):
        libs["base"] = capi.load(os.path.join(ROOT, "openr_amd", "lib", "libopenr_gpu_base.so"))
    unknown = keys - set(DEFAULTS)
    if unknown:
        raise SystemExit(f"no default known for {sorted(unknown)}: add it to DEFAULTS")

    def apply(v):
        """Sets variant v's options; returns the library it runs through."""
        use = libs["base"] if "lib=base" in v else lib
        bench.C3_GROUPS[0] = "c3groups=0" not in v
        for k in keys:
            use.ogs_set_option(k.encode(), DEFAULTS[k])  # the base may lack newer knobs
        for kv in filter(None, v.split(",")):
            k, x = kv.split("=")
            if k not in ("lib", "c3groups"):
                capi.check(use, use.ogs_set_option(k.encode(), int(x)), k)
        return use

    res = {v: [] for v in a.variants}
    digests = {}
    for _ in range(a.pairs):
        for v in a.variants:
            use = apply(v)
            res[v].append(bench.c3_time(use, capi, launches, main_s, side, a.steps, a.warmup))
    for v in a.variants:
        use = apply(v)
        bench.c3_time(use, capi, launches, main_s, side, 1, 0)
        torch.cuda.synchronize(dev)
        digests[v] = f"{shard.combine_digests(bench.c3_digest(L) for L in launches):016x}"
    want = bench.c3_golden_shard(names)
    for v in a.variants:
        ms = sorted(res[v])
        med = ms[len(ms) // 2]
        print(json.dumps({"variant": v, "median_ms": round(med, 4),
                          "frac": round(nbytes / (med * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 4),
                          "ms": [round(x, 4) for x in res[v]], "digest": digests[v],
                          "golden": digests[v] == want}), flush=True)


if __name__ == "__main__":
    main()
