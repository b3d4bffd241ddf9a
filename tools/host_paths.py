#!/usr/bin/env python3
"""The drop-in's host-heavy paths on one box, standalone: f1 incremental
routes (batch split + per-prefix loop), G1 single-source cold / warm split,
f4 publication ingest split. Usage: python tools/host_paths.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

import bench  # noqa: E402


def main():
    import openr_amd
    openr_amd.require_gpu()
    M = openr_amd.decision
    fab = dict(bench.C3_OPTS, prefixesPerNode=100)
    for _ in range(3):
        b, l, same, n, *split = M.incremental_routes_bench("fabric", fab, bench.C3_INC_SOURCE, 100)
        print(json.dumps({"f1": {"batch_ms": round(b, 3), "loop_ms": round(l, 3), "same": same,
                                 "split": [round(x, 3) for x in split]}}), flush=True)
    from openr_amd.workloads import G1_OPTS
    r = M.build_latency_bench("wan", G1_OPTS, "0", 5)
    print(json.dumps({"g1_single": [x if not isinstance(x, float) else round(x, 3) for x in r]},
                     default=str), flush=True)
    d = M.publication_ingest_bench("fabric", fab, 3)
    print(json.dumps({"f4": dict(d)}), flush=True)


if __name__ == "__main__":
    main()
