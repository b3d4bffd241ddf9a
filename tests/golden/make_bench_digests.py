#!/usr/bin/env python3
"""Generates tests/golden/bench_digests.json: the ORACLE's digests of the
exact bench workloads (configs C2-C5 of BASELINE.json),
which bench.py asserts its own digests against and the bench-size parity
tests (tests/test_gpu_bench_size.py) compare with.

Digest spec: openr_amd/csrc/host/route_digest.h (RouteDbs: per unit key the
XOR over routes of a hash of the RibUnicastEntry fields) and
openr_amd/shard.py (C4 change lists, C5 KSP2 path lines). Every value here
comes from oracle/refcpu (test infrastructure), never from the engine.

  python tests/golden/make_bench_digests.py [c1] [c2] [c3] [c3ref] [c4] [c5] [g1] [--threads T]

C3 takes long (2,080 oracle buildRouteDb over 208k prefixes each, ~1.5 h on
8 cores): it is resumable, per-source digests accumulate in
tests/golden/c3_source_digests.json.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import _refcpu as R  # noqa: E402
from openr_amd import shard  # noqa: E402  (pure Python: digest helpers)
from openr_amd.workloads import (C1_OPTS, C1_SOURCE, C2_OPTS, C2_SOURCE, C2_TOPOS, C3_OPTS, C4_OPTS,  # noqa: E402
                                 C4_SOURCE, C4_VARIANTS, C4_SEED, C4_DUAL_PERMILLE,
                                 C5_OPTS, C5_SOURCE, G1_OPTS, G1_SOURCES, c3_source_names,
                                 c5_policy, C3REF_OPTS, c3ref_sample_names)

OUT = os.path.join(HERE, "bench_digests.json")
C3_PART = os.path.join(HERE, "c3_source_digests.json")
C3REF_PART = os.path.join(HERE, "c3ref_source_digests.json")


def load(path):
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return {}


def save(path, d):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
        f.write("\n")
    os.replace(tmp, path)


def gen_c1(out, threads):
    """C1: the oracle's buildRouteDb("1") on the metric-1 10x10 grid (v4 on,
    SR off, best-route selection off), keyed by the source name."""
    out["c1"] = f"{R.gen_route_digests('grid', C1_OPTS, [C1_SOURCE], True, False, False, 1)[0]:016x}"


def gen_c2(out, threads, blocks=8):
    """Per 4096-topology block (weak scaling: rank r of N owns block r), the
    XOR of the per-topology digests."""
    res = []
    for b in range(blocks):
        d = R.grid_batch_digests(C2_OPTS, b * C2_TOPOS, (b + 1) * C2_TOPOS, C2_SOURCE, False,
                                 threads)
        res.append(f"{shard.combine_digests(d):016x}")
    out["c2_blocks"] = res
    out["c2_block_size"] = C2_TOPOS


def gen_c3(out, threads, chunk):
    names = c3_source_names()
    part = load(C3_PART)
    todo = [n for n in names if n not in part]
    while todo:
        batch, todo = todo[:chunk], todo[chunk:]
        t = time.time()
        ds = R.gen_route_digests("fabric", C3_OPTS, batch, True, False, False, threads)
        for n, d in zip(batch, ds):
            part[n] = f"{d:016x}"
        save(C3_PART, part)
        print(f"c3: {len(part)}/{len(names)} sources ({time.time() - t:.0f} s/chunk)",
              flush=True)
    out["c3"] = f"{shard.combine_digests(int(part[n], 16) for n in names):016x}"


def gen_c3ref(out, threads):
    """C3-ref (the reference's own benchmark fabric, full=False): the
    oracle's per-source digests of 64 stratified sources."""
    names = c3ref_sample_names()
    ds = R.gen_route_digests("fabric", C3REF_OPTS, names, True, False, False, threads)
    save(C3REF_PART, {n: f"{d:016x}" for n, d in zip(names, ds)})
    out["c3ref_sample"] = f"{shard.combine_digests(ds):016x}"


def gen_c4(out, threads):
    ch = R.variant_changes("wan", C4_OPTS, C4_SOURCE, C4_VARIANTS, C4_SEED, C4_DUAL_PERMILLE,
                           threads)
    out["c4"] = f"{shard.changes_digest(range(len(ch)), ch):016x}"
    out["c4_changes"] = sum(u + d for u, d, _ in ch)


def gen_c5(out, threads):
    areas, nbrs = R.multiarea_source_info(C5_OPTS, C5_SOURCE)
    pol = c5_policy(areas, nbrs)
    out["c5_routes"] = f"{R.gen_route_digest_multiarea(C5_OPTS, C5_SOURCE, True, False, True, pol):016x}"
    lines = R.kth_paths_all_multiarea(C5_OPTS, C5_SOURCE, threads)
    out["c5_paths"] = f"{shard.lines_digest(lines):016x}"
    out["c5_ksp_lines"] = len(lines)


def gen_g1(out, threads):
    """Per source the RouteDb digest (key = source name), XOR-combined; and
    the first source's alone (the single-source drop-in sub-line)."""
    ds = R.gen_route_digests("wan", G1_OPTS, G1_SOURCES, True, False, False, threads)
    out["g1"] = f"{shard.combine_digests(ds):016x}"
    out["g1_single"] = f"{ds[0]:016x}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c2", "c4", "c5", "c3"])
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--chunk", type=int, default=64)
    a = ap.parse_args()
    out = load(OUT)
    for c in a.configs:
        t = time.time()
        if c == "c1":
            gen_c1(out, a.threads)
        elif c == "c2":
            gen_c2(out, a.threads)
        elif c == "c3":
            gen_c3(out, a.threads, a.chunk)
        elif c == "c3ref":
            gen_c3ref(out, a.threads)
        elif c == "c4":
            gen_c4(out, a.threads)
        elif c == "c5":
            gen_c5(out, a.threads)
        elif c == "g1":
            gen_g1(out, a.threads)
        else:
            raise SystemExit(f"unknown config {c}")
        out["generator"] = "tests/golden/make_bench_digests.py (oracle/refcpu)"
        save(OUT, out)
        print(f"{c}: done in {time.time() - t:.1f} s", flush=True)


if __name__ == "__main__":
    main()
