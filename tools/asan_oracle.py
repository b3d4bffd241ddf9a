"""The CPU oracle (oracle/refcpu) under AddressSanitizer / UBSan: imports the
instrumented build/asan/_refcpu (make asan) and runs every transcribed
reference known-answer test (tests/kat_cases.py ALL_KATS) plus generated
fabric / WAN / grid / multi-area RouteDbs, the C4 variant sweep and KSP2 on
small sizes. Run with libasan preloaded (the Makefile's asan target)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "build", "asan"))
sys.path.insert(1, os.path.join(ROOT, "tests"))
sys.path.insert(2, os.path.join(ROOT, "oracle"))  # thrift_compact.py (after build/asan)
import _refcpu as R  # noqa: E402
import kat_cases  # noqa: E402

assert "build/asan" in R.__file__, R.__file__
n = 0
for kat in kat_cases.ALL_KATS:
    kat(R)
    n += 1
mix = dict(v4Permille=150, anycastPermille=150, minNhPermille=60, drainPermille=50,
           nodeOverloadPermille=30, adjOverloadPermille=20)
fab = dict(pods=4, planes=2, sswPerPlane=6, rswPerPod=8, full=True, prefixesPerNode=2, **mix)
names = [f"1-{p}-{s}" for p in range(2) for s in range(6)] + ["2-0-0", "2-3-1", "3-1-7"]
dbs = R.gen_route_dbs("fabric", fab, names, True, True, True)
wan = dict(nodes=200, seed=0xC4, prefixesPerNode=2, **mix)
dbs += R.gen_route_dbs("wan", wan, ["0", "7", "199", "no-such"], True, False, True)
dbs += R.gen_route_dbs("grid", dict(n=6, metricSeed=0xC2000001, prefixesPerNode=2), ["1", "17"],
                       True, False, False)
ma = dict(areas=3, nodesPerArea=40, abrs=4, prefixesPerNode=2, anycastPermille=200)
dbs += R.gen_route_dbs_multiarea(ma, ["abr-0", "a1-7"], True, True, True)
ch = R.variant_changes("wan", dict(nodes=120, seed=0xC4, prefixesPerNode=1), "0", 60, 0xC4F, 500, 2)
lines = R.kth_paths_all_multiarea(dict(areas=2, nodesPerArea=30, abrs=2, prefixesPerNode=1),
                                  "abr-0", 2)
print(f"asan oracle: {n} KATs, {len(dbs)} RouteDbs, {len(ch)} variants, {len(lines)} KSP2 lines ok")
