"""A/B of the global-state SPF path on the G1 workload (20,000-node WAN, 64
sources, one launch): option OPT (default spf_global_sync) at the values in
VALS, interleaved in one process; prints median launch time per value and
checks every value's RouteDb digest equals the golden one."""
import json
import os
import sys
import time
from statistics import median

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import openr_amd
    import openr_amd.capi as capi
    from openr_amd import shard
    from openr_amd.workloads import G1_OPTS, G1_SOURCES
    openr_amd.require_gpu()
    opt = os.environ.get("OPT", "spf_global_sync").encode()
    vals = [int(x) for x in os.environ.get("VALS", "0,1").split(",")]
    lib = capi.load()
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_digests.json"))).get("g1")
    br = openr_amd.decision.BatchRunner(True, False, False)
    br.add_generated("wan", G1_OPTS, G1_SOURCES)
    br.upload()
    times = {v: [] for v in vals}
    for rnd in range(6):
        for v in vals:
            capi.check(lib, lib.ogs_set_option(opt, v), opt.decode())
            t0 = time.perf_counter()
            br.run()
            dt = time.perf_counter() - t0
            if rnd >= 1:
                times[v].append(dt)
            if rnd == 5:
                br.download()
                d = shard.combine_digests(br.unit_digest(u, G1_SOURCES[u])
                                          for u in range(len(G1_SOURCES)))
                print(f"{opt.decode()}={v}: median {median(times[v]) * 1e3:.3f} ms "
                      f"min {min(times[v]) * 1e3:.3f} ms digest {d:016x} "
                      f"golden={'match' if f'{d:016x}' == golden else 'MISMATCH'}", flush=True)
    capi.check(lib, lib.ogs_set_option(opt, 1 if opt == b"spf_global_sync" else 0), "reset")


if __name__ == "__main__":
    main()
