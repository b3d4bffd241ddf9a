"""A/B of the C1 drop-in latency (SpfSolver::buildRouteDb("1") on the
10x10 grid, cold = fresh objects, warm = same objects) with an engine option
OPT (required) at the values VALS, interleaved in one process. Used to reject a
caching device allocator behind ogs_malloc / ogs_free (cold 171.9 vs 173.9 us:
the ROCm runtime already sub-allocates small buffers)."""
import os
import sys
from statistics import median

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
C1_OPTS = dict(n=10, prefixSeed=0xC1)  # bench.py C1: createGrid(10) wiring, metric 1


def main():
    import torch  # noqa: F401
    import openr_amd
    import openr_amd.capi as capi
    openr_amd.require_gpu()
    lib = capi.load()
    opt = os.environ["OPT"].encode()
    vals = [int(x) for x in os.environ.get("VALS", "0,1").split(",")]
    res = {v: ([], []) for v in vals}
    for rnd in range(4):
        for v in vals:
            capi.check(lib, lib.ogs_set_option(opt, v), opt.decode())
            cold, warm = openr_amd.decision.build_latency_bench("grid", C1_OPTS, "1", 21)[:2]
            if rnd:
                res[v][0].extend(cold)
                res[v][1].extend(warm)
    for v in vals:
        print(f"{opt.decode()}={v}: cold median {median(res[v][0]):.1f} us, "
              f"warm median {median(res[v][1]):.1f} us", flush=True)


if __name__ == "__main__":
    main()
