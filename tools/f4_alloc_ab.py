"""f4 (publication ingest, host only) under two glibc malloc settings, in
child processes interleaved on one box: the default (freed heap returned to
the kernel, so each timed ingest faults its pages in again) and a trim /
mmap threshold that keeps freed memory in the process (the steady state of a
long-running Decision daemon; production builds of the reference link
jemalloc, which also retains freed pages). Explains the box-to-box spread of
`publication_ingest.prefix_insert_ms`; changes nothing in the product.

  python tools/f4_alloc_ab.py [--reps 2]
"""
import argparse
import json
import os
import subprocess
import sys

CHILD = r"""
import json, openr_amd
M = openr_amd.decision
from openr_amd.workloads import C3_OPTS
p = M.publication_ingest_bench("fabric", dict(C3_OPTS), 3)
print(json.dumps({k: round(p[k], 2) for k in
                  ("ingest_ms", "decode_ms", "prefix_keyed_decode_ms", "prefix_insert_ms",
                   "publication_ms")}))
"""

VARIANTS = {
    "default": {},
    "retain": {"GLIBC_TUNABLES": "glibc.malloc.trim_threshold=4294967295:"
                                 "glibc.malloc.mmap_threshold=33554432"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for rep in range(a.reps):
        for name, env in VARIANTS.items():
            e = dict(os.environ, **env)
            e["PYTHONPATH"] = root + os.pathsep + e.get("PYTHONPATH", "")
            r = subprocess.run([sys.executable, "-c", CHILD], env=e, cwd=root,
                               capture_output=True, text=True, timeout=600)
            out = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            print(json.dumps({"variant": name, "rep": rep,
                              **(json.loads(out[-1]) if out else {"error": r.stderr[-300:]})}),
                  flush=True)


if __name__ == "__main__":
    main()
