"""Practical HBM write ceiling on this box beside the C3 build: torch's
fill_ (a store-only kernel) over the C3 build's output volume (5.66 GB), and
a copy of half of it (read + write), HIP events, median of 5; then the C3
line on the same box (bench.py --config c3)."""
import subprocess
import sys

import torch


def timed(fn, reps=5):
    ts = []
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[1:])
    return ts[len(ts) // 2]


def main():
    n = 5_660_000_000 // 4
    x = torch.empty(n, dtype=torch.int32, device="cuda")
    ms = timed(lambda: x.fill_(7))
    print(f"fill_ {n * 4 / 1e9:.2f} GB: {ms:.3f} ms = {n * 4 / ms / 1e9:.2f} TB/s", flush=True)
    h = n // 2
    a, b = x[:h], x[h:2 * h]
    ms = timed(lambda: b.copy_(a))
    print(f"copy_ {h * 4 / 1e9:.2f} GB read + write: {ms:.3f} ms = {2 * h * 4 / ms / 1e9:.2f} TB/s",
          flush=True)
    del x, a, b
    torch.cuda.empty_cache()
    r = subprocess.run([sys.executable, "bench.py", "--config", "c3", "--no-cpu-baseline",
                        "--no-extras", "--steps", "10", "--warmup", "2"],
                       capture_output=True, text=True)
    import json
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    d = json.loads(line[-1])
    print("c3", d["ms_per_step"], d["kernel_ms"], d["roofline"]["achieved"], d["roofline"]["frac"])


if __name__ == "__main__":
    main()
