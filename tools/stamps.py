"""Phase breakdown of the wave SPF+RouteDb kernel from a diagnostic
(-DOGS_STAMPS) build: cycles in staging / SPF rounds / routes per unit, and
the number of relaxation rounds. Run with OGS_LIB=<stamped lib>;
VARIANTS as in ab_unit_width.py."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c2dev import C2, apply, variants  # noqa: E402


def main():
    import torch
    c = C2(int(os.environ.get("TOPOS", "4096")))  # batch size (contention probe)
    pt = c.table()
    o = c.outputs()
    runs = [(v, o) for v in variants("1,1p")
            for o in [int(x) for x in os.environ.get("WAVE_OPTS", "3").split(",")]]
    for (name, uw, order, lds, use_b, upb), wopt in runs:
        apply(c, uw, lds, use_b, upb)
        c.capi.check(c.lib, c.lib.ogs_set_option(b"wave_opt", wopt), "wave_opt")
        name = f"{name}/opt{wopt}"
        g = c.graph(order)
        for _ in range(3):
            c.run(g, pt, o)
        torch.cuda.synchronize()
        raw = o[5].cpu().numpy().reshape(c.U, c.Sp)[:, :7].astype(np.int64)
        raw = raw[raw[:, 0] > 16]  # rows of wave-first units (others: sel bits)
        st = raw[:, :5].astype(np.float64)
        names = ["stage", "spf", "routes", "rounds", "desc"]
        rt0 = raw[:, 5] - raw[:, 5].min()  # 100 MHz realtime, 10 ns ticks
        rt1 = raw[:, 6] - raw[:, 5].min()
        print(f"variant={name}: wave start (us after first) med={np.median(rt0)/100:.2f} "
              f"p90={np.percentile(rt0, 90)/100:.2f} max={rt0.max()/100:.2f}; "
              f"wave end med={np.median(rt1)/100:.2f} max={rt1.max()/100:.2f}; "
              f"wave life med={np.median(rt1 - rt0)/100:.2f}")
        print(f"variant={name}: " + "  ".join(
            f"{n}: med={np.median(st[:, i]):.0f} p90={np.percentile(st[:, i], 90):.0f} "
            f"max={st[:, i].max():.0f}" for i, n in enumerate(names)))
        print(f"   spf cycles/round (median) = {np.median(st[:, 1] / st[:, 3]):.0f}")


if __name__ == "__main__":
    main()
