"""Phase breakdown of the wave SPF+RouteDb kernel from a diagnostic
(-DOGS_STAMPS) build: cycles in staging / SPF rounds / routes per unit, and
the number of relaxation rounds. Run with OGS_LIB=<stamped lib>;
VARIANTS as in ab_unit_width.py."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c2dev import C2, variants  # noqa: E402


def main():
    import torch
    c = C2()
    pt = c.table()
    o = c.outputs()
    for name, uw, order in variants("1,1p"):
        c.capi.check(c.lib, c.lib.ogs_set_option(b"unit_width", uw), "opt")
        g = c.graph(order)
        for _ in range(3):
            c.run(g, pt, o)
        torch.cuda.synchronize()
        st = o[5].cpu().numpy().reshape(c.U, c.Sp)[:, :6].astype(np.float64)
        names = ["stage", "spf", "routes", "rounds", "desc", "evals"]
        print(f"variant={name}: " + "  ".join(
            f"{n}: med={np.median(st[:, i]):.0f} p90={np.percentile(st[:, i], 90):.0f} "
            f"max={st[:, i].max():.0f}" for i, n in enumerate(names)))
        print(f"   spf cycles/round (median) = {np.median(st[:, 1] / st[:, 3]):.0f}")


if __name__ == "__main__":
    main()
