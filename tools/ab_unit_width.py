"""A/B of the SPF+RouteDb kernel variants on the C2 batch, interleaved in ONE
process (cdna_hip_programming.md §5.4 rule 24). VARIANTS lists unit_width
values (0 generic, 1/2 wave, 64/128/256 workgroup), suffix "p" = with the
2-colour slot order. Prints median/min kernel time per variant and checks
every variant's outputs are identical."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c2dev import C2, apply, variants  # noqa: E402


def main():
    import torch
    import openr_amd
    openr_amd.require_gpu()
    c = C2()
    pt = c.table()
    stream = torch.cuda.current_stream(c.dev)
    vs = variants("0,1,1p,64")
    outs = {name: c.outputs() for name, *_ in vs}
    times = {name: [] for name, *_ in vs}
    graphs = {o: c.graph(o) for o in (None, "p", "pi")}
    for rnd in range(12):
        for name, uw, order, lds, use_b, upb in vs:
            apply(c, uw, lds, use_b, upb)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                c.run(graphs[order], pt, outs[name], stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if rnd >= 2:
                times[name].append(e0.elapsed_time(e1) / 10)
    ref = outs[vs[0][0]]
    for name, *_ in vs:
        same = all(torch.equal(a, b) for a, b in zip(ref, outs[name]))
        ts = sorted(times[name])
        print(f"variant={name:>5} median={ts[len(ts)//2]*1e3:8.2f} us "
              f"min={ts[0]*1e3:8.2f} us identical={same}")


if __name__ == "__main__":
    main()
