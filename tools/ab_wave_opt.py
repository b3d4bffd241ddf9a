"""A/B of the wave kernel's paths (option "wave_opt": bit0 = ds_bpermute
SPF words, bit1 = identity-segment route path, bit2 = two units per wave
with 16-bit words) on the C2 batch, interleaved in ONE process against the
base build OGS_LIB_B (without it: this build at wave_opt 2, one unit per
wave); checks every variant's outputs are identical to the base's. SEL=0
hands the kernel no sel output (as bench.py)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c2dev import C2  # noqa: E402


def main():
    import torch
    import openr_amd
    openr_amd.require_gpu()
    c = C2()
    pt = c.table()
    stream = torch.cuda.current_stream(c.dev)
    g = c.graph("pi")
    # OPTS: "wave_opt/wave_upb" pairs, e.g. "2/4,2/8"
    opts = [tuple(int(y) for y in x.split("/")) for x in
            os.environ.get("OPTS", "0/4,2/4,3/4,2/8").split(",")]
    vs = [("base", None)] + [(f"o{o[0]}b{o[1]}", o) for o in opts]
    sel = os.environ.get("SEL", "1") == "1"
    outs = {n: c.outputs() for n, _ in vs}
    times = {n: [] for n, _ in vs}
    for rnd in range(14):
        for name, o in vs:
            c.lib = c.libb if (o is None and c.libb is not None) else c.liba
            if o is None and c.libb is None:
                o = (2, 4)
            if o is not None:
                c.capi.check(c.lib, c.lib.ogs_set_option(b"wave_opt", o[0]), "wave_opt")
                c.capi.check(c.lib, c.lib.ogs_set_option(b"wave_upb", o[1]), "wave_upb")
            out = outs[name] if sel else outs[name][:5] + [None]
            so = c.capi.SpfOut(*[x.data_ptr() if x is not None else None for x in out])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                rc = c.lib.ogs_spf_routes(ctypes.byref(g), ctypes.byref(pt),
                                          ctypes.c_void_p(c.t["units"].data_ptr()), c.U,
                                          c.flags, c.W, ctypes.byref(so),
                                          ctypes.c_void_p(stream.cuda_stream))
                c.capi.check(c.lib, rc, "ogs_spf_routes")
            e1.record(stream)
            torch.cuda.synchronize()
            if rnd >= 2:
                times[name].append(e0.elapsed_time(e1) / 20)
    ref = outs["base"]
    n = 6 if sel else 5
    for name, _ in vs:
        same = all(torch.equal(a, b) for a, b in zip(ref[:n], outs[name][:n]))
        ts = sorted(times[name])
        print(f"variant={name:>5} median={ts[len(ts)//2]*1e3:8.2f} us "
              f"min={ts[0]*1e3:8.2f} us identical={same}", flush=True)


if __name__ == "__main__":
    main()
