"""Shared setup for the GPU tools: the C2 batch (4096 10x10 grids, source
"1") uploaded as torch device tensors, with ctypes views of the C-ABI
structs. `order=False` hands the kernel no slot_node (identity order)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEYS = ("topo_desc", "node_base", "row_ptr", "edges", "node_flags", "pfx_base", "adv_off",
        "adv_node", "adv_metrics", "adv_min_nh", "pfx_flags", "units", "slot_node",
        "slot_edges")


class C2:
    def __init__(self, topos=4096, brs=False):
        import torch
        import openr_amd
        import openr_amd.capi as capi
        self.capi = capi
        self.lib = self.liba = capi.load()
        # optional second build of the C-ABI (OGS_LIB_B) for same-process A/B
        self.libb = None
        if os.environ.get("OGS_LIB_B"):
            self.libb = capi.load(os.environ["OGS_LIB_B"])
        br = openr_amd.decision.BatchRunner(True, False, brs)
        br.add_grid_batch(dict(n=10, metricSeed=0xC2000000, prefixSeed=0xC1), 0, topos, "1")
        h = self.h = br.host_arrays()
        dev = self.dev = torch.device("cuda", 0)
        self.t = {k: torch.from_numpy(h[k]).to(dev) for k in KEYS}
        self.U = len(h["units"]) // 2
        self.Sn, self.Sp, self.W = h["max_nodes"], h["max_prefixes"], h["nh_words"]
        self.flags = h["flags"]

    def graph(self, order="pi"):
        image = order == "pi"
        h, t = self.h, self.t
        g = self.capi.Graph(h["num_topos"], self.Sn, h["max_edges"], h["max_degree"],
                            t["node_base"].data_ptr(), t["row_ptr"].data_ptr(),
                            t["edges"].data_ptr(), t["node_flags"].data_ptr(),
                            t["topo_desc"].data_ptr())
        if order:
            g.slot_node = t["slot_node"].data_ptr()
            g.slot_stride = h["slot_stride"]
            if image and h["slot_degree"]:
                g.slot_edges = t["slot_edges"].data_ptr()
                g.slot_degree = h["slot_degree"]
        return g

    def table(self):
        h, t = self.h, self.t
        return self.capi.PrefixTable(self.Sp, h["max_advertisements"], t["pfx_base"].data_ptr(),
                                     t["adv_off"].data_ptr(), t["adv_node"].data_ptr(),
                                     t["adv_metrics"].data_ptr(), t["adv_min_nh"].data_ptr(),
                                     t["pfx_flags"].data_ptr())

    def outputs(self):
        import torch
        U, Sn, Sp, W = self.U, self.Sn, self.Sp, self.W
        return [torch.zeros(n, dtype=torch.int32, device=self.dev) for n in
                (U * Sn, U * W * Sn, U * Sp, U * Sp, U * W * Sp, U * Sp)]

    def run(self, g, pt, o, stream=None):
        so = self.capi.SpfOut(*[x.data_ptr() for x in o])
        rc = self.lib.ogs_spf_routes(ctypes.byref(g), ctypes.byref(pt),
                                     ctypes.c_void_p(self.t["units"].data_ptr()), self.U,
                                     self.flags, self.W, ctypes.byref(so),
                                     ctypes.c_void_p(stream.cuda_stream if stream else 0))
        self.capi.check(self.lib, rc, "ogs_spf_routes")


def variants(default):
    """VARIANTS="1,1p,1pi,1p@81920,1p#b,64": unit_width, suffix p = with
    slot order, pi = slot order + per-position edge image, @B = wave_wg_lds
    option (minimum LDS bytes per workgroup), #b = run through the OGS_LIB_B
    build."""
    out = []
    for x in os.environ.get("VARIANTS", default).split(","):
        spec, _, which = x.partition("#")
        spec, _, upb = spec.partition("^")  # ^U = wave_upb option
        base, _, lds = spec.partition("@")
        uw = int(base.rstrip("pi"))
        flags = base[len(str(uw)):]
        # order: "p" = slot order only, "pi" = slot order + edge image
        order = {"": None, "p": "p", "pi": "pi"}[flags]
        out.append((x, uw, order, int(lds or 0), which == "b", int(upb or 4)))
    return out


def apply(c, uw, lds, use_b=False, upb=4):
    c.lib = c.libb if use_b else c.liba
    c.capi.check(c.lib, c.lib.ogs_set_option(b"unit_width", uw), "unit_width")
    if lds or not use_b:
        c.capi.check(c.lib, c.lib.ogs_set_option(b"wave_wg_lds", lds), "wave_wg_lds")
    if upb != 4 or not use_b:
        c.capi.check(c.lib, c.lib.ogs_set_option(b"wave_upb", upb), "wave_upb")
