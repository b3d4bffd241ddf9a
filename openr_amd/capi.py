"""ctypes view of the C-ABI (include/openr_gpu.h) — what a Python consumer of
the boundary binds. bench.py drives the kernel through it with torch-owned
device memory and torch's current HIP stream."""
import ctypes

from . import LIB_PATH

OGS_OK = 0
OGS_ABI_VERSION = 6  # include/openr_gpu.h
OGS_F_ENABLE_V4 = 0x01
OGS_F_V4_OVER_V6 = 0x02
OGS_F_BEST_ROUTE_SELECTION = 0x04
OGS_F_HOP_METRIC = 0x08
OGS_F_WIDE_METRIC = 0x10

# every extern "C" entry point declared in include/openr_gpu.h
EXPORTS = [
    "ogs_version", "ogs_last_error", "ogs_device_count", "ogs_set_device",
    "ogs_malloc", "ogs_free", "ogs_memcpy_h2d", "ogs_memcpy_d2h", "ogs_memset",
    "ogs_stream_sync", "ogs_nh_words_for_degree", "ogs_spf_routes",
    "ogs_ksp_paths", "ogs_ksp2_paths", "ogs_set_option", "ogs_routes_multiarea",
    "ogs_spf_routes_variants", "ogs_rib_policy_apply", "ogs_route_changes_gather",
    "ogs_csr_patch", "ogs_host_alloc", "ogs_host_free", "ogs_routes_from_spf",
    "ogs_abi_version", "ogs_spf_routes_groups",
    "ogs_ctx_create", "ogs_ctx_destroy", "ogs_ctx_set_option", "ogs_ctx_spf_routes",
    "ogs_ctx_spf_routes_groups", "ogs_ctx_routes_from_spf", "ogs_ctx_spf_routes_variants",
    "ogs_ctx_ksp_paths", "ogs_ctx_ksp2_paths", "ogs_ctx_routes_multiarea",
    "ogs_ctx_rib_policy_apply",
]


class Graph(ctypes.Structure):
    _fields_ = [("num_topos", ctypes.c_int32), ("max_nodes", ctypes.c_int32),
                ("max_edges", ctypes.c_int32), ("max_degree", ctypes.c_int32),
                ("node_base", ctypes.c_void_p),
                ("row_ptr", ctypes.c_void_p), ("edges", ctypes.c_void_p),
                ("node_flags", ctypes.c_void_p), ("topo_desc", ctypes.c_void_p),
                ("slot_node", ctypes.c_void_p), ("slot_stride", ctypes.c_int32),
                ("slot_edges", ctypes.c_void_p), ("slot_degree", ctypes.c_int32),
                ("edge_src", ctypes.c_void_p), ("rslot_ext", ctypes.c_void_p)]


class PrefixTable(ctypes.Structure):
    _fields_ = [("max_prefixes", ctypes.c_int32), ("max_advertisements", ctypes.c_int32),
                ("pfx_base", ctypes.c_void_p),
                ("adv_off", ctypes.c_void_p), ("adv_node", ctypes.c_void_p),
                ("adv_metrics", ctypes.c_void_p), ("adv_min_nh", ctypes.c_void_p),
                ("pfx_flags", ctypes.c_void_p)]


class SpfOut(ctypes.Structure):
    _fields_ = [("dist", ctypes.c_void_p), ("nh", ctypes.c_void_p),
                ("meta", ctypes.c_void_p), ("metric", ctypes.c_void_p),
                ("mask", ctypes.c_void_p), ("sel", ctypes.c_void_p),
                ("reached", ctypes.c_void_p)]


class RouteGroup(ctypes.Structure):
    _fields_ = [("units", ctypes.c_void_p), ("n_units", ctypes.c_int32),
                ("nh_words", ctypes.c_int32), ("out", SpfOut)]


def load(path=None):
    lib = ctypes.CDLL(path or LIB_PATH)
    lib.ogs_version.restype = ctypes.c_char_p
    if lib.ogs_abi_version() != OGS_ABI_VERSION:
        raise RuntimeError(f"libopenr_gpu ABI {lib.ogs_abi_version()}, "
                           f"this binding expects {OGS_ABI_VERSION}")
    lib.ogs_last_error.restype = ctypes.c_char_p
    lib.ogs_spf_routes.argtypes = [
        ctypes.POINTER(Graph), ctypes.POINTER(PrefixTable), ctypes.c_void_p,
        ctypes.c_int32, ctypes.c_uint32, ctypes.c_int32, ctypes.POINTER(SpfOut),
        ctypes.c_void_p]
    lib.ogs_spf_routes.restype = ctypes.c_int
    lib.ogs_spf_routes_groups.argtypes = [
        ctypes.POINTER(Graph), ctypes.POINTER(PrefixTable), ctypes.POINTER(RouteGroup),
        ctypes.c_int32, ctypes.c_uint32, ctypes.c_void_p]
    lib.ogs_spf_routes_groups.restype = ctypes.c_int
    lib.ogs_set_option.argtypes = [ctypes.c_char_p, ctypes.c_int64]
    lib.ogs_set_option.restype = ctypes.c_int
    # execution contexts (ABI 6): opaque handles
    lib.ogs_ctx_create.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]
    lib.ogs_ctx_create.restype = ctypes.c_int
    lib.ogs_ctx_destroy.argtypes = [ctypes.c_void_p]
    lib.ogs_ctx_destroy.restype = ctypes.c_int
    lib.ogs_ctx_set_option.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]
    lib.ogs_ctx_set_option.restype = ctypes.c_int
    lib.ogs_ctx_spf_routes.argtypes = [ctypes.c_void_p] + lib.ogs_spf_routes.argtypes
    lib.ogs_ctx_spf_routes.restype = ctypes.c_int
    lib.ogs_ctx_spf_routes_groups.argtypes = ([ctypes.c_void_p] +
                                             lib.ogs_spf_routes_groups.argtypes)
    lib.ogs_ctx_spf_routes_groups.restype = ctypes.c_int
    # the remaining compute entry points: structs this module does not model
    # (ogs_path_unit, ogs_unit_mods, ogs_area_table, ogs_rib_policy, ...)
    # pass as c_void_p, so 64-bit handles and device pointers never go
    # through ctypes' default int conversion
    P, I32, U32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32
    plain = {
        "ogs_routes_from_spf": [P, P, P, I32, P, P, P, U32, I32, P, P],
        "ogs_spf_routes_variants": [P, P, P, I32, P, P, U32, I32, P, P],
        "ogs_ksp_paths": [P, P, I32, P, U32, U32, P, P],
        "ogs_ksp2_paths": [P, P, I32, P, I32, U32, P, P, P],
        "ogs_routes_multiarea": [P, P, P, P, I32, P, P, P, U32, I32, P, P],
        "ogs_rib_policy_apply": [P, P, I32, I32, I32, P, P, P, P, P],
    }
    for name, args in plain.items():
        for fn, a in ((name, args), ("ogs_ctx_" + name[4:], [P] + args)):
            f = getattr(lib, fn)
            f.argtypes = a
            f.restype = ctypes.c_int
    return lib


def check(lib, rc, what):
    if rc != OGS_OK:
        raise RuntimeError(f"{what} failed ({rc}): {lib.ogs_last_error().decode()}")
