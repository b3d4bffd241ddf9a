"""openr_amd — MI355X (gfx950) SPF + RouteDb engine for Open/R Decision.

The product is the C-ABI library ``openr_amd/lib/libopenr_gpu.so`` (HIP
kernels, include/openr_gpu.h) plus the C++ drop-in of LinkState / PrefixState
/ SpfSolver / RibPolicy (``openr_amd._decision``). There is no CPU route path:
every SPF and route computation runs on the GPU, and a missing device or
extension raises.
"""
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OGS_LIB") or os.path.join(_HERE, "lib", "libopenr_gpu.so")

try:
    from . import _decision as decision  # noqa: F401
except ImportError as e:  # fail loudly: the HIP path is the product
    raise ImportError(
        "openr_amd native extension is not built (run `make` or "
        "__graft_entry__.build()): " + str(e)) from e


def require_gpu():
    """Raise unless a HIP device is visible to libopenr_gpu.so."""
    n = decision.device_count()
    if n <= 0:
        raise RuntimeError("openr_amd: no HIP device visible (the engine has no CPU path)")
    return n
