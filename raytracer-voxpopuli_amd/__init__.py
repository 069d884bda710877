"""vpx — MI355X-native per-pixel voxel ray-trace path (drop-in for Renderer::Trace).

The product is libvpx_hip.so (csrc/, C-ABI in include/vpx.h).  This package is the host
side around it: ctypes ABI mirror (abi), a context handle (context), the reference
Renderer surface (renderer), scene/world inputs (scene) and tile sharding over
torch.distributed/RCCL (dist).  The directory name is not a Python identifier, so entry
points load it with `load_package()` below (or importlib) under the name `vpx_amd`.
"""
from . import abi  # noqa: F401
from .abi import VpxError, load_library  # noqa: F401


def __getattr__(name):
    import importlib
    if name in ("context", "renderer", "scene", "dist"):
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
