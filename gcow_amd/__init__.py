"""gcow_amd -- MI355X-native ZFP-style gradient codec (drop-in for fpgasystems/gcow's sw/ encoder/decoder).

The product is libgcow.so (gcow_amd/lib, C ABI in include/gcow.h): hand-written gfx950 HIP kernels behind the
reference's sw/ call surface. This package is the Python host binding: ctypes over the C ABI, torch for device
memory, streams and torch.distributed (RCCL).
"""
from ._ffi import GcowError, GcowParams, load  # noqa: F401

__all__ = ["GcowError", "GcowParams", "load", "codec", "dist"]


def __getattr__(name):
    # codec / dist import torch; keep `import gcow_amd` light for the C-ABI-only callers.
    if name in ("codec", "dist"):
        import importlib
        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)
