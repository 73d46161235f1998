"""MI355X-native per-pixel path-tracing kernel for the Trippasch/CudaRayTracer render path.

The product is librt_hip.so (hand-written HIP for gfx950, C ABI in include/rt_hip.h); this package is the
host-side mirror of the reference caller over that ABI:

    abi       ctypes mirror of include/rt_hip.h
    scenes    scene descriptions, built-in scenes, BASELINE configurations, camera → InputStruct
    renderer  Renderer / DeviceScene (CudaLayer's buffers, RNG init, per-frame launch)
    parallel  block-cyclic row-band tiling across ranks + gather over torch.distributed (RCCL)
"""
from . import abi  # noqa: F401

__all__ = ["abi"]
