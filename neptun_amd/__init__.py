"""neptun_amd -- MI355X-native WireGuard transport-data AEAD for NepTUN.

The product is ``libneptun_gpu.so`` (C ABI: include/neptun_gpu.h) built from
``neptun_amd/csrc``; this package is its Python face (ctypes) plus the batched
host-side Tunn semantics.  See DESIGN.md.
"""
from ._native import NeptunGpuError, HEADER_PATH, LIB_PATH, header_functions, load
from .gpu import DESC_DTYPE, STATUS, GpuContext, GpuPipe
from . import tunn
from .tunn import Engine, ReplayWindow, Tunn

__all__ = ["NeptunGpuError", "HEADER_PATH", "LIB_PATH", "header_functions", "load", "DESC_DTYPE", "STATUS",
           "GpuContext", "GpuPipe", "Engine", "ReplayWindow", "Tunn", "tunn"]
