"""Loader for the in-tree C-ABI library ``neptun_amd/libneptun_gpu.so``.

The library is the product: hand-written gfx950 kernels behind the C ABI in
``include/neptun_gpu.h``.  There is no fallback -- if the library or a GPU is
missing, calls raise ``NeptunGpuError``.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libneptun_gpu.so")
# the same library with the latency form's accesses bounds-checked (Makefile CHECKED):
# test infrastructure for that form's audit, never the product path
CHECKED_LIB_PATH = os.path.join(_HERE, "libneptun_gpu_checked.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "neptun_gpu.h")


class NeptunGpuError(RuntimeError):
    pass


_libs: dict[str, ctypes.CDLL] = {}


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Every function the public header declares (the ABI surface)."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(wg_[a-z0-9_]+)\s*\(", text)))


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """The library at `path` (default: the product), bound and checked against the
    tree's sources; loaded once per path."""
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise NeptunGpuError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (or `make -C neptun_amd/csrc`)")
    L = ctypes.CDLL(path)
    c = ctypes
    vp, u32, u64, i32 = c.c_void_p, c.c_uint32, c.c_uint64, c.c_int32
    L.wg_gpu_abi_version.restype = c.c_int
    L.wg_gpu_last_error.restype = c.c_char_p
    L.wg_gpu_build_id.restype = c.c_char_p
    L.wg_gpu_ctx_create.argtypes = [c.c_int, u32, c.POINTER(vp)]
    L.wg_gpu_ctx_destroy.argtypes = [vp]
    L.wg_gpu_ctx_key_slots.argtypes = [vp]
    L.wg_gpu_ctx_key_slots.restype = u32
    L.wg_gpu_set_keys.argtypes = [vp, u32, u32, vp, vp, vp]
    for fn in (L.wg_gpu_seal_batch, L.wg_gpu_open_batch):
        fn.argtypes = [vp, vp, u32, vp, vp, vp, vp]
    L.wg_gpu_plan_batch.argtypes = [vp, c.c_int, vp, u32, vp, vp, vp]
    for fn in (L.wg_gpu_seal_batch_ordered, L.wg_gpu_open_batch_ordered):
        fn.argtypes = [vp, vp, vp, u32, vp, vp, vp, vp]
    L.wg_gpu_ctx_set_xlane_lanes.argtypes = [vp, c.c_int64]
    L.wg_gpu_ctx_set_split.argtypes = [vp, c.c_int]
    L.wg_gpu_strided_split_parts.argtypes = [vp, c.c_int, u32, u32]
    L.wg_gpu_register_host.argtypes = [vp, vp, u64]
    L.wg_gpu_unregister_host.argtypes = [vp, vp]
    L.wg_gpu_host_device_address.argtypes = [vp, vp, u64, c.POINTER(u64)]
    L.wg_gpu_x25519_batch.argtypes = [vp, u32, vp, vp, vp, vp]
    L.wg_gpu_handshake_anon_batch.argtypes = [vp, c.c_char_p, u32, vp, u64, c.c_int, vp, vp]
    L.wg_gpu_handshake_consume_batch.argtypes = [vp, c.c_char_p, u32, vp, u64, vp, vp, vp]
    L.wg_handshake_timestamp_after.argtypes = [c.c_char_p, c.c_char_p]
    L.wg_gpu_handshake_respond_batch.argtypes = [vp, u32, vp, vp, vp, vp]
    L.wg_gpu_mac2_check_batch.argtypes = [vp, c.c_char_p, u64, u32, vp, u64, vp, vp, vp, vp, vp]
    L.wg_gpu_cookie_reply_batch.argtypes = [vp, c.c_char_p, c.c_char_p, u32, vp, vp, vp]
    L.wg_gpu_handshake_initiate_batch.argtypes = [vp, u32, vp, vp, vp]
    L.wg_gpu_handshake_receive_response_batch.argtypes = [vp, c.c_char_p, u32, vp, u64, c.c_int, vp, vp, vp]
    L.wg_gpu_cookie_reply_open_batch.argtypes = [vp, u32, vp, vp, vp]
    L.wg_gpu_route_set.argtypes = [vp, u32, vp, vp]
    L.wg_gpu_route_batch.argtypes = [vp, vp, u32, vp, vp]
    L.wg_gpu_pipe_create.argtypes = [vp, u64, u32, c.POINTER(vp)]
    L.wg_gpu_pipe_destroy.argtypes = [vp]
    L.wg_gpu_pipe_seal_strided.argtypes = [vp, u32, u32, u32, u64, vp, u64, vp, u64, vp]
    L.wg_gpu_pipe_open_strided.argtypes = [vp, u32, u32, u32, vp, u64, vp, u64, vp]
    L.wg_gpu_seal_strided.argtypes = [vp, u32, u32, u32, u64, vp, u64, vp, u64, vp, vp]
    L.wg_gpu_open_strided.argtypes = [vp, u32, u32, u32, vp, u64, vp, u64, vp, vp]
    L.wg_gpu_debug_xlane_check.argtypes = [c.POINTER(c.c_ulonglong), c.c_int]
    L.wg_gpu_debug_xlane_check.restype = c.c_int
    for name in header_functions():
        fn = getattr(L, name)
        if fn.restype is c.c_int and name not in ("wg_gpu_abi_version",):
            fn.restype = i32
    want = source_build_id()
    got = L.wg_gpu_build_id().decode()
    if want is not None and got != want:
        raise NeptunGpuError(
            f"{path} was built from other sources (build id {got}, tree {want}): rebuild it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C neptun_amd/csrc`)")
    _libs[path] = L
    return L


CSRC = os.path.join(_HERE, "csrc")


def source_build_id() -> str | None:
    """The build id the sources in this tree give (neptun_amd/csrc/Makefile
    SRC_FILES / SRC_HASH: the kernel and host sources, the Makefile and the public
    headers, concatenated in that order); None when the sources are not here."""
    if not os.path.isdir(CSRC):
        return None
    inc = os.path.join(os.path.dirname(_HERE), "include")
    if not os.path.isdir(inc):
        return None
    names = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".h")))
    files = [os.path.join(CSRC, f) for f in names] + [os.path.join(CSRC, "Makefile")]
    files += [os.path.join(inc, f) for f in sorted(os.listdir(inc)) if f.endswith(".h")]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def check(rc: int, what: str, lib: ctypes.CDLL | None = None) -> None:
    if rc != 0:
        msg = (lib or load()).wg_gpu_last_error().decode(errors="replace")
        raise NeptunGpuError(f"{what} failed (rc={rc}): {msg}")
