"""The C-ABI library loads and exports every symbol include/*.h declares.

No compute calls here (this runs without a GPU).
"""
import ctypes
import re

import numpy as np
import pytest

import neptun_amd
from neptun_amd import gpu as G
from oracle import pyoracle as o


@pytest.mark.parametrize("header", ["neptun_gpu.h", "neptun_tunn.h"])
def test_library_exports_header_symbols(header):
    import os
    lib = neptun_amd.load()
    path = os.path.join(os.path.dirname(neptun_amd.HEADER_PATH), header)
    names = neptun_amd.header_functions(path)
    assert len(names) >= 9
    for name in names:
        assert hasattr(lib, name), f"{name} declared in include/{header} but not exported"
    assert lib.wg_gpu_abi_version() == 1


def test_library_build_id_matches_the_sources(monkeypatch):
    """The shipped .so carries the hash of the sources it was built from; the
    loader refuses one built from other sources (a stale binary)."""
    from neptun_amd import _native
    lib = neptun_amd.load()
    assert lib.wg_gpu_build_id().decode() == _native.source_build_id()
    monkeypatch.setattr(_native, "_libs", {})
    monkeypatch.setattr(_native, "source_build_id", lambda: "0" * 16)
    with pytest.raises(_native.NeptunGpuError, match="other sources"):
        _native.load()


def test_checked_build_is_a_separate_library():
    """libneptun_gpu_checked.so (the latency form's bounds audit) comes from the same
    sources; the product library reports that it is not the checked build."""
    from neptun_amd import _native
    lib = neptun_amd.load()
    chk = _native.load(_native.CHECKED_LIB_PATH)
    assert chk is not lib
    assert chk.wg_gpu_build_id().decode() == _native.source_build_id()
    out = (ctypes.c_ulonglong * 4)()
    assert lib.wg_gpu_debug_xlane_check(out, 0) == -1


def test_tunn_layouts_match_header():
    from neptun_amd.tunn import Replay, TunnResult
    text = open(neptun_amd.HEADER_PATH.replace("neptun_gpu.h", "neptun_tunn.h")).read()
    assert "#define WG_REPLAY_WORDS 16" in text and "#define WG_N_SESSIONS 8" in text
    assert ctypes.sizeof(Replay) == 8 * 18
    assert ctypes.sizeof(TunnResult) == 32


def test_tunn_entry_points_fail_loudly_on_null():
    from neptun_amd.tunn import _bind
    lib = _bind(neptun_amd.load())
    out = ctypes.c_void_p()
    assert lib.wg_tunn_create(None, 0, ctypes.byref(out)) != 0
    assert b"tunn_create" in lib.wg_gpu_last_error()


def test_engine_entry_points_fail_loudly_on_null():
    """wg_engine_* / multi-peer batches refuse null arguments before touching a GPU."""
    from neptun_amd.tunn import EngineInfo, TunnResult, _bind
    lib = _bind(neptun_amd.load())
    out = ctypes.c_void_p()
    assert lib.wg_engine_create(None, ctypes.byref(out)) == -1
    assert b"engine_create" in lib.wg_gpu_last_error()
    assert lib.wg_tunn_create_on(None, 0, ctypes.byref(out)) == -1
    assert lib.wg_engine_get_info(None, ctypes.byref(EngineInfo())) == -1
    assert lib.wg_engine_destroy(None) == 0
    assert lib.wg_tunn_engine(None) is None
    res = (TunnResult * 1)()
    for fn in (lib.wg_tunn_encapsulate_multi, lib.wg_tunn_decapsulate_multi):
        assert fn(None, 1, None, None, None, None, None, res) == -1
        assert b"_multi: null" in lib.wg_gpu_last_error()
    text = open(neptun_amd.HEADER_PATH.replace("neptun_gpu.h", "neptun_tunn.h")).read()
    body = re.search(r"typedef struct wg_engine_info \{(.*?)\}", text, re.S).group(1)
    fields = [(n.strip(), int(w) // 8) for w, decl in re.findall(r"uint(32|64)_t([^;]*);", body)
              for n in decl.split(",")]
    assert [n for n, _ in fields] == [f for f, _ in EngineInfo._fields_]
    assert [ctypes.sizeof(t) for _, t in EngineInfo._fields_] == [w for _, w in fields]
    assert ctypes.sizeof(EngineInfo) == 4 * 6 + 8 * 2  # (the two 64-bit counters 8-aligned after six words)


def test_library_is_gfx950_code_object():
    data = open(neptun_amd.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"aead_strided_kernel" in data and b"aead_desc_kernel" in data


def header_enum():
    text = open(neptun_amd._native.HEADER_PATH).read()
    return {int(v): k for k, v in re.findall(r"WG_STATUS_([A-Z0-9_]+)\s*=\s*(\d+)", text)}


def test_status_codes_follow_wireguard_error_order():
    # neptun/src/noise/errors.rs:4-28, variant index + 1
    variants = ["DestinationBufferTooSmall", "IncorrectPacketLength", "UnexpectedPacket",
                "WrongPacketType", "WrongIndex", "WrongKey", "InvalidTai64nTimestamp",
                "WrongTai64nTimestamp", "InvalidMac", "InvalidAeadTag", "InvalidCounter",
                "DuplicateCounter", "InvalidPacket", "NoCurrentSession", "LockFailed",
                "ConnectionExpired", "UnderLoad", "CryptoFailed", "InvalidLength",
                "InvalidIndex", "RingUnspecifiedError", "SystemTimeError"]
    enum = header_enum()
    for i, v in enumerate(variants, start=1):
        assert G.STATUS[i] == v
        assert enum[i].replace("_", "") == v.upper(), (enum[i], v)


def test_descriptor_layout_matches_header_and_oracle():
    assert G.DESC_DTYPE.itemsize == 32
    assert G.DESC_DTYPE == o.DESC_DTYPE
    text = open(neptun_amd._native.HEADER_PATH).read()
    body = re.search(r"typedef struct wg_packet_desc \{(.*?)\}", text, re.S).group(1)
    fields = re.findall(r"(uint\d+)_t\s+(\w+);", body)
    assert [f for _, f in fields] == list(G.DESC_DTYPE.names)
    assert [int(t[4:]) // 8 for t, _ in fields] == [G.DESC_DTYPE[n].itemsize for n in G.DESC_DTYPE.names]


def test_no_gpu_means_loud_failure():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(neptun_amd.NeptunGpuError, match="no HIP device"):
        neptun_amd.GpuContext(0, 1)


def test_invalid_arguments_rejected_without_launch():
    lib = neptun_amd.load()
    assert lib.wg_gpu_ctx_create(0, 0, ctypes.byref(ctypes.c_void_p())) == -1
    assert lib.wg_gpu_seal_batch(None, None, 1, None, None, None, None) == -1
    assert b"null" in lib.wg_gpu_last_error()
    assert lib.wg_gpu_ctx_set_slot_padding(None, 1) == -1
    assert b"null context" in lib.wg_gpu_last_error()
