"""Batched Tunn data plane (include/neptun_tunn.h) -- Python face.

`Tunn.encapsulate_batch` / `decapsulate_batch` return what N sequential calls
of neptun's Tunn::encapsulate / Tunn::decapsulate return
(/root/reference/neptun/src/noise/mod.rs:295-380), with the AEAD of the whole
batch on the GPU.  Results mirror TunnResult: (kind, status, len, ip_version,
src_ip); kinds DONE / ERR / WRITE_TO_NETWORK / WRITE_TO_TUNNEL, plus NOT_DATA
for handshake/cookie messages the CPU Tunn must handle.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import check, load
from .gpu import GpuContext

DONE, ERR, WRITE_TO_NETWORK, WRITE_TO_TUNNEL, NOT_DATA = 0, 1, 2, 3, 4
N_SESSIONS = 8


class Replay(ctypes.Structure):
    """wg_replay: ReceivingKeyCounterValidator (session.rs:40-48)."""
    _fields_ = [("next", ctypes.c_uint64), ("receive_cnt", ctypes.c_uint64),
                ("bitmap", ctypes.c_uint64 * 16)]


class TunnResult(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("status", ctypes.c_int32), ("len", ctypes.c_uint32),
                ("ip_version", ctypes.c_uint8), ("src_ip", ctypes.c_uint8 * 16),
                ("pad", ctypes.c_uint8 * 3)]


class Phases(ctypes.Structure):
    """wg_tunn_phases: where a Tunn's batch time goes (cumulative, microseconds)."""
    _fields_ = [("calls", ctypes.c_uint64), ("chunks", ctypes.c_uint64), ("packets", ctypes.c_uint64)] + [
        (f, ctypes.c_double) for f in ("total_us", "checks_us", "pack_us", "submit_us", "wait_us",
                                       "decide_us", "copy_out_us", "dev_h2d_us", "dev_kernel_us",
                                       "dev_d2h_us", "pack_spec_us", "prep_us")]

    def as_dict(self):
        return {f: (round(getattr(self, f), 1) if isinstance(getattr(self, f), float) else getattr(self, f))
                for f, _ in self._fields_}


class EngineInfo(ctypes.Structure):
    """wg_engine_info: what a shared engine holds."""
    _fields_ = [(f, ctypes.c_uint32) for f in ("tunns", "lanes", "max_lanes", "pool_threads", "streams",
                                               "combined")] + [(f, ctypes.c_uint64) for f in
                                                               ("served", "service_launches")]


def _bind(L):
    if getattr(L, "_tunn_bound", False):
        return L
    c = ctypes
    vp, u32, u64 = c.c_void_p, c.c_uint32, c.c_uint64
    L.wg_replay_init.argtypes = [c.POINTER(Replay)]
    L.wg_replay_init.restype = None
    L.wg_replay_will_accept.argtypes = [c.POINTER(Replay), u64]
    L.wg_replay_mark_did_receive.argtypes = [c.POINTER(Replay), u64]
    L.wg_tunn_create.argtypes = [vp, u32, c.POINTER(vp)]
    L.wg_tunn_destroy.argtypes = [vp]
    L.wg_tunn_install_session.argtypes = [vp, u32, u32, c.c_char_p, c.c_char_p, c.c_int]
    L.wg_tunn_stats.argtypes = [vp, c.POINTER(u64), c.POINTER(u64)]
    L.wg_tunn_set_time.argtypes = [vp, u64]
    L.wg_tunn_create_multi.argtypes = [c.POINTER(vp), u32, u32, c.POINTER(vp)]
    L.wg_tunn_engines.argtypes = [vp]
    L.wg_tunn_engines.restype = u32
    L.wg_tunn_engine_info.argtypes = [vp, u32, c.POINTER(c.c_int), c.POINTER(c.c_int)]
    L.wg_tunn_session_counters.argtypes = [vp, u32, c.POINTER(u64), c.POINTER(Replay)]
    L.wg_tunn_get_phases.argtypes = [vp, c.POINTER(Phases)]
    L.wg_tunn_reset_phases.argtypes = [vp]
    L.wg_tunn_set_phase_timing.argtypes = [vp, c.c_int]
    for fn in (L.wg_tunn_encapsulate_batch, L.wg_tunn_decapsulate_batch, L.wg_tunn_decrypt_batch):
        fn.argtypes = [vp, u32, vp, vp, vp, vp, c.POINTER(TunnResult)]
    L.wg_engine_create.argtypes = [vp, c.POINTER(vp)]
    L.wg_engine_destroy.argtypes = [vp]
    L.wg_engine_get_info.argtypes = [vp, c.POINTER(EngineInfo)]
    L.wg_tunn_create_on.argtypes = [vp, u32, c.POINTER(vp)]
    L.wg_tunn_engine.argtypes = [vp]
    L.wg_tunn_engine.restype = vp
    for fn in (L.wg_tunn_encapsulate_multi, L.wg_tunn_decapsulate_multi):
        fn.argtypes = [vp, u32, vp, vp, vp, vp, vp, c.POINTER(TunnResult)]
    L._tunn_bound = True
    return L


class ReplayWindow:
    """The C++ replay window on its own (no GPU needed)."""

    def __init__(self):
        self._lib = _bind(load())
        self.w = Replay()
        self._lib.wg_replay_init(ctypes.byref(self.w))

    def will_accept(self, counter: int) -> int:
        return self._lib.wg_replay_will_accept(ctypes.byref(self.w), counter)

    def mark_did_receive(self, counter: int) -> int:
        return self._lib.wg_replay_mark_did_receive(ctypes.byref(self.w), counter)


def _packet_arrays(blobs, dsts):
    """ctypes pointer / length arrays over Python byte strings and bytearrays (kept alive)."""
    n = len(blobs)
    keep = [ctypes.create_string_buffer(bytes(s), max(len(s), 1)) for s in blobs]
    src_ptr = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in keep])
    src_len = (ctypes.c_uint32 * n)(*[len(s) for s in blobs])
    dbufs = [(ctypes.c_uint8 * max(len(d), 1)).from_buffer(d) if len(d) else
             (ctypes.c_uint8 * 1)() for d in dsts]
    dst_ptr = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in dbufs])
    dst_cap = (ctypes.c_uint32 * n)(*[len(d) for d in dsts])
    return (keep, dbufs), src_ptr, src_len, dst_ptr, dst_cap


def _results(res):
    return [(r.kind, r.status, r.len, r.ip_version, bytes(r.src_ip)) for r in res]


class Engine:
    """wg_engine: a per-GPU engine (host pool, lanes of streams and staging) that any
    number of Tunns share; multi-peer batches mix packets of its Tunns."""

    _close_order = 1  # (GpuContext.close: Tunns and pipes before engines)

    def __init__(self, ctx):
        self._lib = _bind(ctx._lib)
        self._ctx = ctx
        h = ctypes.c_void_p()
        check(self._lib.wg_engine_create(ctx._h, ctypes.byref(h)), "wg_engine_create")
        self._h = h
        ctx._attach(self)

    def tunn(self, first_slot: int) -> "Tunn":
        """A Tunn on this engine over key slots [first_slot, first_slot + 16) of the
        context (refused if a live Tunn on the context holds any of them)."""
        return Tunn(self._ctx, first_slot, engine=self)

    def info(self) -> dict:
        i = EngineInfo()
        check(self._lib.wg_engine_get_info(self._h, ctypes.byref(i)), "wg_engine_get_info")
        return {f: getattr(i, f) for f, _ in EngineInfo._fields_}

    def close(self):
        if getattr(self, "_h", None):
            check(self._lib.wg_engine_destroy(self._h), "wg_engine_destroy")
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        # (its Tunns keep it alive; one attached through the C ABI alone keeps the
        # engine too: wg_engine_destroy refuses while Tunns are attached)
        try:
            self.close()
        except Exception:
            pass

    def _multi(self, fn, name, tunns, blobs, dsts):
        n = len(blobs)
        keep, sp, sl, dp, dc = _packet_arrays(blobs, dsts)
        th = (ctypes.c_void_p * n)(*[t._h.value for t in tunns])
        res = (TunnResult * n)()
        check(fn(self._h, n, th, sp, sl, dp, dc, res), name)
        return _results(res)

    def encapsulate_multi(self, tunns, srcs, dsts):
        """packet i through tunns[i] (wg_tunn_encapsulate_multi)."""
        return self._multi(self._lib.wg_tunn_encapsulate_multi, "wg_tunn_encapsulate_multi", tunns, srcs, dsts)

    def decapsulate_multi(self, tunns, datagrams, dsts):
        return self._multi(self._lib.wg_tunn_decapsulate_multi, "wg_tunn_decapsulate_multi", tunns, datagrams,
                           dsts)

    def _multi_ptrs(self, fn, name, tunn_ptrs, src_ptrs, src_lens, dst_ptrs, dst_caps):
        n = len(src_ptrs)
        res = (TunnResult * n)()
        vp = ctypes.c_void_p
        check(fn(self._h, n, vp(tunn_ptrs.ctypes.data), vp(src_ptrs.ctypes.data), vp(src_lens.ctypes.data),
                 vp(dst_ptrs.ctypes.data), vp(dst_caps.ctypes.data), res), name)
        return _results(res)

    def encapsulate_multi_ptrs(self, tunn_ptrs, src_ptrs, src_lens, dst_ptrs, dst_caps):
        """over raw addresses: tunn_ptrs / src_ptrs / dst_ptrs numpy uint64, lens / caps uint32"""
        return self._multi_ptrs(self._lib.wg_tunn_encapsulate_multi, "wg_tunn_encapsulate_multi", tunn_ptrs,
                                src_ptrs, src_lens, dst_ptrs, dst_caps)

    def decapsulate_multi_ptrs(self, tunn_ptrs, src_ptrs, src_lens, dst_ptrs, dst_caps):
        return self._multi_ptrs(self._lib.wg_tunn_decapsulate_multi, "wg_tunn_decapsulate_multi", tunn_ptrs,
                                src_ptrs, src_lens, dst_ptrs, dst_caps)


def _multi_across(name, tunns, blobs, dsts):
    L = tunns[0]._lib
    n = len(blobs)
    keep, sp, sl, dp, dc = _packet_arrays(blobs, dsts)
    th = (ctypes.c_void_p * n)(*[t._h.value for t in tunns])
    res = (TunnResult * n)()
    check(getattr(L, name)(None, n, th, sp, sl, dp, dc, res), name)
    return _results(res)


def encapsulate_multi(tunns, srcs, dsts):
    """packet i through tunns[i], the Tunns on any engines (one per GPU, say):
    wg_tunn_encapsulate_multi with no engine -- split by engine, shares run
    concurrently, results in packet order."""
    return _multi_across("wg_tunn_encapsulate_multi", tunns, srcs, dsts)


def decapsulate_multi(tunns, datagrams, dsts):
    return _multi_across("wg_tunn_decapsulate_multi", tunns, datagrams, dsts)


def multi_ptrs(seal: bool, tunn_ptrs, src_ptrs, src_lens, dst_ptrs, dst_caps, lib):
    """The engine-free multi-peer call over raw addresses (numpy uint64 / uint32)."""
    n = len(src_ptrs)
    res = (TunnResult * n)()
    vp = ctypes.c_void_p
    name = "wg_tunn_encapsulate_multi" if seal else "wg_tunn_decapsulate_multi"
    check(getattr(lib, name)(None, n, vp(tunn_ptrs.ctypes.data), vp(src_ptrs.ctypes.data),
                             vp(src_lens.ctypes.data), vp(dst_ptrs.ctypes.data), vp(dst_caps.ctypes.data), res),
          name)
    return _results(res)


class Tunn:
    """Tunn mirror bound to a GpuContext; uses 16 key slots from `first_slot`."""

    _close_order = 0  # (GpuContext.close: Tunns and pipes before engines)

    def __init__(self, ctx, first_slot: int = 0, engine: Engine | None = None):
        """ctx: one GpuContext (the Tunn attaches to its default engine, or to `engine`),
        or a list of them (wg_tunn_create_multi: batches are split across the contexts' GPUs)."""
        ctxs = list(ctx) if isinstance(ctx, (list, tuple)) else [ctx]
        self._lib = _bind(ctxs[0]._lib)
        self._ctx = ctxs
        self._engine = engine  # (kept alive while the Tunn is)
        h = ctypes.c_void_p()
        if engine is not None:
            check(self._lib.wg_tunn_create_on(engine._h, first_slot, ctypes.byref(h)), "wg_tunn_create_on")
        elif len(ctxs) == 1:
            check(self._lib.wg_tunn_create(ctxs[0]._h, first_slot, ctypes.byref(h)), "wg_tunn_create")
        else:
            arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value if isinstance(c._h, ctypes.c_void_p) else c._h
                                                  for c in ctxs])
            check(self._lib.wg_tunn_create_multi(arr, len(ctxs), first_slot, ctypes.byref(h)),
                  "wg_tunn_create_multi")
        self._h = h
        for c in ctxs:
            c._attach(self)

    def engines(self):
        """[(device, numa_node)] of the Tunn's engines."""
        out = []
        for e in range(self._lib.wg_tunn_engines(self._h)):
            d, n = ctypes.c_int(), ctypes.c_int()
            check(self._lib.wg_tunn_engine_info(self._h, e, ctypes.byref(d), ctypes.byref(n)),
                  "wg_tunn_engine_info")
            out.append((d.value, n.value))
        return out

    def close(self):
        if getattr(self, "_h", None):
            self._lib.wg_tunn_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def install_session(self, local_index, peer_index, recv_key: bytes, send_key: bytes,
                        make_current: bool = True):
        check(self._lib.wg_tunn_install_session(self._h, local_index, peer_index, recv_key,
                                                send_key, 1 if make_current else 0),
              "wg_tunn_install_session")

    def set_time(self, now: int):
        """timers[TimeCurrent] (the session timer the next install_session records)."""
        check(self._lib.wg_tunn_set_time(self._h, now), "wg_tunn_set_time")

    def _batch_ptrs(self, fn, name, src_ptrs, src_lens, dst_ptrs, dst_caps):
        """Batch over raw addresses (numpy uint64 / uint32 arrays); returns the results."""
        n = len(src_ptrs)
        res = (TunnResult * n)()
        vp = ctypes.c_void_p
        check(fn(self._h, n, vp(src_ptrs.ctypes.data), vp(src_lens.ctypes.data),
                 vp(dst_ptrs.ctypes.data), vp(dst_caps.ctypes.data), res), name)
        return [(r.kind, r.status, r.len, r.ip_version, bytes(r.src_ip)) for r in res]

    def encapsulate_ptrs(self, src_ptrs, src_lens, dst_ptrs, dst_caps):
        return self._batch_ptrs(self._lib.wg_tunn_encapsulate_batch, "wg_tunn_encapsulate_batch",
                                src_ptrs, src_lens, dst_ptrs, dst_caps)

    def decapsulate_ptrs(self, src_ptrs, src_lens, dst_ptrs, dst_caps):
        return self._batch_ptrs(self._lib.wg_tunn_decapsulate_batch, "wg_tunn_decapsulate_batch",
                                src_ptrs, src_lens, dst_ptrs, dst_caps)

    def decrypt_ptrs(self, src_ptrs, src_lens, dst_ptrs, dst_caps):
        return self._batch_ptrs(self._lib.wg_tunn_decrypt_batch, "wg_tunn_decrypt_batch",
                                src_ptrs, src_lens, dst_ptrs, dst_caps)

    def stats(self):
        tx, rx = ctypes.c_uint64(), ctypes.c_uint64()
        check(self._lib.wg_tunn_stats(self._h, ctypes.byref(tx), ctypes.byref(rx)), "wg_tunn_stats")
        return tx.value, rx.value

    def phases(self, reset: bool = False) -> dict:
        """Cumulative phase times (wg_tunn_get_phases); reset=True zeroes them after."""
        p = Phases()
        check(self._lib.wg_tunn_get_phases(self._h, ctypes.byref(p)), "wg_tunn_get_phases")
        if reset:
            check(self._lib.wg_tunn_reset_phases(self._h), "wg_tunn_reset_phases")
        return p.as_dict()

    def set_phase_timing(self, on: bool):
        check(self._lib.wg_tunn_set_phase_timing(self._h, int(bool(on))), "wg_tunn_set_phase_timing")

    def session_counters(self, ring_slot):
        c, w = ctypes.c_uint64(), Replay()
        check(self._lib.wg_tunn_session_counters(self._h, ring_slot, ctypes.byref(c),
                                                 ctypes.byref(w)), "wg_tunn_session_counters")
        return c.value, w

    def _batch(self, fn, name, srcs, dsts):
        n = len(srcs)
        keep, src_ptr, src_len, dst_ptr, dst_cap = _packet_arrays(srcs, dsts)
        res = (TunnResult * n)()
        check(fn(self._h, n, src_ptr, src_len, dst_ptr, dst_cap, res), name)
        return _results(res)

    def encapsulate_batch(self, srcs: list[bytes], dsts: list[bytearray]):
        return self._batch(self._lib.wg_tunn_encapsulate_batch, "wg_tunn_encapsulate_batch",
                           srcs, dsts)

    def decapsulate_batch(self, datagrams: list[bytes], dsts: list[bytearray]):
        return self._batch(self._lib.wg_tunn_decapsulate_batch, "wg_tunn_decapsulate_batch",
                           datagrams, dsts)

    def decrypt_batch(self, datagrams: list[bytes], dsts: list[bytearray]):
        """xray Tunn::decrypt per datagram (no replay window)."""
        return self._batch(self._lib.wg_tunn_decrypt_batch, "wg_tunn_decrypt_batch",
                           datagrams, dsts)
