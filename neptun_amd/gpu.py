"""Python face of the MI355X AEAD batch path (thin wrapper over the C ABI).

Mirrors what NepTUN's Rust side would bind: a context per GPU
holding the device key table (Session::new's keys, session.rs:160-180), batch
seal = N x Session::format_packet_data (session.rs:205-259), batch open = N x
Session::receive_packet_data without the replay window (session.rs:265-302).
PyTorch is used only for device memory and streams; the arithmetic is the
hand-written gfx950 kernels in neptun_amd/csrc/wg_aead.hip.
"""
from __future__ import annotations

import ctypes
import weakref

import numpy as np

from ._native import NeptunGpuError, check, load

DATA_OFFSET = 16        # session.rs:31
AEAD_SIZE = 16          # session.rs:33
DATA_OVERHEAD_SZ = 32   # noise/mod.rs:91

# wg_packet_desc (include/neptun_gpu.h), 32 bytes
DESC_DTYPE = np.dtype([("src_off", "<u8"), ("dst_off", "<u8"), ("counter", "<u8"),
                       ("len", "<u4"), ("key_slot", "<u4")])

# per-packet status = WireGuardError index + 1 (neptun/src/noise/errors.rs:4-28)
KEY_SLOT_NO_SESSION = 0xFFFFFFFF       # include/neptun_gpu.h WG_KEY_SLOT_NO_SESSION
KEY_SLOT_INVALID_PACKET = 0xFFFFFFFE   # WG_KEY_SLOT_INVALID_PACKET

HALF_HANDSHAKE_DTYPE = np.dtype([("peer_index", "<u4"), ("status", "<i4"),
                                 ("peer_static_public", "u1", (32,))])  # wg_half_handshake
# include/neptun_gpu.h responder / cookie records
RESPONDER_PEER_DTYPE = np.dtype([("peer_static_public", "u1", 32), ("static_shared", "u1", 32)])
INIT_RECEIVED_DTYPE = np.dtype([("status", "<i4"), ("peer_index", "<u4"), ("timestamp", "u1", 12),
                                ("chaining_key", "u1", 32), ("hash", "u1", 32),
                                ("peer_ephemeral", "u1", 32), ("pad", "u1", 12)])
RESPONSE_JOB_DTYPE = np.dtype([("ephemeral_private", "u1", 32), ("peer_static_public", "u1", 32),
                               ("preshared_key", "u1", 32), ("mac1_key", "u1", 32),
                               ("cookie", "u1", 16), ("local_index", "<u4"), ("has_cookie", "<u4"),
                               ("pad", "u1", 8)])
RESPONSE_OUT_DTYPE = np.dtype([("message", "u1", 92), ("pad", "u1", 4), ("receiving_key", "u1", 32),
                               ("sending_key", "u1", 32), ("mac1", "u1", 16)])
COOKIE_REPLY_JOB_DTYPE = np.dtype([("cookie", "u1", 16), ("mac1", "u1", 16), ("nonce_ctr", "<u8"),
                                   ("receiver_idx", "<u4"), ("pad", "<u4")])
assert (RESPONDER_PEER_DTYPE.itemsize, INIT_RECEIVED_DTYPE.itemsize, RESPONSE_JOB_DTYPE.itemsize,
        RESPONSE_OUT_DTYPE.itemsize, COOKIE_REPLY_JOB_DTYPE.itemsize) == (64, 128, 160, 176, 48)
# initiator side (include/neptun_gpu.h)
INITIATION_JOB_DTYPE = np.dtype([("ephemeral_private", "u1", 32), ("static_public", "u1", 32),
                                 ("peer_static_public", "u1", 32), ("static_shared", "u1", 32),
                                 ("mac1_key", "u1", 32), ("cookie", "u1", 16), ("timestamp", "u1", 12),
                                 ("local_index", "<u4"), ("has_cookie", "<u4"), ("pad", "u1", 12)])
INIT_SENT_DTYPE = np.dtype([("message", "u1", 148), ("local_index", "<u4"), ("chaining_key", "u1", 32),
                            ("hash", "u1", 32), ("mac1", "u1", 16)])
RESPONSE_RECEIVED_JOB_DTYPE = np.dtype([("chaining_key", "u1", 32), ("hash", "u1", 32),
                                        ("ephemeral_private", "u1", 32), ("preshared_key", "u1", 32)])
SESSION_KEYS_DTYPE = np.dtype([("status", "<i4"), ("peer_index", "<u4"), ("sending_key", "u1", 32),
                               ("receiving_key", "u1", 32), ("receiver_idx", "<u4"), ("pad", "<u4")])
COOKIE_OPEN_JOB_DTYPE = np.dtype([("message", "u1", 64), ("cookie_key", "u1", 32), ("mac1", "u1", 16)])
COOKIE_OPEN_OUT_DTYPE = np.dtype([("status", "<i4"), ("receiver_idx", "<u4"), ("cookie", "u1", 16)])
assert (INITIATION_JOB_DTYPE.itemsize, INIT_SENT_DTYPE.itemsize, RESPONSE_RECEIVED_JOB_DTYPE.itemsize,
        SESSION_KEYS_DTYPE.itemsize, COOKIE_OPEN_JOB_DTYPE.itemsize,
        COOKIE_OPEN_OUT_DTYPE.itemsize) == (208, 232, 128, 80, 112, 24)

STATUS = {
    0: "Ok", 1: "DestinationBufferTooSmall", 2: "IncorrectPacketLength", 3: "UnexpectedPacket",
    4: "WrongPacketType", 5: "WrongIndex", 6: "WrongKey", 7: "InvalidTai64nTimestamp",
    8: "WrongTai64nTimestamp", 9: "InvalidMac", 10: "InvalidAeadTag", 11: "InvalidCounter",
    12: "DuplicateCounter", 13: "InvalidPacket", 14: "NoCurrentSession", 15: "LockFailed",
    16: "ConnectionExpired", 17: "UnderLoad", 18: "CryptoFailed", 19: "InvalidLength",
    20: "InvalidIndex", 21: "RingUnspecifiedError", 22: "SystemTimeError",
    100: "Misaligned", 101: "BadKeySlot",
}
OK = 0
INVALID_AEAD_TAG = 10
INVALID_PACKET = 13
WRONG_INDEX = 5


def _ptr(x) -> int:
    """Device pointer of a torch tensor (or an int already)."""
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    return int(x.data_ptr())


def _stream(stream) -> int:
    if stream is None:
        import torch
        return int(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


class GpuContext:
    """One GPU + device key table.  Replaces per-session ring keys."""

    def __init__(self, device: int = 0, key_slots: int = 1, lib_path: str | None = None):
        # (the Tunns, engines and pipes made on it: their native objects refer to it, so
        # close() closes them first -- Tunns and pipes, then engines)
        self._dependents = weakref.WeakSet()
        # lib_path: another build of the same sources (the tests' checked build)
        self._lib = load(lib_path) if lib_path else load()
        h = ctypes.c_void_p()
        check(self._lib.wg_gpu_ctx_create(device, key_slots, ctypes.byref(h)), "wg_gpu_ctx_create")
        self._h = h
        self.device = device
        self.key_slots = key_slots

    def xlane_check(self, reset: bool = False):
        """Checked build only: (violations, first address, its packet, its lane) of the
        latency form's bounds audit since the last reset; None on the product build."""
        out = (ctypes.c_ulonglong * 4)()
        rc = self._lib.wg_gpu_debug_xlane_check(out, 1 if reset else 0)
        if rc == -1:
            return None
        if rc != 0:
            raise NeptunGpuError(f"wg_gpu_debug_xlane_check failed (rc={rc})")
        return tuple(int(x) for x in out)

    def close(self) -> None:
        for dep in sorted(getattr(self, "_dependents", ()), key=lambda d: d._close_order):
            dep.close()
        if getattr(self, "_h", None):
            self._lib.wg_gpu_ctx_destroy(self._h)
            self._h = None

    def _attach(self, dep) -> None:
        self._dependents.add(dep)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_keys(self, first_slot: int, keys: np.ndarray, indices: np.ndarray, stream=None) -> None:
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, 32)
        indices = np.ascontiguousarray(indices, dtype=np.uint32).reshape(-1)
        if len(keys) != len(indices):
            raise ValueError("keys and indices differ in length")
        check(self._lib.wg_gpu_set_keys(self._h, first_slot, len(keys), keys.ctypes.data,
                                        indices.ctypes.data, _stream(stream)), "wg_gpu_set_keys")

    # --- descriptor batches (device tensors) --------------------------------
    def seal_batch(self, descs, n: int, src, dst, status, stream=None) -> None:
        check(self._lib.wg_gpu_seal_batch(self._h, _ptr(descs), n, _ptr(src), _ptr(dst),
                                          _ptr(status), _stream(stream)), "wg_gpu_seal_batch")

    def open_batch(self, descs, n: int, src, dst, status, stream=None) -> None:
        check(self._lib.wg_gpu_open_batch(self._h, _ptr(descs), n, _ptr(src), _ptr(dst),
                                          _ptr(status), _stream(stream)), "wg_gpu_open_batch")

    # --- mixed-length scheduling -------------------------------------------
    PLAN_SCRATCH_BYTES = 262144  # WG_PLAN_SCRATCH_BYTES

    def plan_batch(self, seal: bool, descs, n: int, order, scratch, stream=None) -> None:
        """Permutation grouping packets by length, longest first (device counting sort)."""
        check(self._lib.wg_gpu_plan_batch(self._h, 1 if seal else 0, _ptr(descs), n, _ptr(order),
                                          _ptr(scratch), _stream(stream)), "wg_gpu_plan_batch")

    def register_host(self, addr: int, nbytes: int) -> None:
        """Register caller host memory (address, size) for copy-free batches."""
        check(self._lib.wg_gpu_register_host(self._h, addr, nbytes), "wg_gpu_register_host")

    def unregister_host(self, addr: int) -> None:
        check(self._lib.wg_gpu_unregister_host(self._h, addr), "wg_gpu_unregister_host")

    def host_device_address(self, addr: int, nbytes: int) -> int:
        dev = ctypes.c_uint64()
        check(self._lib.wg_gpu_host_device_address(self._h, addr, nbytes, ctypes.byref(dev)),
              "wg_gpu_host_device_address")
        return dev.value

    def x25519_batch(self, n: int, scalars, points, out, stream=None) -> None:
        """out[i] = X25519(scalars[i], points[i]), 32-byte rows on the device."""
        check(self._lib.wg_gpu_x25519_batch(self._h, n, _ptr(scalars), _ptr(points), _ptr(out),
                                            _stream(stream)), "wg_gpu_x25519_batch")

    def handshake_anon_batch(self, static_private: bytes, n: int, msgs, stride: int, out,
                             check_mac1: bool = True, stream=None) -> None:
        """mac1 check + parse_handshake_anon for n initiations (device); out: HALF_HANDSHAKE_DTYPE."""
        check(self._lib.wg_gpu_handshake_anon_batch(self._h, bytes(static_private), n, _ptr(msgs),
                                                    stride, 1 if check_mac1 else 0, _ptr(out),
                                                    _stream(stream)),
              "wg_gpu_handshake_anon_batch")

    def handshake_consume_batch(self, static_private: bytes, n: int, msgs, stride: int, peers, out,
                                stream=None) -> None:
        """receive_handshake_initialization crypto (device): peers RESPONDER_PEER_DTYPE,
        out INIT_RECEIVED_DTYPE."""
        check(self._lib.wg_gpu_handshake_consume_batch(self._h, bytes(static_private), n, _ptr(msgs),
                                                       stride, _ptr(peers), _ptr(out), _stream(stream)),
              "wg_gpu_handshake_consume_batch")

    def timestamp_after(self, ts: bytes, last: bytes) -> bool:
        return bool(self._lib.wg_handshake_timestamp_after(bytes(ts), bytes(last)))

    def handshake_respond_batch(self, n: int, states, jobs, out, stream=None) -> None:
        """format_handshake_response + mac1/mac2 (device): jobs RESPONSE_JOB_DTYPE,
        out RESPONSE_OUT_DTYPE."""
        check(self._lib.wg_gpu_handshake_respond_batch(self._h, n, _ptr(states), _ptr(jobs), _ptr(out),
                                                       _stream(stream)),
              "wg_gpu_handshake_respond_batch")

    def mac2_check_batch(self, secret_key: bytes, counter: int, n: int, msgs, stride: int, lens,
                         addrs, cookies, status, stream=None) -> None:
        check(self._lib.wg_gpu_mac2_check_batch(self._h, bytes(secret_key), counter, n, _ptr(msgs),
                                                stride, _ptr(lens), _ptr(addrs), _ptr(cookies),
                                                _ptr(status), _stream(stream)),
              "wg_gpu_mac2_check_batch")

    def handshake_initiate_batch(self, n: int, jobs, out, stream=None) -> None:
        """format_handshake_initiation + mac1/mac2 (device): jobs INITIATION_JOB_DTYPE,
        out INIT_SENT_DTYPE."""
        check(self._lib.wg_gpu_handshake_initiate_batch(self._h, n, _ptr(jobs), _ptr(out), _stream(stream)),
              "wg_gpu_handshake_initiate_batch")

    def handshake_receive_response_batch(self, static_private: bytes, n: int, msgs, stride: int,
                                         jobs, out, check_mac1: bool = True, stream=None) -> None:
        """receive_handshake_response crypto (device): jobs RESPONSE_RECEIVED_JOB_DTYPE,
        out SESSION_KEYS_DTYPE."""
        check(self._lib.wg_gpu_handshake_receive_response_batch(
            self._h, bytes(static_private), n, _ptr(msgs), stride, 1 if check_mac1 else 0, _ptr(jobs),
            _ptr(out), _stream(stream)), "wg_gpu_handshake_receive_response_batch")

    def cookie_reply_open_batch(self, n: int, jobs, out, stream=None) -> None:
        """receive_cookie_reply's XChaCha20-Poly1305 open (device): jobs COOKIE_OPEN_JOB_DTYPE,
        out COOKIE_OPEN_OUT_DTYPE."""
        check(self._lib.wg_gpu_cookie_reply_open_batch(self._h, n, _ptr(jobs), _ptr(out), _stream(stream)),
              "wg_gpu_cookie_reply_open_batch")

    def cookie_reply_batch(self, cookie_key: bytes, nonce_key: bytes, n: int, jobs, out,
                           stream=None) -> None:
        check(self._lib.wg_gpu_cookie_reply_batch(self._h, bytes(cookie_key), bytes(nonce_key), n,
                                                  _ptr(jobs), _ptr(out), _stream(stream)),
              "wg_gpu_cookie_reply_batch")

    def route_set(self, receiver_idx, key_slot) -> None:
        """Replace the device receiver_idx -> key slot table (host arrays)."""
        r = np.ascontiguousarray(receiver_idx, np.uint32)
        k = np.ascontiguousarray(key_slot, np.uint32)
        if r.shape != k.shape:
            raise ValueError("receiver_idx and key_slot must have the same length")
        check(self._lib.wg_gpu_route_set(self._h, len(r), r.ctypes.data, k.ctypes.data),
              "wg_gpu_route_set")

    def route_batch(self, descs, n: int, src, stream=None) -> None:
        """Fill descs[i].key_slot from each datagram's receiver index (device)."""
        check(self._lib.wg_gpu_route_batch(self._h, _ptr(descs), n, _ptr(src), _stream(stream)),
              "wg_gpu_route_batch")

    def seal_batch_ordered(self, descs, order, n: int, src, dst, status, stream=None) -> None:
        check(self._lib.wg_gpu_seal_batch_ordered(self._h, _ptr(descs), _ptr(order), n, _ptr(src),
                                                  _ptr(dst), _ptr(status), _stream(stream)),
              "wg_gpu_seal_batch_ordered")

    def open_batch_ordered(self, descs, order, n: int, src, dst, status, stream=None) -> None:
        check(self._lib.wg_gpu_open_batch_ordered(self._h, _ptr(descs), _ptr(order), n, _ptr(src),
                                                  _ptr(dst), _ptr(status), _stream(stream)),
              "wg_gpu_open_batch_ordered")

    # --- uniform single-session batches -------------------------------------
    def set_slot_padding(self, writable: bool) -> None:
        """Declare the rest of every strided output slot scratch: outputs are then
        zero-filled to their 128-byte line end (whole-line writes)."""
        check(self._lib.wg_gpu_ctx_set_slot_padding(self._h, 1 if writable else 0),
              "wg_gpu_ctx_set_slot_padding")

    def set_xlane_lanes(self, lanes: int) -> None:
        """Latency form of the descriptor and strided batches: n * G <= lanes runs G
        (64..2, narrowed to the packets' keystream blocks) lanes per packet; 0 = off,
        < 0 = default."""
        check(self._lib.wg_gpu_ctx_set_xlane_lanes(self._h, int(lanes)), "wg_gpu_ctx_set_xlane_lanes")

    def set_split(self, parts: int) -> None:
        """Split waves of the strided batches (wg_gpu_ctx_set_split): < 0 the library's
        choice, 1 never, 2 .. 8 forced where every part keeps >= 8 keystream rounds."""
        check(self._lib.wg_gpu_ctx_set_split(self._h, int(parts)), "wg_gpu_ctx_set_split", self._lib)

    def split_parts(self, seal: bool, n: int, length: int) -> int:
        """Parts a throughput-form strided batch's waves would run in (1: unsplit),
        wg_gpu_strided_split_parts."""
        k = self._lib.wg_gpu_strided_split_parts(self._h, int(bool(seal)), int(n), int(length))
        if k < 1:
            check(k, "wg_gpu_strided_split_parts", self._lib)
        return int(k)

    def seal_strided(self, n: int, length: int, key_slot: int, counter_base: int, src,
                     src_stride: int, dst, dst_stride: int, status=None, stream=None) -> None:
        check(self._lib.wg_gpu_seal_strided(self._h, n, length, key_slot, counter_base, _ptr(src),
                                            src_stride, _ptr(dst), dst_stride, _ptr(status),
                                            _stream(stream)), "wg_gpu_seal_strided")

    def open_strided(self, n: int, length: int, key_slot: int, src, src_stride: int, dst,
                     dst_stride: int, status=None, stream=None) -> None:
        check(self._lib.wg_gpu_open_strided(self._h, n, length, key_slot, _ptr(src), src_stride,
                                            _ptr(dst), dst_stride, _ptr(status), _stream(stream)),
              "wg_gpu_open_strided")


class GpuPipe:
    """Host-resident batches: chunked H2D -> kernel -> D2H over `depth` streams.

    The end-to-end shape of NepTUN's data path (TUN/UDP buffers live in host
    memory); pass pinned host tensors for overlapped copies.
    """

    _close_order = 0  # (GpuContext.close: Tunns and pipes before engines)

    def __init__(self, ctx: GpuContext, chunk_bytes: int = 64 << 20, depth: int = 3):
        self._lib = ctx._lib
        self._ctx = ctx  # keep the context alive
        h = ctypes.c_void_p()
        check(self._lib.wg_gpu_pipe_create(ctx._h, chunk_bytes, depth, ctypes.byref(h)),
              "wg_gpu_pipe_create")
        self._h = h
        ctx._attach(self)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.wg_gpu_pipe_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def seal_strided(self, n, length, key_slot, counter_base, h_src, src_stride, h_dst,
                     dst_stride, h_status=None) -> None:
        check(self._lib.wg_gpu_pipe_seal_strided(self._h, n, length, key_slot, counter_base,
                                                 _ptr(h_src), src_stride, _ptr(h_dst), dst_stride,
                                                 _ptr(h_status)), "wg_gpu_pipe_seal_strided")

    def open_strided(self, n, length, key_slot, h_src, src_stride, h_dst, dst_stride,
                     h_status=None) -> None:
        check(self._lib.wg_gpu_pipe_open_strided(self._h, n, length, key_slot, _ptr(h_src),
                                                 src_stride, _ptr(h_dst), dst_stride,
                                                 _ptr(h_status)), "wg_gpu_pipe_open_strided")


__all__ = ["GpuPipe", "GpuContext", "NeptunGpuError", "DESC_DTYPE", "STATUS", "DATA_OFFSET", "AEAD_SIZE",
           "DATA_OVERHEAD_SZ"]
