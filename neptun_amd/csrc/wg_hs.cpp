// wg_hs.cpp -- C ABI of the batched handshake kernels (include/neptun_gpu.h).
// The wave-uniform inputs of handshake_anon_kernel are derived here on the
// host with the same header code the kernel uses.
#include <hip/hip_runtime.h>

#include <cstring>

#include "neptun_gpu.h"
#include "wg_aead_kernels.h"
#include "wg_blake2s.h"
#include "wg_x25519.h"

int wg_pipe_fail(int rc, const char *what, hipError_t e);  // wg_gpu.cpp
int wg_ctx_device(const wg_gpu_ctx *ctx);                   // wg_gpu.cpp

namespace {
struct DevGuard {
  int prev = -1;
  explicit DevGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// INITIAL_CHAIN_HASH = HASH(HASH(CONSTRUCTION) || IDENTIFIER) (handshake.rs:29-39)
void initial_chain_hash(uint32_t out[8]) {
  static const char kConstruction[] = "Noise_IKpsk2_25519_ChaChaPoly_BLAKE2s";  // 37 bytes
  static const char kIdentifier[] = "WireGuard v1 zx2c4 Jason@zx2c4.com";       // 34 bytes
  uint32_t m[16] = {0}, ck[8];
  std::memcpy(m, kConstruction, 37);
  wg::b2s::hash_block(ck, m, 37);
  // 66 bytes: ck || IDENTIFIER[0..32) as one block, IDENTIFIER[32..34) as the last
  std::memcpy(m, ck, 32);
  std::memcpy(reinterpret_cast<uint8_t *>(m) + 32, kIdentifier, 32);
  wg::b2s::init(out, 32, 0);
  wg::b2s::compress(out, m, 64, false);
  std::memset(m, 0, sizeof m);
  std::memcpy(m, kIdentifier + 32, 2);
  wg::b2s::compress(out, m, 66, true);
}
}  // namespace

extern "C" {

int wg_gpu_x25519_batch(wg_gpu_ctx *ctx, uint32_t n, const uint8_t *scalars, const uint8_t *points,
                        uint8_t *out, void *stream) {
  if (!ctx || (n && (!scalars || !points || !out)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "x25519_batch: null argument", hipSuccess);
  if (((uintptr_t)scalars | (uintptr_t)points | (uintptr_t)out) & 15u)
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "x25519_batch: pointers must be 16-byte aligned",
                        hipSuccess);
  if (n == 0) return WG_RC_OK;
  DevGuard g(wg_ctx_device(ctx));
  hipLaunchKernelGGL(wg::x25519_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), n, scalars, points, out);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WG_RC_OK : wg_pipe_fail(WG_RC_HIP_ERROR, "x25519_batch: launch", e);
}

int wg_gpu_handshake_anon_batch(wg_gpu_ctx *ctx, const uint8_t static_private[32], uint32_t n,
                                const uint8_t *msgs, uint64_t stride, int check_mac1,
                                wg_half_handshake *out, void *stream) {
  if (!ctx || !static_private || (n && (!msgs || !out)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "handshake_anon_batch: null argument", hipSuccess);
  if (stride < 148 || (stride & 3u) || ((uintptr_t)msgs & 3u))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT,
                        "handshake_anon_batch: stride >= 148 and 4-byte alignment required", hipSuccess);
  if (n == 0) return WG_RC_OK;
  wg::HandshakeAnonParams prm{};
  prm.msgs = msgs;
  prm.stride = stride;
  prm.out = out;
  prm.n = n;
  prm.check_mac1 = check_mac1 ? 1u : 0u;
  std::memcpy(prm.static_private, static_private, 32);
  // static_public = X25519(static_private, 9); hash0 = HASH(INITIAL_CHAIN_HASH || static_public);
  // mac1_key = HASH(LABEL_MAC1 || static_public) (rate_limiter.rs:67)
  uint32_t base[8] = {9, 0, 0, 0, 0, 0, 0, 0}, pub[8], ich[8];
  wg::x25519::scalarmult(pub, prm.static_private, base);
  initial_chain_hash(ich);
  wg::b2s::hash64(prm.hash0, ich, pub);
  uint32_t m[16] = {0};
  std::memcpy(m, "mac1----", 8);
  std::memcpy(reinterpret_cast<uint8_t *>(m) + 8, pub, 32);
  wg::b2s::hash_block(prm.mac1_key, m, 40);
  DevGuard g(wg_ctx_device(ctx));
  hipLaunchKernelGGL(wg::handshake_anon_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), prm);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WG_RC_OK
                         : wg_pipe_fail(WG_RC_HIP_ERROR, "handshake_anon_batch: launch", e);
}

int wg_gpu_handshake_consume_batch(wg_gpu_ctx *ctx, const uint8_t static_private[32], uint32_t n,
                                   const uint8_t *msgs, uint64_t stride,
                                   const wg_responder_peer *peers, wg_init_received *out,
                                   void *stream) {
  if (!ctx || !static_private || (n && (!msgs || !peers || !out)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "handshake_consume_batch: null argument", hipSuccess);
  if (stride < 148 || (stride & 3u) || (((uintptr_t)msgs | (uintptr_t)peers | (uintptr_t)out) & 3u))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT,
                        "handshake_consume_batch: stride >= 148 and 4-byte alignment required",
                        hipSuccess);
  if (n == 0) return WG_RC_OK;
  wg::HandshakeConsumeParams prm{};
  prm.msgs = msgs;
  prm.stride = stride;
  prm.peers = peers;
  prm.out = out;
  prm.n = n;
  std::memcpy(prm.static_private, static_private, 32);
  uint32_t base[8] = {9, 0, 0, 0, 0, 0, 0, 0}, pub[8], ich[8];
  wg::x25519::scalarmult(pub, prm.static_private, base);
  initial_chain_hash(ich);
  wg::b2s::hash64(prm.hash0, ich, pub);
  DevGuard g(wg_ctx_device(ctx));
  hipLaunchKernelGGL(wg::handshake_consume_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), prm);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WG_RC_OK
                         : wg_pipe_fail(WG_RC_HIP_ERROR, "handshake_consume_batch: launch", e);
}

int wg_handshake_timestamp_after(const uint8_t ts[12], const uint8_t last[12]) {
  return std::memcmp(ts, last, 12) > 0 ? 1 : 0;  // big-endian (secs, nanos): bytewise order
}

int wg_gpu_handshake_respond_batch(wg_gpu_ctx *ctx, uint32_t n, const wg_init_received *states,
                                   const wg_response_job *jobs, wg_response_out *out, void *stream) {
  if (!ctx || (n && (!states || !jobs || !out)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "handshake_respond_batch: null argument", hipSuccess);
  if (((uintptr_t)states | (uintptr_t)jobs | (uintptr_t)out) & 7u)
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "handshake_respond_batch: 8-byte alignment required",
                        hipSuccess);
  if (n == 0) return WG_RC_OK;
  wg::HandshakeRespondParams prm{states, jobs, out, n};
  DevGuard g(wg_ctx_device(ctx));
  hipLaunchKernelGGL(wg::handshake_respond_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), prm);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WG_RC_OK
                         : wg_pipe_fail(WG_RC_HIP_ERROR, "handshake_respond_batch: launch", e);
}

int wg_gpu_mac2_check_batch(wg_gpu_ctx *ctx, const uint8_t secret_key[16], uint64_t cookie_counter,
                            uint32_t n, const uint8_t *msgs, uint64_t stride, const uint32_t *lens,
                            const uint8_t *addrs, uint8_t *cookies, int32_t *status, void *stream) {
  if (!ctx || !secret_key || (n && (!msgs || !lens || !addrs || !cookies || !status)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "mac2_check_batch: null argument", hipSuccess);
  if (stride < 148 || (stride & 3u) ||
      (((uintptr_t)msgs | (uintptr_t)addrs | (uintptr_t)cookies) & 3u))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT,
                        "mac2_check_batch: stride >= 148 and 4-byte alignment required", hipSuccess);
  if (n == 0) return WG_RC_OK;
  wg::Mac2CheckParams prm{};
  prm.msgs = msgs;
  prm.stride = stride;
  prm.lens = lens;
  prm.addrs = addrs;
  prm.cookies = cookies;
  prm.status = status;
  prm.counter = cookie_counter;
  prm.n = n;
  std::memcpy(prm.secret, secret_key, 16);
  DevGuard g(wg_ctx_device(ctx));
  hipLaunchKernelGGL(wg::mac2_check_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), prm);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WG_RC_OK : wg_pipe_fail(WG_RC_HIP_ERROR, "mac2_check_batch: launch", e);
}

int wg_gpu_cookie_reply_batch(wg_gpu_ctx *ctx, const uint8_t cookie_key[32],
                              const uint8_t nonce_key[32], uint32_t n,
                              const wg_cookie_reply_job *jobs, uint8_t *out, void *stream) {
  if (!ctx || !cookie_key || !nonce_key || (n && (!jobs || !out)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "cookie_reply_batch: null argument", hipSuccess);
  if (((uintptr_t)jobs | (uintptr_t)out) & 7u)
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "cookie_reply_batch: 8-byte alignment required",
                        hipSuccess);
  if (n == 0) return WG_RC_OK;
  wg::CookieReplyParams prm{};
  prm.jobs = jobs;
  prm.out = out;
  prm.n = n;
  std::memcpy(prm.cookie_key, cookie_key, 32);
  std::memcpy(prm.nonce_key, nonce_key, 32);
  DevGuard g(wg_ctx_device(ctx));
  hipLaunchKernelGGL(wg::cookie_reply_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), prm);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WG_RC_OK : wg_pipe_fail(WG_RC_HIP_ERROR, "cookie_reply_batch: launch", e);
}

int wg_gpu_handshake_initiate_batch(wg_gpu_ctx *ctx, uint32_t n, const wg_initiation_job *jobs,
                                    wg_init_sent *out, void *stream) {
  if (!ctx || (n && (!jobs || !out)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "handshake_initiate_batch: null argument", hipSuccess);
  if (((uintptr_t)jobs | (uintptr_t)out) & 7u)
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "handshake_initiate_batch: 8-byte alignment required",
                        hipSuccess);
  if (n == 0) return WG_RC_OK;
  wg::HandshakeInitiateParams prm{jobs, out, n};
  DevGuard g(wg_ctx_device(ctx));
  hipLaunchKernelGGL(wg::handshake_initiate_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), prm);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WG_RC_OK
                         : wg_pipe_fail(WG_RC_HIP_ERROR, "handshake_initiate_batch: launch", e);
}

int wg_gpu_handshake_receive_response_batch(wg_gpu_ctx *ctx, const uint8_t static_private[32],
                                            uint32_t n, const uint8_t *msgs, uint64_t stride,
                                            int check_mac1, const wg_response_received_job *jobs,
                                            wg_session_keys *out, void *stream) {
  if (!ctx || !static_private || (n && (!msgs || !jobs || !out)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "handshake_receive_response_batch: null argument",
                        hipSuccess);
  if (stride < 92 || (stride & 3u) || (((uintptr_t)msgs | (uintptr_t)jobs | (uintptr_t)out) & 3u))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT,
                        "handshake_receive_response_batch: stride >= 92 and 4-byte alignment required",
                        hipSuccess);
  if (n == 0) return WG_RC_OK;
  wg::HandshakeResponseParams prm{};
  prm.msgs = msgs;
  prm.stride = stride;
  prm.jobs = jobs;
  prm.out = out;
  prm.n = n;
  prm.check_mac1 = check_mac1 ? 1u : 0u;
  std::memcpy(prm.static_private, static_private, 32);
  // mac1_key = HASH(LABEL_MAC1 || static_public) (rate_limiter.rs:67), static_public = X25519(k, 9)
  uint32_t base[8] = {9, 0, 0, 0, 0, 0, 0, 0}, pub[8];
  wg::x25519::scalarmult(pub, prm.static_private, base);
  uint32_t m[16] = {0};
  std::memcpy(m, "mac1----", 8);
  std::memcpy(reinterpret_cast<uint8_t *>(m) + 8, pub, 32);
  wg::b2s::hash_block(prm.mac1_key, m, 40);
  DevGuard g(wg_ctx_device(ctx));
  hipLaunchKernelGGL(wg::handshake_response_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), prm);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WG_RC_OK
                         : wg_pipe_fail(WG_RC_HIP_ERROR, "handshake_receive_response_batch: launch", e);
}

int wg_gpu_cookie_reply_open_batch(wg_gpu_ctx *ctx, uint32_t n, const wg_cookie_open_job *jobs,
                                   wg_cookie_open_out *out, void *stream) {
  if (!ctx || (n && (!jobs || !out)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "cookie_reply_open_batch: null argument", hipSuccess);
  if (((uintptr_t)jobs | (uintptr_t)out) & 7u)
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "cookie_reply_open_batch: 8-byte alignment required",
                        hipSuccess);
  if (n == 0) return WG_RC_OK;
  wg::CookieOpenParams prm{jobs, out, n};
  DevGuard g(wg_ctx_device(ctx));
  hipLaunchKernelGGL(wg::cookie_open_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), prm);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WG_RC_OK : wg_pipe_fail(WG_RC_HIP_ERROR, "cookie_reply_open_batch: launch", e);
}

}  // extern "C"
