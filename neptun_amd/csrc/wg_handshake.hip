// wg_handshake.hip -- batched handshake-side crypto.
//
//   x25519_kernel          one X25519 (RFC 7748) per lane: per-lane scalar and
//                          point -- the DH of Noise IK (x25519-dalek in the
//                          reference, neptun/src/lib.rs:21-24).
//   handshake_anon_kernel  one handshake initiation per lane: the mac1 check of
//                          RateLimiter::verify_packet (rate_limiter.rs:187-195)
//                          then parse_handshake_anon (handshake.rs:367-412) --
//                          the per-initiation work a device does before it knows
//                          the peer: HASH / HMAC chain, DH(static, ephemeral),
//                          AEAD-open of the initiator's static key.
// The responder's static private key and the two hashes derived from its public
// key are wave-uniform kernel arguments (precomputed on the host with the same
// header code).  Compute-bound integer work: no LDS, no MFMA; X25519 dominates
// (255 ladder steps of 5 mul + 4 sq in radix 2^25.5, then one inversion).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "neptun_gpu.h"
#include "wg_aead_kernels.h"
#include "wg_blake2s.h"
#include "wg_crypto.h"
#include "wg_x25519.h"

namespace wg {

__global__ __launch_bounds__(256) void x25519_kernel(uint32_t n, const uint8_t *scalars,
                                                     const uint8_t *points, uint8_t *out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8], u[8], r[8];
  const uint4 *ks = reinterpret_cast<const uint4 *>(scalars + 32ull * i);
  const uint4 *us = reinterpret_cast<const uint4 *>(points + 32ull * i);
  const uint4 k0 = ks[0], k1 = ks[1], u0 = us[0], u1 = us[1];
  k[0] = k0.x; k[1] = k0.y; k[2] = k0.z; k[3] = k0.w; k[4] = k1.x; k[5] = k1.y; k[6] = k1.z; k[7] = k1.w;
  u[0] = u0.x; u[1] = u0.y; u[2] = u0.z; u[3] = u0.w; u[4] = u1.x; u[5] = u1.y; u[6] = u1.z; u[7] = u1.w;
  x25519::scalarmult(r, k, u);
  uint4 *o = reinterpret_cast<uint4 *>(out + 32ull * i);
  o[0] = make_uint4(r[0], r[1], r[2], r[3]);
  o[1] = make_uint4(r[4], r[5], r[6], r[7]);
}

// INITIAL_CHAIN_KEY = HASH("Noise_IKpsk2_25519_ChaChaPoly_BLAKE2s") (handshake.rs:29-33)
__constant__ uint32_t kChainKey0[8] = {0xae6de260u, 0xc0ef27f3u, 0xe235c32eu, 0xd0d225a0u,
                                       0x0642eb16u, 0xf57772f8u, 0x98d1382du, 0x36cd788bu};

__global__ __launch_bounds__(256) void handshake_anon_kernel(HandshakeAnonParams prm) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= prm.n) return;
  const uint32_t *msg = reinterpret_cast<const uint32_t *>(prm.msgs + prm.stride * i);
  uint32_t w[37];
#pragma unroll
  for (int j = 0; j < 37; ++j) w[j] = msg[j];
  int32_t status = WG_STATUS_OK;
  if (w[0] != 1u) status = WG_STATUS_WRONG_PACKET_TYPE;  // HANDSHAKE_INIT (noise/mod.rs:150)
  if (status == WG_STATUS_OK && prm.check_mac1) {
    uint32_t mac[4];
    b2s::mac16_116(mac, prm.mac1_key, w);
    if ((mac[0] ^ w[29]) | (mac[1] ^ w[30]) | (mac[2] ^ w[31]) | (mac[3] ^ w[32]))
      status = WG_STATUS_INVALID_MAC;
  }
  uint32_t eph[8], h[8], t[8], ck[8], dh[8], key[8], d[16];
#pragma unroll
  for (int j = 0; j < 8; ++j) eph[j] = w[2 + j];
  // hash = HASH(HASH(INITIAL_CHAIN_HASH || static_public) || ephemeral)
  b2s::hash64(h, prm.hash0, eph);
  // chaining_key = HMAC(HMAC(INITIAL_CHAIN_KEY, ephemeral), 0x1)
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j < 8 ? eph[j] : 0u;
  uint32_t ck0[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ck0[j] = kChainKey0[j];
  b2s::hmac(t, ck0, d, 32);
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j == 0 ? 1u : 0u;
  b2s::hmac(ck, t, d, 1);
  // temp = HMAC(chaining_key, DH(static_private, ephemeral))
  x25519::scalarmult(dh, prm.static_private, eph);
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j < 8 ? dh[j] : 0u;
  b2s::hmac(t, ck, d, 32);
  // chaining_key = HMAC(temp, 0x1); key = HMAC(temp, chaining_key || 0x2)
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j == 0 ? 1u : 0u;
  b2s::hmac(ck, t, d, 1);
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j < 8 ? ck[j] : (j == 8 ? 2u : 0u);
  b2s::hmac(key, t, d, 33);
  // encrypted_static = AEAD(key, 0, static_public, hash): open (RFC 8439, AAD = hash)
  uint32_t ks[16];
  chacha20_block(ks, key, 0u, 0u, 0u);
  Poly poly;
  poly_init(poly, ks);
  const uint32_t s[4] = {ks[4], ks[5], ks[6], ks[7]};
  poly_block(poly, h[0], h[1], h[2], h[3]);  // AAD (32 bytes, no padding needed)
  poly_block(poly, h[4], h[5], h[6], h[7]);
  poly_block(poly, w[10], w[11], w[12], w[13]);  // ciphertext
  poly_block(poly, w[14], w[15], w[16], w[17]);
  poly_block(poly, 32u, 0u, 32u, 0u);  // LE64(aad_len) || LE64(ct_len)
  uint32_t tag[4];
  poly_finish(poly, s, tag);
  chacha20_block(ks, key, 1u, 0u, 0u);
  uint32_t pk[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) pk[j] = w[10 + j] ^ ks[j];
  if (status == WG_STATUS_OK &&
      ((tag[0] ^ w[18]) | (tag[1] ^ w[19]) | (tag[2] ^ w[20]) | (tag[3] ^ w[21])))
    status = WG_STATUS_INVALID_AEAD_TAG;
  wg_half_handshake r;
  r.peer_index = status == WG_STATUS_OK || status == WG_STATUS_INVALID_AEAD_TAG ? w[1] : 0u;
  r.status = status;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t v = status == WG_STATUS_OK ? pk[j] : 0u;
    r.peer_static_public[4 * j + 0] = (uint8_t)v;
    r.peer_static_public[4 * j + 1] = (uint8_t)(v >> 8);
    r.peer_static_public[4 * j + 2] = (uint8_t)(v >> 16);
    r.peer_static_public[4 * j + 3] = (uint8_t)(v >> 24);
  }
  prm.out[i] = r;
}

}  // namespace wg
