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

// ---------------------------------------------------------------------------
// Responder side: receive_handshake_initialization split where
// the reference's sequential state sits between its halves -- the device does
// the crypto, the host keeps the TAI64N replay comparison and inc_index().
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ld_words(uint32_t *w, const uint8_t *p, int n) {
  const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
  for (int j = 0; j < n; ++j) w[j] = q[j];
}
__device__ __forceinline__ void st_words(uint8_t *p, const uint32_t *w, int n) {
  uint32_t *q = reinterpret_cast<uint32_t *>(p);
  for (int j = 0; j < n; ++j) q[j] = w[j];
}
__device__ __forceinline__ void hmac_1(uint32_t out[8], const uint32_t key[8], uint32_t byte) {
  uint32_t d[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j == 0 ? byte : 0u;
  b2s::hmac(out, key, d, 1);
}
__device__ __forceinline__ void hmac_32(uint32_t out[8], const uint32_t key[8], const uint32_t a[8]) {
  uint32_t d[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j < 8 ? a[j] : 0u;
  b2s::hmac(out, key, d, 32);
}
// b2s_hmac2(key, a(32 bytes), [byte]) (handshake.rs:58-72)
__device__ __forceinline__ void hmac_33(uint32_t out[8], const uint32_t key[8], const uint32_t a[8],
                                        uint32_t byte) {
  uint32_t d[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j < 8 ? a[j] : (j == 8 ? byte : 0u);
  b2s::hmac(out, key, d, 33);
}
// RFC 8439 AEAD tag over a 32-byte AAD and `ct_len` <= 32 bytes of ciphertext
// (zero-padded words), key block 0 of (key, nonce 0): aead_chacha20_seal/open
// of handshake.rs:101-193 for the handshake's short messages.
__device__ __forceinline__ void tag_aad32(uint32_t tag[4], const uint32_t key[8], const uint32_t aad[8],
                                          const uint32_t ct[8], uint32_t ct_len) {
  uint32_t ks[16];
  chacha20_block(ks, key, 0u, 0u, 0u);
  Poly poly;
  poly_init(poly, ks);
  const uint32_t s[4] = {ks[4], ks[5], ks[6], ks[7]};
  poly_block(poly, aad[0], aad[1], aad[2], aad[3]);
  poly_block(poly, aad[4], aad[5], aad[6], aad[7]);
  if (ct_len > 0) poly_block(poly, ct[0], ct[1], ct[2], ct[3]);  // (pad16 zero-fills)
  if (ct_len > 16) poly_block(poly, ct[4], ct[5], ct[6], ct[7]);
  poly_block(poly, 32u, 0u, ct_len, 0u);
  poly_finish(poly, s, tag);
}

__global__ __launch_bounds__(256) void handshake_consume_kernel(HandshakeConsumeParams prm) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= prm.n) return;
  uint32_t w[37];
  ld_words(w, prm.msgs + prm.stride * i, 37);
  const wg_responder_peer &peer = prm.peers[i];
  uint32_t eph[8], h[8], t[8], ck[8], dh[8], key[8], d[16], tag[4], ks[16];
#pragma unroll
  for (int j = 0; j < 8; ++j) eph[j] = w[2 + j];
  // hash = HASH(HASH(INITIAL_CHAIN_HASH || static_public) || ephemeral)
  b2s::hash64(h, prm.hash0, eph);
  // chaining_key = HMAC(HMAC(INITIAL_CHAIN_KEY, ephemeral), 0x1)
  uint32_t ck0[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ck0[j] = kChainKey0[j];
  hmac_32(t, ck0, eph);
  hmac_1(ck, t, 1u);
  // temp = HMAC(ck, DH(static_private, ephemeral)); ck = HMAC(temp, 1); key = HMAC(temp, ck || 2)
  x25519::scalarmult(dh, prm.static_private, eph);
  hmac_32(t, ck, dh);
  hmac_1(ck, t, 1u);
  hmac_33(key, t, ck, 2u);
  // open encrypted_static (AAD = hash), compare with the configured peer (handshake.rs:562-577)
  int32_t status = w[0] == 1u ? WG_STATUS_OK : WG_STATUS_WRONG_PACKET_TYPE;
  uint32_t ct[8], pk[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ct[j] = w[10 + j];
  tag_aad32(tag, key, h, ct, 32);
  if (status == WG_STATUS_OK && ((tag[0] ^ w[18]) | (tag[1] ^ w[19]) | (tag[2] ^ w[20]) | (tag[3] ^ w[21])))
    status = WG_STATUS_INVALID_AEAD_TAG;
  chacha20_block(ks, key, 1u, 0u, 0u);
  uint32_t want[8], diff = 0;
  ld_words(reinterpret_cast<uint32_t *>(want), peer.peer_static_public, 8);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    pk[j] = ct[j] ^ ks[j];
    diff |= pk[j] ^ want[j];
  }
  if (status == WG_STATUS_OK && diff) status = WG_STATUS_WRONG_KEY;
  // hash = HASH(hash || encrypted_static (48 bytes))
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j < 12 ? w[10 + j] : 0u;
  uint32_t h2[8];
  b2s::hash_cat(h2, h, d, 48);
  // temp = HMAC(ck, static_shared); ck = HMAC(temp, 1); key = HMAC(temp, ck || 2)
  uint32_t ss[8];
  ld_words(ss, peer.static_shared, 8);
  hmac_32(t, ck, ss);
  hmac_1(ck, t, 1u);
  hmac_33(key, t, ck, 2u);
  // open encrypted_timestamp (12 + 16 bytes, AAD = hash)
#pragma unroll
  for (int j = 0; j < 8; ++j) ct[j] = j < 3 ? w[22 + j] : 0u;
  tag_aad32(tag, key, h2, ct, 12);
  if (status == WG_STATUS_OK && ((tag[0] ^ w[25]) | (tag[1] ^ w[26]) | (tag[2] ^ w[27]) | (tag[3] ^ w[28])))
    status = WG_STATUS_INVALID_AEAD_TAG;
  chacha20_block(ks, key, 1u, 0u, 0u);
  uint32_t ts[3] = {w[22] ^ ks[0], w[23] ^ ks[1], w[24] ^ ks[2]};
  // hash = HASH(hash || encrypted_timestamp (28 bytes))
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j < 7 ? w[22 + j] : 0u;
  b2s::hash_cat(h, h2, d, 28);
  wg_init_received &o = prm.out[i];
  const bool ok = status == WG_STATUS_OK;
  o.status = status;
  o.peer_index = status == WG_STATUS_WRONG_PACKET_TYPE ? 0u : w[1];
  uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  st_words(o.timestamp, ok ? ts : z, 3);
  st_words(o.chaining_key, ok ? ck : z, 8);
  st_words(o.hash, ok ? h : z, 8);
  st_words(o.peer_ephemeral, ok ? eph : z, 8);
}

__constant__ uint32_t kBasePoint[8] = {9u, 0, 0, 0, 0, 0, 0, 0};

__global__ __launch_bounds__(256) void handshake_respond_kernel(HandshakeRespondParams prm) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= prm.n) return;
  const wg_init_received &st = prm.states[i];
  const wg_response_job &job = prm.jobs[i];
  wg_response_out &o = prm.out[i];
  if (st.status != WG_STATUS_OK) {
    uint32_t z[23] = {0};
    st_words(o.message, z, 23);
    return;
  }
  uint32_t ck[8], h[8], peph[8], e[8], epub[8], t[8], dh[8], d[16];
  ld_words(ck, st.chaining_key, 8);
  ld_words(h, st.hash, 8);
  ld_words(peph, st.peer_ephemeral, 8);
  ld_words(e, job.ephemeral_private, 8);
  uint32_t base[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) base[j] = kBasePoint[j];
  x25519::scalarmult(epub, e, base);  // DH_PUBKEY(responder.ephemeral_private)
  // hash = HASH(hash || eph_pub); temp = HMAC(ck, eph_pub); ck = HMAC(temp, 1)
  b2s::hash64(d, h, epub);
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = d[j];
  hmac_32(t, ck, epub);
  hmac_1(ck, t, 1u);
  // DH(eph, initiator ephemeral), then DH(eph, initiator static)
  x25519::scalarmult(dh, e, peph);
  hmac_32(t, ck, dh);
  hmac_1(ck, t, 1u);
  uint32_t pst[8];
  ld_words(pst, job.peer_static_public, 8);
  x25519::scalarmult(dh, e, pst);
  hmac_32(t, ck, dh);
  hmac_1(ck, t, 1u);
  // psk (zeros when none, handshake.rs:920)
  uint32_t psk[8], temp[8], temp2[8], key[8];
  ld_words(psk, job.preshared_key, 8);
  hmac_32(temp, ck, psk);
  hmac_1(ck, temp, 1u);
  hmac_33(temp2, temp, ck, 2u);
  hmac_33(key, temp, temp2, 3u);
  b2s::hash64(d, h, temp2);
  // encrypted_nothing = AEAD(key, 0, [], hash)
  uint32_t tag[4], none[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  tag_aad32(tag, key, d, none, 0);
  // message: type 2 | sender (ours) | receiver (theirs) | eph_pub | tag | mac1 | mac2
  uint32_t m[23];
  m[0] = 2u;  // HANDSHAKE_RESP
  m[1] = job.local_index;
  m[2] = st.peer_index;
#pragma unroll
  for (int j = 0; j < 8; ++j) m[3 + j] = epub[j];
#pragma unroll
  for (int j = 0; j < 4; ++j) m[11 + j] = tag[j];
  uint32_t mk[8], mac1[4], mac2[4] = {0, 0, 0, 0};
  ld_words(mk, job.mac1_key, 8);
  b2s::keyed_mac(mac1, 16, mk, 32, m, 60);
#pragma unroll
  for (int j = 0; j < 4; ++j) m[15 + j] = mac1[j];
  if (job.has_cookie) {
    uint32_t ckey[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    ld_words(ckey, job.cookie, 4);
    uint32_t mm[20];
#pragma unroll
    for (int j = 0; j < 20; ++j) mm[j] = j < 19 ? m[j] : 0u;
    b2s::keyed_mac(mac2, 16, ckey, 16, mm, 76);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) m[19 + j] = mac2[j];
  st_words(o.message, m, 23);
  // session keys: temp1 = HMAC(ck, []), temp2 = HMAC(temp1, 1), temp3 = HMAC(temp1, temp2 || 2)
  uint32_t t1[8], t2[8], t3[8], empty[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) empty[j] = 0u;
  b2s::hmac(t1, ck, empty, 0);
  hmac_1(t2, t1, 1u);
  hmac_33(t3, t1, t2, 2u);
  st_words(o.receiving_key, t2, 8);  // Session::new(local, peer, temp2, temp3) (handshake.rs:948)
  st_words(o.sending_key, t3, 8);
  st_words(o.mac1, mac1, 4);
}

// Under load (rate_limiter.rs:197-218): cookie = MAC(secret, LE64(counter) || addr)
// and the mac2 check over msg[..len - 16]; status 0 = valid mac2, 1 = reply with a cookie.
__global__ __launch_bounds__(256) void mac2_check_kernel(Mac2CheckParams prm) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= prm.n) return;
  const uint32_t len = prm.lens[i];
  // only what parse_incoming_packet hands to verify_packet reaches the check:
  // a 148-byte initiation or a 92-byte response (noise/mod.rs:139-199); any
  // other length is rejected there, and here, before anything is read
  // (the host guarantees stride >= 148, so both lengths fit their slot)
  if (len != 148u && len != 92u) {
    prm.status[i] = WG_STATUS_INVALID_PACKET;
    const uint32_t z[4] = {0u, 0u, 0u, 0u};
    st_words(prm.cookies + 16ull * i, z, 4);
    return;
  }
  uint32_t w[37];
  const uint32_t *q = reinterpret_cast<const uint32_t *>(prm.msgs + prm.stride * i);
#pragma unroll
  for (int j = 0; j < 37; ++j) w[j] = 4u * j < len ? q[j] : 0u;
  uint32_t cin[16] = {0}, cookie[4], key[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  cin[0] = (uint32_t)prm.counter;
  cin[1] = (uint32_t)(prm.counter >> 32);
  ld_words(cin + 2, prm.addrs + 16ull * i, 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) key[j] = prm.secret[j];
  b2s::keyed_mac(cookie, 16, key, 16, cin, 24);
  uint32_t ck8[8] = {cookie[0], cookie[1], cookie[2], cookie[3], 0, 0, 0, 0}, mac2[4];
  // msg[..len - 16] = message + mac1; zero the words past it (len - 16 is a multiple of 4)
  const uint32_t mlen = len - 16u;
#pragma unroll
  for (int j = 0; j < 37; ++j) w[j] = 4u * j < mlen ? w[j] : 0u;
  b2s::keyed_mac(mac2, 16, ck8, 16, w, mlen);
  const uint32_t k = mlen / 4u;
  uint32_t diff = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) diff |= mac2[j] ^ q[k + j];
  prm.status[i] = diff ? 1 : 0;
  st_words(prm.cookies + 16ull * i, cookie, 4);
}

// format_cookie_reply (rate_limiter.rs:133-170): nonce = b2s_mac_24(nonce_key,
// LE64(ctr)); XChaCha20-Poly1305(cookie_key, nonce, aad = mac1, cookie).
__global__ __launch_bounds__(256) void cookie_reply_kernel(CookieReplyParams prm) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= prm.n) return;
  const wg_cookie_reply_job &job = prm.jobs[i];
  uint32_t nk[8], nin[16] = {0}, nonce[6];
#pragma unroll
  for (int j = 0; j < 8; ++j) nk[j] = prm.nonce_key[j];
  nin[0] = (uint32_t)job.nonce_ctr;
  nin[1] = (uint32_t)(job.nonce_ctr >> 32);
  b2s::keyed_mac(nonce, 24, nk, 32, nin, 8);
  uint32_t ckey[8], sub[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ckey[j] = prm.cookie_key[j];
  hchacha20(sub, ckey, nonce);
  // RFC 8439 with nonce 0^4 || nonce[16..24): block 0 -> Poly key, block 1 -> keystream
  uint32_t ks[16];
  chacha20_block(ks, sub, 0u, nonce[4], nonce[5]);
  Poly poly;
  poly_init(poly, ks);
  const uint32_t s[4] = {ks[4], ks[5], ks[6], ks[7]};
  uint32_t mac1[4], cookie[4], ct[4];
  ld_words(mac1, job.mac1, 4);
  ld_words(cookie, job.cookie, 4);
  chacha20_block(ks, sub, 1u, nonce[4], nonce[5]);
#pragma unroll
  for (int j = 0; j < 4; ++j) ct[j] = cookie[j] ^ ks[j];
  poly_block(poly, mac1[0], mac1[1], mac1[2], mac1[3]);  // AAD (16 bytes)
  poly_block(poly, ct[0], ct[1], ct[2], ct[3]);
  poly_block(poly, 16u, 0u, 16u, 0u);
  uint32_t tag[4];
  poly_finish(poly, s, tag);
  uint32_t m[16];
  m[0] = 3u;  // COOKIE_REPLY
  m[1] = job.receiver_idx;
#pragma unroll
  for (int j = 0; j < 6; ++j) m[2 + j] = nonce[j];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[8 + j] = ct[j];
    m[12 + j] = tag[j];
  }
  st_words(prm.out + 64ull * i, m, 16);
}

// ---------------------------------------------------------------------------
// Initiator side: format_handshake_initiation (handshake.rs:769-851)
// + append_mac1_and_mac2 (:732-765), receive_handshake_response (:615-695) and
// receive_cookie_reply (:697-727).  The per-peer sequential state (inc_index,
// the InitSent / previous state match by receiver index, cookies.index /
// last_mac1) stays with the caller; the device does the crypto.
// ---------------------------------------------------------------------------
// INITIAL_CHAIN_HASH = HASH(INITIAL_CHAIN_KEY || IDENTIFIER) (handshake.rs:34-39)
__constant__ uint32_t kChainHash0[8] = {0x61b31122u, 0x66c51a08u, 0xdb431269u, 0x32d58a45u,
                                        0x666c9c2du, 0xb7e89322u, 0x659ce10eu, 0xf39e07bau};

// aead_chacha20_seal (handshake.rs:101-117) of <= 32 plaintext bytes under a
// 32-byte AAD with nonce 0: ct = pt ^ keystream block 1, tag over AAD || ct
__device__ __forceinline__ void seal_aad32(uint32_t ct[8], uint32_t tag[4], const uint32_t key[8],
                                           const uint32_t aad[8], const uint32_t pt[8], uint32_t len) {
  uint32_t ks[16];
  chacha20_block(ks, key, 1u, 0u, 0u);
#pragma unroll
  for (int j = 0; j < 8; ++j) ct[j] = 4u * j < len ? pt[j] ^ ks[j] : 0u;
  tag_aad32(tag, key, aad, ct, len);
}

__global__ __launch_bounds__(256) void handshake_initiate_kernel(HandshakeInitiateParams prm) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= prm.n) return;
  const wg_initiation_job &job = prm.jobs[i];
  uint32_t e[8], epub[8], pst[8], h[8], t[8], ck[8], dh[8], key[8], d[16];
  ld_words(e, job.ephemeral_private, 8);
  ld_words(pst, job.peer_static_public, 8);
  uint32_t base[8], c0[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    base[j] = kBasePoint[j];
    c0[j] = kChainHash0[j];
  }
  // hash = HASH(INITIAL_CHAIN_HASH || responder.static_public)
  b2s::hash64(h, c0, pst);
  // msg.unencrypted_ephemeral = DH_PUBKEY(ephemeral_private); hash = HASH(hash || it)
  x25519::scalarmult(epub, e, base);
  b2s::hash64(d, h, epub);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h[j] = d[j];
    c0[j] = kChainKey0[j];
  }
  // chaining_key = HMAC(HMAC(INITIAL_CHAIN_KEY, ephemeral), 0x1)
  hmac_32(t, c0, epub);
  hmac_1(ck, t, 1u);
  // temp = HMAC(ck, DH(ephemeral, responder static)); ck = HMAC(temp, 1); key = HMAC(temp, ck || 2)
  x25519::scalarmult(dh, e, pst);
  hmac_32(t, ck, dh);
  hmac_1(ck, t, 1u);
  hmac_33(key, t, ck, 2u);
  // msg.encrypted_static = AEAD(key, 0, static_public, hash); hash = HASH(hash || it)
  uint32_t spub[8], es[8], tag_s[4];
  ld_words(spub, job.static_public, 8);
  seal_aad32(es, tag_s, key, h, spub, 32u);
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j < 8 ? es[j] : (j < 12 ? tag_s[j - 8] : 0u);
  uint32_t h2[8];
  b2s::hash_cat(h2, h, d, 48);
  // temp = HMAC(ck, static_shared); ck = HMAC(temp, 1); key = HMAC(temp, ck || 2)
  uint32_t ss[8];
  ld_words(ss, job.static_shared, 8);
  hmac_32(t, ck, ss);
  hmac_1(ck, t, 1u);
  hmac_33(key, t, ck, 2u);
  // msg.encrypted_timestamp = AEAD(key, 0, TAI64N, hash); hash = HASH(hash || it)
  uint32_t ts[8] = {0, 0, 0, 0, 0, 0, 0, 0}, et[8], tag_t[4];
  ld_words(ts, job.timestamp, 3);
  seal_aad32(et, tag_t, key, h2, ts, 12u);
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j < 3 ? et[j] : (j < 7 ? tag_t[j - 3] : 0u);
  b2s::hash_cat(h, h2, d, 28);
  // message: type 1 | sender (local index) | eph_pub | enc_static | enc_ts | mac1 | mac2
  uint32_t m[37];
  m[0] = 1u;  // HANDSHAKE_INIT
  m[1] = job.local_index;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[2 + j] = epub[j];
    m[10 + j] = es[j];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) m[18 + j] = tag_s[j];
#pragma unroll
  for (int j = 0; j < 3; ++j) m[22 + j] = et[j];
#pragma unroll
  for (int j = 0; j < 4; ++j) m[25 + j] = tag_t[j];
  uint32_t mk[8], mac1[4], mac2[4] = {0, 0, 0, 0};
  ld_words(mk, job.mac1_key, 8);
  b2s::mac16_116(mac1, mk, m);
#pragma unroll
  for (int j = 0; j < 4; ++j) m[29 + j] = mac1[j];
  if (job.has_cookie) {  // mac2 = MAC(cookie, msg[..mac2_off]) (132 bytes)
    uint32_t ckey[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    ld_words(ckey, job.cookie, 4);
    b2s::keyed_mac(mac2, 16, ckey, 16, m, 132);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) m[33 + j] = mac2[j];
  wg_init_sent &o = prm.out[i];
  st_words(o.message, m, 37);
  o.local_index = job.local_index;
  st_words(o.chaining_key, ck, 8);
  st_words(o.hash, h, 8);
  st_words(o.mac1, mac1, 4);
}

__global__ __launch_bounds__(256) void handshake_response_kernel(HandshakeResponseParams prm) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= prm.n) return;
  uint32_t w[23];
  ld_words(w, prm.msgs + prm.stride * i, 23);
  const wg_response_received_job &job = prm.jobs[i];
  wg_session_keys &o = prm.out[i];
  int32_t status = w[0] == 2u ? WG_STATUS_OK : WG_STATUS_WRONG_PACKET_TYPE;  // HANDSHAKE_RESP
  if (status == WG_STATUS_OK && prm.check_mac1) {  // verify_packet (rate_limiter.rs:182-195)
    uint32_t mac[4];
    b2s::keyed_mac(mac, 16, prm.mac1_key, 32, w, 60);
    if ((mac[0] ^ w[15]) | (mac[1] ^ w[16]) | (mac[2] ^ w[17]) | (mac[3] ^ w[18]))
      status = WG_STATUS_INVALID_MAC;
  }
  uint32_t ck[8], h[8], e[8], peph[8], t[8], dh[8], d[16];
  ld_words(ck, job.chaining_key, 8);
  ld_words(h, job.hash, 8);
  ld_words(e, job.ephemeral_private, 8);
#pragma unroll
  for (int j = 0; j < 8; ++j) peph[j] = w[3 + j];
  // hash = HASH(hash || unencrypted_ephemeral); temp = HMAC(ck, it); ck = HMAC(temp, 1)
  b2s::hash64(d, h, peph);
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = d[j];
  hmac_32(t, ck, peph);
  hmac_1(ck, t, 1u);
  // DH(ephemeral, responder ephemeral), then DH(static, responder ephemeral)
  x25519::scalarmult(dh, e, peph);
  hmac_32(t, ck, dh);
  hmac_1(ck, t, 1u);
  x25519::scalarmult(dh, prm.static_private, peph);
  hmac_32(t, ck, dh);
  hmac_1(ck, t, 1u);
  // psk (zeros when none, handshake.rs:657-661): temp2 / key / hash
  uint32_t psk[8], temp2[8], key[8];
  ld_words(psk, job.preshared_key, 8);
  hmac_32(t, ck, psk);
  hmac_1(ck, t, 1u);
  hmac_33(temp2, t, ck, 2u);
  hmac_33(key, t, temp2, 3u);
  b2s::hash64(d, h, temp2);
  // encrypted_nothing: AEAD-open of the empty plaintext (AAD = hash)
  uint32_t tag[4], none[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  tag_aad32(tag, key, d, none, 0);
  if (status == WG_STATUS_OK && ((tag[0] ^ w[11]) | (tag[1] ^ w[12]) | (tag[2] ^ w[13]) | (tag[3] ^ w[14])))
    status = WG_STATUS_INVALID_AEAD_TAG;
  // temp1 = HMAC(ck, []), temp2 = HMAC(temp1, 1), temp3 = HMAC(temp1, temp2 || 2)
  uint32_t t1[8], t2[8], t3[8], empty[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) empty[j] = 0u;
  b2s::hmac(t1, ck, empty, 0);
  hmac_1(t2, t1, 1u);
  hmac_33(t3, t1, t2, 2u);
  const bool ok = status == WG_STATUS_OK;
  uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  o.status = status;
  o.peer_index = status == WG_STATUS_WRONG_PACKET_TYPE ? 0u : w[1];
  o.receiver_idx = status == WG_STATUS_WRONG_PACKET_TYPE ? 0u : w[2];  // (state match)
  o.pad = 0u;
  // Session::new(local_index, peer_index, temp3, temp2): sending = temp2, receiving = temp3
  st_words(o.sending_key, ok ? t2 : z, 8);
  st_words(o.receiving_key, ok ? t3 : z, 8);
}

// receive_cookie_reply's decryption (handshake.rs:711-724): XChaCha20-Poly1305
// open of the 16-byte cookie with key HASH(LABEL_COOKIE || responder static
// public), the message's 24-byte nonce and aad = the last mac1 sent
__global__ __launch_bounds__(256) void cookie_open_kernel(CookieOpenParams prm) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= prm.n) return;
  const wg_cookie_open_job &job = prm.jobs[i];
  uint32_t m[16], key[8], mac1[4], sub[8];
  ld_words(m, job.message, 16);
  ld_words(key, job.cookie_key, 8);
  ld_words(mac1, job.mac1, 4);
  // m: type 3 | receiver | nonce (6 words) | encrypted cookie (4) | tag (4)
  int32_t status = m[0] == 3u ? WG_STATUS_OK : WG_STATUS_WRONG_PACKET_TYPE;  // COOKIE_REPLY
  hchacha20(sub, key, m + 2);
  uint32_t ks[16];
  chacha20_block(ks, sub, 0u, m[6], m[7]);
  Poly poly;
  poly_init(poly, ks);
  const uint32_t s[4] = {ks[4], ks[5], ks[6], ks[7]};
  poly_block(poly, mac1[0], mac1[1], mac1[2], mac1[3]);  // AAD (16 bytes)
  poly_block(poly, m[8], m[9], m[10], m[11]);
  poly_block(poly, 16u, 0u, 16u, 0u);
  uint32_t tag[4];
  poly_finish(poly, s, tag);
  if (status == WG_STATUS_OK && ((tag[0] ^ m[12]) | (tag[1] ^ m[13]) | (tag[2] ^ m[14]) | (tag[3] ^ m[15])))
    status = WG_STATUS_INVALID_AEAD_TAG;
  chacha20_block(ks, sub, 1u, m[6], m[7]);
  uint32_t cookie[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) cookie[j] = status == WG_STATUS_OK ? m[8 + j] ^ ks[j] : 0u;
  wg_cookie_open_out &o = prm.out[i];
  o.status = status;
  o.receiver_idx = m[1];
  st_words(o.cookie, cookie, 4);
}

}  // namespace wg
