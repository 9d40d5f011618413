// wg_blake2s.h -- BLAKE2s (RFC 7693) and the Noise helpers of NepTUN's
// handshake (neptun/src/noise/handshake.rs:42-91) on 32-bit words, written
// once for the device and the host (the host precomputes the wave-uniform
// hashes; tests/test_handshake_cpu.py checks these functions against hashlib).
// Messages are little-endian 32-bit words; lengths are in bytes.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define WG_HD __host__ __device__ __forceinline__
#else
#define WG_HD static inline
#endif

namespace wg {
namespace b2s {

constexpr uint32_t kIV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                             0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
constexpr uint8_t kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

WG_HD uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

#define WG_B2S_G(a, b, c, d, x, y) \
  a = a + b + (x);                 \
  d = rotr(d ^ a, 16);             \
  c = c + d;                       \
  b = rotr(b ^ c, 12);             \
  a = a + b + (y);                 \
  d = rotr(d ^ a, 8);              \
  c = c + d;                       \
  b = rotr(b ^ c, 7);

// one compression: t = bytes hashed so far including this block (< 2^32 here)
WG_HD void compress(uint32_t h[8], const uint32_t m[16], uint32_t t, bool last) {
  uint32_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint32_t v8 = kIV[0], v9 = kIV[1], v10 = kIV[2], v11 = kIV[3];
  uint32_t v12 = kIV[4] ^ t, v13 = kIV[5], v14 = last ? ~kIV[6] : kIV[6], v15 = kIV[7];
#if defined(__HIPCC__)
#pragma unroll
#endif
  for (int r = 0; r < 10; ++r) {
    const uint8_t *s = kSigma[r];
    WG_B2S_G(v0, v4, v8, v12, m[s[0]], m[s[1]])
    WG_B2S_G(v1, v5, v9, v13, m[s[2]], m[s[3]])
    WG_B2S_G(v2, v6, v10, v14, m[s[4]], m[s[5]])
    WG_B2S_G(v3, v7, v11, v15, m[s[6]], m[s[7]])
    WG_B2S_G(v0, v5, v10, v15, m[s[8]], m[s[9]])
    WG_B2S_G(v1, v6, v11, v12, m[s[10]], m[s[11]])
    WG_B2S_G(v2, v7, v8, v13, m[s[12]], m[s[13]])
    WG_B2S_G(v3, v4, v9, v14, m[s[14]], m[s[15]])
  }
  h[0] ^= v0 ^ v8;
  h[1] ^= v1 ^ v9;
  h[2] ^= v2 ^ v10;
  h[3] ^= v3 ^ v11;
  h[4] ^= v4 ^ v12;
  h[5] ^= v5 ^ v13;
  h[6] ^= v6 ^ v14;
  h[7] ^= v7 ^ v15;
}
#undef WG_B2S_G

// parameter block: digest length, key length, fanout 1, depth 1
WG_HD void init(uint32_t h[8], uint32_t outlen, uint32_t keylen) {
  for (int i = 0; i < 8; ++i) h[i] = kIV[i];
  h[0] ^= 0x01010000u ^ (keylen << 8) ^ outlen;
}

// BLAKE2s-256(a[8] || b[8]) -- b2s_hash of two 32-byte inputs (handshake.rs:42-48)
WG_HD void hash64(uint32_t out[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t m[16];
  for (int i = 0; i < 8; ++i) {
    m[i] = a[i];
    m[8 + i] = b[i];
  }
  init(out, 32, 0);
  compress(out, m, 64, true);
}

// BLAKE2s-256 of one block of n <= 64 bytes given as 16 zero-padded words
WG_HD void hash_block(uint32_t out[8], const uint32_t m[16], uint32_t n) {
  init(out, 32, 0);
  compress(out, m, n, true);
}

// HMAC-BLAKE2s (RFC 2104, 64-byte block) with a 32-byte key and <= 64 bytes of
// data in 16 zero-padded words -- b2s_hmac / b2s_hmac2 (handshake.rs:50-72)
WG_HD void hmac(uint32_t out[8], const uint32_t key[8], const uint32_t data[16], uint32_t n) {
  uint32_t pad[16], ih[8];
  for (int i = 0; i < 16; ++i) pad[i] = (i < 8 ? key[i] : 0u) ^ 0x36363636u;
  init(ih, 32, 0);
  compress(ih, pad, 64, n == 0);  // empty data: the key block is the last block
  if (n) compress(ih, data, 64 + n, true);
  for (int i = 0; i < 16; ++i) pad[i] = (i < 8 ? key[i] : 0u) ^ 0x5c5c5c5cu;
  init(out, 32, 0);
  compress(out, pad, 64, false);
  uint32_t m[16];
  for (int i = 0; i < 16; ++i) m[i] = i < 8 ? ih[i] : 0u;
  compress(out, m, 96, true);
}

// keyed BLAKE2s with a 16-byte digest over the first 116 bytes of a handshake
// initiation (29 words) -- b2s_keyed_mac_16 for mac1 (handshake.rs:75-80,
// rate_limiter.rs:187)
WG_HD void mac16_116(uint32_t out[4], const uint32_t key[8], const uint32_t msg[29]) {
  uint32_t h[8], m[16];
  init(h, 16, 32);
  for (int i = 0; i < 16; ++i) m[i] = i < 8 ? key[i] : 0u;
  compress(h, m, 64, false);
  for (int i = 0; i < 16; ++i) m[i] = msg[i];
  compress(h, m, 128, false);
  for (int i = 0; i < 16; ++i) m[i] = i < 13 ? msg[16 + i] : 0u;
  compress(h, m, 180, true);
  for (int i = 0; i < 4; ++i) out[i] = h[i];
}

// BLAKE2s-256(a[8] || b[0..blen)) for blen <= 64 (b as zero-padded words) --
// b2s_hash(hash, data) of the handshake with a 32-byte chaining hash first
WG_HD void hash_cat(uint32_t out[8], const uint32_t a[8], const uint32_t b[16], uint32_t blen) {
  uint32_t m[16];
  init(out, 32, 0);
  if (blen <= 32) {
    for (int i = 0; i < 16; ++i) m[i] = i < 8 ? a[i] : b[i - 8];
    compress(out, m, 32 + blen, true);
    return;
  }
  for (int i = 0; i < 16; ++i) m[i] = i < 8 ? a[i] : b[i - 8];
  compress(out, m, 64, false);
  for (int i = 0; i < 16; ++i) m[i] = i < 8 ? b[8 + i] : 0u;
  compress(out, m, 32 + blen, true);
}

// Keyed BLAKE2s (RFC 7693 MAC mode) with an outlen-byte digest over dlen bytes
// given as zero-padded words (words past dlen must read as 0 up to the next
// 64-byte boundary): Blake2sMac -- b2s_keyed_mac_16 / _16_2 / b2s_mac_24
// (handshake.rs:74-97).  keylen is 16 or 32 (key words past it are ignored).
WG_HD void keyed_mac(uint32_t *out, uint32_t outlen, const uint32_t key[8], uint32_t keylen,
                     const uint32_t *data, uint32_t dlen) {
  uint32_t h[8], m[16];
  init(h, outlen, keylen);
  for (int i = 0; i < 16; ++i) m[i] = i < (int)(keylen / 4) ? key[i] : 0u;
  compress(h, m, 64, dlen == 0);
  for (uint32_t off = 0; off < dlen; off += 64) {
    const bool last = off + 64 >= dlen;
    for (int i = 0; i < 16; ++i) m[i] = off + 4u * i < dlen ? data[off / 4 + i] : 0u;
    compress(h, m, 64 + (last ? dlen : off + 64), last);
  }
  for (uint32_t i = 0; i < outlen / 4; ++i) out[i] = h[i];
}

}  // namespace b2s
}  // namespace wg
