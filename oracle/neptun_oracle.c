/*
 * neptun_oracle.c -- CPU restatement of NepTUN's transport-data AEAD path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in neptun_amd/ links, loads or calls this
 * file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * use it, and only as the checker (never as the measured or shipped path).
 *
 * What it restates (reference = /root/reference, NordSecurity/NepTUN):
 *   - Session::format_packet_data     neptun/src/noise/session.rs:205-259
 *       header  type=4 LE32 | sending_index LE32 | counter LE64   (:221-227)
 *       nonce   00 00 00 00 | LE64(counter)                        (:230-235)
 *       AAD     empty                                              (:239)
 *       body    ChaCha20-Poly1305 ciphertext, no padding, 16 B tag (:229, :246)
 *   - Session::receive_packet_data    session.rs:265-302 (minus the replay
 *       window, which lives in oracle/tunn_model.py): open_in_place, failure ->
 *       InvalidAeadTag (:290-296)
 *   - Tunn::parse_incoming_packet     neptun/src/noise/mod.rs:139-199 (DATA arm)
 *   - the AEAD itself: ring 0.17.14 LessSafeKey with CHACHA20_POLY1305
 *       (Cargo.lock:1356-1359, not vendored).  Restated from its published
 *       algorithm, RFC 8439 sections 2.1-2.8: ChaCha20 block function (2.3),
 *       Poly1305 (2.5), Poly1305 key generation from block 0 (2.6), AEAD
 *       construction AAD|pad16|CT|pad16|LE64(aad_len)|LE64(ct_len) (2.8).
 *
 * Parity pinning: the primitive is pinned by the reference's own known-answer
 * test, handshake.rs:957-992 (RFC 8439 2.8.2 vector, run through ring); the
 * data-path framing has no reference vectors (every reference data-path test
 * uses OsRng keys), so it is pinned by construction to session.rs and cross-
 * checked against independent RFC 8439 implementations (OpenSSL 3 EVP, node
 * crypto) by oracle/gen_golden.py, which writes tests/golden/.
 *
 * Implementation choices are deliberately different from the GPU kernels so
 * the two do not share mistakes: Poly1305 here uses 64-bit limbs with
 * unsigned __int128 products; the HIP kernel uses 32-bit limbs with
 * v_mad_u64_u32 chains.
 */
#include "neptun_oracle.h"

#include <string.h>

/* ------------------------------------------------------------------ */
/* byte helpers                                                       */
/* ------------------------------------------------------------------ */
static uint32_t ld32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint64_t ld64(const uint8_t *p) { return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32); }
static void st32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static void st64(uint8_t *p, uint64_t v) { st32(p, (uint32_t)v); st32(p + 4, (uint32_t)(v >> 32)); }
static uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* ------------------------------------------------------------------ */
/* RFC 8439 2.3 ChaCha20 block function                               */
/* ------------------------------------------------------------------ */
#define QR(a, b, c, d)                      \
  do {                                      \
    a += b; d ^= a; d = rotl32(d, 16);      \
    c += d; b ^= c; b = rotl32(b, 12);      \
    a += b; d ^= a; d = rotl32(d, 8);       \
    c += d; b ^= c; b = rotl32(b, 7);       \
  } while (0)

void neptun_oracle_chacha20_block(const uint8_t key[32], uint32_t block_counter,
                                  const uint8_t nonce[12], uint8_t out[64]) {
  uint32_t in[16], x[16];
  in[0] = 0x61707865u; in[1] = 0x3320646eu; in[2] = 0x79622d32u; in[3] = 0x6b206574u;
  for (int i = 0; i < 8; ++i) in[4 + i] = ld32(key + 4 * i);
  in[12] = block_counter;
  in[13] = ld32(nonce); in[14] = ld32(nonce + 4); in[15] = ld32(nonce + 8);
  memcpy(x, in, sizeof x);
  for (int i = 0; i < 10; ++i) {
    QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; ++i) st32(out + 4 * i, x[i] + in[i]);
}

/* RFC 8439 2.4: XOR with keystream starting at block `counter`. */
static void chacha20_xor(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                         const uint8_t *in, uint8_t *out, size_t len) {
  uint8_t ks[64];
  for (size_t off = 0; off < len; off += 64, ++counter) {
    neptun_oracle_chacha20_block(key, counter, nonce, ks);
    size_t n = len - off < 64 ? len - off : 64;
    for (size_t i = 0; i < n; ++i) out[off + i] = in[off + i] ^ ks[i];
  }
}

/* ------------------------------------------------------------------ */
/* RFC 8439 2.5 Poly1305, incremental, 64-bit limbs                   */
/* ------------------------------------------------------------------ */
typedef struct {
  uint64_t r0, r1, s1;  /* clamped r, s1 = r1 + r1/4 (r1 is a multiple of 4) */
  uint64_t h0, h1, h2;  /* accumulator, h2 holds bits 128.. */
  uint64_t pad0, pad1;  /* the "s" half of the one-time key */
} poly1305_state;

static void poly_init(poly1305_state *st, const uint8_t key[32]) {
  st->r0 = ld64(key) & 0x0ffffffc0fffffffull;
  st->r1 = ld64(key + 8) & 0x0ffffffc0ffffffcull;
  st->s1 = st->r1 + (st->r1 >> 2);
  st->h0 = st->h1 = st->h2 = 0;
  st->pad0 = ld64(key + 16);
  st->pad1 = ld64(key + 24);
}

/* one 16-byte block with the 2^128 bit set (`hibit`), h = (h + m) * r mod* p */
static void poly_block(poly1305_state *st, const uint8_t m[16], uint64_t hibit) {
  typedef unsigned __int128 u128;
  u128 t = (u128)st->h0 + ld64(m);
  uint64_t h0 = (uint64_t)t;
  t = (u128)st->h1 + ld64(m + 8) + (uint64_t)(t >> 64);
  uint64_t h1 = (uint64_t)t;
  uint64_t h2 = st->h2 + (uint64_t)(t >> 64) + hibit;
  /* h * r, using 2^130 == 5 (mod p):  h1*r1*2^128 = h1*(r1/4)*2^130 -> 5*h1*r1/4 */
  u128 d0 = (u128)h0 * st->r0 + (u128)h1 * st->s1;
  u128 d1 = (u128)h0 * st->r1 + (u128)h1 * st->r0 + (u128)h2 * st->s1;
  uint64_t d2 = h2 * st->r0; /* h2 is tiny (< 8) */
  d1 += (uint64_t)(d0 >> 64);
  d2 += (uint64_t)(d1 >> 64);
  h0 = (uint64_t)d0;
  h1 = (uint64_t)d1;
  /* partial reduction: bits >= 130 times 5 folded back in */
  uint64_t c = (d2 >> 2) * 5;
  h2 = d2 & 3;
  t = (u128)h0 + c;
  h0 = (uint64_t)t;
  t = (u128)h1 + (uint64_t)(t >> 64);
  h1 = (uint64_t)t;
  h2 += (uint64_t)(t >> 64);
  st->h0 = h0; st->h1 = h1; st->h2 = h2;
}

static void poly_finish(poly1305_state *st, uint8_t tag[16]) {
  typedef unsigned __int128 u128;
  uint64_t h0 = st->h0, h1 = st->h1, h2 = st->h2;
  /* full carry: fold bits >= 130 */
  uint64_t c = (h2 >> 2) * 5;
  h2 &= 3;
  u128 t = (u128)h0 + c; h0 = (uint64_t)t;
  t = (u128)h1 + (uint64_t)(t >> 64); h1 = (uint64_t)t;
  h2 += (uint64_t)(t >> 64);
  /* g = h + 5 - 2^130; if g >= 0 (no borrow) take g */
  t = (u128)h0 + 5; uint64_t g0 = (uint64_t)t;
  t = (u128)h1 + (uint64_t)(t >> 64); uint64_t g1 = (uint64_t)t;
  uint64_t g2 = h2 + (uint64_t)(t >> 64);
  if (g2 >> 2) { h0 = g0; h1 = g1; }
  /* tag = (h + s) mod 2^128 */
  t = (u128)h0 + st->pad0; h0 = (uint64_t)t;
  h1 = h1 + st->pad1 + (uint64_t)(t >> 64);
  st64(tag, h0); st64(tag + 8, h1);
}

/* Poly1305 over bytes with RFC 8439 2.5 final-block 0x01 padding. */
void neptun_oracle_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]) {
  poly1305_state st;
  poly_init(&st, key);
  while (len >= 16) { poly_block(&st, msg, 1); msg += 16; len -= 16; }
  if (len) {
    uint8_t b[16] = {0};
    memcpy(b, msg, len);
    b[len] = 1;
    poly_block(&st, b, 0);
  }
  poly_finish(&st, tag);
}

/* RFC 8439 2.8 AEAD MAC input: AAD | pad16 | CT | pad16 | LE64(aad) | LE64(ct) */
static void aead_mac(const uint8_t otk[32], const uint8_t *aad, size_t aad_len,
                     const uint8_t *ct, size_t ct_len, uint8_t tag[16]) {
  poly1305_state st;
  uint8_t b[16];
  poly_init(&st, otk);
  for (size_t i = 0; i < aad_len; i += 16) {
    size_t n = aad_len - i < 16 ? aad_len - i : 16;
    memset(b, 0, 16); memcpy(b, aad + i, n);
    poly_block(&st, b, 1);
  }
  for (size_t i = 0; i < ct_len; i += 16) {
    size_t n = ct_len - i < 16 ? ct_len - i : 16;
    memset(b, 0, 16); memcpy(b, ct + i, n);
    poly_block(&st, b, 1);
  }
  st64(b, (uint64_t)aad_len); st64(b + 8, (uint64_t)ct_len);
  poly_block(&st, b, 1);
  poly_finish(&st, tag);
}

static void otk_gen(const uint8_t key[32], const uint8_t nonce[12], uint8_t otk[32]) {
  uint8_t blk[64];
  neptun_oracle_chacha20_block(key, 0, nonce, blk); /* RFC 8439 2.6 */
  memcpy(otk, blk, 32);
}

void neptun_oracle_aead_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                             size_t aad_len, const uint8_t *pt, size_t len, uint8_t *ct,
                             uint8_t tag[16]) {
  uint8_t otk[32];
  otk_gen(key, nonce, otk);
  chacha20_xor(key, 1, nonce, pt, ct, len);
  aead_mac(otk, aad, aad_len, ct, len, tag);
}

int neptun_oracle_aead_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                            size_t aad_len, const uint8_t *ct, size_t len, const uint8_t tag[16],
                            uint8_t *pt) {
  uint8_t otk[32], want[16];
  otk_gen(key, nonce, otk);
  aead_mac(otk, aad, aad_len, ct, len, want);
  uint8_t diff = 0;
  for (int i = 0; i < 16; ++i) diff |= (uint8_t)(want[i] ^ tag[i]);
  if (diff) {
    /* ring 0.17 open_within: on a tag mismatch the plaintext region is zeroed
     * so unauthenticated bytes are never exposed; neptun then returns
     * InvalidAeadTag (session.rs:296).  The GPU path keeps the same contract. */
    memset(pt, 0, len);
    return -1;
  }
  chacha20_xor(key, 1, nonce, ct, pt, len);
  return 0;
}

/* ------------------------------------------------------------------ */
/* NepTUN framing (session.rs)                                        */
/* ------------------------------------------------------------------ */
static void wg_nonce(uint64_t counter, uint8_t nonce[12]) {
  memset(nonce, 0, 4);          /* session.rs:231  [0u8; 12] */
  st64(nonce + 4, counter);     /* session.rs:232-235 nonce[4..12] = LE64(counter) */
}

int neptun_oracle_format_packet_data(const uint8_t key[32], uint32_t sending_index,
                                     uint64_t counter, const uint8_t *payload, size_t payload_len,
                                     uint8_t *out, size_t out_cap) {
  if (out_cap < payload_len + NEPTUN_DATA_OVERHEAD_SZ) /* session.rs:210-217 */
    return NEPTUN_ERR_INCORRECT_PACKET_LENGTH;
  uint8_t nonce[12];
  st32(out, NEPTUN_MSG_DATA);             /* session.rs:225 */
  st32(out + 4, sending_index);           /* :226 */
  st64(out + 8, counter);                 /* :227 */
  wg_nonce(counter, nonce);
  neptun_oracle_aead_seal(key, nonce, NULL, 0, payload, payload_len, out + NEPTUN_DATA_OFFSET,
                          out + NEPTUN_DATA_OFFSET + payload_len); /* :236-246 */
  return NEPTUN_OK;
}

int neptun_oracle_parse_data_header(const uint8_t *datagram, size_t len, uint32_t *receiver_idx,
                                    uint64_t *counter) {
  /* noise/mod.rs:139-199: len >= 4, type LE32; DATA requires len >= 32 */
  if (len < 4) return NEPTUN_ERR_INVALID_PACKET;
  if (ld32(datagram) != NEPTUN_MSG_DATA || len < NEPTUN_DATA_OVERHEAD_SZ)
    return NEPTUN_ERR_INVALID_PACKET;
  *receiver_idx = ld32(datagram + 4);
  *counter = ld64(datagram + 8);
  return NEPTUN_OK;
}

int neptun_oracle_receive_packet_data(const uint8_t key[32], uint32_t receiving_index,
                                      const uint8_t *datagram, size_t len, uint8_t *out,
                                      size_t out_cap, size_t *out_len) {
  uint32_t ridx; uint64_t counter;
  int rc = neptun_oracle_parse_data_header(datagram, len, &ridx, &counter);
  if (rc) return rc;
  size_t ct_len = len - NEPTUN_DATA_OFFSET; /* ct || tag, session.rs:270 */
  if (out_cap < ct_len) return NEPTUN_ERR_DESTINATION_BUFFER_TOO_SMALL; /* :271-274 */
  if (ridx != receiving_index) return NEPTUN_ERR_WRONG_INDEX;            /* :275-277 */
  uint8_t nonce[12];
  wg_nonce(counter, nonce);
  size_t p = ct_len - NEPTUN_AEAD_SIZE;
  if (neptun_oracle_aead_open(key, nonce, NULL, 0, datagram + NEPTUN_DATA_OFFSET, p,
                              datagram + NEPTUN_DATA_OFFSET + p, out))
    return NEPTUN_ERR_INVALID_AEAD_TAG; /* :296 */
  *out_len = p;
  return NEPTUN_OK;
}

/* ------------------------------------------------------------------ */
/* batch forms mirroring include/neptun_gpu.h (same descriptor meaning) */
/* ------------------------------------------------------------------ */
void neptun_oracle_seal_batch(const neptun_oracle_desc *descs, size_t n, const uint8_t *keys,
                              const uint32_t *key_index, const uint8_t *src, uint8_t *dst,
                              int32_t *status) {
  for (size_t i = 0; i < n; ++i) {
    const neptun_oracle_desc *d = &descs[i];
    status[i] = neptun_oracle_format_packet_data(keys + 32 * (size_t)d->key_slot,
                                                 key_index[d->key_slot], d->counter,
                                                 src + d->src_off, d->len, dst + d->dst_off,
                                                 (size_t)d->len + NEPTUN_DATA_OVERHEAD_SZ);
  }
}

void neptun_oracle_open_batch(const neptun_oracle_desc *descs, size_t n, const uint8_t *keys,
                              const uint32_t *key_index, const uint8_t *src, uint8_t *dst,
                              int32_t *status) {
  for (size_t i = 0; i < n; ++i) {
    const neptun_oracle_desc *d = &descs[i];
    size_t out_len = 0;
    size_t cap = d->len >= NEPTUN_DATA_OFFSET ? d->len - NEPTUN_DATA_OFFSET : 0;
    status[i] = neptun_oracle_receive_packet_data(keys + 32 * (size_t)d->key_slot,
                                                  key_index[d->key_slot], src + d->src_off,
                                                  d->len, dst + d->dst_off, cap, &out_len);
  }
}
