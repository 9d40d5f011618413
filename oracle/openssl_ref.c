/*
 * openssl_ref.c -- independent RFC 8439 implementation used to CROSS-CHECK the
 * oracle and to time the CPU baseline.  TEST INFRASTRUCTURE ONLY.
 *
 * ring 0.17.14 (the crate NepTUN's data path calls, Cargo.lock:1356-1359) is
 * not available offline; OpenSSL 3's EVP_chacha20_poly1305 is the closest
 * stand-in (SIMD assembly, same RFC 8439 construction).  The NepTUN framing
 * around it follows session.rs:205-302 exactly, as in neptun_oracle.c.
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

static void st32(uint8_t *p, uint32_t v) { for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i)); }
static void st64(uint8_t *p, uint64_t v) { for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i)); }
static uint64_t ld64(const uint8_t *p) { uint64_t v = 0; for (int i = 7; i >= 0; --i) v = (v << 8) | p[i]; return v; }

/* One fetched cipher and one context per thread, re-keyed per packet: the
 * per-call EVP_CIPHER_CTX_new + implicit provider fetch serialises threads on
 * OpenSSL's global locks and is not what a tuned caller (or ring) pays. */
static EVP_CIPHER *g_cipher;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void fetch_cipher(void) { g_cipher = EVP_CIPHER_fetch(NULL, "ChaCha20-Poly1305", NULL); }
static __thread EVP_CIPHER_CTX *t_ctx;
static EVP_CIPHER_CTX *thread_ctx(void) {
  pthread_once(&g_once, fetch_cipher);
  if (!t_ctx) t_ctx = EVP_CIPHER_CTX_new();
  return t_ctx;
}

/* Generic AEAD seal/open (used for the RFC 8439 KAT with a 12-byte AAD). */
int ossl_aead_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, int aad_len,
                   const uint8_t *pt, int len, uint8_t *ct, uint8_t tag[16]) {
  EVP_CIPHER_CTX *c = thread_ctx();
  int ok = c && g_cipher && EVP_EncryptInit_ex2(c, g_cipher, key, nonce, NULL);
  int n = 0;
  if (ok && aad_len) ok = EVP_EncryptUpdate(c, NULL, &n, aad, aad_len);
  if (ok && len) ok = EVP_EncryptUpdate(c, ct, &n, pt, len);
  if (ok) ok = EVP_EncryptFinal_ex(c, ct + n, &n);
  if (ok) ok = EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_GET_TAG, 16, tag);
  return ok ? 0 : -1;
}

int ossl_aead_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, int aad_len,
                   const uint8_t *ct, int len, const uint8_t tag[16], uint8_t *pt) {
  EVP_CIPHER_CTX *c = thread_ctx();
  int ok = c && g_cipher && EVP_DecryptInit_ex2(c, g_cipher, key, nonce, NULL);
  int n = 0;
  if (ok && aad_len) ok = EVP_DecryptUpdate(c, NULL, &n, aad, aad_len);
  if (ok && len) ok = EVP_DecryptUpdate(c, pt, &n, ct, len);
  if (ok) ok = EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, 16, (void *)tag);
  if (ok) ok = EVP_DecryptFinal_ex(c, pt + n, &n) > 0;
  return ok ? 0 : -1;
}

/* session.rs:205-259 framing over OpenSSL. */
int ossl_format_packet_data(const uint8_t key[32], uint32_t sending_index, uint64_t counter,
                            const uint8_t *payload, int len, uint8_t *out) {
  uint8_t nonce[12] = {0};
  st64(nonce + 4, counter);
  st32(out, 4u);
  st32(out + 4, sending_index);
  st64(out + 8, counter);
  return ossl_aead_seal(key, nonce, NULL, 0, payload, len, out + 16, out + 16 + len);
}

/* session.rs:265-302 (no replay window) over OpenSSL; returns 0 or -1 (InvalidAeadTag). */
int ossl_receive_packet_data(const uint8_t key[32], const uint8_t *datagram, int len, uint8_t *out) {
  uint8_t nonce[12] = {0};
  st64(nonce + 4, ld64(datagram + 8));
  int p = len - 32;
  return ossl_aead_open(key, nonce, NULL, 0, datagram + 16, p, datagram + 16 + p, out);
}

/* Per-thread X25519 context for the CPU baseline: the private key and the
 * peer key object are created once, the peer's raw public value is replaced per
 * call (EVP_PKEY_new_raw_* per call serialises threads on provider locks). */
typedef struct {
  EVP_PKEY *priv, *peer;
  EVP_PKEY_CTX *ctx;
} x25519_thread;
static __thread x25519_thread t_x;

int ossl_x25519_fast(uint8_t out[32], const uint8_t scalar[32], const uint8_t point[32]) {
  if (!t_x.priv) {
    t_x.priv = EVP_PKEY_new_raw_private_key(EVP_PKEY_X25519, NULL, scalar, 32);
    t_x.peer = EVP_PKEY_new_raw_public_key(EVP_PKEY_X25519, NULL, point, 32);
    t_x.ctx = t_x.priv ? EVP_PKEY_CTX_new(t_x.priv, NULL) : NULL;
    if (!t_x.ctx || EVP_PKEY_derive_init(t_x.ctx) <= 0) return -1;
  }
  if (EVP_PKEY_set1_encoded_public_key(t_x.peer, point, 32) <= 0) return -1;
  size_t len = 32;
  if (EVP_PKEY_derive_set_peer(t_x.ctx, t_x.peer) <= 0) return -1;
  return EVP_PKEY_derive(t_x.ctx, out, &len) > 0 && len == 32 ? 0 : -1;
}

/* X25519 (RFC 7748) through OpenSSL's EVP_PKEY -- an independent check of
 * oracle/handshake_model.py and the CPU baseline of the handshake kernels.
 * Returns 0, or -1 when OpenSSL refuses (it rejects an all-zero shared secret). */
int ossl_x25519(uint8_t out[32], const uint8_t scalar[32], const uint8_t point[32]) {
  EVP_PKEY *priv = EVP_PKEY_new_raw_private_key(EVP_PKEY_X25519, NULL, scalar, 32);
  EVP_PKEY *peer = EVP_PKEY_new_raw_public_key(EVP_PKEY_X25519, NULL, point, 32);
  EVP_PKEY_CTX *c = priv ? EVP_PKEY_CTX_new(priv, NULL) : NULL;
  size_t len = 32;
  int ok = c && peer && EVP_PKEY_derive_init(c) > 0 && EVP_PKEY_derive_set_peer(c, peer) > 0 &&
           EVP_PKEY_derive(c, out, &len) > 0 && len == 32;
  EVP_PKEY_CTX_free(c);
  EVP_PKEY_free(peer);
  EVP_PKEY_free(priv);
  return ok ? 0 : -1;
}
