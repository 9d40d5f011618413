/*
 * gw_cpu_tunn.h -- the gateway's CPU backend (udp_gateway.c built with -DGW_CPU):
 * the same batch calls, done on the calling thread one packet after another with
 * OpenSSL's EVP ChaCha20-Poly1305 -- the way NepTUN's workers run
 * Tunn::encapsulate / Tunn::decapsulate per packet with ring
 * (device/packet_workers.rs:207-287, noise/mod.rs:295-380, session.rs:205-302).
 * It exists to give the GPU gateway a same-box CPU line over the same sockets,
 * threads and batches; no GPU is touched (the replay window is the library's
 * host-side wg_replay_*, session.rs:40-157).
 *
 * One session per Tunn (what the gateway installs): ring slot local_index % 8.
 * Results and destination bytes follow oracle/tunn_model.py (tests/test_udp_gateway.py
 * checks them): encapsulate -> WriteToNetwork(P + 32); decapsulate -> parse, session,
 * capacity, index, replay, ct||tag into dst opened in place (zeroed plaintext on a tag
 * mismatch), replay mark, validate_decapsulated_packet (mod.rs:606-670).
 */
#ifndef GW_CPU_TUNN_H
#define GW_CPU_TUNN_H

#include <openssl/evp.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <string.h>

#include "neptun_gpu.h"
#include "neptun_tunn.h"

typedef struct cpu_tunn {
  uint8_t send_key[32], recv_key[32];
  uint32_t local_idx, peer_idx;
  int has_session;
  uint64_t send_ctr;
  wg_replay win;
  uint64_t tx_bytes, rx_bytes;
  pthread_mutex_t mu; /* Mutex<Tunn> (device/peer.rs:29) */
} cpu_tunn;

/* one EVP context per thread and direction, keyed once: a packet then only sets
 * its nonce (re-selecting the cipher per packet costs OpenSSL 3 a fetch) */
static __thread EVP_CIPHER_CTX *gw_evp[2];
static __thread uint8_t gw_evp_key[2][32];

static EVP_CIPHER_CTX *gw_ctx(int dec, const uint8_t key[32]) {
  if (!gw_evp[dec]) {
    gw_evp[dec] = EVP_CIPHER_CTX_new();
    if (!gw_evp[dec] || EVP_CipherInit_ex(gw_evp[dec], EVP_chacha20_poly1305(), NULL, key, NULL, !dec) != 1)
      return NULL;
    memcpy(gw_evp_key[dec], key, 32);
  } else if (memcmp(gw_evp_key[dec], key, 32) != 0) {
    if (EVP_CipherInit_ex(gw_evp[dec], NULL, NULL, key, NULL, !dec) != 1) return NULL;
    memcpy(gw_evp_key[dec], key, 32);
  }
  return gw_evp[dec];
}

static void gw_nonce(uint64_t ctr, uint8_t n[12]) {
  memset(n, 0, 4); /* session.rs:230-235: 0^4 | LE64(counter) */
  for (int i = 0; i < 8; ++i) n[4 + i] = (uint8_t)(ctr >> (8 * i));
}

static void gw_st32(uint8_t *p, uint32_t v) {
  for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

static uint32_t gw_ld32(const uint8_t *p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

static int cpu_tunn_create(cpu_tunn **out) {
  cpu_tunn *t = calloc(1, sizeof *t);
  if (!t) return WG_RC_OUT_OF_MEMORY;
  wg_replay_init(&t->win);
  pthread_mutex_init(&t->mu, NULL);
  *out = t;
  return 0;
}

static int cpu_tunn_destroy(cpu_tunn *t) {
  pthread_mutex_destroy(&t->mu);
  free(t);
  return 0;
}

static int cpu_tunn_install_session(cpu_tunn *t, uint32_t local, uint32_t peer, const uint8_t rkey[32],
                                    const uint8_t skey[32], int make_current) {
  (void)make_current;
  memcpy(t->recv_key, rkey, 32);
  memcpy(t->send_key, skey, 32);
  t->local_idx = local;
  t->peer_idx = peer;
  t->send_ctr = 0;
  wg_replay_init(&t->win);
  t->has_session = 1;
  return 0;
}

static void gw_set_err(wg_tunn_result *r, int kind, int status) {
  memset(r, 0, sizeof *r);
  r->kind = kind;
  r->status = status;
}

static int cpu_tunn_encapsulate_batch(cpu_tunn *t, uint32_t n, const uint8_t *const *src,
                                      const uint32_t *src_len, uint8_t *const *dst, const uint32_t *dst_cap,
                                      wg_tunn_result *res) {
  pthread_mutex_lock(&t->mu);
  EVP_CIPHER_CTX *c = gw_ctx(0, t->send_key);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t P = src_len[i];
    if (dst_cap[i] < P + 16) { gw_set_err(&res[i], WG_TUNN_ERR, WG_STATUS_INVALID_LENGTH); continue; }
    if (!t->has_session) { gw_set_err(&res[i], WG_TUNN_NOT_DATA, WG_STATUS_NO_CURRENT_SESSION); continue; }
    if (dst_cap[i] < P + 32) { gw_set_err(&res[i], WG_TUNN_ERR, WG_STATUS_INCORRECT_PACKET_LENGTH); continue; }
    const uint64_t ctr = t->send_ctr++;
    uint8_t *o = dst[i], nonce[12];
    gw_st32(o, WG_MSG_DATA);
    gw_st32(o + 4, t->peer_idx);
    for (int k = 0; k < 8; ++k) o[8 + k] = (uint8_t)(ctr >> (8 * k));
    gw_nonce(ctr, nonce);
    int l = 0;
    if (!c || EVP_EncryptInit_ex(c, NULL, NULL, NULL, nonce) != 1 ||
        (P && EVP_EncryptUpdate(c, o + 16, &l, src[i], (int)P) != 1) || EVP_EncryptFinal_ex(c, o + 16 + l, &l) != 1 ||
        EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_GET_TAG, 16, o + 16 + P) != 1) {
      pthread_mutex_unlock(&t->mu);
      return WG_RC_INVALID_ARGUMENT;
    }
    memset(&res[i], 0, sizeof res[i]);
    res[i].kind = WG_TUNN_WRITE_TO_NETWORK;
    res[i].len = P + 32;
    t->tx_bytes += P + 32;
  }
  pthread_mutex_unlock(&t->mu);
  return 0;
}

/* validate_decapsulated_packet (mod.rs:606-670) */
static void gw_validate(cpu_tunn *t, const uint8_t *pt, uint32_t P, wg_tunn_result *r) {
  memset(r, 0, sizeof *r);
  if (P == 0) {
    r->kind = WG_TUNN_DONE;
    t->rx_bytes += 32;
    return;
  }
  uint32_t ip_len;
  const uint8_t v = pt[0] >> 4;
  if (v == 4 && P >= 20) {
    ip_len = (uint32_t)pt[2] << 8 | pt[3];
    r->ip_version = 4;
    memcpy(r->src_ip, pt + 12, 4);
  } else if (v == 6 && P >= 40) {
    ip_len = ((uint32_t)pt[4] << 8 | pt[5]) + 40;
    r->ip_version = 6;
    memcpy(r->src_ip, pt + 8, 16);
  } else {
    gw_set_err(r, WG_TUNN_ERR, WG_STATUS_INVALID_PACKET);
    return;
  }
  if (ip_len > P) {
    gw_set_err(r, WG_TUNN_ERR, WG_STATUS_INVALID_PACKET);
    return;
  }
  r->kind = WG_TUNN_WRITE_TO_TUNNEL;
  r->len = ip_len;
  t->rx_bytes += ip_len + 32;
}

static int cpu_tunn_decapsulate_batch(cpu_tunn *t, uint32_t n, const uint8_t *const *dg, const uint32_t *len,
                                      uint8_t *const *dst, const uint32_t *dst_cap, wg_tunn_result *res) {
  pthread_mutex_lock(&t->mu);
  EVP_CIPHER_CTX *c = gw_ctx(1, t->recv_key);
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *d = dg[i];
    const uint32_t L = len[i];
    wg_tunn_result *r = &res[i];
    if (L == 0) { gw_set_err(r, WG_TUNN_NOT_DATA, 0); continue; }
    if (L < 4) { gw_set_err(r, WG_TUNN_ERR, WG_STATUS_INVALID_PACKET); continue; }
    const uint32_t type = gw_ld32(d);
    if ((type == 1 && L == 148) || (type == 2 && L == 92) || (type == 3 && L == 64)) {
      gw_set_err(r, WG_TUNN_NOT_DATA, 0);
      continue;
    }
    if (type != WG_MSG_DATA || L < 32) { gw_set_err(r, WG_TUNN_ERR, WG_STATUS_INVALID_PACKET); continue; }
    const uint32_t ridx = gw_ld32(d + 4);
    uint64_t ctr = 0;
    for (int k = 0; k < 8; ++k) ctr |= (uint64_t)d[8 + k] << (8 * k);
    if (!t->has_session || ridx % WG_N_SESSIONS != t->local_idx % WG_N_SESSIONS) {
      gw_set_err(r, WG_TUNN_ERR, WG_STATUS_NO_CURRENT_SESSION);
      continue;
    }
    if (dst_cap[i] < L - 16) { gw_set_err(r, WG_TUNN_ERR, WG_STATUS_DESTINATION_BUFFER_TOO_SMALL); continue; }
    if (ridx != t->local_idx) { gw_set_err(r, WG_TUNN_ERR, WG_STATUS_WRONG_INDEX); continue; }
    int e = wg_replay_will_accept(&t->win, ctr);
    if (e) { gw_set_err(r, WG_TUNN_ERR, e); continue; }
    const uint32_t P = L - 32;
    uint8_t nonce[12], tag[16];
    gw_nonce(ctr, nonce);
    memcpy(tag, d + 16 + P, 16);
    int l = 0;
    int ok = c && EVP_DecryptInit_ex(c, NULL, NULL, NULL, nonce) == 1 &&
             (P == 0 || EVP_DecryptUpdate(c, dst[i], &l, d + 16, (int)P) == 1) &&
             EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, 16, tag) == 1 &&
             EVP_DecryptFinal_ex(c, dst[i] + l, &l) == 1;
    memcpy(dst[i] + P, tag, 16); /* session.rs:287-296: ct||tag in dst, opened in place */
    if (!ok) {
      memset(dst[i], 0, P); /* ring zeroes the plaintext on a tag mismatch */
      gw_set_err(r, WG_TUNN_ERR, WG_STATUS_INVALID_AEAD_TAG);
      continue;
    }
    e = wg_replay_mark_did_receive(&t->win, ctr);
    if (e) { gw_set_err(r, WG_TUNN_ERR, e); continue; }
    t->win.receive_cnt++;
    gw_validate(t, dst[i], P, r);
  }
  pthread_mutex_unlock(&t->mu);
  return 0;
}

/* multi-peer batches: packet i under its own Tunn's lock, one after another, as
 * NepTUN's worker does (packet_workers.rs:207-233) */
static int cpu_tunn_encapsulate_multi(uint32_t n, cpu_tunn *const *t, const uint8_t *const *src,
                                      const uint32_t *src_len, uint8_t *const *dst, const uint32_t *dst_cap,
                                      wg_tunn_result *res) {
  for (uint32_t i = 0; i < n; ++i)
    if (cpu_tunn_encapsulate_batch(t[i], 1, &src[i], &src_len[i], &dst[i], &dst_cap[i], &res[i])) return -1;
  return 0;
}

static int cpu_tunn_decapsulate_multi(uint32_t n, cpu_tunn *const *t, const uint8_t *const *dg,
                                      const uint32_t *len, uint8_t *const *dst, const uint32_t *dst_cap,
                                      wg_tunn_result *res) {
  for (uint32_t i = 0; i < n; ++i)
    if (cpu_tunn_decapsulate_batch(t[i], 1, &dg[i], &len[i], &dst[i], &dst_cap[i], &res[i])) return -1;
  return 0;
}

#endif /* GW_CPU_TUNN_H */
