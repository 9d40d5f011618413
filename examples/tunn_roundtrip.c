/*
 * tunn_roundtrip.c -- the C ABI used from plain C, the way NepTUN's Rust side
 * would bind it: two Tunn objects on one GPU context act as
 * the two ends of a WireGuard session; A encapsulates a batch of IPv4 packets
 * (Tunn::encapsulate, noise/mod.rs:295-338), B decapsulates the datagrams
 * (Tunn::decapsulate, mod.rs:346-380), then B sees the same batch again and
 * must reject every packet as a replay (session.rs:279): as a duplicate inside
 * the 1024-packet window, as an invalid counter behind it.
 *
 *   cc -O2 -I include examples/tunn_roundtrip.c -L neptun_amd -lneptun_gpu \
 *      -Wl,-rpath,$PWD/neptun_amd -o build/tunn_roundtrip && build/tunn_roundtrip 4096
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "neptun_gpu.h"
#include "neptun_tunn.h"

#define CHECK(call)                                                             \
  do {                                                                          \
    int rc_ = (call);                                                           \
    if (rc_) {                                                                  \
      fprintf(stderr, "%s failed: %d (%s)\n", #call, rc_, wg_gpu_last_error()); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

static uint64_t rng_state = 0x4E455054554EULL;
static uint8_t rnd8(void) {
  rng_state = rng_state * 6364136223846793005ULL + 1442695040888963407ULL;
  return (uint8_t)(rng_state >> 56);
}

int main(int argc, char **argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1024;
  const uint32_t cap = 1600;
  wg_gpu_ctx *ctx = NULL;
  wg_tunn *a = NULL, *b = NULL;
  CHECK(wg_gpu_ctx_create(0, 32, &ctx));
  CHECK(wg_tunn_create(ctx, 0, &a));
  CHECK(wg_tunn_create(ctx, 16, &b));
  uint8_t k1[32], k2[32];
  for (int i = 0; i < 32; ++i) {
    k1[i] = rnd8();
    k2[i] = rnd8();
  }
  /* A: local 21 sends to peer 34 with k1; B: local 34 receives with k1 */
  CHECK(wg_tunn_install_session(a, 21, 34, k2, k1, 1));
  CHECK(wg_tunn_install_session(b, 34, 21, k1, k2, 1));

  uint8_t *pkt = malloc((size_t)n * cap), *wire = malloc((size_t)n * cap), *back = malloc((size_t)n * cap);
  const uint8_t **src = malloc(n * sizeof *src), **dgram = malloc(n * sizeof *dgram);
  uint8_t **dst = malloc(n * sizeof *dst), **out = malloc(n * sizeof *out);
  uint32_t *len = malloc(n * 4), *wlen = malloc(n * 4), *caps = malloc(n * 4);
  wg_tunn_result *res = malloc(n * sizeof *res);
  for (uint32_t i = 0; i < n; ++i) {
    uint8_t *p = pkt + (size_t)i * cap;
    const uint32_t L = 20 + (uint32_t)(rnd8() | rnd8() << 8) % 1480;
    for (uint32_t j = 0; j < L; ++j) p[j] = rnd8();
    p[0] = 0x45;  /* IPv4, IHL 5 */
    p[2] = (uint8_t)(L >> 8);
    p[3] = (uint8_t)L;
    src[i] = p;
    len[i] = L;
    dst[i] = wire + (size_t)i * cap;
    out[i] = back + (size_t)i * cap;
    caps[i] = cap;
  }
  CHECK(wg_tunn_encapsulate_batch(a, n, src, len, dst, caps, res));
  for (uint32_t i = 0; i < n; ++i) {
    if (res[i].kind != WG_TUNN_WRITE_TO_NETWORK || res[i].len != len[i] + 32) {
      fprintf(stderr, "encap %u: kind %d status %d\n", i, res[i].kind, res[i].status);
      return 1;
    }
    dgram[i] = dst[i];
    wlen[i] = res[i].len;
  }
  CHECK(wg_tunn_decapsulate_batch(b, n, dgram, wlen, out, caps, res));
  for (uint32_t i = 0; i < n; ++i)
    if (res[i].kind != WG_TUNN_WRITE_TO_TUNNEL || res[i].len != len[i] ||
        memcmp(out[i], src[i], len[i]) != 0) {
      fprintf(stderr, "decap %u: kind %d status %d\n", i, res[i].kind, res[i].status);
      return 1;
    }
  /* the replay: counters more than 1024 behind the newest are out of the window
   * (InvalidCounter), the rest are already marked (DuplicateCounter), session.rs:90-104 */
  CHECK(wg_tunn_decapsulate_batch(b, n, dgram, wlen, out, caps, res));
  for (uint32_t i = 0; i < n; ++i)
    if (res[i].kind != WG_TUNN_ERR ||
        res[i].status != ((uint64_t)i + 1024 < n ? WG_STATUS_INVALID_COUNTER
                                                 : WG_STATUS_DUPLICATE_COUNTER)) {
      fprintf(stderr, "replay %u: kind %d status %d\n", i, res[i].kind, res[i].status);
      return 1;
    }
  uint64_t tx, rx;
  CHECK(wg_tunn_stats(a, &tx, NULL));
  CHECK(wg_tunn_stats(b, NULL, &rx));
  printf("ok: %u packets, tx_bytes %llu, rx_bytes %llu\n", n, (unsigned long long)tx,
         (unsigned long long)rx);
  CHECK(wg_tunn_destroy(a));
  CHECK(wg_tunn_destroy(b));
  CHECK(wg_gpu_ctx_destroy(ctx));
  return 0;
}
