/*
 * tunn_threads.c -- T threads, each encapsulating (and decapsulating) batches of B
 * packets on its own Tunn, no sockets: how the per-call time and its phases
 * (wg_tunn_get_phases) change as concurrent callers are added.
 *
 *   tunn_threads T B [calls] [P]   -> one JSON line per run
 * GW_PRIVATE_ENGINES=1: one engine per Tunn (else the context's default engine).
 * TT_REGISTER=1: every thread's buffers registered (wg_gpu_register_host): registered calls.
 * TT_HUGE=1: those buffers on transparent huge pages (one 2 MiB-aligned region).
 * The line also gives how many calls went out in a launch shared with another call
 * (wg_engine_info.combined: the engine's combiner, WG_COMBINE).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include "neptun_gpu.h"
#include "neptun_tunn.h"

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

typedef struct {
  wg_gpu_ctx *ctx;
  wg_tunn *a, *b;
  uint32_t B, calls, P;
  double t_enc, t_dec;
  int rc;
} job_t;

static void *run(void *arg) {
  job_t *j = arg;
  const uint32_t B = j->B, P = j->P, slot = (P + 64 + 127) & ~127u;
  uint8_t *src, *wire, *back;
  if (getenv("TT_HUGE") && atoi(getenv("TT_HUGE"))) {
    /* the three pools in one 2 MiB-aligned region on transparent huge pages (fewer IOMMU
       translations for the kernel's zero-copy reads and writes) */
    const size_t one = ((size_t)B * slot + 4095) & ~(size_t)4095, need = 3 * one;
    const size_t huge = (size_t)2 << 20, len = (need + huge - 1) & ~(huge - 1);
    uint8_t *m = mmap(NULL, len + huge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) {
      j->rc = 98;
      return NULL;
    }
    uint8_t *a = (uint8_t *)(((uintptr_t)m + huge - 1) & ~(uintptr_t)(huge - 1));
    madvise(a, len, MADV_HUGEPAGE);
    memset(a, 0, len);
    src = a, wire = a + one, back = a + 2 * one;
  } else {
    src = calloc((size_t)B, slot), wire = calloc((size_t)B, slot), back = calloc((size_t)B, slot);
  }
  const uint8_t **sp = calloc(B, sizeof *sp), **wp = calloc(B, sizeof *wp);
  uint8_t **wd = calloc(B, sizeof *wd), **bd = calloc(B, sizeof *bd);
  uint32_t *len = calloc(B, 4), *cap = calloc(B, 4), *wlen = calloc(B, 4);
  wg_tunn_result *res = calloc(B, sizeof *res);
  const int reg = getenv("TT_REGISTER") && atoi(getenv("TT_REGISTER"));
  if (reg && (wg_gpu_register_host(j->ctx, src, (uint64_t)B * slot) || wg_gpu_register_host(j->ctx, wire, (uint64_t)B * slot) ||
              wg_gpu_register_host(j->ctx, back, (uint64_t)B * slot))) {
    j->rc = 99;
    return NULL;
  }
  for (uint32_t i = 0; i < B; ++i) {
    uint8_t *p = src + (size_t)i * slot + 16;
    memset(p, (int)i, P);
    p[0] = 0x45;
    p[2] = (uint8_t)(P >> 8);
    p[3] = (uint8_t)P;
    sp[i] = p;
    len[i] = P;
    wd[i] = wire + (size_t)i * slot;
    wp[i] = wd[i];
    bd[i] = back + (size_t)i * slot + 16;
    cap[i] = slot - 16;
    wlen[i] = P + 32;
  }
  for (uint32_t c = 0; c < j->calls && !j->rc; ++c) {
    double t = now();
    j->rc = wg_tunn_encapsulate_batch(j->a, B, sp, len, wd, cap, res);
    j->t_enc += now() - t;
    if (j->rc) break;
    t = now();
    j->rc = wg_tunn_decapsulate_batch(j->b, B, wp, wlen, bd, cap, res);
    j->t_dec += now() - t;
    for (uint32_t i = 0; i < B && !j->rc; ++i)
      if (res[i].kind != WG_TUNN_WRITE_TO_TUNNEL) j->rc = 100 + res[i].status;
  }
  if (reg) {
    wg_gpu_unregister_host(j->ctx, src);
    wg_gpu_unregister_host(j->ctx, wire);
    wg_gpu_unregister_host(j->ctx, back);
  }
  if (!(getenv("TT_HUGE") && atoi(getenv("TT_HUGE")))) {  /* (the huge region is the process's until exit) */
    free(src); free(wire); free(back);
  }
  free(sp); free(wp); free(wd); free(bd); free(len); free(cap); free(wlen);
  free(res);
  return NULL;
}

int main(int argc, char **argv) {
  const uint32_t T = argc > 1 ? (uint32_t)atoi(argv[1]) : 1, B = argc > 2 ? (uint32_t)atoi(argv[2]) : 4096;
  const uint32_t calls = argc > 3 ? (uint32_t)atoi(argv[3]) : 64, P = argc > 4 ? (uint32_t)atoi(argv[4]) : 1350;
  wg_gpu_ctx *ctx = NULL;
  if (wg_gpu_ctx_create(0, 32 * T, &ctx)) {
    fprintf(stderr, "ctx: %s\n", wg_gpu_last_error());
    return 1;
  }
  job_t *jobs = calloc(T, sizeof *jobs);
  uint8_t k1[32], k2[32];
  for (int i = 0; i < 32; ++i) k1[i] = (uint8_t)(3 * i + 1), k2[i] = (uint8_t)(7 * i + 5);
  for (uint32_t t = 0; t < T; ++t) {
    job_t *j = &jobs[t];
    j->ctx = ctx;
    j->B = B, j->calls = calls, j->P = P;
    int rc;
#ifdef TT_ENGINES
    if (getenv("GW_PRIVATE_ENGINES")) {
      wg_engine *ea = NULL, *eb = NULL;
      rc = wg_engine_create(ctx, &ea) || wg_engine_create(ctx, &eb) || wg_tunn_create_on(ea, 32 * t, &j->a) ||
           wg_tunn_create_on(eb, 32 * t + 16, &j->b);
    } else
#endif
      rc = wg_tunn_create(ctx, 32 * t, &j->a) || wg_tunn_create(ctx, 32 * t + 16, &j->b);
    rc = rc || wg_tunn_install_session(j->a, 100 + 256 * t, 200 + 256 * t, k2, k1, 1) ||
         wg_tunn_install_session(j->b, 200 + 256 * t, 100 + 256 * t, k1, k2, 1);
    if (rc) {
      fprintf(stderr, "tunn: %s\n", wg_gpu_last_error());
      return 1;
    }
  }
  /* warm-up: two calls per thread, all threads at once (the engines' lanes and staging
   * are made on first use, one lane per concurrent call) */
  pthread_t *th = calloc(T, sizeof *th);
  for (uint32_t t = 0; t < T; ++t) {
    jobs[t].calls = 2;
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  for (uint32_t t = 0; t < T; ++t) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc) return 1;
    jobs[t].calls = calls;
    jobs[t].t_enc = jobs[t].t_dec = 0;
    wg_tunn_reset_phases(jobs[t].a);
    wg_tunn_reset_phases(jobs[t].b);
  }
  const double t0 = now();
  for (uint32_t t = 0; t < T; ++t) pthread_create(&th[t], NULL, run, &jobs[t]);
  for (uint32_t t = 0; t < T; ++t) pthread_join(th[t], NULL);
  const double secs = now() - t0;
  double te = 0, td = 0;
  wg_tunn_phases pa, pb, sa = {0}, sb = {0};
  for (uint32_t t = 0; t < T; ++t) {
    if (jobs[t].rc) {
      fprintf(stderr, "thread %u failed: %d %s\n", t, jobs[t].rc, wg_gpu_last_error());
      return 1;
    }
    te += jobs[t].t_enc, td += jobs[t].t_dec;
    wg_tunn_get_phases(jobs[t].a, &pa);
    wg_tunn_get_phases(jobs[t].b, &pb);
#define ADD(f) sa.f += pa.f, sb.f += pb.f;
    ADD(calls) ADD(total_us) ADD(checks_us) ADD(pack_us) ADD(submit_us) ADD(wait_us) ADD(decide_us)
    ADD(copy_out_us) ADD(prep_us)
  }
  const double calls_all = (double)T * calls;
  uint32_t combined = 0;
  unsigned long long served = 0, srv_launches = 0;
#ifdef TT_ENGINES
  {
    wg_engine_info info;
    if (!getenv("GW_PRIVATE_ENGINES") && wg_engine_get_info(wg_tunn_engine(jobs[0].a), &info) == 0) {
      combined = info.combined;
      served = info.served;
      srv_launches = info.service_launches;
    }
  }
#endif
  printf("{\"threads\": %u, \"batch\": %u, \"P\": %u, \"calls_per_thread\": %u, \"registered\": %d, "
         "\"combined_calls\": %u, \"served_calls\": %llu, \"service_launches\": %llu, \"seconds\": %.4f, "
         "\"roundtrip_gbps\": %.2f, \"encap_ms_per_call\": %.3f, \"decap_ms_per_call\": %.3f, "
         "\"encap_us\": {\"checks\": %.1f, \"pack\": %.1f, \"submit\": %.1f, \"wait\": %.1f, \"copy_out\": %.1f}, "
         "\"decap_us\": {\"checks\": %.1f, \"pack\": %.1f, \"submit\": %.1f, \"wait\": %.1f, \"decide\": %.1f, "
         "\"copy_out\": %.1f}}\n",
         T, B, P, calls, getenv("TT_REGISTER") && atoi(getenv("TT_REGISTER")), combined, served, srv_launches, secs, calls_all * B * P * 8.0 / secs / 1e9, te / calls_all * 1e3, td / calls_all * 1e3,
         sa.checks_us / calls_all, sa.pack_us / calls_all, sa.submit_us / calls_all, sa.wait_us / calls_all,
         sa.copy_out_us / calls_all, sb.checks_us / calls_all, sb.pack_us / calls_all, sb.submit_us / calls_all,
         sb.wait_us / calls_all, sb.decide_us / calls_all, sb.copy_out_us / calls_all);
  return 0;
}
