/*
 * cpu_baseline.c -- CPU baseline for BASELINE.json config 1 ("CPU
 * encapsulate+decapsulate round-trip, 64k x 1350-byte packets, single session
 * key").  TEST/BENCH INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg runs it.
 *
 * The reference (Rust + ring 0.17.14) cannot be built here (no cargo, no
 * network).  This harness reproduces the NepTUN data path per packet:
 *   seal: Session::format_packet_data  (session.rs:205-259)
 *   open: parse_incoming_packet (noise/mod.rs:139-199) + receive_packet_data
 *         (session.rs:265-302) incl. the ct->dst copy at :287-289
 * with the AEAD from either OpenSSL 3 EVP (--impl openssl, SIMD asm; the
 * closest stand-in for ring's asm) or the scalar restatement in
 * neptun_oracle.c (--impl oracle).  One session per thread, one thread per
 * core, mirroring packet_workers.rs:113-131 (num_cpus::get_physical()).
 *
 * Gbit/s = N * P * 8 / (t_seal + t_open), wall clock, median over reps.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "neptun_oracle.h"

int ossl_format_packet_data(const uint8_t key[32], uint32_t sending_index, uint64_t counter,
                            const uint8_t *payload, int len, uint8_t *out);
int ossl_receive_packet_data(const uint8_t key[32], const uint8_t *datagram, int len, uint8_t *out);

static int g_use_openssl = 1;
static size_t g_pkt = 1350;

typedef struct {
  uint8_t key[32];
  uint8_t *pt, *wire, *out;
  size_t n;
  int bad, cpu, reps;
  uint64_t seed;
  pthread_barrier_t *bar;
  double t_seal, t_open;
} job_t;

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* The worker's own packets, allocated and written by the worker itself (after it
 * pinned itself), so its buffers are local to its core's memory node. */
static void job_init(job_t *j) {
  const size_t P = g_pkt, W = P + 32;
  uint64_t kseed = 0x4E455054554Full; /* "NEPTUN" + 1 */
  for (int k = 0; k < 32; k += 8) { uint64_t v = splitmix64(&kseed); memcpy(j->key + k, &v, 8); }
  j->pt = malloc(j->n * P);
  j->wire = malloc(j->n * W);
  j->out = malloc(j->n * (P + 16));
  uint64_t seed = j->seed;
  for (size_t i = 0; i < j->n * P; i += 8) {
    uint64_t v = splitmix64(&seed);
    memcpy(j->pt + i, &v, (j->n * P - i) < 8 ? (j->n * P - i) : 8);
  }
  memset(j->wire, 0, j->n * W);
  memset(j->out, 0, j->n * (P + 16));
  /* valid IPv4 header (ver 4, IHL 5, total_length = P, proto 17) so that
   * validate_decapsulated_packet keeps all P bytes (noise/mod.rs:613-634) */
  for (size_t i = 0; i < j->n && P >= 20; ++i) {
    uint8_t *h = j->pt + i * P;
    h[0] = 0x45; h[1] = 0; h[2] = (uint8_t)(P >> 8); h[3] = (uint8_t)P; h[9] = 17;
    h[12] = 10; h[13] = 0; h[14] = 0; h[15] = 1; h[16] = 10; h[17] = 0; h[18] = 0; h[19] = 2;
  }
}

static void run_once(job_t *j) {
  const size_t P = g_pkt, W = P + 32;
  double t0 = now();
  for (size_t i = 0; i < j->n; ++i) {
    if (g_use_openssl)
      ossl_format_packet_data(j->key, 0x00ABCD01u, i, j->pt + i * P, (int)P, j->wire + i * W);
    else
      neptun_oracle_format_packet_data(j->key, 0x00ABCD01u, i, j->pt + i * P, P, j->wire + i * W, W);
  }
  double t1 = now();
  for (size_t i = 0; i < j->n; ++i) {
    const uint8_t *d = j->wire + i * W;
    uint32_t ridx; uint64_t ctr;
    if (neptun_oracle_parse_data_header(d, W, &ridx, &ctr)) { j->bad++; continue; }
    int rc;
    if (g_use_openssl) {
      /* session.rs:287-289 copies ct||tag into dst, then opens in place */
      rc = ossl_receive_packet_data(j->key, d, (int)W, j->out + i * P);
    } else {
      size_t ol;
      rc = neptun_oracle_receive_packet_data(j->key, ridx, d, W, j->out + i * (P + 16), P + 16, &ol);
    }
    if (rc) j->bad++;
  }
  double t2 = now();
  if (t1 - t0 < j->t_seal) j->t_seal = t1 - t0;
  if (t2 - t1 < j->t_open) j->t_open = t2 - t1;
}

/* One thread per worker for all reps: pin (optional), build its packets, then per
 * rep wait for the start barrier, run, and meet the main thread at the end barrier. */
static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  if (j->cpu >= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(j->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
  }
  job_init(j);
  j->t_seal = j->t_open = 1e30;
  for (int r = 0; r < j->reps; ++r) {
    pthread_barrier_wait(j->bar);
    run_once(j);
    pthread_barrier_wait(j->bar);
  }
  return NULL;
}

/* --pin: one CPU per physical core, in the order of the process's affinity mask
 * (the first SMT sibling of each core the mask allows). */
static int physical_cpus(int *out, int max) {
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set)) return 0;
  int k = 0;
  for (int c = 0; c < CPU_SETSIZE && k < max; ++c) {
    if (!CPU_ISSET(c, &set)) continue;
    char path[128];
    snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", c);
    FILE *f = fopen(path, "r");
    int first = c;
    if (f) {
      if (fscanf(f, "%d", &first) != 1) first = c;
      fclose(f);
    }
    if (first == c) out[k++] = c;
  }
  return k;
}

static int cmpd(const void *a, const void *b) {
  double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
  size_t n = 65536, per_thread = 0;
  int threads = 1, reps = 5, pin = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--packets") && i + 1 < argc) n = strtoull(argv[++i], 0, 10);
    else if (!strcmp(argv[i], "--packets-per-thread") && i + 1 < argc) per_thread = strtoull(argv[++i], 0, 10);
    else if (!strcmp(argv[i], "--threads") && i + 1 < argc) threads = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--reps") && i + 1 < argc) reps = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--size") && i + 1 < argc) g_pkt = strtoull(argv[++i], 0, 10);
    else if (!strcmp(argv[i], "--impl") && i + 1 < argc) g_use_openssl = !strcmp(argv[++i], "openssl");
    else if (!strcmp(argv[i], "--pin")) pin = 1;
    else { fprintf(stderr, "usage: %s [--packets N | --packets-per-thread N] [--threads T] [--reps R] [--size P] [--impl openssl|oracle] [--pin]\n", argv[0]); return 2; }
  }
  if (threads < 1 || reps < 1) return 2;
  if (per_thread) n = per_thread * (size_t)threads;
  const size_t P = g_pkt;
  int *cpus = calloc(threads, sizeof(int));
  int ncpu = pin ? physical_cpus(cpus, threads) : 0;
  if (pin && ncpu < threads) {
    fprintf(stderr, "--pin: only %d physical cores in the affinity mask for %d threads\n", ncpu, threads);
    return 2;
  }
  job_t *jobs = calloc(threads, sizeof(job_t));
  pthread_t *th = calloc(threads, sizeof(pthread_t));
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, threads + 1);
  uint64_t seed = 0x4E455054554Eull; /* "NEPTUN" */
  size_t per = n / threads;
  for (int t = 0; t < threads; ++t) {
    job_t *j = &jobs[t];
    j->n = per + (t < (int)(n % threads) ? 1 : 0);
    j->cpu = pin ? cpus[t] : -1;
    j->reps = reps;
    j->seed = seed + 0x1000003ull * (uint64_t)t;
    j->bar = &bar;
    pthread_create(&th[t], NULL, worker, j);
  }
  double *walls = calloc(reps, sizeof(double));
  for (int r = 0; r < reps; ++r) {
    pthread_barrier_wait(&bar); /* every worker built its packets / finished the last rep */
    double t0 = now();
    pthread_barrier_wait(&bar);
    walls[r] = now() - t0;
    if (getenv("CPU_BASELINE_DEBUG")) fprintf(stderr, "rep %d wall %.4f\n", r, walls[r]);
  }
  int bad = 0;
  double ms = 0, mo = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    bad += jobs[t].bad;
    if (jobs[t].t_seal > ms) ms = jobs[t].t_seal;
    if (jobs[t].t_open > mo) mo = jobs[t].t_open;
  }
  pthread_barrier_destroy(&bar);
  qsort(walls, reps, sizeof(double), cmpd);
  double med = walls[reps / 2];
  double gbps = (double)n * P * 8 / med / 1e9;
  printf("{\"impl\": \"%s\", \"threads\": %d, \"pinned\": %s, \"packets\": %zu, \"size\": %zu, \"reps\": %d, "
         "\"median_s\": %.6f, \"gbps\": %.4f, \"pkts_per_s\": %.1f, \"seal_gbps_best\": %.4f, "
         "\"open_gbps_best\": %.4f, \"tag_failures\": %d}\n",
         g_use_openssl ? "openssl" : "oracle", threads, pin ? "true" : "false", n, P, reps, med, gbps,
         n / med, (double)n * P * 8 / ms / 1e9, (double)n * P * 8 / mo / 1e9, bad);
  return bad ? 1 : 0;
}
