/*
 * cpu_x25519.c -- CPU baseline for the handshake kernels (test/bench
 * infrastructure, not the product): X25519 operations per second through
 * OpenSSL 3 (the reference uses x25519-dalek, which cannot be built here),
 * one thread per core, each thread running --ops DH computations.
 *   cpu_x25519 [--threads T] [--ops N]   -> one JSON line
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

int ossl_x25519_fast(uint8_t out[32], const uint8_t scalar[32], const uint8_t point[32]);

typedef struct {
  size_t ops;
  uint64_t seed;
  int bad;
} job_t;

static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static void *worker(void *arg) {
  job_t *j = arg;
  uint8_t k[32], u[32], out[32];
  for (int i = 0; i < 32; i += 8) {
    uint64_t v = splitmix64(&j->seed);
    memcpy(k + i, &v, 8);
    v = splitmix64(&j->seed);
    memcpy(u + i, &v, 8);
  }
  for (size_t i = 0; i < j->ops; ++i) {
    if (ossl_x25519_fast(out, k, u)) j->bad++;
    memcpy(u, out, 32);  /* chain: each result is the next point */
  }
  return NULL;
}

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
  int threads = 1;
  size_t ops = 2000;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--threads") && i + 1 < argc) threads = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--ops") && i + 1 < argc) ops = strtoull(argv[++i], 0, 10);
    else { fprintf(stderr, "usage: %s [--threads T] [--ops N]\n", argv[0]); return 2; }
  }
  job_t *jobs = calloc(threads, sizeof(job_t));
  pthread_t *th = calloc(threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t) {
    jobs[t].ops = ops;
    jobs[t].seed = 0x4E455054554Eull + t;
  }
  const double t0 = now();
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &jobs[t]);
  int bad = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    bad += jobs[t].bad;
  }
  const double dt = now() - t0;
  printf("{\"threads\": %d, \"ops\": %zu, \"seconds\": %.4f, \"ops_per_s\": %.1f, \"failed\": %d}\n",
         threads, ops * threads, dt, ops * threads / dt, bad);
  return bad ? 1 : 0;
}
