/*
 * udp_gateway.c -- the batched Tunn behind real UDP sockets, shaped like
 * NepTUN's PacketWorkers (neptun/src/device/packet_workers.rs:99-287):
 *
 *   encrypt worker   (write_to_socket_worker, packet_workers.rs:207-242):
 *       takes a batch of up to B IP packets (read_iface_batch :178-205 reads
 *       them from TUN; here from the input file), Tunn::encapsulate on the GPU
 *       (wg_tunn_encapsulate_batch), one sendmmsg() for the whole batch;
 *   socket reader    (the conn-socket handler, device/mod.rs:1115-1218):
 *       recvmmsg() batches of datagrams off the peer's UDP socket;
 *   decrypt worker   (the handler's Tunn::decapsulate + write_to_tun_worker
 *       :244-287): wg_tunn_decapsulate_batch over everything received so far
 *       (up to B per call), results appended to the output ("the TUN").
 *
 * B is the max_inter_thread_batched_pkts knob (DeviceConfig, device/mod.rs:
 * 162-163; the reference default is 50, packet_workers.rs:27).  Both ends run
 * in this process on 127.0.0.1 with their own Tunn (A sends with key k1 to
 * index b_idx, B receives), on one GPU context.  UDP on loopback drops when
 * the receive buffer overflows, so the sender keeps at most W datagrams in
 * flight (W from the socket's effective SO_RCVBUF).
 *
 *   udp_gateway IN OUT [B]   -> one JSON line on stdout
 * IN : "NGW1" | u32 n | u32 a_idx | u32 b_idx | k1[32] | k2[32] | n x (u32 len | bytes)
 * OUT: "NGWO" | u32 sent | sent x (u32 len | datagram)
 *             | u32 recv | recv x (u32 len | datagram | wg_tunn_result | u32 dst_len | dst bytes)
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "neptun_gpu.h"
#include "neptun_tunn.h"

#define MAX_DGRAM 65536

typedef struct {
  uint32_t n, a_idx, b_idx;
  uint8_t k1[32], k2[32];
  uint8_t **pkt;
  uint32_t *len;
} input_t;

typedef struct {
  input_t *in;
  wg_tunn *a, *b;
  int sa, sb;
  uint32_t batch, window;
  /* sender output */
  uint8_t **sent;
  uint32_t *sent_len;
  _Atomic uint32_t n_sent;
  /* socket reader output (the received datagrams, in arrival order) */
  uint8_t **rx;
  uint32_t *rx_len;
  _Atomic uint32_t n_rx;
  _Atomic int rx_done;
  /* decrypt worker output */
  uint8_t **dst;
  uint32_t *dst_cap;
  wg_tunn_result *res;
  _Atomic uint32_t n_dec;
  _Atomic int failed;
  double t_end;
} gw_t;

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int read_all(FILE *f, void *p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

static int load_input(const char *path, input_t *in) {
  FILE *f = fopen(path, "rb");
  if (!f) return -1;
  char magic[4];
  if (read_all(f, magic, 4) || memcmp(magic, "NGW1", 4) || read_all(f, &in->n, 4) ||
      read_all(f, &in->a_idx, 4) || read_all(f, &in->b_idx, 4) || read_all(f, in->k1, 32) ||
      read_all(f, in->k2, 32)) {
    fclose(f);
    return -1;
  }
  in->pkt = calloc(in->n, sizeof *in->pkt);
  in->len = calloc(in->n, sizeof *in->len);
  for (uint32_t i = 0; i < in->n; ++i) {
    if (read_all(f, &in->len[i], 4) || in->len[i] > MAX_DGRAM - 64) { fclose(f); return -1; }
    in->pkt[i] = malloc(in->len[i] + 1);
    if (read_all(f, in->pkt[i], in->len[i])) { fclose(f); return -1; }
  }
  fclose(f);
  return 0;
}

/* encrypt worker: batch -> GPU encapsulate -> sendmmsg */
static void *sender(void *arg) {
  gw_t *g = arg;
  const uint32_t n = g->in->n, B = g->batch;
  wg_tunn_result *res = calloc(B, sizeof *res);
  uint32_t *cap = calloc(B, sizeof *cap);
  struct mmsghdr *msgs = calloc(B, sizeof *msgs);
  struct iovec *iov = calloc(B, sizeof *iov);
  for (uint32_t i0 = 0; i0 < n && !atomic_load(&g->failed); i0 += B) {
    const uint32_t m = n - i0 < B ? n - i0 : B;
    for (uint32_t j = 0; j < m; ++j) {
      g->sent[i0 + j] = malloc(g->in->len[i0 + j] + 32);
      cap[j] = g->in->len[i0 + j] + 32;
    }
    if (wg_tunn_encapsulate_batch(g->a, m, (const uint8_t *const *)&g->in->pkt[i0], &g->in->len[i0],
                                  &g->sent[i0], cap, res)) {
      fprintf(stderr, "encapsulate_batch: %s\n", wg_gpu_last_error());
      atomic_store(&g->failed, 1);
      break;
    }
    uint32_t k = 0;
    for (uint32_t j = 0; j < m; ++j) {
      g->sent_len[i0 + j] = res[j].kind == WG_TUNN_WRITE_TO_NETWORK ? res[j].len : 0;
      if (!g->sent_len[i0 + j]) continue;  /* (not with a live session) */
      iov[k].iov_base = g->sent[i0 + j];
      iov[k].iov_len = g->sent_len[i0 + j];
      memset(&msgs[k], 0, sizeof msgs[k]);
      msgs[k].msg_hdr.msg_iov = &iov[k];
      msgs[k].msg_hdr.msg_iovlen = 1;
      ++k;
    }
    /* flow control: at most `window` datagrams in the receiver's socket queue */
    uint32_t done = 0;
    while (done < k) {
      const uint32_t inflight = atomic_load(&g->n_sent) - atomic_load(&g->n_rx);
      if (inflight >= g->window) {
        sched_yield();
        continue;
      }
      uint32_t can = g->window - inflight;
      if (can > k - done) can = k - done;
      const int r = sendmmsg(g->sa, &msgs[done], can, 0);
      if (r < 0) {
        perror("sendmmsg");
        atomic_store(&g->failed, 1);
        break;
      }
      done += (uint32_t)r;
      atomic_fetch_add(&g->n_sent, (uint32_t)r);
    }
  }
  free(res); free(cap); free(msgs); free(iov);
  return NULL;
}

/* socket reader: recvmmsg into the arrival-ordered store */
static void *reader(void *arg) {
  gw_t *g = arg;
  const uint32_t n = g->in->n, B = g->batch;
  struct mmsghdr *msgs = calloc(B, sizeof *msgs);
  struct iovec *iov = calloc(B, sizeof *iov);
  double idle_since = now();
  while (atomic_load(&g->n_rx) < n && !atomic_load(&g->failed)) {
    const uint32_t base = atomic_load(&g->n_rx);
    const uint32_t m = n - base < B ? n - base : B;
    for (uint32_t j = 0; j < m; ++j) {
      if (!g->rx[base + j]) g->rx[base + j] = malloc(MAX_DGRAM);
      iov[j].iov_base = g->rx[base + j];
      iov[j].iov_len = MAX_DGRAM;
      memset(&msgs[j], 0, sizeof msgs[j]);
      msgs[j].msg_hdr.msg_iov = &iov[j];
      msgs[j].msg_hdr.msg_iovlen = 1;
    }
    struct timespec to = {0, 50 * 1000 * 1000};
    const int r = recvmmsg(g->sb, msgs, m, MSG_WAITFORONE, &to);
    if (r <= 0) {
      /* every datagram that was sent has arrived or is lost: stop after 2 s idle */
      if (now() - idle_since > 2.0) break;
      continue;
    }
    idle_since = now();
    for (int j = 0; j < r; ++j) g->rx_len[base + j] = msgs[j].msg_len;
    atomic_fetch_add(&g->n_rx, (uint32_t)r);
  }
  atomic_store(&g->rx_done, 1);
  free(msgs); free(iov);
  return NULL;
}

/* decrypt worker: everything received so far, up to B per call, in arrival order */
static void *decryptor(void *arg) {
  gw_t *g = arg;
  for (;;) {
    const uint32_t d = atomic_load(&g->n_dec);
    const int finished = atomic_load(&g->rx_done);
    const uint32_t avail = atomic_load(&g->n_rx);
    if (d == avail) {
      if (finished || atomic_load(&g->failed)) break;
      sched_yield();
      continue;
    }
    const uint32_t m = avail - d < g->batch ? avail - d : g->batch;
    for (uint32_t j = 0; j < m; ++j) {
      const uint32_t L = g->rx_len[d + j];
      g->dst_cap[d + j] = L > 16 ? L - 16 : 0;
      g->dst[d + j] = malloc(g->dst_cap[d + j] + 1);
    }
    if (wg_tunn_decapsulate_batch(g->b, m, (const uint8_t *const *)&g->rx[d], &g->rx_len[d],
                                  &g->dst[d], &g->dst_cap[d], &g->res[d])) {
      fprintf(stderr, "decapsulate_batch: %s\n", wg_gpu_last_error());
      atomic_store(&g->failed, 1);
      break;
    }
    atomic_store(&g->n_dec, d + m);
    g->t_end = now();
  }
  return NULL;
}

static int udp_socket(struct sockaddr_in *addr) {
  const int s = socket(AF_INET, SOCK_DGRAM, 0);
  if (s < 0) return -1;
  const int big = 64 << 20;
  (void)setsockopt(s, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);  /* capped at rmem_max */
  (void)setsockopt(s, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
  memset(addr, 0, sizeof *addr);
  addr->sin_family = AF_INET;
  addr->sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  socklen_t al = sizeof *addr;
  if (bind(s, (struct sockaddr *)addr, sizeof *addr) || getsockname(s, (struct sockaddr *)addr, &al)) {
    close(s);
    return -1;
  }
  return s;
}

#define CHECK(call)                                                             \
  do {                                                                          \
    int rc_ = (call);                                                           \
    if (rc_) {                                                                  \
      fprintf(stderr, "%s failed: %d (%s)\n", #call, rc_, wg_gpu_last_error()); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main(int argc, char **argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s IN OUT [batch]\n", argv[0]);
    return 2;
  }
  input_t in;
  if (load_input(argv[1], &in)) {
    fprintf(stderr, "bad input %s\n", argv[1]);
    return 2;
  }
  gw_t g;
  memset(&g, 0, sizeof g);
  g.in = &in;
  g.batch = argc > 3 ? (uint32_t)atoi(argv[3]) : 512;
  if (g.batch == 0) g.batch = 1;
  wg_gpu_ctx *ctx = NULL;
  CHECK(wg_gpu_ctx_create(0, 32, &ctx));
  CHECK(wg_tunn_create(ctx, 0, &g.a));
  CHECK(wg_tunn_create(ctx, 16, &g.b));
  /* A sends with k1 to b_idx and receives with k2; B the mirror image */
  CHECK(wg_tunn_install_session(g.a, in.a_idx, in.b_idx, in.k2, in.k1, 1));
  CHECK(wg_tunn_install_session(g.b, in.b_idx, in.a_idx, in.k1, in.k2, 1));
  struct sockaddr_in aa, ab;
  g.sa = udp_socket(&aa);
  g.sb = udp_socket(&ab);
  if (g.sa < 0 || g.sb < 0 || connect(g.sa, (struct sockaddr *)&ab, sizeof ab)) {
    perror("socket");
    return 1;
  }
  int rcvbuf = 0;
  socklen_t ol = sizeof rcvbuf;
  (void)getsockopt(g.sb, SOL_SOCKET, SO_RCVBUF, &rcvbuf, &ol);
  /* loopback charges each datagram its skb truesize (~2-4 KiB for <= 1500 B) */
  g.window = rcvbuf / 4096 > 16 ? (uint32_t)(rcvbuf / 4096) : 16;
  const uint32_t n = in.n;
  g.sent = calloc(n, sizeof *g.sent);
  g.sent_len = calloc(n, sizeof *g.sent_len);
  g.rx = calloc(n, sizeof *g.rx);
  g.rx_len = calloc(n, sizeof *g.rx_len);
  g.dst = calloc(n, sizeof *g.dst);
  g.dst_cap = calloc(n, sizeof *g.dst_cap);
  g.res = calloc(n, sizeof *g.res);

  const double t0 = now();
  pthread_t ts, tr, td;
  pthread_create(&tr, NULL, reader, &g);
  pthread_create(&td, NULL, decryptor, &g);
  pthread_create(&ts, NULL, sender, &g);
  pthread_join(ts, NULL);
  pthread_join(tr, NULL);
  pthread_join(td, NULL);
  if (atomic_load(&g.failed)) return 1;

  const uint32_t nrx = atomic_load(&g.n_rx), nsent = atomic_load(&g.n_sent);
  uint64_t bytes = 0;
  for (uint32_t i = 0; i < nrx; ++i)
    if (g.res[i].kind == WG_TUNN_WRITE_TO_TUNNEL) bytes += g.res[i].len;
  const double secs = g.t_end > t0 ? g.t_end - t0 : 1e-9;

  FILE *f = fopen(argv[2], "wb");
  if (!f) return 1;
  fwrite("NGWO", 1, 4, f);
  fwrite(&n, 4, 1, f);
  for (uint32_t i = 0; i < n; ++i) {
    fwrite(&g.sent_len[i], 4, 1, f);
    fwrite(g.sent[i], 1, g.sent_len[i], f);
  }
  fwrite(&nrx, 4, 1, f);
  for (uint32_t i = 0; i < nrx; ++i) {
    fwrite(&g.rx_len[i], 4, 1, f);
    fwrite(g.rx[i], 1, g.rx_len[i], f);
    fwrite(&g.res[i], sizeof g.res[i], 1, f);
    fwrite(&g.dst_cap[i], 4, 1, f);
    fwrite(g.dst[i], 1, g.dst_cap[i], f);
  }
  fclose(f);
  printf("{\"packets\": %u, \"sent\": %u, \"received\": %u, \"lost\": %u, \"batch\": %u, "
         "\"window\": %u, \"rcvbuf\": %d, \"seconds\": %.6f, \"ip_bytes\": %llu, "
         "\"socket_to_socket_gbps\": %.3f}\n",
         n, nsent, nrx, nsent - nrx, g.batch, g.window, rcvbuf, secs, (unsigned long long)bytes,
         bytes * 8.0 / secs / 1e9);
  wg_tunn_destroy(g.a);
  wg_tunn_destroy(g.b);
  wg_gpu_ctx_destroy(ctx);
  return 0;
}
