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
 *   udp_gateway IN OUT [B] [PAIRS] [reg] [mux[=W]]   -> one JSON line on stdout
 * PAIRS > 1 runs that many independent peers side by side (own Tunns, sockets
 * and threads, one GPU context), the way NepTUN serves peers on its n_threads
 * event loops.  "reg": the packet pools (the TUN read buffers the plaintexts land
 * in, the datagram buffers, the decrypted-packet buffers) are one slab registered
 * with wg_gpu_register_host, as INTEGRATION.md advises -- the batches then take the
 * library's DMA path instead of host copies through pinned staging.
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

/* -DGW_CPU: the same gateway with OpenSSL on the CPU in place of the GPU Tunn
 * (gw_cpu_tunn.h) -- the same-box CPU line beside the GPU one */
#ifdef GW_CPU
#include "gw_cpu_tunn.h"
typedef cpu_tunn gw_tunn;
#define GW_BACKEND "cpu"
#define gw_encapsulate_batch cpu_tunn_encapsulate_batch
#define gw_decapsulate_batch cpu_tunn_decapsulate_batch
#define gw_install_session cpu_tunn_install_session
#define gw_destroy cpu_tunn_destroy
#define gw_encapsulate_multi(e, ...) cpu_tunn_encapsulate_multi(__VA_ARGS__)
#define gw_decapsulate_multi(e, ...) cpu_tunn_decapsulate_multi(__VA_ARGS__)
typedef void gw_engine;
#define gw_engine_of(t) NULL
#else
typedef wg_tunn gw_tunn;
#define GW_BACKEND "gpu"
#define gw_encapsulate_batch wg_tunn_encapsulate_batch
#define gw_decapsulate_batch wg_tunn_decapsulate_batch
#define gw_install_session wg_tunn_install_session
#define gw_destroy wg_tunn_destroy
#define gw_encapsulate_multi wg_tunn_encapsulate_multi
#define gw_decapsulate_multi wg_tunn_decapsulate_multi
typedef wg_engine gw_engine;
#define gw_engine_of(t) wg_tunn_engine(t)
#endif

#define MAX_DGRAM 65536

typedef struct {
  uint32_t n, a_idx, b_idx;
  uint8_t k1[32], k2[32];
  uint8_t **pkt;
  uint32_t *len;
} input_t;

typedef struct {
  input_t *in;
  uint32_t i0, i1;  /* this pair's share of the input packets */
  gw_tunn *a, *b;
  int sa, sb;
  uint32_t batch, window, slot;  /* slot: bytes per preallocated packet buffer */
  /* sender output */
  uint8_t **sent;
  uint32_t *sent_len;
  _Atomic uint32_t n_sent;
  /* socket reader output (the received datagrams, in arrival order) */
  uint8_t **rx;
  uint32_t *rx_len;
  _Atomic uint32_t n_rx;
  _Atomic int rx_done;
  _Atomic int send_done;       /* the sender has sent (or given up on) all its datagrams */
  _Atomic uint32_t n_written_off; /* datagrams the sender's flow control counts as lost */
  _Atomic int rx_idle;         /* the reader's last recvmmsg timed out with nothing */
  /* decrypt worker output */
  uint8_t **dst;
  uint32_t *dst_cap;
  wg_tunn_result *res;
  _Atomic uint32_t n_dec;
  _Atomic int failed;
  double t_end;
  /* where the time goes (seconds, per thread) */
  double t_encap, t_send, t_wait, t_recv, t_decap;
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

/* send k prepared datagrams of pair g, keeping its window: 0, or -1 when the run stops */
static int send_window(gw_t *g, struct mmsghdr *msgs, uint32_t k) {
  /* flow control: at most `window` datagrams in the receiver's socket queue.
     Lost datagrams never arrive, so a window that has not moved for 1 s is
     written off (counted as lost) instead of waited for forever; the reader
     ending (rx_done) or a failure stops the sender. */
  double t;
  uint32_t done = 0;
  double stall_since = -1.0;
  uint32_t stall_rx = 0;
  while (done < k) {
    if (atomic_load(&g->rx_done) || atomic_load(&g->failed)) return -1;
    const uint32_t rx = atomic_load(&g->n_rx);
    /* signed: datagrams written off as lost that arrive late after all would
       otherwise underflow the in-flight count */
    const int64_t inflight64 = (int64_t)atomic_load(&g->n_sent) - rx - atomic_load(&g->n_written_off);
    const uint32_t inflight = inflight64 > 0 ? (uint32_t)inflight64 : 0u;
    if (inflight >= g->window) {
      t = now();
      if (stall_since < 0 || rx != stall_rx) {
        stall_since = t;
        stall_rx = rx;
      } else if (t - stall_since > 5.0 && atomic_load(&g->rx_idle)) {
        /* only once the reader has sat idle in recvmmsg (not while it is busy
           decrypting a slow batch) and the window has not moved for 5 s */
        atomic_fetch_add(&g->n_written_off, inflight);
        stall_since = -1.0;
      }
      sched_yield();
      g->t_wait += now() - t;
      continue;
    }
    stall_since = -1.0;
    uint32_t can = g->window - inflight;
    if (can > k - done) can = k - done;
    t = now();
    const int r = sendmmsg(g->sa, &msgs[done], can, 0);
    g->t_send += now() - t;
    if (r < 0) {
      perror("sendmmsg");
      atomic_store(&g->failed, 1);
      return -1;
    }
    done += (uint32_t)r;
    atomic_fetch_add(&g->n_sent, (uint32_t)r);
  }
  return 0;
}

/* encrypt worker: batch -> GPU encapsulate -> sendmmsg */
static void *sender(void *arg) {
  gw_t *g = arg;
  const uint32_t n = g->i1, B = g->batch;
  wg_tunn_result *res = calloc(B, sizeof *res);
  uint32_t *cap = calloc(B, sizeof *cap);
  struct mmsghdr *msgs = calloc(B, sizeof *msgs);
  struct iovec *iov = calloc(B, sizeof *iov);
  for (uint32_t i0 = g->i0; i0 < n && !atomic_load(&g->failed) && !atomic_load(&g->rx_done); i0 += B) {
    const uint32_t m = n - i0 < B ? n - i0 : B;
    for (uint32_t j = 0; j < m; ++j) cap[j] = g->slot;
    double t = now();
    const int erc = gw_encapsulate_batch(g->a, m, (const uint8_t *const *)&g->in->pkt[i0],
                                              &g->in->len[i0], &g->sent[i0], cap, res);
    g->t_encap += now() - t;
    if (erc) {
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
    if (send_window(g, msgs, k)) break;
  }
  atomic_store(&g->send_done, 1);
  free(res); free(cap); free(msgs); free(iov);
  return NULL;
}

/* socket reader: recvmmsg into the arrival-ordered store */
static void *reader(void *arg) {
  gw_t *g = arg;
  const uint32_t n = g->i1 - g->i0, B = g->batch;
  struct mmsghdr *msgs = calloc(B, sizeof *msgs);
  struct iovec *iov = calloc(B, sizeof *iov);
  /* idle clock: from the first datagram on (a slow first GPU batch is not
     idleness), and only once the sender is done may 2 s of silence end the run */
  double idle_since = -1.0;
  const double t_start = now();
  while (atomic_load(&g->n_rx) < n && !atomic_load(&g->failed)) {
    const uint32_t base = atomic_load(&g->n_rx);
    const uint32_t m = n - base < B ? n - base : B;
    for (uint32_t j = 0; j < m; ++j) {
      iov[j].iov_base = g->rx[base + j];
      iov[j].iov_len = g->slot;
      memset(&msgs[j], 0, sizeof msgs[j]);
      msgs[j].msg_hdr.msg_iov = &iov[j];
      msgs[j].msg_hdr.msg_iovlen = 1;
    }
    struct timespec to = {0, 50 * 1000 * 1000};
    const double t = now();
    const int r = recvmmsg(g->sb, msgs, m, MSG_WAITFORONE, &to);
    g->t_recv += now() - t;
    atomic_store(&g->rx_idle, r <= 0);
    if (r <= 0) {
      /* every datagram that was sent has arrived or is lost: stop after 2 s
         idle once the sender is done; nothing at all for 60 s ends it too */
      const double tn = now();
      if (atomic_load(&g->send_done) && tn - (idle_since < 0 ? t_start : idle_since) > 2.0) break;
      if (idle_since < 0 && tn - t_start > 60.0) break;
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
    }
    const double t = now();
    const int drc = gw_decapsulate_batch(g->b, m, (const uint8_t *const *)&g->rx[d], &g->rx_len[d],
                                              &g->dst[d], &g->dst_cap[d], &g->res[d]);
    g->t_decap += now() - t;
    if (drc) {
      fprintf(stderr, "decapsulate_batch: %s\n", wg_gpu_last_error());
      atomic_store(&g->failed, 1);
      break;
    }
    atomic_store(&g->n_dec, d + m);
    g->t_end = now();
  }
  return NULL;
}


/* "mux[=W]": the PacketWorkers shape across peers -- W worker groups (default 1), each
 * serving the pairs p with p % W == its index: ONE encrypt worker whose batches mix its
 * pairs' packets (one at a time round robin, as NepTUN's inter-thread batches mix peers,
 * packet_workers.rs:178-205) in one wg_tunn_encapsulate_multi call, then one sendmmsg
 * per pair within its window; ONE decrypt worker that takes what each of its pairs'
 * readers has received into one wg_tunn_decapsulate_multi call.  The readers stay one
 * per socket.  Threads: 2 W + pairs, whatever the number of peers per worker. */
typedef struct {
  gw_t **gp;   /* this group's pairs */
  uint32_t pairs, batch;
  gw_engine *e;
  double t_encap, t_decap;
} mux_t;

static void *mux_sender(void *arg) {
  mux_t *mx = arg;
  const uint32_t P = mx->pairs, B = mx->batch;
  gw_t **gp = mx->gp;
  const input_t *in = gp[0]->in;
  gw_tunn **tun = calloc(B, sizeof *tun);
  const uint8_t **src = calloc(B, sizeof *src);
  uint8_t **dst = calloc(B, sizeof *dst);
  uint32_t *len = calloc(B, 4), *cap = calloc(B, 4), *who = calloc(B, 4), *idx = calloc(B, 4);
  uint32_t *cur = calloc(P, 4);
  wg_tunn_result *res = calloc(B, sizeof *res);
  struct mmsghdr *msgs = calloc(B, sizeof *msgs);
  struct iovec *iov = calloc(B, sizeof *iov);
  for (uint32_t p = 0; p < P; ++p) cur[p] = gp[p]->i0;
  int stop = 0;
  while (!stop) {
    uint32_t m = 0;
    for (int any = 1; m < B && any;) {
      any = 0;
      for (uint32_t p = 0; p < P && m < B; ++p)
        if (cur[p] < gp[p]->i1) {
          const uint32_t i = cur[p]++;
          who[m] = p;
          idx[m] = i;
          tun[m] = gp[p]->a;
          src[m] = in->pkt[i];
          len[m] = in->len[i];
          dst[m] = gp[p]->sent[i];
          cap[m] = gp[p]->slot;
          ++m;
          any = 1;
        }
    }
    if (m == 0) break;
    const double t = now();
    const int erc = gw_encapsulate_multi(mx->e, m, tun, src, len, dst, cap, res);
    mx->t_encap += now() - t;
    if (erc) {
      fprintf(stderr, "encapsulate_multi: %s\n", wg_gpu_last_error());
      for (uint32_t p = 0; p < P; ++p) atomic_store(&gp[p]->failed, 1);
      break;
    }
    for (uint32_t p = 0; p < P && !stop; ++p) {
      gw_t *g = gp[p];
      uint32_t k = 0;
      for (uint32_t j = 0; j < m; ++j) {
        if (who[j] != p) continue;
        const uint32_t i = idx[j];
        g->sent_len[i] = res[j].kind == WG_TUNN_WRITE_TO_NETWORK ? res[j].len : 0;
        if (!g->sent_len[i]) continue;
        iov[k].iov_base = g->sent[i];
        iov[k].iov_len = g->sent_len[i];
        memset(&msgs[k], 0, sizeof msgs[k]);
        msgs[k].msg_hdr.msg_iov = &iov[k];
        msgs[k].msg_hdr.msg_iovlen = 1;
        ++k;
      }
      if (k && send_window(g, msgs, k)) stop = 1;
    }
  }
  for (uint32_t p = 0; p < P; ++p) atomic_store(&gp[p]->send_done, 1);
  free(tun); free(src); free(dst); free(len); free(cap); free(who); free(idx); free(cur);
  free(res); free(msgs); free(iov);
  return NULL;
}

static void *mux_decryptor(void *arg) {
  mux_t *mx = arg;
  const uint32_t P = mx->pairs, B = mx->batch;
  gw_t **gp = mx->gp;
  gw_tunn **tun = calloc(B, sizeof *tun);
  const uint8_t **dg = calloc(B, sizeof *dg);
  uint8_t **dst = calloc(B, sizeof *dst);
  uint32_t *len = calloc(B, 4), *cap = calloc(B, 4), *took = calloc(P, 4), *from = calloc(P, 4);
  wg_tunn_result *res = calloc(B, sizeof *res);
  uint32_t first = 0;  /* the pair served first (rotates: no pair starves the others) */
  for (;;) {
    uint32_t m = 0;
    int all_done = 1, failed = 0;
    for (uint32_t q = 0; q < P; ++q) {
      const uint32_t p = (first + q) % P;
      gw_t *g = gp[p];
      const int finished = atomic_load(&g->rx_done);
      const uint32_t d = atomic_load(&g->n_dec), avail = atomic_load(&g->n_rx);
      failed |= atomic_load(&g->failed);
      uint32_t take = avail - d;
      if (take > B - m) take = B - m;
      if (!(finished && d + take == avail)) all_done = 0;
      from[p] = d;
      took[p] = take;
      for (uint32_t k = 0; k < take; ++k) {
        const uint32_t L = g->rx_len[d + k];
        g->dst_cap[d + k] = L > 16 ? L - 16 : 0;
        tun[m + k] = g->b;
        dg[m + k] = g->rx[d + k];
        len[m + k] = L;
        dst[m + k] = g->dst[d + k];
        cap[m + k] = g->dst_cap[d + k];
      }
      m += take;
    }
    first = (first + 1) % P;
    if (m == 0) {
      if (all_done || failed) break;
      sched_yield();
      continue;
    }
    const double t = now();
    const int drc = gw_decapsulate_multi(mx->e, m, tun, dg, len, dst, cap, res);
    mx->t_decap += now() - t;
    if (drc) {
      fprintf(stderr, "decapsulate_multi: %s\n", wg_gpu_last_error());
      for (uint32_t p = 0; p < P; ++p) atomic_store(&gp[p]->failed, 1);
      break;
    }
    uint32_t j = 0;
    for (uint32_t q = 0; q < P; ++q) {
      const uint32_t p = (first + P - 1 + q) % P;  /* (the order the batch was built in) */
      gw_t *g = gp[p];
      memcpy(&g->res[from[p]], &res[j], took[p] * sizeof *res);
      j += took[p];
      atomic_store(&g->n_dec, from[p] + took[p]);
      if (took[p]) g->t_end = now();
    }
    if (all_done) break;
  }
  free(tun); free(dg); free(dst); free(len); free(cap); free(took); free(from); free(res);
  return NULL;
}

/* Warm-up before the clock starts, as a long-running gateway is: every pair runs one
 * batch through a scratch Tunn pair on the same engines (the engines' lanes, streams
 * and staging are made on first use), concurrently, so the timed run does not pay for
 * them.  The pairs' own Tunns stay untouched (their counters start at 0). */
typedef struct {
  gw_t *g;
  gw_tunn *t;
  int phase, rc;  /* phase 0: encapsulate into `sent` (side a) or `rx` (side b); 1: decapsulate `sent` */
  int side;
} warm_t;

static void *warm_one(void *arg) {
  warm_t *w = arg;
  gw_t *g = w->g;
  const uint32_t m = g->i1 - g->i0 < g->batch ? g->i1 - g->i0 : g->batch;
  uint32_t *cap = calloc(m, 4), *len = calloc(m, 4);
  wg_tunn_result *res = calloc(m, sizeof *res);
  for (uint32_t j = 0; j < m; ++j) cap[j] = g->slot;
  if (w->phase == 0) {
    w->rc = gw_encapsulate_batch(w->t, m, (const uint8_t *const *)&g->in->pkt[g->i0], &g->in->len[g->i0],
                                 w->side ? &g->rx[0] : &g->sent[g->i0], cap, res);
  } else {
    for (uint32_t j = 0; j < m; ++j) len[j] = g->in->len[g->i0 + j] + 32;
    w->rc = gw_decapsulate_batch(w->t, m, (const uint8_t *const *)&g->sent[g->i0], len, &g->dst[0], cap, res);
  }
  free(cap); free(len); free(res);
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
    fprintf(stderr, "usage: %s IN OUT [batch] [pairs]\n", argv[0]);
    return 2;
  }
  input_t in;
  if (load_input(argv[1], &in)) {
    fprintf(stderr, "bad input %s\n", argv[1]);
    return 2;
  }
  const uint32_t batch = argc > 3 && atoi(argv[3]) > 0 ? (uint32_t)atoi(argv[3]) : 512;
  /* pairs > 1: that many independent peers (Tunn pairs, socket pairs and
   * threads) share the input -- NepTUN's per-peer Mutex<Tunn> + n_threads
   * event loops; the output file is written when every pair received its whole share
   * (pair p's arrivals then sit in rx[n p / pairs, n (p + 1) / pairs)) */
  const uint32_t pairs = argc > 4 && atoi(argv[4]) > 0 ? (uint32_t)atoi(argv[4]) : 1;
  int reg = 0, mux = 0;  /* mux: worker groups (0: one sender + decryptor per pair) */
  for (int a = 5; a < argc; ++a) {
    reg |= strcmp(argv[a], "reg") == 0;
    if (strncmp(argv[a], "mux", 3) == 0) mux = argv[a][3] == '=' ? atoi(argv[a] + 4) : 1;
  }
  wg_gpu_ctx *ctx = NULL;
#ifndef GW_CPU
  CHECK(wg_gpu_ctx_create(0, 64 * pairs, &ctx));  /* (+ the warm-up Tunns' slots) */
#endif
  const uint32_t n = in.n;
  uint8_t **sent = calloc(n, sizeof *sent), **rx = calloc(n, sizeof *rx), **dst = calloc(n, sizeof *dst);
  uint32_t *sent_len = calloc(n, 4), *rx_len = calloc(n, 4), *dst_cap = calloc(n, 4);
  wg_tunn_result *res = calloc(n, sizeof *res);
  /* every packet buffer is preallocated and touched before the clock starts, as
   * a gateway's buffer pools are: the timed region holds no malloc or page fault */
  uint32_t max_len = 0;
  for (uint32_t i = 0; i < n; ++i) max_len = in.len[i] > max_len ? in.len[i] : max_len;
  const uint32_t slot = (max_len + 64 + 63) & ~63u;
  /* (4 regions: datagrams sent, datagrams received, decrypted packets, and -- with
   * "reg" -- the TUN read pool the plaintexts sit in; page-aligned for registration) */
  const size_t slab_bytes = ((size_t)4 * n * slot + 4095) & ~(size_t)4095;
  uint8_t *slabs = aligned_alloc(4096, slab_bytes);
  if (!slabs) return 1;
  memset(slabs, 0, slab_bytes);
  for (uint32_t i = 0; i < n; ++i) {
    sent[i] = slabs + (size_t)i * slot;
    rx[i] = slabs + ((size_t)n + i) * slot;
    dst[i] = slabs + ((size_t)2 * n + i) * slot;
    if (reg) {  /* the read pool: each plaintext in its slot, as a TUN read leaves it */
      uint8_t *b = slabs + ((size_t)3 * n + i) * slot;
      memcpy(b, in.pkt[i], in.len[i]);
      in.pkt[i] = b;
    }
  }
  if (reg && ctx) CHECK(wg_gpu_register_host(ctx, slabs, slab_bytes));
  gw_t *gs = calloc(pairs, sizeof *gs);
  int rcvbuf = 0;
  for (uint32_t p = 0; p < pairs; ++p) {
    gw_t *g = &gs[p];
    g->in = &in;
    g->i0 = (uint32_t)((uint64_t)n * p / pairs);
    g->i1 = (uint32_t)((uint64_t)n * (p + 1) / pairs);
    g->batch = batch;
    g->slot = slot;
#ifdef GW_CPU
    CHECK(cpu_tunn_create(&g->a));
    CHECK(cpu_tunn_create(&g->b));
#else
    if (getenv("GW_PRIVATE_ENGINES")) { /* (A/B: one engine per Tunn) */
      wg_engine *ea = NULL, *eb = NULL;
      CHECK(wg_engine_create(ctx, &ea));
      CHECK(wg_engine_create(ctx, &eb));
      CHECK(wg_tunn_create_on(ea, 32 * p, &g->a));
      CHECK(wg_tunn_create_on(eb, 32 * p + 16, &g->b));
    } else {
      CHECK(wg_tunn_create(ctx, 32 * p, &g->a));
      CHECK(wg_tunn_create(ctx, 32 * p + 16, &g->b));
    }
#endif
    /* A sends with k1 to b_idx and receives with k2; B the mirror image */
    CHECK(gw_install_session(g->a, in.a_idx + 256 * p, in.b_idx + 256 * p, in.k2, in.k1, 1));
    CHECK(gw_install_session(g->b, in.b_idx + 256 * p, in.a_idx + 256 * p, in.k1, in.k2, 1));
    struct sockaddr_in aa, ab;
    g->sa = udp_socket(&aa);
    g->sb = udp_socket(&ab);
    if (g->sa < 0 || g->sb < 0 || connect(g->sa, (struct sockaddr *)&ab, sizeof ab)) {
      perror("socket");
      return 1;
    }
    socklen_t ol = sizeof rcvbuf;
    (void)getsockopt(g->sb, SOL_SOCKET, SO_RCVBUF, &rcvbuf, &ol);
    /* loopback charges each datagram its skb truesize (~2-4 KiB for <= 1500 B) */
    g->window = rcvbuf / 4096 > 16 ? (uint32_t)(rcvbuf / 4096) : 16;
    /* the pair's arrays are windows into the shared ones (sent: input order;
     * rx / dst / res: this pair's arrival order) */
    g->sent = sent;
    g->sent_len = sent_len;
    g->rx = rx + g->i0;
    g->rx_len = rx_len + g->i0;
    g->dst = dst + g->i0;
    g->dst_cap = dst_cap + g->i0;
    g->res = res + g->i0;
  }
  /* Warm-up before the clock starts, as in a long-running gateway: every pair runs a
   * batch through scratch Tunns on its Tunns' engines -- both sides' encapsulate at
   * once (as many concurrent calls as the run has), then one decapsulate -- so that the
   * engines' lanes, streams and staging (made on first use) exist before the timed run.
   * The pairs' own Tunns stay untouched (their counters start at 0). */
  {
    warm_t *ws = calloc(2 * pairs, sizeof *ws);
    pthread_t *wt = calloc(2 * pairs, sizeof *wt);
    for (uint32_t p = 0; p < pairs; ++p)
      for (int side = 0; side < 2; ++side) {
        warm_t *w = &ws[2 * p + side];
        w->g = &gs[p];
        w->side = side;
#ifdef GW_CPU
        CHECK(cpu_tunn_create(&w->t));
#else
        CHECK(wg_tunn_create_on(wg_tunn_engine(side ? gs[p].b : gs[p].a), 32 * (pairs + p) + 16 * side, &w->t));
#endif
        /* side a: session to side b's index 9; side b: the mirror image */
        CHECK(side ? gw_install_session(w->t, 9, 7, in.k1, in.k2, 1) : gw_install_session(w->t, 7, 9, in.k2, in.k1, 1));
      }
    for (int phase = 0; phase < 2; ++phase) {
      uint32_t nt = 0;
      for (uint32_t k = 0; k < 2 * pairs; ++k) {
        if (phase == 1 && ws[k].side == 0) continue;  /* side b opens side a's datagrams */
        ws[k].phase = phase;
        pthread_create(&wt[nt++], NULL, warm_one, &ws[k]);
      }
      for (uint32_t k = 0; k < nt; ++k) pthread_join(wt[k], NULL);
      for (uint32_t k = 0; k < 2 * pairs; ++k) CHECK(ws[k].rc);
    }
    for (uint32_t k = 0; k < 2 * pairs; ++k) gw_destroy(ws[k].t);
    free(ws);
    free(wt);
    memset(slabs, 0, (size_t)3 * n * slot);  /* (the sent / received / decrypted regions) */
  }
  if (mux > (int)pairs) mux = (int)pairs;
  mux_t *mxs = calloc(mux > 0 ? mux : 1, sizeof *mxs);
  gw_t **gps = calloc(pairs, sizeof *gps);
  for (int w = 0, k = 0; w < mux; ++w) {  /* group w: pairs w, w + W, ... */
    mxs[w].gp = gps + k;
    for (uint32_t p = (uint32_t)w; p < pairs; p += (uint32_t)mux) gps[k++] = &gs[p];
    mxs[w].pairs = (uint32_t)(gps + k - mxs[w].gp);
    mxs[w].batch = batch;
    mxs[w].e = gw_engine_of(gs[0].a);
  }
  const double t0 = now();
  pthread_t *th = calloc(3 * pairs + 2 * (mux > 0 ? mux : 0), sizeof *th);
  uint32_t nth = 0;
  for (uint32_t p = 0; p < pairs; ++p) {
    pthread_create(&th[nth++], NULL, reader, &gs[p]);
    if (!mux) {
      pthread_create(&th[nth++], NULL, decryptor, &gs[p]);
      pthread_create(&th[nth++], NULL, sender, &gs[p]);
    }
  }
  for (int w = 0; w < mux; ++w) {
    pthread_create(&th[nth++], NULL, mux_decryptor, &mxs[w]);
    pthread_create(&th[nth++], NULL, mux_sender, &mxs[w]);
  }
  for (uint32_t k = 0; k < nth; ++k) pthread_join(th[k], NULL);
  uint32_t nrx = 0, nsent = 0;
  uint64_t bytes = 0;
  double te = 0, ts = 0, tw = 0, tr = 0, td = 0;
  for (int w = 0; w < mux; ++w) te += mxs[w].t_encap, td += mxs[w].t_decap;
  double t_end = t0;
  for (uint32_t p = 0; p < pairs; ++p) {
    gw_t *g = &gs[p];
    if (atomic_load(&g->failed)) return 1;
    const uint32_t r = atomic_load(&g->n_rx);
    nrx += r;
    nsent += atomic_load(&g->n_sent);
    for (uint32_t i = 0; i < r; ++i)
      if (g->res[i].kind == WG_TUNN_WRITE_TO_TUNNEL) bytes += g->res[i].len;
    if (g->t_end > t_end) t_end = g->t_end;
    te += g->t_encap, ts += g->t_send, tw += g->t_wait, tr += g->t_recv, td += g->t_decap;
  }
  const double secs = t_end > t0 ? t_end - t0 : 1e-9;
  int whole = 1;
  for (uint32_t p = 0; p < pairs; ++p) whole &= atomic_load(&gs[p].n_rx) == gs[p].i1 - gs[p].i0;
  if (pairs == 1 || whole) {
    FILE *f = fopen(argv[2], "wb");
    if (!f) return 1;
    fwrite("NGWO", 1, 4, f);
    fwrite(&n, 4, 1, f);
    for (uint32_t i = 0; i < n; ++i) {
      fwrite(&sent_len[i], 4, 1, f);
      fwrite(sent[i], 1, sent_len[i], f);
    }
    fwrite(&nrx, 4, 1, f);
    for (uint32_t i = 0; i < nrx; ++i) {
      fwrite(&rx_len[i], 4, 1, f);
      fwrite(rx[i], 1, rx_len[i], f);
      fwrite(&res[i], sizeof res[i], 1, f);
      fwrite(&dst_cap[i], 4, 1, f);
      fwrite(dst[i], 1, dst_cap[i], f);
    }
    fclose(f);
  }
  printf("{\"backend\": \"" GW_BACKEND "\", \"packets\": %u, \"sent\": %u, \"received\": %u, \"lost\": %u, \"batch\": %u, "
         "\"pairs\": %u, \"mux\": %d, \"registered\": %d, \"window\": %u, \"rcvbuf\": %d, \"seconds\": %.6f, \"ip_bytes\": %llu, "
         "\"socket_to_socket_gbps\": %.3f, \"thread_seconds\": {\"encapsulate\": %.4f, "
         "\"sendmmsg\": %.4f, \"window_wait\": %.4f, \"recvmmsg\": %.4f, \"decapsulate\": %.4f}",
         n, nsent, nrx, nsent - nrx, batch, pairs, mux, reg, gs[0].window, rcvbuf, secs,
         (unsigned long long)bytes, bytes * 8.0 / secs / 1e9, te, ts, tw, tr, td);
#ifndef GW_CPU
  /* where the library's time went, summed over the pairs' Tunns (wg_tunn_get_phases) */
  for (int side = 0; side < 2; ++side) {
    wg_tunn_phases s = {0}, q;
    for (uint32_t p = 0; p < pairs; ++p) {
      if (wg_tunn_get_phases(side ? gs[p].b : gs[p].a, &q)) continue;
      s.calls += q.calls, s.packets += q.packets, s.total_us += q.total_us, s.checks_us += q.checks_us;
      s.pack_us += q.pack_us, s.submit_us += q.submit_us, s.wait_us += q.wait_us, s.decide_us += q.decide_us;
      s.copy_out_us += q.copy_out_us, s.prep_us += q.prep_us;
    }
    printf(", \"%s_phases_s\": {\"calls\": %llu, \"packets\": %llu, \"total\": %.4f, \"checks\": %.4f, "
           "\"pack\": %.4f, \"submit\": %.4f, \"wait\": %.4f, \"decide\": %.4f, \"copy_out\": %.4f, "
           "\"prep\": %.4f}",
           side ? "decapsulate" : "encapsulate", (unsigned long long)s.calls, (unsigned long long)s.packets,
           s.total_us * 1e-6, s.checks_us * 1e-6, s.pack_us * 1e-6, s.submit_us * 1e-6, s.wait_us * 1e-6,
           s.decide_us * 1e-6, s.copy_out_us * 1e-6, s.prep_us * 1e-6);
  }
#endif
  printf("}\n");
  for (uint32_t p = 0; p < pairs; ++p) {
    gw_destroy(gs[p].a);
    gw_destroy(gs[p].b);
  }
  if (reg && ctx) CHECK(wg_gpu_unregister_host(ctx, slabs));
  if (ctx) wg_gpu_ctx_destroy(ctx);
  return 0;
}
