// wg_tunn.cpp -- batched Tunn data plane (include/neptun_tunn.h).
//
// Host half of the drop-in: everything of Tunn::encapsulate / decapsulate
// that is stateful or sequential stays here, in the reference's order, and
// only the AEAD runs on the GPU (one descriptor batch per call).  A batch
// returns exactly what N sequential calls return: counters are handed out in
// packet order (session.rs:219), the replay window is applied in packet order
// after the GPU has opened everything (a packet's quick check sees the marks of
// the packets before it, session.rs:279 and :300), and byte counters follow
// mod.rs:321 / :667.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "neptun_gpu.h"
#include "neptun_tunn.h"

int wg_pipe_fail(int rc, const char *what, hipError_t e);  // wg_gpu.cpp
int wg_ctx_device(const wg_gpu_ctx *ctx);                   // wg_gpu.cpp

// ---------------------------------------------------------------------------
// replay window: ReceivingKeyCounterValidator, session.rs:40-157
// ---------------------------------------------------------------------------
namespace {
constexpr uint64_t kWordBits = 64, kWords = WG_REPLAY_WORDS, kBits = kWordBits * kWords;

inline void set_bit(wg_replay *w, uint64_t idx) {
  const uint64_t b = idx % kBits;
  w->bitmap[b / kWordBits] |= 1ull << (b % kWordBits);
}
inline void clear_bit(wg_replay *w, uint64_t idx) {
  const uint64_t b = idx % kBits;
  w->bitmap[b / kWordBits] &= ~(1ull << (b % kWordBits));
}
inline void clear_word(wg_replay *w, uint64_t idx) { w->bitmap[(idx % kBits) / kWordBits] = 0; }
inline bool check_bit(const wg_replay *w, uint64_t idx) {
  const uint64_t b = idx % kBits;
  return (w->bitmap[b / kWordBits] >> (b % kWordBits)) & 1ull;
}
}  // namespace

extern "C" {

void wg_replay_init(wg_replay *w) { std::memset(w, 0, sizeof *w); }

int wg_replay_will_accept(const wg_replay *w, uint64_t counter) {
  if (counter >= w->next) return WG_STATUS_OK;                      // :91-94
  if (counter + kBits < w->next) return WG_STATUS_INVALID_COUNTER;  // :95-98
  return check_bit(w, counter) ? WG_STATUS_DUPLICATE_COUNTER : WG_STATUS_OK;
}

int wg_replay_mark_did_receive(wg_replay *w, uint64_t counter) {
  if (counter + kBits < w->next) return WG_STATUS_INVALID_COUNTER;  // :110-113
  if (counter == w->next) {                                         // :114-120
    set_bit(w, counter);
    w->next += 1;
    return WG_STATUS_OK;
  }
  if (counter < w->next) {                                          // :121-128
    if (check_bit(w, counter)) return WG_STATUS_INVALID_COUNTER;
    set_bit(w, counter);
    return WG_STATUS_OK;
  }
  if (counter - w->next >= kBits) {                                 // :130-135
    std::memset(w->bitmap, 0, sizeof w->bitmap);
  } else {
    uint64_t i = w->next;
    while (i % kWordBits != 0 && i < counter) clear_bit(w, i++);    // :137-141
    while (i + kWordBits < counter) {                               // :142-146
      clear_word(w, i);
      i = (i + kWordBits) & (0ull - kWordBits);
    }
    while (i < counter) clear_bit(w, i++);                          // :147-151
  }
  set_bit(w, counter);
  w->next = counter + 1;
  return WG_STATUS_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Tunn mirror
// ---------------------------------------------------------------------------
namespace {

struct Session {  // session.rs:11-18
  bool live = false;
  uint32_t receiving_index = 0, sending_index = 0;
  uint64_t sending_counter = 0;  // AtomicUsize sending_key_counter
  wg_replay window{};
  uint64_t established = 0;      // install sequence: stands in for timers.session_timers
};

inline uint32_t ld32(const uint8_t *p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t ld64(const uint8_t *p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
inline uint32_t round128(uint64_t x) { return (uint32_t)((x + 127) / 128 * 128); }

// device + pinned staging for one batch
struct Staging {
  uint8_t *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
  wg_packet_desc *h_desc = nullptr, *d_desc = nullptr;
  int32_t *h_st = nullptr, *d_st = nullptr;
  size_t bytes = 0, descs = 0;
};

void free_staging(Staging &s) {
  (void)hipHostFree(s.h_in);
  (void)hipHostFree(s.h_out);
  (void)hipHostFree(s.h_desc);
  (void)hipHostFree(s.h_st);
  (void)hipFree(s.d_in);
  (void)hipFree(s.d_out);
  (void)hipFree(s.d_desc);
  (void)hipFree(s.d_st);
  s = Staging{};
}

hipError_t reserve(Staging &s, size_t bytes, size_t descs) {
  hipError_t e = hipSuccess;
  if (bytes > s.bytes) {
    (void)hipHostFree(s.h_in);
    (void)hipHostFree(s.h_out);
    (void)hipFree(s.d_in);
    (void)hipFree(s.d_out);
    s.h_in = s.h_out = s.d_in = s.d_out = nullptr;
    bytes = std::max(bytes, 2 * s.bytes);
    s.bytes = 0;
    if ((e = hipHostMalloc(&s.h_in, bytes)) != hipSuccess) return e;
    if ((e = hipHostMalloc(&s.h_out, bytes)) != hipSuccess) return e;
    if ((e = hipMalloc(&s.d_in, bytes)) != hipSuccess) return e;
    if ((e = hipMalloc(&s.d_out, bytes)) != hipSuccess) return e;
    s.bytes = bytes;
  }
  if (descs > s.descs) {
    (void)hipHostFree(s.h_desc);
    (void)hipHostFree(s.h_st);
    (void)hipFree(s.d_desc);
    (void)hipFree(s.d_st);
    s.h_desc = nullptr; s.d_desc = nullptr; s.h_st = nullptr; s.d_st = nullptr;
    descs = std::max(descs, 2 * s.descs);
    s.descs = 0;
    if ((e = hipHostMalloc(&s.h_desc, descs * sizeof(wg_packet_desc))) != hipSuccess) return e;
    if ((e = hipHostMalloc(&s.h_st, descs * 4)) != hipSuccess) return e;
    if ((e = hipMalloc(&s.d_desc, descs * sizeof(wg_packet_desc))) != hipSuccess) return e;
    if ((e = hipMalloc(&s.d_st, descs * 4)) != hipSuccess) return e;
    s.descs = descs;
  }
  return e;
}

}  // namespace

struct wg_tunn {
  wg_gpu_ctx *ctx = nullptr;
  int device = 0;
  uint32_t first_slot = 0;  // ring slot i: receiving key first_slot + 2i, sending first_slot + 2i + 1
  Session sessions[WG_N_SESSIONS];
  uint64_t current = 0;     // index of the most recently used session (mod.rs:69)
  uint64_t tx_bytes = 0, rx_bytes = 0;
  uint64_t install_seq = 0;
  hipStream_t stream = nullptr;
  Staging st;
};

namespace {

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

#define TUNN_HIP(call, what)                                              \
  do {                                                                    \
    hipError_t e_ = (call);                                               \
    if (e_ != hipSuccess) return wg_pipe_fail(WG_RC_HIP_ERROR, what, e_); \
  } while (0)

// set_current_session (mod.rs:521-532); the timer comparison uses install order
void set_current_session(wg_tunn *t, uint64_t new_idx) {
  const uint64_t cur = t->current;
  if (cur == new_idx) return;
  const Session &c = t->sessions[cur % WG_N_SESSIONS];
  const Session &n = t->sessions[new_idx % WG_N_SESSIONS];
  if (!c.live || n.established >= c.established) t->current = new_idx;
}

inline void set_err(wg_tunn_result &r, int32_t st) {
  std::memset(&r, 0, sizeof r);
  r.kind = WG_TUNN_ERR;
  r.status = st;
}

// run one descriptor batch through the GPU: h_in -> d_in, kernel, d_out -> h_out
int gpu_round(wg_tunn *t, bool seal, uint32_t m, size_t bytes) {
  Staging &s = t->st;
  TUNN_HIP(hipMemcpyAsync(s.d_in, s.h_in, bytes, hipMemcpyHostToDevice, t->stream), "tunn: H2D");
  TUNN_HIP(hipMemcpyAsync(s.d_desc, s.h_desc, (size_t)m * sizeof(wg_packet_desc),
                          hipMemcpyHostToDevice, t->stream),
           "tunn: descs H2D");
  const int rc = seal ? wg_gpu_seal_batch(t->ctx, s.d_desc, m, s.d_in, s.d_out, s.d_st, t->stream)
                      : wg_gpu_open_batch(t->ctx, s.d_desc, m, s.d_in, s.d_out, s.d_st, t->stream);
  if (rc) return rc;
  TUNN_HIP(hipMemcpyAsync(s.h_out, s.d_out, bytes, hipMemcpyDeviceToHost, t->stream), "tunn: D2H");
  TUNN_HIP(hipMemcpyAsync(s.h_st, s.d_st, (size_t)m * 4, hipMemcpyDeviceToHost, t->stream),
           "tunn: status D2H");
  TUNN_HIP(hipStreamSynchronize(t->stream), "tunn: sync");
  return WG_RC_OK;
}

}  // namespace

extern "C" {

int wg_tunn_create(wg_gpu_ctx *ctx, uint32_t first_slot, wg_tunn **out) {
  if (!ctx || !out) return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "tunn_create: null", hipSuccess);
  if ((uint64_t)first_slot + 2 * WG_N_SESSIONS > wg_gpu_ctx_key_slots(ctx))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "tunn_create: needs 16 key slots", hipSuccess);
  wg_tunn *t = new (std::nothrow) wg_tunn;
  if (!t) return wg_pipe_fail(WG_RC_OUT_OF_MEMORY, "tunn_create: host alloc", hipSuccess);
  t->ctx = ctx;
  t->device = wg_ctx_device(ctx);
  t->first_slot = first_slot;
  DevGuard g(t->device);
  const hipError_t e = hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete t;
    return wg_pipe_fail(WG_RC_HIP_ERROR, "tunn_create: stream", e);
  }
  *out = t;
  return WG_RC_OK;
}

int wg_tunn_destroy(wg_tunn *t) {
  if (!t) return WG_RC_OK;
  DevGuard g(t->device);
  (void)hipStreamSynchronize(t->stream);
  free_staging(t->st);
  (void)hipStreamDestroy(t->stream);
  delete t;
  return WG_RC_OK;
}

int wg_tunn_install_session(wg_tunn *t, uint32_t local_index, uint32_t peer_index,
                            const uint8_t receiving_key[32], const uint8_t sending_key[32],
                            int make_current) {
  if (!t || !receiving_key || !sending_key)
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "install_session: null", hipSuccess);
  const uint32_t ring = local_index % WG_N_SESSIONS;
  uint8_t keys[64];
  std::memcpy(keys, receiving_key, 32);
  std::memcpy(keys + 32, sending_key, 32);
  // receiving slot checks our index; sending slot writes the peer's (session.rs:226, :275)
  const uint32_t idx[2] = {local_index, peer_index};
  DevGuard g(t->device);
  const int rc = wg_gpu_set_keys(t->ctx, t->first_slot + 2 * ring, 2, keys, idx, t->stream);
  if (rc) return rc;
  Session &s = t->sessions[ring];
  s = Session{};
  s.live = true;
  s.receiving_index = local_index;
  s.sending_index = peer_index;
  wg_replay_init(&s.window);
  s.established = ++t->install_seq;
  if (make_current) set_current_session(t, local_index);
  return WG_RC_OK;
}

int wg_tunn_stats(const wg_tunn *t, uint64_t *tx_bytes, uint64_t *rx_bytes) {
  if (!t) return WG_RC_INVALID_ARGUMENT;
  if (tx_bytes) *tx_bytes = t->tx_bytes;
  if (rx_bytes) *rx_bytes = t->rx_bytes;
  return WG_RC_OK;
}

int wg_tunn_session_counters(const wg_tunn *t, uint32_t ring_slot, uint64_t *sending_counter,
                             wg_replay *window) {
  if (!t || ring_slot >= WG_N_SESSIONS) return WG_RC_INVALID_ARGUMENT;
  if (sending_counter) *sending_counter = t->sessions[ring_slot].sending_counter;
  if (window) *window = t->sessions[ring_slot].window;
  return WG_RC_OK;
}

int wg_tunn_encapsulate_batch(wg_tunn *t, uint32_t n, const uint8_t *const *src,
                              const uint32_t *src_len, uint8_t *const *dst,
                              const uint32_t *dst_cap, wg_tunn_result *res) {
  if (!t || (n && (!src || !src_len || !dst || !dst_cap || !res)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "encapsulate_batch: null", hipSuccess);
  if (n == 0) return WG_RC_OK;
  DevGuard g(t->device);
  Session &s = t->sessions[t->current % WG_N_SESSIONS];  // mod.rs:310
  const uint32_t slot = t->first_slot + 2 * (uint32_t)(t->current % WG_N_SESSIONS) + 1;
  // pass 1 (host, in order): checks and counter reservation
  std::vector<uint32_t> sel;  // packets that reach format_packet_data
  size_t bytes = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if ((uint64_t)src_len[i] + WG_DATA_OFFSET > dst_cap[i]) {  // encapsulate: dst[16..len+16]
      set_err(res[i], WG_STATUS_INVALID_LENGTH);
      continue;
    }
    std::memcpy(dst[i] + WG_DATA_OFFSET, src[i], src_len[i]);  // mod.rs:296-299, before the session
    if (!s.live) {  // no session: the CPU Tunn queues the packet and starts a handshake
      std::memset(&res[i], 0, sizeof res[i]);
      res[i].kind = WG_TUNN_NOT_DATA;
      res[i].status = WG_STATUS_NO_CURRENT_SESSION;
      continue;
    }
    if ((uint64_t)src_len[i] + WG_DATA_OVERHEAD_SZ > dst_cap[i]) {  // session.rs:210-217
      set_err(res[i], WG_STATUS_INCORRECT_PACKET_LENGTH);
      continue;
    }
    sel.push_back(i);
    bytes += round128((uint64_t)src_len[i] + WG_DATA_OVERHEAD_SZ);
  }
  if (sel.empty()) return WG_RC_OK;
  TUNN_HIP(reserve(t->st, bytes + 128, sel.size()), "encapsulate_batch: staging");
  Staging &st = t->st;
  size_t off = 0;
  for (size_t k = 0; k < sel.size(); ++k) {
    const uint32_t i = sel[k];
    std::memcpy(st.h_in + off + WG_DATA_OFFSET, src[i], src_len[i]);  // NepTUN slot layout
    st.h_desc[k] = wg_packet_desc{off + WG_DATA_OFFSET, off, s.sending_counter++, src_len[i], slot};
    off += round128((uint64_t)src_len[i] + WG_DATA_OVERHEAD_SZ);
  }
  const int rc = gpu_round(t, true, (uint32_t)sel.size(), off);
  if (rc) return rc;
  for (size_t k = 0; k < sel.size(); ++k) {
    const uint32_t i = sel[k];
    const uint32_t w = src_len[i] + WG_DATA_OVERHEAD_SZ;
    if (st.h_st[k] != WG_STATUS_OK) {  // the GPU path has no other failure mode
      set_err(res[i], WG_STATUS_CRYPTO_FAILED);
      continue;
    }
    std::memcpy(dst[i], st.h_out + st.h_desc[k].dst_off, w);
    t->tx_bytes += w;  // mod.rs:321
    std::memset(&res[i], 0, sizeof res[i]);
    res[i].kind = WG_TUNN_WRITE_TO_NETWORK;
    res[i].len = w;
  }
  return WG_RC_OK;
}

}  // extern "C"

// Packet-level pieces shared by decapsulate and decrypt
namespace {

// parse_incoming_packet (mod.rs:139-199): 1 = data, 0 = handshake/cookie, <0 = -InvalidPacket
int parse_kind(const uint8_t *d, uint32_t L) {
  if (L < 4) return -WG_STATUS_INVALID_PACKET;
  const uint32_t type = ld32(d);
  if ((type == 1 && L == 148) || (type == 2 && L == 92) || (type == 3 && L == 64)) return 0;
  if (type != WG_MSG_DATA || L < WG_DATA_OVERHEAD_SZ) return -WG_STATUS_INVALID_PACKET;
  return 1;
}

// stage the selected datagrams (slot layout) and open them on the GPU
int open_selected(wg_tunn *t, const std::vector<uint32_t> &sel, const std::vector<uint32_t> &slot,
                  const uint8_t *const *datagram, const uint32_t *len) {
  if (sel.empty()) return WG_RC_OK;
  size_t bytes = 0;
  for (uint32_t i : sel) bytes += round128(len[i]);
  Staging &st = t->st;
  TUNN_HIP(reserve(st, bytes + 128, sel.size()), "decapsulate: staging");
  size_t off = 0;
  for (size_t k = 0; k < sel.size(); ++k) {
    const uint32_t i = sel[k];
    std::memcpy(st.h_in + off, datagram[i], len[i]);
    st.h_desc[k] = wg_packet_desc{off, off + WG_DATA_OFFSET, 0, len[i], slot[k]};
    off += round128(len[i]);
  }
  return gpu_round(t, false, (uint32_t)sel.size(), off);
}

// session.rs:287-296 result in dst: plaintext (zeros if the tag failed, as ring
// leaves it) followed by the untouched tag bytes
void copy_out(const wg_tunn *t, size_t k, const uint8_t *d, uint32_t P, uint8_t *out) {
  const Staging &st = t->st;
  if (st.h_st[k] == WG_STATUS_OK) std::memcpy(out, st.h_out + st.h_desc[k].dst_off, P);
  else std::memset(out, 0, P);
  std::memcpy(out + P, d + WG_DATA_OFFSET + P, WG_AEAD_SIZE);
}

// validate_decapsulated_packet (mod.rs:606-670) on dst[..P]
void validate(wg_tunn *t, const uint8_t *out, uint32_t P, wg_tunn_result &r) {
  if (P == 0) {
    t->rx_bytes += WG_DATA_OVERHEAD_SZ;  // keepalive
    r.kind = WG_TUNN_DONE;
    return;
  }
  uint32_t ip_len = 0;
  const uint8_t v = out[0] >> 4;
  if (v == 4 && P >= 20) {
    ip_len = (uint32_t)out[2] << 8 | out[3];
    r.ip_version = 4;
    std::memcpy(r.src_ip, out + 12, 4);
  } else if (v == 6 && P >= 40) {
    ip_len = ((uint32_t)out[4] << 8 | out[5]) + 40;
    r.ip_version = 6;
    std::memcpy(r.src_ip, out + 8, 16);
  } else {
    set_err(r, WG_STATUS_INVALID_PACKET);
    return;
  }
  if (ip_len > P) {
    set_err(r, WG_STATUS_INVALID_PACKET);
    return;
  }
  t->rx_bytes += (uint64_t)ip_len + WG_DATA_OVERHEAD_SZ;  // message_data_len, session.rs:357
  r.kind = WG_TUNN_WRITE_TO_TUNNEL;
  r.len = ip_len;
}

}  // namespace

extern "C" {

int wg_tunn_decapsulate_batch(wg_tunn *t, uint32_t n, const uint8_t *const *datagram,
                              const uint32_t *len, uint8_t *const *dst, const uint32_t *dst_cap,
                              wg_tunn_result *res) {
  if (!t || (n && (!datagram || !len || !dst || !dst_cap || !res)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "decapsulate_batch: null", hipSuccess);
  if (n == 0) return WG_RC_OK;
  DevGuard g(t->device);
  // pass 1 (stateless checks, reference order): parse, session, dst size, index
  std::vector<uint32_t> sel, slot;  // DATA packets that reach the AEAD
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *d = datagram[i];
    const uint32_t L = len[i];
    std::memset(&res[i], 0, sizeof res[i]);
    if (L == 0) {  // "repeated call": send_queued_packet is the CPU Tunn's business
      res[i].kind = WG_TUNN_NOT_DATA;
      continue;
    }
    const int pk = parse_kind(d, L);
    if (pk < 0) { set_err(res[i], -pk); continue; }
    if (pk == 0) {  // handshake init / response / cookie (mod.rs:150-181)
      res[i].kind = WG_TUNN_NOT_DATA;
      continue;
    }
    const uint32_t ridx = ld32(d + 4);
    const Session &s = t->sessions[ridx % WG_N_SESSIONS];
    int32_t e = WG_STATUS_OK;
    if (!s.live) e = WG_STATUS_NO_CURRENT_SESSION;                                 // mod.rs:553-556
    else if ((uint64_t)dst_cap[i] < L - WG_DATA_OFFSET) e = WG_STATUS_DESTINATION_BUFFER_TOO_SMALL;  // session.rs:271
    else if (ridx != s.receiving_index) e = WG_STATUS_WRONG_INDEX;                // session.rs:275
    if (e) { set_err(res[i], e); continue; }
    sel.push_back(i);
    slot.push_back(t->first_slot + 2 * (ridx % WG_N_SESSIONS));
  }
  const int rc = open_selected(t, sel, slot, datagram, len);
  if (rc) return rc;
  // pass 2 (sequential, packet order): replay window, copy-out, validation, stats
  for (size_t k = 0; k < sel.size(); ++k) {
    const uint32_t i = sel[k];
    const uint8_t *d = datagram[i];
    const uint32_t P = len[i] - WG_DATA_OVERHEAD_SZ;
    const uint32_t ridx = ld32(d + 4);
    const uint64_t ctr = ld64(d + 8);
    Session &s = t->sessions[ridx % WG_N_SESSIONS];
    int32_t e = wg_replay_will_accept(&s.window, ctr);  // session.rs:279
    if (e) { set_err(res[i], e); continue; }
    copy_out(t, k, d, P, dst[i]);
    if (t->st.h_st[k] != WG_STATUS_OK) { set_err(res[i], t->st.h_st[k]); continue; }
    e = wg_replay_mark_did_receive(&s.window, ctr);  // session.rs:300, :192-199
    if (e) { set_err(res[i], e); continue; }
    s.window.receive_cnt += 1;
    set_current_session(t, ridx);  // mod.rs:562
    validate(t, dst[i], P, res[i]);
  }
  return WG_RC_OK;
}

int wg_tunn_decrypt_batch(wg_tunn *t, uint32_t n, const uint8_t *const *datagram,
                          const uint32_t *len, uint8_t *const *dst, const uint32_t *dst_cap,
                          wg_tunn_result *res) {
  if (!t || (n && (!datagram || !len || !dst || !dst_cap || !res)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "decrypt_batch: null", hipSuccess);
  if (n == 0) return WG_RC_OK;
  DevGuard g(t->device);
  std::vector<uint32_t> sel, slot;
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *d = datagram[i];
    const uint32_t L = len[i];
    std::memset(&res[i], 0, sizeof res[i]);
    const int pk = parse_kind(d, L);
    if (pk < 0) { set_err(res[i], -pk); continue; }
    if (pk == 0) { set_err(res[i], WG_STATUS_WRONG_PACKET_TYPE); continue; }  // mod.rs:416
    const uint32_t ridx = ld32(d + 4);
    int ring = -1;  // sessions.iter().find_map(is_right_session) (mod.rs:394-397, session.rs:311-313)
    for (int r = 0; r < WG_N_SESSIONS && ring < 0; ++r) {
      const Session &s = t->sessions[r];
      if (s.live && (s.receiving_index == ridx || s.sending_index == ridx)) ring = r;
    }
    if (ring < 0) { set_err(res[i], WG_STATUS_NO_CURRENT_SESSION); continue; }
    if ((uint64_t)dst_cap[i] < L - WG_DATA_OFFSET) {  // session.rs:323-326
      set_err(res[i], WG_STATUS_DESTINATION_BUFFER_TOO_SMALL);
      continue;
    }
    // receiving key if the index is ours, else the sending key (session.rs:327-333); the
    // sending slot's key_index is the peer's index, which is what this header carries
    const bool ours = t->sessions[ring].receiving_index == ridx;
    sel.push_back(i);
    slot.push_back(t->first_slot + 2 * (uint32_t)ring + (ours ? 0u : 1u));
  }
  const int rc = open_selected(t, sel, slot, datagram, len);
  if (rc) return rc;
  for (size_t k = 0; k < sel.size(); ++k) {
    const uint32_t i = sel[k];
    const uint32_t P = len[i] - WG_DATA_OVERHEAD_SZ;
    copy_out(t, k, datagram[i], P, dst[i]);
    if (t->st.h_st[k] != WG_STATUS_OK) { set_err(res[i], t->st.h_st[k]); continue; }
    validate(t, dst[i], P, res[i]);
    if (res[i].kind == WG_TUNN_DONE) set_err(res[i], WG_STATUS_UNEXPECTED_PACKET);  // mod.rs:412
  }
  return WG_RC_OK;
}

}  // extern "C"
