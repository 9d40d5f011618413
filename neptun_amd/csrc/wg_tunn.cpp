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
//
// Data movement (the PacketWorkers replacement): a batch is cut
// into ~16 MiB chunks that flow through two pinned-staging buffer sets on two
// HIP streams -- host pack of chunk c+1 and host unpack of chunk c-1 overlap
// the H2D copy + AEAD kernel + D2H copy of chunk c -- and every host byte copy
// is split over a small persistent worker pool.  Sequential semantics are
// untouched: counters are reserved and replay/validation decisions are made
// by one thread in packet order; only the byte copies run in parallel.
//
// Several GPUs (wg_tunn_create_multi): the selected packets of a
// batch are split into contiguous, byte-balanced shares, one per GPU
// ("engine"), AFTER the one counter reservation of the batch (session.rs:219
// fetch_add), so the shares carry disjoint counters.  Each engine has its own
// driver thread, copy threads and pinned staging, bound to the GPU's NUMA node
// (sysfs numa_node of its PCI device; set_mempolicy + hipHostMallocNumaUser),
// and its own streams.  No collective: the shares never exchange data.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "neptun_gpu.h"
#include "neptun_tunn.h"
#include "wg_aead_kernels.h"

int wg_pipe_fail(int rc, const char *what, hipError_t e);  // wg_gpu.cpp
int wg_ctx_device(const wg_gpu_ctx *ctx);                   // wg_gpu.cpp
bool wg_ctx_slot_padding(const wg_gpu_ctx *ctx);            // wg_gpu.cpp
int wg_launch_desc_hinted(wg_gpu_ctx *ctx, bool seal, const wg_packet_desc *descs, uint32_t n,
                          const uint8_t *src, uint8_t *dst, int32_t *status, void *stream,
                          uint32_t max_len, bool host_mem, uint32_t *done_count = nullptr,
                          uint32_t *done_flag = nullptr, uint32_t done_seq = 0,
                          bool *flagged = nullptr, bool xlane_ok = true,
                          bool host_descs = false);  // wg_gpu.cpp
void wg_ctx_reg_snapshot(wg_gpu_ctx *ctx, std::vector<uint64_t> &out);  // wg_gpu.cpp
int wg_ctx_claim_slots(wg_gpu_ctx *ctx, uint32_t first, uint32_t count);  // wg_gpu.cpp
void wg_ctx_release_slots(wg_gpu_ctx *ctx, uint32_t first);              // wg_gpu.cpp
uint64_t wg_ctx_key_gen(const wg_gpu_ctx *ctx);                          // wg_gpu.cpp
const uint8_t *wg_ctx_keys(const wg_gpu_ctx *ctx);                       // wg_gpu.cpp
const uint32_t *wg_ctx_key_index(const wg_gpu_ctx *ctx);                 // wg_gpu.cpp

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
inline uint64_t round128(uint64_t x) { return (x + 127) / 128 * 128; }

// Packet copies into / out of pinned staging with streaming (non-temporal)
// stores: the bytes are read next by the copy engines or the caller, not by this
// core, and a streaming store skips the read-for-ownership of the destination
// line (a third of a cached memcpy's DRAM traffic).  WG_TUNN_NT=0: memcpy.
// Streaming (non-temporal) stores for the host copies into and out of pinned staging:
// they pay for batches far larger than the last-level cache and cost at smaller ones
// (1350-B packets, staged: memcpy 40 vs 66-84 us at 64 packets, 1.7-2.0 vs 2.3 ms at
// 16,384; streaming stores 150-158 vs 146-147 Gbit/s at 262,144; r05y / r05z).
// WG_TUNN_NT=1 / 0 forces either; default: streaming from 32,768 packets on.
bool nt_copies(size_t packets) {
  const char *e = std::getenv("WG_TUNN_NT");
  return e ? std::atoi(e) != 0 : packets >= 32768;
}
// The fewest packets worth a pool part of their own.  A blocked worker wakes tens of
// microseconds late on a loaded host (workers block 20 us after their last part, and a
// small call's GPU wait is longer than that), and a part it takes then holds up its
// caller: steps that only read headers or write descriptors (a few ns per packet) split
// from 2 x WG_TUNN_GRAIN_LIGHT (default 1024) packets; steps that copy payloads split
// into parts of WG_TUNN_GRAIN_COPY (64) packets once a batch has WG_TUNN_COPY_SPLIT
// (512) packets, and run on the caller below that (profiles/r05ai_*: 2-part copies were
// the slowest form, 256 packets copy faster alone, 512+ faster on every worker).
size_t env_count(const char *name, size_t dflt) {
  const char *e = std::getenv(name);
  return e ? (size_t)std::max(1L, std::atol(e)) : dflt;
}
size_t grain_light() {
  static const size_t g = env_count("WG_TUNN_GRAIN_LIGHT", 1024);
  return g;
}
size_t grain_copy(size_t n) {
  static const size_t g = env_count("WG_TUNN_GRAIN_COPY", 64), split = env_count("WG_TUNN_COPY_SPLIT", 512);
  return n < split ? std::max<size_t>(n, 1) : g;
}
void copy_bytes(uint8_t *dst, const uint8_t *src, size_t n, bool nt) {
  if (!nt || n < 256) {
    std::memcpy(dst, src, n);
    return;
  }
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
  std::memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 48), d);
  }
  for (; i + 16 <= n; i += 16)
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i),
                     _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i)));
  std::memcpy(dst + i, src + i, n - i);
  _mm_sfence();  // streaming stores are weakly ordered: visible before the DMA / caller reads
}

// DMA batches' output (WG_TUNN_DMA_OUT, read per call): "direct" -- the AEAD kernel
// stores each packet's output straight into the caller's registered dst; "scatter" --
// into HBM staging, then a scatter kernel copies it out; unset -- direct for the chunks
// whose output runs sit on whole 128-byte lines of host memory (seal: the datagram at a
// line start; open, whose wire grid starts 16 bytes before the plaintext: dst at 16 past
// a line start), scatter for the others.  The kernels store 128-byte runs of 8 packets
// per instruction: on whole lines that writes host memory faster than the scatter's
// contiguous per-packet stores, across line boundaries slower (DESIGN.md section 4,
// profiles/r04al_align.jsonl).  Returns 0 scatter, 1 direct, 2 auto.
int dma_out_mode() {
  const char *e = std::getenv("WG_TUNN_DMA_OUT");
  if (e && std::strcmp(e, "scatter") == 0) return 0;
  if (e && std::strcmp(e, "direct") == 0) return 1;
  return 2;
}

// The chunk's output base for direct output: the lowest of the n device addresses
// addr(j) (each with its extent ext(j)), or 0 when direct output cannot take the chunk
// -- an address not 16-byte aligned (the descriptor kernels' alignment rule), with
// line >= 0 one not `line` bytes past a 128-byte line (auto mode), or a span the
// kernels' per-packet offsets cannot hold (2^43 bytes, 16-byte units in 40 bits)
template <class Addr, class Ext>
uint64_t direct_base(size_t n, Addr addr, Ext ext, int line = -1) {
  uint64_t lo = ~0ull, hi = 0;
  for (size_t j = 0; j < n; ++j) {
    const uint64_t a = addr(j);
    if (a & 15u) return 0;
    if (line >= 0 && (a & 127u) != (uint64_t)line) return 0;
    lo = std::min(lo, a);
    hi = std::max(hi, a + ext(j));
  }
  return n && hi - lo < (1ull << 43) ? lo : 0;
}

// Uniform decapsulate chunks through the strided text-grid open (WG_TUNN_STRIDED=1; off:
// into line-aligned slots it wrote host memory slower than the descriptor kernels +
// scatter, 255-261 vs 267-273 Gbit/s, profiles/r04st_*), read per call
bool dma_strided() {
  const char *e = std::getenv("WG_TUNN_STRIDED");
  return e && std::atoi(e) != 0;
}

// the DMA batches' scatter grid cap (WG_TUNN_SCATTER_BLOCKS, default 0: one block per 4
// jobs), read per call
uint32_t scatter_blocks() {
  const char *e = std::getenv("WG_TUNN_SCATTER_BLOCKS");
  return e ? (uint32_t)std::max(0, std::atoi(e)) : 0u;
}

// DMA batches on a copy, a kernel and an output stream (WG_TUNN_DMA_STREAMS=0: every
// stage of a chunk on its staging set's stream), read per call
bool dma_streams() {
  const char *e = std::getenv("WG_TUNN_DMA_STREAMS");
  return !e || std::atoi(e) != 0;
}

// DMA batches' chunk ramp (make_chunks; WG_TUNN_RAMP=1 turns it on: it measured
// nothing, profiles/r04u_tunn_ramp_ab.jsonl), read per call
bool dma_ramp() {
  const char *e = std::getenv("WG_TUNN_RAMP");
  return e && std::atoi(e) != 0;
}

size_t chunk_bytes() {  // staging bytes per pipeline chunk (WG_TUNN_CHUNK_KB overrides, per call)
  const char *e = std::getenv("WG_TUNN_CHUNK_KB");
  return e ? std::max<size_t>(64, (size_t)std::atol(e)) << 10 : size_t(16) << 20;
}
constexpr uint32_t kSets = 4;                     // staging sets per engine (at most)
// staging sets a pipeline uses (WG_TUNN_SETS overrides, 2..kSets): with n sets the
// host unpacks chunk c - (n - 1) right after submitting chunk c, so n - 1 chunks
// are queued on the GPU's streams while the host copies
uint32_t pipeline_sets() {  // (read per call, like chunk_bytes())
  const char *e = std::getenv("WG_TUNN_SETS");
  const int x = e ? std::atoi(e) : 2;
  return (uint32_t)std::min<int>(kSets, std::max(2, x));
}

// ---------------------------------------------------------------------------
// NUMA placement of an engine's host side (each GPU gets its own
// NUMA-local pinned staging and host threads).  Linux sysfs + raw syscalls:
// the GPU's node from its PCI device, the node's CPUs from its cpulist.
// ---------------------------------------------------------------------------
int device_numa_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return -1;
  for (char *c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
  char path[160];
  std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE *f = std::fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (std::fscanf(f, "%d", &node) != 1) node = -1;
  std::fclose(f);
  return node;
}

std::vector<int> node_cpus(int node) {
  std::vector<int> cpus;
  char path[96];
  std::snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE *f = std::fopen(path, "r");
  if (!f) return cpus;
  char buf[4096] = {0};
  const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
  std::fclose(f);
  buf[n] = 0;
  for (char *tok = std::strtok(buf, ",\n"); tok; tok = std::strtok(nullptr, ",\n")) {
    int a = 0, b = 0;
    const int k = std::sscanf(tok, "%d-%d", &a, &b);
    if (k == 1) b = a;
    if (k >= 1)
      for (int c = a; c <= b && c < CPU_SETSIZE; ++c) cpus.push_back(c);
  }
  return cpus;
}

// Pin the calling thread to the node's CPUs (intersected with what the process
// may use) and make its page allocations prefer that node; pinned staging is
// then allocated with hipHostMallocNumaUser so it follows this policy.
void bind_thread_to_node(int node) {
  if (node < 0) return;
  cpu_set_t allowed, want;
  CPU_ZERO(&want);
  if (sched_getaffinity(0, sizeof allowed, &allowed) == 0) {
    int hits = 0;
    for (int c : node_cpus(node))
      if (CPU_ISSET(c, &allowed)) {
        CPU_SET(c, &want);
        ++hits;
      }
    if (hits) (void)sched_setaffinity(0, sizeof want, &want);
  }
  unsigned long mask[16] = {0};
  if (node < (int)(sizeof mask * 8)) {
    mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
    (void)syscall(SYS_set_mempolicy, 1 /* MPOL_PREFERRED */, mask, sizeof mask * 8);
  }
}

// Persistent worker pool: run(n, fn) calls fn(lo, hi) over a split of [0, n) on the
// workers and the calling thread, and returns when all are done.  The pool belongs to
// an engine whose lanes run batch calls concurrently (one per peer's Tunn, from the
// caller's threads), so several run()s may be active at once: each is a job of parts
// that its caller and any idle worker claim one at a time (under the pool's lock; parts
// are a batch's sixteenths, so the lock is taken a few times per step), the workers
// taking turns over the active jobs.  A caller always works on its own job, so no
// step waits behind another lane's.
class Pool {
 public:
  Pool(unsigned workers, int node) : spin_ns_(spin_ns()) {
    for (unsigned i = 0; i < workers; ++i)
      th_.emplace_back([this, node] {
        bind_thread_to_node(node);
        loop();
      });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      agen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  unsigned size() const { return (unsigned)th_.size() + 1; }
  // (grain: the fewest items worth a part of their own)
  void run(size_t n, const std::function<void(size_t, size_t)> &fn, size_t grain) {
    const unsigned parts = (unsigned)std::min<size_t>(size(), std::max<size_t>(n / std::max<size_t>(grain, 1), 1));
    if (parts <= 1) {
      if (n) fn(0, n);
      return;
    }
    Job j;
    j.fn = &fn;
    j.n = n;
    j.parts = parts;
    j.left.store(parts, std::memory_order_relaxed);
    unsigned wake;
    {
      std::lock_guard<std::mutex> lk(mu_);
      active_.push_back(&j);
      agen_.fetch_add(1, std::memory_order_release);
      wake = std::min(sleepers_, parts - 1);  // (the spinning workers see agen_ change)
    }
    for (unsigned w = 0; w < wake; ++w) cv_.notify_one();
    // the caller's own parts first
    for (;;) {
      unsigned p;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (j.next >= j.parts) break;
        p = claim(&j);
      }
      part(j, p);
    }
    // the parts workers took: spin briefly (they are usually still running), then block
    const auto t0 = std::chrono::steady_clock::now();
    while (j.left.load(std::memory_order_acquire) != 0) {
      if (std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() >
          spin_ns_) {
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return j.left.load(std::memory_order_acquire) == 0; });
        break;
      }
      _mm_pause();
    }
  }

 private:
  struct Job {
    const std::function<void(size_t, size_t)> *fn = nullptr;
    size_t n = 0;
    unsigned parts = 0, next = 0;  // (next: under the pool's lock)
    std::atomic<unsigned> left{0};
  };
  // Workers spin this long for the next job before they block on the condition variable
  // (WG_TUNN_SPIN_US, default 20): a batch call runs several pool steps back to back,
  // and a blocked worker's wake-up costs tens of microseconds on a loaded host.
  static int64_t spin_ns() {
    const char *e = std::getenv("WG_TUNN_SPIN_US");
    return (e ? std::max(0, std::atoi(e)) : 20) * 1000ll;
  }
  // (under mu_) the next part of j; a job whose parts are all claimed leaves the list
  unsigned claim(Job *j) {
    const unsigned p = j->next++;
    if (j->next >= j->parts) active_.erase(std::find(active_.begin(), active_.end(), j));
    return p;
  }
  // run part p of j; the last part to finish wakes the job's caller (j may be gone
  // as soon as `left` reaches 0: only the pool's own members are touched after it)
  void part(Job &j, unsigned p) {
    (*j.fn)(j.n * p / j.parts, j.n * (p + 1) / j.parts);
    if (j.left.fetch_sub(1, std::memory_order_acq_rel) == 1) {
      std::lock_guard<std::mutex> lk(mu_);  // (the caller may be about to block on done_)
      done_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = agen_.load(std::memory_order_acquire);
    size_t rr = 0;
    for (;;) {
      Job *j = nullptr;
      unsigned p = 0;
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (!active_.empty()) {
          j = active_[rr++ % active_.size()];
          p = claim(j);
        } else if (stop_) {
          return;
        }
      }
      if (j) {
        part(*j, p);
        continue;
      }
      // nothing to do: spin on the job generation, then block
      const auto t0 = std::chrono::steady_clock::now();
      while (agen_.load(std::memory_order_acquire) == seen &&
             std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() <
                 spin_ns_)
        _mm_pause();
      std::unique_lock<std::mutex> lk(mu_);
      if (!stop_ && active_.empty() && agen_.load(std::memory_order_acquire) == seen) {
        ++sleepers_;
        cv_.wait(lk, [&] { return stop_ || !active_.empty(); });
        --sleepers_;
      }
      seen = agen_.load(std::memory_order_acquire);
    }
  }
  const int64_t spin_ns_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::vector<Job *> active_;  // jobs with parts not yet claimed
  unsigned sleepers_ = 0;
  std::atomic<uint64_t> agen_{0};
  bool stop_ = false;
};

// One persistent driver thread of a multi-device engine (pinned to the GPU's
// NUMA node): submit() hands it a job, wait() returns the job's result.
class Driver {
 public:
  explicit Driver(int node) : th_([this, node] {
      bind_thread_to_node(node);
      loop();
    }) {}
  ~Driver() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void submit(std::function<int()> job) {
    std::lock_guard<std::mutex> lk(mu_);
    job_ = std::move(job);
    has_ = true;
    done_ = false;
    cv_.notify_all();
  }
  int wait() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return done_; });
    return rc_;
  }

 private:
  void loop() {
    for (;;) {
      std::function<int()> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || has_; });
        if (stop_) return;
        job = std::move(job_);
        has_ = false;
      }
      const int rc = job();
      std::lock_guard<std::mutex> lk(mu_);
      rc_ = rc;
      done_ = true;
      cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::function<int()> job_;
  bool has_ = false, done_ = true, stop_ = false;
  int rc_ = 0;
  std::thread th_;  // last: started after the members it uses
};

// Output scatter (DMA mode): a kernel copies each packet's output bytes from the
// device staging straight into the caller's registered buffer (zero-copy writes
// over PCIe: 54 GB/s device-to-host on MI355X against 30-38 GB/s for the copy
// engines, and it runs beside the copy engines' host-to-device input copies:
// 86 GB/s both ways, tools/microbench_dma.cpp, profiles/r04h_dma.jsonl).  Job:
// a_len bytes from a_base + a_off, then b_len bytes from b_base + b_off, to dst.
struct Scatter {
  uint64_t dst;    // device address of the caller's (registered) destination
  uint32_t a_off, a_len, b_off, b_len;
};

__global__ __launch_bounds__(256) void scatter_kernel(const Scatter *__restrict__ jobs, uint32_t m,
                                                      const uint8_t *__restrict__ a_base,
                                                      const uint8_t *__restrict__ b_base) {
  // one wave per job, the grid striding over the jobs: the launch may be capped so that
  // the next chunk's AEAD kernel finds free CUs beside it (run_dma)
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t j = blockIdx.x * 4u + (threadIdx.x >> 6); j < m; j += gridDim.x * 4u) {
    const Scatter sc = jobs[j];
    uint8_t *dst = reinterpret_cast<uint8_t *>(sc.dst);
    const uint8_t *a = a_base + sc.a_off, *b = b_base + sc.b_off;
    const uint32_t L = sc.a_len + sc.b_len;
    const bool aligned = (sc.dst & 15u) == 0 && (reinterpret_cast<uintptr_t>(a) & 15u) == 0;
    for (uint32_t o = 16u * lane; o < L; o += 1024u) {
      if (aligned && o + 16u <= sc.a_len) {  // a whole piece of segment a
        *reinterpret_cast<uint4 *>(dst + o) = *reinterpret_cast<const uint4 *>(a + o);
        continue;
      }
      uint8_t v[16];
#pragma unroll
      for (uint32_t q = 0; q < 16u; ++q) {
        const uint32_t x = o + q;
        v[q] = x < sc.a_len ? a[x] : (x < L ? b[x - sc.a_len] : 0u);
      }
      if ((sc.dst & 15u) == 0 && o + 16u <= L) {
        uint4 w;
        __builtin_memcpy(&w, v, 16);
        *reinterpret_cast<uint4 *>(dst + o) = w;
      } else {
        for (uint32_t q = 0; q < 16u && o + q < L; ++q) dst[o + q] = v[q];
      }
    }
  }
}

// one pinned + device buffer set of the pipeline
struct CombSlot {
  wg_packet_desc *desc = nullptr;  // pinned (host-written; inlined into the launch when small)
  int32_t *st = nullptr;           // pinned statuses
  uint32_t *h_flag = nullptr, *d_count = nullptr;
  uint32_t seq = 0;
  hipStream_t stream = nullptr;
  std::atomic<int> readers{0};  // calls of the launch that have not taken their statuses yet
};
struct Service;  // (the resident service of the small calls, below)
struct CombSeg {
  const wg_packet_desc *descs = nullptr;
  uint32_t n = 0, max_len = 0;
  uint64_t in_base = 0, out_base = 0;
  // the leader's answer
  std::atomic<int> ready{0};
  int rc = WG_RC_OK;
  CombSlot *slot = nullptr;
  uint32_t off = 0, seq = 0;
};
struct Staging {
  uint8_t *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
  wg_packet_desc *h_desc = nullptr, *d_desc = nullptr;
  struct Scatter *h_sc = nullptr;  // the output scatter's per-packet jobs (pinned, read by the kernel)
  int32_t *h_st = nullptr, *d_st = nullptr;
  size_t bytes = 0, descs = 0;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // phase timing: h2d / kernel / d2h edges
  bool timed = false;     // the chunk in flight recorded ev[]
  bool busy = false;      // work enqueued and not yet waited for
  // explicit-copy chunks: the pack hook copied the input itself (DMA runs out of
  // registered caller memory), the output is DMA'd by a hook (runs into
  // registered caller memory) or deferred until the in-order decisions (mid hook)
  bool in_dma = false, out_dma = false, defer_out = false;
  hipEvent_t done2 = nullptr;  // the deferred outputs (mid) have landed
  bool spec_ok = false;        // decapsulate DMA: outputs scattered on speculated decisions
  uint32_t nsc = 0;            // ... that many scatter jobs (h_sc)
  uint8_t stage = 0;           // run_chunks: kIdle / kSubmitted / kOutputs / kReady
  unsigned host_flags = hipHostMallocDefault;  // + hipHostMallocNumaUser on NUMA-bound engines
  // zero-copy chunks in the latency form: the kernel's completion word (pinned) and its
  // workgroup counter (HBM); `flagged`: the chunk in flight stores done_seq there
  uint32_t *h_flag = nullptr, *d_count = nullptr;
  uint32_t done_seq = 0;
  bool flagged = false;
  bool evented = true;  // `done` was recorded behind the chunk in flight
  // the chunk in flight went out in a combined launch (Combiner below): its word,
  // sequence number, statuses and slot are the combiner's
  CombSeg *comb = nullptr;
  CombSeg cseg;  // (this set's chunk, when it is posted to a combiner)
  // the chunk in flight was posted to the engine's resident service (Service below):
  // its slot and sequence number
  Service *srv = nullptr;
  uint32_t srv_slot = 0, srv_seq = 0;
};

void free_buffers(Staging &s) {
  (void)hipHostFree(s.h_in);
  (void)hipHostFree(s.h_out);
  (void)hipHostFree(s.h_desc);
  (void)hipHostFree(s.h_sc);
  (void)hipHostFree(s.h_st);
  (void)hipFree(s.d_in);
  (void)hipFree(s.d_out);
  (void)hipFree(s.d_desc);
  (void)hipFree(s.d_st);
  (void)hipHostFree(s.h_flag);
  (void)hipFree(s.d_count);
  s.h_flag = s.d_count = nullptr;
  s.h_in = s.h_out = s.d_in = s.d_out = nullptr;
  s.h_desc = s.d_desc = nullptr;
  s.h_sc = nullptr;
  s.h_st = s.d_st = nullptr;
  s.bytes = s.descs = 0;
}

// (WG_TUNN_STAGE_NC=1: packet staging as non-coherent pinned memory -- the kernels'
// zero-copy reads then fill whole L2 lines; an A/B of the small-call cap)
unsigned stage_data_flags(unsigned fl) {
  static const bool nc = [] {
    const char *e = std::getenv("WG_TUNN_STAGE_NC");
    return e && std::atoi(e) != 0;
  }();
  return nc ? (fl | hipHostMallocNonCoherent) : fl;
}

hipError_t reserve(Staging &s, size_t bytes, size_t descs) {
  hipError_t e = hipSuccess;
  const unsigned fl = s.host_flags;
  if (bytes > s.bytes) {
    (void)hipHostFree(s.h_in);
    (void)hipHostFree(s.h_out);
    (void)hipFree(s.d_in);
    (void)hipFree(s.d_out);
    s.h_in = s.h_out = s.d_in = s.d_out = nullptr;
    s.bytes = 0;
    if ((e = hipHostMalloc(&s.h_in, bytes, stage_data_flags(fl))) != hipSuccess) return e;
    if ((e = hipHostMalloc(&s.h_out, bytes, stage_data_flags(fl))) != hipSuccess) return e;
    if ((e = hipMalloc(&s.d_in, bytes)) != hipSuccess) return e;
    if ((e = hipMalloc(&s.d_out, bytes)) != hipSuccess) return e;
    s.bytes = bytes;
  }
  if (descs > s.descs) {
    (void)hipHostFree(s.h_desc);
    (void)hipHostFree(s.h_sc);
    (void)hipHostFree(s.h_st);
    (void)hipFree(s.d_desc);
    (void)hipFree(s.d_st);
    s.h_desc = s.d_desc = nullptr;
    s.h_sc = nullptr;
    s.h_st = s.d_st = nullptr;
    s.descs = 0;
    if ((e = hipHostMalloc(&s.h_desc, descs * sizeof(wg_packet_desc), fl)) != hipSuccess) return e;
    if ((e = hipHostMalloc(&s.h_sc, descs * sizeof(Scatter), fl)) != hipSuccess) return e;
    if ((e = hipHostMalloc(&s.h_st, descs * 4, fl)) != hipSuccess) return e;
    if ((e = hipMalloc(&s.d_desc, descs * sizeof(wg_packet_desc))) != hipSuccess) return e;
    if ((e = hipMalloc(&s.d_st, descs * 4)) != hipSuccess) return e;
    s.descs = descs;
  }
  return e;
}

struct Run {
  const uint8_t *host;
  uint64_t pitch, dev_off, dev_pitch;
  uint32_t width, rows;
};

// a contiguous range [k0, k1) of the selected packets and its staging bytes
struct Chunk {
  size_t k0, k1, bytes;
};

// Stable parallel compaction: emit(o, i) for every i in [0, n) with keep(i), o its
// rank among them, in blocks on the pool (count, prefix, fill); returns the count.
template <class Keep, class Emit>
size_t compact(Pool &pool, size_t n, Keep keep, Emit emit) {
  const size_t blocks = std::max<size_t>(1, std::min<size_t>(256, n / 2048));
  std::vector<size_t> cnt(blocks + 1, 0);
  auto lo_of = [&](size_t b) { return n * b / blocks; };
  pool.run(blocks, [&](size_t b0, size_t b1) {
    for (size_t b = b0; b < b1; ++b) {
      size_t c = 0;
      for (size_t i = lo_of(b); i < lo_of(b + 1); ++i) c += keep(i) ? 1 : 0;
      cnt[b + 1] = c;
    }
  }, 1);
  for (size_t b = 0; b < blocks; ++b) cnt[b + 1] += cnt[b];
  pool.run(blocks, [&](size_t b0, size_t b1) {
    for (size_t b = b0; b < b1; ++b) {
      size_t o = cnt[b];
      for (size_t i = lo_of(b); i < lo_of(b + 1); ++i)
        if (keep(i)) emit(o++, i);
    }
  }, 1);
  return cnt[blocks];
}

// copy threads per engine incl. its driver: WG_TUNN_THREADS, else the CPUs this
// process may run on (its affinity mask, not the machine: a GPU box grants a job a
// share of a larger host) split over the engines, at most 16
unsigned pool_workers(unsigned engines) {
  if (const char *e = std::getenv("WG_TUNN_THREADS")) return (unsigned)std::max(1, std::atoi(e)) - 1;
  cpu_set_t set;
  unsigned cpus = std::max(1u, std::thread::hardware_concurrency());
  if (sched_getaffinity(0, sizeof set, &set) == 0) cpus = std::max(1, CPU_COUNT(&set));
  return std::max(1u, std::min(16u, cpus / std::max(1u, engines))) - 1;
}

// per-call arrays of a batch (a lane's, reused by every Tunn that borrows it, or a
// multi-GPU Tunn's own): a Tunn keeps none of its batches' packet-sized state
struct Scratch {
  std::vector<uint32_t> sel, slot;
  std::vector<int32_t> code;           // pass 1: per packet, key slot if selected, else -1
  std::vector<uint64_t> ctr_all, ctr;  // datagram counters: per packet / per selected packet
  std::vector<uint8_t> act;            // per selected packet: what lands in dst (open_selected)
  std::vector<uint8_t> out_dma;        // per selected packet: its dst bytes were DMA'd (no host copy)
  std::vector<uint8_t> spec;           // per selected packet: speculated to land in dst (DMA decapsulate)
};

// The device side of a batch: one GPU context with its staging sets, streams
// and host copy threads.  As a lane of a shared engine (wg_engine) it is borrowed
// by one batch call at a time; a multi-GPU Tunn has one private engine per GPU it
// spreads batches over (wg_tunn_create_multi), each working on a contiguous range
// [k0, k1) of the batch's selected packets.
struct Engine {
  wg_gpu_ctx *ctx = nullptr;
  int device = 0, numa = -1;
  Staging st[kSets];
  Pool *pool = nullptr;
  bool own_pool = true;       // false: a lane of a shared engine (the engine's pool)
  Scratch scratch;            // the per-call arrays of the calls that borrow this lane
  wg_tunn *owner = nullptr;   // batch owner of the multi-peer calls on this lane
  Driver *driver = nullptr;   // multi-engine Tunns only (the single engine runs on the caller)
  wg_engine *grp = nullptr;   // a lane: its shared engine (combined small launches)
  size_t k0 = 0, k1 = 0;      // this batch's share of the selected packets
  std::vector<Chunk> chunks;
  std::vector<uint64_t> off;  // staging offset of selected packet k0 + j inside its chunk
  std::vector<uint64_t> dsrc, ddst;  // per selected packet: device addresses (direct mode)
  std::vector<uint64_t> reg;         // registered ranges (host, bytes, dev), snapshot per batch
  uint64_t tx = 0;                   // per-call tx_bytes share (summed by the caller)
  wg_tunn_phases ph{};               // this engine's share of the phase times
  bool timing = false;               // record device timing events (wg_tunn_set_phase_timing)
  bool zc = true;                    // this batch's chunks run zero-copy kernels (else explicit copies)
  std::vector<uint8_t> reg_in, reg_out;  // per packet of the share: host buffer registered (DMA runs)
  std::vector<Run> runs;             // scratch
  // DMA batches (run_dma): batch-sized pinned descriptors / statuses / scatter jobs, the
  // chunks' input runs, one completion event per chunk, and the repair path's staging
  wg_packet_desc *b_desc = nullptr;
  int32_t *b_st = nullptr;
  Scatter *b_jobs = nullptr;
  size_t b_cap = 0;
  std::vector<std::vector<Run>> chunk_runs;
  std::vector<hipEvent_t> cev;
  // DMA batches' copy and kernel streams (direct output): the input copies of chunk
  // c + 1 run under chunk c's kernel; per-chunk events order a chunk's stages and a
  // staging set's reuse
  hipStream_t dq[3] = {nullptr, nullptr, nullptr};
  std::vector<hipEvent_t> ev_in, ev_k;
  // direct-output chunks (the AEAD kernel writes the caller's registered dst itself):
  // per chunk 1 = direct, 0 = staged + scatter; and a pinned sink for the plaintext of
  // packets whose speculated decision keeps them out of dst (never read back)
  std::vector<uint8_t> chunk_direct;
  // decapsulate chunks of one length, one key slot and constant dst strides whose
  // packets all land: opened by the strided kernel (text grid on line-aligned plaintext
  // slots) straight into dst -- len == 0: not such a chunk
  struct StridedOpen {
    uint32_t len = 0, slot = 0;
    uint64_t dst = 0, dst_stride = 0;
  };
  std::vector<StridedOpen> chunk_strided;
  uint8_t *sink = nullptr;
  uint64_t sink_dev = 0;
  size_t sink_cap = 0;
  std::vector<void *> sink_old;  // outgrown sinks: kernels in flight may still write them
  Staging aux;
};

struct Combiner;  // (combined small launches, below)

}  // namespace

struct wg_tunn {
  uint32_t first_slot = 0;  // ring slot i: receiving key first_slot + 2i, sending first_slot + 2i + 1
  Session sessions[WG_N_SESSIONS];
  uint64_t current = 0;     // index of the most recently used session (mod.rs:69)
  uint64_t tx_bytes = 0, rx_bytes = 0;
  // timers[TimeCurrent] and timers.session_timers (timers.rs:91, :173-185): the
  // only timer state the data plane reads (set_current_session, mod.rs:530-538)
  uint64_t time_current = 0;
  uint64_t session_timers[WG_N_SESSIONS] = {};
  // the reference's Mutex<Tunn> (device/peer.rs:29): every call on the Tunn, and a
  // multi-peer call on each of its Tunns, holds it
  mutable std::mutex mu;
  wg_engine *group = nullptr;  // the shared engine (nullptr: private engines, wg_tunn_create_multi)
  std::vector<Engine *> eng;   // the private engines, or during a call the borrowed lane
  Scratch own;                 // per-call arrays of a Tunn with private engines
  Scratch *sc = &own;          // ... or, during a call, the borrowed lane's
  bool timing = false;         // wg_tunn_set_phase_timing
  wg_tunn_phases ph{};         // caller-side phases (checks, decide, totals)
  wg_tunn_phases ph_lanes{};   // the lanes' share of this Tunn's calls
  std::atomic<uint64_t> mark{0};  // multi-peer calls: collecting the distinct Tunns
  wg_replay spec_window[WG_N_SESSIONS];  // the speculation's replay windows (this call)
};

// A per-GPU engine shared by Tunns (include/neptun_tunn.h): one host pool, lanes
// made on demand and lent to one batch call at a time.
struct wg_engine {
  wg_gpu_ctx *ctx = nullptr;
  int device = 0;
  Pool *pool = nullptr;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Engine *> lanes, idle;
  uint32_t max_lanes = 8, tunns = 0;
  bool implicit = false;  // a context's default engine (wg_tunn_create): dies with its last Tunn
  // multi-peer calls over several engines (wg_tunn_*_multi with e == NULL): this
  // engine's share runs on its driver thread (made on first use, bound to the GPU's
  // NUMA node), held by one such call at a time
  Driver *driver = nullptr;
  std::mutex driver_mu;
  Combiner *comb[2] = {nullptr, nullptr};  // [seal]: small launches of concurrent calls
  std::mutex comb_mu;                             // (making them, and the service)
  Service *srv = nullptr;                         // resident service of the small calls
};

namespace {

inline double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

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

// longest descriptor length of a chunk (host-visible descriptors)
inline uint32_t max_desc_len(const wg_packet_desc *d, size_t m) {
  uint32_t x = 0;
  for (size_t i = 0; i < m; ++i) x = std::max(x, d[i].len);
  return x;
}

#define TUNN_HIP(call, what)                                              \
  do {                                                                    \
    hipError_t e_ = (call);                                               \
    if (e_ != hipSuccess) return wg_pipe_fail(WG_RC_HIP_ERROR, what, e_); \
  } while (0)

// per batch call: counts the call and its wall time (wg_tunn_get_phases);
// checks_done() ends the pass-1 phase
struct PhaseCall {
  wg_tunn *t;
  double t0, tc = -1.0;
  PhaseCall(wg_tunn *tt, uint32_t n) : t(tt), t0(now_us()) {
    t->ph.calls += 1;
    t->ph.packets += n;
  }
  void checks_done() {
    tc = now_us();
    t->ph.checks_us += tc - t0;
  }
  ~PhaseCall() { t->ph.total_us += now_us() - t0; }
};

// set_current_session (mod.rs:528-542): switch unless the current slot holds a
// session established later than the new one (session_timers compare)
void set_current_session(wg_tunn *t, uint64_t new_idx) {
  const uint64_t cur = t->current;
  if (cur == new_idx) return;
  if (!t->sessions[cur % WG_N_SESSIONS].live ||
      t->session_timers[new_idx % WG_N_SESSIONS] >= t->session_timers[cur % WG_N_SESSIONS])
    t->current = new_idx;
}

inline void set_err(wg_tunn_result &r, int32_t st) {
  std::memset(&r, 0, sizeof r);
  r.kind = WG_TUNN_ERR;
  r.status = st;
}

// device address of [p, p + n) inside memory registered with wg_gpu_register_host
// on this engine's context (E.reg: the batch's snapshot of its ranges)
// (hint: the range the caller's previous lookup hit, tried first -- consecutive packets
// of a pool mostly share one)
bool dev_addr(const Engine &E, const void *p, uint64_t n, uint64_t &dev, size_t &hint) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  if (hint < E.reg.size() / 3) {
    const uint64_t *r = &E.reg[3 * hint];
    if (a >= r[0] && a + n <= r[0] + r[1]) {
      dev = r[2] + (a - r[0]);
      return true;
    }
  }
  size_t lo = 0, hi = E.reg.size() / 3;  // first range with host > a
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (E.reg[3 * mid] <= a) lo = mid + 1;
    else hi = mid;
  }
  if (lo == 0) return false;
  const uint64_t *r = &E.reg[3 * (lo - 1)];
  if (a + n > r[0] + r[1]) return false;
  dev = r[2] + (a - r[0]);
  hint = lo - 1;
  return true;
}
bool dev_addr(const Engine &E, const void *p, uint64_t n, uint64_t &dev) {
  size_t hint = ~size_t(0);
  return dev_addr(E, p, n, dev, hint);
}

// every selected packet k in [a, b) passes ok(k, hint_a, hint_b) -- on the pool
template <class Ok>
bool all_packets(Engine &E, size_t a, size_t b, Ok ok) {
  std::atomic<bool> all{true};
  E.pool->run(b - a, [&](size_t lo, size_t hi) {
    size_t ha = ~size_t(0), hb = ~size_t(0);
    for (size_t j = lo; j < hi && all.load(std::memory_order_relaxed); ++j)
      if (!ok(a + j, ha, hb)) all.store(false, std::memory_order_relaxed);
  }, grain_light());
  return all.load();
}
template <class Ok>
bool all_packets(Engine &E, Ok ok) {
  return all_packets(E, E.k0, E.k1, ok);
}

// append the selected packets [a, b) to the engine's chunks (E.off indexed from E.k0)
template <class SizeFn>
void append_chunks(Engine &E, SizeFn size, size_t a, size_t b, size_t limit) {
  E.off.resize(b - E.k0);
  size_t k0 = a, bytes = 0;
  for (size_t k = a; k < b; ++k) {
    const uint64_t x = size(k);
    if (bytes && bytes + x > limit) {
      E.chunks.push_back(Chunk{k0, k, bytes});
      k0 = k;
      bytes = 0;
    }
    E.off[k - E.k0] = bytes;
    bytes += x;
  }
  if (k0 < b) E.chunks.push_back(Chunk{k0, b, bytes});
}

// cut the engine's selected packets (staging size `size(k)` each) into pipeline chunks;
// ramp (DMA batches, whose input copies of chunk c + 1 run under chunk c's kernel): the
// first chunks grow 1/8, 1/4, 1/2 of the limit and the tail is re-cut into halving
// pieces down to 1/8, so that the copy with no kernel under it at the start and the
// kernel with no copy under it at the end are short
template <class SizeFn>
void make_chunks(Engine &E, SizeFn size, size_t limit = 0, bool ramp = false) {
  if (!limit) limit = chunk_bytes();
  const size_t floor = std::max<size_t>(limit / 8, 1);
  auto lim = [&](size_t idx) { return ramp && idx < 3 ? std::max(floor, limit >> (3 - idx)) : limit; };
  E.chunks.clear();
  E.off.resize(E.k1 - E.k0);
  size_t k0 = E.k0, bytes = 0;
  for (size_t k = E.k0; k < E.k1; ++k) {
    const uint64_t b = size(k);
    if (bytes && bytes + b > lim(E.chunks.size())) {
      E.chunks.push_back(Chunk{k0, k, bytes});
      k0 = k;
      bytes = 0;
    }
    E.off[k - E.k0] = bytes;
    bytes += b;
  }
  if (k0 < E.k1) E.chunks.push_back(Chunk{k0, E.k1, bytes});
  if (!ramp || E.chunks.size() < 4) return;
  // re-cut the last two chunks: each piece half of what is left, until 1/8 of the limit
  const size_t a = E.chunks[E.chunks.size() - 2].k0;
  size_t left = E.chunks[E.chunks.size() - 2].bytes + E.chunks.back().bytes;
  E.chunks.resize(E.chunks.size() - 2);
  k0 = a;
  bytes = 0;
  size_t target = left > 2 * floor ? left / 2 : left;
  for (size_t k = a; k < E.k1; ++k) {
    const uint64_t b = size(k);
    if (bytes && bytes + b > target) {
      E.chunks.push_back(Chunk{k0, k, bytes});
      left -= bytes;
      k0 = k;
      bytes = 0;
      target = left > 2 * floor ? left / 2 : left;
    }
    E.off[k - E.k0] = bytes;
    bytes += b;
  }
  if (k0 < E.k1) E.chunks.push_back(Chunk{k0, E.k1, bytes});
}

// Split the selected packets [a, b) (default: all of them) into contiguous
// engine ranges of about equal staging bytes (size(k) per packet).
template <class SizeFn>
void split(wg_tunn *t, SizeFn size, size_t a = 0, size_t b = ~size_t(0)) {
  const size_t n = std::min(b, t->sc->sel.size()), E = t->eng.size();
  if (E == 1) {
    t->eng[0]->k0 = a;
    t->eng[0]->k1 = n;
    t->eng[0]->tx = 0;
    return;
  }
  uint64_t total = 0;
  for (size_t k = a; k < n; ++k) total += size(k);
  size_t k = a;
  uint64_t acc = 0;
  for (size_t e = 0; e < E; ++e) {
    t->eng[e]->k0 = k;
    const uint64_t goal = total * (e + 1) / E;
    while (k < n && (e + 1 == E || acc + size(k) / 2 < goal)) acc += size(k++);
    t->eng[e]->k1 = k;
    t->eng[e]->tx = 0;
  }
}

// Run job(E) for every engine: on the caller when there is one engine, else
// concurrently on the engines' NUMA-bound driver threads.  First error wins.
int for_engines(wg_tunn *t, const std::function<int(Engine &)> &job) {
  if (t->eng.size() == 1) {
    DevGuard g(t->eng[0]->device);  // staging is allocated on the current device
    return job(*t->eng[0]);
  }
  for (Engine *E : t->eng) {
    Engine *e = E;
    e->driver->submit([e, &job] {
      DevGuard g(e->device);
      return job(*e);
    });
  }
  int rc = WG_RC_OK;
  for (Engine *E : t->eng) {
    const int r = E->driver->wait();
    if (r && !rc) rc = r;
  }
  return rc;
}

// Zero-copy (default; WG_TUNN_ZEROCOPY=0 switches to explicit copies): the AEAD
// kernel reads the pinned input staging and writes the pinned output staging
// directly over PCIe, so reads and writes of a chunk share the link in both
// directions at once instead of running as H2D copy -> kernel -> D2H copy
// (measured: 143 / 156 vs 124 / 112 Gbit/s encap / decap, profiles/r01_tunn_*).
bool zero_copy() {  // (read per batch)
  const char *e = std::getenv("WG_TUNN_ZEROCOPY");
  return !e || std::atoi(e) != 0;
}

// direct mode is possible at all: zero-copy kernels and some registered memory
bool direct_possible(Engine &E) {
  if (!zero_copy()) return false;
  wg_ctx_reg_snapshot(E.ctx, E.reg);
  return !E.reg.empty();
}
// this batch moves registered buffers by DMA runs (explicit copies; one engine, or with
// multi_ok every engine of a multi-GPU Tunn on its own share)
bool dma_possible(wg_tunn *t, Engine &E, bool multi_ok = false);
// DMA runs (explicit-copy mode, registered caller memory): packets whose host
// buffers sit at a constant pitch with one length, and whose staging slots do
// too, move as ONE 2D copy (rows = packets) on the copy engines -- the way the
// pinned pipe reaches the link rate (wg_pipe.cpp) -- instead of a host memcpy
// into pinned staging.  WG_TUNN_DMA=0 turns it off.
bool dma_runs() {  // (read per batch, like the other WG_TUNN_* knobs)
  const char *e = std::getenv("WG_TUNN_DMA");
  return !e || std::atoi(e) != 0;
}
// Registered batches below this many packets take the zero-copy kernels on the caller's
// memory instead of a DMA batch: the copy engine's per-batch setup and completion cost
// more than the kernel's PCIe reads of a few MB (WG_TUNN_DMA_MIN, default 8192; 64 packets
// encapsulate 25 vs 37 us, decapsulate 34 vs 43; 4096: 346-385 vs 346-384 and 384-446 vs
// 445-476; equal at 16,384; profiles/r05q_small_reg.jsonl, r05ab_tunn_small_reg.jsonl).
// Registered decapsulate below dma_min(): the zero-copy open writes landing plaintexts
// straight into the registered dsts (WG_TUNN_DIRECT_OUT=0: into staging, copied out)
bool direct_out_small() {
  const char *e = std::getenv("WG_TUNN_DIRECT_OUT");
  return !e || std::atoi(e) != 0;
}
size_t dma_min() {
  const char *e = std::getenv("WG_TUNN_DMA_MIN");
  return e ? (size_t)std::max(0L, std::atol(e)) : 8192u;
}

// Cut packets [a, b) with use(k) into runs: host(k) pointer, width(k) bytes,
// dev(k) staging offset.  Returns false (runs unusable: too many small copies)
// when there are more than max_runs.
template <class Use, class Host, class Width, class Dev>
bool make_runs(size_t a, size_t b, Use use, Host host, Width width, Dev dev, size_t max_runs,
               std::vector<Run> &out) {
  out.clear();
  for (size_t k = a; k < b; ++k) {
    if (!use(k)) continue;
    const uint8_t *h = host(k);
    const uint32_t w = width(k);
    const uint64_t d = dev(k);
    if (!out.empty()) {
      Run &r = out.back();
      const uint8_t *last = r.host + r.pitch * (r.rows - 1);
      const uint64_t last_dev = r.dev_off + r.dev_pitch * (r.rows - 1);
      if (w == r.width && h > last && d > last_dev) {
        const uint64_t hp = (uint64_t)(h - last), dp = d - last_dev;
        if (r.rows == 1 && hp >= w && dp >= w) {
          r.pitch = hp;
          r.dev_pitch = dp;
          r.rows = 2;
          continue;
        }
        if (r.rows > 1 && hp == r.pitch && dp == r.dev_pitch) {
          ++r.rows;
          continue;
        }
      }
    }
    if (out.size() >= max_runs) return false;
    out.push_back(Run{h, w, d, w, w, 1});
  }
  return true;
}

hipError_t copy_runs(const std::vector<Run> &runs, uint8_t *dev_base, bool h2d, hipStream_t s) {
  for (const Run &r : runs) {
    hipError_t e;
    if (h2d)
      e = hipMemcpy2DAsync(dev_base + r.dev_off, r.dev_pitch, r.host, r.pitch, r.width, r.rows,
                           hipMemcpyHostToDevice, s);
    else
      e = hipMemcpy2DAsync(const_cast<uint8_t *>(r.host), r.pitch, dev_base + r.dev_off, r.dev_pitch,
                           r.width, r.rows, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
size_t max_runs(size_t m) { return std::max<size_t>(16, m / 16); }  // (16: the ramp's small chunks)

bool dma_possible(wg_tunn *t, Engine &E, bool multi_ok) {
  if (!dma_runs() || (!multi_ok && t->eng.size() != 1)) return false;
  wg_ctx_reg_snapshot(E.ctx, E.reg);
  return !E.reg.empty();
}

// Test-only fault injection: WG_TUNN_FAIL_CHUNK=c makes the batch fail with a
// HIP error right after chunk c has been enqueued (read per call).
int injected_failure(size_t c) {
  const char *e = std::getenv("WG_TUNN_FAIL_CHUNK");
  if (e && (size_t)std::atol(e) == c)
    return wg_pipe_fail(WG_RC_HIP_ERROR, "tunn: injected failure (WG_TUNN_FAIL_CHUNK)", hipSuccess);
  return WG_RC_OK;
}

// Every exit from run_chunks -- error paths included -- leaves both staging
// sets idle: work still queued on a set is waited for (its kernel may still be
// writing the pinned staging a later reserve() would free) and `busy` cleared,
// so the next batch starts from a clean pipeline.
// Small zero-copy calls learn that their kernel is done from the kernel's own
// completion word (a host spin: 6 us from launch for an empty kernel against 12 us
// through hipEventSynchronize, profiles/r05am_launch_latency.json) -- chunks of at
// most WG_TUNN_FLAG packets (default 128; 0: never).  Larger grids lose by it: every
// workgroup's system-scope release writes back its L2 (4096 packets staged 518 against
// 389 us, profiles/r05ao).  The event stays recorded behind the kernel: a word that has
// not come after 200 us (a slow or failed launch) hands over to the event, so errors
// surface.
bool flag_completion(size_t packets) {
  const char *e = std::getenv("WG_TUNN_FLAG");
  return packets <= (e ? (size_t)std::max(0L, std::atol(e)) : 128u);
}
// (WG_TUNN_WORD_EVENT=1: record the chunk's event behind a word-completed kernel too)
bool word_event() {
  const char *e = std::getenv("WG_TUNN_WORD_EVENT");
  return e && std::atoi(e) != 0;
}
hipError_t comb_wait(Staging &S, uint32_t m);
hipError_t srv_wait(Staging &S, uint32_t m);
hipError_t wait_chunk(Staging &S, uint32_t m) {
  if (S.comb) {
    S.flagged = false;
    return comb_wait(S, m);
  }
  if (S.srv) {
    S.flagged = false;
    return srv_wait(S, m);
  }
  if (S.flagged) {
    S.flagged = false;
    const volatile uint32_t *f = S.h_flag;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; ++i) {
      if (*f == S.done_seq) {
        std::atomic_thread_fence(std::memory_order_acquire);
        return hipSuccess;
      }
      if ((i & 255u) == 0u &&
          std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count() > 200)
        break;
      _mm_pause();
    }
  }
  return S.evented ? hipEventSynchronize(S.done) : hipStreamSynchronize(S.stream);
}

// Combined small launches.  NepTUN's workers each hand over at most 50 packets
// (packet_workers.rs:27) from up to num_cpus::get_physical() threads at once
// (:113-131).  Each such call is one latency-form launch -- a few microseconds of
// launch and a kernel bound by PCIe latency, not by its 50 packets -- so concurrent
// calls on one engine queue their launches behind each other.  A combiner per engine
// and direction merges them: a call posts its chunk (its descriptors, staging bases)
// and the first poster becomes the leader, which waits for a free launch slot (at most
// WG_COMBINE_DEPTH combined launches in flight: calls arriving meanwhile join the
// next one), takes every posted chunk, writes one descriptor array (absolute
// addresses) and makes ONE launch with one completion word for all of them; each
// call then waits for that word, copies its statuses and goes on with its own
// in-order decisions.  Per packet the kernel does exactly what the call's own launch
// would have done.  Off by default (WG_COMBINE=1 turns it on): measured at 8 threads
// x 50 packets it LOST -- 43 vs 53 Gbit/s staged, 38 vs 54 registered
// (profiles/r06d_tt_*): the calls' time is the kernel's PCIe round trips, which a
// shared launch does not shorten, and the slot wait (12 us) came on top.
constexpr uint32_t kCombSlots = 4, kCombMax = 2048, kCombSegMax = 256;
struct Combiner {
  std::mutex mu;
  std::vector<CombSeg *> pending;
  bool leader = false;
  CombSlot slot[kCombSlots];
  uint32_t next = 0;
  wg_gpu_ctx *ctx = nullptr;
  bool seal = false;
  std::atomic<uint32_t> shared_calls{0};  // chunks that went out in a launch with another call's
};

bool combine_on() {  // (read per call)
  const char *e = std::getenv("WG_COMBINE");
  return e && std::atoi(e) != 0;
}
uint32_t combine_depth() {  // combined launches in flight per engine and direction (1 .. kCombSlots)
  const char *e = std::getenv("WG_COMBINE_DEPTH");
  return e ? (uint32_t)std::min<long>(kCombSlots, std::max(1L, std::atol(e))) : 2u;
}

void comb_free(Combiner *C) {
  if (!C) return;
  for (CombSlot &S : C->slot) {
    if (S.stream) (void)hipStreamSynchronize(S.stream);
    (void)hipHostFree(S.desc);
    (void)hipHostFree(S.st);
    (void)hipHostFree(S.h_flag);
    (void)hipFree(S.d_count);
    if (S.stream) (void)hipStreamDestroy(S.stream);
  }
  delete C;
}

Combiner *comb_get(wg_engine *g, bool seal) {
  std::lock_guard<std::mutex> lk(g->comb_mu);
  if (Combiner *C = g->comb[seal ? 1 : 0]) return C;
  Combiner *C = new (std::nothrow) Combiner;
  if (!C) return nullptr;
  C->ctx = g->ctx;
  C->seal = seal;
  DevGuard dg(g->device);
  bool ok = true;
  for (CombSlot &S : C->slot) {
    ok = ok && hipHostMalloc((void **)&S.desc, kCombMax * sizeof(wg_packet_desc), hipHostMallocDefault) == hipSuccess;
    ok = ok && hipHostMalloc((void **)&S.st, kCombMax * 4, hipHostMallocDefault) == hipSuccess;
    ok = ok && hipHostMalloc((void **)&S.h_flag, 64, hipHostMallocCoherent) == hipSuccess;
    ok = ok && hipMalloc((void **)&S.d_count, 64) == hipSuccess;
    ok = ok && hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMemsetAsync(S.d_count, 0, 64, S.stream) == hipSuccess && hipStreamSynchronize(S.stream) == hipSuccess;
    if (ok) *S.h_flag = 0;
  }
  if (!ok) {
    comb_free(C);
    return nullptr;
  }
  g->comb[seal ? 1 : 0] = C;
  return C;
}

// the launch of slot S has completed (its word, or a stream sync after 200 us)
hipError_t comb_wait_word(const CombSlot &S, uint32_t seq) {
  const volatile uint32_t *f = S.h_flag;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1;; ++i) {
    if ((int32_t)(*f - seq) >= 0) {  // (this launch or a later one of the slot)
      std::atomic_thread_fence(std::memory_order_acquire);
      return hipSuccess;
    }
    if ((i & 255u) == 0u &&
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count() > 200)
      return hipStreamSynchronize(S.stream);
    _mm_pause();
  }
}

// One leader round: a free slot (at most `depth` launches in flight), every posted
// chunk that fits, one launch.  Called with C.mu held and C.leader set; returns with
// C.mu held.
void comb_launch_round(Combiner &C, std::unique_lock<std::mutex> &lk) {
  const uint32_t depth = combine_depth();
  CombSlot &S = C.slot[C.next % depth];
  lk.unlock();
  // the slot's previous launch done and its statuses taken (calls arriving meanwhile
  // join this round)
  (void)comb_wait_word(S, S.seq);
  while (S.readers.load(std::memory_order_acquire) != 0) _mm_pause();
  lk.lock();
  std::vector<CombSeg *> batch;
  uint32_t n = 0, max_len = 0;
  size_t k = 0;
  for (; k < C.pending.size(); ++k) {
    CombSeg *g = C.pending[k];
    if (n + g->n > kCombMax && n) break;
    batch.push_back(g);
    n += g->n;
    max_len = std::max(max_len, g->max_len);
  }
  C.pending.erase(C.pending.begin(), C.pending.begin() + (long)k);
  ++C.next;
  if (batch.size() > 1) C.shared_calls.fetch_add((uint32_t)batch.size(), std::memory_order_relaxed);
  lk.unlock();
  uint32_t off = 0;
  for (CombSeg *g : batch) {
    for (uint32_t j = 0; j < g->n; ++j) {
      wg_packet_desc d = g->descs[j];
      d.src_off += g->in_base;
      d.dst_off += g->out_base;
      S.desc[off + j] = d;
    }
    g->off = off;
    off += g->n;
  }
  const uint32_t seq = S.seq + 1;
  S.readers.store((int)batch.size(), std::memory_order_relaxed);
  bool flagged = false;
  int rc = wg_launch_desc_hinted(C.ctx, C.seal, S.desc, n, nullptr, nullptr, S.st, S.stream, max_len, true,
                                 S.d_count, S.h_flag, seq, &flagged, true, true);
  if (!rc && !flagged) {  // (not the latency form after all: the host publishes the word)
    const hipError_t e = hipStreamSynchronize(S.stream);
    if (e != hipSuccess) rc = wg_pipe_fail(WG_RC_HIP_ERROR, "tunn: combined launch", e);
    else *(volatile uint32_t *)S.h_flag = seq;
  }
  if (rc) S.readers.store(0, std::memory_order_relaxed);
  S.seq = seq;
  for (CombSeg *g : batch) {
    g->rc = rc;
    g->slot = &S;
    g->seq = seq;
    g->ready.store(1, std::memory_order_release);
  }
  lk.lock();
}

// post a chunk; returns once it is launched (g->slot / seq / off) or failed (g->rc)
int comb_submit(Combiner &C, CombSeg &g) {
  g.ready.store(0, std::memory_order_relaxed);
  g.rc = WG_RC_OK;
  std::unique_lock<std::mutex> lk(C.mu);
  C.pending.push_back(&g);
  for (;;) {
    if (!C.leader) {
      C.leader = true;
      // lead until this chunk is out (and whatever else is posted by then)
      while (!g.ready.load(std::memory_order_acquire) && !C.pending.empty()) comb_launch_round(C, lk);
      C.leader = false;
      return g.rc;
    }
    lk.unlock();
    for (uint32_t i = 0; !g.ready.load(std::memory_order_acquire); ++i) {
      _mm_pause();
      if ((i & 63u) == 63u) {  // the leader may have stepped down with this chunk still posted
        lk.lock();
        if (!C.leader && !g.ready.load(std::memory_order_acquire)) break;
        lk.unlock();
      }
    }
    if (g.ready.load(std::memory_order_acquire)) return g.rc;
  }
}

// the combined launch's completion for a chunk: its word, then its statuses
hipError_t comb_wait(Staging &S, uint32_t m) {
  CombSeg *g = S.comb;
  S.comb = nullptr;
  const hipError_t e = comb_wait_word(*g->slot, g->seq);
  if (e == hipSuccess) std::memcpy(S.h_st, g->slot->st + g->off, (size_t)m * 4);
  g->slot->readers.fetch_sub(1, std::memory_order_acq_rel);
  return e;
}

// ---------------------------------------------------------------------------
// Resident service of the small calls (wg_xlane.hip xlane_service_kernel).
//
// A launch per small call costs its ~5 us of launch and, with concurrent callers,
// its turn on the process's hardware queues: 8 threads x 50 packets held each call
// 25-28 us against 13-15 alone (profiles/r06d_tt).  A resident kernel does not: it
// polls kSrvSlots request slots in pinned host memory (a probe of the bare mechanism:
// 3.9 us from post to done, 3.7 M calls/s from 16 threads, other streams' kernels
// unaffected, profiles/r06l/doorbell_*.jsonl), and a call is a post -- its descriptors
// with absolute addresses, then the sequence number -- and a spin on the slot's done
// word.  Per packet the kernel runs xlane_packet exactly as the latency-form launches.
//
// Lifetime: the kernel's workgroups leave on *stop or when their lease (kSrvLeaseUs
// from their start) runs out.  A call posts only while the lease has more than
// kSrvMarginUs left on the host's clock (the kernel's workgroups started after the
// launch, so their leases end later); otherwise, or when the context's key table
// changed since the launch (a resident kernel may hold the old keys in its caches),
// the first caller to see it waits for the calls in flight, stops the kernel and
// launches the next.  A watchdog thread per service stops the kernel once no call has
// been posted for WG_TUNN_SRV_IDLE_US (1000): a resident kernel counts as device work
// to hipDeviceSynchronize, which therefore waits for the engine to go idle that long.
// The watchdog and a poster meet Dekker-style (live / inflight, sequentially
// consistent): a posted call's kernel is never stopped under it.
// Measured against the launches (profiles/r06n, r06o, r06r, r06s: 50 x 1350 B, 1 and 8
// threads, staged and registered): no launch, but the same ~12-15 us of PCIe-bound
// processing per request (device stamps), so 8 callers run 55-60 Gbit/s either way and
// one caller +0-13 %; meanwhile a resident kernel makes hipDeviceSynchronize and hipFree
// anywhere in the process wait for the engine's idle stop.  Off by default: WG_TUNN_SRV=1
// turns it on.
constexpr int64_t kSrvLeaseUs = 1000000, kSrvMarginUs = 5000;
int64_t srv_idle_us() {  // (read per watchdog round)
  const char *e = std::getenv("WG_TUNN_SRV_IDLE_US");
  return e ? std::max(100L, std::atol(e)) : 1000L;
}
int64_t srv_lease_us() {  // (WG_TUNN_SRV_LEASE_US: tests renew it often; read per launch)
  const char *e = std::getenv("WG_TUNN_SRV_LEASE_US");
  return e ? std::max(2000L, std::atol(e)) : kSrvLeaseUs;
}

struct Service {
  wg_gpu_ctx *ctx = nullptr;
  int device = 0;
  wg::SrvSlot *slots = nullptr;  // pinned, coherent
  uint32_t *stop = nullptr;      // pinned, coherent
  uint32_t *d_count = nullptr;   // HBM
  hipStream_t stream = nullptr;
  std::mutex mu;                 // restarts
  std::atomic<int> inflight{0};  // posted calls not yet waited for
  std::atomic<uint32_t> free_mask{(1u << wg::kSrvSlots) - 1u};
  std::atomic<bool> live{false};
  std::atomic<int64_t> post_until{0};  // steady-clock us: no post to the running kernel after
  std::atomic<uint64_t> key_gen{0};
  uint32_t seq[wg::kSrvSlots] = {};    // (each touched by its slot's holder only)
  std::atomic<uint64_t> calls{0}, launches{0};
  std::atomic<int64_t> last_post{0};   // steady-clock us
  std::thread watch;                   // the idle stop
  std::atomic<bool> quit{false};
  // WG_TUNN_SRV_STAMP=path (a diagnostic): per request the device's phase stamps and
  // the host's post-to-seen time, summed; written to path when the service ends
  const char *stamp_path = nullptr;
  std::mutex stamp_mu;
  double st_sum[10] = {};  // us: seen->acquired, ->packets, ->acked, ->published, device total, host total;
                           // packet 0: acquired->descriptor, ->staged, ->tag, ->stores issued
  uint64_t st_n = 0;
  int64_t post_us[wg::kSrvSlots] = {};
};

bool srv_on() {  // (read per call; off by default)
  const char *e = std::getenv("WG_TUNN_SRV");
  return e && std::atoi(e) != 0;
}
int64_t steady_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// every live service is told to stop at exit (host memory only: registered after the
// HIP runtime's own exit handlers, so it runs before them)
std::mutex g_srv_mu;
std::vector<Service *> g_srvs;
void srv_stamp_dump(Service *V);
void srv_atexit() {
  std::lock_guard<std::mutex> lk(g_srv_mu);
  bool any = false;
  for (Service *V : g_srvs) {
    srv_stamp_dump(V);
    V->st_n = 0;
  }
  for (Service *V : g_srvs) {  // (stopped by the watchdog and still draining counts too)
    __atomic_store_n(V->stop, 1u, __ATOMIC_RELEASE);
    V->live.store(false);
    any = true;
  }
  // the grids drained before the runtime tears the queues down (the workgroups see
  // *stop within a poll, ~2 us; bounded at 100 ms)
  const int64_t t0 = steady_us();
  while (any && steady_us() - t0 < 100000) {
    any = false;
    for (Service *V : g_srvs)
      if (V->stream && hipStreamQuery(V->stream) == hipErrorNotReady) any = true;
    if (any) std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}

// stop the kernel and wait (bounded) for its grid to drain; false: it did not
bool srv_halt(Service &V) {
  if (!V.stream) return true;
  __atomic_store_n(V.stop, 1u, __ATOMIC_RELEASE);
  V.live.store(false, std::memory_order_seq_cst);
  const int64_t t0 = steady_us();
  for (;;) {
    const hipError_t q = hipStreamQuery(V.stream);
    if (q != hipErrorNotReady) return true;  // (done, or the stream's error)
    if (steady_us() - t0 > 3 * kSrvLeaseUs) return false;
    std::this_thread::yield();
  }
}

void srv_watch(Service *V) {
  while (!V->quit.load(std::memory_order_acquire)) {
    std::this_thread::sleep_for(std::chrono::microseconds(250));
    const int64_t idle = srv_idle_us();
    if (!V->live.load(std::memory_order_acquire) || steady_us() - V->last_post.load() < idle) continue;
    std::lock_guard<std::mutex> lk(V->mu);
    if (!V->live.load() || steady_us() - V->last_post.load() < idle) continue;
    V->live.store(false, std::memory_order_seq_cst);
    if (V->inflight.load(std::memory_order_seq_cst) != 0) {  // (a post got in: keep it)
      V->live.store(true, std::memory_order_seq_cst);
      continue;
    }
    __atomic_store_n(V->stop, 1u, __ATOMIC_RELEASE);  // (the next post syncs the stream)
  }
}

void srv_stamp_dump(Service *V) {
  if (!V->stamp_path || !V->st_n) return;
  if (FILE *f = std::fopen(V->stamp_path, "a")) {
    const double n = (double)V->st_n;
    std::fprintf(f,
                 "{\"requests\": %llu, \"us\": {\"seen_to_acquired\": %.2f, \"acquired_to_packets\": %.2f, "
                 "\"packets_to_acked\": %.2f, \"acked_to_published\": %.2f, \"device_seen_to_published\": %.2f, "
                 "\"host_post_to_seen_done\": %.2f, \"pkt0_descriptor\": %.2f, \"pkt0_staged\": %.2f, "
                 "\"pkt0_keystream_mac\": %.2f, \"pkt0_store_issue\": %.2f}}\n",
                 (unsigned long long)V->st_n, V->st_sum[0] / n, V->st_sum[1] / n, V->st_sum[2] / n, V->st_sum[3] / n,
                 V->st_sum[4] / n, V->st_sum[5] / n, V->st_sum[6] / n, V->st_sum[7] / n, V->st_sum[8] / n,
                 V->st_sum[9] / n);
    std::fclose(f);
  }
}

void srv_free(Service *V) {
  if (!V) return;
  srv_stamp_dump(V);
  {
    std::lock_guard<std::mutex> lk(g_srv_mu);
    g_srvs.erase(std::remove(g_srvs.begin(), g_srvs.end(), V), g_srvs.end());
  }
  V->quit.store(true, std::memory_order_release);
  if (V->watch.joinable()) V->watch.join();
  DevGuard dg(V->device);
  if (!srv_halt(*V)) return;  // (a grid that does not drain keeps its memory: leaked, not freed under it)
  if (V->stream) (void)hipStreamDestroy(V->stream);
  (void)hipHostFree(V->slots);
  (void)hipHostFree(V->stop);
  (void)hipFree(V->d_count);
  delete V;
}

Service *srv_get(wg_engine *g) {
  std::lock_guard<std::mutex> lk(g->comb_mu);
  if (g->srv) return g->srv;
  Service *V = new (std::nothrow) Service;
  if (!V) return nullptr;
  V->ctx = g->ctx;
  V->device = g->device;
  DevGuard dg(g->device);
  bool ok = hipHostMalloc((void **)&V->slots, sizeof(wg::SrvSlot) * wg::kSrvSlots, hipHostMallocCoherent) == hipSuccess;
  ok = ok && hipHostMalloc((void **)&V->stop, 64, hipHostMallocCoherent) == hipSuccess;
  ok = ok && hipMalloc((void **)&V->d_count, wg::kSrvSlots * 32 * 4) == hipSuccess;
  ok = ok && hipStreamCreateWithFlags(&V->stream, hipStreamNonBlocking) == hipSuccess;
  ok = ok && hipMemsetAsync(V->d_count, 0, wg::kSrvSlots * 32 * 4, V->stream) == hipSuccess &&
       hipStreamSynchronize(V->stream) == hipSuccess;
  if (!ok) {
    srv_free(V);
    return nullptr;
  }
  std::memset(V->slots, 0, sizeof(wg::SrvSlot) * wg::kSrvSlots);
  *V->stop = 0;
  V->stamp_path = std::getenv("WG_TUNN_SRV_STAMP");
  {
    static std::once_flag once;
    std::call_once(once, [] { std::atexit(srv_atexit); });
    std::lock_guard<std::mutex> lk2(g_srv_mu);
    g_srvs.push_back(V);
  }
  V->watch = std::thread(srv_watch, V);
  g->srv = V;
  return V;
}

bool srv_stale(const Service &V) {
  return !V.live.load(std::memory_order_seq_cst) || steady_us() > V.post_until.load(std::memory_order_acquire) ||
         wg_ctx_key_gen(V.ctx) != V.key_gen.load(std::memory_order_acquire);
}

}  // namespace

// a context is being destroyed (wg_gpu.cpp): the services reading its key table stop first
void wg_srv_ctx_closing(wg_gpu_ctx *ctx) {
  std::lock_guard<std::mutex> lk(g_srv_mu);
  for (Service *V : g_srvs)
    if (V->ctx == ctx) {
      std::lock_guard<std::mutex> lk2(V->mu);
      DevGuard dg(V->device);
      (void)srv_halt(*V);
    }
}

namespace {

// a fresh kernel (the caller holds no inflight count)
int srv_restart(Service &V) {
  std::lock_guard<std::mutex> lk(V.mu);
  if (!srv_stale(V)) return WG_RC_OK;
  while (V.inflight.load(std::memory_order_acquire) != 0) _mm_pause();  // (posted calls finish first)
  DevGuard dg(V.device);
  // the previous kernel (live, or stopped by the watchdog and still draining) gone
  __atomic_store_n(V.stop, 1u, __ATOMIC_RELEASE);
  V.live.store(false, std::memory_order_seq_cst);
  TUNN_HIP(hipStreamSynchronize(V.stream), "tunn: service stop");
  // a request left unanswered (a failed wait) is withdrawn: the next kernel starts from
  // every slot's done word and must not find an old sequence number waiting there
  for (uint32_t k = 0; k < wg::kSrvSlots; ++k) {
    const uint32_t done = __atomic_load_n(&V.slots[k].done, __ATOMIC_ACQUIRE);
    __atomic_store_n(&V.slots[k].seq, done, __ATOMIC_RELEASE);
    V.seq[k] = done;
  }
  __atomic_store_n(V.stop, 0u, __ATOMIC_RELEASE);
  TUNN_HIP(hipMemsetAsync(V.d_count, 0, wg::kSrvSlots * 32 * 4, V.stream), "tunn: service counters");
  // (a key update that completes after this read is seen as a new generation next time)
  const uint64_t gen = wg_ctx_key_gen(V.ctx);
  const int64_t t_launch = steady_us(), lease = srv_lease_us();
  wg::SrvParams prm{V.slots, V.stop, V.d_count, wg_ctx_keys(V.ctx), wg_ctx_key_index(V.ctx),
                    wg_gpu_ctx_key_slots(V.ctx), (uint64_t)lease * 100u, V.stamp_path ? 1u : 0u};
  hipLaunchKernelGGL(wg::xlane_service_kernel, dim3(wg::kSrvSlots * wg::kSrvGroup), dim3(wg::kXlaneThreads), 0,
                     V.stream, prm);
  TUNN_HIP(hipGetLastError(), "tunn: service launch");
  V.key_gen.store(gen, std::memory_order_release);
  V.post_until.store(t_launch + lease - std::min(kSrvMarginUs, lease / 4), std::memory_order_release);
  V.last_post.store(t_launch);  // (the watchdog's idle clock starts now)
  V.live.store(true, std::memory_order_seq_cst);
  V.launches.fetch_add(1, std::memory_order_relaxed);
  return WG_RC_OK;
}

// lanes per packet for a request, chosen as the latency-form launches choose them
// (wg_gpu.cpp xlane_group_hinted) within the slot's kSrvLanes lanes and the kernel's
// G = 64 ... 8; 0: not a service request
uint32_t srv_group(uint32_t n, uint32_t max_len, bool seal) {
  if (n * 8u > wg::kSrvLanes) return 0u;
  const uint32_t P = seal ? max_len : (max_len > WG_DATA_OVERHEAD_SZ ? max_len - WG_DATA_OVERHEAD_SZ : 0u);
  const uint32_t nb = 1u + (P + 63u) / 64u;  // keystream blocks of the longest packet
  uint32_t g = 8u;
  while (g < nb && g < 64u) g *= 2u;
  uint32_t G = 64u;
  while (n * G > wg::kSrvLanes) G /= 2u;
  return std::min(G, g);
}

// Post chunk S (m packets, its descriptors relative to in / out) to the service.
// Returns WG_RC_OK (posted: S.srv set), 1 (not taken: no free slot or too large --
// the caller launches), or an error.
int srv_post(Service &V, Staging &S, bool seal, uint32_t m, const uint8_t *in, const uint8_t *out) {
  if (m == 0 || m > wg::kSrvDescs) return 1;
  const uint32_t G = srv_group(m, max_desc_len(S.h_desc, m), seal);
  if (!G) return 1;
  uint32_t fm = V.free_mask.load(std::memory_order_acquire), bit;
  do {
    if (!fm) return 1;
    bit = (uint32_t)__builtin_ctz(fm);
  } while (!V.free_mask.compare_exchange_weak(fm, fm & ~(1u << bit), std::memory_order_acq_rel));
  for (;;) {
    V.inflight.fetch_add(1, std::memory_order_seq_cst);
    if (!srv_stale(V)) break;
    V.inflight.fetch_sub(1, std::memory_order_seq_cst);
    if (const int rc = srv_restart(V)) {
      V.free_mask.fetch_or(1u << bit, std::memory_order_acq_rel);
      return rc;
    }
  }
  wg::SrvSlot &sl = V.slots[bit];
  const uint64_t ib = reinterpret_cast<uint64_t>(in), ob = reinterpret_cast<uint64_t>(out);
  for (uint32_t j = 0; j < m; ++j) {
    wg_packet_desc d = S.h_desc[j];
    d.src_off += ib;
    d.dst_off += ob;
    sl.d[j] = d;
  }
  sl.op = seal ? 1u : 0u;
  sl.n = m;
  sl.G = G;
  const uint32_t q = ++V.seq[bit];
  const int64_t tp = steady_us();
  V.last_post.store(tp, std::memory_order_relaxed);
  V.post_us[bit] = tp;
  __atomic_store_n(&sl.seq, q, __ATOMIC_RELEASE);
  S.srv = &V;
  S.srv_slot = bit;
  S.srv_seq = q;
  V.calls.fetch_add(1, std::memory_order_relaxed);
  return WG_RC_OK;
}

// the posted chunk's done word, then its statuses; the slot and the inflight count
// are given back on every path
hipError_t srv_wait(Staging &S, uint32_t m) {
  Service &V = *S.srv;
  S.srv = nullptr;
  wg::SrvSlot &sl = V.slots[S.srv_slot];
  hipError_t e = hipSuccess;
  const int64_t t0 = steady_us();
  for (uint32_t i = 1;; ++i) {
    if (__atomic_load_n(&sl.done, __ATOMIC_ACQUIRE) == S.srv_seq) break;
    if ((i & 1023u) == 0u) {
      const int64_t dt = steady_us() - t0;
      if (dt > 200) {  // (a slow answer: is the kernel still there?)
        const hipError_t q = hipStreamQuery(V.stream);
        if (q == hipSuccess) {  // ended without answering (never expected: see the lease)
          if (__atomic_load_n(&sl.done, __ATOMIC_ACQUIRE) == S.srv_seq) break;
          e = hipErrorLaunchFailure;
          break;
        }
        if (q != hipErrorNotReady) {
          e = q;
          break;
        }
        if (dt > 2 * std::max(kSrvLeaseUs, srv_lease_us())) {
          e = hipErrorLaunchTimeOut;
          break;
        }
      }
    }
    _mm_pause();
  }
  if (e == hipSuccess) {
    std::memcpy(S.h_st, sl.st, (size_t)m * 4);
    if (V.stamp_path) {
      const double host = (double)(steady_us() - V.post_us[S.srv_slot]);
      const uint64_t *t = sl.stamp;
      std::lock_guard<std::mutex> lk(V.stamp_mu);
      for (int k = 0; k < 4; ++k) V.st_sum[k] += (double)(t[k + 1] - t[k]) / 100.0;
      V.st_sum[4] += (double)(t[4] - t[0]) / 100.0;
      V.st_sum[5] += host;
      V.st_sum[6] += (double)(t[5] - t[1]) / 100.0;
      for (int k = 0; k < 3; ++k) V.st_sum[7 + k] += (double)(t[6 + k] - t[5 + k]) / 100.0;
      ++V.st_n;
    }
  } else {
    V.live.store(false, std::memory_order_release);  // (the next post restarts it)
  }
  V.inflight.fetch_sub(1, std::memory_order_acq_rel);
  V.free_mask.fetch_or(1u << S.srv_slot, std::memory_order_acq_rel);
  return e;
}

struct PipelineDrain {
  Engine &E;
  explicit PipelineDrain(Engine &e) : E(e) { drain(); }
  ~PipelineDrain() { drain(); }
  void drain() {
    for (auto &S : E.st)
      if (S.comb) {  // (an error path left a combined chunk unwaited: its kernel may still use the staging)
        CombSeg *g = S.comb;
        S.comb = nullptr;
        (void)comb_wait_word(*g->slot, g->seq);
        g->slot->readers.fetch_sub(1, std::memory_order_acq_rel);
      }
    for (auto &S : E.st)
      if (S.srv) (void)srv_wait(S, 0);  // (an error path left a posted chunk unwaited)
    for (auto &S : E.st)
      if (S.busy) {
        (void)hipStreamSynchronize(S.stream);
        S.busy = false;
        S.stage = 0;
      }
    for (hipStream_t q : E.dq)
      if (q) (void)hipStreamSynchronize(q);
  }
};

// Pipeline driver over one engine: pack(c, S) fills set S for chunk c (descs +
// bytes), the GPU runs chunk c on S's stream, unpack(c, S) consumes the
// results.  abs_src / abs_dst: descriptors carry absolute device addresses of
// registered caller memory on that side (no staging bytes there).
struct NoHook {
  int operator()(const Chunk &, Staging &) const { return 0; }
};

// post_kernel(ch, S): after the kernel is enqueued (explicit-copy mode), may
// enqueue the output's DMA runs itself (S.out_dma).  mid(ch, S): once the chunk's
// statuses are on the host, before unpack, strictly in chunk order (the in-order
// decisions); returns 1 when it enqueued more device work (outputs that waited for
// its decisions: S.done2 then marks them), 0 if not, < 0 on a HIP error.
// Stages per chunk: submitted -> [status back] mid -> [outputs back] unpack.
// After chunk c is submitted the driver runs mid for chunk c - 1 and unpacks the
// chunks whose outputs are in flight one chunk longer (c - 2 when outputs waited
// for mid, else c - 1), so a chunk's deferred output copies overlap the next
// chunk's input copies and kernel instead of the host waiting for them.
enum : uint8_t { kIdle = 0, kSubmitted = 1, kOutputs = 2, kReady = 3 };

template <class Pack, class Unpack, class Post = NoHook, class Mid = NoHook>
int run_chunks(Engine &E, bool seal, Pack pack, Unpack unpack, bool abs_src = false,
               bool abs_dst = false, Post post_kernel = Post(), Mid mid = Mid()) {
  PipelineDrain drain_guard(E);
  const size_t nc = E.chunks.size();
  const size_t sets = pipeline_sets();
  const bool zc = E.zc;
  E.ph.chunks += nc;
  size_t next_mid = 0, next_unpack = 0;
  auto stage_mid = [&](size_t c) -> int {
    Staging &S = E.st[c % sets];
    const double a = now_us();
    TUNN_HIP(wait_chunk(S, (uint32_t)(E.chunks[c].k1 - E.chunks[c].k0)), "tunn: chunk wait");
    E.ph.wait_us += now_us() - a;
    const int mr = (int)mid(E.chunks[c], S);
    if (mr == -2)
      return wg_pipe_fail(WG_RC_HIP_ERROR, "tunn: a speculated replay decision was not kept", hipSuccess);
    if (mr < 0) return wg_pipe_fail(WG_RC_HIP_ERROR, "tunn: output copies", hipGetLastError());
    if (mr > 0) {  // outputs that waited for the in-order decisions
      if (S.timed) TUNN_HIP(hipEventRecord(S.ev[3], S.stream), "tunn: event");  // (d2h incl. the decide gap)
      TUNN_HIP(hipEventRecord(S.done2, S.stream), "tunn: event");
      S.stage = kOutputs;
    } else {
      S.stage = kReady;
    }
    return WG_RC_OK;
  };
  auto stage_unpack = [&](size_t c) -> int {
    Staging &S = E.st[c % sets];
    if (S.stage == kOutputs) {
      const double a = now_us();
      TUNN_HIP(hipEventSynchronize(S.done2), "tunn: chunk output wait");
      E.ph.wait_us += now_us() - a;
    }
    if (S.timed) {  // device time per stage (wg_tunn_set_phase_timing)
      float ms = 0.f;
      if (!zc && hipEventElapsedTime(&ms, S.ev[0], S.ev[1]) == hipSuccess) E.ph.dev_h2d_us += 1e3 * ms;
      if (hipEventElapsedTime(&ms, S.ev[1], S.ev[2]) == hipSuccess) E.ph.dev_kernel_us += 1e3 * ms;
      if (!zc && hipEventElapsedTime(&ms, S.ev[2], S.ev[3]) == hipSuccess) E.ph.dev_d2h_us += 1e3 * ms;
      S.timed = false;
    }
    S.busy = false;
    S.stage = kIdle;
    unpack(E.chunks[c], S);
    return WG_RC_OK;
  };
  // run mid for every chunk < c_mid and unpack every chunk < c_unpack (in order),
  // plus chunk c_unpack itself when its outputs did not wait for mid
  auto advance = [&](size_t c_mid, size_t c_unpack, bool ready_too) -> int {
    while (next_mid < c_mid)
      if (const int rc = stage_mid(next_mid++)) return rc;
    while (next_unpack < next_mid &&
           (next_unpack < c_unpack ||
            (ready_too && next_unpack == c_unpack && E.st[next_unpack % sets].stage == kReady)))
      if (const int rc = stage_unpack(next_unpack++)) return rc;
    return WG_RC_OK;
  };
  for (size_t c = 0; c < nc; ++c) {
    Staging &S = E.st[c % sets];
    if (S.busy)  // chunk c - sets still owns this set
      if (const int rc = advance(c - sets + 1, c - sets + 1, false)) return rc;
    const Chunk &ch = E.chunks[c];
    const size_t m = ch.k1 - ch.k0;
    const double pa = now_us();
    TUNN_HIP(reserve(S, (abs_src && abs_dst) ? 128 : ch.bytes + 128, m), "tunn: staging");
    S.in_dma = S.out_dma = S.defer_out = S.flagged = false;
    const bool timed = E.timing;
    if (timed && !S.ev[0])
      for (auto &e : S.ev) TUNN_HIP(hipEventCreate(&e), "tunn: timing event");
    if (!zc && timed) TUNN_HIP(hipEventRecord(S.ev[0], S.stream), "tunn: event");
    pack(ch, S);  // (may enqueue the chunk's input DMA runs: S.in_dma; ev[0] goes first)
    const double pb = now_us();
    E.ph.pack_us += pb - pa;
    if (zc) {
      const uint8_t *in = abs_src ? nullptr : S.h_in;
      uint8_t *out = abs_dst ? nullptr : S.h_out;
      if (timed) TUNN_HIP(hipEventRecord(S.ev[1], S.stream), "tunn: event");
      // (the latency form's completion word: the set's own, made on first use)
      const bool word = !timed && flag_completion(m);
      if (word && !S.h_flag) {
        TUNN_HIP(hipHostMalloc((void **)&S.h_flag, 64, hipHostMallocCoherent), "tunn: completion word");
        TUNN_HIP(hipMalloc((void **)&S.d_count, 64), "tunn: completion counter");
        TUNN_HIP(hipMemsetAsync(S.d_count, 0, 64, S.stream), "tunn: completion counter");
        *S.h_flag = 0;
        S.done_seq = 0;
      }
      // (a call of one chunk only: a caller never holds a slot's statuses while it
      // leads another round, whose slot may be that one)
      int posted = 1;  // (the engine's resident service took the chunk: 0)
      if (word && nc == 1 && E.grp && srv_on()) {
        if (Service *V = srv_get(E.grp)) {
          posted = srv_post(*V, S, seal, (uint32_t)m, in, out);
          if (posted < 0) return posted;
          if (posted == 0) S.flagged = true;
        }
      }
      if (posted == 0) {
        // (posted: no launch, no event -- srv_wait)
      } else if (word && nc == 1 && m <= kCombSegMax && E.grp && combine_on()) {
        // one launch with the engine's other small calls of this direction (Combiner)
        Combiner *C = comb_get(E.grp, seal);
        if (!C) return wg_pipe_fail(WG_RC_OUT_OF_MEMORY, "tunn: combiner", hipSuccess);
        S.cseg.descs = S.h_desc;
        S.cseg.n = (uint32_t)m;
        S.cseg.max_len = max_desc_len(S.h_desc, m);
        S.cseg.in_base = reinterpret_cast<uint64_t>(in);
        S.cseg.out_base = reinterpret_cast<uint64_t>(out);
        if (const int rc = comb_submit(*C, S.cseg)) return rc;
        S.comb = &S.cseg;
        S.flagged = true;
      } else {
        if (word) ++S.done_seq;
        // (the kernel reads the packets over PCIe: hint the latency form's choice)
        const int rc = wg_launch_desc_hinted(E.ctx, seal, S.h_desc, (uint32_t)m, in, out, S.h_st, S.stream,
                                             max_desc_len(S.h_desc, m), true, word ? S.d_count : nullptr,
                                             word ? S.h_flag : nullptr, S.done_seq, &S.flagged, true, true);
        if (rc) return rc;
      }
      if (timed) TUNN_HIP(hipEventRecord(S.ev[2], S.stream), "tunn: event");
    } else {
      if (!S.in_dma)
        TUNN_HIP(hipMemcpyAsync(S.d_in, S.h_in, ch.bytes, hipMemcpyHostToDevice, S.stream), "tunn: H2D");
      TUNN_HIP(hipMemcpyAsync(S.d_desc, S.h_desc, m * sizeof(wg_packet_desc),
                              hipMemcpyHostToDevice, S.stream),
               "tunn: descs H2D");
      if (timed) TUNN_HIP(hipEventRecord(S.ev[1], S.stream), "tunn: event");
      const int rc = wg_launch_desc_hinted(E.ctx, seal, S.d_desc, (uint32_t)m, S.d_in, S.d_out, S.d_st,
                                           S.stream, max_desc_len(S.h_desc, m), false);
      if (rc) return rc;
      if (timed) TUNN_HIP(hipEventRecord(S.ev[2], S.stream), "tunn: event");
      post_kernel(ch, S);  // (may DMA the outputs straight to registered dst: S.out_dma)
      if (!S.out_dma && !S.defer_out)
        TUNN_HIP(hipMemcpyAsync(S.h_out, S.d_out, ch.bytes, hipMemcpyDeviceToHost, S.stream),
                 "tunn: D2H");
      TUNN_HIP(hipMemcpyAsync(S.h_st, S.d_st, m * 4, hipMemcpyDeviceToHost, S.stream),
               "tunn: status D2H");
      if (timed) TUNN_HIP(hipEventRecord(S.ev[3], S.stream), "tunn: event");
    }
    // (a chunk on the completion word needs no event: its fallback syncs the stream)
    if (!S.flagged || word_event()) TUNN_HIP(hipEventRecord(S.done, S.stream), "tunn: event");
    S.evented = !S.flagged || word_event();
    S.busy = true;
    S.stage = kSubmitted;
    S.timed = timed;
    E.ph.submit_us += now_us() - pb;
    if (const int rc = injected_failure(c)) return rc;
    // overlap: with sets - 1 chunks still queued behind this one, decide the
    // oldest and unpack what has landed (see above)
    if (c + 2 >= sets)
      if (const int rc = advance(c + 2 - sets, c + 2 - sets > 0 ? c + 1 - sets : 0, true)) return rc;
  }
  return advance(nc, nc, true);
}

// DMA batch (registered buffers, one engine): unlike the staged pipeline, the host
// never waits for a chunk before enqueueing the next -- every chunk's input runs,
// descriptor copy, AEAD kernel, output scatter and status copy go onto the streams
// at once (the chunks take the staging sets round robin, and the streams' own order
// keeps a set's device buffers from being reused early), with the descriptors,
// statuses and scatter jobs in batch-sized pinned arrays; the host then takes each
// chunk's results in order as its event completes, overlapping the later chunks.
// fill(ch, j0, d_out) writes the chunk's descriptors (E.b_desc + j0) and scatter jobs
// and returns the AEAD kernel's dst base: d_out (the set's HBM staging; descriptors hold
// staging offsets, scatter jobs copy out) or a host base (direct output: descriptors
// hold the caller's dst relative to it, no jobs); done(ch, j0) consumes its statuses
// (E.b_st + j0).  Returns 1 (nothing done) when the
// batch does not qualify: a packet outside registered memory, or inputs that do not
// form few enough runs.
// the direct-output sink, at least `bytes` (pinned, device-mapped); false on failure
bool grow_sink(Engine &E, size_t bytes) {
  bytes = std::max<size_t>(bytes, 65536);  // (a UDP datagram's plaintext always fits)
  if (bytes <= E.sink_cap) return true;
  if (E.sink) E.sink_old.push_back(E.sink);  // freed with the engine, after its streams drain
  E.sink = nullptr;
  E.sink_cap = 0;
  void *p = nullptr, *d = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocMapped) != hipSuccess) return false;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    (void)hipHostFree(p);
    return false;
  }
  E.sink = static_cast<uint8_t *>(p);
  E.sink_dev = reinterpret_cast<uint64_t>(d);
  E.sink_cap = bytes;
  return true;
}

hipError_t reserve_batch(Engine &E, size_t n) {
  if (n <= E.b_cap) return hipSuccess;
  (void)hipHostFree(E.b_desc);
  (void)hipHostFree(E.b_st);
  (void)hipHostFree(E.b_jobs);
  E.b_desc = nullptr;
  E.b_st = nullptr;
  E.b_jobs = nullptr;
  E.b_cap = 0;
  const unsigned fl = E.st[0].host_flags;
  hipError_t e;
  if ((e = hipHostMalloc(&E.b_desc, n * sizeof(wg_packet_desc), fl)) != hipSuccess) return e;
  if ((e = hipHostMalloc(&E.b_st, n * 4, fl)) != hipSuccess) return e;
  if ((e = hipHostMalloc(&E.b_jobs, n * sizeof(Scatter), fl)) != hipSuccess) return e;
  E.b_cap = n;
  return hipSuccess;
}

// more() runs once, right after chunk 0 is enqueued: 0 -- it appended chunks (the rest
// of a batch whose selection was cut short to start the device early), 1 -- nothing to
// add, 2 -- the rest cannot take a DMA batch.  Returns WG_RC_OK, an error, 1 (the batch
// does not qualify, nothing done) or 2 (the chunks [0, E.chunks.size()) are done and
// the selected packets from E.k1 on are left for the caller).  n_cap bounds the
// packets of the whole batch (the batch arrays are sized for it up front).
// launch(c, S, stream) may run chunk c's AEAD itself: it returns -1 when it does not
// (the descriptor kernels then run), else the launch's rc.
template <class InHost, class InLen, class Fill, class Done, class More, class Launch>
int run_dma(Engine &E, bool seal, double t_prep, size_t n_cap, InHost in_host, InLen in_len, Fill fill, Done done,
            More more, Launch launch) {
  // (seal: the plaintext goes 16 bytes into its staging slot, NepTUN's layout; open: the datagram at 0)
  const uint64_t in_shift = seal ? WG_DATA_OFFSET : 0u;
  const size_t nc0 = E.chunks.size(), n = E.k1 - E.k0;
  if (!nc0) return WG_RC_OK;
  const bool may_grow = n_cap > n;
  // the inputs of every chunk as runs (else the staged pipeline takes the batch)
  // the input runs of chunks [c0, c1) (false: too many runs for copies)
  auto build_runs = [&](size_t c0, size_t c1) {
    E.chunk_runs.resize(c1);
    std::atomic<bool> runs_ok{true};
    E.pool->run(c1 - c0, [&](size_t lo, size_t hi) {
      for (size_t c = c0 + lo; c < c0 + hi; ++c) {
        const Chunk &ch = E.chunks[c];
        if (!make_runs(
                ch.k0, ch.k1, [](size_t) { return true; }, in_host, in_len,
                [&](size_t k) { return E.off[k - E.k0] + in_shift; }, max_runs(ch.k1 - ch.k0), E.chunk_runs[c]))
          runs_ok.store(false, std::memory_order_relaxed);
      }
    }, 1);
    return runs_ok.load();
  };
  // staging: the chunks there are, or a full chunk when more may come (the sets are
  // in use by then: they cannot grow)
  size_t max_bytes = may_grow ? chunk_bytes() : 0, max_m = may_grow ? chunk_bytes() / 128 + 1 : 0;
  for (const Chunk &ch : E.chunks) {
    max_bytes = std::max(max_bytes, ch.bytes);
    max_m = std::max(max_m, ch.k1 - ch.k0);
  }
  if (!build_runs(0, nc0)) return 1;
  PipelineDrain drain_guard(E);
  // outgrown direct-output sinks of earlier batches: their kernels have drained
  for (void *p : E.sink_old) (void)hipHostFree(p);
  E.sink_old.clear();
  const bool split_streams = dma_streams();
  const uint32_t scatter_cap = scatter_blocks();
  const bool split_scatter = std::getenv("WG_TUNN_SPLIT_SCATTER") != nullptr;  // (A/B only)
  // Staging sets (WG_TUNN_SETS overrides): decided by chunk 0's output form -- all kSets
  // when it takes the scatter, whose copy, kernel and scatter then overlap the neighbours'
  // (decapsulate into line-aligned slots 263-269 Gbit/s with 2 sets, 278-285 with 4),
  // 2 for direct output, which 4 sets slowed (profiles/r04se_sets.jsonl, r04f8_*).
  size_t sets = std::getenv("WG_TUNN_SETS") ? pipeline_sets() : 0;
  TUNN_HIP(reserve_batch(E, std::max(n, n_cap)), "tunn: batch arrays");
  // (each set reserved at its first use in the batch: no chunk of this batch holds it yet)
  TUNN_HIP(reserve(E.st[0], max_bytes + 128, max_m), "tunn: staging");
  auto events = [&](size_t count) -> hipError_t {
    for (auto *v : {&E.cev, &E.ev_in, &E.ev_k})
      while (v->size() < count) {
        hipEvent_t ev;
        if (const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming); e != hipSuccess) return e;
        v->push_back(ev);
      }
    return hipSuccess;
  };
  TUNN_HIP(events(nc0), "tunn: event");
  E.ph.prep_us += now_us() - t_prep;
  bool left_over = false;  // more() left the rest of the batch to the caller
  size_t next_done = 0;
  auto finish_one = [&](size_t c) {
    const Chunk &ch = E.chunks[c];
    done(ch, ch.k0 - E.k0);
  };
  for (size_t c = 0; c < E.chunks.size(); ++c) {
    const Chunk &ch = E.chunks[c];
    const size_t m = ch.k1 - ch.k0, j0 = ch.k0 - E.k0;
    if (c > 0 && c < sets) TUNN_HIP(reserve(E.st[c], max_bytes + 128, max_m), "tunn: staging");
    Staging &S = E.st[sets ? c % sets : 0];
    const double pa = now_us();
    uint8_t *const out_base = fill(ch, j0, S.d_out);
    const bool scatter = out_base == S.d_out;
    if (!sets) sets = scatter ? kSets : 2;  // (chunk 0)
    const double pb = now_us();
    E.ph.pack_us += pb - pa;
    // Direct output: the input copies on the copy stream, the kernel on the kernel
    // stream, so that chunk c + 1's copies run under chunk c's kernel (the two move data
    // in opposite directions).  Staged output: copies, kernel and scatter on the set's
    // stream -- splitting those too (the scatter on a third stream beside the next
    // chunk's kernel, its grid capped by WG_TUNN_SCATTER_BLOCKS) measured 3-15 % slower
    // (profiles/r04sc_scatter.jsonl).  WG_TUNN_DMA_STREAMS=0: every stage on the set's
    // stream.  Either way a set's reuse by chunk c waits for chunk c - sets.
    const bool split = split_streams && (!scatter || split_scatter);
    hipStream_t qi = split ? E.dq[0] : S.stream, qk = split ? E.dq[1] : S.stream, qo = split ? E.dq[2] : S.stream;
    if (c >= sets) TUNN_HIP(hipStreamWaitEvent(qi, E.cev[c - sets], 0), "tunn: set reuse");
    TUNN_HIP(copy_runs(E.chunk_runs[c], S.d_in, true, qi), "tunn: input runs");
    if (split) {
      TUNN_HIP(hipEventRecord(E.ev_in[c], qi), "tunn: event");
      TUNN_HIP(hipStreamWaitEvent(qk, E.ev_in[c], 0), "tunn: event wait");
    }
    // the kernel reads the descriptors from, and writes the statuses into, the pinned
    // batch arrays itself: no small copies, which the copy engine would take in
    // submission order -- chunk c + 1's descriptors behind chunk c's statuses, i.e.
    // behind chunk c's kernel
    int rc = launch(c, S, qk);
    if (rc < 0)
      // (decapsulate chunks keep the throughput open: the latency form's open cost
      // 262,144-packet registered batches 280 -> 233 Gbit/s, where the seal gains 279 ->
      // 296; profiles/r05ba)
      rc = wg_launch_desc_hinted(E.ctx, seal, E.b_desc + j0, (uint32_t)m, S.d_in, out_base, E.b_st + j0, qk,
                                 max_desc_len(E.b_desc + j0, m), false, nullptr, nullptr, 0, nullptr, seal);
    if (rc) return rc;
    if (scatter) {
      if (split) {
        TUNN_HIP(hipEventRecord(E.ev_k[c], qk), "tunn: event");
        TUNN_HIP(hipStreamWaitEvent(qo, E.ev_k[c], 0), "tunn: event wait");
      }
      const uint32_t blocks = (uint32_t)((m + 3) / 4);
      hipLaunchKernelGGL(scatter_kernel, dim3(scatter_cap ? std::min(blocks, scatter_cap) : blocks), dim3(256), 0,
                         qo, E.b_jobs + j0, (uint32_t)m, (const uint8_t *)S.d_out, (const uint8_t *)S.d_in);
      TUNN_HIP(hipGetLastError(), "tunn: scatter launch");
    }
    TUNN_HIP(hipEventRecord(E.cev[c], scatter ? qo : qk), "tunn: event");
    S.busy = true;
    E.ph.submit_us += now_us() - pb;
    if (const int rc2 = injected_failure(c)) return rc2;
    if (c == 0) {  // the rest of the batch (chunk 0 is on the device meanwhile)
      const double a = now_us();
      const size_t had = E.chunks.size(), k_had = E.k1;
      const int mr = more();
      if (mr == 0) {
        bool fits = true;
        for (size_t x = had; x < E.chunks.size(); ++x)
          fits = fits && E.chunks[x].bytes <= max_bytes && E.chunks[x].k1 - E.chunks[x].k0 <= max_m;
        if (!fits || !build_runs(had, E.chunks.size())) {
          E.chunks.resize(had);  // (the rest goes back to the caller)
          E.k1 = k_had;
          left_over = true;
        }
        TUNN_HIP(events(E.chunks.size()), "tunn: event");
      } else if (mr == 2) {
        left_over = true;
      }
      E.ph.prep_us += now_us() - a;
    }
    // take whatever has landed meanwhile, in order
    while (next_done < c && hipEventQuery(E.cev[next_done]) == hipSuccess) finish_one(next_done++);
  }
  const size_t nc = E.chunks.size();
  E.ph.chunks += nc;
  while (next_done < nc) {
    const double a = now_us();
    TUNN_HIP(hipEventSynchronize(E.cev[next_done]), "tunn: chunk wait");
    E.ph.wait_us += now_us() - a;
    finish_one(next_done++);
  }
  return left_over ? 2 : WG_RC_OK;
}

// parse_incoming_packet (mod.rs:139-199): 1 = data, 0 = handshake/cookie, <0 = -InvalidPacket
int parse_kind(const uint8_t *d, uint32_t L) {
  if (L < 4) return -WG_STATUS_INVALID_PACKET;
  const uint32_t type = ld32(d);
  if ((type == 1 && L == 148) || (type == 2 && L == 92) || (type == 3 && L == 64)) return 0;
  if (type != WG_MSG_DATA || L < WG_DATA_OVERHEAD_SZ) return -WG_STATUS_INVALID_PACKET;
  return 1;
}

// validate_decapsulated_packet (mod.rs:606-670) on the plaintext pt[..P]; returns
// what it adds to rx_bytes (the pool threads sum it, the caller adds it to the Tunn)
uint64_t validate(const uint8_t *pt, uint32_t P, wg_tunn_result &r) {
  if (P == 0) {
    r.kind = WG_TUNN_DONE;
    return WG_DATA_OVERHEAD_SZ;  // keepalive
  }
  uint32_t ip_len = 0;
  const uint8_t v = pt[0] >> 4;
  if (v == 4 && P >= 20) {
    ip_len = (uint32_t)pt[2] << 8 | pt[3];
    r.ip_version = 4;
    std::memcpy(r.src_ip, pt + 12, 4);
  } else if (v == 6 && P >= 40) {
    ip_len = ((uint32_t)pt[4] << 8 | pt[5]) + 40;
    r.ip_version = 6;
    std::memcpy(r.src_ip, pt + 8, 16);
  } else {
    set_err(r, WG_STATUS_INVALID_PACKET);
    return 0;
  }
  if (ip_len > P) {
    set_err(r, WG_STATUS_INVALID_PACKET);
    return 0;
  }
  r.kind = WG_TUNN_WRITE_TO_TUNNEL;
  r.len = ip_len;
  return (uint64_t)ip_len + WG_DATA_OVERHEAD_SZ;  // message_data_len, session.rs:357
}

// Open the selected datagrams.  decide(k, S, kk) runs in packet order on one
// thread (kk = index of packet k inside its chunk's staging S) and returns what
// lands in dst: 0 nothing, 1 plaintext + tag bytes, 2 zeros + tag bytes
// (session.rs:287-296: ct||tag copied into dst, opened in place, ring zeroes
// the plaintext on a tag mismatch), | kFinish when finish(k, plaintext, P) must
// run.  decide only touches the per-packet arrays (counters, statuses), so the
// in-order pass stays in cache; finish (validate_decapsulated_packet: reads the
// plaintext's IP header, fills the result, returns its rx_bytes share) runs with
// the byte copies on the pools.
//  * one engine: a double-buffered chunk pipeline; each chunk is decided as it
//    returns while the next runs on the GPU;
//  * several engines: the selection is cut into rounds of about
//    engines x chunk_bytes() staging bytes; in each round every engine opens
//    its share as one chunk (in parallel on its own GPU and NUMA node), then
//    the caller decides the round's packets in order, then every engine copies
//    its share out.  Pinned staging per engine stays one chunk whatever the
//    batch size (a 16M-packet batch over 2 GPUs needs no more than 1 GPU does).
constexpr uint8_t kFinish = 0x80;

// partial: t->sc->sel holds only the selection of the batch's first packets, and grow()
// appends the rest (in order) -- so that a registered DMA batch can put its first chunk
// on the device while the host is still checking the rest (pass 1); every other path
// grows the selection first.  n_cap: the batch's packet count.
template <class Decide, class Finish, class Speculate, class Grow>
int open_selected(wg_tunn *t, const uint8_t *const *datagram, const uint32_t *len,
                  uint8_t *const *dst, Decide decide, Finish finish, Speculate speculate, Grow grow,
                  bool partial, size_t n_cap) {
  const bool multi = t->eng.size() > 1;
  if (partial && (multi || !dma_runs())) {
    grow();
    partial = false;
  }
  auto size = [&](size_t k) { return round128(len[t->sc->sel[k]]); };
  if (!multi) split(t, size);
  t->sc->act.assign(t->sc->sel.size(), 0);
  t->sc->out_dma.assign(t->sc->sel.size(), 0);
  t->sc->spec.assign(t->sc->sel.size(), 0);
  auto grow_all = [&]() {  // the full selection, and the per-packet state sized for it
    if (!partial) return;
    grow();
    partial = false;
    t->sc->act.resize(t->sc->sel.size(), 0);
    t->sc->out_dma.resize(t->sc->sel.size(), 0);
    t->sc->spec.resize(t->sc->sel.size(), 0);
  };
  const bool nt = nt_copies(n_cap);
  std::atomic<uint64_t> rx{0};
  // what lands in dst from pinned staging (pt: the plaintext there), then finish
  auto copy_out = [&](Engine &E, const Chunk &ch, const uint8_t *h_out, const wg_packet_desc *h_desc) {
    const double a = now_us();
    E.pool->run(ch.k1 - ch.k0, [&](size_t lo, size_t hi) {
      uint64_t my_rx = 0;
      for (size_t kk = lo; kk < hi; ++kk) {
        const size_t k = ch.k0 + kk;
        const uint8_t a = t->sc->act[k];
        if (!a) continue;
        const uint32_t i = t->sc->sel[k];
        const uint32_t P = len[i] - WG_DATA_OVERHEAD_SZ;
        // plaintext (or ring's zeros): scattered into dst already, else in the pinned staging
        const bool in_dst = t->sc->out_dma[k];
        const uint8_t *pt = in_dst ? dst[i] : h_out + h_desc[kk].dst_off;
        if (!in_dst) {
          if ((a & 3) == 1) copy_bytes(dst[i], pt, P, nt);
          else std::memset(dst[i], 0, P);
          std::memcpy(dst[i] + P, datagram[i] + WG_DATA_OFFSET + P, WG_AEAD_SIZE);
        } else if (t->sc->out_dma[k] == 2) {  // direct output: the kernel wrote the plaintext only
          std::memcpy(dst[i] + P, datagram[i] + WG_DATA_OFFSET + P, WG_AEAD_SIZE);
        }
        if (a & kFinish) my_rx += finish(k, in_dst ? dst[i] : pt, P);
      }
      rx.fetch_add(my_rx, std::memory_order_relaxed);
    }, grain_copy(ch.k1 - ch.k0));
    E.ph.copy_out_us += now_us() - a;
  };
  auto decide_range = [&](size_t k0, size_t k1, const int32_t *st) {
    const double a = now_us();
    for (size_t k = k0; k < k1; ++k) t->sc->act[k] = decide(k, st[k - k0]);
    t->ph.decide_us += now_us() - a;
  };
  // Several engines over registered pools (multi_dma): every engine runs its share as a
  // DMA batch of its own, concurrently; the speculation is taken for the whole selection
  // in packet order first (pre_spec: it assumes every tag good, so it needs no result),
  // and each chunk's decisions, repairs and copy-out wait until every engine is back
  // (defer_done), then run in packet order.  inline_decide: the staged chunks decide as
  // they return (one engine; or a multi-GPU engine whose share could not take the DMA
  // batch, run on the caller in its turn).
  bool multi_dma = false, pre_spec = false, defer_done = false, inline_decide = !multi;
  int dma_err = WG_RC_OK;  // a chunk's results could not be taken (reported after the batch)
  // DMA batch (registered datagrams and destinations, one engine): run_dma with the
  // replay decisions speculated per chunk (every tag assumed good) so the plaintexts
  // are scattered into dst right behind the kernel.  The speculation never lands a
  // packet the real decisions would not -- a failed tag only removes replay marks, so
  // the speculative window is the stricter one -- and the kernel has zeroed a failed
  // packet's plaintext already, which is what lands for it (session.rs:290-296).  The
  // packets it missed (a counter the speculation saw taken by a packet whose tag then
  // failed) are opened again from their datagrams into E.aux's pinned staging and
  // copied out by the host.
  auto registered = [&](Engine &E, size_t a, size_t b) {  // datagrams and dsts of [a, b)
    E.ddst.resize(b - E.k0);
    return all_packets(E, a, b, [&](size_t k, size_t &ha, size_t &hb) {
      const uint32_t i = t->sc->sel[k];
      uint64_t unused;
      return dev_addr(E, datagram[i], len[i], unused, ha) &&
             dev_addr(E, dst[i], len[i] - WG_DATA_OFFSET, E.ddst[k - E.k0], hb);
    });
  };
  // a DMA chunk's results: in-order decisions, repairs of the packets the speculation
  // missed, validation and copy-out
  // after a speculated chunk's decisions: which outputs are in dst (landed: 2 = the
  // kernel wrote the plaintext, the tag still to write; 1 = all of it) and the repairs
  // of the packets the speculation missed; false (dma_err set) on an error
  auto settle = [&](Engine &E, const Chunk &ch, uint8_t landed) -> bool {
    std::vector<size_t> rep;
    for (size_t k = ch.k0; k < ch.k1; ++k) {
      const bool lands = (t->sc->act[k] & 3) != 0;
      if (lands && !t->sc->spec[k]) rep.push_back(k);
      t->sc->out_dma[k] = lands && t->sc->spec[k] ? landed : 0;
      if (!lands && t->sc->spec[k]) {  // (cannot happen: see above)
        dma_err = wg_pipe_fail(WG_RC_HIP_ERROR, "tunn: a speculated replay decision was not kept", hipSuccess);
        return false;
      }
    }
    if (!rep.empty()) {
      // open the missed packets again into pinned staging; their decisions stand
      Staging &A = E.aux;
      uint64_t bytes = 0;
      for (size_t k : rep) bytes += round128(len[t->sc->sel[k]]);
      if (const hipError_t e = reserve(A, bytes + 128, rep.size()); e != hipSuccess) {
        dma_err = wg_pipe_fail(WG_RC_HIP_ERROR, "tunn: repair staging", e);
        return false;
      }
      uint64_t o = 0;
      for (size_t r = 0; r < rep.size(); ++r) {
        const uint32_t i = t->sc->sel[rep[r]];
        std::memcpy(A.h_in + o, datagram[i], len[i]);
        A.h_desc[r] = wg_packet_desc{o, o + WG_DATA_OFFSET, 0, len[i], t->sc->slot[rep[r]]};
        o += round128(len[i]);
      }
      if (const int rc = wg_gpu_open_batch(E.ctx, A.h_desc, (uint32_t)rep.size(), A.h_in, A.h_out, A.h_st,
                                           A.stream)) {
        dma_err = rc;
        return false;
      }
      if (const hipError_t e = hipStreamSynchronize(A.stream); e != hipSuccess) {
        dma_err = wg_pipe_fail(WG_RC_HIP_ERROR, "tunn: repair open", e);
        return false;
      }
      for (size_t r = 0; r < rep.size(); ++r) {
        const size_t k = rep[r];
        const uint32_t i = t->sc->sel[k];
        const uint32_t P = len[i] - WG_DATA_OVERHEAD_SZ;
        if ((t->sc->act[k] & 3) == 1) std::memcpy(dst[i], A.h_out + A.h_desc[r].dst_off, P);
        else std::memset(dst[i], 0, P);
        std::memcpy(dst[i] + P, datagram[i] + WG_DATA_OFFSET + P, WG_AEAD_SIZE);
        t->sc->out_dma[k] = 1;  // (in dst now)
      }
    }
    return true;
  };
  auto done_chunk = [&](Engine &E, const Chunk &ch, size_t j0) -> void {
    if (dma_err) return;
    decide_range(ch.k0, ch.k1, E.b_st + j0);
    if (!settle(E, ch, E.chunk_direct[&ch - E.chunks.data()] ? 2 : 1)) return;
    copy_out(E, ch, nullptr, nullptr);
  };
  auto dma_batch = [&](Engine &E) -> int {
    const double t_prep = now_us();
    if (!multi_dma && (multi || n_cap < dma_min() || !dma_possible(t, E) || !registered(E, E.k0, E.k1))) {
      if (partial) {  // not for a DMA batch after all: the staged path takes the whole selection
        grow_all();
        split(t, size);
      }
      return 1;
    }
    make_chunks(E, size, 0, dma_ramp());
    const int out_mode = dma_out_mode();
    const bool strided_ok = out_mode == 2 && !wg_ctx_slot_padding(E.ctx) && dma_strided();
    E.chunk_direct.assign(E.chunks.size(), 0);
    E.chunk_strided.assign(E.chunks.size(), Engine::StridedOpen{});
    auto fill = [&](const Chunk &ch, size_t j0, uint8_t *d_out) -> uint8_t * {
      const double a = now_us();
      const size_t m = ch.k1 - ch.k0;
      uint32_t pmax = 0;
      for (size_t k = ch.k0; k < ch.k1; ++k) {  // (in packet order)
        if (!pre_spec) t->sc->spec[k] = speculate(k);
        if (!t->sc->spec[k]) pmax = std::max(pmax, len[t->sc->sel[k]] - (uint32_t)WG_DATA_OVERHEAD_SZ);
      }
      E.ph.pack_spec_us += now_us() - a;
      // direct output: the open kernel writes the plaintext of every packet the
      // speculation lands straight into its dst (the tag follows from the host, in
      // copy_out), and that of the others into the pinned sink
      const size_t c = &ch - E.chunks.data();
      // a chunk the strided text-grid open takes: every packet lands, one length and one
      // key slot, plaintext slots at a constant stride on whole 128-byte lines
      if (strided_ok && pmax == 0 && m >= 64) {
        const uint32_t L = len[t->sc->sel[ch.k0]], sl = t->sc->slot[ch.k0];
        const uint64_t d0 = E.ddst[j0], ds = m > 1 ? E.ddst[j0 + 1] - d0 : 0;
        bool uni = L >= WG_DATA_OVERHEAD_SZ && d0 % 128 == 0 && ds % 128 == 0 && ds >= L - WG_DATA_OVERHEAD_SZ &&
                   ds < (1ull << 25) && 63 * ds + L + 64 < (1ull << 31);
        for (size_t kk = 0; uni && kk < m; ++kk) {
          const size_t k = ch.k0 + kk;
          uni = t->sc->spec[k] && len[t->sc->sel[k]] == L && t->sc->slot[k] == sl && E.ddst[j0 + kk] == d0 + kk * ds;
        }
        if (uni) {
          E.chunk_strided[c] = Engine::StridedOpen{L, sl, d0, ds};
          E.chunk_direct[c] = 1;
          return reinterpret_cast<uint8_t *>(d0);  // (not d_out: no scatter)
        }
      }
      uint64_t base = 0;
      // (the sink target sits 16 bytes past a line, like the dsts auto mode takes)
      if (out_mode != 0 && (pmax + 16 <= E.sink_cap || grow_sink(E, pmax + 16))) {
        auto addr = [&](size_t kk) { return t->sc->spec[ch.k0 + kk] ? E.ddst[j0 + kk] : E.sink_dev + 16; };
        auto ext = [&](size_t kk) { return (uint64_t)len[t->sc->sel[ch.k0 + kk]] - WG_DATA_OVERHEAD_SZ; };
        base = direct_base(m, addr, ext, out_mode == 2 ? 16 : -1);
      }
      E.chunk_direct[&ch - E.chunks.data()] = base != 0;
      E.pool->run(m, [&](size_t lo, size_t hi) {
        for (size_t kk = lo; kk < hi; ++kk) {
          const size_t k = ch.k0 + kk, j = j0 + kk;
          const uint32_t i = t->sc->sel[k];
          const uint32_t P = len[i] - WG_DATA_OVERHEAD_SZ, o = (uint32_t)E.off[j] + WG_DATA_OFFSET;
          if (base) {
            E.b_desc[j] = wg_packet_desc{E.off[j], (t->sc->spec[k] ? E.ddst[j] : E.sink_dev + 16) - base, 0, len[i],
                                         t->sc->slot[k]};
          } else {
            E.b_desc[j] = wg_packet_desc{E.off[j], o, 0, len[i], t->sc->slot[k]};
            // plaintext then the received tag (ct||tag lands in dst, session.rs:287-289)
            E.b_jobs[j] = t->sc->spec[k] ? Scatter{E.ddst[j], o, P, o + P, WG_AEAD_SIZE} : Scatter{0, 0, 0, 0, 0};
          }
        }
      }, grain_light());
      return base ? reinterpret_cast<uint8_t *>(base) : d_out;
    };
    auto done = [&](const Chunk &ch, size_t j0) -> void {
      if (!defer_done) done_chunk(E, ch, j0);
    };
    auto more = [&]() -> int {
      if (!partial) return 1;
      const size_t had = t->sc->sel.size();
      grow_all();
      if (t->sc->sel.size() == had) return 1;
      if (!registered(E, had, t->sc->sel.size())) return 2;
      append_chunks(E, size, had, t->sc->sel.size(), chunk_bytes());
      E.k1 = t->sc->sel.size();
      E.chunk_direct.resize(E.chunks.size(), 0);
      E.chunk_strided.resize(E.chunks.size(), Engine::StridedOpen{});
      return 0;
    };
    auto launch = [&](size_t c, Staging &S, hipStream_t q) -> int {
      if (c >= E.chunk_strided.size() || !E.chunk_strided[c].len) return -1;
      const Chunk &ch = E.chunks[c];
      const Engine::StridedOpen &so = E.chunk_strided[c];
      // (staging offsets: one length, so packet kk sits at kk * round128(len))
      return wg_gpu_open_strided(E.ctx, (uint32_t)(ch.k1 - ch.k0), so.len, so.slot, S.d_in, round128(so.len),
                                 reinterpret_cast<uint8_t *>(so.dst), so.dst_stride, E.b_st + (ch.k0 - E.k0), q);
    };
    const int r = run_dma(
        E, false, t_prep, n_cap, [&](size_t k) { return datagram[t->sc->sel[k]]; },
        [&](size_t k) { return len[t->sc->sel[k]]; }, fill, done, more, launch);
    if (r == 1 && partial) {  // (nothing was done)
      grow_all();
      split(t, size);
    }
    return dma_err ? dma_err : r;
  };
  auto engine_job = [&](Engine &E) -> int {
    if (const int r = dma_batch(E); r == 2) {  // the rest of the batch: staged
      grow_all();
      E.k0 = E.k1;
      E.k1 = t->sc->sel.size();
    } else if (r != 1) {
      return r;
    }
    E.zc = zero_copy();
    make_chunks(E, size, inline_decide ? 0 : ~size_t(0));
    // direct input (zero-copy): every datagram 16-byte aligned inside registered memory
    bool direct = direct_possible(E);
    E.dsrc.resize(E.k1 - E.k0);
    for (size_t k = E.k0; direct && k < E.k1; ++k) {
      const uint32_t i = t->sc->sel[k];
      direct = (reinterpret_cast<uint64_t>(datagram[i]) & 15u) == 0 &&
               dev_addr(E, datagram[i], len[i], E.dsrc[k - E.k0]);
    }
    // direct output too (every dst registered and 16-byte aligned, one engine): the open
    // kernel writes each plaintext the speculated replay decisions land straight into
    // its dst and the others' into the pinned sink, as the DMA batches' direct output
    // does; the in-order decisions then only add the tags (and repair what the
    // speculation missed) -- no plaintext copy-out from staging
    bool dout = direct && inline_decide && direct_out_small();
    if (dout) {
      E.ddst.resize(E.k1 - E.k0);
      uint32_t pmax = 0;
      for (size_t k = E.k0; dout && k < E.k1; ++k) {
        const uint32_t i = t->sc->sel[k];
        dout = (reinterpret_cast<uint64_t>(dst[i]) & 15u) == 0 &&
               dev_addr(E, dst[i], len[i] - WG_DATA_OFFSET, E.ddst[k - E.k0]);
        pmax = std::max(pmax, len[i] - (uint32_t)WG_DATA_OVERHEAD_SZ);
      }
      dout = dout && (pmax + 16 <= E.sink_cap || grow_sink(E, pmax + 16));
    }
    auto pack = [&](const Chunk &ch, Staging &S) {
      if (dout) {  // (packet order)
        const double a = now_us();
        for (size_t k = ch.k0; k < ch.k1; ++k) t->sc->spec[k] = speculate(k);
        E.ph.pack_spec_us += now_us() - a;
      }
      E.pool->run(ch.k1 - ch.k0, [&](size_t lo, size_t hi) {
        for (size_t kk = lo; kk < hi; ++kk) {
          const size_t k = ch.k0 + kk, j = k - E.k0;
          const uint32_t i = t->sc->sel[k];
          if (dout) {
            S.h_desc[kk] = wg_packet_desc{E.dsrc[j], t->sc->spec[k] ? E.ddst[j] : E.sink_dev + 16, 0, len[i],
                                          t->sc->slot[k]};
          } else if (direct) {
            // dst is staging: the replay decision comes after the GPU (session.rs:279-300)
            S.h_desc[kk] = wg_packet_desc{E.dsrc[j], E.off[j] + WG_DATA_OFFSET, 0, len[i], t->sc->slot[k]};
          } else {
            copy_bytes(S.h_in + E.off[j], datagram[i], len[i], nt);
            S.h_desc[kk] = wg_packet_desc{E.off[j], E.off[j] + WG_DATA_OFFSET, 0, len[i], t->sc->slot[k]};
          }
        }
      }, direct ? grain_light() : grain_copy(ch.k1 - ch.k0));
    };
    // statuses are back: decide in packet order (the copies follow in unpack)
    auto mid = [&](const Chunk &ch, Staging &S) -> int {
      if (inline_decide) decide_range(ch.k0, ch.k1, S.h_st);  // (several engines: after all are back)
      if (dout && !dma_err) (void)settle(E, ch, 2);
      return 0;
    };
    auto unpack = [&](const Chunk &ch, Staging &S) {
      if (dout) {
        if (!dma_err) copy_out(E, ch, nullptr, nullptr);
      } else if (inline_decide) {
        copy_out(E, ch, S.h_out, S.h_desc);
      }
    };
    const int r = run_chunks(E, false, pack, unpack, direct, dout, NoHook(), mid);
    return r ? r : dma_err;
  };
  int rc = WG_RC_OK;
  if (multi) {
    // registered pools on every engine's share: one DMA batch per engine (see multi_dma)
    split(t, size);
    bool all = dma_runs() && n_cap >= dma_min();
    for (size_t e = 0; all && e < t->eng.size(); ++e) {
      Engine &E = *t->eng[e];
      DevGuard g(E.device);
      all = dma_possible(t, E, true) && registered(E, E.k0, E.k1);
    }
    if (all) {
      for (size_t k = 0; k < t->sc->sel.size(); ++k) t->sc->spec[k] = speculate(k);
      multi_dma = pre_spec = defer_done = true;
      std::vector<int> verdict(t->eng.size(), 1);
      rc = for_engines(t, [&](Engine &E) -> int {
        const size_t e = std::find(t->eng.begin(), t->eng.end(), &E) - t->eng.begin();
        E.zc = zero_copy();
        const int r = dma_batch(E);
        verdict[e] = r;
        return r == 1 ? WG_RC_OK : r;
      });
      // (a verdict-1 share re-runs as the staged pipeline: dma_batch must then decline
      // it at once rather than build its chunks and runs again)
      defer_done = multi_dma = false;
      // in packet order: each engine's DMA chunks, or -- a share whose input could not
      // move as runs (verdict 1) -- the staged pipeline on the caller, deciding inline
      for (size_t e = 0; !rc && e < t->eng.size(); ++e) {
        Engine &E = *t->eng[e];
        DevGuard g(E.device);
        if (verdict[e] == 1) {
          inline_decide = true;
          rc = engine_job(E);
          inline_decide = false;
        } else {
          for (const Chunk &ch : E.chunks) done_chunk(E, ch, ch.k0 - E.k0);
          if (dma_err) rc = dma_err;
        }
      }
      t->rx_bytes += rx.load();
      return rc;
    }
  }
  if (!multi) {
    rc = for_engines(t, engine_job);
  } else {
    // several engines: rounds of about engines x chunk_bytes() staging bytes
    const size_t n = t->sc->sel.size();
    const uint64_t cap = (uint64_t)chunk_bytes() * t->eng.size();
    for (size_t a = 0; a < n && !rc;) {
      size_t b = a;
      uint64_t acc = 0;
      while (b < n && (b == a || acc + size(b) <= cap)) acc += size(b++);
      split(t, size, a, b);
      rc = for_engines(t, engine_job);
      if (rc) break;
      // one chunk per engine, its results still in staging set 0; decided in
      // packet order (engine ranges are contiguous and ordered)
      for (Engine *E : t->eng)
        if (!E->chunks.empty()) decide_range(E->k0, E->k1, E->st[0].h_st);
      rc = for_engines(t, [&](Engine &E) -> int {
        if (!E.chunks.empty()) copy_out(E, E.chunks[0], E.st[0].h_out, E.st[0].h_desc);
        return WG_RC_OK;
      });
      a = b;
    }
  }
  t->rx_bytes += rx.load();
  return rc;
}

void destroy_engine(Engine *E) {
  if (!E) return;
  delete E->driver;  // joins the driver thread first
  {
    DevGuard g(E->device);
    if (E->aux.stream) (void)hipStreamSynchronize(E->aux.stream);
    for (hipStream_t q : E->dq)
      if (q) (void)hipStreamSynchronize(q);
    for (hipStream_t q : E->dq)
      if (q) (void)hipStreamDestroy(q);
    (void)hipHostFree(E->sink);
    for (void *p : E->sink_old) (void)hipHostFree(p);
    for (hipEvent_t ev : E->ev_in) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : E->ev_k) (void)hipEventDestroy(ev);
    (void)hipHostFree(E->b_desc);
    (void)hipHostFree(E->b_st);
    (void)hipHostFree(E->b_jobs);
    for (hipEvent_t ev : E->cev) (void)hipEventDestroy(ev);
    free_buffers(E->aux);
    if (E->aux.stream) (void)hipStreamDestroy(E->aux.stream);
    for (auto &S : E->st) {
      if (S.stream) (void)hipStreamSynchronize(S.stream);
      free_buffers(S);
      if (S.done) (void)hipEventDestroy(S.done);
      if (S.done2) (void)hipEventDestroy(S.done2);
      for (auto &e : S.ev)
        if (e) (void)hipEventDestroy(e);
      if (S.stream) (void)hipStreamDestroy(S.stream);
    }
  }
  if (E->own_pool) delete E->pool;
  delete E->owner;
  delete E;
}

// The HIP runtime spreads a process's streams over GPU_MAX_HW_QUEUES hardware queues
// (default 4) in creation order, and kernels of one hardware queue run one after
// another.  Every lane makes the same number of streams (a multiple of 4), so without
// care st[0] -- the stream of every single-chunk call -- of all lanes shares one or two
// queues: 8 concurrent 50-packet calls then ran on 2 queues, one after another
// (profiles/r05av trace).  A lane therefore makes its streams in an order rotated by
// its index, st[0] of lanes 0, 1, 2, 3 ... landing on consecutive queues.
unsigned hw_queues() {
  const char *e = std::getenv("GPU_MAX_HW_QUEUES");
  return e && std::atoi(e) > 0 ? (unsigned)std::atoi(e) : 4u;
}

// shared: the engine's pool (a lane), else the engine makes its own; rot: the lane's
// index (stream order, above)
int make_engine(wg_gpu_ctx *ctx, bool multi, unsigned engines, Engine **out, Pool *shared = nullptr,
                unsigned rot = 0) {
  Engine *E = new (std::nothrow) Engine;
  if (!E) return wg_pipe_fail(WG_RC_OUT_OF_MEMORY, "tunn_create: host alloc", hipSuccess);
  E->ctx = ctx;
  if (shared) {
    E->pool = shared;
    E->own_pool = false;
  }
  E->device = wg_ctx_device(ctx);
  if (multi) {
    E->numa = device_numa_node(E->device);
    for (auto &S : E->st) S.host_flags = E->numa >= 0 ? hipHostMallocNumaUser : hipHostMallocDefault;
  }
  DevGuard g(E->device);
  std::vector<hipStream_t *> streams;  // (st[0] first, then the rest, rotated below)
  for (auto &S : E->st) streams.push_back(&S.stream);
  streams.push_back(&E->aux.stream);
  for (hipStream_t &q : E->dq) streams.push_back(&q);
  const size_t ns = streams.size(), r = rot % hw_queues() % ns;
  for (size_t j = 0; j < ns; ++j)  // st[0] is made r-th
    if (const hipError_t e = hipStreamCreateWithFlags(streams[(j + ns - r) % ns], hipStreamNonBlocking);
        e != hipSuccess) {
      destroy_engine(E);
      return wg_pipe_fail(WG_RC_HIP_ERROR, "tunn_create: stream", e);
    }
  for (auto &S : E->st) {
    hipError_t e = hipEventCreateWithFlags(&S.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&S.done2, hipEventDisableTiming);
    if (e != hipSuccess) {
      destroy_engine(E);
      return wg_pipe_fail(WG_RC_HIP_ERROR, "tunn_create: event", e);
    }
  }
  if (!shared) E->pool = new (std::nothrow) Pool(pool_workers(engines), E->numa);
  if (multi && E->pool) E->driver = new (std::nothrow) Driver(E->numa);
  if (!E->pool || (multi && !E->driver)) {
    destroy_engine(E);
    return wg_pipe_fail(WG_RC_OUT_OF_MEMORY, "tunn_create: threads", hipSuccess);
  }
  *out = E;
  return WG_RC_OK;
}

// lanes of a shared engine: streams per lane (staging sets + repair + DMA streams)
constexpr uint32_t kLaneStreams = kSets + 1 + 3;

uint32_t engine_max_lanes() {  // WG_ENGINE_LANES (1..64, default 8), read when an engine is made
  const char *e = std::getenv("WG_ENGINE_LANES");
  return e ? (uint32_t)std::min(64, std::max(1, std::atoi(e))) : 8u;
}

// borrow a lane (made on first need, up to max_lanes; else wait for one)
int lane_acquire(wg_engine *g, Engine **out) {
  std::unique_lock<std::mutex> lk(g->mu);
  for (;;) {
    if (!g->idle.empty()) {
      *out = g->idle.back();
      g->idle.pop_back();
      return WG_RC_OK;
    }
    if (g->lanes.size() < g->max_lanes) {
      Engine *E = nullptr;
      if (const int rc = make_engine(g->ctx, false, 1, &E, g->pool, (unsigned)g->lanes.size())) return rc;
      E->grp = g;
      g->lanes.push_back(E);
      *out = E;
      return WG_RC_OK;
    }
    g->cv.wait(lk);
  }
}

void lane_release(wg_engine *g, Engine *E) {
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->idle.push_back(E);
  }
  g->cv.notify_one();
}

void add_lane_phases(wg_tunn_phases &to, const wg_tunn_phases &p) {
  to.chunks += p.chunks;
  to.pack_us += p.pack_us;
  to.submit_us += p.submit_us;
  to.wait_us += p.wait_us;
  to.copy_out_us += p.copy_out_us;
  to.dev_h2d_us += p.dev_h2d_us;
  to.dev_kernel_us += p.dev_kernel_us;
  to.dev_d2h_us += p.dev_d2h_us;
  to.pack_spec_us += p.pack_spec_us;
  to.prep_us += p.prep_us;
}

// A batch call's lane: a Tunn on a shared engine borrows one for the call (its
// engine list and per-call arrays point at the lane meanwhile); the lane's phase
// times go to the Tunn.  Private engines (multi-GPU Tunns): nothing to do.
struct Lease {
  wg_tunn *t;
  Engine *E = nullptr;
  int rc = WG_RC_OK;
  explicit Lease(wg_tunn *tt, Engine *lane = nullptr) : t(tt) {
    if (!t->group) return;
    if (lane) E = lane;
    else if ((rc = lane_acquire(t->group, &E)) != WG_RC_OK) return;
    E->timing = t->timing;
    E->ph = wg_tunn_phases{};
    t->eng.assign(1, E);
    t->sc = &E->scratch;
  }
  ~Lease() {
    if (!E) return;
    add_lane_phases(t->ph_lanes, E->ph);
    E->ph = wg_tunn_phases{};
    t->eng.clear();
    t->sc = &t->own;
    lane_release(t->group, E);
  }
};

// every context's default engine (wg_tunn_create)
std::mutex g_default_mu;
std::vector<std::pair<wg_gpu_ctx *, wg_engine *>> g_default;

int engine_make(wg_gpu_ctx *ctx, wg_engine **out) {
  wg_engine *g = new (std::nothrow) wg_engine;
  if (!g) return wg_pipe_fail(WG_RC_OUT_OF_MEMORY, "engine_create: host alloc", hipSuccess);
  g->ctx = ctx;
  g->device = wg_ctx_device(ctx);
  g->max_lanes = engine_max_lanes();
  g->pool = new (std::nothrow) Pool(pool_workers(1), -1);
  if (!g->pool) {
    delete g;
    return wg_pipe_fail(WG_RC_OUT_OF_MEMORY, "engine_create: threads", hipSuccess);
  }
  *out = g;
  return WG_RC_OK;
}

void engine_free(wg_engine *g) {
  srv_free(g->srv);
  for (Engine *E : g->lanes) destroy_engine(E);
  comb_free(g->comb[0]);
  comb_free(g->comb[1]);
  delete g->driver;
  delete g->pool;
  delete g;
}

int tunn_attach(wg_engine *g, uint32_t first_slot, wg_tunn **out) {
  if ((uint64_t)first_slot + 2 * WG_N_SESSIONS > wg_gpu_ctx_key_slots(g->ctx))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "tunn_create: needs 16 key slots", hipSuccess);
  wg_tunn *t = new (std::nothrow) wg_tunn;
  if (!t) return wg_pipe_fail(WG_RC_OUT_OF_MEMORY, "tunn_create: host alloc", hipSuccess);
  if (const int rc = wg_ctx_claim_slots(g->ctx, first_slot, 2 * WG_N_SESSIONS)) {
    delete t;
    return rc;
  }
  t->first_slot = first_slot;
  t->group = g;
  std::lock_guard<std::mutex> lk(g->mu);
  ++g->tunns;
  *out = t;
  return WG_RC_OK;
}

// The distinct Tunns of a multi-peer batch, sorted by address (the lock order);
// false if one is null or not attached to g.
bool collect_peers(wg_engine *g, uint32_t n, wg_tunn *const *peer, std::vector<wg_tunn *> &out) {
  static std::atomic<uint64_t> epoch{1};
  const uint64_t ep = epoch.fetch_add(1, std::memory_order_relaxed);
  out.clear();
  const wg_tunn *last = nullptr;
  for (uint32_t i = 0; i < n; ++i) {
    wg_tunn *p = peer[i];
    if (!p) return false;
    if (p == last) continue;
    last = p;
    // (a concurrent call may re-mark a Tunn: duplicates are removed below)
    if (p->mark.load(std::memory_order_relaxed) != ep) {
      p->mark.store(ep, std::memory_order_relaxed);
      out.push_back(p);
    }
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  for (const wg_tunn *p : out)
    if (p->group != g) return false;
  return true;
}

}  // namespace

extern "C" {

int wg_engine_create(wg_gpu_ctx *ctx, wg_engine **out) {
  if (!ctx || !out) return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "engine_create: null", hipSuccess);
  return engine_make(ctx, out);
}

int wg_engine_destroy(wg_engine *e) {
  if (!e) return WG_RC_OK;
  {
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->tunns || e->implicit)
      return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "engine_destroy: Tunns are still attached", hipSuccess);
  }
  engine_free(e);
  return WG_RC_OK;
}

int wg_engine_get_info(const wg_engine *e, wg_engine_info *out) {
  if (!e || !out) return WG_RC_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(const_cast<wg_engine *>(e)->mu);
  *out = wg_engine_info{};
  out->tunns = e->tunns;
  out->lanes = (uint32_t)e->lanes.size();
  out->max_lanes = e->max_lanes;
  out->pool_threads = e->pool->size();
  out->streams = out->lanes * kLaneStreams;
  {
    std::lock_guard<std::mutex> cl(const_cast<wg_engine *>(e)->comb_mu);
    for (const Combiner *C : e->comb)
      if (C) out->combined += C->shared_calls.load(std::memory_order_relaxed);
    if (const Service *V = e->srv) {
      out->served = V->calls.load(std::memory_order_relaxed);
      out->service_launches = V->launches.load(std::memory_order_relaxed);
    }
  }
  return WG_RC_OK;
}

int wg_tunn_create_on(wg_engine *e, uint32_t first_slot, wg_tunn **out) {
  if (!e || !out) return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "tunn_create_on: null", hipSuccess);
  return tunn_attach(e, first_slot, out);
}

wg_engine *wg_tunn_engine(const wg_tunn *t) { return t ? t->group : nullptr; }

int wg_tunn_create_multi(wg_gpu_ctx *const *ctxs, uint32_t nctx, uint32_t first_slot,
                         wg_tunn **out) {
  if (!ctxs || !out || nctx == 0 || nctx > WG_TUNN_MAX_ENGINES)
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "tunn_create: bad contexts", hipSuccess);
  for (uint32_t e = 0; e < nctx; ++e) {
    if (!ctxs[e]) return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "tunn_create: null context", hipSuccess);
    if ((uint64_t)first_slot + 2 * WG_N_SESSIONS > wg_gpu_ctx_key_slots(ctxs[e]))
      return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "tunn_create: needs 16 key slots", hipSuccess);
  }
  if (nctx == 1) return wg_tunn_create(ctxs[0], first_slot, out);  // (the context's shared engine)
  wg_tunn *t = new (std::nothrow) wg_tunn;
  if (!t) return wg_pipe_fail(WG_RC_OUT_OF_MEMORY, "tunn_create: host alloc", hipSuccess);
  t->first_slot = first_slot;
  for (uint32_t e = 0; e < nctx; ++e) {
    Engine *E = nullptr;
    int rc = make_engine(ctxs[e], nctx > 1, nctx, &E);
    if (!rc) {
      rc = wg_ctx_claim_slots(ctxs[e], first_slot, 2 * WG_N_SESSIONS);
      if (rc) destroy_engine(E);
    }
    if (rc) {
      wg_tunn_destroy(t);
      return rc;
    }
    t->eng.push_back(E);
  }
  *out = t;
  return WG_RC_OK;
}

int wg_tunn_create(wg_gpu_ctx *ctx, uint32_t first_slot, wg_tunn **out) {
  if (!ctx || !out) return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "tunn_create: null", hipSuccess);
  if ((uint64_t)first_slot + 2 * WG_N_SESSIONS > wg_gpu_ctx_key_slots(ctx))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "tunn_create: needs 16 key slots", hipSuccess);
  std::lock_guard<std::mutex> lk(g_default_mu);
  wg_engine *g = nullptr;
  for (auto &d : g_default)
    if (d.first == ctx) g = d.second;
  const bool made = g == nullptr;
  if (made) {
    if (const int rc = engine_make(ctx, &g)) return rc;
    g->implicit = true;
    g_default.emplace_back(ctx, g);
  }
  const int rc = tunn_attach(g, first_slot, out);
  if (rc && made) {
    g_default.pop_back();
    engine_free(g);
  }
  return rc;
}

int wg_tunn_destroy(wg_tunn *t) {
  if (!t) return WG_RC_OK;
  if (wg_engine *g = t->group) {
    wg_ctx_release_slots(g->ctx, t->first_slot);
    std::lock_guard<std::mutex> dl(g_default_mu);
    bool last;
    {
      std::lock_guard<std::mutex> lk(g->mu);
      last = --g->tunns == 0 && g->implicit;
    }
    if (last) {  // a context's default engine goes with its last Tunn
      for (size_t k = 0; k < g_default.size(); ++k)
        if (g_default[k].second == g) {
          g_default.erase(g_default.begin() + (long)k);
          break;
        }
      engine_free(g);
    }
  } else {
    for (Engine *E : t->eng) {
      wg_ctx_release_slots(E->ctx, t->first_slot);
      destroy_engine(E);
    }
  }
  delete t;
  return WG_RC_OK;
}

uint32_t wg_tunn_engines(const wg_tunn *t) {
  if (!t) return 0u;
  return t->group ? 1u : (uint32_t)t->eng.size();
}

int wg_tunn_engine_info(const wg_tunn *t, uint32_t engine, int *device, int *numa_node) {
  if (!t || engine >= wg_tunn_engines(t)) return WG_RC_INVALID_ARGUMENT;
  if (t->group) {
    if (device) *device = t->group->device;
    if (numa_node) *numa_node = -1;  // (a shared engine's pool is not bound)
    return WG_RC_OK;
  }
  if (device) *device = t->eng[engine]->device;
  if (numa_node) *numa_node = t->eng[engine]->numa;
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
  std::lock_guard<std::mutex> lk(t->mu);
  if (t->group) {  // (synchronous: the copy has landed when set_keys returns)
    DevGuard g(t->group->device);
    const int rc = wg_gpu_set_keys(t->group->ctx, t->first_slot + 2 * ring, 2, keys, idx, nullptr);
    if (rc) return rc;
  }
  for (Engine *E : t->eng) {  // every GPU holds the session's keys
    DevGuard g(E->device);
    const int rc = wg_gpu_set_keys(E->ctx, t->first_slot + 2 * ring, 2, keys, idx, E->st[0].stream);
    if (rc) return rc;
  }
  Session &s = t->sessions[ring];
  s = Session{};
  s.live = true;
  s.receiving_index = local_index;
  s.sending_index = peer_index;
  wg_replay_init(&s.window);
  // timer_tick_session_established (timers.rs:173-185)
  t->session_timers[ring] = t->time_current;
  if (make_current) set_current_session(t, local_index);
  return WG_RC_OK;
}

int wg_tunn_set_time(wg_tunn *t, uint64_t now) {
  if (!t) return WG_RC_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(t->mu);
  t->time_current = now;  // update_timers: timers[TimeCurrent] = now (timers.rs:228-233)
  return WG_RC_OK;
}

int wg_tunn_stats(const wg_tunn *t, uint64_t *tx_bytes, uint64_t *rx_bytes) {
  if (!t) return WG_RC_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(t->mu);
  if (tx_bytes) *tx_bytes = t->tx_bytes;
  if (rx_bytes) *rx_bytes = t->rx_bytes;
  return WG_RC_OK;
}

int wg_tunn_session_counters(const wg_tunn *t, uint32_t ring_slot, uint64_t *sending_counter,
                             wg_replay *window) {
  if (!t || ring_slot >= WG_N_SESSIONS) return WG_RC_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(t->mu);
  if (sending_counter) *sending_counter = t->sessions[ring_slot].sending_counter;
  if (window) *window = t->sessions[ring_slot].window;
  return WG_RC_OK;
}

// n x Tunn::encapsulate.  t: the batch owner (the Tunn of a single-Tunn call, whose
// lane / engines and per-call arrays the batch runs on; a lane's owner for a
// multi-peer call).  peer: nullptr (every packet is t's), or packet i's Tunn.
static int encap_impl(wg_tunn *t, wg_tunn *const *peer, uint32_t n, const uint8_t *const *src,
                      const uint32_t *src_len, uint8_t *const *dst, const uint32_t *dst_cap,
                      wg_tunn_result *res) {
  PhaseCall pc(t, n);
  const bool many = peer != nullptr;
  Session &s = t->sessions[t->current % WG_N_SESSIONS];  // mod.rs:310 (single-Tunn batches)
  const uint32_t slot = t->first_slot + 2 * (uint32_t)(t->current % WG_N_SESSIONS) + 1;
  // pass 1 (stateless checks, on the pool; the counters are reserved below) over
  // packets [lo, hi), appending to the selection
  t->sc->code.resize(n);
  t->sc->sel.clear();
  const bool live = s.live;
  auto live_of = [&](size_t i) {  // the packet's Tunn has a current session (mod.rs:310)
    if (!many) return live;
    const wg_tunn *T = peer[i];
    return T->sessions[T->current % WG_N_SESSIONS].live;
  };
  auto pass1 = [&](size_t lo0, size_t hi0) {
    t->eng[0]->pool->run(hi0 - lo0, [&](size_t lo, size_t hi) {
      for (size_t i = lo0 + lo; i < lo0 + hi; ++i) {
        t->sc->code[i] = -1;
        if ((uint64_t)src_len[i] + WG_DATA_OFFSET > dst_cap[i]) {  // encapsulate: dst[16..len+16]
          set_err(res[i], WG_STATUS_INVALID_LENGTH);
          continue;
        }
        if (!live_of(i)) {  // no session: the CPU Tunn queues the packet and starts a handshake
          std::memset(&res[i], 0, sizeof res[i]);
          res[i].kind = WG_TUNN_NOT_DATA;
          res[i].status = WG_STATUS_NO_CURRENT_SESSION;
        } else if ((uint64_t)src_len[i] + WG_DATA_OVERHEAD_SZ > dst_cap[i]) {  // session.rs:210-217
          set_err(res[i], WG_STATUS_INCORRECT_PACKET_LENGTH);
        } else {
          // until its chunk comes back a selected packet reads as failed (a batch that
          // errors part-way leaves no stale or zeroed results behind)
          set_err(res[i], WG_STATUS_CRYPTO_FAILED);
          t->sc->code[i] = 0;
          continue;
        }
        // mod.rs:296-299 copies src into dst[16..] before looking at the session
        std::memcpy(dst[i] + WG_DATA_OFFSET, src[i], src_len[i]);
      }
    }, grain_light());  // (payload copies only for packets not sent: rare)
    const size_t had = t->sc->sel.size();
    t->sc->sel.resize(had + (hi0 - lo0));
    t->sc->sel.resize(had + compact(
        *t->eng[0]->pool, hi0 - lo0, [&](size_t j) { return t->sc->code[lo0 + j] >= 0; },
        [&](size_t o, size_t j) { t->sc->sel[had + o] = (uint32_t)(lo0 + j); }));
  };
  // one fetch_add per batch (session.rs:219), BEFORE the split: every engine's
  // packets carry counters ctr0 + k (k: the packet's rank in the selection), disjoint
  // across GPUs.  A large batch on one engine checks its first sixteenth first, so that
  // a registered DMA batch puts that part's first chunk on the device while pass 1
  // covers the rest; the reservation grows with the selection.
  const uint64_t ctr0 = s.sending_counter;
  const size_t n0 = n >= 16384 && dma_runs() && t->eng.size() == 1 && !many ? n / 16 : n;
  pass1(0, n0);
  bool partial = n0 < n;
  auto grow = [&]() {
    if (!partial) return;
    partial = false;
    const double a = now_us();
    pass1(n0, n);
    s.sending_counter = ctr0 + t->sc->sel.size();
    t->ph.checks_us += now_us() - a;
  };
  if (!many) s.sending_counter = ctr0 + t->sc->sel.size();
  if (t->sc->sel.empty()) grow();
  if (t->sc->sel.empty()) return WG_RC_OK;
  if (many) {
    // each Tunn's counters in the order of its packets (session.rs:219 per packet), and
    // the key slot of its current session (mod.rs:310)
    Scratch &q = *t->sc;
    q.ctr.resize(q.sel.size());
    q.slot.resize(q.sel.size());
    for (size_t k = 0; k < q.sel.size(); ++k) {
      wg_tunn *T = peer[q.sel[k]];
      const uint32_t ring = (uint32_t)(T->current % WG_N_SESSIONS);
      q.ctr[k] = T->sessions[ring].sending_counter++;
      q.slot[k] = T->first_slot + 2 * ring + 1;
    }
  }
  // the sending counter and key slot of selected packet k
  auto ctr_of = [&](size_t k) -> uint64_t { return many ? t->sc->ctr[k] : ctr0 + k; };
  auto slot_of = [&](size_t k) -> uint32_t { return many ? t->sc->slot[k] : slot; };
  pc.checks_done();
  auto size = [&](size_t k) { return round128((uint64_t)src_len[t->sc->sel[k]] + WG_DATA_OVERHEAD_SZ); };
  split(t, size);
  const bool nt = nt_copies(n);
  const int rc = for_engines(t, [&](Engine &E) -> int {
    E.zc = zero_copy();
    // registered src and dst (one engine): the DMA batch -- plaintexts in as runs, the
    // datagrams scattered straight into dst, no host copies and no waits between chunks
    const double t_prep = now_us();
    auto registered = [&](size_t a, size_t b) {  // srcs and dsts of [a, b)
      E.ddst.resize(b - E.k0);
      return all_packets(E, a, b, [&](size_t k, size_t &ha, size_t &hb) {
        const uint32_t i = t->sc->sel[k];
        uint64_t unused;
        return dev_addr(E, src[i], src_len[i], unused, ha) &&
               dev_addr(E, dst[i], (uint64_t)src_len[i] + WG_DATA_OVERHEAD_SZ, E.ddst[k - E.k0], hb);
      });
    };
    auto grow_all = [&]() {  // the full selection on this (the only) engine
      if (!partial) return;
      grow();
      split(t, size);
    };
    int left = 1;  // run_dma's verdict: 1 nothing done, 2 the packets from E.k1 on are left
    // (encapsulate has no in-order decisions: every engine of a multi-GPU Tunn runs its
    // contiguous share as a DMA batch of its own, the counters reserved before the split)
    const bool dma_ok = dma_possible(t, E, true) && n >= dma_min();
    if (!dma_ok) grow_all();
    if (dma_ok) {
      const bool all = registered(E.k0, E.k1);
      if (all) {
        make_chunks(E, size, 0, dma_ramp());
        const int out_mode = dma_out_mode();
        auto fill = [&](const Chunk &ch, size_t j0, uint8_t *d_out) -> uint8_t * {
          const size_t m = ch.k1 - ch.k0;
          // direct output: the seal kernel writes each datagram into the caller's dst
          const uint64_t base = out_mode != 0 ? direct_base(
                                                    m, [&](size_t kk) { return E.ddst[j0 + kk]; },
                                                    [&](size_t kk) {
                                                      return (uint64_t)src_len[t->sc->sel[ch.k0 + kk]] + WG_DATA_OVERHEAD_SZ;
                                                    },
                                                    out_mode == 2 ? 0 : -1)
                                              : 0;
          E.pool->run(m, [&](size_t lo, size_t hi) {
            for (size_t kk = lo; kk < hi; ++kk) {
              const size_t k = ch.k0 + kk, j = j0 + kk;
              const uint32_t i = t->sc->sel[k];
              if (base) {
                E.b_desc[j] = wg_packet_desc{E.off[j] + WG_DATA_OFFSET, E.ddst[j] - base, ctr_of(k), src_len[i],
                                             slot_of(k)};
              } else {
                E.b_desc[j] = wg_packet_desc{E.off[j] + WG_DATA_OFFSET, E.off[j], ctr_of(k), src_len[i], slot_of(k)};
                E.b_jobs[j] = Scatter{E.ddst[j], (uint32_t)E.off[j], src_len[i] + WG_DATA_OVERHEAD_SZ, 0, 0};
              }
            }
          }, grain_light());
          return base ? reinterpret_cast<uint8_t *>(base) : d_out;
        };
        auto done = [&](const Chunk &ch, size_t j0) {
          const double a = now_us();
          std::atomic<uint64_t> tx{0};
          E.pool->run(ch.k1 - ch.k0, [&](size_t lo, size_t hi) {
            uint64_t my_tx = 0;
            for (size_t kk = lo; kk < hi; ++kk) {
              const uint32_t i = t->sc->sel[ch.k0 + kk];
              if (E.b_st[j0 + kk] != WG_STATUS_OK) {  // the GPU path has no other failure mode
                set_err(res[i], WG_STATUS_CRYPTO_FAILED);
                continue;
              }
              std::memset(&res[i], 0, sizeof res[i]);
              res[i].kind = WG_TUNN_WRITE_TO_NETWORK;
              res[i].len = src_len[i] + WG_DATA_OVERHEAD_SZ;
              my_tx += res[i].len;  // mod.rs:321
            }
            tx.fetch_add(my_tx, std::memory_order_relaxed);
          }, grain_light());
          E.tx += tx.load();
          E.ph.copy_out_us += now_us() - a;
        };
        auto more = [&]() -> int {
          if (!partial) return 1;
          const size_t had = t->sc->sel.size();
          grow();
          if (t->sc->sel.size() == had) return 1;
          if (!registered(had, t->sc->sel.size())) return 2;
          append_chunks(E, size, had, t->sc->sel.size(), chunk_bytes());
          E.k1 = t->sc->sel.size();
          return 0;
        };
        left = run_dma(
            E, true, t_prep, n, [&](size_t k) { return src[t->sc->sel[k]]; },
            [&](size_t k) { return src_len[t->sc->sel[k]]; }, fill, done, more,
            [](size_t, Staging &, hipStream_t) { return -1; });
        if (left != 1 && left != 2) return left;
      }
    }
    if (left == 2) {  // the rest of the batch takes the paths below
      grow();
      E.k0 = E.k1;
      E.k1 = t->sc->sel.size();
    } else {
      grow_all();
    }
    // direct mode (zero-copy, WG_TUNN_DMA=0): src and dst of every packet 16-byte aligned
    // inside memory registered on this engine -> the kernel reads the caller's plaintext and
    // writes the caller's datagram over PCIe, no host copies at all
    bool direct = direct_possible(E);
    E.dsrc.resize(E.k1 - E.k0);
    E.ddst.resize(E.k1 - E.k0);
    for (size_t k = E.k0; direct && k < E.k1; ++k) {
      const uint32_t i = t->sc->sel[k];
      const size_t j = k - E.k0;
      direct = ((reinterpret_cast<uint64_t>(src[i]) | reinterpret_cast<uint64_t>(dst[i])) & 15u) == 0 &&
               dev_addr(E, src[i], src_len[i], E.dsrc[j]) &&
               dev_addr(E, dst[i], (uint64_t)src_len[i] + WG_DATA_OVERHEAD_SZ, E.ddst[j]);
    }
    make_chunks(E, size, direct ? ~size_t(0) : 0);
    auto pack = [&](const Chunk &ch, Staging &S) {
      E.pool->run(ch.k1 - ch.k0, [&](size_t lo, size_t hi) {
        for (size_t kk = lo; kk < hi; ++kk) {
          const size_t k = ch.k0 + kk, j = k - E.k0;
          const uint32_t i = t->sc->sel[k];
          if (direct) {
            S.h_desc[kk] = wg_packet_desc{E.dsrc[j], E.ddst[j], ctr_of(k), src_len[i], slot_of(k)};
          } else {
            copy_bytes(S.h_in + E.off[j] + WG_DATA_OFFSET, src[i], src_len[i], nt);  // NepTUN slot layout
            S.h_desc[kk] = wg_packet_desc{E.off[j] + WG_DATA_OFFSET, E.off[j], ctr_of(k), src_len[i], slot_of(k)};
          }
        }
      }, direct ? grain_light() : grain_copy(ch.k1 - ch.k0));
    };
    auto unpack = [&](const Chunk &ch, Staging &S) {
      const double a = now_us();
      E.pool->run(ch.k1 - ch.k0, [&](size_t lo, size_t hi) {
        for (size_t kk = lo; kk < hi; ++kk) {
          const uint32_t i = t->sc->sel[ch.k0 + kk];
          const uint32_t w = src_len[i] + WG_DATA_OVERHEAD_SZ;
          if (S.h_st[kk] != WG_STATUS_OK) {  // the GPU path has no other failure mode
            set_err(res[i], WG_STATUS_CRYPTO_FAILED);
            continue;
          }
          // the whole dst[..P+32]: header, ciphertext, tag (dst[16..] held src before)
          if (!direct) copy_bytes(dst[i], S.h_out + S.h_desc[kk].dst_off, w, nt);
          std::memset(&res[i], 0, sizeof res[i]);
          res[i].kind = WG_TUNN_WRITE_TO_NETWORK;
          res[i].len = w;
        }
      }, direct ? grain_light() : grain_copy(ch.k1 - ch.k0));
      for (size_t kk = 0; kk < ch.k1 - ch.k0; ++kk)  // mod.rs:321
        if (S.h_st[kk] == WG_STATUS_OK) E.tx += src_len[t->sc->sel[ch.k0 + kk]] + WG_DATA_OVERHEAD_SZ;
      E.ph.copy_out_us += now_us() - a;
    };
    return run_chunks(E, true, pack, unpack, direct, direct);
  });
  for (Engine *E : t->eng) t->tx_bytes += E->tx;
  // a batch that failed while pass 1 still covered only its first part: the rest gets
  // pass 1 now, so every packet's result is this call's (selected ones read as failed,
  // their counters stay consumed like the rest of the failed batch's)
  if (rc) grow();
  if (many)  // tx_bytes of each packet's own Tunn (mod.rs:321)
    for (uint32_t i = 0; i < n; ++i)
      if (res[i].kind == WG_TUNN_WRITE_TO_NETWORK) peer[i]->tx_bytes += res[i].len;
  return rc;
}

// n x Tunn::decapsulate; t and peer as in encap_impl, peers: the distinct Tunns of a
// multi-peer batch
static int decap_impl(wg_tunn *t, wg_tunn *const *peer, const std::vector<wg_tunn *> *peers, uint32_t n,
                      const uint8_t *const *datagram, const uint32_t *len, uint8_t *const *dst,
                      const uint32_t *dst_cap, wg_tunn_result *res) {
  PhaseCall pc(t, n);
  const bool many = peer != nullptr;
  // pass 1 (stateless checks, reference order; on the pool): parse, session, dst
  // size, index -- and each datagram's counter, so the in-order pass never reads
  // the datagrams again.  Over packets [lo, hi), appending to the selection.
  t->sc->code.resize(n);
  t->sc->ctr_all.resize(n);
  t->sc->sel.clear();
  t->sc->slot.clear();
  t->sc->ctr.clear();
  auto pass1 = [&](size_t lo0, size_t hi0) {
    t->eng[0]->pool->run(hi0 - lo0, [&](size_t lo, size_t hi) {
      for (size_t i = lo0 + lo; i < lo0 + hi; ++i) {
        const uint8_t *d = datagram[i];
        const uint32_t L = len[i];
        std::memset(&res[i], 0, sizeof res[i]);
        t->sc->code[i] = -1;
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
        const wg_tunn *T = many ? peer[i] : t;  // (the packet's Tunn)
        const Session &s = T->sessions[ridx % WG_N_SESSIONS];
        int32_t e = WG_STATUS_OK;
        if (!s.live) e = WG_STATUS_NO_CURRENT_SESSION;                                 // mod.rs:553-556
        else if ((uint64_t)dst_cap[i] < L - WG_DATA_OFFSET) e = WG_STATUS_DESTINATION_BUFFER_TOO_SMALL;  // session.rs:271
        else if (ridx != s.receiving_index) e = WG_STATUS_WRONG_INDEX;                // session.rs:275
        if (e) { set_err(res[i], e); continue; }
        // until its chunk returns a selected packet reads as failed
        set_err(res[i], WG_STATUS_CRYPTO_FAILED);
        t->sc->code[i] = (int32_t)(T->first_slot + 2 * (ridx % WG_N_SESSIONS));
        t->sc->ctr_all[i] = ld64(d + 8);
      }
    }, grain_light());
    const size_t had = t->sc->sel.size();
    t->sc->sel.resize(had + (hi0 - lo0));
    t->sc->slot.resize(t->sc->sel.size());
    t->sc->ctr.resize(t->sc->sel.size());
    const size_t got = compact(
        *t->eng[0]->pool, hi0 - lo0, [&](size_t j) { return t->sc->code[lo0 + j] >= 0; },
        [&](size_t o, size_t j) {
          const size_t i = lo0 + j;
          t->sc->sel[had + o] = (uint32_t)i;
          t->sc->slot[had + o] = (uint32_t)t->sc->code[i];
          t->sc->ctr[had + o] = t->sc->ctr_all[i];
        });
    t->sc->sel.resize(had + got);
    t->sc->slot.resize(had + got);
    t->sc->ctr.resize(had + got);
  };
  // a large batch checks its first sixteenth first: a registered DMA batch puts that
  // part's first chunk on the device while pass 1 covers the rest (open_selected)
  const size_t n0 = n >= 16384 && dma_runs() && t->eng.size() == 1 && !many ? n / 16 : n;
  pass1(0, n0);
  bool grown = n0 == n;
  auto grow = [&]() {
    if (grown) return;
    grown = true;
    const double a = now_us();
    pass1(n0, n);
    t->ph.checks_us += now_us() - a;
  };
  if (t->sc->sel.empty()) grow();
  pc.checks_done();
  if (t->sc->sel.empty()) return WG_RC_OK;
  if (!many)
    for (int r = 0; r < WG_N_SESSIONS; ++r) t->spec_window[r] = t->sessions[r].window;
  else
    for (wg_tunn *T : *peers)
      for (int r = 0; r < WG_N_SESSIONS; ++r) T->spec_window[r] = T->sessions[r].window;
  // pass 2 (sequential, packet order, per chunk as it returns): replay window,
  // stats; validation and the byte copies follow on the pools
  const int rc = open_selected(
      t, datagram, len, dst,
      [&](size_t k, int32_t g_st) -> uint8_t {
        const uint32_t i = t->sc->sel[k];
        wg_tunn *T = many ? peer[i] : t;
        const uint64_t ctr = t->sc->ctr[k];
        const uint32_t ring = (t->sc->slot[k] - T->first_slot) / 2;
        Session &s = T->sessions[ring];
        int32_t e = wg_replay_will_accept(&s.window, ctr);  // session.rs:279
        if (e) { set_err(res[i], e); return 0; }
        if (g_st != WG_STATUS_OK) { set_err(res[i], g_st); return 2; }
        e = wg_replay_mark_did_receive(&s.window, ctr);  // session.rs:300, :192-199
        if (e) { set_err(res[i], e); return 1; }
        s.window.receive_cnt += 1;
        set_current_session(T, s.receiving_index);  // mod.rs:562 (pass 1: ridx == receiving_index)
        return 1 | kFinish;
      },
      [&](size_t k, const uint8_t *pt, uint32_t P) -> uint64_t {
        wg_tunn_result &r = res[t->sc->sel[k]];
        std::memset(&r, 0, sizeof r);
        return validate(pt, P, r);
      },
      [&](size_t k) -> bool {  // the same decision with every tag assumed good
        wg_tunn *T = many ? peer[t->sc->sel[k]] : t;
        wg_replay &w = T->spec_window[(t->sc->slot[k] - T->first_slot) / 2];
        if (wg_replay_will_accept(&w, t->sc->ctr[k])) return false;
        (void)wg_replay_mark_did_receive(&w, t->sc->ctr[k]);
        return true;
      },
      grow, !grown, n);
  // failed while pass 1 covered only the batch's first part: the rest gets its pass-1
  // results now (selected packets read as failed), none from an earlier call
  if (rc) grow();
  if (many)  // rx_bytes of each packet's own Tunn: validate()'s share (mod.rs:606-670)
    for (uint32_t i = 0; i < n; ++i) {
      const wg_tunn_result &r = res[i];
      if (r.kind == WG_TUNN_DONE) peer[i]->rx_bytes += WG_DATA_OVERHEAD_SZ;
      else if (r.kind == WG_TUNN_WRITE_TO_TUNNEL) peer[i]->rx_bytes += (uint64_t)r.len + WG_DATA_OVERHEAD_SZ;
    }
  return rc;
}

int wg_tunn_encapsulate_batch(wg_tunn *t, uint32_t n, const uint8_t *const *src,
                              const uint32_t *src_len, uint8_t *const *dst,
                              const uint32_t *dst_cap, wg_tunn_result *res) {
  if (!t || (n && (!src || !src_len || !dst || !dst_cap || !res)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "encapsulate_batch: null", hipSuccess);
  if (n == 0) return WG_RC_OK;
  std::lock_guard<std::mutex> lk(t->mu);
  Lease lease(t);
  if (lease.rc) return lease.rc;
  return encap_impl(t, nullptr, n, src, src_len, dst, dst_cap, res);
}

int wg_tunn_decapsulate_batch(wg_tunn *t, uint32_t n, const uint8_t *const *datagram,
                              const uint32_t *len, uint8_t *const *dst, const uint32_t *dst_cap,
                              wg_tunn_result *res) {
  if (!t || (n && (!datagram || !len || !dst || !dst_cap || !res)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "decapsulate_batch: null", hipSuccess);
  if (n == 0) return WG_RC_OK;
  std::lock_guard<std::mutex> lk(t->mu);
  Lease lease(t);
  if (lease.rc) return lease.rc;
  return decap_impl(t, nullptr, nullptr, n, datagram, len, dst, dst_cap, res);
}

// A multi-peer call: the distinct Tunns locked in address order, one lane borrowed,
// the lane's owner object as the batch owner
struct MultiCall {
  std::vector<wg_tunn *> peers;
  std::vector<std::unique_lock<std::mutex>> locks;
  Engine *lane = nullptr;
  wg_tunn *owner = nullptr;
  int rc = WG_RC_OK;
  MultiCall(wg_engine *g, uint32_t n, wg_tunn *const *tunn) {
    if (!collect_peers(g, n, tunn, peers)) {
      rc = wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "multi batch: a Tunn is null or not on this engine", hipSuccess);
      return;
    }
    locks.reserve(peers.size());
    for (wg_tunn *p : peers) locks.emplace_back(p->mu);
    if ((rc = lane_acquire(g, &lane)) != WG_RC_OK) return;
    if (!lane->owner) lane->owner = new (std::nothrow) wg_tunn;
    if (!lane->owner) {
      lane_release(g, lane);
      lane = nullptr;
      rc = wg_pipe_fail(WG_RC_OUT_OF_MEMORY, "multi batch: host alloc", hipSuccess);
      return;
    }
    owner = lane->owner;
    owner->group = g;
  }
  ~MultiCall() {}  // (the lease below returns the lane; the locks go last)
};

static int multi_on_engine(bool seal, wg_engine *e, uint32_t n, wg_tunn *const *tunn, const uint8_t *const *in,
                    const uint32_t *len, uint8_t *const *dst, const uint32_t *dst_cap, wg_tunn_result *res) {
  MultiCall mc(e, n, tunn);
  if (mc.rc) return mc.rc;
  Lease lease(mc.owner, mc.lane);
  return seal ? encap_impl(mc.owner, tunn, n, in, len, dst, dst_cap, res)
              : decap_impl(mc.owner, tunn, &mc.peers, n, in, len, dst, dst_cap, res);
}

// Multi-peer batches over several engines (e == NULL; normally one engine per GPU,
// NepTUN's PacketWorkers serving every peer from one channel, packet_workers.rs:
// 113-131, 178-233, with one Mutex<Tunn> per peer, device/peer.rs:29): the batch is
// split by the packets' engines, each engine's packets kept in batch order -- a Tunn
// belongs to one engine, so every Tunn still sees its packets in order and the
// results equal the sequential calls -- and the shares run concurrently: each on its
// engine's driver thread (while another such call holds that driver: on the caller),
// the last on the caller.  Results are scattered back into packet order.
struct EngineShare {
  wg_engine *g = nullptr;
  std::vector<uint32_t> idx;
  std::vector<wg_tunn *> tunn;
  std::vector<const uint8_t *> in;
  std::vector<uint32_t> len, cap;
  std::vector<uint8_t *> dst;
  std::vector<wg_tunn_result> res;
  int rc = WG_RC_OK;
  bool on_driver = false;
};

static int multi_across(bool seal, uint32_t n, wg_tunn *const *tunn, const uint8_t *const *in, const uint32_t *len,
                 uint8_t *const *dst, const uint32_t *dst_cap, wg_tunn_result *res) {
  thread_local std::vector<EngineShare> shares;
  size_t used = 0, last = 0;
  for (uint32_t i = 0; i < n; ++i) {
    wg_engine *g = tunn[i] ? tunn[i]->group : nullptr;
    if (!g)
      return wg_pipe_fail(WG_RC_INVALID_ARGUMENT,
                          "multi batch: a Tunn is null or has private engines (wg_tunn_create_multi)", hipSuccess);
    if (last >= used || shares[last].g != g) {
      last = 0;
      while (last < used && shares[last].g != g) ++last;
      if (last == used) {
        if (used == shares.size()) shares.emplace_back();
        EngineShare &S = shares[used++];
        S.g = g;
        S.idx.clear();
        S.tunn.clear();
        S.in.clear();
        S.len.clear();
        S.cap.clear();
        S.dst.clear();
        S.rc = WG_RC_OK;
        S.on_driver = false;
      }
    }
    EngineShare &S = shares[last];
    S.idx.push_back(i);
    S.tunn.push_back(tunn[i]);
    S.in.push_back(in[i]);
    S.len.push_back(len[i]);
    S.dst.push_back(dst[i]);
    S.cap.push_back(dst_cap[i]);
  }
  if (used == 1) return multi_on_engine(seal, shares[0].g, n, tunn, in, len, dst, dst_cap, res);
  auto run_share = [seal](EngineShare &S) {
    S.res.resize(S.idx.size());
    return multi_on_engine(seal, S.g, (uint32_t)S.idx.size(), S.tunn.data(), S.in.data(), S.len.data(),
                           S.dst.data(), S.cap.data(), S.res.data());
  };
  for (size_t k = 0; k + 1 < used; ++k) {
    EngineShare &S = shares[k];
    wg_engine *g = S.g;
    if (!g->driver_mu.try_lock()) continue;
    if (!g->driver) g->driver = new (std::nothrow) Driver(device_numa_node(g->device));
    if (!g->driver) {
      g->driver_mu.unlock();
      continue;
    }
    S.on_driver = true;
    EngineShare *ps = &S;
    g->driver->submit([ps, run_share]() mutable {
      DevGuard dg(ps->g->device);
      return run_share(*ps);
    });
  }
  int rc = WG_RC_OK;
  for (size_t k = used; k-- > 0;)  // (the caller's shares while the drivers run theirs)
    if (!shares[k].on_driver) shares[k].rc = run_share(shares[k]);
  for (size_t k = 0; k < used; ++k) {
    EngineShare &S = shares[k];
    if (S.on_driver) {
      S.rc = S.g->driver->wait();
      S.g->driver_mu.unlock();
    }
    if (S.rc && !rc) rc = S.rc;
    for (size_t j = 0; j < S.idx.size(); ++j) res[S.idx[j]] = S.res[j];
  }
  return rc;
}

int wg_tunn_encapsulate_multi(wg_engine *e, uint32_t n, wg_tunn *const *tunn,
                              const uint8_t *const *src, const uint32_t *src_len,
                              uint8_t *const *dst, const uint32_t *dst_cap, wg_tunn_result *res) {
  if (n && (!tunn || !src || !src_len || !dst || !dst_cap || !res))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "encapsulate_multi: null", hipSuccess);
  if (n == 0) return WG_RC_OK;
  if (!e) return multi_across(true, n, tunn, src, src_len, dst, dst_cap, res);
  return multi_on_engine(true, e, n, tunn, src, src_len, dst, dst_cap, res);
}

int wg_tunn_decapsulate_multi(wg_engine *e, uint32_t n, wg_tunn *const *tunn,
                              const uint8_t *const *datagram, const uint32_t *len,
                              uint8_t *const *dst, const uint32_t *dst_cap, wg_tunn_result *res) {
  if (n && (!tunn || !datagram || !len || !dst || !dst_cap || !res))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "decapsulate_multi: null", hipSuccess);
  if (n == 0) return WG_RC_OK;
  if (!e) return multi_across(false, n, tunn, datagram, len, dst, dst_cap, res);
  return multi_on_engine(false, e, n, tunn, datagram, len, dst, dst_cap, res);
}

int wg_tunn_decrypt_batch(wg_tunn *t, uint32_t n, const uint8_t *const *datagram,
                          const uint32_t *len, uint8_t *const *dst, const uint32_t *dst_cap,
                          wg_tunn_result *res) {
  if (!t || (n && (!datagram || !len || !dst || !dst_cap || !res)))
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "decrypt_batch: null", hipSuccess);
  if (n == 0) return WG_RC_OK;
  std::lock_guard<std::mutex> lk(t->mu);
  Lease lease(t);
  if (lease.rc) return lease.rc;
  PhaseCall pc(t, n);
  t->sc->sel.clear();
  t->sc->slot.clear();
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
    t->sc->sel.push_back(i);
    t->sc->slot.push_back(t->first_slot + 2 * (uint32_t)ring + (ours ? 0u : 1u));
  }
  if (t->sc->sel.empty()) return WG_RC_OK;
  for (uint32_t i : t->sc->sel) set_err(res[i], WG_STATUS_CRYPTO_FAILED);  // until its chunk returns
  pc.checks_done();
  return open_selected(
      t, datagram, len, dst,
      [&](size_t k, int32_t g_st) -> uint8_t {
        const uint32_t i = t->sc->sel[k];
        if (g_st != WG_STATUS_OK) { set_err(res[i], g_st); return 2; }
        return 1 | kFinish;
      },
      [&](size_t k, const uint8_t *pt, uint32_t P) -> uint64_t {
        wg_tunn_result &r = res[t->sc->sel[k]];
        std::memset(&r, 0, sizeof r);
        const uint64_t rx = validate(pt, P, r);
        if (r.kind == WG_TUNN_DONE) set_err(r, WG_STATUS_UNEXPECTED_PACKET);  // mod.rs:412
        return rx;
      },
      [](size_t) { return true; },  // (no replay window: every opened packet lands)
      [] {}, false, n);
}

int wg_tunn_get_phases(const wg_tunn *t, wg_tunn_phases *out) {
  if (!t || !out) return WG_RC_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(t->mu);
  *out = t->ph;
  add_lane_phases(*out, t->ph_lanes);
  for (const Engine *E : t->eng) add_lane_phases(*out, E->ph);
  return WG_RC_OK;
}

int wg_tunn_reset_phases(wg_tunn *t) {
  if (!t) return WG_RC_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(t->mu);
  t->ph = wg_tunn_phases{};
  t->ph_lanes = wg_tunn_phases{};
  for (Engine *E : t->eng) E->ph = wg_tunn_phases{};
  return WG_RC_OK;
}

int wg_tunn_set_phase_timing(wg_tunn *t, int on) {
  if (!t) return WG_RC_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(t->mu);
  t->timing = on != 0;
  for (Engine *E : t->eng) E->timing = on != 0;
  return WG_RC_OK;
}

}  // extern "C"
