// wg_gpu.cpp -- C ABI (include/neptun_gpu.h) over the gfx950 AEAD kernels.
//
// Host side of the drop-in boundary: context + device key table (replaces the
// per-session ring::LessSafeKey objects built in Session::new,
// neptun/src/noise/session.rs:160-180) and batch launchers.  Nothing here
// falls back to a CPU implementation: without a usable HIP device every call
// fails with WG_RC_NO_DEVICE / WG_RC_HIP_ERROR.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "neptun_gpu.h"
#include "wg_aead_kernels.h"

struct wg_gpu_ctx {
  int device = 0;
  uint32_t key_slots = 0;
  uint8_t *d_keys = nullptr;       // key_slots * 32
  uint32_t *d_key_index = nullptr; // key_slots
  uint2 *d_route = nullptr;        // receiver_idx -> key slot (wg_route.hip), 2^route_bits
  uint32_t route_bits = 0;
  uint32_t cus = 0;                // compute units (persistent strided grid)
  bool pad_slots = false;          // wg_gpu_ctx_set_slot_padding
  int64_t xlane_lanes = -1;        // wg_gpu_ctx_set_xlane_lanes (< 0: default)
  int split_parts = -1;            // wg_gpu_ctx_set_split (< 0: default)
  struct Range {
    uint64_t host, bytes, dev;
  };
  std::vector<Range> reg;          // registered host memory, sorted by host address
  // key-slot ranges [first, first + count) held by Tunns (wg_tunn.cpp): a Tunn's
  // install_session writes its slots, so two Tunns may never share one
  std::vector<std::pair<uint32_t, uint32_t>> claims;
  std::mutex mu;                   // serialises key-table and route-table updates
  // key-table updates completed so far (wg_gpu_set_keys): a resident kernel holding the
  // table in its caches since an older generation is relaunched (wg_tunn.cpp Service)
  std::atomic<uint64_t> key_gen{0};
};

void wg_srv_ctx_closing(wg_gpu_ctx *ctx);  // wg_tunn.cpp: resident kernels on this context stop

// open into line-aligned plaintext slots on the text grid (1) or on the wire grid
// with its output runs straddling the destination's lines (0: A/B only)
#ifndef WG_TEXT_GRID
#define WG_TEXT_GRID 1
#endif

namespace {

thread_local std::string g_last_error;

int fail(int rc, const char *what, hipError_t e = hipSuccess) {
  char buf[256];
  if (e != hipSuccess)
    std::snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
  else
    std::snprintf(buf, sizeof buf, "%s", what);
  g_last_error = buf;
  return rc;
}

#define WG_HIP(call, what)                                   \
  do {                                                       \
    hipError_t e_ = (call);                                  \
    if (e_ != hipSuccess) return fail(WG_RC_HIP_ERROR, what, e_); \
  } while (0)

inline uint32_t grid_for(uint32_t n) { return (n + wg::kBlockThreads - 1) / wg::kBlockThreads; }

// Launch on the caller's device; restore the previous current device after.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

// shared with wg_pipe.cpp / wg_tunn.cpp
int wg_pipe_fail(int rc, const char *what, hipError_t e) { return fail(rc, what, e); }
int wg_ctx_device(const wg_gpu_ctx *ctx) { return ctx->device; }
bool wg_ctx_slot_padding(const wg_gpu_ctx *ctx) { return ctx->pad_slots; }
// a Tunn's key slots: claimed at create (an overlap with a live Tunn's range on this
// context is refused), released at destroy
int wg_ctx_claim_slots(wg_gpu_ctx *ctx, uint32_t first, uint32_t count) {
  std::lock_guard<std::mutex> lk(ctx->mu);
  if ((uint64_t)first + count > ctx->key_slots)
    return fail(WG_RC_INVALID_ARGUMENT, "tunn_create: needs 16 key slots");
  for (const auto &c : ctx->claims)
    if (first < c.first + c.second && c.first < first + count)
      return fail(WG_RC_INVALID_ARGUMENT, "tunn_create: key slots overlap another Tunn's on this context");
  ctx->claims.emplace_back(first, count);
  return WG_RC_OK;
}
void wg_ctx_release_slots(wg_gpu_ctx *ctx, uint32_t first) {
  std::lock_guard<std::mutex> lk(ctx->mu);
  for (size_t k = 0; k < ctx->claims.size(); ++k)
    if (ctx->claims[k].first == first) {
      ctx->claims.erase(ctx->claims.begin() + (long)k);
      return;
    }
}
uint64_t wg_ctx_key_gen(const wg_gpu_ctx *ctx) { return ctx->key_gen.load(std::memory_order_acquire); }
const uint8_t *wg_ctx_keys(const wg_gpu_ctx *ctx) { return ctx->d_keys; }
const uint32_t *wg_ctx_key_index(const wg_gpu_ctx *ctx) { return ctx->d_key_index; }
// snapshot of the registered ranges as (host, bytes, dev) triples, sorted by host
void wg_ctx_reg_snapshot(wg_gpu_ctx *ctx, std::vector<uint64_t> &out) {
  std::lock_guard<std::mutex> lk(ctx->mu);
  out.clear();
  for (const auto &r : ctx->reg) {
    out.push_back(r.host);
    out.push_back(r.bytes);
    out.push_back(r.dev);
  }
}
// device address of host [p, p + n) if it lies inside one registered range
bool wg_ctx_dev_addr(wg_gpu_ctx *ctx, const void *p, uint64_t n, uint64_t *dev) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  std::lock_guard<std::mutex> lk(ctx->mu);
  auto it = std::upper_bound(ctx->reg.begin(), ctx->reg.end(), a,
                             [](uint64_t x, const wg_gpu_ctx::Range &r) { return x < r.host; });
  if (it == ctx->reg.begin()) return false;
  --it;
  if (a + n > it->host + it->bytes) return false;
  *dev = it->dev + (a - it->host);
  return true;
}

// Host ranges pinned by hipHostRegister, shared by every context that registers them
// (a multi-GPU Tunn registers the caller's pools on each GPU's context): one pin per
// range, released with its last registration.  A range must be registered with the
// same base and size everywhere.
namespace {
struct Pin {
  uint64_t bytes;
  int refs;
};
std::mutex g_pin_mu;
std::map<uint64_t, Pin> g_pins;

int pin_acquire(uint64_t a, uint64_t bytes) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pins.upper_bound(a);
  if (it != g_pins.begin()) {
    auto p = std::prev(it);
    if (p->first == a && p->second.bytes == bytes) {
      ++p->second.refs;
      return WG_RC_OK;
    }
    if (p->first + p->second.bytes > a)
      return fail(WG_RC_INVALID_ARGUMENT, "register_host: overlaps a range another context registered differently");
  }
  if (it != g_pins.end() && it->first < a + bytes)
    return fail(WG_RC_INVALID_ARGUMENT, "register_host: overlaps a range another context registered differently");
  WG_HIP(hipHostRegister(reinterpret_cast<void *>(a), bytes, hipHostRegisterMapped | hipHostRegisterPortable),
         "register_host: hipHostRegister");
  g_pins[a] = Pin{bytes, 1};
  return WG_RC_OK;
}

int pin_release(uint64_t a) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pins.find(a);
  if (it == g_pins.end()) return fail(WG_RC_INVALID_ARGUMENT, "unregister_host: not pinned");
  if (--it->second.refs > 0) return WG_RC_OK;
  g_pins.erase(it);
  WG_HIP(hipHostUnregister(reinterpret_cast<void *>(a)), "unregister_host: hipHostUnregister");
  return WG_RC_OK;
}
}  // namespace

extern "C" {

int wg_gpu_abi_version(void) { return WG_GPU_ABI_VERSION; }

#ifndef WG_BUILD_ID
#define WG_BUILD_ID "unknown"
#endif
const char *wg_gpu_build_id(void) { return WG_BUILD_ID; }

const char *wg_gpu_last_error(void) { return g_last_error.c_str(); }

int wg_gpu_ctx_create(int device, uint32_t key_slots, wg_gpu_ctx **out) {
  if (!out || key_slots == 0) return fail(WG_RC_INVALID_ARGUMENT, "ctx_create: bad argument");
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
    return fail(WG_RC_NO_DEVICE, "ctx_create: no HIP device");
  if (device < 0 || device >= count) return fail(WG_RC_INVALID_ARGUMENT, "ctx_create: bad device");
  wg_gpu_ctx *ctx = new (std::nothrow) wg_gpu_ctx;
  if (!ctx) return fail(WG_RC_OUT_OF_MEMORY, "ctx_create: host alloc");
  ctx->device = device;
  ctx->key_slots = key_slots;
  DeviceGuard g(device);
  int cus = 0;
  hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  ctx->cus = (e == hipSuccess && cus > 0) ? (uint32_t)cus : 256u;
  e = hipMalloc(&ctx->d_keys, (size_t)key_slots * 32);
  if (e == hipSuccess) e = hipMalloc(&ctx->d_key_index, (size_t)key_slots * 4);
  if (e == hipSuccess) e = hipMemset(ctx->d_keys, 0, (size_t)key_slots * 32);
  if (e == hipSuccess) e = hipMemset(ctx->d_key_index, 0, (size_t)key_slots * 4);
  if (e != hipSuccess) {
    (void)hipFree(ctx->d_keys);
    (void)hipFree(ctx->d_key_index);
    delete ctx;
    return fail(WG_RC_HIP_ERROR, "ctx_create: device alloc", e);
  }
  *out = ctx;
  return WG_RC_OK;
}

int wg_gpu_ctx_destroy(wg_gpu_ctx *ctx) {
  if (!ctx) return WG_RC_OK;
  DeviceGuard g(ctx->device);
  wg_srv_ctx_closing(ctx);
  (void)hipDeviceSynchronize();
  (void)hipFree(ctx->d_keys);
  (void)hipFree(ctx->d_key_index);
  (void)hipFree(ctx->d_route);
  // (through the shared pins: another context may still hold the same range)
  for (const auto &r : ctx->reg) (void)pin_release(r.host);
  delete ctx;
  return WG_RC_OK;
}

uint32_t wg_gpu_ctx_key_slots(const wg_gpu_ctx *ctx) { return ctx ? ctx->key_slots : 0; }

int wg_gpu_set_keys(wg_gpu_ctx *ctx, uint32_t first_slot, uint32_t n, const uint8_t *keys,
                    const uint32_t *indices, void *stream) {
  if (!ctx || !keys || !indices) return fail(WG_RC_INVALID_ARGUMENT, "set_keys: null argument");
  if (n == 0) return WG_RC_OK;
  if ((uint64_t)first_slot + n > ctx->key_slots)
    return fail(WG_RC_INVALID_ARGUMENT, "set_keys: slot range exceeds the key table");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  // pageable host source: hipMemcpyAsync stages it before returning
  WG_HIP(hipMemcpyAsync(ctx->d_keys + (size_t)first_slot * 32, keys, (size_t)n * 32,
                        hipMemcpyHostToDevice, s),
         "set_keys: key copy");
  WG_HIP(hipMemcpyAsync(ctx->d_key_index + first_slot, indices, (size_t)n * 4,
                        hipMemcpyHostToDevice, s),
         "set_keys: index copy");
  WG_HIP(hipStreamSynchronize(s), "set_keys: sync");
  ctx->key_gen.fetch_add(1, std::memory_order_acq_rel);
  return WG_RC_OK;
}

// Persistent grid for `waves` waves of 64 packets (strided / phase-locked descriptor
// kernels): kStridedBlocksPerCU workgroups per CU walking workgroup-sized groups, or,
// when the waves do not fill those slots, one workgroup per slot (at most one per
// wave) with an even share each (`spread`, wg_aead_kernels.h WG_SPREAD)
// WG_SPREAD_ROT: 0 none, 1 odd blockIdx, 2 blockIdx bit 8, 3 blockIdx bit 3 (A/B)
static uint32_t spread_rot() {
  static const uint32_t m = [] {
    const char *e = std::getenv("WG_SPREAD_ROT");
    return e ? (uint32_t)std::min(3, std::max(0, std::atoi(e))) : 0u;
  }();
  return m;
}

static dim3 persistent_grid(const wg_gpu_ctx *ctx, uint32_t waves, uint32_t &spread) {
  const uint32_t slots = ctx->cus * wg::kStridedBlocksPerCU, per_block = wg::kStridedThreads / 64u;
  if (WG_SPREAD && waves <= per_block * slots) {
    spread = 1u;
    return dim3(std::min(waves, slots));
  }
  spread = 0u;
  return dim3(std::min((waves + per_block - 1u) / per_block, slots));
}

// Latency form (wg_xlane.hip): a batch that would fill only a small part of the
// chip as one packet per lane runs G lanes per packet instead -- the largest G of
// 64 .. 2 with n * G within a lane budget (wg_gpu_ctx_set_xlane_lanes, else
// WG_XLANE_LANES, else cus * 256: one wave per SIMD).  0: the throughput forms.
// Measured (profiles/r05c_xlane_*.jsonl): 1350 B packets gain up to n = 32768
// (G = 2: 37 us against 65 us), lose from 131072 on; 8192 B gain to 16384 (G = 4).
// (smallest group the selection takes: WG_XLANE_MIN_G, 2 .. 64, default 2)
static uint32_t xlane_min_group() {
  static const uint32_t g = [] {
    const char *e = std::getenv("WG_XLANE_MIN_G");
    const long v = e ? std::atol(e) : 2L;
    uint32_t m = 2;
    while (m < 64 && (long)m < v) m *= 2;
    return m;
  }();
  return g;
}

// (WG_XLANE_INLINE=0: small host-described batches read their descriptors from the
// pinned host array like the others -- A/B only)
static bool xlane_inline() {
  static const bool on = [] {
    const char *e = std::getenv("WG_XLANE_INLINE");
    return !e || std::atoi(e) != 0;
  }();
  return on;
}

static uint32_t xlane_group(const wg_gpu_ctx *ctx, uint32_t n) {
  static const long long env = [] {
    const char *e = std::getenv("WG_XLANE_LANES");
    return e ? std::atoll(e) : -1LL;
  }();
  const uint64_t budget = ctx->xlane_lanes >= 0 ? (uint64_t)ctx->xlane_lanes
                          : env >= 0            ? (uint64_t)env
                                                : (uint64_t)ctx->cus * 256u;
  for (uint32_t G = 64; G >= xlane_min_group(); G /= 2)
    if ((uint64_t)n * G <= budget) return G;
  return 0;
}

// What a caller may know about a descriptor batch (the Tunn does: it wrote the
// descriptors): its longest packet, and whether the kernel reaches src / dst in
// host memory over PCIe.
struct DescHint {
  uint32_t max_len = 0;   // 0: unknown
  bool host_mem = false;
  // a completion word the latency form stores when done (DescParams::done_flag); the
  // launch sets *flagged when the chosen form does so (other forms leave it false)
  uint32_t *done_count = nullptr, *done_flag = nullptr;
  uint32_t done_seq = 0;
  bool *flagged = nullptr;
  bool xlane_ok = true;  // false: the throughput forms only
  bool host_descs = false;  // the host can read descs (pinned): small latency-form batches inline them
};

// The latency form's group for a batch: the budget's G (xlane_group), narrowed to
// the longest packet's keystream blocks when known (a 128-byte packet has 3 blocks:
// a 64-lane group would leave 61 lanes idle and measured 2x slower than 4 lanes,
// profiles/r05d_xlane.jsonl).  Reading host memory over PCIe, its 16-byte lane loads
// cost more than the throughput form's whole-line loads beyond a few thousand
// packets (Tunn staged batches of 16,384: 1.62 ms against 1.03, r05b_tunn_small).
static uint32_t xlane_group_hinted(const wg_gpu_ctx *ctx, bool seal, uint32_t n, const DescHint &h) {
  uint32_t G = h.xlane_ok ? xlane_group(ctx, n) : 0u;
  if (!G || (h.host_mem && n > 4096u)) return 0u;
  if (h.max_len) {
    const uint32_t P = seal ? h.max_len : (h.max_len > WG_DATA_OVERHEAD_SZ ? h.max_len - WG_DATA_OVERHEAD_SZ : 0u);
    const uint32_t nb = 1u + (P + 63u) / 64u;
    uint32_t g = 2;
    while (g < nb && g < 64u) g *= 2;
    G = std::max(std::min(G, g), xlane_min_group());
  }
  return G;
}

static int launch_desc(wg_gpu_ctx *ctx, bool seal, const wg_packet_desc *descs,
                       const uint32_t *order, uint32_t n, const uint8_t *src, uint8_t *dst,
                       int32_t *status, void *stream, const DescHint &hint = DescHint{}) {
  // src / dst may be NULL: descriptor offsets are then absolute device addresses
  if (!ctx || (n && (!descs || !status))) return fail(WG_RC_INVALID_ARGUMENT, "batch: null argument");
  if (n == 0) return WG_RC_OK;
  DeviceGuard g(ctx->device);
  wg::DescParams prm{ctx->d_keys, ctx->d_key_index, descs, order, src, dst, status, n,
                     ctx->key_slots, 0u};
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hint.flagged) *hint.flagged = false;
  if (const uint32_t G = xlane_group_hinted(ctx, seal, n, hint)) {
    if (hint.done_flag && hint.done_count) {
      prm.done_count = hint.done_count;
      prm.done_flag = hint.done_flag;
      prm.done_seq = hint.done_seq;
      if (hint.flagged) *hint.flagged = true;
    }
    const uint32_t form = 6u - (uint32_t)__builtin_ctz(G);  // 64 -> 0 ... 2 -> 5
    const uint32_t per_block = wg::kXlaneThreads / G;
    if (hint.host_descs && !order && n <= wg::kXlaneInlineDescs && xlane_inline()) {
      // the descriptors travel in the kernel arguments: no PCIe read before the packets'
      wg::XlaneInlineParams ip;
      ip.prm = prm;
      std::memcpy(ip.d, descs, (size_t)n * sizeof(wg_packet_desc));
      using KI = void (*)(wg::XlaneInlineParams);
      static const KI ikernels[2][6] = {
          {wg::aead_xlane_inline_kernel<false, 64>, wg::aead_xlane_inline_kernel<false, 32>,
           wg::aead_xlane_inline_kernel<false, 16>, wg::aead_xlane_inline_kernel<false, 8>,
           wg::aead_xlane_inline_kernel<false, 4>, wg::aead_xlane_inline_kernel<false, 2>},
          {wg::aead_xlane_inline_kernel<true, 64>, wg::aead_xlane_inline_kernel<true, 32>,
           wg::aead_xlane_inline_kernel<true, 16>, wg::aead_xlane_inline_kernel<true, 8>,
           wg::aead_xlane_inline_kernel<true, 4>, wg::aead_xlane_inline_kernel<true, 2>}};
      hipLaunchKernelGGL(ikernels[seal ? 1 : 0][form], dim3((n + per_block - 1u) / per_block),
                         dim3(wg::kXlaneThreads), 0, s, ip);
      WG_HIP(hipGetLastError(), "batch: launch");
      return WG_RC_OK;
    }
    using K = void (*)(wg::DescParams);
    static const K kernels[2][6] = {  // [seal][64, 32, 16, 8, 4, 2]
        {wg::aead_xlane_kernel<false, 64>, wg::aead_xlane_kernel<false, 32>,
         wg::aead_xlane_kernel<false, 16>, wg::aead_xlane_kernel<false, 8>,
         wg::aead_xlane_kernel<false, 4>, wg::aead_xlane_kernel<false, 2>},
        {wg::aead_xlane_kernel<true, 64>, wg::aead_xlane_kernel<true, 32>,
         wg::aead_xlane_kernel<true, 16>, wg::aead_xlane_kernel<true, 8>,
         wg::aead_xlane_kernel<true, 4>, wg::aead_xlane_kernel<true, 2>}};
    hipLaunchKernelGGL(kernels[seal ? 1 : 0][form], dim3((n + per_block - 1u) / per_block),
                       dim3(wg::kXlaneThreads), 0, s, prm);
  } else if (WG_DESC_SYNC && src && dst) {
    // phase-locked, persistent (wg_aead.hip aead_desc_sync_kernel); its compact
    // per-packet tables hold buffer-relative offsets, hence non-null bases
    const dim3 grid = persistent_grid(ctx, (n + 63u) / 64u, prm.spread);
    // unordered launches may hold affine workgroups (fixed slots, one length);
    // a plan's permutation gathers packets from all over the batch
    const bool affine = WG_DESC_AFFINE && order == nullptr;
    // a single-slot context: every packet that passes the slot check uses key 0
    const bool key1 = WG_DESC_KEY1 && ctx->key_slots == 1;
    using K = void (*)(wg::DescParams);
    static const K kernels[2][2][2] = {  // [seal][affine][key1]
        {{wg::aead_desc_sync_kernel<false>, wg::aead_desc_sync_key1_kernel<false>},
         {wg::aead_desc_affine_kernel<false>, wg::aead_desc_affine_key1_kernel<false>}},
        {{wg::aead_desc_sync_kernel<true>, wg::aead_desc_sync_key1_kernel<true>},
         {wg::aead_desc_affine_kernel<true>, wg::aead_desc_affine_key1_kernel<true>}}};
    hipLaunchKernelGGL(kernels[seal ? 1 : 0][affine ? 1 : 0][key1 ? 1 : 0], grid,
                       dim3(wg::kStridedThreads), 0, s, prm);
  } else if (seal) {
    hipLaunchKernelGGL(wg::aead_desc_kernel<true>, dim3(grid_for(n)), dim3(wg::kBlockThreads), 0,
                       s, prm);
  } else {
    hipLaunchKernelGGL(wg::aead_desc_kernel<false>, dim3(grid_for(n)), dim3(wg::kBlockThreads), 0,
                       s, prm);
  }
  WG_HIP(hipGetLastError(), "batch: launch");
  return WG_RC_OK;
}

}  // extern "C"

// Tunn-internal launch (wg_tunn.cpp) with the batch's longest packet and memory kind
int wg_launch_desc_hinted(wg_gpu_ctx *ctx, bool seal, const wg_packet_desc *descs, uint32_t n,
                          const uint8_t *src, uint8_t *dst, int32_t *status, void *stream,
                          uint32_t max_len, bool host_mem, uint32_t *done_count, uint32_t *done_flag,
                          uint32_t done_seq, bool *flagged, bool xlane_ok, bool host_descs) {
  DescHint h;
  h.host_descs = host_descs;
  h.max_len = max_len;
  h.host_mem = host_mem;
  h.done_count = done_count;
  h.done_flag = done_flag;
  h.done_seq = done_seq;
  h.flagged = flagged;
  h.xlane_ok = xlane_ok;
  return launch_desc(ctx, seal, descs, nullptr, n, src, dst, status, stream, h);
}

extern "C" {

int wg_gpu_seal_batch(wg_gpu_ctx *ctx, const wg_packet_desc *descs, uint32_t n,
                      const uint8_t *src, uint8_t *dst, int32_t *status, void *stream) {
  return launch_desc(ctx, true, descs, nullptr, n, src, dst, status, stream);
}

int wg_gpu_open_batch(wg_gpu_ctx *ctx, const wg_packet_desc *descs, uint32_t n,
                      const uint8_t *src, uint8_t *dst, int32_t *status, void *stream) {
  return launch_desc(ctx, false, descs, nullptr, n, src, dst, status, stream);
}

int wg_gpu_seal_batch_ordered(wg_gpu_ctx *ctx, const wg_packet_desc *descs,
                              const uint32_t *order, uint32_t n, const uint8_t *src,
                              uint8_t *dst, int32_t *status, void *stream) {
  if (n && !order) return fail(WG_RC_INVALID_ARGUMENT, "batch_ordered: null order");
  return launch_desc(ctx, true, descs, order, n, src, dst, status, stream);
}

int wg_gpu_open_batch_ordered(wg_gpu_ctx *ctx, const wg_packet_desc *descs,
                              const uint32_t *order, uint32_t n, const uint8_t *src,
                              uint8_t *dst, int32_t *status, void *stream) {
  if (n && !order) return fail(WG_RC_INVALID_ARGUMENT, "batch_ordered: null order");
  return launch_desc(ctx, false, descs, order, n, src, dst, status, stream);
}

int wg_gpu_plan_batch(wg_gpu_ctx *ctx, int seal, const wg_packet_desc *descs, uint32_t n,
                      uint32_t *order, uint32_t *scratch, void *stream) {
  if (!ctx || (n && (!descs || !order || !scratch)))
    return fail(WG_RC_INVALID_ARGUMENT, "plan_batch: null argument");
  if (n == 0) return WG_RC_OK;
  DeviceGuard g(ctx->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t extra = seal ? WG_DATA_OVERHEAD_SZ : 0u;  // rounds follow the datagram size
  hipLaunchKernelGGL(wg::plan_hist_kernel, dim3(wg::kPlanTiles), dim3(wg::kPlanThreads), 0, s, descs, n, extra,
                     scratch);
  hipLaunchKernelGGL(wg::plan_scan_kernel, dim3(1), dim3(1024), 0, s, scratch);
  hipLaunchKernelGGL(wg::plan_scatter_kernel, dim3(wg::kPlanTiles), dim3(wg::kPlanThreads), 0, s, descs, n,
                     extra, scratch, order);
  WG_HIP(hipGetLastError(), "plan_batch: launch");
  return WG_RC_OK;
}

// Split waves (StridedParams::split): a launch whose full waves fill only part of the
// persistent grid's wave slots (cus x 16: 4 per SIMD) leaves SIMDs with 2-3 waves,
// whose phase-locked rounds then issue far below the VALU rate: 172,544 x 8192 B ran
// at 0.456 of HBM with 2,696 waves on 4,096 slots, the same packets as a full grid of
// 4,096 waves at 0.544 (profiles/r06c_bench_p8192_*).  Cutting every wave into K parts
// of its rounds (K = 2 .. 8, >= 8 rounds a part; part 0 takes the rounds K does not
// divide) multiplies the wave jobs by K; K is chosen by a fill model -- per pass of up
// to `slots` jobs, time ~ occupancy / (K e(occupancy)), e(o) = o^0.45 fitted to those
// two runs -- plus 1.5 % per extra part (its Poly1305 key block and the finish kernel's
// combine).  172,544 x 8192 B (2,696 waves): K = 3, 8,088 jobs in 1.97 passes (K = 4,
// the best divisor of the 64 rounds, leaves a third pass at 0.63).
// WG_SPLIT_K: 1 = never, 2 .. 8 = forced where a part keeps 8 rounds, unset = the model.
static uint32_t split_parts(const wg_gpu_ctx *ctx, uint32_t waves, uint32_t rk) {
  static const long env = [] {
    const char *e = std::getenv("WG_SPLIT_K");
    return e ? std::atol(e) : -1L;
  }();
  auto ok = [&](uint32_t K) { return K == 1u || rk / K >= 8u; };
  const long forced = ctx->split_parts >= 1 ? ctx->split_parts : env;
  if (forced >= 1) return forced <= 8 && ok((uint32_t)forced) ? (uint32_t)forced : 1u;
  const double slots = (double)ctx->cus * 16.0;
  auto model = [&](uint32_t K) {
    double t = 0.0;
    for (double u = (double)waves * K; u > 0.0; u -= slots) {
      const double occ = std::min(u, slots) / slots;
      t += occ / (K * std::pow(occ, 0.45));
    }
    return t * (1.0 + 0.015 * (K - 1u));
  };
  uint32_t best = 1u;
  for (uint32_t K = 2u; K <= 8u; ++K)
    if (ok(K) && model(K) < model(best)) best = K;
  return best;
}

// the parts of a throughput-form strided batch's full waves (1: unsplit); (open with
// datagrams shorter than 32 bytes fails every packet at parse: never split)
static uint32_t strided_split(const wg_gpu_ctx *ctx, bool seal, uint32_t n, uint32_t len) {
  const uint32_t full_waves = n / 64u;
  return WG_SPLIT && full_waves && (seal || len >= WG_DATA_OVERHEAD_SZ)
             ? split_parts(ctx, full_waves, ((seal ? len : len - WG_DATA_OVERHEAD_SZ) + 127u) / 128u)
             : 1u;
}

static int launch_strided(wg_gpu_ctx *ctx, bool seal, uint32_t n, uint32_t len, uint32_t key_slot,
                          uint64_t counter_base, const uint8_t *src, uint64_t src_stride,
                          uint8_t *dst, uint64_t dst_stride, int32_t *status, void *stream) {
  if (!ctx || (n && (!src || !dst))) return fail(WG_RC_INVALID_ARGUMENT, "strided: null argument");
  if (key_slot >= ctx->key_slots) return fail(WG_RC_INVALID_ARGUMENT, "strided: bad key slot");
  if (((uintptr_t)src | (uintptr_t)dst | src_stride | dst_stride) & 15u)
    return fail(WG_RC_INVALID_ARGUMENT, "strided: pointers and strides must be 16-byte aligned");
  // packets must not overlap their neighbours: the datagram / plaintext of
  // packet i lies in [i * stride, i * stride + its length)
  const uint64_t in_len = len, out_len = seal ? (uint64_t)len + WG_DATA_OVERHEAD_SZ
                                               : (len >= WG_DATA_OVERHEAD_SZ ? len - WG_DATA_OVERHEAD_SZ : 0);
  if (in_len > src_stride || out_len > dst_stride)
    return fail(WG_RC_INVALID_ARGUMENT, "strided: packet length exceeds its stride (slots would overlap)");
  // the uniform kernels reach a wave's 64 slots through one buffer resource
  // with 32-bit offsets (num_records = 63 * stride + the last packet's extent)
  // and mask idle lanes with the out-of-range offset wg::kNoAccessOffset
  if (63u * std::max(src_stride, dst_stride) + (uint64_t)len + 64u >= wg::kNoAccessOffset)
    return fail(WG_RC_INVALID_ARGUMENT, "strided: stride too large (63 * stride + len must stay below 2 GiB)");
  if (n == 0) return WG_RC_OK;
  DeviceGuard g(ctx->device);
  wg::StridedParams prm{ctx->d_keys, ctx->d_key_index, src, dst, status, src_stride,
                        dst_stride, counter_base, n, len, key_slot, 0u, 0u, 0u};
  // open into plaintext slots that start on 128-byte boundaries: the text
  // run grid keeps every output line whole (wg_aead.hip Ranges)
  const bool text_grid = WG_TEXT_GRID && !seal && ((uintptr_t)dst % 128u) == 0 && dst_stride % 128u == 0;
  if (ctx->pad_slots) {
    // zero-fill to the line end only where the output runs sit on whole lines
    // and that line end stays inside the slot (the uniform kernels' grid origin:
    // seal and the text grid at dst, open's wire grid 16 bytes before it)
    const uint64_t origin = seal || text_grid ? (uintptr_t)dst : (uintptr_t)dst - 16u;
    const uint64_t out_hi = seal ? (uint64_t)len + WG_DATA_OVERHEAD_SZ
                                 : (text_grid ? out_len : out_len + 16u);
    const uint64_t line_end = (out_hi + 127u) & ~127ull;
    prm.pad_tail = origin % 128u == 0 && dst_stride % 128u == 0 && line_end <= dst_stride &&
                   (seal || len >= WG_DATA_OVERHEAD_SZ);
  }
  // input grid origin on a 128-byte line with whole-line slots: the uniform
  // kernels load every round as whole lines (wg_aead.hip stage_in; the lines
  // hold packet bytes, so they are mapped, and what lies around the packet is
  // never output)
  {
    const uint64_t in_origin = seal ? (uintptr_t)src - 16u : text_grid ? (uintptr_t)src + 16u : (uintptr_t)src;
    prm.full_in = in_origin % 128u == 0 && src_stride % 128u == 0;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  // small batches: the latency form (G lanes per packet, wg_xlane.hip), its group
  // narrowed to the packets' blocks; not with slot padding (its kernels write no padding)
  if (!prm.pad_tail) {
    DescHint h;
    h.max_len = len;
    if (const uint32_t G = xlane_group_hinted(ctx, seal, n, h)) {
      using K = void (*)(wg::StridedParams);
      static const K kernels[2][6] = {  // [seal][64, 32, 16, 8, 4, 2]
          {wg::aead_xlane_strided_kernel<false, 64>, wg::aead_xlane_strided_kernel<false, 32>,
           wg::aead_xlane_strided_kernel<false, 16>, wg::aead_xlane_strided_kernel<false, 8>,
           wg::aead_xlane_strided_kernel<false, 4>, wg::aead_xlane_strided_kernel<false, 2>},
          {wg::aead_xlane_strided_kernel<true, 64>, wg::aead_xlane_strided_kernel<true, 32>,
           wg::aead_xlane_strided_kernel<true, 16>, wg::aead_xlane_strided_kernel<true, 8>,
           wg::aead_xlane_strided_kernel<true, 4>, wg::aead_xlane_strided_kernel<true, 2>}};
      const uint32_t per_block = wg::kXlaneThreads / G;
      hipLaunchKernelGGL(kernels[seal ? 1 : 0][6u - (uint32_t)__builtin_ctz(G)],
                         dim3((n + per_block - 1u) / per_block), dim3(wg::kXlaneThreads), 0, s, prm);
      WG_HIP(hipGetLastError(), "strided: launch");
      return WG_RC_OK;
    }
  }
  const uint32_t full_waves = n / 64u;
  const uint32_t split = strided_split(ctx, seal, n, len);
  void *scratch = nullptr;
  wg::StridedSplitParams sp;
  if (split > 1u) {
    // the parts' accumulators, stream-ordered (concurrent launches on other streams
    // get their own): [part][packet] 16 + 4 bytes, then [packet] r and s (32 bytes)
    const size_t np = (size_t)full_waves * 64u, m = np * split;
    WG_HIP(hipMallocAsync(&scratch, m * 20u + np * 32u, s), "strided: split scratch");
    sp.sa.split = split;
    const uint32_t rk = ((seal ? len : len - WG_DATA_OVERHEAD_SZ) + 127u) / 128u;
    sp.sa.split_q = rk / split;
    sp.sa.split_rem = rk - split * sp.sa.split_q;
    sp.sa.part_h = static_cast<uint4 *>(scratch);
    sp.sa.rs = reinterpret_cast<uint4 *>(static_cast<uint8_t *>(scratch) + m * 16u);
    sp.sa.part_h4 = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(scratch) + m * 16u + np * 32u);
  }
  if (full_waves) {
    // persistent: kStridedBlocksPerCU resident workgroups per CU walk the
    // workgroup-sized packet groups (wg_aead.hip aead_strided_kernel); split: the
    // waves' parts
    const dim3 grid = persistent_grid(ctx, full_waves * split, prm.spread);
    // (strided kernels: the spread's live-wave rotation, wg_aead.hip strided_body)
    if (prm.spread) prm.spread |= spread_rot() << 8;
    sp.prm = prm;
    if (split > 1u) {
      if (seal)
        hipLaunchKernelGGL((wg::aead_strided_split_kernel<true, false>), grid, dim3(wg::kStridedThreads), 0, s, sp);
      else if (text_grid)
        hipLaunchKernelGGL((wg::aead_strided_split_kernel<false, true>), grid, dim3(wg::kStridedThreads), 0, s, sp);
      else
        hipLaunchKernelGGL((wg::aead_strided_split_kernel<false, false>), grid, dim3(wg::kStridedThreads), 0, s,
                           sp);
    } else if (seal)
      hipLaunchKernelGGL((wg::aead_strided_kernel<true, false>), grid, dim3(wg::kStridedThreads),
                         0, s, prm);
    else if (text_grid)
      hipLaunchKernelGGL(wg::aead_strided_open_text_kernel, grid, dim3(wg::kStridedThreads), 0, s,
                         prm);
    else
      hipLaunchKernelGGL((wg::aead_strided_kernel<false, false>), grid, dim3(wg::kStridedThreads),
                         0, s, prm);
    if (split > 1u) {
      const dim3 fg((full_waves * 64u + 255u) / 256u);
      if (seal)
        hipLaunchKernelGGL((wg::aead_strided_finish_kernel<true, false>), fg, dim3(256), 0, s, sp);
      else if (text_grid)
        hipLaunchKernelGGL((wg::aead_strided_finish_kernel<false, true>), fg, dim3(256), 0, s, sp);
      else
        hipLaunchKernelGGL((wg::aead_strided_finish_kernel<false, false>), fg, dim3(256), 0, s, sp);
      WG_HIP(hipFreeAsync(scratch, s), "strided: split scratch");
    }
  }
  if (n % 64u) {  // the last, partial wave: generic per-lane geometry
    if (seal)
      hipLaunchKernelGGL((wg::aead_strided_kernel<true, true>), dim3(1), dim3(wg::kBlockThreads), 0,
                         s, prm);
    else
      hipLaunchKernelGGL((wg::aead_strided_kernel<false, true>), dim3(1), dim3(wg::kBlockThreads),
                         0, s, prm);
  }
  WG_HIP(hipGetLastError(), "strided: launch");
  return WG_RC_OK;
}

int wg_gpu_seal_strided(wg_gpu_ctx *ctx, uint32_t n, uint32_t len, uint32_t key_slot,
                        uint64_t counter_base, const uint8_t *src, uint64_t src_stride,
                        uint8_t *dst, uint64_t dst_stride, int32_t *status, void *stream) {
  return launch_strided(ctx, true, n, len, key_slot, counter_base, src, src_stride, dst,
                        dst_stride, status, stream);
}

int wg_gpu_open_strided(wg_gpu_ctx *ctx, uint32_t n, uint32_t len, uint32_t key_slot,
                        const uint8_t *src, uint64_t src_stride, uint8_t *dst,
                        uint64_t dst_stride, int32_t *status, void *stream) {
  return launch_strided(ctx, false, n, len, key_slot, 0, src, src_stride, dst, dst_stride, status,
                        stream);
}

int wg_gpu_ctx_set_slot_padding(wg_gpu_ctx *ctx, int writable) {
  if (!ctx) return fail(WG_RC_INVALID_ARGUMENT, "set_slot_padding: null context");
  ctx->pad_slots = writable != 0;
  return WG_RC_OK;
}

int wg_gpu_ctx_set_xlane_lanes(wg_gpu_ctx *ctx, int64_t lanes) {
  if (!ctx) return fail(WG_RC_INVALID_ARGUMENT, "set_xlane_lanes: null context");
  ctx->xlane_lanes = lanes < 0 ? -1 : lanes;
  return WG_RC_OK;
}

int wg_gpu_ctx_set_split(wg_gpu_ctx *ctx, int parts) {
  if (!ctx) return fail(WG_RC_INVALID_ARGUMENT, "set_split: null context");
  ctx->split_parts = parts < 0 ? -1 : parts;
  return WG_RC_OK;
}

int wg_gpu_strided_split_parts(wg_gpu_ctx *ctx, int seal, uint32_t n, uint32_t len) {
  if (!ctx) return fail(WG_RC_INVALID_ARGUMENT, "strided_split_parts: null context");
  return (int)strided_split(ctx, seal != 0, n, len);
}

int wg_gpu_register_host(wg_gpu_ctx *ctx, void *base, uint64_t bytes) {
  if (!ctx || !base || !bytes) return fail(WG_RC_INVALID_ARGUMENT, "register_host: bad argument");
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  std::lock_guard<std::mutex> lk(ctx->mu);
  for (const auto &r : ctx->reg)
    if (a < r.host + r.bytes && r.host < a + bytes)
      return fail(WG_RC_INVALID_ARGUMENT, "register_host: overlaps a registered range");
  DeviceGuard g(ctx->device);
  if (const int rc = pin_acquire(a, bytes)) return rc;
  void *dev = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&dev, base, 0);
  if (e != hipSuccess) {
    (void)pin_release(a);
    return fail(WG_RC_HIP_ERROR, "register_host: device pointer", e);
  }
  const wg_gpu_ctx::Range r{a, bytes, reinterpret_cast<uint64_t>(dev)};
  ctx->reg.insert(std::upper_bound(ctx->reg.begin(), ctx->reg.end(), r,
                                   [](const wg_gpu_ctx::Range &x, const wg_gpu_ctx::Range &y) {
                                     return x.host < y.host;
                                   }),
                  r);
  return WG_RC_OK;
}

int wg_gpu_unregister_host(wg_gpu_ctx *ctx, void *base) {
  if (!ctx || !base) return fail(WG_RC_INVALID_ARGUMENT, "unregister_host: bad argument");
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  std::lock_guard<std::mutex> lk(ctx->mu);
  for (auto it = ctx->reg.begin(); it != ctx->reg.end(); ++it)
    if (it->host == a) {
      DeviceGuard g(ctx->device);
      WG_HIP(hipDeviceSynchronize(), "unregister_host: sync");  // no batch may still use it
      ctx->reg.erase(it);
      return pin_release(a);
    }
  return fail(WG_RC_INVALID_ARGUMENT, "unregister_host: not registered");
}

int wg_gpu_host_device_address(wg_gpu_ctx *ctx, const void *host, uint64_t bytes, uint64_t *dev) {
  if (!ctx || !host || !dev) return fail(WG_RC_INVALID_ARGUMENT, "host_device_address: null argument");
  if (!wg_ctx_dev_addr(ctx, host, bytes, dev))
    return fail(WG_RC_INVALID_ARGUMENT, "host_device_address: not inside a registered range");
  return WG_RC_OK;
}

int wg_gpu_route_set(wg_gpu_ctx *ctx, uint32_t n, const uint32_t *receiver_idx,
                     const uint32_t *key_slot) {
  if (!ctx || (n && (!receiver_idx || !key_slot)))
    return fail(WG_RC_INVALID_ARGUMENT, "route_set: null argument");
  if (n > (1u << 22)) return fail(WG_RC_INVALID_ARGUMENT, "route_set: more than 2^22 entries");
  uint32_t bits = 4;
  while ((1u << bits) < 2u * n) ++bits;  // load factor <= 1/2
  const uint32_t cap = 1u << bits, mask = cap - 1u;
  std::vector<uint2> tab(cap, uint2{0u, WG_KEY_SLOT_NO_SESSION});
  for (uint32_t i = 0; i < n; ++i) {
    if (key_slot[i] >= ctx->key_slots)
      return fail(WG_RC_INVALID_ARGUMENT, "route_set: key slot outside the key table");
    uint32_t pos = wg::route_hash(receiver_idx[i], bits);
    while (tab[pos].y != WG_KEY_SLOT_NO_SESSION) {
      if (tab[pos].x == receiver_idx[i])
        return fail(WG_RC_INVALID_ARGUMENT, "route_set: duplicate receiver index");
      pos = (pos + 1u) & mask;
    }
    tab[pos] = uint2{receiver_idx[i], key_slot[i]};
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  uint2 *d = nullptr;
  WG_HIP(hipMalloc(&d, (size_t)cap * sizeof(uint2)), "route_set: device alloc");
  hipError_t e = hipMemcpy(d, tab.data(), (size_t)cap * sizeof(uint2), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(d);
    return fail(WG_RC_HIP_ERROR, "route_set: copy", e);
  }
  // launches already queued may still read the old table
  WG_HIP(hipDeviceSynchronize(), "route_set: sync");
  (void)hipFree(ctx->d_route);
  ctx->d_route = d;
  ctx->route_bits = bits;
  return WG_RC_OK;
}

int wg_gpu_route_batch(wg_gpu_ctx *ctx, wg_packet_desc *descs, uint32_t n, const uint8_t *src,
                       void *stream) {
  if (!ctx || (n && (!descs || !src))) return fail(WG_RC_INVALID_ARGUMENT, "route_batch: null argument");
  if (n == 0) return WG_RC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);  // the table pointer is swapped by route_set
  DeviceGuard g(ctx->device);
  hipLaunchKernelGGL(wg::route_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), descs, n, src, ctx->d_route, ctx->route_bits);
  WG_HIP(hipGetLastError(), "route_batch: launch");
  return WG_RC_OK;
}

}  // extern "C"
