// wg_aead_kernels.h -- kernel parameter blocks shared by wg_aead.hip and wg_gpu.cpp.
#pragma once
#include <stdint.h>

#include "neptun_gpu.h"

namespace wg {

constexpr uint32_t kBlockThreads = 256;
// buffer offset past every num_records the uniform kernels use: a lane given it
// moves nothing (launch_strided keeps 63 * stride + len below it)
constexpr uint32_t kNoAccessOffset = 0x7ffffff0u;  // 4 waves per workgroup (descriptor / tail kernels)

// Uniform strided kernel: with WG_SYNC the ChaCha20 steps are phase-locked by
// s_barrier (wg_crypto.h chacha20_block2_sync), which needs waves that share a
// SIMD to be in one workgroup.  512 threads = 2 waves per SIMD per workgroup,
// two workgroups per CU (<= 128 VGPRs): while one waits for its DMA the other
// computes (one 1024-thread workgroup per CU exposes every round's DMA).
#ifndef WG_SYNC
#define WG_SYNC 1
#endif
#ifndef WG_STRIDED_THREADS
#define WG_STRIDED_THREADS (WG_SYNC ? 512 : 256)
#endif
constexpr uint32_t kStridedThreads = WG_STRIDED_THREADS;
#ifndef WG_STRIDED_MIN_WAVES
#define WG_STRIDED_MIN_WAVES 4
#endif
constexpr uint32_t kStridedMinWaves = WG_STRIDED_MIN_WAVES;  // __launch_bounds__ waves per SIMD: 128-VGPR cap
#ifndef WG_STRIDED_BLOCKS_PER_CU
#define WG_STRIDED_BLOCKS_PER_CU (4u * kStridedMinWaves * 64u / kStridedThreads)
#endif
constexpr uint32_t kStridedBlocksPerCU = WG_STRIDED_BLOCKS_PER_CU;
#ifndef WG_DESC_SYNC
#define WG_DESC_SYNC 1  // descriptor batches with non-null bases use the phase-locked kernel
#endif
// Under-filled launches -- fewer waves of 64 packets than the persistent grid has
// wave slots (8 KiB packets at the bench's step payload, a Tunn chunk of a few
// thousand packets): the host sizes the grid to the waves and sets `spread`, and
// every workgroup runs its even share of them (at most a workgroup's waves) in one
// pass.  Without it the first workgroups take whole groups of a workgroup's waves
// and the rest of the chip idles (172,544 x 8 KiB: 337 groups on 512 slots, 81 CUs
// with two workgroups, 175 with one).  0: the plain persistent walk.
#ifndef WG_SPREAD
#define WG_SPREAD 1
#endif
// first wave of workgroup b of `grid` in a spread launch of `waves` waves
__host__ __device__ inline uint32_t spread_lo(uint32_t waves, uint32_t b, uint32_t grid) {
  return (uint32_t)(((uint64_t)waves * b) / grid);
}

struct StridedParams {
  const uint8_t *keys;        // device key table, 32 B per slot
  const uint32_t *key_index;  // device session index per slot
  const uint8_t *src;
  uint8_t *dst;
  int32_t *status;            // may be null
  uint64_t src_stride, dst_stride;
  uint64_t counter_base;      // seal only
  uint32_t n, len, key_slot;
  uint32_t pad_tail;          // 1: zero-fill each output to its 128-byte line end (slot padding)
  uint32_t full_in;           // 1: input runs are whole 128-byte lines (launch_strided)
  uint32_t spread;            // 1: under-filled launch, even wave shares in one pass (WG_SPREAD)
};

// Split (under-filled launches of long packets, wg_gpu.cpp): every wave of 64 packets
// is cut into `split` parts, every part a wave job of its own, so that the grid fills
// the chip: part 0 takes rounds [0, split_q + split_rem), part j > 0 rounds
// [j split_q + split_rem, (j + 1) split_q + split_rem), the last part to the end; the
// parts' Poly1305 accumulators go to part_h / part_h4 ([part][packet]) and
// aead_strided_finish_kernel combines them,
// writes the tags (seal) or checks them (open) and the statuses.  (Kernels of their
// own with their own argument block: the unsplit kernels are compiled as before.)
struct SplitArgs {
  uint32_t split, split_q, split_rem;
  uint4 *part_h;
  uint32_t *part_h4;
  uint4 *rs;  // [packet][2]: part 0's clamped r and s (the finish kernel's Poly1305 key)
};
struct StridedSplitParams {
  StridedParams prm;
  SplitArgs sa;
};
#ifndef WG_SPLIT
#define WG_SPLIT 1
#endif
template <bool kSeal, bool kText> __global__ void aead_strided_split_kernel(StridedSplitParams sp);
template <bool kSeal, bool kText> __global__ void aead_strided_finish_kernel(StridedSplitParams sp);

struct DescParams {
  const uint8_t *keys;
  const uint32_t *key_index;
  const wg_packet_desc *descs;
  const uint32_t *order;  // optional permutation (wg_gpu_plan_batch); null = identity
  const uint8_t *src;
  uint8_t *dst;
  int32_t *status;
  uint32_t n, key_slots;
  uint32_t spread;  // as StridedParams::spread (persistent descriptor kernels)
  // latency form only (aead_xlane_kernel): when done_flag is set, the grid's last
  // workgroup stores done_seq there (pinned host memory, system scope) once every
  // workgroup's outputs and statuses are out; done_count is its arrival counter
  // (device memory, 0 between launches).  The host spins on the word instead of an
  // event (wg_tunn.cpp small zero-copy calls).
  uint32_t *done_count = nullptr;
  uint32_t *done_flag = nullptr;
  uint32_t done_seq = 0;
};

template <bool kSeal, bool kTail> __global__ void aead_strided_kernel(StridedParams prm);
__global__ void aead_strided_open_text_kernel(StridedParams prm);
template <bool kSeal> __global__ void aead_desc_kernel(DescParams prm);
template <bool kSeal> __global__ void aead_desc_sync_kernel(DescParams prm);
// Descriptor batches launched without a plan go to aead_desc_affine_kernel, whose
// workgroups with affine packets (one length, constant slot strides) run the
// uniform geometry with per-packet keys (0: aead_desc_sync_kernel for every launch).
#ifndef WG_DESC_AFFINE
#define WG_DESC_AFFINE 1
#endif
// ... and contexts with a single key slot to the *_key1 forms (SGPR key)
template <bool kSeal> __global__ void aead_desc_sync_key1_kernel(DescParams prm);
template <bool kSeal> __global__ void aead_desc_affine_key1_kernel(DescParams prm);
#ifndef WG_DESC_KEY1
#define WG_DESC_KEY1 1
#endif
template <bool kSeal> __global__ void aead_desc_affine_kernel(DescParams prm);

// Latency form (wg_xlane.hip): G lanes per packet for batches that fill a small
// part of the chip; wg_gpu.cpp picks G from the batch size.
constexpr uint32_t kXlaneThreads = 256;
template <bool kSeal, uint32_t G> __global__ void aead_xlane_kernel(DescParams prm);
// ... with the batch's descriptors carried in the kernel arguments (the host can read
// them: the Tunn's small calls, whose descriptors sit in pinned host memory that the
// kernel would otherwise read over PCIe before anything else)
constexpr uint32_t kXlaneInlineDescs = 64;
struct XlaneInlineParams {
  DescParams prm;
  wg_packet_desc d[kXlaneInlineDescs];
};
template <bool kSeal, uint32_t G> __global__ void aead_xlane_inline_kernel(XlaneInlineParams ip);
template <bool kSeal, uint32_t G> __global__ void aead_xlane_strided_kernel(StridedParams prm);

// Resident service (wg_xlane.hip xlane_service_kernel, host side wg_tunn.cpp Service):
// the Tunn's small calls posted to slots in pinned host memory instead of a launch
// each.  Slot s is served by workgroups [s kSrvGroup, (s + 1) kSrvGroup) of the grid,
// kSrvGroup x kXlaneThreads lanes, G per packet.  The host writes op / n / G and the
// descriptors (absolute device addresses in src_off / dst_off), then seq; the
// workgroups poll {seq, op, n, G} as one 16-byte load, run the packets exactly as the
// latency-form kernels do (statuses into st), and the last of them to finish stores
// seq to `done`.  A workgroup leaves when the host sets *stop or its lease runs out
// (s_memrealtime), so the grid always drains.
constexpr uint32_t kSrvSlots = 8, kSrvGroup = 8, kSrvDescs = 64;
constexpr uint32_t kSrvLanes = kSrvGroup * kXlaneThreads;
struct alignas(128) SrvSlot {
  uint32_t seq, op, n, G;  // op: 1 seal, 0 open; seq written last
  uint32_t pad0[28];
  wg_packet_desc d[kSrvDescs];
  int32_t st[kSrvDescs];
  alignas(128) uint32_t done;
  uint32_t pad1[31];
  // (SrvParams::stamp) s_memrealtime of the request's phases: seen, acquired, the
  // packets done, their stores acknowledged (workgroup 0 of the slot), published (the
  // last workgroup); then inside packet 0 (its group's lane 0): descriptor read, input
  // staged, tag formed, output stores issued
  uint64_t stamp[9];
  uint64_t pad2[7];
};
struct SrvParams {
  SrvSlot *slots;
  const uint32_t *stop;
  uint32_t *d_count;  // [slot * 32]: arrivals of the slot's workgroups (HBM)
  const uint8_t *keys;
  const uint32_t *key_index;
  uint32_t key_slots;
  uint64_t lease_ticks;  // s_memrealtime ticks (100 MHz) from each workgroup's start
  uint32_t stamp;        // 1: record SrvSlot::stamp (WG_TUNN_SRV_STAMP, a diagnostic)
};
__global__ void xlane_service_kernel(SrvParams p);

// wg_plan.hip: counting sort of a descriptor batch by rounds (longest first)
constexpr uint32_t kPlanBins = 256;   // rounds 0..254, 255+ share the top bin
constexpr uint32_t kPlanTiles = 256;  // contiguous descriptor tiles, one block each
constexpr uint32_t kPlanThreads = 512, kPlanWaves = kPlanThreads / 64u;  // hist / scatter blocks
constexpr uint32_t kPlanPer = 8;                            // descriptors per lane per chunk
constexpr uint32_t kPlanChunk = kPlanThreads * kPlanPer;  // descriptors per chunk
static_assert(kPlanBins * kPlanTiles * 4 == WG_PLAN_SCRATCH_BYTES, "scratch size");
__global__ void plan_hist_kernel(const wg_packet_desc *descs, uint32_t n, uint32_t extra,
                                 uint32_t *table);
__global__ void plan_scan_kernel(uint32_t *table);
__global__ void plan_scatter_kernel(const wg_packet_desc *descs, uint32_t n, uint32_t extra,
                                    const uint32_t *table, uint32_t *order);


// wg_route.hip: receiver_idx -> key slot (linear probing, capacity 2^bits, empty
// entries carry slot WG_KEY_SLOT_NO_SESSION); the same hash on host and device
__host__ __device__ inline uint32_t route_hash(uint32_t x, uint32_t bits) {
  return (x * 0x9E3779B1u) >> (32u - bits);
}
__global__ void route_kernel(wg_packet_desc *descs, uint32_t n, const uint8_t *src,
                             const uint2 *table, uint32_t bits);


// wg_handshake.hip
struct HandshakeAnonParams {
  const uint8_t *msgs;  // n handshake initiations, 148 bytes each at `stride`
  uint64_t stride;
  wg_half_handshake *out;
  uint32_t n, check_mac1;
  uint32_t static_private[8];  // responder static key (wave-uniform)
  uint32_t hash0[8];           // HASH(INITIAL_CHAIN_HASH || static_public)
  uint32_t mac1_key[8];        // HASH(LABEL_MAC1 || static_public)
};
struct HandshakeConsumeParams {
  const uint8_t *msgs;  // n handshake initiations, 148 bytes each at `stride`
  uint64_t stride;
  const wg_responder_peer *peers;
  wg_init_received *out;
  uint32_t n;
  uint32_t static_private[8];
  uint32_t hash0[8];  // HASH(INITIAL_CHAIN_HASH || static_public)
};
struct HandshakeRespondParams {
  const wg_init_received *states;
  const wg_response_job *jobs;
  wg_response_out *out;
  uint32_t n;
};
struct Mac2CheckParams {
  const uint8_t *msgs;
  uint64_t stride;
  const uint32_t *lens;
  const uint8_t *addrs;  // 16 bytes each
  uint8_t *cookies;      // 16 bytes each (out)
  int32_t *status;       // out: 0 valid mac2, 1 cookie reply needed
  uint64_t counter;      // cur_counter (rate_limiter.rs:104)
  uint32_t n;
  uint32_t secret[4];
};
struct CookieReplyParams {
  const wg_cookie_reply_job *jobs;
  uint8_t *out;  // 64 bytes each
  uint32_t n;
  uint32_t cookie_key[8], nonce_key[8];
};
struct HandshakeInitiateParams {
  const wg_initiation_job *jobs;
  wg_init_sent *out;
  uint32_t n;
};
struct HandshakeResponseParams {
  const uint8_t *msgs;  // n handshake responses, 92 bytes each at `stride`
  uint64_t stride;
  const wg_response_received_job *jobs;
  wg_session_keys *out;
  uint32_t n, check_mac1;
  uint32_t static_private[8];  // the initiator's static key (wave-uniform)
  uint32_t mac1_key[8];        // HASH(LABEL_MAC1 || static_public)
};
struct CookieOpenParams {
  const wg_cookie_open_job *jobs;
  wg_cookie_open_out *out;
  uint32_t n;
};
__global__ void x25519_kernel(uint32_t n, const uint8_t *scalars, const uint8_t *points,
                              uint8_t *out);
__global__ void handshake_initiate_kernel(HandshakeInitiateParams prm);
__global__ void handshake_response_kernel(HandshakeResponseParams prm);
__global__ void cookie_open_kernel(CookieOpenParams prm);
__global__ void handshake_anon_kernel(HandshakeAnonParams prm);
__global__ void handshake_consume_kernel(HandshakeConsumeParams prm);
__global__ void handshake_respond_kernel(HandshakeRespondParams prm);
__global__ void mac2_check_kernel(Mac2CheckParams prm);
__global__ void cookie_reply_kernel(CookieReplyParams prm);

}  // namespace wg
