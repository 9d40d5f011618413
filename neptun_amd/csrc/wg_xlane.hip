// wg_xlane.hip -- latency form of the descriptor batches: G lanes per packet.
//
// NepTUN hands the data plane batches of at most 50 packets
// (/root/reference/neptun/src/device/packet_workers.rs:27,
// MAX_INTERTHREAD_BATCHED_PKTS).  The throughput kernels (wg_aead.hip) run one
// packet per lane, so such a batch is one or two waves whose lanes each walk their
// packet's 23 ChaCha20 blocks and 85 Poly1305 blocks (1350 B) one after another
// while the rest of the chip idles: ~70 us for 64 packets.  Here a packet is spread
// over a group of G consecutive lanes of one wave (G = 64, 32, ..., 2, chosen by
// the host from the batch size, wg_gpu.cpp):
//
//   blocks   the packet's NB = 1 + ceil(P / 64) keystream blocks (block 0 = the
//            Poly1305 key, RFC 8439 2.6) are dealt out in contiguous spans of
//            C = ceil(NB / G) blocks, lane l taking [l C, l C + C); each lane loads
//            its input pieces, XORs them with its keystream and stores the output;
//   r        lane 0 of the group broadcasts r and s of block 0 (ds_bpermute);
//   Horner   each lane absorbs its ciphertext pieces: h_l = sum m_i r^(k_l - i + 1)
//            over its k_l pieces (lane 0's span starts with block 0, i.e. 4 empty
//            slots in front, which Horner from h = 0 ignores);
//   combine  every lane but the last holds S = 4 C slots, so with d = Lu - 2 - l
//            (Lu lanes in use) T = sum_{l < Lu-1} h_l r^(S d) is a binary tree over
//            the group with one power per level for all lanes (r^S, r^2S, r^4S, ...,
//            by squaring); the last lane then forms D = T r^(c_last) + h_last, its
//            c_last pieces following T's, then the length block and + s (the tag).
//   open     the last lane compares the tag and broadcasts the verdict; on a
//            mismatch every lane zeroes the plaintext it wrote (ring's open_within
//            behaviour, as the throughput kernels do), status InvalidAeadTag.
//
// Per-packet checks, statuses and bytes written are those of aead_desc_kernel:
// seal = Session::format_packet_data (session.rs:205-259), open =
// parse_incoming_packet's DATA arm (noise/mod.rs:139-199) + receive_packet_data
// without the replay window (session.rs:265-302).  The general multiply of the
// combine step is radix 2^26 (wg_crypto.h f26_mul: powers of r are not clamped).
#include <hip/hip_runtime.h>

#include "wg_aead_kernels.h"
#include "wg_crypto.h"

// Checked build (WG_XLANE_CHECK=1 -> neptun_amd/libneptun_gpu_checked.so, the
// tests' bounds audit of this form): every global access of a packet is checked
// against that packet's own extents -- input [src, src + round_up(in bytes, 16)),
// output [dst, dst + out bytes) -- and a stray one is counted (first address,
// packet and lane kept) and not made.  wg_gpu_debug_xlane_check reads the record.
#ifndef WG_XLANE_CHECK
#define WG_XLANE_CHECK 0
#endif

// (A/B: 0 = the staged path's key in vector loads, as the other paths)
#ifndef WG_XLANE_SCALAR_KEY
#define WG_XLANE_SCALAR_KEY 1
#endif

namespace wg {
#if WG_XLANE_CHECK
__device__ unsigned long long g_xlane_check[4];  // violations, first address, its packet, its lane
#endif
namespace {

// a packet's extents (checked build) and who it is
struct XBounds {
  uint64_t in_lo, in_hi, out_lo, out_hi;
  uint32_t pkt, lane;
};

__device__ __forceinline__ bool xok(uint64_t a, uint32_t bytes, uint64_t lo, uint64_t hi, const XBounds &B) {
#if WG_XLANE_CHECK
  if (a >= lo && a + bytes <= hi) return true;
  if (atomicAdd(&g_xlane_check[0], 1ull) == 0ull) {
    atomicExch(&g_xlane_check[1], (unsigned long long)a);
    atomicExch(&g_xlane_check[2], (unsigned long long)B.pkt);
    atomicExch(&g_xlane_check[3], (unsigned long long)B.lane);
  }
  return false;
#else
  (void)a; (void)bytes; (void)lo; (void)hi; (void)B;
  return true;
#endif
}
__device__ __forceinline__ uint4 xld16(const uint8_t *p, const XBounds &B) {
  return xok((uint64_t)p, 16u, B.in_lo, B.in_hi, B) ? ld16(p) : make_uint4(0, 0, 0, 0);
}
// a system-coherent 16-byte load (sc0 sc1: past the caches to memory): the resident
// service's host-memory reads (kSys), made without a launch's cache invalidate
typedef unsigned int xl_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16_sys(const uint8_t *p) {
  // (a volatile global load: sc0 sc1 on gfx950, and the compiler places its waits)
  const xl_u32x4 v =
      *reinterpret_cast<const volatile __attribute__((address_space(1))) xl_u32x4 *>(reinterpret_cast<uint64_t>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 xld16_sys(const uint8_t *p, const XBounds &B) {
  return xok((uint64_t)p, 16u, B.in_lo, B.in_hi, B) ? ld16_sys(p) : make_uint4(0, 0, 0, 0);
}
// a global-address-space 16-byte load: a flat load also counts against the LDS counter,
// and the compiler then waits for every load at once (vmcnt(0) lgkmcnt(0)) where a
// global one lets the key loads issued before the input be waited for alone
__device__ __forceinline__ uint4 xld16_g(const uint8_t *p, const XBounds &B) {
  if (!xok((uint64_t)p, 16u, B.in_lo, B.in_hi, B)) return make_uint4(0, 0, 0, 0);
  const xl_u32x4 v = *reinterpret_cast<const __attribute__((address_space(1))) xl_u32x4 *>(reinterpret_cast<uint64_t>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void xst16(uint8_t *p, uint32_t a, uint32_t b, uint32_t c, uint32_t d, const XBounds &B) {
  if (xok((uint64_t)p, 16u, B.out_lo, B.out_hi, B)) st16(p, a, b, c, d);
}
__device__ __forceinline__ void xstore_partial(uint8_t *p, const uint32_t w[4], int k, const XBounds &B) {
  if (xok((uint64_t)p, (uint32_t)k, B.out_lo, B.out_hi, B)) store_partial(p, w, k);
}

// The key of `slot` in scalar registers, for groups of a whole or half wave (the staged
// path): a scalar load counts against lgkmcnt, not vmcnt, so the first keystream block
// waits for the key alone and runs while the input's vector loads are in flight (a key
// of vector loads issued before them is waited for with vmcnt(0), the input included).
// readlane of a lane whose group has no packet gives a stray slot: clamped, and unused.
template <uint32_t G>
__device__ __forceinline__ void key_issue_scalar(const uint8_t *keys, const uint32_t *key_index, uint32_t slot,
                                                 uint32_t key_slots, uint32_t (&kr)[2][9]) {
  static_assert(G == 64u || G == 32u, "one or two groups per wave");
  typedef const __attribute__((address_space(4))) uint32_t kc_u32;
  auto sload = [&](uint32_t s, uint32_t (&k)[9]) {
    s = s < key_slots ? s : 0u;
    const kc_u32 *q = reinterpret_cast<const kc_u32 *>(reinterpret_cast<uint64_t>(keys) + 32ull * s);
#pragma unroll
    for (int j = 0; j < 8; ++j) k[j] = q[j];
    k[8] = reinterpret_cast<const kc_u32 *>(reinterpret_cast<uint64_t>(key_index))[s];
  };
  if constexpr (G == 64u) {
    sload(__builtin_amdgcn_readfirstlane(slot), kr[0]);
  } else {
    sload(__builtin_amdgcn_readlane(slot, 0), kr[0]);
    sload(__builtin_amdgcn_readlane(slot, 32), kr[1]);
  }
}

// Open's header (the packet's first 16 bytes, the nonce) the same way, for the launched
// kernel only: a launch starts with the scalar cache invalidated, so it cannot hold an
// earlier call's bytes (the resident service reads packets with vector loads past the
// caches).  A half wave without a packet (exec) reads the other half's header: its lanes'
// addresses are stale.  (Addresses are chosen before the loads, not loads under a branch:
// a join's copy of the result waits for every scalar load.)
template <uint32_t G>
__device__ __forceinline__ void hdr_issue_scalar(const uint8_t *src, uint4 (&hr)[2]) {
  static_assert(G == 64u || G == 32u, "one or two groups per wave");
  typedef const __attribute__((address_space(4))) xl_u32x4 hc_u32x4;
  const uint64_t a = reinterpret_cast<uint64_t>(src);
  const uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
  auto addr = [&](int ln) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, ln) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, ln) << 32);
  };
  auto sload = [&](uint64_t q) {
    const xl_u32x4 v = *reinterpret_cast<const hc_u32x4 *>(q);
    return make_uint4(v.x, v.y, v.z, v.w);
  };
  if constexpr (G == 64u) {
    hr[0] = hr[1] = sload(addr(0));  // (the group is the wave: lane 0 is active)
  } else {
    const uint64_t ex = __builtin_amdgcn_read_exec();
    const uint64_t p0 = addr(0), p1 = addr(32);
    const uint64_t q0 = (ex & 1ull) ? p0 : p1;  // (some half is active)
    const uint64_t q1 = ((ex >> 32) & 1ull) ? p1 : q0;
    hr[0] = sload(q0);
    hr[1] = sload(q1);
  }
}

// value of lane `src` (0 .. G-1) of this lane's group
template <uint32_t G>
__device__ __forceinline__ uint32_t gshfl(uint32_t x, uint32_t src) {
  return (uint32_t)__shfl((int)x, (int)src, (int)G);
}

template <uint32_t G>
__device__ __forceinline__ F26 gshfl26(const F26 &a, uint32_t src) {
  F26 r;
#pragma unroll
  for (int q = 0; q < 5; ++q) r.v[q] = gshfl<G>(a.v[q], src);
  return r;
}

__device__ __forceinline__ F26 f26_zero() {
  F26 z;
#pragma unroll
  for (int q = 0; q < 5; ++q) z.v[q] = 0u;
  return z;
}

}  // namespace

// LDS staging of packets in host memory (kStage: the Tunn's zero-copy small calls).
// The lane-span layout has every lane read and write its own blocks 16 bytes at a time,
// C 64-byte blocks apart: over PCIe each piece is a request of its own.  50 packets of
// 1350 B from 8 concurrent callers are then ~0.9 G read requests and as many 16-byte
// writes per second -- with their headers about the whole upstream PCIe link, where 8
// callers flattened at 54 Gbit/s with launches and with the resident service alike
// (profiles/r06n/tt_*).  Staged, the group moves its packet through LDS: its G lanes
// load consecutive pieces (one load instruction covers G x 16 contiguous bytes, which
// the memory pipeline merges), every lane then reads and writes its blocks in LDS, and
// the group stores the output the same contiguous way -- the same bytes in 4-8x fewer,
// larger transactions, and every input piece in flight at once (one round trip).
constexpr uint32_t kXlaneStagePieces = 3072;  // 48 KiB of 16-byte pieces per workgroup
template <uint32_t G>
__device__ __forceinline__ constexpr uint32_t stage_cap() {  // pieces per group
  return kXlaneStagePieces / (kXlaneThreads / G);
}
// (cross-lane LDS traffic inside one wave: the wave's LDS operations complete in order;
// this keeps the compiler from moving a lane's read above another lane's write)
__device__ __forceinline__ void lds_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// One packet on the G lanes of its group (l = the lane's index in the group): the
// checks, the spread keystream / Poly1305 spans, the combine, the tag.  align: the
// packet's offsets OR-ed (misaligned -> WG_STATUS_MISALIGNED); st: its status (or null).
// kStage: through the group's LDS region gb (stage_cap<G>() pieces; the caller checks
// that the packet's (P + 31) / 16 pieces fit).
template <bool kSeal, uint32_t G, bool kStage = false, bool kSys = false>
__device__ __forceinline__ void xlane_packet(uint32_t l, const uint8_t *src, uint8_t *dst, uint32_t len,
                                             uint32_t slot, uint64_t counter, uint64_t align, int32_t *st,
                                             const uint8_t *keys, const uint32_t *key_index, uint32_t key_slots,
                                             uint32_t pkt, uint4 *gb = nullptr, uint64_t *stamps = nullptr) {
  // (stamps: the service's phase stamps of this packet, its group's lane 0 writes them)
  const bool stamp = stamps && l == 0u;
  int32_t status = WG_STATUS_OK;
  if (!kSeal && slot == WG_KEY_SLOT_INVALID_PACKET) status = WG_STATUS_INVALID_PACKET;
  else if (!kSeal && slot == WG_KEY_SLOT_NO_SESSION) status = WG_STATUS_NO_CURRENT_SESSION;
  else if (slot >= key_slots) status = WG_STATUS_BAD_KEY_SLOT;
  else if ((align & 15u) != 0u) status = WG_STATUS_MISALIGNED;
  else if (!kSeal && len < WG_DATA_OVERHEAD_SZ) status = WG_STATUS_INVALID_PACKET;  // mod.rs:170

  // (seal: plaintext in, datagram out; open: datagram in, plaintext out)
  const uint32_t in_bytes = (len + 15u) & ~15u;
  const uint32_t out_bytes = kSeal ? len + WG_DATA_OVERHEAD_SZ : (len >= WG_DATA_OVERHEAD_SZ ? len - WG_DATA_OVERHEAD_SZ : 0u);
  const XBounds B{(uint64_t)src, (uint64_t)src + in_bytes, (uint64_t)dst, (uint64_t)dst + out_bytes, pkt, l};
  if (status != WG_STATUS_OK) {  // group-uniform: nothing of the packet is read or written
    if (l == 0u && st) *st = status;
    return;
  }

  const uint32_t P = kSeal ? len : len - WG_DATA_OVERHEAD_SZ;
  const uint8_t *in = kSeal ? src : src + WG_DATA_OFFSET;  // plaintext / ciphertext
  uint8_t *out = kSeal ? dst + WG_DATA_OFFSET : dst;      // ciphertext / plaintext
  const uint32_t NB = 1u + (P + 63u) / 64u;
  const uint32_t C = (NB + G - 1u) / G;
  const uint32_t Lu = (NB + C - 1u) / C;  // lanes in use; lane Lu - 1 holds block NB - 1
  const uint32_t b0 = l * C, b1 = min(b0 + C, NB);

  // the span's first input pieces go out with open's header load: over PCIe (the
  // Tunn's zero-copy calls) one round trip instead of two.  A header that fails its
  // checks below then only suppresses every store (wr): its packet's bytes are read
  // but nothing of it is written.
  auto load_block = [&](uint32_t b, uint4 (&x)[4]) {
    const uint32_t off = 64u * (b - 1u);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool has = b >= 1u && off + 16u * (uint32_t)q < P;
      if constexpr (kStage) x[q] = has ? gb[(off >> 4) + (uint32_t)q] : make_uint4(0, 0, 0, 0);
      else x[q] = has ? xld16(in + off + 16u * (uint32_t)q, B) : make_uint4(0, 0, 0, 0);
    }
  };
  uint4 x[4];
  const bool any = b0 < NB;
  // staged: the group's input pieces (seal: the plaintext; open: ciphertext + tag),
  // G consecutive pieces per load instruction, up to 8 per lane in flight at once
  constexpr uint32_t kBatch = 8;
  const uint32_t np_in = kSeal ? (P + 15u) / 16u : (P + 31u) / 16u;
  uint4 sv[kBatch];
  uint32_t key[8];
  uint32_t sidx = 0, n1 = 0, n2 = 0;
  // (the service's open reads its header with a vector load past the caches, and waits for
  // it -- and so for the input -- before its first block)
  constexpr bool kScalarKey = kStage && G >= 32u && (kSeal || !kSys) && WG_XLANE_SCALAR_KEY;
  uint32_t kr[2][9];  // (kScalarKey: each half wave's key and index, and open's header)
  uint4 hr[2];
  auto header_checks = [&](const uint4 &h) {  // header: type, receiver_idx, counter (mod.rs:170-180)
    if (h.x != WG_MSG_DATA) status = WG_STATUS_INVALID_PACKET;
    else if (h.y != sidx) status = WG_STATUS_WRONG_INDEX;  // session.rs:275-277
    n1 = h.z;
    n2 = h.w;
  };
  auto load_key = [&]() {
    if (kSeal) {
      n1 = (uint32_t)counter;
      n2 = (uint32_t)(counter >> 32);
    }
    if constexpr (kScalarKey) {  // (issued here, taken by settle_key)
      key_issue_scalar<G>(keys, key_index, slot, key_slots, kr);
      if constexpr (!kSeal) hdr_issue_scalar<G>(src, hr);
    } else {
      const uint4 a = ld16(keys + 32u * slot), b = ld16(keys + 32u * slot + 16u);
      key[0] = a.x; key[1] = a.y; key[2] = a.z; key[3] = a.w;
      key[4] = b.x; key[5] = b.y; key[6] = b.z; key[7] = b.w;
      sidx = key_index[slot];
      if constexpr (!kSeal) header_checks(kSys ? xld16_sys(src, B) : kStage ? xld16_g(src, B) : xld16(src, B));
    }
  };
  // (kScalarKey, after the input's loads: a scheduling barrier and an empty asm per value,
  // so no use or copy of them -- and no wait for the header's PCIe round trip -- lands
  // among the loads)
  auto settle_key = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    constexpr int kHalves = G == 64u ? 1 : 2;
#pragma unroll
    for (int q = 0; q < kHalves; ++q) {
#pragma unroll
      for (int j = 0; j < 9; ++j) asm volatile("" : "+s"(kr[q][j]));
      if constexpr (!kSeal) asm volatile("" : "+s"(hr[q].x), "+s"(hr[q].y), "+s"(hr[q].z), "+s"(hr[q].w));
    }
    const bool h1 = kHalves == 2 && (threadIdx.x & 32u) != 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) key[j] = h1 ? kr[kHalves - 1][j] : kr[0][j];
    sidx = h1 ? kr[kHalves - 1][8] : kr[0][8];
    if constexpr (!kSeal) header_checks(h1 ? hr[kHalves - 1] : hr[0]);
  };
  // staged: the key (HBM) and the nonce -- seal's descriptor counter, or open's header
  // in a scalar load -- go out first, and the span's first keystream block, the Poly1305
  // key and the combine's first power of r are computed while the input crosses PCIe
  constexpr bool kEarlyKs = kStage && (kSeal || kScalarKey);
  if constexpr (kEarlyKs) {
    load_key();
    asm volatile("" ::: "memory");  // (the key and header loads go out before the input's)
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (kStage) {
    // (straight-line loads: a lane past the input reloads the input's last piece -- the
    // line its neighbours fetch in the same instruction -- and does not stage it.  A
    // per-lane zero default, or a branch around each load, makes the compiler copy, and
    // wait, after every load.  An empty seal reads nothing: its source may be null.)
    if (!kSeal || np_in != 0u) {  // (group-uniform; an open always has its tag)
#pragma unroll
      for (uint32_t k = 0; k < kBatch; ++k) {
        const uint32_t p = l + k * G, pp = p < np_in ? p : np_in - 1u;
        sv[k] = kSys ? xld16_sys(in + 16u * pp, B) : xld16_g(in + 16u * pp, B);
      }
    }
  } else {
    if (any) load_block(b0, x);
  }
  if constexpr (kScalarKey) settle_key();
  if constexpr (!kEarlyKs) load_key();
  const bool wr = kSeal || status == WG_STATUS_OK;  // (group-uniform)
  Poly ps;
  uint32_t ks[16];
  uint32_t rk[8];
  F26 r26, R0;  // (r, and r^(4 C): the combine's first level)
  // first block of the span (lane 0: block 0, the one-time key), r and s to every lane
  auto first_block = [&]() {
    if (any) {
      chacha20_block(ks, key, b0, n1, n2);
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) ks[j] = 0u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) rk[j] = gshfl<G>(ks[j], 0u);
    poly_init(ps, rk);
    r26 = f26_from32(ps.r0, ps.r1, ps.r2, ps.r3, 0u);
    R0 = Lu > 2u ? f26_pow(r26, 4u * C) : r26;
  };
  if constexpr (kEarlyKs) {
    asm volatile("" ::: "memory");  // (the input loads above go out before the keystream)
    first_block();
  }
  uint32_t tw[8] = {0, 0, 0, 0, 0, 0, 0, 0};          // open: the received tag's two pieces
  if constexpr (kStage) {
    lds_wave_sync();  // (the group's previous packet has left the stage)
#pragma unroll
    for (uint32_t k = 0; k < kBatch; ++k) {
      const uint32_t p = l + k * G;
      if (p < np_in) gb[p] = sv[k];
    }
    for (uint32_t p0 = kBatch * G; p0 < np_in; p0 += kBatch * G) {  // (packets past 8 G pieces)
#pragma unroll
      for (uint32_t k = 0; k < kBatch; ++k) {
        const uint32_t p = p0 + l + k * G;
        sv[k] = p < np_in ? (kSys ? xld16_sys(in + 16u * p, B) : xld16_g(in + 16u * p, B)) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (uint32_t k = 0; k < kBatch; ++k) {
        const uint32_t p = p0 + l + k * G;
        if (p < np_in) gb[p] = sv[k];
      }
    }
    lds_wave_sync();
    if (stamp) stamps[1] = wall_clock64();
    if (any) load_block(b0, x);
    if (!kSeal && l == Lu - 1u) {  // (before this lane's last block overwrites the tag's first bytes)
      const uint4 ta = gb[P >> 4], tb = (P & 15u) ? gb[(P >> 4) + 1u] : make_uint4(0, 0, 0, 0);
      tw[0] = ta.x; tw[1] = ta.y; tw[2] = ta.z; tw[3] = ta.w;
      tw[4] = tb.x; tw[5] = tb.y; tw[6] = tb.z; tw[7] = tb.w;
    }
  }

  uint32_t kpieces = 0;  // pieces this lane absorbed
  // one data block b >= 1: XOR, store, and (once r is known) absorb its pieces
  auto data_block = [&](uint32_t b, const uint32_t (&ks)[16], const uint4 (&x)[4]) {
    const uint32_t off = 64u * (b - 1u);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t o = off + 16u * (uint32_t)q;
      if (o >= P) break;
      const uint32_t valid = min(16u, P - o);
      uint32_t w[4] = {x[q].x ^ ks[4 * q], x[q].y ^ ks[4 * q + 1], x[q].z ^ ks[4 * q + 2], x[q].w ^ ks[4 * q + 3]};
      uint32_t c[4] = {kSeal ? w[0] : x[q].x, kSeal ? w[1] : x[q].y, kSeal ? w[2] : x[q].z, kSeal ? w[3] : x[q].w};
      if (valid < 16u) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          w[j] &= byte_mask((int)valid, j);
          c[j] &= byte_mask((int)valid, j);
        }
        if constexpr (kStage) gb[o >> 4] = make_uint4(w[0], w[1], w[2], w[3]);  // (in place, zeros past P)
        else if (wr) xstore_partial(out + o, w, (int)valid, B);
      } else if constexpr (kStage) {
        gb[o >> 4] = make_uint4(w[0], w[1], w[2], w[3]);
      } else if (wr) {
        xst16(out + o, w[0], w[1], w[2], w[3], B);
      }
      poly_block(ps, c[0], c[1], c[2], c[3]);
      ++kpieces;
    }
  };

  if constexpr (!kEarlyKs) first_block();
  if (any && b0 >= 1u) data_block(b0, ks, x);
  for (uint32_t b = b0 + 1u; b < b1; ++b) {
    load_block(b, x);
    chacha20_block(ks, key, b, n1, n2);
    data_block(b, ks, x);
  }

  // combine: T = sum_{l < Lu-1} h_l r^(S (Lu - 2 - l)) in lane Lu - 2, by levels
  F26 v = l + 1u < Lu ? f26_from32(ps.h0, ps.h1, ps.h2, ps.h3, ps.h4) : f26_zero();
  if (Lu > 2u) {
    F26 R = R0;
    const int dd = (int)Lu - 2 - (int)l;
    for (uint32_t k = 0; (1u << k) < Lu - 1u; ++k) {
      const uint32_t step = 1u << k;
      const F26 pv = gshfl26<G>(v, l >= step ? l - step : 0u);  // node d + 2^k
      if (dd >= 0 && ((uint32_t)dd & (2u * step - 1u)) == 0u && (uint32_t)dd + step <= Lu - 2u)
        v = f26_add(v, f26_mul(pv, R));
      if ((2u << k) < Lu - 1u) R = f26_mul(R, R);
    }
  }
  const F26 T = gshfl26<G>(v, Lu >= 2u ? Lu - 2u : 0u);
  uint32_t bad = 0u;
  if (l == Lu - 1u) {
    if (Lu >= 2u) {  // D = T r^(c_last) + h_last
      const F26 D = f26_add(f26_mul(T, f26_pow(r26, kpieces)),
                            f26_from32(ps.h0, ps.h1, ps.h2, ps.h3, ps.h4));
      f26_to32(D, ps.h0, ps.h1, ps.h2, ps.h3, ps.h4);
    }
    poly_block(ps, 0u, 0u, P, 0u);  // le64(AAD len = 0) | le64(P)
    const uint32_t s[4] = {rk[4], rk[5], rk[6], rk[7]};
    uint32_t tag[4];
    poly_finish(ps, s, tag);
    if (kSeal) {
      if constexpr (kStage) {  // (into the stage, after this lane's last ciphertext piece)
        uint8_t *t = reinterpret_cast<uint8_t *>(gb) + P;
#pragma unroll
        for (int q = 0; q < 16; ++q) t[q] = (uint8_t)(tag[q / 4] >> (8 * (q % 4)));
      } else {
        uint8_t *t = out + P;  // right after the ciphertext (session.rs:247-252)
        if (xok((uint64_t)t, 16u, B.out_lo, B.out_hi, B)) {
#pragma unroll
          for (int q = 0; q < 16; ++q) t[q] = (uint8_t)(tag[q / 4] >> (8 * (q % 4)));
        }
      }
    } else {
      // received tag = bytes [P, P + 16) after the header: two aligned pieces
      if constexpr (!kStage) {
        const uint32_t o = P & ~15u;
        const uint4 ta = xld16(in + o, B);
        const uint4 tb = (P & 15u) ? xld16(in + o + 16u, B) : make_uint4(0, 0, 0, 0);
        tw[0] = ta.x; tw[1] = ta.y; tw[2] = ta.z; tw[3] = ta.w;
        tw[4] = tb.x; tw[5] = tb.y; tw[6] = tb.z; tw[7] = tb.w;
      }
      const int sh = (int)(P & 15u);
#pragma unroll
      for (int j = 0; j < 4; ++j) bad |= bytes_at(tw, sh + 4 * j) ^ tag[j];
    }
  }
  if constexpr (kStage) {
    // the group's output, G consecutive pieces per store instruction (seal: ciphertext
    // + tag after the header; open: the plaintext, or ring's zeros on a failed tag)
    if (!kSeal) {
      bad = gshfl<G>(bad, Lu - 1u);
      if (bad && wr) status = WG_STATUS_INVALID_AEAD_TAG;
    }
    lds_wave_sync();
    if (stamp) stamps[2] = wall_clock64();
    if (wr) {
      const uint32_t nb_out = kSeal ? P + 16u : P, np_out = (nb_out + 15u) / 16u;
      for (uint32_t p = l; p < np_out; p += G) {
        const uint4 y = bad ? make_uint4(0, 0, 0, 0) : gb[p];
        const uint32_t o = 16u * p;
        if (o + 16u <= nb_out) {
          xst16(out + o, y.x, y.y, y.z, y.w, B);
        } else {
          const uint32_t yw[4] = {y.x, y.y, y.z, y.w};
          xstore_partial(out + o, yw, (int)(nb_out - o), B);
        }
      }
      if (kSeal && l == 0u) xst16(dst, WG_MSG_DATA, sidx, n1, n2, B);  // header (session.rs:224-229)
    }
    if (stamp) stamps[3] = wall_clock64();
  } else if (kSeal) {
    if (l == 0u) xst16(dst, WG_MSG_DATA, sidx, n1, n2, B);  // header (session.rs:224-229)
  } else {
    bad = gshfl<G>(bad, Lu - 1u);
    if (bad && wr) {
      status = WG_STATUS_INVALID_AEAD_TAG;
      // never leave unauthenticated plaintext behind: this lane's own stores land first
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t lo = b0 >= 1u ? 64u * (b0 - 1u) : 0u;
      const uint32_t hi = b1 >= 1u ? min(64u * (b1 - 1u), P) : 0u;
      const uint32_t zw[4] = {0, 0, 0, 0};
      for (uint32_t o = lo; o < hi; o += 16u) {
        if (o + 16u <= P) xst16(out + o, 0u, 0u, 0u, 0u, B);
        else xstore_partial(out + o, zw, (int)(P - o), B);
      }
    }
  }
  if (l == 0u && st) *st = status;
}

// The grid's completion word (DescParams::done_flag): each wave waits for its own
// stores (outputs and status) to be acknowledged, the workgroup meets at a barrier, and
// its thread 0 arrives on done_count with a system-scope release (one L2 write-back per
// workgroup; no acquire: nothing is read after it, and an acquire's L2 invalidate per
// wave cost 1024-packet calls 50 us, profiles/r05an); the last to arrive takes one
// system-scope acquire, resets the counter for the stream's next launch and
// publishes seq.  (Thread-indexed addresses:
// the counter and the word take vector memory operations.)
__device__ __forceinline__ void grid_done(uint32_t *count, uint32_t *flag, uint32_t seq) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0u) {
    const uint32_t prev = __hip_atomic_fetch_add(count + threadIdx.x, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (prev == gridDim.x - 1u) {
      // the one last arrival acquires every other workgroup's release, so the word
      // it publishes orders their outputs and statuses too (one invalidate per grid)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      __hip_atomic_store(count + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(flag + threadIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <bool kSeal, uint32_t G>
__global__ __launch_bounds__(kXlaneThreads) void aead_xlane_kernel(DescParams prm) {
  static_assert(G >= 2u && G <= 64u && (G & (G - 1u)) == 0u, "group = power of two within a wave");
  const uint32_t gid = blockIdx.x * (kXlaneThreads / G) + threadIdx.x / G;  // packet (batch position)
  const uint32_t l = threadIdx.x & (G - 1u);
  if (gid < prm.n) {  // (the whole group)
    const uint32_t idx = prm.order ? prm.order[gid] : gid;
    const wg_packet_desc d = prm.descs[idx];
    // (null bases: the offsets are absolute device addresses)
    const uint8_t *src = reinterpret_cast<const uint8_t *>(reinterpret_cast<uint64_t>(prm.src) + d.src_off);
    uint8_t *dst = reinterpret_cast<uint8_t *>(reinterpret_cast<uint64_t>(prm.dst) + d.dst_off);
    xlane_packet<kSeal, G>(l, src, dst, d.len, d.key_slot, d.counter, d.src_off | d.dst_off, prm.status + idx,
                           prm.keys, prm.key_index, prm.key_slots, idx);
  }
  if (prm.done_flag) grid_done(prm.done_count, prm.done_flag, prm.done_seq);  // (kernel-uniform)
}

// a packet of `len` input bytes fits a group's stage (xlane_packet kStage)
template <bool kSeal, uint32_t G>
__device__ __forceinline__ bool stage_fits(uint32_t len) {
  const uint32_t P = kSeal ? len : (len >= WG_DATA_OVERHEAD_SZ ? len - WG_DATA_OVERHEAD_SZ : 0u);
  return (P + 31u) / 16u <= stage_cap<G>();
}

// (the Tunn's small calls: packets in host memory -- staged where they fit)
template <bool kSeal, uint32_t G>
__global__ __launch_bounds__(kXlaneThreads) void aead_xlane_inline_kernel(XlaneInlineParams ip) {
  __shared__ uint4 stage[kXlaneStagePieces];
  const DescParams &prm = ip.prm;
  const uint32_t gid = blockIdx.x * (kXlaneThreads / G) + threadIdx.x / G;  // packet (batch position)
  const uint32_t l = threadIdx.x & (G - 1u);
  if (gid < prm.n) {  // (the host keeps n <= kXlaneInlineDescs)
    const wg_packet_desc d = ip.d[gid];
    const uint8_t *src = reinterpret_cast<const uint8_t *>(reinterpret_cast<uint64_t>(prm.src) + d.src_off);
    uint8_t *dst = reinterpret_cast<uint8_t *>(reinterpret_cast<uint64_t>(prm.dst) + d.dst_off);
    if (stage_fits<kSeal, G>(d.len))  // (group-uniform)
      xlane_packet<kSeal, G, true>(l, src, dst, d.len, d.key_slot, d.counter, d.src_off | d.dst_off,
                                   prm.status + gid, prm.keys, prm.key_index, prm.key_slots, gid,
                                   stage + (threadIdx.x / G) * stage_cap<G>());
    else
      xlane_packet<kSeal, G>(l, src, dst, d.len, d.key_slot, d.counter, d.src_off | d.dst_off, prm.status + gid,
                             prm.keys, prm.key_index, prm.key_slots, gid);
  }
  if (prm.done_flag) grid_done(prm.done_count, prm.done_flag, prm.done_seq);  // (kernel-uniform)
}

// Strided batches (wg_gpu_seal_strided / wg_gpu_open_strided without slot padding):
// packet i at src + i src_stride / dst + i dst_stride, one length and key slot, seal
// counter counter_base + i; the host has checked alignment and the slot
template <bool kSeal, uint32_t G>
__global__ __launch_bounds__(kXlaneThreads) void aead_xlane_strided_kernel(StridedParams prm) {
  const uint32_t i = blockIdx.x * (kXlaneThreads / G) + threadIdx.x / G;
  const uint32_t l = threadIdx.x & (G - 1u);
  if (i >= prm.n) return;
  xlane_packet<kSeal, G>(l, prm.src + (uint64_t)i * prm.src_stride, prm.dst + (uint64_t)i * prm.dst_stride, prm.len,
                         prm.key_slot, prm.counter_base + i, 0u, prm.status ? prm.status + i : nullptr, prm.keys,
                         prm.key_index, 0xffffffffu, i);
}

// ---------------------------------------------------------------------------
// Resident service (wg_aead_kernels.h SrvSlot; host side wg_tunn.cpp Service).
// NepTUN's workers hand the data plane at most 50 packets at a time from every
// physical core (packet_workers.rs:27, :113-131).  As launches, concurrent calls of
// this size queue on the process's hardware queues (~13 us of queue time each: 8
// callers ran 54 Gbit/s); posted to this kernel's slots, a call costs
// its PCIe round trips and no launch.
// ---------------------------------------------------------------------------
namespace {

// {seq, op, n, G} of a slot in one system-coherent 16-byte load (the host writes seq
// last, so a new seq comes with its own op / n / G)
typedef unsigned int srv_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 srv_poll(const SrvSlot *sl) {
  srv_u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
               : "=v"(v)
               : "v"(reinterpret_cast<uint64_t>(sl))
               : "memory");
  return make_uint4(v.x, v.y, v.z, v.w);
}

// this workgroup's packets of the request (lane: its index among the slot's lanes)
template <bool kSeal, uint32_t G>
__device__ __forceinline__ void srv_packets(SrvSlot *sl, uint32_t lane, uint32_t n, const SrvParams &p,
                                            uint4 *stage) {
  const uint32_t l = lane & (G - 1u);
  uint4 *gb = stage + ((lane % kXlaneThreads) / G) * stage_cap<G>();
  for (uint32_t i = lane / G; i < n; i += kSrvLanes / G) {  // (group-uniform)
    // the descriptor, past the caches (the host rewrote the slot since the last request)
    const uint4 d0 = ld16_sys(reinterpret_cast<const uint8_t *>(&sl->d[i]));
    const uint4 d1 = ld16_sys(reinterpret_cast<const uint8_t *>(&sl->d[i]) + 16u);
    const uint64_t so = (uint64_t)d0.x | ((uint64_t)d0.y << 32), dn = (uint64_t)d0.z | ((uint64_t)d0.w << 32);
    const uint64_t ctr = (uint64_t)d1.x | ((uint64_t)d1.y << 32);
    const uint32_t len = d1.z, kslot = d1.w;
    const uint8_t *src = reinterpret_cast<const uint8_t *>(so);
    uint8_t *dst = reinterpret_cast<uint8_t *>(dn);
    uint64_t *stamps = p.stamp && i == 0u ? sl->stamp + 5 : nullptr;  // (packet 0: stamp[5 ..])
    if (stamps && l == 0u) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamps[0] = wall_clock64();
    }
    if (stage_fits<kSeal, G>(len)) {
      xlane_packet<kSeal, G, true, true>(l, src, dst, len, kslot, ctr, so | dn, sl->st + i, p.keys, p.key_index,
                                         p.key_slots, i, gb, stamps);
    } else {  // (its plain loads: first drop what the caches hold of earlier requests)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      xlane_packet<kSeal, G>(l, src, dst, len, kslot, ctr, so | dn, sl->st + i, p.keys, p.key_index, p.key_slots, i);
    }
  }
}

}  // namespace

__global__ __launch_bounds__(kXlaneThreads) void xlane_service_kernel(SrvParams p) {
  __shared__ uint32_t s_req[5];
  __shared__ uint4 stage[kXlaneStagePieces];
  const uint32_t slot = blockIdx.x / kSrvGroup, part = blockIdx.x % kSrvGroup;
  SrvSlot *sl = p.slots + slot;
  const uint64_t t0 = wall_clock64();
  // the last request of this slot the host saw done (it posts the next one only then)
  uint32_t last = 0;
  if (threadIdx.x == 0u) last = __hip_atomic_load(&sl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    if (threadIdx.x == 0u) {
      uint32_t go = 0u;
      uint4 h = make_uint4(last, 0u, 0u, 0u);
      for (uint32_t i = 0;; ++i) {
        h = srv_poll(sl);
        if (h.x != last) {
          go = 1u;
          break;
        }
        if ((i & 15u) == 0u && (__hip_atomic_load(p.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u ||
                                wall_clock64() - t0 > p.lease_ticks))
          break;
        __builtin_amdgcn_s_sleep(1);
      }
      s_req[0] = go;
      s_req[1] = h.x;
      s_req[2] = h.y;
      s_req[3] = h.z;
      s_req[4] = h.w;
    }
    __syncthreads();
    const uint32_t go = s_req[0], seq = s_req[1], op = s_req[2], n = s_req[3], G = s_req[4];
    __syncthreads();  // (s_req is rewritten by the next poll)
    if (!go) return;  // (workgroup-uniform: stop or lease)
    const bool stamp = p.stamp && part == 0u && threadIdx.x == 0u;
    if (stamp) sl->stamp[0] = wall_clock64();
    // (the request's bytes -- descriptors, packets -- are read past the caches; no
    // per-request invalidate: with a slot's workgroups on many CUs it cost 3-4 us a
    // request under load, profiles/r06r)
    if (stamp) sl->stamp[1] = wall_clock64();
    const uint32_t lane = part * kXlaneThreads + threadIdx.x;
    if (n <= kSrvDescs && n * G <= kSrvLanes) {  // (the host never posts more)
      switch ((op ? 128u : 0u) | G) {
        case 128u | 64u: srv_packets<true, 64>(sl, lane, n, p, stage); break;
        case 128u | 32u: srv_packets<true, 32>(sl, lane, n, p, stage); break;
        case 128u | 16u: srv_packets<true, 16>(sl, lane, n, p, stage); break;
        case 128u | 8u: srv_packets<true, 8>(sl, lane, n, p, stage); break;
        case 64u: srv_packets<false, 64>(sl, lane, n, p, stage); break;
        case 32u: srv_packets<false, 32>(sl, lane, n, p, stage); break;
        case 16u: srv_packets<false, 16>(sl, lane, n, p, stage); break;
        case 8u: srv_packets<false, 8>(sl, lane, n, p, stage); break;
        default: break;
      }
    }
    // arrival: this workgroup's outputs and statuses acknowledged, one system-scope
    // release each; the last of the slot's workgroups publishes seq (grid_done's shape)
    if (stamp) sl->stamp[2] = wall_clock64();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (stamp) sl->stamp[3] = wall_clock64();
    if (threadIdx.x == 0u) {
      uint32_t *cnt = p.d_count + (threadIdx.x + slot * 32u);
      const uint32_t prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (prev == kSrvGroup - 1u) {
        if (p.stamp) sl->stamp[4] = wall_clock64();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sl->done + threadIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      last = seq;
    }
  }
}

template __global__ void aead_xlane_kernel<true, 64>(DescParams);
template __global__ void aead_xlane_kernel<false, 64>(DescParams);
template __global__ void aead_xlane_kernel<true, 32>(DescParams);
template __global__ void aead_xlane_kernel<false, 32>(DescParams);
template __global__ void aead_xlane_kernel<true, 16>(DescParams);
template __global__ void aead_xlane_kernel<false, 16>(DescParams);
template __global__ void aead_xlane_kernel<true, 8>(DescParams);
template __global__ void aead_xlane_kernel<false, 8>(DescParams);
template __global__ void aead_xlane_kernel<true, 4>(DescParams);
template __global__ void aead_xlane_kernel<false, 4>(DescParams);
template __global__ void aead_xlane_kernel<true, 2>(DescParams);
template __global__ void aead_xlane_kernel<false, 2>(DescParams);

#define WG_XLANE_INLINE(S, G) template __global__ void aead_xlane_inline_kernel<S, G>(XlaneInlineParams);
WG_XLANE_INLINE(true, 64) WG_XLANE_INLINE(false, 64) WG_XLANE_INLINE(true, 32) WG_XLANE_INLINE(false, 32)
WG_XLANE_INLINE(true, 16) WG_XLANE_INLINE(false, 16) WG_XLANE_INLINE(true, 8) WG_XLANE_INLINE(false, 8)
WG_XLANE_INLINE(true, 4) WG_XLANE_INLINE(false, 4) WG_XLANE_INLINE(true, 2) WG_XLANE_INLINE(false, 2)
#undef WG_XLANE_INLINE

template __global__ void aead_xlane_strided_kernel<true, 64>(StridedParams);
template __global__ void aead_xlane_strided_kernel<false, 64>(StridedParams);
template __global__ void aead_xlane_strided_kernel<true, 32>(StridedParams);
template __global__ void aead_xlane_strided_kernel<false, 32>(StridedParams);
template __global__ void aead_xlane_strided_kernel<true, 16>(StridedParams);
template __global__ void aead_xlane_strided_kernel<false, 16>(StridedParams);
template __global__ void aead_xlane_strided_kernel<true, 8>(StridedParams);
template __global__ void aead_xlane_strided_kernel<false, 8>(StridedParams);
template __global__ void aead_xlane_strided_kernel<true, 4>(StridedParams);
template __global__ void aead_xlane_strided_kernel<false, 4>(StridedParams);
template __global__ void aead_xlane_strided_kernel<true, 2>(StridedParams);
template __global__ void aead_xlane_strided_kernel<false, 2>(StridedParams);

}  // namespace wg

// Checked build's record: out = {violations, first address, its packet, its lane};
// reset != 0 clears it.  Returns 0, or -1 when this library is not the checked build.
extern "C" int wg_gpu_debug_xlane_check(unsigned long long *out, int reset) {
#if WG_XLANE_CHECK
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(wg::g_xlane_check), sizeof(wg::g_xlane_check)) != hipSuccess)
    return -2;
  if (reset) {
    const unsigned long long z[4] = {0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(wg::g_xlane_check), z, sizeof z) != hipSuccess) return -2;
  }
  return 0;
#else
  (void)out; (void)reset;
  return -1;
#endif
}
