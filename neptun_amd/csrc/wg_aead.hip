// wg_aead.hip -- MI355X (gfx950 / CDNA4) WireGuard transport-data AEAD kernels.
//
// Hand-written HIP for NepTUN's per-packet ChaCha20-Poly1305 seal/open:
//   seal = Session::format_packet_data   (neptun/src/noise/session.rs:205-259)
//   open = parse_incoming_packet DATA arm (noise/mod.rs:139-199) +
//          Session::receive_packet_data  (session.rs:265-302, replay window on host)
// The AEAD is RFC 8439 (what ring 0.17.14's CHACHA20_POLY1305 computes).
//
// Execution model (DESIGN.md "Kernels"):
//   * compute: one packet per wavefront lane.  A wave64 owns 64 packets and
//     walks them in lockstep, one 128-byte "run" of every packet per round;
//     the 16 ChaCha20 state words of the lane's packet live in VGPRs (the key
//     in SGPRs for single-session batches), two 64-byte keystream blocks per
//     round, Poly1305 accumulated per lane in radix 2^32.
//   * memory: runs are staged through LDS.  Loads are LDS-DMA
//     (global_load_lds_dwordx4), 8 packets x 128 contiguous bytes per 1 KiB
//     wave instruction; stores go LDS -> VGPR -> global_store_dwordx4 in the
//     same shape.  Every 128-byte line of a 128-byte-aligned slot is read or
//     written whole by one instruction (measured: the lane-strided alternative
//     moved 2.5-2.9x the algorithmic bytes through HBM, profiles/r01_*).  The
//     LDS image is XOR-swizzled so a lane reading its own run is bank-
//     conflict-free.
//   * coordinates: everything is indexed in "wire coordinates" w = byte offset
//     in the datagram (header 0..15, ciphertext 16..16+P, tag after it).  The
//     plaintext side is addressed as base - 16 + w, so when plaintext sits 16
//     bytes into a slot (NepTUN's WG_HEADER_OFFSET layout, device/mod.rs:76)
//     both sides' runs are 128-byte aligned.  Any 16-byte-aligned layout is
//     correct; that one is also fastest.
// No MFMA: this is a stream cipher + MAC, not a contraction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "neptun_gpu.h"
#include "wg_aead_kernels.h"
#include "wg_crypto.h"

namespace wg {

constexpr uint32_t kRun = 128;    // bytes of one packet per round (one cache line)
constexpr uint32_t kChunks = 8;   // 16-byte chunks per run
constexpr uint32_t kWaves = kBlockThreads / 64;  // generic kernels

// timing-only ablations (wrong outputs): skip the HBM traffic / skip the crypto
#ifndef WG_ABLATE_NO_MEM
#define WG_ABLATE_NO_MEM 0
#endif
#ifndef WG_ABLATE_NO_CRYPT
#define WG_ABLATE_NO_CRYPT 0
#endif

// timing-only energy / bound probes (wrong outputs): no Poly1305 blocks / no
// LDS traffic of the crypt step (text words taken from registers, results
// dropped).  DESIGN.md 3.1 has what they showed.
#ifndef WG_ABLATE_NO_POLY
#define WG_ABLATE_NO_POLY 0
#endif
#ifndef WG_ABLATE_NO_LDS_CRYPT
#define WG_ABLATE_NO_LDS_CRYPT 0
#endif
#ifndef WG_ABLATE_ALL_INTERIOR
#define WG_ABLATE_ALL_INTERIOR 0  // every round staged as a full 128-byte run (edge bytes wrong)
#endif
#ifndef WG_ABLATE_NO_KEYBLOCK
#define WG_ABLATE_NO_KEYBLOCK 0  // seal: skip the per-packet Poly1305 key block
#endif
// Wave priority of the memory phase of a phase-locked round (0: unchanged):
// from the landing wait (WG_MEM_PRIO_AT 0) or from the stores (1) until the
// next round's keystream steps set their own (WG_CHACHA_PRIO).
#ifndef WG_MEM_PRIO
#define WG_MEM_PRIO 0
#endif
#ifndef WG_MEM_PRIO_AT
#define WG_MEM_PRIO_AT 0
#endif
#ifndef WG_ABLATE_PURE_COPY
#define WG_ABLATE_PURE_COPY 0  // uniform kernels: staging loop only (a copy), no setup, no crypto
#endif

#ifndef WG_WAVES_PER_SIMD
#define WG_WAVES_PER_SIMD 1  // __launch_bounds__ min waves per SIMD (VGPR cap)
#endif

#ifndef WG_FULL_LINES
#define WG_FULL_LINES 1  // uniform kernels: edge rounds moved as whole lines where the host allows it
#endif

// The lane index and P opaque to the optimiser once per round (run_wave):
// lane-derived LDS addresses, buffer offsets and the tail chunk's byte masks are
// then recomputed each round instead of being computed once per kernel and held
// in VGPRs through every round.  Descriptor kernels: fewer spills, config 4
// -1.2 %; uniform kernels: +1 % open, off.
#ifndef WG_OPAQUE_LANE
#define WG_OPAQUE_LANE 0
#endif
#ifndef WG_OPAQUE_LANE_DESC
#define WG_OPAQUE_LANE_DESC 1
#endif

// descriptor kernels (per-lane keys): the shared first diagonal round too (the
// two blocks' columns 1-3 are equal after the first column round whatever the key)
#ifndef WG_SHARED_DIAG_DESC
#define WG_SHARED_DIAG_DESC 0
#endif

// descriptor kernels: the SGPR-key form for waves whose live packets share one
// key slot.  Measured -0.5 % on config 3 (its only single-key config) and -0.3 %
// on config 4: off (profiles/r03_ab_desc_forms.txt)
#ifndef WG_DESC_UNIFORM_KEY
#define WG_DESC_UNIFORM_KEY 0
#endif
// descriptor kernels: the full-round fast path (run_wave).  Measured +0.3 % on
// config 4 and +0.1 % on config 3 (noise level), but its register pressure spills
// 6-7 VGPRs per group (+1.5 % config-4 HBM traffic): off
// (profiles/r03_ab_desc_forms.txt)
#ifndef WG_DESC_FULL_ROUNDS
#define WG_DESC_FULL_ROUNDS 0
#endif

// uniform kernels' persistent walk: each XCD's workgroups on one contiguous eighth of
// the batch (A/B knob, off: profiles/r03v_ab_xcd_walk.txt)
#ifndef WG_XCD_CONTIG
#define WG_XCD_CONTIG 0
#endif

#ifndef WG_HDR_NT
#define WG_HDR_NT 0  // open's early header fetch with the streaming (nt) policy
#endif
// uniform open: each group's headers prefetched into the tag park during the
// previous group (its round 1), when the tag lies wholly in the last round and a
// stage chunk past the datagram is free there (the tag is then checked inside the
// last round, and the park is free from round 1 on): the group start no longer
// waits for a header fetch before its one-time key
#ifndef WG_OPEN_HDR_PREFETCH
#define WG_OPEN_HDR_PREFETCH 0
#endif
#ifndef WG_HDR_DMA
#define WG_HDR_DMA 1  // uniform open: headers by LDS-DMA ahead of round 0, counted vmcnt(8) wait
#endif

#ifndef WG_ABLATE_ZEROING
#define WG_ABLATE_ZEROING 0  // timing-only: forged packets keep their plaintext
#endif

// Cache policy of the streaming traffic (every byte is read once and written
// once), as LLVM CPol bits for gfx940+: 1 = sc0, 2 = nt, 16 = sc1 (and sums).
// The kernels are power-capped (PPT 1400 W, profiles/r02_power.json), so what
// the memory hierarchy spends per byte is clock the VALU does not get:
// non-temporal loads and stores (nt) run config 2's round trip 2.5 % and
// config 4's 2.9 % faster than the default policy (profiles/r02_ab_cache_policy.txt;
// nt stores alone let the seal run at 2.09 instead of 1.90 GHz under the same
// limit).  (Round 1 measured nt 8 % slower, on kernels not yet at the limit.)
#ifndef WG_LOAD_CPOL
#define WG_LOAD_CPOL 2
#endif
#ifndef WG_STORE_CPOL
#define WG_STORE_CPOL 2
#endif
// the text grid's loads (open into offset-0 destinations): each 128-byte run of
// the datagram starts 16 bytes into a line, so every line is read by two rounds
// (its head in round r, the rest in round r + 1).  As nt loads HBM served such
// a line twice (PMC: 2.80 GB read per 1M x 1350 B open against 1.48 GB on the
// wire grid, profiles/pmc_traffic_config2_neptun.json); with the default policy
// the line stays in L2 for the second read: open 0.815 -> 0.758 ms
// (profiles/r03_ab_text_grid.txt)
#ifndef WG_TEXT_LOAD_CPOL
#define WG_TEXT_LOAD_CPOL 0
#endif
// the text grid's two kinds of load piece, each its own instruction (exec-masked):
// a run's chunk 7 is the HEAD of the next datagram line (its first access, read
// again by the next round) and chunks 0-6 the BODY of this line (its last access)
#ifndef WG_TEXT_SPLIT
#define WG_TEXT_SPLIT 0
#endif
#ifndef WG_TEXT_HEAD_CPOL
#define WG_TEXT_HEAD_CPOL 0
#endif
#ifndef WG_TEXT_BODY_CPOL
#define WG_TEXT_BODY_CPOL 2
#endif
// (equal policies: the compiler merges the two arms into one load per piece, and
// open's header wait, which counts 16 load instructions per round, runs early)
#if WG_TEXT_SPLIT && WG_TEXT_HEAD_CPOL == WG_TEXT_BODY_CPOL
#error "WG_TEXT_SPLIT needs two different cache policies"
#endif
// Measured (profiles/r03l_ab_text_split.txt): body nt / head default cut the open's
// HBM reads 2.76 -> 2.36 GB per launch (the head lines stay in L2 more often) but
// not its time (0.775 vs 0.773 ms): off.
// the owner-lane stores of a packet's partial last chunk (dword / short / byte,
// no slot padding) keep the default policy: as nt stores their partial writes
// made an unpadded round trip 18 % slower
#ifndef WG_PARTIAL_STORE_CPOL
#define WG_PARTIAL_STORE_CPOL 0
#endif
#ifndef WG_EDGE_STORE_NT
#define WG_EDGE_STORE_NT 0  // unpadded edge rounds' 16-byte stores: 0 = default policy
#endif
#define WG_CPOL_ASM_0 ""
#define WG_CPOL_ASM_1 " sc0"
#define WG_CPOL_ASM_2 " nt"
#define WG_CPOL_ASM_3 " sc0 nt"
#define WG_CPOL_ASM_16 " sc1"
#define WG_CPOL_ASM_17 " sc0 sc1"
#define WG_CPOL_ASM_18 " nt sc1"
#define WG_CPOL_ASM_19 " sc0 nt sc1"
#define WG_CPOL_ASM_(x) WG_CPOL_ASM_##x
#define WG_CPOL_ASM(x) WG_CPOL_ASM_(x)
#define WG_LOAD_NT_ASM WG_CPOL_ASM(WG_LOAD_CPOL)
#define WG_STORE_NT_ASM WG_CPOL_ASM(WG_STORE_CPOL)
#define WG_PARTIAL_STORE_ASM WG_CPOL_ASM(WG_PARTIAL_STORE_CPOL)

#ifndef WG_SYNC_KEY_BLOCK
#define WG_SYNC_KEY_BLOCK 1  // phase-locked Poly1305 key block on the sync paths
#endif
#ifndef WG_SYNC_OPEN_KEY
#define WG_SYNC_OPEN_KEY 1  // open (uniform batches): phase-locked key block once the headers landed
#endif

// Diagnostic build only (-DWG_STAMP=1): s_memtime at the phase boundaries of
// the phase-locked loop, wave 0 of every workgroup, read back with
// wg_gpu_debug_stamps() (tools/stamps.py).  Never part of the product build.
#ifndef WG_STAMP
#define WG_STAMP 0
#endif
#if WG_STAMP
constexpr int kStampBlocks = 4096, kStampRounds = 16, kStampPhases = 6;
__device__ uint64_t g_stamps[2][kStampBlocks][kStampRounds][kStampPhases];
// s_memrealtime (100 MHz) beside each round's start stamp: the in-kernel shader
// clock is d(s_memtime) / d(s_memrealtime) x 100 MHz (tools/clock_trace.py)
__device__ uint64_t g_realtime[2][kStampBlocks][kStampRounds];
#define WG_STAMP_AT(seal, r, ph)                                                              \
  do {                                                                                      \
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0 && lane == 0 &&                \
        blockIdx.x < kStampBlocks && (r) < kStampRounds) {                                  \
      g_stamps[seal][blockIdx.x][r][ph] = __builtin_amdgcn_s_memtime();                     \
      if ((ph) == 0) g_realtime[seal][blockIdx.x][r] = __builtin_amdgcn_s_memrealtime();   \
    }                                                                                       \
  } while (0)
#else
#define WG_STAMP_AT(seal, r, ph) do {} while (0)
#endif

// LDS of one wave.  Generic geometry: one 8 KiB run buffer + per-packet tables.
struct WaveStage {
  uint4 run[1][64 * kChunks];  // [buffer][packet][chunk ^ swz(packet)], 8 KiB
  uint64_t in_base[64];        // wire-coordinate origin of the input side
  uint64_t out_base[64];       // wire-coordinate origin of the output side
  uint32_t wlen[64];           // W = datagram length (P + 32)
  uint32_t nruns[64];          // rounds this packet takes part in; 0 = none
  uint4 park[64];              // per-packet Poly1305 "s" half of the one-time key
  static constexpr bool kTagPark = false;
};
// Uniform geometry: one run buffer, no tables (addresses are arithmetic).
struct WaveStageUniform {
  uint4 run[1][64 * kChunks];
  uint4 park[64];  // per-packet Poly1305 "s" (parked here: VGPRs are the scarce resource)
  uint4 tagp[64];  // open: the received tag (ditto; 2 x 8 waves x 10 KiB = the whole LDS)
  static constexpr bool kTagPark = true;
};

// XOR swizzle of a packet's 8 chunk slots: lane L reading or writing chunk k
// of its own run hits slot 8L + (k ^ swz(L)).  Conflict-free for both banking
// modes of MI355X_MICROARCH.md "LDS": ds_read_b128 (lane groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31}, ..., 64 banks: 16-byte slot
// 8(L&1) + (k ^ swz)) and ds_write_b128 (8 contiguous lanes, 32 banks: slot
// k ^ swz).  (L>>1)&7 alone left every write 2-way conflicted (L, L^1 on one
// slot): PMC SQ_LDS_BANK_CONFLICT was a third of SQ_LDS_IDX_ACTIVE.
__device__ __forceinline__ uint32_t swz(uint32_t p) { return ((p >> 1) & 7u) ^ ((p & 1u) << 2); }

__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, 64));
  return x;
}

__device__ __forceinline__ uint64_t rl64(uint64_t x, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t wave_min32(uint32_t x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o, 64));
  return __builtin_amdgcn_readfirstlane(x);
}
// wave-uniform copy of lane 0's 64-bit value.  (readfirstlane returns int:
// each half must be taken back to uint32_t before widening, or a low half with
// bit 31 set sign-extends over the high half.)
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t y = (uint64_t)__shfl_xor((long long)x, o, 64);
    x = y < x ? y : x;
  }
  return uniform64(x);
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t y = (uint64_t)__shfl_xor((long long)x, o, 64);
    x = y > x ? y : x;
  }
  return uniform64(x);
}

__device__ __forceinline__ void lds_wait_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Run grids.  The wire grid (kText = false) cuts every packet into 128-byte
// runs of the DATAGRAM (grid coordinate = wire offset): seal's output and
// NepTUN's TUN-buffer plaintext (16 bytes in) both sit on it.  The text grid
// (open only) cuts the TEXT into runs (grid coordinate = wire offset - 16): for
// plaintext destinations that start on a 128-byte boundary, so every output
// line is written whole, in one round (the datagram header is then outside the
// grid and fetched on its own).
template <bool kSeal, bool kText = false>
struct Ranges {
  // input bytes live in [in_lo, in_hi) and output bytes in [out_lo, out_hi) of grid coordinates
  static_assert(!(kSeal && kText), "the text grid is for open");
  __device__ static uint32_t in_lo() { return kSeal ? 16u : 0u; }
  __device__ static uint32_t in_hi(uint32_t W) { return kSeal || kText ? W - 16u : W; }
  __device__ static uint32_t out_lo() { return kSeal || kText ? 0u : 16u; }
  __device__ static uint32_t out_hi(uint32_t W) { return kSeal ? W : kText ? W - 32u : W - 16u; }
};

// Per-packet geometry of the wave's 64 packets, two flavours:
//  * LdsGeom: arbitrary per-packet layout (descriptor batches, or the last,
//    partial wave of a strided batch) -- read from the WaveStage tables;
//  * UniformGeom: one length, strided slots, all 64 lanes live -- arithmetic,
//    wave-uniform lengths, so every length-dependent branch is a scalar one.
struct LdsGeom {
  static constexpr bool kTextGrid = false;
  WaveStage &S;
  __device__ bool live(uint32_t p, uint32_t r) const { return r < S.nruns[p]; }
  __device__ uint32_t wlen(uint32_t p) const { return S.wlen[p]; }
  __device__ uint64_t in_base(uint32_t p) const { return S.in_base[p]; }
  __device__ uint64_t out_base(uint32_t p) const { return S.out_base[p]; }
};

// Phase-locked descriptor batches: 8 waves x (this + 1 KiB of park) must fit
// twice in 160 KiB, so the per-packet tables are compact -- stage origins in
// 16-byte units from base - 16 (64 GiB reach), one length word (0 = no part).
struct WaveStageDesc {
  uint4 run[1][64 * kChunks];
  uint32_t in16[64], out16[64];  // wire-coordinate origins: ref + 16 * (hi:lo)
  uint8_t in_hi[64], out_hi[64];
  uint32_t wlen[64];             // W = datagram length; 0 = not staged
  uint4 park[64];
  static constexpr bool kTagPark = false;  // (no LDS left for it)
};

struct DescGeom {
  static constexpr bool kTextGrid = false;
  WaveStageDesc &S;
  uint64_t in_ref, out_ref;      // src - 16, dst - 16
  uint32_t *wg_rounds;           // [waves] round counts of the workgroup's waves
  uint32_t wave, alive;          // this wave, waves of the workgroup with packets
  // Fast addressing (per group, wave-uniform; set by set()): when every staged
  // packet of the wave lies within +-1 GiB of the wave's first staged packet on
  // each side, in16 / out16 hold BYTE offsets from that anchor - 1 GiB
  // (kNoAccess for packets not staged) and every round goes through one buffer
  // resource per side with 32-bit offsets: the rounds in [r_in0, r_in1) /
  // [r_out0, r_out1), where every staged packet moves a full 128-byte run, with
  // 1 VALU op per piece; the edge rounds with per-piece range masks (offset
  // kNoAccess = no access) and owner-lane stores of each packet's partial last
  // chunk (stage_in / stage_out overloads below).  Otherwise per-lane 64-bit
  // addresses (the generic path).
  bool fast = false;
  uint64_t in_wave = 0, out_wave = 0;
  uint32_t r_in0 = 0, r_in1 = 0, r_out0 = 0, r_out1 = 0;
  __device__ bool live(uint32_t p, uint32_t r) const { return kRun * r < S.wlen[p]; }
  __device__ uint32_t wlen(uint32_t p) const { return S.wlen[p]; }
  __device__ uint64_t in_base(uint32_t p) const {
    if (fast) return in_wave + S.in16[p];
    return in_ref + 16ull * (((uint64_t)S.in_hi[p] << 32) | S.in16[p]);
  }
  __device__ uint64_t out_base(uint32_t p) const {
    if (fast) return out_wave + S.out16[p];
    return out_ref + 16ull * (((uint64_t)S.out_hi[p] << 32) | S.out16[p]);
  }
  // the anchor of the fast offsets: the first staged lane's origin - 1 GiB
  __device__ static uint64_t anchor(uint64_t x, int l0) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l0);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l0);
    const uint64_t a = ((uint64_t)hi << 32) | lo;
    return a > (1ull << 30) ? a - (1ull << 30) : 0ull;
  }
  // (host side: src and dst are non-null, so offsets stay below 2^44 bytes)
  template <bool kSeal>
  __device__ void set(uint32_t lane, uint64_t in_base, uint64_t out_base, uint32_t W, bool ok) {
    const uint32_t ihi = ok ? (kSeal ? W - 16u : W) : 0u;   // Ranges<kSeal>::in_hi
    const uint32_t ohi = ok ? (kSeal ? W : W - 16u) : 0u;   // Ranges<kSeal>::out_hi
    const uint64_t live_lanes = __ballot(ok);
    fast = live_lanes != 0ull;
    if (fast) {
      const int l0 = (int)__builtin_amdgcn_readfirstlane((uint32_t)__builtin_ctzll(live_lanes));
      const uint64_t ia = anchor(in_base, l0), oa = anchor(out_base, l0);
      const uint64_t io = in_base - ia, oo = out_base - oa;
      // every byte a staged packet moves (its extent + a 16-byte tail chunk)
      // stays below kNoAccess, and kNoAccess + 128 r never wraps; a packet
      // more than 1 GiB below the anchor would wrap io / oo:
      // such a wave takes the generic path
      const bool far = ok && (in_base < ia || out_base < oa ||
                              io + ihi + 16u >= kNoAccessOffset - 1024u ||
                              oo + ohi + 16u >= kNoAccessOffset - 1024u);
      fast = __ballot(far) == 0ull;
      if (fast) {
        in_wave = ia;
        out_wave = oa;
        // full-run rounds: 128 r >= lo and 128 (r + 1) <= hi for every staged packet
        r_in0 = kSeal ? 1u : 0u;
        r_out0 = kSeal ? 0u : 1u;
        r_in1 = wave_min32(ok ? ihi / kRun : 0xffffffffu);
        r_out1 = wave_min32(ok ? ohi / kRun : 0xffffffffu);
        S.in16[lane] = ok ? (uint32_t)io : kNoAccessOffset;
        S.out16[lane] = ok ? (uint32_t)oo : kNoAccessOffset;
      }
    }
    if (!fast) {
      const uint64_t i16 = (in_base - in_ref) >> 4, o16 = (out_base - out_ref) >> 4;
      S.in16[lane] = (uint32_t)i16;
      S.in_hi[lane] = (uint8_t)(i16 >> 32);
      S.out16[lane] = (uint32_t)o16;
      S.out_hi[lane] = (uint8_t)(o16 >> 32);
    }
    S.wlen[lane] = ok ? W : 0u;
  }
  __device__ void kill(uint32_t lane) {
    S.wlen[lane] = 0u;
    if (fast) {
      S.in16[lane] = kNoAccessOffset;
      S.out16[lane] = kNoAccessOffset;
    }
  }
  // the workgroup's round count (every wave must run the same barrier steps)
  __device__ uint32_t wg_max(uint32_t wave_rounds) const {
    if ((threadIdx.x & 63u) == 0u) wg_rounds[wave] = wave_rounds;
    __syncthreads();
    uint32_t m = 0;
    for (uint32_t w = 0; w < alive; ++w) m = max(m, wg_rounds[w]);
    __syncthreads();  // the slots are rewritten by the next group
    return m;
  }
};

template <bool kText>
struct UniformGeomT {
  static constexpr bool kTextGrid = kText;
  uint64_t in0, out0, in_stride, out_stride;  // grid origins of packet 0, slot strides
  uint64_t dead;   // wave mask of packets dropped at the header check (open)
  uint32_t W, nr;  // datagram length and rounds, same for every packet
  uint32_t pad;    // slot padding: zero-fill each output to its 128-byte line end
  uint32_t full_in;  // input runs on whole 128-byte lines: every round loads whole lines
  __device__ bool live(uint32_t p, uint32_t r) const { return r < nr && !((dead >> p) & 1u); }
  __device__ uint32_t wlen(uint32_t) const { return W; }
  __device__ uint64_t in_base(uint32_t p) const { return in0 + (uint64_t)p * in_stride; }
  __device__ uint64_t out_base(uint32_t p) const { return out0 + (uint64_t)p * out_stride; }
};
using UniformGeom = UniformGeomT<false>;

// Memory instructions of the generic (per-packet address) staging, written so
// that the compiler inserts no waits of its own between them:
//  * the LDS-DMA is inline asm -- for the builtin the compiler drains vmcnt
//    before every later LDS read (here: the per-packet tables read for the
//    next piece), which serialised the 8 pieces of a round;
//  * stores go to the global address space -- a flat store may alias LDS, so
//    the compiler drained every in-flight LDS-DMA before each one;
//  * asm instructions carry their own wait states (the compiler's hazard
//    recognizer does not look inside inline asm): five after an SGPR/m0
//    write before the DMA reads them, two after a 16-byte store before its
//    data registers may be rewritten.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) uint8_t gbyte;
typedef __attribute__((address_space(1))) uint16_t gshort;
typedef __attribute__((address_space(1))) uint32_t gword;

__device__ __forceinline__ uint32_t lds_offset(const uint4 *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint4 *)p;
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// kStream = false: the default cache policy -- for open's early header fetch,
// whose line round 0 loads again right after (as nt, HBM served that line
// twice: +1.1 % of open's traffic, PMC)
template <bool kStream = true>
__device__ __forceinline__ void dma_global(uint32_t lds, const uint8_t *src) {
  if constexpr (kStream)
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 4\n\tglobal_load_lds_dwordx4 %1, off" WG_LOAD_NT_ASM
                 :: "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(src) : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 4\n\tglobal_load_lds_dwordx4 %1, off"
                 :: "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(src) : "memory", "m0");
}
#pragma clang diagnostic pop

// kStream = false: the default cache policy (stores into partly written lines,
// see store16)
template <bool kStream = true>
__device__ __forceinline__ void gstore16(uint8_t *dst, const uint4 v) {
  const u32x4 vv = {v.x, v.y, v.z, v.w};
  if constexpr (kStream)
    asm volatile("global_store_dwordx4 %0, %1, off" WG_STORE_NT_ASM "\n\ts_nop 1" :: "v"(dst), "v"(vv)
                 : "memory");
  else
    asm volatile("global_store_dwordx4 %0, %1, off" WG_PARTIAL_STORE_ASM "\n\ts_nop 1" :: "v"(dst),
                 "v"(vv) : "memory");
}

// the first k (1..15) bytes of a chunk, through global-address-space pointers
__device__ __forceinline__ void gstore_partial(uint8_t *p, const uint32_t w[4], int k) {
  gbyte *g = (gbyte *)p;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int v = k - 4 * j;
    if (v >= 4) {
      *(gword *)(g + 4 * j) = w[j];
    } else if (v > 0) {
      gbyte *pb = g + 4 * j;
      if (v >= 2) {
        *(gshort *)pb = (uint16_t)w[j];
        if (v == 3) pb[2] = (uint8_t)(w[j] >> 16);
      } else {
        pb[0] = (uint8_t)w[j];
      }
    }
  }
}

// Cooperative LDS-DMA load of round r: instruction j carries packets 8j..8j+7,
// lane i moves 16 bytes (chunk (i&7)^swz(p)) of packet p = 8j + i/8.
template <bool kSeal, class Geom>
__device__ __forceinline__ void stage_in(uint4 *run, const Geom &g, uint32_t lane, uint32_t r) {
#pragma unroll
  for (uint32_t j = 0; j < kChunks; ++j) {
    const uint32_t p = 8u * j + (lane >> 3);
    const uint32_t k = (lane & 7u) ^ swz(p);
    const uint32_t w = kRun * r + 16u * k;
    if (g.live(p, r) && w >= Ranges<kSeal>::in_lo() && w < Ranges<kSeal>::in_hi(g.wlen(p)))
      dma_global(lds_offset(&run[64u * j]), reinterpret_cast<const uint8_t *>(g.in_base(p)) + w);
  }
}

// Cooperative store of round r (same shape); the last chunk of a packet may be partial.
template <bool kSeal, class Geom>
__device__ __forceinline__ void stage_out(uint4 *run, const Geom &g, uint32_t lane, uint32_t r) {
#pragma unroll
  for (uint32_t j = 0; j < kChunks; ++j) {
    const uint32_t p = 8u * j + (lane >> 3);
    const uint32_t k = (lane & 7u) ^ swz(p);
    const uint32_t w = kRun * r + 16u * k;
    const uint32_t hi = Ranges<kSeal>::out_hi(g.wlen(p));
    if (g.live(p, r) && w >= Ranges<kSeal>::out_lo() && w < hi) {
      const uint4 v = run[64u * j + lane];
      uint8_t *dst = reinterpret_cast<uint8_t *>(g.out_base(p)) + w;
      const uint32_t n = hi - w;
      if (n >= 16u) {
        gstore16<WG_EDGE_STORE_NT != 0>(dst, v);  // (edge rounds: lines partly written)
      } else {
        const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
        gstore_partial(dst, wv, (int)n);
      }
    }
  }
}

// Uniform-geometry forms: buffer instructions with a wave-uniform resource
// (SGPRs) whose base is the wave's first packet, a wave-uniform soffset
// (8j packets + 128r bytes) and a 32-bit per-lane voffset -- 2 offset VGPRs
// for all 16 memory instructions of a round instead of 16 64-bit addresses.
// For p = 8j + (lane>>3): swz(p) = (lane>>4) ^ 4*(j&1) ^ 4*((lane>>3)&1).
// Every round issues exactly 8 loads and 8 full-chunk stores: a lane with no
// byte to move gets an offset past the resource's num_records, which the
// buffer range check turns into no memory access.  That keeps vmcnt counts
// static, which the double-buffered prefetch relies on.
constexpr uint32_t kNoAccess = kNoAccessOffset;  // >= any num_records used below

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(uint64_t base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), (short)0, (int)bytes,
                                           0x00020000);
}

// 16-byte buffer store with wait states after it.  The store reads its data
// VGPRs a few cycles after issue; for a buffer store with an SGPR soffset the
// compiler does not model that hazard and may overwrite the data registers in
// the very next VALU instruction -- measured on MI355X: some lanes then store
// the new values (tools/diff_variants.py found 1 % of packets corrupted in a
// build whose register allocation did that).  The asm form keeps two wait
// states between the store and any later write of its data registers.
// kStream = false: the default cache policy, for stores into lines that are
// only partly written (an unpadded packet's last line): as nt stores those cost
// an unpadded round trip several % (profiles/r02_ab_cache_policy.txt).
template <bool kStream = true>
__device__ __forceinline__ void store16(u32x4 data, uint64_t base, uint32_t bytes, uint32_t voff,
                                        uint32_t soff) {
  const u32x4 rs = {(uint32_t)base, (uint32_t)(base >> 32) & 0xffffu, bytes, 0x00020000u};
  if constexpr (kStream)
    asm volatile("buffer_store_dwordx4 %0, %1, %2, %3 offen" WG_STORE_NT_ASM "\n\ts_nop 1"
                 :: "v"(data), "v"(voff), "s"(rs), "s"(soff) : "memory");
  else
    asm volatile("buffer_store_dwordx4 %0, %1, %2, %3 offen" WG_PARTIAL_STORE_ASM "\n\ts_nop 1"
                 :: "v"(data), "v"(voff), "s"(rs), "s"(soff) : "memory");
}

// Per-piece LDS destinations (m0) and soffsets of a uniform round, derived
// from two values made opaque to the optimiser each round: otherwise it hoists
// the 8 destinations and 8 soffsets out of the round loop, runs out of SGPRs
// and restores them from VGPR lanes -- 16 v_readlane (VALU, energy at the power
// limit) per round.  Recomputed, they cost one SALU add each.
#ifndef WG_STAGE_CHAIN
#define WG_STAGE_CHAIN 1
#endif
struct StageChain {
  uint32_t lds0, step, soff0;
  __device__ StageChain(uint4 *run, uint32_t stride, uint32_t r)
      : lds0(lds_offset(run)), step(8u * stride), soff0(kRun * r) {
    asm volatile("" : "+s"(lds0), "+s"(step));
  }
  __device__ __attribute__((address_space(3))) void *lds(uint32_t j) const {
    return (__attribute__((address_space(3))) void *)(uintptr_t)(lds0 + 1024u * j);
  }
  __device__ uint32_t soff(uint32_t j) const { return soff0 + j * step; }
};

template <bool kSeal, bool kText>
__device__ __forceinline__ void stage_in(uint4 *run, const UniformGeomT<kText> &g, uint32_t lane,
                                         uint32_t r) {
  using R = Ranges<kSeal, kText>;
  constexpr int kCpol = kText ? WG_TEXT_LOAD_CPOL : WG_LOAD_CPOL;
  const uint32_t stride = (uint32_t)g.in_stride;
  const uint32_t hi = R::in_hi(g.W);
  // num_records = the end of the wave's last packet's input, rounded up to its
  // 16-byte chunk: the range check drops a WHOLE 16-byte access that crosses
  // num_records (the tail chunk reads up to 15 bytes past the packet -- inside
  // the same 16-byte-aligned, so mapped, granule).  launch_strided bounds
  // 63 * stride + hi below kNoAccess.
  // With full_in (input grid lines 128-byte aligned) the edge rounds load
  // whole lines as well: a line holding any byte of the packet is mapped, and
  // the bytes around the packet never reach an output (header chunk replaced,
  // tail chunk masked, chunks past the end not processed and zeroed or not
  // stored).  The resource then ends at the last packet's line end.
  const bool full = WG_FULL_LINES && g.full_in;
  const uint32_t rec_hi = full ? ((hi + 127u) & ~127u) : ((hi + 15u) & ~15u);
  const __amdgpu_buffer_rsrc_t rs = wave_rsrc(g.in0, 63u * stride + rec_hi);
  const uint32_t y = lane >> 3, k0 = (lane & 7u) ^ swz(y), k1 = k0 ^ 4u;
  // (open: packets dropped at the header check are loaded like the others --
  // harmless, their lanes skip the crypto and stage_out never writes them back)
  // (a round past the input -- open / seal grids end apart -- loads nothing;
  // r > 0 keeps round 0 straight-line: exactly 8 loads on every path, which
  // open's header wait counts on)
  if (full && r > 0u && kRun * r >= hi) return;
  if (WG_ABLATE_ALL_INTERIOR || full || (kRun * r >= R::in_lo() && kRun * r + kRun <= hi)) {
    // interior round (wave-uniform test): every lane moves a full chunk, the
    // per-lane offsets are round-independent -- no range checks
    const uint32_t v0 = y * stride + 16u * k0, v1 = y * stride + 16u * k1;
#if WG_STAGE_CHAIN
    StageChain c(run, stride, r);
    if constexpr (kText && WG_TEXT_SPLIT) {
#pragma unroll
      for (uint32_t j = 0; j < kChunks; ++j) {
        if (((j & 1u) ? k1 : k0) != 7u)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, c.lds(j), 16, (j & 1u) ? v1 : v0, c.soff(j), 0,
                                                   WG_TEXT_BODY_CPOL);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, c.lds(j), 16, (j & 1u) ? v1 : v0, c.soff(j), 0,
                                                   WG_TEXT_HEAD_CPOL);
      }
      return;
    }
#pragma unroll
    for (uint32_t j = 0; j < kChunks; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, c.lds(j), 16, (j & 1u) ? v1 : v0, c.soff(j), 0,
                                               kCpol);
#else
#pragma unroll
    for (uint32_t j = 0; j < kChunks; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, &run[64u * j], 16, (j & 1u) ? v1 : v0,
                                               8u * j * stride + kRun * r, 0, kCpol);
#endif
    return;
  }
#if WG_STAGE_CHAIN
  StageChain c(run, stride, r);
#endif
#pragma unroll
  for (uint32_t j = 0; j < kChunks; ++j) {
    const uint32_t k = (j & 1u) ? k1 : k0;
    const uint32_t w = kRun * r + 16u * k;
    const bool ok = w >= R::in_lo() && w < hi;
#if WG_STAGE_CHAIN
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, c.lds(j), 16, ok ? y * stride + 16u * k : kNoAccess,
                                             c.soff(j), 0, kCpol);
#else
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, &run[64u * j], 16,
                                             ok ? y * stride + 16u * k : kNoAccess,
                                             8u * j * stride + kRun * r, 0, kCpol);
#endif
  }
}

// kSkip0 (a split part's first round, wire grid): chunk 0 of every packet is the
// previous part's (its last piece, finished there) and is not stored
template <bool kSeal, bool kText, bool kSkip0 = false>
__device__ __forceinline__ void stage_out(uint4 *run, const UniformGeomT<kText> &g, uint32_t lane,
                                          uint32_t r) {
  using R = Ranges<kSeal, kText>;
  const uint32_t stride = (uint32_t)g.out_stride;
  const uint32_t hi = R::out_hi(g.W);
  // (see stage_in; with slot padding the last packet's line end)
  const uint32_t records = 63u * stride + (g.pad ? ((hi + 127u) & ~127u) : ((hi + 15u) & ~15u));
  const __amdgpu_buffer_rsrc_t rs = wave_rsrc(g.out0, records);
  const uint32_t y = lane >> 3, k0 = (lane & 7u) ^ swz(y), k1 = k0 ^ 4u;
  // open's drop mask, opaque to the optimiser: otherwise it hoists 8 per-lane
  // 64-bit masks 1 << (8j + y) out of the round loop, and their spill reloads
  // drain the DMA in flight
  uint64_t dead = kSeal ? 0ull : g.dead;
  if constexpr (!kSeal) asm volatile("" : "+s"(dead));
  // slot padding with no packet dropped: every output line is written whole,
  // edge rounds included -- run_wave zeroed the stage chunks outside the
  // output (zero_outside) -- and rounds past the output's line end store nothing
  const bool full = WG_FULL_LINES && g.pad && dead == 0;
  if (full && kRun * r >= hi) return;
  if (!kSkip0 && (WG_ABLATE_ALL_INTERIOR || full || (kRun * r >= R::out_lo() && kRun * r + kRun <= hi && dead == 0))) {
    // interior round: 8 full-chunk stores at round-independent per-lane offsets
    // (all 8 LDS reads first: the asm stores are memory barriers to the
    // compiler, which otherwise serialises read -> wait -> store per piece)
    const uint32_t v0 = y * stride + 16u * k0, v1 = y * stride + 16u * k1;
    uint4 v[kChunks];
#pragma unroll
    for (uint32_t j = 0; j < kChunks; ++j) v[j] = run[64u * j + lane];
#pragma unroll
    for (uint32_t j = 0; j < kChunks; ++j) {
      const u32x4 vv = {v[j].x, v[j].y, v[j].z, v[j].w};
      store16(vv, g.out0, records, (j & 1u) ? v1 : v0, 8u * j * stride + kRun * r);
    }
    return;
  }
  uint4 v[kChunks];
#pragma unroll
  for (uint32_t j = 0; j < kChunks; ++j) v[j] = run[64u * j + lane];
#pragma unroll
  for (uint32_t j = 0; j < kChunks; ++j) {
    const uint32_t k = (j & 1u) ? k1 : k0;
    const uint32_t w = kRun * r + 16u * k;
    const bool gone = (!kSeal && ((((uint32_t)(dead >> (8u * j))) >> y) & 1u)) || (kSkip0 && k == 0u);
    const bool ok = !gone && w >= R::out_lo() && w < hi;
    if (g.pad) {  // (wave-uniform) the partial chunk and the rest of its line, zero-filled
      const int valid = ok ? (int)min(hi - w, 16u) : 0;
      // (open on the wire grid: also the 16 slot bytes before the plaintext, so
      // the first line is written whole too)
      const bool mine = ok || (!gone && ((w >= hi && w < ((hi + 127u) & ~127u)) || w < R::out_lo()));
      const u32x4 vv = {v[j].x & byte_mask(valid, 0), v[j].y & byte_mask(valid, 1),
                        v[j].z & byte_mask(valid, 2), v[j].w & byte_mask(valid, 3)};
      store16(vv, g.out0, records, mine ? y * stride + 16u * k : kNoAccess, 8u * j * stride + kRun * r);
    } else {
      const u32x4 vv = {v[j].x, v[j].y, v[j].z, v[j].w};
      store16<WG_EDGE_STORE_NT != 0>(vv, g.out0, records, ok && hi - w >= 16u ? y * stride + 16u * k : kNoAccess,
              8u * j * stride + kRun * r);
    }
  }
  // The packets' last, partial chunk: q = hi % 16 bytes at wire offset wp, the
  // same for every packet of the wave (uniform length).  Its owner lane stores
  // it straight from its per-packet LDS row: at most 3 dword + 1 short + 1 byte
  // stores for the whole wave (wave-uniform branches, so the compiler's vmcnt
  // bookkeeping stays exact), instead of the cooperative shape's 5 per piece.
  const uint32_t q = hi & 15u, wp = hi & ~15u;
  if (!g.pad && q && (wp >> 7) == r && wp >= R::out_lo()) {
    const bool gone = !kSeal && ((dead >> lane) & 1ull);
    const uint4 c = run[8u * lane + (((wp >> 4) & 7u) ^ swz(lane))];
    const uint32_t base = gone ? kNoAccess : lane * stride + wp;
    if (q >= 4u) __builtin_amdgcn_raw_buffer_store_b32(c.x, rs, base, 0, WG_PARTIAL_STORE_CPOL);
    if (q >= 8u) __builtin_amdgcn_raw_buffer_store_b32(c.y, rs, base + 4u, 0, WG_PARTIAL_STORE_CPOL);
    if (q >= 12u) __builtin_amdgcn_raw_buffer_store_b32(c.z, rs, base + 8u, 0, WG_PARTIAL_STORE_CPOL);
    const uint32_t nd = q >> 2, rem = q & 3u;
    const uint32_t last = nd == 0 ? c.x : nd == 1 ? c.y : nd == 2 ? c.z : c.w;
    if (rem >= 2u)
      __builtin_amdgcn_raw_buffer_store_b16((unsigned short)last, rs, base + 4u * nd, 0, WG_PARTIAL_STORE_CPOL);
    if (rem & 1u)
      __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(last >> (8u * (rem & 2u))), rs,
                                           base + 4u * nd + (rem & 2u), 0, WG_PARTIAL_STORE_CPOL);
  }
}

// Descriptor-batch forms (DescGeom, fast waves): one wave-uniform buffer
// resource per side (base = the anchor, num_records = kNoAccess) and the 32-bit
// per-packet offsets from LDS.  Rounds where every staged packet moves a full
// 128-byte run: one v_add per piece, no range checks (packets not staged carry
// offset kNoAccess).  Edge rounds (the first / last ones, ragged lengths): each
// piece masked by its packet's range (kNoAccess = no access), full chunks only
// on the store side, then each packet's partial last chunk stored by its owner
// lane (dword / short / byte, masked the same way) -- no per-lane 64-bit
// addresses and no divergent branches.  The 8 offsets are read before the 8
// DMAs: an LDS read after a builtin LDS-DMA makes the compiler drain it.
// (measured: config 3 -1.2 %, config 4 +-0.2 % against the generic edge rounds,
// profiles/r03_ab_desc_addressing.txt -- off by default)
// aead_desc_affine_kernel (WG_DESC_AFFINE, wg_aead_kernels.h): the shared first
// diagonal round with the affine groups' per-lane keys
#ifndef WG_AFFINE_SHARED_DIAG
#define WG_AFFINE_SHARED_DIAG 0
#endif
#ifndef WG_DESC_MASKED_EDGES
#define WG_DESC_MASKED_EDGES 0
#endif
template <bool kSeal>
__device__ __forceinline__ void stage_in(uint4 *run, const DescGeom &g, uint32_t lane, uint32_t r) {
  const bool interior = r >= g.r_in0 && r < g.r_in1;
  if (!g.fast || (!WG_DESC_MASKED_EDGES && !interior)) {
    stage_in<kSeal, DescGeom>(run, g, lane, r);
    return;
  }
  const uint32_t y = lane >> 3, k0 = 16u * ((lane & 7u) ^ swz(y)), k1 = k0 ^ 64u;
  const __amdgpu_buffer_rsrc_t rs = wave_rsrc(g.in_wave, kNoAccessOffset);
  uint32_t off[kChunks];
  if (interior) {
#pragma unroll
    for (uint32_t j = 0; j < kChunks; ++j) off[j] = g.S.in16[8u * j + y] + ((j & 1u) ? k1 : k0);
  } else {
#pragma unroll
    for (uint32_t j = 0; j < kChunks; ++j) {
      const uint32_t p = 8u * j + y, kb = (j & 1u) ? k1 : k0, w = kRun * r + kb;
      const bool ok = w >= Ranges<kSeal>::in_lo() && w < Ranges<kSeal>::in_hi(g.S.wlen[p]);
      off[j] = ok ? g.S.in16[p] + kb : kNoAccessOffset;
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < kChunks; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, &run[64u * j], 16, off[j], kRun * r, 0, WG_LOAD_CPOL);
}

template <bool kSeal>
__device__ __forceinline__ void stage_out(uint4 *run, const DescGeom &g, uint32_t lane, uint32_t r) {
  const bool interior = r >= g.r_out0 && r < g.r_out1;
  if (!g.fast || (!WG_DESC_MASKED_EDGES && !interior)) {
    stage_out<kSeal, DescGeom>(run, g, lane, r);
    return;
  }
  const uint32_t y = lane >> 3, k0 = 16u * ((lane & 7u) ^ swz(y)), k1 = k0 ^ 64u;
  uint32_t off[kChunks];
  uint4 v[kChunks];
  if (interior) {
#pragma unroll
    for (uint32_t j = 0; j < kChunks; ++j) {
      off[j] = g.S.out16[8u * j + y] + ((j & 1u) ? k1 : k0);
      v[j] = run[64u * j + lane];
    }
#pragma unroll
    for (uint32_t j = 0; j < kChunks; ++j) {
      const u32x4 vv = {v[j].x, v[j].y, v[j].z, v[j].w};
      store16(vv, g.out_wave, kNoAccessOffset, off[j], kRun * r);
    }
    return;
  }
  // edge round: whole 16-byte chunks of the output (lines partly written: the
  // default cache policy, as the uniform kernels' unpadded edges)
#pragma unroll
  for (uint32_t j = 0; j < kChunks; ++j) {
    const uint32_t p = 8u * j + y, kb = (j & 1u) ? k1 : k0, w = kRun * r + kb;
    const bool ok = w >= Ranges<kSeal>::out_lo() && w + 16u <= Ranges<kSeal>::out_hi(g.S.wlen[p]);
    off[j] = ok ? g.S.out16[p] + kb : kNoAccessOffset;
    v[j] = run[64u * j + lane];
  }
#pragma unroll
  for (uint32_t j = 0; j < kChunks; ++j) {
    const u32x4 vv = {v[j].x, v[j].y, v[j].z, v[j].w};
    store16<WG_EDGE_STORE_NT != 0>(vv, g.out_wave, kNoAccessOffset, off[j], kRun * r);
  }
  // the packet's partial last chunk (q = hi % 16 bytes at wire offset wp), by its
  // owner lane straight from its LDS row, when it falls in this round
  const uint32_t W = g.S.wlen[lane];
  const uint32_t hi = Ranges<kSeal>::out_hi(W), q = hi & 15u, wp = hi & ~15u;
  const bool mine = W != 0u && q != 0u && (wp >> 7) == r && wp >= Ranges<kSeal>::out_lo();
  if (__ballot(mine) != 0ull) {  // (wave-uniform)
    const __amdgpu_buffer_rsrc_t rs = wave_rsrc(g.out_wave, kNoAccessOffset);
    const uint4 c = run[8u * lane + (((wp >> 4) & 7u) ^ swz(lane))];
    const uint32_t base = mine ? g.S.out16[lane] + wp : kNoAccessOffset;
    const uint32_t nd = q >> 2, rem = q & 3u;
    const uint32_t last = nd == 0 ? c.x : nd == 1 ? c.y : nd == 2 ? c.z : c.w;
    __builtin_amdgcn_raw_buffer_store_b32(c.x, rs, q >= 4u ? base : kNoAccessOffset, 0, WG_PARTIAL_STORE_CPOL);
    __builtin_amdgcn_raw_buffer_store_b32(c.y, rs, q >= 8u ? base + 4u : kNoAccessOffset, 0, WG_PARTIAL_STORE_CPOL);
    __builtin_amdgcn_raw_buffer_store_b32(c.z, rs, q >= 12u ? base + 8u : kNoAccessOffset, 0, WG_PARTIAL_STORE_CPOL);
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)last, rs, rem >= 2u ? base + 4u * nd : kNoAccessOffset,
                                          0, WG_PARTIAL_STORE_CPOL);
    __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(last >> (8u * (rem & 2u))), rs,
                                         (rem & 1u) ? base + 4u * nd + (rem & 2u) : kNoAccessOffset, 0,
                                         WG_PARTIAL_STORE_CPOL);
  }
}

// One lane's chunk of ciphertext work.  m = plaintext/ciphertext byte index of
// the chunk (wire w - 16); `ks` = its 4 keystream words.  Returns via LDS.
// kFull: the caller knows the chunk is a whole one (no tail mask)
template <bool kSeal, bool kFull = false>
__device__ __forceinline__ void crypt_chunk(uint4 &slot, Poly &p, int m, uint32_t P,
                                            uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
#if WG_ABLATE_NO_LDS_CRYPT
  uint32_t i0 = (uint32_t)m, i1 = P, i2 = a + (uint32_t)m, i3 = b ^ P;
#else
  const uint4 v = slot;
  uint32_t i0 = v.x, i1 = v.y, i2 = v.z, i3 = v.w;
#endif
  uint32_t o0 = i0 ^ a, o1 = i1 ^ b, o2 = i2 ^ c, o3 = i3 ^ d;
  const int valid = (int)P - m;
  if (!kFull && valid < 16) {  // the packet's last, partial chunk: AEAD pad16 zero-fills it
    const uint32_t m0 = byte_mask(valid, 0), m1 = byte_mask(valid, 1), m2 = byte_mask(valid, 2),
                   m3 = byte_mask(valid, 3);
    i0 &= m0; i1 &= m1; i2 &= m2; i3 &= m3;
    o0 &= m0; o1 &= m1; o2 &= m2; o3 &= m3;
  }
#if WG_ABLATE_NO_POLY
  p.h0 ^= o0 ^ i1; p.h1 ^= o1 ^ i2; p.h2 ^= o2 ^ i3; p.h3 ^= o3 ^ i0;
#else
  if (kSeal) poly_block(p, o0, o1, o2, o3);  // MAC the ciphertext
  else poly_block(p, i0, i1, i2, i3);
#endif
#if WG_ABLATE_NO_LDS_CRYPT
  p.h4 ^= o0 ^ o1 ^ o2 ^ o3;
#else
  slot = make_uint4(o0, o1, o2, o3);
#endif
}

// Process round r of this lane's packet: chunk k sits at wire w = 128r + 16k,
// i.e. text byte m = 128r - 16 + 16k.  Keystream: chunk 0 is the last chunk of
// block 2r (saved from the previous round), chunks 1-4 are block 2r+1, chunks
// 5-7 the first three of block 2r+2 (its fourth is saved for round r+1).
template <bool kSeal>
__device__ __forceinline__ void crypt_round(uint4 *run, uint32_t lane, uint32_t r, uint32_t P,
                                            const uint32_t key[8], uint32_t n1, uint32_t n2,
                                            Poly &p, uint32_t ks_save[4]) {
  const int m0 = (int)(kRun * r) - 16;
  const uint32_t row = 8u * lane, sw = swz(lane);
  if (r > 0 && m0 < (int)P)
    crypt_chunk<kSeal>(run[row + (0u ^ sw)], p, m0, P, ks_save[0], ks_save[1], ks_save[2],
                       ks_save[3]);
  if ((int)(kRun * r) < (int)P) {
    uint32_t ks[16];
    chacha20_block(ks, key, 2u * r + 1u, n1, n2);
#pragma unroll
    for (int k = 1; k <= 4; ++k) {
      const int m = m0 + 16 * k;
      if (m < (int)P)
        crypt_chunk<kSeal>(run[row + ((uint32_t)k ^ sw)], p, m, P, ks[4 * k - 4],
                           ks[4 * k - 3], ks[4 * k - 2], ks[4 * k - 1]);
    }
  }
  if ((int)(kRun * r) + 64 < (int)P) {
    uint32_t ks[16];
    chacha20_block(ks, key, 2u * r + 2u, n1, n2);
#pragma unroll
    for (int k = 5; k <= 7; ++k) {
      const int m = m0 + 16 * k;
      if (m < (int)P)
        crypt_chunk<kSeal>(run[row + ((uint32_t)k ^ sw)], p, m, P, ks[4 * k - 20],
                           ks[4 * k - 19], ks[4 * k - 18], ks[4 * k - 17]);
    }
    ks_save[0] = ks[12]; ks_save[1] = ks[13]; ks_save[2] = ks[14]; ks_save[3] = ks[15];
  }
}

// The same round with both keystream blocks computed beforehand
// (chacha20_block2_sync(ka, kb, key, 2r + 1, ...)): chunk 0 (keystream saved
// from the previous round), then chunks 1-7.
// (text grid: chunk k of round r is text 128r + 16k -- blocks 2r + 1 and
// 2r + 2 cover the round exactly, nothing is carried between rounds)
// kFull (descriptor batches): every live packet of the wave has ciphertext
// through the end of the round (128 r + 112 <= the wave's shortest P), so no
// per-chunk length test and no tail mask (wave-uniform, decided per round)
template <bool kSeal, bool kText = false, bool kFull = false>
__device__ __forceinline__ void apply_chunk0(uint4 *run, uint32_t lane, uint32_t r, uint32_t P,
                                             Poly &p, const uint32_t ks_save[4]) {
  if constexpr (kText) return;
  const int m0 = (int)(kRun * r) - 16;
  if (r > 0 && (kFull || m0 < (int)P))
    crypt_chunk<kSeal, kFull>(run[8u * lane + (0u ^ swz(lane))], p, m0, P, ks_save[0], ks_save[1],
                              ks_save[2], ks_save[3]);
}

template <bool kSeal, bool kText = false, bool kFull = false>
__device__ __forceinline__ void apply_blocks(uint4 *run, uint32_t lane, uint32_t r, uint32_t P,
                                             const uint32_t (&ka)[16], const uint32_t (&kb)[16],
                                             Poly &p, uint32_t ks_save[4]) {
  const uint32_t row = 8u * lane, sw = swz(lane);
  if constexpr (kText) {
    const int m0 = (int)(kRun * r);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int m = m0 + 16 * k;
      if (m < (int)P)
        crypt_chunk<kSeal>(run[row + ((uint32_t)k ^ sw)], p, m, P, ka[4 * k], ka[4 * k + 1],
                           ka[4 * k + 2], ka[4 * k + 3]);
    }
#pragma unroll
    for (int k = 4; k < 8; ++k) {
      const int m = m0 + 16 * k;
      if (m < (int)P)
        crypt_chunk<kSeal>(run[row + ((uint32_t)k ^ sw)], p, m, P, kb[4 * k - 16], kb[4 * k - 15],
                           kb[4 * k - 14], kb[4 * k - 13]);
    }
    return;
  }
  const int m0 = (int)(kRun * r) - 16;
#pragma unroll
  for (int k = 1; k <= 4; ++k) {
    const int m = m0 + 16 * k;
    if (kFull || m < (int)P)
      crypt_chunk<kSeal, kFull>(run[row + ((uint32_t)k ^ sw)], p, m, P, ka[4 * k - 4], ka[4 * k - 3],
                                ka[4 * k - 2], ka[4 * k - 1]);
  }
#pragma unroll
  for (int k = 5; k <= 7; ++k) {
    const int m = m0 + 16 * k;
    if (kFull || m < (int)P)
      crypt_chunk<kSeal, kFull>(run[row + ((uint32_t)k ^ sw)], p, m, P, kb[4 * k - 20], kb[4 * k - 19],
                                kb[4 * k - 18], kb[4 * k - 17]);
  }
  ks_save[0] = kb[12]; ks_save[1] = kb[13]; ks_save[2] = kb[14]; ks_save[3] = kb[15];
}

// 32 bytes starting at the tail chunk: k ciphertext bytes then the 16-byte tag
__device__ __forceinline__ void tail_words(const uint32_t (&ct)[4], const uint32_t (&tag)[4], int q,
                                           uint32_t out[8]) {
  const uint32_t r[8] = {ct[0], ct[1], ct[2], ct[3], 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = r[j] | bytes_at(tag, 4 * j - q);
}

// A uniform batch's one session key, loaded once per kernel into SGPRs: a
// per-group key load would be a vector load whose wait drains the previous
// group's stores at every group start.
struct SessionKey {
  uint32_t k[8];
  uint32_t sidx;
};

struct PacketJob {
  uint64_t in_base, out_base;  // wire-coordinate origins (see WaveStage)
  uint64_t counter;            // seal: nonce counter; open: from the header
  uint32_t len;                // seal: payload P; open: datagram length
  uint32_t slot;
  int32_t status;
};

// One part of a split wave (StridedParams::split): rounds [r0, r1) of its 64 packets;
// the lane's accumulator goes to h[idx] / h4[idx]
struct SplitPart {
  uint32_t r0, r1, idx;
  uint4 *h;
  uint32_t *h4;
  uint4 *rs;  // part 0 only (else null): the packet's r and s for the finish kernel
};
#if WG_SPLIT && WG_POLY_RADIX26
#error "split waves hand over radix-2^32 accumulators: build WG_POLY_RADIX26 with -DWG_SPLIT=0"
#endif

// The owner lane's side of a packet: everything but the cooperative memory
// moves.  kUniform = every lane of the wave is live with the same length
// (strided batches); then P, W and the round count are wave-uniform.
// kUKey (descriptor batches, phase-locked): every live packet of the wave uses
// the key slot `pre` carries, loaded once into SGPRs -- the keystream then runs
// as for uniform batches (wave-uniform columns on the SALU, shared diagonal)
// kLaneKeys (uniform geometry, descriptor batches): a key per packet in VGPRs
// (pre unused) -- the keystream keeps the in-place first diagonal round.
// kInDesc: uniform geometry inside a descriptor kernel (the affine groups).
template <bool kSeal, bool kUniform, bool kSync, bool kUKey = false, bool kLaneKeys = false,
          bool kInDesc = false, bool kSplit = false, class Stage, class Geom>
__device__ __forceinline__ bool run_wave(Stage &S, Geom &g, uint32_t lane, PacketJob job,
                                         const uint8_t *keys, const uint32_t *key_index,
                                         int32_t *status_out, const SessionKey *pre = nullptr,
                                         uint64_t next_hdr = 0, bool hdr_ready = false,
                                         const SplitPart *sp = nullptr) {
  // run grid (Ranges): kG = grid coordinate of text byte 0
  constexpr bool kText = Geom::kTextGrid;
  constexpr uint32_t kG = kText ? 0u : 16u;
  // the descriptor kernel's forms: the lane made opaque where its derived
  // offsets would otherwise be hoisted across groups and spilled
  constexpr bool kOpaqueDesc = (!kUniform || kLaneKeys || kInDesc) && WG_OPAQUE_LANE_DESC;
  static_assert(!kText || (kSync && kUniform && !kSeal), "text grid: uniform phase-locked open only");
  // phase-locked: every wave of the workgroup runs the same number of rounds
  // (uniform batches by construction, descriptor batches via DescGeom::wg_max)
  // ---- per-packet setup (owner lane) ------------------------------------
  uint32_t W = 0, P = 0;
  if (kUniform || job.status == WG_STATUS_OK) {
    if (kSeal) {
      P = job.len;
      W = P + WG_DATA_OVERHEAD_SZ;
    } else if (job.len < WG_DATA_OVERHEAD_SZ) {
      job.status = WG_STATUS_INVALID_PACKET;  // parse_incoming_packet: DATA needs len >= 32
    } else {
      W = job.len;
      P = W - WG_DATA_OVERHEAD_SZ;
    }
  }
  // runs covering the grid span of the datagram (text grid: without its header)
  uint32_t my_runs = job.status == WG_STATUS_OK ? (W - (16u - kG) + kRun - 1) / kRun : 0u;
  uint32_t rounds;
  uint32_t p_min = 0u;  // descriptor batches, phase-locked: the wave's shortest live payload
  // a split part runs rounds [r_begin, r_end) (wave-uniform; parts differ by at most
  // the rem rounds of part 0, see strided_body)
  constexpr bool split = kUniform && kSync && kSplit;
  uint32_t r_begin = 0u;
  if constexpr (kUniform) {
    rounds = my_runs;  // uniform: job.len is a kernel argument
    if constexpr (split) {
      r_begin = sp->r0;
      rounds = min(sp->r1, my_runs);
    }
  } else if constexpr (kSync) {
    p_min = wave_min32(my_runs ? P : 0xffffffffu);
    uint32_t ls = lane;  // (opaque: no kernel-lifetime LDS addresses to hold and spill)
    if constexpr (WG_OPAQUE_LANE_DESC) asm volatile("" : "+v"(ls));
    g.template set<kSeal>(ls, job.in_base, job.out_base, W, my_runs != 0u);
    rounds = g.wg_max(wave_max(my_runs));
  } else {
    S.in_base[lane] = job.in_base;
    S.out_base[lane] = job.out_base;
    S.wlen[lane] = W;
    S.nruns[lane] = my_runs;
    rounds = wave_max(my_runs);
  }

  uint32_t key[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t sidx = 0;
  if ((kUniform || kUKey) && !kLaneKeys && pre) {
#pragma unroll
    for (int j = 0; j < 8; ++j) key[j] = pre->k[j];
    sidx = pre->sidx;
  } else if (kUniform || job.status == WG_STATUS_OK) {
    const uint4 a = ld16(keys + 32u * job.slot), b = ld16(keys + 32u * job.slot + 16u);
    key[0] = a.x; key[1] = a.y; key[2] = a.z; key[3] = a.w;
    key[4] = b.x; key[5] = b.y; key[6] = b.z; key[7] = b.w;
    sidx = key_index[job.slot];
  }

  Poly poly;
  uint32_t ks_save[4] = {0, 0, 0, 0};
  uint32_t n1 = (uint32_t)job.counter, n2 = (uint32_t)(job.counter >> 32);
  const uint32_t q = P & 15u;                    // bytes in the partial ciphertext chunk
  const uint32_t wt = kG + (P & ~15u);           // grid offset of the tail chunk
  uint32_t tailB[4] = {0, 0, 0, 0};              // seal: chunk after the tail chunk (tag rest)
  uint32_t tg[4] = {0, 0, 0, 0};                 // open: the received tag, bytes [W - 16, W)
  // header prefetch (WG_OPEN_HDR_PREFETCH; wave- and workgroup-uniform: P and the
  // round count are launch constants): the tag's chunks in the last round, and
  // that round's chunk 7 past the datagram's grid end (the tag is parked there)
  constexpr bool kPfBuild = !kSeal && kUniform && kSync && WG_HDR_DMA && WG_OPEN_HDR_PREFETCH &&
                            Stage::kTagPark && !kInDesc && !kLaneKeys && !WG_ABLATE_NO_MEM;
  bool pf = false;
  uint32_t tag_bad = 0u;  // pf: the tag check's result, from the last round
  if constexpr (kPfBuild) {
    const uint32_t last = rounds - 1u, gend = W - (16u - kG);
    pf = !split && rounds >= 2u && (wt >> 7) == last && (q == 0u || ((wt + 16u) >> 7) == last) &&
         gend <= kRun * last + 112u;
  }

  auto one_time_key = [&]() {
    uint32_t ks[16];
    constexpr bool kSyncOpenKey = kSync && kUniform && !kSeal && WG_SYNC_OPEN_KEY;
    // RFC 8439 2.6: block 0 -> r | s.  Phase-locked for seal on the sync
    // paths, where every wave calls this once per group right after issuing
    // round 0's DMA (wave-uniform call site).  Open computes it per lane as
    // soon as the lane's header has landed: locking it there made every wave
    // wait for the slowest header (-4 %).
    if constexpr ((kSync && kSeal && WG_SYNC_KEY_BLOCK) || kSyncOpenKey) {
      chacha20_block_sync(ks, key, 0u, n1, n2);
    } else {
      chacha20_block(ks, key, 0u, n1, n2);
    }
    poly_init(poly, ks);
    // s, read back for the tag.  An inline-asm LDS write: the compiler cannot
    // tell the park from the run buffer that round 0's LDS-DMA (in flight
    // here) fills, and put a vmcnt(0) before a plain store -- draining the DMA
    // before round 0's keystream at every group start.  (LDS accesses of one
    // wave execute in order, so later reads of the park see this write.)
    const u32x4 sv = {ks[4], ks[5], ks[6], ks[7]};
    asm volatile("ds_write_b128 %0, %1" :: "v"(lds_offset(&S.park[lane])), "v"(sv) : "memory");
  };
  if (kSeal && !kSync && my_runs) one_time_key();

  // open, round 0: the datagram header (noise/mod.rs:170-180) decides the
  // packet's fate and supplies the nonce counter
  auto open_header = [&](const uint4 h) {
    if (job.status == WG_STATUS_OK) {  // (lanes already failed keep their status)
      if (h.x != WG_MSG_DATA) job.status = WG_STATUS_INVALID_PACKET;
      else if (h.y != sidx) job.status = WG_STATUS_WRONG_INDEX;  // session.rs:275-277
    }
    if constexpr (kSync && kUniform && WG_SYNC_OPEN_KEY) {
      // every lane of every wave runs the phase-locked block (dropped lanes on
      // garbage; their results are never used)
      n1 = h.z;
      n2 = h.w;
      one_time_key();
      if (job.status != WG_STATUS_OK) my_runs = 0;
    } else if (job.status != WG_STATUS_OK) {
      my_runs = 0;  // nothing of this packet is stored
      if constexpr (kSync && !kUniform) g.kill(lane);
      else if constexpr (!kUniform) S.nruns[lane] = 0;
    } else {
      n1 = h.z;
      n2 = h.w;
      one_time_key();
    }
    // (the non-phase-locked loop calls this in a divergent branch: it takes the
    // ballot itself, outside it)
    if constexpr (kUniform && kSync) g.dead = __ballot(job.status != WG_STATUS_OK);
  };
  // open: collect the received tag before the slots are decrypted in place.
  // It is bytes [q, q + 16) of the 32 raw bytes [wt, wt + 32), which sit in
  // two chunks (possibly two rounds); each chunk contributes its bytes (the
  // other half read as zero) and the parts are OR-ed together.
  // With an LDS tag slot (uniform stage) the parts go there instead of
  // registers: 4 fewer VGPRs through every round measured +3 % on open.
  // (descriptor batches: the lane made opaque in the tail helpers too -- else its
  // row / swizzle are computed once per kernel, held, and spilled)
  auto tail_lane = [&]() {
    uint32_t l = lane;
    if constexpr (kOpaqueDesc) asm volatile("" : "+v"(l));
    return l;
  };
  auto open_keep_tail = [&](uint4 *run, uint32_t r) {
    const uint32_t tl = tail_lane(), row = 8u * tl, sw = swz(tl);
    const uint32_t ra = wt >> 7, rb = (wt + 16u) >> 7;
    uint32_t t[4] = {0u, 0u, 0u, 0u};
    if (ra == r) {
      const uint4 v = run[row + (((wt >> 4) & 7u) ^ sw)];
      const uint32_t w[8] = {v.x, v.y, v.z, v.w, 0u, 0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] |= bytes_at(w, (int)q + 4 * j);
    }
    if (q && rb == r) {
      const uint4 v = run[row + ((((wt + 16u) >> 4) & 7u) ^ sw)];
      const uint32_t w[8] = {0u, 0u, 0u, 0u, v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] |= bytes_at(w, (int)q + 4 * j);
    }
    if constexpr (Stage::kTagPark) {
      if (kPfBuild && pf) {  // (ra == rb == the last round: the whole tag at once)
        if (ra == r) run[row + (7u ^ sw)] = make_uint4(t[0], t[1], t[2], t[3]);
      } else if (ra == r) {
        S.tagp[lane] = make_uint4(t[0], t[1], t[2], t[3]);
      } else if (q && rb == r) {
        const uint4 o = S.tagp[lane];
        S.tagp[lane] = make_uint4(o.x | t[0], o.y | t[1], o.z | t[2], o.w | t[3]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) tg[j] |= t[j];
    }
  };
  // seal: place the tag (and the tag bytes that spill into the next round)
  auto seal_tail = [&](uint4 *run, uint32_t r) {
    const uint32_t tl = tail_lane(), row = 8u * tl, sw = swz(tl);
    if (r > 0 && ((wt + 16u) >> 7) == r && (wt >> 7) == r - 1u && q) {
      // tag remainder spilled into this round's first chunk
      run[row + (0u ^ sw)] = make_uint4(tailB[0], tailB[1], tailB[2], tailB[3]);
    }
    if ((wt >> 7) == r) {
      // all ciphertext is MACed: LE64(aad_len=0) | LE64(ct_len), then the tag
      // (a split part holds only its share of the MAC: zeros here, the finish kernel
      // writes the tag over them)
      uint32_t tag[4] = {0u, 0u, 0u, 0u};
      if (!split) {
        poly_block(poly, 0u, 0u, P, 0u);
        const uint4 sp4 = S.park[tl];
        const uint32_t s[4] = {sp4.x, sp4.y, sp4.z, sp4.w};
        poly_finish(poly, s, tag);
      }
      const uint32_t ka = (wt >> 4) & 7u;
      uint32_t ct[4] = {0, 0, 0, 0};
      if (q) {
        const uint4 v = run[row + (ka ^ sw)];
        ct[0] = v.x; ct[1] = v.y; ct[2] = v.z; ct[3] = v.w;
      }
      uint32_t w8[8];
      tail_words(ct, tag, (int)q, w8);
      run[row + (ka ^ sw)] = make_uint4(w8[0], w8[1], w8[2], w8[3]);
      tailB[0] = w8[4]; tailB[1] = w8[5]; tailB[2] = w8[6]; tailB[3] = w8[7];
      if (q && ka < 7u) run[row + ((ka + 1u) ^ sw)] = make_uint4(w8[4], w8[5], w8[6], w8[7]);
    }
  };

  // Slot padding (uniform batches): stage_out writes whole output lines, so the
  // stage chunks of the round that lie outside the output are zeroed here --
  // those wholly past its end (input bytes, or bytes loaded past the packet),
  // and on open's wire grid the 16 slot bytes before the plaintext (the
  // header).  The partial chunks are zero past the end already (crypt_chunk,
  // tail_words).  Wave-uniform: at most the last output round and round 0.
  auto zero_outside = [&](uint4 *run, uint32_t ln, uint32_t r) {
    if constexpr (kUniform) {
      using R = Ranges<kSeal, kText>;
      const uint32_t zlo = (R::out_hi(g.W) + 15u) & ~15u;  // first chunk wholly past the output
      // (addresses from an opaque copy of the lane, computed inside the
      // wave-uniform branches: only the rounds that zero pay for them, and
      // nothing is hoisted and held in VGPRs)
      auto slots = [&](uint32_t &row, uint32_t &sw, uint4 &z) {
        uint32_t lz = ln, zero = 0u;
        asm volatile("" : "+v"(lz), "+v"(zero));
        row = 8u * lz;
        sw = swz(lz);
        z = make_uint4(zero, zero, zero, zero);
      };
      if ((zlo >> 7) == r) {
        const uint32_t kz = (zlo >> 4) & 7u;
        uint32_t row, sw;
        uint4 z;
        slots(row, sw, z);
#pragma unroll
        for (uint32_t k = 1; k < kChunks; ++k)
          if (k >= kz) run[row + (k ^ sw)] = z;
      }
      if (R::out_lo() > 0u && r == 0u) {
        uint32_t row, sw;
        uint4 z;
        slots(row, sw, z);
        run[row + (0u ^ sw)] = z;
      }
    }
  };

  if constexpr (kSync) {
    // Phase-locked path (workgroup-uniform control flow, one LDS stage per
    // wave): the round's DMA is issued first and its two keystream blocks are
    // computed while it is in flight -- the keystream does not depend on the
    // data.  Only open's round 0 has to wait first: the nonce is in the header.
    uint4 *run = S.run[0];
    // open: each lane fetches its own header ahead of round 0's DMA, so the
    // round-0 keystream waits for 16 bytes, not for the whole stage
    // (round 0's DMA is issued before the loop so the header is consumed, and
    // its registers freed, before the loop body; a split part: its first round's)
    if (rounds > r_begin) {
      uint4 hdr = make_uint4(0u, 0u, 0u, 0u);
      if constexpr (!kSeal && kUniform && WG_HDR_DMA && !WG_ABLATE_NO_MEM) {
        // Uniform open: the 64 headers go to the tag park by one LDS-DMA piece
        // issued before round 0's 8 pieces, and are read back after an
        // explicit vmcnt(8) -- header landed, round 0's DMA still in flight
        // under the key block and round 0's keystream.  (With a register load
        // the compiler placed the header's use, and its wait, between the
        // pieces, issuing most of round 0's DMA a memory latency late.)  The
        // tag park is free until round 0's tag bytes land (open_keep_tail).
        if (my_runs && !(kPfBuild && hdr_ready))
          dma_global<WG_HDR_NT != 0>(lds_offset(&S.tagp[0]), reinterpret_cast<const uint8_t *>(job.in_base - (16u - kG)));
        stage_in<kSeal>(run, g, lane, r_begin);  // exactly 8 pieces (the first round is straight-line)
        u32x4 h;
        if (kPfBuild && hdr_ready)  // (landed during the previous group: its rounds waited vmcnt(0))
          asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                       : "=v"(h) : "v"(lds_offset(&S.tagp[lane])) : "memory");
        else if constexpr (kText && WG_TEXT_SPLIT)  // (16 load instructions per round)
          asm volatile("s_waitcnt vmcnt(16)\n\tds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                       : "=v"(h) : "v"(lds_offset(&S.tagp[lane])) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(8)\n\tds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                       : "=v"(h) : "v"(lds_offset(&S.tagp[lane])) : "memory");
        hdr = make_uint4(h.x, h.y, h.z, h.w);
      } else {
        // (a global-address-space load: a flat one may alias LDS and makes the
        // compiler drain the LDS-DMA in flight before it)
        if (!kSeal && my_runs) {
          const u32x4 h = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(
              job.in_base - (16u - kG));  // (the datagram start)
          hdr = make_uint4(h.x, h.y, h.z, h.w);
        }
#if !WG_ABLATE_NO_MEM
        // (descriptor batches: the lane opaque here as in do_round -- else the
        // compiler computes round 0's lane-derived offsets once per kernel, holds
        // them through every group and spills them: ~40 scratch reloads per group)
        uint32_t ln0 = lane;
        if constexpr (kOpaqueDesc) asm volatile("" : "+v"(ln0));
        stage_in<kSeal>(run, g, ln0, r_begin);
#endif
      }
      if (kSeal && !WG_ABLATE_NO_KEYBLOCK) one_time_key();  // while round 0's DMA is in flight (every wave: phase-locked)
      if (!kSeal && my_runs) open_header(hdr);
    }
    // one round of the phase-locked loop
    auto do_round = [&](uint32_t r) {
      // (WG_OPAQUE_LANE / WG_OPAQUE_LANE_DESC: see the knob)
      uint32_t ln = lane;
      uint32_t Pr = P;
#if WG_OPAQUE_LANE
      if constexpr (kUniform) {
        asm volatile("" : "+v"(ln));
        Pr = __builtin_amdgcn_readfirstlane(P);
        asm volatile("" : "+s"(Pr));
      } else {
        asm volatile("" : "+v"(ln));
        asm volatile("" : "+v"(Pr));
      }
#elif WG_OPAQUE_LANE_DESC
      if constexpr (!kUniform) {
        asm volatile("" : "+v"(ln));
        asm volatile("" : "+v"(Pr));
      } else if constexpr (kLaneKeys || kInDesc) {
        asm volatile("" : "+v"(ln));
        Pr = __builtin_amdgcn_readfirstlane(P);
        asm volatile("" : "+s"(Pr));
      }
#endif
      WG_STAMP_AT(kSeal, r, 0);
#if !WG_ABLATE_NO_MEM
      if (r > r_begin) stage_in<kSeal>(run, g, ln, r);
#endif
      if constexpr (kPfBuild) {  // the next group's headers into the (free) tag park
        if (pf && r == 1u && next_hdr)
          dma_global<WG_HDR_NT != 0>(lds_offset(&S.tagp[0]), reinterpret_cast<const uint8_t *>(next_hdr));
      }
      WG_STAMP_AT(kSeal, r, 1);
      // descriptor batches: a round every live packet fills with ciphertext
      // (wave-uniform) runs without per-chunk length tests, tail masks or tag work
      const bool full = !kUniform && WG_DESC_FULL_ROUNDS && kRun * r + 112u <= p_min;
      // a later split part's first round (wire grid): its chunk 0 -- the tail of block
      // 2 r -- is the previous part's last piece, done there (no carry block here)
      const bool skip0 = split && !kText && r == r_begin && r_begin > 0u;
      auto landed = [&]() {
#if WG_MEM_PRIO && !WG_MEM_PRIO_AT
        __builtin_amdgcn_s_setprio(WG_MEM_PRIO);
#endif
        lds_wait_dma();
        WG_STAMP_AT(kSeal, r, 3);
        // (no tag byte lies in a full round: the tag starts past 128 r + 128)
        if (!kSeal && my_runs && !full) open_keep_tail(run, r);
        if (kSeal && r == 0)  // header: LE32 4 | LE32 sending_index | LE64 counter (session.rs:221-227)
          run[8u * ln + (0u ^ swz(ln))] = make_uint4(WG_MSG_DATA, sidx, n1, n2);
      };
      // workgroup-uniform: P for uniform batches; every round for descriptor
      // batches (lanes without ciphertext in the round ignore the keystream)
      if ((!kUniform || (int)(kRun * r) < (int)Pr) && !WG_ABLATE_NO_CRYPT) {
        // the keystream lives only inside this branch (kept out of phis, the
        // compiler would otherwise carry it as a register tuple and spill it)
        uint32_t ka[16], kb[16];
        chacha20_block2_sync<WG_SHARED_DIAG && ((kUniform && (!kLaneKeys || WG_AFFINE_SHARED_DIAG)) ||
                                                kUKey || WG_SHARED_DIAG_DESC)>(ka, kb, key, 2u * r + 1u, n1, n2);
        WG_STAMP_AT(kSeal, r, 2);
        landed();
        if (full) {
          if (my_runs) {
            apply_chunk0<kSeal, kText, true>(run, ln, r, Pr, poly, ks_save);
            apply_blocks<kSeal, kText, true>(run, ln, r, Pr, ka, kb, poly, ks_save);
          }
        } else if (my_runs) {
          if (!skip0) apply_chunk0<kSeal, kText>(run, ln, r, Pr, poly, ks_save);
          apply_blocks<kSeal, kText>(run, ln, r, Pr, ka, kb, poly, ks_save);
          if (kSeal) seal_tail(run, r);
        }
      } else {
        landed();
        if (my_runs && !WG_ABLATE_NO_CRYPT) {
          if (!skip0) apply_chunk0<kSeal, kText>(run, ln, r, Pr, poly, ks_save);
          if (kSeal) seal_tail(run, r);
        }
      }
      if constexpr (kPfBuild) {  // the tag check, from the parked chunk 7 (before zero_outside)
        if (pf && r == rounds - 1u && my_runs) {
          const uint32_t tl = tail_lane();
          const uint4 tv = run[8u * tl + (7u ^ swz(tl))];
          poly_block(poly, 0u, 0u, P, 0u);
          uint32_t tag[4];
          const uint4 sp = S.park[tl];
          const uint32_t sk4[4] = {sp.x, sp.y, sp.z, sp.w};
          poly_finish(poly, sk4, tag);
          tag_bad = (tv.x ^ tag[0]) | (tv.y ^ tag[1]) | (tv.z ^ tag[2]) | (tv.w ^ tag[3]);
        }
      }
      if constexpr (kUniform) {
        if (WG_FULL_LINES && g.pad) zero_outside(run, ln, r);
      }
      WG_STAMP_AT(kSeal, r, 4);
#if WG_MEM_PRIO && WG_MEM_PRIO_AT
      __builtin_amdgcn_s_setprio(WG_MEM_PRIO);
#endif
#if !WG_ABLATE_NO_MEM
      if constexpr (split && !kText) {
        if (skip0) stage_out<kSeal, kText, true>(run, g, ln, r);
        else stage_out<kSeal>(run, g, ln, r);
      } else {
        stage_out<kSeal>(run, g, ln, r);
      }
#endif
      WG_STAMP_AT(kSeal, r, 5);
    };
    for (uint32_t r = r_begin; r < rounds; ++r) do_round(r);
  } else {
    uint4 *run = S.run[0];
    for (uint32_t r = 0; r < rounds; ++r) {
#if !WG_ABLATE_NO_MEM
      stage_in<kSeal>(run, g, lane, r);
#endif
      lds_wait_dma();
      if (r < my_runs) {
        if (!kSeal) {
          if (r == 0) open_header(run[8u * lane + (0u ^ swz(lane))]);
          if (my_runs) open_keep_tail(run, r);
        } else if (r == 0) {
          // header: LE32 4 | LE32 sending_index | LE64 counter (session.rs:221-227)
          run[8u * lane + (0u ^ swz(lane))] = make_uint4(WG_MSG_DATA, sidx, n1, n2);
        }
        if (my_runs && !WG_ABLATE_NO_CRYPT) {
          crypt_round<kSeal>(run, lane, r, P, key, n1, n2, poly, ks_save);
          if (kSeal) seal_tail(run, r);
        }
      }
      if constexpr (kUniform && !kSeal) {
        if (r == 0) g.dead = __ballot(job.status != WG_STATUS_OK);
      }
      // (uniform geometry built with WG_SYNC=0: slot padding writes whole lines
      // here too, so the stage chunks outside the output are zeroed first)
      if constexpr (kUniform) {
        if (WG_FULL_LINES && g.pad) zero_outside(run, lane, r);
      }
#if !WG_ABLATE_NO_MEM
      stage_out<kSeal>(run, g, lane, r);
#endif
    }
  }

  if constexpr (split) {
    if constexpr (!kText) {
      // (wire grid, all parts but the last) chunk 0 of the next part's first round: the
      // tail of block 2 r_end, whose keystream this part holds (ks_save) -- a whole
      // 16-byte piece (the packets' ciphertext goes on past the next part's start)
      if (sp->r1 != 0xffffffffu && my_runs) {
        const uint32_t w = kRun * rounds;
        const u32x4 v = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(job.in_base + w);
        const uint32_t o0 = v.x ^ ks_save[0], o1 = v.y ^ ks_save[1], o2 = v.z ^ ks_save[2], o3 = v.w ^ ks_save[3];
        if (kSeal) poly_block(poly, o0, o1, o2, o3);
        else poly_block(poly, v.x, v.y, v.z, v.w);
        gstore16<false>(reinterpret_cast<uint8_t *>(job.out_base + w), make_uint4(o0, o1, o2, o3));
      }
    }
    // this part's share of the MAC (the finish kernel combines the parts; the open's
    // header statuses, tag check and zeroing are its too)
    sp->h[sp->idx] = make_uint4(poly.h0, poly.h1, poly.h2, poly.h3);
    sp->h4[sp->idx] = poly.h4;
    if (sp->rs) {  // (part 0: the Poly1305 key, so the finish kernel computes no block)
      sp->rs[2u * sp->idx] = make_uint4(poly.r0, poly.r1, poly.r2, poly.r3);
      sp->rs[2u * sp->idx + 1u] = S.park[lane];
    }
    return false;
  }
  if (!kSeal && job.status == WG_STATUS_OK) {
    uint32_t diff = 0;
    if (kPfBuild && pf) {
      diff = tag_bad;  // (checked in the last round)
    } else {
      poly_block(poly, 0u, 0u, P, 0u);
      uint32_t tag[4];
      const uint4 sp = S.park[lane];
      const uint32_t s[4] = {sp.x, sp.y, sp.z, sp.w};
      poly_finish(poly, s, tag);
      if constexpr (Stage::kTagPark) {
        const uint4 o = S.tagp[lane];
        tg[0] = o.x; tg[1] = o.y; tg[2] = o.z; tg[3] = o.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) diff |= tg[j] ^ tag[j];
    }
    if (diff) {
      // tag mismatch: never expose unauthenticated plaintext (ring open_within
      // zeroes it); the streamed stores of this wave land first (same wave, in order)
      job.status = WG_STATUS_INVALID_AEAD_TAG;
#if !WG_ABLATE_ZEROING
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // (global-address-space stores: a flat store may alias LDS and would
      // make the compiler drain in-flight LDS-DMA around it)
      uint8_t *pt = reinterpret_cast<uint8_t *>(job.out_base) + kG;
      const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
      for (uint32_t off = 0; off + 16u <= P; off += 16u) gstore16(pt + off, zero);
      if (q) {
        const uint32_t z[4] = {0, 0, 0, 0};
        gstore_partial(pt + (P & ~15u), z, (int)q);
      }
#endif
    }
  }
  if (status_out) *status_out = job.status;
  return kPfBuild && pf && next_hdr != 0u;  // the next group's headers are in the tag park
}

// The persistent kernels' walk over workgroup-sized packet groups: workgroup b
// takes groups b, b + grid, ... (round-robin), or, with xcd (WG_XCD_CONTIG),
// the workgroups of each XCD -- dispatched round-robin over the 8 XCDs, so b runs
// on XCD b % 8 -- walk one contiguous eighth of the batch.  Either way the last
// group is the last iteration of the workgroup that takes it.
struct GroupWalk {
  uint32_t first, end, step;
  __device__ GroupWalk(uint32_t groups, bool xcd) {
    if (xcd && gridDim.x % 8u == 0u) {
      const uint32_t x = blockIdx.x % 8u, span = (groups + 7u) / 8u;
      first = x * span + blockIdx.x / 8u;
      end = min(groups, x * span + span);
      step = gridDim.x / 8u;
    } else {
      first = blockIdx.x;
      end = groups;
      step = gridDim.x;
    }
  }
};

// ---------------------------------------------------------------------------
// kernels: 4 independent waves per workgroup, each with its own LDS stage
// ---------------------------------------------------------------------------
// Strided batches: kTail = false covers the whole waves [0, n & ~63) with the
// uniform geometry; kTail = true is a one-wave launch for the n % 64 packets
// left over (generic geometry), so the hot kernel carries no generic path.
// one wave's 64 packets [pkt0, pkt0 + 64) of a strided batch
template <bool kSeal, bool kTail, bool kText, class Stage, bool kSplit = false>
__device__ __forceinline__ bool strided_group(Stage &stage, const StridedParams &prm,
                                              uint32_t pkt0, uint32_t lane,
                                              const SessionKey *sk = nullptr,
                                              uint64_t next_hdr = 0, bool hdr_ready = false,
                                              const SplitPart *sp = nullptr) {
  const uint32_t i = pkt0 + lane;
  PacketJob job;
  job.slot = prm.key_slot;
  job.len = prm.len;
  job.counter = prm.counter_base + i;
  const uint64_t src0 = reinterpret_cast<uint64_t>(prm.src) + (uint64_t)pkt0 * prm.src_stride;
  const uint64_t dst0 = reinterpret_cast<uint64_t>(prm.dst) + (uint64_t)pkt0 * prm.dst_stride;
  // grid origins (Ranges): wire grid -- the plaintext side sits at grid
  // coordinate 16; text grid (open) -- the ciphertext starts at grid 0
  const uint64_t in0 = kSeal ? src0 - 16u : kText ? src0 + 16u : src0;
  const uint64_t out0 = kSeal || kText ? dst0 : dst0 - 16u;
  job.in_base = in0 + (uint64_t)lane * prm.src_stride;
  job.out_base = out0 + (uint64_t)lane * prm.dst_stride;
  int32_t *st = (prm.status && i < prm.n) ? prm.status + i : nullptr;
  if constexpr (!kTail) {
    job.status = WG_STATUS_OK;
    const uint32_t W = kSeal ? prm.len + WG_DATA_OVERHEAD_SZ : prm.len;
    UniformGeomT<kText> g{in0, out0, prm.src_stride, prm.dst_stride, 0ull, W,
                          (kSeal || prm.len >= WG_DATA_OVERHEAD_SZ)
                              ? (W - (kText ? 16u : 0u) + kRun - 1) / kRun : 0u,
                          prm.pad_tail, prm.full_in};
#if WG_ABLATE_PURE_COPY
    // timing-only probe: the kernel's own staging instructions and nothing else
    // (DMA in, wait, LDS read-out, stores), to compare with the memory-only
    // ablation on the same box, buffers and process
    {
      uint4 *run = stage.run[0];
      for (uint32_t r = 0; r < g.nr; ++r) {
        stage_in<kSeal>(run, g, lane, r);
        lds_wait_dma();
        stage_out<kSeal>(run, g, lane, r);
      }
      return false;
    }
#endif
    // (the text grid exists only in the phase-locked form)
    return run_wave<kSeal, true, WG_SYNC != 0 || kText, false, false, false, kSplit>(
        stage, g, lane, job, prm.keys, prm.key_index, st, sk, next_hdr, hdr_ready, sp);
  } else {
    job.status = i < prm.n ? WG_STATUS_OK : -1;  // -1: lane past the batch end
    LdsGeom g{stage};
    run_wave<kSeal, false, false>(stage, g, lane, job, prm.keys, prm.key_index, st);
    return false;
  }
}

template <bool kSeal, bool kTail, bool kText, bool kSplit = false>
__device__ __forceinline__ void strided_body(const StridedParams &prm, const SplitArgs *sa = nullptr) {
  using Stage = typename std::conditional<kTail, WaveStage, WaveStageUniform>::type;
  constexpr uint32_t kWaves = (kTail ? kBlockThreads : kStridedThreads) / 64u;
  __shared__ Stage stage[kWaves];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably uniform
  if constexpr (kTail) {
    if (wave == 0) strided_group<kSeal, true, false>(stage[wave], prm, prm.n & ~63u, lane);
  } else {
    // persistent walk over workgroup-sized packet groups: the resident
    // workgroups stay in their steady, mutually de-phased rhythm (one DMA
    // in flight while the other computes) instead of restarting in step
    const uint32_t groups = (prm.n / 64u + kWaves - 1u) / kWaves;
    SessionKey sk;
    {
      const uint8_t *kp = prm.keys + 32u * prm.key_slot;
      const uint4 a = ld16(kp), b = ld16(kp + 16u);
      const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) sk.k[j] = __builtin_amdgcn_readfirstlane(w[j]);
      sk.sidx = __builtin_amdgcn_readfirstlane(prm.key_index[prm.key_slot]);
    }
    bool hdr_ready = false;  // (WG_OPEN_HDR_PREFETCH) this group's headers already in the tag park
    (void)hdr_ready;
    uint32_t g_first = blockIdx.x, g_end = groups, g_step = gridDim.x;
#if WG_XCD_CONTIG
    {
      const GroupWalk walk(groups, true);
      g_first = walk.first;
      g_end = walk.end;
      g_step = walk.step;
    }
#endif
    // spread launch (WG_SPREAD): one pass over this workgroup's share [s_lo, s_hi) of the full waves
    const uint32_t s_lo = prm.spread ? spread_lo(prm.n / 64u, blockIdx.x, gridDim.x) : 0u;
    const uint32_t s_hi = prm.spread ? spread_lo(prm.n / 64u, blockIdx.x + 1u, gridDim.x) : 0u;
    if (prm.spread) {
      g_first = 0u;
      g_end = 1u;
      g_step = 1u;
    }
#define WALK_STEP g_step
#define WALK_END g_end
    // spread: which of the workgroup's waves carry its share -- waves w and w + 4 share a
    // SIMD, so a share of 5 or 6 waves doubles up on one or two SIMDs; rotating the live
    // set by 2 on every other workgroup lets the two workgroups of a CU double up on
    // different SIMDs (WG_SPREAD_ROT, wg_gpu.cpp: which workgroups are "every other")
    uint32_t vwave = wave;
    if (prm.spread >> 8) {
      const uint32_t mode = prm.spread >> 8;
      const uint32_t b = blockIdx.x;
      const uint32_t odd = mode == 1u ? (b & 1u) : mode == 2u ? ((b >> 8) & 1u) : ((b >> 3) & 1u);
      vwave = (wave + kWaves - 2u * odd) % kWaves;
    }
#if WG_SPLIT && WG_SYNC
    if constexpr (kSplit) {  // (a kernel of its own: the unsplit kernels keep their registers)
      // split waves: unit u = part * W64 + wave-of-packets (part-major: the waves of a
      // workgroup mostly run the same part), a part's rounds [part q + rem, part q + q +
      // rem) (part 0 from 0: it carries the rem < K rounds K does not divide), the last
      // part to the packets' end.  Parts of unequal length may share a workgroup: the
      // strided rounds meet only at the phase-locked s_barriers, which pace the waves and
      // guard no LDS (each wave stages its own), so a wave one round ahead stays locked
      // one step off, and a wave that ends leaves the barrier
      const uint32_t w64 = prm.n / 64u, units = w64 * sa->split;
      uint32_t u_first = blockIdx.x * kWaves + wave, u_end = units, u_step = gridDim.x * kWaves;
      if (prm.spread) {  // (one pass: this workgroup's even share of the units)
        u_first = spread_lo(units, blockIdx.x, gridDim.x) + vwave;
        u_end = spread_lo(units, blockIdx.x + 1u, gridDim.x);
        u_step = kWaves;
      }
      for (uint32_t u = u_first; u < u_end; u += u_step) {
        const uint32_t part = u / w64, pkt0 = (u - part * w64) * 64u;
        SplitPart spt;
        spt.r0 = part == 0u ? 0u : part * sa->split_q + sa->split_rem;
        spt.r1 = part + 1u == sa->split ? 0xffffffffu : (part + 1u) * sa->split_q + sa->split_rem;
        spt.idx = pkt0 + lane;
        spt.h = sa->part_h + (size_t)part * (w64 * 64u);
        spt.h4 = sa->part_h4 + (size_t)part * (w64 * 64u);
        spt.rs = part == 0u ? sa->rs : nullptr;
        strided_group<kSeal, false, kText, Stage, true>(stage[wave], prm, pkt0, lane, &sk, 0, false, &spt);
      }
      return;
    }
#endif
    for (uint32_t grp = g_first; grp < g_end; grp += g_step) {
      const uint32_t pkt0 = prm.spread ? (s_lo + vwave) * 64u : (grp * kWaves + wave) * 64u;
      // only the last group can be partial, and it is this workgroup's last
      // iteration: a wave without packets ends (ended waves leave the barrier)
      if (prm.spread ? s_lo + vwave >= s_hi : pkt0 + 64u > prm.n) return;
#if WG_OPEN_HDR_PREFETCH
      // open: this lane's datagram in the wave's next group (0: none), whose header
      // run_wave may prefetch into the tag park
      uint64_t next_hdr = 0;
      if constexpr (!kSeal) {
        const uint32_t npkt0 = ((grp + WALK_STEP) * kWaves + wave) * 64u;
        if (grp + WALK_STEP < WALK_END && npkt0 + 64u <= prm.n)
          next_hdr = reinterpret_cast<uint64_t>(prm.src) + (uint64_t)(npkt0 + lane) * prm.src_stride;
      }
      hdr_ready = strided_group<kSeal, false, kText>(stage[wave], prm, pkt0, lane, &sk, next_hdr, hdr_ready);
#else
      strided_group<kSeal, false, kText>(stage[wave], prm, pkt0, lane, &sk);
#endif
    }
#undef WALK_STEP
#undef WALK_END
  }
}

template <bool kSeal, bool kTail>
__global__ __launch_bounds__(kTail ? kBlockThreads : kStridedThreads,
                             kTail ? WG_WAVES_PER_SIMD : kStridedMinWaves) void
aead_strided_kernel(StridedParams prm) {
  strided_body<kSeal, kTail, false>(prm);
}

// The split waves' finish (StridedParams::split): one thread per packet of the full
// waves.  The parts' accumulators are Horner sums over their own ciphertext pieces,
// so the packet's is h = (..(h_0 r^k_1 + h_1) r^k_2 + ..) + h_last (k_j: part j's
// pieces), taken in radix 2^26 (powers of r are not clamped, wg_crypto.h f26_*); then
// the length block and + s as always (RFC 8439 2.8).  Seal writes the tag over the
// zeros the last part left; open checks the header (noise/mod.rs:170-180,
// session.rs:275-277) and the tag, zeroes a failed packet's plaintext (ring's
// open_within), and every packet gets its status here.
template <bool kSeal, bool kText>
__global__ __launch_bounds__(256) void aead_strided_finish_kernel(StridedSplitParams sp) {
  const StridedParams &prm = sp.prm;
  const SplitArgs &sa = sp.sa;
  const uint32_t n = prm.n & ~63u;
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint32_t P = kSeal ? prm.len : prm.len - WG_DATA_OVERHEAD_SZ;  // (open: len >= 32, the host checks)
  const uint8_t *src = prm.src + (uint64_t)i * prm.src_stride;
  uint8_t *dst = prm.dst + (uint64_t)i * prm.dst_stride;
  int32_t status = WG_STATUS_OK;
  if (!kSeal) {
    const uint32_t sidx = prm.key_index[prm.key_slot];
    const uint4 h = ld16(src);
    if (h.x != WG_MSG_DATA) status = WG_STATUS_INVALID_PACKET;
    else if (h.y != sidx) status = WG_STATUS_WRONG_INDEX;
  }
  if (status == WG_STATUS_OK) {
    // the Poly1305 key part 0 computed (r clamped, s)
    const uint4 rq = sa.rs[2u * i], sq = sa.rs[2u * i + 1u];
    const uint32_t rk[8] = {rq.x, rq.y, rq.z, rq.w, 0u, 0u, 0u, 0u};
    Poly ps;
    poly_init(ps, rk);
    const F26 r26 = f26_from32(ps.r0, ps.r1, ps.r2, ps.r3, 0u);
    // pieces (16-byte ciphertext chunks, the last one partial) of the part over rounds
    // [a, b): text [128 a, 128 b) on both grids (on the wire grid a part also finishes
    // chunk 0 of the next part's first round and skips its own first), those below P
    const uint32_t P16 = (P + 15u) & ~15u;
    auto pieces = [&](uint32_t a, uint32_t b) -> uint32_t {
      return (min(128u * b, P16) - min(128u * a, P16)) / 16u;
    };
    const size_t stride = (size_t)n;
    // parts 1 .. K-2 have the same piece count (8 Q): their power of r once
    const uint32_t pq = sa.split_q, prem = sa.split_rem;
    const uint32_t k_mid = pieces(pq + prem, 2u * pq + prem);
    const F26 r_mid = sa.split > 2u ? f26_pow(r26, k_mid) : r26;
    F26 acc;
    for (uint32_t j = 0; j < sa.split; ++j) {
      const uint4 hq = sa.part_h[j * stride + i];
      const F26 hj = f26_from32(hq.x, hq.y, hq.z, hq.w, sa.part_h4[j * stride + i]);
      if (j == 0) {
        acc = hj;
      } else if (j + 1u < sa.split) {
        acc = f26_add(f26_mul(acc, r_mid), hj);
      } else {
        const uint32_t k = pieces(j * pq + prem, 0x7fffffffu / 128u);
        acc = f26_add(k ? f26_mul(acc, f26_pow(r26, k)) : acc, hj);
      }
    }
    f26_to32(acc, ps.h0, ps.h1, ps.h2, ps.h3, ps.h4);
    poly_block(ps, 0u, 0u, P, 0u);  // le64(AAD len = 0) | le64(P)
    const uint32_t s4[4] = {sq.x, sq.y, sq.z, sq.w};
    uint32_t tag[4];
    poly_finish(ps, s4, tag);
    if (kSeal) {
      uint8_t *t = dst + WG_DATA_OFFSET + P;  // (session.rs:247-252)
      if ((P & 15u) == 0u) {
        st16(t, tag[0], tag[1], tag[2], tag[3]);
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) t[q] = (uint8_t)(tag[q / 4] >> (8 * (q % 4)));
      }
    } else {
      // received tag: bytes [16 + P, 32 + P) of the datagram, in two aligned pieces
      const uint8_t *in = src + WG_DATA_OFFSET;
      const uint32_t o = P & ~15u;
      const uint4 ta = ld16(in + o);
      const uint4 tb = (P & 15u) ? ld16(in + o + 16u) : make_uint4(0, 0, 0, 0);
      const uint32_t tw[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
      uint32_t bad = 0u;
#pragma unroll
      for (int j = 0; j < 4; ++j) bad |= bytes_at(tw, (int)(P & 15u) + 4 * j) ^ tag[j];
      if (bad) {
        status = WG_STATUS_INVALID_AEAD_TAG;
        for (uint32_t off = 0; off + 16u <= P; off += 16u) st16(dst + off, 0u, 0u, 0u, 0u);
        if (P & 15u) {
          const uint32_t z[4] = {0, 0, 0, 0};
          store_partial(dst + (P & ~15u), z, (int)(P & 15u));
        }
      }
    }
  }
  if (prm.status) prm.status[i] = status;
}

// the split waves' kernels (StridedParams::split > 1; kText: open on the text grid)
template <bool kSeal, bool kText>
__global__ __launch_bounds__(kStridedThreads, kStridedMinWaves) void aead_strided_split_kernel(StridedSplitParams sp) {
  strided_body<kSeal, false, kText, true>(sp.prm, &sp.sa);
}

// open on the text grid (Ranges): destinations whose plaintext slots start on
// 128-byte boundaries (launch_strided picks it); the full waves only -- the
// last, partial wave stays on aead_strided_kernel<false, true>
__global__ __launch_bounds__(kStridedThreads, kStridedMinWaves) void aead_strided_open_text_kernel(
    StridedParams prm) {
  strided_body<false, false, true>(prm);
}

template <bool kSeal>
__global__ __launch_bounds__(kBlockThreads, WG_WAVES_PER_SIMD) void aead_desc_kernel(
    DescParams prm) {
  __shared__ WaveStage stage[kWaves];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t pkt0 = (blockIdx.x * kWaves + wave) * 64u;
  if (pkt0 >= prm.n) return;
  const uint32_t i = pkt0 + lane;
  uint32_t idx = i;  // descriptor (and status) index this lane serves
  PacketJob job;
  job.status = -1;
  job.in_base = job.out_base = 0;
  job.counter = 0;
  job.len = 0;
  job.slot = 0;
  if (i < prm.n) {
    if (prm.order) idx = prm.order[i];
    const wg_packet_desc d = prm.descs[idx];
    job.len = d.len;
    job.slot = d.key_slot;
    job.counter = d.counter;
    const uint64_t src = reinterpret_cast<uint64_t>(prm.src) + d.src_off;
    const uint64_t dst = reinterpret_cast<uint64_t>(prm.dst) + d.dst_off;
    job.in_base = kSeal ? src - 16u : src;
    job.out_base = kSeal ? dst : dst - 16u;
    if (!kSeal && d.key_slot == WG_KEY_SLOT_INVALID_PACKET) job.status = WG_STATUS_INVALID_PACKET;
    else if (!kSeal && d.key_slot == WG_KEY_SLOT_NO_SESSION) job.status = WG_STATUS_NO_CURRENT_SESSION;
    else if (d.key_slot >= prm.key_slots) job.status = WG_STATUS_BAD_KEY_SLOT;
    else if (((d.src_off | d.dst_off) & 15u) != 0u) job.status = WG_STATUS_MISALIGNED;
    else job.status = WG_STATUS_OK;
  }
  LdsGeom g{stage[wave]};
  run_wave<kSeal, false, false>(stage[wave], g, lane, job, prm.keys, prm.key_index,
                         i < prm.n ? prm.status + idx : nullptr);
}

// Phase-locked descriptor batches (configs 3/4): persistent 512-thread
// workgroups like the strided kernel; each group of 512 descriptors runs the
// workgroup's longest packet's rounds (the length-sorted plan,
// wg_gpu_plan_batch, keeps a group's packets alike).
// kAffine (aead_desc_affine_kernel, unordered launches): workgroups whose packets
// are affine take the uniform geometry (below).  A separate kernel, so that the
// ordered launches of mixed batches (whose groups gather packets from all over
// the batch and are never affine) keep the plain form's register allocation.
// kOneKey (the *_key1 kernels, contexts with one key slot -- a single session,
// BASELINE config 3): the key is loaded once per kernel into SGPRs as in the
// strided kernels, and every group runs the SGPR-key forms (wave-uniform first
// column on the SALU, shared first diagonal round).  Packets naming any other
// slot fail with BAD_KEY_SLOT before the crypto, so no lane needs another key.
template <bool kSeal, bool kAffine, bool kOneKey>
__device__ __forceinline__ void desc_sync_body(const DescParams &prm) {
  constexpr uint32_t kWaves = kStridedThreads / 64u;
  // The descriptor stages and, with kAffine, the uniform stages of the affine
  // groups share the LDS; the workgroup's round / vote slots sit in the
  // descriptor layout's slack (the last wave's uniform tag park: 2 workgroups x
  // 80 KiB = the whole LDS).
  static_assert(kWaves * sizeof(WaveStageDesc) + 4u * kWaves <= kWaves * sizeof(WaveStageUniform),
                "vote slots in the slack");
  constexpr uint32_t kLdsBytes =
      kAffine ? kWaves * sizeof(WaveStageUniform) : (kWaves * sizeof(WaveStageDesc) + 4u * kWaves + 15u) & ~15u;
  __shared__ uint4 lds_raw[kLdsBytes / 16u];
  auto stage_d = [&](uint32_t w) { return reinterpret_cast<WaveStageDesc *>(lds_raw) + w; };
  auto stage_u = [&](uint32_t w) { return reinterpret_cast<WaveStageUniform *>(lds_raw) + w; };
  uint32_t *wg_rounds = reinterpret_cast<uint32_t *>(stage_d(kWaves));
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t groups = (prm.n + 64u * kWaves - 1u) / (64u * kWaves);
  SessionKey sk;
  if constexpr (kOneKey) {
    const uint4 a = ld16(prm.keys), b = ld16(prm.keys + 16u);
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) sk.k[j] = __builtin_amdgcn_readfirstlane(w[j]);
    sk.sidx = __builtin_amdgcn_readfirstlane(prm.key_index[0]);
  }
  uint32_t g_first = blockIdx.x, g_end = groups, g_step = gridDim.x;
  // (a plan's order is length-sorted: contiguous ranges would hand whole XCDs the
  // long packets, so only unordered launches may take the XCD walk)
#if WG_XCD_CONTIG
  {
    const GroupWalk walk(groups, kAffine);
    g_first = walk.first;
    g_end = walk.end;
    g_step = walk.step;
  }
#endif
  // spread launch (WG_SPREAD): one pass over this workgroup's share [s_lo, s_hi) of
  // the waves (the last one may be partial)
  const uint32_t waves_all = (prm.n + 63u) / 64u;
  const uint32_t s_lo = prm.spread ? spread_lo(waves_all, blockIdx.x, gridDim.x) : 0u;
  const uint32_t s_hi = prm.spread ? spread_lo(waves_all, blockIdx.x + 1u, gridDim.x) : 0u;
  if (prm.spread) {
    g_first = 0u;
    g_end = 1u;
    g_step = 1u;
  }
  for (uint32_t grp = g_first; grp < g_end; grp += g_step) {
    const uint32_t pkt0 = prm.spread ? (s_lo + wave) * 64u : (grp * kWaves + wave) * 64u;
    // only the last group can lack waves; it is this workgroup's last iteration
    if (prm.spread ? s_lo + wave >= s_hi : pkt0 >= prm.n) return;
    const uint32_t alive = prm.spread ? s_hi - s_lo : min(kWaves, (prm.n - grp * kWaves * 64u + 63u) / 64u);
    const uint32_t i = pkt0 + lane;
    uint32_t idx = i;
    PacketJob job;
    job.status = -1;
    job.in_base = reinterpret_cast<uint64_t>(prm.src);
    job.out_base = reinterpret_cast<uint64_t>(prm.dst);
    job.counter = 0;
    job.len = 0;
    job.slot = 0;
    if (i < prm.n) {
      if (prm.order) idx = prm.order[i];
      const wg_packet_desc d = prm.descs[idx];
      job.len = d.len;
      job.slot = d.key_slot;
      job.counter = d.counter;
      const uint64_t src = reinterpret_cast<uint64_t>(prm.src) + d.src_off;
      const uint64_t dst = reinterpret_cast<uint64_t>(prm.dst) + d.dst_off;
      job.in_base = kSeal ? src - 16u : src;
      job.out_base = kSeal ? dst : dst - 16u;
      if (!kSeal && d.key_slot == WG_KEY_SLOT_INVALID_PACKET) job.status = WG_STATUS_INVALID_PACKET;
      else if (!kSeal && d.key_slot == WG_KEY_SLOT_NO_SESSION) job.status = WG_STATUS_NO_CURRENT_SESSION;
      else if (d.key_slot >= prm.key_slots) job.status = WG_STATUS_BAD_KEY_SLOT;
      else if (((d.src_off | d.dst_off) & 15u) != 0u) job.status = WG_STATUS_MISALIGNED;
      else job.status = WG_STATUS_OK;
    }
    int32_t *st = i < prm.n ? prm.status + idx : nullptr;
    // Affine groups: when every wave of the workgroup holds 64 live packets of one
    // length in slots at a constant stride on each side (MTU-sized traffic in
    // fixed receive / send slots: config 4, a Tunn's bulk batches), the group runs
    // the strided kernels' uniform geometry -- SGPR addressing, wave-uniform
    // lengths and branches -- with the keys still per packet.  The vote is
    // workgroup-wide because the two forms run different barrier sequences.
    if constexpr (kAffine) {
      const uint32_t Wl = kSeal ? job.len + WG_DATA_OVERHEAD_SZ : job.len;
      const uint32_t W0 = __builtin_amdgcn_readfirstlane(Wl);
      const uint64_t i0 = rl64(job.in_base, 0), o0 = rl64(job.out_base, 0);
      const uint64_t si = rl64(job.in_base, 1) - i0, so = rl64(job.out_base, 1) - o0;
      const uint64_t span = (W0 + 15u) & ~15u;
      const bool shape = pkt0 + 64u <= prm.n && (kSeal || W0 >= WG_DATA_OVERHEAD_SZ) &&
                         si >= span && so >= span &&
                         63u * (si > so ? si : so) + W0 + 256u < (uint64_t)kNoAccessOffset;
      const bool mine = job.status == WG_STATUS_OK && Wl == W0 &&
                        job.in_base == i0 + (uint64_t)lane * si && job.out_base == o0 + (uint64_t)lane * so;
      const uint32_t vote = shape && __ballot(!mine) == 0ull ? W0 : 0u;
      __syncthreads();  // the previous group is done with the LDS (the slots overlap a tag park)
      if (lane == 0u) wg_rounds[wave] = vote;
      __syncthreads();
      bool uni = wg_rounds[0] != 0u;
      for (uint32_t w = 1; w < alive; ++w) uni = uni && wg_rounds[w] == wg_rounds[0];
      __syncthreads();  // read before a uniform stage or the next vote overwrites them
      if (uni) {
        const uint32_t nr = (W0 + kRun - 1u) / kRun;
        const uint32_t full_in = (i0 % 128u == 0u && si % 128u == 0u) ? 1u : 0u;
        UniformGeom ug{i0, o0, si, so, 0ull, W0, nr, 0u, full_in};
        // (equal on every lane: constants / SGPRs, so the uniform form's branches stay scalar)
        job.len = __builtin_amdgcn_readfirstlane(job.len);
        job.status = WG_STATUS_OK;
        if constexpr (kOneKey)
          run_wave<kSeal, true, true, false, false, true>(*stage_u(wave), ug, lane, job, prm.keys,
                                                          prm.key_index, st, &sk);
        else
          run_wave<kSeal, true, true, false, true, true>(*stage_u(wave), ug, lane, job, prm.keys,
                                                         prm.key_index, st);
        continue;
      }
    }
    DescGeom g{*stage_d(wave), reinterpret_cast<uint64_t>(prm.src) - 16u,
               reinterpret_cast<uint64_t>(prm.dst) - 16u, wg_rounds, wave, alive};
    if constexpr (kOneKey) {
      run_wave<kSeal, false, true, true>(*stage_d(wave), g, lane, job, prm.keys, prm.key_index, st, &sk);
      continue;
    }
#if WG_DESC_UNIFORM_KEY
    // a wave whose live packets all use one key slot (single-session batches:
    // config 3, a Tunn's batches) takes the SGPR-key form; the two forms run
    // the same barrier sequence, so the waves of a workgroup may mix them
    const uint64_t live = __ballot(job.status == WG_STATUS_OK);
    if (live) {
      const int l0 = (int)__builtin_amdgcn_readfirstlane((uint32_t)__builtin_ctzll(live));
      const uint32_t us = (uint32_t)__builtin_amdgcn_readlane((int)job.slot, l0);
      if (__ballot(job.status == WG_STATUS_OK && job.slot != us) == 0ull) {
        SessionKey sk;
        const uint4 a = ld16(prm.keys + 32u * us), b = ld16(prm.keys + 32u * us + 16u);
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) sk.k[j] = __builtin_amdgcn_readfirstlane(w[j]);
        sk.sidx = __builtin_amdgcn_readfirstlane(prm.key_index[us]);
        run_wave<kSeal, false, true, true>(*stage_d(wave), g, lane, job, prm.keys, prm.key_index, st, &sk);
        continue;
      }
    }
#endif
    run_wave<kSeal, false, true>(*stage_d(wave), g, lane, job, prm.keys, prm.key_index, st);
  }
}

template <bool kSeal>
__global__ __launch_bounds__(kStridedThreads, kStridedMinWaves) void aead_desc_sync_kernel(
    DescParams prm) {
  desc_sync_body<kSeal, false, false>(prm);
}

template <bool kSeal>
__global__ __launch_bounds__(kStridedThreads, kStridedMinWaves) void aead_desc_affine_kernel(
    DescParams prm) {
  desc_sync_body<kSeal, true, false>(prm);
}

template <bool kSeal>
__global__ __launch_bounds__(kStridedThreads, kStridedMinWaves) void aead_desc_sync_key1_kernel(
    DescParams prm) {
  desc_sync_body<kSeal, false, true>(prm);
}

template <bool kSeal>
__global__ __launch_bounds__(kStridedThreads, kStridedMinWaves) void aead_desc_affine_key1_kernel(
    DescParams prm) {
  desc_sync_body<kSeal, true, true>(prm);
}

template __global__ void aead_strided_split_kernel<true, false>(StridedSplitParams);
template __global__ void aead_strided_split_kernel<false, false>(StridedSplitParams);
template __global__ void aead_strided_split_kernel<false, true>(StridedSplitParams);
template __global__ void aead_strided_finish_kernel<true, false>(StridedSplitParams);
template __global__ void aead_strided_finish_kernel<false, false>(StridedSplitParams);
template __global__ void aead_strided_finish_kernel<false, true>(StridedSplitParams);
template __global__ void aead_strided_kernel<true, false>(StridedParams);
template __global__ void aead_strided_kernel<false, false>(StridedParams);
template __global__ void aead_strided_kernel<true, true>(StridedParams);
template __global__ void aead_strided_kernel<false, true>(StridedParams);
template __global__ void aead_desc_kernel<true>(DescParams);
template __global__ void aead_desc_kernel<false>(DescParams);
template __global__ void aead_desc_sync_kernel<true>(DescParams);
template __global__ void aead_desc_sync_kernel<false>(DescParams);
template __global__ void aead_desc_affine_kernel<true>(DescParams);
template __global__ void aead_desc_affine_kernel<false>(DescParams);
template __global__ void aead_desc_sync_key1_kernel<true>(DescParams);
template __global__ void aead_desc_sync_key1_kernel<false>(DescParams);
template __global__ void aead_desc_affine_key1_kernel<true>(DescParams);
template __global__ void aead_desc_affine_key1_kernel<false>(DescParams);

}  // namespace wg

#if WG_STAMP
extern "C" int wg_gpu_debug_stamps(void *out, size_t bytes) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(wg::g_stamps), bytes) == hipSuccess ? 0 : -1;
}
extern "C" int wg_gpu_debug_realtime(void *out, size_t bytes) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(wg::g_realtime), bytes) == hipSuccess ? 0 : -1;
}
// device-side snapshot of both stamp arrays into `dst` (device memory, stamps then
// realtime), queued on `stream` behind the launch it records: no host sync per step
extern "C" int wg_gpu_debug_snapshot(void *dst, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  const size_t a = sizeof(wg::g_stamps), b = sizeof(wg::g_realtime);
  if (hipMemcpyFromSymbolAsync(dst, HIP_SYMBOL(wg::g_stamps), a, 0, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return -1;
  return hipMemcpyFromSymbolAsync((char *)dst + a, HIP_SYMBOL(wg::g_realtime), b, 0,
                                  hipMemcpyDeviceToDevice, st) == hipSuccess ? 0 : -1;
}
#endif
