// wg_crypto.h -- device primitives for the gfx950 AEAD kernels: ChaCha20 block
// function (RFC 8439 2.3), Poly1305 in radix 2^32 (RFC 8439 2.5) and the
// byte-granular helpers used once per packet at its tail.
//
// Poly1305 radix choice: on MI355X v_mad_u64_u32 issues at the same rate as
// v_alignbit_b32 (tools/microbench_valu.hip, profiles/r01_microbench_valu.txt),
// so 4 x 32-bit limbs + a 3-bit top limb (20 mads per 16-byte block, no limb
// splitting) beat radix 2^26 (25 mads + splitting + 64-bit carries).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wg {


// ---------------------------------------------------------------------------
// ChaCha20 (RFC 8439 2.3)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, 32u - n);  // v_alignbit_b32: 1 VALU op
}

#ifndef WG_ROT_PERM
#define WG_ROT_PERM 0  // 1: byte rotations (16, 8) as v_perm_b32
#endif
#if WG_ROT_PERM
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x01000302u); }
__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x02010003u); }
#else
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return rotl(x, 16); }
__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return rotl(x, 8); }
#endif

#define WG_QR(a, b, c, d)                   \
  a += b; d ^= a; d = rotl16(d);            \
  c += d; b ^= c; b = rotl(b, 12);          \
  a += b; d ^= a; d = rotl8(d);             \
  c += d; b ^= c; b = rotl(b, 7);

constexpr uint32_t kSigma0 = 0x61707865u, kSigma1 = 0x3320646eu, kSigma2 = 0x79622d32u,
                   kSigma3 = 0x6b206574u;

// Keystream block `blk` for key k[8] and nonce (0, n1, n2) -- WireGuard's nonce
// is 4 zero bytes then LE64(counter) (session.rs:230-235), so word 13 is 0.
__device__ __forceinline__ void chacha20_block(uint32_t ks[16], const uint32_t k[8], uint32_t blk,
                                               uint32_t n1, uint32_t n2) {
  uint32_t x0 = kSigma0, x1 = kSigma1, x2 = kSigma2, x3 = kSigma3;
  uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3];
  uint32_t x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
  uint32_t x12 = blk, x13 = 0, x14 = n1, x15 = n2;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    WG_QR(x0, x4, x8, x12) WG_QR(x1, x5, x9, x13) WG_QR(x2, x6, x10, x14) WG_QR(x3, x7, x11, x15)
    WG_QR(x0, x5, x10, x15) WG_QR(x1, x6, x11, x12) WG_QR(x2, x7, x8, x13) WG_QR(x3, x4, x9, x14)
  }
  ks[0] = x0 + kSigma0; ks[1] = x1 + kSigma1; ks[2] = x2 + kSigma2; ks[3] = x3 + kSigma3;
  ks[4] = x4 + k[0]; ks[5] = x5 + k[1]; ks[6] = x6 + k[2]; ks[7] = x7 + k[3];
  ks[8] = x8 + k[4]; ks[9] = x9 + k[5]; ks[10] = x10 + k[6]; ks[11] = x11 + k[7];
  ks[12] = x12 + blk; ks[13] = x13; ks[14] = x14 + n1; ks[15] = x15 + n2;
}

// HChaCha20 (draft-irtf-cfrg-xchacha 2.2): the 20 rounds over (sigma, key,
// n[0..3]) without the feed-forward; out = words 0-3 and 12-15.  The subkey of
// XChaCha20-Poly1305 (chacha20poly1305 0.10, the cookie AEAD of
// rate_limiter.rs:156-164 / handshake.rs:719).
__device__ __forceinline__ void hchacha20(uint32_t out[8], const uint32_t k[8], const uint32_t n[4]) {
  uint32_t x0 = kSigma0, x1 = kSigma1, x2 = kSigma2, x3 = kSigma3;
  uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3];
  uint32_t x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
  uint32_t x12 = n[0], x13 = n[1], x14 = n[2], x15 = n[3];
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    WG_QR(x0, x4, x8, x12) WG_QR(x1, x5, x9, x13) WG_QR(x2, x6, x10, x14) WG_QR(x3, x7, x11, x15)
    WG_QR(x0, x5, x10, x15) WG_QR(x1, x6, x11, x12) WG_QR(x2, x7, x8, x13) WG_QR(x3, x4, x9, x14)
  }
  out[0] = x0; out[1] = x1; out[2] = x2; out[3] = x3;
  out[4] = x12; out[5] = x13; out[6] = x14; out[7] = x15;
}

// ---------------------------------------------------------------------------
// Two consecutive keystream blocks in phase-locked steps.
//
// gfx950 issues the "simple" VALU ops (v_add_u32, v_xor_b32, ...) of two waves
// of a SIMD together, i.e. at twice the rate of v_alignbit_b32 -- but only
// while the waves' streams run in step: once the waves drift apart, every op
// costs the single-issue rate (tools/microbench_valu6.hip, microbench_chacha2.hip,
// profiles/r01_microbench_valu6.txt, r01_microbench_chacha2.txt).  So the two
// blocks' 8 quarter-rounds of a step are issued as 8 adds, 8 xors, 8 rotates,
// and the workgroup's waves (4 per SIMD) re-align with s_barrier after every
// step: 2375 SIMD-cycles per wave-block instead of 3840 for the compiler-
// scheduled block function.
//
// Every wave of the workgroup must call this the same number of times (the
// barriers have to match); callers guarantee that with wave-uniform control flow.
// ---------------------------------------------------------------------------
#ifndef WG_CHACHA_PRIO
#define WG_CHACHA_PRIO 3  // wave priority during the phase-locked steps (0: unchanged)
#endif
// One rotate of a phase-locked step: v_alignbit_b32 (x, x, SH) = rotl(x, 32 - SH);
// with WG_STEP_PERM the byte rotations (SH 16: rotl 16, SH 24: rotl 8) are
// v_perm_b32 byte selects whose selector sits in an SGPR operand (%SEL; VOP3
// takes no literal on gfx950) -- the same issue cost, measured for energy.
#ifndef WG_STEP_PERM
#define WG_STEP_PERM 0
#endif
#define WG_ROT_A(R, SH) "v_alignbit_b32 %" #R ", %" #R ", %" #R ", " #SH "\n\t"
#define WG_ROT_P(R, SEL) "v_perm_b32 %" #R ", %" #R ", %" #R ", %" #SEL "\n\t"
#if WG_STEP_PERM
#define WG_ROT_16(R, SEL) WG_ROT_P(R, SEL)
#define WG_ROT_24(R, SEL) WG_ROT_P(R, SEL)
#else
#define WG_ROT_16(R, SEL) WG_ROT_A(R, 16)
#define WG_ROT_24(R, SEL) WG_ROT_A(R, 24)
#endif
#define WG_ROT_20(R, SEL) WG_ROT_A(R, 20)
#define WG_ROT_25(R, SEL) WG_ROT_A(R, 25)
#define WG_ROT(R, SH, SEL) WG_ROT_##SH(R, SEL)
// the selector operand of the byte rotations (unused by the other steps)
constexpr uint32_t kPermRotl16 = 0x01000302u, kPermRotl8 = 0x02010003u;
__device__ __forceinline__ uint32_t perm_sel(int sh) { return sh == 16 ? kPermRotl16 : kPermRotl8; }
#if WG_STEP_PERM
#define WG_PERM_SEL(SH) , "s"(perm_sel(SH))
#else
#define WG_PERM_SEL(SH)
#endif
#define WG_STEP8_ASM(SH)                                                                  \
  "v_add_u32 %0, %0, %16\n\tv_add_u32 %1, %1, %17\n\tv_add_u32 %2, %2, %18\n\t"           \
  "v_add_u32 %3, %3, %19\n\tv_add_u32 %4, %4, %20\n\tv_add_u32 %5, %5, %21\n\t"           \
  "v_add_u32 %6, %6, %22\n\tv_add_u32 %7, %7, %23\n\t"                                    \
  "v_xor_b32 %8, %8, %0\n\tv_xor_b32 %9, %9, %1\n\tv_xor_b32 %10, %10, %2\n\t"            \
  "v_xor_b32 %11, %11, %3\n\tv_xor_b32 %12, %12, %4\n\tv_xor_b32 %13, %13, %5\n\t"        \
  "v_xor_b32 %14, %14, %6\n\tv_xor_b32 %15, %15, %7\n\t"                                  \
  WG_ROT(8, SH, 24) WG_ROT(9, SH, 24) WG_ROT(10, SH, 24) WG_ROT(11, SH, 24)                 \
  WG_ROT(12, SH, 24) WG_ROT(13, SH, 24) WG_ROT(14, SH, 24) WG_ROT(15, SH, 24)                 \
  "s_barrier"
// Single-block form of the phase-locked steps (4 quarter-rounds per step:
// 4 v_add + 4 v_xor + 4 v_alignbit + s_barrier), for the Poly1305 key block.
#define WG_STEP4_ASM(SH)                                                                  \
  "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %9\n\tv_add_u32 %2, %2, %10\n\t"            \
  "v_add_u32 %3, %3, %11\n\t"                                                            \
  "v_xor_b32 %4, %4, %0\n\tv_xor_b32 %5, %5, %1\n\tv_xor_b32 %6, %6, %2\n\t"              \
  "v_xor_b32 %7, %7, %3\n\t"                                                             \
  WG_ROT(4, SH, 12) WG_ROT(5, SH, 12) WG_ROT(6, SH, 12) WG_ROT(7, SH, 12)                     \
  "s_barrier"
#define WG_COLUMN_ROUND1 \
  asm volatile(WG_STEP4_ASM(16) : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p12), "+v"(p13), "+v"(p14), "+v"(p15) : "v"(p4), "v"(p5), "v"(p6), "v"(p7) WG_PERM_SEL(16)); \
  asm volatile(WG_STEP4_ASM(20) : "+v"(p8), "+v"(p9), "+v"(p10), "+v"(p11), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7) : "v"(p12), "v"(p13), "v"(p14), "v"(p15) WG_PERM_SEL(20)); \
  asm volatile(WG_STEP4_ASM(24) : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p12), "+v"(p13), "+v"(p14), "+v"(p15) : "v"(p4), "v"(p5), "v"(p6), "v"(p7) WG_PERM_SEL(24)); \
  asm volatile(WG_STEP4_ASM(25) : "+v"(p8), "+v"(p9), "+v"(p10), "+v"(p11), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7) : "v"(p12), "v"(p13), "v"(p14), "v"(p15) WG_PERM_SEL(25));
#define WG_DIAGONAL_ROUND1 \
  asm volatile(WG_STEP4_ASM(16) : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p15), "+v"(p12), "+v"(p13), "+v"(p14) : "v"(p5), "v"(p6), "v"(p7), "v"(p4) WG_PERM_SEL(16)); \
  asm volatile(WG_STEP4_ASM(20) : "+v"(p10), "+v"(p11), "+v"(p8), "+v"(p9), "+v"(p5), "+v"(p6), "+v"(p7), "+v"(p4) : "v"(p15), "v"(p12), "v"(p13), "v"(p14) WG_PERM_SEL(20)); \
  asm volatile(WG_STEP4_ASM(24) : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p15), "+v"(p12), "+v"(p13), "+v"(p14) : "v"(p5), "v"(p6), "v"(p7), "v"(p4) WG_PERM_SEL(24)); \
  asm volatile(WG_STEP4_ASM(25) : "+v"(p10), "+v"(p11), "+v"(p8), "+v"(p9), "+v"(p5), "+v"(p6), "+v"(p7), "+v"(p4) : "v"(p15), "v"(p12), "v"(p13), "v"(p14) WG_PERM_SEL(25));

// Keystream block blk, phase-locked (same barrier contract as chacha20_block2_sync).
__device__ __forceinline__ void chacha20_block_sync(uint32_t (&ks)[16], const uint32_t k[8],
                                                    uint32_t blk, uint32_t n1, uint32_t n2) {
  uint32_t p0 = kSigma0, p1 = kSigma1, p2 = kSigma2, p3 = kSigma3;
  uint32_t p4 = k[0], p5 = k[1], p6 = k[2], p7 = k[3], p8 = k[4], p9 = k[5], p10 = k[6], p11 = k[7];
  uint32_t p12 = blk, p13 = 0, p14 = n1, p15 = n2;
  WG_QR(p0, p4, p8, p12) WG_QR(p1, p5, p9, p13) WG_QR(p2, p6, p10, p14) WG_QR(p3, p7, p11, p15)
  __builtin_amdgcn_s_barrier();
#if WG_CHACHA_PRIO
  __builtin_amdgcn_s_setprio(WG_CHACHA_PRIO);
#endif
  WG_DIAGONAL_ROUND1
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    WG_COLUMN_ROUND1
    WG_DIAGONAL_ROUND1
  }
#if WG_CHACHA_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
  ks[0] = p0 + kSigma0; ks[1] = p1 + kSigma1; ks[2] = p2 + kSigma2; ks[3] = p3 + kSigma3;
  ks[4] = p4 + k[0]; ks[5] = p5 + k[1]; ks[6] = p6 + k[2]; ks[7] = p7 + k[3];
  ks[8] = p8 + k[4]; ks[9] = p9 + k[5]; ks[10] = p10 + k[6]; ks[11] = p11 + k[7];
  ks[12] = p12 + blk; ks[13] = p13; ks[14] = p14 + n1; ks[15] = p15 + n2;
}

// One column round and one diagonal round of both blocks (p = block blk,
// q = block blk + 1, 16 named state words each), 4 steps per round.  Named
// scalars, not arrays: the compiler keeps arrays that are addressed through
// pointers in register tuples and spills them whole.
#define WG_COLUMN_ROUND2 \
  asm volatile(WG_STEP8_ASM(16) : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(p12), "+v"(p13), "+v"(p14), "+v"(p15), "+v"(q12), "+v"(q13), "+v"(q14), "+v"(q15) : "v"(p4), "v"(p5), "v"(p6), "v"(p7), "v"(q4), "v"(q5), "v"(q6), "v"(q7) WG_PERM_SEL(16)); \
  asm volatile(WG_STEP8_ASM(20) : "+v"(p8), "+v"(p9), "+v"(p10), "+v"(p11), "+v"(q8), "+v"(q9), "+v"(q10), "+v"(q11), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7) : "v"(p12), "v"(p13), "v"(p14), "v"(p15), "v"(q12), "v"(q13), "v"(q14), "v"(q15) WG_PERM_SEL(20)); \
  asm volatile(WG_STEP8_ASM(24) : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(p12), "+v"(p13), "+v"(p14), "+v"(p15), "+v"(q12), "+v"(q13), "+v"(q14), "+v"(q15) : "v"(p4), "v"(p5), "v"(p6), "v"(p7), "v"(q4), "v"(q5), "v"(q6), "v"(q7) WG_PERM_SEL(24)); \
  asm volatile(WG_STEP8_ASM(25) : "+v"(p8), "+v"(p9), "+v"(p10), "+v"(p11), "+v"(q8), "+v"(q9), "+v"(q10), "+v"(q11), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7) : "v"(p12), "v"(p13), "v"(p14), "v"(p15), "v"(q12), "v"(q13), "v"(q14), "v"(q15) WG_PERM_SEL(25));
#define WG_DIAGONAL_ROUND2 \
  asm volatile(WG_STEP8_ASM(16) : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(p15), "+v"(p12), "+v"(p13), "+v"(p14), "+v"(q15), "+v"(q12), "+v"(q13), "+v"(q14) : "v"(p5), "v"(p6), "v"(p7), "v"(p4), "v"(q5), "v"(q6), "v"(q7), "v"(q4) WG_PERM_SEL(16)); \
  asm volatile(WG_STEP8_ASM(20) : "+v"(p10), "+v"(p11), "+v"(p8), "+v"(p9), "+v"(q10), "+v"(q11), "+v"(q8), "+v"(q9), "+v"(p5), "+v"(p6), "+v"(p7), "+v"(p4), "+v"(q5), "+v"(q6), "+v"(q7), "+v"(q4) : "v"(p15), "v"(p12), "v"(p13), "v"(p14), "v"(q15), "v"(q12), "v"(q13), "v"(q14) WG_PERM_SEL(20)); \
  asm volatile(WG_STEP8_ASM(24) : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(p15), "+v"(p12), "+v"(p13), "+v"(p14), "+v"(q15), "+v"(q12), "+v"(q13), "+v"(q14) : "v"(p5), "v"(p6), "v"(p7), "v"(p4), "v"(q5), "v"(q6), "v"(q7), "v"(q4) WG_PERM_SEL(24)); \
  asm volatile(WG_STEP8_ASM(25) : "+v"(p10), "+v"(p11), "+v"(p8), "+v"(p9), "+v"(q10), "+v"(q11), "+v"(q8), "+v"(q9), "+v"(p5), "+v"(p6), "+v"(p7), "+v"(p4), "+v"(q5), "+v"(q6), "+v"(q7), "+v"(q4) : "v"(p15), "v"(p12), "v"(p13), "v"(p14), "v"(q15), "v"(q12), "v"(q13), "v"(q14) WG_PERM_SEL(25));

#ifndef WG_SHARED_DIAG
#define WG_SHARED_DIAG 1  // first diagonal round with the two blocks' common words shared
#endif

// keystream blocks blk and blk+1 (same key and nonce) into ka, kb.  kShared:
// the first diagonal round on the blocks' common words (below); the descriptor
// kernels (per-lane keys) keep the in-place form, where it cost one more spill.
// chacha20_block_pair_sync: any two blocks blk, blk_b of one key and nonce (they too
// differ in word 12 only) -- the split strided kernels' first call of a part, block 0
// (the Poly1305 key) with the block whose last 16 bytes the part's first round needs.
template <bool kShared = WG_SHARED_DIAG>
__device__ __forceinline__ void chacha20_block_pair_sync(uint32_t (&ka)[16], uint32_t (&kb)[16],
                                                         const uint32_t k[8], uint32_t blk, uint32_t blk_b,
                                                         uint32_t n1, uint32_t n2) {
  uint32_t p0 = kSigma0, p1 = kSigma1, p2 = kSigma2, p3 = kSigma3;
  uint32_t p4 = k[0], p5 = k[1], p6 = k[2], p7 = k[3], p8 = k[4], p9 = k[5], p10 = k[6], p11 = k[7];
  uint32_t p12 = blk, p13 = 0, p14 = n1, p15 = n2;
  uint32_t q0 = kSigma0, q1 = kSigma1, q2 = kSigma2, q3 = kSigma3;
  uint32_t q4 = k[0], q5 = k[1], q6 = k[2], q7 = k[3], q8 = k[4], q9 = k[5], q10 = k[6], q11 = k[7];
  uint32_t q12 = blk_b, q13 = 0, q14 = n1, q15 = n2;
  // the first column round stays compiler-scheduled: with a wave-uniform key
  // and counter its wave-uniform columns run on the scalar unit
  WG_QR(p0, p4, p8, p12) WG_QR(p1, p5, p9, p13) WG_QR(p2, p6, p10, p14) WG_QR(p3, p7, p11, p15)
  if constexpr (!kShared) {
    WG_QR(q0, q4, q8, q12) WG_QR(q1, q5, q9, q13) WG_QR(q2, q6, q10, q14) WG_QR(q3, q7, q11, q15)
  }
  __builtin_amdgcn_s_barrier();
#if WG_CHACHA_PRIO
  __builtin_amdgcn_s_setprio(WG_CHACHA_PRIO);  // the phase-locked steps go first
#endif
  if constexpr (kShared) {
    // The blocks differ only in word 12, so after the first column round their
    // columns 1-3 are equal (s*: the compiler computes them once per packet and
    // holds them) and only column 0 is per block.  The first diagonal round
    // reads the common words as inputs and writes fresh registers -- in-place
    // steps made the compiler copy every common word into both blocks first
    // (24 v_mov per round) -- and the ops whose operands are all common (words
    // 1 and 2's first add, word 13's first xor-rotate) run once for both.
    WG_QR(q0, q4, q8, q12)
    const uint32_t s1 = p1, s2 = p2, s3 = p3, s5 = p5, s6 = p6, s7 = p7;
    const uint32_t s9 = p9, s10 = p10, s11 = p11, s13 = p13, s14 = p14, s15 = p15;
    uint32_t a1, a2, d13;
    // step 1: a += b; d ^= a; d <<<= 16   (6 + 7 + 7 ops instead of 8 + 8 + 8)
    asm volatile(
        "v_add_u32 %[p0], %[p0], %[s5]\n\tv_add_u32 %[q0], %[q0], %[s5]\n\t"
        "v_add_u32 %[a1], %[s1], %[s6]\n\tv_add_u32 %[a2], %[s2], %[s7]\n\t"
        "v_add_u32 %[p3], %[s3], %[p4]\n\tv_add_u32 %[q3], %[s3], %[q4]\n\t"
        "v_xor_b32 %[p15], %[s15], %[p0]\n\tv_xor_b32 %[q15], %[s15], %[q0]\n\t"
        "v_xor_b32 %[p12], %[p12], %[a1]\n\tv_xor_b32 %[q12], %[q12], %[a1]\n\t"
        "v_xor_b32 %[d13], %[s13], %[a2]\n\t"
        "v_xor_b32 %[p14], %[s14], %[p3]\n\tv_xor_b32 %[q14], %[s14], %[q3]\n\t"
        "v_alignbit_b32 %[p15], %[p15], %[p15], 16\n\tv_alignbit_b32 %[q15], %[q15], %[q15], 16\n\t"
        "v_alignbit_b32 %[p12], %[p12], %[p12], 16\n\tv_alignbit_b32 %[q12], %[q12], %[q12], 16\n\t"
        "v_alignbit_b32 %[d13], %[d13], %[d13], 16\n\t"
        "v_alignbit_b32 %[p14], %[p14], %[p14], 16\n\tv_alignbit_b32 %[q14], %[q14], %[q14], 16\n\t"
        "s_barrier"
        : [p0] "+v"(p0), [q0] "+v"(q0), [a1] "=&v"(a1), [a2] "=&v"(a2), [p3] "=&v"(p3),
          [q3] "=&v"(q3), [p15] "=&v"(p15), [q15] "=&v"(q15), [p12] "+v"(p12), [q12] "+v"(q12),
          [d13] "=&v"(d13), [p14] "=&v"(p14), [q14] "=&v"(q14)
        : [s5] "v"(s5), [s1] "v"(s1), [s6] "v"(s6), [s2] "v"(s2), [s7] "v"(s7), [s3] "v"(s3),
          [p4] "v"(p4), [q4] "v"(q4), [s15] "v"(s15), [s13] "v"(s13), [s14] "v"(s14));
    // step 2: c += d; b ^= c; b <<<= 12
    asm volatile(
        "v_add_u32 %[p10], %[s10], %[p15]\n\tv_add_u32 %[q10], %[s10], %[q15]\n\t"
        "v_add_u32 %[p11], %[s11], %[p12]\n\tv_add_u32 %[q11], %[s11], %[q12]\n\t"
        "v_add_u32 %[p8], %[p8], %[d13]\n\tv_add_u32 %[q8], %[q8], %[d13]\n\t"
        "v_add_u32 %[p9], %[s9], %[p14]\n\tv_add_u32 %[q9], %[s9], %[q14]\n\t"
        "v_xor_b32 %[p5], %[s5], %[p10]\n\tv_xor_b32 %[q5], %[s5], %[q10]\n\t"
        "v_xor_b32 %[p6], %[s6], %[p11]\n\tv_xor_b32 %[q6], %[s6], %[q11]\n\t"
        "v_xor_b32 %[p7], %[s7], %[p8]\n\tv_xor_b32 %[q7], %[s7], %[q8]\n\t"
        "v_xor_b32 %[p4], %[p4], %[p9]\n\tv_xor_b32 %[q4], %[q4], %[q9]\n\t"
        "v_alignbit_b32 %[p5], %[p5], %[p5], 20\n\tv_alignbit_b32 %[q5], %[q5], %[q5], 20\n\t"
        "v_alignbit_b32 %[p6], %[p6], %[p6], 20\n\tv_alignbit_b32 %[q6], %[q6], %[q6], 20\n\t"
        "v_alignbit_b32 %[p7], %[p7], %[p7], 20\n\tv_alignbit_b32 %[q7], %[q7], %[q7], 20\n\t"
        "v_alignbit_b32 %[p4], %[p4], %[p4], 20\n\tv_alignbit_b32 %[q4], %[q4], %[q4], 20\n\t"
        "s_barrier"
        : [p10] "=&v"(p10), [q10] "=&v"(q10), [p11] "=&v"(p11), [q11] "=&v"(q11), [p8] "+v"(p8),
          [q8] "+v"(q8), [p9] "=&v"(p9), [q9] "=&v"(q9), [p5] "=&v"(p5), [q5] "=&v"(q5),
          [p6] "=&v"(p6), [q6] "=&v"(q6), [p7] "=&v"(p7), [q7] "=&v"(q7), [p4] "+v"(p4),
          [q4] "+v"(q4)
        : [s10] "v"(s10), [s11] "v"(s11), [s9] "v"(s9), [p15] "v"(p15), [q15] "v"(q15),
          [p12] "v"(p12), [q12] "v"(q12), [d13] "v"(d13), [p14] "v"(p14), [q14] "v"(q14),
          [s5] "v"(s5), [s6] "v"(s6), [s7] "v"(s7));
    // step 3: a += b; d ^= a; d <<<= 8   (words 1, 2 and 13 split into the two blocks here)
    asm volatile(
        "v_add_u32 %[p0], %[p0], %[p5]\n\tv_add_u32 %[q0], %[q0], %[q5]\n\t"
        "v_add_u32 %[p1], %[a1], %[p6]\n\tv_add_u32 %[q1], %[a1], %[q6]\n\t"
        "v_add_u32 %[p2], %[a2], %[p7]\n\tv_add_u32 %[q2], %[a2], %[q7]\n\t"
        "v_add_u32 %[p3], %[p3], %[p4]\n\tv_add_u32 %[q3], %[q3], %[q4]\n\t"
        "v_xor_b32 %[p15], %[p15], %[p0]\n\tv_xor_b32 %[q15], %[q15], %[q0]\n\t"
        "v_xor_b32 %[p12], %[p12], %[p1]\n\tv_xor_b32 %[q12], %[q12], %[q1]\n\t"
        "v_xor_b32 %[p13], %[d13], %[p2]\n\tv_xor_b32 %[q13], %[d13], %[q2]\n\t"
        "v_xor_b32 %[p14], %[p14], %[p3]\n\tv_xor_b32 %[q14], %[q14], %[q3]\n\t"
        "v_alignbit_b32 %[p15], %[p15], %[p15], 24\n\tv_alignbit_b32 %[q15], %[q15], %[q15], 24\n\t"
        "v_alignbit_b32 %[p12], %[p12], %[p12], 24\n\tv_alignbit_b32 %[q12], %[q12], %[q12], 24\n\t"
        "v_alignbit_b32 %[p13], %[p13], %[p13], 24\n\tv_alignbit_b32 %[q13], %[q13], %[q13], 24\n\t"
        "v_alignbit_b32 %[p14], %[p14], %[p14], 24\n\tv_alignbit_b32 %[q14], %[q14], %[q14], 24\n\t"
        "s_barrier"
        : [p0] "+v"(p0), [q0] "+v"(q0), [p1] "=&v"(p1), [q1] "=&v"(q1), [p2] "=&v"(p2),
          [q2] "=&v"(q2), [p3] "+v"(p3), [q3] "+v"(q3), [p15] "+v"(p15), [q15] "+v"(q15),
          [p12] "+v"(p12), [q12] "+v"(q12), [p13] "=&v"(p13), [q13] "=&v"(q13), [p14] "+v"(p14),
          [q14] "+v"(q14)
        : [p5] "v"(p5), [q5] "v"(q5), [a1] "v"(a1), [p6] "v"(p6), [q6] "v"(q6), [a2] "v"(a2),
          [p7] "v"(p7), [q7] "v"(q7), [d13] "v"(d13), [p4] "v"(p4), [q4] "v"(q4));
    // step 4: the ordinary in-place step (no common words left)
    asm volatile(WG_STEP8_ASM(25) : "+v"(p10), "+v"(p11), "+v"(p8), "+v"(p9), "+v"(q10), "+v"(q11), "+v"(q8), "+v"(q9), "+v"(p5), "+v"(p6), "+v"(p7), "+v"(p4), "+v"(q5), "+v"(q6), "+v"(q7), "+v"(q4) : "v"(p15), "v"(p12), "v"(p13), "v"(p14), "v"(q15), "v"(q12), "v"(q13), "v"(q14) WG_PERM_SEL(25));
  } else {
    WG_DIAGONAL_ROUND2
  }
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    WG_COLUMN_ROUND2
    WG_DIAGONAL_ROUND2
  }
#if WG_CHACHA_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
  ka[0] = p0 + kSigma0; ka[1] = p1 + kSigma1; ka[2] = p2 + kSigma2; ka[3] = p3 + kSigma3;
  ka[4] = p4 + k[0]; ka[5] = p5 + k[1]; ka[6] = p6 + k[2]; ka[7] = p7 + k[3];
  ka[8] = p8 + k[4]; ka[9] = p9 + k[5]; ka[10] = p10 + k[6]; ka[11] = p11 + k[7];
  ka[12] = p12 + blk; ka[13] = p13; ka[14] = p14 + n1; ka[15] = p15 + n2;
  kb[0] = q0 + kSigma0; kb[1] = q1 + kSigma1; kb[2] = q2 + kSigma2; kb[3] = q3 + kSigma3;
  kb[4] = q4 + k[0]; kb[5] = q5 + k[1]; kb[6] = q6 + k[2]; kb[7] = q7 + k[3];
  kb[8] = q8 + k[4]; kb[9] = q9 + k[5]; kb[10] = q10 + k[6]; kb[11] = q11 + k[7];
  kb[12] = q12 + blk_b; kb[13] = q13; kb[14] = q14 + n1; kb[15] = q15 + n2;
}
template <bool kShared = WG_SHARED_DIAG>
__device__ __forceinline__ void chacha20_block2_sync(uint32_t (&ka)[16], uint32_t (&kb)[16],
                                                     const uint32_t k[8], uint32_t blk,
                                                     uint32_t n1, uint32_t n2) {
  chacha20_block_pair_sync<kShared>(ka, kb, k, blk, blk + 1u, n1, n2);
}

// ---------------------------------------------------------------------------
// Poly1305 (RFC 8439 2.5) -- two limb schemes, same results bit for bit:
//  * radix 2^32 (default): 4 x 32-bit limbs + a 3-bit top limb, 21
//    v_mad_u64_u32 on full 32-bit operands, 39 VALU per 16-byte block;
//  * radix 2^26 (-DWG_POLY_RADIX26=1): 5 x 26-bit limbs (poly1305-donna-32),
//    25 v_mad_u64_u32 whose operands carry <= 27 / 29 significant bits, 54
//    VALU per block.  More instructions, narrower multiplies: built to measure
//    energy per block at the package power limit, where time
//    follows energy, not issue slots.
// ---------------------------------------------------------------------------
#ifndef WG_POLY_RADIX26
#define WG_POLY_RADIX26 0
#endif

#if WG_POLY_RADIX26
struct Poly {
  uint32_t h0, h1, h2, h3, h4;  // 26-bit limbs (h1 may carry a few bits more between blocks)
  uint32_t r0, r1, r2, r3, r4;  // clamped r, 26-bit limbs
  uint32_t s1, s2, s3, s4;      // 5 * r_i (2^130 == 5)
};

__device__ __forceinline__ void poly_init(Poly &p, const uint32_t ks0[8]) {
  const uint32_t w0 = ks0[0] & 0x0fffffffu, w1 = ks0[1] & 0x0ffffffcu, w2 = ks0[2] & 0x0ffffffcu,
                 w3 = ks0[3] & 0x0ffffffcu;
  p.r0 = w0 & 0x3ffffffu;
  p.r1 = ((w0 >> 26) | (w1 << 6)) & 0x3ffffffu;
  p.r2 = ((w1 >> 20) | (w2 << 12)) & 0x3ffffffu;
  p.r3 = ((w2 >> 14) | (w3 << 18)) & 0x3ffffffu;
  p.r4 = w3 >> 8;
  p.s1 = 5u * p.r1;
  p.s2 = 5u * p.r2;
  p.s3 = 5u * p.r3;
  p.s4 = 5u * p.r4;
  p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0;
}

// h = (h + m + 2^128) * r, partially reduced.  Bounds: h_i < 2^27 after the
// add, s_i < 2^29, so each product < 2^56 and each 5-term chain + seed < 2^59;
// d4 (no s terms) < 2^55.4, so its carry fits 32 bits and 5 * it fits too.
__device__ __forceinline__ void poly_block(Poly &p, uint32_t m0, uint32_t m1, uint32_t m2,
                                           uint32_t m3) {
  // m + 2^128 in 26-bit limbs (funnel shifts), added to h
  const uint32_t a0 = p.h0 + (m0 & 0x3ffffffu);
  const uint32_t a1 = p.h1 + (__builtin_amdgcn_alignbit(m1, m0, 26) & 0x3ffffffu);
  const uint32_t a2 = p.h2 + (__builtin_amdgcn_alignbit(m2, m1, 20) & 0x3ffffffu);
  const uint32_t a3 = p.h3 + (__builtin_amdgcn_alignbit(m3, m2, 14) & 0x3ffffffu);
  const uint32_t a4 = p.h4 + ((m3 >> 8) | (1u << 24));
  uint64_t d0, d1, d2, d3, d4, seed, sc;
  asm volatile(
      // d0 = h0 r0 + h1 s4 + h2 s3 + h3 s2 + h4 s1
      "v_mad_u64_u32 %[d0], %[sc], %[a0], %[r0], 0\n\t"
      "v_mad_u64_u32 %[d0], %[sc], %[a1], %[s4], %[d0]\n\t"
      "v_mad_u64_u32 %[d0], %[sc], %[a2], %[s3], %[d0]\n\t"
      "v_mad_u64_u32 %[d0], %[sc], %[a3], %[s2], %[d0]\n\t"
      "v_mad_u64_u32 %[d0], %[sc], %[a4], %[s1], %[d0]\n\t"
      // d1 = (d0 >> 26) + h0 r1 + h1 r0 + h2 s4 + h3 s3 + h4 s2
      "v_lshrrev_b64 %[seed], 26, %[d0]\n\t"
      "v_mad_u64_u32 %[d1], %[sc], %[a0], %[r1], %[seed]\n\t"
      "v_mad_u64_u32 %[d1], %[sc], %[a1], %[r0], %[d1]\n\t"
      "v_mad_u64_u32 %[d1], %[sc], %[a2], %[s4], %[d1]\n\t"
      "v_mad_u64_u32 %[d1], %[sc], %[a3], %[s3], %[d1]\n\t"
      "v_mad_u64_u32 %[d1], %[sc], %[a4], %[s2], %[d1]\n\t"
      // d2 = (d1 >> 26) + h0 r2 + h1 r1 + h2 r0 + h3 s4 + h4 s3
      "v_lshrrev_b64 %[seed], 26, %[d1]\n\t"
      "v_mad_u64_u32 %[d2], %[sc], %[a0], %[r2], %[seed]\n\t"
      "v_mad_u64_u32 %[d2], %[sc], %[a1], %[r1], %[d2]\n\t"
      "v_mad_u64_u32 %[d2], %[sc], %[a2], %[r0], %[d2]\n\t"
      "v_mad_u64_u32 %[d2], %[sc], %[a3], %[s4], %[d2]\n\t"
      "v_mad_u64_u32 %[d2], %[sc], %[a4], %[s3], %[d2]\n\t"
      // d3 = (d2 >> 26) + h0 r3 + h1 r2 + h2 r1 + h3 r0 + h4 s4
      "v_lshrrev_b64 %[seed], 26, %[d2]\n\t"
      "v_mad_u64_u32 %[d3], %[sc], %[a0], %[r3], %[seed]\n\t"
      "v_mad_u64_u32 %[d3], %[sc], %[a1], %[r2], %[d3]\n\t"
      "v_mad_u64_u32 %[d3], %[sc], %[a2], %[r1], %[d3]\n\t"
      "v_mad_u64_u32 %[d3], %[sc], %[a3], %[r0], %[d3]\n\t"
      "v_mad_u64_u32 %[d3], %[sc], %[a4], %[s4], %[d3]\n\t"
      // d4 = (d3 >> 26) + h0 r4 + h1 r3 + h2 r2 + h3 r1 + h4 r0
      "v_lshrrev_b64 %[seed], 26, %[d3]\n\t"
      "v_mad_u64_u32 %[d4], %[sc], %[a0], %[r4], %[seed]\n\t"
      "v_mad_u64_u32 %[d4], %[sc], %[a1], %[r3], %[d4]\n\t"
      "v_mad_u64_u32 %[d4], %[sc], %[a2], %[r2], %[d4]\n\t"
      "v_mad_u64_u32 %[d4], %[sc], %[a3], %[r1], %[d4]\n\t"
      "v_mad_u64_u32 %[d4], %[sc], %[a4], %[r0], %[d4]"
      : [d0] "=&v"(d0), [d1] "=&v"(d1), [d2] "=&v"(d2), [d3] "=&v"(d3), [d4] "=&v"(d4),
        [seed] "=&v"(seed), [sc] "=&s"(sc)
      : [a0] "v"(a0), [a1] "v"(a1), [a2] "v"(a2), [a3] "v"(a3), [a4] "v"(a4),
        [r0] "v"(p.r0), [r1] "v"(p.r1), [r2] "v"(p.r2), [r3] "v"(p.r3), [r4] "v"(p.r4),
        [s1] "v"(p.s1), [s2] "v"(p.s2), [s3] "v"(p.s3), [s4] "v"(p.s4));
  // bits >= 130: c = d4 >> 26 (< 2^30), folded as 5c into limb 0, one carry into limb 1
  const uint32_t c = __builtin_amdgcn_alignbit((uint32_t)(d4 >> 32), (uint32_t)d4, 26);
  const uint32_t h0 = ((uint32_t)d0 & 0x3ffffffu) + 5u * c;
  p.h0 = h0 & 0x3ffffffu;
  p.h1 = ((uint32_t)d1 & 0x3ffffffu) + (h0 >> 26);
  p.h2 = (uint32_t)d2 & 0x3ffffffu;
  p.h3 = (uint32_t)d3 & 0x3ffffffu;
  p.h4 = (uint32_t)d4 & 0x3ffffffu;
}

// tag = (h mod p) + s mod 2^128 (full carry, h + 5 >= 2^130 <=> h >= p)
__device__ __forceinline__ void poly_finish(const Poly &p, const uint32_t s[4], uint32_t tag[4]) {
  uint32_t h0 = p.h0, h1 = p.h1, h2 = p.h2, h3 = p.h3, h4 = p.h4, c;
  c = h1 >> 26; h1 &= 0x3ffffffu; h2 += c;
  c = h2 >> 26; h2 &= 0x3ffffffu; h3 += c;
  c = h3 >> 26; h3 &= 0x3ffffffu; h4 += c;
  c = h4 >> 26; h4 &= 0x3ffffffu; h0 += 5u * c;
  c = h0 >> 26; h0 &= 0x3ffffffu; h1 += c;
  // g = h + 5 - 2^130
  uint32_t g0 = h0 + 5u; c = g0 >> 26; g0 &= 0x3ffffffu;
  uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffffu;
  uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffffu;
  uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffffu;
  const uint32_t g4 = h4 + c - (1u << 26);
  const bool ge = (g4 >> 31) == 0u;  // no borrow: h >= p
  if (ge) { h0 = g0; h1 = g1; h2 = g2; h3 = g3; h4 = g4; }
  const uint32_t f0 = h0 | (h1 << 26), f1 = (h1 >> 6) | (h2 << 20), f2 = (h2 >> 12) | (h3 << 14),
                 f3 = (h3 >> 18) | (h4 << 8);
  uint64_t t = (uint64_t)f0 + s[0];
  tag[0] = (uint32_t)t;
  t = (uint64_t)f1 + s[1] + (t >> 32);
  tag[1] = (uint32_t)t;
  t = (uint64_t)f2 + s[2] + (t >> 32);
  tag[2] = (uint32_t)t;
  tag[3] = f3 + s[3] + (uint32_t)(t >> 32);
}

#else  // radix 2^32

// radix 2^32: h = h0..h3 (32-bit) + h4 (< 8)
struct Poly {
  uint32_t h0, h1, h2, h3, h4;
  uint32_t r0, r1, r2, r3;  // clamped r
  uint32_t s1, s2, s3;      // 5*r_i/4 (r1..r3 are multiples of 4)
};

__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * b + c;  // v_mad_u64_u32
}

__device__ __forceinline__ void poly_init(Poly &p, const uint32_t ks0[8]) {
  p.r0 = ks0[0] & 0x0fffffffu;
  p.r1 = ks0[1] & 0x0ffffffcu;
  p.r2 = ks0[2] & 0x0ffffffcu;
  p.r3 = ks0[3] & 0x0ffffffcu;
  p.s1 = p.r1 + (p.r1 >> 2);
  p.s2 = p.r2 + (p.r2 >> 2);
  p.s3 = p.r3 + (p.r3 >> 2);
  p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0;
}

#ifndef WG_POLY_ASM
#define WG_POLY_ASM 1
#endif

#if WG_POLY_ASM
// 32x32+64 -> 64 multiply-add, kept as written: hipcc otherwise re-associates
// the carry-seeded chains below into zero-seeded mads + v_lshl_add_u64 adds,
// which costs ~13 extra half-rate ops per 16-byte block.
__device__ __forceinline__ uint64_t mad_c(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t d, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(cc) : "v"(a), "v"(b), "v"(c));
  return d;
}
#else
__device__ __forceinline__ uint64_t mad_c(uint32_t a, uint32_t b, uint64_t c) { return mad(a, b, c); }
#endif

#ifndef WG_POLY_ONE_ASM
#define WG_POLY_ONE_ASM 1
#endif

#if WG_POLY_ONE_ASM
// h = (h + m + 2^128) * r  (partially reduced mod 2^130 - 5).
// The 21 multiply-accumulates are ONE asm statement: the compiler pads every
// separate asm statement that writes an SGPR (the mads' carry-out) with an
// s_nop, which cost 21 issue slots per block.  Inside: the h + m + 2^128 carry
// chain, four carry-seeded chains d0..d3 (2^130 == 5 folding via s_i = 5 r_i / 4;
// seed = (d_{j-1} >> 32) by a 64-bit shift), and h4 * r0.  The carry-out goes to
// a scratch SGPR pair nothing reads.
__device__ __forceinline__ void poly_block(Poly &p, uint32_t m0, uint32_t m1, uint32_t m2,
                                           uint32_t m3) {
  uint32_t a0, a1, a2, a3, a4;  // h + m + 2^128
  uint64_t d0, d1, d2, d3, e4, seed, sc;
  asm volatile(
      "v_add_co_u32 %[a0], vcc, %[h0], %[m0]\n\t"
      "v_addc_co_u32 %[a1], vcc, %[h1], %[m1], vcc\n\t"
      "v_addc_co_u32 %[a2], vcc, %[h2], %[m2], vcc\n\t"
      "v_addc_co_u32 %[a3], vcc, %[h3], %[m3], vcc\n\t"
      "v_addc_co_u32 %[a4], vcc, 1, %[h4], vcc\n\t"
      // d0 = h0 r0 + h1 s3 + h2 s2 + h3 s1
      "v_mad_u64_u32 %[d0], %[sc], %[a0], %[r0], 0\n\t"
      "v_mad_u64_u32 %[d0], %[sc], %[a1], %[s3], %[d0]\n\t"
      "v_mad_u64_u32 %[d0], %[sc], %[a2], %[s2], %[d0]\n\t"
      "v_mad_u64_u32 %[d0], %[sc], %[a3], %[s1], %[d0]\n\t"
      // d1 = (d0 >> 32) + h0 r1 + h1 r0 + h2 s3 + h3 s2 + h4 s1
      "v_lshrrev_b64 %[seed], 32, %[d0]\n\t"
      "v_mad_u64_u32 %[d1], %[sc], %[a0], %[r1], %[seed]\n\t"
      "v_mad_u64_u32 %[d1], %[sc], %[a1], %[r0], %[d1]\n\t"
      "v_mad_u64_u32 %[d1], %[sc], %[a2], %[s3], %[d1]\n\t"
      "v_mad_u64_u32 %[d1], %[sc], %[a3], %[s2], %[d1]\n\t"
      "v_mad_u64_u32 %[d1], %[sc], %[a4], %[s1], %[d1]\n\t"
      // d2 = (d1 >> 32) + h0 r2 + h1 r1 + h2 r0 + h3 s3 + h4 s2
      "v_lshrrev_b64 %[seed], 32, %[d1]\n\t"
      "v_mad_u64_u32 %[d2], %[sc], %[a0], %[r2], %[seed]\n\t"
      "v_mad_u64_u32 %[d2], %[sc], %[a1], %[r1], %[d2]\n\t"
      "v_mad_u64_u32 %[d2], %[sc], %[a2], %[r0], %[d2]\n\t"
      "v_mad_u64_u32 %[d2], %[sc], %[a3], %[s3], %[d2]\n\t"
      "v_mad_u64_u32 %[d2], %[sc], %[a4], %[s2], %[d2]\n\t"
      // d3 = (d2 >> 32) + h0 r3 + h1 r2 + h2 r1 + h3 r0 + h4 s3
      "v_lshrrev_b64 %[seed], 32, %[d2]\n\t"
      "v_mad_u64_u32 %[d3], %[sc], %[a0], %[r3], %[seed]\n\t"
      "v_mad_u64_u32 %[d3], %[sc], %[a1], %[r2], %[d3]\n\t"
      "v_mad_u64_u32 %[d3], %[sc], %[a2], %[r1], %[d3]\n\t"
      "v_mad_u64_u32 %[d3], %[sc], %[a3], %[r0], %[d3]\n\t"
      "v_mad_u64_u32 %[d3], %[sc], %[a4], %[s3], %[d3]\n\t"
      // h4' = (d3 >> 32) + h4 r0  (< 2^32)
      "v_lshrrev_b64 %[seed], 32, %[d3]\n\t"
      "v_mad_u64_u32 %[e4], %[sc], %[a4], %[r0], %[seed]"
      : [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [a4] "=&v"(a4),
        [d0] "=&v"(d0), [d1] "=&v"(d1), [d2] "=&v"(d2), [d3] "=&v"(d3), [e4] "=&v"(e4),
        [seed] "=&v"(seed), [sc] "=&s"(sc)
      : [h0] "v"(p.h0), [h1] "v"(p.h1), [h2] "v"(p.h2), [h3] "v"(p.h3), [h4] "v"(p.h4),
        [m0] "v"(m0), [m1] "v"(m1), [m2] "v"(m2), [m3] "v"(m3),
        [r0] "v"(p.r0), [r1] "v"(p.r1), [r2] "v"(p.r2), [r3] "v"(p.r3),
        [s1] "v"(p.s1), [s2] "v"(p.s2), [s3] "v"(p.s3)
      : "vcc");
  // fold bits >= 130: c = 5 * (h4' >> 2), then one carry chain
  uint32_t h4 = (uint32_t)e4;
  const uint32_t c = (h4 >> 2) + (h4 & ~3u);
  h4 &= 3u;
  asm volatile(
      "v_add_co_u32 %0, vcc, %5, %6\n\t"
      "v_addc_co_u32 %1, vcc, 0, %7, vcc\n\t"
      "v_addc_co_u32 %2, vcc, 0, %8, vcc\n\t"
      "v_addc_co_u32 %3, vcc, 0, %9, vcc\n\t"
      "v_addc_co_u32 %4, vcc, 0, %10, vcc"
      : "=&v"(p.h0), "=&v"(p.h1), "=&v"(p.h2), "=&v"(p.h3), "=&v"(p.h4)
      : "v"(c), "v"((uint32_t)d0), "v"((uint32_t)d1), "v"((uint32_t)d2), "v"((uint32_t)d3),
        "v"(h4)
      : "vcc");
}
#else
// h = (h + m + 2^128) * r  (partially reduced mod 2^130 - 5)
__device__ __forceinline__ void poly_block(Poly &p, uint32_t m0, uint32_t m1, uint32_t m2,
                                           uint32_t m3) {
  uint32_t h0, h1, h2, h3, h4;
#if WG_POLY_ASM
  // h += m + 2^128: one carry chain through vcc
  asm("v_add_co_u32 %0, vcc, %5, %6\n\t"
      "v_addc_co_u32 %1, vcc, %7, %8, vcc\n\t"
      "v_addc_co_u32 %2, vcc, %9, %10, vcc\n\t"
      "v_addc_co_u32 %3, vcc, %11, %12, vcc\n\t"
      "v_addc_co_u32 %4, vcc, 1, %13, vcc"
      : "=&v"(h0), "=&v"(h1), "=&v"(h2), "=&v"(h3), "=&v"(h4)
      : "v"(p.h0), "v"(m0), "v"(p.h1), "v"(m1), "v"(p.h2), "v"(m2), "v"(p.h3), "v"(m3), "v"(p.h4)
      : "vcc");
#else
  uint64_t t = (uint64_t)p.h0 + m0;
  h0 = (uint32_t)t;
  t = (uint64_t)p.h1 + m1 + (t >> 32);
  h1 = (uint32_t)t;
  t = (uint64_t)p.h2 + m2 + (t >> 32);
  h2 = (uint32_t)t;
  t = (uint64_t)p.h3 + m3 + (t >> 32);
  h3 = (uint32_t)t;
  h4 = p.h4 + (uint32_t)(t >> 32) + 1u;  // + 2^128 (full 16-byte block)
#endif
  // d_j = sum_i h_i r_{j-i} with 2^128 == 5/4 folding (h_i r_j, i+j >= 4 -> h_i s_j);
  // each chain is seeded with the carry out of the previous one
  const uint64_t d0 = mad_c(h3, p.s1, mad_c(h2, p.s2, mad_c(h1, p.s3, mad_c(h0, p.r0, 0ull))));
  const uint64_t d1 =
      mad_c(h4, p.s1, mad_c(h3, p.s2, mad_c(h2, p.s3, mad_c(h1, p.r0, mad_c(h0, p.r1, d0 >> 32)))));
  const uint64_t d2 =
      mad_c(h4, p.s2, mad_c(h3, p.s3, mad_c(h2, p.r0, mad_c(h1, p.r1, mad_c(h0, p.r2, d1 >> 32)))));
  const uint64_t d3 =
      mad_c(h4, p.s3, mad_c(h3, p.r0, mad_c(h2, p.r1, mad_c(h1, p.r2, mad_c(h0, p.r3, d2 >> 32)))));
  h4 = (uint32_t)mad_c(h4, p.r0, d3 >> 32);
  // fold bits >= 130: c = 5 * (h4 >> 2)
  const uint32_t c = (h4 >> 2) + (h4 & ~3u);
  h4 &= 3u;
#if WG_POLY_ASM
  asm("v_add_co_u32 %0, vcc, %5, %6\n\t"
      "v_addc_co_u32 %1, vcc, 0, %7, vcc\n\t"
      "v_addc_co_u32 %2, vcc, 0, %8, vcc\n\t"
      "v_addc_co_u32 %3, vcc, 0, %9, vcc\n\t"
      "v_addc_co_u32 %4, vcc, 0, %10, vcc"
      : "=&v"(p.h0), "=&v"(p.h1), "=&v"(p.h2), "=&v"(p.h3), "=&v"(p.h4)
      : "v"(c), "v"((uint32_t)d0), "v"((uint32_t)d1), "v"((uint32_t)d2), "v"((uint32_t)d3),
        "v"(h4)
      : "vcc");
#else
  uint64_t t2 = (uint64_t)(uint32_t)d0 + c;
  p.h0 = (uint32_t)t2;
  t2 = (uint64_t)(uint32_t)d1 + (t2 >> 32);
  p.h1 = (uint32_t)t2;
  t2 = (uint64_t)(uint32_t)d2 + (t2 >> 32);
  p.h2 = (uint32_t)t2;
  t2 = (uint64_t)(uint32_t)d3 + (t2 >> 32);
  p.h3 = (uint32_t)t2;
  p.h4 = h4 + (uint32_t)(t2 >> 32);
#endif
}

#endif  // WG_POLY_ONE_ASM

// tag = (h mod p) + s mod 2^128; h < 5*2^128 < 2p so one conditional subtract
__device__ __forceinline__ void poly_finish(const Poly &p, const uint32_t s[4], uint32_t tag[4]) {
  uint64_t t = (uint64_t)p.h0 + 5u;
  const uint32_t g0 = (uint32_t)t;
  t = (uint64_t)p.h1 + (t >> 32);
  const uint32_t g1 = (uint32_t)t;
  t = (uint64_t)p.h2 + (t >> 32);
  const uint32_t g2 = (uint32_t)t;
  t = (uint64_t)p.h3 + (t >> 32);
  const uint32_t g3 = (uint32_t)t;
  const uint32_t g4 = p.h4 + (uint32_t)(t >> 32);
  const bool ge = (g4 >> 2) != 0u;  // h + 5 >= 2^130  <=>  h >= p
  const uint32_t f0 = ge ? g0 : p.h0, f1 = ge ? g1 : p.h1, f2 = ge ? g2 : p.h2,
                 f3 = ge ? g3 : p.h3;
  t = (uint64_t)f0 + s[0];
  tag[0] = (uint32_t)t;
  t = (uint64_t)f1 + s[1] + (t >> 32);
  tag[1] = (uint32_t)t;
  t = (uint64_t)f2 + s[2] + (t >> 32);
  tag[2] = (uint32_t)t;
  tag[3] = f3 + s[3] + (uint32_t)(t >> 32);
}

#endif  // WG_POLY_RADIX26

// ---------------------------------------------------------------------------
// byte-granular helpers for the packet tail (run once per packet)
// ---------------------------------------------------------------------------
// mask of the valid low bytes of word j when `valid` bytes of a 16-byte chunk are live
__device__ __forceinline__ uint32_t byte_mask(int valid, int j) {
  const int v = valid - 4 * j;
  return v >= 4 ? 0xffffffffu : (v <= 0 ? 0u : ((1u << (8 * v)) - 1u));
}

// select word idx (runtime, may be out of [0,n)) of w[n], 0 outside
template <int N>
__device__ __forceinline__ uint32_t pick(const uint32_t (&w)[N], int idx) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) r = (idx == j) ? w[j] : r;
  return r;
}

// 4 bytes of the little-endian stream w[] starting at byte offset `off` (off may be < 0)
template <int N>
__device__ __forceinline__ uint32_t bytes_at(const uint32_t (&w)[N], int off) {
  const int q = off >> 2;  // floor division (arithmetic shift)
  const uint32_t b = (uint32_t)(off & 3);
  return __builtin_amdgcn_alignbyte(pick(w, q + 1), pick(w, q), b);
}

// store the first k (1..15) bytes of a 16-byte-aligned chunk
__device__ __forceinline__ void store_partial(uint8_t *p, const uint32_t w[4], int k) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int v = k - 4 * j;
    if (v >= 4) {
      *reinterpret_cast<uint32_t *>(p + 4 * j) = w[j];
    } else if (v > 0) {
      uint8_t *pb = p + 4 * j;
      if (v >= 2) {
        *reinterpret_cast<uint16_t *>(pb) = (uint16_t)w[j];
        if (v == 3) pb[2] = (uint8_t)(w[j] >> 16);
      } else {
        pb[0] = (uint8_t)w[j];
      }
    }
  }
}

__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
  return *reinterpret_cast<const uint4 *>(p);
}
__device__ __forceinline__ void st16(uint8_t *p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  *reinterpret_cast<uint4 *>(p) = make_uint4(a, b, c, d);
}

// ---------------------------------------------------------------------------
// General multiply mod 2^130 - 5 for combining partial Poly1305 accumulators
// (several lanes per packet, wg_xlane.hip): h = sum m_i r^(n - i + 1) splits into
// spans, each span's Horner sum weighted by a power of r.  poly_block's radix
// 2^32 form relies on a clamped r; powers of r are not clamped, so these use
// radix 2^26 (poly1305-donna-32's multiply, valid for any operand whose limbs are
// below ~2^27).
// ---------------------------------------------------------------------------
constexpr uint32_t kM26 = 0x3ffffffu;

struct F26 {
  uint32_t v[5];
};

// radix 2^32 accumulator (h4 small) -> radix 2^26
__device__ __forceinline__ F26 f26_from32(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3, uint32_t h4) {
  F26 a;
  a.v[0] = h0 & kM26;
  a.v[1] = ((h0 >> 26) | (h1 << 6)) & kM26;
  a.v[2] = ((h1 >> 20) | (h2 << 12)) & kM26;
  a.v[3] = ((h2 >> 14) | (h3 << 18)) & kM26;
  a.v[4] = (h3 >> 8) | (h4 << 24);
  return a;
}

// a * b mod 2^130 - 5; result limbs < 2^26 (+ a small carry in limb 1)
__device__ __forceinline__ F26 f26_mul(const F26 &a, const F26 &b) {
  const uint32_t s1 = b.v[1] * 5u, s2 = b.v[2] * 5u, s3 = b.v[3] * 5u, s4 = b.v[4] * 5u;
  const uint64_t a0 = a.v[0], a1 = a.v[1], a2 = a.v[2], a3 = a.v[3], a4 = a.v[4];
  uint64_t d0 = a0 * b.v[0] + a1 * s4 + a2 * s3 + a3 * s2 + a4 * s1;
  uint64_t d1 = a0 * b.v[1] + a1 * b.v[0] + a2 * s4 + a3 * s3 + a4 * s2;
  uint64_t d2 = a0 * b.v[2] + a1 * b.v[1] + a2 * b.v[0] + a3 * s4 + a4 * s3;
  uint64_t d3 = a0 * b.v[3] + a1 * b.v[2] + a2 * b.v[1] + a3 * b.v[0] + a4 * s4;
  uint64_t d4 = a0 * b.v[4] + a1 * b.v[3] + a2 * b.v[2] + a3 * b.v[1] + a4 * b.v[0];
  F26 r;
  d1 += d0 >> 26;
  r.v[0] = (uint32_t)d0 & kM26;
  d2 += d1 >> 26;
  r.v[1] = (uint32_t)d1 & kM26;
  d3 += d2 >> 26;
  r.v[2] = (uint32_t)d2 & kM26;
  d4 += d3 >> 26;
  r.v[3] = (uint32_t)d3 & kM26;
  const uint64_t c = (d4 >> 26) * 5u + r.v[0];
  r.v[4] = (uint32_t)d4 & kM26;
  r.v[0] = (uint32_t)c & kM26;
  r.v[1] += (uint32_t)(c >> 26);
  return r;
}

__device__ __forceinline__ F26 f26_add(const F26 &a, const F26 &b) {
  F26 r;
#pragma unroll
  for (int q = 0; q < 5; ++q) r.v[q] = a.v[q] + b.v[q];
  return r;
}

// r^e, e >= 1 (square and multiply, MSB first)
__device__ __forceinline__ F26 f26_pow(const F26 &r, uint32_t e) {
  F26 x = r;
  for (int bit = 30 - __builtin_clz(e); bit >= 0; --bit) {
    x = f26_mul(x, x);
    if ((e >> bit) & 1u) x = f26_mul(x, r);
  }
  return x;
}

// radix 2^26 (limbs < 2^29) -> radix 2^32, the same value (no reduction): limb j
// sits at bit 26 j, so each 32-bit word collects its limbs' shifted parts plus the
// carry out of the word below; h4 < 2^5
__device__ __forceinline__ void f26_to32(const F26 &a, uint32_t &h0, uint32_t &h1, uint32_t &h2, uint32_t &h3,
                                         uint32_t &h4) {
  uint64_t t = (uint64_t)a.v[0] + ((uint64_t)a.v[1] << 26);
  h0 = (uint32_t)t;
  t = (t >> 32) + ((uint64_t)a.v[2] << 20);
  h1 = (uint32_t)t;
  t = (t >> 32) + ((uint64_t)a.v[3] << 14);
  h2 = (uint32_t)t;
  t = (t >> 32) + ((uint64_t)a.v[4] << 8);
  h3 = (uint32_t)t;
  h4 = (uint32_t)(t >> 32);
}

}  // namespace wg
