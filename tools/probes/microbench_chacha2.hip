// ChaCha20 issue-rate probe for gfx950, part 2: two keystream blocks per lane
// with the 8 quarter-rounds of a step issued as 8 adds, 8 xors, 8 rotates
// (inline asm, so the grouping is exact), and an s_barrier every BAR steps to
// keep the waves that share a SIMD in phase (tools/microbench_valu6.hip: that
// took an add8/xor8/rot8 stream from 3.96 to 2.4-2.8 cycles per instruction).
//   hipcc --offload-arch=gfx950 -O3 -I neptun_amd/csrc tools/microbench_chacha2.hip -o tools/microbench_chacha2
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <cstdio>

#include "wg_crypto.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kPairs = 64;  // block pairs per lane

// one step of 8 quarter-rounds: a += b; d ^= a; d = rotl(d, n)
#define STEP_ASM(SH)                                                                        \
  "v_add_u32 %0, %0, %16\n v_add_u32 %1, %1, %17\n v_add_u32 %2, %2, %18\n v_add_u32 %3, %3, %19\n" \
  "v_add_u32 %4, %4, %20\n v_add_u32 %5, %5, %21\n v_add_u32 %6, %6, %22\n v_add_u32 %7, %7, %23\n" \
  "v_xor_b32 %8, %8, %0\n v_xor_b32 %9, %9, %1\n v_xor_b32 %10, %10, %2\n v_xor_b32 %11, %11, %3\n" \
  "v_xor_b32 %12, %12, %4\n v_xor_b32 %13, %13, %5\n v_xor_b32 %14, %14, %6\n v_xor_b32 %15, %15, %7\n" \
  "v_alignbit_b32 %8, %8, %8, " #SH "\n v_alignbit_b32 %9, %9, %9, " #SH "\n"                          \
  "v_alignbit_b32 %10, %10, %10, " #SH "\n v_alignbit_b32 %11, %11, %11, " #SH "\n"                    \
  "v_alignbit_b32 %12, %12, %12, " #SH "\n v_alignbit_b32 %13, %13, %13, " #SH "\n"                    \
  "v_alignbit_b32 %14, %14, %14, " #SH "\n v_alignbit_b32 %15, %15, %15, " #SH "\n"

template <int BAR>
__device__ __forceinline__ void bar(int step) {
  if (BAR > 0 && (step % BAR) == BAR - 1) __builtin_amdgcn_s_barrier();
}

// 8 QRs (2 blocks x 4 columns or diagonals); x[blk][16]
#define Q8(A0, B0, C0, D0, A1, B1, C1, D1, A2, B2, C2, D2, A3, B3, C3, D3)                      \
  step<SH16, MODE>(x[0][A0], x[0][A1], x[0][A2], x[0][A3], x[1][A0], x[1][A1], x[1][A2], x[1][A3],     \
             x[0][D0], x[0][D1], x[0][D2], x[0][D3], x[1][D0], x[1][D1], x[1][D2], x[1][D3],     \
             x[0][B0], x[0][B1], x[0][B2], x[0][B3], x[1][B0], x[1][B1], x[1][B2], x[1][B3]);    \
  bar<BAR>(s++);                                                                                  \
  step<SH12, MODE>(x[0][C0], x[0][C1], x[0][C2], x[0][C3], x[1][C0], x[1][C1], x[1][C2], x[1][C3],     \
             x[0][B0], x[0][B1], x[0][B2], x[0][B3], x[1][B0], x[1][B1], x[1][B2], x[1][B3],     \
             x[0][D0], x[0][D1], x[0][D2], x[0][D3], x[1][D0], x[1][D1], x[1][D2], x[1][D3]);    \
  bar<BAR>(s++);                                                                                  \
  step<SH8, MODE>(x[0][A0], x[0][A1], x[0][A2], x[0][A3], x[1][A0], x[1][A1], x[1][A2], x[1][A3],      \
            x[0][D0], x[0][D1], x[0][D2], x[0][D3], x[1][D0], x[1][D1], x[1][D2], x[1][D3],      \
            x[0][B0], x[0][B1], x[0][B2], x[0][B3], x[1][B0], x[1][B1], x[1][B2], x[1][B3]);     \
  bar<BAR>(s++);                                                                                  \
  step<SH7, MODE>(x[0][C0], x[0][C1], x[0][C2], x[0][C3], x[1][C0], x[1][C1], x[1][C2], x[1][C3],      \
            x[0][B0], x[0][B1], x[0][B2], x[0][B3], x[1][B0], x[1][B1], x[1][B2], x[1][B3],      \
            x[0][D0], x[0][D1], x[0][D2], x[0][D3], x[1][D0], x[1][D1], x[1][D2], x[1][D3]);     \
  bar<BAR>(s++);

enum { SH16 = 16, SH12 = 20, SH8 = 24, SH7 = 25 };  // alignbit shift = 32 - rotl amount

// MODE 0: add8 xor8 rot8; 1: add8 xor8 s_barrier rot8; 2: (add xor rot) x 8
#define STEP_H(SH)                                                                          \
  "v_add_u32 %0, %0, %16\n v_add_u32 %1, %1, %17\n v_add_u32 %2, %2, %18\n v_add_u32 %3, %3, %19\n" \
  "v_add_u32 %4, %4, %20\n v_add_u32 %5, %5, %21\n v_add_u32 %6, %6, %22\n v_add_u32 %7, %7, %23\n" \
  "v_xor_b32 %8, %8, %0\n v_xor_b32 %9, %9, %1\n v_xor_b32 %10, %10, %2\n v_xor_b32 %11, %11, %3\n" \
  "v_xor_b32 %12, %12, %4\n v_xor_b32 %13, %13, %5\n v_xor_b32 %14, %14, %6\n v_xor_b32 %15, %15, %7\n" \
  "s_barrier\n"                                                                              \
  "v_alignbit_b32 %8, %8, %8, " #SH "\n v_alignbit_b32 %9, %9, %9, " #SH "\n"                \
  "v_alignbit_b32 %10, %10, %10, " #SH "\n v_alignbit_b32 %11, %11, %11, " #SH "\n"          \
  "v_alignbit_b32 %12, %12, %12, " #SH "\n v_alignbit_b32 %13, %13, %13, " #SH "\n"          \
  "v_alignbit_b32 %14, %14, %14, " #SH "\n v_alignbit_b32 %15, %15, %15, " #SH "\n"
#define AXR(A, D, B, SH) "v_add_u32 %" #A ", %" #A ", %" #B "\n v_xor_b32 %" #D ", %" #D ", %" #A "\n v_alignbit_b32 %" #D ", %" #D ", %" #D ", " #SH "\n"
#define STEP_I(SH) AXR(0, 8, 16, SH) AXR(1, 9, 17, SH) AXR(2, 10, 18, SH) AXR(3, 11, 19, SH) \
                   AXR(4, 12, 20, SH) AXR(5, 13, 21, SH) AXR(6, 14, 22, SH) AXR(7, 15, 23, SH)
#define OPS : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), \
  "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)              \
  : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)
#define STEP4(M)                                                                  \
  if constexpr (SH == SH16) asm volatile(M(16) OPS);                              \
  else if constexpr (SH == SH12) asm volatile(M(20) OPS);                         \
  else if constexpr (SH == SH8) asm volatile(M(24) OPS);                          \
  else asm volatile(M(25) OPS);

template <int SH, int MODE>
__device__ __forceinline__ void step(uint32_t &a0, uint32_t &a1, uint32_t &a2, uint32_t &a3,
                                     uint32_t &a4, uint32_t &a5, uint32_t &a6, uint32_t &a7,
                                     uint32_t &d0, uint32_t &d1, uint32_t &d2, uint32_t &d3,
                                     uint32_t &d4, uint32_t &d5, uint32_t &d6, uint32_t &d7,
                                     uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3,
                                     uint32_t b4, uint32_t b5, uint32_t b6, uint32_t b7) {
  if constexpr (MODE == 0) { STEP4(STEP_ASM) }
  else if constexpr (MODE == 1) { STEP4(STEP_H) }
  else { STEP4(STEP_I) }
}

// in the step: "a" operand = first arg group (updated by +=), "d" = xor/rot target,
// "b" = addend.  For a QR (a,b,c,d): step1 a+=b, d^=a, d<<<16 -> step(a, d, b)
// step2 c+=d, b^=c, b<<<12 -> step(c, b, d), etc.
template <int BAR, int MODE>
__device__ __forceinline__ void chacha2(uint32_t (&x)[2][16]) {
  int s = 0;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    Q8(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15)
    Q8(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14)
  }
}

template <int BAR, int WG, int MODE = 0>
__global__ __launch_bounds__(WG) void k_asm(uint32_t* out, const uint32_t* keys) {
  uint32_t key[8];
  for (int i = 0; i < 8; ++i) key[i] = keys[i];  // uniform key (SGPRs)
  uint32_t acc = 0;
  const uint32_t n1 = blockIdx.x * WG + threadIdx.x;
  for (int b = 0; b < kPairs; ++b) {
    uint32_t x[2][16];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      x[j][0] = wg::kSigma0; x[j][1] = wg::kSigma1; x[j][2] = wg::kSigma2; x[j][3] = wg::kSigma3;
#pragma unroll
      for (int i = 0; i < 8; ++i) x[j][4 + i] = key[i];
      x[j][12] = 2 * b + j; x[j][13] = 0; x[j][14] = n1; x[j][15] = 0;
    }
    chacha2<BAR, MODE>(x);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc ^= x[j][i] + (i < 4 ? 0u : i < 12 ? key[i - 4] : 0u);
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

// reference: the compiled chacha20_block of the product, 2 blocks per iteration
template <int WG>
__global__ __launch_bounds__(WG) void k_c(uint32_t* out, const uint32_t* keys) {
  uint32_t key[8];
  for (int i = 0; i < 8; ++i) key[i] = keys[i];
  uint32_t acc = 0;
  const uint32_t n1 = blockIdx.x * WG + threadIdx.x;
  for (int b = 0; b < 2 * kPairs; ++b) {
    uint32_t ks[16];
    wg::chacha20_block(ks, key, (uint32_t)b, n1, 0u);
#pragma unroll
    for (int j = 0; j < 16; ++j) acc ^= ks[j];
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

typedef void (*kfn)(uint32_t*, const uint32_t*);

int main(int argc, char** argv) {
  const bool sustained = argc > 1;
  const int reps = sustained ? 10 : 1;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device CUs %d clock %d kHz\n", cus, prop.clockRate);
  uint32_t *out, *keys;
  CHECK(hipMalloc(&out, 256 << 20));
  CHECK(hipMalloc(&keys, 64));
  CHECK(hipMemset(keys, 0x5a, 64));
  for (auto f : {k_asm<1, 1024>, k_asm<1, 512>, k_asm<1, 768>, k_asm<0, 1024>, k_c<256>})
    CHECK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  struct { const char* name; kfn f; int wg; int lds = 0; } ks[] = {
    {"compiled chacha20_block    wg256", k_c<256>, 256},
    {"compiled chacha20_block    wg1024", k_c<1024>, 1024},
    {"asm 8-QR steps, no barrier wg256", k_asm<0, 256>, 256},
    {"asm 8-QR steps, no barrier wg1024", k_asm<0, 1024>, 1024},
    {"asm, barrier/step          wg256", k_asm<1, 256>, 256},
    {"asm, barrier/step          wg512", k_asm<1, 512>, 512},
    {"asm, barrier/step          wg1024", k_asm<1, 1024>, 1024},
    {"asm, barrier/2 steps       wg1024", k_asm<2, 1024>, 1024},
    {"asm, barrier/step          wg768", k_asm<1, 768>, 768},
    {"asm interleaved QRs, bar   wg1024", k_asm<1, 1024, 2>, 1024},
    {"asm, barrier/half-step     wg1024", k_asm<1, 1024, 1>, 1024},
    {"asm, barrier/4 steps       wg1024", k_asm<4, 1024>, 1024},
    {"asm, barrier/8 steps       wg1024", k_asm<8, 1024>, 1024},
    {"asm, bar/step wg1024 1 WG/CU (LDS)", k_asm<1, 1024>, 1024, 96 << 10},
    {"asm, bar/step wg512 2 WG/CU (LDS)", k_asm<1, 512>, 512, 64 << 10},
    {"asm, bar/step wg768 1 WG/CU (LDS)", k_asm<1, 768>, 768, 96 << 10},
    {"asm, no bar wg1024 1 WG/CU (LDS)", k_asm<0, 1024>, 1024, 96 << 10},
    {"compiled wg256 4 WG/CU (LDS)", k_c<256>, 256, 36 << 10},
  };
  // `microbench_chacha2 only IDX SECONDS`: one variant back to back for ~SECONDS
  // (tools/power_probe.py: energy per block of the phase-locked vs the
  // compiler-scheduled keystream)
  if (argc > 3 && !strcmp(argv[1], "only")) {
    auto& k = ks[atoi(argv[2])];
    const int threads_total = cus * 4 * 4 * 64 * 8;
    const int blocks = threads_total / k.wg;
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(k.wg), k.lds, 0, out, keys);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(k.wg), k.lds, 0, out, keys);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms1;
    CHECK(hipEventElapsedTime(&ms1, e0, e1));
    const int n = (int)(atof(argv[3]) * 1e3 / ms1) + 1;
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(k.wg), k.lds, 0, out, keys);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double blocks_total = (double)threads_total * 2 * kPairs * n;
    printf("{\"variant\": \"%s\", \"seconds\": %.3f, \"wave_blocks_per_s\": %.4e}\n", k.name,
           ms * 1e-3, blocks_total / 64.0 / (ms * 1e-3));
    return 0;
  }
  // total waves = 4 waves/SIMD resident x 8 rounds; per wave 2*kPairs blocks
  for (auto& k : ks) {
    for (int wps : {4}) {
      const int threads_total = cus * 4 * wps * 64 * 8;
      const int blocks = threads_total / k.wg;
      // sustained: ~40 launches of warm-up (DVFS settles), then time 10
      for (int i = 0; i < (sustained ? 40 : 1); ++i)
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(k.wg), k.lds, 0, out, keys);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(k.wg), k.lds, 0, out, keys);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      const double blocks_total = (double)threads_total * 2 * kPairs;
      const double per_simd = blocks_total / 64.0 / (cus * 4);  // wave-blocks per SIMD
      printf("%-36s grid waves/SIMD %2d x8: %7.3f ms  %7.1f SIMD-cycles per wave-block @2.4GHz  %6.1f Gblk/s\n",
             k.name, wps, ms, ms * 1e-3 * 2.4e9 / per_simd, blocks_total / (ms * 1e-3) * 1e-9);
    }
  }
  return 0;
}
