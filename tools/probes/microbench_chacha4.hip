// ChaCha20 issue-rate probe for gfx950, part 4: the rotate-by-16 step as two
// SDWA xors (word selects) instead of v_xor + v_alignbit.
//   t.hi = d.lo ^ a.lo  (dst_sel WORD_1, low half zeroed)
//   t.lo = d.hi ^ a.hi  (dst_sel WORD_0, high half preserved)   -> t = rotl(d ^ a, 16)
// SDWA ops are VOP2 encodings; the question is whether two waves' SDWA ops pair
// like v_xor (2 cycles per wave64 instruction) or cost 4 like v_alignbit.
// Same harness as microbench_chacha2 (phase-locked: s_barrier after every step,
// 512-thread workgroups, 2 per CU).
//   hipcc --offload-arch=gfx950 -O3 -I neptun_amd/csrc tools/microbench_chacha4.hip -o tools/microbench_chacha4
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "wg_crypto.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kPairs = 64;  // block pairs per lane

#define ADD8 \
  "v_add_u32 %0, %0, %16\n v_add_u32 %1, %1, %17\n v_add_u32 %2, %2, %18\n v_add_u32 %3, %3, %19\n" \
  "v_add_u32 %4, %4, %20\n v_add_u32 %5, %5, %21\n v_add_u32 %6, %6, %22\n v_add_u32 %7, %7, %23\n"
#define XOR8 \
  "v_xor_b32 %8, %8, %0\n v_xor_b32 %9, %9, %1\n v_xor_b32 %10, %10, %2\n v_xor_b32 %11, %11, %3\n" \
  "v_xor_b32 %12, %12, %4\n v_xor_b32 %13, %13, %5\n v_xor_b32 %14, %14, %6\n v_xor_b32 %15, %15, %7\n"
#define ROT8(SH) \
  "v_alignbit_b32 %8, %8, %8, " #SH "\n v_alignbit_b32 %9, %9, %9, " #SH "\n"                \
  "v_alignbit_b32 %10, %10, %10, " #SH "\n v_alignbit_b32 %11, %11, %11, " #SH "\n"          \
  "v_alignbit_b32 %12, %12, %12, " #SH "\n v_alignbit_b32 %13, %13, %13, " #SH "\n"          \
  "v_alignbit_b32 %14, %14, %14, " #SH "\n v_alignbit_b32 %15, %15, %15, " #SH "\n"
#define OPS : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), \
  "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)              \
  : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)

// SDWA rot16: outputs t0..t7 (%0..%7, early clobber), a (%8..%15, +v), d (%16..%23), b (%24..%31)
#define SX_HI(T, D, A) "v_xor_b32_sdwa %" #T ", %" #D ", %" #A " dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n"
#define SX_LO(T, D, A) "v_xor_b32_sdwa %" #T ", %" #D ", %" #A " dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n"
#define ADD8S \
  "v_add_u32 %8, %8, %24\n v_add_u32 %9, %9, %25\n v_add_u32 %10, %10, %26\n v_add_u32 %11, %11, %27\n" \
  "v_add_u32 %12, %12, %28\n v_add_u32 %13, %13, %29\n v_add_u32 %14, %14, %30\n v_add_u32 %15, %15, %31\n"
#define SDWA16 ADD8S \
  SX_HI(0, 16, 8) SX_HI(1, 17, 9) SX_HI(2, 18, 10) SX_HI(3, 19, 11)   \
  SX_HI(4, 20, 12) SX_HI(5, 21, 13) SX_HI(6, 22, 14) SX_HI(7, 23, 15) \
  SX_LO(0, 16, 8) SX_LO(1, 17, 9) SX_LO(2, 18, 10) SX_LO(3, 19, 11)   \
  SX_LO(4, 20, 12) SX_LO(5, 21, 13) SX_LO(6, 22, 14) SX_LO(7, 23, 15)
// v_perm_b32 rot16 (VOP3, for comparison)
#define PERM8 \
  "v_perm_b32 %8, %8, %8, %24\n v_perm_b32 %9, %9, %9, %24\n v_perm_b32 %10, %10, %10, %24\n v_perm_b32 %11, %11, %11, %24\n" \
  "v_perm_b32 %12, %12, %12, %24\n v_perm_b32 %13, %13, %13, %24\n v_perm_b32 %14, %14, %14, %24\n v_perm_b32 %15, %15, %15, %24\n"

// MODE 0: add8 xor8 alignbit8 for every step; 1: rot16 steps as SDWA pairs; 2: rot16 as v_perm
template <int SH, int MODE>
__device__ __forceinline__ void step(uint32_t &a0, uint32_t &a1, uint32_t &a2, uint32_t &a3,
                                     uint32_t &a4, uint32_t &a5, uint32_t &a6, uint32_t &a7,
                                     uint32_t &d0, uint32_t &d1, uint32_t &d2, uint32_t &d3,
                                     uint32_t &d4, uint32_t &d5, uint32_t &d6, uint32_t &d7,
                                     uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3,
                                     uint32_t b4, uint32_t b5, uint32_t b6, uint32_t b7) {
  if constexpr (SH == 16 && MODE == 1) {
    uint32_t t0, t1, t2, t3, t4, t5, t6, t7;
    asm volatile(SDWA16 "s_barrier\n"
                 : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "=&v"(t5), "=&v"(t6), "=&v"(t7),
                   "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(d0), "v"(d1), "v"(d2), "v"(d3), "v"(d4), "v"(d5), "v"(d6), "v"(d7),
                   "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7));
    d0 = t0; d1 = t1; d2 = t2; d3 = t3; d4 = t4; d5 = t5; d6 = t6; d7 = t7;
  } else if constexpr (SH == 16 && MODE == 2) {
    const uint32_t sel = 0x01000302u;  // bytes 1,0,3,2 -> rotl 16
    asm volatile(ADD8 XOR8
                 "v_perm_b32 %8, %8, %8, %24\n v_perm_b32 %9, %9, %9, %24\n v_perm_b32 %10, %10, %10, %24\n"
                 "v_perm_b32 %11, %11, %11, %24\n v_perm_b32 %12, %12, %12, %24\n v_perm_b32 %13, %13, %13, %24\n"
                 "v_perm_b32 %14, %14, %14, %24\n v_perm_b32 %15, %15, %15, %24\n s_barrier\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                   "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                 : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7), "s"(sel));
  } else if constexpr (SH == 16) {
    asm volatile(ADD8 XOR8 ROT8(16) "s_barrier\n" OPS);
  } else if constexpr (SH == 20) {
    asm volatile(ADD8 XOR8 ROT8(20) "s_barrier\n" OPS);
  } else if constexpr (SH == 24) {
    asm volatile(ADD8 XOR8 ROT8(24) "s_barrier\n" OPS);
  } else {
    asm volatile(ADD8 XOR8 ROT8(25) "s_barrier\n" OPS);
  }
}

#define Q8(A0, B0, C0, D0, A1, B1, C1, D1, A2, B2, C2, D2, A3, B3, C3, D3)                      \
  step<16, MODE>(x[0][A0], x[0][A1], x[0][A2], x[0][A3], x[1][A0], x[1][A1], x[1][A2], x[1][A3], \
             x[0][D0], x[0][D1], x[0][D2], x[0][D3], x[1][D0], x[1][D1], x[1][D2], x[1][D3],     \
             x[0][B0], x[0][B1], x[0][B2], x[0][B3], x[1][B0], x[1][B1], x[1][B2], x[1][B3]);    \
  step<20, MODE>(x[0][C0], x[0][C1], x[0][C2], x[0][C3], x[1][C0], x[1][C1], x[1][C2], x[1][C3], \
             x[0][B0], x[0][B1], x[0][B2], x[0][B3], x[1][B0], x[1][B1], x[1][B2], x[1][B3],     \
             x[0][D0], x[0][D1], x[0][D2], x[0][D3], x[1][D0], x[1][D1], x[1][D2], x[1][D3]);    \
  step<24, MODE>(x[0][A0], x[0][A1], x[0][A2], x[0][A3], x[1][A0], x[1][A1], x[1][A2], x[1][A3], \
            x[0][D0], x[0][D1], x[0][D2], x[0][D3], x[1][D0], x[1][D1], x[1][D2], x[1][D3],      \
            x[0][B0], x[0][B1], x[0][B2], x[0][B3], x[1][B0], x[1][B1], x[1][B2], x[1][B3]);     \
  step<25, MODE>(x[0][C0], x[0][C1], x[0][C2], x[0][C3], x[1][C0], x[1][C1], x[1][C2], x[1][C3], \
            x[0][B0], x[0][B1], x[0][B2], x[0][B3], x[1][B0], x[1][B1], x[1][B2], x[1][B3],      \
            x[0][D0], x[0][D1], x[0][D2], x[0][D3], x[1][D0], x[1][D1], x[1][D2], x[1][D3]);

template <int MODE>
__device__ __forceinline__ void chacha2(uint32_t (&x)[2][16]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    Q8(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15)
    Q8(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14)
  }
}

template <int MODE>
__global__ __launch_bounds__(512) void k_asm(uint32_t* out, const uint32_t* keys) {
  uint32_t key[8];
  for (int i = 0; i < 8; ++i) key[i] = keys[i];
  uint32_t acc = 0;
  const uint32_t n1 = blockIdx.x * 512 + threadIdx.x;
  for (int b = 0; b < kPairs; ++b) {
    uint32_t x[2][16];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      x[j][0] = wg::kSigma0; x[j][1] = wg::kSigma1; x[j][2] = wg::kSigma2; x[j][3] = wg::kSigma3;
#pragma unroll
      for (int i = 0; i < 8; ++i) x[j][4 + i] = key[i];
      x[j][12] = 2 * b + j; x[j][13] = 0; x[j][14] = n1; x[j][15] = 0;
    }
    chacha2<MODE>(x);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc ^= x[j][i] + (i < 4 ? 0u : i < 12 ? key[i - 4] : 0u);
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc;
}

typedef void (*kfn)(uint32_t*, const uint32_t*);

int main(int argc, char** argv) {
  const int reps = 10;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device CUs %d\n", cus);
  uint32_t *out, *keys;
  const int threads_total = cus * 4 * 4 * 64 * 8;
  CHECK(hipMalloc(&out, threads_total * 4 * 3));
  CHECK(hipMalloc(&keys, 64));
  CHECK(hipMemset(keys, 0x5a, 64));
  const int lds = 64 << 10;  // 2 workgroups per CU, as the product
  kfn fs[3] = {k_asm<0>, k_asm<1>, k_asm<2>};
  const char* names[3] = {"xor + alignbit (product)", "rot16 as 2 SDWA xors", "rot16 as v_perm"};
  for (auto f : fs) CHECK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int blocks = threads_total / 512;
  for (int pass = 0; pass < 2; ++pass)
    for (int m = 0; m < 3; ++m) {
      for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(fs[m], dim3(blocks), dim3(512), lds, 0, out + m * threads_total, keys);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(fs[m], dim3(blocks), dim3(512), lds, 0, out + m * threads_total, keys);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      const double blocks_total = (double)threads_total * 2 * kPairs;
      const double per_simd = blocks_total / 64.0 / (cus * 4);
      printf("pass %d %-28s %7.3f ms  %7.1f SIMD-cycles per wave-block @2.4GHz\n", pass, names[m], ms,
             ms * 1e-3 * 2.4e9 / per_simd);
    }
  // all three must compute the same keystream
  uint32_t* h = new uint32_t[threads_total * 3];
  CHECK(hipMemcpy(h, out, threads_total * 4 * 3, hipMemcpyDeviceToHost));
  printf("outputs %s\n", memcmp(h, h + threads_total, threads_total * 4) == 0 &&
                                 memcmp(h, h + 2 * threads_total, threads_total * 4) == 0 ? "identical" : "DIFFER");
  return 0;
}
