// VALU issue-model follow-up for gfx950: why does one rotate poison a stream
// of full-rate adds/xors?  Each kernel runs 8 independent chains per lane;
// reported = SIMD cycles per wave-instruction at 2.4 GHz (lower is better).
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_valu2.hip -o tools/microbench_valu2
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 2048
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define BODY8(OP) OP OP OP OP OP OP OP OP

#define KERN(NAME, ASM)                                                         \
__global__ void NAME(uint32_t* out, uint32_t seed) {                            \
  uint32_t a0 = seed + threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3;      \
  uint32_t a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;                  \
  uint32_t b = seed * 3 + 1, c = seed * 7 + 5;                                  \
  for (int i = 0; i < ITERS; ++i) {                                             \
    asm volatile(BODY8(ASM) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3),          \
                 "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));     \
  }                                                                             \
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
}
#define OP8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define ADD(k) "v_add_u32 %" #k ", %" #k ", %8\n"
#define ADDE64(k) "v_add_u32_e64 %" #k ", %" #k ", %8\n"
#define XOR(k) "v_xor_b32 %" #k ", %" #k ", %9\n"
#define XORE64(k) "v_xor_b32_e64 %" #k ", %" #k ", %9\n"
#define ROT(k) "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 20\n"
#define ROTB(k) "v_alignbit_b32 %" #k ", %" #k ", %8, 20\n"
#define SHR(k) "v_lshrrev_b32 %" #k ", 7, %" #k "\n"
#define LSHLOR(k) "v_lshl_or_b32 %" #k ", %" #k ", 7, %9\n"
#define BITOP3(k) "v_bitop3_b32 %" #k ", %" #k ", %8, %9 bitop3:0x96\n"
#define ROT1(k) "v_alignbit_b32 %0, %0, %0, 20\n"

KERN(k_add, OP8(ADD))
KERN(k_add_e64, OP8(ADDE64))
KERN(k_xor_e64, OP8(XORE64))
KERN(k_ax_e64, OP8(ADDE64) OP8(XORE64))
KERN(k_rot, OP8(ROT))
KERN(k_rotb, OP8(ROTB))
KERN(k_shr, OP8(SHR))
KERN(k_64s_1r, OP8(ADD) OP8(XOR) OP8(ADD) OP8(XOR) OP8(ADD) OP8(XOR) OP8(ADD) OP8(XOR) ROT1(0))
KERN(k_16s_1r, OP8(ADD) OP8(XOR) ROT1(0))
KERN(k_ax_bitop3, OP8(ADD) OP8(BITOP3))
KERN(k_ax_shr, OP8(ADD) OP8(XOR) OP8(SHR))
KERN(k_ax_lshlor, OP8(ADD) OP8(XOR) OP8(LSHLOR))
KERN(k_axr, OP8(ADD) OP8(XOR) OP8(ROT))
// one ChaCha-like column step: 4 adds, 4 xors, 4 rotates on 4 independent QRs x 2
KERN(k_qr_sw, OP8(ADD) OP8(XOR) OP8(ROT) OP8(ADD) OP8(XOR) OP8(ROT))

// half the waves run pure adds, the other half pure rotates (same SIMDs)
__global__ void k_split(uint32_t* out, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3;
  uint32_t a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;
  uint32_t b = seed * 3 + 1, c = seed * 7 + 5;
  if (blockIdx.x & 1) {
    for (int i = 0; i < ITERS; ++i)
      asm volatile(BODY8(OP8(ROT)) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
  } else {
    for (int i = 0; i < 2 * ITERS; ++i)
      asm volatile(BODY8(OP8(ADD)) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device CUs %d clock %d kHz\n", cus, prop.clockRate);
  struct { const char* name; kfn f; double per_asm; } ks[] = {
    {"add", k_add, 8}, {"add_e64", k_add_e64, 8}, {"xor_e64", k_xor_e64, 8},
    {"add_e64+xor_e64", k_ax_e64, 16}, {"alignbit x,x,x", k_rot, 8}, {"alignbit x,b,x", k_rotb, 8},
    {"lshrrev", k_shr, 8}, {"64 simple + 1 rot", k_64s_1r, 65}, {"16 simple + 1 rot", k_16s_1r, 17},
    {"add8 bitop3_8", k_ax_bitop3, 16}, {"add8 xor8 shr8", k_ax_shr, 24},
    {"add8 xor8 lshl_or8", k_ax_lshlor, 24}, {"add8 xor8 rot8", k_axr, 24},
    {"qr-shaped (a x r a x r)", k_qr_sw, 48},
    {"split: add waves | rot waves (2x adds)", k_split, 8 * 1.5},
  };
  const int threads = 256;
  for (int wps : {1, 4, 8}) {
    const int blocks = cus * wps;
    uint32_t* out;
    CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1u);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, (uint32_t)r);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      // wave-instructions per SIMD (split kernel: average of its two halves' counts)
      const double instr = (double)wps * 3 * ITERS * 8 * k.per_asm;
      const double cyc = ms * 1e-3 * 2.4e9 / instr;
      printf("wps=%d %-40s %8.3f ms  %5.2f SIMD-cycles/wave-instr\n", wps, k.name, ms, cyc);
    }
    CHECK(hipFree(out));
  }
  return 0;
}
