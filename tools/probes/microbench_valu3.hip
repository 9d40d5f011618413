// VALU co-issue probe for gfx950, part 3: does the 2-cycle rate of simple ops
// need the waves sharing a SIMD to run the same instruction stream in step?
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_valu3.hip -o tools/microbench_valu3
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 2048
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define BODY8(OP) OP OP OP OP OP OP OP OP
#define OP8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define ADD(k) "v_add_u32 %" #k ", %" #k ", %8\n"
#define XOR(k) "v_xor_b32 %" #k ", %" #k ", %9\n"
#define OR(k) "v_or_b32 %" #k ", %" #k ", %9\n"
#define SHL(k) "v_lshlrev_b32 %" #k ", 3, %" #k "\n"
#define SHL12(k) "v_lshlrev_b32 %" #k ", 12, %" #k "\n"
#define SHR(k) "v_lshrrev_b32 %" #k ", 7, %" #k "\n"
#define ROT(k) "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 20\n"
#define ROT1 "v_alignbit_b32 %0, %0, %0, 20\n"
// rotate via shifts: t = x >> 20 (into b? no: scratch c), x = x << 12, x |= t
#define SROT(k) "v_lshrrev_b32 %9, 20, %" #k "\n" "v_lshlrev_b32 %" #k ", 12, %" #k "\n" "v_or_b32 %" #k ", %" #k ", %9\n"

#define REGS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define PROLOG                                                                  \
  uint32_t a0 = seed + threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3;      \
  uint32_t a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;                  \
  uint32_t b = seed * 3 + 1, c = seed * 7 + 5;                                  \
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#define EPILOG out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ c;
#define LOOP(ASM) for (int i = 0; i < ITERS; ++i) asm volatile(BODY8(ASM) : REGS : "v"(b), "v"(c));
#define LOOPC(ASM) for (int i = 0; i < ITERS; ++i) asm volatile(BODY8(ASM) : REGS, "+v"(c) : "v"(b));
#define STAGGER if (stagger) for (uint32_t s = 0; s < wave; ++s) __builtin_amdgcn_s_sleep(7);

#define KERN(NAME, ASM) __global__ void NAME(uint32_t* out, uint32_t seed, int stagger) { PROLOG STAGGER LOOP(ASM) EPILOG }
#define KERNC(NAME, ASM) __global__ void NAME(uint32_t* out, uint32_t seed, int stagger) { PROLOG STAGGER LOOPC(ASM) EPILOG }
KERN(k_add, OP8(ADD))
KERN(k_or, OP8(OR))
KERN(k_shl3, OP8(SHL))
KERN(k_shl12, OP8(SHL12))
KERN(k_shr, OP8(SHR))
KERN(k_64s_1r, OP8(ADD) OP8(XOR) OP8(ADD) OP8(XOR) OP8(ADD) OP8(XOR) OP8(ADD) OP8(XOR) ROT1)
KERN(k_axr, OP8(ADD) OP8(XOR) OP8(ROT))
KERNC(k_ax_srot, OP8(ADD) OP8(XOR) OP8(SROT))
// waves alternate roles: even waves pure add, odd waves pure xor (different PCs)
__global__ void k_add_or_xor(uint32_t* out, uint32_t seed, int stagger) {
  PROLOG STAGGER
  if (wave & 1) { LOOP(OP8(XOR)) } else { LOOP(OP8(ADD)) }
  EPILOG
}
__global__ void k_add_or_rot(uint32_t* out, uint32_t seed, int stagger) {
  PROLOG STAGGER
  if (wave & 1) { LOOP(OP8(ROT)) } else { LOOP(OP8(ADD)) }
  EPILOG
}

typedef void (*kfn)(uint32_t*, uint32_t, int);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device CUs %d clock %d kHz\n", cus, prop.clockRate);
  struct { const char* name; kfn f; double per_asm; } ks[] = {
    {"add", k_add, 8}, {"or", k_or, 8}, {"lshlrev 3", k_shl3, 8}, {"lshlrev 12", k_shl12, 8},
    {"lshrrev 7", k_shr, 8}, {"64 simple + 1 rot", k_64s_1r, 65}, {"add8 xor8 rot8", k_axr, 24},
    {"add8 xor8 shiftrot8 (5 ops)", k_ax_srot, 40},
    {"waves: add | xor", k_add_or_xor, 8}, {"waves: add | rot", k_add_or_rot, 8},
  };
  // 1024-thread blocks: 16 waves, 4 per SIMD; wave w sits on SIMD w % 4 (so waves
  // w and w + 4 share a SIMD and have opposite parity only if ... see 'odd4' below)
  for (int threads : {256, 512, 1024}) {
    for (int stagger : {0, 1}) {
      const int blocks = cus * 2;
      uint32_t* out;
      CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0));
      CHECK(hipEventCreate(&e1));
      for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1u, stagger);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, (uint32_t)r, stagger);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double wps = 2.0 * threads / 256;  // waves per SIMD
        const double instr = wps * 3 * ITERS * 8 * k.per_asm;
        printf("thr=%4d wps=%g stagger=%d %-32s %8.3f ms  %5.2f SIMD-cycles/wave-instr\n", threads,
               wps, stagger, k.name, ms, ms * 1e-3 * 2.4e9 / instr);
      }
      CHECK(hipFree(out));
    }
  }
  return 0;
}
