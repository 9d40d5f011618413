// VALU co-issue probe for gfx950, part 5: is the 2-cycle rate a property of
// the wave (lost for good once it issues a "slow" opcode) or of the stream?
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_valu5.hip -o tools/microbench_valu5
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 1024
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define BODY8(OP) OP OP OP OP OP OP OP OP
#define OP8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define REGS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define ADD(k) "v_add_u32 %" #k ", %" #k ", %8\n"
#define XOR(k) "v_xor_b32 %" #k ", %" #k ", %9\n"
#define FAST16 OP8(ADD) OP8(XOR)
#define PRE(ASM) asm volatile(ASM : REGS : "v"(b), "v"(c));
#define KERN(NAME, BEFORE, AFTER)                                               \
__global__ void NAME(uint32_t* out, uint32_t seed) {                            \
  uint32_t a0 = seed + threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3;      \
  uint32_t a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;                  \
  uint32_t b = seed * 3 + 1, c = seed * 7 + 5;                                  \
  BEFORE                                                                        \
  for (int i = 0; i < ITERS; ++i) asm volatile(BODY8(FAST16) : REGS : "v"(b), "v"(c)); \
  AFTER                                                                         \
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
}
KERN(k_plain, , )
KERN(k_rot_first, PRE("v_alignbit_b32 %0, %0, %0, 20\n"), )
KERN(k_rot_last, , PRE("v_alignbit_b32 %0, %0, %0, 20\n"))
KERN(k_shl_first, PRE("v_lshlrev_b32 %0, 3, %0\n"), )
KERN(k_mul_first, PRE("v_mul_lo_u32 %0, %0, %8\n"), )
KERN(k_rot_first_nop, PRE("v_alignbit_b32 %0, %0, %0, 20\ns_nop 7\ns_nop 7\n"), )

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  struct { const char* name; kfn f; } ks[] = {
    {"fast loop", k_plain}, {"1 alignbit, then fast loop", k_rot_first},
    {"fast loop, then 1 alignbit", k_rot_last}, {"1 lshlrev, then fast loop", k_shl_first},
    {"1 mul_lo, then fast loop", k_mul_first}, {"1 alignbit + s_nops, then fast loop", k_rot_first_nop},
  };
  for (int threads : {512, 1024}) {
    const int blocks = cus * 2;
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
      const double wps = 2.0 * threads / 256;
      const double instr = wps * 3 * ITERS * 8 * 16;
      printf("wps=%g %-38s %8.3f ms  %5.2f SIMD-cycles/wave-instr\n", wps, k.name, ms,
             ms * 1e-3 * 2.4e9 / instr);
    }
    CHECK(hipFree(out));
  }
  return 0;
}
