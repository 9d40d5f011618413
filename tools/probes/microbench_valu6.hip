// VALU co-issue probe for gfx950, part 6: which waves pair for the 2-cycle
// rate?  Earlier probes split roles by wave parity, but waves w and w+4 share a
// SIMD, so both halves of a SIMD ran the same code.  Here roles are chosen from
// the hardware wave slot (HW_REG_HW_ID) so that waves sharing a SIMD really run
// different code, and the wave -> SIMD map is printed.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_valu6.hip -o tools/microbench_valu6
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 2048
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define BODY8(OP) OP OP OP OP OP OP OP OP
#define OP8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define ADD(k) "v_add_u32 %" #k ", %" #k ", %8\n"
#define ADDC(k) "v_add_u32 %" #k ", %8, %" #k "\n"   /* same op, commuted encoding */
#define XOR(k) "v_xor_b32 %" #k ", %" #k ", %9\n"
#define ROT(k) "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 20\n"
#define REGS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define PROLOG                                                                  \
  uint32_t a0 = seed + threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3;      \
  uint32_t a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;                  \
  uint32_t b = seed * 3 + 1, c = seed * 7 + 5;                                  \
  const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);              \
  const uint32_t slot = hwid & 15; (void)slot;                                  \
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); (void)wave;
#define EPILOG out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ c;
#define LOOP(ASM) for (int i = 0; i < ITERS; ++i) asm volatile(BODY8(ASM) : REGS : "v"(b), "v"(c));

__global__ void k_map(uint32_t* out, uint32_t) {
  const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = hwid;
}
// same code in every wave
__global__ void k_same(uint32_t* out, uint32_t seed) { PROLOG LOOP(OP8(ADD)) EPILOG }
// two copies of the add loop (different PCs), chosen by the hardware wave slot
__global__ void k_pc_by_slot(uint32_t* out, uint32_t seed) {
  PROLOG
  if (slot & 1) { LOOP(OP8(ADDC)) } else { LOOP(OP8(ADD)) }
  EPILOG
}
// two copies chosen by wave index bit 2 (waves w, w+4 differ if SIMD = w % 4)
__global__ void k_pc_by_w4(uint32_t* out, uint32_t seed) {
  PROLOG
  if (wave & 4) { LOOP(OP8(ADDC)) } else { LOOP(OP8(ADD)) }
  EPILOG
}
// roles by bit 2: add waves | rot waves on one SIMD
__global__ void k_add_rot_w4(uint32_t* out, uint32_t seed) {
  PROLOG
  if (wave & 4) { LOOP(OP8(ROT)) } else { LOOP(OP8(ADD)) }
  EPILOG
}
// roles by bit 2: (add,xor) waves | rot waves, 2:1 instruction ratio
__global__ void k_ax_rot_w4(uint32_t* out, uint32_t seed) {
  PROLOG
  if (wave & 4) { LOOP(OP8(ROT)) } else { LOOP(OP8(ADD) OP8(XOR)) }
  EPILOG
}
// one wave stream: add8 xor8 rot8 (ChaCha step shape)
__global__ void k_axr(uint32_t* out, uint32_t seed) { PROLOG LOOP(OP8(ADD) OP8(XOR) OP8(ROT)) EPILOG }
// same, a barrier after each 24-instruction group (re-aligns the waves' PCs)
__global__ void k_axr_bar(uint32_t* out, uint32_t seed) {
  PROLOG LOOP(OP8(ADD) OP8(XOR) OP8(ROT) "s_barrier\n") EPILOG
}
// same, barrier every 3 groups
__global__ void k_axr_bar3(uint32_t* out, uint32_t seed) {
  PROLOG
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(OP8(ADD) OP8(XOR) OP8(ROT) OP8(ADD) OP8(XOR) OP8(ROT) OP8(ADD) OP8(XOR) OP8(ROT) "s_barrier\n"
                 OP8(ADD) OP8(XOR) OP8(ROT) OP8(ADD) OP8(XOR) OP8(ROT) OP8(ADD) OP8(XOR) OP8(ROT) "s_barrier\n"
                 OP8(ADD) OP8(XOR) OP8(ROT) OP8(ADD) OP8(XOR) OP8(ROT) "s_barrier\n" : REGS : "v"(b), "v"(c));
  }
  EPILOG
}
// pure rot stream with a barrier each body (barrier cost reference)
__global__ void k_add_bar(uint32_t* out, uint32_t seed) { PROLOG LOOP(OP8(ADD) OP8(XOR) OP8(ADD) "s_barrier\n") EPILOG }

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device CUs %d clock %d kHz\n", cus, prop.clockRate);
  {
    uint32_t* m;
    CHECK(hipMalloc(&m, 64 * 16 * 4));
    hipLaunchKernelGGL(k_map, dim3(4), dim3(1024), 0, 0, m, 0u);
    uint32_t h[64];
    CHECK(hipMemcpy(h, m, sizeof(h), hipMemcpyDeviceToHost));
    for (int blk = 0; blk < 2; ++blk) {
      printf("block %d wave -> (simd, slot, cu):", blk);
      for (int w = 0; w < 16; ++w) {
        uint32_t v = h[blk * 16 + w];
        printf(" %d:(%u,%u,%u)", w, (v >> 4) & 3, v & 15, (v >> 8) & 15);
      }
      printf("\n");
    }
    CHECK(hipFree(m));
  }
  struct { const char* name; kfn f; double per_asm; } ks[] = {
    {"same code: add", k_same, 8},
    {"2 PCs by hw slot: add|add", k_pc_by_slot, 8},
    {"2 PCs by wave&4: add|add", k_pc_by_w4, 8},
    {"wave&4 roles: add|rot", k_add_rot_w4, 8},
    {"wave&4 roles: add+xor|rot (per-wave count)", k_ax_rot_w4, 0},
    {"add8 xor8 rot8", k_axr, 24},
    {"add8 xor8 rot8 + s_barrier", k_axr_bar, 24},
    {"(add8 xor8 rot8)x3 + s_barrier", k_axr_bar3, 24},
    {"add8 xor8 add8 + s_barrier", k_add_bar, 24},
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
      const double wps = 2.0 * threads / 256;  // waves per SIMD
      // per_asm 0: half the waves run 16-instruction bodies, half 8: average 12
      const double per = k.per_asm > 0 ? k.per_asm : 12.0;
      const double instr = wps * 3 * ITERS * 8 * per;
      printf("wps=%g %-44s %8.3f ms  %5.2f SIMD-cycles/wave-instr\n", wps, k.name, ms,
             ms * 1e-3 * 2.4e9 / instr);
    }
    CHECK(hipFree(out));
  }
  return 0;
}
