// VALU throughput microbenchmark for gfx950 (MI355X).
// Measures wave-instructions/cycle/CU for the integer ops the ChaCha20/Poly1305
// kernels lean on. Each kernel runs 8 independent dependency chains per lane so
// the number is issue-throughput, not latency. Build:
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_valu.hip -o tools/microbench_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define BODY32(OP) OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP OP

#define KERNEL32(NAME, ASM)                                                     \
__global__ void NAME(uint32_t* out, uint32_t seed) {                            \
  uint32_t a0 = seed + threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3;      \
  uint32_t a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;                  \
  uint32_t b = seed * 3 + 1, c = seed * 7 + 5;                                  \
  for (int i = 0; i < ITERS; ++i) {                                             \
    asm volatile(BODY32(ASM) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3),         \
                 "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));     \
  }                                                                             \
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
}
// 8 instructions per ASM string (one per chain) -> 32*8 = 256 instr / iter
#define OP8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)

#define ADD(k) "v_add_u32 %" #k ", %" #k ", %8\n"
#define XOR(k) "v_xor_b32 %" #k ", %" #k ", %8\n"
#define ALIGNBIT(k) "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 20\n"
#define PERM(k) "v_perm_b32 %" #k ", %" #k ", %" #k ", %9\n"
#define ADD3(k) "v_add3_u32 %" #k ", %" #k ", %8, %9\n"
#define XAD(k) "v_xad_u32 %" #k ", %" #k ", %8, %9\n"
#define BITOP3(k) "v_bitop3_b32 %" #k ", %" #k ", %8, %9 bitop3:0x96\n"
#define MULLO(k) "v_mul_lo_u32 %" #k ", %" #k ", %8\n"
#define MULHI(k) "v_mul_hi_u32 %" #k ", %" #k ", %8\n"
#define MUL24(k) "v_mul_u32_u24 %" #k ", %" #k ", %8\n"
#define MULHI24(k) "v_mul_hi_u32_u24 %" #k ", %" #k ", %8\n"
#define DOT2(k) "v_dot2_u32_u16 %" #k ", %" #k ", %8, %9\n"
#define LSHLADD(k) "v_lshl_add_u32 %" #k ", %" #k ", 3, %9\n"
#define XORSDWA(k) "v_xor_b32_sdwa %" #k ", %" #k ", %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n"
#define ADDSDWA(k) "v_add_u32_sdwa %" #k ", %" #k ", %8 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n"
#define PKADD16(k) "v_pk_add_u16 %" #k ", %" #k ", %8\n"
#define LSHLOR(k) "v_lshl_or_b32 %" #k ", %" #k ", 7, %9\n"
#define ALIGNBYTE(k) "v_alignbyte_b32 %" #k ", %" #k ", %" #k ", 2\n"
#define ADDCO(k) "v_add_co_u32 %" #k ", vcc, %" #k ", %8\n"

KERNEL32(k_add, OP8(ADD))
KERNEL32(k_xor, OP8(XOR))
KERNEL32(k_alignbit, OP8(ALIGNBIT))
KERNEL32(k_perm, OP8(PERM))
KERNEL32(k_add3, OP8(ADD3))
KERNEL32(k_xad, OP8(XAD))
KERNEL32(k_bitop3, OP8(BITOP3))
KERNEL32(k_mullo, OP8(MULLO))
KERNEL32(k_mulhi, OP8(MULHI))
KERNEL32(k_mul24, OP8(MUL24))
KERNEL32(k_mulhi24, OP8(MULHI24))
KERNEL32(k_dot2, OP8(DOT2))
KERNEL32(k_lshladd, OP8(LSHLADD))
KERNEL32(k_xorsdwa, OP8(XORSDWA))
KERNEL32(k_addsdwa, OP8(ADDSDWA))
KERNEL32(k_pkadd16, OP8(PKADD16))
KERNEL32(k_lshlor, OP8(LSHLOR))
KERNEL32(k_alignbyte, OP8(ALIGNBYTE))
KERNEL32(k_addco, OP8(ADDCO))
// mixes: per chain k one add, one xor, one alignbit (ChaCha's 2:1 full:half ratio)
#define MIX_AXR(k) "v_add_u32 %" #k ", %" #k ", %8\n" "v_xor_b32 %" #k ", %" #k ", %9\n" "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 20\n"
#define MIX_AX(k) "v_add_u32 %" #k ", %" #k ", %8\n" "v_xor_b32 %" #k ", %" #k ", %9\n"
#define MIX_AR(k) "v_add_u32 %" #k ", %" #k ", %8\n" "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 20\n"
#define SHL(k) "v_lshlrev_b32 %" #k ", 3, %" #k "\n"
#define ORR(k) "v_or_b32 %" #k ", %" #k ", %8\n"
#define ANDD(k) "v_and_b32 %" #k ", %" #k ", %8\n"
KERNEL32(k_mix_axr, OP8(MIX_AXR))
KERNEL32(k_mix_ax, OP8(MIX_AX))
KERNEL32(k_mix_ar, OP8(MIX_AR))
KERNEL32(k_shl, OP8(SHL))
KERNEL32(k_or, OP8(ORR))
KERNEL32(k_and, OP8(ANDD))
// grouped runs: all 8 chains' adds, then all xors, then all rotates (4 parallel QRs' shape)
#define GRP_AXR OP8(ADD) OP8(XOR) OP8(ALIGNBIT)
#define GRP_AR OP8(ADD) OP8(ALIGNBIT)
#define GRP_AAXR OP8(ADD) OP8(XOR) OP8(ADD) OP8(ALIGNBIT)
#define GRP_16R OP8(ADD) OP8(XOR) OP8(ADD) OP8(XOR) OP8(ADD) OP8(XOR) OP8(ADD) OP8(XOR) OP8(ALIGNBIT)
KERNEL32(k_grp_axr, GRP_AXR)
KERNEL32(k_grp_ar, GRP_AR)
KERNEL32(k_grp_aaxr, GRP_AAXR)
KERNEL32(k_grp_16r, GRP_16R)

// 64-bit destination ops: 8 chains of u64
#define KERNEL64(NAME, ASM)                                                     \
__global__ void NAME(uint32_t* out, uint32_t seed) {                            \
  uint64_t a0 = seed + threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3;      \
  uint64_t a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;                  \
  uint32_t b = seed * 3 + 1, c = seed * 7 + 5;                                  \
  for (int i = 0; i < ITERS; ++i) {                                             \
    asm volatile(BODY32(ASM) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3),         \
                 "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));     \
  }                                                                             \
  uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                            \
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)r ^ (uint32_t)(r >> 32); \
}
#define MAD64(k) "v_mad_u64_u32 %" #k ", vcc, %8, %9, %" #k "\n"
#define FMA64(k) "v_fma_f64 %" #k ", %" #k ", %" #k ", %" #k "\n"
#define LSHLADD64(k) "v_lshl_add_u64 %" #k ", %" #k ", 2, %" #k "\n"
#define LSHR64(k) "v_lshrrev_b64 %" #k ", 3, %" #k "\n"
KERNEL64(k_mad64, OP8(MAD64))
KERNEL64(k_fma64, OP8(FMA64))
KERNEL64(k_lshladd64, OP8(LSHLADD64))
KERNEL64(k_lshr64, OP8(LSHR64))

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", prop.name, cus, prop.clockRate);
  struct { const char* name; kfn f; } ks[] = {
    {"v_add_u32", k_add}, {"v_xor_b32", k_xor}, {"v_alignbit_b32", k_alignbit},
    {"v_perm_b32", k_perm}, {"v_add3_u32", k_add3}, {"v_xad_u32", k_xad},
    {"v_bitop3_b32", k_bitop3}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
    {"v_mul_u32_u24", k_mul24}, {"v_mul_hi_u32_u24", k_mulhi24}, {"v_dot2_u32_u16", k_dot2},
    {"v_lshl_add_u32", k_lshladd}, {"v_xor_b32_sdwa", k_xorsdwa}, {"v_add_u32_sdwa", k_addsdwa},
    {"v_pk_add_u16", k_pkadd16}, {"v_lshl_or_b32", k_lshlor}, {"v_alignbyte_b32", k_alignbyte},
    {"v_add_co_u32(vcc)", k_addco}, {"mix add,xor,alignbit /3", k_mix_axr},
    {"mix add,xor /2", k_mix_ax}, {"mix add,alignbit /2", k_mix_ar}, {"v_lshlrev_b32", k_shl},
    {"v_or_b32", k_or}, {"v_and_b32", k_and}, {"grp add8,xor8,rot8 /3", k_grp_axr},
    {"grp add8,rot8 /2", k_grp_ar}, {"grp add8,xor8,add8,rot8 /4", k_grp_aaxr},
    {"grp 64 simple, rot8 /9", k_grp_16r}, {"v_mad_u64_u32", k_mad64}, {"v_fma_f64", k_fma64},
    {"v_lshl_add_u64", k_lshladd64}, {"v_lshrrev_b64", k_lshr64},
  };
  const int threads = 256;
  for (int wps : {2, 4}) {  // waves per SIMD
    int blocks = cus * wps;  // 256 threads = 4 waves = 1 per SIMD per block
    uint32_t* out;
    CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1u);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, (uint32_t)r);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      double waves = (double)blocks * (threads / 64) * 5;
      double instr = waves * ITERS * 256.0;           // wave-instructions
      double lane_ops = instr * 64.0;
      double per_s = lane_ops / (ms * 1e-3);
      // wave-instr per CU per cycle at nominal 2.4 GHz
      double ipc = instr / cus / (ms * 1e-3 * 2.4e9);
      printf("wps=%d %-18s %8.3f ms  %7.2f T lane-op/s  %5.3f wave-instr/CU/cyc@2.4GHz\n",
             wps, k.name, ms, per_s / 1e12, ipc);
    }
    CHECK(hipFree(out));
  }
  return 0;
}
