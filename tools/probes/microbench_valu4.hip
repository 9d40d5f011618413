// VALU co-issue probe for gfx950, part 4: which opcodes run at the 2-cycle
// (dual-issue) rate, and how rare must a slow opcode be to leave it intact?
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_valu4.hip -o tools/microbench_valu4
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 1024
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define BODY8(OP) OP OP OP OP OP OP OP OP
#define OP8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define REGS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define KERN(NAME, ASM)                                                         \
__global__ void NAME(uint32_t* out, uint32_t seed) {                            \
  uint32_t a0 = seed + threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3;      \
  uint32_t a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;                  \
  uint32_t b = seed * 3 + 1, c = seed * 7 + 5;                                  \
  for (int i = 0; i < ITERS; ++i) asm volatile(BODY8(ASM) : REGS : "v"(b), "v"(c)); \
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
}
#define I1(name, text) KERN(name, OP8(text))
#define ADD(k) "v_add_u32 %" #k ", %" #k ", %8\n"
#define XOR(k) "v_xor_b32 %" #k ", %" #k ", %9\n"
#define X_SHL_E64(k) "v_lshlrev_b32_e64 %" #k ", 3, %" #k "\n"
#define X_SHL_V(k) "v_lshlrev_b32 %" #k ", %8, %" #k "\n"
#define X_SHR_V(k) "v_lshrrev_b32 %" #k ", %8, %" #k "\n"
#define X_ASHR(k) "v_ashrrev_i32 %" #k ", 3, %" #k "\n"
#define X_SUB(k) "v_sub_u32 %" #k ", %" #k ", %8\n"
#define X_SUBREV(k) "v_subrev_u32 %" #k ", %" #k ", %8\n"
#define X_NOT(k) "v_not_b32 %" #k ", %" #k "\n"
#define X_XNOR(k) "v_xnor_b32 %" #k ", %" #k ", %8\n"
#define X_MAX(k) "v_max_u32 %" #k ", %" #k ", %8\n"
#define X_BFE(k) "v_bfe_u32 %" #k ", %" #k ", 3, 12\n"
#define X_BFI(k) "v_bfi_b32 %" #k ", %8, %" #k ", %9\n"
#define X_CND(k) "v_cndmask_b32 %" #k ", %" #k ", %8, vcc\n"
#define X_MOV(k) "v_mov_b32 %" #k ", %8\n"
#define X_SHL16(k) "v_lshlrev_b16 %" #k ", 3, %" #k "\n"
#define X_PKSHL16(k) "v_pk_lshlrev_b16 %" #k ", 3, %" #k "\n"
#define X_PKSHR16(k) "v_pk_lshrrev_b16 %" #k ", 3, %" #k "\n"
#define X_MUL24(k) "v_mul_u32_u24 %" #k ", %" #k ", 8\n"
#define X_ADDC(k) "v_addc_co_u32 %" #k ", vcc, %" #k ", %8, vcc\n"
#define X_LSHLADD(k) "v_lshl_add_u32 %" #k ", %" #k ", 3, %9\n"
#define X_ADDLSHL(k) "v_add_lshl_u32 %" #k ", %" #k ", %8, 3\n"
#define X_ANDOR(k) "v_and_or_b32 %" #k ", %" #k ", %8, %9\n"
#define X_OR3(k) "v_or3_b32 %" #k ", %" #k ", %8, %9\n"
#define X_XOR3(k) "v_xor3_b32 %" #k ", %" #k ", %8, %9\n"
#define X_BITOP3S(k) "v_bitop3_b32 %" #k ", %" #k ", %8, %9 bitop3:0x96\n"
#define X_PKADD32(k) "v_pk_add_u32 %" #k ", %" #k ", %8\n"
#define X_PKMOV(k) "v_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[0,1]\n"
#define X_ALIGN(k) "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 20\n"
#define X_MADU24(k) "v_mad_u32_u24 %" #k ", %" #k ", 8, %9\n"
#define X_PKFMA(k) "v_pk_fma_f32 v[40:41], v[42:43], v[44:45], v[40:41]\n"
I1(k_shl_e64, X_SHL_E64) I1(k_shl_v, X_SHL_V) I1(k_shr_v, X_SHR_V) I1(k_ashr, X_ASHR)
I1(k_sub, X_SUB) I1(k_subrev, X_SUBREV) I1(k_not, X_NOT) I1(k_xnor, X_XNOR) I1(k_max, X_MAX)
I1(k_bfe, X_BFE) I1(k_bfi, X_BFI) I1(k_cnd, X_CND) I1(k_mov, X_MOV) I1(k_shl16, X_SHL16)
I1(k_pkshl16, X_PKSHL16) I1(k_pkshr16, X_PKSHR16) I1(k_mul24, X_MUL24) I1(k_addc, X_ADDC)
I1(k_lshladd, X_LSHLADD) I1(k_addlshl, X_ADDLSHL) I1(k_andor, X_ANDOR) I1(k_or3, X_OR3)
I1(k_bitop3, X_BITOP3S) I1(k_madu24, X_MADU24)
// rare slow op: 1 alignbit per 8*R fast ops (R groups of add8/xor8 ... )
#define FAST16 OP8(ADD) OP8(XOR)
#define ROT1 "v_alignbit_b32 %0, %0, %0, 20\n"
#define SHL1 "v_lshlrev_b32 %0, 3, %0\n"
KERN(k_rare16, FAST16 ROT1)
KERN(k_rare64, FAST16 FAST16 FAST16 FAST16 ROT1)
KERN(k_rare256, FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 FAST16 ROT1)
KERN(k_rare64shl, FAST16 FAST16 FAST16 FAST16 SHL1)
// slow op with no dependent consumer nearby (writes a dead register)
#define ROTDEAD "v_alignbit_b32 v60, %0, %0, 20\n"
KERN(k_rare64dead, FAST16 FAST16 FAST16 FAST16 ROTDEAD)
KERN(k_rare16dead, FAST16 ROTDEAD)

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device CUs %d clock %d kHz\n", cus, prop.clockRate);
  struct { const char* name; kfn f; double per_asm; } ks[] = {
    {"lshlrev_e64 imm", k_shl_e64, 8}, {"lshlrev vgpr amt", k_shl_v, 8}, {"lshrrev vgpr amt", k_shr_v, 8},
    {"ashrrev", k_ashr, 8}, {"sub", k_sub, 8}, {"subrev", k_subrev, 8}, {"not", k_not, 8},
    {"xnor", k_xnor, 8}, {"max_u32", k_max, 8}, {"bfe_u32", k_bfe, 8}, {"bfi_b32", k_bfi, 8},
    {"cndmask", k_cnd, 8}, {"mov", k_mov, 8}, {"lshlrev_b16", k_shl16, 8},
    {"pk_lshlrev_b16", k_pkshl16, 8}, {"pk_lshrrev_b16", k_pkshr16, 8}, {"mul_u32_u24", k_mul24, 8},
    {"addc_co", k_addc, 8}, {"lshl_add", k_lshladd, 8}, {"add_lshl", k_addlshl, 8},
    {"and_or", k_andor, 8}, {"or3", k_or3, 8}, {"bitop3", k_bitop3, 8},
    {"mad_u32_u24", k_madu24, 8},
    {"16 fast + 1 rot", k_rare16, 17}, {"64 fast + 1 rot", k_rare64, 65},
    {"256 fast + 1 rot", k_rare256, 257}, {"64 fast + 1 shl", k_rare64shl, 65},
    {"64 fast + 1 rot (dead dst)", k_rare64dead, 65}, {"16 fast + 1 rot (dead dst)", k_rare16dead, 17},
  };
  const int threads = 512;  // 8 waves -> 2 per SIMD; 2 blocks per CU -> 4 per SIMD
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
    const double instr = 4.0 * 3 * ITERS * 8 * k.per_asm;
    printf("wps=4 %-30s %8.3f ms  %5.2f SIMD-cycles/wave-instr\n", k.name, ms, ms * 1e-3 * 2.4e9 / instr);
  }
  return 0;
}
