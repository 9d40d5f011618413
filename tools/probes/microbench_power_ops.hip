// Energy per VALU instruction type on MI355X (gfx950), for the power-capped
// AEAD kernels (profiles/r02_power.json: 1400 W PPT active).  Each variant runs
// one instruction type back to back (16 independent chains per lane, 4 waves
// per SIMD, every CU) for ~SECONDS; tools/power_probe.py samples socket power
// and clock meanwhile.  Energy per op ~ (P - P_base) / rate.
//   microbench_power_ops VARIANT SECONDS   -> one JSON line
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench_power_ops.hip -o tools/microbench_power_ops
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

#define R16(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7) OP(8) OP(9) OP(10) OP(11) OP(12) OP(13) OP(14) OP(15)

template <int V>
__global__ __launch_bounds__(256) void ops(uint32_t *out, uint32_t iters, uint32_t seed) {
  uint32_t x[16];
  const uint32_t t = threadIdx.x + blockIdx.x * 256u;
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = t * 2654435761u + seed * (i + 1);
  const uint32_t k = seed | 1u;
  for (uint32_t it = 0; it < iters; ++it) {
#define ADD(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(x[(i + 1) & 15]));
#define XOR(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[i]) : "v"(x[(i + 1) & 15]));
#define ALIGN(i) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(x[i]));
#define PERM(i) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x[i]) : "s"(0x01000302u));
#define ALIGNB(i) asm volatile("v_alignbyte_b32 %0, %0, %0, 2" : "+v"(x[i]));
#define MAD(i) { uint64_t d; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(d) : "v"(x[i]), "v"(x[(i + 1) & 15]) : "vcc"); x[i] = (uint32_t)d; }
#define ARX(i) asm volatile("v_add_u32 %0, %0, %2\n\tv_xor_b32 %1, %1, %0\n\tv_alignbit_b32 %1, %1, %1, 16" : "+v"(x[i]), "+v"(x[(i + 8) & 15]) : "v"(x[(i + 4) & 15]));
    if constexpr (V == 0) { R16(ADD) }
    if constexpr (V == 1) { R16(XOR) }
    if constexpr (V == 2) { R16(ALIGN) }
    if constexpr (V == 3) { R16(PERM) }
    if constexpr (V == 4) { R16(ALIGNB) }
    if constexpr (V == 5) { R16(MAD) }
    if constexpr (V == 6) { R16(ARX) }
  }
  uint32_t acc = k;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc ^= x[i];
  out[t] = acc;
}

int main(int argc, char **argv) {
  const char *names[] = {"add", "xor", "alignbit", "perm", "alignbyte", "mad_u64", "arx_step"};
  int v = -1;
  for (int i = 0; i < 7; ++i)
    if (argc > 1 && !strcmp(argv[1], names[i])) v = i;
  if (v < 0) {
    printf("usage: %s add|xor|alignbit|perm|alignbyte|mad_u64|arx_step SECONDS\n", argv[0]);
    return 2;
  }
  const double secs = argc > 2 ? atof(argv[2]) : 3.0;
  const uint32_t blocks = 256 * 16, iters = 4096;  // 4 waves per SIMD
  uint32_t *out;
  CHECK(hipMalloc(&out, blocks * 256 * 4));
  auto launch = [&] {
    switch (v) {
      case 0: hipLaunchKernelGGL(ops<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u); break;
      case 1: hipLaunchKernelGGL(ops<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u); break;
      case 2: hipLaunchKernelGGL(ops<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u); break;
      case 3: hipLaunchKernelGGL(ops<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u); break;
      case 4: hipLaunchKernelGGL(ops<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u); break;
      case 5: hipLaunchKernelGGL(ops<5>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u); break;
      default: hipLaunchKernelGGL(ops<6>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u); break;
    }
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  launch();
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms1;
  CHECK(hipEventElapsedTime(&ms1, e0, e1));
  const int reps = (int)(secs * 1e3 / ms1) + 1;
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double instr = (double)blocks * 4 /* waves */ * iters * 16 * (v == 6 ? 3 : 1) * reps;
  printf("{\"variant\": \"%s\", \"ms\": %.2f, \"wave_instr_per_s\": %.4e, \"lane_ops_per_s\": %.4e}\n",
         names[v], ms, instr / (ms * 1e-3), instr * 64 / (ms * 1e-3));
  return 0;
}
