// Memory-pattern microbenchmark #2: LDS-staged layouts for one packet per lane.
// Slot stride S = 1408 = 11 runs of 128 B; a wave owns 64 packets and moves one
// 128-byte run per packet per round (8 packets x 128 B = one 1 KiB instruction).
//   D  LDS-DMA loads (global_load_lds_dwordx4), lane reads its run from LDS
//      (XOR-swizzled, conflict-free ds_read_b128), direct lane-strided stores
//   E  LDS-DMA loads + stores staged back through LDS and issued coalesced
//   F  register loads (coalesced) + ds_write transpose, stores as E
//   G  D with the next round's DMA issued before the current round's reads
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench_mem2.hip -o tools/microbench_mem2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr uint32_t S = 1408, RUNS = 11, WAVES = 4;

__device__ __forceinline__ uint32_t swz(uint32_t p) { return (p >> 1) & 7u; }

template <int MODE>
__global__ __launch_bounds__(256) void kern(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint32_t n) {
  __shared__ uint4 lds[WAVES][2][512];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t base = (blockIdx.x * WAVES + wave) * 64;
  if (base >= n) return;  // n is a multiple of 64 here
  const uint32_t jp = lane >> 3;          // packet within an instruction group
  auto gaddr = [&](const uint8_t* b, uint32_t j, uint32_t r) {
    uint32_t p = 8 * j + jp;               // packet within wave
    uint32_t k = (lane & 7) ^ swz(p);
    return b + (uint64_t)(base + p) * S + 128 * r + 16 * k;
  };
  auto issue = [&](uint32_t r, uint32_t buf) {
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j)
      __builtin_amdgcn_global_load_lds((const void*)gaddr(src, j, r), &lds[wave][buf][64 * j], 16, 0, 0);
  };
  if (MODE == 3) issue(0, 0);
  for (uint32_t r = 0; r < RUNS; ++r) {
    uint32_t buf = (MODE == 3) ? (r & 1) : 0;
    if (MODE == 0 || MODE == 1) {
      issue(r, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (MODE == 2) {
      uint4 v[8];
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) v[j] = *(const uint4*)gaddr(src, j, r);
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) lds[wave][0][64 * j + lane] = v[j];
    } else {  // MODE 3: prefetch next
      if (r + 1 < RUNS) issue(r + 1, buf ^ 1);
      if (r + 1 < RUNS) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_wave_barrier();
    uint4 c[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) c[k] = lds[wave][buf][8 * lane + (k ^ swz(lane))];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) c[k].x ^= 0x5a5a5a5au;
    if (MODE == 0 || MODE == 3) {
      uint8_t* d = dst + (uint64_t)(base + lane) * S + 128 * r;
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k) *(uint4*)(d + 16 * k) = c[k];
    } else {
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k) lds[wave][0][8 * lane + (k ^ swz(lane))] = c[k];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) *(uint4*)gaddr(dst, j, r) = lds[wave][0][64 * j + lane];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

int main() {
  const uint32_t n = 1u << 20;
  uint8_t *src, *dst;
  CHECK(hipMalloc(&src, (size_t)n * S + 4096));
  CHECK(hipMalloc(&dst, (size_t)n * S + 4096));
  CHECK(hipMemset(src, 3, (size_t)n * S));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const double bytes = 2.0 * n * S;
  uint8_t* ref;
  CHECK(hipHostMalloc(&ref, 4096));
  auto run = [&](const char* name, auto launch) -> int {
    CHECK(hipMemset(dst, 0, (size_t)n * S));
    launch();
    CHECK(hipDeviceSynchronize());
    // spot check: byte 0 of packet 12345 run 5 must be 3 ^ 0x5a
    CHECK(hipMemcpy(ref, dst + (size_t)12345 * S + 128 * 5, 64, hipMemcpyDeviceToHost));
    int ok = ref[0] == (3 ^ 0x5a) && ref[1] == (3 ^ 0x5a) && ref[4] == 3;
    const int R = 20;
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < R; ++r) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-44s %8.3f ms/copy  %7.1f GB/s  %s\n", name, ms / R, bytes / (ms / R * 1e-3) / 1e9, ok ? "ok" : "WRONG");
    return 0;
  };
  uint32_t grid = n / 256;
  run("D  DMA in, lane-strided stores", [&] { hipLaunchKernelGGL(kern<0>, dim3(grid), dim3(256), 0, 0, src, dst, n); });
  run("E  DMA in, LDS-staged coalesced stores", [&] { hipLaunchKernelGGL(kern<1>, dim3(grid), dim3(256), 0, 0, src, dst, n); });
  run("F  reg loads+ds_write, coalesced stores", [&] { hipLaunchKernelGGL(kern<2>, dim3(grid), dim3(256), 0, 0, src, dst, n); });
  run("G  DMA in (prefetch 1), lane-strided stores", [&] { hipLaunchKernelGGL(kern<3>, dim3(grid), dim3(256), 0, 0, src, dst, n); });
  return 0;
}
