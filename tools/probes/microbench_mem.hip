// Memory-pattern microbenchmark for the one-packet-per-lane AEAD layout (gfx950).
// Copies N packets of P bytes between slot buffers (slot stride S) with the
// access patterns the AEAD kernels could use, no arithmetic, and reports GB/s
// of algorithmic bytes (2 * N * P per copy).
//   A  lane-strided:   lane = packet, 4 x dwordx4 per 64-byte block (current kernel)
//   A16 lane-strided, destination shifted by +16 bytes (the seal wire offset)
//   B  coalesced:      contiguous dwordx4 copy of the same slot bytes (upper bound)
//   C  LDS transpose:  wave loads 16 packets' 64-byte blocks per instruction
//                      (lanes 4p..4p+3 -> packet p), transposes through LDS so
//                      lane L holds packet L's block, and stores back the same way
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench_mem.hip -o tools/microbench_mem
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void copy_lane(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                 uint32_t n, uint32_t P, uint32_t S, uint32_t dshift) {
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint8_t* s = src + (uint64_t)i * S;
  uint8_t* d = dst + (uint64_t)i * S + dshift;
  uint32_t nblk = (P + 63) / 64;
  uint32_t acc = 0;
  for (uint32_t b = 0; b < nblk; ++b) {
    const uint4* sp = (const uint4*)(s + 64 * b);
    uint4 a0 = sp[0], a1 = sp[1], a2 = sp[2], a3 = sp[3];
    uint4* dp = (uint4*)(d + 64 * b);
    dp[0] = a0; dp[1] = a1; dp[2] = a2; dp[3] = a3;
  }
}

__global__ __launch_bounds__(256) void copy_flat(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16) {
  uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}

// lane L of each wave owns packet (wave_base + L); 64 packets per wave
__global__ __launch_bounds__(256) void copy_lds(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                uint32_t n, uint32_t P, uint32_t S) {
  __shared__ uint4 tile[4][64 * 4 + 64];  // per wave: 64 packets x 4 chunks (+pad per 16 rows)
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t base = (blockIdx.x * 4 + wave) * 64;
  if (base >= n) return;
  uint4* t = tile[wave];
  const uint32_t nblk = (P + 63) / 64;
  // padded index: chunk c of packet p at p*4 + c + (p/16)*? -> keep simple, pad every 16 chunks
  auto idx = [](uint32_t p, uint32_t c) { return p * 4 + c + (p >> 4); };
  for (uint32_t b = 0; b < nblk; ++b) {
    // 4 coalesced-ish loads: instruction q covers packets 16q..16q+15, lane -> (p = 16q + lane/4, c = lane%4)
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      uint32_t p = 16 * q + (lane >> 2), c = lane & 3;
      uint32_t pk = base + p;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (pk < n) v = *(const uint4*)(src + (uint64_t)pk * S + 64 * b + 16 * c);
      t[idx(p, c)] = v;
    }
    __builtin_amdgcn_wave_barrier();
    uint4 a0 = t[idx(lane, 0)], a1 = t[idx(lane, 1)], a2 = t[idx(lane, 2)], a3 = t[idx(lane, 3)];
    // (compute on a0..a3 would go here) -- write back transposed
    a0.x ^= 1u;
    t[idx(lane, 0)] = a0; t[idx(lane, 1)] = a1; t[idx(lane, 2)] = a2; t[idx(lane, 3)] = a3;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      uint32_t p = 16 * q + (lane >> 2), c = lane & 3;
      uint32_t pk = base + p;
      uint4 v = t[idx(p, c)];
      if (pk < n) *(uint4*)(dst + (uint64_t)pk * S + 64 * b + 16 * c) = v;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

int main() {
  const uint32_t n = 1u << 20, P = 1350 + 42;  // 22 blocks of 64 B per packet
  const uint32_t S = 1408;
  uint8_t *src, *dst;
  CHECK(hipMalloc(&src, (size_t)n * S + 4096));
  CHECK(hipMalloc(&dst, (size_t)n * S + 4096));
  CHECK(hipMemset(src, 1, (size_t)n * S));
  CHECK(hipMemset(dst, 0, (size_t)n * S));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const double bytes = 2.0 * n * 1408;  // bytes moved per copy (22 blocks x 64 B each way)
  auto run = [&](const char* name, auto launch) -> int {
    launch();
    CHECK(hipDeviceSynchronize());
    const int R = 20;
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < R; ++r) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-34s %8.3f ms/copy  %7.1f GB/s\n", name, ms / R, bytes / (ms / R * 1e-3) / 1e9);
    return 0;
  };
  uint32_t grid = (n + 255) / 256;
  run("A  lane-strided (64B blocks)", [&] { hipLaunchKernelGGL(copy_lane, dim3(grid), dim3(256), 0, 0, src, dst, n, P, S, 0u); });
  run("A16 lane-strided, dst +16", [&] { hipLaunchKernelGGL(copy_lane, dim3(grid), dim3(256), 0, 0, src, dst, n, P - 16, S, 16u); });
  run("B  coalesced flat copy", [&] { hipLaunchKernelGGL(copy_flat, dim3(2048), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst, (uint64_t)n * S / 16); });
  run("B' coalesced flat copy (grid n/256)", [&] { hipLaunchKernelGGL(copy_flat, dim3((uint32_t)((uint64_t)n * S / 16 / 256)), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst, (uint64_t)n * S / 16); });
  run("C  LDS-transposed 16 pkts/instr", [&] { hipLaunchKernelGGL(copy_lds, dim3(grid), dim3(256), 0, 0, src, dst, n, P, S); });
  return 0;
}
