// Pure-compute throughput of the AEAD building blocks on gfx950 (no memory):
// cycles per ChaCha20 block and per Poly1305 16-byte block, per wave, at a
// given occupancy.  Compares against the issue-rate model (full-rate add/xor
// 2 cycles, half-rate alignbit/mad 4 cycles per wave64 instruction).
// Build: hipcc --offload-arch=gfx950 -O3 -I neptun_amd/csrc tools/microbench_chacha.hip -o tools/microbench_chacha
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "wg_crypto.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kBlocks = 256;

template <int WPS>
__global__ __launch_bounds__(256, WPS) void k_chacha(uint32_t* out, uint32_t seed) {
  uint32_t key[8];
  for (int i = 0; i < 8; ++i) key[i] = seed * (i + 1) + threadIdx.x;  // per-lane key (VGPRs)
  uint32_t acc = 0;
  const uint32_t n1 = blockIdx.x * 256 + threadIdx.x, n2 = seed;
  for (int b = 0; b < kBlocks; ++b) {
    uint32_t ks[16];
    wg::chacha20_block(ks, key, (uint32_t)b, n1, n2);
#pragma unroll
    for (int j = 0; j < 16; ++j) acc ^= ks[j];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int WPS>
__global__ __launch_bounds__(256, WPS) void k_chacha_ukey(uint32_t* out, const uint32_t* keys) {
  uint32_t key[8];
  for (int i = 0; i < 8; ++i) key[i] = keys[i];  // uniform key (SGPRs)
  uint32_t acc = 0;
  const uint32_t n1 = blockIdx.x * 256 + threadIdx.x, n2 = 0;
  for (int b = 0; b < kBlocks; ++b) {
    uint32_t ks[16];
    wg::chacha20_block(ks, key, (uint32_t)b, n1, n2);
#pragma unroll
    for (int j = 0; j < 16; ++j) acc ^= ks[j];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int WPS>
__global__ __launch_bounds__(256, WPS) void k_poly(uint32_t* out, uint32_t seed) {
  wg::Poly p;
  uint32_t k0[8];
  for (int i = 0; i < 8; ++i) k0[i] = seed * 0x9E3779B9u * (i + 1) + threadIdx.x * 77u;
  wg::poly_init(p, k0);
  uint32_t m = threadIdx.x;
  for (int b = 0; b < 4 * kBlocks; ++b) {
    wg::poly_block(p, m, m ^ 1u, m + 7u, (uint32_t)b);
    m = p.h0;
  }
  out[blockIdx.x * 256 + threadIdx.x] = p.h0 ^ p.h1 ^ p.h2 ^ p.h3 ^ p.h4;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t *out, *keys;
  CHECK(hipMalloc(&out, 64 << 20));
  CHECK(hipMalloc(&keys, 64));
  CHECK(hipMemset(keys, 0x5a, 64));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  auto run = [&](const char* name, int wps, double units_per_item, int items, auto launch) -> int {
    const int blocks = cus * wps * 8;  // 8 rounds of resident waves
    launch(blocks);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    launch(blocks);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double waves_per_simd = (double)blocks * 4 / (cus * 4);
    const double cycles = ms * 1e-3 * 2.4e9;  // at the nominal 2.4 GHz
    const double per_item = cycles / (waves_per_simd * items);
    printf("%-28s wps=%d  %8.3f ms  %8.1f SIMD-cycles/item/wave @2.4GHz  model %6.0f  eff %.2f\n",
           name, wps, ms, per_item, units_per_item, units_per_item / per_item);
    return 0;
  };
  // model: ChaCha block = 656 full-rate (2 cyc) + 320 half-rate (4 cyc) + 16 acc xor (2)
  const double chacha_model = 656 * 2 + 320 * 4 + 16 * 2;
  const double poly_model = 20 * 4 + 10 * 4 + 8 * 2;
  run("chacha per-lane key", 4, chacha_model, kBlocks, [&](int b) { hipLaunchKernelGGL(k_chacha<4>, dim3(b), dim3(256), 0, 0, out, 1u); });
  run("chacha per-lane key", 2, chacha_model, kBlocks, [&](int b) { hipLaunchKernelGGL(k_chacha<2>, dim3(b), dim3(256), 0, 0, out, 1u); });
  run("chacha uniform key", 4, chacha_model, kBlocks, [&](int b) { hipLaunchKernelGGL(k_chacha_ukey<4>, dim3(b), dim3(256), 0, 0, out, keys); });
  run("chacha uniform key", 8, chacha_model, kBlocks, [&](int b) { hipLaunchKernelGGL(k_chacha_ukey<8>, dim3(b), dim3(256), 0, 0, out, keys); });
  run("poly1305 block", 4, poly_model, 4 * kBlocks, [&](int b) { hipLaunchKernelGGL(k_poly<4>, dim3(b), dim3(256), 0, 0, out, 1u); });
  run("poly1305 block", 8, poly_model, 4 * kBlocks, [&](int b) { hipLaunchKernelGGL(k_poly<8>, dim3(b), dim3(256), 0, 0, out, 1u); });
  return 0;
}
