// Memory-locality microbenchmark for the one-packet-per-lane layout (gfx950).
//
// Question: is the kernel's memory-only rate (~5.0 TB/s) capped by
// the access ORDER -- each round touches one 128-byte line of each of 64
// packets 1408 bytes apart, so every HBM row is opened ~11 times per packet --
// rather than by the staging mechanism?  Every variant copies the same bytes
// (1M packets x 11 lines x 128 B, slot stride 1408) with the same per-wave
// structure (batches of 8 x 16-byte loads per lane, then 8 stores); only the
// order in which a wave walks its 64 packets x 11 lines differs:
//   P1   batch = line l of all 64 packets (the AEAD kernels' round)
//   P2   batch = lines l, l+1 of 32 packets (256 contiguous bytes per packet)
//   P4   batch = lines l..l+3 of 16 packets
//   P8   batch = lines l..l+7 of 8 packets (1 KiB contiguous per packet)
//   FLAT batch = the next 8 KiB of the wave's contiguous 64-packet region
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench_mem3.hip -o tools/microbench_mem3
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__);            \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

constexpr uint32_t kS = 1408, kLines = 11;

// byte offset (inside the wave's 64-packet region) of 16-byte piece `lane` of
// instruction j of batch b, for packet-group width G lines (G = 1, 2, 4, 8) or flat (G = 0)
template <int G>
__device__ __forceinline__ uint32_t piece(uint32_t b, uint32_t j, uint32_t lane) {
  if constexpr (G == 0) {
    return (b * 8u + j) * 1024u + lane * 16u;  // contiguous
  } else {
    // a batch covers G lines of 64/G packets; instruction j covers 8/G packets x G lines
    // lane -> (packet, line, chunk): 8 lanes per 128-byte line
    constexpr uint32_t kPk = 64u / G;                 // packets per batch
    const uint32_t lines0 = (b % ((kLines + G - 1) / G)) * G;
    const uint32_t pgrp = b / ((kLines + G - 1) / G);  // which group of kPk packets
    const uint32_t idx = j * 8u + (lane >> 3);        // 0..63 = (packet, line) pair in the batch
    const uint32_t pk = pgrp * kPk + idx / G, ln = lines0 + idx % G;
    return pk * kS + ln * 128u + (lane & 7u) * 16u;
  }
}

template <int G>
__device__ __forceinline__ uint32_t batches() {
  if constexpr (G == 0) return (64u * kS + 8191u) / 8192u;
  else return ((kLines + G - 1) / G) * G;  // (64/G packet groups) x ceil(11/G) line groups
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool kNT>
__device__ __forceinline__ uint4 ld(const uint8_t *p) {
  if constexpr (kNT) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *(const uint4 *)p;
  }
}
template <bool kNT>
__device__ __forceinline__ void st(uint8_t *p, uint4 v) {
  if constexpr (kNT) __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (u32x4 *)p);
  else *(uint4 *)p = v;
}

// kNT: nontemporal loads and stores; kPipe: the next batch's loads are issued
// before this batch's stores; LDS padding (dynamic) sets workgroups per CU
template <int G, bool kNT, bool kPipe>
__global__ __launch_bounds__(512) void copy_order(const uint8_t *__restrict__ src,
                                                  uint8_t *__restrict__ dst, uint32_t waves) {
  extern __shared__ uint32_t pad[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = blockIdx.x * 8u + (threadIdx.x >> 6);
  if (wv >= waves) return;
  if (lane == 65u) pad[0] = 0;  // keep the LDS allocation
  const uint64_t base = (uint64_t)wv * 64u * kS;
  const uint32_t nb = batches<G>();
  auto okf = [&](uint32_t off) { return off < 64u * kS && (G == 0 || (off % kS) < kLines * 128u); };
  uint4 v[8];
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) {
    const uint32_t off = piece<G>(0, j, lane);
    v[j] = okf(off) ? ld<kNT>(src + base + off) : make_uint4(0, 0, 0, 0);
  }
  for (uint32_t b = 0; b < nb; ++b) {
    uint4 w[8];
    if (kPipe && b + 1 < nb) {
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t off = piece<G>(b + 1, j, lane);
        w[j] = okf(off) ? ld<kNT>(src + base + off) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t off = piece<G>(b, j, lane);
      if (okf(off)) st<kNT>(dst + base + off, v[j]);
    }
    if (!kPipe && b + 1 < nb) {
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t off = piece<G>(b + 1, j, lane);
        w[j] = okf(off) ? ld<kNT>(src + base + off) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) v[j] = w[j];
  }
}

// window probes (FLAT order): kSweep = batch b of wave w is global 8-KiB batch
// b * waves + w (the chip-wide working window stays compact, like a grid-stride
// copy); kOneShot = every wave does one batch (11x the waves, no loop)
template <bool kSweep, bool kOneShot>
__global__ __launch_bounds__(512) void copy_window(const uint8_t *__restrict__ src,
                                                   uint8_t *__restrict__ dst, uint32_t waves) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = blockIdx.x * 8u + (threadIdx.x >> 6);
  const uint32_t nb = kOneShot ? 1u : 11u, total = kOneShot ? waves * 11u : waves;
  if (wv >= total) return;
  for (uint32_t b = 0; b < nb; ++b) {
    const uint64_t batch = kOneShot ? wv : kSweep ? (uint64_t)b * waves + wv : (uint64_t)wv * 11u + b;
    const uint64_t base = batch * 8192u;
    uint4 v[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) v[j] = *(const uint4 *)(src + base + j * 1024u + lane * 16u);
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) *(uint4 *)(dst + base + j * 1024u + lane * 16u) = v[j];
  }
}

// K loads then K stores per lane, one-shot waves (K = 1 is the guide's float4 copy)
template <int K, int kThreads>
__global__ __launch_bounds__(kThreads) void copy_k(const uint8_t *__restrict__ src,
                                                   uint8_t *__restrict__ dst, uint64_t bytes) {
  const uint64_t base = ((uint64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6)) * 1024u * K;
  const uint32_t lane = threadIdx.x & 63u;
  if (base >= bytes) return;
  uint4 v[K];
#pragma unroll
  for (int j = 0; j < K; ++j) v[j] = *(const uint4 *)(src + base + j * 1024u + lane * 16u);
#pragma unroll
  for (int j = 0; j < K; ++j) *(uint4 *)(dst + base + j * 1024u + lane * 16u) = v[j];
}

// looping per-wave FLAT region, store j of batch b interleaved with load j of
// batch b + 1 (kMode 0), loads only (1), stores only (2)
template <int kMode>
__global__ __launch_bounds__(512) void copy_mix(const uint8_t *__restrict__ src,
                                                uint8_t *__restrict__ dst, uint32_t waves) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = blockIdx.x * 8u + (threadIdx.x >> 6);
  if (wv >= waves) return;
  const uint64_t base = (uint64_t)wv * 11u * 8192u;
  uint4 v[8];
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j)
    v[j] = kMode == 2 ? make_uint4(lane, j, 0, 0) : *(const uint4 *)(src + base + j * 1024u + lane * 16u);
  for (uint32_t b = 0; b < 11; ++b) {
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint64_t o = base + b * 8192u + j * 1024u + lane * 16u;
      if (kMode != 1) *(uint4 *)(dst + o) = v[j];
      else acc ^= v[j].x ^ v[j].w;
      if (b + 1 < 11 && kMode != 2) v[j] = *(const uint4 *)(src + o + 8192u);
    }
  }
  if (kMode == 1 && acc == 0x12345678u) dst[wv] = 1;
}

int main(int argc, char **argv) {
  const uint32_t n = 1u << 20, waves = n / 64u;
  // `microbench_mem3 P1|FLAT|K1 SECONDS`: run one variant alone for ~SECONDS (for
  // tools/power_probe.py: is the strided order more expensive in ENERGY?)
  const char *only = argc > 2 ? argv[1] : nullptr;
  const double secs = argc > 2 ? atof(argv[2]) : 0.0;
  uint8_t *src, *dst;
  CHECK(hipMalloc(&src, (size_t)n * kS + 65536));
  CHECK(hipMalloc(&dst, (size_t)n * kS + 65536));
  CHECK(hipMemset(src, 1, (size_t)n * kS));
  CHECK(hipMemset(dst, 0, (size_t)n * kS));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double bytes = 2.0 * n * kLines * 128.0;
  auto run = [&](const char *name, auto launch) -> int {
    launch();
    CHECK(hipDeviceSynchronize());
    const int R = 20;
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < R; ++r) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-44s %8.3f ms/copy  %7.1f GB/s\n", name, ms / R, bytes / (ms / R * 1e-3) / 1e9);
    return 0;
  };
  const dim3 grid((waves + 7) / 8), blk(512);
  if (only) {
    const uint64_t tot1 = (uint64_t)n * kLines * 128u;
    auto launch = [&] {
      if (!strcmp(only, "P1")) hipLaunchKernelGGL((copy_order<1, false, false>), grid, blk, 0, 0, src, dst, waves);
      else if (!strcmp(only, "FLAT")) hipLaunchKernelGGL((copy_order<0, false, false>), grid, blk, 0, 0, src, dst, waves);
      else hipLaunchKernelGGL((copy_k<1, 256>), dim3((uint32_t)(tot1 / 1024 / 4)), dim3(256), 0, 0, src, dst, tot1);
    };
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    const int reps = (int)(secs / 0.55e-3);
    for (int r = 0; r < reps; ++r) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"variant\": \"%s\", \"ms_per_copy\": %.4f, \"GBps\": %.1f}\n", only, ms / reps,
           bytes / (ms / reps * 1e-3) / 1e9);
    return 0;
  }
  char name[128];
  for (uint32_t lds : {0u, 60u * 1024u}) {  // 0: up to 4 WG/CU by VGPRs; 60 KiB: 2 WG/CU (the AEAD kernels)
    const char *occ = lds ? "2WG/CU" : "free  ";
#define V(G, NT, PIPE, label)                                                                     \
    snprintf(name, sizeof name, "%s %s nt=%d pipe=%d", occ, label, NT, PIPE);                      \
    run(name, [&] { hipLaunchKernelGGL((copy_order<G, NT, PIPE>), grid, blk, lds, 0, src, dst, waves); });
    V(1, false, false, "P1  ") V(1, true, false, "P1  ") V(1, false, true, "P1  ") V(1, true, true, "P1  ")
    V(8, false, false, "P8  ") V(0, false, false, "FLAT") V(0, true, false, "FLAT") V(0, true, true, "FLAT")
  }
  const uint64_t tot = (uint64_t)n * kLines * 128u;
  for (int rep = 0; rep < 2; ++rep) {
    run("copy K=1 256 thr", [&] { hipLaunchKernelGGL((copy_k<1, 256>), dim3((uint32_t)(tot / 1024 / 4)), dim3(256), 0, 0, src, dst, tot); });
    run("copy K=1 512 thr", [&] { hipLaunchKernelGGL((copy_k<1, 512>), dim3((uint32_t)(tot / 1024 / 8)), dim3(512), 0, 0, src, dst, tot); });
    run("copy K=2 256 thr", [&] { hipLaunchKernelGGL((copy_k<2, 256>), dim3((uint32_t)(tot / 2048 / 4)), dim3(256), 0, 0, src, dst, tot); });
    run("copy K=4 256 thr", [&] { hipLaunchKernelGGL((copy_k<4, 256>), dim3((uint32_t)(tot / 4096 / 4)), dim3(256), 0, 0, src, dst, tot); });
    run("copy K=8 256 thr", [&] { hipLaunchKernelGGL((copy_k<8, 256>), dim3((uint32_t)(tot / 8192 / 4)), dim3(256), 0, 0, src, dst, tot); });
  }
  for (int rep = 0; rep < 2; ++rep) {
    run("mix: store j / load j interleaved", [&] { hipLaunchKernelGGL((copy_mix<0>), grid, blk, 0, 0, src, dst, waves); });
    run("mix: loads only (bytes x2 in the GB/s)", [&] { hipLaunchKernelGGL((copy_mix<1>), grid, blk, 0, 0, src, dst, waves); });
    run("mix: stores only (bytes x2 in the GB/s)", [&] { hipLaunchKernelGGL((copy_mix<2>), grid, blk, 0, 0, src, dst, waves); });
  }
  for (int rep = 0; rep < 2; ++rep) {
    run("window: per-wave region (FLAT)", [&] { hipLaunchKernelGGL((copy_window<false, false>), grid, blk, 0, 0, src, dst, waves); });
    run("window: sweep (grid-stride order)", [&] { hipLaunchKernelGGL((copy_window<true, false>), grid, blk, 0, 0, src, dst, waves); });
    run("window: one batch per wave (11x waves)", [&] { hipLaunchKernelGGL((copy_window<false, true>), dim3((waves * 11 + 7) / 8), blk, 0, 0, src, dst, waves); });
  }
  return 0;
}
