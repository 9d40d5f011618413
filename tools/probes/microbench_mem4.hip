// Memory-only staging microbenchmark #4: why does the AEAD kernels' staging
// path alone (WG_ABLATE_NO_CRYPT, 0.655 ms for config 2's seal) run ~20 %
// slower per byte than tools/microbench_mem2.hip's variant E (LDS-DMA in,
// LDS read-out, coalesced stores)?  Every variant moves 1M packets x 11 runs of
// 128 B (slot stride 1408) the way the kernels do: per round a wave issues 8
// LDS-DMA pieces (8 packets x 128 B each), waits for them, reads the 8 KiB
// stage back (ds_read_b128, lane = 16 B of a packet run) and stores it with 8
// 16-byte stores.  Factors:
//   L  load : G = global_load_lds_dwordx4 (64-bit lane address)
//             B = buffer_load_dwordx4 ... lds (wave resource + 32-bit offsets)
//   S  store: G = global_store_dwordx4,  B = buffer_store_dwordx4
//   P  launch: O = one group of 64 packets per wave, grid = n / 512 workgroups
//             W = persistent, 2 x 512-thread workgroups per CU walking groups
//                 (grp += gridDim.x), as aead_strided_kernel
// All variants: 512-thread workgroups, 80 KiB LDS per workgroup (2 per CU).
// Depth variants (global loads/stores, one group per wave):
//   D  two 8 KiB stages per wave: round r + 1's DMA is issued before round r
//      is read out (128 KiB per workgroup, 1 workgroup = 8 waves per CU)
//   H  half rounds (64 B per packet, 4 KiB pieces), two 4 KiB stages per wave:
//      the next half's DMA goes out before this half is read (2 workgroups/CU)
// Loop-granularity variants (flat copy of the same byte count, register loads):
//   LK persistent waves (WPC waves per CU), grid-stride over K-KiB chunks: K loads
//      then K stores per lane per iteration -- does a persistent loop with small K
//      reach the one-shot float4 copy's rate?
//   microbench_mem4 -> one line per variant
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench_mem4.hip -o tools/microbench_mem4
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__);            \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

constexpr uint32_t kS = 1408, kRuns = 11, kWaves = 8;
constexpr uint32_t kStageBytes = 10240;  // 8 KiB stage + 2 KiB (80 KiB per workgroup)

__device__ __forceinline__ uint32_t swz(uint32_t p) { return (p >> 1) & 7u; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}

template <char L, char S>
__device__ __forceinline__ void group(uint4 *run, const uint8_t *src, uint8_t *dst, uint32_t pkt0,
                                      uint32_t lane) {
  const uint32_t y = lane >> 3;
  const uint64_t base = (uint64_t)pkt0 * kS;
  const uint32_t rec = 64u * kS;
  const __amdgpu_buffer_rsrc_t rs = rsrc(src + base, rec), rd = rsrc(dst + base, rec);
  for (uint32_t r = 0; r < kRuns; ++r) {
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t p = 8u * j + y, k = (lane & 7u) ^ swz(p);
      const uint32_t off = p * kS + 128u * r + 16u * k;
      if constexpr (L == 'G')
        __builtin_amdgcn_global_load_lds((const void *)(src + base + off), &run[64u * j], 16, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, &run[64u * j], 16, y * kS + 16u * k,
                                                 8u * j * kS + 128u * r, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint4 v[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) v[j] = run[64u * j + lane];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t p = 8u * j + y, k = (lane & 7u) ^ swz(p);
      const uint32_t off = p * kS + 128u * r + 16u * k;
      if constexpr (S == 'G') {
        *(uint4 *)(dst + base + off) = v[j];
      } else {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 vv = {v[j].x, v[j].y, v[j].z, v[j].w};
        __builtin_amdgcn_raw_buffer_store_b128(vv, rd, y * kS + 16u * k, 8u * j * kS + 128u * r, 0);
      }
    }
  }
}

// K = 8 pieces of 16 B per lane per full round (D) or 4 per half round (H)
template <int kHalf>
__device__ __forceinline__ void group_pipe(uint4 *st0, uint4 *st1, const uint8_t *src, uint8_t *dst,
                                           uint32_t pkt0, uint32_t lane) {
  constexpr uint32_t K = kHalf ? 4u : 8u, kPieces = kHalf ? 2u * kRuns : kRuns;
  const uint32_t y = lane >> 3;
  const uint64_t base = (uint64_t)pkt0 * kS;
  // piece j of step t: packet p = 8j + y (full) / 16j + (lane>>2) (half), chunk k
  auto addr = [&](uint32_t t, uint32_t j) -> uint32_t {
    if constexpr (kHalf) {
      const uint32_t p = 16u * j + (lane >> 2), k = lane & 3u;
      return p * kS + 64u * t + 16u * k;
    } else {
      const uint32_t p = 8u * j + y, k = (lane & 7u) ^ swz(p);
      return p * kS + 128u * t + 16u * k;
    }
  };
  auto issue = [&](uint32_t t, uint4 *st) {
#pragma unroll
    for (uint32_t j = 0; j < K; ++j)
      __builtin_amdgcn_global_load_lds((const void *)(src + base + addr(t, j)), &st[64u * j], 16, 0, 0);
  };
  issue(0, st0);
  for (uint32_t t = 0; t < kPieces; ++t) {
    uint4 *cur = (t & 1u) ? st1 : st0, *nxt = (t & 1u) ? st0 : st1;
    if (t + 1 < kPieces) {
      issue(t + 1, nxt);
      if constexpr (kHalf) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    uint4 v[K];
#pragma unroll
    for (uint32_t j = 0; j < K; ++j) v[j] = cur[64u * j + lane];
#pragma unroll
    for (uint32_t j = 0; j < K; ++j) *(uint4 *)(dst + base + addr(t, j)) = v[j];
  }
}

template <int kHalf>
__global__ __launch_bounds__(512) void kern_pipe(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                 uint32_t n) {
  constexpr uint32_t kStage = kHalf ? 4096u : 8192u;
  __shared__ uint8_t lds[kWaves][2][kStage];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  group_pipe<kHalf>(reinterpret_cast<uint4 *>(lds[wave][0]), reinterpret_cast<uint4 *>(lds[wave][1]), src,
                    dst, (blockIdx.x * kWaves + wave) * 64u, lane);
}

template <int K>
__global__ __launch_bounds__(256) void copy_loop(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                uint64_t chunks) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6), waves = (uint64_t)gridDim.x * 4u;
  for (uint64_t c = wave; c < chunks; c += waves) {
    const uint64_t base = c * 1024u * K;
    uint4 v[K];
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = *(const uint4 *)(src + base + j * 1024u + lane * 16u);
#pragma unroll
    for (int j = 0; j < K; ++j) *(uint4 *)(dst + base + j * 1024u + lane * 16u) = v[j];
  }
}

template <char L, char S, char P>
__global__ __launch_bounds__(512) void kern(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                            uint32_t n) {
  __shared__ uint8_t lds[kWaves][kStageBytes];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint4 *run = reinterpret_cast<uint4 *>(lds[wave]);
  const uint32_t groups = n / 64u / kWaves;
  if constexpr (P == 'O') {
    group<L, S>(run, src, dst, (blockIdx.x * kWaves + wave) * 64u, lane);
  } else {
    for (uint32_t g = blockIdx.x; g < groups; g += gridDim.x) group<L, S>(run, src, dst, (g * kWaves + wave) * 64u, lane);
  }
}

int main() {
  const uint32_t n = 1u << 20;
  uint8_t *src, *dst;
  CHECK(hipMalloc(&src, (size_t)n * kS + 4096));
  CHECK(hipMalloc(&dst, (size_t)n * kS + 4096));
  CHECK(hipMemset(src, 3, (size_t)n * kS));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double bytes = 2.0 * n * kRuns * 128.0;
  auto run = [&](const char *name, auto launch) -> int {
    launch();
    CHECK(hipDeviceSynchronize());
    float best = 1e9f, sum = 0.f;
    const int R = 30;
    for (int i = 0; i < R; ++i) {
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    uint8_t h[16];
    CHECK(hipMemcpy(h, dst + (size_t)12345 * kS + 128 * 5, 16, hipMemcpyDeviceToHost));
    printf("%-36s mean %.4f ms  min %.4f ms  %7.1f GB/s  %s\n", name, sum / R, best,
           bytes / (sum / R * 1e-3) / 1e9, h[0] == 3 && h[15] == 3 ? "ok" : "WRONG");
    return 0;
  };
  const dim3 one(n / 64u / kWaves), pers(2u * cus), blk(512);
#define V(L, S, P, grid) \
  run("L=" #L " S=" #S " P=" #P, [&] { hipLaunchKernelGGL((kern<#L[0], #S[0], #P[0]>), grid, blk, 0, 0, src, dst, n); })
  for (int rep = 0; rep < 2; ++rep) {
    V(G, G, O, one);
    V(B, G, O, one);
    V(G, B, O, one);
    V(B, B, O, one);
    V(G, G, W, pers);
    V(B, B, W, pers);
    run("D  two 8 KiB stages, prefetch 1 round", [&] { hipLaunchKernelGGL(kern_pipe<0>, one, blk, 0, 0, src, dst, n); });
    run("H  two 4 KiB half-round stages", [&] { hipLaunchKernelGGL(kern_pipe<1>, one, blk, 0, 0, src, dst, n); });
  }
  const uint64_t tot = (uint64_t)n * kRuns * 128u;  // same byte count, flat
  for (int wpc : {16, 32}) {
    const dim3 g((uint32_t)(cus * wpc / 4));
    char name[64];
    snprintf(name, sizeof name, "LK K=1 %d waves/CU", wpc);
    run(name, [&] { hipLaunchKernelGGL(copy_loop<1>, g, dim3(256), 0, 0, src, dst, tot / 1024); });
    snprintf(name, sizeof name, "LK K=2 %d waves/CU", wpc);
    run(name, [&] { hipLaunchKernelGGL(copy_loop<2>, g, dim3(256), 0, 0, src, dst, tot / 2048); });
    snprintf(name, sizeof name, "LK K=8 %d waves/CU", wpc);
    run(name, [&] { hipLaunchKernelGGL(copy_loop<8>, g, dim3(256), 0, 0, src, dst, tot / 8192); });
  }
  return 0;
}
