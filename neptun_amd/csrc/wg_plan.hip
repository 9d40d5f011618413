// wg_plan.hip -- scheduling pass for mixed-length descriptor batches.
//
// The AEAD kernels run one packet per lane in lockstep, so a wave costs as
// many rounds as its longest packet.  A batch that interleaves 64-byte and
// 8900-byte datagrams (BASELINE config 3) would leave most lanes idle.  This
// counting sort groups packets by their round count (128-byte runs), longest
// first, so each wave's 64 lanes carry similar work and the long waves start
// early.  Results do not depend on the order: every packet is independent.
//
// Three passes, no global atomics (a handful of hot bins would serialise
// them): per-tile histograms -> one scan over [bin][tile] -> per-tile scatter
// with wave-aggregated LDS counters.  The order inside a bin follows the tile
// and wave order, so the permutation is deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "neptun_gpu.h"
#include "wg_aead_kernels.h"

namespace wg {

// bin 0 = longest: rounds of the larger side of the op, clamped to kPlanBins-1
__device__ __forceinline__ uint32_t plan_bin(const wg_packet_desc &d, uint32_t extra) {
  const uint32_t rounds = (uint32_t)(((uint64_t)d.len + extra + 127u) >> 7);
  return kPlanBins - 1u - min(rounds, kPlanBins - 1u);
}

__device__ __forceinline__ uint32_t tile_begin(uint32_t n, uint32_t t) {
  return (uint32_t)(((uint64_t)n * t) / kPlanTiles);
}

// Wave-aggregated "ticket" on an LDS counter array: lanes with equal bins get
// consecutive slots; one LDS atomic per distinct bin in the wave.
__device__ __forceinline__ uint32_t wave_ticket(uint32_t *cnt, uint32_t bin, bool active) {
  uint64_t pending = __ballot(active);
  uint32_t mine = 0;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t below = (1ull << lane) - 1ull;
  while (pending) {
    const uint32_t leader = (uint32_t)__builtin_ctzll(pending);
    const uint32_t b = __shfl(bin, leader, 64);
    const uint64_t same = __ballot(active && bin == b) & pending;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&cnt[b], (uint32_t)__builtin_popcountll(same));
    base = __shfl(base, leader, 64);
    if (active && bin == b) mine = base + (uint32_t)__builtin_popcountll(same & below);
    pending &= ~same;
  }
  return mine;
}

// pass 1: tile t counts its bins into table[bin * kPlanTiles + t]
__global__ __launch_bounds__(256) void plan_hist_kernel(const wg_packet_desc *descs, uint32_t n,
                                                        uint32_t extra, uint32_t *table) {
  __shared__ uint32_t h[kPlanBins];
  const uint32_t t = blockIdx.x;
  for (uint32_t b = threadIdx.x; b < kPlanBins; b += 256) h[b] = 0;
  __syncthreads();
  const uint32_t lo = tile_begin(n, t), hi = tile_begin(n, t + 1);
  for (uint32_t i0 = lo; i0 < hi; i0 += 256) {
    const uint32_t i = i0 + threadIdx.x;
    const bool active = i < hi;
    const uint32_t bin = active ? plan_bin(descs[i], extra) : 0u;
    (void)wave_ticket(h, bin, active);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kPlanBins; b += 256) table[b * kPlanTiles + t] = h[b];
}

// pass 2: exclusive scan of the kPlanBins x kPlanTiles table (bin-major), one block
__global__ __launch_bounds__(1024) void plan_scan_kernel(uint32_t *table) {
  constexpr uint32_t kN = kPlanBins * kPlanTiles, kPer = kN / 1024;
  __shared__ uint32_t part[1024];
  const uint32_t tid = threadIdx.x;
  uint32_t *seg = table + tid * kPer;
  uint32_t s = 0;
  for (uint32_t j = 0; j < kPer; ++j) s += seg[j];
  part[tid] = s;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    const uint32_t x = tid >= o ? part[tid - o] : 0u;
    __syncthreads();
    part[tid] += x;
    __syncthreads();
  }
  uint32_t run = part[tid] - s;
  for (uint32_t j = 0; j < kPer; ++j) {
    const uint32_t v = seg[j];
    seg[j] = run;
    run += v;
  }
}

// pass 3: tile t places its packets at table[bin][t] + their rank inside the tile
__global__ __launch_bounds__(256) void plan_scatter_kernel(const wg_packet_desc *descs,
                                                           uint32_t n, uint32_t extra,
                                                           const uint32_t *table,
                                                           uint32_t *order) {
  __shared__ uint32_t next[kPlanBins];
  const uint32_t t = blockIdx.x;
  for (uint32_t b = threadIdx.x; b < kPlanBins; b += 256) next[b] = table[b * kPlanTiles + t];
  __syncthreads();
  const uint32_t lo = tile_begin(n, t), hi = tile_begin(n, t + 1);
  const uint32_t wave = threadIdx.x >> 6;
  for (uint32_t i0 = lo; i0 < hi; i0 += 256) {
    // waves take tickets one after another so the tile keeps its index order
    const uint32_t i = i0 + threadIdx.x;
    const bool active = i < hi;
    const uint32_t bin = active ? plan_bin(descs[i], extra) : 0u;
    for (uint32_t w = 0; w < 4; ++w) {
      if (wave == w) {
        const uint32_t pos = wave_ticket(next, bin, active);
        if (active) order[pos] = i;
      }
      __syncthreads();
    }
  }
}

}  // namespace wg
