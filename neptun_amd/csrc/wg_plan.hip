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
// with wave-aggregated LDS counters.  The order inside a bin is the index
// order, so the permutation is deterministic.
//
// Tiles walk their descriptors in chunks of kPlanChunk: every lane loads its
// kPlanPer lengths up front (the loads overlap), each wave owns a contiguous
// slice of the chunk, and the scatter places the waves' slices by a per-bin
// prefix over the waves instead of letting the waves take turns.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "neptun_gpu.h"
#include "wg_aead_kernels.h"

namespace wg {

// bin 0 = longest: rounds of the larger side of the op, clamped to kPlanBins-1
__device__ __forceinline__ uint32_t plan_bin(uint32_t len, uint32_t extra) {
  const uint32_t rounds = (uint32_t)(((uint64_t)len + extra + 127u) >> 7);
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

// The lane's kPlanPer bins of the chunk at c0: wave w owns [c0 + 64 kPlanPer w, + 64 kPlanPer),
// element u of the lane is index c0 + 64 (kPlanPer w + u) + lane (index order = (u, lane)).
// live[u]: the element exists (offsets relative to c0, so nothing wraps near 2^32).
__device__ __forceinline__ void load_bins(const wg_packet_desc *descs, uint32_t c0, uint32_t hi,
                                          uint32_t extra, uint32_t (&bin)[kPlanPer],
                                          uint32_t (&idx)[kPlanPer], bool (&live)[kPlanPer]) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t len[kPlanPer];
#pragma unroll
  for (uint32_t u = 0; u < kPlanPer; ++u) {
    const uint32_t off = 64u * (kPlanPer * wave + u) + lane;
    live[u] = off < hi - c0;
    idx[u] = c0 + off;
    len[u] = live[u] ? descs[idx[u]].len : 0u;
  }
#pragma unroll
  for (uint32_t u = 0; u < kPlanPer; ++u) bin[u] = plan_bin(len[u], extra);
}

__device__ __forceinline__ uint32_t next_chunk(uint32_t c0, uint32_t hi) {
  return c0 + min(kPlanChunk, hi - c0);
}

// pass 1: tile t counts its bins into table[bin * kPlanTiles + t]
__global__ __launch_bounds__(kPlanThreads) void plan_hist_kernel(const wg_packet_desc *descs,
                                                                 uint32_t n, uint32_t extra,
                                                                 uint32_t *table) {
  __shared__ uint32_t h[kPlanBins];
  const uint32_t t = blockIdx.x;
  for (uint32_t b = threadIdx.x; b < kPlanBins; b += kPlanThreads) h[b] = 0;
  __syncthreads();
  const uint32_t lo = tile_begin(n, t), hi = tile_begin(n, t + 1);
  for (uint32_t c0 = lo; c0 < hi; c0 = next_chunk(c0, hi)) {
    uint32_t bin[kPlanPer], idx[kPlanPer];
    bool live[kPlanPer];
    load_bins(descs, c0, hi, extra, bin, idx, live);
    // counts only: fire-and-forget LDS adds (no return value to wait for)
#pragma unroll
    for (uint32_t u = 0; u < kPlanPer; ++u)
      if (live[u]) __hip_atomic_fetch_add(&h[bin[u]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kPlanBins; b += kPlanThreads) table[b * kPlanTiles + t] = h[b];
}

// pass 2: exclusive scan of the kPlanBins x kPlanTiles table (bin-major), one
// block.  Wave w takes rows (bins) w, w + 16, ...: one coalesced 16-byte load per
// lane covers a whole row, a lane-level scan ranks it, and the row totals get a
// block scan in LDS before every row is written back with its offset.
__global__ __launch_bounds__(1024) void plan_scan_kernel(uint32_t *table) {
  static_assert(kPlanTiles == 256 && kPlanBins % 16 == 0, "one uint4 per lane covers a row");
  constexpr uint32_t kRows = kPlanBins / 16;  // rows per wave
  __shared__ uint32_t rowsum[kPlanBins];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint4 v[kRows];
  uint32_t pre[kRows];  // exclusive prefix of the lane's 4 entries inside the row
#pragma unroll
  for (uint32_t k = 0; k < kRows; ++k)
    v[k] = reinterpret_cast<const uint4 *>(table + (wave + 16u * k) * kPlanTiles)[lane];
#pragma unroll
  for (uint32_t k = 0; k < kRows; ++k) {
    const uint32_t mine = v[k].x + v[k].y + v[k].z + v[k].w;
    uint32_t inc = mine;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t x = (uint32_t)__shfl_up((int)inc, o, 64);
      if (lane >= o) inc += x;
    }
    pre[k] = inc - mine;
    if (lane == 63u) rowsum[wave + 16u * k] = inc;
  }
  __syncthreads();
  if (wave == 0) {  // exclusive scan of the kPlanBins row totals, 4 per lane
    uint32_t r[kPlanBins / 64], t = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPlanBins / 64; ++j) { r[j] = rowsum[4u * lane + j]; t += r[j]; }
    uint32_t inc = t;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t x = (uint32_t)__shfl_up((int)inc, o, 64);
      if (lane >= o) inc += x;
    }
    uint32_t run = inc - t;
#pragma unroll
    for (uint32_t j = 0; j < kPlanBins / 64; ++j) { rowsum[4u * lane + j] = run; run += r[j]; }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kRows; ++k) {
    uint32_t run = rowsum[wave + 16u * k] + pre[k];
    uint4 o;
    o.x = run; run += v[k].x;
    o.y = run; run += v[k].y;
    o.z = run; run += v[k].z;
    o.w = run;
    reinterpret_cast<uint4 *>(table + (wave + 16u * k) * kPlanTiles)[lane] = o;
  }
}

// pass 3: tile t places its packets at table[bin][t] + their rank inside the
// tile.  Per chunk: each wave ranks its slice on its own LDS counters, one
// thread per bin turns the per-wave counts into positions, then every lane
// writes its kPlanPer entries of `order`.
__global__ __launch_bounds__(kPlanThreads) void plan_scatter_kernel(const wg_packet_desc *descs,
                                                                    uint32_t n, uint32_t extra,
                                                                    const uint32_t *table,
                                                                    uint32_t *order) {
  __shared__ uint32_t next[kPlanBins];             // the tile's next position per bin
  __shared__ uint32_t cnt[kPlanWaves][kPlanBins];  // per-wave counts, then starts
  const uint32_t t = blockIdx.x, wave = threadIdx.x >> 6;
  for (uint32_t b = threadIdx.x; b < kPlanBins; b += kPlanThreads) next[b] = table[b * kPlanTiles + t];
  const uint32_t lo = tile_begin(n, t), hi = tile_begin(n, t + 1);
  for (uint32_t c0 = lo; c0 < hi; c0 = next_chunk(c0, hi)) {
    uint32_t bin[kPlanPer], idx[kPlanPer], rank[kPlanPer];
    bool live[kPlanPer];
    load_bins(descs, c0, hi, extra, bin, idx, live);
    for (uint32_t b = threadIdx.x; b < kPlanBins * kPlanWaves; b += kPlanThreads) (&cnt[0][0])[b] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < kPlanPer; ++u) rank[u] = wave_ticket(cnt[wave], bin[u], live[u]);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < kPlanBins; b += kPlanThreads) {
      uint32_t run = next[b];
#pragma unroll
      for (uint32_t w = 0; w < kPlanWaves; ++w) {
        const uint32_t c = cnt[w][b];
        cnt[w][b] = run;
        run += c;
      }
      next[b] = run;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < kPlanPer; ++u)
      if (live[u]) order[cnt[wave][bin[u]] + rank[u]] = idx[u];
    __syncthreads();  // cnt is reset by the next chunk
  }
}

}  // namespace wg
