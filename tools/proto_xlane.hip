// proto_xlane.hip -- round-4 prototype (SURVEY §7 hard part 2):
// ChaCha20-Poly1305 SEAL with K lanes per packet instead of one packet per lane.
//
// Bounded on purpose: uniform payload length P, strided NepTUN slots (plaintext at
// slot + 16, datagram at slot + 0, slots with room for whole 16-byte pieces), one
// key (kernel arguments -> SGPRs), counters base + packet index.  It answers one
// question by measurement: does spreading a packet over K lanes -- each lane
// loading its own contiguous span of 64-byte blocks with direct float4 loads (no
// LDS staging), accumulating Poly1305 over its span with the packet's clamped r,
// and one lane combining the K partial accumulators through LDS with powers of r
// -- seal a batch with less energy than the product's one-packet-per-lane kernel
// (neptun_amd/csrc/wg_aead.hip)?  Not part of libneptun_gpu.so; tools/proto_xlane.py
// checks it bit for bit against the product and A/B-times it.
//
// Per packet: NB = 1 + ceil(P / 64) ChaCha20 blocks (block 0 = the Poly1305 key),
// lane l of the packet owns blocks [l * SPL, (l + 1) * SPL), SPL = ceil(NB / K),
// computed as phase-locked pairs (chacha20_block2_sync) plus one single block when
// SPL is odd.  Poly1305: lane l's span of 16-byte messages m_a..m_b gives
// h_l = sum m_i r^(b - i + 1); the combining lane (the one holding the last data
// block, which also appends the length block) forms X = sum_l h_l r^(messages
// after span l) by Horner over the lanes, X <- X * r^(cnt_l) + h_l, with the
// powers in radix 2^26 (poly1305-donna-32 multiply, valid for any multiplier, not
// only a clamped r), then tag = X + s.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../neptun_amd/csrc/wg_crypto.h"
#include "neptun_gpu.h"

namespace {
using namespace wg;

constexpr uint32_t kThreads = 512;
constexpr uint32_t M26 = 0x3ffffffu;

struct F26 {
  uint32_t v[5];
};

__device__ __forceinline__ F26 f26_from32(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3, uint32_t h4) {
  F26 a;
  a.v[0] = h0 & M26;
  a.v[1] = ((h0 >> 26) | (h1 << 6)) & M26;
  a.v[2] = ((h1 >> 20) | (h2 << 12)) & M26;
  a.v[3] = ((h2 >> 14) | (h3 << 18)) & M26;
  a.v[4] = (h3 >> 8) | (h4 << 24);
  return a;
}

// a * b mod 2^130 - 5, limbs of the result < 2^26 (+ a small carry in limb 1)
__device__ __forceinline__ F26 f26_mul(const F26 &a, const F26 &b) {
  const uint32_t s1 = b.v[1] * 5u, s2 = b.v[2] * 5u, s3 = b.v[3] * 5u, s4 = b.v[4] * 5u;
  const uint64_t a0 = a.v[0], a1 = a.v[1], a2 = a.v[2], a3 = a.v[3], a4 = a.v[4];
  uint64_t d0 = a0 * b.v[0] + a1 * s4 + a2 * s3 + a3 * s2 + a4 * s1;
  uint64_t d1 = a0 * b.v[1] + a1 * b.v[0] + a2 * s4 + a3 * s3 + a4 * s2;
  uint64_t d2 = a0 * b.v[2] + a1 * b.v[1] + a2 * b.v[0] + a3 * s4 + a4 * s3;
  uint64_t d3 = a0 * b.v[3] + a1 * b.v[2] + a2 * b.v[1] + a3 * b.v[0] + a4 * s4;
  uint64_t d4 = a0 * b.v[4] + a1 * b.v[3] + a2 * b.v[2] + a3 * b.v[1] + a4 * b.v[0];
  F26 r;
  d1 += d0 >> 26;
  r.v[0] = (uint32_t)d0 & M26;
  d2 += d1 >> 26;
  r.v[1] = (uint32_t)d1 & M26;
  d3 += d2 >> 26;
  r.v[2] = (uint32_t)d2 & M26;
  d4 += d3 >> 26;
  r.v[3] = (uint32_t)d3 & M26;
  const uint64_t c = (d4 >> 26) * 5u + r.v[0];
  r.v[4] = (uint32_t)d4 & M26;
  r.v[0] = (uint32_t)c & M26;
  r.v[1] += (uint32_t)(c >> 26);
  return r;
}

// r^e for a wave-uniform e >= 1 (square and multiply, MSB first)
__device__ __forceinline__ F26 f26_pow(const F26 &r, uint32_t e) {
  F26 x = r;
  for (int bit = 30 - __builtin_clz(e); bit >= 0; --bit) {
    x = f26_mul(x, x);
    if ((e >> bit) & 1u) x = f26_mul(x, r);
  }
  return x;
}

// radix 2^26 -> Poly (radix 2^32) accumulator, fully carried (value < 2^130 + small)
__device__ __forceinline__ void f26_to_poly(F26 a, Poly &p) {
  a.v[1] += a.v[0] >> 26; a.v[0] &= M26;
  a.v[2] += a.v[1] >> 26; a.v[1] &= M26;
  a.v[3] += a.v[2] >> 26; a.v[2] &= M26;
  a.v[4] += a.v[3] >> 26; a.v[3] &= M26;
  a.v[0] += (a.v[4] >> 26) * 5u; a.v[4] &= M26;
  a.v[1] += a.v[0] >> 26; a.v[0] &= M26;
  p.h0 = a.v[0] | (a.v[1] << 26);
  p.h1 = (a.v[1] >> 6) | (a.v[2] << 20);
  p.h2 = (a.v[2] >> 12) | (a.v[3] << 14);
  p.h3 = (a.v[3] >> 18) | (a.v[4] << 8);
  p.h4 = a.v[4] >> 24;
}

// the packet's K lanes are consecutive lanes of one wave: lane 0 of the group
template <uint32_t K>
__device__ __forceinline__ uint32_t from_lane0(uint32_t x) {
  const int src = (int)((threadIdx.x & 63u) & ~(K - 1u));
  return (uint32_t)__shfl((int)x, src, 64);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint8_t *p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(uint8_t *p, uint4 v) {
  const u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(p));
}

struct Span {
  const uint8_t *in;
  uint8_t *out;
  uint32_t P;
  bool live;
};

// one 64-byte block b (>= 1) of data: the 16-byte pieces inside P (a prefix of the
// block's 4) are loaded, XORed with the keystream and stored; w keeps the
// ciphertext pieces (zero-padded past P) for Poly1305, nv = how many
__device__ __forceinline__ void load_block(const Span &sp, uint32_t b, uint4 (&x)[4]) {
  const uint32_t off = 64u * (b - 1u);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    x[q] = (b >= 1u && off + 16u * q < sp.P) ? ld_nt(sp.in + off + 16u * q) : make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ uint32_t crypt_block(const Span &sp, uint32_t b, const uint4 (&x)[4],
                                                const uint32_t (&ks)[16], uint32_t (&w)[4][4]) {
  const uint32_t off = 64u * (b - 1u);
  const uint32_t nv = (b < 1u || off >= sp.P) ? 0u : min(4u, (sp.P - off + 15u) / 16u);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    w[q][0] = x[q].x ^ ks[4 * q];
    w[q][1] = x[q].y ^ ks[4 * q + 1];
    w[q][2] = x[q].z ^ ks[4 * q + 2];
    w[q][3] = x[q].w ^ ks[4 * q + 3];
    if ((uint32_t)q >= nv) continue;
    const uint32_t o = off + 16u * q;
    const uint32_t valid = min(16u, sp.P - o);
    if (valid < 16u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) w[q][j] &= byte_mask((int)valid, j);
      if (sp.live) store_partial(sp.out + 16u + o, w[q], (int)valid);
    } else if (sp.live) {
      st_nt(sp.out + 16u + o, make_uint4(w[q][0], w[q][1], w[q][2], w[q][3]));
    }
  }
  return nv;
}

__device__ __forceinline__ void poly_pieces(Poly &ps, uint32_t &cnt, const uint32_t (&w)[4][4], uint32_t nv) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if ((uint32_t)q < nv) poly_block(ps, w[q][0], w[q][1], w[q][2], w[q][3]);
  cnt += nv;
}

template <uint32_t K>
__global__ __launch_bounds__(kThreads, 2) void xlane_seal_kernel(
    const uint8_t *__restrict__ src, uint64_t src_stride, uint8_t *__restrict__ dst, uint64_t dst_stride,
    uint32_t n, uint32_t P, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint32_t k4, uint32_t k5,
    uint32_t k6, uint32_t k7, uint32_t receiver, uint64_t ctr_base) {
  __shared__ uint32_t park[kThreads][6];  // each lane's h0..h4 and message count
  const uint32_t tid = threadIdx.x;
  const uint32_t l = tid % K;
  const uint32_t pk = (blockIdx.x * kThreads + tid) / K;
  const bool live = pk < n;
  const uint32_t pkc = live ? pk : n - 1u;  // lanes past the batch run packet n - 1, store nothing
  const uint64_t ctr = ctr_base + pkc;
  const uint32_t n1 = (uint32_t)ctr, n2 = (uint32_t)(ctr >> 32);
  const uint32_t key[8] = {k0, k1, k2, k3, k4, k5, k6, k7};
  const uint32_t NB = 1u + (P + 63u) / 64u;
  const uint32_t SPL = (NB + K - 1u) / K;
  const uint32_t b0 = l * SPL;
  const uint32_t last_lane = (NB - 1u) / SPL;
  const Span sp{src + (uint64_t)pkc * src_stride + 16u, dst + (uint64_t)pkc * dst_stride, P, live};

  Poly ps;
  uint32_t cnt = 0, s_key[4];
  // first pair: lane 0's block 0 is the Poly1305 key; every lane keeps its pair's
  // ciphertext until r has been broadcast from lane 0
  {
    uint4 xa[4], xb[4];
    load_block(sp, b0, xa);
    load_block(sp, b0 + 1u, xb);
    uint32_t ka[16], kb[16];
    chacha20_block2_sync(ka, kb, key, b0, n1, n2);
    uint32_t wa[4][4], wb[4][4];
    const uint32_t na = crypt_block(sp, b0, xa, ka, wa);
    const uint32_t nb = crypt_block(sp, b0 + 1u, xb, kb, wb);
    uint32_t rb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) rb[j] = from_lane0<K>(ka[j]);
    poly_init(ps, rb);
#pragma unroll
    for (int j = 0; j < 4; ++j) s_key[j] = rb[4 + j];
    poly_pieces(ps, cnt, wa, na);
    poly_pieces(ps, cnt, wb, nb);
  }
  // the rest of the span: pairs, then a single block when SPL is odd
  for (uint32_t t = 2; t + 1u < 2u * (SPL / 2u); t += 2) {
    uint4 xa[4], xb[4];
    load_block(sp, b0 + t, xa);
    load_block(sp, b0 + t + 1u, xb);
    uint32_t ka[16], kb[16];
    chacha20_block2_sync(ka, kb, key, b0 + t, n1, n2);
    uint32_t wa[4][4], wb[4][4];
    const uint32_t na = crypt_block(sp, b0 + t, xa, ka, wa);
    const uint32_t nb = crypt_block(sp, b0 + t + 1u, xb, kb, wb);
    poly_pieces(ps, cnt, wa, na);
    poly_pieces(ps, cnt, wb, nb);
  }
  if (SPL & 1u) {
    const uint32_t b = b0 + SPL - 1u;
    uint4 x[4];
    load_block(sp, b, x);
    uint32_t ks[16];
    chacha20_block_sync(ks, key, b, n1, n2);
    uint32_t w[4][4];
    poly_pieces(ps, cnt, w, crypt_block(sp, b, x, ks, w));
  }
  // the length block (AAD empty): le64(0) | le64(P), after the last data block
  if (l == last_lane) {
    poly_block(ps, 0u, 0u, P, 0u);
    ++cnt;
  }

  // combine the packet's K accumulators in the lane that holds the last block
  park[tid][0] = ps.h0; park[tid][1] = ps.h1; park[tid][2] = ps.h2; park[tid][3] = ps.h3;
  park[tid][4] = ps.h4; park[tid][5] = cnt;
  __syncthreads();
  if (l == last_lane) {
    const uint32_t base = tid - l;
    const F26 r26 = f26_from32(ps.r0, ps.r1, ps.r2, ps.r3, 0u);
    // lanes 1 .. last_lane - 1 each hold 4 * SPL messages (no tail): one power for all
    const F26 r_mid = f26_pow(r26, 4u * SPL);
    F26 x = f26_from32(park[base][0], park[base][1], park[base][2], park[base][3], park[base][4]);
    for (uint32_t j = 1; j <= last_lane; ++j) {
      const uint32_t c = park[base + j][5];
      const F26 rp = j < last_lane ? r_mid : f26_pow(r26, c);
      x = f26_mul(x, rp);
      const F26 h = f26_from32(park[base + j][0], park[base + j][1], park[base + j][2], park[base + j][3],
                               park[base + j][4]);
#pragma unroll
      for (int q = 0; q < 5; ++q) x.v[q] += h.v[q];
    }
    Poly fin;
    f26_to_poly(x, fin);
    uint32_t tag[4];
    poly_finish(fin, s_key, tag);
    if (live) {
      uint8_t *t = sp.out + 16u + P;
#pragma unroll
      for (int q = 0; q < 16; ++q) t[q] = (uint8_t)(tag[q / 4] >> (8 * (q % 4)));
    }
  }
  if (l == 0u && live) st_nt(sp.out, make_uint4(WG_MSG_DATA, receiver, n1, n2));
}

}  // namespace

extern "C" int xlane_seal(uint32_t K, const void *src, uint64_t src_stride, void *dst, uint64_t dst_stride,
                          uint32_t n, uint32_t P, const uint8_t key[32], uint32_t receiver, uint64_t ctr_base,
                          void *stream) {
  uint32_t k[8];
  for (int j = 0; j < 8; ++j)
    k[j] = (uint32_t)key[4 * j] | (uint32_t)key[4 * j + 1] << 8 | (uint32_t)key[4 * j + 2] << 16 |
           (uint32_t)key[4 * j + 3] << 24;
  const uint32_t NB = 1u + (P + 63u) / 64u;
  // every lane must own at least one whole pair, and the last block's lane must be the
  // last lane holding data (tools/proto_xlane.py keeps to P >= 128 K)
  if (n == 0 || P < 128u * K || (NB + K - 1u) / K < 2u) return 1;
  const uint64_t threads = (uint64_t)n * K;
  const dim3 grid((uint32_t)((threads + kThreads - 1) / kThreads));
  hipStream_t s = (hipStream_t)stream;
#define XL(KK)                                                                                          \
  hipLaunchKernelGGL(xlane_seal_kernel<KK>, grid, dim3(kThreads), 0, s, (const uint8_t *)src, src_stride, \
                     (uint8_t *)dst, dst_stride, n, P, k[0], k[1], k[2], k[3], k[4], k[5], k[6], k[7],      \
                     receiver, ctr_base)
  switch (K) {
    case 2: XL(2); break;
    case 4: XL(4); break;
    case 8: XL(8); break;
    default: return 2;
  }
#undef XL
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
