// wg_aead.hip -- MI355X (gfx950 / CDNA4) WireGuard transport-data AEAD.
//
// Hand-written HIP for NepTUN's per-packet ChaCha20-Poly1305 seal/open:
//   seal = Session::format_packet_data   (neptun/src/noise/session.rs:205-259)
//   open = parse_incoming_packet DATA arm (noise/mod.rs:139-199) +
//          Session::receive_packet_data  (session.rs:265-302, replay window on host)
// The AEAD is RFC 8439 (what ring 0.17.14's CHACHA20_POLY1305 computes).
//
// Execution model (DESIGN.md "Kernels"):
//   * one packet per wavefront lane; a wave64 works on 64 packets in lockstep,
//     so for a uniform batch every branch below is wave-uniform;
//   * the 16 ChaCha20 state words live in VGPRs (single-key batches keep the
//     key in SGPRs), one 64-byte keystream block per loop trip;
//   * data moves as 16-byte global_load/store_dwordx4 (4 per 64-byte block);
//   * Poly1305 runs per lane in radix 2^32 (4 x 32-bit limbs + a 3-bit top
//     limb) on v_mad_u64_u32 chains: measured on MI355X, v_mad_u64_u32 issues at
//     the same rate as v_alignbit_b32 (tools/microbench_valu.hip), so 20 mads
//     per 16-byte block beat radix 2^26 (25 mads + limb splitting);
//   * the nonce is 0^4 | LE64(counter); in the strided form the counter is
//     counter_base + packet index (derived from the lane index).
// No MFMA: this is a stream cipher + MAC, not a contraction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "neptun_gpu.h"
#include "wg_aead_kernels.h"

namespace wg {

// ---------------------------------------------------------------------------
// ChaCha20 (RFC 8439 2.3)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, 32u - n);  // v_alignbit_b32: 1 VALU op
}

#define WG_QR(a, b, c, d)                   \
  a += b; d ^= a; d = rotl(d, 16);          \
  c += d; b ^= c; b = rotl(b, 12);          \
  a += b; d ^= a; d = rotl(d, 8);           \
  c += d; b ^= c; b = rotl(b, 7);

constexpr uint32_t kSigma0 = 0x61707865u, kSigma1 = 0x3320646eu, kSigma2 = 0x79622d32u,
                   kSigma3 = 0x6b206574u;

// Keystream block `blk` for key k[8] and nonce (0, n1, n2) -- WireGuard's nonce
// is 4 zero bytes then LE64(counter) (session.rs:230-235), so word 13 is 0.
__device__ __forceinline__ void chacha20_block(uint32_t ks[16], const uint32_t k[8], uint32_t blk,
                                               uint32_t n1, uint32_t n2) {
  uint32_t x0 = kSigma0, x1 = kSigma1, x2 = kSigma2, x3 = kSigma3;
  uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3];
  uint32_t x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
  uint32_t x12 = blk, x13 = 0, x14 = n1, x15 = n2;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    WG_QR(x0, x4, x8, x12) WG_QR(x1, x5, x9, x13) WG_QR(x2, x6, x10, x14) WG_QR(x3, x7, x11, x15)
    WG_QR(x0, x5, x10, x15) WG_QR(x1, x6, x11, x12) WG_QR(x2, x7, x8, x13) WG_QR(x3, x4, x9, x14)
  }
  ks[0] = x0 + kSigma0; ks[1] = x1 + kSigma1; ks[2] = x2 + kSigma2; ks[3] = x3 + kSigma3;
  ks[4] = x4 + k[0]; ks[5] = x5 + k[1]; ks[6] = x6 + k[2]; ks[7] = x7 + k[3];
  ks[8] = x8 + k[4]; ks[9] = x9 + k[5]; ks[10] = x10 + k[6]; ks[11] = x11 + k[7];
  ks[12] = x12 + blk; ks[13] = x13; ks[14] = x14 + n1; ks[15] = x15 + n2;
}

// ---------------------------------------------------------------------------
// Poly1305 (RFC 8439 2.5), radix 2^32: h = h0..h3 (32-bit) + h4 (< 8)
// ---------------------------------------------------------------------------
struct Poly {
  uint32_t h0, h1, h2, h3, h4;
  uint32_t r0, r1, r2, r3;  // clamped r
  uint32_t s1, s2, s3;      // 5*r_i/4 (r1..r3 are multiples of 4)
};

__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * b + c;  // v_mad_u64_u32
}

__device__ __forceinline__ void poly_init(Poly &p, const uint32_t ks0[8]) {
  p.r0 = ks0[0] & 0x0fffffffu;
  p.r1 = ks0[1] & 0x0ffffffcu;
  p.r2 = ks0[2] & 0x0ffffffcu;
  p.r3 = ks0[3] & 0x0ffffffcu;
  p.s1 = p.r1 + (p.r1 >> 2);
  p.s2 = p.r2 + (p.r2 >> 2);
  p.s3 = p.r3 + (p.r3 >> 2);
  p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0;
}

// h = (h + m + 2^128) * r  (partially reduced mod 2^130 - 5)
__device__ __forceinline__ void poly_block(Poly &p, uint32_t m0, uint32_t m1, uint32_t m2,
                                           uint32_t m3) {
  uint64_t t = (uint64_t)p.h0 + m0;
  const uint32_t h0 = (uint32_t)t;
  t = (uint64_t)p.h1 + m1 + (t >> 32);
  const uint32_t h1 = (uint32_t)t;
  t = (uint64_t)p.h2 + m2 + (t >> 32);
  const uint32_t h2 = (uint32_t)t;
  t = (uint64_t)p.h3 + m3 + (t >> 32);
  const uint32_t h3 = (uint32_t)t;
  uint32_t h4 = p.h4 + (uint32_t)(t >> 32) + 1u;  // + 2^128 (full 16-byte block)
  // d_j = sum_i h_i r_{j-i} with 2^128 == 5/4 folding (h_i r_j, i+j >= 4 -> h_i s_j)
  const uint64_t d0 = mad(h3, p.s1, mad(h2, p.s2, mad(h1, p.s3, (uint64_t)h0 * p.r0)));
  const uint64_t d1 =
      mad(h4, p.s1, mad(h3, p.s2, mad(h2, p.s3, mad(h1, p.r0, mad(h0, p.r1, d0 >> 32)))));
  const uint64_t d2 =
      mad(h4, p.s2, mad(h3, p.s3, mad(h2, p.r0, mad(h1, p.r1, mad(h0, p.r2, d1 >> 32)))));
  const uint64_t d3 =
      mad(h4, p.s3, mad(h3, p.r0, mad(h2, p.r1, mad(h1, p.r2, mad(h0, p.r3, d2 >> 32)))));
  h4 = h4 * p.r0 + (uint32_t)(d3 >> 32);
  // fold bits >= 130: c = 5 * (h4 >> 2)
  const uint32_t c = (h4 >> 2) + (h4 & ~3u);
  h4 &= 3u;
  t = (uint64_t)(uint32_t)d0 + c;
  p.h0 = (uint32_t)t;
  t = (uint64_t)(uint32_t)d1 + (t >> 32);
  p.h1 = (uint32_t)t;
  t = (uint64_t)(uint32_t)d2 + (t >> 32);
  p.h2 = (uint32_t)t;
  t = (uint64_t)(uint32_t)d3 + (t >> 32);
  p.h3 = (uint32_t)t;
  p.h4 = h4 + (uint32_t)(t >> 32);
}

// tag = (h mod p) + s mod 2^128; h < 5*2^128 < 2p so one conditional subtract
__device__ __forceinline__ void poly_finish(const Poly &p, const uint32_t s[4], uint32_t tag[4]) {
  uint64_t t = (uint64_t)p.h0 + 5u;
  const uint32_t g0 = (uint32_t)t;
  t = (uint64_t)p.h1 + (t >> 32);
  const uint32_t g1 = (uint32_t)t;
  t = (uint64_t)p.h2 + (t >> 32);
  const uint32_t g2 = (uint32_t)t;
  t = (uint64_t)p.h3 + (t >> 32);
  const uint32_t g3 = (uint32_t)t;
  const uint32_t g4 = p.h4 + (uint32_t)(t >> 32);
  const bool ge = (g4 >> 2) != 0u;  // h + 5 >= 2^130  <=>  h >= p
  const uint32_t f0 = ge ? g0 : p.h0, f1 = ge ? g1 : p.h1, f2 = ge ? g2 : p.h2,
                 f3 = ge ? g3 : p.h3;
  t = (uint64_t)f0 + s[0];
  tag[0] = (uint32_t)t;
  t = (uint64_t)f1 + s[1] + (t >> 32);
  tag[1] = (uint32_t)t;
  t = (uint64_t)f2 + s[2] + (t >> 32);
  tag[2] = (uint32_t)t;
  tag[3] = f3 + s[3] + (uint32_t)(t >> 32);
}

// ---------------------------------------------------------------------------
// byte-granular helpers for the packet tail (run once per packet)
// ---------------------------------------------------------------------------
// mask of the valid low bytes of word j when `valid` bytes of a 16-byte chunk are live
__device__ __forceinline__ uint32_t byte_mask(int valid, int j) {
  const int v = valid - 4 * j;
  return v >= 4 ? 0xffffffffu : (v <= 0 ? 0u : ((1u << (8 * v)) - 1u));
}

// select word idx (runtime, may be out of [0,n)) of w[n], 0 outside
template <int N>
__device__ __forceinline__ uint32_t pick(const uint32_t (&w)[N], int idx) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) r = (idx == j) ? w[j] : r;
  return r;
}

// 4 bytes of the little-endian stream w[] starting at byte offset `off` (off may be < 0)
template <int N>
__device__ __forceinline__ uint32_t bytes_at(const uint32_t (&w)[N], int off) {
  const int q = off >> 2;  // floor division (arithmetic shift)
  const uint32_t b = (uint32_t)(off & 3);
  return __builtin_amdgcn_alignbyte(pick(w, q + 1), pick(w, q), b);
}

// store the first k (1..15) bytes of a 16-byte-aligned chunk
__device__ __forceinline__ void store_partial(uint8_t *p, const uint32_t w[4], int k) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int v = k - 4 * j;
    if (v >= 4) {
      *reinterpret_cast<uint32_t *>(p + 4 * j) = w[j];
    } else if (v > 0) {
      uint8_t *pb = p + 4 * j;
      if (v >= 2) {
        *reinterpret_cast<uint16_t *>(pb) = (uint16_t)w[j];
        if (v == 3) pb[2] = (uint8_t)(w[j] >> 16);
      } else {
        pb[0] = (uint8_t)w[j];
      }
    }
  }
}

__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
  return *reinterpret_cast<const uint4 *>(p);
}
__device__ __forceinline__ void st16(uint8_t *p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  *reinterpret_cast<uint4 *>(p) = make_uint4(a, b, c, d);
}

// ---------------------------------------------------------------------------
// one packet, one lane
// ---------------------------------------------------------------------------
// body = plaintext (seal: in, open: out) / ciphertext (seal: out, open: in)
// Returns the per-packet status.
template <bool kSeal>
__device__ __forceinline__ int32_t process_packet(const uint8_t *in, uint8_t *out,
                                                  const uint32_t key[8], uint32_t sess_index,
                                                  uint64_t counter_in, uint32_t len) {
  uint64_t counter = counter_in;
  uint32_t body_len;  // P
  const uint8_t *body_in;
  uint8_t *body_out;
  if (kSeal) {
    body_len = len;
    body_in = in;
    body_out = out + WG_DATA_OFFSET;
    // header: LE32 DATA | LE32 sending_index | LE64 counter  (session.rs:221-227)
    st16(out, WG_MSG_DATA, sess_index, (uint32_t)counter, (uint32_t)(counter >> 32));
  } else {
    // parse_incoming_packet DATA arm (noise/mod.rs:139-199): type 4, len >= 32
    if (len < WG_DATA_OVERHEAD_SZ) return WG_STATUS_INVALID_PACKET;
    const uint4 hdr = ld16(in);
    if (hdr.x != WG_MSG_DATA) return WG_STATUS_INVALID_PACKET;
    // receive_packet_data: receiver_idx == receiving_index (session.rs:275-277)
    if (hdr.y != sess_index) return WG_STATUS_WRONG_INDEX;
    counter = (uint64_t)hdr.z | ((uint64_t)hdr.w << 32);
    body_len = len - WG_DATA_OVERHEAD_SZ;
    body_in = in + WG_DATA_OFFSET;
    body_out = out;
  }
  const uint32_t n1 = (uint32_t)counter, n2 = (uint32_t)(counter >> 32);

  // Poly1305 one-time key = keystream block 0 (RFC 8439 2.6)
  Poly p;
  uint32_t s[4];
  {
    uint32_t ks[16];
    chacha20_block(ks, key, 0u, n1, n2);
    poly_init(p, ks);
    s[0] = ks[4]; s[1] = ks[5]; s[2] = ks[6]; s[3] = ks[7];
  }

  const uint32_t nfull = body_len >> 6;  // whole 64-byte keystream blocks
  for (uint32_t b = 0; b < nfull; ++b) {
    const uint8_t *ip = body_in + 64u * b;
    uint8_t *op = body_out + 64u * b;
    const uint4 c0 = ld16(ip), c1 = ld16(ip + 16), c2 = ld16(ip + 32), c3 = ld16(ip + 48);
    uint32_t ks[16];
    chacha20_block(ks, key, b + 1u, n1, n2);
    const uint32_t o0 = c0.x ^ ks[0], o1 = c0.y ^ ks[1], o2 = c0.z ^ ks[2], o3 = c0.w ^ ks[3];
    const uint32_t o4 = c1.x ^ ks[4], o5 = c1.y ^ ks[5], o6 = c1.z ^ ks[6], o7 = c1.w ^ ks[7];
    const uint32_t o8 = c2.x ^ ks[8], o9 = c2.y ^ ks[9], o10 = c2.z ^ ks[10], o11 = c2.w ^ ks[11];
    const uint32_t o12 = c3.x ^ ks[12], o13 = c3.y ^ ks[13], o14 = c3.z ^ ks[14],
                   o15 = c3.w ^ ks[15];
    st16(op, o0, o1, o2, o3);
    st16(op + 16, o4, o5, o6, o7);
    st16(op + 32, o8, o9, o10, o11);
    st16(op + 48, o12, o13, o14, o15);
    if (kSeal) {  // MAC the ciphertext
      poly_block(p, o0, o1, o2, o3);
      poly_block(p, o4, o5, o6, o7);
      poly_block(p, o8, o9, o10, o11);
      poly_block(p, o12, o13, o14, o15);
    } else {
      poly_block(p, c0.x, c0.y, c0.z, c0.w);
      poly_block(p, c1.x, c1.y, c1.z, c1.w);
      poly_block(p, c2.x, c2.y, c2.z, c2.w);
      poly_block(p, c3.x, c3.y, c3.z, c3.w);
    }
  }

  // last, partial keystream block (1..63 bytes)
  const int rem = (int)(body_len & 63u);
  const int k = (int)(body_len & 15u);        // bytes in the partial 16-byte chunk
  const uint32_t tail_off = body_len & ~15u;  // offset of that chunk (or of the tag if k == 0)
  uint32_t tail_in[4] = {0, 0, 0, 0};         // input bytes of the partial chunk (masked)
  uint32_t tail_out[4] = {0, 0, 0, 0};        // output bytes of the partial chunk (masked)
  if (rem) {
    uint32_t ks[16];
    chacha20_block(ks, key, nfull + 1u, n1, n2);
    const uint8_t *ip = body_in + 64u * nfull;
    uint8_t *op = body_out + 64u * nfull;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int valid = rem - 16 * c;
      if (valid > 0) {
        const uint4 v = ld16(ip + 16 * c);  // aligned 16-byte chunk: over-read stays in it
        uint32_t iw[4] = {v.x, v.y, v.z, v.w}, ow[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t m = byte_mask(valid, j);
          iw[j] &= m;
          ow[j] = (iw[j] ^ ks[4 * c + j]) & m;
        }
        if (valid >= 16) {
          st16(op + 16 * c, ow[0], ow[1], ow[2], ow[3]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) { tail_in[j] = iw[j]; tail_out[j] = ow[j]; }
        }
        // AEAD pad16: the zero-padded chunk is MACed as a full block
        if (kSeal) poly_block(p, ow[0], ow[1], ow[2], ow[3]);
        else poly_block(p, iw[0], iw[1], iw[2], iw[3]);
      }
    }
  }
  // LE64(aad_len = 0) | LE64(ct_len)   (RFC 8439 2.8)
  poly_block(p, 0u, 0u, body_len, 0u);
  uint32_t tag[4];
  poly_finish(p, s, tag);

  if (kSeal) {
    // tail region at ct + tail_off: k ciphertext bytes then the 16-byte tag
    uint8_t *tp = body_out + tail_off;
    const uint32_t r[8] = {tail_out[0], tail_out[1], tail_out[2], tail_out[3], 0, 0, 0, 0};
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = r[j] | bytes_at(tag, 4 * j - k);
    st16(tp, w[0], w[1], w[2], w[3]);
    if (k) store_partial(tp + 16, &w[4], k);
    return WG_STATUS_OK;
  }

  // open: the received tag sits at ct + body_len (k bytes into the tail chunk)
  const uint8_t *tp = body_in + tail_off;
  uint32_t rx[8];
  if (k) {
    // tail_in holds only the k ciphertext bytes; the chunk (L1/L2-hot) carries tag bytes too
    const uint4 lo = ld16(tp), hi = ld16(tp + 16);
    rx[0] = lo.x; rx[1] = lo.y; rx[2] = lo.z; rx[3] = lo.w;
    rx[4] = hi.x; rx[5] = hi.y; rx[6] = hi.z; rx[7] = hi.w;
  } else {
    const uint4 lo = ld16(tp);
    rx[0] = lo.x; rx[1] = lo.y; rx[2] = lo.z; rx[3] = lo.w;
    rx[4] = rx[5] = rx[6] = rx[7] = 0;
  }
  uint32_t diff = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) diff |= bytes_at(rx, k + 4 * j) ^ tag[j];
  if (diff == 0u) {
    if (k) store_partial(body_out + tail_off, tail_out, k);
    return WG_STATUS_OK;
  }
  // tag mismatch: never expose unauthenticated plaintext (ring open_within zeroes it)
  for (uint32_t off = 0; off + 16u <= body_len; off += 16u) st16(body_out + off, 0, 0, 0, 0);
  if (k) {
    const uint32_t z[4] = {0, 0, 0, 0};
    store_partial(body_out + tail_off, z, k);
  }
  return WG_STATUS_INVALID_AEAD_TAG;
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_key(const uint8_t *keys, uint32_t slot, uint32_t k[8]) {
  const uint4 a = ld16(keys + 32u * slot), b = ld16(keys + 32u * slot + 16u);
  k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w;
  k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
}

template <bool kSeal>
__global__ __launch_bounds__(kBlockThreads) void aead_strided_kernel(StridedParams prm) {
  const uint32_t i = blockIdx.x * kBlockThreads + threadIdx.x;
  if (i >= prm.n) return;
  // single session: key and index are wave-uniform (scalar loads, SGPRs)
  uint32_t key[8];
  load_key(prm.keys, prm.key_slot, key);
  const uint32_t sidx = prm.key_index[prm.key_slot];
  const uint8_t *in = prm.src + (uint64_t)i * prm.src_stride;
  uint8_t *out = prm.dst + (uint64_t)i * prm.dst_stride;
  const int32_t st =
      process_packet<kSeal>(in, out, key, sidx, prm.counter_base + i, prm.len);
  if (prm.status) prm.status[i] = st;
}

template <bool kSeal>
__global__ __launch_bounds__(kBlockThreads) void aead_desc_kernel(DescParams prm) {
  const uint32_t i = blockIdx.x * kBlockThreads + threadIdx.x;
  if (i >= prm.n) return;
  const wg_packet_desc d = prm.descs[i];
  int32_t st;
  if (d.key_slot >= prm.key_slots) {
    st = WG_STATUS_BAD_KEY_SLOT;
  } else if (((d.src_off | d.dst_off) & 15u) != 0u) {
    st = WG_STATUS_MISALIGNED;
  } else {
    uint32_t key[8];
    load_key(prm.keys, d.key_slot, key);
    const uint32_t sidx = prm.key_index[d.key_slot];
    st = process_packet<kSeal>(prm.src + d.src_off, prm.dst + d.dst_off, key, sidx, d.counter,
                               d.len);
  }
  prm.status[i] = st;
}

template __global__ void aead_strided_kernel<true>(StridedParams);
template __global__ void aead_strided_kernel<false>(StridedParams);
template __global__ void aead_desc_kernel<true>(DescParams);
template __global__ void aead_desc_kernel<false>(DescParams);

}  // namespace wg
