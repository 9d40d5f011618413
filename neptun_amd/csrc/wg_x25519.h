// wg_x25519.h -- X25519 (RFC 7748) for the handshake kernels, written once for
// the device (hipcc) and the host (g++: tests/test_handshake_cpu.py compiles it
// to check the arithmetic against oracle/handshake_model.py without a GPU, and
// oracle-independent CPU timing uses it as the "port" baseline).
//
// Field GF(2^255 - 19) in radix 2^25.5: ten signed limbs, even limbs 26 bits,
// odd limbs 25 bits (value = sum f_i 2^ceil(25.5 i)).  Products of two limbs
// fit an int64 with room for the ten-term sums (v_mad_i64_i32 on gfx950); the
// wrap 2^255 == 19 folds high terms with a factor 19, and a product of two odd
// limbs carries an extra factor 2 (25.5-bit radix).  One lane per scalar
// multiplication; the Montgomery ladder runs all 255 steps with branch-free
// conditional swaps.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define WG_HD __host__ __device__ __forceinline__
#else
#define WG_HD static inline
#endif

namespace wg {
namespace x25519 {

struct Fe {
  int32_t v[10];
};

WG_HD void fe_copy(Fe &h, const Fe &f) {
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i];
}
WG_HD void fe_set(Fe &h, int32_t x) {
  h.v[0] = x;
  for (int i = 1; i < 10; ++i) h.v[i] = 0;
}
WG_HD void fe_add(Fe &h, const Fe &f, const Fe &g) {
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}
WG_HD void fe_sub(Fe &h, const Fe &f, const Fe &g) {
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] - g.v[i];
}
// constant-time conditional swap (b = 0 or 1)
WG_HD void fe_cswap(Fe &f, Fe &g, int32_t b) {
  const int32_t m = -b;
  for (int i = 0; i < 10; ++i) {
    const int32_t x = (f.v[i] ^ g.v[i]) & m;
    f.v[i] ^= x;
    g.v[i] ^= x;
  }
}

// carry chain shared by mul / sq / mul_small: 64-bit limbs -> reduced 32-bit limbs
WG_HD void fe_carry(Fe &out, int64_t h[10]) {
  int64_t c;
#define WG_C(i, s)                                   \
  c = (h[i] + ((int64_t)1 << (s - 1))) >> s;         \
  h[i + 1] += c;                                     \
  h[i] -= c * ((int64_t)1 << s);
  WG_C(0, 26) WG_C(4, 26) WG_C(1, 25) WG_C(5, 25) WG_C(2, 26) WG_C(6, 26) WG_C(3, 25) WG_C(7, 25)
  WG_C(4, 26) WG_C(8, 26)
#undef WG_C
  c = (h[9] + ((int64_t)1 << 24)) >> 25;
  h[0] += c * 19;
  h[9] -= c * ((int64_t)1 << 25);
  c = (h[0] + ((int64_t)1 << 25)) >> 26;
  h[1] += c;
  h[0] -= c * ((int64_t)1 << 26);
  for (int i = 0; i < 10; ++i) out.v[i] = (int32_t)h[i];
}

// h = f * g: h_k = sum_{i+j = k (mod 10)} (2 if i, j odd) (19 if i+j >= 10) f_i g_j
WG_HD void fe_mul(Fe &out, const Fe &f, const Fe &g) {
  int32_t g19[10], f2[10];
  for (int i = 0; i < 10; ++i) {
    g19[i] = 19 * g.v[i];
    f2[i] = (i & 1) ? 2 * f.v[i] : f.v[i];
  }
  int64_t h[10];
  for (int k = 0; k < 10; ++k) h[k] = 0;
  for (int i = 0; i < 10; ++i)
    for (int j = 0; j < 10; ++j) {
      const int32_t a = (j & 1) ? f2[i] : f.v[i];  // the extra 2 only for odd i and odd j
      const int32_t b = (i + j >= 10) ? g19[j] : g.v[j];
      h[(i + j) % 10] += (int64_t)a * b;
    }
  fe_carry(out, h);
}

// h = f^2 (the symmetric half of fe_mul, cross terms doubled)
WG_HD void fe_sq(Fe &out, const Fe &f) {
  int32_t f19[10], f2[10];
  for (int i = 0; i < 10; ++i) {
    f19[i] = 19 * f.v[i];
    f2[i] = 2 * f.v[i];
  }
  int64_t h[10];
  for (int k = 0; k < 10; ++k) h[k] = 0;
  for (int i = 0; i < 10; ++i)
    for (int j = i; j < 10; ++j) {
      // coefficient: (i != j ? 2 : 1) * (odd*odd ? 2 : 1) * (i + j >= 10 ? 19 : 1)
      const bool oo = (i & 1) && (j & 1);
      int32_t a = (i != j) ? f2[i] : f.v[i];
      if (oo) a *= 2;
      const int32_t b = (i + j >= 10) ? f19[j] : f.v[j];
      h[(i + j) % 10] += (int64_t)a * b;
    }
  fe_carry(out, h);
}

WG_HD void fe_mul_small(Fe &out, const Fe &f, int32_t s) {
  int64_t h[10];
  for (int i = 0; i < 10; ++i) h[i] = (int64_t)f.v[i] * s;
  fe_carry(out, h);
}

WG_HD void fe_sqn(Fe &out, const Fe &f, int n) {
  fe_sq(out, f);
  for (int i = 1; i < n; ++i) fe_sq(out, out);
}

// z^(p-2) = z^(2^255 - 21)
WG_HD void fe_invert(Fe &out, const Fe &z) {
  Fe t0, t1, t2, t3;
  fe_sq(t0, z);                 // 2
  fe_sqn(t1, t0, 2);            // 8
  fe_mul(t1, z, t1);            // 9
  fe_mul(t0, t0, t1);           // 11
  fe_sq(t2, t0);                // 22
  fe_mul(t1, t1, t2);           // 2^5 - 1
  fe_sqn(t2, t1, 5);
  fe_mul(t1, t2, t1);           // 2^10 - 1
  fe_sqn(t2, t1, 10);
  fe_mul(t2, t2, t1);           // 2^20 - 1
  fe_sqn(t3, t2, 20);
  fe_mul(t2, t3, t2);           // 2^40 - 1
  fe_sqn(t2, t2, 10);
  fe_mul(t1, t2, t1);           // 2^50 - 1
  fe_sqn(t2, t1, 50);
  fe_mul(t2, t2, t1);           // 2^100 - 1
  fe_sqn(t3, t2, 100);
  fe_mul(t2, t3, t2);           // 2^200 - 1
  fe_sqn(t2, t2, 50);
  fe_mul(t1, t2, t1);           // 2^250 - 1
  fe_sqn(t1, t1, 5);            // 2^255 - 32
  fe_mul(out, t1, t0);          // 2^255 - 21
}

WG_HD uint32_t ld32le(const uint8_t *p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

// RFC 7748 decodeUCoordinate: little endian, bit 255 masked (values >= p are fine)
WG_HD void fe_frombytes(Fe &h, const uint32_t w[8]) {
  // bit offsets of limbs: 0, 26, 51, 77, 102, 128, 153, 179, 204, 230
  const int off[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
  const int bits[10] = {26, 25, 26, 25, 26, 25, 26, 25, 26, 25};
  for (int i = 0; i < 10; ++i) {
    const int o = off[i], q = o >> 5, r = o & 31;
    uint64_t x = w[q];
    if (q + 1 < 8) x |= (uint64_t)w[q + 1] << 32;
    x >>= r;
    uint32_t v = (uint32_t)x & ((1u << bits[i]) - 1u);
    if (i == 9) v &= (1u << 25) - 1u;  // bit 255 dropped
    h.v[i] = (int32_t)v;
  }
}

// canonical encoding (value mod p), 8 little-endian words
WG_HD void fe_tobytes(uint32_t w[8], const Fe &f) {
  int32_t h[10];
  for (int i = 0; i < 10; ++i) h[i] = f.v[i];
  // q = floor((h + 19) / 2^255) in {0, 1} for the carried input range
  int32_t q = (19 * h[9] + ((int32_t)1 << 24)) >> 25;
  for (int i = 0; i < 10; ++i) q = (h[i] + q) >> ((i & 1) ? 25 : 26);
  h[0] += 19 * q;
  for (int i = 0; i < 9; ++i) {
    const int s = (i & 1) ? 25 : 26;
    const int32_t c = h[i] >> s;
    h[i + 1] += c;
    h[i] -= c * ((int32_t)1 << s);
  }
  h[9] &= (1 << 25) - 1;
  const int off[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
  uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 10; ++i) {
    const int o = off[i], q2 = o >> 5, r = o & 31;
    const uint64_t x = (uint64_t)(uint32_t)h[i] << r;
    acc[q2] |= x & 0xffffffffu;
    if (q2 + 1 < 8) acc[q2 + 1] |= x >> 32;
  }
  for (int i = 0; i < 8; ++i) w[i] = (uint32_t)acc[i];
}

// RFC 7748 section 5: X25519(k, u); scalar and point as 8 little-endian words
WG_HD void scalarmult(uint32_t out[8], const uint32_t scalar[8], const uint32_t point[8]) {
  uint32_t k[8];
  for (int i = 0; i < 8; ++i) k[i] = scalar[i];
  k[0] &= ~7u;                  // clamp (decodeScalar25519)
  k[7] = (k[7] & 0x7fffffffu) | 0x40000000u;
  Fe x1, x2, z2, x3, z3, a, aa, b, bb, e, c, d, da, cb, t;
  fe_frombytes(x1, point);
  fe_set(x2, 1);
  fe_set(z2, 0);
  fe_copy(x3, x1);
  fe_set(z3, 1);
  int32_t swap = 0;
  for (int pos = 254; pos >= 0; --pos) {
    const int32_t kt = (int32_t)((k[pos >> 5] >> (pos & 31)) & 1u);
    swap ^= kt;
    fe_cswap(x2, x3, swap);
    fe_cswap(z2, z3, swap);
    swap = kt;
    fe_add(a, x2, z2);
    fe_sq(aa, a);
    fe_sub(b, x2, z2);
    fe_sq(bb, b);
    fe_sub(e, aa, bb);
    fe_add(c, x3, z3);
    fe_sub(d, x3, z3);
    fe_mul(da, d, a);
    fe_mul(cb, c, b);
    fe_add(t, da, cb);
    fe_sq(x3, t);
    fe_sub(t, da, cb);
    fe_sq(t, t);
    fe_mul(z3, x1, t);
    fe_mul(x2, aa, bb);
    fe_mul_small(t, e, 121665);
    fe_add(t, aa, t);
    fe_mul(z2, e, t);
  }
  fe_cswap(x2, x3, swap);
  fe_cswap(z2, z3, swap);
  fe_invert(z2, z2);
  fe_mul(x2, x2, z2);
  fe_tobytes(out, x2);
}

}  // namespace x25519
}  // namespace wg
