// field.h — secp256k1 arithmetic for gfx950, one field element per lane.
//
// Field F_p, p = 2^256 - 2^32 - 977 (btcec S256, the curve of
// src/crypto/keys/curve.go:20-22), held as 8 x 32-bit little-endian limbs in
// VGPRs.  Elements are kept *weakly reduced* (any value < 2^256 congruent to
// the element); fe_canon() gives the unique representative < p for
// comparisons.  Products use v_mad_u64_u32 (32x32+64 -> 64; ~31.8 T/s
// measured chip-wide, tools/ubench_int.hip) and carry chains lower to
// v_add_co/v_addc_co through __builtin_addc/__builtin_subc.  Reduction mod p
// folds the high half with 2^256 = 2^32 + 977 (pseudo-Mersenne), which is
// cheaper than Montgomery for this p.
//
// Scalars mod N (the group order, curve.go:13) use 8-limb Montgomery
// multiplication (R = 2^256): only ~20 of them run per verify (s^-1 via a
// batched Montgomery trick, u1, u2).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __host__ __device__ __forceinline__

struct fe {
  uint32_t v[8];
};

// p, little-endian limbs
#define P0 0xFFFFFC2Fu
#define P1 0xFFFFFFFEu
#define PX 0xFFFFFFFFu

DEV uint32_t addc32(uint32_t a, uint32_t b, uint32_t &c) {
  uint32_t co;
  uint32_t r = __builtin_addc(a, b, c, &co);
  c = co;
  return r;
}
DEV uint32_t subb32(uint32_t a, uint32_t b, uint32_t &br) {
  uint32_t bo;
  uint32_t r = __builtin_subc(a, b, br, &bo);
  br = bo;
  return r;
}

DEV void fe_set(fe &r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = 0;
}

DEV bool fe_is_zero_raw(const fe &a) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a.v[i];
  return x == 0;
}

// a >= p  (a < 2^256)
DEV bool fe_ge_p(const fe &a) {
  uint32_t hi = a.v[7] & a.v[6] & a.v[5] & a.v[4] & a.v[3] & a.v[2];
  if (hi != PX) return false;
  if (a.v[1] != P1) return a.v[1] > P1;
  return a.v[0] >= P0;
}

// Canonical representative in [0, p).
DEV void fe_canon(fe &a) {
  // a - p = a + c - 2^256 where c = 2^32 + 977; subtract p iff a >= p.
  uint32_t c = 0;
  fe t;
  t.v[0] = addc32(a.v[0], 977u, c);
  t.v[1] = addc32(a.v[1], 1u, c);
#pragma unroll
  for (int i = 2; i < 8; i++) t.v[i] = addc32(a.v[i], 0u, c);
  // carry out == 1  <=>  a + c >= 2^256  <=>  a >= p
  if (c) a = t;
}

DEV bool fe_is_zero(const fe &a) {  // a == 0 mod p
  fe t = a;
  fe_canon(t);
  return fe_is_zero_raw(t);
}

DEV bool fe_eq(const fe &a, const fe &b) {
  fe x = a, y = b;
  fe_canon(x);
  fe_canon(y);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d |= x.v[i] ^ y.v[i];
  return d == 0;
}

// r = a + b mod p (weak)
DEV void fe_add(fe &r, const fe &a, const fe &b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc32(a.v[i], b.v[i], c);
  // wrapped past 2^256: add 2^256 mod p = 2^32 + 977 (may wrap once more)
  uint32_t m = 0u - c;  // all-ones if carry
  uint32_t c2 = 0;
  r.v[0] = addc32(r.v[0], 977u & m, c2);
  r.v[1] = addc32(r.v[1], 1u & m, c2);
#pragma unroll
  for (int i = 2; i < 8; i++) r.v[i] = addc32(r.v[i], 0u, c2);
  if (c2) {  // astronomically rare: result was within 2^32+977 of 2^256
    uint32_t c3 = 0;
    r.v[0] = addc32(r.v[0], 977u, c3);
    r.v[1] = addc32(r.v[1], 1u, c3);
#pragma unroll
    for (int i = 2; i < 8; i++) r.v[i] = addc32(r.v[i], 0u, c3);
  }
}

// r = a - b mod p (weak)
DEV void fe_sub(fe &r, const fe &a, const fe &b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = subb32(a.v[i], b.v[i], br);
  // negative: add p == subtract (2^32 + 977) modulo 2^256
  uint32_t m = 0u - br;
  uint32_t b2 = 0;
  r.v[0] = subb32(r.v[0], 977u & m, b2);
  r.v[1] = subb32(r.v[1], 1u & m, b2);
#pragma unroll
  for (int i = 2; i < 8; i++) r.v[i] = subb32(r.v[i], 0u, b2);
  if (b2) {  // still negative (b > p and a < b - p): add p once more
    uint32_t b3 = 0;
    r.v[0] = subb32(r.v[0], 977u, b3);
    r.v[1] = subb32(r.v[1], 1u, b3);
#pragma unroll
    for (int i = 2; i < 8; i++) r.v[i] = subb32(r.v[i], 0u, b3);
  }
}

DEV void fe_neg(fe &r, const fe &a) {
  fe z;
  fe_set(z, 0);
  fe_sub(r, z, a);
}

// 256 x 256 -> 512, operand scanning; each step a*b + w + c <= 2^64 - 1.
DEV void mul_512(uint32_t w[16], const fe &a, const fe &b) {
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t t = (uint64_t)a.v[i] * b.v[j] + w[i + j] + c;
      w[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    w[i + 8] = (uint32_t)c;
  }
}

DEV void sqr_512(uint32_t w[16], const fe &a) {
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = 0;
  // cross products a_i a_j, i < j
#pragma unroll
  for (int i = 0; i < 7; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; j++) {
      uint64_t t = (uint64_t)a.v[i] * a.v[j] + w[i + j] + c;
      w[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    w[i + 8] = (uint32_t)c;
  }
  // double
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = addc32(w[i], w[i], c);
  // add diagonal squares
  c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t p = (uint64_t)a.v[i] * a.v[i];
    w[2 * i] = addc32(w[2 * i], (uint32_t)p, c);
    w[2 * i + 1] = addc32(w[2 * i + 1], (uint32_t)(p >> 32), c);
  }
}

// r = w mod p (weak), w < 2^512.  2^256 = 2^32 + 977 (mod p).
DEV void fe_reduce(fe &r, const uint32_t w[16]) {
  // m = H * 977  (9 limbs)
  uint32_t m[9];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t t = (uint64_t)w[8 + i] * 977u + c;
    m[i] = (uint32_t)t;
    c = t >> 32;
  }
  m[8] = (uint32_t)c;
  // t = L + m + (H << 32)
  uint32_t t[9];
  uint32_t cc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = addc32(w[i], m[i], cc);
  t[8] = m[8] + cc;  // m[8] < 977, no overflow
  cc = 0;
  t[1] = addc32(t[1], w[8], cc);
#pragma unroll
  for (int i = 2; i < 9; i++) t[i] = addc32(t[i], w[7 + i], cc);
  // t[8] <= 2^32 - 1 + 977 + carry : cc can only be set if t[8] wrapped;
  // fold hi = t[8] + cc*2^32 (as a 64-bit value) once more.
  // Y = hi * (2^32 + 977) as three limbs (hi < 2^33 so Y < 2^66)
  uint64_t hi = (uint64_t)t[8] + ((uint64_t)cc << 32);
  uint64_t y = hi * 977u;
  uint64_t rest = (y >> 32) + hi;
  uint32_t c2 = 0;
  r.v[0] = addc32(t[0], (uint32_t)y, c2);
  r.v[1] = addc32(t[1], (uint32_t)rest, c2);
  r.v[2] = addc32(t[2], (uint32_t)(rest >> 32), c2);
#pragma unroll
  for (int i = 3; i < 8; i++) r.v[i] = addc32(t[i], 0u, c2);
  if (c2) {  // rare: wrapped past 2^256 again; the remainder is tiny
    uint32_t c4 = 0;
    r.v[0] = addc32(r.v[0], 977u, c4);
    r.v[1] = addc32(r.v[1], 1u, c4);
#pragma unroll
    for (int i = 2; i < 8; i++) r.v[i] = addc32(r.v[i], 0u, c4);
  }
}

DEV void fe_mul(fe &r, const fe &a, const fe &b) {
  uint32_t w[16];
  mul_512(w, a, b);
  fe_reduce(r, w);
}
DEV void fe_sqr(fe &r, const fe &a) {
  uint32_t w[16];
  sqr_512(w, a);
  fe_reduce(r, w);
}

// small multiples (for 2x, 3x, 8x in point formulas)
DEV void fe_dbl(fe &r, const fe &a) { fe_add(r, a, a); }

// a^(p-2): standard addition chain, 255 S + 15 M
DEV void fe_sqrn(fe &r, const fe &a, int n) {
  r = a;
  for (int i = 0; i < n; i++) fe_sqr(r, r);
}
DEV void fe_inv(fe &r, const fe &a) {
  fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fe_sqr(x2, a);
  fe_mul(x2, x2, a);
  fe_sqr(x3, x2);
  fe_mul(x3, x3, a);
  fe_sqrn(x6, x3, 3);
  fe_mul(x6, x6, x3);
  fe_sqrn(x9, x6, 3);
  fe_mul(x9, x9, x3);
  fe_sqrn(x11, x9, 2);
  fe_mul(x11, x11, x2);
  fe_sqrn(x22, x11, 11);
  fe_mul(x22, x22, x11);
  fe_sqrn(x44, x22, 22);
  fe_mul(x44, x44, x22);
  fe_sqrn(x88, x44, 44);
  fe_mul(x88, x88, x44);
  fe_sqrn(x176, x88, 88);
  fe_mul(x176, x176, x88);
  fe_sqrn(x220, x176, 44);
  fe_mul(x220, x220, x44);
  fe_sqrn(x223, x220, 3);
  fe_mul(x223, x223, x3);
  fe_sqrn(t, x223, 23);
  fe_mul(t, t, x22);
  fe_sqrn(t, t, 5);
  fe_mul(t, t, a);
  fe_sqrn(t, t, 3);
  fe_mul(t, t, x2);
  fe_sqrn(t, t, 2);
  fe_mul(r, t, a);
}

// ---------------------------------------------------------------------------
// Scalars mod N (Montgomery, R = 2^256)
// ---------------------------------------------------------------------------
struct sc {
  uint32_t v[8];
};

static constexpr uint32_t SC_N[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                                                          0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
// R^2 mod N
static constexpr uint32_t SC_R2[8] = {0x67D7D140u, 0x896CF214u, 0x0E7CF878u, 0x741496C2u,
                                                           0x5BCD07C6u, 0xE697F5E4u, 0x81C69BC5u, 0x9D671CD5u};
// R mod N  (Montgomery one)
static constexpr uint32_t SC_R1[8] = {0x2FC9BEBFu, 0x402DA173u, 0x50B75FC4u, 0x45512319u,
                                                           0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u};
#define SC_NINV 0x5588B13Fu  // -N^-1 mod 2^32

DEV bool sc_ge_n(const sc &a) {
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    if (a.v[i] != SC_N[i]) return a.v[i] > SC_N[i];
  }
  return true;
}
DEV void sc_sub_n(sc &a) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) a.v[i] = subb32(a.v[i], SC_N[i], br);
}

// r = a * b * R^-1 mod N; requires a*b < N*R (true when a < R, b < N).
DEV void sc_mont(sc &r, const sc &a, const sc &b) {
  uint32_t t[10];
#pragma unroll
  for (int i = 0; i < 10; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    // t += a_i * b
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t x = (uint64_t)a.v[i] * b.v[j] + t[j] + c;
      t[j] = (uint32_t)x;
      c = x >> 32;
    }
    uint32_t cc = 0;
    t[8] = addc32(t[8], (uint32_t)c, cc);
    t[9] = cc;
    // t += m * N, m = t0 * (-N^-1) mod 2^32; then t >>= 32
    uint32_t m = t[0] * SC_NINV;
    c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t x = (uint64_t)m * SC_N[j] + t[j] + c;
      t[j] = (uint32_t)x;
      c = x >> 32;
    }
    cc = 0;
    t[8] = addc32(t[8], (uint32_t)c, cc);
    t[9] += cc;
#pragma unroll
    for (int j = 0; j < 9; j++) t[j] = t[j + 1];
    t[9] = 0;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  if (t[8] || sc_ge_n(r)) sc_sub_n(r);
}

DEV void sc_load_const(sc &r, const uint32_t *c) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
}

// r = a + b mod N (a, b < N)
DEV void sc_add(sc &r, const sc &a, const sc &b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc32(a.v[i], b.v[i], c);
  if (c || sc_ge_n(r)) sc_sub_n(r);
}
// r = a - b mod N (a, b < N)
DEV void sc_sub(sc &r, const sc &a, const sc &b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = subb32(a.v[i], b.v[i], br);
  if (br) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = addc32(r.v[i], SC_N[i], c);
  }
}

// ---------------------------------------------------------------------------
// GLV endomorphism of secp256k1: lambda * (x, y) = (beta * x, y).
// k = k1 + k2 * lambda (mod N) with |k1|, |k2| < 2^128 (the lattice split of
// Gallant-Lambert-Vanstone; constants checked in tests/test_emu.py).
// ---------------------------------------------------------------------------
static constexpr uint32_t FE_BETA[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u,
                                        0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};
// round(2^384 * b2 / N), round(2^384 * (-b1) / N)
static constexpr uint32_t GLV_G1[8] = {0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u,
                                       0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};
static constexpr uint32_t GLV_G2[8] = {0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu,
                                       0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};
// -b1 * R, -b2 * R, lambda * R (mod N): Montgomery forms for sc_mont
static constexpr uint32_t GLV_MB1R[8] = {0x0AD9263Cu, 0xC50468D0u, 0xFAA6ED42u, 0x1B1C8205u,
                                         0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu};
static constexpr uint32_t GLV_MB2R[8] = {0x6A144696u, 0x0CAC5E50u, 0xF3BA5939u, 0x1E8A8DC5u,
                                         0xBA244FCEu, 0x176CDF65u, 0x8E173580u, 0xC25575EBu};
static constexpr uint32_t GLV_LAMR[8] = {0xC9926C9Eu, 0xF07DEB3Du, 0x83C6944Cu, 0x2C93E7ADu,
                                         0x52697D91u, 0x73A96606u, 0x8558D639u, 0x53284017u};
// (N - 1) / 2
static constexpr uint32_t SC_HALF_N[8] = {0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u,
                                          0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};

// round(k * g / 2^384) for 256-bit k, g (result < 2^129)
DEV void glv_mulshift(sc &c, const sc &k, const uint32_t *g) {
  fe a, b;
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.v[i] = k.v[i];
    b.v[i] = g[i];
  }
  mul_512(w, a, b);
  uint32_t cy = w[11] >> 31;  // rounding bit (bit 383)
#pragma unroll
  for (int i = 0; i < 4; i++) c.v[i] = addc32(w[12 + i], 0u, cy);
  c.v[4] = cy;
#pragma unroll
  for (int i = 5; i < 8; i++) c.v[i] = 0;
}

// k -> (|k1|, |k2|) as 128-bit magnitudes (4 limbs each) and sign bits
// (bit 0: k1 negative, bit 1: k2 negative), k = k1 + k2 lambda (mod N).
DEV void glv_split(uint32_t mag1[4], uint32_t mag2[4], uint32_t &signs, const sc &k) {
  sc c1, c2, t, r1, r2, mb;
  glv_mulshift(c1, k, GLV_G1);
  glv_mulshift(c2, k, GLV_G2);
  sc_load_const(mb, GLV_MB1R);
  sc_mont(c1, c1, mb);  // c1 * (-b1) mod N
  sc_load_const(mb, GLV_MB2R);
  sc_mont(c2, c2, mb);  // c2 * (-b2) mod N
  sc_add(r2, c1, c2);
  sc_load_const(mb, GLV_LAMR);
  sc_mont(t, r2, mb);   // r2 * lambda mod N
  sc_sub(r1, k, t);
  signs = 0;
  sc h;
  sc_load_const(h, SC_HALF_N);
  sc n;
  sc_load_const(n, SC_N);
  // r > (N-1)/2 -> negative: magnitude N - r
  bool gt1 = false, gt2 = false;
  {
    bool decided = false;
#pragma unroll
    for (int i = 7; i >= 0; i--) {
      if (!decided && r1.v[i] != h.v[i]) {
        gt1 = r1.v[i] > h.v[i];
        decided = true;
      }
    }
    decided = false;
#pragma unroll
    for (int i = 7; i >= 0; i--) {
      if (!decided && r2.v[i] != h.v[i]) {
        gt2 = r2.v[i] > h.v[i];
        decided = true;
      }
    }
  }
  if (gt1) {
    sc z;
    sc_sub(z, n, r1);
    r1 = z;
    signs |= 1u;
  }
  if (gt2) {
    sc z;
    sc_sub(z, n, r2);
    r2 = z;
    signs |= 2u;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    mag1[i] = r1.v[i];
    mag2[i] = r2.v[i];
  }
}
