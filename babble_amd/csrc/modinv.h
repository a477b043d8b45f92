// modinv.h — variable-time modular inversion by Bernstein–Yang divsteps
// ("safegcd", https://gcd.cr.yp.to) for the two moduli of the verify path:
// p (field, point normalisation in the table builders) and N (group order,
// the batched s^-1 of ecdsa.Verify step 5).
//
// Why: Fermat inversion is a serial chain of ~270 dependent 256-bit
// multiplications (~0.2 ms of latency on one gfx950 lane).  Every
// inversion on this path sits on a critical latency chain — one lane per
// block inverts the block's product (k_table_fill / k_table_pair), one lane
// per 16 items inverts in k_sinv — so latency, not throughput, is what
// matters, and divsteps on 32-bit words plus 20-odd 2x2 matrix
// applications to 9-limb numbers are ~10x shorter.  Variable time is fine:
// every operand is public (keys, signatures, table points).
//
// Representation: "signed30", 9 limbs of 30 bits (int32), value =
// sum v[i] 2^(30 i), low limbs in [0, 2^30), the top limb signed.
// Algorithm (Bernstein & Yang 2019, with the variable-time batching of
// zero-divsteps and the 6-bit cancellation of Pornin/Wuille):
//   f = m, g = x, d = 0, e = 1, eta = -1
//   repeat: 30 divsteps on the low words of f, g -> 2x2 matrix t (entries
//   bounded by 2^30); (d, e) <- t (d, e) / 2^30 mod m; (f, g) <- t (f, g) /
//   2^30 (exact); until g = 0.  Then f = +-1 and x^-1 = +-d mod m.
// Invariants (as in the published analysis): d, e in (-2m, m).
//
// Attribution: the structure of this implementation (signed30 limbs, the
// divsteps matrix, update_de / update_fg, the modinfo constants) follows
// libsecp256k1's src/modinv32_impl.h (Copyright (c) 2020 Peter Dettman,
// Pieter Wuille; MIT license, https://github.com/bitcoin-core/secp256k1),
// restated here for one GPU lane; the safegcd paper is Bernstein & Yang,
// "Fast constant-time gcd computation and modular inversion", TCHES 2019.
#pragma once
#include <stdint.h>

struct s30 {
  int32_t v[9];
};

struct modinfo30 {
  int32_t m[9];      // modulus, signed30 (non-negative limbs)
  uint32_t inv30;    // m^-1 mod 2^30
};

#define M30 0x3FFFFFFFu

DEV void s30_from_u256(s30 &r, const uint32_t a[8]) {
  // bit 30 i .. 30 i + 29
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 30 * i, w = bit >> 5, sh = bit & 31;
    uint32_t lo = a[w] >> sh;
    if (sh > 2 && w + 1 < 8) lo |= a[w + 1] << (32 - sh);
    r.v[i] = (int32_t)(lo & M30);
  }
}

DEV void s30_to_u256(uint32_t a[8], const s30 &r) {  // r in [0, 2^256), limbs normalised
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const int bit = 32 * w, i = bit / 30, sh = bit % 30;
    uint32_t x = (uint32_t)r.v[i] >> sh;
    x |= (uint32_t)r.v[i + 1] << (30 - sh);
    if (sh > 28 && i + 2 < 9) x |= (uint32_t)r.v[i + 2] << (60 - sh);
    a[w] = x;
  }
}

// Count trailing zeros of a non-zero word.
DEV int ctz32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_ctz(x);
#else
  return __builtin_ctz(x);
#endif
}

// 30 divsteps on the low words f0, g0 (f0 odd); returns the new eta and the
// transition matrix (u v; q r) with (f', g') 2^30 = (u f + v g, q f + r g).
DEV int32_t divsteps_30_var(int32_t eta, uint32_t f0, uint32_t g0, int32_t t[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1, f = f0, g = g0;
  int i = 30;
  for (;;) {
    const int zeros = ctz32(g | (0xFFFFFFFFu << i));  // sentinel bit: at most i
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {  // (f, g) <- (g, -f) and the matching matrix rows
      uint32_t tmp;
      eta = -eta;
      tmp = f; f = g; g = 0u - tmp;
      tmp = u; u = q; q = 0u - tmp;
      tmp = v; v = r; r = 0u - tmp;
    }
    // cancel the low min(eta + 1, i, 6) bits of g with a multiple of f:
    // w = -g f^-1 mod 2^6, f^-1 = f (2 - f^2) mod 2^6 (f^2 = 1 mod 8)
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xFFFFFFFFu >> (32 - limit)) & 63u;
    const uint32_t w = (f * g * (f * f - 2u)) & m;
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t[0] = (int32_t)u;
  t[1] = (int32_t)v;
  t[2] = (int32_t)q;
  t[3] = (int32_t)r;
  return eta;
}

// (d, e) <- t (d, e) / 2^30 mod m, keeping d, e in (-2m, m).
DEV void update_de_30(s30 &d, s30 &e, const int32_t t[4], const modinfo30 &mi) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;  // -1 if negative
  int32_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  // add md, me multiples of m so the low 30 bits vanish
  md -= (int32_t)((mi.inv30 * (uint32_t)cd + (uint32_t)md) & M30);
  me -= (int32_t)((mi.inv30 * (uint32_t)ce + (uint32_t)me) & M30);
  cd += (int64_t)mi.m[0] * md;
  ce += (int64_t)mi.m[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cd += (int64_t)u * d.v[i] + (int64_t)v * e.v[i] + (int64_t)mi.m[i] * md;
    ce += (int64_t)q * d.v[i] + (int64_t)r * e.v[i] + (int64_t)mi.m[i] * me;
    d.v[i - 1] = (int32_t)((uint32_t)cd & M30);
    e.v[i - 1] = (int32_t)((uint32_t)ce & M30);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}

// (f, g) <- t (f, g) / 2^30 (exact division)
DEV void update_fg_30(s30 &f, s30 &g, const int32_t t[4]) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
  int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cf += (int64_t)u * f.v[i] + (int64_t)v * g.v[i];
    cg += (int64_t)q * f.v[i] + (int64_t)r * g.v[i];
    f.v[i - 1] = (int32_t)((uint32_t)cf & M30);
    g.v[i - 1] = (int32_t)((uint32_t)cg & M30);
    cf >>= 30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}

// x = sign * d mod m in [0, m), for d in (-2m, m), sign = +-1 (f's sign).
DEV void normalize_30(s30 &d, int32_t f_sign_mask, const modinfo30 &mi) {
  // conditional negation: d <- (d ^ s) - s on the whole value
  int32_t c = 0;
  if (f_sign_mask) {
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      acc += -(int64_t)d.v[i];
      if (i < 8) {
        d.v[i] = (int32_t)((uint32_t)acc & M30);
        acc >>= 30;
      } else {
        d.v[i] = (int32_t)acc;
      }
    }
  }
  (void)c;
  // now d in (-m, 2m): add m while negative, subtract m while >= m
  for (int pass = 0; pass < 3; pass++) {
    if (d.v[8] < 0) {
      int64_t acc = 0;
#pragma unroll
      for (int i = 0; i < 9; i++) {
        acc += (int64_t)d.v[i] + mi.m[i];
        if (i < 8) {
          d.v[i] = (int32_t)((uint32_t)acc & M30);
          acc >>= 30;
        } else {
          d.v[i] = (int32_t)acc;
        }
      }
    }
  }
  // d >= m ?  (limbs normalised, d >= 0)
  bool ge = true;
  for (int i = 8; i >= 0; i--) {
    if (d.v[i] != mi.m[i]) {
      ge = d.v[i] > mi.m[i];
      break;
    }
  }
  if (ge) {
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      acc += (int64_t)d.v[i] - mi.m[i];
      if (i < 8) {
        d.v[i] = (int32_t)((uint32_t)acc & M30);
        acc >>= 30;
      } else {
        d.v[i] = (int32_t)acc;
      }
    }
  }
}

// r = x^-1 mod m for 0 < x < m (x = 0 gives 0).
DEV void modinv_var(uint32_t r[8], const uint32_t x[8], const modinfo30 &mi) {
  s30 d, e, f, g;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    d.v[i] = 0;
    e.v[i] = 0;
    f.v[i] = mi.m[i];
  }
  e.v[0] = 1;
  s30_from_u256(g, x);
  int32_t eta = -1;
  for (;;) {
    int32_t t[4];
    eta = divsteps_30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de_30(d, e, t, mi);
    update_fg_30(f, g, t);
    int32_t z = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) z |= g.v[i];
    if (z == 0) break;
  }
  normalize_30(d, f.v[8] >> 31, mi);
  s30_to_u256(r, d);
}

// p = 2^256 - 2^32 - 977 and N (curve.go:13), signed30
DEV void modinfo_p(modinfo30 &mi) {
  const int32_t m[9] = {1073740847, 1073741819, 1073741823, 1073741823, 1073741823,
                        1073741823, 1073741823, 1073741823, 65535};
#pragma unroll
  for (int i = 0; i < 9; i++) mi.m[i] = m[i];
  mi.inv30 = 769313487u;
}
DEV void modinfo_n(modinfo30 &mi) {
  const int32_t m[9] = {271991105, 1061780019, 881460155, 733428139, 1073741498,
                        1073741823, 1073741823, 1073741823, 65535};
#pragma unroll
  for (int i = 0; i < 9; i++) mi.m[i] = m[i];
  mi.inv30 = 712462017u;
}
