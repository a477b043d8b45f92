// verify_core.h — the per-unit work of every kernel, as __host__ __device__
// functions.  kernels.hip maps them onto the grid; tests/emu compiles the
// same source for the host so index logic and arithmetic are exercised on
// the CPU (with sanitizers) before a GPU run.  Nothing here is a CPU path of
// the product: libbabbleverify.so only ever runs these on gfx950.
#pragma once
#include <type_traits>
#include <stdint.h>

#include "../../include/babbleverify.h"
#include "geometry.h"
#include "coop.h"
#include "point.h"
#include "sha256.h"

// key status (k_key_decode output)
#define KS_OK 0
#define KS_EMPTY 1
#define KS_BAD 2

// p - N: r + N < p  <=>  r < p - N
static constexpr uint32_t P_MINUS_N[8] = {0x2FC9BAEEu, 0x402DA172u, 0x50B75FC4u, 0x45512319u,
                                          0x00000001u, 0u, 0u, 0u};

// ---------------------------------------------------------------------------
// loads / stores
// ---------------------------------------------------------------------------
DEV void fe_load_be(fe &r, const uint8_t *b) {  // 32 big-endian bytes, any alignment
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint8_t *q = b + 4 * (7 - i);
    r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}
DEV void fe_load_be_words(fe &r, const uint32_t *w) {  // 8 dwords holding 32 BE bytes
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = bswap32(w[7 - i]);
}
DEV void sc_load_be_words(sc &r, const uint32_t *w) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = bswap32(w[7 - i]);
}
DEV void fe_store(uint32_t *p, const fe &a) {
#pragma unroll
  for (int i = 0; i < 8; i++) p[i] = a.v[i];
}
DEV void fe_load(fe &a, const uint32_t *p) {
#pragma unroll
  for (int i = 0; i < 8; i++) a.v[i] = p[i];
}
DEV void fe_load4(fe &a, const uint32_t *p) {  // 16-byte aligned: 2 x dwordx4
#if defined(__HIP_DEVICE_COMPILE__)
  // table entries live in global memory: global_load, not flat_load (a flat
  // access also counts against lgkmcnt and takes the aperture check)
  typedef const __attribute__((address_space(1))) uint4 *gptr;
  const gptr q = (gptr)p;
#else
  const uint4 *q = (const uint4 *)p;
#endif
  uint4 l = q[0], h = q[1];
  a.v[0] = l.x; a.v[1] = l.y; a.v[2] = l.z; a.v[3] = l.w;
  a.v[4] = h.x; a.v[5] = h.y; a.v[6] = h.z; a.v[7] = h.w;
}
DEV void store16(uint32_t *p, const uint32_t *v) {  // 64 bytes, 16-byte aligned
  uint4 *q = (uint4 *)p;
#pragma unroll
  for (int c = 0; c < 4; c++) q[c] = make_uint4(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);
}
DEV bool u256_lt(const uint32_t *a, const uint32_t *b) {
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] < b[i];
  }
  return false;
}
DEV bool u256_is_zero(const uint32_t *a) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a[i];
  return x == 0;
}

// ---------------------------------------------------------------------------
// SHA-256 of message m -> 8 dwords holding the 32 big-endian digest bytes
// (crypto.SHA256, src/crypto/hash.go:8)
// ---------------------------------------------------------------------------
DEV void sha256_one(uint64_t m, const uint8_t *bytes, const uint64_t *off, uint32_t *digest_words) {
  const uint64_t o = off[m];
  const uint64_t len = off[m + 1] - o;
  uint32_t h[8];
  sha256_msg(h, bytes, o, len);
  uint32_t be[8];
#pragma unroll
  for (int i = 0; i < 8; i++) be[i] = bswap32(h[i]);
  uint4 *dst = (uint4 *)(digest_words + 8 * m);
  dst[0] = make_uint4(be[0], be[1], be[2], be[3]);
  dst[1] = make_uint4(be[4], be[5], be[6], be[7]);
}

// ---------------------------------------------------------------------------
// elliptic.Unmarshal(btcec.S256(), b) (src/crypto/keys/public_key.go:14-20):
// len 65, prefix 0x04, x < p, y < p, y^2 == x^3 + 7.  len 0 -> ToPublicKey
// returns nil (KS_EMPTY: ecdsa.Verify panics at pub.Curve).
// ---------------------------------------------------------------------------
DEV void key_decode_point(const uint8_t *kbytes, uint64_t o, uint64_t len, uint8_t &st, fe &x, fe &y) {
  st = KS_BAD;
  fe_set(x, 0);
  fe_set(y, 0);
  if (len == 0) {
    st = KS_EMPTY;
  } else if (len == 65 && kbytes[o] == 4) {
#if defined(__HIP_DEVICE_COMPILE__)
    // 17 aligned dword loads issued together (bytewise loads of an unaligned
    // key serialise on memory latency: 80 us for one wave of 64 keys); the
    // last dword may extend <= 7 bytes past the key (key_bytes is padded)
    const uint32_t *w = (const uint32_t *)(kbytes + (o & ~(uint64_t)3));
    const uint32_t sh = (uint32_t)(o & 3);
    uint32_t d[18];
#pragma unroll
    for (int i = 0; i < 18; i++) d[i] = w[i];
#pragma unroll
    for (int i = 0; i < 8; i++) {  // big-endian bytes 1 + 4 (7 - i) .. and 33 + 4 (7 - i) ..
      const uint32_t bx = 1 + 4 * (7 - i) + sh, by = 33 + 4 * (7 - i) + sh;
      x.v[i] = bswap32(alignbyte(d[bx / 4 + 1], d[bx / 4], bx % 4));
      y.v[i] = bswap32(alignbyte(d[by / 4 + 1], d[by / 4], by % 4));
    }
#else
    fe_load_be(x, kbytes + o + 1);
    fe_load_be(y, kbytes + o + 33);
#endif
    if (!fe_ge_p(x) && !fe_ge_p(y)) {
      fe y2, x3, seven;
      fe_sqr(y2, y);
      fe_sqr(x3, x);
      fe_mul(x3, x3, x);
      fe_set(seven, 7);
      fe_add(x3, x3, seven);
      if (fe_eq(y2, x3)) st = KS_OK;
    }
  }
}

DEV void key_decode_one(uint32_t k, const uint8_t *kbytes, const uint64_t *koff, uint8_t *kstatus, uint32_t *kxy) {
  uint8_t st;
  fe x, y;
  key_decode_point(kbytes, koff[k], koff[k + 1] - koff[k], st, x, y);
  kstatus[k] = st;
  fe_store(kxy + 16 * k, x);
  fe_store(kxy + 16 * k + 8, y);
}

// ---------------------------------------------------------------------------
// Fixed-base tables
// ---------------------------------------------------------------------------
// B_j = 2^(w j) P_b (Jacobian, 24 words each), j < nwin: a serial doubling
// chain per base.
template <bool LAT = false>
DEV void table_bases_one(uint32_t b, const uint32_t *bxy, uint32_t *bases_jac, int w, int nwin) {
  gej P;
  fe_load(P.X, bxy + 16 * b);
  fe_load(P.Y, bxy + 16 * b + 8);
  fe_set(P.Z, 1);
  uint32_t *out = bases_jac + (uint64_t)b * nwin * 24;
  for (int j = 0; j < nwin; j++) {
    fe_store(out + 24 * j, P.X);
    fe_store(out + 24 * j + 8, P.Y);
    fe_store(out + 24 * j + 16, P.Z);
    if (j + 1 < nwin) {
      for (int k = 0; k < w; k++) gej_double_sel<LAT>(P, P);  // one wave per 64 keys: latency bound
    }
  }
}

#if defined(__HIPCC__)
// The same chain, wave-cooperative (coop.h): ONE wave per base, the
// doubling's three product levels spread over the wave's DPP rows; lanes
// 0..7 (row 0) store.  Same formulas, so the same Jacobian representatives
// as table_bases_one.
__device__ __forceinline__ void coop_bases_one(uint32_t b, const uint32_t *bxy, uint32_t *bases_jac, int w, int nwin) {
  const uint32_t k = coop::pos(), lane = __lane_id();
  uint32_t X = k < 8 ? bxy[16 * (uint64_t)b + k] : 0u, Y = k < 8 ? bxy[16 * (uint64_t)b + 8 + k] : 0u;
  uint32_t Z = k == 0 ? 1u : 0u;
  uint32_t *out = bases_jac + (uint64_t)b * nwin * 24;
  for (int j = 0; j < nwin; j++) {
    if (lane < 8) {
      out[24 * j + lane] = X;
      out[24 * j + 8 + lane] = Y;
      out[24 * j + 16 + lane] = Z;
    }
    if (j + 1 < nwin)
      for (int i = 0; i < w; i++) coop::dbl(X, Y, Z);
  }
}
#endif

// d * B (B affine), MSB-first double-and-add over `bits` bits of d.  The
// returned Z is 1 for d == 0 so it can join a batch inversion.
template <bool LAT = false>
DEV void table_point(gej &R, bool &inf, fe &Z, const fe &bx, const fe &by, uint32_t d, int bits) {
  inf = true;
  fe_set(R.X, 0);
  fe_set(R.Y, 0);
  fe_set(R.Z, 0);
  for (int bit = bits - 1; bit >= 0; bit--) {
    if (!inf) gej_double_sel<LAT>(R, R);
    if ((d >> bit) & 1) gej_add_ge_sel<LAT>(R, inf, bx, by);
  }
  if (inf) fe_set(Z, 1);
  else Z = R.Z;
}

// Store one entry given Z^-1 (canonical affine; d == 0 stored as zeros).
// With `phi` != null also store phi(entry) = (beta x, y) there.
DEV void table_store(uint32_t *entry, uint32_t *phi, uint32_t d, const gej &R, bool inf, const fe &zi) {
  fe zi2, zi3, x, y;
  fe_sqr(zi2, zi);
  fe_mul(zi3, zi2, zi);
  fe_mul(x, R.X, zi2);
  fe_mul(y, R.Y, zi3);
  fe_canon(x);
  fe_canon(y);
  if (d == 0 || inf) {
    fe_set(x, 0);
    fe_set(y, 0);
  }
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    v[i] = x.v[i];
    v[8 + i] = y.v[i];
  }
  store16(entry, v);
  if (phi) {
    fe beta, bx;
    fe_load(beta, FE_BETA);
    fe_mul(bx, x, beta);
    fe_canon(bx);
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = bx.v[i];
    store16(phi, v);
  }
}

// K12 entry (j, d) = S_2j[lo] + S_2j+1[hi], lo = d mod 2^L, hi = d >> L,
// with S_k[x] = x 2^(Lk) Q affine (zeros for x == 0).  The two points are
// distinct multiples lo 2^(Wj) Q and hi 2^(Wj+L) Q of Q with
// 0 < lo < 2^L <= hi 2^L and lo + hi 2^L < 2^W << N, so they are neither
// equal nor opposite and the affine chord formula applies:
//   lambda = (y2 - y1) / (x2 - x1), x3 = lambda^2 - x1 - x2,
//   y3 = lambda (x1 - x3) - y1.
// The denominators H = x2 - x1 of a block are inverted together
// (Montgomery's trick, k_table_pair).  kind: 0 zero entry, 1 copy S_lo,
// 2 copy S_hi, 3 chord sum.
DEV int pair_kind(uint32_t lo, uint32_t hi) { return (lo ? 1 : 0) | (hi ? 2 : 0); }

// K12 builder slot -> digit: slot 0 of a window block builds the window's
// top digit 2^(W-1) = ENT (stored at window j+1's unused slot 0).
DEV uint32_t k12_digit(uint32_t d, uint32_t ent) { return d ? d : ent; }

DEV void pair_load(const uint32_t *s_lo, const uint32_t *s_hi, uint32_t lo, uint32_t hi, fe &x1, fe &y1, fe &x2,
                   fe &y2) {
  fe_load(x1, s_lo + BV_ENTRY_U32 * lo);
  fe_load(y1, s_lo + BV_ENTRY_U32 * lo + 8);
  fe_load(x2, s_hi + BV_ENTRY_U32 * hi);
  fe_load(y2, s_hi + BV_ENTRY_U32 * hi + 8);
}

// the value joining the batch inversion (1 unless the entry is a sum)
DEV void pair_denominator(fe &H, int kind, const fe &x1, const fe &x2) {
  if (kind == 3) fe_sub(H, x2, x1);
  else fe_set(H, 1);
}

DEV void pair_store(uint32_t *entry, uint32_t *phi, int kind, const fe &x1, const fe &y1, const fe &x2, const fe &y2,
                    const fe &Hinv) {
  fe x, y;
  if (kind == 3) {
    fe lam, t;
    fe_sub(t, y2, y1);
    fe_mul(lam, t, Hinv);
    fe_sqr(x, lam);
    fe_sub(x, x, x1);
    fe_sub(x, x, x2);
    fe_sub(t, x1, x);
    fe_mul(y, lam, t);
    fe_sub(y, y, y1);
  } else if (kind == 1) {
    x = x1;
    y = y1;
  } else {
    x = x2;  // kind 2, or kind 0 with S_hi[0] = zeros
    y = y2;
  }
  fe_canon(x);
  fe_canon(y);
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    v[i] = x.v[i];
    v[8 + i] = y.v[i];
  }
  store16(entry, v);
  if (!phi) return;
  fe beta, bx;
  fe_load(beta, FE_BETA);
  fe_mul(bx, x, beta);
  fe_canon(bx);
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = bx.v[i];
  store16(phi, v);
}

// ---------------------------------------------------------------------------
// Scalars: u1 = e * s^-1, u2 = r * s^-1 (mod N)  (ecdsa.Verify steps 4-6)
// ---------------------------------------------------------------------------
DEV void sc_sqrn(sc &a, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) sc_mont(a, a, a);
}

// x^(N-2) in the Montgomery domain (xR -> x^-1 R): 255 S + 45 M.
// The top 128 bits of N-2 are 2^128 - 2 (runs of ones, built from
// x^(2^k - 1)); the low 128 bits use a 4-bit sliding window (chain generated
// offline; tests/test_emu.py checks inverses against Python ints).
DEV void sc_inverse(sc &r, const sc &x) {
  sc x2, x3, x5, x7, x9, x11, x13, x15;
  sc_mont(x2, x, x);
  sc_mont(x3, x2, x);
  sc_mont(x5, x3, x2);
  sc_mont(x7, x5, x2);
  sc_mont(x9, x7, x2);
  sc_mont(x11, x9, x2);
  sc_mont(x13, x11, x2);
  sc_mont(x15, x13, x2);
  sc a2 = x3, a4, a8, a16, a32, a64, t;
  a4 = a2; sc_sqrn(a4, 2); sc_mont(a4, a4, a2);
  a8 = a4; sc_sqrn(a8, 4); sc_mont(a8, a8, a4);
  a16 = a8; sc_sqrn(a16, 8); sc_mont(a16, a16, a8);
  a32 = a16; sc_sqrn(a32, 16); sc_mont(a32, a32, a16);
  a64 = a32; sc_sqrn(a64, 32); sc_mont(a64, a64, a32);
  t = a64;
  sc_sqrn(t, 32); sc_mont(t, t, a32);
  sc_sqrn(t, 16); sc_mont(t, t, a16);
  sc_sqrn(t, 8); sc_mont(t, t, a8);
  sc_sqrn(t, 4); sc_mont(t, t, a4);
  sc_sqrn(t, 2); sc_mont(t, t, a2);
  sc_sqrn(t, 1); sc_mont(t, t, x);  // x^(2^127 - 1)
  sc_sqrn(t, 1);                    // x^(2^128 - 2)
#define SQM(n, m) sc_sqrn(t, n); sc_mont(t, t, m);
  SQM(4, x11) SQM(3, x5) SQM(4, x5) SQM(4, x7) SQM(5, x13) SQM(2, x3) SQM(5, x7) SQM(6, x13)
  SQM(5, x11) SQM(4, x13) SQM(3, x) SQM(6, x5) SQM(10, x7) SQM(4, x7) SQM(5, x15) SQM(4, x15)
  SQM(5, x9) SQM(6, x11) SQM(4, x13) SQM(5, x3) SQM(6, x13) SQM(10, x13) SQM(4, x9) SQM(9, x9)
  SQM(4, x15) SQM(1, x)
#undef SQM
  r = t;
}

DEV bool s_usable(const uint8_t *pre, uint64_t i, const sc &s) {
  return (pre == nullptr || pre[i] == 0) && !u256_is_zero(s.v) && u256_lt(s.v, SC_N);
}

// k_sinv, thread t of T: w_i = s_i^-1 R mod N (Montgomery form) for items
// t, t+T, ..., t+(M-1)T with one inversion (Montgomery's trick).
// Needs only s and pre, so it runs on its own stream concurrently with
// SHA-256 and the key tables; the digest-dependent products u1 = e w and
// u2 = r w are formed by k_verify_g (item_scalars).  Unusable items
// contribute s = 1 and get a w that is never read.
//
// The raw s_k enter the Montgomery products unconverted (no s R^2 -> s R
// step): after k items the prefix is acc_k = R^(1-k) prod_{i<=k} s_i, the
// inverse of the total (xR -> x^-1 R) is R^(1+K) / prod s, one extra
// product by 1 makes it R^K / prod s, and walking back w_k = inv acc_(k-1)
// / R = R / s_k while inv loses one s_k and one R per step.
DEV void sinv_thread(uint64_t t, uint64_t T, uint64_t n_items, uint32_t M, const uint32_t *s_be, const uint8_t *pre,
                     uint32_t *w_out) {
  sc R1, one;
  sc_load_const(R1, SC_R1);
#pragma unroll
  for (int k = 0; k < 8; k++) one.v[k] = k == 0 ? 1u : 0u;
  sc acc = R1;
  for (uint32_t m = 0; m < M; m++) {
    const uint64_t i = t + (uint64_t)m * T;
    if (i >= n_items) break;
    sc s;
    sc_load_be_words(s, s_be + 8 * i);
    if (!s_usable(pre, i, s)) s = one;
    uint4 *q = (uint4 *)(w_out + 8 * i);
    q[0] = make_uint4(acc.v[0], acc.v[1], acc.v[2], acc.v[3]);
    q[1] = make_uint4(acc.v[4], acc.v[5], acc.v[6], acc.v[7]);
    sc_mont(acc, acc, s);
  }
  sc inv;
  sc_inverse_var(inv, acc);
  sc_mont(inv, inv, one);
  for (int m = (int)M - 1; m >= 0; m--) {
    const uint64_t i = t + (uint64_t)m * T;
    if (i >= n_items) continue;
    sc s, pfx, w;
    sc_load_be_words(s, s_be + 8 * i);
    if (!s_usable(pre, i, s)) s = one;
    uint4 *q = (uint4 *)(w_out + 8 * i);
    const uint4 a = q[0], b = q[1];
    pfx.v[0] = a.x; pfx.v[1] = a.y; pfx.v[2] = a.z; pfx.v[3] = a.w;
    pfx.v[4] = b.x; pfx.v[5] = b.y; pfx.v[6] = b.z; pfx.v[7] = b.w;
    sc_mont(w, inv, pfx);  // s^-1 R
    sc_mont(inv, inv, s);
    q[0] = make_uint4(w.v[0], w.v[1], w.v[2], w.v[3]);
    q[1] = make_uint4(w.v[4], w.v[5], w.v[6], w.v[7]);
  }
}

// u1 = e s^-1 and the GLV split of u2 = r s^-1 (mod N) for an item that
// reaches the math (ecdsa.Verify steps 4-6: e = the 256-bit digest,
// unreduced; w = s^-1 R from k_sinv).
DEV void item_scalars(uint64_t i, const uint32_t *r_be, const uint32_t *item_msg, const uint32_t *digest_words,
                      const uint32_t *w_in, uint32_t u1[8], uint32_t k1[4], uint32_t k2[4], uint32_t &signs) {
  sc w, e, r, a, b;
  const uint4 *q = (const uint4 *)(w_in + 8 * i);
  const uint4 x = q[0], y = q[1];
  w.v[0] = x.x; w.v[1] = x.y; w.v[2] = x.z; w.v[3] = x.w;
  w.v[4] = y.x; w.v[5] = y.y; w.v[6] = y.z; w.v[7] = y.w;
  sc_load_be_words(e, digest_words + 8 * (uint64_t)item_msg[i]);
  sc_load_be_words(r, r_be + 8 * i);
  sc_mont(a, e, w);  // e * s^-1 mod N  (e < 2^256 = R, w < N)
  sc_mont(b, r, w);  // r * s^-1 mod N
#pragma unroll
  for (int k = 0; k < 8; k++) u1[k] = a.v[k];
  glv_split(k1, k2, signs, b);
}

// Key-cache batches with a few keys that have no table yet (bv_kc_prepare's
// partial mode): their items reach the math without a table; the
// KC kernels leave them as BV_DEFERRED (accept bit 0) and k_verify_deferred
// finishes them by the generic path.  Never returned to a caller.
#define BV_DEFERRED 0xFE

// ---------------------------------------------------------------------------
// Item decision table.  Returns 0xFF when the item must run
// the math, else its final status.  The host pre-class is re-checked against
// the r/s bytes so an inconsistent pre byte cannot skip a range check.
// ---------------------------------------------------------------------------
DEV uint8_t classify(uint8_t pre, uint8_t ks, const fe &r, const fe &s) {
  if (pre & BV_PRE_PARTS_BAD) return BV_REJECT_ERR;
  if (ks == KS_EMPTY) return BV_REF_PANIC;
  uint32_t rc = pre & 3u, scl = (pre >> 2) & 3u;
  if (rc == BV_SC_OK) rc = u256_is_zero(r.v) ? BV_SC_NONPOS : (u256_lt(r.v, SC_N) ? BV_SC_OK : BV_SC_GE_N);
  if (scl == BV_SC_OK) scl = u256_is_zero(s.v) ? BV_SC_NONPOS : (u256_lt(s.v, SC_N) ? BV_SC_OK : BV_SC_GE_N);
  if (rc == BV_SC_NIL) return BV_REF_PANIC;
  if (rc == BV_SC_NONPOS) return BV_REJECT;
  if (scl == BV_SC_NIL) return BV_REF_PANIC;
  if (scl == BV_SC_NONPOS) return BV_REJECT;
  if (rc == BV_SC_GE_N || scl == BV_SC_GE_N) return BV_REJECT;
  if (ks != KS_OK) return BV_REF_PANIC;
  return 0xFF;
}

DEV uint8_t classify_item(uint64_t i, const uint32_t *item_key, const uint32_t *r_be, const uint32_t *s_be,
                          const uint8_t *pre, const uint8_t *kstatus, fe &r) {
  fe s;
  fe_load_be_words(r, r_be + 8 * i);
  fe_load_be_words(s, s_be + 8 * i);
  return classify(pre ? pre[i] : 0, kstatus[item_key[i]], r, s);
}

// x(R) mod N == r, projectively: X == r Z^2, or (r + N < p and X == (r+N) Z^2)
DEV bool final_check(const gej &R, bool inf, const fe &r) {
  if (inf) return false;
  fe z2, t;
  fe_sqr(z2, R.Z);
  fe_mul(t, r, z2);
  if (fe_eq(t, R.X)) return true;
  if (u256_lt(r.v, P_MINUS_N)) {
    fe rn;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) rn.v[i] = addc32(r.v[i], SC_N[i], c);
    fe_mul(t, rn, z2);
    if (fe_eq(t, R.X)) return true;
  }
  return false;
}

// The same check on an XYZZ accumulator: x = X / ZZ, so X == r ZZ (or
// (r + N) ZZ): one multiply, no squaring.
DEV bool final_check(const gexz &R, bool inf, const fe &r) {
  if (inf) return false;
  fe t;
  fe_mul(t, r, R.ZZ);
  if (fe_eq(t, R.X)) return true;
  if (u256_lt(r.v, P_MINUS_N)) {
    fe rn;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) rn.v[i] = addc32(r.v[i], SC_N[i], c);
    fe_mul(t, rn, R.ZZ);
    if (fe_eq(t, R.X)) return true;
  }
  return false;
}

// R += sum_j T[j][digit_j(u)] over the 256-bit u1 (8 limbs, consumed:
// shifted right W bits per window, so digits never straddle limbs) with
// SIGNED digits in (-2^(W-1), 2^(W-1)] by carry recoding: T[j][|d|], y
// negated for d < 0 (geometry.h).  u < N < 2^256 and W NWIN >= 257, so no
// carry is left after the top window.
// FROM_INF (XYZZ only): R enters as the identity, so after window 0 it is
// that window's affine entry and window 1 adds with the 4M + 2S affine step
// (gexz_add_ge_aff) — 4 multiplies fewer per item.
template <int W, int NWIN, bool LAT = false, class PT = gej, bool FROM_INF = false>
DEV void g_table_add(PT &R, bool &inf, const uint32_t *tab, uint32_t u[8]) {
  constexpr uint32_t ENT = 1u << (W - 1);
  static_assert(W * NWIN >= 257 && W < 32, "signed G windows must absorb the last carry");
  uint32_t carry = 0;
  for (int j = 0; j < NWIN; j++) {
    uint32_t d = (u[0] & ((1u << W) - 1u)) + carry;
#pragma unroll
    for (int c = 0; c < 7; c++) u[c] = (u[c] >> W) | (u[c + 1] << (32 - W));
    u[7] >>= W;
    carry = d > ENT ? 1u : 0u;
    const bool dneg = carry != 0;
    if (dneg) d = (1u << W) - d;  // |d - 2^W|, 0 when d == 2^W
    // loaded unconditionally (d == 0 reads the window's slot 0, a valid
    // entry that is then not added): no per-lane branch around the lookup
    const uint32_t *e = tab + ((uint64_t)j * ENT + d) * BV_ENTRY_U32;
    fe x, y;
    fe_load4(x, e);
    fe_load4(y, e + 8);
    fe_cneg_canon(y, dneg);
    if constexpr (FROM_INF) {
      if (j == 1 && !inf) {  // R = window 0's entry (affine)
        if (d != 0) gexz_add_ge_aff<LAT>(R, inf, x, y);
        continue;
      }
    }
    pt_add_ge_step<LAT>(R, inf, x, y, d != 0);
  }
}

// k1 magnitude, k2 magnitude (4 limbs each) and the sign word
DEV void load_k(uint32_t k1[4], uint32_t k2[4], uint32_t &signs, const uint32_t *u12, uint64_t i) {
  const uint4 *q = (const uint4 *)(u12 + (uint64_t)BV_U_STRIDE * i);
  uint4 a = q[0], b = q[1], c = q[2];
  k1[0] = a.x; k1[1] = a.y; k1[2] = a.z; k1[3] = a.w;
  k2[0] = b.x; k2[1] = b.y; k2[2] = b.z; k2[3] = b.w;
  signs = c.x;
}

// Partial point R_G = u1 G (XYZZ), kept in HBM between k_verify_g and
// k_verify_q as 33 SoA words per item (X, Y, ZZ, ZZZ limbs, inf flag) for
// coalesced access.
#define RG_WORDS 33
DEV void rg_store(uint32_t *rg, uint64_t n, uint64_t i, const gexz &R, bool inf) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    rg[(uint64_t)k * n + i] = R.X.v[k];
    rg[(uint64_t)(8 + k) * n + i] = R.Y.v[k];
    rg[(uint64_t)(16 + k) * n + i] = R.ZZ.v[k];
    rg[(uint64_t)(24 + k) * n + i] = R.ZZZ.v[k];
  }
  rg[(uint64_t)32 * n + i] = inf ? 1u : 0u;
}
DEV void rg_load(const uint32_t *rg, uint64_t n, uint64_t i, gexz &R, bool &inf) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    R.X.v[k] = rg[(uint64_t)k * n + i];
    R.Y.v[k] = rg[(uint64_t)(8 + k) * n + i];
    R.ZZ.v[k] = rg[(uint64_t)(16 + k) * n + i];
    R.ZZZ.v[k] = rg[(uint64_t)(24 + k) * n + i];
  }
  inf = rg[(uint64_t)32 * n + i] != 0;
}

// Phase 1 (overlaps the key-table build): R_G = u1 G for items that reach
// the math.
// k_glv_split, item i (per-batch key tables, device entry): u2 = r s^-1 and
// its GLV split into u12 as soon as s^-1 is known — on the s^-1 stream,
// beside SHA-256 and the key tables — so k_verify_g forms only u1 = e s^-1
// (the digest's product).  Items whose s is unusable get a split of a
// dummy w that k_verify_q never reads (it classifies first).
DEV void glv_split_item(uint64_t i, const uint32_t *r_be, const uint32_t *w_in, uint32_t *u12) {
  sc w, r, b;
  const uint4 *q = (const uint4 *)(w_in + 8 * i);
  const uint4 x = q[0], y = q[1];
  w.v[0] = x.x; w.v[1] = x.y; w.v[2] = x.z; w.v[3] = x.w;
  w.v[4] = y.x; w.v[5] = y.y; w.v[6] = y.z; w.v[7] = y.w;
  sc_load_be_words(r, r_be + 8 * i);
  sc_mont(b, r, w);  // r * s^-1 mod N
  uint32_t k1[4], k2[4], signs;
  glv_split(k1, k2, signs, b);
  uint4 *o = (uint4 *)(u12 + (uint64_t)BV_U_STRIDE * i);
  o[0] = make_uint4(k1[0], k1[1], k1[2], k1[3]);
  o[1] = make_uint4(k2[0], k2[1], k2[2], k2[3]);
  o[2] = make_uint4(signs, 0u, 0u, 0u);
}

// SPLIT: u12 already holds the GLV split (k_glv_split); else it is formed
// here with u1.
template <bool LAT = false, bool SPLIT = false>
DEV void verify_item_g(uint64_t i, uint64_t n, const uint32_t *item_key, const uint32_t *r_be, const uint32_t *s_be,
                       const uint8_t *pre, const uint8_t *kstatus, const uint32_t *item_msg,
                       const uint32_t *digest_words, const uint32_t *w_in, uint32_t *u12, const uint32_t *g_table,
                       uint32_t *rg) {
  fe r;
  if (classify_item(i, item_key, r_be, s_be, pre, kstatus, r) != 0xFF) return;
  uint32_t u[8];
  if (SPLIT) {
    sc w, e, a;
    const uint4 *q = (const uint4 *)(w_in + 8 * i);
    const uint4 x = q[0], y = q[1];
    w.v[0] = x.x; w.v[1] = x.y; w.v[2] = x.z; w.v[3] = x.w;
    w.v[4] = y.x; w.v[5] = y.y; w.v[6] = y.z; w.v[7] = y.w;
    sc_load_be_words(e, digest_words + 8 * (uint64_t)item_msg[i]);
    sc_mont(a, e, w);  // e * s^-1 mod N
#pragma unroll
    for (int k = 0; k < 8; k++) u[k] = a.v[k];
  } else {
    uint32_t k1[4], k2[4], signs;
    item_scalars(i, r_be, item_msg, digest_words, w_in, u, k1, k2, signs);
    uint4 *q = (uint4 *)(u12 + (uint64_t)BV_U_STRIDE * i);
    q[0] = make_uint4(k1[0], k1[1], k1[2], k1[3]);
    q[1] = make_uint4(k2[0], k2[1], k2[2], k2[3]);
    q[2] = make_uint4(signs, 0u, 0u, 0u);
  }
  gexz R;
  bool inf = true;
  fe_set(R.X, 0);
  fe_set(R.Y, 0);
  fe_set(R.ZZ, 0);
  fe_set(R.ZZZ, 0);
  g_table_add<BV_GW, BV_GNWIN, LAT, gexz, true>(R, inf, g_table, u);
  rg_store(rg, n, i, R, inf);
}

// R += sum_j T[j][digit_j(k)] over a 128-bit GLV half k (4 limbs; consumed:
// shifted right W bits per window, so digits never straddle limbs).
// SIGNED (K12): digits in (-2^(W-1), 2^(W-1)] by carry recoding, T[j][|d|]
// with y negated for d < 0; a window holds ENT = 2^(W-1) slots.  k < 2^128
// and W NWIN >= 129 bits, so no carry is left after the top window.
// `phi`: the table holds T (the k1 half) and this half needs phi(T) =
// (beta x, y): one multiply per lookup instead of a stored phi half (KC).
// `from_inf` (uniform; XYZZ only): R enters as the identity, so window 1
// adds to window 0's affine entry with the 4M + 2S step (as g_table_add).
template <int W, int NWIN, bool SIGNED, bool LAT = false, class PT = gexz>
DEV void key_table_add(PT &R, bool &inf, const uint32_t *tab, uint32_t k[4], bool neg, bool phi = false,
                       bool from_inf = false) {
  constexpr uint32_t ENT = SIGNED ? (1u << (W - 1)) : (1u << W);
  static_assert(!SIGNED || W * NWIN >= 129, "signed windows must absorb the last carry");
  if (neg) fe_neg(R.Y, R.Y);
  uint32_t carry = 0;
  for (int j = 0; j < NWIN; j++) {
    uint32_t d = (k[0] & ((1u << W) - 1u)) + carry;
    k[0] = (k[0] >> W) | (k[1] << (32 - W));
    k[1] = (k[1] >> W) | (k[2] << (32 - W));
    k[2] = (k[2] >> W) | (k[3] << (32 - W));
    k[3] >>= W;
    bool dneg = false;
    if (SIGNED) {
      carry = d > ENT ? 1u : 0u;
      if (carry) {
        d = (1u << W) - d;  // |d - 2^W|, 0 when d == 2^W
        dneg = true;
      }
    }
    const uint32_t *e = tab + ((uint64_t)j * ENT + d) * BV_ENTRY_U32;  // d == 0: a valid, unused slot
    fe x, y;
    fe_load4(x, e);
    fe_load4(y, e + 8);
    if (phi) {
      fe beta;
      fe_load(beta, FE_BETA);
      fe_mul(x, x, beta);
    }
    fe_cneg_canon(y, dneg);
    if constexpr (std::is_same<PT, gexz>::value) {
      if (from_inf && j == 1 && !inf) {  // R = window 0's entry (affine)
        if (d != 0) gexz_add_ge_aff<LAT>(R, inf, x, y);
        continue;
      }
    }
    pt_add_ge_step<LAT>(R, inf, x, y, d != 0);
  }
  if (neg) fe_neg(R.Y, R.Y);
}

// Phase 2: R = R_G + k1 Q + k2 phi(Q) with the key's two half-tables;
// final check -> status.
// key_tabs != null (key cache): per-batch-key table base addresses, else
// the tables are contiguous in key_table (per-batch K8 / K12 build).
template <int W, int NWIN, bool LAT = false>
DEV uint8_t verify_item_q(uint64_t i, uint64_t n, const uint32_t *item_key, const uint32_t *r_be,
                          const uint32_t *s_be, const uint8_t *pre, const uint8_t *kstatus, const uint32_t *u12,
                          const uint32_t *key_table, const uint64_t *key_tabs, const uint32_t *rg) {
  constexpr bool SIGNED = W != BV_KW;
  constexpr bool KC = W == BV_KCW;  // one stored half, phi(T) formed per lookup
  constexpr uint64_t half =
      SIGNED ? ((uint64_t)NWIN * (1ull << (W - 1)) + 1) * BV_ENTRY_U32 : (uint64_t)NWIN * (1ull << W) * BV_ENTRY_U32;
  static_assert(W != BV_K12W || half == BV_K12HALF_U32, "K12 geometry");
  static_assert(!KC || half == BV_KCHALF_U32, "KC geometry");
  fe r;
  const uint8_t st = classify_item(i, item_key, r_be, s_be, pre, kstatus, r);
  if (st != 0xFF) return st;
  uint32_t k1[4], k2[4], signs;
  load_k(k1, k2, signs, u12, i);
  gexz R;
  bool inf;
  rg_load(rg, n, i, R, inf);
  const uint32_t *tab = key_tabs ? (const uint32_t *)key_tabs[item_key[i]]
                                 : key_table + (uint64_t)item_key[i] * (KC ? 1 : 2) * half;
  if (!tab) return BV_DEFERRED;  // key cache, partial batch: no table for this key
  // One loop body for both GLV halves (one inlined copy of the point
  // addition: smaller code, fewer live registers than two calls).
#pragma unroll 1
  for (int h = 0; h < 2; h++) {
    uint32_t kk[4];
#pragma unroll
    for (int c = 0; c < 4; c++) kk[c] = h ? k2[c] : k1[c];
    key_table_add<W, NWIN, SIGNED, LAT>(R, inf, tab + (h && !KC ? half : 0), kk, (signs >> h) & 1u, KC && h);
  }
  fe_load_be_words(r, r_be + 8 * i);  // reloaded: not kept live through the loop
  return final_check(R, inf, r) ? BV_ACCEPT : BV_REJECT;
}

// Key part first, for host entries whose messages are still crossing PCIe:
// u2 = r s^-1 needs no digest, so R_Q = k1 Q + k2 phi(Q) is summed as soon
// as r, s, the keys and their tables are in HBM (k_verify_qf), and only
// u1 G and the decision wait for each chunk's digests (k_verify_gf).  The
// same additions as verify_item_g + verify_item_q in the other order; R_Q
// goes through the R_G buffer (rg_store), and no u12 round trip.
template <int W, int NWIN, bool LAT = false>
DEV void verify_item_qfirst(uint64_t i, uint64_t n, const uint32_t *item_key, const uint32_t *r_be,
                            const uint32_t *s_be, const uint8_t *pre, const uint8_t *kstatus, const uint32_t *w_in,
                            const uint32_t *key_table, const uint64_t *key_tabs, uint32_t *rq) {
  constexpr bool SIGNED = W != BV_KW;
  constexpr bool KC = W == BV_KCW;
  constexpr uint64_t half =
      SIGNED ? ((uint64_t)NWIN * (1ull << (W - 1)) + 1) * BV_ENTRY_U32 : (uint64_t)NWIN * (1ull << W) * BV_ENTRY_U32;
  fe r;
  if (classify_item(i, item_key, r_be, s_be, pre, kstatus, r) != 0xFF) return;
  uint32_t k1[4], k2[4], signs;
  {
    sc w, rs, b;
    const uint4 *q = (const uint4 *)(w_in + 8 * i);
    const uint4 x = q[0], y = q[1];
    w.v[0] = x.x; w.v[1] = x.y; w.v[2] = x.z; w.v[3] = x.w;
    w.v[4] = y.x; w.v[5] = y.y; w.v[6] = y.z; w.v[7] = y.w;
    sc_load_be_words(rs, r_be + 8 * i);
    sc_mont(b, rs, w);  // r * s^-1 mod N
    glv_split(k1, k2, signs, b);
  }
  gexz R;
  bool inf = true;
  fe_set(R.X, 0);
  fe_set(R.Y, 0);
  fe_set(R.ZZ, 0);
  fe_set(R.ZZZ, 0);
  const uint32_t *tab = key_tabs ? (const uint32_t *)key_tabs[item_key[i]]
                                 : key_table + (uint64_t)item_key[i] * (KC ? 1 : 2) * half;
  if (!tab) {  // key cache, partial batch: k_verify_gf leaves the item BV_DEFERRED
    rq[(uint64_t)32 * n + i] = 2u;
    return;
  }
#pragma unroll 1
  for (int h = 0; h < 2; h++) {
    uint32_t kk[4];
#pragma unroll
    for (int c = 0; c < 4; c++) kk[c] = h ? k2[c] : k1[c];
    key_table_add<W, NWIN, SIGNED, LAT>(R, inf, tab + (h && !KC ? half : 0), kk, (signs >> h) & 1u, KC && h,
                                        h == 0);
  }
  rg_store(rq, n, i, R, inf);
}

template <bool LAT = false>
DEV uint8_t verify_item_gfinish(uint64_t i, uint64_t n, const uint32_t *item_key, const uint32_t *r_be,
                                const uint32_t *s_be, const uint8_t *pre, const uint8_t *kstatus,
                                const uint32_t *item_msg, const uint32_t *digest_words, const uint32_t *w_in,
                                const uint32_t *g_table, const uint32_t *rq) {
  fe r;
  const uint8_t st = classify_item(i, item_key, r_be, s_be, pre, kstatus, r);
  if (st != 0xFF) return st;
  if (rq[(uint64_t)32 * n + i] == 2u) return BV_DEFERRED;  // no key table (k_verify_qf)
  uint32_t u[8];
  {
    sc w, e, a;
    const uint4 *q = (const uint4 *)(w_in + 8 * i);
    const uint4 x = q[0], y = q[1];
    w.v[0] = x.x; w.v[1] = x.y; w.v[2] = x.z; w.v[3] = x.w;
    w.v[4] = y.x; w.v[5] = y.y; w.v[6] = y.z; w.v[7] = y.w;
    sc_load_be_words(e, digest_words + 8 * (uint64_t)item_msg[i]);
    sc_mont(a, e, w);  // e * s^-1 mod N  (e < 2^256 = R, w < N)
#pragma unroll
    for (int k = 0; k < 8; k++) u[k] = a.v[k];
  }
  gexz R;
  bool inf;
  rg_load(rq, n, i, R, inf);
  g_table_add<BV_GW, BV_GNWIN, LAT>(R, inf, g_table, u);
  fe_load_be_words(r, r_be + 8 * i);
  return final_check(R, inf, r) ? BV_ACCEPT : BV_REJECT;
}

// Key-cache path in ONE pass (k_verify_gq): R = u1 G + k1 T + k2 phi(T) with
// the G table and the key's cached table, R_G kept in registers (no HBM
// round trip of R_G / u12 between two kernels, no kernel boundary).  Same
// decisions as verify_item_g followed by verify_item_q.
template <bool LAT = false>
DEV uint8_t verify_item_gq_kc(uint64_t i, const uint32_t *item_key, const uint32_t *r_be, const uint32_t *s_be,
                              const uint8_t *pre, const uint8_t *kstatus, const uint32_t *item_msg,
                              const uint32_t *digest_words, const uint32_t *w_in, const uint32_t *g_table,
                              const uint64_t *key_tabs) {
  fe r;
  const uint8_t st = classify_item(i, item_key, r_be, s_be, pre, kstatus, r);
  if (st != 0xFF) return st;
  const uint32_t *tab = (const uint32_t *)key_tabs[item_key[i]];
  if (!tab) return BV_DEFERRED;  // partial batch: no table for this key
  uint32_t u[8], k1[4], k2[4], signs;
  item_scalars(i, r_be, item_msg, digest_words, w_in, u, k1, k2, signs);
  gexz R;
  bool inf = true;
  fe_set(R.X, 0);
  fe_set(R.Y, 0);
  fe_set(R.ZZ, 0);
  fe_set(R.ZZZ, 0);
  g_table_add<BV_GW, BV_GNWIN, LAT, gexz, true>(R, inf, g_table, u);
#pragma unroll 1
  for (int h = 0; h < 2; h++) {
    uint32_t kk[4];
#pragma unroll
    for (int c = 0; c < 4; c++) kk[c] = h ? k2[c] : k1[c];
    key_table_add<BV_KCW, BV_KCNWIN, true, LAT>(R, inf, tab, kk, (signs >> h) & 1u, h != 0);
  }
  fe_load_be_words(r, r_be + 8 * i);
  return final_check(R, inf, r) ? BV_ACCEPT : BV_REJECT;
}

// One signature item without a key table: k1 Q + k2 phi(Q) by a joint
// (Strauss-Shamir) per-lane double-and-add over the 128-bit GLV halves.
template <bool LAT = false>
DEV uint8_t verify_item_generic(uint64_t i, const uint32_t *item_key, const uint32_t *r_be, const uint32_t *s_be,
                                const uint8_t *pre, const uint8_t *kstatus, const uint32_t *kxy,
                                const uint32_t *item_msg, const uint32_t *digest_words, const uint32_t *w_in,
                                const uint32_t *g_table) {
  fe r;
  const uint8_t st = classify_item(i, item_key, r_be, s_be, pre, kstatus, r);
  if (st != 0xFF) return st;
  const uint32_t k = item_key[i];
  uint32_t u1[8], k1[4], k2[4], signs;
  item_scalars(i, r_be, item_msg, digest_words, w_in, u1, k1, k2, signs);
  fe q1x, q1y, q2x, q2y, beta;
  fe_load(q1x, kxy + 16 * k);
  fe_load(q1y, kxy + 16 * k + 8);
  fe_load(beta, FE_BETA);
  fe_mul(q2x, q1x, beta);  // phi(Q) = (beta x, y)
  q2y = q1y;
  if (signs & 1u) fe_neg(q1y, q1y);
  if (signs & 2u) fe_neg(q2y, q2y);
  gej R;
  bool inf = true;
  fe_set(R.X, 0);
  fe_set(R.Y, 0);
  fe_set(R.Z, 0);
  for (int bit = 127; bit >= 0; bit--) {
    if (!inf) gej_double_sel<LAT>(R, R);
    if ((k1[bit >> 5] >> (bit & 31)) & 1u) gej_add_ge_sel<LAT>(R, inf, q1x, q1y);
    if ((k2[bit >> 5] >> (bit & 31)) & 1u) gej_add_ge_sel<LAT>(R, inf, q2x, q2y);
  }
  g_table_add<BV_GW, BV_GNWIN, LAT>(R, inf, g_table, u1);
  return final_check(R, inf, r) ? BV_ACCEPT : BV_REJECT;
}

// ---------------------------------------------------------------------------
// Small batches (k_small: one workgroup per item, every step of one item's
// verification in one launch).  The pieces below are the
// per-lane work of its roles.
// ---------------------------------------------------------------------------
// w = s^-1 R (Montgomery form, as k_sinv makes it) for one item: the plain
// inverse R^2 / s of s (taken as (s/R) R), times 1.
DEV void sinv_one(sc &w, const sc &s) {
  sc t, one;
#pragma unroll
  for (int k = 0; k < 8; k++) one.v[k] = k == 0 ? 1u : 0u;
  sc_inverse_var(t, s);
  sc_mont(w, t, one);
}

// u1 = e w and the GLV split of u2 = r w (item_scalars over values)
DEV void scalars_from(const sc &w, const sc &e, const sc &r, uint32_t u1[8], uint32_t k1[4], uint32_t k2[4],
                      uint32_t &signs) {
  sc a, b;
  sc_mont(a, e, w);
  sc_mont(b, r, w);
#pragma unroll
  for (int k = 0; k < 8; k++) u1[k] = a.v[k];
  glv_split(k1, k2, signs, b);
}

// g_table_add over windows [j0, j1) only: the signed recoding runs over
// every window (a digit depends on the carry out of the window below), the
// table additions only in the range — so lanes can sum disjoint ranges.
template <int W, int NWIN, bool LAT = false, class PT = gexz>
DEV void g_table_add_range(PT &R, bool &inf, const uint32_t *tab, uint32_t u[8], int j0, int j1) {
  constexpr uint32_t ENT = 1u << (W - 1);
  uint32_t carry = 0;
  for (int j = 0; j < NWIN; j++) {
    uint32_t d = (u[0] & ((1u << W) - 1u)) + carry;
#pragma unroll
    for (int c = 0; c < 7; c++) u[c] = (u[c] >> W) | (u[c + 1] << (32 - W));
    u[7] >>= W;
    carry = d > ENT ? 1u : 0u;
    const bool dneg = carry != 0;
    if (dneg) d = (1u << W) - d;
    if (j < j0 || j >= j1) continue;
    const uint32_t *e = tab + ((uint64_t)j * ENT + d) * BV_ENTRY_U32;
    fe x, y;
    fe_load4(x, e);
    fe_load4(y, e + 8);
    fe_cneg_canon(y, dneg);
    pt_add_ge_step<LAT>(R, inf, x, y, d != 0);
  }
}

// R = k P for an affine P and a 128-bit k (4 limbs), MSB-first over the
// non-adjacent form of k (digits in {-1, 0, 1}, ~k/3 additions): a key
// without a table (the small-batch kernel's cold path).  pos / neg digit
// masks: c = 3k ^ k, pos = (c & 3k) >> 1, neg = (c & k) >> 1.
template <bool LAT = false>
DEV void naf_mul(gej &R, bool &inf, const fe &px, const fe &py, const uint32_t k[4]) {
  uint32_t h[5], kk[5], pos[5], neg[5];
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) kk[i] = k[i];
  kk[4] = 0;
  // h = 3k = k + 2k
  uint32_t prev = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint32_t k2 = (kk[i] << 1) | (prev >> 31);
    prev = kk[i];
    h[i] = addc32(kk[i], k2, c);
  }
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint32_t x = h[i] ^ kk[i];
    pos[i] = x & h[i];
    neg[i] = x & kk[i];
  }
#pragma unroll
  for (int i = 0; i < 5; i++) {  // >> 1
    pos[i] = (pos[i] >> 1) | (i < 4 ? pos[i + 1] << 31 : 0u);
    neg[i] = (neg[i] >> 1) | (i < 4 ? neg[i + 1] << 31 : 0u);
  }
  fe ny;
  fe_neg(ny, py);
  inf = true;
  fe_set(R.X, 0);
  fe_set(R.Y, 0);
  fe_set(R.Z, 0);
  for (int bit = 129; bit >= 0; bit--) {
    if (!inf) gej_double_sel<LAT>(R, R);
    const uint32_t p = (pos[bit >> 5] >> (bit & 31)) & 1u, n = (neg[bit >> 5] >> (bit & 31)) & 1u;
    if (p | n) gej_add_ge_sel<LAT>(R, inf, px, n ? ny : py);
  }
}

// One leaf of k_small's sum tree: the entry window j of u (NW limbs of 32
// bits, consumed; W-bit SIGNED digits by carry recoding, as g_table_add /
// key_table_add) contributes: (x, y) with y negated for a negative digit,
// XOR `neg` (the GLV half's sign); `phi`: (beta x, y) of the stored entry;
// *zero: the digit is 0 (the leaf is the identity).  The recoding runs over
// windows 0..j (a digit depends on the carry out of the window below).
template <int W, int NW>
DEV void table_leaf(fe &x, fe &y, bool &zero, const uint32_t *tab, uint32_t u[NW], int j, bool neg, bool phi) {
  constexpr uint32_t ENT = 1u << (W - 1);
  uint32_t carry = 0, d = 0;
  for (int w = 0; w <= j; w++) {
    d = (u[0] & ((1u << W) - 1u)) + carry;
#pragma unroll
    for (int c = 0; c < NW - 1; c++) u[c] = (u[c] >> W) | (u[c + 1] << (32 - W));
    u[NW - 1] >>= W;
    carry = d > ENT ? 1u : 0u;
  }
  const bool dneg = carry != 0;
  if (dneg) d = (1u << W) - d;  // |d - 2^W|, 0 when d == 2^W
  zero = d == 0;
  const uint32_t *e = tab + ((uint64_t)j * ENT + d) * BV_ENTRY_U32;  // d == 0: a valid, unused slot
  fe_load4(x, e);
  fe_load4(y, e + 8);
  if (phi) {
    fe beta;
    fe_load(beta, FE_BETA);
    fe_mul(x, x, beta);
  }
  fe_cneg_canon(y, dneg != neg);
}

// One XYZZ partial sum (+ identity flag) in 33 words (LDS hand-off)
DEV void part_store(uint32_t *p, const gexz &R, bool inf) {
#pragma unroll
  for (int k = 0; k < 8; k++) p[k] = R.X.v[k], p[8 + k] = R.Y.v[k], p[16 + k] = R.ZZ.v[k], p[24 + k] = R.ZZZ.v[k];
  p[32] = inf ? 1u : 0u;
}
DEV void part_load(const uint32_t *p, gexz &R, bool &inf) {
#pragma unroll
  for (int k = 0; k < 8; k++) R.X.v[k] = p[k], R.Y.v[k] = p[8 + k], R.ZZ.v[k] = p[16 + k], R.ZZZ.v[k] = p[24 + k];
  inf = p[32] != 0;
}
