/*
 * CPU ORACLE — test infrastructure only (checker + cpu_baseline "port" leg).
 * Never linked into, loaded by, or called from the product path
 * (babble_amd/, libbabbleverify.so).
 *
 * Plain-C restatement of the reference's verification path, following its
 * control flow call by call:
 *   crypto.SHA256                          src/crypto/hash.go:8-13  (FIPS 180-4)
 *   keys.ToPublicKey -> elliptic.Unmarshal  src/crypto/keys/public_key.go:14-20
 *   keys.Verify -> ecdsa.Verify (Go 1.13 generic path, curve = btcec.S256()):
 *       src/crypto/keys/signature.go:20-22, curve.go:20-22
 *       w = ModInverse(s, N); u1 = e*w mod N; u2 = r*w mod N
 *       (x1,y1) = ScalarBaseMult(u1)      btcec: 8-bit byte-point tables
 *       (x2,y2) = ScalarMult(Q, u2)        btcec: GLV+NAF; restated as a 4-bit
 *                                          fixed window (same group element)
 *       (x,y)   = Add(x1,y1,x2,y2)         btcec: (0,0) identity, doubling,
 *                                          P+(-P) = (0,0)
 *       x==0 && y==0 -> false; return x mod N == r
 *   and the pre-class/panic ordering of SURVEY §8a-9 (event.go:219-247).
 * Third-party semantics (btcec v0.0.0-20190523000118-16327141da8c, Go 1.13
 * stdlib) are absent from the container and restated from their published
 * algorithms; see DESIGN.md §Oracle for how parity is pinned.
 *
 * Arithmetic: 4 x 64-bit limbs with unsigned __int128, fully reduced values.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/babbleverify.h"

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------ */
/* SHA-256 (FIPS 180-4)                                                      */
/* ------------------------------------------------------------------------ */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t h[8], const uint8_t *p) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROTR(w[i - 15], 7) ^ ROTR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROTR(w[i - 2], 17) ^ ROTR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void oracle_sha256(const uint8_t *data, uint64_t len, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint64_t full = len / 64;
  for (uint64_t i = 0; i < full; i++) sha256_block(h, data + 64 * i);
  uint8_t tail[128];
  uint64_t rem = len - 64 * full;
  memset(tail, 0, sizeof tail);
  memcpy(tail, data + 64 * full, rem);
  tail[rem] = 0x80;
  uint64_t tl = (rem + 9 <= 64) ? 64 : 128;
  uint64_t bits = len * 8;
  for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
  sha256_block(h, tail);
  if (tl == 128) sha256_block(h, tail + 64);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = h[i] >> 24; out[4 * i + 1] = h[i] >> 16; out[4 * i + 2] = h[i] >> 8; out[4 * i + 3] = h[i];
  }
}

/* ------------------------------------------------------------------------ */
/* Field mod p = 2^256 - 2^32 - 977                                          */
/* ------------------------------------------------------------------------ */
typedef struct { uint64_t v[4]; } fe;
static const fe FE_P = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
static const uint64_t FE_C = 0x1000003D1ULL; /* 2^256 mod p */

static int u256_ge(const uint64_t *a, const uint64_t *b) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return 1;
}
static uint64_t u256_sub(uint64_t *r, const uint64_t *a, const uint64_t *b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a[i] - b[i] - br;
    r[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
  return br;
}
static uint64_t u256_add(uint64_t *r, const uint64_t *a, const uint64_t *b) {
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a[i] + b[i];
    r[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}
static int fe_is_zero(const fe *a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
static int fe_eq(const fe *a, const fe *b) { return memcmp(a, b, sizeof(fe)) == 0; }

static void fe_add(fe *r, const fe *a, const fe *b) {
  uint64_t c = u256_add(r->v, a->v, b->v);
  if (c || u256_ge(r->v, FE_P.v)) u256_sub(r->v, r->v, FE_P.v);
}
static void fe_sub(fe *r, const fe *a, const fe *b) {
  uint64_t br = u256_sub(r->v, a->v, b->v);
  if (br) u256_add(r->v, r->v, FE_P.v);
}
static void fe_reduce512(fe *r, const uint64_t w[8]) {
  uint64_t t[4];
  u128 acc = 0;
  for (int i = 0; i < 4; i++) {
    acc += (u128)w[i + 4] * FE_C + w[i];
    t[i] = (uint64_t)acc;
    acc >>= 64;
  }
  uint64_t hi = (uint64_t)acc; /* < 2^34 */
  acc = (u128)hi * FE_C + t[0];
  t[0] = (uint64_t)acc;
  acc >>= 64;
  for (int i = 1; i < 4; i++) {
    acc += t[i];
    t[i] = (uint64_t)acc;
    acc >>= 64;
  }
  if (acc) { /* one more wrap: add 2^256 mod p */
    u128 a2 = (u128)t[0] + FE_C;
    t[0] = (uint64_t)a2;
    a2 >>= 64;
    for (int i = 1; i < 4 && a2; i++) {
      a2 += t[i];
      t[i] = (uint64_t)a2;
      a2 >>= 64;
    }
  }
  memcpy(r->v, t, sizeof t);
  if (u256_ge(r->v, FE_P.v)) u256_sub(r->v, r->v, FE_P.v);
}
static void mul256(uint64_t w[8], const uint64_t *a, const uint64_t *b) {
  memset(w, 0, 8 * sizeof(uint64_t));
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a[i] * b[j] + w[i + j];
      w[i + j] = (uint64_t)c;
      c >>= 64;
    }
    w[i + 4] = (uint64_t)c;
  }
}
static void fe_mul(fe *r, const fe *a, const fe *b) {
  uint64_t w[8];
  mul256(w, a->v, b->v);
  fe_reduce512(r, w);
}
static void fe_sqr(fe *r, const fe *a) { fe_mul(r, a, a); }
static void fe_sqrn(fe *r, const fe *a, int n) {
  *r = *a;
  for (int i = 0; i < n; i++) fe_sqr(r, r);
}
/* a^(p-2) via the standard secp256k1 addition chain (255 S + 15 M). */
static void fe_inv(fe *r, const fe *a) {
  fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fe_sqr(&x2, a); fe_mul(&x2, &x2, a);
  fe_sqr(&x3, &x2); fe_mul(&x3, &x3, a);
  fe_sqrn(&x6, &x3, 3); fe_mul(&x6, &x6, &x3);
  fe_sqrn(&x9, &x6, 3); fe_mul(&x9, &x9, &x3);
  fe_sqrn(&x11, &x9, 2); fe_mul(&x11, &x11, &x2);
  fe_sqrn(&x22, &x11, 11); fe_mul(&x22, &x22, &x11);
  fe_sqrn(&x44, &x22, 22); fe_mul(&x44, &x44, &x22);
  fe_sqrn(&x88, &x44, 44); fe_mul(&x88, &x88, &x44);
  fe_sqrn(&x176, &x88, 88); fe_mul(&x176, &x176, &x88);
  fe_sqrn(&x220, &x176, 44); fe_mul(&x220, &x220, &x44);
  fe_sqrn(&x223, &x220, 3); fe_mul(&x223, &x223, &x3);
  fe_sqrn(&t, &x223, 23); fe_mul(&t, &t, &x22);
  fe_sqrn(&t, &t, 5); fe_mul(&t, &t, a);
  fe_sqrn(&t, &t, 3); fe_mul(&t, &t, &x2);
  fe_sqrn(&t, &t, 2); fe_mul(r, &t, a);
}
static void fe_from_be(fe *r, const uint8_t *b) {
  for (int i = 0; i < 4; i++) {
    uint64_t x = 0;
    for (int j = 0; j < 8; j++) x = (x << 8) | b[(3 - i) * 8 + j];
    r->v[i] = x;
  }
}

/* ------------------------------------------------------------------------ */
/* Scalars mod N                                                             */
/* ------------------------------------------------------------------------ */
static const uint64_t SC_N[4] = {0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL};
static const uint64_t SC_CN[3] = {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 0x1ULL}; /* 2^256 - N */

/* r = (hi * CN + lo) folded until < 2^256, then < N */
static void sc_reduce512(uint64_t r[4], const uint64_t w[8]) {
  uint64_t t[8];
  memcpy(t, w, sizeof t);
  for (int round = 0; round < 4; round++) {
    uint64_t hi[4] = {t[4], t[5], t[6], t[7]};
    if ((hi[0] | hi[1] | hi[2] | hi[3]) == 0) break;
    uint64_t acc[8] = {t[0], t[1], t[2], t[3], 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
      u128 c = 0;
      for (int j = 0; j < 3; j++) {
        c += (u128)hi[i] * SC_CN[j] + acc[i + j];
        acc[i + j] = (uint64_t)c;
        c >>= 64;
      }
      for (int k = i + 3; k < 8 && c; k++) {
        c += acc[k];
        acc[k] = (uint64_t)c;
        c >>= 64;
      }
    }
    memcpy(t, acc, sizeof t);
  }
  memcpy(r, t, 4 * sizeof(uint64_t));
  while (u256_ge(r, SC_N)) u256_sub(r, r, SC_N);
}
static void sc_mul(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t w[8];
  mul256(w, a, b);
  sc_reduce512(r, w);
}
static void sc_inv(uint64_t r[4], const uint64_t a[4]) { /* a^(N-2), square-and-multiply */
  uint64_t e[4], acc[4] = {1, 0, 0, 0};
  const uint64_t two[4] = {2, 0, 0, 0};
  u256_sub(e, SC_N, two);
  for (int i = 255; i >= 0; i--) {
    sc_mul(acc, acc, acc);
    if ((e[i / 64] >> (i % 64)) & 1) sc_mul(acc, acc, a);
  }
  memcpy(r, acc, sizeof acc);
}
static void u256_from_be(uint64_t r[4], const uint8_t *b) {
  fe t;
  fe_from_be(&t, b);
  memcpy(r, t.v, sizeof t.v);
}

/* ------------------------------------------------------------------------ */
/* Points (Jacobian; Z = 0 is infinity)                                      */
/* ------------------------------------------------------------------------ */
typedef struct { fe X, Y, Z; } gej;
typedef struct { fe x, y; int inf; } ge;

static void gej_set_inf(gej *r) { memset(r, 0, sizeof *r); }
static int gej_is_inf(const gej *a) { return fe_is_zero(&a->Z); }

static void gej_double(gej *r, const gej *a) { /* dbl-2009-l, a = 0 */
  if (gej_is_inf(a) || fe_is_zero(&a->Y)) { gej_set_inf(r); return; }
  fe A, B, C, D, E, F, t, X3, Y3, Z3;
  fe_sqr(&A, &a->X);
  fe_sqr(&B, &a->Y);
  fe_sqr(&C, &B);
  fe_add(&t, &a->X, &B); fe_sqr(&t, &t); fe_sub(&t, &t, &A); fe_sub(&t, &t, &C); fe_add(&D, &t, &t);
  fe_add(&E, &A, &A); fe_add(&E, &E, &A);
  fe_sqr(&F, &E);
  fe_add(&t, &D, &D); fe_sub(&X3, &F, &t);
  fe_sub(&t, &D, &X3); fe_mul(&Y3, &E, &t);
  fe_add(&t, &C, &C); fe_add(&t, &t, &t); fe_add(&t, &t, &t); fe_sub(&Y3, &Y3, &t);
  fe_mul(&Z3, &a->Y, &a->Z); fe_add(&Z3, &Z3, &Z3);
  r->X = X3; r->Y = Y3; r->Z = Z3;
}

static void gej_add(gej *r, const gej *a, const gej *b) { /* add-2007-bl + exceptional cases */
  if (gej_is_inf(a)) { *r = *b; return; }
  if (gej_is_inf(b)) { *r = *a; return; }
  fe Z1Z1, Z2Z2, U1, U2, S1, S2, H, Rr, t, HH, HHH, V, X3, Y3, Z3;
  fe_sqr(&Z1Z1, &a->Z);
  fe_sqr(&Z2Z2, &b->Z);
  fe_mul(&U1, &a->X, &Z2Z2);
  fe_mul(&U2, &b->X, &Z1Z1);
  fe_mul(&t, &b->Z, &Z2Z2); fe_mul(&S1, &a->Y, &t);
  fe_mul(&t, &a->Z, &Z1Z1); fe_mul(&S2, &b->Y, &t);
  fe_sub(&H, &U2, &U1);
  fe_sub(&Rr, &S2, &S1);
  if (fe_is_zero(&H)) {
    if (fe_is_zero(&Rr)) { gej_double(r, a); return; }
    gej_set_inf(r);
    return;
  }
  fe_sqr(&HH, &H);
  fe_mul(&HHH, &H, &HH);
  fe_mul(&V, &U1, &HH);
  fe_sqr(&X3, &Rr); fe_sub(&X3, &X3, &HHH); fe_sub(&X3, &X3, &V); fe_sub(&X3, &X3, &V);
  fe_sub(&t, &V, &X3); fe_mul(&Y3, &Rr, &t); fe_mul(&t, &S1, &HHH); fe_sub(&Y3, &Y3, &t);
  fe_mul(&Z3, &a->Z, &b->Z); fe_mul(&Z3, &Z3, &H);
  r->X = X3; r->Y = Y3; r->Z = Z3;
}

static void gej_to_ge(ge *r, const gej *a) { /* fieldJacobianToBigAffine: inf -> (0,0) */
  if (gej_is_inf(a)) { memset(r, 0, sizeof *r); r->inf = 1; return; }
  fe zi, zi2, zi3;
  fe_inv(&zi, &a->Z);
  fe_sqr(&zi2, &zi);
  fe_mul(&zi3, &zi2, &zi);
  fe_mul(&r->x, &a->X, &zi2);
  fe_mul(&r->y, &a->Y, &zi3);
  r->inf = 0;
}
static void ge_to_gej(gej *r, const ge *a) {
  if (a->inf) { gej_set_inf(r); return; }
  r->X = a->x; r->Y = a->y;
  memset(&r->Z, 0, sizeof r->Z);
  r->Z.v[0] = 1;
}

static const uint8_t G_BE[65] = {
    0x04, 0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0, 0x62, 0x95, 0xCE, 0x87, 0x0B, 0x07,
    0x02, 0x9B, 0xFC, 0xDB, 0x2D, 0xCE, 0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98,
    0x48, 0x3A, 0xDA, 0x77, 0x26, 0xA3, 0xC4, 0x65, 0x5D, 0xA4, 0xFB, 0xFC, 0x0E, 0x11, 0x08, 0xA8,
    0xFD, 0x17, 0xB4, 0x48, 0xA6, 0x85, 0x54, 0x19, 0x9C, 0x47, 0xD0, 0x8F, 0xFB, 0x10, 0xD4, 0xB8};

/* btcec-style ScalarBaseMult tables: BYTEPTS[i][b] = b * 256^(31-i) * G (affine). */
static ge BYTEPTS[32][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void init_tables(void) {
  ge g;
  fe_from_be(&g.x, G_BE + 1);
  fe_from_be(&g.y, G_BE + 33);
  g.inf = 0;
  gej base;
  ge_to_gej(&base, &g);
  for (int i = 31; i >= 0; i--) {
    gej acc;
    gej_set_inf(&acc);
    BYTEPTS[i][0].inf = 1;
    for (int b = 1; b < 256; b++) {
      gej_add(&acc, &acc, &base);
      gej_to_ge(&BYTEPTS[i][b], &acc);
    }
    for (int d = 0; d < 8; d++) gej_double(&base, &base);
  }
}

/* ScalarBaseMult(k) with k given as 32 BE bytes (u1 < N). */
static void scalar_base_mult(gej *r, const uint8_t k[32]) {
  gej_set_inf(r);
  for (int i = 0; i < 32; i++) {
    if (k[i] == 0) continue;
    gej p;
    ge_to_gej(&p, &BYTEPTS[i][k[i]]);
    gej_add(r, r, &p);
  }
}

/* ScalarMult(Q, k): 4-bit fixed window, MSB first. */
static void scalar_mult(gej *r, const ge *q, const uint8_t k[32]) {
  gej tab[16];
  gej_set_inf(&tab[0]);
  ge_to_gej(&tab[1], q);
  for (int i = 2; i < 16; i++) gej_add(&tab[i], &tab[i - 1], &tab[1]);
  gej_set_inf(r);
  for (int i = 0; i < 64; i++) {
    for (int d = 0; d < 4; d++) gej_double(r, r);
    int nib = (k[i / 2] >> ((i & 1) ? 0 : 4)) & 15;
    if (nib) gej_add(r, r, &tab[nib]);
  }
}

static void u256_to_be(uint8_t *b, const uint64_t v[4]) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) b[(3 - i) * 8 + j] = (uint8_t)(v[i] >> (56 - 8 * j));
}

/* elliptic.Unmarshal(btcec.S256(), pub): 1 = ok. */
int oracle_unmarshal(const uint8_t *pub, uint64_t len, uint8_t xy_out[64]) {
  if (len != 65 || pub[0] != 4) return 0;
  fe x, y, y2, x3;
  fe_from_be(&x, pub + 1);
  fe_from_be(&y, pub + 33);
  if (u256_ge(x.v, FE_P.v) || u256_ge(y.v, FE_P.v)) return 0;
  fe_sqr(&y2, &y);
  fe_sqr(&x3, &x);
  fe_mul(&x3, &x3, &x);
  fe seven = {{7, 0, 0, 0}};
  fe_add(&x3, &x3, &seven);
  if (!fe_eq(&y2, &x3)) return 0;
  if (xy_out) memcpy(xy_out, pub + 1, 64);
  return 1;
}

/* ecdsa.Verify steps 4-10 for r, s in [1, N-1] and a valid key. */
static int ecdsa_math(const uint8_t *pub65, const uint8_t digest[32], const uint8_t r_be[32], const uint8_t s_be[32]) {
  pthread_once(&g_once, init_tables);
  uint64_t e[4], r[4], s[4], w[4], u1[4], u2[4];
  u256_from_be(e, digest);
  u256_from_be(r, r_be);
  u256_from_be(s, s_be);
  sc_inv(w, s);                 /* w = ModInverse(s, N) */
  sc_mul(u1, e, w);             /* e may be >= N: sc_mul reduces the product */
  sc_mul(u2, r, w);
  uint8_t u1b[32], u2b[32];
  u256_to_be(u1b, u1);
  u256_to_be(u2b, u2);
  ge q;
  fe_from_be(&q.x, pub65 + 1);
  fe_from_be(&q.y, pub65 + 33);
  q.inf = 0;
  gej j1, j2, jr;
  ge a1, a2, ar;
  scalar_base_mult(&j1, u1b);
  gej_to_ge(&a1, &j1);          /* big affine, inf -> (0,0) */
  scalar_mult(&j2, &q, u2b);
  gej_to_ge(&a2, &j2);
  /* Add(x1,y1,x2,y2): (0,0) is the identity */
  if (a1.inf) ar = a2;
  else if (a2.inf) ar = a1;
  else {
    gej p1, p2;
    ge_to_gej(&p1, &a1);
    ge_to_gej(&p2, &a2);
    gej_add(&jr, &p1, &p2);
    gej_to_ge(&ar, &jr);
  }
  if (ar.inf) return 0;         /* x.Sign()==0 && y.Sign()==0 */
  uint64_t x[4];
  memcpy(x, ar.x.v, sizeof x);
  if (u256_ge(x, SC_N)) u256_sub(x, x, SC_N); /* x mod N (x < p < 2N) */
  return memcmp(x, r, sizeof x) == 0;
}

/* Steps (1)-(6) of SURVEY §8a-9: the final status, or -1 when the item
 * reaches the ECDSA math. */
static int oracle_item_status_pre(const uint8_t *pub, uint64_t publen, uint8_t pre, const uint8_t r_be[32],
                                  const uint8_t s_be[32]) {
  if (pre & BV_PRE_PARTS_BAD) return BV_REJECT_ERR;
  if (publen == 0) return BV_REF_PANIC;
  int rc = pre & 3, sc = (pre >> 2) & 3;
  /* ABI rule (babbleverify.h): a class-OK value is re-checked against its
   * bytes, so r = 0 reads as "<= 0" and r >= N as ">= N". */
  uint64_t rv[4], sv[4];
  u256_from_be(rv, r_be);
  u256_from_be(sv, s_be);
  if (rc == BV_SC_OK) rc = (rv[0] | rv[1] | rv[2] | rv[3]) == 0 ? BV_SC_NONPOS : (u256_ge(rv, SC_N) ? BV_SC_GE_N : BV_SC_OK);
  if (sc == BV_SC_OK) sc = (sv[0] | sv[1] | sv[2] | sv[3]) == 0 ? BV_SC_NONPOS : (u256_ge(sv, SC_N) ? BV_SC_GE_N : BV_SC_OK);
  if (rc == BV_SC_NIL) return BV_REF_PANIC;
  if (rc == BV_SC_NONPOS) return BV_REJECT;
  if (sc == BV_SC_NIL) return BV_REF_PANIC;
  if (sc == BV_SC_NONPOS) return BV_REJECT;
  if (rc == BV_SC_GE_N || sc == BV_SC_GE_N) return BV_REJECT;
  if (!oracle_unmarshal(pub, publen, NULL)) return BV_REF_PANIC;
  return -1;
}

/* One item, SURVEY §8a-9 ordering. */
int oracle_item_status(const uint8_t *pub, uint64_t publen, const uint8_t digest[32], uint8_t pre,
                       const uint8_t r_be[32], const uint8_t s_be[32]) {
  const int st = oracle_item_status_pre(pub, publen, pre, r_be, s_be);
  if (st >= 0) return st;
  return ecdsa_math(pub, digest, r_be, s_be) ? BV_ACCEPT : BV_REJECT;
}

/* Point helpers exposed for known-answer tests: k*G affine (64 BE bytes). */
int oracle_scalar_base_mult(const uint8_t k_be[32], uint8_t xy_out[64]) {
  pthread_once(&g_once, init_tables);
  gej j;
  ge a;
  scalar_base_mult(&j, k_be);
  gej_to_ge(&a, &j);
  if (a.inf) return 0;
  uint8_t *o = xy_out;
  u256_to_be(o, a.x.v);
  u256_to_be(o + 32, a.y.v);
  return 1;
}

/* ------------------------------------------------------------------------ */
/* Batch driver (pthreads)                                                   */
/* ------------------------------------------------------------------------ */
int port_item_status(const uint8_t *pub, uint64_t publen, const uint8_t digest[32], uint8_t pre,
                     const uint8_t r_be[32], const uint8_t s_be[32]);

typedef struct {
  const bv_batch *b;
  uint8_t *hash;
  uint8_t *status;
  uint64_t lo, hi;
  int phase;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  const bv_batch *b = j->b;
  if (j->phase == 0) {
    for (uint64_t m = j->lo; m < j->hi; m++)
      oracle_sha256(b->msg_bytes + b->msg_off[m], b->msg_off[m + 1] - b->msg_off[m], j->hash + 32 * m);
  } else {
    for (uint64_t i = j->lo; i < j->hi; i++) {
      uint32_t k = b->item_key[i];
      const uint8_t *pub = b->key_bytes + b->key_off[k];
      uint64_t publen = b->key_off[k + 1] - b->key_off[k];
      uint8_t pre = b->pre ? b->pre[i] : 0;
      const uint8_t *dg = j->hash + 32 * (uint64_t)b->item_msg[i];
      j->status[i] = (uint8_t)(j->phase == 2 ? port_item_status(pub, publen, dg, pre, b->r_be + 32 * i, b->s_be + 32 * i)
                                              : oracle_item_status(pub, publen, dg, pre, b->r_be + 32 * i, b->s_be + 32 * i));
    }
  }
  return NULL;
}

/* A persistent pool (the CPU comparators must not pay a
 * thread spawn and join per call): workers are created on first need and
 * sleep between calls; a phase uses min(n_threads, items) participants —
 * the caller plus workers — pulling chunks from an atomic counter, and a
 * one-participant phase runs inline on the caller. */
#define POOL_MAX 256
static pthread_mutex_t g_pmu = PTHREAD_MUTEX_INITIALIZER;   /* one phase at a time */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_go = PTHREAD_COND_INITIALIZER, g_fin = PTHREAD_COND_INITIALIZER;
static int g_workers, g_want, g_left;
static uint64_t g_gen;
static struct {
  const bv_batch *b;
  uint8_t *hash, *status;
  uint64_t n, chunk;
  int phase;
  uint64_t next; /* atomic */
} g_task;

static void run_chunks(void) {
  for (;;) {
    const uint64_t lo = __atomic_fetch_add(&g_task.next, g_task.chunk, __ATOMIC_RELAXED);
    if (lo >= g_task.n) return;
    job_t j = {g_task.b, g_task.hash, g_task.status, lo, lo + g_task.chunk < g_task.n ? lo + g_task.chunk : g_task.n,
               g_task.phase};
    worker(&j);
  }
}

static void *pool_main(void *arg) {
  const int id = (int)(intptr_t)arg;
  uint64_t seen = 0;
  pthread_mutex_lock(&g_mu);
  for (;;) {
    while (g_gen == seen || id >= g_want) {
      if (g_gen != seen) seen = g_gen; /* not a participant of this phase */
      pthread_cond_wait(&g_go, &g_mu);
    }
    seen = g_gen;
    pthread_mutex_unlock(&g_mu);
    run_chunks();
    pthread_mutex_lock(&g_mu);
    if (--g_left == 0) pthread_cond_signal(&g_fin);
  }
  return NULL;
}

static void run_phase(const bv_batch *b, uint8_t *hash, uint8_t *status, uint64_t n, int phase, int nt) {
  if (nt < 1) nt = 1;
  if (nt > POOL_MAX) nt = POOL_MAX;
  /* hashing is ~1 us a message: don't wake a thread for fewer than 256 */
  const uint64_t grain = phase == 0 ? 256 : 1;
  const uint64_t max_part = (n + grain - 1) / grain;
  const int k = (uint64_t)nt < max_part ? nt : (int)max_part;
  if (k <= 1) {
    job_t j = {b, hash, status, 0, n, phase};
    worker(&j);
    return;
  }
  pthread_mutex_lock(&g_pmu);
  pthread_mutex_lock(&g_mu);
  while (g_workers < k - 1) {
    pthread_t t;
    pthread_create(&t, NULL, pool_main, (void *)(intptr_t)g_workers);
    pthread_detach(t);
    g_workers++;
  }
  g_task.b = b;
  g_task.hash = hash;
  g_task.status = status;
  g_task.n = n;
  g_task.phase = phase;
  g_task.chunk = n / ((uint64_t)k * 4) ? n / ((uint64_t)k * 4) : 1;
  g_task.chunk = g_task.chunk > grain ? g_task.chunk : grain;
  __atomic_store_n(&g_task.next, 0, __ATOMIC_RELAXED);
  g_want = k - 1;
  g_left = k - 1;
  g_gen++;
  pthread_cond_broadcast(&g_go);
  pthread_mutex_unlock(&g_mu);
  run_chunks();
  pthread_mutex_lock(&g_mu);
  while (g_left > 0) pthread_cond_wait(&g_fin, &g_mu);
  pthread_mutex_unlock(&g_mu);
  pthread_mutex_unlock(&g_pmu);
}

/* Verify a whole batch on the CPU: the oracle for parity tests and the
 * cpu_baseline "port" timing.  msg_hash must hold 32*n_msgs bytes. */
int oracle_verify_batch(const bv_batch *b, uint8_t *msg_hash, uint8_t *status, uint64_t *accept_bits, int n_threads) {
  pthread_once(&g_once, init_tables);
  run_phase(b, msg_hash, status, b->n_msgs, 0, n_threads);
  run_phase(b, msg_hash, status, b->n_items, 1, n_threads);
  if (accept_bits) {
    uint64_t nw = (b->n_items + 63) / 64;
    memset(accept_bits, 0, nw * 8);
    for (uint64_t i = 0; i < b->n_items; i++)
      if (status[i] == BV_ACCEPT) accept_bits[i / 64] |= 1ULL << (i % 64);
  }
  return 0;
}

/* The same batch through the btcec-algorithm port (cpu_baseline timing). */
int port_verify_batch(const bv_batch *b, uint8_t *msg_hash, uint8_t *status, int n_threads) {
  pthread_once(&g_once, init_tables);
  run_phase(b, msg_hash, status, b->n_msgs, 0, n_threads);
  run_phase(b, msg_hash, status, b->n_items, 2, n_threads);
  return 0;
}

void oracle_init(void) { pthread_once(&g_once, init_tables); }

/* ------------------------------------------------------------------------ */
/* btcec-algorithm PORT — the cpu_baseline "port" leg (timing only; the     */
/* checker above stays the simple restatement).  Same decisions as          */
/* oracle_item_status; the two scalar multiplications follow the reference  */
/* stack's own algorithms (btcec v0.0.0-20190523000118-16327141da8c, called  */
/* by Go 1.13 ecdsa.Verify, src/crypto/keys/signature.go:20-22):            */
/*   ScalarBaseMult: the 32 x 256 byte-point tables, mixed additions;       */
/*   ScalarMult:     GLV split k = k1 + k2 lambda (|k1|, |k2| < 2^128), NAF */
/*                   of both halves, one joint double-and-add over Q and    */
/*                   phi(Q) = (beta x, y) with mixed additions;             */
/*   Add:            affine in, Jacobian sum, affine out (3 inversions in   */
/*                   all, as fieldJacobianToBigAffine does).                */
/* ------------------------------------------------------------------------ */
static const uint64_t GLV_G1[4] = {0xE893209A45DBB031ULL, 0x3DAA8A1471E8CA7FULL, 0xE86C90E49284EB15ULL, 0x3086D221A7D46BCDULL};
static const uint64_t GLV_G2[4] = {0x1571B4AE8AC47F71ULL, 0x221208AC9DF506C6ULL, 0x6F547FA90ABFE4C4ULL, 0xE4437ED6010E8828ULL};
static const uint64_t GLV_MB1[4] = {0x6F547FA90ABFE4C3ULL, 0xE4437ED6010E8828ULL, 0, 0};
static const uint64_t GLV_MB2[4] = {0xD765CDA83DB1562CULL, 0x8A280AC50774346DULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL};
static const uint64_t GLV_LAM[4] = {0xDF02967C1B23BD72ULL, 0x122E22EA20816678ULL, 0xA5261C028812645AULL, 0x5363AD4CC05C30E0ULL};
static const fe FE_BETA64 = {{0xC1396C28719501EEULL, 0x9CF0497512F58995ULL, 0x6E64479EAC3434E9ULL, 0x7AE96A2B657C0710ULL}};

/* round(k g / 2^384) */
static void glv_mulshift(uint64_t c[4], const uint64_t k[4], const uint64_t g[4]) {
  uint64_t w[8];
  mul256(w, k, g);
  const uint64_t rnd = (w[5] >> 63) & 1; /* bit 383 */
  u128 s = (u128)w[6] + rnd;
  c[0] = (uint64_t)s; s >>= 64;
  s += w[7];
  c[1] = (uint64_t)s;
  c[2] = c[3] = 0;
}

/* k = k1 + k2 lambda (mod N): magnitudes < 2^128 and signs (1 = negative) */
static void glv_split(const uint64_t k[4], uint64_t m1[2], int *neg1, uint64_t m2[2], int *neg2) {
  uint64_t c1[4], c2[4], t1[4], t2[4], k1[4], k2[4], half[4];
  glv_mulshift(c1, k, GLV_G1);
  glv_mulshift(c2, k, GLV_G2);
  sc_mul(t1, c1, GLV_MB1);
  sc_mul(t2, c2, GLV_MB2);
  if (u256_add(k2, t1, t2) || u256_ge(k2, SC_N)) u256_sub(k2, k2, SC_N);
  sc_mul(t1, k2, GLV_LAM);
  if (u256_sub(k1, k, t1)) u256_add(k1, k1, SC_N);
  /* N/2 rounded up: values above it are negative */
  memcpy(half, SC_N, sizeof half);
  for (int i = 0; i < 3; i++) half[i] = (half[i] >> 1) | (half[i + 1] << 63);
  half[3] >>= 1;
  uint64_t *ks[2] = {k1, k2}, *ms[2] = {m1, m2};
  int *ns[2] = {neg1, neg2};
  for (int h = 0; h < 2; h++) {
    uint64_t v[4];
    memcpy(v, ks[h], sizeof v);
    *ns[h] = u256_ge(v, half) && !(v[0] == half[0] && v[1] == half[1] && v[2] == half[2] && v[3] == half[3]);
    if (*ns[h]) u256_sub(v, SC_N, v);
    ms[h][0] = v[0];
    ms[h][1] = v[1];
  }
}

/* width-2 NAF of a < 2^128 magnitude: digits in {-1, 0, 1}, LSB first; returns the length */
static int naf128(int8_t d[130], const uint64_t m[2]) {
  u128 k = ((u128)m[1] << 64) | m[0];
  uint64_t top = 0; /* k may become 2^128 after a -1 digit */
  int n = 0;
  while (k || top) {
    int8_t z = 0;
    if (k & 1) {
      z = (k & 3) == 3 ? -1 : 1;
      if (z == 1) k -= 1;
      else { u128 k2 = k + 1; if (k2 == 0) top = 1; k = k2; }
    }
    d[n++] = z;
    k = (k >> 1) | ((u128)top << 127);
    top = 0;
  }
  return n;
}

/* r += b (affine, not the identity): btcec's addZ2EqualsOne, 8M + 3S, with
 * its doubling and P + (-P) cases */
static void gej_add_ge(gej *r, const ge *b) {
  if (gej_is_inf(r)) { ge_to_gej(r, b); return; }
  fe Z1Z1, U2, S2, H, R, HH, HHH, V, t;
  fe_sqr(&Z1Z1, &r->Z);
  fe_mul(&U2, &b->x, &Z1Z1);
  fe_mul(&t, &r->Z, &Z1Z1);
  fe_mul(&S2, &b->y, &t);
  fe_sub(&H, &U2, &r->X);
  fe_sub(&R, &S2, &r->Y);
  if (fe_is_zero(&H)) {
    if (fe_is_zero(&R)) gej_double(r, r);
    else gej_set_inf(r);
    return;
  }
  fe_sqr(&HH, &H);
  fe_mul(&HHH, &H, &HH);
  fe_mul(&V, &r->X, &HH);
  fe_mul(&r->Z, &r->Z, &H);
  fe X3;
  fe_sqr(&X3, &R); fe_sub(&X3, &X3, &HHH); fe_sub(&X3, &X3, &V); fe_sub(&X3, &X3, &V);
  fe_sub(&t, &V, &X3); fe_mul(&t, &R, &t);
  fe_mul(&HHH, &r->Y, &HHH);
  fe_sub(&r->Y, &t, &HHH);
  r->X = X3;
}

static void port_scalar_base_mult(gej *r, const uint8_t k[32]) {
  gej_set_inf(r);
  for (int i = 0; i < 32; i++)
    if (k[i]) gej_add_ge(r, &BYTEPTS[i][k[i]]);
}

static void port_scalar_mult(gej *r, const ge *q, const uint64_t k[4]) {
  uint64_t m1[2], m2[2];
  int n1, n2;
  glv_split(k, m1, &n1, m2, &n2);
  ge p1 = *q, p2 = *q, p1n, p2n;
  fe_mul(&p2.x, &q->x, &FE_BETA64); /* phi(Q) = (beta x, y) */
  const fe zero = {{0, 0, 0, 0}};
  if (n1) fe_sub(&p1.y, &zero, &p1.y);
  if (n2) fe_sub(&p2.y, &zero, &p2.y);
  p1n = p1; fe_sub(&p1n.y, &zero, &p1.y);
  p2n = p2; fe_sub(&p2n.y, &zero, &p2.y);
  int8_t d1[130] = {0}, d2[130] = {0};
  const int l1 = naf128(d1, m1), l2 = naf128(d2, m2);
  gej_set_inf(r);
  for (int i = (l1 > l2 ? l1 : l2) - 1; i >= 0; i--) {
    if (!gej_is_inf(r)) gej_double(r, r);
    if (d1[i] == 1) gej_add_ge(r, &p1);
    else if (d1[i] == -1) gej_add_ge(r, &p1n);
    if (d2[i] == 1) gej_add_ge(r, &p2);
    else if (d2[i] == -1) gej_add_ge(r, &p2n);
  }
}

static int port_ecdsa_math(const uint8_t *pub65, const uint8_t digest[32], const uint8_t r_be[32],
                           const uint8_t s_be[32]) {
  uint64_t e[4], r[4], s[4], w[4], u1[4], u2[4];
  u256_from_be(e, digest);
  u256_from_be(r, r_be);
  u256_from_be(s, s_be);
  sc_inv(w, s);
  sc_mul(u1, e, w);
  sc_mul(u2, r, w);
  uint8_t u1b[32];
  u256_to_be(u1b, u1);
  ge q;
  fe_from_be(&q.x, pub65 + 1);
  fe_from_be(&q.y, pub65 + 33);
  q.inf = 0;
  gej j1, j2, jr;
  ge a1, a2, ar;
  port_scalar_base_mult(&j1, u1b);
  gej_to_ge(&a1, &j1);
  port_scalar_mult(&j2, &q, u2);
  gej_to_ge(&a2, &j2);
  if (a1.inf) ar = a2;
  else if (a2.inf) ar = a1;
  else {
    gej p1;
    ge_to_gej(&p1, &a1);
    jr = p1;
    gej_add_ge(&jr, &a2);
    gej_to_ge(&ar, &jr);
  }
  if (ar.inf) return 0;
  uint64_t x[4];
  memcpy(x, ar.x.v, sizeof x);
  if (u256_ge(x, SC_N)) u256_sub(x, x, SC_N);
  return memcmp(x, r, sizeof x) == 0;
}

/* One item through the port: the oracle's decision order, btcec's algorithms. */
int port_item_status(const uint8_t *pub, uint64_t publen, const uint8_t digest[32], uint8_t pre,
                     const uint8_t r_be[32], const uint8_t s_be[32]) {
  pthread_once(&g_once, init_tables);
  const int st = oracle_item_status_pre(pub, publen, pre, r_be, s_be);
  if (st >= 0) return st;
  return port_ecdsa_math(pub, digest, r_be, s_be) ? BV_ACCEPT : BV_REJECT;
}
