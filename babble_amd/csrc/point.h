// point.h — secp256k1 group law on gfx950 (Jacobian coordinates, a = 0).
//
// Semantics follow btcec's KoblitzCurve (src/crypto/keys/curve.go:21):
// the identity is tracked as an explicit flag (btcec's (0,0) / Z = 0), and
// addJacobian's exceptional cases are honoured: P + P doubles, P + (-P) is
// the identity.  These cases are data-dependent and rare, so they are
// branches; an adversarial key or signature that hits them still gets the
// exact group-law answer.
#pragma once
#include "field.h"

struct gej {
  fe X, Y, Z;
};

// dbl-2009-l (a = 0): 2M + 5S.  Caller guarantees the input is not the
// identity; Y == 0 cannot occur on secp256k1 (no 2-torsion, b = 7).
DEV void gej_double(gej &r, const gej &a) {
  fe A, B, C, D, E, F, t;
  fe_sqr(A, a.X);
  fe_sqr(B, a.Y);
  fe_sqr(C, B);
  fe_add(t, a.X, B);
  fe_sqr(t, t);
  fe_sub(t, t, A);
  fe_sub(t, t, C);
  fe_dbl(D, t);
  fe_dbl(E, A);
  fe_add(E, E, A);
  fe_sqr(F, E);
  fe Z3;
  fe_mul(Z3, a.Y, a.Z);
  fe_dbl(r.Z, Z3);
  fe_dbl(t, D);
  fe_sub(r.X, F, t);
  fe_sub(t, D, r.X);
  fe_mul(r.Y, E, t);
  fe_dbl(t, C);
  fe_dbl(t, t);
  fe_dbl(t, t);
  fe_sub(r.Y, r.Y, t);
}

// The same doubling for latency-bound single-wave chains (k_table_bases):
// dbl-2009-l's seven multiplies form three dependent levels,
// {X^2, Y^2, Y Z} -> {B^2, (X + B)^2, E^2} -> E (D - X3), and each of the
// first two runs as ONE interleaved asm program (field_asm.h, gen_zip), so
// a lone wave issues from three independent streams instead of stalling on
// every dependent instruction.  Same values as gej_double; r may alias a.
DEV void gej_double_lat(gej &r, const gej &a) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe A, B, YZ, C, t, E, F, D;
  fe_sqr_sqr_mul_zip_asm(A, a.X, B, a.Y, YZ, a.Y, a.Z);
  fe_add(t, a.X, B);
  fe_dbl(E, A);
  fe_add(E, E, A);
  fe_sqr_sqr_sqr_zip_asm(C, B, t, t, F, E);
  fe_sub(t, t, A);
  fe_sub(t, t, C);
  fe_dbl(D, t);
  fe_dbl(r.Z, YZ);
  fe_dbl(t, D);
  fe_sub(r.X, F, t);
  fe_sub(t, D, r.X);
  fe_mul(r.Y, E, t);
  fe_dbl(t, C);
  fe_dbl(t, t);
  fe_dbl(t, t);
  fe_sub(r.Y, r.Y, t);
#else
  gej_double(r, a);
#endif
}

// r += (x2, y2) (affine): 8M + 3S + 7 add/sub (madd with Z3 = Z1 H; fewer
// additions and live temporaries than madd-2007-bl's 7M + 4S + 11: trading
// one squaring for a multiply costs 30 VALU on gfx950 — fe_sqr 132 against
// fe_mul 162, field_asm.h — while the four extra add/sub would cost 52).
// `inf` is r's identity flag.
DEV void gej_add_ge(gej &r, bool &inf, const fe &x2, const fe &y2) {
  if (inf) {
    r.X = x2;
    r.Y = y2;
    fe_set(r.Z, 1);
    inf = false;
    return;
  }
  fe Z1Z1, U2, S2, H, R, t;
  fe_sqr(Z1Z1, r.Z);
  fe_mul(U2, x2, Z1Z1);
  fe_mul(t, r.Z, Z1Z1);
  fe_mul(S2, y2, t);
  fe_sub(H, U2, r.X);
  fe_sub(R, S2, r.Y);
  if (fe_is_zero(H)) {
    if (fe_is_zero(R)) {
      gej d;
      gej_double(d, r);
      r = d;
    } else {
      inf = true;
    }
    return;
  }
  fe HH, HHH, V;
  fe_sqr(HH, H);
  fe_mul(HHH, H, HH);
  fe_mul(V, r.X, HH);
  fe_mul(r.Z, r.Z, H);
  // X3 = R^2 - HHH - 2V
  fe_sqr(t, R);
  fe_sub(t, t, HHH);
  fe_sub(t, t, V);
  fe_sub(r.X, t, V);
  // Y3 = R (V - X3) - Y1 HHH
  fe_sub(t, V, r.X);
  fe_mul(t, R, t);
  fe_mul(HHH, r.Y, HHH);
  fe_sub(r.Y, t, HHH);
}

// The same mixed addition for latency-bound launches (one or two waves per
// SIMD: small batches, the table fills): its multiplies run as five levels
// {Z1^2} -> {x2 Z1Z1, Z1 Z1Z1} -> {y2 t, H^2} -> {H HH, X1 HH, Z1 H, R^2} ->
// {R (V - X3), Y1 HHH}, each level one interleaved asm program (field_asm.h
// gen_zip).  Same values and exceptional cases as gej_add_ge.
DEV void gej_add_ge_lat(gej &r, bool &inf, const fe &x2, const fe &y2) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (inf) {
    r.X = x2;
    r.Y = y2;
    fe_set(r.Z, 1);
    inf = false;
    return;
  }
  fe Z1Z1, U2, S2, H, R, t, HH, HHH, V, Z3, RR;
  fe_sqr(Z1Z1, r.Z);
  fe_mul_mul_zip_asm(U2, x2, Z1Z1, t, r.Z, Z1Z1);
  fe_sub(H, U2, r.X);
  fe_mul_sqr_zip_asm(S2, y2, t, HH, H);
  fe_sub(R, S2, r.Y);
  if (fe_is_zero(H)) {
    if (fe_is_zero(R)) {
      gej d;
      gej_double_lat(d, r);
      r = d;
    } else {
      inf = true;
    }
    return;
  }
  fe_mul_mul_mul_sqr_zip_asm(HHH, H, HH, V, r.X, HH, Z3, r.Z, H, RR, R);
  r.Z = Z3;
  // X3 = R^2 - HHH - 2V;  Y3 = R (V - X3) - Y1 HHH
  fe_sub(t, RR, HHH);
  fe_sub(t, t, V);
  fe_sub(r.X, t, V);
  fe_sub(t, V, r.X);
  fe_mul_mul_zip_asm(t, R, t, HHH, r.Y, HHH);
  fe_sub(r.Y, t, HHH);
#else
  gej_add_ge(r, inf, x2, y2);
#endif
}

// Point-op selection for kernels with a latency variant (LAT: zipped).
template <bool LAT>
DEV void gej_add_ge_sel(gej &r, bool &inf, const fe &x2, const fe &y2) {
  if (LAT) gej_add_ge_lat(r, inf, x2, y2);
  else gej_add_ge(r, inf, x2, y2);
}
template <bool LAT>
DEV void gej_double_sel(gej &r, const gej &a) {
  if (LAT) gej_double_lat(r, a);
  else gej_double(r, a);
}

// r += b (both Jacobian), add-2007-bl with exceptional cases: 11M + 5S.
DEV void gej_add(gej &r, bool &rinf, const gej &b, bool binf) {
  if (binf) return;
  if (rinf) {
    r = b;
    rinf = false;
    return;
  }
  fe Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, t;
  fe_sqr(Z1Z1, r.Z);
  fe_sqr(Z2Z2, b.Z);
  fe_mul(U1, r.X, Z2Z2);
  fe_mul(U2, b.X, Z1Z1);
  fe_mul(t, b.Z, Z2Z2);
  fe_mul(S1, r.Y, t);
  fe_mul(t, r.Z, Z1Z1);
  fe_mul(S2, b.Y, t);
  fe_sub(H, U2, U1);
  fe_sub(rr, S2, S1);
  if (fe_is_zero(H)) {
    if (fe_is_zero(rr)) {
      gej d;
      gej_double(d, r);
      r = d;
    } else {
      rinf = true;
    }
    return;
  }
  fe_dbl(I, H);
  fe_sqr(I, I);
  fe_mul(J, H, I);
  fe_dbl(rr, rr);
  fe_mul(V, U1, I);
  // Z3 = ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H
  fe_add(t, r.Z, b.Z);
  fe_sqr(t, t);
  fe_sub(t, t, Z1Z1);
  fe_sub(t, t, Z2Z2);
  fe_mul(r.Z, t, H);
  fe_sqr(t, rr);
  fe_sub(t, t, J);
  fe_sub(t, t, V);
  fe_sub(r.X, t, V);
  fe_sub(t, V, r.X);
  fe_mul(t, rr, t);
  fe_mul(J, S1, J);
  fe_dbl(J, J);
  fe_sub(r.Y, t, J);
}

// ---------------------------------------------------------------------------
// Extended Jacobian "XYZZ" coordinates for the verify kernels' accumulators
// (x = X / ZZ, y = Y / ZZZ, ZZ^3 = ZZZ^2): a mixed addition is madd-2008-s,
// 8M + 2S, against 8M + 3S for Jacobian madd (the accumulator's ZZ and ZZZ
// replace Z1^2 and Z1^3: one squaring fewer per table lookup), and the final
// check x(R) == r needs X == r ZZ (1M instead of 1S + 1M).  The verify
// kernels only add affine table points to an accumulator (no doublings), so
// the dearer XYZZ doubling (dbl-2008-s-1) is only the exceptional P + P case.
// Same group law and identity handling as gej (btcec's exceptional cases).
// ---------------------------------------------------------------------------
struct gexz {
  fe X, Y, ZZ, ZZZ;
};

// r = 2 a (dbl-2008-s-1, a = 0): 6M + 3S.  a is not the identity; Y == 0
// cannot occur on secp256k1.
DEV void gexz_double(gexz &r, const gexz &a) {
  fe U, V, W, S, M, t;
  fe_dbl(U, a.Y);
  fe_sqr(V, U);
  fe_mul(W, U, V);
  fe_mul(S, a.X, V);
  fe_sqr(M, a.X);
  fe_dbl(t, M);
  fe_add(M, M, t);            // 3 X1^2
  fe_sqr(t, M);
  fe_dbl(r.X, S);
  fe_sub(r.X, t, r.X);        // M^2 - 2S
  fe_sub(t, S, r.X);
  fe_mul(t, M, t);
  fe_mul(U, W, a.Y);
  fe_sub(r.Y, t, U);          // M (S - X3) - W Y1
  fe_mul(r.ZZ, V, a.ZZ);
  fe_mul(r.ZZZ, W, a.ZZZ);
}

DEV void gexz_set_ge(gexz &r, const fe &x, const fe &y) {
  r.X = x;
  r.Y = y;
  fe_set(r.ZZ, 1);
  fe_set(r.ZZZ, 1);
}

// r += (x2, y2) (affine), madd-2008-s: 8M + 2S + 6 add/sub.
DEV void gexz_add_ge(gexz &r, bool &inf, const fe &x2, const fe &y2) {
  if (inf) {
    gexz_set_ge(r, x2, y2);
    inf = false;
    return;
  }
  fe P, R, PP, PPP, Q, t;
  fe_mul(P, x2, r.ZZ);       // U2
  fe_sub(P, P, r.X);         // P = U2 - X1
  fe_mul(R, y2, r.ZZZ);      // S2
  fe_sub(R, R, r.Y);         // R = S2 - Y1
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) {
      gexz d;
      gexz_double(d, r);
      r = d;
    } else {
      inf = true;
    }
    return;
  }
  fe_sqr(PP, P);
  fe_mul(PPP, P, PP);
  fe_mul(Q, r.X, PP);
  fe_mul(r.ZZ, r.ZZ, PP);
  // X3 = R^2 - PPP - 2Q
  fe_sqr(t, R);
  fe_sub(t, t, PPP);
  fe_sub(t, t, Q);
  fe_sub(r.X, t, Q);
  // Y3 = R (Q - X3) - Y1 PPP, ZZZ3 = ZZZ1 PPP
  fe_sub(t, Q, r.X);
  fe_mul(t, R, t);
  fe_mul(r.ZZZ, r.ZZZ, PPP);
  fe_mul(PPP, r.Y, PPP);
  fe_sub(r.Y, t, PPP);
}

// The same for latency-bound launches: four dependent levels of
// multiplies, each one interleaved asm program (field_asm.h gen_zip):
// {x2 ZZ1, y2 ZZZ1} -> {P^2, R^2} -> {P PP, X1 PP, ZZ1 PP} ->
// {R (Q - X3), Y1 PPP, ZZZ1 PPP}.  Same values and exceptional cases.
DEV void gexz_add_ge_lat(gexz &r, bool &inf, const fe &x2, const fe &y2) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (inf) {
    gexz_set_ge(r, x2, y2);
    inf = false;
    return;
  }
  fe P, R, PP, RR, PPP, Q, ZZ3, t, u;
  fe_mul_mul_zip_asm(P, x2, r.ZZ, R, y2, r.ZZZ);
  fe_sub(P, P, r.X);
  fe_sub(R, R, r.Y);
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) {
      gexz d;
      gexz_double(d, r);
      r = d;
    } else {
      inf = true;
    }
    return;
  }
  fe_sqr_sqr_zip_asm(PP, P, RR, R);
  fe_mul_mul_mul_zip_asm(PPP, P, PP, Q, r.X, PP, ZZ3, r.ZZ, PP);
  r.ZZ = ZZ3;
  fe_sub(t, RR, PPP);
  fe_sub(t, t, Q);
  fe_sub(r.X, t, Q);
  fe_sub(t, Q, r.X);
  fe_mul_mul_mul_zip_asm(t, R, t, u, r.Y, PPP, ZZ3, r.ZZZ, PPP);
  r.ZZZ = ZZ3;
  fe_sub(r.Y, t, u);
#else
  gexz_add_ge(r, inf, x2, y2);
#endif
}

// r += b, both XYZZ (add-2008-s: 12M + 2S) with the exceptional cases:
// either operand the identity, P + P (doubles), P + (-P) (the identity).
// Combines the partial sums of the small-batch kernel (k_small).
DEV void gexz_add(gexz &r, bool &rinf, const gexz &b, bool binf) {
  if (binf) return;
  if (rinf) {
    r = b;
    rinf = false;
    return;
  }
  fe U1, U2, S1, S2, P, R, PP, PPP, Q, t;
  fe_mul(U1, r.X, b.ZZ);
  fe_mul(U2, b.X, r.ZZ);
  fe_mul(S1, r.Y, b.ZZZ);
  fe_mul(S2, b.Y, r.ZZZ);
  fe_sub(P, U2, U1);
  fe_sub(R, S2, S1);
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) {
      gexz d;
      gexz_double(d, r);
      r = d;
    } else {
      rinf = true;
    }
    return;
  }
  fe_sqr(PP, P);
  fe_mul(PPP, P, PP);
  fe_mul(Q, U1, PP);
  fe_sqr(t, R);
  fe_sub(t, t, PPP);
  fe_sub(t, t, Q);
  fe_sub(r.X, t, Q);          // X3 = R^2 - PPP - 2Q
  fe_sub(t, Q, r.X);
  fe_mul(t, R, t);
  fe_mul(S1, S1, PPP);
  fe_sub(r.Y, t, S1);         // Y3 = R (Q - X3) - S1 PPP
  fe_mul(r.ZZ, r.ZZ, b.ZZ);
  fe_mul(r.ZZ, r.ZZ, PP);     // ZZ3 = ZZ1 ZZ2 PP
  fe_mul(r.ZZZ, r.ZZZ, b.ZZZ);
  fe_mul(r.ZZZ, r.ZZZ, PPP);  // ZZZ3 = ZZZ1 ZZZ2 PPP
}

// gexz_add for latency-bound single lanes (k_small's sum tree): its 14
// products in five levels of independent multiplies, each level one zipped
// asm program — {U1, U2, S1} {S2, ZZ1 ZZ2, ZZZ1 ZZZ2} -> {P^2, R^2} ->
// {P PP, U1 PP, ZZ12 PP} -> {R (Q - X3), S1 PPP, ZZZ12 PPP}.  Same values
// and exceptional cases.
DEV void gexz_add_lat(gexz &r, bool &rinf, const gexz &b, bool binf) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (binf) return;
  if (rinf) {
    r = b;
    rinf = false;
    return;
  }
  fe U1, U2, S1, S2, Z12, W12, P, R, PP, RR, PPP, Q, t, u;
  fe_mul_mul_mul_zip_asm(U1, r.X, b.ZZ, U2, b.X, r.ZZ, S1, r.Y, b.ZZZ);
  fe_mul_mul_mul_zip_asm(S2, b.Y, r.ZZZ, Z12, r.ZZ, b.ZZ, W12, r.ZZZ, b.ZZZ);
  fe_sub(P, U2, U1);
  fe_sub(R, S2, S1);
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) {
      gexz d;
      gexz_double(d, r);
      r = d;
    } else {
      rinf = true;
    }
    return;
  }
  fe_sqr_sqr_zip_asm(PP, P, RR, R);
  fe_mul_mul_mul_zip_asm(PPP, P, PP, Q, U1, PP, r.ZZ, Z12, PP);
  fe_sub(t, RR, PPP);
  fe_sub(t, t, Q);
  fe_sub(r.X, t, Q);  // X3 = R^2 - PPP - 2Q
  fe_sub(t, Q, r.X);
  fe_mul_mul_mul_zip_asm(t, R, t, u, S1, PPP, r.ZZZ, W12, PPP);
  fe_sub(r.Y, t, u);  // Y3 = R (Q - X3) - S1 PPP
#else
  gexz_add(r, rinf, b, binf);
#endif
}

// r = (x1, y1) + (x2, y2), two affine points (either may be the identity:
// i1 / i2) into XYZZ — madd-2008-s with Z1 = 1: 4M + 2S in three zipped
// levels {P^2, R^2} -> {P PP, x1 PP} -> {R (Q - X3), y1 PPP}.  The first
// level of k_small's sum tree (table entries are affine).
DEV void gexz_sum_ge_lat(gexz &r, bool &rinf, const fe &x1, const fe &y1, bool i1, const fe &x2, const fe &y2,
                         bool i2) {
  rinf = i1 && i2;
  if (i1 || i2) {
    if (!rinf) gexz_set_ge(r, i1 ? x2 : x1, i1 ? y2 : y1);
    return;
  }
  fe P, R;
  fe_sub(P, x2, x1);
  fe_sub(R, y2, y1);
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) {
      gexz a;
      gexz_set_ge(a, x1, y1);
      gexz_double(r, a);
    } else {
      rinf = true;
    }
    return;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  fe PP, RR, PPP, Q, t, u;
  fe_sqr_sqr_zip_asm(PP, P, RR, R);
  fe_mul_mul_zip_asm(PPP, P, PP, Q, x1, PP);
  fe_sub(t, RR, PPP);
  fe_sub(t, t, Q);
  fe_sub(r.X, t, Q);
  fe_sub(t, Q, r.X);
  fe_mul_mul_zip_asm(t, R, t, u, y1, PPP);
  fe_sub(r.Y, t, u);
  r.ZZ = PP;
  r.ZZZ = PPP;
#else
  gexz_set_ge(r, x1, y1);
  gexz_add_ge(r, rinf, x2, y2);
#endif
}

// Jacobian (X, Y, Z) -> XYZZ (X, Y, Z^2, Z^3): the same point
DEV void gexz_from_gej(gexz &r, const gej &a) {
  r.X = a.X;
  r.Y = a.Y;
  fe_sqr(r.ZZ, a.Z);
  fe_mul(r.ZZZ, r.ZZ, a.Z);
}

template <bool LAT>
DEV void pt_add_ge(gexz &r, bool &inf, const fe &x2, const fe &y2) {
  if (LAT) gexz_add_ge_lat(r, inf, x2, y2);
  else gexz_add_ge(r, inf, x2, y2);
}

// r += (x2, y2) for r AFFINE (ZZ = ZZZ = 1, not the identity: the first
// table entry of a sum), mmadd-2008-s: 4M + 2S — the products by ZZ1 and
// ZZZ1 of the general step drop out (U2 = x2, S2 = y2, ZZ3 = PP, ZZZ3 =
// PPP).  Same exceptional cases as gexz_add_ge.
template <bool LAT>
DEV void gexz_add_ge_aff(gexz &r, bool &inf, const fe &x2, const fe &y2) {
  fe P, R, PP, RR, PPP, Q, t, u, v;
  fe_sub(P, x2, r.X);
  fe_sub(R, y2, r.Y);
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) {
      gexz d;
      gexz_double(d, r);
      r = d;
    } else {
      inf = true;
    }
    return;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  if (LAT) {
    fe_sqr_sqr_zip_asm(PP, P, RR, R);
    fe_mul_mul_zip_asm(PPP, P, PP, Q, r.X, PP);
  } else
#endif
  {
    fe_sqr(PP, P);
    fe_sqr(RR, R);
    fe_mul(PPP, P, PP);
    fe_mul(Q, r.X, PP);
  }
  fe_sub(t, RR, PPP);
  fe_sub(t, t, Q);
  fe_sub(t, t, Q);  // X3
  fe_sub(u, Q, t);
  r.X = t;
  r.ZZ = PP;
  r.ZZZ = PPP;
#if defined(__HIP_DEVICE_COMPILE__)
  if (LAT) {
    fe_mul_mul_zip_asm(t, R, u, v, r.Y, PPP);
  } else
#endif
  {
    fe_mul(t, R, u);
    fe_mul(v, r.Y, PPP);
  }
  fe_sub(r.Y, t, v);
}

// One table lookup step of the verify kernels: r += (x2, y2) in lanes with
// `take` (a nonzero digit).  Measured alternatives (profiles/r03_ab_step.log,
// same-box PMC A/B): a straight-line common path under wave-uniform
// branches for the identity / P == 0 lanes cuts the compiler's phi moves
// (VALU -2 %) but needs more live registers than the 128 of 4 waves per SIMD
// (scratch spills in the loop: k_verify_q +3 %), and the zipped latency
// variants at 2-3 waves per SIMD run 10-15 % slower; this per-lane form
// stays.
template <bool LAT>
DEV void pt_add_ge_step(gexz &r, bool &inf, const fe &x2, const fe &y2, bool take) {
  if (take) pt_add_ge<LAT>(r, inf, x2, y2);
}
template <bool LAT>
DEV void pt_add_ge_step(gej &r, bool &inf, const fe &x2, const fe &y2, bool take) {
  if (take) gej_add_ge_sel<LAT>(r, inf, x2, y2);
}
template <bool LAT>
DEV void pt_add_ge(gej &r, bool &inf, const fe &x2, const fe &y2) {
  gej_add_ge_sel<LAT>(r, inf, x2, y2);
}
