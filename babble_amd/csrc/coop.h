// coop.h — wave-cooperative field arithmetic mod p for latency-bound chains
// (the north star's "wavefront-cooperative carry propagation").
//
// A lone wave that walks a serial chain (the key tables' base chain
// 2^(L j) Q: ~120 doublings per key) is bound by the dependent-instruction
// latency of ONE lane's field multiply (~440 ns, profiles/r03_ubench_coop.txt),
// not by issue slots: 63 lanes idle.  Here a field element lives in a 16-lane
// DPP row — limb k (32 bits) in lane k < 8 of the row, zeros in lanes 8..15 —
// so one multiply is ~8 short column steps per lane instead of ~160
// instructions, and the wave's four rows run up to four DIFFERENT multiplies
// at once (the independent products of one doubling level).
//
// Carries between limbs are resolved with a carry-lookahead over wave-wide
// lane masks: G = lanes whose digit carries out, P = lanes whose digit is
// 0xFFFFFFFF; the carries INTO the lanes are ((G << 1) + P) ^ P.  A product
// or a norm() runs ONE such resolve (two ballots and the scalar adds on its
// dependent chain): the 2^256 folds work on unresolved 33-bit digits, with
// one DPP carry-save step each (round 6; three resolves before).  The bounds
// are checked digit by digit by a Python model of these functions
// (tests/test_coop_model.py).
//
// Forms:  NORMAL  lanes 0..7 hold the limbs of a value < 2^256 (weakly
//                 reduced mod p), lanes 8..15 hold 0 — what mul() takes and
//                 returns;
//         WIDE    a 64-bit value per lane (lanes 0..8), value =
//                 sum w_k 2^(32 k), w_k < 2^40 — sums and differences of
//                 normal values without carry handling; norm() brings them
//                 back (one carry pass + the 2^256 = 2^32 + 977 fold).
// Subtraction adds a multiple of p whose redundant limbs are all >= 2^32
// (M4 = 4p below), so every lane stays non-negative.
//
// Every step is exact for all inputs: the rare carry out of limb 7 after a
// fold is taken by a wave-uniform branch.  gfx950 only (DPP row controls).
#pragma once
#include "field.h"

#if defined(__HIPCC__)
namespace coop {

__device__ __forceinline__ uint32_t pos() { return __lane_id() & 15u; }
__device__ __forceinline__ uint32_t row() { return __lane_id() >> 4; }
// per-lane masks and multipliers (lane-constant, so the compiler keeps
// them in registers instead of branching on the lane index)
__device__ __forceinline__ uint32_t lo8() { return pos() < 8 ? 0xFFFFFFFFu : 0u; }  // limb lanes
__device__ __forceinline__ uint32_t f977() { return pos() == 0 ? 977u : (pos() == 1 ? 1u : 0u); }

// DPP (gfx9 encoding): row_shl:n 0x100+n (lane k reads lane k+n of its row),
// row_shr:n 0x110+n (lane k reads lane k-n), row_newbcast:n 0x150+n (every
// lane reads lane n of its row); lanes without a source read 0 (bound_ctrl)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}

// v + (carry into this lane), carries generated where `gen` and rippling
// through lanes holding 0xFFFFFFFF.  A row's top lane never generates here
// (every caller keeps its values below the row's width), so rows stay
// independent.
__device__ __forceinline__ uint32_t resolve(uint32_t v, bool gen) {
  const uint64_t G = __ballot(gen), P = __ballot(v == 0xFFFFFFFFu);
  const uint64_t C = ((G << 1) + P) ^ P;
  return v + (uint32_t)((C >> __lane_id()) & 1u);
}

// lanes 0..8 hold w_k < 2^32 + 2^20 (lanes 9..15: 0), the value
// sum w_k 2^(32 k): fold w_8 (2^256 = 2^32 + 977) into lanes 0 and 1
// unresolved, then resolve the carries ONCE.  The lanes 0..7 part is below
// 2^256 + 2^245 and w_8 (2^32 + 977) below 2^53, so the resolved lane 8 is 0
// or 1, and when it is 1 the rest is below 2^245: the rare second fold
// cannot carry out of limb 7.  Whether lane 8 ends nonzero is read off the
// scalar carry word (its input digit, or a carry into it), so the branch
// needs no vector compare after the resolve.  N values at once (N = 1, 2):
// their steps interleave in one basic block, one branch for all.
constexpr uint64_t kLane8 = 0x0100010001000100ull;  // lane 8 of each row
template <int N>
__device__ __forceinline__ void tail_n(const uint64_t (&w)[N], uint32_t (&d)[N]) {
  const uint32_t m = lo8(), f = f977();
  uint64_t y[N], C[N], rare = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint64_t w8 = ((uint64_t)dpp<0x158>((uint32_t)(w[i] >> 32)) << 32) | dpp<0x158>((uint32_t)w[i]);
    const uint64_t z = (pos() < 8 ? w[i] : 0ull) + w8 * f;  // lane 0: + 977 w_8, lane 1: + w_8 (< 2^43)
    y[i] = (uint64_t)(uint32_t)z + dpp<0x111>((uint32_t)(z >> 32));  // < 2^33; lane 8: <= 1
  }
#pragma unroll
  for (int i = 0; i < N; i++) {  // resolve(), with lane 8's outcome kept in `rare`
    const uint64_t G = __ballot((y[i] >> 32) != 0), P = __ballot((uint32_t)y[i] == 0xFFFFFFFFu);
    C[i] = ((G << 1) + P) ^ P;
    rare |= (__ballot((uint32_t)y[i] != 0) | C[i]) & kLane8;
  }
  // v + (bit `lane` of C): ONE v_addc with the scalar carry word as its
  // carry-in mask (instead of a 64-bit shift, an and and an add)
#pragma unroll
  for (int i = 0; i < N; i++) {
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(d[i]), "=s"(co) : "v"((uint32_t)y[i]), "s"(C[i]));
  }
  if (rare) {  // rare (a value within ~2^235 of 2^256), wave-uniform
#pragma unroll
    for (int i = 0; i < N; i++) {  // (a no-op for a value whose lane 8 is 0)
      const uint32_t o = dpp<0x158>(d[i]);
      const uint64_t z2 = (uint64_t)(d[i] & m) + (uint64_t)o * f;
      const uint64_t y2 = (uint64_t)(uint32_t)z2 + dpp<0x111>((uint32_t)(z2 >> 32));
      d[i] = resolve((uint32_t)y2, (y2 >> 32) != 0);  // the rest is < 2^245: no carry out
    }
  }
  // (lane 8 is 0 here: without the rare fold y_8 = 0 and no carry reached
  // it; after it, the rest had no carry out; lanes 9..15 stayed 0)
}
__device__ __forceinline__ uint32_t tail(uint64_t w) {
  const uint64_t in[1] = {w};
  uint32_t out[1];
  tail_n<1>(in, out);
  return out[0];
}

// WIDE -> NORMAL: one carry-save step (lane 9 stays 0: a WIDE lane 8 is
// small), then tail()
__device__ __forceinline__ uint64_t carry_save(uint64_t w) {
  return (uint64_t)(uint32_t)w + dpp<0x111>((uint32_t)(w >> 32));  // < 2^32 + 2^8
}
__device__ __forceinline__ uint32_t norm(uint64_t w) { return tail(carry_save(w)); }
// two independent WIDE values side by side
__device__ __forceinline__ void norm2(uint32_t &a, uint64_t wa, uint32_t &b, uint64_t wb) {
  const uint64_t in[2] = {carry_save(wa), carry_save(wb)};
  uint32_t out[2];
  tail_n<2>(in, out);
  a = out[0];
  b = out[1];
}

// a b mod p; a, b NORMAL (row-local), result NORMAL
__device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b) {
  const uint32_t k = pos();
  uint64_t acc = 0;
  uint32_t cnt = 0, bs = b;
  // lane k accumulates column k = sum_s a_s b_(k-s) (b shifts up one lane a step)
  // acc += as bs, cnt += the carry out: one v_mad_u64_u32 (its carry-out
  // SGPR pair) and one v_addc (gfx950 wants 2 wait states between the VALU
  // write of an SGPR and a VALU carry-in read of it: the s_nop)
#define COOP_STEP(s)                                                                            \
  {                                                                                             \
    const uint32_t as = dpp<0x150 + (s)>(a);                                                    \
    if (s) bs = dpp<0x111>(bs);                                                                 \
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc" \
                 : "+v"(acc), "+v"(cnt)                                                         \
                 : "v"(as), "v"(bs)                                                             \
                 : "vcc");                                                                      \
  }
  COOP_STEP(0) COOP_STEP(1) COOP_STEP(2) COOP_STEP(3) COOP_STEP(4) COOP_STEP(5) COOP_STEP(6) COOP_STEP(7)
#undef COOP_STEP
  // column k = lo_k + 2^32 hi_k + 2^64 cnt_k (columns 14, 15 carry nothing
  // out of the row) -> u_k < 2^34 with sum u_k 2^(32 k) = a b, then the
  // product's digit E_k = (u_k mod 2^32) + (u_(k-1) div 2^32) < 2^32 + 3
  // (E_15 < 2^32, as a b < 2^512) — left unresolved
  const uint32_t lo = (uint32_t)acc, hi = (uint32_t)(acc >> 32);
  const uint64_t u = (uint64_t)lo + dpp<0x111>(hi) + dpp<0x112>(cnt);
  const uint64_t v = (uint64_t)(uint32_t)u + dpp<0x111>((uint32_t)(u >> 32));
  const uint32_t vl = (uint32_t)v, vh = (uint32_t)(v >> 32);  // vh <= 1
  // 2^256 = 2^32 + 977: lane k < 8 gets E_k + 977 E_(k+8) + [k >= 1] E_(k+7),
  // lane 8 gets E_15 (row_shl:8 / :7 read zeros past the row's end); < 2^42
  const uint64_t e8 = ((uint64_t)dpp<0x108>(vh) << 32) | dpp<0x108>(vl);
  const uint32_t m7 = (k == 0 || k > 8) ? 0u : 0xFFFFFFFFu;
  const uint64_t e7 = ((uint64_t)(dpp<0x107>(vh) & m7) << 32) | (dpp<0x107>(vl) & m7);
  const uint64_t t = (k < 8 ? v : 0ull) + e8 * 977u + e7;
  // one carry-save step: lanes 0..8, each < 2^32 + 2^10 (lane 9: E_15 div 2^32 = 0)
  return tail((uint64_t)(uint32_t)t + dpp<0x111>((uint32_t)(t >> 32)));
}

// 4p in redundant limbs all >= 2^32 (lane k's limb; lane 8: 2): a + M4 - b
// keeps every lane non-negative for NORMAL b.  sum M4_k 2^(32 k) = 4p.
__device__ __forceinline__ uint64_t m4() {
  const uint32_t k = pos();
  const uint32_t lo = k == 0 ? 0xFFFFF0BCu : k == 1 ? 0xFFFFFFFAu : k < 8 ? 0xFFFFFFFEu : (k == 8 ? 2u : 0u);
  return ((uint64_t)(k < 8 ? 1u : 0u) << 32) | lo;
}
// WIDE multiples: a + (M4 - b) for NORMAL b
__device__ __forceinline__ uint64_t negw(uint32_t b) { return m4() - b; }

// the value of row `r` in every row (one ds_bpermute)
__device__ __forceinline__ uint32_t from_row(uint32_t x, uint32_t r) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((r << 4) | pos()) << 2), (int)x);
}

// Jacobian doubling dbl-2009-l (a = 0; the same formulas, hence the same
// representative, as point.h gej_double) with the state (X, Y, Z, NORMAL)
// replicated in every row: its seven products form three levels,
// {X^2, Y^2, Y Z} -> {B^2, E^2, (X + B)^2} -> E (D - X3), and the products of
// a level run in rows 0..2 at once.  The input is not the identity.
__device__ __forceinline__ void dbl(uint32_t &X, uint32_t &Y, uint32_t &Z) {
  const uint32_t r = row();
  // level 1: A = X^2 (row 0), B = Y^2 (row 1), YZ (row 2)
  uint32_t m = mul(r == 0 || r == 3 ? X : Y, r == 1 ? Y : r == 2 ? Z : X);
  const uint32_t A = from_row(m, 0), B = from_row(m, 1), YZ = from_row(m, 2);
  uint32_t E, XB;
  norm2(E, 3ull * A, XB, (uint64_t)X + B);
  // level 2: C = B^2 (row 0), F = E^2 (row 1), W = (X + B)^2 (row 2)
  const uint32_t s = r == 1 ? E : r == 2 ? XB : B;
  m = mul(s, s);
  const uint32_t C = from_row(m, 0), F = from_row(m, 1), W = from_row(m, 2);
  const uint32_t D = norm(2ull * ((uint64_t)W + negw(A) + negw(C)));  // 2 ((X + B)^2 - A - C)
  uint32_t t;  // X3 = F - 2 D, D - X3 = 3 D - F
  norm2(X, (uint64_t)F + 2ull * negw(D), t, 3ull * D + negw(F));
  // level 3: E (D - X3), every row
  m = mul(E, t);
  norm2(Y, (uint64_t)m + 8ull * negw(C), Z, 2ull * YZ);  // E (D - X3) - 8 C, 2 Y Z
}

// a NORMAL value (replicated in every row) is 0 mod p: 0 or p itself
__device__ __forceinline__ bool is_zero(uint32_t a) {
  const uint32_t k = __lane_id();
  const uint64_t z = __ballot(k < 8 && a == 0u), pp = __ballot(k < 8 && a == (k == 0 ? 0xFFFFFC2Fu : k == 1 ? 0xFFFFFFFEu : 0xFFFFFFFFu));
  return (z & 0xFFu) == 0xFFu || (pp & 0xFFu) == 0xFFu;
}

// r += (x2, y2) affine (NORMAL), the same formulas and exceptional cases as
// point.h gej_add_ge (Z3 = Z1 H): its products form five levels
// {Z1^2} -> {x2 Z1Z1, Z1 Z1Z1} -> {y2 t, H^2} -> {H HH, X1 HH, Z1 H, R^2} ->
// {R (V - X3), Y1 HHH}, each level's products in rows 0..3 at once.  `inf`
// (wave-uniform) is r's identity flag.
__device__ __forceinline__ void madd(uint32_t &X, uint32_t &Y, uint32_t &Z, bool &inf, uint32_t x2, uint32_t y2) {
  if (inf) {
    X = x2;
    Y = y2;
    Z = pos() == 0 ? 1u : 0u;
    inf = false;
    return;
  }
  const uint32_t r = row();
  const uint32_t ZZ = mul(Z, Z);
  uint32_t m = mul(r == 1 ? Z : x2, ZZ);  // row 0: U2 = x2 Z1Z1, row 1: Z1 Z1Z1
  const uint32_t U2 = from_row(m, 0), t = from_row(m, 1);
  const uint32_t H = norm((uint64_t)U2 + negw(X));
  m = mul(r == 1 ? H : y2, r == 1 ? H : t);  // row 0: S2 = y2 Z1^3, row 1: HH = H^2
  const uint32_t S2 = from_row(m, 0), HH = from_row(m, 1);
  const uint32_t R = norm((uint64_t)S2 + negw(Y));
  if (is_zero(H)) {  // wave-uniform
    if (is_zero(R)) dbl(X, Y, Z);
    else inf = true;
    return;
  }
  // row 0: HHH = H HH, row 1: V = X1 HH, row 2: Z3 = Z1 H, row 3: R^2
  m = mul(r == 0 ? H : r == 1 ? X : r == 2 ? Z : R, r == 2 ? H : r == 3 ? R : HH);
  const uint32_t HHH = from_row(m, 0), V = from_row(m, 1), Z3 = from_row(m, 2), RR = from_row(m, 3);
  const uint32_t X3 = norm((uint64_t)RR + negw(HHH) + 2ull * negw(V));  // R^2 - HHH - 2V
  const uint32_t t2 = norm((uint64_t)V + negw(X3));                      // V - X3
  m = mul(r == 1 ? Y : R, r == 1 ? HHH : t2);  // row 0: R (V - X3), row 1: Y1 HHH
  const uint32_t a = from_row(m, 0), b = from_row(m, 1);
  Y = norm((uint64_t)a + negw(b));
  X = X3;
  Z = Z3;
}

// beta's limb for this lane (phi(x, y) = (beta x, y))
__device__ __forceinline__ uint32_t beta_limb() { return pos() < 8 ? FE_BETA[pos()] : 0u; }

// XYZZ doubling dbl-2008-s-1 (a = 0; x = X / ZZ, y = Y / ZZZ; the values
// of point.h gexz_double mod p), state replicated in every row; the nine
// products form three levels {Y^2, X^2} -> {Y V, X V, V ZZ, M^2} ->
// {M (S - X3), H Y, H ZZZ, beta X3} with V = U^2 = 4 Y^2 (U = 2Y),
// H = Y V (so W = U V = 2H), M = 3X^2; the fourth product of the last level
// is beta X3 of the result (phi's x for free).  Every reduction between two
// levels runs beside another (V | M, X3 | S - X3 = 3S - M^2, Y3 | ZZZ3):
// three norm() latencies on the chain.  The input is not the identity;
// Y == 0 cannot occur on secp256k1.
__device__ __forceinline__ void dbl_xyzz(uint32_t &X, uint32_t &Y, uint32_t &ZZ, uint32_t &ZZZ, uint32_t &BX) {
  const uint32_t r = row();
  uint32_t m = mul(r == 0 ? Y : X, r == 0 ? Y : X);  // row 0: Y^2, row 1: X^2
  const uint32_t YY = from_row(m, 0), XX = from_row(m, 1);
  uint32_t V, M;
  norm2(V, 4ull * YY, M, 3ull * XX);
  // row 0: H = Y V, row 1: S = X V, row 2: ZZ3 = V ZZ, row 3: M^2
  m = mul(r == 0 ? Y : r == 1 ? X : r == 2 ? ZZ : M, r == 3 ? M : V);
  const uint32_t H = from_row(m, 0), S = from_row(m, 1), ZZ3 = from_row(m, 2), MM = from_row(m, 3);
  uint32_t X3, t;  // M^2 - 2 S, S - X3 = 3 S - M^2
  norm2(X3, (uint64_t)MM + 2ull * negw(S), t, 3ull * S + negw(MM));
  // row 0: M (S - X3), row 1: H Y, row 2: H ZZZ, row 3: beta X3
  m = mul(r == 0 ? M : r == 3 ? X3 : H, r == 0 ? t : r == 1 ? Y : r == 2 ? ZZZ : beta_limb());
  const uint32_t Mt = from_row(m, 0), HY = from_row(m, 1), HZ = from_row(m, 2), B3 = from_row(m, 3);
  norm2(Y, (uint64_t)Mt + 2ull * negw(HY), ZZZ, 2ull * HZ);  // M (S - X3) - W Y, W ZZZ
  X = X3;
  ZZ = ZZ3;
  BX = B3;
}

// (X1, Y1, ZZ1, ZZZ1) += (X2, Y2, ZZ2, ZZZ2), both XYZZ (add-2008-s, the
// formulas of point.h gexz_add), the second operand finite; complete: the
// identity (`inf`, wave-uniform), P + P (doubling) and P + (-P).  Fourteen
// products in four levels {U1, U2, S1, S2} -> {P^2, R^2, ZZ1 ZZ2, ZZZ1 ZZZ2}
// -> {P PP, U1 PP, ZZ12 PP} -> {R (Q - X3), S1 PPP, ZZZ12 PPP}.
__device__ __forceinline__ void add_xyzz(uint32_t &X1, uint32_t &Y1, uint32_t &ZZ1, uint32_t &ZZZ1, bool &inf,
                                         uint32_t X2, uint32_t Y2, uint32_t ZZ2, uint32_t ZZZ2) {
  if (inf) {
    X1 = X2;
    Y1 = Y2;
    ZZ1 = ZZ2;
    ZZZ1 = ZZZ2;
    inf = false;
    return;
  }
  const uint32_t r = row();
  // row 0: U1 = X1 ZZ2, row 1: U2 = X2 ZZ1, row 2: S1 = Y1 ZZZ2, row 3: S2 = Y2 ZZZ1
  uint32_t m = mul(r == 0 ? X1 : r == 1 ? X2 : r == 2 ? Y1 : Y2, r == 0 ? ZZ2 : r == 1 ? ZZ1 : r == 2 ? ZZZ2 : ZZZ1);
  const uint32_t U1 = from_row(m, 0), U2 = from_row(m, 1), S1 = from_row(m, 2), S2 = from_row(m, 3);
  uint32_t P, R;
  norm2(P, (uint64_t)U2 + negw(U1), R, (uint64_t)S2 + negw(S1));
  if (is_zero(P)) {  // wave-uniform: the same x
    if (is_zero(R)) {
      uint32_t bx;
      dbl_xyzz(X1, Y1, ZZ1, ZZZ1, bx);
    } else {
      inf = true;
    }
    return;
  }
  // row 0: PP = P^2, row 1: R^2, row 2: ZZ1 ZZ2, row 3: ZZZ1 ZZZ2
  m = mul(r == 0 ? P : r == 1 ? R : r == 2 ? ZZ1 : ZZZ1, r == 0 ? P : r == 1 ? R : r == 2 ? ZZ2 : ZZZ2);
  const uint32_t PP = from_row(m, 0), RR = from_row(m, 1), Z12 = from_row(m, 2), ZZZ12 = from_row(m, 3);
  // row 0: PPP = P PP, row 1: Q = U1 PP, rows 2-3: ZZ3 = ZZ1 ZZ2 PP
  m = mul(r == 0 ? P : r == 1 ? U1 : Z12, PP);
  const uint32_t PPP = from_row(m, 0), Q = from_row(m, 1), ZZ3 = from_row(m, 2);
  uint32_t X3, t;  // R^2 - PPP - 2 Q, Q - X3 = 3 Q + PPP - R^2
  norm2(X3, (uint64_t)RR + negw(PPP) + 2ull * negw(Q), t, 3ull * Q + PPP + negw(RR));
  // row 0: R (Q - X3), row 1: S1 PPP, rows 2-3: ZZZ3 = ZZZ1 ZZZ2 PPP
  m = mul(r == 0 ? R : r == 1 ? S1 : ZZZ12, r == 0 ? t : PPP);
  const uint32_t Rt = from_row(m, 0), SP = from_row(m, 1), ZZZ3 = from_row(m, 2);
  Y1 = norm((uint64_t)Rt + negw(SP));
  X1 = X3;
  ZZ1 = ZZ3;
  ZZZ1 = ZZZ3;
}

// (X, Y, Z) = k P for an affine P (NORMAL, replicated) and a 128-bit k
// (4 limbs, wave-uniform): MSB-first over the non-adjacent form of k (~k/3
// additions; verify_core.h naf_mul, per lane), every step cooperative.
__device__ __forceinline__ void naf_mul(uint32_t &X, uint32_t &Y, uint32_t &Z, bool &inf, uint32_t px, uint32_t py,
                                        const uint32_t k[4]) {
  uint32_t pos_[5], neg_[5];
  ::naf_masks(k, pos_, neg_);
  const uint32_t ny = norm(negw(py));
  inf = true;
  X = Y = Z = 0;
  for (int bit = 129; bit >= 0; bit--) {
    if (!inf) dbl(X, Y, Z);
    const uint32_t p = (pos_[bit >> 5] >> (bit & 31)) & 1u, n = (neg_[bit >> 5] >> (bit & 31)) & 1u;
    if (p | n) madd(X, Y, Z, inf, px, n ? ny : py);
  }
}

}  // namespace coop
#endif
