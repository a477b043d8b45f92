// kernels.hip — gfx950 kernels of the batch verifier (per-unit work lives in
// verify_core.h; bv_api.cpp drives them).
//
// One batch (streams owned by the library, one set per device):
//   lane (the call's)            s^-1 stream                keys stream (high priority)
//   k_sha256 (hash.go:8)         k_key_decode (Unmarshal,
//        |                         public_key.go:14)  ---> k_table_bases  2^(L k) Q, serial
//        |                       k_sinv (batched s^-1)      k_table_fill   sub-tables
//        |<------ join ---------------'                     k_table_pair   chord sums
//   k_verify_g   u1, u2, GLV split; R_G = u1 G: 9 XYZZ adds from the    |
//                26-bit signed G table (10 windows)                      |
//        |<------ join ----------------------------------------------------'
//   k_verify_q   R = R_G + k1 Q + k2 phi(Q): 22 adds from the key's K12
//                (12-bit signed, GLV) tables; decision table; X == r ZZ;
//                status + __ballot accept bits
// Key cache (BV_F_KEY_CACHE): the validator's KC tables (22-bit signed
// windows, built once by k_table_pair_kc) replace the keys stream and
// k_verify_gq does g + q in one pass.  k_verify_generic covers keys with too
// few items for a table.  The G table (k_table_pair_g, 21.5 GB) is built once
// per process and device.  Host batches of <= 256 items take k_small (one
// workgroup per item, one launch).  bv_verify_events' bulk batches hash each
// body as it is serialised from wire fields (k_ev_body_hash: no body stored).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "evjson.h"
#include "hostscalar.h"

#include "verify_core.h"


#ifndef BV_SHA_WAVES
#define BV_SHA_WAVES 1
#endif
// one message per lane; messages longer than max_len are left to the host
// (their digests arrive by k_put_digests)
__global__ void __launch_bounds__(256, BV_SHA_WAVES) k_sha256(uint64_t n_msgs, const uint8_t *__restrict__ bytes,
                                                const uint64_t *__restrict__ off,
                                                uint32_t *__restrict__ digest_words, uint64_t max_len) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m < n_msgs && off[m + 1] - off[m] <= max_len) sha256_one(m, bytes, off, digest_words);
}

// digests computed elsewhere (the host, for long messages): message idx[i]
// gets the 8 words vals[8 i ..]
__global__ void __launch_bounds__(256) k_put_digests(uint64_t n, const uint64_t *__restrict__ idx,
                                                     const uint32_t *__restrict__ vals, uint32_t *__restrict__ dig) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < 8 * n) dig[8 * idx[t / 8] + t % 8] = vals[t];
}

// PeerSet.Hash (src/peers/peer_set.go:104-115): h = [] then, for each peer
// in order, h = SHA256(h || pubkey) (crypto.SimpleHashFromTwoHashes,
// src/crypto/hash.go:17-22).  An inherently serial chain: ONE lane walks it
// in one launch (instead of one host round trip per peer); `scratch` holds
// 32 + max key length + 64 bytes.
__global__ void __launch_bounds__(64) k_sha256_chain(uint32_t n, const uint8_t *__restrict__ bytes,
                                                     const uint64_t *__restrict__ off, uint8_t *__restrict__ scratch,
                                                     uint32_t *__restrict__ out_words) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t hlen = 0;  // 0 before the first peer ([]byte{}), then 32
  for (uint32_t i = 0; i < n; i++) {
    const uint64_t o = off[i], len = off[i + 1] - o;
    for (int k = 0; k < 8; k++) {  // previous digest, big-endian bytes
      const uint32_t be = bswap32(h[k]);
      for (int q = 0; q < 4; q++) scratch[4 * k + q] = (uint8_t)(be >> (8 * q));
    }
    for (uint64_t q = 0; q < len; q++) scratch[hlen + q] = bytes[o + q];
    for (int q = 0; q < 8; q++) scratch[hlen + len + q] = 0;  // the over-read pad
    sha256_msg(h, scratch, 0, hlen + len);
    hlen = 32;  // re-serialised at the top of the next iteration
  }
  for (int k = 0; k < 8; k++) out_words[k] = bswap32(h[k]);
}

// ---------------------------------------------------------------------------
// Events from wire fields (evjson.h): body lengths, bodies, level hashing
// ---------------------------------------------------------------------------
// Bodies serialised straight into SHA-256, one lane per event (batches
// without in-batch parents; those are hashed on the host, hostdag.cpp): no
// body, length or offset array in HBM.  Each lane keeps its chaining value
// and current block in a 25-word LDS row (odd stride: the 64 lanes' rows
// start in distinct banks); bytes are packed big-endian into a register and
// stored a word at a time; a full block is compressed by evh_block, one
// out-of-line copy of the rounds for every put() call site of the
// serialiser.
#define EVH_NT 256
#define EVH_ROW 25
__global__ void __launch_bounds__(EVH_NT) k_ev_body_hash(bv_event_batch b, uint64_t e0, uint64_t e1,
                                                         uint32_t *__restrict__ dig) {
  __shared__ uint32_t rows[EVH_NT * EVH_ROW];
  const uint64_t e = e0 + (uint64_t)blockIdx.x * EVH_NT + threadIdx.x;
  if (e >= e1) return;  // no barriers below
  EvjSha o = evj_sha_begin(rows + threadIdx.x * EVH_ROW);
  evj_emit(b, e, o);
  uint32_t be[8];
  evj_sha_finish(o, be);
  uint4 *dst = (uint4 *)(dig + 8 * e);
  dst[0] = make_uint4(be[0], be[1], be[2], be[3]);
  dst[1] = make_uint4(be[4], be[5], be[6], be[7]);
}

// keys.DecodeSignature + the range checks on the device, one lane per event
// (bv_event_batch sig_text): the same rules as bv_decode_signature
// (hostparse.cpp, Go 1.13 strings.Split + big.Int.SetString(., 36)): exactly
// one '|'; each part an optional '+' / '-', then base-36 digits only, at
// least one; classes NIL / NONPOS / GE_N / OK; r and s as 32 big-endian
// bytes (zero unless OK) and the pre byte.  Six digits at a time (36^6 <
// 2^32) are folded into a 288-bit value with one mad per limb.
namespace {
DEV uint32_t digit36(uint32_t c) {
  if (c - '0' < 10u) return c - '0';
  if (c - 'a' < 26u) return c - 'a' + 10;
  if (c - 'A' < 26u) return c - 'A' + 10;
  return 0xFFu;
}
DEV uint8_t sig_part36(const uint8_t *s, uint64_t len, uint8_t *out) {
  uint32_t v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  bool big = false;
  uint64_t i = 0;
  bool neg = false;
  if (len && (s[0] == '-' || s[0] == '+')) neg = s[0] == '-', i = 1;
  const uint64_t first = i;
  while (i < len) {
    uint32_t chunk = 0, scale = 1, k = 0;
    for (; k < 6 && i < len; k++, i++) {
      const uint32_t d = digit36(s[i]);
      if (d == 0xFFu) break;
      chunk = chunk * 36u + d;
      scale *= 36u;
    }
    if (k && !big) {
      uint64_t carry = chunk;
#pragma unroll
      for (int j = 0; j < 9; j++) {
        const uint64_t t = (uint64_t)v[j] * scale + carry;
        v[j] = (uint32_t)t;
        carry = t >> 32;
      }
      big = carry != 0;
    }
    if (k < 6 && i < len) break;  // not a digit
  }
  uint4 *o = (uint4 *)out;
  o[0] = o[1] = make_uint4(0, 0, 0, 0);
  if (len == 0 || i == first || i != len) return BV_SC_NIL;
  bool zero = !big;
#pragma unroll
  for (int j = 0; j < 9; j++) zero = zero && v[j] == 0;
  if (zero || neg) return BV_SC_NONPOS;
  if (big || v[8]) return BV_SC_GE_N;
  if (!u256_lt(v, SC_N)) return BV_SC_GE_N;
  const uint32_t w[8] = {__builtin_bswap32(v[7]), __builtin_bswap32(v[6]), __builtin_bswap32(v[5]),
                         __builtin_bswap32(v[4]), __builtin_bswap32(v[3]), __builtin_bswap32(v[2]),
                         __builtin_bswap32(v[1]), __builtin_bswap32(v[0])};
  o[0] = make_uint4(w[0], w[1], w[2], w[3]);
  o[1] = make_uint4(w[4], w[5], w[6], w[7]);
  return BV_SC_OK;
}
}  // namespace

__global__ void __launch_bounds__(256) k_sig_decode(uint64_t n, const uint64_t *__restrict__ off,
                                                     const uint8_t *__restrict__ text, uint8_t *__restrict__ r_be,
                                                     uint8_t *__restrict__ s_be, uint8_t *__restrict__ pre) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint8_t *s = text + off[e];
  const uint64_t len = off[e + 1] - off[e];
  uint64_t bar = len, parts = 1;
  for (uint64_t i = 0; i < len; i++)
    if (s[i] == '|') {
      if (parts == 1) bar = i;
      parts++;
    }
  uint8_t *r = r_be + 32 * e, *sv = s_be + 32 * e;
  if (parts != 2) {
    ((uint4 *)r)[0] = ((uint4 *)r)[1] = ((uint4 *)sv)[0] = ((uint4 *)sv)[1] = make_uint4(0, 0, 0, 0);
    pre[e] = BV_PRE_PARTS_BAD;
    return;
  }
  const uint8_t rc = sig_part36(s, bar, r), sc = sig_part36(s + bar + 1, len - bar - 1, sv);
  pre[e] = BV_PRE(rc, sc);
}

__global__ void __launch_bounds__(256) k_iota(uint64_t n, uint32_t *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (uint32_t)i;
}

__global__ void __launch_bounds__(64) k_key_decode(uint32_t n_keys, const uint8_t *__restrict__ kbytes,
                                                   const uint64_t *__restrict__ koff, uint8_t *__restrict__ kstatus,
                                                   uint32_t *__restrict__ kxy) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n_keys) key_decode_one(k, kbytes, koff, kstatus, kxy);
}

template <bool LAT>
__global__ void __launch_bounds__(64) k_table_bases(uint32_t n_bases, const uint32_t *__restrict__ bxy,
                                                    const uint8_t *__restrict__ bstatus,
                                                    uint32_t *__restrict__ bases_jac, int w, int nwin) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_bases) return;
  if (bstatus && bstatus[b] != KS_OK) return;
  table_bases_one<LAT>(b, bxy, bases_jac, w, nwin);
}

// The same chain, one wave per base, wave-cooperative (coop.h): 126
// doublings of 64 keys 0.46 -> 0.28 ms (profiles/r04_coop_chain.log).
__global__ void __launch_bounds__(64) k_table_bases_coop(uint32_t n_bases, const uint32_t *__restrict__ bxy,
                                                         const uint8_t *__restrict__ bstatus,
                                                         uint32_t *__restrict__ bases_jac, int w, int nwin) {
  const uint32_t b = blockIdx.x;
  if (b >= n_bases) return;
  if (bstatus && bstatus[b] != KS_OK) return;  // wave-uniform
  coop_bases_one(b, bxy, bases_jac, w, nwin);
}

// Montgomery batch inversion over a block of N threads, one non-zero value
// each: an in-place binary product tree in LDS (heap order; T holds 2N - 1
// elements, the leaves at N - 1 + t).  N - 1 products up, ONE field
// inversion at the root (thread 0), 2N - 2 products down (a child's inverse
// is its parent's inverse times its sibling): ~3 products per thread where a
// prefix / suffix scan of the block spends 16, in 2 log2(N) levels.
// v <- v^-1.
template <int N>
__device__ __forceinline__ void block_inverse(fe *T, fe &v, uint32_t t) {
  static_assert((N & (N - 1)) == 0, "power of two");
  T[N - 1 + t] = v;
  __syncthreads();
#pragma unroll 1
  for (uint32_t n = N / 2; n >= 1; n >>= 1) {  // nodes n-1 .. 2n-2 from their children
    if (t < n) {
      const uint32_t p = n - 1 + t;
      fe a = T[2 * p + 1], b = T[2 * p + 2], r;
      fe_mul(r, a, b);
      T[p] = r;
    }
    __syncthreads();
  }
  if (t == 0) {
    fe x, root = T[0];
    fe_inv_var(x, root);
    T[0] = x;
  }
  __syncthreads();
#pragma unroll 1
  for (uint32_t n = 1; n < N; n <<= 1) {  // the 2n nodes 2n-1 .. 4n-2
    const uint32_t c = 2 * n - 1 + t;
    fe r;
    if (t < 2 * n) {
      fe a = T[(c - 1) / 2], b = T[(c & 1u) ? c + 1 : c - 1];
      fe_mul(r, a, b);
    }
    __syncthreads();
    if (t < 2 * n) T[c] = r;
    __syncthreads();
  }
  v = T[N - 1 + t];
}

// blockDim = BLOCK, grid (NWIN * 2^W / BLOCK, n_bases).  Thread t of block c
// computes the entry f = BLOCK c + t of the key's flat (window, digit) list
// — window j = f / 2^W, digit d = f mod 2^W; a block spans part of one
// window or (BLOCK > 2^W: the K8 sub-tables) several — and the block
// normalises its entries to affine with one field inversion (prefix/suffix
// products in LDS).  PHI: also write the phi(T) half of a GLV key table.
template <int W, int NWIN, bool PHI, int BLOCK = 256, bool LAT = true>
__global__ void __launch_bounds__(BLOCK) k_table_fill(const uint32_t *__restrict__ bases_jac,
                                                      const uint8_t *__restrict__ bstatus,
                                                      uint32_t *__restrict__ table) {
  static_assert(((NWIN << W) % BLOCK) == 0, "blocks cover whole keys");
  constexpr uint64_t half_u32 = (uint64_t)NWIN * (1ull << W) * BV_ENTRY_U32;
  const uint32_t b = blockIdx.y;
  const uint32_t f = blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t j = f >> W;
  const uint32_t d = f & ((1u << W) - 1u);
  const uint32_t t = threadIdx.x;
  if (bstatus && bstatus[b] != KS_OK) return;  // uniform per block
  __shared__ fe sT[2 * BLOCK - 1];
  // The base B = (X, Y, Z) stays Jacobian: (X, Y) is an affine point of the
  // isomorphic curve y^2 = x^3 + 7 Z^6, and the a = 0 doubling / mixed-add
  // formulas never use b, so d (X, Y) computed there as (X', Y', Z') is
  // d B = (X', Y', Z' Z) on secp256k1.  No inversion before the entries.
  const uint32_t *bj = bases_jac + ((uint64_t)b * NWIN + j) * 24;
  fe bx, by, bz;
  fe_load(bx, bj);
  fe_load(by, bj + 8);
  fe_load(bz, bj + 16);
  gej R;
  bool inf;
  fe Z;
  table_point<LAT>(R, inf, Z, bx, by, d, W);
  if (!inf) fe_mul(Z, Z, bz);
  fe zi = Z;
  block_inverse<BLOCK>(sT, zi, t);  // Z_t^-1
  uint32_t *entry = table + (uint64_t)b * (PHI ? 2 : 1) * half_u32 + (((uint64_t)j << W) + d) * BV_ENTRY_U32;
  table_store(entry, PHI ? entry + half_u32 : nullptr, d, R, inf, zi);
}

// K12 key tables from the 6-bit sub-tables (verify_core.h: pair_*).
// One block of 256 threads per (window j, key): digit d = 256 e + t for
// e < E (E = 2^(W-1) / 256; signed digits, geometry.h), so a wave shares hi
// and reads 64 distinct lo; d = 0 stands for digit 2^(W-1), stored in slot 0
// of window j+1 (k12_digit).
// S_2j and S_2j+1 are staged in LDS; the window's chord denominators are
// inverted with ONE field inversion (per-thread running products whose
// prefixes go to `pscr`, then block prefix/suffix products in LDS), so the
// serial inversion latency is paid once per window and the whole grid is
// resident in one round.  The top window only needs digits
// <= 2^(128 - W j): its blocks stop after the live entries.
template <int W, int L, int NWIN>
__global__ void __launch_bounds__(256) k_table_pair(const uint32_t *__restrict__ sub,
                                                    const uint8_t *__restrict__ bstatus,
                                                    uint32_t *__restrict__ table, uint4 *__restrict__ pscr) {
  constexpr uint32_t ENT = 1u << (W - 1), E = ENT / 256u, NS = 1u << L;
  constexpr uint64_t half_u32 = ((uint64_t)NWIN * ENT + 1) * BV_ENTRY_U32;
  static_assert(half_u32 == BV_K12HALF_U32, "K12 geometry");
  const uint32_t b = blockIdx.y, j = blockIdx.x, t = threadIdx.x;
  if (bstatus && bstatus[b] != KS_OK) return;
  const int live_bits = 128 - W * (int)j;
  const uint32_t e_live = live_bits >= W - 1 ? E : ((1u << live_bits) + 1u + 255u) / 256u;
  __shared__ uint32_t sLo[NS * BV_ENTRY_U32], sHi[NS * BV_ENTRY_U32];
  __shared__ fe sT[511];
  const uint32_t *sk = sub + ((uint64_t)b * 2 * NWIN + 2 * j) * NS * BV_ENTRY_U32;
  for (uint32_t x = t; x < NS * BV_ENTRY_U32; x += 256) {
    sLo[x] = sk[x];
    sHi[x] = sk[NS * BV_ENTRY_U32 + x];
  }
  __syncthreads();
  uint4 *ps = pscr + ((uint64_t)b * NWIN + j) * E * 2 * 256 + t;
  fe acc;
  fe_set(acc, 1);
#pragma unroll 1
  for (uint32_t e = 0; e < e_live; e++) {
    const uint32_t d = k12_digit(256 * e + t, ENT), lo = d & (NS - 1), hi = d >> L;
    fe x1, y1, x2, y2, H;
    pair_load(sLo, sHi, lo, hi, x1, y1, x2, y2);
    pair_denominator(H, pair_kind(lo, hi), x1, x2);
    ps[(2 * e) * 256] = make_uint4(acc.v[0], acc.v[1], acc.v[2], acc.v[3]);
    ps[(2 * e + 1) * 256] = make_uint4(acc.v[4], acc.v[5], acc.v[6], acc.v[7]);
    fe_mul(acc, acc, H);
  }
  fe q = acc;
  block_inverse<256>(sT, q, t);  // (this thread's product)^-1
  uint32_t *base = table + (uint64_t)b * 2 * half_u32 + (uint64_t)j * ENT * BV_ENTRY_U32;
#pragma unroll 1
  for (int e = (int)e_live - 1; e >= 0; e--) {
    const uint32_t d = k12_digit(256 * e + t, ENT), lo = d & (NS - 1), hi = d >> L;
    const int kind = pair_kind(lo, hi);
    fe x1, y1, x2, y2, H, Hinv, pre;
    pair_load(sLo, sHi, lo, hi, x1, y1, x2, y2);
    pair_denominator(H, kind, x1, x2);
    const uint4 p0 = ps[(2 * e) * 256], p1 = ps[(2 * e + 1) * 256];
    pre.v[0] = p0.x; pre.v[1] = p0.y; pre.v[2] = p0.z; pre.v[3] = p0.w;
    pre.v[4] = p1.x; pre.v[5] = p1.y; pre.v[6] = p1.z; pre.v[7] = p1.w;
    fe_mul(Hinv, q, pre);
    fe_mul(q, q, H);
    uint32_t *entry = base + (uint64_t)d * BV_ENTRY_U32;
    pair_store(entry, entry + half_u32, kind, x1, y1, x2, y2, Hinv);
  }
}

// K8 key tables from the 4-bit sub-tables: one block of 256
// threads per WPB windows of a key; thread t builds digit d = t = lo + 16 hi
// of each of its windows j as the affine chord S_2j[lo] + S_2j+1[hi] (the
// two are never equal or opposite: lo < 16 <= 16 hi), and the block's chord
// denominators are inverted with ONE field inversion: per-thread running
// products (their prefixes in `pscr`, coalesced), then block_inverse.
// Replaces the per-entry double-and-add of k_table_fill<8, 16, true> (~12
// point operations and a 256-entry inversion share per entry) with one
// affine addition; digit 0 stays the (0, 0) identity.  WPB = 16 (one
// inversion per key) when many keys fill the chip, 1 when a few keys' latency
// is the point.  The block's sub-tables are staged in LDS.
template <int W, int L, int NWIN, int WPB>
__global__ void __launch_bounds__(256) k_table_pair_u(const uint32_t *__restrict__ sub,
                                                      const uint8_t *__restrict__ bstatus,
                                                      uint32_t *__restrict__ table, uint4 *__restrict__ pscr) {
  constexpr uint32_t NS = 1u << L, SUB_U32 = 2 * WPB * NS * BV_ENTRY_U32;
  constexpr uint64_t half_u32 = (uint64_t)NWIN * (1ull << W) * BV_ENTRY_U32;
  static_assert((1u << W) == 256 && W == 2 * L && half_u32 == BV_KHALF_U32 && NWIN % WPB == 0, "K8 geometry");
  const uint32_t b = blockIdx.y, j0 = blockIdx.x * WPB, t = threadIdx.x;
  if (bstatus && bstatus[b] != KS_OK) return;
  __shared__ uint32_t sS[SUB_U32];
  __shared__ fe sT[511];
  const uint32_t *sk = sub + ((uint64_t)b * 2 * NWIN + 2 * j0) * NS * BV_ENTRY_U32;
  for (uint32_t x = t; x < SUB_U32; x += 256) sS[x] = sk[x];
  __syncthreads();
  const uint32_t lo = t & (NS - 1), hi = t >> L;
  const int kind = pair_kind(lo, hi);
  uint4 *ps = pscr + ((uint64_t)b * NWIN + j0) * 2 * 256 + t;
  fe acc;
  fe_set(acc, 1);
#pragma unroll 1
  for (uint32_t e = 0; e < WPB; e++) {
    fe x1, y1, x2, y2, H;
    pair_load(sS + 2 * e * NS * BV_ENTRY_U32, sS + (2 * e + 1) * NS * BV_ENTRY_U32, lo, hi, x1, y1, x2, y2);
    pair_denominator(H, kind, x1, x2);
    if (WPB > 1) {
      ps[(2 * e) * 256] = make_uint4(acc.v[0], acc.v[1], acc.v[2], acc.v[3]);
      ps[(2 * e + 1) * 256] = make_uint4(acc.v[4], acc.v[5], acc.v[6], acc.v[7]);
    }
    fe_mul(acc, acc, H);
  }
  fe q = acc;
  block_inverse<256>(sT, q, t);  // (this thread's product)^-1
  uint32_t *base = table + (uint64_t)b * 2 * half_u32 + (((uint64_t)j0 << W) + t) * BV_ENTRY_U32;
#pragma unroll 1
  for (int e = WPB - 1; e >= 0; e--) {
    fe x1, y1, x2, y2, H, Hinv;
    pair_load(sS + 2 * e * NS * BV_ENTRY_U32, sS + (2 * e + 1) * NS * BV_ENTRY_U32, lo, hi, x1, y1, x2, y2);
    if (WPB > 1) {
      fe pre;
      pair_denominator(H, kind, x1, x2);
      const uint4 p0 = ps[(2 * e) * 256], p1 = ps[(2 * e + 1) * 256];
      pre.v[0] = p0.x; pre.v[1] = p0.y; pre.v[2] = p0.z; pre.v[3] = p0.w;
      pre.v[4] = p1.x; pre.v[5] = p1.y; pre.v[6] = p1.z; pre.v[7] = p1.w;
      fe_mul(Hinv, q, pre);
      fe_mul(q, q, H);
    } else {
      Hinv = q;
    }
    uint32_t *entry = base + ((uint64_t)e << W) * BV_ENTRY_U32;
    pair_store(entry, entry + half_u32, kind, x1, y1, x2, y2, Hinv);
  }
}

// Generator table window j from the G sub-tables (geometry.h, signed
// digits): block c holds slots s = 4096 c + 256 e + t (e < 16) of window j,
// digit k12_digit(s) (slot 0 builds digit 2^(W-1), which lands in window
// j+1's slot 0), so a wave reads 64 consecutive S_lo points and one S_hi point
// (the sub-tables, 5 MiB, stay in L2/MALL; no LDS staging).  One field
// inversion per block; prefix products in `pscr` (4096 fe per block).
// Launched once per window chunk.
template <int W, int L>
__global__ void __launch_bounds__(256) k_table_pair_g(const uint32_t *__restrict__ sub, uint32_t *__restrict__ table,
                                                      uint4 *__restrict__ pscr, uint32_t j, uint32_t c0) {
  constexpr uint32_t E = 16, NS = 1u << L, ENT = 1u << (W - 1);
  const uint32_t c = c0 + blockIdx.x, t = threadIdx.x;
  const uint32_t *s_lo = sub + (uint64_t)(2 * j) * NS * BV_ENTRY_U32;
  const uint32_t *s_hi = s_lo + (uint64_t)NS * BV_ENTRY_U32;
  __shared__ fe sT[511];
  uint4 *ps = pscr + (uint64_t)blockIdx.x * E * 2 * 256 + t;
  fe acc;
  fe_set(acc, 1);
#pragma unroll 1
  for (uint32_t e = 0; e < E; e++) {
    const uint32_t d = k12_digit(4096u * c + 256u * e + t, ENT), lo = d & (NS - 1), hi = d >> L;
    fe x1, y1, x2, y2, H;
    pair_load(s_lo, s_hi, lo, hi, x1, y1, x2, y2);
    pair_denominator(H, pair_kind(lo, hi), x1, x2);
    ps[(2 * e) * 256] = make_uint4(acc.v[0], acc.v[1], acc.v[2], acc.v[3]);
    ps[(2 * e + 1) * 256] = make_uint4(acc.v[4], acc.v[5], acc.v[6], acc.v[7]);
    fe_mul(acc, acc, H);
  }
  fe q = acc;
  block_inverse<256>(sT, q, t);  // (this thread's product)^-1
  uint32_t *base = table + (uint64_t)j * ENT * BV_ENTRY_U32;
#pragma unroll 1
  for (int e = (int)E - 1; e >= 0; e--) {
    const uint32_t d = k12_digit(4096u * c + 256u * e + t, ENT), lo = d & (NS - 1), hi = d >> L;
    const int kind = pair_kind(lo, hi);
    fe x1, y1, x2, y2, H, Hinv, pre;
    pair_load(s_lo, s_hi, lo, hi, x1, y1, x2, y2);
    pair_denominator(H, kind, x1, x2);
    const uint4 p0 = ps[(2 * e) * 256], p1 = ps[(2 * e + 1) * 256];
    pre.v[0] = p0.x; pre.v[1] = p0.y; pre.v[2] = p0.z; pre.v[3] = p0.w;
    pre.v[4] = p1.x; pre.v[5] = p1.y; pre.v[6] = p1.z; pre.v[7] = p1.w;
    fe_mul(Hinv, q, pre);
    fe_mul(q, q, H);
    pair_store(base + (uint64_t)d * BV_ENTRY_U32, nullptr, kind, x1, y1, x2, y2, Hinv);
  }
}

__global__ void __launch_bounds__(256) k_sinv(uint64_t n_items, uint32_t M, const uint32_t *__restrict__ s_be,
                                              const uint8_t *__restrict__ pre, uint32_t *__restrict__ w_out) {
  const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  sinv_thread(t, T, n_items, M, s_be, pre, w_out);
}

// Items [lo, hi) of a launch, lo a multiple of 64: each wave owns whole
// 64-bit words of the accept bitmask (hi is a multiple of 64 or the end).
__device__ __forceinline__ void write_status(uint64_t i, uint64_t hi, uint8_t st, uint8_t *status, uint64_t *bits) {
  if (i < hi) status[i] = st;
  const uint64_t mask = __ballot(i < hi && st == BV_ACCEPT);
  if ((threadIdx.x & 63) == 0 && i < hi) bits[i >> 6] = mask;
}

#ifndef BV_GWAVES
#define BV_GWAVES 1
#endif
#ifndef BV_LWAVES  // latency variants (zipped point ops, small batches)
#define BV_LWAVES 1
#endif
__global__ void __launch_bounds__(256) k_glv_split(uint64_t n_items, const uint32_t *__restrict__ r_be,
                                                   const uint32_t *__restrict__ w_in, uint32_t *__restrict__ u12) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_items) glv_split_item(i, r_be, w_in, u12);
}

template <bool LAT, bool SPLIT>
__global__ void __launch_bounds__(256, LAT ? BV_LWAVES : BV_GWAVES) k_verify_g(uint64_t n_items, uint64_t lo, uint64_t hi,
                                                  const uint32_t *__restrict__ item_key,
                                                  const uint32_t *__restrict__ r_be, const uint32_t *__restrict__ s_be,
                                                  const uint8_t *__restrict__ pre, const uint8_t *__restrict__ kstatus,
                                                  const uint32_t *__restrict__ item_msg,
                                                  const uint32_t *__restrict__ digest_words,
                                                  const uint32_t *__restrict__ w_in, uint32_t *__restrict__ u12,
                                                  const uint32_t *__restrict__ g_table, uint32_t *__restrict__ rg) {
  const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < hi)
    verify_item_g<LAT, SPLIT>(i, n_items, item_key, r_be, s_be, pre, kstatus, item_msg, digest_words, w_in, u12,
                              g_table, rg);
}

// Throughput variants: BV_QWAVES waves per SIMD (4: 128 VGPRs, the XYZZ
// accumulator fits; at 3 waves the bulk launch loses a quarter of its
// latency hiding).
#ifndef BV_QWAVES
#define BV_QWAVES 4
#endif
template <int W, int NWIN, bool LAT>
__global__ void __launch_bounds__(256, LAT ? BV_LWAVES : BV_QWAVES) k_verify_q(uint64_t n_items, uint64_t lo, uint64_t hi,
                                                  const uint32_t *__restrict__ item_key,
                                                  const uint32_t *__restrict__ r_be, const uint32_t *__restrict__ s_be,
                                                  const uint8_t *__restrict__ pre, const uint8_t *__restrict__ kstatus,
                                                  const uint32_t *__restrict__ u12,
                                                  const uint32_t *__restrict__ key_table,
                                                  const uint64_t *__restrict__ key_tabs,
                                                  const uint32_t *__restrict__ rg, uint8_t *__restrict__ status,
                                                  uint64_t *__restrict__ bits) {
  const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t st = BV_REJECT;
  if (i < hi)
    st = verify_item_q<W, NWIN, LAT>(i, n_items, item_key, r_be, s_be, pre, kstatus, u12, key_table, key_tabs, rg);
  write_status(i, hi, st, status, bits);
}

// Key part first (verify_core.h: verify_item_qfirst / verify_item_gfinish):
// host entries run k_verify_qf over the whole batch while its messages
// cross PCIe, then k_verify_gf per hashed chunk.
template <int W, int NWIN, bool LAT>
__global__ void __launch_bounds__(256, LAT ? BV_LWAVES : BV_QWAVES) k_verify_qf(uint64_t n_items, uint64_t lo, uint64_t hi,
                                                   const uint32_t *__restrict__ item_key,
                                                   const uint32_t *__restrict__ r_be, const uint32_t *__restrict__ s_be,
                                                   const uint8_t *__restrict__ pre, const uint8_t *__restrict__ kstatus,
                                                   const uint32_t *__restrict__ w_in,
                                                   const uint32_t *__restrict__ key_table,
                                                   const uint64_t *__restrict__ key_tabs, uint32_t *__restrict__ rq) {
  const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < hi)
    verify_item_qfirst<W, NWIN, LAT>(i, n_items, item_key, r_be, s_be, pre, kstatus, w_in, key_table, key_tabs, rq);
}

template <bool LAT>
__global__ void __launch_bounds__(256, LAT ? BV_LWAVES : BV_QWAVES) k_verify_gf(uint64_t n_items, uint64_t lo, uint64_t hi,
                                                   const uint32_t *__restrict__ item_key,
                                                   const uint32_t *__restrict__ r_be, const uint32_t *__restrict__ s_be,
                                                   const uint8_t *__restrict__ pre, const uint8_t *__restrict__ kstatus,
                                                   const uint32_t *__restrict__ item_msg,
                                                   const uint32_t *__restrict__ digest_words,
                                                   const uint32_t *__restrict__ w_in,
                                                   const uint32_t *__restrict__ g_table,
                                                   const uint32_t *__restrict__ rq, uint8_t *__restrict__ status,
                                                   uint64_t *__restrict__ bits) {
  const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t st = BV_REJECT;
  if (i < hi)
    st = verify_item_gfinish<LAT>(i, n_items, item_key, r_be, s_be, pre, kstatus, item_msg, digest_words, w_in, g_table,
                                  rq);
  write_status(i, hi, st, status, bits);
}

// Key-cache path, G and Q parts fused (verify_core.h: verify_item_gq_kc).
#ifndef BV_GQWAVES
#define BV_GQWAVES BV_QWAVES
#endif
template <bool LAT>
__global__ void __launch_bounds__(256, LAT ? BV_LWAVES : BV_GQWAVES) k_verify_gq(uint64_t n_items, uint64_t lo, uint64_t hi,
                                                   const uint32_t *__restrict__ item_key,
                                                   const uint32_t *__restrict__ r_be, const uint32_t *__restrict__ s_be,
                                                   const uint8_t *__restrict__ pre, const uint8_t *__restrict__ kstatus,
                                                   const uint32_t *__restrict__ item_msg,
                                                   const uint32_t *__restrict__ digest_words,
                                                   const uint32_t *__restrict__ w_in,
                                                   const uint32_t *__restrict__ g_table,
                                                   const uint64_t *__restrict__ key_tabs, uint8_t *__restrict__ status,
                                                   uint64_t *__restrict__ bits) {
  const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t st = BV_REJECT;
  if (i < hi)
    st = verify_item_gq_kc<LAT>(i, item_key, r_be, s_be, pre, kstatus, item_msg, digest_words, w_in, g_table, key_tabs);
  write_status(i, hi, st, status, bits);
}

// Key-cache (KC) table windows from the 11-bit sub-tables: block (c, key)
// holds slots s = BV_KCPAIR_ENT c' + 256 e + t (e < 16) of window
// j = c / (ENT / BV_KCPAIR_ENT), c' = c mod that; digit k12_digit(s) (signed
// windows: slot 0 builds digit ENT, stored in window j+1's slot 0).  A wave
// reads 64 consecutive S_lo points and one S_hi point from L2 (the key's
// sub-tables are 1.5 MB).  One field inversion per block (Montgomery's trick
// over 4096 chord denominators, prefix products in `pscr`), then each entry
// is stored (no phi half: k_verify_q forms phi(T) = (beta x, y)).  Blocks
// beyond the top window's live digits (<= 2^(128 - W j) + 1) return at once.
// `tabs[b]` is key b's table.
template <int W, int L, int NWIN>
__global__ void __launch_bounds__(256) k_table_pair_kc(const uint32_t *__restrict__ sub,
                                                       const uint8_t *__restrict__ bstatus,
                                                       const uint64_t *__restrict__ tabs, uint4 *__restrict__ pscr) {
  constexpr uint32_t ENT = 1u << (W - 1), NS = 1u << L, E = BV_KCPAIR_ENT / 256u, CH = ENT / BV_KCPAIR_ENT;
  const uint32_t b = blockIdx.y, j = blockIdx.x / CH, c = blockIdx.x % CH, t = threadIdx.x;
  if (bstatus && bstatus[b] != KS_OK) return;
  const int live_bits = 128 - W * (int)j;
  if (live_bits < W - 1 && (uint64_t)BV_KCPAIR_ENT * c > (1ull << live_bits) + 1) return;  // uniform per block
  const uint32_t *s_lo = sub + ((uint64_t)b * 2 * NWIN + 2 * j) * NS * BV_ENTRY_U32;
  const uint32_t *s_hi = s_lo + (uint64_t)NS * BV_ENTRY_U32;
  __shared__ fe sT[511];
  uint4 *ps = pscr + ((uint64_t)b * gridDim.x + blockIdx.x) * E * 2 * 256 + t;
  fe acc;
  fe_set(acc, 1);
#pragma unroll 1
  for (uint32_t e = 0; e < E; e++) {
    const uint32_t d = k12_digit(BV_KCPAIR_ENT * c + 256u * e + t, ENT), lo = d & (NS - 1), hi = d >> L;
    fe x1, y1, x2, y2, H;
    pair_load(s_lo, s_hi, lo, hi, x1, y1, x2, y2);
    pair_denominator(H, pair_kind(lo, hi), x1, x2);
    ps[(2 * e) * 256] = make_uint4(acc.v[0], acc.v[1], acc.v[2], acc.v[3]);
    ps[(2 * e + 1) * 256] = make_uint4(acc.v[4], acc.v[5], acc.v[6], acc.v[7]);
    fe_mul(acc, acc, H);
  }
  fe q = acc;
  block_inverse<256>(sT, q, t);  // (this thread's product)^-1
  uint32_t *base = (uint32_t *)tabs[b] + (uint64_t)j * ENT * BV_ENTRY_U32;
#pragma unroll 1
  for (int e = (int)E - 1; e >= 0; e--) {
    const uint32_t d = k12_digit(BV_KCPAIR_ENT * c + 256u * e + t, ENT), lo = d & (NS - 1), hi = d >> L;
    const int kind = pair_kind(lo, hi);
    fe x1, y1, x2, y2, H, Hinv, pre;
    pair_load(s_lo, s_hi, lo, hi, x1, y1, x2, y2);
    pair_denominator(H, kind, x1, x2);
    const uint4 p0 = ps[(2 * e) * 256], p1 = ps[(2 * e + 1) * 256];
    pre.v[0] = p0.x; pre.v[1] = p0.y; pre.v[2] = p0.z; pre.v[3] = p0.w;
    pre.v[4] = p1.x; pre.v[5] = p1.y; pre.v[6] = p1.z; pre.v[7] = p1.w;
    fe_mul(Hinv, q, pre);
    fe_mul(q, q, H);
    pair_store(base + (uint64_t)d * BV_ENTRY_U32, nullptr, kind, x1, y1, x2, y2, Hinv);  // no phi half (geometry.h)
  }
}

template <bool LAT>
__global__ void __launch_bounds__(256) k_verify_generic(uint64_t n_items, uint64_t lo, uint64_t hi,
                                                        const uint32_t *__restrict__ item_key,
                                                        const uint32_t *__restrict__ r_be,
                                                        const uint32_t *__restrict__ s_be,
                                                        const uint8_t *__restrict__ pre,
                                                        const uint8_t *__restrict__ kstatus,
                                                        const uint32_t *__restrict__ kxy,
                                                        const uint32_t *__restrict__ item_msg,
                                                        const uint32_t *__restrict__ digest_words,
                                                        const uint32_t *__restrict__ w_in,
                                                        const uint32_t *__restrict__ g_table,
                                                        uint8_t *__restrict__ status, uint64_t *__restrict__ bits) {
  const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t st = BV_REJECT;
  if (i < hi)
    st = verify_item_generic<LAT>(i, item_key, r_be, s_be, pre, kstatus, kxy, item_msg, digest_words, w_in, g_table);
  write_status(i, hi, st, status, bits);
}

// Key cache, partial batch (verify_core.h BV_DEFERRED): the deferred items'
// indices, appended in any order (`list[n]` counts them), then the generic
// per-lane path over that list, grid-stride (they are few: keys without a
// table yet).  A deferred item's accept bit is OR-ed into its word, whose
// other bits the KC kernel already wrote.
__global__ void __launch_bounds__(256) k_defer_list(uint64_t n, const uint8_t *__restrict__ status,
                                                    uint32_t *__restrict__ list) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && status[i] == BV_DEFERRED) list[atomicAdd(list + n, 1u)] = (uint32_t)i;
}
__global__ void __launch_bounds__(64) k_verify_deferred(uint64_t n, const uint32_t *__restrict__ list,
                                                        const uint32_t *__restrict__ item_key,
                                                        const uint32_t *__restrict__ r_be,
                                                        const uint32_t *__restrict__ s_be,
                                                        const uint8_t *__restrict__ pre,
                                                        const uint8_t *__restrict__ kstatus,
                                                        const uint32_t *__restrict__ kxy,
                                                        const uint32_t *__restrict__ item_msg,
                                                        const uint32_t *__restrict__ digest_words,
                                                        const uint32_t *__restrict__ w_in,
                                                        const uint32_t *__restrict__ g_table,
                                                        uint8_t *__restrict__ status, uint64_t *__restrict__ bits) {
  const uint32_t cnt = list[n];
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < cnt; t += gridDim.x * blockDim.x) {
    const uint64_t i = list[t];
    const uint8_t st =
        verify_item_generic<true>(i, item_key, r_be, s_be, pre, kstatus, kxy, item_msg, digest_words, w_in, g_table);
    status[i] = st;
    if (st == BV_ACCEPT) atomicOr((unsigned long long *)bits + (i >> 6), 1ull << (i & 63));
  }
}

// ---------------------------------------------------------------------------
// Small batches: k_small, ONE launch per batch, one 256-thread workgroup per
// item.  A small batch is bound by its longest serial chain, not by
// throughput, so one item's work is spread over the workgroup (lanes of
// different waves run different code at the same time; lanes of one wave
// only when they run the same code).  The host has hashed the messages
// (SHA-NI, hostsha.cpp) and sends the digests.
//   phase 1  waves 1 + 3: s^-1 (one Bernstein-Yang inversion split over two
//            waves, lane 0 each: wave-uniform, so it runs on the scalar unit)
//            wave 2: elliptic.Unmarshal of the item's key (Q); without a
//            key-cache table it then doubles Q (kColdD0 doublings)
//            wave 0: the item's r, digest, pre and table address
//            (latency batches, <= BV_HOST_SCALARS items: `rec` holds one
//            256-byte host record per item — key bytes, r, s, pre, table
//            address and u1, k1, k2 computed on the host, hostscalar.h —
//            read by ONE wave-wide load; no inversion, wave 2 decodes Q)
//   phase 2  wave 0 lane 0: decision table, u1 = e w;  wave 1 lane 0:
//            u2 = r w, its GLV split (k1, k2, signs) and, without a table,
//            the chain length and the phase count; wave 2: kColdD1 doublings
//   phase 3  key with a key-cache table: 22 leaves in lanes 0..21 of wave
//            0, every table entry loaded at once — G windows 0..9 of u1,
//            KC windows 0..5 of k1 (T) and of k2 (phi(T)) — summed by a
//            binary tree (affine pairs, then XYZZ sums: 5 levels of zipped
//            point additions, nodes handed over through LDS);
//            key without one: right to left in barrier-separated phases
//            (see SmallCold above): wave 2 doubles kColdChunk more entries
//            per phase, waves 1 / 3 add the entries of earlier phases for
//            k1 Q / k2 phi(Q); wave 3 first adds the G sum (wave 0 sums
//            the G leaves in phase 2); then wave 1 adds wave 3's sum
//   phase 4  x(R) mod N == r (wave 0 lane 0 with a table, wave 1 lane 0
//            without)
// Statuses only; the host packs a small batch's accept bits.  `stamps`
// (BV_SMALL_STAMPS diagnostics): workgroup 0's shader clocks per phase.
// ---------------------------------------------------------------------------
namespace {
constexpr int kSmallLeaves = BV_GNWIN + 2 * BV_KCNWIN;  // 22
struct SmallNode {
  uint32_t w[33];
};
// one level of the wave-0 sum tree: node i <- node 2i + node 2i+1 (the last
// node of an odd count moves up alone); nodes in `from`, results in `to`
DEV void small_tree_level(const SmallNode *from, SmallNode *to, int n, uint32_t lane) {
  if (lane < (uint32_t)(n + 1) / 2) {
    gexz A, B;
    bool ia, ib = true;
    part_load(from[2 * lane].w, A, ia);
    if (2 * (int)lane + 1 < n) part_load(from[2 * lane + 1].w, B, ib);
    gexz_add_lat(A, ia, B, ib);
    part_store(to[lane].w, A, ia);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // this wave's LDS writes land before the next level reads
  __builtin_amdgcn_wave_barrier();
}
// the leaves' first level: affine pairs (2i, 2i+1) -> XYZZ node i
DEV void small_leaf_pairs(const fe &x, const fe &y, bool zero, SmallNode *to, SmallNode *scratch, int n,
                          uint32_t lane) {
  if (lane < (uint32_t)n) {  // the leaf, affine: (x, y, zero) in the node's X, Y, identity slots
#pragma unroll
    for (int k = 0; k < 8; k++) scratch[lane].w[k] = x.v[k], scratch[lane].w[8 + k] = y.v[k];
    scratch[lane].w[32] = zero ? 1u : 0u;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
  if (lane < (uint32_t)(n + 1) / 2) {
    fe x1, y1, x2, y2;
    bool i1, i2 = true;
#pragma unroll
    for (int k = 0; k < 8; k++) x1.v[k] = scratch[2 * lane].w[k], y1.v[k] = scratch[2 * lane].w[8 + k];
    i1 = scratch[2 * lane].w[32] != 0;
    if (2 * (int)lane + 1 < n) {
#pragma unroll
      for (int k = 0; k < 8; k++) x2.v[k] = scratch[2 * lane + 1].w[k], y2.v[k] = scratch[2 * lane + 1].w[8 + k];
      i2 = scratch[2 * lane + 1].w[32] != 0;
    }
    gexz R;
    bool inf;
    gexz_sum_ge_lat(R, inf, x1, y1, i1, x2, y2, i2);
    part_store(to[lane].w, R, inf);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
// s^-1 of one item split over two waves (both run it on the scalar unit).
// The Bernstein-Yang batches' critical chain is divsteps + the (f, g)
// update: each batch's 2x2 matrix depends on the new f, g low words only.
// The (d, e) update of each batch (whose result is needed only at the end)
// runs on another wave, fed the matrices through an LDS ring.
constexpr int kSinvRing = 16;
struct SinvMail {
  int32_t t[kSinvRing][4];
  uint32_t produced, consumed, done;  // matrices published / applied; total + 1 once g = 0 (0: running)
  int32_t f_sign;
};
// A flag read, made wave-uniform (every lane takes lane 0's value, so a
// branch on it is a scalar branch and no lane can see a different value of
// a flag another wave is writing).
DEV uint32_t lds_acquire(const uint32_t *p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
DEV void lds_release(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }
// BV_SINV_VALU (A/B, off): the split inversion's values in VGPRs (lane 0 of
// each of the two waves), so the divsteps, the matrix products (one
// v_mad_i64_i32 each) and the loop tests run on the VECTOR unit.  Alone it
// is 13 % faster than the scalar unit (69k against 79k clocks per
// inversion, profiles/r06_ubench_sinv.txt); inside k_small, beside the
// other waves' vector work, the split inversion measured 75k-105k clocks
// against 70k-75k on the scalar unit (profiles/r06_small_lat_b.log)
#ifndef BV_SINV_VALU
#define BV_SINV_VALU 0
#endif
DEV uint32_t in_vgpr(uint32_t x) {
#if BV_SINV_VALU
  asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(x));
#endif
  return x;
}
// producer (the s^-1 chain): divsteps and the (f, g) updates
DEV void sinv_split_fg(SinvMail &mb, const sc &s_in) {
  modinfo30 mi;
  modinfo_n(mi);
  sc s;
#pragma unroll
  for (int i = 0; i < 8; i++) s.v[i] = in_vgpr(s_in.v[i]);
  s30 f, g;
#pragma unroll
  for (int i = 0; i < 9; i++) f.v[i] = mi.m[i];
  s30_from_u256(g, s.v);
  int32_t eta = -1;
  uint32_t k = 0;
  for (;;) {
    int32_t t[4];
    eta = divsteps_30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    while (k - lds_acquire(&mb.consumed) >= (uint32_t)kSinvRing) __builtin_amdgcn_s_sleep(1);  // ring full
#pragma unroll
    for (int i = 0; i < 4; i++) mb.t[k % kSinvRing][i] = t[i];
    lds_release(&mb.produced, ++k);
    update_fg_30(f, g, t);
    int32_t z = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) z |= g.v[i];
    if (z == 0) break;
  }
  mb.f_sign = f.v[8] >> 31;
  lds_release(&mb.done, k + 1);
}
// consumer: the (d, e) updates, then inv = s^-1 mod N (plain, < N): phase
// 2 forms u1 = e s^-1 and u2 = r s^-1 as ONE Montgomery product each, of inv
// and the e R, r R that wave 0 prepared beside the inversion
DEV void sinv_split_de(SinvMail &mb, sc &inv) {
  modinfo30 mi;
  modinfo_n(mi);
  s30 d, e;
#pragma unroll
  for (int i = 0; i < 9; i++) d.v[i] = 0, e.v[i] = 0;
  e.v[0] = 1;
  for (uint32_t k = 0;; k++) {
    uint32_t done;
    while (k >= lds_acquire(&mb.produced) && !(done = lds_acquire(&mb.done))) __builtin_amdgcn_s_sleep(1);
    if (k >= lds_acquire(&mb.produced)) break;  // (done: every matrix applied)
    int32_t t[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
      t[i] = BV_SINV_VALU ? (int32_t)in_vgpr((uint32_t)mb.t[k % kSinvRing][i])
                          : __builtin_amdgcn_readfirstlane(mb.t[k % kSinvRing][i]);
    update_de_30(d, e, t, mi);
    lds_release(&mb.consumed, k + 1);
  }
  normalize_30(d, __builtin_amdgcn_readfirstlane(mb.f_sign), mi);
  s30_to_u256(inv.v, d);
}

// ---- the cold path (no key-cache table), right to left in lockstep phases.
// Wave 2 doubles Q from the moment it is decoded (2^i Q in XYZZ with beta X,
// coop.h dbl_xyzz) into LDS; waves 1 and 3 add +-2^i Q / +-phi(2^i Q) for
// the non-zero NAF digits of k1 / k2 (coop.h add_xyzz); wave 0 sums the G
// leaves.  Every hand-over between waves goes through a workgroup barrier:
// the doubling chain runs in chunks of kColdChunk doublings, one barrier
// after each, and an entry is read only in a phase after the one that wrote
// it.  What each wave does in phase j is a function of (j, k1, k2) alone,
// so the additions happen in the same order whatever the waves' timing, and
// no wave leaves the kernel before the last one has finished (the round-5
// flag-driven form of this pipeline, withdrawn, had neither property;
// DESIGN.md section 4).
constexpr uint32_t kChainBits = 130;  // NAF digits of a GLV half (|k| < 2^129)
constexpr uint32_t kColdD0 = 16;      // doublings beside s^-1 (phase 1: ~70k clocks, ~4.4k per doubling)
constexpr uint32_t kColdD1 = 20;      // doublings beside u1, u2, the GLV split and the G sum (phase 2: ~90k clocks)
constexpr uint32_t kColdPre = 1 + kColdD0 + kColdD1;  // entries published before the chunk loop
constexpr uint32_t kColdChunk = 6;    // doublings per loop phase
constexpr uint32_t kColdBudget = 4;   // additions per half per phase (an addition ~1.33 doublings)
constexpr uint32_t kColdGJoin = 0;    // the phase in which wave 3 adds the G sum (wave 0 sums it in phase 2)
struct ChainPt {
  uint32_t x[8], bx[8], y[8], zz[8], zzz[8];
};
struct SmallCold {
  ChainPt pt[kChainBits];
  SmallNode acc3;  // wave 3's sum: k2 phi(Q) + u1 G
};
__device__ __forceinline__ uint32_t row_limb(const uint32_t *p) { return coop::pos() < 8 ? p[coop::pos()] : 0u; }
__device__ __forceinline__ void row_store(uint32_t *p, uint32_t v) {
  if (__lane_id() < 8) p[__lane_id()] = v;
}
// entries 2^i Q visible in phase j of the chunk loop (all written before
// the barrier that opened it)
DEV uint32_t cold_pub(uint32_t j, uint32_t nb) { return min(nb, kColdPre + j * kColdChunk); }
// the digits a half takes in one phase: from `pos` up to `end`, stopping
// before its (budget + 1)-th non-zero digit.  The kernel's additions and
// the phase count (cold_phases) both follow this rule.
DEV uint32_t cold_take(const uint32_t m[5], uint32_t pos, uint32_t end, uint32_t budget) {
  for (; pos < end; pos++)
    if ((m[pos >> 5] >> (pos & 31)) & 1u) {
      if (budget == 0) break;
      budget--;
    }
  return pos;
}
// phases until both halves have taken every digit (and wave 3 the G sum)
DEV uint32_t cold_phases(const uint32_t m1[5], const uint32_t m3[5], uint32_t nb) {
  uint32_t p1 = 0, p3 = 0, j = 0;
  for (; j < 64 && (p1 < nb || p3 < nb || j <= kColdGJoin); j++) {
    p1 = cold_take(m1, p1, cold_pub(j, nb), kColdBudget);
    p3 = cold_take(m3, p3, cold_pub(j, nb), kColdBudget - (j == kColdGJoin ? 1u : 0u));
  }
  return j;
}
// wave 2: 2^i Q -> entry i (lanes 0..7 of row 0 store)
__device__ __forceinline__ void cold_store(SmallCold &cs, uint32_t i, uint32_t X, uint32_t Y, uint32_t ZZ, uint32_t ZZZ,
                                           uint32_t BX) {
  ChainPt &e = cs.pt[i];
  row_store(e.x, X), row_store(e.bx, BX), row_store(e.y, Y), row_store(e.zz, ZZ), row_store(e.zzz, ZZZ);
}
// R += node (a SmallNode in LDS: X Y ZZ ZZZ + identity flag), cooperatively
__device__ __forceinline__ void cold_add_node(uint32_t &X, uint32_t &Y, uint32_t &ZZ, uint32_t &ZZZ, bool &inf,
                                              const SmallNode &nd) {
  if (!__builtin_amdgcn_readfirstlane(nd.w[32]))
    coop::add_xyzz(X, Y, ZZ, ZZZ, inf, row_limb(nd.w), row_limb(nd.w + 8), row_limb(nd.w + 16), row_limb(nd.w + 24));
}
// `to` = the sum of nodes [lo, hi) of `from` (one wave, cooperatively)
__device__ __forceinline__ void coop_sum_nodes(const SmallNode *from, uint32_t lo, uint32_t hi, SmallNode &to) {
  uint32_t X = 0, Y = 0, ZZ = 0, ZZZ = 0;
  bool inf = true;
  for (uint32_t j = lo; j < hi; j++) cold_add_node(X, Y, ZZ, ZZZ, inf, from[j]);
  row_store(to.w, X), row_store(to.w + 8, Y), row_store(to.w + 16, ZZ), row_store(to.w + 24, ZZZ);
  if (__lane_id() == 0) to.w[32] = inf ? 1u : 0u;
}
// the warm tree's first level: wave w sums leaf-pair nodes [kWarmSplit[w], kWarmSplit[w + 1])
constexpr uint32_t kWarmSplit[5] = {0, 3, 6, 9, (kSmallLeaves + 1) / 2};
}  // namespace

__global__ void __launch_bounds__(256) k_small(uint32_t n_items, const uint32_t *__restrict__ digest_words,
                                               const uint8_t *__restrict__ key_bytes,
                                               const uint64_t *__restrict__ key_off,
                                               const uint32_t *__restrict__ item_msg,
                                               const uint32_t *__restrict__ item_key,
                                               const uint32_t *__restrict__ r_be, const uint32_t *__restrict__ s_be,
                                               const uint8_t *__restrict__ pre, const uint64_t *__restrict__ kc_tabs,
                                               const uint32_t *__restrict__ g_table, uint8_t *__restrict__ status,
                                               uint64_t *__restrict__ stamps, const uint32_t *__restrict__ rec,
                                               uint64_t *__restrict__ clk) {
  const uint32_t b = blockIdx.x, t = threadIdx.x, wave = t >> 6, lane = t & 63;
  // the launch's span on the 100 MHz constant clock, in host memory:
  // clk[0] = workgroup 0's start, clk[1 + b] = workgroup b's end, written
  // before its status byte (no timing events around the launch)
  if (b == 0 && t == 0) clk[0] = __builtin_amdgcn_s_memrealtime();
#define SMALL_DONE(value)                                \
  do {                                                   \
    const uint8_t st_ = (value);                         \
    clk[1 + b] = __builtin_amdgcn_s_memrealtime();       \
    __threadfence_system();                              \
    status[b] = st_;                                     \
  } while (0)
#define SMALL_STAMP(k)                                                     \
  do {                                                                     \
    if (stamps && b == 0) stamps[k] = __builtin_amdgcn_s_memtime();        \
  } while (0)
  if (t == 0) SMALL_STAMP(0);
  __shared__ uint32_t sh_w[8], sh_q[16], sh_u1[8], sh_k[8], sh_r[8], sh_s[8], sh_eR[8], sh_rR[8];
  __shared__ uint32_t sh_ks, sh_go, sh_signs, sh_pre, sh_nb, sh_nphase;
  __shared__ uint64_t sh_tab;
  __shared__ SinvMail sh_mail;
  __shared__ uint32_t sh_sok, sh_cls;
  __shared__ SmallNode sh_a[kSmallLeaves], sh_b[kSmallLeaves / 2 + 1], sh_c[kSmallLeaves / 4 + 2];
  __shared__ SmallCold cs;
  __shared__ uint32_t sh_rec[hrec::kWords];
  if (b >= n_items) return;  // (the grid is n_items)
  if (t == 0) sh_mail.produced = sh_mail.consumed = sh_mail.done = 0;
  __syncthreads();
  // wave 2's doubling state (the cold path; replicated in every DPP row)
  uint32_t dX = 0, dY = 0, dZZ = 0, dZZZ = 0, dBX = 0;
  bool chain = false;  // wave 2: this item doubles Q (no table, Q decoded)
  // ---- phase 1 (the inputs live in host memory, read in place: wave 0
  // fetches what phases 2-4 need while s^-1 runs).  With host records
  // (hostscalar.h; `rec` is a kernel argument, so the branch is uniform):
  // ONE 256-byte read, the scalars already there, wave 2 decodes Q.
  if (rec) {
    if (wave == 0) sh_rec[lane] = rec[hrec::kWords * (uint64_t)b + lane];
    __syncthreads();
    if (lane == 0 && wave == 0) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        sh_r[k] = sh_rec[hrec::kR + k], sh_s[k] = sh_rec[hrec::kS + k], sh_u1[k] = sh_rec[hrec::kU1 + k];
        sh_k[k] = sh_rec[hrec::kK + k];
      }
      sh_signs = sh_rec[hrec::kSigns];
      sh_pre = sh_rec[hrec::kPre];
      sh_tab = (uint64_t)sh_rec[hrec::kTab] | (uint64_t)sh_rec[hrec::kTab + 1] << 32;
      SMALL_STAMP(2);
    } else if (lane == 0 && wave == 2) {
      if (sh_rec[hrec::kTab] | sh_rec[hrec::kTab + 1]) {
        // a key-cache table exists only for these exact bytes decoded
        // KS_OK: phase 2 decides with that, and wave 2 decodes the key
        // again in phase 3, beside the leaf loads, for the final decision
        sh_ks = KS_OK;
      } else {
        uint8_t st;
        fe x, y;
        key_decode_point((const uint8_t *)(sh_rec + hrec::kKey), 0, sh_rec[hrec::kKeyLen], st, x, y);
#pragma unroll
        for (int c = 0; c < 8; c++) sh_q[c] = x.v[c], sh_q[8 + c] = y.v[c];
        sh_ks = st;
        chain = st == KS_OK;
      }
      SMALL_STAMP(3);
    }
  } else if (lane == 0 && wave == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) sh_r[k] = r_be[8 * (uint64_t)b + k];
    const uint32_t m = item_msg[b];
    sh_pre = pre ? pre[b] : 0u;
    sh_tab = kc_tabs ? kc_tabs[item_key[b]] : 0;
    // e R and r R mod N beside the inversion (Montgomery form), so u1 and
    // u2 are one product of each with s^-1 after it
    sc e, r, R2, eR, rR;
    sc_load_be_words(e, digest_words + 8 * (uint64_t)m);
    sc_load_be_words(r, r_be + 8 * (uint64_t)b);
    sc_load_const(R2, SC_R2);
    sc_mont(eR, e, R2);  // (e < 2^256 = R unreduced, R2 < N)
    sc_mont(rR, r, R2);
#pragma unroll
    for (int k = 0; k < 8; k++) sh_eR[k] = eR.v[k], sh_rR[k] = rR.v[k];
  } else if (lane == 0 && wave == 1) {  // s^-1: divsteps and (f, g) (wave 3 applies (d, e))
    sc s;
    sc_load_be_words(s, s_be + 8 * (uint64_t)b);
#pragma unroll
    for (int k = 0; k < 8; k++) sh_s[k] = s_be[8 * (uint64_t)b + k];
    const bool ok = s_usable(pre, b, s);
    sh_sok = ok;
    if (ok) sinv_split_fg(sh_mail, s);
    else lds_release(&sh_mail.done, 1);
  } else if (lane == 0 && wave == 3) {
    sc inv;
    sinv_split_de(sh_mail, inv);
    if (!__builtin_amdgcn_readfirstlane(sh_sok)) {  // (published before done)
#pragma unroll
      for (int k = 0; k < 8; k++) inv.v[k] = 0;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) sh_w[k] = inv.v[k];  // s^-1 mod N
    SMALL_STAMP(2);
  } else if (lane == 0 && wave == 2) {
    const uint32_t k = item_key[b];
    uint8_t st;
    fe x, y;
    key_decode_point(key_bytes, key_off[k], key_off[k + 1] - key_off[k], st, x, y);
#pragma unroll
    for (int c = 0; c < 8; c++) sh_q[c] = x.v[c], sh_q[8 + c] = y.v[c];
    sh_ks = st;
    // (wave 2 reads the table address itself: wave 0's copy is not
    // published before the barrier)
    chain = st == KS_OK && !(kc_tabs && kc_tabs[k]);
    SMALL_STAMP(3);
  }
  if (wave == 2) {
    chain = __builtin_amdgcn_readfirstlane(chain ? 1u : 0u) != 0;
    if (chain) {  // entries 0..kColdD0: Q, 2Q, ..., 2^kColdD0 Q
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // lane 0's sh_q, for the whole wave
      __builtin_amdgcn_wave_barrier();
      dX = row_limb(sh_q), dY = row_limb(sh_q + 8), dZZ = coop::pos() == 0 ? 1u : 0u, dZZZ = dZZ;
      dBX = coop::mul(dX, coop::beta_limb());
      cold_store(cs, 0, dX, dY, dZZ, dZZZ, dBX);
      for (uint32_t i = 1; i <= kColdD0; i++) {
        coop::dbl_xyzz(dX, dY, dZZ, dZZZ, dBX);
        cold_store(cs, i, dX, dY, dZZ, dZZZ, dBX);
      }
      if (lane == 0) SMALL_STAMP(4);
    }
  }
  __syncthreads();
  if (t == 0) SMALL_STAMP(5);
  // ---- phase 2: the decision table and u1 (wave 0), u2 + GLV (wave 1)
  if (lane == 0 && wave == 0) {
    fe r, sv;
    fe_load_be_words(r, sh_r);
    fe_load_be_words(sv, sh_s);
    const uint8_t cls = classify((uint8_t)sh_pre, (uint8_t)sh_ks, r, sv);
    sh_go = cls == 0xFF;
    if (cls != 0xFF) {
      SMALL_DONE(cls);
    } else if (!rec) {  // (a host record holds u1)
      sc inv, eR, a;
#pragma unroll
      for (int k = 0; k < 8; k++) inv.v[k] = sh_w[k], eR.v[k] = sh_eR[k];
      sc_mont(a, eR, inv);  // e R s^-1 R^-1 = e s^-1 mod N
#pragma unroll
      for (int k = 0; k < 8; k++) sh_u1[k] = a.v[k];
    }
  } else if (lane == 0 && wave == 1) {
    uint32_t k1[4], k2[4];
    if (!rec) {
      sc inv, rR, u2;
#pragma unroll
      for (int k = 0; k < 8; k++) inv.v[k] = sh_w[k], rR.v[k] = sh_rR[k];
      sc_mont(u2, rR, inv);  // r s^-1 mod N (only used when the item reaches the math)
      uint32_t signs;
      glv_split(k1, k2, signs, u2);
#pragma unroll
      for (int k = 0; k < 4; k++) sh_k[k] = k1[k], sh_k[4 + k] = k2[k];
      sh_signs = signs;
    } else {  // (the host record's split, in sh_k since phase 1)
#pragma unroll
      for (int k = 0; k < 4; k++) k1[k] = sh_k[k], k2[k] = sh_k[4 + k];
    }
    if (!sh_tab) {  // the cold path's chain length and phase count
      uint32_t p1[5], n1[5], p2[5], n2[5], m1[5], m3[5], nb = 0;
      naf_masks(k1, p1, n1);
      naf_masks(k2, p2, n2);
      for (int i = 0; i < 5; i++) m1[i] = p1[i] | n1[i], m3[i] = p2[i] | n2[i];
      for (int i = 4; i >= 0 && nb == 0; i--)
        if (m1[i] | m3[i]) nb = 32 * i + 32 - __builtin_clz(m1[i] | m3[i]);
      nb = min(nb, kChainBits);
      sh_nb = nb;
      sh_nphase = cold_phases(m1, m3, nb);
    }
  } else if (wave == 2 && chain) {  // entries kColdD0 + 1 .. kColdPre - 1
    for (uint32_t i = kColdD0 + 1; i < kColdPre; i++) {
      coop::dbl_xyzz(dX, dY, dZZ, dZZZ, dBX);
      cold_store(cs, i, dX, dY, dZZ, dZZZ, dBX);
    }
  }
  if (wave == 0 && !sh_tab) {  // no table: the G leaves of u1 and their sum, 10 -> 5 -> 3 -> 2 -> 1 (sh_c[0])
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // lane 0's sh_go and sh_u1, for the whole wave
    __builtin_amdgcn_wave_barrier();
    if (__builtin_amdgcn_readfirstlane(sh_go)) {
      fe x, y;
      bool zero = true;
      if (lane < BV_GNWIN) {
        uint32_t u[8];
#pragma unroll
        for (int k = 0; k < 8; k++) u[k] = sh_u1[k];
        table_leaf<BV_GW, 8>(x, y, zero, g_table, u, (int)lane, false, false);
      }
      small_leaf_pairs(x, y, zero, sh_b, sh_a, BV_GNWIN, lane);
      small_tree_level(sh_b, sh_c, 5, lane);
      small_tree_level(sh_c, sh_b, 3, lane);
      small_tree_level(sh_b, sh_c, 2, lane);
      if (lane == 0) SMALL_STAMP(7);
    }
  }
  __syncthreads();
  if (t == 0) SMALL_STAMP(6);
  if (!sh_go) return;  // decided by the table (uniform)
  const uint32_t signs = sh_signs;
  const uint64_t tab = sh_tab;  // wave-uniform
  // ---- phase 3
  if (tab) {
    if (wave == 0) {
      fe x, y;
      bool zero = true;
      if (lane < BV_GNWIN) {  // G window `lane` of u1
        uint32_t u[8];
#pragma unroll
        for (int k = 0; k < 8; k++) u[k] = sh_u1[k];
        table_leaf<BV_GW, 8>(x, y, zero, g_table, u, (int)lane, false, false);
      } else if (lane < (uint32_t)kSmallLeaves) {  // KC window j of k1 (T) or of k2 (phi(T))
        const uint32_t q = lane - BV_GNWIN, h = q / BV_KCNWIN;
        uint32_t kk[4];
#pragma unroll
        for (int k = 0; k < 4; k++) kk[k] = sh_k[4 * h + k];
        table_leaf<BV_KCW, 4>(x, y, zero, (const uint32_t *)tab, kk, (int)(q % BV_KCNWIN), (signs >> h) & 1u,
                              h != 0);
      }
      if (lane == 0) SMALL_STAMP(7);
      small_leaf_pairs(x, y, zero, sh_b, sh_a, kSmallLeaves, lane);  // 22 leaves -> 11 nodes (per lane)
      if (lane == 0) SMALL_STAMP(8);
    } else if (rec && wave == 2 && lane == 0) {  // the record's key, decoded off the critical path
      uint8_t st;
      fe x, y;
      key_decode_point((const uint8_t *)(sh_rec + hrec::kKey), 0, sh_rec[hrec::kKeyLen], st, x, y);
      sh_ks = st;
    }
    __syncthreads();
    // the XYZZ tree on DPP rows (coop.h add_xyzz, ~6k clocks an addition
    // against ~21k for one lane's): 11 -> 4 (wave w sums nodes
    // kWarmSplit[w] .. kWarmSplit[w + 1] - 1), 4 -> 2 (waves 0, 1), 2 -> 1
    coop_sum_nodes(sh_b, kWarmSplit[wave], kWarmSplit[wave + 1], sh_c[wave]);
    __syncthreads();
    if (wave < 2) {
      coop_sum_nodes(sh_c, 2 * wave, 2 * wave + 2, sh_a[wave]);
    } else if (rec && wave == 2 && lane == 0) {  // the decision table with the key's own decode, meanwhile
      fe r, sv;
      fe_load_be_words(r, sh_r);
      fe_load_be_words(sv, sh_s);
      sh_cls = classify((uint8_t)sh_pre, (uint8_t)sh_ks, r, sv);
    }
    __syncthreads();
    if (wave == 0) {
      coop_sum_nodes(sh_a, 0, 2, sh_b[0]);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) SMALL_STAMP(11);
    }
    // ---- phase 4: the root (sh_b[0]) -> the decision
    if (t == 0) {
      gexz A;
      bool ia;
      part_load(sh_b[0].w, A, ia);
      fe r;
      fe_load_be_words(r, sh_r);
      uint8_t st = final_check(A, ia, r) ? BV_ACCEPT : BV_REJECT;
      if (rec && sh_cls != 0xFF) st = (uint8_t)sh_cls;  // (the key's own decode says otherwise)
      SMALL_DONE(st);
      SMALL_STAMP(13);
    }
    __syncthreads();  // no wave leaves before the last cooperative step of the workgroup
    return;
  }
  // ---- phase 3 without a table: the chunk loop (every wave runs every
  // phase and its barrier; the counts are uniform, read from LDS)
  const uint32_t nb = __builtin_amdgcn_readfirstlane(sh_nb), nphase = __builtin_amdgcn_readfirstlane(sh_nphase);
  const uint32_t h = wave == 3 ? 1u : 0u;  // (waves 1 and 3: the GLV half)
  uint32_t pm[5] = {}, nm[5] = {}, m[5] = {}, pos = 0;
  uint32_t X = 0, Y = 0, ZZ = 0, ZZZ = 0;
  bool inf = true;
  const bool neg_all = (signs >> h) & 1u;
  if (wave == 1 || wave == 3) {
    uint32_t kk[4];
#pragma unroll
    for (int k = 0; k < 4; k++) kk[k] = __builtin_amdgcn_readfirstlane(sh_k[4 * h + k]);
    naf_masks(kk, pm, nm);
#pragma unroll
    for (int i = 0; i < 5; i++) m[i] = pm[i] | nm[i];
  }
  for (uint32_t j = 0; j < nphase; j++) {
    if (wave == 2) {  // the chain: entries cold_pub(j) .. cold_pub(j + 1) - 1
      for (uint32_t i = cold_pub(j, nb); i < cold_pub(j + 1, nb); i++) {
        coop::dbl_xyzz(dX, dY, dZZ, dZZZ, dBX);
        cold_store(cs, i, dX, dY, dZZ, dZZZ, dBX);
      }
    } else if (wave != 0) {  // waves 1 / 3: +-2^i Q (h = 1: +-phi(2^i Q)) for the non-zero digits the phase takes
      uint32_t budget = kColdBudget;
      if (h && j == kColdGJoin) {  // the G sum (wave 0, phase 2)
        cold_add_node(X, Y, ZZ, ZZZ, inf, sh_c[0]);
        budget--;
      }
      for (const uint32_t end = cold_pub(j, nb); pos < end; pos++) {
        if (!((m[pos >> 5] >> (pos & 31)) & 1u)) continue;
        if (budget == 0) break;
        budget--;
        const ChainPt &e = cs.pt[pos];
        uint32_t y = row_limb(e.y);
        if ((((nm[pos >> 5] >> (pos & 31)) & 1u) != 0) != neg_all) y = coop::norm(coop::negw(y));
        coop::add_xyzz(X, Y, ZZ, ZZZ, inf, row_limb(h ? e.bx : e.x), y, row_limb(e.zz), row_limb(e.zzz));
      }
    }
    __syncthreads();
  }
  if (wave == 3) {  // k2 phi(Q) + u1 G to wave 1
    row_store(cs.acc3.w, X), row_store(cs.acc3.w + 8, Y), row_store(cs.acc3.w + 16, ZZ),
        row_store(cs.acc3.w + 24, ZZZ);
    if (lane == 0) cs.acc3.w[32] = inf ? 1u : 0u;
    if (lane == 0) SMALL_STAMP(10);
  }
  __syncthreads();
  if (wave == 1) {  // k1 Q + (k2 phi(Q) + u1 G), then the decision
    cold_add_node(X, Y, ZZ, ZZZ, inf, cs.acc3);
    row_store(sh_b[0].w, X), row_store(sh_b[0].w + 8, Y), row_store(sh_b[0].w + 16, ZZ), row_store(sh_b[0].w + 24, ZZZ);
    if (lane == 0) sh_b[0].w[32] = inf ? 1u : 0u;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      gexz A;
      bool ia;
      part_load(sh_b[0].w, A, ia);
      fe r;
      fe_load_be_words(r, sh_r);
      SMALL_DONE(final_check(A, ia, r) ? BV_ACCEPT : BV_REJECT);
      SMALL_STAMP(13);
    }
  }
  __syncthreads();  // no wave leaves before the last cooperative step of the workgroup
#undef SMALL_STAMP
#undef SMALL_DONE
}

// ---------------------------------------------------------------------------
// Launch wrappers (called from bv_api.cpp)
// ---------------------------------------------------------------------------
namespace bvk {

static inline dim3 grid1(uint64_t n, uint32_t block) { return dim3((uint32_t)((n + block - 1) / block)); }

// Verify kernels come in two variants: the throughput one (one multiply at a
// time, few VGPRs, 4+ waves per SIMD hide the latency) and the latency one
// (gej_*_lat: independent multiplies interleaved in one asm program) for
// batches too small to put more than ~2 waves on each of the 1024 SIMDs.
#ifndef BV_LAT_MAX_ITEMS
#define BV_LAT_MAX_ITEMS 131072
#endif
static inline bool lat_variant(uint64_t n) { return n <= BV_LAT_MAX_ITEMS; }
// The generic per-lane kernel's latency variant pays only up to 32k items:
// with two batches in flight its larger VGPR footprint halves the rate at
// 64k-128k items (1000 keys: 28.2 -> 45.9 / 28.6 -> 59.1 M/s without it),
// while single calls at <= 32k keep its 2.6-3.2 ms (r04_ab_generic_lat.log).
#ifndef BV_GEN_LAT_MAX_ITEMS
#define BV_GEN_LAT_MAX_ITEMS 32768
#endif

hipError_t sha256(hipStream_t st, uint64_t n, const uint8_t *bytes, const uint64_t *off, uint32_t *dig,
                  uint64_t max_len) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sha256, grid1(n, 256), dim3(256), 0, st, n, bytes, off, dig, max_len);
  return hipGetLastError();
}

hipError_t put_digests(hipStream_t st, uint64_t n, const uint64_t *idx, const uint32_t *vals, uint32_t *dig) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_put_digests, grid1(8 * n, 256), dim3(256), 0, st, n, idx, vals, dig);
  return hipGetLastError();
}

hipError_t ev_body_hash(hipStream_t st, const bv_event_batch &b, uint64_t e0, uint64_t e1, uint32_t *dig) {
  if (e1 <= e0) return hipSuccess;
  hipLaunchKernelGGL(k_ev_body_hash, grid1(e1 - e0, EVH_NT), dim3(EVH_NT), 0, st, b, e0, e1, dig);
  return hipGetLastError();
}

hipError_t sig_decode(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *text, uint8_t *r_be,
                      uint8_t *s_be, uint8_t *pre) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sig_decode, grid1(n, 256), dim3(256), 0, st, n, off, text, r_be, s_be, pre);
  return hipGetLastError();
}

hipError_t iota(hipStream_t st, uint64_t n, uint32_t *out) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_iota, grid1(n, 256), dim3(256), 0, st, n, out);
  return hipGetLastError();
}

hipError_t sha256_chain(hipStream_t st, uint32_t n, const uint8_t *bytes, const uint64_t *off, uint8_t *scratch,
                        uint32_t *out) {
  hipLaunchKernelGGL(k_sha256_chain, dim3(1), dim3(64), 0, st, n, bytes, off, scratch, out);
  return hipGetLastError();
}

hipError_t key_decode(hipStream_t st, uint32_t n, const uint8_t *kb, const uint64_t *ko, uint8_t *kst, uint32_t *kxy) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_key_decode, grid1(n, 64), dim3(64), 0, st, n, kb, ko, kst, kxy);
  return hipGetLastError();
}

// Point-op variant of the K12 table build (bit 0: base chains, bit 1:
// sub-table fills; 1 = zipped).  Beside a large batch's bulk kernels (`busy`)
// the fills take the throughput ops: with 4 bulk waves on a SIMD a wave needs
// a small VGPR footprint to be placed at all (same-box A/B: 415 -> 424 M
// verifies/s), while the lone-wave base chain keeps its zipped doubling.
// BV_K12_LAT overrides for A/B runs.
static int k12_lat_mask(bool busy) {
  static const int env = [] {
    const char *s = getenv("BV_K12_LAT");
    return s ? atoi(s) : -1;
  }();
  return env >= 0 ? env : busy ? 1 : 3;
}

// kw = 0: the generator table (BV_GW-bit windows over 256 bits from
// BV_GL-bit sub-tables, built once per process and device); kw = 8 / 12: the K8 / K12
// GLV key tables (verify_core.h).  `sub`
// is the K12 sub-table scratch (n_bases * BV_K12SUB_U32 words), `pscr` the
// K12 prefix-product scratch (n_bases * BV_K12HALF_U32 / 2 words).
// the base chains run wave-cooperative (BV_COOP_BASES=0 at process start:
// the per-lane chain, for A/B)
static const bool g_coop_bases = [] {
  const char *s = getenv("BV_COOP_BASES");
  return s == nullptr || atoi(s) != 0;
}();

// K8 for at most this many keys: each entry by its own double-and-add from
// the 8-bit bases (k_table_fill<8, 16, true>: one launch after the chain,
// the shortest chain for a few keys); above it the 4-bit sub-tables and
// chord sums (k_table_pair_u: ~12x less work per key).  Cold latency,
// 1000 / 4000 events: 4 keys 0.741 / 0.763 ms direct against 0.768 / 0.816
// chord, 16 keys 0.744 / 0.775 against 0.768 / 0.796, 32 keys equal
// (profiles/r05_ab_k8_direct.log); 64 keys chord 0.80 against 0.955
// (r05_ab_k8_lat.log).  BV_K8_DIRECT_KEYS.
static const uint32_t g_k8_direct_keys = [] {
  const char *s = getenv("BV_K8_DIRECT_KEYS");
  return s ? (uint32_t)atoi(s) : 24u;
}();

hipError_t build_tables(hipStream_t st, int kw, uint32_t n_bases, const uint32_t *bxy, const uint8_t *bstatus,
                        uint32_t *bases_jac, uint32_t *sub, uint32_t *pscr, uint32_t *table, uint64_t n_items) {
  const bool k8_direct = kw == 8 && n_bases <= g_k8_direct_keys;
  if (n_bases == 0) return hipSuccess;
  const int w = kw == 0 ? BV_GL : kw == 8 ? (k8_direct ? BV_KW : BV_KL) : BV_K12L;
  const int nwin = kw == 0 ? BV_GNSUB : kw == 8 ? (k8_direct ? BV_KNWIN : BV_KNSUB) : BV_K12NSUB;
  // K12 (large batches) builds beside the bulk kernels on a busy chip, where
  // a kernel's VGPR footprint decides when its waves get a SIMD: there the
  // throughput point ops (fewer VGPRs) win; elsewhere the zipped ones.
  const int lat = kw == 12 ? k12_lat_mask(!lat_variant(n_items)) : 3;
  if (g_coop_bases)
    hipLaunchKernelGGL(k_table_bases_coop, dim3(n_bases), dim3(64), 0, st, n_bases, bxy, bstatus, bases_jac, w, nwin);
  else if (lat & 1)
    hipLaunchKernelGGL(k_table_bases<true>, grid1(n_bases, 64), dim3(64), 0, st, n_bases, bxy, bstatus, bases_jac, w,
                       nwin);
  else
    hipLaunchKernelGGL(k_table_bases<false>, grid1(n_bases, 64), dim3(64), 0, st, n_bases, bxy, bstatus, bases_jac, w,
                       nwin);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (kw == 0) {  // n_bases == 1 (G); `pscr` holds BV_GPAIR_BLOCKS blocks x 4096 fe
    hipLaunchKernelGGL((k_table_fill<BV_GL, BV_GNSUB, false>), dim3(BV_GNSUB * ((1u << BV_GL) / 256u), 1), dim3(256),
                       0, st, bases_jac, bstatus, sub);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    for (uint32_t j = 0; j < BV_GNWIN; j++) {
      // slots needed: all of a full window; the top window's digits are
      // <= 2^(256 - W j) (its value bits plus the carry)
      const int live_bits = 256 - BV_GW * (int)j;
      const uint64_t live = live_bits >= BV_GW - 1 ? BV_GENT : (1ull << live_bits) + 1;
      const uint32_t blocks = (uint32_t)((live + 4095) / 4096);
      for (uint32_t c0 = 0; c0 < blocks; c0 += BV_GPAIR_BLOCKS) {
        const uint32_t nb = blocks - c0 < BV_GPAIR_BLOCKS ? blocks - c0 : BV_GPAIR_BLOCKS;
        hipLaunchKernelGGL((k_table_pair_g<BV_GW, BV_GL>), dim3(nb), dim3(256), 0, st, sub, table, (uint4 *)pscr, j,
                           c0);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
      }
    }
  } else if (k8_direct) {
    hipLaunchKernelGGL((k_table_fill<BV_KW, BV_KNWIN, true>), dim3(BV_KNWIN * ((1u << BV_KW) / 256u), n_bases),
                       dim3(256), 0, st, bases_jac, bstatus, table);
  } else if (kw == 8) {
    // 4-bit sub-tables (16 per block of 256: one inversion per block), then
    // the chord sums.  The zipped point ops only for few keys and a small
    // batch: their VGPRs allow 2 blocks per CU, and 1000 keys' 2000 blocks
    // then take 4 rounds (0.55 ms per fill)
    constexpr uint32_t fill_blocks = (BV_KNSUB << BV_KL) / 256u;
    if (lat_variant(n_items) && n_bases <= 256)
      hipLaunchKernelGGL((k_table_fill<BV_KL, BV_KNSUB, false, 256, true>), dim3(fill_blocks, n_bases), dim3(256), 0,
                         st, bases_jac, bstatus, sub);
    else
      hipLaunchKernelGGL((k_table_fill<BV_KL, BV_KNSUB, false, 256, false>), dim3(fill_blocks, n_bases), dim3(256), 0,
                         st, bases_jac, bstatus, sub);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (n_bases <= 64)  // latency: 16 blocks (one inversion each) per key
      hipLaunchKernelGGL((k_table_pair_u<BV_KW, BV_KL, BV_KNWIN, 1>), dim3(BV_KNWIN, n_bases), dim3(256), 0, st, sub,
                         bstatus, table, (uint4 *)pscr);
    else if (n_bases <= 256)
      hipLaunchKernelGGL((k_table_pair_u<BV_KW, BV_KL, BV_KNWIN, 4>), dim3(BV_KNWIN / 4, n_bases), dim3(256), 0, st, sub,
                         bstatus, table, (uint4 *)pscr);
    else  // throughput: one inversion per key
      hipLaunchKernelGGL((k_table_pair_u<BV_KW, BV_KL, BV_KNWIN, BV_KNWIN>), dim3(1, n_bases), dim3(256), 0, st, sub,
                         bstatus, table, (uint4 *)pscr);
  } else {
    if (lat & 2)
      hipLaunchKernelGGL((k_table_fill<BV_K12L, BV_K12NSUB, false, 1 << BV_K12L, true>), dim3(BV_K12NSUB, n_bases),
                         dim3(1 << BV_K12L), 0, st, bases_jac, bstatus, sub);
    else
      hipLaunchKernelGGL((k_table_fill<BV_K12L, BV_K12NSUB, false, 1 << BV_K12L, false>), dim3(BV_K12NSUB, n_bases),
                         dim3(1 << BV_K12L), 0, st, bases_jac, bstatus, sub);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_table_pair<BV_K12W, BV_K12L, BV_K12NWIN>), dim3(BV_K12NWIN, n_bases), dim3(256), 0, st, sub,
                       bstatus, table, (uint4 *)pscr);
  }
  return hipGetLastError();
}

hipError_t sinv(hipStream_t st, uint64_t n, uint32_t M, const uint32_t *s_be, const uint8_t *pre, uint32_t *w) {
  if (n == 0) return hipSuccess;
  const uint64_t threads = (n + M - 1) / M;
  hipLaunchKernelGGL(k_sinv, grid1(threads, 256), dim3(256), 0, st, n, M, s_be, pre, w);
  return hipGetLastError();
}

// Items [lo, hi) of an n-item batch (R_G is stored SoA with stride n).
hipError_t glv_split(hipStream_t st, uint64_t n, const uint32_t *r_be, const uint32_t *w, uint32_t *u12) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_glv_split, grid1(n, 256), dim3(256), 0, st, n, r_be, w, u12);
  return hipGetLastError();
}

// split: u12 holds the GLV split already (k_glv_split on the s^-1 stream)
hipError_t verify_g(hipStream_t st, uint64_t n, uint64_t lo, uint64_t hi, const uint32_t *item_key,
                    const uint32_t *r_be, const uint32_t *s_be, const uint8_t *pre, const uint8_t *kst,
                    const uint32_t *item_msg, const uint32_t *dig, const uint32_t *w, uint32_t *u12,
                    const uint32_t *g_table, uint32_t *rg, bool split) {
  if (hi <= lo) return hipSuccess;
  const bool lat = lat_variant(n);
  auto k = lat ? (split ? k_verify_g<true, true> : k_verify_g<true, false>)
               : (split ? k_verify_g<false, true> : k_verify_g<false, false>);
  hipLaunchKernelGGL(k, grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key, r_be, s_be, pre, kst, item_msg,
                     dig, w, u12, g_table, rg);
  return hipGetLastError();
}

// kw = 8 / 12: contiguous per-batch tables in key_table; kw = 22: the key
// cache (KC), table base address per batch key in key_tabs.
hipError_t verify_q(hipStream_t st, int kw, uint64_t n, uint64_t lo, uint64_t hi, const uint32_t *item_key,
                    const uint32_t *r_be, const uint32_t *s_be, const uint8_t *pre, const uint8_t *kst,
                    const uint32_t *u12, const uint32_t *key_table, const uint64_t *key_tabs, const uint32_t *rg,
                    uint8_t *status, uint64_t *bits) {
  if (hi <= lo) return hipSuccess;
  const bool lat = lat_variant(n);
#define BV_LAUNCH_Q(W, NWIN, KT, KTABS)                                                                             \
  if (lat)                                                                                                       \
    hipLaunchKernelGGL((k_verify_q<W, NWIN, true>), grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key,  \
                       r_be, s_be, pre, kst, u12, KT, KTABS, rg, status, bits);                                  \
  else                                                                                                           \
    hipLaunchKernelGGL((k_verify_q<W, NWIN, false>), grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key,   \
                       r_be, s_be, pre, kst, u12, KT, KTABS, rg, status, bits);
  if (kw == 8) {
    BV_LAUNCH_Q(BV_KW, BV_KNWIN, key_table, nullptr)
  } else if (kw == 12) {
    BV_LAUNCH_Q(BV_K12W, BV_K12NWIN, key_table, nullptr)
  } else {
    BV_LAUNCH_Q(BV_KCW, BV_KCNWIN, nullptr, key_tabs)
  }
#undef BV_LAUNCH_Q
  return hipGetLastError();
}

// Key part first: R_Q of items [lo, hi) into rq (SoA, stride n); kw as
// verify_q.
hipError_t verify_qf(hipStream_t st, int kw, uint64_t n, uint64_t lo, uint64_t hi, const uint32_t *item_key,
                     const uint32_t *r_be, const uint32_t *s_be, const uint8_t *pre, const uint8_t *kst,
                     const uint32_t *w, const uint32_t *key_table, const uint64_t *key_tabs, uint32_t *rq) {
  if (hi <= lo) return hipSuccess;
  const bool lat = lat_variant(n);
#define BV_LAUNCH_QF(W, NWIN, KT, KTABS)                                                                            \
  if (lat)                                                                                                       \
    hipLaunchKernelGGL((k_verify_qf<W, NWIN, true>), grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key, \
                       r_be, s_be, pre, kst, w, KT, KTABS, rq);                                                  \
  else                                                                                                           \
    hipLaunchKernelGGL((k_verify_qf<W, NWIN, false>), grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key, \
                       r_be, s_be, pre, kst, w, KT, KTABS, rq);
  if (kw == 8) {
    BV_LAUNCH_QF(BV_KW, BV_KNWIN, key_table, nullptr)
  } else if (kw == 12) {
    BV_LAUNCH_QF(BV_K12W, BV_K12NWIN, key_table, nullptr)
  } else {
    BV_LAUNCH_QF(BV_KCW, BV_KCNWIN, nullptr, key_tabs)
  }
#undef BV_LAUNCH_QF
  return hipGetLastError();
}

// ... then u1 G and the decision for items [lo, hi) once their digests are in.
hipError_t verify_gf(hipStream_t st, uint64_t n, uint64_t lo, uint64_t hi, const uint32_t *item_key,
                     const uint32_t *r_be, const uint32_t *s_be, const uint8_t *pre, const uint8_t *kst,
                     const uint32_t *item_msg, const uint32_t *dig, const uint32_t *w, const uint32_t *g_table,
                     const uint32_t *rq, uint8_t *status, uint64_t *bits) {
  if (hi <= lo) return hipSuccess;
  if (lat_variant(n))
    hipLaunchKernelGGL(k_verify_gf<true>, grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key, r_be, s_be, pre,
                       kst, item_msg, dig, w, g_table, rq, status, bits);
  else
    hipLaunchKernelGGL(k_verify_gf<false>, grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key, r_be, s_be, pre,
                       kst, item_msg, dig, w, g_table, rq, status, bits);
  return hipGetLastError();
}

hipError_t verify_gq(hipStream_t st, uint64_t n, uint64_t lo, uint64_t hi, const uint32_t *item_key,
                     const uint32_t *r_be, const uint32_t *s_be, const uint8_t *pre, const uint8_t *kst,
                     const uint32_t *item_msg, const uint32_t *dig, const uint32_t *w, const uint32_t *g_table,
                     const uint64_t *key_tabs, uint8_t *status, uint64_t *bits) {
  if (hi <= lo) return hipSuccess;
  if (lat_variant(n))
    hipLaunchKernelGGL(k_verify_gq<true>, grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key, r_be, s_be, pre,
                       kst, item_msg, dig, w, g_table, key_tabs, status, bits);
  else
    hipLaunchKernelGGL(k_verify_gq<false>, grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key, r_be, s_be, pre,
                       kst, item_msg, dig, w, g_table, key_tabs, status, bits);
  return hipGetLastError();
}

// Key-cache tables for n keys (decoded affine points kxy, statuses kst):
// bases 2^(11 k) Q (k < 12), the 11-bit sub-tables into `sub`
// (n * BV_KCSUB_U32 words), then every window's chord sums into
// tabs[b] (BV_KCTABLE_U32 words each; k_verify_q forms the phi half).
// `pscr`: n * kc_pscr_bytes() bytes.
size_t kc_pscr_bytes() {
  return (size_t)BV_KCNWIN * (BV_KCENT / BV_KCPAIR_ENT) * BV_KCPAIR_ENT * 32;
}
hipError_t build_kc(hipStream_t st, uint32_t n, const uint32_t *kxy, const uint8_t *kst, uint32_t *bases_jac,
                    uint32_t *sub, uint32_t *pscr, const uint64_t *tabs) {
  if (n == 0) return hipSuccess;
  if (g_coop_bases)
    hipLaunchKernelGGL(k_table_bases_coop, dim3(n), dim3(64), 0, st, n, kxy, kst, bases_jac, BV_KCL, BV_KCNSUB);
  else
    hipLaunchKernelGGL(k_table_bases<true>, grid1(n, 64), dim3(64), 0, st, n, kxy, kst, bases_jac, BV_KCL, BV_KCNSUB);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_table_fill<BV_KCL, BV_KCNSUB, false>), dim3(BV_KCNSUB * ((1u << BV_KCL) / 256u), n),
                     dim3(256), 0, st, bases_jac, kst, sub);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_table_pair_kc<BV_KCW, BV_KCL, BV_KCNWIN>),
                     dim3(BV_KCNWIN * (BV_KCENT / BV_KCPAIR_ENT), n), dim3(256), 0, st, sub, kst, tabs, (uint4 *)pscr);
  return hipGetLastError();
}

// (no timing events around a latency-bound launch: the kernel writes its
// own span on the constant clock into `clk`, host memory)
hipError_t verify_small(hipStream_t st, uint32_t n_items, const uint8_t *dig, const uint8_t *key_bytes,
                        const uint64_t *key_off, const uint32_t *item_msg, const uint32_t *item_key,
                        const uint8_t *r_be, const uint8_t *s_be, const uint8_t *pre, const uint64_t *kc_tabs,
                        const uint32_t *g_table, uint8_t *status, uint64_t *stamps, const uint32_t *rec,
                        uint64_t *clk) {
  if (n_items == 0) return hipSuccess;
  hipLaunchKernelGGL(k_small, dim3(n_items), dim3(256), 0, st, n_items, (const uint32_t *)dig, key_bytes, key_off,
                     item_msg, item_key, (const uint32_t *)r_be, (const uint32_t *)s_be, pre, kc_tabs, g_table,
                     status, stamps, rec, clk);
  return hipGetLastError();
}

hipError_t verify_deferred(hipStream_t st, uint64_t n, uint32_t *list, const uint32_t *item_key,
                           const uint32_t *r_be, const uint32_t *s_be, const uint8_t *pre, const uint8_t *kst,
                           const uint32_t *kxy, const uint32_t *item_msg, const uint32_t *dig, const uint32_t *w,
                           const uint32_t *g_table, uint8_t *status, uint64_t *bits) {
  if (n == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(list + n, 0, 4, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_defer_list, grid1(n, 256), dim3(256), 0, st, n, status, list);
  hipLaunchKernelGGL(k_verify_deferred, dim3((unsigned)std::min<uint64_t>(1024, (n + 63) / 64)), dim3(64), 0, st, n,
                     list, item_key, r_be, s_be, pre, kst, kxy, item_msg, dig, w, g_table, status, bits);
  return hipGetLastError();
}

hipError_t verify_generic(hipStream_t st, uint64_t n, uint64_t lo, uint64_t hi, const uint32_t *item_key,
                          const uint32_t *r_be, const uint32_t *s_be, const uint8_t *pre, const uint8_t *kst,
                          const uint32_t *kxy, const uint32_t *item_msg, const uint32_t *dig, const uint32_t *w,
                          const uint32_t *g_table, uint8_t *status, uint64_t *bits) {
  if (hi <= lo) return hipSuccess;
  if (n <= BV_GEN_LAT_MAX_ITEMS)
    hipLaunchKernelGGL(k_verify_generic<true>, grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key, r_be, s_be,
                       pre, kst, kxy, item_msg, dig, w, g_table, status, bits);
  else
    hipLaunchKernelGGL(k_verify_generic<false>, grid1(hi - lo, 256), dim3(256), 0, st, n, lo, hi, item_key, r_be,
                       s_be, pre, kst, kxy, item_msg, dig, w, g_table, status, bits);
  return hipGetLastError();
}

}  // namespace bvk
