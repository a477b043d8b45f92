// geometry.h — fixed-base table geometry shared by the kernels (verify_core.h)
// and the host driver (bv_api.cpp).
//
// Fixed-base tables: T[j][d] = d * 2^(W j) * P (affine, 64 bytes), d < 2^W.
//
// Generator table: a constant, built once per process and device with wide
// SIGNED-digit windows over the 256-bit u1, sized for the GPU's 288 GB of
// HBM: 26-bit windows x 10 (260 bits >= 257 for the signed recoding; digits
// in (-2^25, 2^25], y negated for negative digits) = 2^25 entries per window,
// 21.5 GB, so u1 G costs 9 mixed additions (the first window lands on the
// identity) and no doublings.  Entries are chord sums of two 13-bit
// sub-table points S_k[x] = x 2^(13 k) G; the digit 2^25 of window j lives
// in the never-read slot 0 of window j+1 (one pad entry after the top
// window), as in the K12 / KC key tables.  The host emulator (tests/emu, test
// infrastructure) overrides BV_GW/BV_GNWIN/BV_GL/BV_GNSUB with smaller
// geometries (host memory); the code paths are the same templates.
// Key tables are built per batch over 128 bits only: u2 is split GLV-style
// (u2 = k1 + k2 lambda, |k1|, |k2| < 2^128) and the second half of a key
// table holds phi(T) = (beta x, y), so the serial doubling chain per key
// covers 128 bits instead of 256.  Two key-table geometries:
//   K8:  8-bit windows x 16 (+ phi) = 512 KiB per key, 32 adds per item;
//        entries by per-thread double-and-add (mid-size batches);
//   K12: 12-bit signed-digit windows x 11 (+ phi) = 2.75 MiB per key, 22
//        adds per item; digits |d| <= 2^11, so a window holds 2^11 entries
//        (entry 2^11 of window j lives in the never-read slot 0 of window
//        j+1; one pad entry after the top window); entries as chord sums of
//        two 6-bit sub-table points with one batched inversion per window
//        (large batches: ~16k items per key).
#pragma once

#define BV_ENTRY_U32 16  // affine x, y = 16 words (64 bytes)
#ifndef BV_GW
#define BV_GW 26         // G window bits (signed digits)
#define BV_GNWIN 10      //   x 10 windows (260 bits) x 2^25 entries = 21.5 GB
#define BV_GL 13         // G sub-table bits: S_k[x] = x 2^(13k) G, x < 8192
#define BV_GNSUB 20      //   k < 20
#endif
#define BV_GENT (1u << (BV_GW - 1))  // entry slots per G window
#define BV_GTABLE_U32 (((uint64_t)BV_GNWIN * BV_GENT + 1) * BV_ENTRY_U32)
#define BV_GSUB_U32 ((uint64_t)BV_GNSUB * (1ull << BV_GL) * BV_ENTRY_U32)
#define BV_GPAIR_BLOCKS 1024  // k_table_pair_g blocks per launch (4096 entries each)
#define BV_KW 8          // K8 window bits
#define BV_KNWIN 16      //   x 16 windows (128 bits) x 256 entries
#define BV_KHALF_U32 ((uint64_t)BV_KNWIN * (1ull << BV_KW) * BV_ENTRY_U32)
#define BV_KTABLE_U32 (2 * BV_KHALF_U32)
#define BV_KL 4          // K8 sub-table bits: S_k[x] = x 2^(4k) Q, x < 16
#define BV_KNSUB 32      //   k < 32; entry (j, d) = S_2j[d mod 16] + S_2j+1[d / 16]
#define BV_KSUB_U32 ((uint64_t)BV_KNSUB * (1ull << BV_KL) * BV_ENTRY_U32)
#define BV_K12W 12       // K12 window bits
#define BV_K12NWIN 11    //   x 11 windows (132 bits; the top one holds 8)
#define BV_K12L 6        // K12 sub-table bits: S_k[x] = x 2^(6k) Q, x < 64
#define BV_K12NSUB 22    //   k < 22 (offsets 0, 6, ..., 126)
#define BV_K12ENT (1u << (BV_K12W - 1))  // entry slots per window (signed digits)
#define BV_K12HALF_U32 (((uint64_t)BV_K12NWIN * BV_K12ENT + 1) * BV_ENTRY_U32)
#define BV_K12TABLE_U32 (2 * BV_K12HALF_U32)
#define BV_K12SUB_U32 ((uint64_t)BV_K12NSUB * (1ull << BV_K12L) * BV_ENTRY_U32)
// KC: the key-cache geometry (BV_F_KEY_CACHE).  Validator sets are stable
// (peers/peer_set.go), so a key's table is built once and kept in HBM across
// calls; the build cost is amortised and the windows can be wide: 22-bit
// signed-digit windows x 6 (132 bits >= 129) = 12 adds per item for u2 Q
// (K12: 22).  Only the k1 half is stored; the k2 half's entries are
// phi(T) = (beta x, y), formed in k_verify_q with one multiply per lookup
// (12 adds + 6 multiplies instead of the 14 adds of 20-bit windows with a
// stored phi half): 805 MB per key (64 keys: 52 GB, 100 validators: 81 GB
// of the GPU's 288 GB).  Entries are chord sums of two 11-bit sub-table
// points S_k[x] = x 2^(11 k) Q, k < 12, same scheme as the generator table.
#define BV_KCW 22
#define BV_KCNWIN 6
#define BV_KCL 11
#define BV_KCNSUB 12
#define BV_KCENT (1u << (BV_KCW - 1))
#define BV_KCHALF_U32 (((uint64_t)BV_KCNWIN * BV_KCENT + 1) * BV_ENTRY_U32)
#define BV_KCTABLE_U32 BV_KCHALF_U32  // no stored phi half
#define BV_KCSUB_U32 ((uint64_t)BV_KCNSUB * (1ull << BV_KCL) * BV_ENTRY_U32)
#define BV_KCPAIR_ENT 4096  // entries per k_table_pair_kc block (16 per thread)
// per-item GLV halves of u2 (k_verify_g -> k_verify_q): k1[4] | k2[4] | signs | pad
#define BV_U_STRIDE 12
