// sha256.h — FIPS 180-4 SHA-256 on gfx950, one message per lane.
//
// Replaces crypto.SHA256 (src/crypto/hash.go:8-13) as used by
// EventBody.Hash (event.go:58-64), BlockBody.Hash (block.go:49-55) and
// InternalTransactionBody.Hash (internal_transaction.go:59-65).
// Message bytes are read as aligned dwords and re-aligned in registers with
// v_alignbyte (byte offsets of canonical JSON bodies are arbitrary); the
// device buffer is padded so the over-read of the last dword is in bounds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __host__ __device__ __forceinline__

static constexpr uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

DEV uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// a ^ b ^ c in one v_bitop3_b32 (truth table 0x96) on gfx950; the compiler
// does not fuse the xor pairs of the Sigma / sigma functions by itself.
DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}
// Maj(a, b, c) in one v_bitop3_b32 (truth table 0xE8); left to itself the
// compiler emits xor + and + bitop3 (three VALU) per round.
DEV uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
#else
  return (a & b) ^ (a & c) ^ (b & c);
#endif
}
DEV uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
// bytes sh..sh+3 of the little-endian pair (lo, hi) (v_alignbyte_b32 on gfx950)
DEV uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) {
  return (uint32_t)(((uint64_t)hi << 32 | lo) >> (8 * sh));
}

// bswap32(alignbyte(hi, lo, sh)): the big-endian word of bytes sh..sh+3 of
// the little-endian pair (lo, hi), one v_perm_b32 on gfx950 (selector
// 0x00010203 + sh * 0x01010101: out byte 3 - k = pair byte sh + k).
DEV uint32_t be_word_at(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(hi, lo, 0x00010203u + sh * 0x01010101u);
#else
  return bswap32(alignbyte(hi, lo, sh));
#endif
}

DEV void sha256_compress(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t t1 = hh + xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25)) + ((e & f) ^ (~e & g)) + SHA_K[i] + wi;
    uint32_t t2 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22)) + maj3(a, b, c);
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

DEV void sha256_init(uint32_t h[8]) {
  h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}

DEV uint64_t sha256_nblocks(uint64_t len) { return (len + 9 + 63) / 64; }

// 17 aligned dwords of a full data block (the realignment reads one past):
// 4 dwordx4 loads at dword alignment (gfx950 global loads need not be
// 16-byte aligned): a quarter of the load instructions, and each lane
// touches a cache line once per load instead of four times
DEV void sha256_load17(uint32_t d[17], const uint32_t *src) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
  const u32x4a4 *v = (const u32x4a4 *)src;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const u32x4a4 x = v[i];
    d[4 * i] = x.x;
    d[4 * i + 1] = x.y;
    d[4 * i + 2] = x.z;
    d[4 * i + 3] = x.w;
  }
  d[16] = src[16];
#else
#pragma unroll
  for (int i = 0; i < 17; i++) d[i] = src[i];
#endif
}

// The 16 big-endian message words of block `blk` of a len-byte message
// (FIPS padding and length included).  `src0` is the 4-byte aligned dword
// holding message byte 64 blk0, `sh` that byte's offset within it; the
// buffer is padded by >= 8 bytes past the message end (the realignment
// over-reads one dword).
DEV void sha256_block_words(uint32_t w[16], const uint32_t *src0, uint32_t sh, uint64_t len, uint64_t blk0,
                            uint64_t blk) {
  const uint64_t p0 = blk * 64;  // byte position of this block in the message
  if (p0 + 64 <= len) {
    // full data block: 17 aligned dwords, realigned
    uint32_t d[17];
    sha256_load17(d, src0 + (blk - blk0) * 16);
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = be_word_at(d[i + 1], d[i], sh);
    return;
  }
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint64_t p = p0 + 4 * i;
    uint32_t x = 0;
    if (p < len) {
      const uint32_t *src = src0 + ((p - blk0 * 64) >> 2);
      x = alignbyte(src[1], src[0], sh);  // LE word of bytes p..p+3
      const uint64_t rem = len - p;        // bytes of message left
      if (rem < 4) {
        const uint32_t keep = (uint32_t)rem * 8u;
        x = (x & ((1u << keep) - 1u)) | (0x80u << keep);
      }
    } else if (p == len) {
      x = 0x80u;
    }
    w[i] = bswap32(x);
  }
  if (blk == sha256_nblocks(len) - 1) {
    const uint64_t bitlen = len * 8;
    w[14] = (uint32_t)(bitlen >> 32);
    w[15] = (uint32_t)bitlen;
  }
}

// Compress blocks [blk0, blk1) of a len-byte message into h (see
// sha256_block_words for src0 / sh).
DEV void sha256_blocks(uint32_t h[8], const uint32_t *src0, uint32_t sh, uint64_t len, uint64_t blk0,
                       uint64_t blk1) {
  for (uint64_t blk = blk0; blk < blk1; blk++) {
    uint32_t w[16];
    sha256_block_words(w, src0, sh, len, blk0, blk);
    sha256_compress(h, w);
  }
}

// SHA-256 of bytes [off, off+len) of `base` (a 4-byte aligned buffer padded
// by >= 8 bytes past its end).  Output: the 8 state words h[0..7] (digest =
// big-endian serialisation of h).
DEV void sha256_msg(uint32_t h[8], const uint8_t *base, uint64_t off, uint64_t len) {
  sha256_init(h);
  sha256_blocks(h, (const uint32_t *)(base + (off & ~(uint64_t)3)), (uint32_t)(off & 3), len, 0,
                sha256_nblocks(len));
}
