// hostsha.cpp — host SHA-256 (hostsha.h).  Two compressors: the x86 SHA
// extensions (sha256rnds2 does two rounds, sha256msg1/msg2 the message
// schedule, four words at a time) and a portable one; the choice is made once
// per process from CPUID.
#include "hostsha.h"

#include <immintrin.h>
#include <string.h>

#include <atomic>

namespace {

alignas(16) const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void compress_portable(uint32_t h[8], const uint8_t *p, size_t nblocks) {
  for (; nblocks--; p += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
      w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
      const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 64; i++) {
      const uint32_t t1 = k + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      k = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
    h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e, h[5] += f, h[6] += g, h[7] += k;
  }
}

// The state lives as ABEF / CDGH register pairs (the layout sha256rnds2
// works on); message words are byte-swapped on load.
__attribute__((target("sha,sse4.1,ssse3"))) void compress_shani(uint32_t h[8], const uint8_t *p, size_t nblocks) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *)&h[0]), 0xB1);  // CDAB
  __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *)&h[4]), 0x1B);  // EFGH
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                          // ABEF
  s1 = _mm_blend_epi16(s1, t, 0xF0);                                               // CDGH
  for (; nblocks--; p += 64) {
    const __m128i abef = s0, cdgh = s1;
    __m128i w[4];
    // 16 groups of 4 rounds; w[i & 3] holds message words 4i .. 4i+3
#define HSHA_RND4(i)                                                                                         \
  {                                                                                                          \
    if ((i) < 4)                                                                                             \
      w[(i) & 3] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 16 * (i))), bswap);                \
    else                                                                                                     \
      w[(i) & 3] = _mm_sha256msg2_epu32(                                                                     \
          _mm_add_epi32(_mm_sha256msg1_epu32(w[(i) & 3], w[((i) + 1) & 3]),                                  \
                        _mm_alignr_epi8(w[((i) + 3) & 3], w[((i) + 2) & 3], 4)),                             \
          w[((i) + 3) & 3]);                                                                                 \
    const __m128i m = _mm_add_epi32(w[(i) & 3], _mm_load_si128((const __m128i *)&K[4 * (i)]));              \
    s1 = _mm_sha256rnds2_epu32(s1, s0, m);                                                                   \
    s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(m, 0x0E));                                          \
  }
    HSHA_RND4(0) HSHA_RND4(1) HSHA_RND4(2) HSHA_RND4(3) HSHA_RND4(4) HSHA_RND4(5) HSHA_RND4(6) HSHA_RND4(7)
    HSHA_RND4(8) HSHA_RND4(9) HSHA_RND4(10) HSHA_RND4(11) HSHA_RND4(12) HSHA_RND4(13) HSHA_RND4(14) HSHA_RND4(15)
#undef HSHA_RND4
    s0 = _mm_add_epi32(s0, abef);
    s1 = _mm_add_epi32(s1, cdgh);
  }
  t = _mm_shuffle_epi32(s0, 0x1B);                                     // FEBA
  s1 = _mm_shuffle_epi32(s1, 0xB1);                                    // DCHG
  _mm_storeu_si128((__m128i *)&h[0], _mm_blend_epi16(t, s1, 0xF0));   // DCBA
  _mm_storeu_si128((__m128i *)&h[4], _mm_alignr_epi8(s1, t, 8));      // HGFE
}

// Two independent single-block compressions, their rounds interleaved: the
// sha256rnds2 chain of one block is latency-bound, so a second message's
// rounds fill the gaps (the serial DAG levels of a SyncResponse hash their
// 2-3 events this way, hostdag.cpp).
__attribute__((target("sha,sse4.1,ssse3"))) void compress2_shani(uint32_t ha[8], const uint8_t *pa, uint32_t hb[8],
                                                                 const uint8_t *pb) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i ta = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *)&ha[0]), 0xB1);
  __m128i a1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *)&ha[4]), 0x1B);
  __m128i a0 = _mm_alignr_epi8(ta, a1, 8);
  a1 = _mm_blend_epi16(a1, ta, 0xF0);
  __m128i tb = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *)&hb[0]), 0xB1);
  __m128i b1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *)&hb[4]), 0x1B);
  __m128i b0 = _mm_alignr_epi8(tb, b1, 8);
  b1 = _mm_blend_epi16(b1, tb, 0xF0);
  const __m128i abef_a = a0, cdgh_a = a1, abef_b = b0, cdgh_b = b1;
  __m128i wa[4], wb[4];
#define HSHA_SCHED(w, p, i)                                                                                  \
  if ((i) < 4)                                                                                               \
    w[(i) & 3] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)((p) + 16 * (i))), bswap);               \
  else                                                                                                       \
    w[(i) & 3] = _mm_sha256msg2_epu32(_mm_add_epi32(_mm_sha256msg1_epu32(w[(i) & 3], w[((i) + 1) & 3]),    \
                                                    _mm_alignr_epi8(w[((i) + 3) & 3], w[((i) + 2) & 3], 4)), \
                                      w[((i) + 3) & 3]);
#define HSHA_RND4X2(i)                                                                 \
  {                                                                                    \
    HSHA_SCHED(wa, pa, i)                                                              \
    HSHA_SCHED(wb, pb, i)                                                              \
    const __m128i k = _mm_load_si128((const __m128i *)&K[4 * (i)]);                   \
    const __m128i ma = _mm_add_epi32(wa[(i) & 3], k), mb = _mm_add_epi32(wb[(i) & 3], k); \
    a1 = _mm_sha256rnds2_epu32(a1, a0, ma);                                            \
    b1 = _mm_sha256rnds2_epu32(b1, b0, mb);                                            \
    a0 = _mm_sha256rnds2_epu32(a0, a1, _mm_shuffle_epi32(ma, 0x0E));                   \
    b0 = _mm_sha256rnds2_epu32(b0, b1, _mm_shuffle_epi32(mb, 0x0E));                   \
  }
  HSHA_RND4X2(0) HSHA_RND4X2(1) HSHA_RND4X2(2) HSHA_RND4X2(3) HSHA_RND4X2(4) HSHA_RND4X2(5) HSHA_RND4X2(6)
  HSHA_RND4X2(7) HSHA_RND4X2(8) HSHA_RND4X2(9) HSHA_RND4X2(10) HSHA_RND4X2(11) HSHA_RND4X2(12) HSHA_RND4X2(13)
  HSHA_RND4X2(14) HSHA_RND4X2(15)
#undef HSHA_RND4X2
#undef HSHA_SCHED
  a0 = _mm_add_epi32(a0, abef_a);
  a1 = _mm_add_epi32(a1, cdgh_a);
  b0 = _mm_add_epi32(b0, abef_b);
  b1 = _mm_add_epi32(b1, cdgh_b);
  ta = _mm_shuffle_epi32(a0, 0x1B);
  a1 = _mm_shuffle_epi32(a1, 0xB1);
  _mm_storeu_si128((__m128i *)&ha[0], _mm_blend_epi16(ta, a1, 0xF0));
  _mm_storeu_si128((__m128i *)&ha[4], _mm_alignr_epi8(a1, ta, 8));
  tb = _mm_shuffle_epi32(b0, 0x1B);
  b1 = _mm_shuffle_epi32(b1, 0xB1);
  _mm_storeu_si128((__m128i *)&hb[0], _mm_blend_epi16(tb, b1, 0xF0));
  _mm_storeu_si128((__m128i *)&hb[4], _mm_alignr_epi8(b1, tb, 8));
}

bool cpu_has_sha() {
  __builtin_cpu_init();
  return __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
}
const bool kHasSha = cpu_has_sha();
std::atomic<bool> g_portable{false};

}  // namespace

namespace hsha {

void init(uint32_t h[8]) {
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(h, iv, sizeof iv);
}

int accelerated() { return kHasSha && !g_portable.load(std::memory_order_relaxed); }
void force_portable(bool on) { g_portable.store(on); }

void compress(uint32_t h[8], const uint8_t *blocks, size_t nblocks) {
  if (accelerated())
    compress_shani(h, blocks, nblocks);
  else
    compress_portable(h, blocks, nblocks);
}

void finish(uint32_t h[8], const uint8_t *msg, size_t from, size_t len, uint8_t out[32]) {
  const size_t whole = (len - from) / 64;
  compress(h, msg + from, whole);
  const size_t rest = len - from - whole * 64;
  uint8_t tail[128] = {0};
  memcpy(tail, msg + from + whole * 64, rest);
  tail[rest] = 0x80;
  const size_t tb = rest + 9 <= 64 ? 1 : 2;
  const uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) tail[tb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
  compress(h, tail, tb);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h[i] >> 8);
    out[4 * i + 3] = (uint8_t)h[i];
  }
}

namespace {
// The blocks still to compress for one message after `from`: its whole data
// blocks in place, then the FIPS tail (padding and length) in `tail`.
struct Pending {
  const uint8_t *msg;
  size_t whole, nb;  // whole data blocks, all blocks
  uint8_t tail[128];
  void set(const uint8_t *m, size_t from, size_t len) {
    msg = m + from;
    whole = (len - from) / 64;
    const size_t rest = len - from - whole * 64;
    memset(tail, 0, sizeof tail);
    memcpy(tail, msg + whole * 64, rest);
    tail[rest] = 0x80;
    const size_t tb = rest + 9 <= 64 ? 1 : 2;
    const uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; i++) tail[tb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    nb = whole + tb;
  }
  const uint8_t *block(size_t j) const { return j < whole ? msg + 64 * j : tail + 64 * (j - whole); }
};

void put_digest(const uint32_t h[8], uint8_t out[32]) {
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h[i] >> 8);
    out[4 * i + 3] = (uint8_t)h[i];
  }
}
}  // namespace

void finish2(uint32_t ha[8], const uint8_t *ma, size_t from_a, size_t len_a, uint8_t out_a[32], uint32_t hb[8],
             const uint8_t *mb, size_t from_b, size_t len_b, uint8_t out_b[32]) {
  if (!accelerated()) {
    finish(ha, ma, from_a, len_a, out_a);
    finish(hb, mb, from_b, len_b, out_b);
    return;
  }
  Pending a, b;
  a.set(ma, from_a, len_a);
  b.set(mb, from_b, len_b);
  const size_t both = a.nb < b.nb ? a.nb : b.nb;
  for (size_t j = 0; j < both; j++) compress2_shani(ha, a.block(j), hb, b.block(j));
  for (size_t j = both; j < a.nb; j++) compress_shani(ha, a.block(j), 1);
  for (size_t j = both; j < b.nb; j++) compress_shani(hb, b.block(j), 1);
  put_digest(ha, out_a);
  put_digest(hb, out_b);
}

void digest(const uint8_t *msg, size_t len, uint8_t out[32]) {
  uint32_t h[8];
  init(h);
  finish(h, msg, 0, len, out);
}

}  // namespace hsha
