// hostparse.cpp — host helpers of the C ABI that mirror the Go parsing the
// reference performs before the math (no device involved).
//
//   bv_decode_signature  keys.DecodeSignature (src/crypto/keys/signature.go:31-39):
//                        strings.Split(sig, "|") must give exactly 2 parts;
//                        each part goes through big.Int.SetString(part, 36)
//                        (Go 1.13 math/big: optional single '+'/'-', digits
//                        0-9a-zA-Z, no '_' for base 36, at least one digit,
//                        whole string consumed; failure -> nil, error ignored),
//                        then classified for ecdsa.Verify's r.Sign() <= 0 /
//                        r.Cmp(N) >= 0 checks.
//   bv_hex_decode        common.DecodeFromString (src/common/hex.go:15-17):
//                        hex.DecodeString(s[2:]) returning the bytes decoded
//                        before the first error (Babble ignores the error,
//                        src/peers/peer.go:51-54); len(s) < 2 panics in Go.
#include <cstdint>
#include <cstring>

#include "../../include/babbleverify.h"

namespace {

const uint32_t kN[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                        0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

// digit value of a byte in base 36 (0-9, a-z, A-Z), 0xFF otherwise
struct Digits36 {
  uint8_t v[256];
  constexpr Digits36() : v() {
    for (int c = 0; c < 256; c++) v[c] = 0xFF;
    for (int c = '0'; c <= '9'; c++) v[c] = (uint8_t)(c - '0');
    for (int c = 'a'; c <= 'z'; c++) v[c] = (uint8_t)(c - 'a' + 10);
    for (int c = 'A'; c <= 'Z'; c++) v[c] = (uint8_t)(c - 'A' + 10);
  }
};
constexpr Digits36 kDigit36;

// Parse one base-36 part.  Returns the class; for BV_SC_OK writes 32 BE bytes.
// Up to 12 digits at a time are gathered into one word (36^12 < 2^63) and
// folded into a 320-bit accumulator with one 64 x 64 -> 128-bit product per
// limb (the Go shim decodes every event's signature on the host: ~10x fewer
// operations than a 32-bit limb pass per digit).
uint8_t parse36(const char *s, size_t len, uint8_t out[32]) {
  memset(out, 0, 32);
  if (len == 0) return BV_SC_NIL;  // scanSign hits EOF
  size_t i = 0;
  bool neg = false;
  if (s[0] == '-') {
    neg = true;
    i = 1;
  } else if (s[0] == '+') {
    i = 1;
  }
  uint64_t v[5] = {0, 0, 0, 0, 0};  // 320-bit accumulator
  bool big = false;                 // value >= 2^320 (certainly >= N)
  const size_t first = i;
  while (i < len) {
    uint64_t chunk = 0, scale = 1;
    size_t k = 0;
    for (; k < 12 && i < len; k++, i++) {
      const uint8_t d = kDigit36.v[(unsigned char)s[i]];
      if (d == 0xFF) break;
      chunk = chunk * 36u + d;
      scale *= 36u;
    }
    if (k && !big) {  // v = v * 36^k + chunk
      unsigned __int128 carry = chunk;
      for (int j = 0; j < 5; j++) {
        const unsigned __int128 t = (unsigned __int128)v[j] * scale + carry;
        v[j] = (uint64_t)t;
        carry = t >> 64;
      }
      if (carry) big = true;
    }
    if (k < 12 && i < len) break;  // a byte that is not a digit
  }
  if (i == first) return BV_SC_NIL;  // errNoDigits
  if (i != len) return BV_SC_NIL;    // trailing garbage: not fully consumed
  bool zero = !big;
  for (int k = 0; k < 5 && zero; k++) zero = v[k] == 0;
  if (zero) return BV_SC_NONPOS;     // "-0" and "0" are 0
  if (neg) return BV_SC_NONPOS;
  if (big || v[4] != 0) return BV_SC_GE_N;
  uint32_t w32[8];
  for (int k = 0; k < 4; k++) w32[2 * k] = (uint32_t)v[k], w32[2 * k + 1] = (uint32_t)(v[k] >> 32);
  // compare with N
  bool ge = true;
  for (int k = 7; k >= 0; k--) {
    if (w32[k] != kN[k]) {
      ge = w32[k] > kN[k];
      break;
    }
  }
  if (ge) return BV_SC_GE_N;
  for (int k = 0; k < 8; k++) {
    const uint32_t w = w32[7 - k];
    out[4 * k] = (uint8_t)(w >> 24);
    out[4 * k + 1] = (uint8_t)(w >> 16);
    out[4 * k + 2] = (uint8_t)(w >> 8);
    out[4 * k + 3] = (uint8_t)w;
  }
  return BV_SC_OK;
}

int from_hex(unsigned char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

}  // namespace

extern "C" uint8_t bv_decode_signature(const char *sig, size_t len, uint8_t r_be[32], uint8_t s_be[32]) {
  memset(r_be, 0, 32);
  memset(s_be, 0, 32);
  size_t bar = (size_t)-1;
  int parts = 1;
  for (size_t i = 0; i < len; i++)
    if (sig[i] == '|') {
      parts++;
      if (bar == (size_t)-1) bar = i;
    }
  if (parts != 2) return BV_PRE_PARTS_BAD;
  const uint8_t rc = parse36(sig, bar, r_be);
  const uint8_t sc = parse36(sig + bar + 1, len - bar - 1, s_be);
  return BV_PRE(rc, sc);
}

extern "C" int64_t bv_hex_decode(const char *s, size_t len, uint8_t *out) {
  if (len < 2) return -1;
  const char *src = s + 2;
  const size_t n = len - 2;
  int64_t k = 0;
  for (size_t i = 0; i < n / 2; i++) {
    const int a = from_hex((unsigned char)src[2 * i]);
    if (a < 0) return k;
    const int b = from_hex((unsigned char)src[2 * i + 1]);
    if (b < 0) return k;
    out[k++] = (uint8_t)((a << 4) | b);
  }
  return k;
}
