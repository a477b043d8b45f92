// hostscalar.cpp — the item record of a latency batch (hostscalar.h):
// the scalar half of ecdsa.Verify on the host with field.h's own functions.
// Plain clang, no offload (field.h's device-only assembly is behind
// __HIP_DEVICE_COMPILE__; the host bodies are the portable ones).
#include "hostscalar.h"

#include <string.h>

#include "field.h"

namespace {
void load_be(sc &r, const uint8_t b[32]) {
  for (int i = 0; i < 8; i++) {
    const uint8_t *p = b + 4 * (7 - i);
    r.v[i] = (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
  }
}
bool is_zero(const sc &a) {
  uint32_t z = 0;
  for (int i = 0; i < 8; i++) z |= a.v[i];
  return z == 0;
}
}  // namespace

void bv_host_item_record(uint32_t rec[hrec::kWords], const uint8_t digest[32], const uint8_t r_be[32],
                         const uint8_t s_be[32], uint8_t pre, const uint8_t *key, uint64_t key_len, uint64_t table) {
  memset(rec, 0, hrec::kWords * 4);
  const uint64_t kl = key_len > 65 ? 66 : key_len;  // (a longer key is malformed by its length alone)
  if (kl == 65) memcpy(rec + hrec::kKey, key, 65);
  rec[hrec::kKeyLen] = (uint32_t)kl;
  rec[hrec::kPre] = pre;
  memcpy(rec + hrec::kR, r_be, 32);
  memcpy(rec + hrec::kS, s_be, 32);
  memcpy(rec + hrec::kTab, &table, 8);
  sc e, r, s;
  load_be(e, digest);
  load_be(r, r_be);
  load_be(s, s_be);
  if (pre != 0 || is_zero(s) || sc_ge_n(s)) return;  // verify_core.h s_usable
  // as k_small: w = s^-1 (plain), eR = e R, rR = r R (e, r < 2^256 = R
  // unreduced), u1 = eR w R^-1 = e w, u2 = r w, then the GLV split of u2
  sc w, R2, eR, rR, u1, u2;
  modinfo30 mi;
  modinfo_n(mi);
  modinv_var(w.v, s.v, mi);
  sc_load_const(R2, SC_R2);
  sc_mont(eR, e, R2);
  sc_mont(rR, r, R2);
  sc_mont(u1, eR, w);
  sc_mont(u2, rR, w);
  uint32_t k1[4], k2[4], signs;
  glv_split(k1, k2, signs, u2);
  memcpy(rec + hrec::kU1, u1.v, 32);
  memcpy(rec + hrec::kK, k1, 16);
  memcpy(rec + hrec::kK + 4, k2, 16);
  rec[hrec::kSigns] = signs;
}
