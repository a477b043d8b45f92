// hostscalar.cpp — the item records of a latency batch (hostscalar.h):
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
// verify_core.h s_usable
bool usable(const HostRecItem &it, sc &s) {
  load_be(s, it.s);
  return it.pre == 0 && !is_zero(s) && !sc_ge_n(s);
}
void fill_fields(uint32_t rec[hrec::kWords], const HostRecItem &it) {
  memset(rec, 0, hrec::kWords * 4);
  const uint64_t kl = it.key_len > 65 ? 66 : it.key_len;  // (a longer key is malformed by its length alone)
  if (kl == 65) memcpy(rec + hrec::kKey, it.key, 65);
  rec[hrec::kKeyLen] = (uint32_t)kl;
  rec[hrec::kPre] = it.pre;
  memcpy(rec + hrec::kR, it.r, 32);
  memcpy(rec + hrec::kS, it.s, 32);
  memcpy(rec + hrec::kTab, &it.table, 8);
}
// u1 = e w / R, u2 = r w / R for w = s^-1 R (Montgomery form; e, r < 2^256
// = R unreduced, w < N), then the GLV split of u2
void put_scalars(uint32_t rec[hrec::kWords], const HostRecItem &it, const sc &w) {
  sc e, r, u1, u2;
  load_be(e, it.digest);
  load_be(r, it.r);
  sc_mont(u1, e, w);
  sc_mont(u2, r, w);
  uint32_t k1[4], k2[4], signs;
  glv_split(k1, k2, signs, u2);
  memcpy(rec + hrec::kU1, u1.v, 32);
  memcpy(rec + hrec::kK, k1, 16);
  memcpy(rec + hrec::kK + 4, k2, 16);
  rec[hrec::kSigns] = signs;
}
}  // namespace

void bv_host_item_records(uint32_t *recs, const HostRecItem *items, uint64_t n) {
  if (n == 0) return;
  // Montgomery's trick over the usable items, as k_sinv does per lane: the
  // prefix products of s R, ONE inversion (modinv.h's divsteps), then the
  // walk back gives every w = s^-1 R
  constexpr uint64_t kMax = 64;
  sc sR[kMax], pfx[kMax], s, R2, acc, inv;
  bool ok[kMax];
  sc_load_const(R2, SC_R2);
  for (uint64_t lo = 0; lo < n; lo += kMax) {
    const uint64_t m = n - lo < kMax ? n - lo : kMax;
    sc_load_const(acc, SC_R1);  // R: the Montgomery one
    for (uint64_t k = 0; k < m; k++) {
      const HostRecItem &it = items[lo + k];
      fill_fields(recs + hrec::kWords * (lo + k), it);
      ok[k] = usable(it, s);
      pfx[k] = acc;
      if (!ok[k]) continue;  // (scalars stay zero: the kernel's decision table rejects the item first)
      sc_mont(sR[k], s, R2);
      sc_mont(acc, acc, sR[k]);
    }
    sc_inverse_var(inv, acc);  // (prod s)^-1 R
    for (uint64_t k = m; k-- > 0;) {
      if (!ok[k]) continue;
      sc w;
      sc_mont(w, inv, pfx[k]);   // s_k^-1 R
      sc_mont(inv, inv, sR[k]);  // (prod_{< k} s)^-1 R
      put_scalars(recs + hrec::kWords * (lo + k), items[lo + k], w);
    }
  }
}
