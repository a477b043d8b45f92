// Host emulation of the device pipeline — TEST INFRASTRUCTURE ONLY.
//
// Compiles babble_amd/csrc/verify_core.h (the exact per-unit source the
// gfx950 kernels run) for the host and replays kernels.hip's grid mapping
// serially, so tests can check index logic and arithmetic on the CPU (and
// under AddressSanitizer, tests/emu/Makefile `asan`) before a GPU run.
// Not linked into libbabbleverify.so; the product never runs this.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <functional>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../babble_amd/csrc/evjson.h"
#include "../../babble_amd/csrc/hostdag.h"
#include "../../babble_amd/csrc/hostsha.h"
#include "../../babble_amd/csrc/verify_core.h"

namespace {

template <class F>
void parallel_for(uint64_t n, int nt, F f) {
  if (nt < 1) nt = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < nt; t++)
    th.emplace_back([=]() {
      for (uint64_t i = t; i < n; i += nt) f(i);
    });
  for (auto &x : th) x.join();
}

// k_table_bases + k_table_fill<w, nwin, phi, block>: one (b, window, chunk)
// block per task; the block's prefix/suffix scans run serially.
void emu_fill(uint32_t n_bases, const uint8_t *bstatus, const uint32_t *bases, int w, uint32_t nwin, bool phi,
              uint32_t block, uint32_t *table, int nt) {
  const uint32_t chunks = (1u << w) / block;
  const uint64_t half_u32 = (uint64_t)nwin * (1ull << w) * BV_ENTRY_U32;
  parallel_for((uint64_t)n_bases * nwin * chunks, nt, [&](uint64_t task) {
    const uint32_t b = (uint32_t)(task / ((uint64_t)nwin * chunks));
    const uint32_t jc = (uint32_t)(task % ((uint64_t)nwin * chunks));
    const uint32_t j = jc / chunks, c = jc % chunks;
    if (bstatus && bstatus[b] != KS_OK) return;
    // as the kernel: the Jacobian base's (X, Y) on the isomorphic curve
    // y^2 = x^3 + 7 Z^6, entries' Z scaled by the base's Z
    fe bx, by, bz;
    const uint32_t *bj = bases + ((uint64_t)b * nwin + j) * 24;
    fe_load(bx, bj);
    fe_load(by, bj + 8);
    fe_load(bz, bj + 16);
    std::vector<gej> R(block);
    std::vector<fe> Z(block), pre(block), suf(block);
    std::vector<char> inf(block);
    for (uint32_t t = 0; t < block; t++) {
      bool f;
      table_point(R[t], f, Z[t], bx, by, c * block + t, w);
      if (!f) fe_mul(Z[t], Z[t], bz);
      inf[t] = f;
    }
    pre[0] = Z[0];
    for (uint32_t t = 1; t < block; t++) fe_mul(pre[t], pre[t - 1], Z[t]);
    suf[block - 1] = Z[block - 1];
    for (int t = (int)block - 2; t >= 0; t--) fe_mul(suf[t], suf[t + 1], Z[t]);
    fe inv;
    fe_inv_var(inv, pre[block - 1]);
    for (uint32_t t = 0; t < block; t++) {
      fe zi = inv;
      if (t > 0) fe_mul(zi, zi, pre[t - 1]);
      if (t < block - 1) fe_mul(zi, zi, suf[t + 1]);
      const uint32_t d = c * block + t;
      uint32_t *entry = table + (uint64_t)b * (phi ? 2 : 1) * half_u32 + (((uint64_t)j << w) + d) * BV_ENTRY_U32;
      table_store(entry, phi ? entry + half_u32 : nullptr, d, R[t], inf[t] != 0, zi);
    }
  });
}

void emu_bases(uint32_t n_bases, const uint32_t *bxy, const uint8_t *bstatus, std::vector<uint32_t> &bases, int w,
               uint32_t nwin, int nt) {
  bases.assign((size_t)n_bases * nwin * 24, 0);
  parallel_for(n_bases, nt, [&](uint64_t b) {
    if (bstatus && bstatus[b] != KS_OK) return;
    table_bases_one((uint32_t)b, bxy, bases.data(), w, nwin);
  });
}

// One chunk of chord-sum entries d in [d0, d0 + n) of a window (k_table_pair
// / k_table_pair_g): one batched inversion, then pair_store.
void emu_pair_chunk(const uint32_t *s_lo, const uint32_t *s_hi, uint32_t L, uint32_t d0, uint32_t n, uint32_t *base,
                    uint64_t phi_off, uint32_t zero_as = 0) {
  const uint32_t NS = 1u << L;
  std::vector<fe> H(n), pre(n);
  fe acc;
  fe_set(acc, 1);
  for (uint32_t k = 0; k < n; k++) {
    const uint32_t d = zero_as ? k12_digit(d0 + k, zero_as) : d0 + k;
    fe x1, y1, x2, y2;
    pair_load(s_lo, s_hi, d & (NS - 1), d >> L, x1, y1, x2, y2);
    pair_denominator(H[k], pair_kind(d & (NS - 1), d >> L), x1, x2);
    pre[k] = acc;
    fe_mul(acc, acc, H[k]);
  }
  fe q;
  fe_inv_var(q, acc);
  for (int k = (int)n - 1; k >= 0; k--) {
    const uint32_t d = zero_as ? k12_digit(d0 + k, zero_as) : d0 + k;
    fe x1, y1, x2, y2, Hinv;
    pair_load(s_lo, s_hi, d & (NS - 1), d >> L, x1, y1, x2, y2);
    fe_mul(Hinv, q, pre[k]);
    fe_mul(q, q, H[k]);
    uint32_t *entry = base + (uint64_t)d * BV_ENTRY_U32;
    pair_store(entry, phi_off ? entry + phi_off : nullptr, pair_kind(d & (NS - 1), d >> L), x1, y1, x2, y2, Hinv);
  }
}

// kw = 0: generator table (11-bit sub-tables, then k_table_pair_g's chunks
// of 4096 entries); 8: K8 key tables; 12: K12 key tables (sub-tables, then
// k_table_pair's one block per window).
void emu_build_tables(int kw, uint32_t n_bases, const uint32_t *bxy, const uint8_t *bstatus, uint32_t *table,
                      int nt) {
  std::vector<uint32_t> bases;
  if (kw == 8) {  // 4-bit sub-tables, then k_table_pair_u's chord sums (one block per window and key)
    emu_bases(n_bases, bxy, bstatus, bases, BV_KL, BV_KNSUB, nt);
    std::vector<uint32_t> sub((size_t)n_bases * BV_KSUB_U32 + 16);
    emu_fill(n_bases, bstatus, bases.data(), BV_KL, BV_KNSUB, false, 1u << BV_KL, sub.data(), nt);
    constexpr uint32_t NS = 1u << BV_KL;
    parallel_for((uint64_t)n_bases * BV_KNWIN, nt, [&](uint64_t task) {
      const uint32_t b = (uint32_t)(task / BV_KNWIN), j = (uint32_t)(task % BV_KNWIN);
      if (bstatus && bstatus[b] != KS_OK) return;
      const uint32_t *s_lo = sub.data() + ((uint64_t)b * BV_KNSUB + 2 * j) * NS * BV_ENTRY_U32;
      uint32_t *base = table + (uint64_t)b * BV_KTABLE_U32 + ((uint64_t)j << BV_KW) * BV_ENTRY_U32;
      emu_pair_chunk(s_lo, s_lo + NS * BV_ENTRY_U32, BV_KL, 0, 1u << BV_KW, base, BV_KHALF_U32);
    });
    return;
  }
  if (kw == 0) {
    emu_bases(1, bxy, nullptr, bases, BV_GL, BV_GNSUB, nt);
    std::vector<uint32_t> sub(BV_GSUB_U32 + 16);
    emu_fill(1, nullptr, bases.data(), BV_GL, BV_GNSUB, false, 256, sub.data(), nt);
    const uint32_t NS = 1u << BV_GL;
    for (uint32_t j = 0; j < BV_GNWIN; j++) {
      const int live_bits = 256 - BV_GW * (int)j;
      const uint64_t live = live_bits >= BV_GW - 1 ? BV_GENT : (1ull << live_bits) + 1;
      const uint32_t *s_lo = sub.data() + (uint64_t)(2 * j) * NS * BV_ENTRY_U32, *s_hi = s_lo + NS * BV_ENTRY_U32;
      uint32_t *base = table + (uint64_t)j * BV_GENT * BV_ENTRY_U32;
      parallel_for((live + 4095) / 4096, nt, [&](uint64_t c) {
        emu_pair_chunk(s_lo, s_hi, BV_GL, (uint32_t)(c * 4096), 4096, base, 0, BV_GENT);
      });
    }
    return;
  }
  constexpr uint32_t W = BV_K12W, L = BV_K12L, NWIN = BV_K12NWIN, NS = 1u << L;
  emu_bases(n_bases, bxy, bstatus, bases, L, BV_K12NSUB, nt);
  std::vector<uint32_t> sub((size_t)n_bases * BV_K12SUB_U32 + 16);
  emu_fill(n_bases, bstatus, bases.data(), L, BV_K12NSUB, false, NS, sub.data(), nt);
  const uint64_t half_u32 = BV_K12HALF_U32;
  // k_table_pair: one block per (window, key); the top window stops after
  // its live digits.  Entry order within the block does not change results.
  parallel_for((uint64_t)n_bases * NWIN, nt, [&](uint64_t task) {
    const uint32_t b = (uint32_t)(task / NWIN), j = (uint32_t)(task % NWIN);
    if (bstatus && bstatus[b] != KS_OK) return;
    const int live_bits = 128 - (int)(W * j);
    const uint32_t n_live =
        live_bits >= (int)W - 1 ? BV_K12ENT : (((1u << live_bits) + 1u + 255u) / 256u) * 256u;
    const uint32_t *s_lo = sub.data() + ((uint64_t)b * 2 * NWIN + 2 * j) * NS * BV_ENTRY_U32;
    const uint32_t *s_hi = s_lo + NS * BV_ENTRY_U32;
    uint32_t *base = table + (uint64_t)b * 2 * half_u32 + (uint64_t)j * BV_K12ENT * BV_ENTRY_U32;
    emu_pair_chunk(s_lo, s_hi, L, 0, n_live, base, half_u32, BV_K12ENT);
  });
}

// The generator table is a constant: built once per process (like bv_create).
const uint32_t *emu_g_table(int nt) {
  static std::vector<uint8_t> store;
  static uint32_t *gt = nullptr;
  static std::once_flag once;
  std::call_once(once, [&]() {
    store.assign(BV_GTABLE_U32 * 4 + 64, 0);
    gt = (uint32_t *)(((uintptr_t)store.data() + 15) & ~(uintptr_t)15);
    alignas(16) static const uint32_t G[16] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                                               0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu,
                                               0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                                               0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
    emu_build_tables(0, 1, G, nullptr, gt, nt);
  });
  return gt;
}

// k_small's per-item steps (kernels.hip) run one after another: the same
// verify_core.h / point.h pieces the workgroup's waves run concurrently
// (s^-1, key decode, decision table, u1 / u2 + GLV, the 10 G leaves and
// their sum tree — affine pairs, then XYZZ sums — the NAF chains of k1 Q and
// k2 phi(Q), the root sums and the final check).  The digest is SHA-256 of
// the message (the library hashes small batches on the host).  The key
// cache's table leaves are exercised on the GPU.
namespace {
void tree_sum(std::vector<gexz> &n, std::vector<bool> &inf) {
  while (n.size() > 1) {  // node i <- node 2i + node 2i+1, an odd last node moves up alone
    std::vector<gexz> m;
    std::vector<bool> mi;
    for (size_t i = 0; i < n.size(); i += 2) {
      gexz a = n[i];
      bool ia = inf[i];
      if (i + 1 < n.size()) gexz_add_lat(a, ia, n[i + 1], inf[i + 1]);
      m.push_back(a);
      mi.push_back(ia);
    }
    n.swap(m);
    inf.swap(mi);
  }
}
}  // namespace

uint8_t small_item(uint64_t i, const bv_batch *b, const uint8_t *msg, const uint32_t *r, const uint32_t *s,
                   const uint32_t *gt) {
  const uint32_t m = b->item_msg[i], k = b->item_key[i];
  uint32_t h[8], e_words[8];
  sha256_msg(h, msg, b->msg_off[m], b->msg_off[m + 1] - b->msg_off[m]);
  for (int c = 0; c < 8; c++) e_words[c] = bswap32(h[c]);
  sc sv, w;
  sc_load_be_words(sv, s + 8 * i);
  if (s_usable(b->pre, i, sv)) sinv_one(w, sv);
  else for (int c = 0; c < 8; c++) w.v[c] = 0;
  uint8_t ks;
  fe qx, qy;
  key_decode_point(b->key_bytes, b->key_off[k], b->key_off[k + 1] - b->key_off[k], ks, qx, qy);
  fe rf, sf;
  fe_load_be_words(rf, r + 8 * i);
  fe_load_be_words(sf, s + 8 * i);
  const uint8_t cls = classify(b->pre ? b->pre[i] : 0, ks, rf, sf);
  if (cls != 0xFF) return cls;
  sc e, rs;
  sc_load_be_words(e, e_words);
  for (int c = 0; c < 8; c++) rs.v[c] = rf.v[c];
  uint32_t u1[8], k1[4], k2[4], signs;
  scalars_from(w, e, rs, u1, k1, k2, signs);
  fe lx[BV_GNWIN], ly[BV_GNWIN];
  bool lz[BV_GNWIN];
  for (int j = 0; j < BV_GNWIN; j++) {
    uint32_t u[8];
    for (int c = 0; c < 8; c++) u[c] = u1[c];
    table_leaf<BV_GW, 8>(lx[j], ly[j], lz[j], gt, u, j, false, false);
  }
  std::vector<gexz> nodes;
  std::vector<bool> ninf;
  for (int j = 0; j < BV_GNWIN; j += 2) {
    gexz R;
    bool inf;
    const bool last = j + 1 >= BV_GNWIN;
    gexz_sum_ge_lat(R, inf, lx[j], ly[j], lz[j], last ? lx[j] : lx[j + 1], last ? ly[j] : ly[j + 1],
                    last ? true : lz[j + 1]);
    nodes.push_back(R);
    ninf.push_back(inf);
  }
  tree_sum(nodes, ninf);  // the G sum
  // the cold path (no key-cache table) in k_small's order: the doubling
  // chain 2^i Q in XYZZ; half 1 (wave 3) starts from the G sum and adds
  // +-phi(2^i Q), half 0 (wave 1) +-2^i Q, each over its non-zero NAF digits
  // in increasing i (the kernel's phases only decide WHEN, never the order);
  // then half 0 + half 1
  uint32_t pm[2][5], nm[2][5];
  naf_masks(k1, pm[0], nm[0]);
  naf_masks(k2, pm[1], nm[1]);
  gexz acc[2];
  bool ai[2] = {true, true};
  acc[1] = nodes[0];
  ai[1] = ninf[0];
  fe beta;
  fe_load(beta, FE_BETA);
  gexz P;
  P.X = qx, P.Y = qy;
  for (int c = 0; c < 8; c++) P.ZZ.v[c] = P.ZZZ.v[c] = c == 0 ? 1u : 0u;
  for (uint32_t bit = 0; bit < 130; bit++) {
    if (bit) {
      gexz D;
      gexz_double(D, P);
      P = D;
    }
    for (int hh = 0; hh < 2; hh++) {
      const uint32_t p = (pm[hh][bit >> 5] >> (bit & 31)) & 1u, n = (nm[hh][bit >> 5] >> (bit & 31)) & 1u;
      if (!(p | n)) continue;
      gexz T = P;
      if (hh) fe_mul(T.X, T.X, beta);
      if ((n != 0) != (((signs >> hh) & 1u) != 0)) fe_neg(T.Y, T.Y);
      gexz_add_lat(acc[hh], ai[hh], T, false);
    }
  }
  gexz_add_lat(acc[0], ai[0], acc[1], ai[1]);  // k1 Q + (u1 G + k2 phi(Q))
  return final_check(acc[0], ai[0], rf) ? BV_ACCEPT : BV_REJECT;
}

template <class T>
T *aligned(std::vector<uint8_t> &store, size_t bytes) {
  store.assign(bytes + 64, 0);
  uintptr_t p = ((uintptr_t)store.data() + 15) & ~(uintptr_t)15;
  return (T *)p;
}

}  // namespace

extern "C" {

// Same pipeline and mode choice as bv_api.cpp run_device, on the host.
// force_mode: -1 = same rule as the library, 0 = generic, 1 = K8 tables,
// 2 = K12 tables, 3 = the small-batch kernel's steps (k_small).  Returns the
// mode used.
int emu_verify_batch(const bv_batch *b, uint8_t *msg_hash, uint8_t *status, uint64_t *bits, int n_threads,
                     int force_mode) {
  const uint64_t n_msgs = b->n_msgs, n_items = b->n_items;
  const uint32_t n_keys = b->n_keys;
  // device-style aligned + padded copies of the inputs
  std::vector<uint8_t> s_msg, s_dig, s_kst, s_kxy, s_r, s_s, s_scr, s_u12, s_kt;
  const uint64_t msg_len = n_msgs ? b->msg_off[n_msgs] : 0;
  uint8_t *msg = aligned<uint8_t>(s_msg, msg_len + 64);
  if (msg_len) memcpy(msg, b->msg_bytes, msg_len);
  uint32_t *dig = aligned<uint32_t>(s_dig, (n_msgs + 1) * 32);
  uint8_t *kst = aligned<uint8_t>(s_kst, n_keys + 1);
  uint32_t *kxy = aligned<uint32_t>(s_kxy, (n_keys + 1) * 64ull);
  uint32_t *r = aligned<uint32_t>(s_r, n_items * 32 + 32);
  uint32_t *s = aligned<uint32_t>(s_s, n_items * 32 + 32);
  if (n_items) {
    memcpy(r, b->r_be, n_items * 32);
    memcpy(s, b->s_be, n_items * 32);
  }
  uint32_t *scratch = aligned<uint32_t>(s_scr, n_items * 32 + 32);
  uint32_t *u12 = aligned<uint32_t>(s_u12, n_items * BV_U_STRIDE * 4 + 64);
  parallel_for(n_msgs, n_threads, [&](uint64_t m) { sha256_one(m, msg, b->msg_off, dig); });
  for (uint32_t k = 0; k < n_keys; k++) key_decode_one(k, b->key_bytes, b->key_off, kst, kxy);
  // force_mode 5 / 6: K8 / K12 with the key part first (verify_item_qfirst,
  // then verify_item_gfinish), as the host entries run them; returns 1 / 2
  const bool qfirst = force_mode == 5 || force_mode == 6;
  int mode = qfirst ? force_mode - 4 : force_mode;
  if (mode < 0) {
    mode = (n_keys <= 8192 && n_items >= 16ull * n_keys) ? 1 : 0;
    if (mode == 1 && n_keys <= 1024 && n_items >= 2048ull * n_keys) mode = 2;
  }
  const bool table_mode = mode == 1 || mode == 2;
  const uint32_t *gt = emu_g_table(n_threads);
  uint32_t *kt = nullptr;
  if (table_mode) {
    const uint64_t per_key = mode == 2 ? BV_K12TABLE_U32 : BV_KTABLE_U32;
    kt = aligned<uint32_t>(s_kt, (uint64_t)(n_keys ? n_keys : 1) * per_key * 4);
    emu_build_tables(mode == 2 ? 12 : 8, n_keys, kxy, kst, kt, n_threads);
  }
  std::vector<uint8_t> s_rg;
  uint32_t *rg = table_mode ? aligned<uint32_t>(s_rg, (n_items + 1) * RG_WORDS * 4) : nullptr;
  const uint32_t M = 16;
  const uint64_t T = ((n_items + M - 1) / M + 255) / 256 * 256;  // kernel grid size
  parallel_for(T, n_threads, [&](uint64_t t) { sinv_thread(t, T, n_items, M, s, b->pre, scratch); });
  std::vector<uint8_t> st(n_items + 1);
  if (mode == 3) {
    parallel_for(n_items, n_threads, [&](uint64_t i) { st[i] = small_item(i, b, msg, r, s, gt); });
  } else if (table_mode && qfirst) {
    parallel_for(n_items, n_threads, [&](uint64_t i) {
      if (mode == 2)
        verify_item_qfirst<BV_K12W, BV_K12NWIN>(i, n_items, b->item_key, r, s, b->pre, kst, scratch, kt, nullptr, rg);
      else
        verify_item_qfirst<BV_KW, BV_KNWIN>(i, n_items, b->item_key, r, s, b->pre, kst, scratch, kt, nullptr, rg);
    });
    parallel_for(n_items, n_threads, [&](uint64_t i) {
      st[i] = verify_item_gfinish(i, n_items, b->item_key, r, s, b->pre, kst, b->item_msg, dig, scratch, gt, rg);
    });
  } else if (table_mode) {
    parallel_for(n_items, n_threads,
                 [&](uint64_t i) {
                   verify_item_g(i, n_items, b->item_key, r, s, b->pre, kst, b->item_msg, dig, scratch, u12, gt, rg);
                 });
    parallel_for(n_items, n_threads, [&](uint64_t i) {
      st[i] = mode == 2 ? verify_item_q<BV_K12W, BV_K12NWIN>(i, n_items, b->item_key, r, s, b->pre, kst, u12, kt, nullptr, rg)
                        : verify_item_q<BV_KW, BV_KNWIN>(i, n_items, b->item_key, r, s, b->pre, kst, u12, kt, nullptr, rg);
    });
  } else {
    parallel_for(n_items, n_threads, [&](uint64_t i) {
      st[i] = verify_item_generic(i, b->item_key, r, s, b->pre, kst, kxy, b->item_msg, dig, scratch, gt);
    });
  }
  if (msg_hash && n_msgs) memcpy(msg_hash, dig, n_msgs * 32);
  if (status && n_items) memcpy(status, st.data(), n_items);
  if (bits) {
    const uint64_t nw = (n_items + 63) / 64;
    memset(bits, 0, nw * 8);
    for (uint64_t i = 0; i < n_items; i++)
      if (st[i] == BV_ACCEPT) bits[i / 64] |= 1ull << (i % 64);
  }
  return mode;
}

// The product's host DAG hasher (hostdag.cpp) over a batch: levels and order
// as bv_events.cpp computes them; `threads` > 1 runs the parallel steps on
// that many threads; `portable` selects the portable SHA-256 compressor.
void emu_host_dag_hash(const bv_event_batch *b, uint8_t *digests, int threads, int portable) {
  const uint64_t n = b->n_events;
  std::vector<uint32_t> level(n, 0), order(n), level_off;
  uint32_t nl = 1;
  for (uint64_t e = 0; e < n; e++) {
    uint32_t l = 0;
    for (int p = 0; p < 2; p++)
      if (b->parent_kind[2 * e + p] == BV_PARENT_EVENT) l = std::max(l, level[b->parent_ref[2 * e + p]] + 1);
    level[e] = l;
    nl = std::max(nl, l + 1);
  }
  level_off.assign(nl + 1, 0);
  for (uint64_t e = 0; e < n; e++) level_off[level[e] + 1]++;
  for (uint32_t l = 0; l < nl; l++) level_off[l + 1] += level_off[l];
  std::vector<uint32_t> fill(level_off.begin(), level_off.end() - 1);
  for (uint64_t e = 0; e < n; e++) order[fill[level[e]]++] = (uint32_t)e;
  const HostParFor pf = [threads](uint64_t cnt, uint64_t grain, const std::function<void(uint64_t, uint64_t)> &fn) {
    if (threads <= 1 || cnt <= grain) return fn(0, cnt);
    std::vector<std::thread> th;
    std::atomic<uint64_t> next{0};
    for (int t = 0; t < threads; t++)
      th.emplace_back([&]() {
        for (uint64_t lo; (lo = next.fetch_add(grain)) < cnt;) fn(lo, std::min(cnt, lo + grain));
      });
    for (auto &x : th) x.join();
  };
  hsha::force_portable(portable != 0);
  HostDagScratch w;
  bv_host_dag_hash(*b, order.data(), level_off.data(), nl, pf, w, digests);
  hsha::force_portable(false);
}

void emu_host_sha256(const uint8_t *msg, uint64_t len, uint8_t *out, int portable) {
  hsha::force_portable(portable != 0);
  hsha::digest(msg, len, out);
  hsha::force_portable(false);
}

int emu_host_sha_accelerated() { return hsha::accelerated(); }

// bv_verify_events' body construction (the device kernels' per-event code,
// evjson.h) and hashing (sha256.h), in event order (parents precede
// children): the in-batch parents' hex spliced in once their digests exist.
// bodies: sum of lengths + 64 bytes; offs: n + 1; digests: 32 * n.  Returns
// the total body bytes.
uint64_t emu_ev_bodies(const bv_event_batch *b, uint8_t *bodies, uint64_t cap, uint64_t *offs, uint8_t *digests) {
  const uint64_t n = b->n_events;
  std::vector<uint32_t> ppos(2 * n);
  offs[0] = 0;
  for (uint64_t e = 0; e < n; e++) offs[e + 1] = offs[e] + evj_len(*b, e, &ppos[2 * e]);
  if (offs[n] + 64 > cap) return 0;
  memset(bodies + offs[n], 0, 64);
  for (uint64_t e = 0; e < n; e++) evj_write(*b, e, bodies + offs[e]);
  for (uint64_t e = 0; e < n; e++) {
    for (int p = 0; p < 2; p++)
      if (ppos[2 * e + p] != EVJ_NOPOS) evj_hex32(bodies + offs[e] + ppos[2 * e + p], digests + 32 * b->parent_ref[2 * e + p]);
    uint32_t h[8];
    sha256_msg(h, bodies, offs[e], offs[e + 1] - offs[e]);
    for (int k = 0; k < 32; k++) digests[32 * e + k] = (uint8_t)(h[k / 4] >> (24 - 8 * (k % 4)));
  }
  return offs[n];
}

// k_ev_body_hash: each body serialised straight into the streaming SHA-256
// sink (batches without in-batch parents); digests[n, 32].
void emu_ev_body_hash(const bv_event_batch *b, uint8_t *digests) {
  for (uint64_t e = 0; e < b->n_events; e++) {
    uint32_t row[25];
    EvjSha o = evj_sha_begin(row);
    evj_emit(*b, e, o);
    uint32_t be[8];
    evj_sha_finish(o, be);
    memcpy(digests + 32 * e, be, 32);
  }
}

void emu_sc_inverse(const uint32_t s_le[8], uint32_t out_le[8]) {
  sc s, sM, R2, inv, one, r;
  for (int i = 0; i < 8; i++) s.v[i] = s_le[i];
  sc_load_const(R2, SC_R2);
  sc_mont(sM, s, R2);
  sc_inverse(inv, sM);
  for (int i = 0; i < 8; i++) one.v[i] = i == 0;
  sc_mont(r, inv, one);
  for (int i = 0; i < 8; i++) out_le[i] = r.v[i];
}

// the same through the variable-time divsteps inversion (modinv.h)
void emu_sc_inverse_var(const uint32_t s_le[8], uint32_t out_le[8]) {
  sc s, sM, R2, inv, one, r;
  for (int i = 0; i < 8; i++) s.v[i] = s_le[i];
  sc_load_const(R2, SC_R2);
  sc_mont(sM, s, R2);
  sc_inverse_var(inv, sM);
  for (int i = 0; i < 8; i++) one.v[i] = i == 0;
  sc_mont(r, inv, one);
  for (int i = 0; i < 8; i++) out_le[i] = r.v[i];
}

// GLV split of k (< N): magnitudes |k1|, |k2| (4 limbs each) and signs
void emu_glv_split(const uint32_t k_le[8], uint32_t out[9]) {
  sc k;
  for (int i = 0; i < 8; i++) k.v[i] = k_le[i];
  uint32_t signs;
  glv_split(out, out + 4, signs, k);
  out[8] = signs;
}

// a * b mod p, canonical (field arithmetic known-answer tests)
void emu_fe_mul(const uint32_t a[8], const uint32_t b[8], uint32_t out[8]) {
  fe x, y, z;
  for (int i = 0; i < 8; i++) {
    x.v[i] = a[i];
    y.v[i] = b[i];
  }
  fe_mul(z, x, y);
  fe_canon(z);
  for (int i = 0; i < 8; i++) out[i] = z.v[i];
}
void emu_fe_sqr(const uint32_t a[8], uint32_t out[8]) {
  fe x, z;
  for (int i = 0; i < 8; i++) x.v[i] = a[i];
  fe_sqr(z, x);
  fe_canon(z);
  for (int i = 0; i < 8; i++) out[i] = z.v[i];
}
void emu_fe_add(const uint32_t a[8], const uint32_t b[8], uint32_t out[8]) {
  fe x, y, z;
  for (int i = 0; i < 8; i++) {
    x.v[i] = a[i];
    y.v[i] = b[i];
  }
  fe_add(z, x, y);
  fe_canon(z);
  for (int i = 0; i < 8; i++) out[i] = z.v[i];
}
void emu_fe_sub(const uint32_t a[8], const uint32_t b[8], uint32_t out[8]) {
  fe x, y, z;
  for (int i = 0; i < 8; i++) {
    x.v[i] = a[i];
    y.v[i] = b[i];
  }
  fe_sub(z, x, y);
  fe_canon(z);
  for (int i = 0; i < 8; i++) out[i] = z.v[i];
}
void emu_fe_inv(const uint32_t a[8], uint32_t out[8]) {
  fe x, z;
  for (int i = 0; i < 8; i++) x.v[i] = a[i];
  fe_inv(z, x);
  fe_canon(z);
  for (int i = 0; i < 8; i++) out[i] = z.v[i];
}
void emu_fe_inv_var(const uint32_t a[8], uint32_t out[8]) {
  fe x, z;
  for (int i = 0; i < 8; i++) x.v[i] = a[i];
  fe_inv_var(z, x);
  fe_canon(z);
  for (int i = 0; i < 8; i++) out[i] = z.v[i];
}
// a * b * R^-1 mod N
void emu_sc_mont(const uint32_t a[8], const uint32_t b[8], uint32_t out[8]) {
  sc x, y, z;
  for (int i = 0; i < 8; i++) {
    x.v[i] = a[i];
    y.v[i] = b[i];
  }
  sc_mont(z, x, y);
  for (int i = 0; i < 8; i++) out[i] = z.v[i];
}

}  // extern "C"
