// Sanitizer driver for the host emulation — TEST INFRASTRUCTURE ONLY.
//
// Built by `make -C tests/emu asan` as a host-only executable with
// AddressSanitizer + UBSan (the device code is never built with sanitizers).
// Reads a bv_batch dumped by tests/emu/emu.py:dump_batch, runs the emulated
// pipeline (emu.cpp: the same verify_core.h per-unit code the gfx950 kernels
// run) in every key-table mode, and compares digests, statuses and accept
// bits with the C oracle (oracle/oracle.c).  Exit 0 = all equal and no
// sanitizer report; any mismatch exits 1, a sanitizer finding aborts.
//
// File format (little-endian): magic "BVB1", then u64 n_msgs, n_keys, n_items,
// msg_len, key_len, has_pre; then msg_off[n_msgs+1] u64, msg_bytes,
// key_off[n_keys+1] u64, key_bytes, item_msg u32[n], item_key u32[n],
// r_be[32n], s_be[32n], pre[n] (if has_pre).
//
// `emu_asan dag <seed> [n]`: a random event wire batch (keys of 0 / 33 / 65 /
// 70 bytes, nil and empty transaction lists, nil transactions, ITX and
// BlockSignature fragments, no / known-hash / in-batch parents) in
// exactly-sized heap buffers; the product's host DAG hasher (hostdag.cpp,
// hostsha.cpp) on 1 and 4 threads and with the portable compressor must give
// the digests of the plain in-order build (emu_ev_bodies).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/babbleverify.h"

extern "C" {
int emu_verify_batch(const bv_batch *b, uint8_t *msg_hash, uint8_t *status, uint64_t *bits, int n_threads,
                     int force_mode);
int oracle_verify_batch(const bv_batch *b, uint8_t *msg_hash, uint8_t *status, uint64_t *accept_bits,
                        int n_threads);
void oracle_init(void);
void emu_host_dag_hash(const bv_event_batch *b, uint8_t *digests, int threads, int portable);
uint64_t emu_ev_bodies(const bv_event_batch *b, uint8_t *bodies, uint64_t cap, uint64_t *offs, uint8_t *digests);
}

namespace {

template <class T>
bool rd(FILE *f, std::vector<T> &v, uint64_t n) {
  v.resize(n ? n : 1);
  return n == 0 || fread(v.data(), sizeof(T), n, f) == n;
}

struct Rng {
  uint64_t x;
  uint64_t next() {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    return x;
  }
  uint64_t below(uint64_t n) { return next() % n; }
};

// every array in its own exactly-sized heap block (ASan sees any over-read)
template <class T>
T *exact(const std::vector<T> &v, std::vector<std::unique_ptr<char[]>> &keep) {
  if (v.empty()) return nullptr;
  keep.emplace_back(new char[v.size() * sizeof(T)]);
  memcpy(keep.back().get(), v.data(), v.size() * sizeof(T));
  return (T *)keep.back().get();
}

int dag_main(uint64_t seed, uint64_t n) {
  Rng r{seed * 0x9E3779B97F4A7C15ull + 1};
  std::vector<uint64_t> key_off{0};
  std::vector<uint8_t> keys;
  const int lens[4] = {0, 33, 65, 70};
  for (int k = 0; k < 6; k++) {
    const int L = lens[r.below(4)];
    for (int i = 0; i < L; i++) keys.push_back((uint8_t)r.next());
    key_off.push_back(keys.size());
  }
  std::vector<uint32_t> creator(n);
  std::vector<int64_t> index(n), ts(n);
  std::vector<uint8_t> pkind(2 * n), tx_list_nil(n), tx_nil, tx_bytes, phash, itx, bsig;
  std::vector<uint64_t> pref(2 * n), tx_start{0}, tx_off{0}, itx_off{0}, bsig_off{0};
  for (uint64_t e = 0; e < n; e++) {
    creator[e] = (uint32_t)r.below(6);
    index[e] = (int64_t)r.next() >> r.below(64);
    ts[e] = (int64_t)r.next() >> r.below(64);
    for (int p = 0; p < 2; p++) {
      const uint64_t c = r.below(10);
      if (c < 2 || e == 0) {
        pkind[2 * e + p] = BV_PARENT_NONE;
      } else if (c < 5) {
        pkind[2 * e + p] = BV_PARENT_HASH;
        pref[2 * e + p] = phash.size() / 32;
        for (int i = 0; i < 32; i++) phash.push_back((uint8_t)r.next());
      } else {
        pkind[2 * e + p] = BV_PARENT_EVENT;
        pref[2 * e + p] = e - 1 - r.below(e < 8 ? e : 8);
      }
    }
    tx_list_nil[e] = r.below(8) == 0;
    const uint64_t ntx = tx_list_nil[e] ? 0 : r.below(4);
    for (uint64_t t = 0; t < ntx; t++) {
      tx_nil.push_back(r.below(10) == 0);
      const uint64_t L = r.below(200);
      for (uint64_t i = 0; i < L; i++) tx_bytes.push_back((uint8_t)r.next());
      tx_off.push_back(tx_bytes.size());
    }
    tx_start.push_back(tx_off.size() - 1);
    const uint64_t il = r.below(6) == 0 ? 1 + r.below(90) : 0, bl = r.below(6) == 0 ? 1 + r.below(90) : 0;
    for (uint64_t i = 0; i < il; i++) itx.push_back((uint8_t)(' ' + r.below(90)));
    for (uint64_t i = 0; i < bl; i++) bsig.push_back((uint8_t)(' ' + r.below(90)));
    itx_off.push_back(itx.size());
    bsig_off.push_back(bsig.size());
  }
  std::vector<std::unique_ptr<char[]>> keep;
  bv_event_batch b{};
  b.n_events = n;
  b.n_keys = 6;
  b.key_bytes = exact(keys, keep);
  b.key_off = exact(key_off, keep);
  b.creator = exact(creator, keep);
  b.index = exact(index, keep);
  b.timestamp = exact(ts, keep);
  b.parent_kind = exact(pkind, keep);
  b.parent_ref = exact(pref, keep);
  b.n_parent_hashes = phash.size() / 32;
  b.parent_hashes = exact(phash, keep);
  b.tx_start = exact(tx_start, keep);
  b.tx_off = exact(tx_off, keep);
  b.tx_bytes = exact(tx_bytes, keep);
  b.tx_list_nil = exact(tx_list_nil, keep);
  b.tx_nil = exact(tx_nil, keep);
  b.itx_off = exact(itx_off, keep);
  b.itx_json = exact(itx, keep);
  b.bsig_off = exact(bsig_off, keep);
  b.bsig_json = exact(bsig, keep);
  const uint64_t cap = 4096 * n + 4 * tx_bytes.size() + itx.size() + bsig.size() + 4096;
  std::vector<uint8_t> bodies(cap), want(32 * n), got(32 * n);
  std::vector<uint64_t> offs(n + 1);
  if (!emu_ev_bodies(&b, bodies.data(), cap, offs.data(), want.data())) return 2;
  int bad = 0;
  for (int threads : {1, 4})
    for (int portable : {0, 1}) {
      std::fill(got.begin(), got.end(), 0);
      emu_host_dag_hash(&b, got.data(), threads, portable);
      const bool eq = memcmp(got.data(), want.data(), 32 * n) == 0;
      printf("dag threads %d portable %d: %s (%llu events)\n", threads, portable, eq ? "equal" : "MISMATCH",
             (unsigned long long)n);
      bad += !eq;
    }
  return bad ? 1 : 0;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc >= 3 && strcmp(argv[1], "dag") == 0)
    return dag_main(strtoull(argv[2], nullptr, 10), argc > 3 ? strtoull(argv[3], nullptr, 10) : 700);
  if (argc < 2) {
    fprintf(stderr, "usage: %s batch.bin [threads]\n", argv[0]);
    return 2;
  }
  const int nt = argc > 2 ? atoi(argv[2]) : 4;
  FILE *f = fopen(argv[1], "rb");
  if (!f) {
    perror("open");
    return 2;
  }
  char magic[4];
  uint64_t hdr[6];
  if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "BVB1", 4) != 0 || fread(hdr, 8, 6, f) != 6) {
    fprintf(stderr, "bad header\n");
    return 2;
  }
  const uint64_t n_msgs = hdr[0], n_keys = hdr[1], n_items = hdr[2], msg_len = hdr[3], key_len = hdr[4];
  std::vector<uint64_t> msg_off, key_off;
  std::vector<uint8_t> msg, key, r, s, pre;
  std::vector<uint32_t> im, ik;
  bool ok = rd(f, msg_off, n_msgs + 1) && rd(f, msg, msg_len) && rd(f, key_off, n_keys + 1) &&
            rd(f, key, key_len) && rd(f, im, n_items) && rd(f, ik, n_items) && rd(f, r, 32 * n_items) &&
            rd(f, s, 32 * n_items) && (!hdr[5] || rd(f, pre, n_items));
  fclose(f);
  if (!ok) {
    fprintf(stderr, "short file\n");
    return 2;
  }
  bv_batch b{};
  b.n_msgs = n_msgs;
  b.msg_bytes = msg.data();
  b.msg_off = msg_off.data();
  b.n_keys = (uint32_t)n_keys;
  b.key_bytes = key.data();
  b.key_off = key_off.data();
  b.n_items = n_items;
  b.item_msg = im.data();
  b.item_key = ik.data();
  b.r_be = r.data();
  b.s_be = s.data();
  b.pre = hdr[5] ? pre.data() : nullptr;

  const uint64_t nw = (n_items + 63) / 64;
  std::vector<uint8_t> h0(32 * n_msgs + 1), st0(n_items + 1);
  std::vector<uint64_t> b0(nw + 1);
  oracle_init();
  oracle_verify_batch(&b, h0.data(), st0.data(), b0.data(), nt);

  int bad = 0;
  for (int mode = 0; mode <= 3; mode++) {
    std::vector<uint8_t> h(32 * n_msgs + 1), st(n_items + 1);
    std::vector<uint64_t> bits(nw + 1);
    const int m = emu_verify_batch(&b, h.data(), st.data(), bits.data(), nt, mode);
    const bool eq = m == mode && memcmp(h.data(), h0.data(), 32 * n_msgs) == 0 &&
                    memcmp(st.data(), st0.data(), n_items) == 0 && memcmp(bits.data(), b0.data(), 8 * nw) == 0;
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n_items; i++) acc += st[i] == BV_ACCEPT;
    printf("mode %d: %s (%llu items, %llu accepted)\n", mode, eq ? "equal" : "MISMATCH",
           (unsigned long long)n_items, (unsigned long long)acc);
    bad += !eq;
  }
  return bad ? 1 : 0;
}
