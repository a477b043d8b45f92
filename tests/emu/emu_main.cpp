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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/babbleverify.h"

extern "C" {
int emu_verify_batch(const bv_batch *b, uint8_t *msg_hash, uint8_t *status, uint64_t *bits, int n_threads,
                     int force_mode);
int oracle_verify_batch(const bv_batch *b, uint8_t *msg_hash, uint8_t *status, uint64_t *accept_bits,
                        int n_threads);
void oracle_init(void);
}

namespace {

template <class T>
bool rd(FILE *f, std::vector<T> &v, uint64_t n) {
  v.resize(n ? n : 1);
  return n == 0 || fread(v.data(), sizeof(T), n, f) == n;
}

}  // namespace

int main(int argc, char **argv) {
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
  for (int mode = 0; mode <= 2; mode++) {
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
