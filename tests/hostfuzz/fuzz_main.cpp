// fuzz_main.cpp — ASan/UBSan driver for the product's host-only C++ (test
// infrastructure only): hostparse.cpp (bv_decode_signature, bv_hex_decode —
// attacker-controlled text: processJoinRequest reaches it outside coreLock,
// node_rpc.go:250-260) and hostplan.cpp (bv_plan_shards, bv_plan_group,
// bv_merge_shard_bits).  Reads one case per line on stdin, writes one result
// line per case; tests/test_hostfuzz.py generates the cases and compares the
// results with oracle/gosemantics.py and babble_amd/shard.py.
//
//   S <hex bytes>                         -> S <pre> <r hex> <s hex>
//   H <hex bytes>                         -> H <n> <out hex>      (n = -1: Go panics)
//   G <D> <n_msgs> <item_msg,...|->       -> G <rc> <perm,...> <item bounds,...> <msg bounds,...>
//   M <words> <D> <bounds,...> <hex64,...> -> M <rc> <out hex64,...>
//
// Inputs are copied into exactly-sized heap buffers so any over-read is an
// ASan report (the process aborts and the test fails).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/babbleverify.h"
#include "../../babble_amd/csrc/hostscalar.h"

static std::vector<uint8_t> unhex(const std::string &h) {
  std::vector<uint8_t> out(h.size() / 2);
  for (size_t i = 0; i < out.size(); i++) out[i] = (uint8_t)std::stoul(h.substr(2 * i, 2), nullptr, 16);
  return out;
}

static std::string hex(const uint8_t *p, size_t n) {
  static const char H[] = "0123456789abcdef";
  std::string o;
  for (size_t i = 0; i < n; i++) o += H[p[i] >> 4], o += H[p[i] & 15];
  return o.empty() ? "-" : o;
}

template <class T>
static std::vector<T> csv(const std::string &s, int base = 10) {
  std::vector<T> v;
  if (s == "-") return v;
  std::stringstream ss(s);
  std::string t;
  while (std::getline(ss, t, ',')) v.push_back((T)std::stoull(t, nullptr, base));
  return v;
}

template <class T>
static std::string join(const T *p, size_t n) {
  std::string o;
  for (size_t i = 0; i < n; i++) o += (i ? "," : "") + std::to_string(p[i]);
  return o.empty() ? "-" : o;
}

// bv_host_item_records over the queued R lines, in batches of cycling sizes
// (1, 2, 7, 64, 65, 100: one inversion per 64 items inside), one output
// line per item in order: "R" and the record's 64 words
struct RItem {
  std::vector<uint8_t> d, r, s, key;
  uint8_t pre;
};
static std::vector<RItem> pending;
static void flush_records() {
  static const size_t sizes[] = {1, 2, 7, 64, 65, 100};
  size_t at = 0, c = 0;
  while (at < pending.size()) {
    const size_t n = std::min(sizes[c++ % 6], pending.size() - at);
    std::vector<std::unique_ptr<uint8_t[]>> keys;  // exact-size copies: an over-read aborts
    std::vector<HostRecItem> items(n);
    for (size_t k = 0; k < n; k++) {
      const RItem &p = pending[at + k];
      keys.emplace_back(new uint8_t[p.key.size() ? p.key.size() : 1]);
      if (!p.key.empty()) memcpy(keys.back().get(), p.key.data(), p.key.size());
      items[k] = {p.d.data(), p.r.data(), p.s.data(), keys.back().get(), p.key.size(), 0x1122334455667788ull, p.pre};
    }
    std::vector<uint32_t> recs(n * hrec::kWords);
    bv_host_item_records(recs.data(), items.data(), n);
    for (size_t k = 0; k < n; k++) {
      std::cout << "R";
      for (uint32_t w = 0; w < hrec::kWords; w++) {
        char t[12];
        snprintf(t, sizeof t, " %08x", recs[k * hrec::kWords + w]);
        std::cout << t;
      }
      std::cout << "\n";
    }
    at += n;
  }
  pending.clear();
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    std::stringstream in(line);
    std::string op;
    in >> op;
    if (op != "R") flush_records();
    if (op == "S" || op == "H") {
      std::string h;
      in >> h;
      if (h == "-") h.clear();
      const std::vector<uint8_t> raw = unhex(h);
      std::unique_ptr<char[]> buf(new char[raw.size() ? raw.size() : 1]);  // exact size: no terminator
      if (!raw.empty()) memcpy(buf.get(), raw.data(), raw.size());
      if (op == "S") {
        uint8_t r[32], s[32];
        const uint8_t pre = bv_decode_signature(buf.get(), raw.size(), r, s);
        std::cout << "S " << (int)pre << " " << hex(r, 32) << " " << hex(s, 32) << "\n";
      } else {
        std::unique_ptr<uint8_t[]> out(new uint8_t[raw.size() >= 2 ? (raw.size() - 2) / 2 + 1 : 1]);
        const int64_t n = bv_hex_decode(buf.get(), raw.size(), out.get());
        std::cout << "H " << n << " " << (n > 0 ? hex(out.get(), (size_t)n) : "-") << "\n";
      }
    } else if (op == "G") {
      int D;
      uint64_t n_msgs;
      std::string ims;
      in >> D >> n_msgs >> ims;
      const std::vector<uint32_t> im = csv<uint32_t>(ims);
      const size_t n = im.size();
      std::unique_ptr<uint32_t[]> item_msg(new uint32_t[n ? n : 1]), item_key(new uint32_t[n ? n : 1]);
      std::unique_ptr<uint8_t[]> r(new uint8_t[32 * n + 1]), s(new uint8_t[32 * n + 1]);
      for (size_t i = 0; i < n; i++) item_msg[i] = im[i], item_key[i] = 0;
      memset(r.get(), 0, 32 * n + 1);
      memset(s.get(), 0, 32 * n + 1);
      bv_batch b = {};
      b.n_msgs = n_msgs;
      b.n_items = n;
      b.item_msg = item_msg.get();
      b.item_key = item_key.get();
      b.r_be = r.get();
      b.s_be = s.get();
      std::unique_ptr<uint64_t[]> ib(new uint64_t[D + 1]), mb(new uint64_t[D + 1]);
      std::unique_ptr<uint32_t[]> perm(new uint32_t[n ? n : 1]);
      const int rc = bv_plan_group(&b, D, ib.get(), mb.get(), perm.get());
      std::cout << "G " << rc;
      if (rc >= 0) std::cout << " " << join(perm.get(), n) << " " << join(ib.get(), D + 1) << " " << join(mb.get(), D + 1);
      std::cout << "\n";
    } else if (op == "M") {
      uint64_t words;
      int D;
      std::string bs, gs;
      in >> words >> D >> bs >> gs;
      const std::vector<uint64_t> bounds = csv<uint64_t>(bs), g = csv<uint64_t>(gs, 16);
      std::unique_ptr<uint64_t[]> bd(new uint64_t[bounds.size()]), gathered(new uint64_t[g.size() ? g.size() : 1]);
      for (size_t i = 0; i < bounds.size(); i++) bd[i] = bounds[i];
      for (size_t i = 0; i < g.size(); i++) gathered[i] = g[i];
      const uint64_t W = (bounds.back() + 63) / 64;
      std::unique_ptr<uint64_t[]> out(new uint64_t[W ? W : 1]);
      const int rc = bv_merge_shard_bits(gathered.get(), words, D, bd.get(), out.get());
      std::cout << "M " << rc;
      if (rc == BV_OK) {
        std::cout << " ";
        for (uint64_t w = 0; w < W; w++) {
          char t[24];
          snprintf(t, sizeof t, "%s%llx", w ? "," : "", (unsigned long long)out[w]);
          std::cout << t;
        }
        if (!W) std::cout << "-";
      }
      std::cout << "\n";
    } else if (op == "R") {  // R <digest> <r> <s> <pre> <key|->: queued; run by the next flush
      std::string dh, rh, sh, kh;
      int pre;
      in >> dh >> rh >> sh >> pre >> kh;
      if (kh == "-") kh.clear();
      pending.push_back({unhex(dh), unhex(rh), unhex(sh), unhex(kh), (uint8_t)pre});
      continue;
    } else {
      return 2;
    }
  }
  flush_records();
  return 0;
}
