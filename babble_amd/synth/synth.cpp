// synth.cpp — seeded synthetic workload generator (bench and test input only;
// not part of the verification path).
//
// Produces the SURVEY §8d configurations as packed SoA batches:
//   synth_events  C1/C2/C3: a hashgraph of signed Events.  Creator c's event
//                 n has self-parent = c's event n-1 and other-parent = the
//                 latest event of creator (c+1) mod n_creators (the play
//                 pattern of src/hashgraph/hashgraph_test.go:102-112);
//                 index-0 events carry Parents ["",""].  Bodies are the
//                 canonical encoding/json bytes of EventBody
//                 (src/hashgraph/event.go:21-45), signed like Event.Sign
//                 (event.go:201-215) with EncodeSignature's r|s.
//   synth_blocks  C5: BlockBodies (block.go:16-55), each signed by every
//                 validator (Block.Sign, block.go:318-334).
// Key and nonce material comes from a SHA-256 counter DRBG keyed by the
// seed; signing uses OpenSSL (independent of both the device code and the
// CPU oracle) with per-signer nonce pools so generation stays cheap.
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>

#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct Drbg {
  uint8_t key[32];
  uint64_t ctr = 0;
  Drbg(uint64_t seed, const char *label) {
    std::string s = "babble-synth:" + std::to_string(seed) + ":" + label;
    SHA256((const uint8_t *)s.data(), s.size(), key);
  }
  void block(uint8_t out[32]) {
    uint8_t buf[40];
    memcpy(buf, key, 32);
    memcpy(buf + 32, &ctr, 8);
    ctr++;
    SHA256(buf, 40, out);
  }
};

struct SplitMix {
  uint64_t s;
  explicit SplitMix(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  void fill(uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i += 8) {
      uint64_t v = next();
      size_t k = n - i < 8 ? n - i : 8;
      memcpy(p + i, &v, k);
    }
  }
};

const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

void b64(std::string &o, const uint8_t *p, size_t n) {
  size_t i = 0;
  for (; i + 3 <= n; i += 3) {
    uint32_t v = (p[i] << 16) | (p[i + 1] << 8) | p[i + 2];
    o += kB64[v >> 18];
    o += kB64[(v >> 12) & 63];
    o += kB64[(v >> 6) & 63];
    o += kB64[v & 63];
  }
  if (n - i == 1) {
    uint32_t v = p[i] << 16;
    o += kB64[v >> 18];
    o += kB64[(v >> 12) & 63];
    o += "==";
  } else if (n - i == 2) {
    uint32_t v = (p[i] << 16) | (p[i + 1] << 8);
    o += kB64[v >> 18];
    o += kB64[(v >> 12) & 63];
    o += kB64[(v >> 6) & 63];
    o += '=';
  }
}

struct Signer {
  BIGNUM *d = nullptr;
  std::vector<BIGNUM *> kinv;  // nonce pool: k^-1 mod N
  std::vector<BIGNUM *> r;     // x(kG) mod N
  uint8_t pub[65];
};

struct Ctx {
  EC_GROUP *g;
  BIGNUM *n;
  BN_CTX *bn;
  Ctx() {
    g = EC_GROUP_new_by_curve_name(NID_secp256k1);
    n = BN_new();
    bn = BN_CTX_new();
    EC_GROUP_get_order(g, n, bn);
  }
  ~Ctx() {
    BN_free(n);
    BN_CTX_free(bn);
    EC_GROUP_free(g);
  }
  // uniform in [1, N-1] from the DRBG
  BIGNUM *scalar(Drbg &dr) {
    uint8_t b[32];
    BIGNUM *x = BN_new();
    for (;;) {
      dr.block(b);
      BN_bin2bn(b, 32, x);
      if (!BN_is_zero(x) && BN_cmp(x, n) < 0) return x;
    }
  }
  // Nonce pool: k_j = k_0 + j delta (mod N) with k_0, delta from the DRBG,
  // so R_j = R_(j-1) + delta G is one point addition instead of a full
  // scalar multiplication per nonce (generation-side cost only; r = x(R_j)
  // still varies like a random nonce's, the verifier cannot exploit it).
  void make_signer(Signer &s, Drbg &dr, uint32_t pool) {
    s.d = scalar(dr);
    EC_POINT *P = EC_POINT_new(g), *D = EC_POINT_new(g);
    EC_POINT_mul(g, P, s.d, nullptr, nullptr, bn);
    EC_POINT_point2oct(g, P, POINT_CONVERSION_UNCOMPRESSED, s.pub, 65, bn);
    BIGNUM *k = scalar(dr), *delta = scalar(dr);
    EC_POINT_mul(g, P, k, nullptr, nullptr, bn);
    EC_POINT_mul(g, D, delta, nullptr, nullptr, bn);
    BIGNUM *x = BN_new(), *y = BN_new();
    for (uint32_t i = 0; i < pool; i++) {
      if (i) {
        EC_POINT_add(g, P, P, D, bn);
        BN_mod_add(k, k, delta, n, bn);
      }
      EC_POINT_get_affine_coordinates(g, P, x, y, bn);
      BIGNUM *rr = BN_new();
      BN_nnmod(rr, x, n, bn);
      s.kinv.push_back(BN_mod_inverse(nullptr, k, n, bn));
      s.r.push_back(rr);
    }
    BN_free(k);
    BN_free(delta);
    BN_free(x);
    BN_free(y);
    EC_POINT_free(P);
    EC_POINT_free(D);
  }
  // s = k^-1 (e + r d) mod N with pool entry j; writes 32-byte BE r, s
  void sign(const Signer &sg, uint32_t j, const uint8_t digest[32], uint8_t r_out[32], uint8_t s_out[32]) {
    BN_CTX_start(bn);
    BIGNUM *e = BN_CTX_get(bn), *t = BN_CTX_get(bn);
    BN_bin2bn(digest, 32, e);
    BN_mod_mul(t, sg.r[j], sg.d, n, bn);
    BN_mod_add(t, t, e, n, bn);
    BN_mod_mul(t, t, sg.kinv[j], n, bn);
    BN_bn2binpad(sg.r[j], r_out, 32);
    BN_bn2binpad(t, s_out, 32);
    BN_CTX_end(bn);
  }
  void free_signer(Signer &s) {
    BN_free(s.d);
    for (auto *b : s.kinv) BN_free(b);
    for (auto *b : s.r) BN_free(b);
  }
};

}  // namespace

extern "C" {

// Upper bound of the body bytes synth_events will produce.
uint64_t synth_events_capacity(uint64_t n_events, uint32_t n_tx, uint32_t tx_bytes) {
  const uint64_t per = 400 + (uint64_t)n_tx * (4 * ((tx_bytes + 2) / 3) + 3) + 64;
  return n_events * per;
}

// Returns total body bytes written, or 0 on failure.
// Outputs: msg_bytes/msg_off (n_events+1), key_bytes (65 * n_creators),
// item_key[n_events], r_be/s_be[32 * n_events]; optionally (non-null) the
// wire fields of every event for bv_verify_events: digests (32 * n), parent
// event indices (2 * n, -1 = none), Index and Timestamp (n each) and the raw
// transactions (n * n_tx * tx_bytes).
uint64_t synth_events_fields(uint64_t seed, uint32_t n_creators, uint64_t n_events, uint32_t n_tx, uint32_t tx_bytes,
                             uint32_t nonce_pool, int64_t ts0, uint8_t *msg_bytes, uint64_t msg_cap,
                             uint64_t *msg_off, uint8_t *key_bytes, uint32_t *item_key, uint8_t *r_be, uint8_t *s_be,
                             uint8_t *digest_out, int64_t *parent_out, int64_t *index_out, int64_t *ts_out,
                             uint8_t *tx_out);
uint64_t synth_events(uint64_t seed, uint32_t n_creators, uint64_t n_events, uint32_t n_tx, uint32_t tx_bytes,
                      uint32_t nonce_pool, int64_t ts0, uint8_t *msg_bytes, uint64_t msg_cap, uint64_t *msg_off,
                      uint8_t *key_bytes, uint32_t *item_key, uint8_t *r_be, uint8_t *s_be) {
  return synth_events_fields(seed, n_creators, n_events, n_tx, tx_bytes, nonce_pool, ts0, msg_bytes, msg_cap, msg_off,
                             key_bytes, item_key, r_be, s_be, nullptr, nullptr, nullptr, nullptr, nullptr);
}
uint64_t synth_events_fields(uint64_t seed, uint32_t n_creators, uint64_t n_events, uint32_t n_tx, uint32_t tx_bytes,
                             uint32_t nonce_pool, int64_t ts0, uint8_t *msg_bytes, uint64_t msg_cap,
                             uint64_t *msg_off, uint8_t *key_bytes, uint32_t *item_key, uint8_t *r_be, uint8_t *s_be,
                             uint8_t *digest_out, int64_t *parent_out, int64_t *index_out, int64_t *ts_out,
                             uint8_t *tx_out) {
  if (n_creators == 0 || nonce_pool == 0) return 0;
  Ctx cx;
  Drbg dr(seed, "keys");
  std::vector<Signer> sg(n_creators);
  for (uint32_t c = 0; c < n_creators; c++) {
    cx.make_signer(sg[c], dr, nonce_pool);
    memcpy(key_bytes + 65 * c, sg[c].pub, 65);
  }
  SplitMix rng(seed * 0x2545F4914F6CDD1Dull + 7);
  // the body is written in place (no per-event allocation): constant JSON
  // pieces, each creator's base64 key computed once, parents' "0X..." hex
  // kept per creator (66 chars)
  std::vector<std::string> creator_b64(n_creators);
  for (uint32_t c = 0; c < n_creators; c++) b64(creator_b64[c], sg[c].pub, 65);
  std::vector<std::array<char, 66>> last_hex(n_creators);  // "0X..." of each creator's latest event
  std::vector<int64_t> last_ev(n_creators, -1);            // ... and its batch index
  std::vector<int64_t> next_index(n_creators, 0);
  std::vector<uint8_t> txs((size_t)n_tx * tx_bytes);
  std::string tmp;
  uint64_t pos = 0;
  msg_off[0] = 0;
  const uint64_t per_max = 400 + (uint64_t)n_tx * (4 * ((tx_bytes + 2) / 3) + 3) + 64;
  for (uint64_t i = 0; i < n_events; i++) {
    const uint32_t c = (uint32_t)(i % n_creators);
    const uint32_t other = (c + 1) % n_creators;
    for (uint32_t t = 0; t < n_tx; t++) rng.fill(txs.data() + (size_t)t * tx_bytes, tx_bytes);
    const int64_t idx = next_index[c]++;
    const bool has_p1 = idx > 0 && last_ev[other] >= 0;  // the other creator may have no event yet
    if (parent_out) {
      parent_out[2 * i] = idx > 0 ? last_ev[c] : -1;
      parent_out[2 * i + 1] = has_p1 ? last_ev[other] : -1;
    }
    if (index_out) index_out[i] = idx;
    if (ts_out) ts_out[i] = ts0 + (int64_t)i;
    if (tx_out) memcpy(tx_out + (uint64_t)i * n_tx * tx_bytes, txs.data(), (size_t)n_tx * tx_bytes);
    if (pos + per_max > msg_cap) return 0;
    char *o = (char *)msg_bytes + pos, *const o0 = o;
    auto put = [&o](const char *p, size_t n) {
      memcpy(o, p, n);
      o += n;
    };
    auto lit = [&put](const char *p) { put(p, strlen(p)); };
    lit("{\"Transactions\":");
    if (n_tx == 0) {
      lit("null");
    } else {
      *o++ = '[';
      for (uint32_t t = 0; t < n_tx; t++) {
        if (t) *o++ = ',';
        *o++ = '"';
        tmp.clear();
        b64(tmp, txs.data() + (size_t)t * tx_bytes, tx_bytes);
        put(tmp.data(), tmp.size());
        *o++ = '"';
      }
      *o++ = ']';
    }
    lit(",\"InternalTransactions\":null,\"Parents\":[\"");
    if (idx > 0) put(last_hex[c].data(), 66);
    lit("\",\"");
    if (has_p1) put(last_hex[other].data(), 66);
    lit("\"],\"Creator\":\"");
    put(creator_b64[c].data(), creator_b64[c].size());
    lit("\",\"Index\":");
    o += snprintf(o, 24, "%lld", (long long)idx);
    lit(",\"BlockSignatures\":null,\"Timestamp\":");
    o += snprintf(o, 24, "%lld", (long long)(ts0 + (int64_t)i));
    lit("}\n");
    const size_t len = (size_t)(o - o0);
    pos += len;
    msg_off[i + 1] = pos;
    uint8_t dig[32];
    SHA256((const uint8_t *)o0, len, dig);
    static const char H[] = "0123456789ABCDEF";
    char *hx = last_hex[c].data();
    hx[0] = '0';
    hx[1] = 'X';
    for (int k = 0; k < 32; k++) hx[2 + 2 * k] = H[dig[k] >> 4], hx[3 + 2 * k] = H[dig[k] & 15];
    last_ev[c] = (int64_t)i;
    if (digest_out) memcpy(digest_out + 32 * i, dig, 32);
    item_key[i] = c;
    cx.sign(sg[c], (uint32_t)(idx % nonce_pool), dig, r_be + 32 * i, s_be + 32 * i);
  }
  for (auto &s : sg) cx.free_signer(s);
  return pos;
}

uint64_t synth_blocks_capacity(uint64_t n_blocks, uint32_t n_tx, uint32_t tx_bytes) {
  const uint64_t per = 400 + (uint64_t)n_tx * (4 * ((tx_bytes + 2) / 3) + 3) + 64;
  return n_blocks * per;
}

// C5: n_blocks BlockBodies, each signed by all n_validators.  Items are
// block-major (item = b * n_validators + v).  peers_hash (32 bytes) is the
// PeerSet.Hash chain over the validator keys (peer_set.go:104-115) and is
// returned so the caller can run CheckBlock.
uint64_t synth_blocks(uint64_t seed, uint32_t n_validators, uint64_t n_blocks, uint32_t n_tx, uint32_t tx_bytes,
                      uint32_t nonce_pool, int64_t ts0, uint8_t *msg_bytes, uint64_t msg_cap, uint64_t *msg_off,
                      uint8_t *key_bytes, uint8_t *peers_hash, uint32_t *item_msg, uint32_t *item_key, uint8_t *r_be,
                      uint8_t *s_be) {
  if (n_validators == 0 || nonce_pool == 0) return 0;
  Ctx cx;
  Drbg dr(seed, "validators");
  std::vector<Signer> sg(n_validators);
  uint8_t h[32];
  std::vector<uint8_t> chain;  // h = SHA256(h || pk), h starts empty
  for (uint32_t v = 0; v < n_validators; v++) {
    cx.make_signer(sg[v], dr, nonce_pool);
    memcpy(key_bytes + 65 * v, sg[v].pub, 65);
    std::vector<uint8_t> buf(chain);
    buf.insert(buf.end(), sg[v].pub, sg[v].pub + 65);
    SHA256(buf.data(), buf.size(), h);
    chain.assign(h, h + 32);
  }
  memcpy(peers_hash, chain.data(), 32);
  SplitMix rng(seed * 0x9E3779B97F4A7C15ull + 11);
  std::vector<uint8_t> tx(tx_bytes);
  uint64_t pos = 0;
  msg_off[0] = 0;
  for (uint64_t b = 0; b < n_blocks; b++) {
    uint8_t state_hash[32], frame_hash[32];
    rng.fill(state_hash, 32);
    rng.fill(frame_hash, 32);
    std::string o;
    o.reserve(512 + n_tx * 96);
    o += "{\"Index\":";
    o += std::to_string(b);
    o += ",\"RoundReceived\":";
    o += std::to_string(b + 1);
    o += ",\"Timestamp\":";
    o += std::to_string(ts0 + (int64_t)b);
    o += ",\"StateHash\":\"";
    b64(o, state_hash, 32);
    o += "\",\"FrameHash\":\"";
    b64(o, frame_hash, 32);
    o += "\",\"PeersHash\":\"";
    b64(o, peers_hash, 32);
    o += "\",\"Transactions\":[";
    for (uint32_t t = 0; t < n_tx; t++) {
      rng.fill(tx.data(), tx.size());
      if (t) o += ',';
      o += '"';
      b64(o, tx.data(), tx.size());
      o += '"';
    }
    o += "],\"InternalTransactions\":[],\"InternalTransactionReceipts\":null}\n";
    if (pos + o.size() > msg_cap) return 0;
    memcpy(msg_bytes + pos, o.data(), o.size());
    pos += o.size();
    msg_off[b + 1] = pos;
    uint8_t dig[32];
    SHA256((const uint8_t *)o.data(), o.size(), dig);
    for (uint32_t v = 0; v < n_validators; v++) {
      const uint64_t it = b * n_validators + v;
      item_msg[it] = (uint32_t)b;
      item_key[it] = v;
      cx.sign(sg[v], (uint32_t)(b % nonce_pool), dig, r_be + 32 * it, s_be + 32 * it);
    }
  }
  for (auto &s : sg) cx.free_signer(s);
  return pos;
}

}  // extern "C"
