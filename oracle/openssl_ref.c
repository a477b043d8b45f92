/*
 * openssl_ref.c — OpenSSL libcrypto proxy of the reference's CPU path:
 * TEST AND BASELINE INFRASTRUCTURE ONLY (never linked into the product).
 *
 * The Go reference (crypto/ecdsa.Verify over btcec) cannot run
 * here (no Go toolchain, no btcd module).  SURVEY §8d's CPU-baseline proxy is
 * an all-core harness over OpenSSL: per item, SHA-256 of the message
 * (crypto.SHA256, src/crypto/hash.go:8), SEC1 decode of the creator key
 * (keys.ToPublicKey, src/crypto/keys/public_key.go:14 — done per item, as
 * Event.Verify does at src/hashgraph/event.go:234) and ECDSA_do_verify
 * (keys.Verify, src/crypto/keys/signature.go:20).  It is also the independent
 * cross-check of the oracle's ECDSA math on every WELL-FORMED item (r, s in
 * [1, N-1], 65-byte uncompressed on-curve key): OpenSSL is no oracle for the
 * Go parsing / panic rules (it accepts compressed keys), so other items are
 * reported as OSSL_SKIP.
 */
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include "../include/babbleverify.h"

#define OSSL_SKIP 0xFE

static const uint8_t N_BE[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                 0xFF, 0xFF, 0xFF, 0xFF, 0xFE, 0xBA, 0xAE, 0xDC, 0xE6, 0xAF, 0x48,
                                 0xA0, 0x3B, 0xBF, 0xD2, 0x5E, 0x8C, 0xD0, 0x36, 0x41, 0x41};

static int in_range(const uint8_t *v) { /* 0 < v < N, 32 BE bytes */
  int nz = 0;
  for (int i = 0; i < 32; i++) nz |= v[i];
  if (!nz) return 0;
  return memcmp(v, N_BE, 32) < 0;
}

typedef struct {
  const bv_batch *b;
  uint8_t *status;
  uint64_t lo, hi;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  const bv_batch *b = j->b;
  EC_KEY *key = EC_KEY_new_by_curve_name(NID_secp256k1);
  ECDSA_SIG *sig = ECDSA_SIG_new();
  for (uint64_t i = j->lo; i < j->hi; i++) {
    const uint32_t m = b->item_msg[i], k = b->item_key[i];
    const uint8_t *pub = b->key_bytes + b->key_off[k];
    const uint64_t publen = b->key_off[k + 1] - b->key_off[k];
    const uint8_t *r = b->r_be + 32 * i, *s = b->s_be + 32 * i;
    if ((b->pre && b->pre[i]) || publen != 65 || pub[0] != 4 || !in_range(r) || !in_range(s)) {
      j->status[i] = OSSL_SKIP;
      continue;
    }
    uint8_t digest[32];
    SHA256(b->msg_bytes + b->msg_off[m], b->msg_off[m + 1] - b->msg_off[m], digest);
    const unsigned char *p = pub;
    if (!o2i_ECPublicKey(&key, &p, 65)) { /* off-curve or x, y >= p */
      j->status[i] = OSSL_SKIP;
      continue;
    }
    BIGNUM *rb = BN_bin2bn(r, 32, NULL), *sb = BN_bin2bn(s, 32, NULL);
    ECDSA_SIG_set0(sig, rb, sb);
    const int rv = ECDSA_do_verify(digest, 32, sig, key);
    j->status[i] = rv == 1 ? 1 : rv == 0 ? 0 : OSSL_SKIP;
  }
  ECDSA_SIG_free(sig);
  EC_KEY_free(key);
  return NULL;
}

/* status[i]: 1 accept, 0 reject, OSSL_SKIP (0xFE) not well-formed. */
int ossl_verify_batch(const bv_batch *b, uint8_t *status, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  pthread_t th[256];
  job_t jobs[256];
  const uint64_t n = b->n_items;
  for (int t = 0; t < n_threads; t++) {
    jobs[t].b = b;
    jobs[t].status = status;
    jobs[t].lo = n * t / n_threads;
    jobs[t].hi = n * (t + 1) / n_threads;
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  return 0;
}
