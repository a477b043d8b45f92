/*
 * shim_harness.c — TEST AND BENCH INFRASTRUCTURE, not part of the product.
 *
 * Replays, in C through the C ABI (include/babbleverify.h), the exact call
 * sequence of the cgo shim in INTEGRATION.md section 2 (Go is not installed
 * here, so the Go source there cannot run; this harness is its stand-in):
 *
 *   verifier()        one process context, bv_create(BV_F_KEY_CACHE)
 *   setPeers          bv_kc_register of the PeerSet's PubKeyBytes
 *                     (core.setPeers, src/node/core.go:186)
 *   builder pool      sync.Pool of batch builders; each owns a bv_arena
 *                     (bv_arena_reserve replaces cbuf.grow's per-call
 *                     bv_host_alloc / bv_host_free)
 *   VerifySync        core.sync (core.go:210-245) after ReadWireBatch: the
 *                     resolved WireEvents written into the arena in two
 *                     passes over chunks of events (sizes, then the fill at
 *                     exact offsets; creators keyed by id; each Signature's
 *                     text bytes copied: the library decodes them on the
 *                     device), ONE bv_verify_events, digests and statuses
 *                     copied out (C.GoBytes) by chunk
 *   VerifyEvents      Event.Verify (event.go:219-247) for one event through
 *                     bv_verify_batch (addSelfEvent, core.go:291)
 *
 * tests/test_cabi.py checks its results against the C oracle; bench.py's
 * `shim_path` leg times it.  Built by tests/cabi/Makefile (gcc, linked
 * against babble_amd/libbabbleverify.so).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "babbleverify.h"

enum {
  S_KEYS, S_KOFF, S_CREATOR, S_INDEX, S_TS, S_PKIND, S_PREF, S_PHASH, S_TXSTART, S_TXOFF, S_TXB, S_TXLNIL,
  S_TXNIL, S_ITXOFF, S_ITX, S_BSOFF, S_BS, S_R, S_S, S_PRE, S_OUT, S_MSGS, S_MOFF, S_IMSG, S_IKEY, S_SIGOFF,
  S_SIGTXT, S_NSLOTS
};

/* a batch builder: arena blocks + fill levels (Go: the cbufs of `batch`)
 * and the key map (Go: map[string]uint32) */
typedef struct {
  bv_arena *arena;
  uint8_t *p[S_NSLOTS];
  size_t n[S_NSLOTS], cap[S_NSLOTS];
  uint32_t *kmap;       /* open addressing: key index + 1, 0 = empty */
  uint32_t kmap_cap, n_keys;
  uint32_t *cid, cid_cap, n_cid; /* creator id -> key index + 1 (Go: map[uint32]uint32) */
} builder;

static int put(builder *b, int slot, const void *src, size_t len) {
  if (b->n[slot] + len > b->cap[slot]) { /* cbuf.grow: only past the high-water mark */
    void *np;
    if (bv_arena_reserve(b->arena, (uint32_t)slot, b->n[slot] + len, b->n[slot], &np, &b->cap[slot]) != BV_OK)
      return -1;
    b->p[slot] = (uint8_t *)np;
  }
  if (len) memcpy(b->p[slot] + b->n[slot], src, len);
  b->n[slot] += len;
  return 0;
}
static int put_u8(builder *b, int s, uint8_t v) { return put(b, s, &v, 1); }
static int put_u32(builder *b, int s, uint32_t v) { return put(b, s, &v, 4); }
static int put_u64(builder *b, int s, uint64_t v) { return put(b, s, &v, 8); }

static uint64_t fnv(const uint8_t *p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

/* batch.key: the key's index, appending it on first sight */
static int64_t key_index(builder *b, const uint8_t *pub, size_t len) {
  if (2 * (b->n_keys + 1) > b->kmap_cap) { /* rehash */
    uint32_t nc = b->kmap_cap ? 2 * b->kmap_cap : 256;
    uint32_t *nm = (uint32_t *)calloc(nc, 4);
    if (!nm) return -1;
    const uint64_t *ko = (const uint64_t *)b->p[S_KOFF];
    for (uint32_t k = 0; k < b->n_keys; k++) {
      uint64_t h = fnv(b->p[S_KEYS] + ko[k], ko[k + 1] - ko[k]) & (nc - 1);
      while (nm[h]) h = (h + 1) & (nc - 1);
      nm[h] = k + 1;
    }
    free(b->kmap);
    b->kmap = nm, b->kmap_cap = nc;
  }
  const uint64_t *ko = (const uint64_t *)b->p[S_KOFF];
  uint64_t h = fnv(pub, len) & (b->kmap_cap - 1);
  for (; b->kmap[h]; h = (h + 1) & (b->kmap_cap - 1)) {
    const uint32_t k = b->kmap[h] - 1;
    if (ko[k + 1] - ko[k] == len && memcmp(b->p[S_KEYS] + ko[k], pub, len) == 0) return k;
  }
  if (put(b, S_KEYS, pub, len) || put_u64(b, S_KOFF, b->n[S_KEYS])) return -1;
  b->kmap[h] = b->n_keys + 1;
  return b->n_keys++;
}

static void reset(builder *b) {
  for (int s = 0; s < S_NSLOTS; s++) b->n[s] = 0;
  if (b->kmap) memset(b->kmap, 0, (size_t)b->kmap_cap * 4);
  if (b->cid) memset(b->cid, 0, (size_t)b->cid_cap * 8);
  b->n_cid = 0;
  b->n_keys = 0;
}

/* ---- the process state: verifier() and the builder pool ---- */
#define POOL 4
static bv_ctx *g_ctx;
static builder *g_free[POOL];
static int g_nfree;

static builder *pool_get(void) {
  if (g_nfree) return g_free[--g_nfree];
  builder *b = (builder *)calloc(1, sizeof *b);
  if (b && bv_arena_create(&b->arena) != BV_OK) free(b), b = NULL;
  return b;
}
static void pool_put(builder *b) {
  if (g_nfree < POOL) {
    g_free[g_nfree++] = b;
    return;
  }
  bv_arena_destroy(b->arena);
  free(b->kmap);
  free(b->cid);
  free(b);
}

int shim_open(int device, uint32_t flags) {
  if (g_ctx) return BV_OK;
  return bv_create(&g_ctx, device, flags);
}

void shim_close(void) {
  while (g_nfree) {
    builder *b = g_free[--g_nfree];
    bv_arena_destroy(b->arena);
    free(b->kmap);
    free(b->cid);
    free(b);
  }
  if (g_ctx) bv_destroy(g_ctx);
  g_ctx = NULL;
}

const char *shim_last_error(void) { return g_ctx ? bv_last_error(g_ctx) : "no context"; }

/* core.setPeers (core.go:186): the PeerSet's keys get their tables now */
int shim_set_peers(uint32_t n, const uint8_t *key_bytes, const uint64_t *key_off) {
  return g_ctx ? bv_kc_register(g_ctx, n, key_bytes, key_off) : BV_E_ARGS;
}

/* The resolved WireEvents of one SyncResponse, as the Go shim holds them
 * after ReadWireBatch (hashgraph.go:1540-1595): per event the creator's
 * PubKeyBytes (from the repertoire: `rep_*`, indexed by creator id), Index,
 * Timestamp, both parents (none / a store hash / an earlier event of the
 * response), the transactions, the ITX / BlockSignature JSON fragments and
 * the Signature text. */
typedef struct {
  uint64_t n_events;
  const uint8_t *rep_bytes;
  const uint64_t *rep_off;
  const uint32_t *creator_id;
  const int64_t *index, *timestamp;
  const uint8_t *parent_kind;   /* 2 per event, BV_PARENT_* */
  const uint64_t *parent_event; /* 2 per event: the event index (BV_PARENT_EVENT) */
  const uint8_t *parent_hash;   /* 2 x 32 bytes per event (BV_PARENT_HASH) */
  const uint64_t *tx_start, *tx_off;
  const uint8_t *tx_bytes, *tx_list_nil, *tx_nil; /* (nil flags may be NULL) */
  const uint64_t *itx_off, *bsig_off;             /* (may be NULL: all nil) */
  const uint8_t *itx_json, *bsig_json;
  const uint64_t *sig_off;
  const char *sig_text;
} shim_wire;

static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

/* ---- VerifySync's fill: two passes over chunks of events ----
 * Pass 1 sizes every slot per chunk (and collects the chunk's creator ids
 * in first-seen order), the creators get their batch key indices in event
 * order, every slot is reserved ONCE at its exact size, and pass 2 writes
 * each chunk at its prefix offsets: no per-field capacity check, chunks on
 * their own threads for large batches (Go: goroutines).
 * Pass 3 copies the digests and statuses out the same way. */
typedef struct { uint64_t tx, txb, itx, bs, sig, nh; } fill_at;

typedef struct fill_job {
  void (*fn)(struct fill_job *);
  const shim_wire *w;
  builder *b;
  uint64_t e0, e1;
  fill_at at;           /* pass 1: the chunk's sizes; pass 2: its start offsets */
  uint32_t *ids, n_ids; /* pass 1: the chunk's distinct creator ids, first-seen order */
  uint32_t *set, set_cap;
  uint8_t *dig, *st;    /* pass 3 */
  const bv_result *res;
} fill_job;

#define MAX_JOBS 8

static void *job_main(void *p) {
  fill_job *j = (fill_job *)p;
  j->fn(j);
  return NULL;
}

static void run_jobs(fill_job *jobs, int nj, void (*fn)(fill_job *)) {
  pthread_t th[MAX_JOBS];
  int started[MAX_JOBS] = {0};
  for (int i = 0; i < nj; i++) jobs[i].fn = fn;
  for (int i = 1; i < nj; i++) started[i] = pthread_create(&th[i], NULL, job_main, &jobs[i]) == 0;
  fn(&jobs[0]);
  for (int i = 1; i < nj; i++) {
    if (started[i]) pthread_join(th[i], NULL);
    else fn(&jobs[i]);
  }
}

/* id -> value + 1 in an open-addressed table of 2 * cap words (id, value+1) */
static uint32_t *idmap_slot(uint32_t *m, uint32_t cap, uint32_t id) {
  uint32_t h = (id * 2654435761u) & (cap - 1);
  while (m[2 * h + 1] && m[2 * h] != id) h = (h + 1) & (cap - 1);
  return m + 2 * h;
}

static int local_id(fill_job *j, uint32_t id) {
  if (2 * (j->n_ids + 1) > j->set_cap) {
    const uint32_t nc = j->set_cap ? 2 * j->set_cap : 64;
    uint32_t *ns = (uint32_t *)calloc(2 * (size_t)nc, 4), *nl = (uint32_t *)realloc(j->ids, 4 * (size_t)nc);
    if (!ns || !nl) return free(ns), j->ids = nl ? nl : j->ids, -1;
    j->ids = nl;
    for (uint32_t i = 0; i < j->n_ids; i++) {
      uint32_t *s = idmap_slot(ns, nc, j->ids[i]);
      s[0] = j->ids[i], s[1] = 1;
    }
    free(j->set);
    j->set = ns, j->set_cap = nc;
  }
  uint32_t *s = idmap_slot(j->set, j->set_cap, id);
  if (!s[1]) s[0] = id, s[1] = 1, j->ids[j->n_ids++] = id;
  return 0;
}

static void size_chunk(fill_job *j) {
  const shim_wire *w = j->w;
  fill_at z = {0, 0, 0, 0, 0, 0};
  uint32_t last = 0;
  int have_last = 0;
  for (uint64_t e = j->e0; e < j->e1; e++) {
    const uint32_t c = w->creator_id[e];
    if (!have_last || c != last) {
      if (local_id(j, c)) j->n_ids = UINT32_MAX; /* (out of memory: the caller fails) */
      if (j->n_ids == UINT32_MAX) return;
      last = c, have_last = 1;
    }
    z.nh += (w->parent_kind[2 * e] == BV_PARENT_HASH) + (w->parent_kind[2 * e + 1] == BV_PARENT_HASH);
    for (uint64_t t = w->tx_start[e]; t < w->tx_start[e + 1]; t++) z.txb += w->tx_off[t + 1] - w->tx_off[t];
    z.tx += w->tx_start[e + 1] - w->tx_start[e];
    if (w->itx_off) z.itx += w->itx_off[e + 1] - w->itx_off[e];
    if (w->bsig_off) z.bs += w->bsig_off[e + 1] - w->bsig_off[e];
    z.sig += w->sig_off[e + 1] - w->sig_off[e];
  }
  j->at = z;
}

static void fill_chunk(fill_job *j) {
  const shim_wire *w = j->w;
  builder *b = j->b;
  fill_at a = j->at;
  uint32_t *cr = (uint32_t *)b->p[S_CREATOR];
  int64_t *idx = (int64_t *)b->p[S_INDEX], *ts = (int64_t *)b->p[S_TS];
  uint8_t *pk = b->p[S_PKIND], *ph = b->p[S_PHASH];
  uint64_t *pref = (uint64_t *)b->p[S_PREF], *txs = (uint64_t *)b->p[S_TXSTART], *txo = (uint64_t *)b->p[S_TXOFF];
  uint8_t *txb = b->p[S_TXB], *txn = b->p[S_TXNIL], *tln = b->p[S_TXLNIL];
  uint64_t *io = (uint64_t *)b->p[S_ITXOFF], *bo = (uint64_t *)b->p[S_BSOFF], *so = (uint64_t *)b->p[S_SIGOFF];
  uint8_t *ij = b->p[S_ITX], *bj = b->p[S_BS], *sg = b->p[S_SIGTXT];
  uint32_t last = 0, lastk = 0;
  int have_last = 0;
  for (uint64_t e = j->e0; e < j->e1; e++) {
    const uint32_t c = w->creator_id[e];
    if (!have_last || c != last) lastk = idmap_slot(b->cid, b->cid_cap, c)[1] - 1, last = c, have_last = 1;
    cr[e] = lastk;
    idx[e] = w->index[e];
    ts[e] = w->timestamp[e];
    for (int k = 0; k < 2; k++) {
      const uint8_t kind = w->parent_kind[2 * e + k];
      uint64_t ref = 0;
      if (kind == BV_PARENT_HASH) {
        memcpy(ph + 32 * a.nh, w->parent_hash + 64 * e + 32 * k, 32);
        ref = a.nh++;
      } else if (kind == BV_PARENT_EVENT) {
        ref = w->parent_event[2 * e + k];
      }
      pk[2 * e + k] = kind;
      pref[2 * e + k] = ref;
    }
    for (uint64_t t = w->tx_start[e]; t < w->tx_start[e + 1]; t++) {
      const uint64_t len = w->tx_off[t + 1] - w->tx_off[t];
      if (len) memcpy(txb + a.txb, w->tx_bytes + w->tx_off[t], len);
      a.txb += len;
      txo[a.tx + 1] = a.txb;
      txn[a.tx++] = w->tx_nil ? w->tx_nil[t] : 0;
    }
    txs[e + 1] = a.tx;
    tln[e] = w->tx_list_nil ? w->tx_list_nil[e] : 0;
    if (w->itx_off) {
      const uint64_t len = w->itx_off[e + 1] - w->itx_off[e];
      if (len) memcpy(ij + a.itx, w->itx_json + w->itx_off[e], len);
      a.itx += len;
    }
    io[e + 1] = a.itx;
    if (w->bsig_off) {
      const uint64_t len = w->bsig_off[e + 1] - w->bsig_off[e];
      if (len) memcpy(bj + a.bs, w->bsig_json + w->bsig_off[e], len);
      a.bs += len;
    }
    bo[e + 1] = a.bs;
    const uint64_t len = w->sig_off[e + 1] - w->sig_off[e];
    if (len) memcpy(sg + a.sig, w->sig_text + w->sig_off[e], len);
    a.sig += len;
    so[e + 1] = a.sig;
  }
}

static void copy_chunk(fill_job *j) { /* C.GoBytes, per chunk */
  const uint64_t n = j->e1 - j->e0;
  if (j->dig) memcpy(j->dig + 32 * j->e0, j->res->msg_hash + 32 * j->e0, 32 * n);
  if (j->st) memcpy(j->st + j->e0, j->res->status + j->e0, n);
}

/* slot s reserved at exactly `bytes` (at least 64: a non-null block) */
static int size_slot(builder *b, int s, size_t bytes) {
  void *np;
  if (bv_arena_reserve(b->arena, (uint32_t)s, bytes < 64 ? 64 : bytes, 0, &np, &b->cap[s]) != BV_OK) return -1;
  b->p[s] = (uint8_t *)np;
  b->n[s] = bytes;
  return 0;
}

static double g_phase[3]; /* the last shim_sync: build, library call, copy-out (ms) */

void shim_last_phases(double out[3]) { memcpy(out, g_phase, sizeof g_phase); }

/* VerifySync: the batch built in the arena, one bv_verify_events, results
 * copied out.  digests: 32 * n, status: n.  *ms: wall time of the whole
 * call (build + verify + copy-out). */
int shim_sync(const shim_wire *w, uint8_t *digests, uint8_t *status, double *ms) {
  if (!g_ctx || !w) return BV_E_ARGS;
  const double t0 = now_ms();
  builder *b = pool_get();
  if (!b) return BV_E_OOM;
  reset(b);
  int rc = BV_E_OOM;
  const uint64_t n = w->n_events;
  int nj = n >= 8192 ? (int)(n / 4096) : 1;
  if (nj > MAX_JOBS) nj = MAX_JOBS;
  fill_job jobs[MAX_JOBS];
  memset(jobs, 0, sizeof jobs);
  for (int i = 0; i < nj; i++) {
    jobs[i].w = w, jobs[i].b = b;
    jobs[i].e0 = n * i / nj, jobs[i].e1 = n * (i + 1) / nj;
  }
  double t1 = t0, t2 = t0;
  run_jobs(jobs, nj, size_chunk);
  fill_at tot = {0, 0, 0, 0, 0, 0};
  if (put_u64(b, S_KOFF, 0)) goto out;
  for (int i = 0; i < nj; i++) { /* the creators' key indices, in event order; chunk sizes -> offsets */
    if (jobs[i].n_ids == UINT32_MAX) goto out;
    for (uint32_t q = 0; q < jobs[i].n_ids; q++) {
      const uint32_t c = jobs[i].ids[q];
      if (2 * (b->n_cid + 1) > b->cid_cap) { /* (a repertoire larger than the map: grow it) */
        const uint32_t nc = b->cid_cap ? 2 * b->cid_cap : 256;
        uint32_t *nm = (uint32_t *)calloc(2 * (size_t)nc, 4);
        if (!nm) goto out;
        for (uint32_t h = 0; h < b->cid_cap; h++)
          if (b->cid[2 * h + 1]) memcpy(idmap_slot(nm, nc, b->cid[2 * h]), b->cid + 2 * h, 8);
        free(b->cid);
        b->cid = nm, b->cid_cap = nc;
      }
      uint32_t *s = idmap_slot(b->cid, b->cid_cap, c);
      if (s[1]) continue;
      const int64_t k = key_index(b, w->rep_bytes + w->rep_off[c], w->rep_off[c + 1] - w->rep_off[c]);
      if (k < 0) goto out;
      s[0] = c, s[1] = (uint32_t)k + 1;
      b->n_cid++;
    }
    const fill_at z = jobs[i].at;
    jobs[i].at = tot;
    tot.tx += z.tx, tot.txb += z.txb, tot.itx += z.itx, tot.bs += z.bs, tot.sig += z.sig, tot.nh += z.nh;
  }
  if (size_slot(b, S_CREATOR, 4 * n) || size_slot(b, S_INDEX, 8 * n) || size_slot(b, S_TS, 8 * n) ||
      size_slot(b, S_PKIND, 2 * n) || size_slot(b, S_PREF, 16 * n) || size_slot(b, S_PHASH, 32 * tot.nh) ||
      size_slot(b, S_TXSTART, 8 * (n + 1)) || size_slot(b, S_TXOFF, 8 * (tot.tx + 1)) ||
      size_slot(b, S_TXB, tot.txb) || size_slot(b, S_TXLNIL, n) || size_slot(b, S_TXNIL, tot.tx) ||
      size_slot(b, S_ITXOFF, 8 * (n + 1)) || size_slot(b, S_ITX, tot.itx) || size_slot(b, S_BSOFF, 8 * (n + 1)) ||
      size_slot(b, S_BS, tot.bs) || size_slot(b, S_SIGOFF, 8 * (n + 1)) || size_slot(b, S_SIGTXT, tot.sig + 1))
    goto out;
  ((uint64_t *)b->p[S_TXSTART])[0] = ((uint64_t *)b->p[S_TXOFF])[0] = 0;
  ((uint64_t *)b->p[S_ITXOFF])[0] = ((uint64_t *)b->p[S_BSOFF])[0] = ((uint64_t *)b->p[S_SIGOFF])[0] = 0;
  b->p[S_SIGTXT][tot.sig] = 0; /* (a non-null text pointer even when every signature is empty) */
  run_jobs(jobs, nj, fill_chunk);
  t1 = now_ms();
  {
    const size_t words = (n + 63) / 64, out_bytes = 32 * n + n + 8 * words + 8;
    void *op;
    if (bv_arena_reserve(b->arena, S_OUT, out_bytes, 0, &op, &b->cap[S_OUT]) != BV_OK) goto out;
    b->p[S_OUT] = (uint8_t *)op;
    bv_event_batch in;
    memset(&in, 0, sizeof in);
    in.n_events = n;
    in.n_keys = b->n_keys;
    in.key_bytes = b->p[S_KEYS];
    in.key_off = (const uint64_t *)b->p[S_KOFF];
    in.creator = (const uint32_t *)b->p[S_CREATOR];
    in.index = (const int64_t *)b->p[S_INDEX];
    in.timestamp = (const int64_t *)b->p[S_TS];
    in.parent_kind = b->p[S_PKIND];
    in.parent_ref = (const uint64_t *)b->p[S_PREF];
    in.n_parent_hashes = tot.nh;
    in.parent_hashes = b->p[S_PHASH];
    in.tx_start = (const uint64_t *)b->p[S_TXSTART];
    in.tx_off = (const uint64_t *)b->p[S_TXOFF];
    in.tx_bytes = b->p[S_TXB];
    in.tx_list_nil = w->tx_list_nil ? b->p[S_TXLNIL] : NULL;
    in.tx_nil = w->tx_nil ? b->p[S_TXNIL] : NULL;
    in.itx_off = w->itx_off ? (const uint64_t *)b->p[S_ITXOFF] : NULL;
    in.itx_json = b->p[S_ITX];
    in.bsig_off = w->bsig_off ? (const uint64_t *)b->p[S_BSOFF] : NULL;
    in.bsig_json = b->p[S_BS];
    in.sig_off = (const uint64_t *)b->p[S_SIGOFF];
    in.sig_text = b->p[S_SIGTXT];
    bv_result res;
    res.msg_hash = b->p[S_OUT];
    res.status = b->p[S_OUT] + 32 * n;
    res.accept_bits = (uint64_t *)(b->p[S_OUT] + ((32 * n + n + 7) & ~(size_t)7));
    rc = bv_verify_events(g_ctx, &in, &res);
    t2 = now_ms();
    if (rc == BV_OK) {
      for (int i = 0; i < nj; i++) jobs[i].dig = digests, jobs[i].st = status, jobs[i].res = &res;
      run_jobs(jobs, nj, copy_chunk);
    }
  }
out:
  for (int i = 0; i < nj; i++) free(jobs[i].ids), free(jobs[i].set);
  pool_put(b);
  const double t3 = now_ms();
  g_phase[0] = t1 - t0, g_phase[1] = t2 - t1, g_phase[2] = t3 - t2;
  if (ms) *ms = t3 - t0;
  return rc;
}

/* VerifyEvents([ev]) without ITX: the body (EventBody.Marshal), the
 * creator key and the Signature text -> one bv_verify_batch item. */
int shim_verify_event(const uint8_t *body, size_t body_len, const uint8_t *key, size_t key_len, const char *sig,
                      size_t sig_len, uint8_t digest[32], uint8_t *status, double *ms) {
  if (!g_ctx) return BV_E_ARGS;
  const double t0 = now_ms();
  builder *b = pool_get();
  if (!b) return BV_E_OOM;
  reset(b);
  int rc = BV_E_OOM;
  uint8_t r[32], s[32];
  const uint8_t pre = bv_decode_signature(sig, sig_len, r, s);
  int64_t k;
  if (put_u64(b, S_MOFF, 0) || put(b, S_MSGS, body, body_len) || put_u64(b, S_MOFF, body_len) ||
      put_u64(b, S_KOFF, 0) || (k = key_index(b, key, key_len)) < 0 || put_u32(b, S_IMSG, 0) ||
      put_u32(b, S_IKEY, (uint32_t)k) || put(b, S_R, r, 32) || put(b, S_S, s, 32) || put_u8(b, S_PRE, pre))
    goto out;
  {
    void *op;
    if (bv_arena_reserve(b->arena, S_OUT, 64, 0, &op, &b->cap[S_OUT]) != BV_OK) goto out;
    b->p[S_OUT] = (uint8_t *)op;
    bv_batch in;
    in.n_msgs = 1;
    in.msg_bytes = b->p[S_MSGS];
    in.msg_off = (const uint64_t *)b->p[S_MOFF];
    in.n_keys = b->n_keys;
    in.key_bytes = b->p[S_KEYS];
    in.key_off = (const uint64_t *)b->p[S_KOFF];
    in.n_items = 1;
    in.item_msg = (const uint32_t *)b->p[S_IMSG];
    in.item_key = (const uint32_t *)b->p[S_IKEY];
    in.r_be = b->p[S_R];
    in.s_be = b->p[S_S];
    in.pre = b->p[S_PRE];
    bv_result res;
    res.msg_hash = b->p[S_OUT];
    res.status = b->p[S_OUT] + 32;
    res.accept_bits = NULL;
    rc = bv_verify_batch(g_ctx, &in, &res);
    if (rc == BV_OK) {
      memcpy(digest, res.msg_hash, 32);
      *status = res.status[0];
    }
  }
out:
  pool_put(b);
  if (ms) *ms = now_ms() - t0;
  return rc;
}

/* keys.EncodeSignature (signature.go:25-27) for test data: base-36 text of
 * r and s, "r|s", lower-case digits as big.Int.Text(36).  text holds 2 x 50
 * + 1 bytes per signature; off: n + 1 offsets.  (Data preparation only.) */
static size_t text36(const uint8_t be[32], char *out) {
  uint32_t w[8];
  for (int i = 0; i < 8; i++)
    w[i] = ((uint32_t)be[4 * i] << 24) | ((uint32_t)be[4 * i + 1] << 16) | ((uint32_t)be[4 * i + 2] << 8) | be[4 * i + 3];
  char tmp[64];
  size_t n = 0;
  for (;;) {
    int nz = 0;
    uint64_t rem = 0;
    for (int i = 0; i < 8; i++) {
      const uint64_t cur = (rem << 32) | w[i];
      w[i] = (uint32_t)(cur / 36);
      rem = cur % 36;
      nz |= w[i] != 0;
    }
    tmp[n++] = "0123456789abcdefghijklmnopqrstuvwxyz"[rem];
    if (!nz) break;
  }
  for (size_t i = 0; i < n; i++) out[i] = tmp[n - 1 - i];
  return n;
}

int shim_encode_signatures(uint64_t n, const uint8_t *r_be, const uint8_t *s_be, char *text, uint64_t *off) {
  uint64_t o = 0;
  off[0] = 0;
  for (uint64_t i = 0; i < n; i++) {
    o += text36(r_be + 32 * i, text + o);
    text[o++] = '|';
    o += text36(s_be + 32 * i, text + o);
    off[i + 1] = o;
  }
  return BV_OK;
}
