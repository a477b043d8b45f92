/*
 * babbleverify.h — C ABI of libbabbleverify.so, the MI355X batch verifier for
 * Babble's event-ingestion hot path (SHA-256 of canonical bodies + ECDSA over
 * secp256k1).  Plain C types only: this is what a Go cgo shim (see
 * INTEGRATION.md) or any other FFI binds.
 *
 * Reference interfaces each entry point replaces (paths under the reference
 * tree, sikoba/babble v0.8.4):
 *   bv_verify_batch   N x { crypto.SHA256(body)              src/crypto/hash.go:8
 *                           keys.ToPublicKey(pub)             src/crypto/keys/public_key.go:14
 *                           keys.Verify(pub, hash, r, s) }    src/crypto/keys/signature.go:20
 *                     as composed by Event.Verify             src/hashgraph/event.go:219-247
 *                     InternalTransaction.Verify              src/hashgraph/internal_transaction.go:139-154
 *                     Block.Verify                            src/hashgraph/block.go:343-357
 *   bv_sha256_batch   N x crypto.SHA256                       src/crypto/hash.go:8-13
 *   bv_decode_signature  keys.DecodeSignature + the sign/range
 *                     pre-checks of ecdsa.Verify              src/crypto/keys/signature.go:31-39
 *   bv_hex_decode     common.DecodeFromString                 src/common/hex.go:15-17
 *
 * Threading: every entry point is re-entrant.  A bv_ctx serialises its own
 * calls with an internal mutex (processJoinRequest, node_rpc.go:250-260, calls
 * the verifier outside Node.coreLock); use one ctx per thread for concurrency.
 * Ownership: all pointers are caller-owned and only read/written during the
 * call; nothing is retained.  There is no CPU fallback: if no gfx950 device is
 * usable the calls fail with BV_E_NODEVICE.
 */
#ifndef BABBLEVERIFY_H
#define BABBLEVERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BV_ABI_VERSION 6

/* Return codes (per-item outcomes are never errors; they go to status[]). */
#define BV_OK 0
#define BV_E_ARGS (-1)
#define BV_E_NODEVICE (-2)
#define BV_E_OOM (-3)
#define BV_E_LAUNCH (-4)
#define BV_E_COMM (-5)

/* Item status (SURVEY §8a-9 decision table). */
#define BV_REJECT 0     /* keys.Verify returned false                          */
#define BV_ACCEPT 1     /* keys.Verify returned true                           */
#define BV_REJECT_ERR 2 /* DecodeSignature returned an error (parts != 2)      */
#define BV_REF_PANIC 3  /* the Go reference would panic on this input          */

/* Pre-class byte per item, decided on the host from the signature text.
 * bits 0-1: class of r, bits 2-3: class of s, bit 7: parts != 2.
 * pre == 0 means "r and s parsed and both in [1, N-1]": run the math.       */
#define BV_SC_OK 0     /* 0 < v < N                                          */
#define BV_SC_NIL 1    /* big.Int SetString failed -> nil (Go would panic)   */
#define BV_SC_NONPOS 2 /* v <= 0                                             */
#define BV_SC_GE_N 3   /* v >= N (possibly wider than 256 bits)              */
#define BV_PRE_PARTS_BAD 0x80
#define BV_PRE(rc, sc) ((uint8_t)((rc) | ((sc) << 2)))

/* Flags for bv_create (any other bit is BV_E_ARGS). */
#define BV_F_DEFAULT 0u
#define BV_F_KEY_CACHE 1u /* keep per-key tables in HBM across calls, keyed by
                             the raw pubkey bytes (validator sets are stable,
                             peers/peer_set.go): 22-bit signed-window GLV
                             tables, 805 MB per valid key.  A key gets a table
                             when it is registered (bv_kc_register: the
                             PeerSet) or once it has been seen in 2 batches
                             (env BV_KC_ADMIT); tables are LRU-evicted past
                             the cache budget (env BV_KEY_CACHE_GB, default
                             96), registered keys only for other registered
                             keys.  Malformed keys are never given a table.
                             A batch whose valid keys without a table are at
                             most 1 in 16 of its valid keys, carrying at most
                             1 in 16 of its items, keeps the cache (their
                             items are finished by the generic path after the
                             cached ones); otherwise the batch takes the
                             per-batch table path.  Off by default:
                             tables are then rebuilt for every batch.          */
#define BV_F_K8 2u        /* per-batch tables: never use the 12-bit tables
                             (2.75 MiB per key); 8-bit only (512 KiB per key) */
#define BV_F_KNOWN (BV_F_KEY_CACHE | BV_F_K8)

typedef struct bv_ctx bv_ctx;

/* One batch, struct-of-arrays.  Messages are hashed once each; items point
 * at a message and a key, so one BlockBody serves its 100 signatures. */
typedef struct {
  uint64_t n_msgs;
  const uint8_t *msg_bytes;  /* concatenated canonical JSON bodies            */
  const uint64_t *msg_off;   /* n_msgs + 1 offsets into msg_bytes            */
  uint32_t n_keys;
  const uint8_t *key_bytes;  /* concatenated raw pubkey bytes (any length)   */
  const uint64_t *key_off;   /* n_keys + 1 offsets into key_bytes            */
  uint64_t n_items;
  const uint32_t *item_msg;  /* message index per item                       */
  const uint32_t *item_key;  /* key index per item                           */
  const uint8_t *r_be;       /* 32 * n_items, big-endian r (valid if class OK) */
  const uint8_t *s_be;       /* 32 * n_items, big-endian s                    */
  const uint8_t *pre;        /* n_items pre-class bytes (NULL = all 0)       */
} bv_batch;

typedef struct {
  uint8_t *msg_hash;     /* 32 * n_msgs digests (NULL: not returned)          */
  uint8_t *status;       /* n_items BV_* statuses (NULL: not returned)        */
  uint64_t *accept_bits; /* ceil(n_items/64) words, bit i = item i ACCEPT,
                            LSB-first (NULL: not returned)                     */
} bv_result;

/* Timing of the last call, device-side (HIP events on the ctx stream). */
typedef struct {
  float ms_total;    /* first kernel start -> last kernel end                  */
  float ms_sha256;   /* k_sha256: message hashing                              */
  float ms_keyprep;  /* key decode + per-key table build (own stream, overlaps
                        hashing, s^-1 and the u1 G phase)                       */
  float ms_scalar;   /* k_sinv: batched s^-1 (own stream, from batch start)     */
  float ms_verify_g; /* k_verify_g: u1, u2 + GLV split, u1 G from the G table   */
  float ms_verify;   /* k_verify_q (+ u2 Q, decision, bits) or k_verify_generic */
  float ms_h2d;      /* host -> device staging (host-buffer entry point only):
                        call start -> last input byte in HBM                    */
  float ms_d2h;      /* device -> host results after the last kernel            */
  float ms_host;     /* wall clock of the whole call on the host (host entry
                        point: staging, PCIe, kernels, copy-out)                */
  float ms_host_prep; /* host: validation + staging copies, call start -> the
                         last input copy enqueued                               */
  float ms_host_out;  /* host: results copied out after the device finished    */
  uint32_t key_path; /* 0: per-lane generic path; 8 / 12: per-batch K8 / K12
                        key tables; 22: key-cache (KC) tables                   */
  uint32_t kc_hits;   /* batch keys found in the key cache                      */
  uint32_t kc_builds; /* key tables built into the cache by this call           */
  uint32_t kc_keys;   /* keys held by the cache after the call                  */
} bv_timing;

int bv_abi_version(void);

/* Create a context on `device` (HIP ordinal; -1 = current device). */
int bv_create(bv_ctx **out, int device, uint32_t flags);
void bv_destroy(bv_ctx *ctx);
const char *bv_last_error(const bv_ctx *ctx);

/* Key cache (BV_F_KEY_CACHE contexts only): set the registered keys — the
 * PeerSet's PubKeyBytes (src/peers/peer_set.go; Babble calls this where the
 * peer set changes) — replacing the previous set, and build the tables of the
 * registered valid keys that have none, before returning.  Registered tables
 * are never evicted for unregistered keys.  BV_E_ARGS on a ctx without the
 * cache or more than 4096 keys.  Cap: the budget holds floor(BV_KEY_CACHE_GB
 * / 0.805) tables (119 at the default 96 GB); past it, the first registered
 * keys in the caller's order that fit get tables and the rest none (their
 * batches take the per-batch path), still BV_OK.  bv_get_timing's kc_builds
 * / kc_keys report what was built and what the cache holds. */
int bv_kc_register(bv_ctx *ctx, uint32_t n_keys, const uint8_t *key_bytes, const uint64_t *key_off);

/* Synchronous batch verify from host buffers (the cgo entry point).  Any
 * input array or result buffer that lies in memory from bv_host_alloc is
 * moved by DMA from / to where it is; other (pageable) buffers go through
 * the ctx's pinned staging, one extra host copy each. */
int bv_verify_batch(bv_ctx *ctx, const bv_batch *batch, bv_result *result);

/* Page-locked host memory (hipHostMalloc, portable to every device) for
 * callers that build their batches in place (the cgo shim allocates its
 * bv_batch arrays here instead of C.CBytes copies).  bv_host_free ignores
 * pointers it did not allocate.  No device context is needed. */
int bv_host_alloc(size_t bytes, void **out);
void bv_host_free(void *p);

/* A pinned arena: BV_ARENA_SLOTS growable blocks of bv_host_alloc memory
 * that persist until bv_arena_destroy.  A caller that keeps its arena across
 * calls (the cgo shim's pooled batch builders)
 * page-locks and frees nothing per call: hipHostMalloc / hipHostFree cost
 * tens of microseconds each and hipHostFree synchronises the device.  Arena
 * memory is bv_host_alloc memory, so batches built in it are DMA'd in place.
 * An arena is not thread-safe: one per concurrent builder.  No device
 * context is needed. */
#define BV_ARENA_SLOTS 32
typedef struct bv_arena bv_arena;
int bv_arena_create(bv_arena **out);
void bv_arena_destroy(bv_arena *arena);
/* Block `slot` (< BV_ARENA_SLOTS) with capacity >= `bytes`.  When it must
 * grow, the new block holds max(bytes, 2 x the old capacity) bytes and its
 * first `keep` bytes (<= the old capacity) are copied from the old one, which
 * is freed.  *out = the block's base, *cap (may be NULL) = its capacity.
 * BV_E_ARGS, BV_E_OOM (the old block is then kept). */
int bv_arena_reserve(bv_arena *arena, uint32_t slot, size_t bytes, size_t keep, void **out, size_t *cap);

/* Same, with every bv_batch / bv_result pointer in device memory of the ctx's
 * device (inputs already resident in HBM).  `stream` is a hipStream_t (NULL =
 * the ctx stream); the call returns after the work is enqueued when
 * `async` != 0, else after it completes.  msg_bytes and key_bytes must stay
 * readable for 64 bytes past their last byte (the kernels read them with
 * aligned vector loads; the host entry points pad their staging copies). */
int bv_verify_batch_device(bv_ctx *ctx, const bv_batch *dbatch, bv_result *dresult,
                           void *stream, int async);
/* Streams: a process holds ONE set per device, shared by all its contexts
 * (HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES hardware
 * queues, 4 by default; streams sharing a queue run serially): one lane per
 * work slot, the s^-1 stream and a high-priority key-table stream, plus a
 * copy stream created by the first host-entry call.  A NULL `stream` above
 * runs the call on its slot's lane, so consecutive async calls overlap
 * without the caller creating streams.  bv_last_stream returns the stream
 * the ctx's last call ran on (a hipStream_t), to order the caller's own
 * work after an async NULL-stream call. */
void *bv_last_stream(const bv_ctx *ctx);
/* The ctx holds two sets of work buffers.  Consecutive bv_verify_batch_device
 * calls alternate them, and each waits (on the device) only for the last call
 * that used the same set — and for the call before it when their result
 * buffers overlap: two async calls on different streams writing different
 * results overlap, one call's key tables building beside the other's verify
 * (the caller orders a call whose inputs an earlier in-flight call's results
 * write, as for any two streams).  Every other entry
 * point first waits for all earlier calls.  bv_sync waits for every call's
 * work and updates bv_get_timing (the last call's). */
int bv_sync(bv_ctx *ctx);

/* Events from their wire fields.  Instead of the
 * serialized bodies, the caller passes what a WireEvent carries
 * (src/hashgraph/event.go:413-449) with the parents resolved as in
 * Hashgraph.ReadWireInfo (hashgraph.go:1540-1595); the device builds every
 * canonical EventBody JSON (event.go:38-45, Go 1.13 encoding/json, bit-exact),
 * hashes it and verifies the creator's signature over it.  A parent may be an
 * EARLIER event of the same batch (the in-batch DAG dependency of core.sync,
 * core.go:214-245): its "0X"+hex is spliced into the child's body once the
 * parent's digest is known.  Such a batch (a SyncResponse) is built and
 * hashed in topological order on the host while the device decodes the keys,
 * builds the key tables and inverts s; then only the digests cross PCIe and
 * the device verifies.  Batches without in-batch parents are built and hashed
 * on the device; ~2-3x fewer bytes cross PCIe than the serialized bodies
 * (64-B tx: ~250 B per event instead of ~530).
 * Per-event result: msg_hash (the body digest = Event.Hash) and status of the
 * event signature (keys.Verify as composed by Event.Verify, event.go:232-247).
 * InternalTransactions are serialized from the verbatim fragment but their
 * own signatures are NOT verified here (use bv_verify_batch items, as the Go
 * shim does for Event.Verify's ITX loop). */
#define BV_PARENT_NONE 0  /* "" (wire index < 0)                              */
#define BV_PARENT_HASH 1  /* known hash: parent_ref indexes parent_hashes     */
#define BV_PARENT_EVENT 2 /* an earlier event of this batch: parent_ref = its
                             index (< the child's)                            */
typedef struct {
  uint64_t n_events;
  uint32_t n_keys;
  const uint8_t *key_bytes;      /* creator keys, raw bytes (as bv_batch)      */
  const uint64_t *key_off;       /* n_keys + 1                                 */
  const uint32_t *creator;       /* key index per event (EventBody.Creator)    */
  const int64_t *index;          /* EventBody.Index                            */
  const int64_t *timestamp;      /* EventBody.Timestamp                        */
  const uint8_t *parent_kind;    /* 2 per event: self-parent, other-parent     */
  const uint64_t *parent_ref;    /* 2 per event (see BV_PARENT_*)              */
  uint64_t n_parent_hashes;
  const uint8_t *parent_hashes;  /* 32 bytes each                              */
  const uint64_t *tx_start;      /* n_events + 1: event e has transactions
                                    [tx_start[e], tx_start[e+1])               */
  const uint64_t *tx_off;        /* n_tx + 1 byte offsets into tx_bytes        */
  const uint8_t *tx_bytes;
  const uint8_t *tx_list_nil;    /* per event, 1: Transactions is nil (NULL: none) */
  const uint8_t *tx_nil;         /* per tx, 1: that []byte is nil (NULL: none)  */
  const uint64_t *itx_off;       /* n_events + 1 into itx_json: encoding/json of
                                    InternalTransactions; empty = nil (NULL: all nil) */
  const uint8_t *itx_json;
  const uint64_t *bsig_off;      /* same for BlockSignatures (creator = Validator) */
  const uint8_t *bsig_json;
  const uint8_t *r_be;           /* the event signature, as in bv_batch        */
  const uint8_t *s_be;
  const uint8_t *pre;
  /* OR the Event.Signature text of every event (sig_off: n_events + 1 byte
   * offsets into sig_text).  When sig_text is non-NULL, r_be / s_be / pre are
   * ignored (may be NULL): the device decodes each signature as
   * bv_decode_signature does (keys.DecodeSignature + the range checks) beside
   * the key decode, so a caller holding Go strings copies bytes and makes no
   * call per event. */
  const uint64_t *sig_off;
  const uint8_t *sig_text;
} bv_event_batch;

/* Host buffers in, results out (msg_hash: 32 * n_events; status, accept_bits
 * per event).  BV_E_ARGS for a bad reference (an EVENT parent not earlier in
 * the batch, an out-of-range key / hash / offset).  As for bv_verify_batch,
 * arrays and result buffers in bv_host_alloc memory are DMA'd in place. */
int bv_verify_events(bv_ctx *ctx, const bv_event_batch *events, bv_result *result);

/* Multi-GPU: one verifier over several devices of this process (one bv_ctx
 * per device, the caller's device ordinals).  bv_group_verify_batch shards
 * the items into contiguous ranges that never split the items of one
 * message (a BlockBody's signatures stay on one device), balanced by item
 * count (bv_plan_shards); each device stages, hashes and verifies its shard
 * (messages of the shard only), and the per-device accept bitmasks come back
 * through ONE RCCL all-gather (ncclAllGather over xGMI, librccl loaded at
 * bv_group_create) into device 0, from which the merged bitmask is copied
 * once.  Digests and statuses come back per device.  Errors: BV_E_COMM if
 * RCCL is unavailable or a collective fails; BV_E_ARGS if a device appears
 * twice in a list of several devices.  A list naming ONE device n times
 * makes n logical shards on it (one ctx each, no RCCL: the shard bitmasks
 * are gathered by device copies; the key-cache budget is split between the
 * shards). */
typedef struct bv_group bv_group;
int bv_group_create(bv_group **out, const int *devices, int n_devices, uint32_t flags);
void bv_group_destroy(bv_group *g);
const char *bv_group_last_error(const bv_group *g);
int bv_group_verify_batch(bv_group *g, const bv_batch *batch, bv_result *result);
/* Timing of the last group call on device slot `i` (its ctx's bv_timing). */
int bv_group_get_timing(const bv_group *g, int i, bv_timing *out);
/* Host helper (no device): the shard plan bv_group_verify_batch uses.
 * Writes n_shards + 1 item bounds (bounds[0] = 0, bounds[n] = n_items). */
int bv_plan_shards(const bv_batch *batch, int n_shards, uint64_t *bounds);
/* Host helper (no device): the bitmask merge bv_group_verify_batch does
 * after its all-gather.  Shard d's words start at gathered[d *
 * words_per_shard]; its bit 0 is item bounds[d].  Writes
 * ceil(bounds[n_shards] / 64) words to `out`; BV_E_ARGS on non-monotone
 * bounds or a shard wider than words_per_shard words.
 * bv_group_verify_batch accepts items in any message order: the items are
 * sorted by message (stably) for sharding, the messages are partitioned into
 * contiguous device ranges (each hashed once, also messages no item names),
 * and statuses / bits come back in the caller's item order. */
int bv_merge_shard_bits(const uint64_t *gathered, uint64_t words_per_shard, int n_shards,
                        const uint64_t *bounds, uint64_t *out);
/* Host helper (no device): the whole plan of bv_group_verify_batch.  perm
 * (n_items entries, may be NULL): the item order used, perm[j] = the caller's
 * index of the j-th item (identity when item_msg is non-decreasing);
 * item_bounds (n_shards + 1): the shards over that order (bv_plan_shards);
 * msg_bounds (n_shards + 1): device d hashes messages [msg_bounds[d],
 * msg_bounds[d+1]) — a partition of [0, n_msgs).  Returns 1 when the items
 * were permuted, 0 when not, BV_E_ARGS on bad arguments. */
int bv_plan_group(const bv_batch *batch, int n_shards, uint64_t *item_bounds, uint64_t *msg_bounds,
                  uint32_t *perm);

/* SHA-256 of n messages (host buffers) -> 32*n bytes. */
int bv_sha256_batch(bv_ctx *ctx, uint64_t n_msgs, const uint8_t *msg_bytes,
                    const uint64_t *msg_off, uint8_t *out_hash);

/* PeerSet.Hash (src/peers/peer_set.go:104-115): h = [] then h = SHA256(h ||
 * pubkey) over the n peers' raw key bytes in order (PubKeyBytes), as ONE
 * device launch (the chain is serial).  n_peers == 0: the hash is empty
 * ([]byte{}) and out_hash is not written. */
int bv_peer_set_hash(bv_ctx *ctx, uint32_t n_peers, const uint8_t *key_bytes, const uint64_t *key_off,
                     uint8_t out_hash[32]);

/* Device-timing breakdown of the last verify call on this ctx. */
int bv_get_timing(const bv_ctx *ctx, bv_timing *out);

/* Host helpers mirroring the Go parsing semantics (no device needed). */
/* keys.DecodeSignature + classification: writes 32-byte BE r,s (zero when the
 * class is not OK) and returns the pre byte. */
uint8_t bv_decode_signature(const char *sig, size_t len, uint8_t r_be[32], uint8_t s_be[32]);
/* common.DecodeFromString: hex.DecodeString(s[2:]) keeping the prefix decoded
 * before the first error.  Returns the decoded length, or -1 where Go panics
 * (len < 2).  `out` must hold (len-2)/2 bytes. */
int64_t bv_hex_decode(const char *s, size_t len, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif /* BABBLEVERIFY_H */
