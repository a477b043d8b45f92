// bv_internal.h — ctx layout and internal entry points shared by bv_api.cpp
// (single device) and bv_group.cpp (multi-device group).  Not installed.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <array>

#ifndef BV_SLOTS
#define BV_SLOTS 2  // work-buffer slots: device calls that may be in flight at once (3: -4 % in a same-box A/B)
#endif
#include <vector>

#include "../../include/babbleverify.h"
#include "hostscalar.h"
#include "geometry.h"
#include "hostdag.h"

#define KS_OK 0  // k_key_decode statuses (verify_core.h)

namespace bvk {
hipError_t sha256(hipStream_t, uint64_t, const uint8_t *, const uint64_t *, uint32_t *, uint64_t max_len = ~0ull);
hipError_t put_digests(hipStream_t, uint64_t, const uint64_t *, const uint32_t *, uint32_t *);
hipError_t key_decode(hipStream_t, uint32_t, const uint8_t *, const uint64_t *, uint8_t *, uint32_t *);
hipError_t sha256_chain(hipStream_t, uint32_t, const uint8_t *, const uint64_t *, uint8_t *, uint32_t *);
hipError_t ev_body_hash(hipStream_t st, const bv_event_batch &b, uint64_t e0, uint64_t e1, uint32_t *dig);
hipError_t iota(hipStream_t, uint64_t, uint32_t *);
hipError_t sig_decode(hipStream_t, uint64_t n, const uint64_t *off, const uint8_t *text, uint8_t *r_be, uint8_t *s_be,
                      uint8_t *pre);
hipError_t build_tables(hipStream_t, int, uint32_t, const uint32_t *, const uint8_t *, uint32_t *, uint32_t *,
                        uint32_t *, uint32_t *, uint64_t n_items);
hipError_t build_kc(hipStream_t, uint32_t, const uint32_t *, const uint8_t *, uint32_t *, uint32_t *, uint32_t *,
                    const uint64_t *);
size_t kc_pscr_bytes();
hipError_t sinv(hipStream_t, uint64_t, uint32_t, const uint32_t *, const uint8_t *, uint32_t *);
hipError_t glv_split(hipStream_t, uint64_t n, const uint32_t *r_be, const uint32_t *w, uint32_t *u12);
// verify kernels over items [lo, hi) of an n-item batch (lo a multiple of 64)
hipError_t verify_gq(hipStream_t, uint64_t, uint64_t, uint64_t, const uint32_t *, const uint32_t *, const uint32_t *,
                     const uint8_t *, const uint8_t *, const uint32_t *, const uint32_t *, const uint32_t *,
                     const uint32_t *, const uint64_t *, uint8_t *, uint64_t *);
// list: n + 1 words (the deferred items' indices, then their count)
hipError_t verify_deferred(hipStream_t, uint64_t, uint32_t *, const uint32_t *, const uint32_t *, const uint32_t *,
                           const uint8_t *, const uint8_t *, const uint32_t *, const uint32_t *, const uint32_t *,
                           const uint32_t *, const uint32_t *, uint8_t *, uint64_t *);
hipError_t verify_qf(hipStream_t, int, uint64_t, uint64_t, uint64_t, const uint32_t *, const uint32_t *,
                     const uint32_t *, const uint8_t *, const uint8_t *, const uint32_t *, const uint32_t *,
                     const uint64_t *, uint32_t *);
hipError_t verify_gf(hipStream_t, uint64_t, uint64_t, uint64_t, const uint32_t *, const uint32_t *, const uint32_t *,
                     const uint8_t *, const uint8_t *, const uint32_t *, const uint32_t *, const uint32_t *,
                     const uint32_t *, const uint32_t *, uint8_t *, uint64_t *);
hipError_t verify_g(hipStream_t, uint64_t, uint64_t, uint64_t, const uint32_t *, const uint32_t *, const uint32_t *,
                    const uint8_t *, const uint8_t *, const uint32_t *, const uint32_t *, const uint32_t *, uint32_t *,
                    const uint32_t *, uint32_t *, bool split);
hipError_t verify_q(hipStream_t, int, uint64_t, uint64_t, uint64_t, const uint32_t *, const uint32_t *,
                    const uint32_t *, const uint8_t *, const uint8_t *, const uint32_t *, const uint32_t *,
                    const uint64_t *, const uint32_t *, uint8_t *, uint64_t *);
hipError_t verify_small(hipStream_t, uint32_t n_items, const uint8_t *dig, const uint8_t *key_bytes,
                        const uint64_t *key_off, const uint32_t *item_msg, const uint32_t *item_key,
                        const uint8_t *r_be, const uint8_t *s_be, const uint8_t *pre, const uint64_t *kc_tabs,
                        const uint32_t *g_table, uint8_t *status, uint64_t *stamps, const uint32_t *rec,
                        uint64_t *clk);
hipError_t verify_generic(hipStream_t, uint64_t, uint64_t, uint64_t, const uint32_t *, const uint32_t *,
                          const uint32_t *, const uint8_t *, const uint8_t *, const uint32_t *, const uint32_t *,
                          const uint32_t *, const uint32_t *, const uint32_t *, uint8_t *, uint64_t *);
}  // namespace bvk

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes);
  void release();
  template <class T>
  T *as() const {
    return (T *)p;
  }
};

struct PinnedBuf {
  void *p = nullptr;
  size_t cap = 0;
  unsigned flags = hipHostMallocDefault;  // hipHostMalloc flags of the next allocation
  hipError_t ensure(size_t bytes);
  void release();
};

// ---------------------------------------------------------------------------
// host copy pool: parallel memcpy into / out of pinned staging
// ---------------------------------------------------------------------------
struct CopyPool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::vector<std::function<void()>> q;
  size_t pending = 0;
  bool stop = false;
  explicit CopyPool(int n) {
    for (int i = 0; i < n; i++)
      th.emplace_back([this]() {
        for (;;) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [this]() { return stop || !q.empty(); });
            if (stop && q.empty()) return;
            f = std::move(q.back());
            q.pop_back();
          }
          f();
          std::lock_guard<std::mutex> lk(mu);
          if (--pending == 0) done_cv.notify_all();
        }
      });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
  // fn(lo, hi) over [0, n) in `grain`-sized ranges on the pool and the
  // caller; returns false if any range returned false.
  bool parallel_for(uint64_t n, uint64_t grain, const std::function<bool(uint64_t, uint64_t)> &fn) {
    if (n <= grain || th.empty()) return fn(0, n);
    const uint64_t parts = (n + grain - 1) / grain;
    std::atomic<bool> ok{true};
    {
      std::lock_guard<std::mutex> lk(mu);
      for (uint64_t i = 1; i < parts; i++) {
        const uint64_t lo = i * grain, hi = std::min(n, lo + grain);
        q.push_back([&fn, &ok, lo, hi]() {
          if (!fn(lo, hi)) ok = false;
        });
        pending++;
      }
    }
    cv.notify_all();
    if (!fn(0, std::min(n, grain))) ok = false;
    std::unique_lock<std::mutex> lk(mu);
    done_cv.wait(lk, [this]() { return pending == 0; });
    return ok;
  }
  // dst <- src (n bytes); returns when done.  Small copies stay on the caller.
  void copy(void *dst, const void *src, size_t n) {
    constexpr size_t kPiece = 2ull << 20;
    if (n <= kPiece || th.empty()) {
      if (n) memcpy(dst, src, n);
      return;
    }
    const size_t pieces = (n + kPiece - 1) / kPiece;
    {
      std::lock_guard<std::mutex> lk(mu);
      for (size_t i = 1; i < pieces; i++) {
        const size_t o = i * kPiece, len = std::min(kPiece, n - o);
        q.push_back([=]() { memcpy((uint8_t *)dst + o, (const uint8_t *)src + o, len); });
        pending++;
      }
    }
    cv.notify_all();
    memcpy(dst, src, std::min(kPiece, n));  // the caller copies the first piece
    std::unique_lock<std::mutex> lk(mu);
    done_cv.wait(lk, [this]() { return pending == 0; });
  }
  // several copies at once (the pieces of one staging chunk), split into
  // 1 MB parts spread over the pool; returns when all are done
  struct Piece {
    void *dst;
    const void *src;
    size_t n;
  };
  void copy_many(const std::vector<Piece> &v) {
    constexpr size_t kPart = 1ull << 20;
    std::vector<Piece> parts;
    for (const Piece &p : v)
      for (size_t o = 0; o < p.n; o += kPart)
        parts.push_back({(uint8_t *)p.dst + o, (const uint8_t *)p.src + o, std::min(kPart, p.n - o)});
    if (parts.size() <= 1 || th.empty()) {
      for (const Piece &p : parts) memcpy(p.dst, p.src, p.n);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      for (size_t i = 1; i < parts.size(); i++) {
        const Piece p = parts[i];
        q.push_back([p]() { memcpy(p.dst, p.src, p.n); });
        pending++;
      }
    }
    cv.notify_all();
    memcpy(parts[0].dst, parts[0].src, parts[0].n);
    std::unique_lock<std::mutex> lk(mu);
    done_cv.wait(lk, [this]() { return pending == 0; });
  }
};


inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// timing / ordering events (see bv_read_timing)
enum {
  E_START, E_FORK, E_SHA, E_SCALAR, E_G, E_JOINED, E_END, E_KEYS, E_SINV,
  E_CALL, E_SMALL, E_HASH0, E_STAGED, E_HASHED, E_OUT, E_CSDONE, E_READY, E_KREADY, E_SREADY, E_RREADY, E_KCTAB, E_KDEC, E_KCDEC, E_SDEC, E_COUNT
};

constexpr uint32_t kKcMaxBatchKeys = 4096;  // key cache: batches with more keys use per-batch tables

struct KcSlot {
  std::string bytes;      // raw pubkey bytes (the cache key)
  void *table = nullptr;  // KC table (valid keys only)
  uint64_t last_use = 0;
  bool free = false;
};

// The streams a context runs on are per device and per PROCESS, shared by
// every ctx of that device (refcounted): HIP maps a process's streams onto
// GPU_MAX_HW_QUEUES hardware queues (4 by default) and two streams on one
// queue serialise.  A process holds one lane per work slot (the default
// stream of that slot's calls), the s^-1 stream and the high-priority keys
// stream — 3 normal-priority queues, so the caller's own stream (or torch's
// default) still gets a queue of its own; the copy stream is created only
// when a host-entry call first needs it.
struct bv_ctx {
  int device = 0;
  uint32_t flags = 0;
  static constexpr int kSlots = BV_SLOTS;
  hipStream_t lane[kSlots] = {};  // slot k's default stream
  hipStream_t stream = nullptr;   // lane[0]: host entry points, one-launch helpers
  hipStream_t kstream = nullptr;  // per-batch key tables (high priority)
  hipStream_t sstream = nullptr;  // batched s^-1 (+ key decode)
  hipStream_t cstream = nullptr;  // host-entry copies (bv_copy_stream: created on first use)
  hipStream_t last = nullptr;     // the stream of the last device call (bv_last_stream)
  std::mutex mu;
  std::string err;
  const uint32_t *g_table = nullptr;  // process-wide, per device (gtable_acquire)
  CopyPool *pool = nullptr;
  // host-entry staging: one layout in pinned memory and in HBM
  PinnedBuf pin_in, pin_out;
  PinnedBuf small_io;  // k_small's inputs and statuses, read / written by the kernel in place (mapped, coherent)
  uint8_t *small_io_host = nullptr, *small_io_dev = nullptr;  // small_io.p (of capacity small_io_cap) and its
  size_t small_io_cap = 0;                                      // device alias
  double wall_khz = 1e5;  // the device's constant clock (hipDeviceAttributeWallClockRate)
  DevBuf d_in;
  DevBuf d_stamps;  // BV_SMALL_STAMPS: k_small phase clocks (diagnostics)
  DevBuf d_sig;     // bv_verify_events with signature text: the decoded r, s, pre
  // host entry: messages longer than kHostHashLen hashed on the host (their
  // index and digest), uploaded beside the device hashing
  PinnedBuf pin_long;
  DevBuf d_long;
  // work buffers
  // Per-call work buffers in kSlots slots: device-resident calls rotate
  // through them, so a call waits only for the last user of its slot and
  // kSlots batches can be in flight, e.g. the next batch's key tables
  // building during this batch's k_verify_q when the caller alternates
  // streams.
  struct Slot {
    DevBuf digests, kstatus, kxy, bases_jac, key_sub, key_pscr, key_table, scratch, u12, rg, status, bits;
    DevBuf kc_tabs;          // key-cache table address per batch key
    PinnedBuf pin_small;     // its host staging
    bool kc_decoded = false; // bv_kc_prepare already ran k_key_decode into kstatus / kxy on the call stream
    // key cache, partial batch: a few valid keys have no table; their items
    // are left BV_DEFERRED by the KC kernels and finished by bv_run_deferred
    bool kc_partial = false;
    bool glv_split = false;  // this call's u12 was filled by k_glv_split (k_verify_g forms only u1)
    DevBuf defer;  // the deferred items' indices, then their count
    // caller result ranges [lo, hi) of this slot's device calls that the
    // other slots' calls have not yet been ordered after (deduplicated)
    std::vector<std::array<uintptr_t, 6>> uncovered;
    hipEvent_t ev[E_COUNT] = {};  // the slot's call's fork/join and timing events
    hipEvent_t done = nullptr;  // end of the last call that used this slot
    bool has_done = false;
  };
  Slot slot[kSlots];
  int cur = 0;
  Slot &S() { return slot[cur]; }
  std::vector<hipEvent_t> chunk_ev;
  hipEvent_t ev_done = nullptr;  // end of the last call's device work (both slots: bv_wait_all)
  hipEvent_t ev_host = nullptr;  // host waits on this ctx's own work on a shared lane (bv_host_wait)
  bool has_done = false;
  bool table_mode = false;
  int key_w = 0;  // 8, 12 or 20 (KC) in table mode
  bv_timing timing = {};
  // key cache (BV_F_KEY_CACHE, bv_keycache.cpp)
  std::unordered_map<std::string, int> kc_index;  // keys whose table build has been enqueued
  std::vector<KcSlot> kc_slots;
  std::unordered_set<std::string> kc_registered;  // bv_kc_register: the validator set
  std::unordered_map<std::string, uint32_t> kc_seen;  // valid keys without a table: batches seen (bounded)
  std::unordered_set<std::string> kc_bad;  // 65-byte 0x04 keys off the curve (bounded)
  uint32_t kc_admit = 2;                   // batches before an unregistered valid key gets a table
  bool kc_partial_on = false;              // BV_KC_PARTIAL=1: partial mode (bv_kc_prepare; off: measured slower)
  int kc_fail_alloc = 0, kc_fail_build = 0;  // fault injection (BV_KC_FAIL), tests only
  uint64_t kc_allocs = 0, kc_build_calls = 0;
  uint64_t kc_clock = 0, kc_bytes = 0, kc_budget = 0;
  DevBuf kc_kxy, kc_btabs;
  // bv_verify_events: body lengths, parent-hex positions, offsets, bodies
  DevBuf ev_iota;
  HostDagScratch dag_scratch;  // in-batch DAG batches: bodies built and hashed on the host (hostdag.cpp)
  // A/B knobs, read once at bv_create (never per call): host-entry message
  // chunk (BV_HOST_CHUNK_MB, >= 1 MB), event staging chunk (BV_EV_CHUNK_MB,
  // 0 = one chunk; chunks hold >= 256 events), bulk events' verify beside the next chunk
  // (BV_EV_VERIFY_STREAM=0: on the main stream)
  // small host batches through k_small (BV_SMALL=0: the bulk pipeline);
  // host entries sum the key part of every item before the messages land
  // (BV_QFIRST=0: G part first, as device-resident batches)
  uint64_t host_msg_chunk = 64ull << 20, ev_chunk = 64ull << 20;
  bool ev_split_verify = true, small_path = true, qfirst = true;
  // host entries' digests to the host (BV_EV_D2H): 1 = one copy per hashed
  // chunk, 0 = one copy after the last chunk, 2 = bulk events only: each
  // chunk's copy by SDMA on the copy stream behind the next chunk's H2D
  // (profiles/r05_ab_ev_qfirst.log: 5.42-5.49 against 5.16-5.28 ms; stores
  // by the hashing kernel through the pinned buffer's alias: no better)
  int ev_d2h = 1;
  int ev_tail = 0;  // bulk events' chunk plan (BV_EV_TAIL): 0 equal, 1 halving, 2 equal + one small last chunk
  uint64_t table_min_items = 8;    // per-batch tables (not the generic path) from this many items per key
  uint64_t table_min_items_many = 48;  // the same above kManyKeys keys
  uint64_t k12_min_items = 8192;  // per-batch K12 (not K8) tables from this many items per key
  bool small_stamps = false;      // BV_SMALL_STAMPS=1: print k_small's phase clocks to stderr
  bool host_stamps = false;       // BV_HOST_STAMPS=1: print the host entry's phases to stderr
  bool glv_in_sstream = true;     // BV_GLV_SSTREAM (A/B): device entry's GLV split in k_glv_split
  uint32_t host_scalar_max = 16;  // BV_HOST_SCALARS: k_small batches up to this many items may get host
                                  // item records (hostscalar.h; 0: the device inverts every item)
  std::vector<HostRecItem> rec_items;  // (their inputs, reused across calls)
  uint64_t small_max = 256;       // k_small for batches of at most this many items and messages (BV_SMALL_MAX)
  uint64_t small_warm_max = 1024;  // k_small for batches whose keys are all cached (BV_SMALL_WARM_MAX)
  uint32_t lat_table_keys = 256;  // latency rule: K8 tables for batches of <= 4096 items from up to this many keys (BV_LAT_TABLE_KEYS)
};

// one in-flight host-entry call (bv_host_launch -> bv_host_finish)
struct bv_host_call {
  std::chrono::steady_clock::time_point t0;
  float ms_prep = 0;
  uint8_t *pout = nullptr;
  size_t o_st = 0, o_bits = 0;
  bool direct_in = false;                          // message bytes DMA'd from the caller's pinned buffer
  bool direct_hash = false, direct_status = false;  // results DMA'd into the caller's pinned buffers
  double h_call = -1;                               // (BV_HOST_STAMPS) host ms when E_CALL was first seen done
};
bool bv_is_pinned(const void *p, size_t n);  // [p, p+n) inside one bv_host_alloc block

int bv_fail(bv_ctx *c, int code, const char *what, hipError_t e = hipSuccess);
hipStream_t bv_copy_stream(bv_ctx *ctx);   // the device's copy stream (created on first use; nullptr on failure)
// After a failed call: wait until nothing the call may have enqueued on the
// ctx's streams (and on `st`) is still running, so no slot keeps orphaned
// kernels that a later call would not wait for.  Returns `rc`.
int bv_drain(bv_ctx *ctx, hipStream_t st, int rc);
int bv_wait_all(bv_ctx *ctx);              // host: every call's device work has finished
int bv_mark_done(bv_ctx *ctx, hipStream_t st);
// Wait on the host for the work this ctx has enqueued on `st` so far (an
// event, not hipStreamSynchronize: the lanes are shared with other contexts)
hipError_t bv_host_wait(bv_ctx *ctx, hipStream_t st);
// Next slot for a device call writing `res`: st waits for the slot's last
// call, and for the other slot's last call when their result ranges overlap.
int bv_slot_begin(bv_ctx *ctx, hipStream_t st, const bv_batch *b, const bv_result *res);  // record the end of this call (its slot and ev_done)
int bv_validate_host_batch(bv_ctx *ctx, const bv_batch *b);
int bv_run_device(bv_ctx *ctx, const bv_batch *b, uint8_t *d_msg_hash, uint8_t *d_status, uint64_t *d_bits,
                  hipStream_t st, bool hashed, bool kc);
// split_ok: r is in HBM by s_ready too, so u2's GLV split may run on the
// s^-1 stream (k_glv_split) instead of in k_verify_g (the device entry)
int bv_run_keys(bv_ctx *ctx, const bv_batch *b, hipEvent_t keys_ready, hipEvent_t s_ready, bool kc,
                bool split_ok = false);
struct bv_out {  // device outputs of one verify
  uint32_t *dig = nullptr;
  uint8_t *status = nullptr;
  uint64_t *bits = nullptr;
};
int bv_out_bufs(bv_ctx *ctx, const bv_batch *b, uint8_t *d_msg_hash, uint8_t *d_status, uint64_t *d_bits,
                bool hashed, bv_out *o);
int bv_launch_items(bv_ctx *ctx, const bv_batch *b, const bv_out &o, hipStream_t st, bool kc, uint64_t lo,
                    uint64_t hi, int part);
// Host entry points: items verified in order on `st` as their messages get
// hashed (after bv_run_keys); upto(end) launches items [done, end), end a
// multiple of 64 or n_items.  The first launch orders `st` after s^-1 and
// the key tables.
struct bv_item_pipe {
  bv_ctx *ctx;
  const bv_batch *b;
  bv_out o;
  hipStream_t st;
  bool kc;
  bool qf = false;  // key part launched for every item (key_part): upto runs k_verify_gf
  uint64_t done = 0;
  // table mode, BV_QFIRST: R_Q of every item on `ks` after s^-1, the key
  // tables and `ready` (r and the item keys in HBM); the first upto orders
  // `st` after it.  Key cache: also after the call's kc_prepare work on
  // ctx->stream (kc_tabs), so call it right after bv_run_keys.
  int key_part(hipStream_t ks, hipEvent_t ready);
  int upto(uint64_t end);
  int finish();  // the rest, and the timing events even when there are no items
};
int bv_run_verify(bv_ctx *ctx, const bv_batch *b, uint8_t *d_msg_hash, uint8_t *d_status, uint64_t *d_bits,
                  hipStream_t st, bool hashed, bool kc);
// key cache, partial batch (kc_partial): the BV_DEFERRED items by the
// generic per-lane path, on `st` after the call's last verify kernel
int bv_run_deferred(bv_ctx *ctx, const bv_batch *b, const bv_out &o, hipStream_t st);
// the batch's item -> key map for the partial-mode item bound (host copy,
// or the device one, copied back only when the batch has table-less keys)
struct bv_kc_items {
  uint64_t n_items = 0;
  const uint32_t *h_item_key = nullptr;
  const uint32_t *d_item_key = nullptr;
};
int bv_kc_prepare(bv_ctx *ctx, uint32_t n_keys, const uint8_t *hkb, const uint64_t *hko, const uint8_t *dkb,
                  const uint64_t *dko, hipStream_t st, bool *use, bool force_build = false,
                  const bv_kc_items *items = nullptr);
uint32_t bv_kc_lookup(bv_ctx *ctx, uint32_t n_keys, const uint8_t *hkb, const uint64_t *hko, uint64_t *tabs);
bool bv_kc_all_cached(bv_ctx *ctx, uint32_t n_keys, const uint8_t *hkb, const uint64_t *hko);
void bv_kc_init(bv_ctx *ctx);     // budget, admission and fault-injection settings (bv_create)
void bv_kc_release(bv_ctx *ctx);  // free every cached table (bv_destroy, after all calls finished)
// `res` (may be null): the caller's result buffers, written by DMA directly
// when they are bv_host_alloc memory (else bv_host_finish copies them).
int bv_host_launch(bv_ctx *ctx, const bv_batch *b, bv_host_call *call, const bv_result *res = nullptr);
int bv_host_finish(bv_ctx *ctx, const bv_batch *b, bv_result *res, bv_host_call *call, bool bits_out);
void bv_read_timing(bv_ctx *ctx);
