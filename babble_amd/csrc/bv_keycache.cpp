// bv_keycache.cpp — the key cache of a bv_ctx (BV_F_KEY_CACHE): per-validator
// KC tables (22-bit signed GLV windows, 805 MB each) kept in HBM across calls,
// keyed by the raw pubkey bytes.  Babble's validator set is stable
// (src/peers/peer_set.go), so the tables of the PeerSet's keys are built once
// and every later batch of their events skips the per-batch table build.
//
// Invariants:
//  * kc_index maps a key ONLY to a slot whose table build has been enqueued
//    successfully on the call's stream (and every later call on the ctx is
//    ordered after that stream's work).  A call that fails part-way — a
//    table hipMalloc, a scratch allocation or a build launch — frees and
//    unindexes every slot it allocated, so no later call can hit an unbuilt
//    table.
//  * Admission: a valid key gets a table when it is registered
//    (bv_kc_register: the PeerSet) or once it has been seen in kc_admit
//    batches (default 2).  Registered tables are never evicted to make room
//    for unregistered keys.  Keys that are malformed by their form (length !=
//    65 or prefix != 0x04) are never remembered; 65-byte keys found off the
//    curve and valid keys waiting for admission are remembered in two sets of
//    at most kKcMemoMax entries each (cleared when full), so attacker-chosen
//    keys (processJoinRequest, src/node/node_rpc.go:250-260) bound host memory
//    and cannot evict a validator's table.
//  * Key statuses never come from the cache: every batch runs k_key_decode
//    (the product's elliptic.Unmarshal), so a cached table is only ever read
//    for a key whose batch decode says KS_OK.
//  * Fault injection for tests (BV_KC_FAIL="alloc:N" or "build:N", read once
//    at bv_create): the N-th KC table allocation / build launch of the ctx
//    fails once.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "bv_internal.h"

#define HIPCHK(expr, code, what)                               \
  do {                                                         \
    hipError_t _e = (expr);                                    \
    if (_e != hipSuccess) return bv_fail(ctx, code, what, _e); \
  } while (0)

namespace {
constexpr uint64_t kKcTableBytes = BV_KCTABLE_U32 * 4;  // 805 MB per cached key
constexpr uint64_t kKcSubBytes = BV_KCSUB_U32 * 4;
constexpr uint32_t kKcBases = 22;       // bases_jac allocation per key (>= BV_KCNSUB)
constexpr uint32_t kKcBuildGroup = 8;   // keys per KC build launch (pscr: 403 MB per key)
constexpr size_t kKcMemoMax = 4096;     // entries of kc_seen / kc_bad
constexpr uint64_t kKcPartialRatio = 16;  // partial batches: at most 1 valid key in 16 without a table

bool key_form_ok(const uint8_t *p, uint64_t len) { return len == 65 && p[0] == 4; }

template <class Set>
void memo_insert(Set &s, const std::string &k) {
  if (s.size() >= kKcMemoMax) s.clear();  // bounded: forget everything rather than grow
  s.insert(k);
}
}  // namespace

void bv_kc_init(bv_ctx *ctx) {
  double gb = 96.0;  // 119 KC tables: C5's 100 validators fit
  if (const char *s = getenv("BV_KEY_CACHE_GB")) gb = atof(s);
  ctx->kc_budget = (uint64_t)(std::max(gb, 0.0) * 1e9);
  if (const char *s = getenv("BV_KC_ADMIT")) ctx->kc_admit = (uint32_t)std::max(1, atoi(s));
  if (const char *s = getenv("BV_KC_PARTIAL")) ctx->kc_partial_on = atoi(s) != 0;
  if (const char *s = getenv("BV_KC_FAIL")) {
    int n = 0;
    if (sscanf(s, "alloc:%d", &n) == 1) ctx->kc_fail_alloc = n;
    else if (sscanf(s, "build:%d", &n) == 1) ctx->kc_fail_build = n;
  }
}

void bv_kc_release(bv_ctx *ctx) {
  for (auto &s : ctx->kc_slots)
    if (s.table) (void)hipFree(s.table);
  ctx->kc_slots.clear();
  ctx->kc_index.clear();
  ctx->kc_bytes = 0;
}

static hipError_t kc_table_alloc(bv_ctx *ctx, void **p) {
  if (++ctx->kc_allocs == (uint64_t)ctx->kc_fail_alloc) return hipErrorOutOfMemory;  // injected
  hipError_t e = hipMalloc(p, kKcTableBytes);
  if (e != hipSuccess) (void)hipGetLastError();
  return e;
}

// Resolves the batch's keys against the cache.  On BV_OK with *use = true the
// slot's kc_tabs holds one table address per batch key (null for keys whose
// decode is not KS_OK, never read) and every valid key has a built table;
// *use = false sends the batch down the per-batch table path (too many keys,
// a valid key not admitted yet, budget or HBM exhausted).  `force_build`
// (bv_kc_register) builds the admitted keys even when the batch itself could
// not use the cache.  hkb/hko: host copies of the key bytes; dkb/dko: device.
int bv_kc_prepare(bv_ctx *ctx, uint32_t n_keys, const uint8_t *hkb, const uint64_t *hko, const uint8_t *dkb,
                  const uint64_t *dko, hipStream_t st, bool *use, bool force_build, const bv_kc_items *items) {
  *use = false;
  ctx->S().kc_decoded = false;
  ctx->S().kc_partial = false;
  if (n_keys == 0 || n_keys > kKcMaxBatchKeys) return BV_OK;
  if (ctx->S().has_done)  // the slot's pin_small may still feed its previous (async) call
    HIPCHK(hipEventSynchronize(ctx->S().done), BV_E_LAUNCH, "sync slot");
  const uint64_t clock = ++ctx->kc_clock;
  std::vector<int> slot_of(n_keys, -1);
  std::vector<uint32_t> alias(n_keys);  // a repeated key -> its first index in the batch
  std::unordered_map<std::string, uint32_t> first;
  std::vector<uint32_t> unknown, admit;
  std::vector<uint8_t> is_blocked(n_keys, 0);  // per batch key (first occurrence): valid, no table, not admitted
  bool blocked = false;
  uint32_t n_blocked = 0;  // distinct valid keys without a table that may not get one yet
  uint32_t hits = 0;
  auto key_of = [&](uint32_t k) { return std::string((const char *)hkb + hko[k], (size_t)(hko[k + 1] - hko[k])); };
  auto admitted = [&](const std::string &key, uint32_t seen) {
    return ctx->kc_registered.count(key) != 0 || seen >= ctx->kc_admit;
  };
  for (uint32_t k = 0; k < n_keys; k++) {
    alias[k] = k;
    if (!key_form_ok(hkb + hko[k], hko[k + 1] - hko[k])) continue;  // malformed by form: no table, no memo
    const std::string key = key_of(k);
    auto f = first.emplace(key, k);
    if (!f.second) {
      alias[k] = f.first->second;
      continue;
    }
    auto it = ctx->kc_index.find(key);
    if (it != ctx->kc_index.end()) {
      slot_of[k] = it->second;
      ctx->kc_slots[it->second].last_use = clock;
      hits++;
      continue;
    }
    if (ctx->kc_bad.count(key)) continue;
    auto s = ctx->kc_seen.find(key);
    if (s != ctx->kc_seen.end()) {
      if (admitted(key, ++s->second)) admit.push_back(k);
      else blocked = true, n_blocked++, is_blocked[k] = 1;
      continue;
    }
    unknown.push_back(k);
  }
  if (!unknown.empty()) {
    // classify the new 65-byte keys: k_key_decode on the device (the product
    // path of elliptic.Unmarshal), one small synchronous copy back
    HIPCHK(ctx->S().kstatus.ensure(n_keys), BV_E_OOM, "alloc kstatus");
    HIPCHK(ctx->S().kxy.ensure((uint64_t)n_keys * 64), BV_E_OOM, "alloc kxy");
    HIPCHK(bvk::key_decode(st, n_keys, dkb, dko, ctx->S().kstatus.as<uint8_t>(), ctx->S().kxy.as<uint32_t>()),
           BV_E_LAUNCH, "k_key_decode");
    HIPCHK(hipEventRecord(ctx->S().ev[E_KCDEC], st), BV_E_LAUNCH, "event");
    std::vector<uint8_t> kst(n_keys);
    HIPCHK(hipMemcpyAsync(kst.data(), ctx->S().kstatus.p, n_keys, hipMemcpyDeviceToHost, st), BV_E_LAUNCH, "d2h kst");
    HIPCHK(bv_host_wait(ctx, st), BV_E_LAUNCH, "sync");
    ctx->S().kc_decoded = true;  // this batch's statuses and points are in the slot (bv_run_keys reuses them)
    for (uint32_t k : unknown) {
      const std::string key = key_of(k);
      if (kst[k] != KS_OK) {
        memo_insert(ctx->kc_bad, key);
        continue;
      }
      if (ctx->kc_seen.size() >= kKcMemoMax) ctx->kc_seen.clear();
      ctx->kc_seen[key] = 1;
      if (admitted(key, 1)) admit.push_back(k);
      else blocked = true, n_blocked++, is_blocked[k] = 1;
    }
  }
  // Every return below that leaves *use false after this call's k_key_decode
  // was launched on `st` waits for it first: the per-batch path then decodes
  // the batch again on the s^-1 stream into the same buffers.
  auto bail = [&]() -> int {
    ctx->S().kc_partial = false;
    ctx->timing.kc_hits = hits;
    ctx->timing.kc_builds = 0;
    ctx->timing.kc_keys = (uint32_t)ctx->kc_index.size();
    if (ctx->S().kc_decoded) {
      ctx->S().kc_decoded = false;
      if (bv_host_wait(ctx, st) != hipSuccess) return bv_fail(ctx, BV_E_LAUNCH, "sync", hipGetLastError());
    }
    return BV_OK;
  };
  // A valid key without a table: when such keys are few against the batch's
  // cached / admitted keys (at most 1 in kKcPartialRatio), the batch keeps
  // the cache and only their items take the generic path afterwards
  // (bv_run_deferred; ADVICE r4: a fresh key in every batch used to send the
  // whole batch, cached validators included, to the per-batch tables);
  // otherwise the per-batch path.  The deferred items run the per-lane
  // generic path after the batch's last verify kernel (a ~2.6 ms serial
  // chain of 128 doublings per lane), so they are bounded by ITEM count too
  // (ADVICE r5): when the table-less keys carry more than 1 item in
  // kKcPartialRatio, the per-batch tables take the batch.
  // Partial mode is OFF by default (BV_KC_PARTIAL=1 turns it on): measured
  // with 1 fresh key of 20 (profiles/r06_ab_partial.log), its deferred tail
  // costs +2.4 ms (20k-400k events) to +3 ms (1M) over the full key cache,
  // while the per-batch tables cost +0.2-0.3 ms, so a fresh key now sends
  // the batch to the per-batch tables.
  if (blocked && !force_build && !ctx->kc_partial_on) return bail();
  if (blocked && !force_build) {
    const uint64_t tabled = hits + admit.size();
    if (tabled == 0 || (uint64_t)n_blocked * kKcPartialRatio > tabled + n_blocked) return bail();
    if (items && items->n_items) {
      std::vector<uint32_t> keys;  // the caller's item -> key map, on the host
      const uint32_t *ik = items->h_item_key;
      if (!ik) {  // (device entry) one copy, only on this rare path
        keys.resize(items->n_items);
        HIPCHK(hipMemcpyAsync(keys.data(), items->d_item_key, items->n_items * 4, hipMemcpyDeviceToHost, st),
               BV_E_LAUNCH, "d2h item_key");
        HIPCHK(bv_host_wait(ctx, st), BV_E_LAUNCH, "sync");
        ik = keys.data();
      }
      uint64_t deferred = 0;
      for (uint64_t i = 0; i < items->n_items; i++) {
        const uint32_t k = ik[i];
        deferred += k < n_keys && is_blocked[alias[k]];
      }
      if (deferred * kKcPartialRatio > items->n_items) return bail();
    }
    ctx->S().kc_partial = true;
  }

  // Registration builds as many registered keys as the budget holds (in the
  // caller's order); the rest stay uncached (timing.kc_keys tells).  A
  // batch whose own keys alone exceed the budget takes the per-batch path.
  const uint64_t fit = ctx->kc_budget / kKcTableBytes;
  if (admit.size() > fit) {
    if (!force_build) return bail();
    admit.resize(fit);
  }
  uint32_t builds = 0;
  if (!admit.empty()) {
    if (!ctx->S().kc_decoded) {  // the admitted keys' points: decode the batch now
      HIPCHK(ctx->S().kstatus.ensure(n_keys), BV_E_OOM, "alloc kstatus");
      HIPCHK(ctx->S().kxy.ensure((uint64_t)n_keys * 64), BV_E_OOM, "alloc kxy");
      HIPCHK(bvk::key_decode(st, n_keys, dkb, dko, ctx->S().kstatus.as<uint8_t>(), ctx->S().kxy.as<uint32_t>()),
             BV_E_LAUNCH, "k_key_decode");
      HIPCHK(hipEventRecord(ctx->S().ev[E_KCDEC], st), BV_E_LAUNCH, "event");
      ctx->S().kc_decoded = true;  // ordered before the builds and the verify on `st`; sstream waits (bv_run_keys)
    }
    const uint64_t need = (uint64_t)admit.size() * kKcTableBytes;
    bool all_registered = true;
    for (uint32_t k : admit) all_registered = all_registered && ctx->kc_registered.count(key_of(k));
    // evict least-recently-used tables this batch does not use: unregistered
    // keys first; a registered key's table only to make room for registered keys
    while (ctx->kc_bytes + need > ctx->kc_budget) {
      int victim = -1;
      bool victim_reg = true;
      for (size_t i = 0; i < ctx->kc_slots.size(); i++) {
        const auto &s = ctx->kc_slots[i];
        if (s.free || !s.table || s.last_use == clock) continue;
        const bool reg = ctx->kc_registered.count(s.bytes) != 0;
        if (reg && !all_registered) continue;
        if (victim < 0 || (victim_reg && !reg) ||
            (victim_reg == reg && s.last_use < ctx->kc_slots[victim].last_use)) {
          victim = (int)i;
          victim_reg = reg;
        }
      }
      if (victim < 0) return bail();
      if (bv_wait_all(ctx) != BV_OK) return BV_E_LAUNCH;  // no call in flight may still read it
      auto &s = ctx->kc_slots[victim];
      HIPCHK(hipFree(s.table), BV_E_LAUNCH, "free cached table");
      ctx->kc_index.erase(s.bytes);
      s = KcSlot{};
      s.free = true;
      ctx->kc_bytes -= kKcTableBytes;
    }
    // Allocate this call's slots.  They are indexed only after their build
    // is enqueued; `rollback` frees them on any failure.
    std::vector<int> fresh;
    bool launched = false;
    auto rollback = [&]() {
      if (launched) (void)bv_host_wait(ctx, st);  // enqueued builds may still write the tables
      for (int si : fresh) {
        auto &s = ctx->kc_slots[si];
        if (s.table) {
          (void)hipFree(s.table);
          ctx->kc_bytes -= kKcTableBytes;
        }
        s = KcSlot{};
        s.free = true;
      }
      (void)hipGetLastError();
    };
    for (uint32_t k : admit) {
      int si = -1;
      for (size_t i = 0; i < ctx->kc_slots.size(); i++)
        if (ctx->kc_slots[i].free) {
          si = (int)i;
          break;
        }
      if (si < 0) {
        ctx->kc_slots.emplace_back();
        si = (int)ctx->kc_slots.size() - 1;
      }
      auto &s = ctx->kc_slots[si];
      s = KcSlot{};
      s.bytes = key_of(k);
      s.last_use = clock;
      fresh.push_back(si);
      if (kc_table_alloc(ctx, &s.table) != hipSuccess) {
        s.table = nullptr;
        rollback();
        return bail();  // HBM exhausted: per-batch path for this call, nothing indexed
      }
      ctx->kc_bytes += kKcTableBytes;
      slot_of[k] = si;
    }
    // build the new tables, kKcBuildGroup keys per launch
    auto fail = [&](int code, const char *what, hipError_t e) {
      rollback();
      return bv_fail(ctx, code, what, e);
    };
    const uint32_t G = std::min<uint32_t>(kKcBuildGroup, (uint32_t)admit.size());
    hipError_t e;
    if ((e = ctx->kc_kxy.ensure((uint64_t)G * 64)) != hipSuccess ||
        (e = ctx->kc_btabs.ensure((uint64_t)G * 8)) != hipSuccess ||
        (e = ctx->S().bases_jac.ensure((uint64_t)G * kKcBases * 96)) != hipSuccess ||
        (e = ctx->S().key_sub.ensure((uint64_t)G * kKcSubBytes)) != hipSuccess ||
        (e = ctx->S().key_pscr.ensure((uint64_t)G * bvk::kc_pscr_bytes())) != hipSuccess ||
        (e = ctx->S().pin_small.ensure(4096)) != hipSuccess)
      return fail(BV_E_OOM, "alloc KC build scratch", e);
    for (size_t g0 = 0; g0 < admit.size(); g0 += G) {
      const uint32_t n = (uint32_t)std::min<size_t>(G, admit.size() - g0);
      uint64_t *tabs = (uint64_t *)ctx->S().pin_small.p;
      if (launched && (e = bv_host_wait(ctx, st)) != hipSuccess) return fail(BV_E_LAUNCH, "sync", e);  // pin_small reuse
      for (uint32_t i = 0; i < n; i++) {
        const uint32_t k = admit[g0 + i];
        if ((e = hipMemcpyAsync(ctx->kc_kxy.as<uint8_t>() + 64ull * i, ctx->S().kxy.as<uint8_t>() + 64ull * k, 64,
                                hipMemcpyDeviceToDevice, st)) != hipSuccess)
          return fail(BV_E_LAUNCH, "gather kxy", e);
        tabs[i] = (uint64_t)(uintptr_t)ctx->kc_slots[slot_of[k]].table;
      }
      if ((e = hipMemcpyAsync(ctx->kc_btabs.p, tabs, n * 8ull, hipMemcpyHostToDevice, st)) != hipSuccess)
        return fail(BV_E_LAUNCH, "h2d tabs", e);
      launched = true;
      e = ++ctx->kc_build_calls == (uint64_t)ctx->kc_fail_build
              ? hipErrorLaunchFailure  // injected
              : bvk::build_kc(st, n, ctx->kc_kxy.as<uint32_t>(), nullptr, ctx->S().bases_jac.as<uint32_t>(),
                              ctx->S().key_sub.as<uint32_t>(), ctx->S().key_pscr.as<uint32_t>(),
                              ctx->kc_btabs.as<uint64_t>());
      if (e != hipSuccess) return fail(BV_E_LAUNCH, "KC key tables", e);
      builds += n;
    }
    // every build is enqueued on `st`, ahead of this call's verify and of
    // every later call (they order after this one): index the slots now
    for (int si : fresh) {
      ctx->kc_index[ctx->kc_slots[si].bytes] = si;
      ctx->kc_seen.erase(ctx->kc_slots[si].bytes);
    }
    if ((e = bv_host_wait(ctx, st)) != hipSuccess) return bv_fail(ctx, BV_E_LAUNCH, "sync", e);  // pin_small
  }
  for (uint32_t k = 0; k < n_keys; k++)
    if (alias[k] != k) slot_of[k] = slot_of[alias[k]];
  ctx->timing.kc_hits = hits;
  ctx->timing.kc_builds = builds;
  ctx->timing.kc_keys = (uint32_t)ctx->kc_index.size();
  if (blocked && !ctx->S().kc_partial) return BV_OK;  // force_build: the tables are built, this batch still takes the per-batch path
  // per-batch array: the table address of every batch key (null: no table;
  // only keys whose batch decode is not KS_OK have none, and theirs is never read)
  HIPCHK(ctx->S().pin_small.ensure((uint64_t)n_keys * 8 + 64), BV_E_OOM, "alloc pinned");
  uint64_t *tabs = (uint64_t *)ctx->S().pin_small.p;
  for (uint32_t k = 0; k < n_keys; k++)
    tabs[k] = slot_of[k] >= 0 ? (uint64_t)(uintptr_t)ctx->kc_slots[slot_of[k]].table : 0;
  HIPCHK(ctx->S().kc_tabs.ensure((uint64_t)n_keys * 8), BV_E_OOM, "alloc kc tabs");
  HIPCHK(hipMemcpyAsync(ctx->S().kc_tabs.p, tabs, n_keys * 8ull, hipMemcpyHostToDevice, st), BV_E_LAUNCH, "h2d tabs");
  *use = true;
  return BV_OK;
}

// Host-only lookup for the small-batch path (no device work, no sync): the
// table of every batch key that has one built, else 0.  Small batches never
// build tables (registration and bulk batches do).  Returns the hits.
uint32_t bv_kc_lookup(bv_ctx *ctx, uint32_t n_keys, const uint8_t *hkb, const uint64_t *hko, uint64_t *tabs) {
  uint32_t hits = 0;  // distinct keys, as bv_kc_prepare counts them
  const uint64_t clock = ++ctx->kc_clock;
  for (uint32_t k = 0; k < n_keys; k++) {
    tabs[k] = 0;
    if (!key_form_ok(hkb + hko[k], hko[k + 1] - hko[k])) continue;
    auto it = ctx->kc_index.find(std::string((const char *)hkb + hko[k], (size_t)(hko[k + 1] - hko[k])));
    if (it == ctx->kc_index.end()) continue;
    auto &slot = ctx->kc_slots[it->second];
    hits += slot.last_use != clock;
    slot.last_use = clock;
    tabs[k] = (uint64_t)(uintptr_t)slot.table;
  }
  return hits;
}

// Every well-formed key of the batch has a built table (host-only).
bool bv_kc_all_cached(bv_ctx *ctx, uint32_t n_keys, const uint8_t *hkb, const uint64_t *hko) {
  for (uint32_t k = 0; k < n_keys; k++) {
    if (!key_form_ok(hkb + hko[k], hko[k + 1] - hko[k])) continue;
    if (!ctx->kc_index.count(std::string((const char *)hkb + hko[k], (size_t)(hko[k + 1] - hko[k])))) return false;
  }
  return true;
}

extern "C" int bv_kc_register(bv_ctx *ctx, uint32_t n_keys, const uint8_t *key_bytes, const uint64_t *key_off) {
  if (!ctx || (n_keys && !key_off)) return BV_E_ARGS;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!(ctx->flags & BV_F_KEY_CACHE)) return bv_fail(ctx, BV_E_ARGS, "bv_kc_register needs BV_F_KEY_CACHE");
  if (n_keys > kKcMaxBatchKeys) return bv_fail(ctx, BV_E_ARGS, "more than 4096 registered keys");
  if (n_keys && key_off[0] != 0) return bv_fail(ctx, BV_E_ARGS, "key_off[0] != 0");
  for (uint32_t k = 0; k < n_keys; k++)
    if (key_off[k] > key_off[k + 1]) return bv_fail(ctx, BV_E_ARGS, "key_off not monotone");
  const uint64_t len = n_keys ? key_off[n_keys] : 0;
  if (len && !key_bytes) return bv_fail(ctx, BV_E_ARGS, "null key bytes");
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  ctx->kc_registered.clear();
  for (uint32_t k = 0; k < n_keys; k++)
    if (key_form_ok(key_bytes + key_off[k], key_off[k + 1] - key_off[k]))
      ctx->kc_registered.emplace((const char *)key_bytes + key_off[k], (size_t)(key_off[k + 1] - key_off[k]));
  ctx->timing = bv_timing{};
  if (ctx->kc_registered.empty()) return BV_OK;
  // the keys on the device (k_key_decode reads 64 bytes past the last one)
  if (bv_wait_all(ctx) != BV_OK) return BV_E_LAUNCH;
  hipStream_t st = ctx->stream;
  const size_t o_off = align256(len + 64), total = o_off + align256((n_keys + 1) * 8ull);
  HIPCHK(ctx->pin_in.ensure(total), BV_E_OOM, "alloc pinned staging");
  HIPCHK(ctx->d_in.ensure(total), BV_E_OOM, "alloc device staging");
  uint8_t *pin = (uint8_t *)ctx->pin_in.p, *dev = ctx->d_in.as<uint8_t>();
  if (len) memcpy(pin, key_bytes, len);
  memset(pin + len, 0, 64);
  memcpy(pin + o_off, key_off, (n_keys + 1) * 8ull);
  HIPCHK(hipMemcpyAsync(dev, pin, total, hipMemcpyHostToDevice, st), BV_E_LAUNCH, "h2d keys");
  ctx->cur = (ctx->cur + 1) % bv_ctx::kSlots;
  bool use = false;
  int rc = bv_kc_prepare(ctx, n_keys, key_bytes, key_off, dev, (const uint64_t *)(dev + o_off), st, &use, true);
  if (rc != BV_OK) return bv_drain(ctx, st, rc);
  rc = bv_mark_done(ctx, st);
  if (rc != BV_OK) return bv_drain(ctx, st, rc);
  HIPCHK(bv_host_wait(ctx, st), BV_E_LAUNCH, "sync");
  return BV_OK;
}
