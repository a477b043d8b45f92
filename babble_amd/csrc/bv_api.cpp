// bv_api.cpp — host side of libbabbleverify.so: the C ABI declared in
// include/babbleverify.h (single-device contexts; bv_group.cpp adds the
// multi-device group on top).
//
// One bv_ctx owns three HIP streams (main, keys, s^-1) plus a copy stream
// for the host entry point, growable device work buffers, pinned
// (hipHostMalloc) staging buffers, and optionally the key cache
// (BV_F_KEY_CACHE).  The generator table (geometry.h: 26-bit signed
// windows, 21.5 GB) is a per-process, per-device constant shared by every ctx.  There
// is no CPU fallback: a missing or non-gfx950 device is BV_E_NODEVICE.
//
// Host entry point (bv_verify_batch, what cgo calls): every input array is
// staged into one pinned buffer by a small thread pool and streamed to HBM on
// the copy stream in ~16 MB chunks; the message bytes go last, chunked on
// message boundaries, and each chunk is hashed (k_sha256 on the main stream)
// as soon as it lands, so hashing overlaps the PCIe transfer of the next
// chunk.  Digests are copied back as soon as hashing ends (overlapping the
// verify kernels), statuses and bits after the last kernel.
#include "bv_internal.h"
#include "hostscalar.h"
#include "hostsha.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <new>
#include <thread>

#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace {

constexpr uint64_t kGTableBytes = BV_GTABLE_U32 * 4;                       // 21.5 GB (geometry.h)
constexpr uint64_t kGSubBytes = BV_GSUB_U32 * 4;
constexpr uint64_t kGPrefixBytes = (uint64_t)BV_GPAIR_BLOCKS * 4096 * 32;  // one k_table_pair_g launch
constexpr uint64_t kKTableBytes = BV_KTABLE_U32 * 4;
constexpr uint64_t kK12TableBytes = BV_K12TABLE_U32 * 4;
constexpr uint64_t kK12SubBytes = BV_K12SUB_U32 * 4;
constexpr uint64_t kK12PrefixBytes = (uint64_t)BV_K12NWIN * BV_K12ENT * 32;  // one fe per entry
constexpr uint64_t kKSubBytes = BV_KSUB_U32 * 4;
constexpr uint64_t kKPrefixBytes = (uint64_t)BV_KNWIN * (1u << BV_KW) * 32;  // one fe per entry
constexpr uint32_t kBasesPerKey = 32;       // max(K8 32, K12 22, KC 12) bases per key
// Per-batch K12 (22 lookups per item) or K8 (32) tables.  K8 entries are
// chord sums of 4-bit sub-table points (k_table_pair_u, one field inversion
// per key), so a K8 key costs ~12x less to build than a K12 key; K12's
// cheaper lookups pay only from ctx->k12_min_items (8192, BV_K12_MIN_ITEMS)
// items per key, with at most kMaxK12Keys keys.  Same-box A/Bs, two batches
// in flight (profiles/r05_ab_k8_rule.log): 64 keys 16k / 125k / 1M events
// K8 34.4 / 236.6 / 438.0 against K12 31.1 / 213.8 / 489.4 M/s; 200 keys
// 50k / 200k / 1M 98.3 / 302.1 / 426.6 against 53.5 / 213.5 / 416.1;
// 1000 keys 1M 348.0 against 222.7.
constexpr uint32_t kMaxTableKeys = 8192;       // K8: 4 GiB of key tables
constexpr uint32_t kMaxK12Keys = 1024;         // K12: 2.8 GiB
// Table or generic: the generic path costs ~16.5 ns per item with a floor
// of ~1.2 ms per batch; the K8 build grows with the key count.  Up to
// kManyKeys keys tables win from 8 items per key (ctx->table_min_items;
// 1000 keys, 8k / 16k / 32k / 128k events: K8 8.7 / 17.0 / 34.0 / 127.0
// against generic 6.5 / 12.9 / 25.8 / 59.2 M/s), above it from 48
// (ctx->table_min_items_many; 2000 keys 32 / 64 per key: generic 46.0
// against 42.8, K8 82.2 against 59.2; 3000 keys 32 / 48 / 64 per key:
// generic 55.8 / 60.3 / 62.0 against K8 46.6 / 68.3 / 88.4;
// profiles/r05_ab_k8_rule.log, r05_ab_k8_rule2.log, r05_ab_k8_chord_1000.log).
constexpr uint32_t kManyKeys = 1024;
// Latency rule: a small batch is bound by its longest serial chain, not by
// total work.  The per-lane generic path runs 128 doublings AND ~128
// additions in one lane per item (~2.6 ms); the K8 tables cost one wave's
// 120 doublings per key plus the fills, so they finish first even at one
// item per key: up to 256 keys (1.85 ms; 0.8 ms at 32 keys), measured in
// profiles/r04_ab_lat_keys.log.  ctx->lat_table_keys (BV_LAT_TABLE_KEYS).
constexpr uint64_t kLatTableItems = 4096;
#ifndef BV_PREP_M
#define BV_PREP_M 16
#endif
constexpr uint32_t kPrepM = BV_PREP_M;         // items per s^-1 batch
constexpr uint32_t kRgWords = 33;              // R_G words per item (XYZZ + inf: verify_core.h RG_WORDS)
#ifndef BV_FUSED_KC
#define BV_FUSED_KC 1
#endif
constexpr bool kFusedKc = BV_FUSED_KC;         // key cache: one fused verify kernel (k_verify_gq)
constexpr size_t kChunk = 16ull << 20;         // host-entry staging / PCIe chunk
// message bytes hashed (and their items verified) per chunk: ctx->host_msg_chunk,
// 64 MB by default — it keeps each chunk's verify launches at full occupancy
// (1M C2 events from pinned arrays, same box: 16 / 64 / 128 MB = 15.0-15.7 /
// 11.0 / 10.9-11.0 ms per call; pageable 15.2 / 12.0 ms, tools/host_prof.py)
// host batches whose whole staging layout is at most this cross PCIe as ONE
// copy: each extra small H2D costs ~20 us of DMA latency on a lone call
constexpr size_t kSmallStage = 1ull << 20;
// Host entry: a message longer than this is hashed on the host (hostsha.cpp,
// the SHA extensions) instead of by one GPU lane — SHA-256 of one message is
// a serial chain, ~3.2 us a block on a lone lane against ~40 ns on a CPU
// core: the 54 KB anchor Frame of C5 (853 blocks) took 2.8 ms of device time
// on its lane (profiles/r04_bench_midround.json c5_fast_sync).
constexpr uint64_t kHostHashLen = 16 << 10;

}  // namespace

// ---------------------------------------------------------------------------
// buffers
// ---------------------------------------------------------------------------
hipError_t DevBuf::ensure(size_t bytes) {
  if (bytes <= cap) return hipSuccess;
  if (p) {
    hipError_t e = hipFree(p);
    if (e != hipSuccess) return e;
    p = nullptr;
    cap = 0;
  }
  size_t want = std::max(bytes, cap * 3 / 2);
  want = (want + 255) & ~(size_t)255;
  hipError_t e = hipMalloc(&p, want);
  if (e != hipSuccess) {
    p = nullptr;
    (void)hipGetLastError();
    return e;
  }
  cap = want;
  return hipSuccess;
}
void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
}
hipError_t PinnedBuf::ensure(size_t bytes) {
  if (bytes <= cap) return hipSuccess;
  if (p) {
    hipError_t e = hipHostFree(p);
    if (e != hipSuccess) return e;
    p = nullptr;
    cap = 0;
  }
  size_t want = std::max(bytes, cap * 3 / 2);
  want = (want + 4095) & ~(size_t)4095;
  hipError_t e = hipHostMalloc(&p, want, flags);
  if (e != hipSuccess) {
    p = nullptr;
    (void)hipGetLastError();
    return e;
  }
  cap = want;
  return hipSuccess;
}
void PinnedBuf::release() {
  if (p) (void)hipHostFree(p);
  p = nullptr;
  cap = 0;
}

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
int bv_fail(bv_ctx *c, int code, const char *what, hipError_t e) {
  if (c) {
    char buf[256];
    if (e != hipSuccess)
      snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    else
      snprintf(buf, sizeof buf, "%s", what);
    c->err = buf;
  }
  return code;
}

#define HIPCHK(expr, code, what)                               \
  do {                                                         \
    hipError_t _e = (expr);                                    \
    if (_e != hipSuccess) return bv_fail(ctx, code, what, _e); \
  } while (0)

// ---------------------------------------------------------------------------
// caller-visible pinned memory (bv_host_alloc): a host-entry call whose
// arrays live in it is DMA'd straight from them, without the staging copy
// ---------------------------------------------------------------------------
namespace {
std::mutex g_pin_mu;
std::map<uintptr_t, size_t> g_pinned;  // base -> bytes
}  // namespace

extern "C" int bv_host_alloc(size_t bytes, void **out) {
  if (!out) return BV_E_ARGS;
  *out = nullptr;
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess) {
    (void)hipGetLastError();
    return BV_E_OOM;
  }
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pinned[(uintptr_t)p] = bytes ? bytes : 1;
  *out = p;
  return BV_OK;
}

extern "C" void bv_host_free(void *p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pinned.find((uintptr_t)p);
    if (it == g_pinned.end()) return;  // not ours: ignored
    g_pinned.erase(it);
  }
  (void)hipHostFree(p);
}

// The pinned arena (babbleverify.h): blocks that outlive calls.
struct bv_arena {
  void *p[BV_ARENA_SLOTS] = {};
  size_t cap[BV_ARENA_SLOTS] = {};
};

extern "C" int bv_arena_create(bv_arena **out) {
  if (!out) return BV_E_ARGS;
  *out = new (std::nothrow) bv_arena();
  return *out ? BV_OK : BV_E_OOM;
}

extern "C" void bv_arena_destroy(bv_arena *a) {
  if (!a) return;
  for (void *p : a->p) bv_host_free(p);
  delete a;
}

// (diagnostics) the NUMA node of the page holding p (get_mempolicy
// MPOL_F_NODE | MPOL_F_ADDR), or of the calling thread's CPU when p is null;
// -1 when unknown
static int numa_node_of(const void *p) {
  int node = -1;
  if (!p) {
    unsigned cpu = 0, n = 0;
    return syscall(SYS_getcpu, &cpu, &n, nullptr) == 0 ? (int)n : -1;
  }
  const long MPOL_F_NODE_ = 1, MPOL_F_ADDR_ = 2;
  if (syscall(SYS_get_mempolicy, &node, nullptr, 0, p, MPOL_F_NODE_ | MPOL_F_ADDR_) != 0) return -1;
  return node;
}

extern "C" int bv_arena_reserve(bv_arena *a, uint32_t slot, size_t bytes, size_t keep, void **out, size_t *cap) {
  if (!a || !out || slot >= BV_ARENA_SLOTS || keep > a->cap[slot]) return BV_E_ARGS;
  if (bytes > a->cap[slot]) {
    const size_t nc = std::max(bytes, 2 * a->cap[slot]);
    void *np = nullptr;
    const int rc = bv_host_alloc(nc, &np);
    if (rc != BV_OK) return rc;
    if (keep) memcpy(np, a->p[slot], keep);
    bv_host_free(a->p[slot]);
    a->p[slot] = np;
    a->cap[slot] = nc;
  }
  *out = a->p[slot];
  if (cap) *cap = a->cap[slot];
  return BV_OK;
}

bool bv_is_pinned(const void *p, size_t n) {
  if (!p || !n) return false;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pinned.upper_bound((uintptr_t)p);
  if (it == g_pinned.begin()) return false;
  --it;
  return (uintptr_t)p + n <= it->first + it->second;
}

int bv_wait_all(bv_ctx *ctx) {
  for (auto &sl : ctx->slot)
    if (sl.has_done) HIPCHK(hipEventSynchronize(sl.done), BV_E_LAUNCH, "sync previous calls");
  for (auto &sl : ctx->slot) sl.uncovered.clear();
  return BV_OK;
}

int bv_slot_begin(bv_ctx *ctx, hipStream_t st, const bv_batch *b, const bv_result *res) {
  ctx->cur = (ctx->cur + 1) % bv_ctx::kSlots;
  bv_ctx::Slot &sl = ctx->S();
  if (sl.has_done) HIPCHK(hipStreamWaitEvent(st, sl.done, 0), BV_E_LAUNCH, "order after the slot's last call");
  // The caller's result buffers: a call writing buffers that a call still in
  // flight on another slot writes (e.g. the same DeviceBatch issued on two
  // streams) is ordered after that slot's last call, as if serial.
  const void *p[3] = {res->msg_hash, res->status, res->accept_bits};
  const uint64_t n[3] = {b->n_msgs * 32, b->n_items, (b->n_items + 63) / 64 * 8};
  std::array<uintptr_t, 6> r{};
  for (int i = 0; i < 3; i++)
    if (p[i] && n[i]) r[2 * i] = (uintptr_t)p[i], r[2 * i + 1] = (uintptr_t)p[i] + n[i];
  for (auto &other : ctx->slot) {
    if (&other == &sl) continue;
    bool overlap = other.uncovered.size() >= 8;
    for (const auto &u : other.uncovered)
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) overlap |= u[2 * j] < r[2 * i + 1] && r[2 * i] < u[2 * j + 1];
    if (overlap) {
      HIPCHK(hipStreamWaitEvent(st, other.done, 0), BV_E_LAUNCH, "order after an overlapping call");
      other.uncovered.clear();
    }
  }
  if (std::find(sl.uncovered.begin(), sl.uncovered.end(), r) == sl.uncovered.end()) sl.uncovered.push_back(r);
  return BV_OK;
}

hipError_t bv_host_wait(bv_ctx *ctx, hipStream_t st) {
  hipError_t e = hipEventRecord(ctx->ev_host, st);
  return e != hipSuccess ? e : hipEventSynchronize(ctx->ev_host);
}

int bv_mark_done(bv_ctx *ctx, hipStream_t st) {
  HIPCHK(hipEventRecord(ctx->S().done, st), BV_E_LAUNCH, "event");
  HIPCHK(hipEventRecord(ctx->ev_done, st), BV_E_LAUNCH, "event");
  ctx->S().has_done = true;
  ctx->has_done = true;
  return BV_OK;
}

static const uint8_t kGenerator[64] = {
    0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0, 0x62, 0x95, 0xCE, 0x87, 0x0B, 0x07,
    0x02, 0x9B, 0xFC, 0xDB, 0x2D, 0xCE, 0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98,
    0x48, 0x3A, 0xDA, 0x77, 0x26, 0xA3, 0xC4, 0x65, 0x5D, 0xA4, 0xFB, 0xFC, 0x0E, 0x11, 0x08, 0xA8,
    0xFD, 0x17, 0xB4, 0x48, 0xA6, 0x85, 0x54, 0x19, 0x9C, 0x47, 0xD0, 0x8F, 0xFB, 0x10, 0xD4, 0xB8};

extern "C" int bv_abi_version(void) { return BV_ABI_VERSION; }

extern "C" const char *bv_last_error(const bv_ctx *ctx) { return ctx ? ctx->err.c_str() : "null ctx"; }

// The generator table is a constant: one copy per device and process,
// shared by every context (refcounted), built on first use.
// T[j][d] = d 2^(BV_GW j) G, j < BV_GNWIN, 0 < d <= 2^(BV_GW-1) (signed, geometry.h);
// sub-tables and prefix scratch are freed after the build.
namespace {
struct GTableSlot {
  void *table = nullptr;
  int refs = 0;
};
std::mutex g_gtable_mu;
GTableSlot g_gtables[64];
}  // namespace

static const uint32_t *gtable_acquire(int device, hipStream_t st) {
  if (device < 0 || device >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_gtable_mu);
  GTableSlot &slot = g_gtables[device];
  if (slot.table) {
    slot.refs++;
    return (const uint32_t *)slot.table;
  }
  void *table = nullptr, *xy = nullptr, *bases = nullptr, *sub = nullptr, *pscr = nullptr;
  bool ok = hipMalloc(&table, kGTableBytes) == hipSuccess && hipMalloc(&xy, 64) == hipSuccess &&
            hipMalloc(&bases, BV_GNSUB * 96) == hipSuccess && hipMalloc(&sub, kGSubBytes) == hipSuccess &&
            hipMalloc(&pscr, kGPrefixBytes) == hipSuccess;
  if (ok) {
    uint32_t gxy[16];
    for (int half = 0; half < 2; half++)
      for (int i = 0; i < 8; i++) {
        const uint8_t *q = kGenerator + 32 * half + 4 * (7 - i);
        gxy[8 * half + i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
      }
    ok = hipMemcpyAsync(xy, gxy, sizeof gxy, hipMemcpyHostToDevice, st) == hipSuccess &&
         bvk::build_tables(st, 0, 1, (const uint32_t *)xy, nullptr, (uint32_t *)bases, (uint32_t *)sub,
                           (uint32_t *)pscr, (uint32_t *)table, 0) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
  }
  for (void *p : {xy, bases, sub, pscr})
    if (p) (void)hipFree(p);
  if (!ok) {
    if (table) (void)hipFree(table);
    (void)hipGetLastError();
    return nullptr;
  }
  slot.table = table;
  slot.refs = 1;
  return (const uint32_t *)table;
}

static void gtable_release(int device) {
  std::lock_guard<std::mutex> lk(g_gtable_mu);
  GTableSlot &slot = g_gtables[device];
  if (--slot.refs == 0) {
    (void)hipFree(slot.table);
    slot.table = nullptr;
  }
}

// Per-device, per-process stream set shared by every ctx (bv_internal.h).
namespace {
struct DevStreams {
  hipStream_t lane[BV_SLOTS] = {};
  hipStream_t kstream = nullptr, sstream = nullptr, cstream = nullptr;
  int refs = 0;
};
std::mutex g_streams_mu;
DevStreams g_streams[64];

void streams_destroy(DevStreams &d) {
  for (hipStream_t &s : d.lane)
    if (s) (void)hipStreamDestroy(s), s = nullptr;
  for (hipStream_t *s : {&d.kstream, &d.sstream, &d.cstream})
    if (*s) (void)hipStreamDestroy(*s), *s = nullptr;
}
}  // namespace

#ifndef BV_KPRIO
#define BV_KPRIO 1
#endif
#ifndef BV_SPRIO
#define BV_SPRIO 0
#endif

static int streams_acquire(bv_ctx *ctx) {
  if (ctx->device < 0 || ctx->device >= 64) return bv_fail(ctx, BV_E_NODEVICE, "device ordinal >= 64");
  std::lock_guard<std::mutex> lk(g_streams_mu);
  DevStreams &d = g_streams[ctx->device];
  if (d.refs == 0) {
    // the key-table stream runs a latency-bound chain (k_table_bases): give
    // it the higher priority so its waves are scheduled ahead of bulk kernels
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    bool ok = true;
    for (hipStream_t &s : d.lane) ok = ok && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipStreamCreateWithPriority(&d.sstream, hipStreamNonBlocking, BV_SPRIO ? hi : lo) == hipSuccess;
    ok = ok && hipStreamCreateWithPriority(&d.kstream, hipStreamNonBlocking, BV_KPRIO ? hi : lo) == hipSuccess;
    if (!ok) {
      (void)hipGetLastError();
      streams_destroy(d);
      return bv_fail(ctx, BV_E_NODEVICE, "hipStreamCreate");
    }
  }
  d.refs++;
  for (int k = 0; k < bv_ctx::kSlots; k++) ctx->lane[k] = d.lane[k];
  ctx->stream = d.lane[0];
  ctx->kstream = d.kstream;
  ctx->sstream = d.sstream;
  ctx->cstream = d.cstream;
  return BV_OK;
}

static void streams_release(bv_ctx *ctx) {
  if (!ctx->stream) return;
  std::lock_guard<std::mutex> lk(g_streams_mu);
  DevStreams &d = g_streams[ctx->device];
  if (--d.refs == 0) streams_destroy(d);
}

hipStream_t bv_copy_stream(bv_ctx *ctx) {
  if (ctx->cstream) return ctx->cstream;
  std::lock_guard<std::mutex> lk(g_streams_mu);
  DevStreams &d = g_streams[ctx->device];
  if (!d.cstream && hipStreamCreateWithFlags(&d.cstream, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    d.cstream = nullptr;
  }
  ctx->cstream = d.cstream;
  return ctx->cstream;
}

// After a failed call: wait for everything this ctx enqueued.  The streams
// are shared with the process's other contexts, so each wait is an event of
// the ctx's own recorded behind its work (bv_host_wait), not a stream
// synchronize that would also wait for other contexts' later work.
int bv_drain(bv_ctx *ctx, hipStream_t st, int rc) {
  for (hipStream_t s : {st, ctx->sstream, ctx->kstream, ctx->cstream})
    if (s && bv_host_wait(ctx, s) != hipSuccess) (void)hipStreamSynchronize(s);
  for (auto &sl : ctx->slot) sl.uncovered.clear();
  (void)hipGetLastError();
  return rc;
}

static int create_impl(bv_ctx *ctx) {
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  if (streams_acquire(ctx) != BV_OK) return BV_E_NODEVICE;
  for (auto &sl : ctx->slot)
    for (auto &e : sl.ev) HIPCHK(hipEventCreate(&e), BV_E_NODEVICE, "hipEventCreate");
  HIPCHK(hipEventCreateWithFlags(&ctx->ev_done, hipEventDisableTiming), BV_E_NODEVICE, "hipEventCreate");
  HIPCHK(hipEventCreateWithFlags(&ctx->ev_host, hipEventDisableTiming), BV_E_NODEVICE, "hipEventCreate");
  for (auto &sl : ctx->slot)
    HIPCHK(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming), BV_E_NODEVICE, "hipEventCreate");
  ctx->chunk_ev.resize(64);
  for (auto &e : ctx->chunk_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming), BV_E_NODEVICE, "event");
  {  // s_memrealtime's rate (k_small's own span; 100 MHz on gfx950)
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device) == hipSuccess && khz > 0)
      ctx->wall_khz = khz;
    (void)hipGetLastError();
  }
  ctx->g_table = gtable_acquire(ctx->device, ctx->stream);
  if (!ctx->g_table) return bv_fail(ctx, BV_E_OOM, "generator table (geometry.h, ~21.5 GB of HBM) build failed");
  const unsigned hw = std::thread::hardware_concurrency();
  int copy_threads = (int)std::min<unsigned>(hw ? hw - 1 : 0, 7);
  if (const char *s = getenv("BV_COPY_THREADS")) copy_threads = std::max(0, std::min(63, atoi(s)));  // (A/B knob)
  ctx->pool = new CopyPool(copy_threads);
  if (ctx->flags & BV_F_KEY_CACHE) bv_kc_init(ctx);
  // A/B knobs (bv_internal.h), read once here
  if (const char *s = getenv("BV_HOST_CHUNK_MB")) ctx->host_msg_chunk = (uint64_t)(std::max(1.0, atof(s)) * (1 << 20));
  if (const char *s = getenv("BV_EV_CHUNK_MB")) {
    const double mb = atof(s);
    ctx->ev_chunk = mb <= 0 ? 0 : std::max<uint64_t>(1, (uint64_t)(mb * (1 << 20)));  // >= 256 events a chunk anyway
  }
  if (const char *s = getenv("BV_EV_VERIFY_STREAM")) ctx->ev_split_verify = atoi(s) != 0;
  if (const char *s = getenv("BV_SMALL")) ctx->small_path = atoi(s) != 0;
  if (const char *s = getenv("BV_QFIRST")) ctx->qfirst = atoi(s) != 0;
  if (const char *s = getenv("BV_GLV_SSTREAM")) ctx->glv_in_sstream = atoi(s) != 0;
  if (const char *s = getenv("BV_EV_D2H")) ctx->ev_d2h = atoi(s);
  if (const char *s = getenv("BV_EV_TAIL")) ctx->ev_tail = atoi(s);
  if (const char *s = getenv("BV_SMALL_STAMPS")) ctx->small_stamps = atoi(s) != 0;
  if (const char *s = getenv("BV_HOST_STAMPS")) ctx->host_stamps = atoi(s) != 0;
  if (const char *s = getenv("BV_HOST_SCALARS")) ctx->host_scalar_max = (uint32_t)atoi(s);
  if (const char *s = getenv("BV_TABLE_MIN_ITEMS")) ctx->table_min_items = (uint64_t)std::max(1, atoi(s));
  if (const char *s = getenv("BV_TABLE_MIN_ITEMS_MANY")) ctx->table_min_items_many = (uint64_t)std::max(1, atoi(s));
  if (const char *s = getenv("BV_K12_MIN_ITEMS")) ctx->k12_min_items = (uint64_t)std::max(1, atoi(s));
  if (const char *s = getenv("BV_SMALL_WARM_MAX")) ctx->small_warm_max = (uint64_t)std::max(0, atoi(s));
  if (const char *s = getenv("BV_SMALL_MAX")) ctx->small_max = (uint64_t)std::max(0, atoi(s));
  if (const char *s = getenv("BV_FORCE_K8"))  // (A/B knob: as the BV_F_K8 flag)
    if (atoi(s) != 0) ctx->flags |= BV_F_K8;
  if (const char *s = getenv("BV_LAT_TABLE_KEYS")) ctx->lat_table_keys = (uint32_t)atoi(s);
  return BV_OK;
}

extern "C" int bv_create(bv_ctx **out, int device, uint32_t flags) {
  if (!out) return BV_E_ARGS;
  *out = nullptr;
  if (flags & ~BV_F_KNOWN) return BV_E_ARGS;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return BV_E_NODEVICE;
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) return BV_E_NODEVICE;
  }
  if (device >= ndev) return BV_E_NODEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return BV_E_NODEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return BV_E_NODEVICE;
  bv_ctx *ctx = new bv_ctx();
  ctx->device = device;
  ctx->flags = flags;
  int rc = create_impl(ctx);
  if (rc != BV_OK) {
    bv_destroy(ctx);
    return rc;
  }
  *out = ctx;
  return BV_OK;
}

extern "C" void bv_destroy(bv_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  // every call of this ctx has finished before anything is released (an
  // async call may still be reading slot buffers and key-cache tables)
  if (ctx->stream) {
    (void)bv_wait_all(ctx);
    if (ctx->has_done) (void)hipEventSynchronize(ctx->ev_done);
  }
  if (ctx->g_table) gtable_release(ctx->device);
  DevBuf *bufs[] = {&ctx->d_in, &ctx->kc_kxy, &ctx->kc_btabs, &ctx->ev_iota, &ctx->d_stamps, &ctx->d_sig};
  for (auto *b : bufs) b->release();
  for (auto &sl : ctx->slot) {
    DevBuf *sb[] = {&sl.digests,   &sl.kstatus, &sl.kxy, &sl.bases_jac, &sl.key_sub, &sl.key_pscr,
                    &sl.key_table, &sl.scratch, &sl.u12, &sl.rg,        &sl.status,  &sl.bits,
                    &sl.kc_tabs,   &sl.defer};
    for (auto *b : sb) b->release();
    sl.pin_small.release();
    if (sl.done) (void)hipEventDestroy(sl.done);
  }
  bv_kc_release(ctx);
  ctx->pin_in.release();
  ctx->pin_out.release();
  ctx->small_io.release();
  ctx->pin_long.release();
  ctx->d_long.release();
  for (auto &sl : ctx->slot)
    for (auto &e : sl.ev)
      if (e) (void)hipEventDestroy(e);
  for (auto &e : ctx->chunk_ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->ev_done) (void)hipEventDestroy(ctx->ev_done);
  if (ctx->ev_host) (void)hipEventDestroy(ctx->ev_host);
  streams_release(ctx);
  delete ctx->pool;
  delete ctx;
}

extern "C" void *bv_last_stream(const bv_ctx *ctx) { return ctx ? (void *)ctx->last : nullptr; }

static float elapsed(hipEvent_t a, hipEvent_t b);

extern "C" int bv_get_timing(const bv_ctx *ctx, bv_timing *out) {
  if (!ctx || !out) return BV_E_ARGS;
  // under the ctx's lock: a call on another thread writes the timing
  bv_ctx *c = const_cast<bv_ctx *>(ctx);
  std::lock_guard<std::mutex> lk(c->mu);
  *out = c->timing;
  return BV_OK;
}

// ---------------------------------------------------------------------------
// device pipeline
// ---------------------------------------------------------------------------
// Over device-resident inputs.  msg_hash/status/bits may be null (ctx
// buffers are used).  Caller holds ctx->mu and has set the device.
// `hashed`: the digests are already in ctx->S().digests (host entry point,
// hashed chunk by chunk as the bytes landed).  `kc`: use the key cache
// arrays prepared by kc_prepare.  Every call starts after the previous call
// on this ctx that used the same work-buffer slot has finished on the device
// (ctx->slot[].done), whatever its stream.
// Phase A of a verify: batched s^-1 on the s^-1 stream after `s_ready` (s
// and pre in HBM), key decode + per-batch key tables on the keys stream after
// `keys_ready` (the keys in HBM).  The host entry points stage the keys
// first, then s and pre, so the key tables build while the rest of the batch
// still crosses PCIe.
int bv_run_keys(bv_ctx *ctx, const bv_batch *b, hipEvent_t keys_ready, hipEvent_t s_ready, bool kc, bool split_ok) {
  const uint64_t n_items = b->n_items;
  const uint32_t n_keys = b->n_keys;
  if (n_items > 0 && (!b->item_msg || !b->item_key || !b->r_be || !b->s_be))
    return bv_fail(ctx, BV_E_ARGS, "null item arrays");
  if (n_items > 0 && n_keys == 0) return bv_fail(ctx, BV_E_ARGS, "items without keys");
  if (n_keys > 0 && !b->key_off) return bv_fail(ctx, BV_E_ARGS, "null key_off");
  if (((uintptr_t)b->r_be | (uintptr_t)b->s_be) & 15)
    return bv_fail(ctx, BV_E_ARGS, "r_be/s_be must be 16-byte aligned");
  HIPCHK(ctx->S().kstatus.ensure(std::max<uint32_t>(n_keys, 1)), BV_E_OOM, "alloc kstatus");
  HIPCHK(ctx->S().kxy.ensure(std::max<uint32_t>(n_keys, 1) * 64ull), BV_E_OOM, "alloc kxy");
  HIPCHK(ctx->S().scratch.ensure(std::max<uint64_t>(n_items, 1) * 32), BV_E_OOM, "alloc scratch");
  HIPCHK(ctx->S().u12.ensure(std::max<uint64_t>(n_items, 1) * BV_U_STRIDE * 4), BV_E_OOM, "alloc u12");

  // Key path: the key cache when prepared; otherwise per-batch fixed-base
  // tables once a key signs enough items (K12 for large batches, K8 for
  // mid-size), else the generic per-lane path.
  const uint64_t min_items = n_keys <= kManyKeys ? ctx->table_min_items : ctx->table_min_items_many;
  const bool table_mode = kc || (n_keys <= kMaxTableKeys && n_items >= min_items * n_keys) ||
                          (n_keys <= ctx->lat_table_keys && n_items <= kLatTableItems && n_items > 0);
  const int key_w = kc ? BV_KCW
                    : !table_mode ? 0
                    : (n_keys <= kMaxK12Keys && n_items >= ctx->k12_min_items * n_keys && !(ctx->flags & BV_F_K8))
                        ? 12
                        : 8;
  ctx->table_mode = table_mode;
  ctx->key_w = key_w;
  if (table_mode) {
    HIPCHK(ctx->S().rg.ensure(std::max<uint64_t>(n_items, 1) * kRgWords * 4), BV_E_OOM, "alloc R_G");
    if (!kc) {
      const uint64_t nk = std::max<uint32_t>(n_keys, 1);
      HIPCHK(ctx->S().bases_jac.ensure(nk * kBasesPerKey * 96ull), BV_E_OOM, "alloc bases");
      HIPCHK(ctx->S().key_sub.ensure(nk * (key_w == 12 ? kK12SubBytes : kKSubBytes)), BV_E_OOM,
             "alloc key sub-tables");
      HIPCHK(ctx->S().key_pscr.ensure(nk * (key_w == 12 ? kK12PrefixBytes : kKPrefixBytes)), BV_E_OOM,
             "alloc key prefix scratch");
      HIPCHK(ctx->S().key_table.ensure(nk * (key_w == 12 ? kK12TableBytes : kKTableBytes)), BV_E_OOM,
             "alloc key tables");
    }
  }
  hipEvent_t *ev = ctx->S().ev;
  // The key statuses (k_key_decode) go on the s^-1 stream ahead of s^-1:
  // k_verify_g reads them and is ordered after s^-1, while the key tables
  // (kstream) may queue behind another in-flight call's build.
  HIPCHK(hipStreamWaitEvent(ctx->sstream, keys_ready, 0), BV_E_LAUNCH, "fork");
  HIPCHK(hipEventRecord(ev[E_START], ctx->sstream), BV_E_LAUNCH, "event");
  // (key cache: every batch decodes its keys too — statuses never come from
  // the cache — unless bv_kc_prepare already did on the call's stream)
  if (kc && ctx->S().kc_decoded)  // its statuses are read on this stream too (k_verify_g)
    HIPCHK(hipStreamWaitEvent(ctx->sstream, ctx->S().ev[E_KCDEC], 0), BV_E_LAUNCH, "join");
  else
    HIPCHK(bvk::key_decode(ctx->sstream, n_keys, b->key_bytes, b->key_off, ctx->S().kstatus.as<uint8_t>(),
                           ctx->S().kxy.as<uint32_t>()),
           BV_E_LAUNCH, "k_key_decode");
  HIPCHK(hipEventRecord(ev[E_KDEC], ctx->sstream), BV_E_LAUNCH, "event");
  // s^-1 needs only s: concurrent with everything up to k_verify_g
  HIPCHK(hipStreamWaitEvent(ctx->sstream, s_ready, 0), BV_E_LAUNCH, "fork");
  // items per lane: kPrepM amortises the inversion in large batches; a small
  // batch spreads over ~64k lanes instead, since there the serial chain of
  // one lane (M products, the inversion, 2M products) is the latency
  const uint32_t M = (uint32_t)std::min<uint64_t>(kPrepM, std::max<uint64_t>(1, (n_items + 65535) / 65536));
  HIPCHK(bvk::sinv(ctx->sstream, n_items, M, (const uint32_t *)b->s_be, b->pre, ctx->S().scratch.as<uint32_t>()),
         BV_E_LAUNCH, "k_sinv");
  // u2 = r s^-1 and its GLV split for k_verify_q, off k_verify_g's path
  // (per-batch tables; the fused key-cache kernel forms its own)
  ctx->S().glv_split = split_ok && ctx->glv_in_sstream && table_mode && !(kc && kFusedKc);
  if (ctx->S().glv_split)
    HIPCHK(bvk::glv_split(ctx->sstream, n_items, (const uint32_t *)b->r_be, ctx->S().scratch.as<uint32_t>(),
                          ctx->S().u12.as<uint32_t>()),
           BV_E_LAUNCH, "k_glv_split");
  HIPCHK(hipEventRecord(ev[E_SINV], ctx->sstream), BV_E_LAUNCH, "event");
  HIPCHK(hipStreamWaitEvent(ctx->kstream, ev[E_KDEC], 0), BV_E_LAUNCH, "fork");
  if (!kc) {
    if (table_mode)
      HIPCHK(bvk::build_tables(ctx->kstream, key_w, n_keys, ctx->S().kxy.as<uint32_t>(), ctx->S().kstatus.as<uint8_t>(),
                               ctx->S().bases_jac.as<uint32_t>(), ctx->S().key_sub.as<uint32_t>(),
                               ctx->S().key_pscr.as<uint32_t>(), ctx->S().key_table.as<uint32_t>(), n_items),
             BV_E_LAUNCH, "key tables");
  }
  HIPCHK(hipEventRecord(ev[E_KEYS], ctx->kstream), BV_E_LAUNCH, "event");
  return BV_OK;
}

// Output buffers of a verify: the caller's device buffers when given (and
// usable), else the ctx's own.
int bv_out_bufs(bv_ctx *ctx, const bv_batch *b, uint8_t *d_msg_hash, uint8_t *d_status, uint64_t *d_bits,
                bool hashed, bv_out *o) {
  const uint64_t n_msgs = b->n_msgs, n_items = b->n_items;
  o->dig = (uint32_t *)d_msg_hash;
  if (hashed || !o->dig || ((uintptr_t)o->dig & 15)) {
    HIPCHK(ctx->S().digests.ensure(std::max<uint64_t>(n_msgs, 1) * 32), BV_E_OOM, "alloc digests");
    o->dig = ctx->S().digests.as<uint32_t>();
  }
  o->status = d_status;
  if (!o->status) {
    HIPCHK(ctx->S().status.ensure(std::max<uint64_t>(n_items, 1)), BV_E_OOM, "alloc status");
    o->status = ctx->S().status.as<uint8_t>();
  }
  o->bits = d_bits;
  if (!o->bits) {
    HIPCHK(ctx->S().bits.ensure(std::max<uint64_t>((n_items + 63) / 64, 1) * 8), BV_E_OOM, "alloc bits");
    o->bits = ctx->S().bits.as<uint64_t>();
  }
  return BV_OK;
}

// The verify kernels for items [lo, hi) (lo a multiple of 64) on `st`, after
// bv_run_keys; the caller orders `st` after s^-1 (E_SINV) and, for part 2,
// the key tables (E_KEYS).  part 1: k_verify_g (per-batch tables only: it
// needs no key table); part 2: the rest (k_verify_q, the fused key-cache
// kernel or the generic path) with statuses and bits.
int bv_launch_items(bv_ctx *ctx, const bv_batch *b, const bv_out &o, hipStream_t st, bool kc, uint64_t lo,
                    uint64_t hi, int part) {
  const uint64_t n = b->n_items;
  const uint8_t *kst = ctx->S().kstatus.as<uint8_t>();
  const uint32_t *r32 = (const uint32_t *)b->r_be, *s32 = (const uint32_t *)b->s_be;
  uint32_t *w = ctx->S().scratch.as<uint32_t>(), *u12 = ctx->S().u12.as<uint32_t>();
  const bool fused = kc && kFusedKc;  // key cache: G and Q parts in one kernel (R_G stays in registers)
  if (part == 1) {
    if (ctx->table_mode && !fused)
      HIPCHK(bvk::verify_g(st, n, lo, hi, b->item_key, r32, s32, b->pre, kst, b->item_msg, o.dig, w, u12,
                           ctx->g_table, ctx->S().rg.as<uint32_t>(), ctx->S().glv_split),
             BV_E_LAUNCH, "k_verify_g");
    return BV_OK;
  }
  if (fused)
    HIPCHK(bvk::verify_gq(st, n, lo, hi, b->item_key, r32, s32, b->pre, kst, b->item_msg, o.dig, w, ctx->g_table,
                          ctx->S().kc_tabs.as<uint64_t>(), o.status, o.bits),
           BV_E_LAUNCH, "k_verify_gq");
  else if (ctx->table_mode)
    HIPCHK(bvk::verify_q(st, ctx->key_w, n, lo, hi, b->item_key, r32, s32, b->pre, kst, u12,
                         ctx->S().key_table.as<uint32_t>(), kc ? ctx->S().kc_tabs.as<uint64_t>() : nullptr,
                         ctx->S().rg.as<uint32_t>(), o.status, o.bits),
           BV_E_LAUNCH, "k_verify_q");
  else
    HIPCHK(bvk::verify_generic(st, n, lo, hi, b->item_key, r32, s32, b->pre, kst, ctx->S().kxy.as<uint32_t>(),
                               b->item_msg, o.dig, w, ctx->g_table, o.status, o.bits),
           BV_E_LAUNCH, "k_verify_generic");
  return BV_OK;
}

int bv_item_pipe::key_part(hipStream_t ks, hipEvent_t ready) {
  if (!ctx->table_mode || !ctx->qfirst || b->n_items == 0) return BV_OK;
  hipEvent_t *ev = ctx->S().ev;
  HIPCHK(hipStreamWaitEvent(ks, ev[E_SINV], 0), BV_E_LAUNCH, "join");
  HIPCHK(hipStreamWaitEvent(ks, ready, 0), BV_E_LAUNCH, "join");
  HIPCHK(hipStreamWaitEvent(ks, ev[E_KEYS], 0), BV_E_LAUNCH, "join");
  if (kc && ks != ctx->stream) {  // kc_tabs (and any KC build) enqueued on ctx->stream by bv_kc_prepare
    HIPCHK(hipEventRecord(ev[E_KCTAB], ctx->stream), BV_E_LAUNCH, "event");
    HIPCHK(hipStreamWaitEvent(ks, ev[E_KCTAB], 0), BV_E_LAUNCH, "join");
  }
  HIPCHK(hipEventRecord(ev[E_SCALAR], ks), BV_E_LAUNCH, "event");  // ms_verify_g: the key part
  HIPCHK(hipEventRecord(ev[E_JOINED], ks), BV_E_LAUNCH, "event");  // ms_verify: key part to the last decision
  const uint64_t n = b->n_items;
  HIPCHK(bvk::verify_qf(ks, ctx->key_w, n, 0, n, b->item_key, (const uint32_t *)b->r_be, (const uint32_t *)b->s_be,
                        b->pre, ctx->S().kstatus.as<uint8_t>(), ctx->S().scratch.as<uint32_t>(),
                        ctx->S().key_table.as<uint32_t>(), kc ? ctx->S().kc_tabs.as<uint64_t>() : nullptr,
                        ctx->S().rg.as<uint32_t>()),
         BV_E_LAUNCH, "k_verify_qf");
  HIPCHK(hipEventRecord(ev[E_G], ks), BV_E_LAUNCH, "event");
  qf = true;
  return BV_OK;
}

int bv_item_pipe::upto(uint64_t end) {
  if (end <= done) return BV_OK;
  if (qf) {  // the key part is in rg: u1 G and the decision
    const uint64_t n = b->n_items;
    if (done == 0) HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_G], 0), BV_E_LAUNCH, "join key part");
    HIPCHK(bvk::verify_gf(st, n, done, end, b->item_key, (const uint32_t *)b->r_be, (const uint32_t *)b->s_be, b->pre,
                          ctx->S().kstatus.as<uint8_t>(), b->item_msg, o.dig, ctx->S().scratch.as<uint32_t>(),
                          ctx->g_table, ctx->S().rg.as<uint32_t>(), o.status, o.bits),
           BV_E_LAUNCH, "k_verify_gf");
    done = end;
    return BV_OK;
  }
  if (done == 0) {
    HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_SINV], 0), BV_E_LAUNCH, "join");
    HIPCHK(hipEventRecord(ctx->S().ev[E_SCALAR], st), BV_E_LAUNCH, "event");
    HIPCHK(hipEventRecord(ctx->S().ev[E_G], st), BV_E_LAUNCH, "event");
    HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_KEYS], 0), BV_E_LAUNCH, "join");
    HIPCHK(hipEventRecord(ctx->S().ev[E_JOINED], st), BV_E_LAUNCH, "event");
  }
  for (int part = 1; part <= 2; part++) {
    const int r = bv_launch_items(ctx, b, o, st, kc, done, end, part);
    if (r != BV_OK) return r;
  }
  done = end;
  return BV_OK;
}

int bv_run_deferred(bv_ctx *ctx, const bv_batch *b, const bv_out &o, hipStream_t st) {
  if (!ctx->S().kc_partial || b->n_items == 0) return BV_OK;
  const uint64_t n = b->n_items;
  HIPCHK(ctx->S().defer.ensure((n + 1) * 4), BV_E_OOM, "alloc deferred list");
  HIPCHK(bvk::verify_deferred(st, n, ctx->S().defer.as<uint32_t>(), b->item_key, (const uint32_t *)b->r_be,
                              (const uint32_t *)b->s_be, b->pre, ctx->S().kstatus.as<uint8_t>(),
                              ctx->S().kxy.as<uint32_t>(), b->item_msg, o.dig, ctx->S().scratch.as<uint32_t>(),
                              ctx->g_table, o.status, o.bits),
         BV_E_LAUNCH, "k_verify_deferred");
  return BV_OK;
}

int bv_item_pipe::finish() {
  const uint64_t n = b->n_items;
  if (n == 0) {
    HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_SINV], 0), BV_E_LAUNCH, "join");
    HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_KEYS], 0), BV_E_LAUNCH, "join");
    for (int e : {E_SCALAR, E_G, E_JOINED}) HIPCHK(hipEventRecord(ctx->S().ev[e], st), BV_E_LAUNCH, "event");
  }
  int r = upto(n);
  if (r != BV_OK) return r;
  if (kc && (r = bv_run_deferred(ctx, b, o, st)) != BV_OK) return r;
  HIPCHK(hipEventRecord(ctx->S().ev[E_END], st), BV_E_LAUNCH, "event");
  return bv_mark_done(ctx, st);
}

// Phase B on `st` (after bv_run_keys): SHA-256 of the messages (unless
// `hashed`: digests already in ctx->S().digests), then the verify kernels once
// s^-1 and the key tables are ready; statuses and bits.  k_verify_g needs
// no key table, so it runs while the keys stream still builds them.
int bv_run_verify(bv_ctx *ctx, const bv_batch *b, uint8_t *d_msg_hash, uint8_t *d_status, uint64_t *d_bits,
                  hipStream_t st, bool hashed, bool kc) {
  const uint64_t n_msgs = b->n_msgs, n_items = b->n_items;
  if (n_msgs > 0 && !b->msg_off) return bv_fail(ctx, BV_E_ARGS, "null msg_off");
  bv_out o;
  int rc = bv_out_bufs(ctx, b, d_msg_hash, d_status, d_bits, hashed, &o);
  if (rc != BV_OK) return rc;
  hipEvent_t *ev = ctx->S().ev;
  HIPCHK(hipEventRecord(ev[E_FORK], st), BV_E_LAUNCH, "event");
  if (!hashed) HIPCHK(bvk::sha256(st, n_msgs, b->msg_bytes, b->msg_off, o.dig), BV_E_LAUNCH, "k_sha256");
  HIPCHK(hipEventRecord(ev[E_SHA], st), BV_E_LAUNCH, "event");
  HIPCHK(hipStreamWaitEvent(st, ev[E_SINV], 0), BV_E_LAUNCH, "join");
  HIPCHK(hipEventRecord(ev[E_SCALAR], st), BV_E_LAUNCH, "event");
  rc = bv_launch_items(ctx, b, o, st, kc, 0, n_items, 1);
  if (rc != BV_OK) return rc;
  HIPCHK(hipEventRecord(ev[E_G], st), BV_E_LAUNCH, "event");
  HIPCHK(hipStreamWaitEvent(st, ev[E_KEYS], 0), BV_E_LAUNCH, "join");
  HIPCHK(hipEventRecord(ev[E_JOINED], st), BV_E_LAUNCH, "event");
  rc = bv_launch_items(ctx, b, o, st, kc, 0, n_items, 2);
  if (rc != BV_OK) return rc;
  if (kc && (rc = bv_run_deferred(ctx, b, o, st)) != BV_OK) return rc;
  HIPCHK(hipEventRecord(ev[E_END], st), BV_E_LAUNCH, "event");
  if (d_msg_hash && (uint8_t *)o.dig != d_msg_hash)
    HIPCHK(hipMemcpyAsync(d_msg_hash, o.dig, n_msgs * 32, hipMemcpyDeviceToDevice, st), BV_E_LAUNCH, "copy digests");
  return bv_mark_done(ctx, st);
}

// The whole verify of a batch already in HBM on `st` (which has waited for
// the last call on the current work-buffer slot: bv_slot_begin).
int bv_run_device(bv_ctx *ctx, const bv_batch *b, uint8_t *d_msg_hash, uint8_t *d_status, uint64_t *d_bits,
                  hipStream_t st, bool hashed, bool kc) {
  HIPCHK(hipEventRecord(ctx->S().ev[E_READY], st), BV_E_LAUNCH, "event");
  int rc = bv_run_keys(ctx, b, ctx->S().ev[E_READY], ctx->S().ev[E_READY], kc, true);
  if (rc != BV_OK) return rc;
  return bv_run_verify(ctx, b, d_msg_hash, d_status, d_bits, st, hashed, kc);
}

// (an event this call did not record gives -1; the failed query's error is
// cleared, so the next launch check does not report it)
static float elapsed(hipEvent_t a, hipEvent_t b) {
  float t;
  if (hipEventElapsedTime(&t, a, b) == hipSuccess) return t;
  (void)hipGetLastError();
  return -1.f;
}

void bv_read_timing(bv_ctx *ctx) {
  hipEvent_t *ev = ctx->S().ev;
  bv_timing &t = ctx->timing;
  t.ms_sha256 = elapsed(ev[E_FORK], ev[E_SHA]);
  t.key_path = (uint32_t)ctx->key_w;
  t.ms_keyprep = elapsed(ev[E_START], ev[E_KEYS]);
  t.ms_scalar = elapsed(ev[E_START], ev[E_SINV]);
  t.ms_verify_g = elapsed(ev[E_SCALAR], ev[E_G]);
  t.ms_verify = elapsed(ev[E_JOINED], ev[E_END]);
  t.ms_total = elapsed(ev[E_START], ev[E_END]);
}

static int verify_device_impl(bv_ctx *ctx, const bv_batch *dbatch, bv_result *dresult, hipStream_t st);

extern "C" int bv_verify_batch_device(bv_ctx *ctx, const bv_batch *dbatch, bv_result *dresult, void *stream,
                                      int async) {
  if (!ctx || !dbatch || !dresult) return BV_E_ARGS;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  const auto t0 = std::chrono::steady_clock::now();
  // NULL stream: the lane of the work slot this call takes (bv_slot_begin
  // advances ctx->cur), so consecutive async calls land on two queues
  hipStream_t st = stream ? (hipStream_t)stream : ctx->lane[(ctx->cur + 1) % bv_ctx::kSlots];
  ctx->last = st;
  ctx->timing = bv_timing{};
  int rc = verify_device_impl(ctx, dbatch, dresult, st);
  if (rc != BV_OK) return bv_drain(ctx, st, rc);
  if (!async) {
    HIPCHK(hipStreamSynchronize(st), BV_E_LAUNCH, "verify sync");
    bv_read_timing(ctx);
    ctx->timing.ms_host =
        std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return BV_OK;
}

static int verify_device_impl(bv_ctx *ctx, const bv_batch *dbatch, bv_result *dresult, hipStream_t st) {
  bool kc = false;
  if (bv_slot_begin(ctx, st, dbatch, dresult) != BV_OK) return BV_E_LAUNCH;
  if ((ctx->flags & BV_F_KEY_CACHE) && dbatch->n_keys && dbatch->n_keys <= kKcMaxBatchKeys) {
    // the cache is keyed by the raw key bytes: bring them (small) to the host
    const uint32_t nk = dbatch->n_keys;
    std::vector<uint64_t> hko(nk + 1);
    HIPCHK(hipMemcpyAsync(hko.data(), dbatch->key_off, (nk + 1) * 8ull, hipMemcpyDeviceToHost, st), BV_E_LAUNCH,
           "d2h key_off");
    HIPCHK(bv_host_wait(ctx, st), BV_E_LAUNCH, "sync");
    if (hko[0] != 0) return bv_fail(ctx, BV_E_ARGS, "key_off[0] != 0");
    for (uint32_t k = 0; k < nk; k++)
      if (hko[k] > hko[k + 1]) return bv_fail(ctx, BV_E_ARGS, "key_off not monotone");
    std::vector<uint8_t> hkb(hko[nk] + 1);
    if (hko[nk]) {
      HIPCHK(hipMemcpyAsync(hkb.data(), dbatch->key_bytes, hko[nk], hipMemcpyDeviceToHost, st), BV_E_LAUNCH,
             "d2h key bytes");
      HIPCHK(bv_host_wait(ctx, st), BV_E_LAUNCH, "sync");
    }
    bv_kc_items items;
    items.n_items = dbatch->n_items;
    items.d_item_key = dbatch->item_key;
    int rc = bv_kc_prepare(ctx, nk, hkb.data(), hko.data(), dbatch->key_bytes, dbatch->key_off, st, &kc, false, &items);
    if (rc != BV_OK) return rc;
  }
  return bv_run_device(ctx, dbatch, dresult->msg_hash, dresult->status, dresult->accept_bits, st, false, kc);
}

extern "C" int bv_sync(bv_ctx *ctx) {
  if (!ctx) return BV_E_ARGS;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!ctx->has_done) return BV_OK;
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  const int rc = bv_wait_all(ctx);
  if (rc != BV_OK) return rc;
  bv_read_timing(ctx);
  return BV_OK;
}

// ---------------------------------------------------------------------------
// host entry point
// ---------------------------------------------------------------------------
int bv_validate_host_batch(bv_ctx *ctx, const bv_batch *b) {
  const uint64_t n_msgs = b->n_msgs, n_items = b->n_items;
  const uint32_t n_keys = b->n_keys;
  if ((n_msgs && !b->msg_off) || (n_keys && !b->key_off) ||
      (n_items && (!b->item_msg || !b->item_key || !b->r_be || !b->s_be)))
    return bv_fail(ctx, BV_E_ARGS, "null input array");
  if (n_items && !n_keys) return bv_fail(ctx, BV_E_ARGS, "items without keys");
  const uint64_t msg_len = n_msgs ? b->msg_off[n_msgs] : 0;
  const uint64_t key_len = n_keys ? b->key_off[n_keys] : 0;
  // byte arrays may be null only when empty (all-empty messages or keys)
  if ((msg_len && !b->msg_bytes) || (key_len && !b->key_bytes)) return bv_fail(ctx, BV_E_ARGS, "null byte array");
  // validate host offsets (a bad offset must not become an OOB device read)
  if (n_msgs && b->msg_off[0] != 0) return bv_fail(ctx, BV_E_ARGS, "msg_off[0] != 0");
  if (n_keys && b->key_off[0] != 0) return bv_fail(ctx, BV_E_ARGS, "key_off[0] != 0");
  for (uint32_t k = 0; k < n_keys; k++)
    if (b->key_off[k] > b->key_off[k + 1]) return bv_fail(ctx, BV_E_ARGS, "key_off not monotone");
  // the O(n) checks run on the copy pool (1M items: ~0.3 ms instead of ~3)
  constexpr uint64_t kGrain = 1 << 17;
  if (!ctx->pool->parallel_for(n_msgs, kGrain, [b](uint64_t lo, uint64_t hi) {
        for (uint64_t m = lo; m < hi; m++)
          if (b->msg_off[m] > b->msg_off[m + 1]) return false;
        return true;
      }))
    return bv_fail(ctx, BV_E_ARGS, "msg_off not monotone");
  if (!ctx->pool->parallel_for(n_items, kGrain, [b, n_msgs, n_keys](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; i++)
          if (b->item_msg[i] >= n_msgs || b->item_key[i] >= n_keys) return false;
        return true;
      }))
    return bv_fail(ctx, BV_E_ARGS, "item index out of range");
  return BV_OK;
}


// Stage a host batch into HBM (pinned chunks on the copy stream), hash the
// messages chunk by chunk as they land and launch the verify pipeline.
// Returns with the work enqueued; bv_host_finish waits and copies results.
int bv_host_launch(bv_ctx *ctx, const bv_batch *b, bv_host_call *call, const bv_result *res) {
  const auto t0 = std::chrono::steady_clock::now();
  call->t0 = t0;
  int rc = bv_validate_host_batch(ctx, b);
  if (rc != BV_OK) return rc;
  // BV_HOST_STAMPS (diagnostics): the host phases of this call on stderr
  auto stamp_ms = [t0]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  double st_validated = ctx->host_stamps ? stamp_ms() : 0, st_items = 0, st_first = 0, st_copy = 0;
  int n_chunks = 0;
  hipStream_t st = ctx->stream, cs = bv_copy_stream(ctx);
  if (!cs) return bv_fail(ctx, BV_E_NODEVICE, "copy stream");
  ctx->last = st;
  ctx->timing = bv_timing{};
  const uint64_t n_msgs = b->n_msgs, n_items = b->n_items;
  const uint32_t n_keys = b->n_keys;
  const uint64_t msg_len = n_msgs ? b->msg_off[n_msgs] : 0;
  const uint64_t key_len = n_keys ? b->key_off[n_keys] : 0;
  // long messages (hashed on the host, below)
  std::vector<uint64_t> longm;
  if (n_msgs && !ctx->pool->parallel_for(n_msgs, 1 << 17, [b](uint64_t lo, uint64_t hi) {
        for (uint64_t m = lo; m < hi; m++)
          if (b->msg_off[m + 1] - b->msg_off[m] > kHostHashLen) return false;
        return true;
      }))
    for (uint64_t m = 0; m < n_msgs; m++)
      if (b->msg_off[m + 1] - b->msg_off[m] > kHostHashLen) longm.push_back(m);

  // one staging layout, identical in pinned host memory and in HBM
  struct Seg {
    const void *src;
    size_t n;
    size_t off;
  };
  Seg segs[9];
  size_t total = 0;
  auto add = [&](int i, const void *src, size_t n, size_t pad) {
    segs[i] = {src, n, total};
    total += align256(n + pad);
  };
  // staging order: the keys (the key tables start once they land), s and
  // pre (s^-1), the other item arrays, then the message bytes
  add(1, b->key_off, n_keys ? (n_keys + 1) * 8ull : 0, 0);
  add(2, b->key_bytes, key_len, 64);
  add(6, b->s_be, n_items * 32, 0);
  add(7, b->pre, b->pre ? n_items : 0, 0);
  add(0, b->msg_off, n_msgs ? (n_msgs + 1) * 8 : 0, 0);
  add(3, b->item_msg, n_items * 4, 0);
  add(4, b->item_key, n_items * 4, 0);
  add(5, b->r_be, n_items * 32, 0);
  add(8, b->msg_bytes, msg_len, 64);
  // previous work on this ctx must be done before its staging is reused
  if (bv_wait_all(ctx) != BV_OK) return BV_E_LAUNCH;  // previous calls' work buffers / staging
  HIPCHK(ctx->pin_in.ensure(total), BV_E_OOM, "alloc pinned staging");
  HIPCHK(ctx->d_in.ensure(total), BV_E_OOM, "alloc device staging");
  uint8_t *pin = (uint8_t *)ctx->pin_in.p, *dev = ctx->d_in.as<uint8_t>();
  HIPCHK(hipEventRecord(ctx->S().ev[E_CALL], cs), BV_E_LAUNCH, "event");
  // arrays in bv_host_alloc memory are DMA'd from where they are
  bool direct[9];
  for (int i = 0; i < 9; i++) direct[i] = bv_is_pinned(segs[i].src, segs[i].n);
  call->direct_in = direct[8];

  // keys and item arrays first (one contiguous region of the layout), in
  // kChunk pieces: the pool fills piece c+1 while the DMA engine moves piece c
  size_t ev_i = 0;
  auto chunk_event = [&]() -> hipEvent_t {
    hipEvent_t e = ctx->chunk_ev[ev_i % ctx->chunk_ev.size()];
    ev_i++;
    return e;
  };
  // layout bytes [a0, a1) of segments 0-7, in kChunk pieces: the pool fills
  // piece c+1 while the DMA engine moves piece c
  auto stage = [&](size_t a0, size_t a1) -> int {
    for (size_t a = a0; a < a1; a += kChunk) {
      const size_t z = std::min(a1, a + kChunk);
      std::vector<CopyPool::Piece> pieces;
      bool any_direct = false;
      for (int i = 0; i < 8; i++) {
        const Seg &s = segs[i];
        const size_t lo = std::max(a, s.off), hi = std::min(z, s.off + s.n);
        if (lo >= hi) continue;
        if (direct[i]) {
          any_direct = true;
          HIPCHK(hipMemcpyAsync(dev + lo, (const uint8_t *)s.src + (lo - s.off), hi - lo, hipMemcpyHostToDevice, cs),
                 BV_E_LAUNCH, "h2d (pinned caller buffer)");
        } else {
          pieces.push_back({pin + lo, (const uint8_t *)s.src + (lo - s.off), hi - lo});
        }
      }
      ctx->pool->copy_many(pieces);
      if (!any_direct) {
        HIPCHK(hipMemcpyAsync(dev + a, pin + a, z - a, hipMemcpyHostToDevice, cs), BV_E_LAUNCH, "h2d");
      } else {
        for (const CopyPool::Piece &q : pieces) {
          const size_t o = (uint8_t *)q.dst - pin;
          HIPCHK(hipMemcpyAsync(dev + o, q.dst, q.n, hipMemcpyHostToDevice, cs), BV_E_LAUNCH, "h2d");
        }
      }
    }
    return BV_OK;
  };
  // a small batch (every array in pageable memory) crosses in ONE copy: the
  // whole layout, message bytes and their zero pad included
  bool one_copy = total <= kSmallStage;
  for (int i = 0; i < 9; i++) one_copy = one_copy && !direct[i];
  if (one_copy) {
    for (int i = 0; i < 9; i++)
      if (segs[i].n) memcpy(pin + segs[i].off, segs[i].src, segs[i].n);
    if (msg_len) memset(pin + segs[8].off + msg_len, 0, 64);
    HIPCHK(hipMemcpyAsync(dev, pin, total, hipMemcpyHostToDevice, cs), BV_E_LAUNCH, "h2d (one copy)");
    for (int e : {E_KREADY, E_SREADY, E_SMALL}) HIPCHK(hipEventRecord(ctx->S().ev[e], cs), BV_E_LAUNCH, "event");
  } else {
    rc = stage(0, segs[6].off);  // the keys
    if (rc != BV_OK) return rc;
    HIPCHK(hipEventRecord(ctx->S().ev[E_KREADY], cs), BV_E_LAUNCH, "event");
    rc = stage(segs[6].off, segs[0].off);  // s, pre
    if (rc != BV_OK) return rc;
    HIPCHK(hipEventRecord(ctx->S().ev[E_SREADY], cs), BV_E_LAUNCH, "event");
    rc = stage(segs[0].off, segs[8].off);  // msg_off, item_msg, item_key, r
    if (rc != BV_OK) return rc;
    // zero the message-bytes pad (the SHA kernel over-reads the last dword of
    // a message into it): in the staging, or on the device for direct bytes
    if (msg_len && !direct[8]) memset(pin + segs[8].off + msg_len, 0, 64);
    if (msg_len && direct[8])
      HIPCHK(hipMemsetAsync(dev + segs[8].off + msg_len, 0, 64, cs), BV_E_LAUNCH, "zero message pad");
    HIPCHK(hipEventRecord(ctx->S().ev[E_SMALL], cs), BV_E_LAUNCH, "event");
  }

  bv_batch d = {};
  d.n_msgs = n_msgs;
  d.msg_bytes = dev + segs[8].off;
  d.msg_off = (const uint64_t *)(dev + segs[0].off);
  d.n_keys = n_keys;
  d.key_bytes = dev + segs[2].off;
  d.key_off = (const uint64_t *)(dev + segs[1].off);
  d.n_items = n_items;
  d.item_msg = (const uint32_t *)(dev + segs[3].off);
  d.item_key = (const uint32_t *)(dev + segs[4].off);
  d.r_be = dev + segs[5].off;
  d.s_be = dev + segs[6].off;
  d.pre = b->pre ? dev + segs[7].off : nullptr;

  if (ctx->host_stamps) st_items = stamp_ms();
  // key cache resolution needs the keys on the device (decode of misses)
  bool kc = false;
  if ((ctx->flags & BV_F_KEY_CACHE) && n_keys && n_keys <= kKcMaxBatchKeys) {
    HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_KREADY], 0), BV_E_LAUNCH, "join");
    bv_kc_items items;
    items.n_items = b->n_items;
    items.h_item_key = b->item_key;
    rc = bv_kc_prepare(ctx, n_keys, b->key_bytes, b->key_off, d.key_bytes, d.key_off, st, &kc, false, &items);
    if (rc != BV_OK) return rc;
  }
  // the key tables need only the keys and s^-1 only s: they run while the
  // rest of the batch still crosses PCIe
  rc = bv_run_keys(ctx, &d, ctx->S().ev[E_KREADY], ctx->S().ev[E_SREADY], kc);
  if (rc != BV_OK) return rc;

  // Items in message order (item_msg non-decreasing: events, blocks) are
  // verified chunk by chunk as their messages are hashed, so the verify
  // kernels also run under the PCIe transfer; otherwise after the last chunk.
  const bool in_order = longm.empty() &&  // (long messages' digests land after the last chunk)
                        ctx->pool->parallel_for(n_items > 0 ? n_items - 1 : 0, 1 << 17, [b](uint64_t lo, uint64_t hi) {
                          for (uint64_t i = lo; i < hi; i++)
                            if (b->item_msg[i] > b->item_msg[i + 1]) return false;
                          return true;
                        });
  bv_item_pipe pipe{ctx, &d, {}, st, kc};
  rc = bv_out_bufs(ctx, &d, nullptr, nullptr, nullptr, true, &pipe.o);
  if (rc != BV_OK) return rc;
  // the key part of every item (R_Q) on the s^-1 stream once r and the item
  // keys are in: it needs no digest, so it runs under the message transfer
  rc = pipe.key_part(ctx->sstream, ctx->S().ev[E_SMALL]);
  if (rc != BV_OK) return rc;

  // results into pinned memory (straight into the caller's bv_host_alloc
  // buffers when they are): digests chunk by chunk on `st` as each chunk is
  // hashed (ctx->ev_d2h; after the last chunk, on the copy stream, when long
  // messages' digests are put in afterwards), statuses and bits at the end
  const size_t o_st = align256(n_msgs * 32), o_bits = o_st + align256(n_items);
  HIPCHK(ctx->pin_out.ensure(o_bits + align256((n_items + 63) / 64 * 8) + 256), BV_E_OOM, "alloc pinned results");
  uint8_t *pout = (uint8_t *)ctx->pin_out.p;
  call->pout = pout;
  call->o_st = o_st;
  call->o_bits = o_bits;
  call->direct_hash = res && bv_is_pinned(res->msg_hash, n_msgs * 32);
  call->direct_status = res && bv_is_pinned(res->status, n_items);
  uint8_t *hout = call->direct_hash ? res->msg_hash : pout;
  const bool d2h_chunks = ctx->ev_d2h == 1 && longm.empty();

  // message bytes: chunks on message boundaries, each hashed once it lands
  if (ctx->has_done) HIPCHK(hipStreamWaitEvent(st, ctx->ev_done, 0), BV_E_LAUNCH, "order");
  HIPCHK(hipEventRecord(ctx->S().ev[E_HASH0], st), BV_E_LAUNCH, "event");
  HIPCHK(hipEventRecord(ctx->S().ev[E_FORK], st), BV_E_LAUNCH, "event");
  const uint64_t msg_chunk = ctx->host_msg_chunk;
  uint64_t m0 = 0;
  while (m0 < n_msgs) {
    // messages [m0, m1) holding about msg_chunk bytes (at least one message)
    const uint64_t base = b->msg_off[m0];
    uint64_t m1 = std::upper_bound(b->msg_off + m0 + 1, b->msg_off + n_msgs + 1, base + msg_chunk) - b->msg_off - 1;
    if (m1 <= m0) m1 = m0 + 1;
    const uint64_t end = b->msg_off[m1];
    if (one_copy) {
      // already on the device
    } else if (direct[8]) {
      HIPCHK(hipMemcpyAsync(dev + segs[8].off + base, b->msg_bytes + base, end - base, hipMemcpyHostToDevice, cs),
             BV_E_LAUNCH, "h2d msgs (pinned caller buffer)");
    } else {
      const size_t len = end - base + (m1 == n_msgs ? 64 : 0);
      const double c0 = ctx->host_stamps ? stamp_ms() : 0;
      ctx->pool->copy(pin + segs[8].off + base, b->msg_bytes + base, end - base);
      if (ctx->host_stamps) st_copy += stamp_ms() - c0;
      HIPCHK(hipMemcpyAsync(dev + segs[8].off + base, pin + segs[8].off + base, len, hipMemcpyHostToDevice, cs),
             BV_E_LAUNCH, "h2d msgs");
    }
    hipEvent_t e = chunk_event();
    HIPCHK(hipEventRecord(e, cs), BV_E_LAUNCH, "event");
    HIPCHK(hipStreamWaitEvent(st, e, 0), BV_E_LAUNCH, "join chunk");
    if (m0 == 0 && ctx->host_stamps) st_first = stamp_ms();
    n_chunks++;
    if (ctx->host_stamps && call->h_call < 0) {  // (diagnostics) has the device reached the call yet?
      const hipError_t q = hipEventQuery(ctx->S().ev[E_CALL]);
      if (q == hipSuccess) call->h_call = stamp_ms();
      else if (q != hipErrorNotReady) (void)hipGetLastError();
    }
    if (m0 == 0) HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_SMALL], 0), BV_E_LAUNCH, "join offsets");
    HIPCHK(bvk::sha256(st, m1 - m0, d.msg_bytes, d.msg_off + m0, pipe.o.dig + 8 * m0, kHostHashLen), BV_E_LAUNCH,
           "k_sha256");
    HIPCHK(hipEventRecord(ctx->S().ev[E_HASHED], st), BV_E_LAUNCH, "event");  // the last chunk's record is the one used
    if (in_order) {  // items up to the first one of a message >= m1, in whole 64-item words
      const uint64_t i_end = m1 == n_msgs ? n_items
                                          : (uint64_t)(std::lower_bound(b->item_msg, b->item_msg + n_items, m1) -
                                                       b->item_msg) / 64 * 64;
      rc = pipe.upto(i_end);
      if (rc != BV_OK) return rc;
    }
    if (d2h_chunks)
      HIPCHK(hipMemcpyAsync(hout + 32 * m0, pipe.o.dig + 8 * m0, (m1 - m0) * 32, hipMemcpyDeviceToHost, st),
             BV_E_LAUNCH, "d2h digests");
    m0 = m1;
  }
  if (!longm.empty()) {
    // the long messages on the host (pool threads, SHA extensions) while the
    // device hashes the rest; then their digests cross and are put in place
    const uint64_t nl = longm.size();
    HIPCHK(ctx->pin_long.ensure(nl * 40), BV_E_OOM, "alloc pinned long digests");
    HIPCHK(ctx->d_long.ensure(nl * 40), BV_E_OOM, "alloc long digests");
    uint64_t *lidx = (uint64_t *)ctx->pin_long.p;
    uint8_t *ldig = (uint8_t *)(lidx + nl);
    memcpy(lidx, longm.data(), nl * 8);
    ctx->pool->parallel_for(nl, 1, [&](uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi; i++) {
        const uint64_t m = longm[i];
        hsha::digest(b->msg_bytes + b->msg_off[m], b->msg_off[m + 1] - b->msg_off[m], ldig + 32 * i);
      }
      return true;
    });
    HIPCHK(hipMemcpyAsync(ctx->d_long.p, lidx, nl * 40, hipMemcpyHostToDevice, cs), BV_E_LAUNCH, "h2d long digests");
    hipEvent_t e = chunk_event();
    HIPCHK(hipEventRecord(e, cs), BV_E_LAUNCH, "event");
    HIPCHK(hipStreamWaitEvent(st, e, 0), BV_E_LAUNCH, "join long digests");
    HIPCHK(bvk::put_digests(st, nl, ctx->d_long.as<uint64_t>(), (const uint32_t *)(ctx->d_long.as<uint8_t>() + nl * 8),
                            pipe.o.dig),
           BV_E_LAUNCH, "k_put_digests");
    HIPCHK(hipEventRecord(ctx->S().ev[E_HASHED], st), BV_E_LAUNCH, "event");
  }
  HIPCHK(hipEventRecord(ctx->S().ev[E_STAGED], cs), BV_E_LAUNCH, "event");
  call->ms_prep = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (ctx->host_stamps)
    fprintf(stderr,
            "bv_host_launch ms: validated %.3f items_staged %.3f first_msg_chunk %.3f staged %.3f (message copies "
            "%.3f in %d chunks; msgs %.1f MB, %d copy threads; staging on NUMA node %d..%d, caller on node %d)\n",
            st_validated, st_items, st_first, (double)call->ms_prep, st_copy, n_chunks, msg_len / 1e6,
            (int)ctx->pool->th.size(), numa_node_of(pin), numa_node_of(pin + total - 1), numa_node_of(nullptr));
  HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_STAGED], 0), BV_E_LAUNCH, "join staging");
  HIPCHK(hipEventRecord(ctx->S().ev[E_SHA], st), BV_E_LAUNCH, "event");
  if (n_msgs == 0) HIPCHK(hipEventRecord(ctx->S().ev[E_HASHED], st), BV_E_LAUNCH, "event");
  rc = pipe.finish();
  if (rc != BV_OK) return rc;

  if (n_msgs && !d2h_chunks) {  // the digests as soon as hashing ended, beside the verify kernels
    HIPCHK(hipStreamWaitEvent(cs, ctx->S().ev[E_HASHED], 0), BV_E_LAUNCH, "join");
    HIPCHK(hipMemcpyAsync(hout, ctx->S().digests.p, n_msgs * 32, hipMemcpyDeviceToHost, cs), BV_E_LAUNCH,
           "d2h digests");
  }
  if (n_items) {
    HIPCHK(hipMemcpyAsync(call->direct_status ? res->status : pout + o_st, ctx->S().status.p, n_items,
                          hipMemcpyDeviceToHost, st),
           BV_E_LAUNCH, "d2h status");
    HIPCHK(hipMemcpyAsync(pout + o_bits, ctx->S().bits.p, (n_items + 63) / 64 * 8, hipMemcpyDeviceToHost, st),
           BV_E_LAUNCH, "d2h bits");
  }
  HIPCHK(hipEventRecord(ctx->S().ev[E_OUT], st), BV_E_LAUNCH, "event");
  HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_STAGED], 0), BV_E_LAUNCH, "join");  // staging free after this point
  HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_HASHED], 0), BV_E_LAUNCH, "join");
  // the digests' d2h on the copy stream also precedes ev_done
  HIPCHK(hipEventRecord(ctx->S().ev[E_CSDONE], cs), BV_E_LAUNCH, "event");
  HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_CSDONE], 0), BV_E_LAUNCH, "join");
  return bv_mark_done(ctx, st);
}

int bv_host_finish(bv_ctx *ctx, const bv_batch *b, bv_result *res, bv_host_call *call, bool bits_out) {
  double h_in = -1, h_staged = -1, h_done = -1;
  if (ctx->host_stamps) {  // (diagnostics) host ms at which the staging end and the call's end are seen
    auto ms = [call]() {
      return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - call->t0).count();
    };
    h_in = ms();
    if (call->h_call < 0 && hipEventQuery(ctx->S().ev[E_CALL]) == hipSuccess) call->h_call = h_in;
    while (h_done < 0) {
      if (h_staged < 0 && hipEventQuery(ctx->S().ev[E_STAGED]) == hipSuccess) h_staged = ms();
      const hipError_t q = hipEventQuery(ctx->ev_done);
      if (q == hipSuccess) h_done = ms();
      else if (q != hipErrorNotReady) break;
    }
    (void)hipGetLastError();
  }
  HIPCHK(hipEventSynchronize(ctx->ev_done), BV_E_LAUNCH, "verify sync");
  const auto t_out = std::chrono::steady_clock::now();
  const uint64_t n_msgs = b->n_msgs, n_items = b->n_items;
  if (res->msg_hash && n_msgs && !call->direct_hash) ctx->pool->copy(res->msg_hash, call->pout, n_msgs * 32);
  if (res->status && n_items && !call->direct_status) ctx->pool->copy(res->status, call->pout + call->o_st, n_items);
  if (bits_out && res->accept_bits && n_items)
    memcpy(res->accept_bits, call->pout + call->o_bits, (n_items + 63) / 64 * 8);
  bv_read_timing(ctx);
  ctx->timing.ms_h2d = elapsed(ctx->S().ev[E_CALL], ctx->S().ev[E_STAGED]);
  ctx->timing.ms_d2h = elapsed(ctx->S().ev[E_END], ctx->S().ev[E_OUT]);
  const auto t_end = std::chrono::steady_clock::now();
  if (ctx->host_stamps) {  // the device timeline from E_CALL (the first copy-stream command of the call)
    hipEvent_t *ev = ctx->S().ev;
    fprintf(stderr,
            "bv_host_finish ms: synced %.3f (host, from the call; seen: call %.3f finish_in %.3f staged %.3f "
            "done %.3f) | device from E_CALL: hash0 %.3f staged %.3f hashed %.3f verify_start %.3f verify_end %.3f "
            "out %.3f\n",
            std::chrono::duration<double, std::milli>(t_out - call->t0).count(), call->h_call, h_in, h_staged, h_done,
            elapsed(ev[E_CALL], ev[E_HASH0]),
            elapsed(ev[E_CALL], ev[E_STAGED]), elapsed(ev[E_CALL], ev[E_HASHED]), elapsed(ev[E_CALL], ev[E_START]),
            elapsed(ev[E_CALL], ev[E_END]), elapsed(ev[E_CALL], ev[E_OUT]));
  }
  ctx->timing.ms_host = std::chrono::duration<float, std::milli>(t_end - call->t0).count();
  ctx->timing.ms_host_prep = call->ms_prep;
  ctx->timing.ms_host_out = std::chrono::duration<float, std::milli>(t_end - t_out).count();
  return BV_OK;
}

// ---------------------------------------------------------------------------
// Small batches (addSelfEvent's own event, core.go:292; processJoinRequest's
// ITX, node_rpc.go:250-260; a short SyncResponse): latency, not throughput.
// ONE copy in, ONE k_small launch (every step of an item in one workgroup,
// kernels.hip), ONE copy out; key-cache tables are resolved on the host
// without a device round trip, keys without one take k_small's cooperative
// NAF chain (1 cold event 0.55 ms against 0.78 ms through the per-batch K8
// tables; with the key cache 0.18 ms against 0.47 ms,
// profiles/r04_small_lat.log).
// ---------------------------------------------------------------------------
constexpr uint64_t kSmallMsgLen = 16 << 10;  // longest message (hashed on the host, inside the call)
constexpr uint64_t kHostRecGrain = 16;       // host item records per pool task
constexpr uint8_t kSmallPending = 0xFF;      // status sentinel (statuses are 0..3)

// Small batches: <= ctx->small_max (256) items, or up to ctx->small_warm_max
// (1024) items when every well-formed key already has a key-cache table (no
// item needs the cooperative NAF chains).  Warm, same box, 4 creators
// (profiles/r05_ab_small_max.log): 0.14 / 0.18 / 0.29 / 0.52 ms at 256 / 512
// / 1000 / 2000 items against 0.45-0.70 / 0.52 for the bulk pipeline.  The
// cold limit is round 4's (profiles/r04_small_lat.log): the right-to-left
// cold path that measured 0.32 / 0.40 ms at 256 / 512 items gave a false
// REJECT on ~1 in 3000 items of a process's first batch and was withdrawn
// (DESIGN.md section 4, round 5).
static bool small_batch(bv_ctx *ctx, const bv_batch *b) {
  if (b->n_items == 0) return false;
  const uint64_t n = std::max<uint64_t>(b->n_items, b->n_msgs);
  if (n > ctx->small_max) {
    if (n > ctx->small_warm_max || !(ctx->flags & BV_F_KEY_CACHE) || b->n_keys == 0 || b->n_keys > kKcMaxBatchKeys)
      return false;
    // the key bytes are read below: only a well-formed batch (the bulk path
    // reports a malformed one through its own validation)
    if (bv_validate_host_batch(ctx, b) != BV_OK || !bv_kc_all_cached(ctx, b->n_keys, b->key_bytes, b->key_off))
      return false;
  }
  if (b->n_msgs && !b->msg_off) return false;  // (validation reports it)
  for (uint64_t m = 0; m < b->n_msgs; m++)
    if (b->msg_off[m + 1] - b->msg_off[m] > kSmallMsgLen) return false;
  return true;
}

static int small_verify(bv_ctx *ctx, const bv_batch *b, bv_result *res) {
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t n_msgs = b->n_msgs, n_items = b->n_items;
  const uint32_t n_keys = b->n_keys;
  const uint64_t key_len = n_keys ? b->key_off[n_keys] : 0;
  hipStream_t st = ctx->stream;
  ctx->last = st;
  ctx->timing = bv_timing{};
  size_t total = 0;
  auto at = [&](size_t bytes) {
    const size_t o = total;
    total += align256(bytes);
    return o;
  };
  // ONE mapped, coherent pinned buffer the kernel reads and writes in place
  // (no copy either way): the digests (hashed here), keys, item arrays, the
  // key cache's table address per key; then the statuses
  const size_t o_dig = at(n_msgs * 32), o_key = at(key_len + 64), o_koff = at((n_keys + 1) * 8ull),
               o_im = at(n_items * 4), o_ik = at(n_items * 4), o_r = at(n_items * 32), o_s = at(n_items * 32),
               o_pre = at(n_items), o_tab = at(n_keys * 8ull), o_st = at(n_items);
  // a latency batch: one host record per item (hostscalar.h) instead
  const bool rec_room = n_items <= ctx->host_scalar_max;
  const size_t o_rec = at(rec_room ? n_items * hrec::kWords * 4 : 0), o_clk = at((n_items + 1) * 8);
  if (bv_wait_all(ctx) != BV_OK) return BV_E_LAUNCH;  // the previous call may still read the buffer
  const auto t_waited = std::chrono::steady_clock::now();
  ctx->small_io.flags = hipHostMallocMapped | hipHostMallocCoherent;
  HIPCHK(ctx->small_io.ensure(total), BV_E_OOM, "alloc small-batch buffer");
  uint8_t *pin = (uint8_t *)ctx->small_io.p;
  if (ctx->small_io_host != pin || ctx->small_io_cap != ctx->small_io.cap) {  // the alias, once per allocation
    HIPCHK(hipHostGetDevicePointer((void **)&ctx->small_io_dev, pin, 0), BV_E_LAUNCH, "device pointer (small batch)");
    ctx->small_io_host = pin;
    ctx->small_io_cap = ctx->small_io.cap;
  }
  uint8_t *dev = ctx->small_io_dev;
  auto put = [&](size_t o, const void *src, size_t n) {
    if (n) memcpy(pin + o, src, n);
  };
  // SHA-256 of every message on the host (SHA extensions; the messages are
  // <= 16 KB, a few hundred at most): the kernel's first phase is s^-1 alone
  uint8_t *dig = pin + o_dig;
  auto hash = [b, dig](uint64_t lo, uint64_t hi) {
    for (uint64_t m = lo; m < hi; m++)
      hsha::digest(b->msg_bytes + b->msg_off[m], b->msg_off[m + 1] - b->msg_off[m], dig + 32 * m);
    return true;
  };
  if (n_msgs <= 16) hash(0, n_msgs);
  else ctx->pool->parallel_for(n_msgs, 16, hash);
  put(o_key, b->key_bytes, key_len);
  memset(pin + o_key + key_len, 0, 64);
  put(o_koff, b->key_off, (n_keys + 1) * 8ull);
  put(o_im, b->item_msg, n_items * 4);
  put(o_ik, b->item_key, n_items * 4);
  put(o_r, b->r_be, n_items * 32);
  put(o_s, b->s_be, n_items * 32);
  if (b->pre) put(o_pre, b->pre, n_items);
  // statuses start as a sentinel no status takes: the host sees each one
  // land in this (coherent) buffer and returns without waiting for the
  // kernel's completion signal
  volatile uint8_t *stv = pin + o_st;
  memset(pin + o_st, kSmallPending, n_items);
  memset(pin + o_clk, 0, (n_items + 1) * 8);
  const bool kc = (ctx->flags & BV_F_KEY_CACHE) && n_keys;
  uint32_t hits = 0;
  if (kc) hits = bv_kc_lookup(ctx, n_keys, b->key_bytes, b->key_off, (uint64_t *)(pin + o_tab));
  // Records when the scalar chain is the kernel's critical path: up to 4
  // items always, up to host_scalar_max when every item's key has a
  // key-cache table.  A table-less key's Q chain (~0.25 ms) hides the device's s^-1,
  // and there the host's records only add host time; past ~16 items the
  // host batch costs more than the device's parallel inversions (measured:
  // profiles/r06_small_lat_hs128.log / r06_small_lat_hs4.log).
  bool recs = rec_room && (n_items <= 4 || kc);
  if (recs && n_items > 4)
    for (uint64_t i = 0; i < n_items && recs; i++) recs = ((const uint64_t *)(pin + o_tab))[b->item_key[i]] != 0;
  if (recs) {  // the items' scalar halves, kHostRecGrain items per pool task (one inversion each)
    const uint64_t *tabs = (const uint64_t *)(pin + o_tab);
    std::vector<HostRecItem> &it = ctx->rec_items;
    it.resize(n_items);
    for (uint64_t i = 0; i < n_items; i++) {
      const uint32_t k = b->item_key[i];
      it[i] = {dig + 32ull * b->item_msg[i], b->r_be + 32 * i, b->s_be + 32 * i, b->key_bytes + b->key_off[k],
               b->key_off[k + 1] - b->key_off[k], kc ? tabs[k] : 0, (uint8_t)(b->pre ? b->pre[i] : 0)};
    }
    uint32_t *rp = (uint32_t *)(pin + o_rec);
    ctx->pool->parallel_for(n_items, kHostRecGrain, [&](uint64_t lo, uint64_t hi) {
      bv_host_item_records(rp + hrec::kWords * lo, it.data() + lo, hi - lo);
      return true;
    });
  }
  const auto t_staged = std::chrono::steady_clock::now();
  uint64_t *stamps = nullptr;
  if (ctx->small_stamps) {
    HIPCHK(ctx->d_stamps.ensure(16 * 8), BV_E_OOM, "alloc stamps");
    HIPCHK(hipMemsetAsync(ctx->d_stamps.p, 0, 16 * 8, st), BV_E_LAUNCH, "memset stamps");
    stamps = ctx->d_stamps.as<uint64_t>();
  }
  HIPCHK(bvk::verify_small(st, (uint32_t)n_items, dev + o_dig, dev + o_key, (const uint64_t *)(dev + o_koff),
                           (const uint32_t *)(dev + o_im), (const uint32_t *)(dev + o_ik), dev + o_r, dev + o_s,
                           b->pre ? dev + o_pre : nullptr, kc ? (const uint64_t *)(dev + o_tab) : nullptr,
                           ctx->g_table, dev + o_st, stamps, recs ? (const uint32_t *)(dev + o_rec) : nullptr,
                           (uint64_t *)(dev + o_clk)),
         BV_E_LAUNCH, "k_small");
  int rc = bv_mark_done(ctx, st);
  if (rc != BV_OK) return rc;
  const auto t_enq = std::chrono::steady_clock::now();
  if (res->msg_hash && n_msgs) memcpy(res->msg_hash, dig, n_msgs * 32);  // while the device works
  // Wait for the statuses themselves (each workgroup's one byte, written
  // last).  The completion event is polled beside them, so a launch that
  // ends without writing them all (a fault) is an error, never a hang; the
  // next call on this ctx waits for the event before touching the buffer.
  uint64_t seen = 0;
  for (uint64_t spins = 0;; spins++) {
    while (seen < n_items && stv[seen] != kSmallPending) seen++;
    if (seen == n_items) break;
    if ((spins & 255) == 255) {
      const hipError_t q = hipEventQuery(ctx->ev_done);
      if (q == hipSuccess) {
        while (seen < n_items && stv[seen] != kSmallPending) seen++;
        if (seen < n_items) return bv_fail(ctx, BV_E_LAUNCH, "k_small ended without every status", hipSuccess);
        break;
      }
      if (q != hipErrorNotReady) return bv_fail(ctx, BV_E_LAUNCH, "small batch sync", q);
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  const auto t_sync = std::chrono::steady_clock::now();
  if (res->status) memcpy(res->status, (const uint8_t *)stv, n_items);
  if (res->accept_bits) {
    memset(res->accept_bits, 0, (n_items + 63) / 64 * 8);
    for (uint64_t i = 0; i < n_items; i++)
      if (stv[i] == BV_ACCEPT) res->accept_bits[i / 64] |= 1ull << (i % 64);
  }
  bv_timing &t = ctx->timing;
  {  // the kernel's span from its own clock writes (wall_khz; each end lands before its status)
    const volatile uint64_t *clk = (const volatile uint64_t *)(pin + o_clk);
    uint64_t end = 0;
    for (uint64_t i = 0; i < n_items; i++) end = std::max<uint64_t>(end, (uint64_t)clk[1 + i]);
    const uint64_t start = clk[0];
    t.ms_total = t.ms_verify = start && end >= start ? (float)((double)(end - start) / ctx->wall_khz) : 0.f;
  }
  t.key_path = kc && hits ? BV_KCW : 0;
  t.kc_hits = hits;
  t.kc_keys = (uint32_t)ctx->kc_index.size();
  t.ms_host = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (stamps) {  // diagnostics: workgroup 0's phase clocks, relative to its start
    uint64_t h[16];
    HIPCHK(hipMemcpy(h, stamps, sizeof h, hipMemcpyDeviceToHost), BV_E_LAUNCH, "d2h stamps");
    auto us = [&](std::chrono::steady_clock::time_point a) {
      return std::chrono::duration<double, std::micro>(a - t0).count();
    };
    fprintf(stderr, "k_small host_us waited=%.1f staged=%.1f enqueued=%.1f synced=%.1f\n", us(t_waited),
            us(t_staged), us(t_enq), us(t_sync));
    fprintf(stderr, "k_small stamps n=%llu kernel_ms=%.4f:", (unsigned long long)n_items, t.ms_total);
    for (int k = 1; k < 14; k++) fprintf(stderr, " %d:%lld", k, h[k] ? (long long)(h[k] - h[0]) : -1ll);
    fprintf(stderr, "\n");
  }
  return BV_OK;
}

extern "C" int bv_verify_batch(bv_ctx *ctx, const bv_batch *b, bv_result *res) {
  if (!ctx || !b || !res) return BV_E_ARGS;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  if (ctx->small_path && small_batch(ctx, b)) {
    int rc = bv_validate_host_batch(ctx, b);
    if (rc != BV_OK) return rc;
    rc = small_verify(ctx, b, res);
    return rc == BV_OK ? rc : bv_drain(ctx, ctx->stream, rc);
  }
  bv_host_call call;
  int rc = bv_host_launch(ctx, b, &call, res);
  if (rc != BV_OK) return bv_drain(ctx, ctx->stream, rc);
  return bv_host_finish(ctx, b, res, &call, true);
}

extern "C" int bv_sha256_batch(bv_ctx *ctx, uint64_t n_msgs, const uint8_t *msg_bytes, const uint64_t *msg_off,
                               uint8_t *out_hash) {
  if (!ctx || (n_msgs && (!msg_bytes || !msg_off || !out_hash))) return BV_E_ARGS;
  if (n_msgs == 0) return BV_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  if (msg_off[0] != 0) return bv_fail(ctx, BV_E_ARGS, "msg_off[0] != 0");
  for (uint64_t m = 0; m < n_msgs; m++)
    if (msg_off[m] > msg_off[m + 1]) return bv_fail(ctx, BV_E_ARGS, "msg_off not monotone");
  hipStream_t st = ctx->stream;
  const uint64_t len = msg_off[n_msgs];
  if (bv_wait_all(ctx) != BV_OK) return BV_E_LAUNCH;  // previous calls' work buffers / staging
  const size_t o_off = align256(len + 64), total = o_off + align256((n_msgs + 1) * 8);
  HIPCHK(ctx->pin_in.ensure(total), BV_E_OOM, "alloc pinned staging");
  HIPCHK(ctx->d_in.ensure(total), BV_E_OOM, "alloc device staging");
  HIPCHK(ctx->pin_out.ensure(n_msgs * 32), BV_E_OOM, "alloc pinned results");
  HIPCHK(ctx->S().digests.ensure(n_msgs * 32), BV_E_OOM, "alloc digests");
  uint8_t *pin = (uint8_t *)ctx->pin_in.p, *dev = ctx->d_in.as<uint8_t>();
  ctx->pool->copy(pin, msg_bytes, len);
  memset(pin + len, 0, 64);
  memcpy(pin + o_off, msg_off, (n_msgs + 1) * 8);
  HIPCHK(hipMemcpyAsync(dev, pin, total, hipMemcpyHostToDevice, st), BV_E_LAUNCH, "h2d");
  HIPCHK(bvk::sha256(st, n_msgs, dev, (const uint64_t *)(dev + o_off), ctx->S().digests.as<uint32_t>()), BV_E_LAUNCH,
         "k_sha256");
  HIPCHK(hipMemcpyAsync(ctx->pin_out.p, ctx->S().digests.p, n_msgs * 32, hipMemcpyDeviceToHost, st), BV_E_LAUNCH, "d2h");
  if (bv_mark_done(ctx, st) != BV_OK) return BV_E_LAUNCH;
  HIPCHK(hipStreamSynchronize(st), BV_E_LAUNCH, "sync");
  memcpy(out_hash, ctx->pin_out.p, n_msgs * 32);
  return BV_OK;
}

extern "C" int bv_peer_set_hash(bv_ctx *ctx, uint32_t n_peers, const uint8_t *key_bytes, const uint64_t *key_off,
                                uint8_t out_hash[32]) {
  if (!ctx || !out_hash || (n_peers && !key_off)) return BV_E_ARGS;
  if (n_peers == 0) return BV_OK;  // []byte{}: nothing written
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  if (key_off[0] != 0) return bv_fail(ctx, BV_E_ARGS, "key_off[0] != 0");
  uint64_t maxlen = 0;
  for (uint32_t i = 0; i < n_peers; i++) {
    if (key_off[i] > key_off[i + 1]) return bv_fail(ctx, BV_E_ARGS, "key_off not monotone");
    maxlen = std::max<uint64_t>(maxlen, key_off[i + 1] - key_off[i]);
  }
  const uint64_t len = key_off[n_peers];
  if (len && !key_bytes) return bv_fail(ctx, BV_E_ARGS, "null key bytes");
  hipStream_t st = ctx->stream;
  if (bv_wait_all(ctx) != BV_OK) return BV_E_LAUNCH;  // previous calls' work buffers / staging
  const size_t o_off = align256(len + 8), o_scr = o_off + align256((n_peers + 1) * 8ull);
  const size_t total = o_scr + align256(32 + maxlen + 72);
  HIPCHK(ctx->pin_in.ensure(total), BV_E_OOM, "alloc pinned staging");
  HIPCHK(ctx->d_in.ensure(total + 32), BV_E_OOM, "alloc device staging");
  HIPCHK(ctx->pin_out.ensure(32), BV_E_OOM, "alloc pinned results");
  uint8_t *pin = (uint8_t *)ctx->pin_in.p, *dev = ctx->d_in.as<uint8_t>();
  if (len) memcpy(pin, key_bytes, len);
  memcpy(pin + o_off, key_off, (n_peers + 1) * 8ull);
  HIPCHK(hipMemcpyAsync(dev, pin, o_scr, hipMemcpyHostToDevice, st), BV_E_LAUNCH, "h2d");
  uint32_t *dout = (uint32_t *)(dev + total);
  HIPCHK(bvk::sha256_chain(st, n_peers, dev, (const uint64_t *)(dev + o_off), dev + o_scr, dout), BV_E_LAUNCH,
         "k_sha256_chain");
  HIPCHK(hipMemcpyAsync(ctx->pin_out.p, dout, 32, hipMemcpyDeviceToHost, st), BV_E_LAUNCH, "d2h");
  if (bv_mark_done(ctx, st) != BV_OK) return BV_E_LAUNCH;
  HIPCHK(hipStreamSynchronize(st), BV_E_LAUNCH, "sync");
  memcpy(out_hash, ctx->pin_out.p, 32);
  return BV_OK;
}
