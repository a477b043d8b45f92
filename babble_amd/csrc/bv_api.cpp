// bv_api.cpp — host side of libbabbleverify.so: the C ABI declared in
// include/babbleverify.h.
//
// One bv_ctx owns two HIP streams (main + keys), the generator table (16-bit
// windows, 64 MiB, built on the device at bv_create and kept resident in
// HBM) and growable device work buffers.  bv_verify_batch stages host
// buffers to HBM and runs the same device pipeline as
// bv_verify_batch_device.  There is no CPU fallback: a missing or
// non-gfx950 device is BV_E_NODEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/babbleverify.h"
#include "geometry.h"

namespace bvk {
hipError_t sha256(hipStream_t, uint64_t, const uint8_t *, const uint64_t *, uint32_t *);
hipError_t key_decode(hipStream_t, uint32_t, const uint8_t *, const uint64_t *, uint8_t *, uint32_t *);
hipError_t build_tables(hipStream_t, int, uint32_t, const uint32_t *, const uint8_t *, uint32_t *, uint32_t *,
                        uint32_t *, uint32_t *);
hipError_t sinv(hipStream_t, uint64_t, uint32_t, const uint32_t *, const uint8_t *, uint32_t *);
hipError_t verify_g(hipStream_t, uint64_t, const uint32_t *, const uint32_t *, const uint32_t *, const uint8_t *,
                    const uint8_t *, const uint32_t *, const uint32_t *, const uint32_t *, uint32_t *,
                    const uint32_t *, uint32_t *);
hipError_t verify_q(hipStream_t, int, uint64_t, const uint32_t *, const uint32_t *, const uint32_t *, const uint8_t *,
                    const uint8_t *, const uint32_t *, const uint32_t *, const uint32_t *, uint8_t *, uint64_t *);
hipError_t verify_generic(hipStream_t, uint64_t, const uint32_t *, const uint32_t *, const uint32_t *,
                          const uint8_t *, const uint8_t *, const uint32_t *, const uint32_t *, const uint32_t *,
                          const uint32_t *, const uint32_t *, uint8_t *, uint64_t *);
}  // namespace bvk

namespace {

// Table geometry (must match verify_core.h): generator 16-bit windows x 16
// (64 MiB, once per ctx); GLV key tables K8 (8-bit windows x 16 + phi,
// 512 KiB per key) or K12 (12-bit signed windows x 11 + phi, 2.75 MiB per key, from
// 22 six-bit sub-tables).
constexpr uint32_t kKNwin = 16;
constexpr uint64_t kGTableBytes = BV_GTABLE_U32 * 4;                 // 10.7 GB (geometry.h)
constexpr uint64_t kGSubBytes = BV_GSUB_U32 * 4;
constexpr uint64_t kGPrefixBytes = (uint64_t)BV_GPAIR_BLOCKS * 4096 * 32;  // one k_table_pair_g launch
constexpr uint64_t kKTableBytes = 2ull * kKNwin * (1ull << 8) * 64ull;
constexpr uint64_t kK12TableBytes = BV_K12TABLE_U32 * 4ull;
constexpr uint64_t kK12SubBytes = 22ull * 64 * 64;
constexpr uint64_t kK12PrefixBytes = (uint64_t)BV_K12NWIN * BV_K12ENT * 32;  // one fe per entry
constexpr uint32_t kBasesPerKey = 22;       // max(K8 16 windows, K12 22 sub-tables)
constexpr uint64_t kK12MinItemsPerKey = 2048;  // K12 pays for its 11x larger build above this
constexpr uint32_t kUStride = 12;  // per-item GLV words (k1, k2, signs)
constexpr uint32_t kMaxTableKeys = 8192;                                // K8: 4 GiB of key tables
constexpr uint32_t kMaxK12Keys = 1024;                                  // K12: 2.8 GiB
constexpr uint32_t kPrepM = 16;                                         // items per s^-1 batch
constexpr uint32_t kRgWords = 25;                                       // R_G words per item

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
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
      return e;
    }
    cap = want;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *as() const {
    return (T *)p;
  }
};

// timing events (see read_timing)
enum { E_START, E_FORK, E_SHA, E_SCALAR, E_G, E_JOINED, E_END, E_KEYS, E_SINV, E_COUNT };

}  // namespace

struct bv_ctx {
  int device = 0;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;   // main
  hipStream_t kstream = nullptr;  // key tables
  hipStream_t sstream = nullptr;  // batched s^-1
  std::mutex mu;
  std::string err;
  const uint32_t *g_table = nullptr;  // process-wide, per device (gtable_acquire)
  // staging for the host entry point
  DevBuf h_msg_bytes, h_msg_off, h_key_bytes, h_key_off, h_item_msg, h_item_key, h_r, h_s, h_pre;
  // work buffers
  DevBuf digests, kstatus, kxy, bases_jac, key_sub, key_pscr, key_table, scratch, u12, rg, status, bits;
  hipEvent_t ev[E_COUNT] = {};
  bool table_mode = false;
  int key_w = 0;  // 8 or 12 in table mode
  bv_timing timing = {};
};

static int fail(bv_ctx *c, int code, const char *what, hipError_t e = hipSuccess) {
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

#define HIPCHK(expr, code, what)                            \
  do {                                                      \
    hipError_t _e = (expr);                                 \
    if (_e != hipSuccess) return fail(ctx, code, what, _e); \
  } while (0)

static const uint8_t kGenerator[64] = {
    0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0, 0x62, 0x95, 0xCE, 0x87, 0x0B, 0x07,
    0x02, 0x9B, 0xFC, 0xDB, 0x2D, 0xCE, 0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98,
    0x48, 0x3A, 0xDA, 0x77, 0x26, 0xA3, 0xC4, 0x65, 0x5D, 0xA4, 0xFB, 0xFC, 0x0E, 0x11, 0x08, 0xA8,
    0xFD, 0x17, 0xB4, 0x48, 0xA6, 0x85, 0x54, 0x19, 0x9C, 0x47, 0xD0, 0x8F, 0xFB, 0x10, 0xD4, 0xB8};

extern "C" int bv_abi_version(void) { return BV_ABI_VERSION; }

extern "C" const char *bv_last_error(const bv_ctx *ctx) { return ctx ? ctx->err.c_str() : "null ctx"; }

extern "C" void bv_destroy(bv_ctx *ctx);

// The generator table is a constant: one copy per device and process,
// shared by every context (refcounted), built on first use.
// T[j][d] = d 2^(BV_GW j) G, j < BV_GNWIN, d < 2^BV_GW (geometry.h);
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
                           (uint32_t *)pscr, (uint32_t *)table) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
  }
  for (void *p : {xy, bases, sub, pscr})
    if (p) (void)hipFree(p);
  if (!ok) {
    if (table) (void)hipFree(table);
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

static int create_impl(bv_ctx *ctx) {
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking), BV_E_NODEVICE, "hipStreamCreate");
  HIPCHK(hipStreamCreateWithFlags(&ctx->kstream, hipStreamNonBlocking), BV_E_NODEVICE, "hipStreamCreate");
  HIPCHK(hipStreamCreateWithFlags(&ctx->sstream, hipStreamNonBlocking), BV_E_NODEVICE, "hipStreamCreate");
  for (auto &e : ctx->ev) HIPCHK(hipEventCreate(&e), BV_E_NODEVICE, "hipEventCreate");
  ctx->g_table = gtable_acquire(ctx->device, ctx->stream);
  if (!ctx->g_table) return fail(ctx, BV_E_OOM, "generator table (geometry.h, ~10.7 GB of HBM) build failed");
  return BV_OK;
}

extern "C" int bv_create(bv_ctx **out, int device, uint32_t flags) {
  if (!out) return BV_E_ARGS;
  *out = nullptr;
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
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->kstream) (void)hipStreamSynchronize(ctx->kstream);
  if (ctx->sstream) (void)hipStreamSynchronize(ctx->sstream);
  if (ctx->g_table) gtable_release(ctx->device);
  DevBuf *bufs[] = {&ctx->h_msg_bytes, &ctx->h_msg_off,
                    &ctx->h_key_bytes, &ctx->h_key_off, &ctx->h_item_msg, &ctx->h_item_key,  &ctx->h_r,
                    &ctx->h_s,         &ctx->h_pre,     &ctx->digests,    &ctx->kstatus,     &ctx->kxy,
                    &ctx->bases_jac,   &ctx->key_sub,     &ctx->key_pscr,    &ctx->key_table, &ctx->scratch,    &ctx->u12,         &ctx->rg,
                    &ctx->status,      &ctx->bits};
  for (auto *b : bufs) b->release();
  for (auto &e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->kstream) (void)hipStreamDestroy(ctx->kstream);
  if (ctx->sstream) (void)hipStreamDestroy(ctx->sstream);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

extern "C" int bv_get_timing(const bv_ctx *ctx, bv_timing *out) {
  if (!ctx || !out) return BV_E_ARGS;
  *out = ctx->timing;
  return BV_OK;
}

// Device pipeline over device-resident inputs.  msg_hash/status/bits may be
// null (ctx buffers are used).  Caller holds ctx->mu and has set the device.
static int run_device(bv_ctx *ctx, const bv_batch *b, uint8_t *d_msg_hash, uint8_t *d_status, uint64_t *d_bits,
                      hipStream_t st) {
  const uint64_t n_msgs = b->n_msgs, n_items = b->n_items;
  const uint32_t n_keys = b->n_keys;
  if (n_items > 0 && (!b->item_msg || !b->item_key || !b->r_be || !b->s_be))
    return fail(ctx, BV_E_ARGS, "null item arrays");
  if (n_msgs > 0 && !b->msg_off) return fail(ctx, BV_E_ARGS, "null msg_off");
  if (n_items > 0 && n_keys == 0) return fail(ctx, BV_E_ARGS, "items without keys");
  if (n_keys > 0 && !b->key_off) return fail(ctx, BV_E_ARGS, "null key_off");
  if (((uintptr_t)b->r_be | (uintptr_t)b->s_be) & 15)
    return fail(ctx, BV_E_ARGS, "r_be/s_be must be 16-byte aligned");

  uint32_t *dig = (uint32_t *)d_msg_hash;
  if (!dig || ((uintptr_t)dig & 15)) {
    HIPCHK(ctx->digests.ensure(std::max<uint64_t>(n_msgs, 1) * 32), BV_E_OOM, "alloc digests");
    dig = ctx->digests.as<uint32_t>();
  }
  uint8_t *status = d_status;
  if (!status) {
    HIPCHK(ctx->status.ensure(std::max<uint64_t>(n_items, 1)), BV_E_OOM, "alloc status");
    status = ctx->status.as<uint8_t>();
  }
  uint64_t *bits = d_bits;
  if (!bits) {
    HIPCHK(ctx->bits.ensure(std::max<uint64_t>((n_items + 63) / 64, 1) * 8), BV_E_OOM, "alloc bits");
    bits = ctx->bits.as<uint64_t>();
  }
  HIPCHK(ctx->kstatus.ensure(std::max<uint32_t>(n_keys, 1)), BV_E_OOM, "alloc kstatus");
  HIPCHK(ctx->kxy.ensure(std::max<uint32_t>(n_keys, 1) * 64ull), BV_E_OOM, "alloc kxy");
  HIPCHK(ctx->scratch.ensure(std::max<uint64_t>(n_items, 1) * 32), BV_E_OOM, "alloc scratch");
  HIPCHK(ctx->u12.ensure(std::max<uint64_t>(n_items, 1) * kUStride * 4), BV_E_OOM, "alloc u12");

  // Per-key fixed-base tables pay off once a key signs enough items; with
  // few items per key the generic per-lane path is cheaper.
  const bool table_mode = n_keys <= kMaxTableKeys && n_items >= 16ull * n_keys;
  const int key_w = !table_mode ? 0
                    : (n_keys <= kMaxK12Keys && n_items >= kK12MinItemsPerKey * n_keys && !(ctx->flags & BV_F_K8))
                        ? 12
                        : 8;
  ctx->table_mode = table_mode;
  ctx->key_w = key_w;
  if (table_mode) {
    const uint64_t nk = std::max<uint32_t>(n_keys, 1);
    HIPCHK(ctx->bases_jac.ensure(nk * kBasesPerKey * 96ull), BV_E_OOM, "alloc bases");
    if (key_w == 12) {
      HIPCHK(ctx->key_sub.ensure(nk * kK12SubBytes), BV_E_OOM, "alloc key sub-tables");
      HIPCHK(ctx->key_pscr.ensure(nk * kK12PrefixBytes), BV_E_OOM, "alloc key prefix scratch");
    }
    HIPCHK(ctx->key_table.ensure(nk * (key_w == 12 ? kK12TableBytes : kKTableBytes)), BV_E_OOM,
           "alloc key tables");
    HIPCHK(ctx->rg.ensure(std::max<uint64_t>(n_items, 1) * kRgWords * 4), BV_E_OOM, "alloc R_G");
  }

  hipEvent_t *ev = ctx->ev;
  const uint32_t *r32 = (const uint32_t *)b->r_be, *s32 = (const uint32_t *)b->s_be;
  uint32_t *w = ctx->scratch.as<uint32_t>(), *u12 = ctx->u12.as<uint32_t>();
  HIPCHK(hipEventRecord(ev[E_START], st), BV_E_LAUNCH, "event");
  // s^-1 needs only s: its own stream, concurrent with everything up to k_verify_g
  HIPCHK(hipStreamWaitEvent(ctx->sstream, ev[E_START], 0), BV_E_LAUNCH, "fork");
  HIPCHK(bvk::sinv(ctx->sstream, n_items, kPrepM, s32, b->pre, w), BV_E_LAUNCH, "k_sinv");
  HIPCHK(hipEventRecord(ev[E_SINV], ctx->sstream), BV_E_LAUNCH, "event");
  HIPCHK(bvk::key_decode(st, n_keys, b->key_bytes, b->key_off, ctx->kstatus.as<uint8_t>(), ctx->kxy.as<uint32_t>()),
         BV_E_LAUNCH, "k_key_decode");
  HIPCHK(hipEventRecord(ev[E_FORK], st), BV_E_LAUNCH, "event");
  if (table_mode) {  // key tables on the keys stream, concurrent with the main stream below
    HIPCHK(hipStreamWaitEvent(ctx->kstream, ev[E_FORK], 0), BV_E_LAUNCH, "fork");
    HIPCHK(bvk::build_tables(ctx->kstream, key_w, n_keys, ctx->kxy.as<uint32_t>(), ctx->kstatus.as<uint8_t>(),
                             ctx->bases_jac.as<uint32_t>(), ctx->key_sub.as<uint32_t>(),
                             ctx->key_pscr.as<uint32_t>(), ctx->key_table.as<uint32_t>()),
           BV_E_LAUNCH, "key tables");
    HIPCHK(hipEventRecord(ev[E_KEYS], ctx->kstream), BV_E_LAUNCH, "event");
  }
  HIPCHK(bvk::sha256(st, n_msgs, b->msg_bytes, b->msg_off, dig), BV_E_LAUNCH, "k_sha256");
  HIPCHK(hipEventRecord(ev[E_SHA], st), BV_E_LAUNCH, "event");
  HIPCHK(hipStreamWaitEvent(st, ev[E_SINV], 0), BV_E_LAUNCH, "join");
  HIPCHK(hipEventRecord(ev[E_SCALAR], st), BV_E_LAUNCH, "event");
  if (table_mode) {
    HIPCHK(bvk::verify_g(st, n_items, b->item_key, r32, s32, b->pre, ctx->kstatus.as<uint8_t>(), b->item_msg, dig, w,
                         u12, ctx->g_table, ctx->rg.as<uint32_t>()),
           BV_E_LAUNCH, "k_verify_g");
    HIPCHK(hipEventRecord(ev[E_G], st), BV_E_LAUNCH, "event");
    HIPCHK(hipStreamWaitEvent(st, ev[E_KEYS], 0), BV_E_LAUNCH, "join");
    HIPCHK(hipEventRecord(ev[E_JOINED], st), BV_E_LAUNCH, "event");
    HIPCHK(bvk::verify_q(st, key_w, n_items, b->item_key, r32, s32, b->pre, ctx->kstatus.as<uint8_t>(), u12,
                         ctx->key_table.as<uint32_t>(), ctx->rg.as<uint32_t>(), status, bits),
           BV_E_LAUNCH, "k_verify_q");
  } else {
    HIPCHK(hipEventRecord(ev[E_G], st), BV_E_LAUNCH, "event");
    HIPCHK(hipEventRecord(ev[E_JOINED], st), BV_E_LAUNCH, "event");
    HIPCHK(bvk::verify_generic(st, n_items, b->item_key, r32, s32, b->pre, ctx->kstatus.as<uint8_t>(),
                               ctx->kxy.as<uint32_t>(), b->item_msg, dig, w, ctx->g_table, status,
                               bits),
           BV_E_LAUNCH, "k_verify_generic");
  }
  HIPCHK(hipEventRecord(ev[E_END], st), BV_E_LAUNCH, "event");
  if (d_msg_hash && (uint8_t *)dig != d_msg_hash)
    HIPCHK(hipMemcpyAsync(d_msg_hash, dig, n_msgs * 32, hipMemcpyDeviceToDevice, st), BV_E_LAUNCH, "copy digests");
  return BV_OK;
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
  float t;
  return hipEventElapsedTime(&t, a, b) == hipSuccess ? t : -1.f;
}

static void read_timing(bv_ctx *ctx) {
  hipEvent_t *ev = ctx->ev;
  bv_timing &t = ctx->timing;
  t.ms_sha256 = elapsed(ev[E_FORK], ev[E_SHA]);
  t.key_path = (uint32_t)ctx->key_w;
  t.ms_keyprep = ctx->table_mode ? elapsed(ev[E_START], ev[E_KEYS]) : elapsed(ev[E_START], ev[E_FORK]);
  t.ms_scalar = elapsed(ev[E_START], ev[E_SINV]);
  t.ms_verify_g = elapsed(ev[E_SCALAR], ev[E_G]);
  t.ms_verify = elapsed(ev[E_JOINED], ev[E_END]);
  t.ms_total = elapsed(ev[E_START], ev[E_END]);
}

extern "C" int bv_verify_batch_device(bv_ctx *ctx, const bv_batch *dbatch, bv_result *dresult, void *stream,
                                      int async) {
  if (!ctx || !dbatch || !dresult) return BV_E_ARGS;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
  int rc = run_device(ctx, dbatch, dresult->msg_hash, dresult->status, dresult->accept_bits, st);
  if (rc != BV_OK) return rc;
  if (!async) {
    HIPCHK(hipStreamSynchronize(st), BV_E_LAUNCH, "verify sync");
    read_timing(ctx);
  }
  return BV_OK;
}

extern "C" int bv_verify_batch(bv_ctx *ctx, const bv_batch *b, bv_result *res) {
  if (!ctx || !b || !res) return BV_E_ARGS;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  hipStream_t st = ctx->stream;
  const uint64_t n_msgs = b->n_msgs, n_items = b->n_items;
  const uint32_t n_keys = b->n_keys;
  if ((n_msgs && !b->msg_off) || (n_keys && !b->key_off) ||
      (n_items && (!b->item_msg || !b->item_key || !b->r_be || !b->s_be)))
    return fail(ctx, BV_E_ARGS, "null input array");
  const uint64_t msg_len = n_msgs ? b->msg_off[n_msgs] : 0;
  const uint64_t key_len = n_keys ? b->key_off[n_keys] : 0;
  // byte arrays may be null only when empty (all-empty messages or keys)
  if ((msg_len && !b->msg_bytes) || (key_len && !b->key_bytes)) return fail(ctx, BV_E_ARGS, "null byte array");
  // validate host offsets (a bad offset must not become an OOB device read)
  if (n_msgs && b->msg_off[0] != 0) return fail(ctx, BV_E_ARGS, "msg_off[0] != 0");
  if (n_keys && b->key_off[0] != 0) return fail(ctx, BV_E_ARGS, "key_off[0] != 0");
  for (uint64_t m = 0; m < n_msgs; m++)
    if (b->msg_off[m] > b->msg_off[m + 1]) return fail(ctx, BV_E_ARGS, "msg_off not monotone");
  for (uint32_t k = 0; k < n_keys; k++)
    if (b->key_off[k] > b->key_off[k + 1]) return fail(ctx, BV_E_ARGS, "key_off not monotone");
  for (uint64_t i = 0; i < n_items; i++)
    if (b->item_msg[i] >= n_msgs || b->item_key[i] >= n_keys) return fail(ctx, BV_E_ARGS, "item index out of range");

  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0), BV_E_LAUNCH, "event");
  HIPCHK(hipEventCreate(&e1), BV_E_LAUNCH, "event");
  HIPCHK(hipEventRecord(e0, st), BV_E_LAUNCH, "event");
  HIPCHK(ctx->h_msg_bytes.ensure(msg_len + 64), BV_E_OOM, "alloc msg bytes");
  HIPCHK(ctx->h_msg_off.ensure((n_msgs + 1) * 8), BV_E_OOM, "alloc msg off");
  HIPCHK(ctx->h_key_bytes.ensure(key_len + 64), BV_E_OOM, "alloc key bytes");
  HIPCHK(ctx->h_key_off.ensure((uint64_t)(n_keys + 1) * 8), BV_E_OOM, "alloc key off");
  HIPCHK(ctx->h_item_msg.ensure(std::max<uint64_t>(n_items, 1) * 4), BV_E_OOM, "alloc item msg");
  HIPCHK(ctx->h_item_key.ensure(std::max<uint64_t>(n_items, 1) * 4), BV_E_OOM, "alloc item key");
  HIPCHK(ctx->h_r.ensure(std::max<uint64_t>(n_items, 1) * 32), BV_E_OOM, "alloc r");
  HIPCHK(ctx->h_s.ensure(std::max<uint64_t>(n_items, 1) * 32), BV_E_OOM, "alloc s");
  HIPCHK(ctx->h_pre.ensure(std::max<uint64_t>(n_items, 1)), BV_E_OOM, "alloc pre");
  auto h2d = [&](DevBuf &d, const void *src, size_t n) -> hipError_t {
    if (n == 0) return hipSuccess;
    return hipMemcpyAsync(d.p, src, n, hipMemcpyHostToDevice, st);
  };
  HIPCHK(h2d(ctx->h_msg_bytes, b->msg_bytes, msg_len), BV_E_LAUNCH, "h2d msg");
  if (n_msgs) HIPCHK(h2d(ctx->h_msg_off, b->msg_off, (n_msgs + 1) * 8), BV_E_LAUNCH, "h2d msg off");
  HIPCHK(h2d(ctx->h_key_bytes, b->key_bytes, key_len), BV_E_LAUNCH, "h2d keys");
  if (n_keys) HIPCHK(h2d(ctx->h_key_off, b->key_off, (uint64_t)(n_keys + 1) * 8), BV_E_LAUNCH, "h2d key off");
  HIPCHK(h2d(ctx->h_item_msg, b->item_msg, n_items * 4), BV_E_LAUNCH, "h2d item msg");
  HIPCHK(h2d(ctx->h_item_key, b->item_key, n_items * 4), BV_E_LAUNCH, "h2d item key");
  HIPCHK(h2d(ctx->h_r, b->r_be, n_items * 32), BV_E_LAUNCH, "h2d r");
  HIPCHK(h2d(ctx->h_s, b->s_be, n_items * 32), BV_E_LAUNCH, "h2d s");
  if (b->pre) HIPCHK(h2d(ctx->h_pre, b->pre, n_items), BV_E_LAUNCH, "h2d pre");
  bv_batch d = {};
  d.n_msgs = n_msgs;
  d.msg_bytes = ctx->h_msg_bytes.as<uint8_t>();
  d.msg_off = ctx->h_msg_off.as<uint64_t>();
  d.n_keys = n_keys;
  d.key_bytes = ctx->h_key_bytes.as<uint8_t>();
  d.key_off = ctx->h_key_off.as<uint64_t>();
  d.n_items = n_items;
  d.item_msg = ctx->h_item_msg.as<uint32_t>();
  d.item_key = ctx->h_item_key.as<uint32_t>();
  d.r_be = ctx->h_r.as<uint8_t>();
  d.s_be = ctx->h_s.as<uint8_t>();
  d.pre = b->pre ? ctx->h_pre.as<uint8_t>() : nullptr;
  int rc = run_device(ctx, &d, nullptr, nullptr, nullptr, st);
  if (rc != BV_OK) return rc;
  if (res->msg_hash && n_msgs)
    HIPCHK(hipMemcpyAsync(res->msg_hash, ctx->digests.p, n_msgs * 32, hipMemcpyDeviceToHost, st), BV_E_LAUNCH,
           "d2h digests");
  if (res->status && n_items)
    HIPCHK(hipMemcpyAsync(res->status, ctx->status.p, n_items, hipMemcpyDeviceToHost, st), BV_E_LAUNCH, "d2h status");
  if (res->accept_bits && n_items)
    HIPCHK(hipMemcpyAsync(res->accept_bits, ctx->bits.p, (n_items + 63) / 64 * 8, hipMemcpyDeviceToHost, st),
           BV_E_LAUNCH, "d2h bits");
  HIPCHK(hipEventRecord(e1, st), BV_E_LAUNCH, "event");
  HIPCHK(hipStreamSynchronize(st), BV_E_LAUNCH, "verify sync");
  read_timing(ctx);
  ctx->timing.ms_h2d = elapsed(e0, ctx->ev[E_START]);
  ctx->timing.ms_d2h = elapsed(ctx->ev[E_END], e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return BV_OK;
}

extern "C" int bv_sha256_batch(bv_ctx *ctx, uint64_t n_msgs, const uint8_t *msg_bytes, const uint64_t *msg_off,
                               uint8_t *out_hash) {
  if (!ctx || (n_msgs && (!msg_bytes || !msg_off || !out_hash))) return BV_E_ARGS;
  if (n_msgs == 0) return BV_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  if (msg_off[0] != 0) return fail(ctx, BV_E_ARGS, "msg_off[0] != 0");
  for (uint64_t m = 0; m < n_msgs; m++)
    if (msg_off[m] > msg_off[m + 1]) return fail(ctx, BV_E_ARGS, "msg_off not monotone");
  hipStream_t st = ctx->stream;
  const uint64_t len = msg_off[n_msgs];
  HIPCHK(ctx->h_msg_bytes.ensure(len + 64), BV_E_OOM, "alloc msg bytes");
  HIPCHK(ctx->h_msg_off.ensure((n_msgs + 1) * 8), BV_E_OOM, "alloc msg off");
  HIPCHK(ctx->digests.ensure(n_msgs * 32), BV_E_OOM, "alloc digests");
  if (len) HIPCHK(hipMemcpyAsync(ctx->h_msg_bytes.p, msg_bytes, len, hipMemcpyHostToDevice, st), BV_E_LAUNCH, "h2d");
  HIPCHK(hipMemcpyAsync(ctx->h_msg_off.p, msg_off, (n_msgs + 1) * 8, hipMemcpyHostToDevice, st), BV_E_LAUNCH, "h2d");
  HIPCHK(bvk::sha256(st, n_msgs, ctx->h_msg_bytes.as<uint8_t>(), ctx->h_msg_off.as<uint64_t>(),
                     ctx->digests.as<uint32_t>()),
         BV_E_LAUNCH, "k_sha256");
  HIPCHK(hipMemcpyAsync(out_hash, ctx->digests.p, n_msgs * 32, hipMemcpyDeviceToHost, st), BV_E_LAUNCH, "d2h");
  HIPCHK(hipStreamSynchronize(st), BV_E_LAUNCH, "sync");
  return BV_OK;
}
