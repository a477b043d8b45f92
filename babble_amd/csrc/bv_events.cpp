// bv_verify_events: canonical EventBody JSON built from wire fields, hashed,
// then the verify pipeline (include/babbleverify.h).
//
// Bulk batches (no in-batch parent: a store / bootstrap replay, parents by
// known hash): host work is validation and the staging of the compact wire
// arrays; each chunk's bodies are serialised straight into SHA-256 on the
// device (k_ev_body_hash, one lane per event: no body ever stored) while the
// next chunk crosses PCIe, and each chunk's items are verified beside the
// next chunk's hashing.  Batches with in-batch parents (a SyncResponse's DAG:
// each body embeds its parents' hashes) are built and hashed on the host in
// topological order instead (hostdag.cpp; the serial chain is ~50x faster on
// one CPU core than on one GPU wave: 0.8 vs 5.5 ms per 1000-event
// SyncResponse, profiles/r04_ab_dag.log) while the device runs key decode,
// key tables and s^-1; only the digests cross PCIe.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "bv_internal.h"

#define HIPCHK(expr, code, what)                               \
  do {                                                         \
    hipError_t _e = (expr);                                    \
    if (_e != hipSuccess) return bv_fail(ctx, code, what, _e); \
  } while (0)

namespace {

// staged bytes per PCIe piece / event chunk: 64 MB (~250k C2 events) keeps
// each chunk's verify launches at full occupancy while the next chunk
// crosses PCIe (1M bulk events, same box: 16 / 32 / 64 / 128 MB / one
// chunk = 8.6-9.0 / 7.8-8.3 / 7.25-7.5 / 7.7 / 7.7-8.2 ms per call from
// pinned arrays, tools/events_prof.py)
constexpr size_t kChunk = 64ull << 20;
constexpr uint64_t kEvTailMin = 65536;  // events: the smallest chunk the halving tail splits off

int validate(bv_ctx *ctx, const bv_event_batch *b) {
  const uint64_t n = b->n_events;
  if (!n) return BV_OK;
  if (!b->creator || !b->index || !b->timestamp || !b->parent_kind || !b->parent_ref || !b->tx_start ||
      (!b->sig_text && (!b->r_be || !b->s_be)) || !b->key_off)
    return bv_fail(ctx, BV_E_ARGS, "null event array");
  if (b->sig_text) {  // signature text: offsets from 0, monotone
    if (!b->sig_off || b->sig_off[0] != 0) return bv_fail(ctx, BV_E_ARGS, "sig_off missing or sig_off[0] != 0");
    if (!ctx->pool->parallel_for(n, 1 << 17, [b](uint64_t lo, uint64_t hi) {
          for (uint64_t e = lo; e < hi; e++)
            if (b->sig_off[e] > b->sig_off[e + 1]) return false;
          return true;
        }))
      return bv_fail(ctx, BV_E_ARGS, "sig_off not monotone");
  }
  if (b->key_off[0] != 0) return bv_fail(ctx, BV_E_ARGS, "key_off[0] != 0");
  for (uint32_t k = 0; k < b->n_keys; k++)
    if (b->key_off[k] > b->key_off[k + 1]) return bv_fail(ctx, BV_E_ARGS, "key_off not monotone");
  if (b->key_off[b->n_keys] && !b->key_bytes) return bv_fail(ctx, BV_E_ARGS, "null key bytes");
  if (b->tx_start[0] != 0) return bv_fail(ctx, BV_E_ARGS, "tx_start[0] != 0");
  const uint64_t n_tx = b->tx_start[n];
  if (n_tx && !b->tx_off) return bv_fail(ctx, BV_E_ARGS, "null tx_off");
  if (n_tx && b->tx_off[0] != 0) return bv_fail(ctx, BV_E_ARGS, "tx_off[0] != 0");
  constexpr uint64_t kGrain = 1 << 17;
  if (!ctx->pool->parallel_for(n_tx, kGrain, [b](uint64_t lo, uint64_t hi) {
        for (uint64_t t = lo; t < hi; t++)
          if (b->tx_off[t] > b->tx_off[t + 1]) return false;
        return true;
      }))
    return bv_fail(ctx, BV_E_ARGS, "tx_off not monotone");
  if (n_tx && b->tx_off[n_tx] && !b->tx_bytes) return bv_fail(ctx, BV_E_ARGS, "null tx bytes");
  for (const uint64_t *off : {b->itx_off, b->bsig_off})
    if (off && off[0] != 0) return bv_fail(ctx, BV_E_ARGS, "fragment offsets must start at 0");
  if ((b->itx_off && b->itx_off[n] && !b->itx_json) || (b->bsig_off && b->bsig_off[n] && !b->bsig_json))
    return bv_fail(ctx, BV_E_ARGS, "null fragment bytes");
  for (const uint64_t *off : {b->itx_off, b->bsig_off})
    if (off && !ctx->pool->parallel_for(n, kGrain, [off](uint64_t lo, uint64_t hi) {
          for (uint64_t e = lo; e < hi; e++)
            if (off[e] > off[e + 1]) return false;
          return true;
        }))
      return bv_fail(ctx, BV_E_ARGS, "fragment offsets not monotone");
  if (!ctx->pool->parallel_for(n, kGrain, [b](uint64_t lo, uint64_t hi) {
        for (uint64_t e = lo; e < hi; e++) {
          if (b->creator[e] >= b->n_keys || b->tx_start[e] > b->tx_start[e + 1]) return false;
          for (int p = 0; p < 2; p++) {
            const uint8_t k = b->parent_kind[2 * e + p];
            const uint64_t r = b->parent_ref[2 * e + p];
            if (k > BV_PARENT_EVENT) return false;
            if (k == BV_PARENT_HASH && (r >= b->n_parent_hashes || !b->parent_hashes)) return false;
            if (k == BV_PARENT_EVENT && r >= e) return false;  // an in-batch parent precedes its child
          }
        }
        return true;
      }))
    return bv_fail(ctx, BV_E_ARGS,
                   "bad event reference (creator, tx_start, or a parent not earlier in the batch / out of range)");
  return BV_OK;
}

// Signature text (eb->sig_text): the device decodes r, s and pre into
// ctx->d_sig on the s^-1 stream once the text has landed (`text_ready`),
// ahead of s^-1; E_SDEC marks them written.  Returns the device arrays.
struct SigOut {
  uint8_t *r = nullptr, *s = nullptr, *pre = nullptr;
};
int sig_decode_on_device(bv_ctx *ctx, uint64_t n, const uint64_t *d_off, const uint8_t *d_text, hipEvent_t text_ready,
                         SigOut *out) {
  const size_t rs = align256(n * 32);
  HIPCHK(ctx->d_sig.ensure(2 * rs + align256(n)), BV_E_OOM, "alloc decoded signatures");
  uint8_t *base = ctx->d_sig.as<uint8_t>();
  out->r = base, out->s = base + rs, out->pre = base + 2 * rs;
  HIPCHK(hipStreamWaitEvent(ctx->sstream, text_ready, 0), BV_E_LAUNCH, "join signature text");
  HIPCHK(bvk::sig_decode(ctx->sstream, n, d_off, d_text, out->r, out->s, out->pre), BV_E_LAUNCH, "k_sig_decode");
  HIPCHK(hipEventRecord(ctx->S().ev[E_SDEC], ctx->sstream), BV_E_LAUNCH, "event");
  return BV_OK;
}

}  // namespace

static int verify_events_impl(bv_ctx *ctx, const bv_event_batch *eb, bv_result *res);

// A batch with in-batch parents (a SyncResponse, core.go:214-245): the host
// builds and hashes the bodies in topological order (hostdag.cpp) while the
// device runs key decode, the key tables and s^-1 on the keys / s / pre that
// crossed PCIe first; then only the 32-byte digests cross and the verify
// kernels run.  The bodies never reach the device.
static int verify_events_dag_host(bv_ctx *ctx, const bv_event_batch *eb, bv_result *res,
                                  const std::vector<uint32_t> &order, const std::vector<uint32_t> &level_off,
                                  bv_host_call &call) {
  const uint64_t n = eb->n_events;
  hipStream_t st = ctx->stream;
  const uint64_t key_len = eb->key_off[eb->n_keys];
  // staging layout: keys | s, pre | r, creators | digests
  size_t total = 0;
  auto at = [&](size_t bytes, size_t pad = 0) {
    const size_t o = total;
    total += align256(bytes + pad);
    return o;
  };
  const size_t o_koff = at((eb->n_keys + 1) * 8ull), o_kb = at(key_len, 64), keys_end = total;
  // s and pre, or the signature text (decoded on the device: r, s, pre)
  const bool text = eb->sig_text != nullptr;
  const uint64_t text_len = text ? eb->sig_off[n] : 0;
  const size_t o_s = at(text ? (n + 1) * 8 : n * 32), o_pre = at(text ? text_len : (eb->pre ? n : 0)), s_end = total;
  const size_t o_r = at(text ? 0 : n * 32), o_cr = at(n * 4), small_end = total;
  const size_t o_dig = at(n * 32);
  if (bv_wait_all(ctx) != BV_OK) return BV_E_LAUNCH;  // previous calls' work buffers / staging
  HIPCHK(ctx->pin_in.ensure(total), BV_E_OOM, "alloc pinned staging");
  HIPCHK(ctx->d_in.ensure(total), BV_E_OOM, "alloc device staging");
  HIPCHK(ctx->ev_iota.ensure(n * 4), BV_E_OOM, "alloc item index");
  uint8_t *pin = (uint8_t *)ctx->pin_in.p, *dev = ctx->d_in.as<uint8_t>();
  hipStream_t cs = bv_copy_stream(ctx);
  if (!cs) return bv_fail(ctx, BV_E_NODEVICE, "copy stream");
  HIPCHK(hipEventRecord(ctx->S().ev[E_CALL], cs), BV_E_LAUNCH, "event");
  auto put = [&](size_t o, const void *src, size_t bytes) {
    if (bytes) memcpy(pin + o, src, bytes);
  };
  auto h2d = [&](size_t a, size_t z) -> int {
    HIPCHK(hipMemcpyAsync(dev + a, pin + a, z - a, hipMemcpyHostToDevice, cs), BV_E_LAUNCH, "h2d");
    return BV_OK;
  };
  put(o_koff, eb->key_off, (eb->n_keys + 1) * 8ull);
  put(o_kb, eb->key_bytes, key_len);
  memset(pin + o_kb + key_len, 0, 64);
  int rc = h2d(0, keys_end);
  if (rc != BV_OK) return rc;
  HIPCHK(hipEventRecord(ctx->S().ev[E_KREADY], cs), BV_E_LAUNCH, "event");
  bv_batch vb = {};
  vb.n_msgs = n;
  vb.n_keys = eb->n_keys;
  vb.key_bytes = dev + o_kb;
  vb.key_off = (const uint64_t *)(dev + o_koff);
  vb.n_items = n;
  vb.item_msg = ctx->ev_iota.as<uint32_t>();
  vb.item_key = (const uint32_t *)(dev + o_cr);
  vb.r_be = dev + o_r;
  vb.s_be = dev + o_s;
  vb.pre = eb->pre ? dev + o_pre : nullptr;
  bool kc = false;
  if (ctx->flags & BV_F_KEY_CACHE) {
    HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_KREADY], 0), BV_E_LAUNCH, "join");
    bv_kc_items items;
    items.n_items = eb->n_events;
    items.h_item_key = eb->creator;
    rc = bv_kc_prepare(ctx, eb->n_keys, eb->key_bytes, eb->key_off, vb.key_bytes, vb.key_off, st, &kc, false, &items);
    if (rc != BV_OK) return rc;
  }
  if (text) {
    put(o_s, eb->sig_off, (n + 1) * 8);
    put(o_pre, eb->sig_text, text_len);
  } else {
    put(o_s, eb->s_be, n * 32);
    if (eb->pre) put(o_pre, eb->pre, n);
  }
  if ((rc = h2d(keys_end, s_end)) != BV_OK) return rc;
  HIPCHK(hipEventRecord(ctx->S().ev[E_SREADY], cs), BV_E_LAUNCH, "event");
  if (text) {
    SigOut so;
    rc = sig_decode_on_device(ctx, n, (const uint64_t *)(dev + o_s), dev + o_pre, ctx->S().ev[E_SREADY], &so);
    if (rc != BV_OK) return rc;
    vb.r_be = so.r, vb.s_be = so.s, vb.pre = so.pre;
  }
  rc = bv_run_keys(ctx, &vb, ctx->S().ev[E_KREADY], ctx->S().ev[E_SREADY], kc);
  if (rc != BV_OK) return rc;
  if (!text) put(o_r, eb->r_be, n * 32);
  put(o_cr, eb->creator, n * 4);
  if ((rc = h2d(s_end, small_end)) != BV_OK) return rc;
  HIPCHK(hipEventRecord(ctx->S().ev[E_SMALL], cs), BV_E_LAUNCH, "event");
  HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_SMALL], 0), BV_E_LAUNCH, "join");
  if (text) HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_SDEC], 0), BV_E_LAUNCH, "join decoded signatures");
  HIPCHK(bvk::iota(st, n, ctx->ev_iota.as<uint32_t>()), BV_E_LAUNCH, "k_iota");
  HIPCHK(hipEventRecord(ctx->S().ev[E_FORK], st), BV_E_LAUNCH, "event");

  // the host's part, overlapping the device's key / s^-1 work
  const HostParFor pf = [ctx](uint64_t cnt, uint64_t grain, const std::function<void(uint64_t, uint64_t)> &fn) {
    ctx->pool->parallel_for(cnt, grain, [&fn](uint64_t lo, uint64_t hi) {
      fn(lo, hi);
      return true;
    });
  };
  bv_host_dag_hash(*eb, order.data(), level_off.data(), (uint32_t)level_off.size() - 1, pf, ctx->dag_scratch,
                   pin + o_dig);
  if ((rc = h2d(o_dig, o_dig + n * 32)) != BV_OK) return rc;
  HIPCHK(hipEventRecord(ctx->S().ev[E_STAGED], cs), BV_E_LAUNCH, "event");
  call.ms_prep = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - call.t0).count();
  HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_STAGED], 0), BV_E_LAUNCH, "join digests");
  HIPCHK(hipEventRecord(ctx->S().ev[E_SHA], st), BV_E_LAUNCH, "event");
  HIPCHK(hipEventRecord(ctx->S().ev[E_HASHED], st), BV_E_LAUNCH, "event");
  bv_item_pipe pipe{ctx, &vb, {}, st, kc};
  rc = bv_out_bufs(ctx, &vb, nullptr, nullptr, nullptr, true, &pipe.o);
  if (rc != BV_OK) return rc;
  pipe.o.dig = (uint32_t *)(dev + o_dig);
  rc = pipe.finish();
  if (rc != BV_OK) return rc;
  const size_t o_bits = align256(n);
  HIPCHK(ctx->pin_out.ensure(o_bits + align256((n + 63) / 64 * 8) + 256), BV_E_OOM, "alloc pinned results");
  uint8_t *pout = (uint8_t *)ctx->pin_out.p;
  call.pout = pout;
  call.o_st = 0;
  call.o_bits = o_bits;
  call.direct_hash = true;  // the digests are already on the host: copied below
  call.direct_status = res && bv_is_pinned(res->status, n);
  HIPCHK(hipMemcpyAsync(call.direct_status ? res->status : pout, pipe.o.status, n, hipMemcpyDeviceToHost, st),
         BV_E_LAUNCH, "d2h status");
  HIPCHK(hipMemcpyAsync(pout + o_bits, pipe.o.bits, (n + 63) / 64 * 8, hipMemcpyDeviceToHost, st), BV_E_LAUNCH,
         "d2h bits");
  HIPCHK(hipEventRecord(ctx->S().ev[E_OUT], st), BV_E_LAUNCH, "event");
  rc = bv_mark_done(ctx, st);
  if (rc != BV_OK) return rc;
  if (res->msg_hash) memcpy(res->msg_hash, pin + o_dig, n * 32);
  bv_batch sizes = {};
  sizes.n_msgs = n;
  sizes.n_items = n;
  return bv_host_finish(ctx, &sizes, res, &call, true);
}

extern "C" int bv_verify_events(bv_ctx *ctx, const bv_event_batch *eb, bv_result *res) {
  if (!ctx || !eb || !res) return BV_E_ARGS;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device), BV_E_NODEVICE, "hipSetDevice");
  const int rc = verify_events_impl(ctx, eb, res);
  return rc == BV_OK ? rc : bv_drain(ctx, ctx->stream, rc);
}

static int verify_events_impl(bv_ctx *ctx, const bv_event_batch *eb, bv_result *res) {
  bv_host_call call;
  call.t0 = std::chrono::steady_clock::now();
  int rc = validate(ctx, eb);
  if (rc != BV_OK) return rc;
  ctx->timing = bv_timing{};
  const uint64_t n = eb->n_events;
  hipStream_t st = ctx->stream;
  ctx->last = st;
  if (n == 0) return BV_OK;

  // DAG levels over in-batch parents (refs point backwards: one pass)
  std::vector<uint32_t> level, order, level_off;
  const bool dag = memchr(eb->parent_kind, BV_PARENT_EVENT, 2 * n) != nullptr;
  if (dag) {
    level.assign(n, 0);
    uint32_t nl = 1;
    for (uint64_t e = 0; e < n; e++) {
      uint32_t l = 0;
      for (int p = 0; p < 2; p++)
        if (eb->parent_kind[2 * e + p] == BV_PARENT_EVENT) l = std::max(l, level[eb->parent_ref[2 * e + p]] + 1);
      level[e] = l;
      nl = std::max(nl, l + 1);
    }
    level_off.assign(nl + 1, 0);
    for (uint64_t e = 0; e < n; e++) level_off[level[e] + 1]++;
    for (uint32_t l = 0; l < nl; l++) level_off[l + 1] += level_off[l];
    order.resize(n);
    std::vector<uint32_t> fill(level_off.begin(), level_off.end() - 1);
    for (uint64_t e = 0; e < n; e++) order[fill[level[e]]++] = (uint32_t)e;
    return verify_events_dag_host(ctx, eb, res, order, level_off, call);
  }

  // staging layout (pinned host and HBM): the compact wire arrays
  const uint64_t n_tx = eb->tx_start[n];
  const uint64_t tx_len = n_tx ? eb->tx_off[n_tx] : 0;
  const uint64_t key_len = eb->key_off[eb->n_keys];
  const uint64_t itx_len = eb->itx_off ? eb->itx_off[n] : 0, bsig_len = eb->bsig_off ? eb->bsig_off[n] : 0;
  // How a segment splits over an event chunk [e0, e1): ALL = whole, in the
  // first part; EV = `unit` bytes per event; EV1 = an n + 1 offset array
  // (elements e0 ..= e1); TX / TX1 = the same per transaction of the chunk's
  // events; TXB / ITX / BSIG = the chunk's bytes of tx_bytes / itx_json /
  // bsig_json.
  enum Kind { ALL, EV, EV1, TX, TX1, TXB, ITX, BSIG };
  struct Seg {
    const void *src;
    size_t n, off;
    Kind kind;
    size_t unit;
  };
  std::vector<Seg> segs;
  size_t total = 0;
  auto add = [&](const void *src, size_t bytes, Kind kind, size_t unit = 1, size_t pad = 0) -> size_t {
    segs.push_back({src, bytes, total, kind, unit});
    const size_t o = total;
    total += align256(bytes + pad);
    return o;
  };
  // keys first (the key tables start once they land), then s and pre (s^-1)
  // and the parent hashes (any event may name any of them); the per-event
  // fields, r and the creators among them, follow chunk by chunk (each
  // chunk's bodies are hashed and its items verified while the next one
  // crosses PCIe)
  const size_t o_koff = add(eb->key_off, (eb->n_keys + 1) * 8ull, ALL);
  const size_t o_kb = add(eb->key_bytes, key_len, ALL, 1, 64);
  const size_t keys_end = total;
  // s and pre, or the signature text (decoded on the device into r, s, pre)
  const bool text = eb->sig_text != nullptr;
  const size_t o_s = text ? add(eb->sig_off, (n + 1) * 8, ALL) : add(eb->s_be, n * 32, ALL);
  const size_t o_pre = text ? add(eb->sig_text, eb->sig_off[n], ALL) : add(eb->pre, eb->pre ? n : 0, ALL);
  const size_t s_end = total;
  // key part first (ctx->qfirst): r and the creators cross before the
  // chunks, so every item's k1 Q + k2 phi(Q) is summed under the transfer
  // of the bodies and only u1 G waits for each chunk's digests
  const bool qf = ctx->qfirst;
  const size_t o_r = qf && !text ? add(eb->r_be, n * 32, ALL) : 0;
  const size_t o_cr = qf ? add(eb->creator, n * 4, ALL) : 0;
  const size_t r_end = total;
  const size_t o_ph = add(eb->parent_hashes, eb->parent_hashes ? eb->n_parent_hashes * 32 : 0, ALL);
  const size_t small_end = total;
  const size_t o_r_ev = qf || text ? o_r : add(eb->r_be, n * 32, EV, 32);
  const size_t o_cr_ev = qf ? o_cr : add(eb->creator, n * 4, EV, 4);
  const size_t o_ix = add(eb->index, n * 8, EV, 8);
  const size_t o_ts = add(eb->timestamp, n * 8, EV, 8);
  const size_t o_pk = add(eb->parent_kind, n * 2, EV, 2);
  const size_t o_pr = add(eb->parent_ref, n * 16, EV, 16);
  const size_t o_txs = add(eb->tx_start, (n + 1) * 8, EV1, 8);
  const size_t o_txo = add(eb->tx_off, n_tx ? (n_tx + 1) * 8 : 0, TX1, 8);
  const size_t o_txb = add(eb->tx_bytes, tx_len, TXB, 1, 64);
  const size_t o_tln = add(eb->tx_list_nil, eb->tx_list_nil ? n : 0, EV, 1);
  const size_t o_txn = add(eb->tx_nil, eb->tx_nil ? n_tx : 0, TX, 1);
  const size_t o_io = add(eb->itx_off, eb->itx_off ? (n + 1) * 8 : 0, EV1, 8);
  const size_t o_ij = add(eb->itx_json, itx_len, ITX);
  const size_t o_bo = add(eb->bsig_off, eb->bsig_off ? (n + 1) * 8 : 0, EV1, 8);
  const size_t o_bj = add(eb->bsig_json, bsig_len, BSIG);
  auto seg_range = [&](const Seg &g, uint64_t e0, uint64_t e1, size_t *lo, size_t *hi) {
    const uint64_t t0 = eb->tx_start[e0], t1 = eb->tx_start[e1];
    switch (g.kind) {
      case ALL: *lo = 0; *hi = g.n; break;
      case EV: *lo = e0 * g.unit; *hi = e1 * g.unit; break;
      case EV1: *lo = e0 * g.unit; *hi = (e1 + 1) * g.unit; break;
      case TX: *lo = t0 * g.unit; *hi = t1 * g.unit; break;
      case TX1: *lo = t0 * g.unit; *hi = (t1 + 1) * g.unit; break;
      case TXB: *lo = n_tx ? eb->tx_off[t0] : 0; *hi = n_tx ? eb->tx_off[t1] : 0; break;
      case ITX: *lo = eb->itx_off ? eb->itx_off[e0] : 0; *hi = eb->itx_off ? eb->itx_off[e1] : 0; break;
      case BSIG: *lo = eb->bsig_off ? eb->bsig_off[e0] : 0; *hi = eb->bsig_off ? eb->bsig_off[e1] : 0; break;
    }
    *hi = std::min(*hi, g.n);
    *lo = std::min(*lo, *hi);
  };

  // event chunks of ~kChunk staged bytes (whole 256-event groups, so each
  // chunk's items fill whole words of the accept bitmask)
  // chunks: at most ~ev_chunk bytes; with ev_tail (BV_EV_TAIL=1), each
  // takes at most half of what is left (down to kEvTailMin events), so the
  // last chunk to land, whose hashing and verify are the call's tail, is
  // small.  Not the default: each chunk costs one DMA command per wire
  // field, and equal chunks measured 5.18-5.26 ms per 1M pinned events
  // against 5.37-5.39 (profiles/r05_ab_ev_qfirst.log)
  std::vector<uint64_t> cb{0};
  const uint64_t chunk_bytes = ctx->ev_chunk;  // 0 = one chunk (A/B knob, bv_create)
  if (chunk_bytes > 0) {
    const uint64_t per_ev = std::max<uint64_t>(1, (total - small_end) / n);
    const uint64_t per = std::max<uint64_t>(256, chunk_bytes / per_ev / 256 * 256);
    if (ctx->ev_tail == 2 && n > 2 * kEvTailMin) {  // equal chunks, then one of kEvTailMin events
      const uint64_t body = (n - kEvTailMin) / 256 * 256, k = (body + per - 1) / per;
      const uint64_t c = ((body + k - 1) / k + 255) / 256 * 256;
      for (uint64_t e = c; e < body; e += c) cb.push_back(e);
      cb.push_back(body);
    } else {
      for (uint64_t e = 0; e < n;) {
        uint64_t c = per;
        if (ctx->ev_tail == 1) c = std::min(per, ((n - e) / 2 + 255) / 256 * 256);
        if (n - e <= c || (ctx->ev_tail == 1 && n - e - c < kEvTailMin)) break;
        e += c;
        cb.push_back(e);
      }
    }
  }
  cb.push_back(n);

  if (bv_wait_all(ctx) != BV_OK) return BV_E_LAUNCH;  // previous calls' work buffers / staging
  HIPCHK(ctx->pin_in.ensure(total), BV_E_OOM, "alloc pinned staging");
  HIPCHK(ctx->d_in.ensure(total), BV_E_OOM, "alloc device staging");
  HIPCHK(ctx->ev_iota.ensure(n * 4), BV_E_OOM, "alloc item index");
  uint8_t *pin = (uint8_t *)ctx->pin_in.p, *dev = ctx->d_in.as<uint8_t>();

  // the same batch over device pointers
  bv_event_batch d = *eb;
  d.key_off = (const uint64_t *)(dev + o_koff);
  d.key_bytes = dev + o_kb;
  d.creator = (const uint32_t *)(dev + o_cr_ev);
  d.index = (const int64_t *)(dev + o_ix);
  d.timestamp = (const int64_t *)(dev + o_ts);
  d.parent_kind = dev + o_pk;
  d.parent_ref = (const uint64_t *)(dev + o_pr);
  d.parent_hashes = eb->parent_hashes ? dev + o_ph : nullptr;
  d.tx_start = (const uint64_t *)(dev + o_txs);
  d.tx_off = n_tx ? (const uint64_t *)(dev + o_txo) : nullptr;
  d.tx_bytes = dev + o_txb;
  d.tx_list_nil = eb->tx_list_nil ? dev + o_tln : nullptr;
  d.tx_nil = eb->tx_nil ? dev + o_txn : nullptr;
  d.itx_off = eb->itx_off ? (const uint64_t *)(dev + o_io) : nullptr;
  d.itx_json = dev + o_ij;
  d.bsig_off = eb->bsig_off ? (const uint64_t *)(dev + o_bo) : nullptr;
  d.bsig_json = dev + o_bj;
  d.r_be = dev + o_r_ev;
  d.s_be = dev + o_s;
  d.pre = eb->pre ? dev + o_pre : nullptr;

  // verification items: item e = (body e, creator key, r, s); the bodies
  // are never stored (k_ev_body_hash writes their digests only)
  bv_batch vb = {};
  vb.n_msgs = n;
  vb.n_keys = eb->n_keys;
  vb.key_bytes = d.key_bytes;
  vb.key_off = d.key_off;
  vb.n_items = n;
  vb.item_msg = ctx->ev_iota.as<uint32_t>();
  vb.item_key = d.creator;
  vb.r_be = d.r_be;
  vb.s_be = d.s_be;
  vb.pre = d.pre;
  bool kc = false;
  // bulk batches: each chunk's verify kernels go on the s^-1 stream (idle
  // once this batch's s^-1 is done; normal priority — the high-priority keys
  // stream stays for the latency-bound table chains), so they run
  // beside the next chunk's body build and hashing on the main stream
  // instead of after them (1M bulk events from pinned arrays, same box:
  // 7.37-7.41 -> 6.90-7.01 ms per call; BV_EV_VERIFY_STREAM=0 keeps them on
  // the main stream)
  const bool split_verify = ctx->ev_split_verify;
  hipStream_t vst = split_verify ? ctx->sstream : st;
  bv_item_pipe pipe{ctx, &vb, {}, vst, false};
  rc = bv_out_bufs(ctx, &vb, nullptr, nullptr, nullptr, true, &pipe.o);
  if (rc != BV_OK) return rc;
  uint32_t *dig = pipe.o.dig;

  // the first part: pinned copies by the pool, H2D on the copy stream
  hipStream_t cs = bv_copy_stream(ctx);
  if (!cs) return bv_fail(ctx, BV_E_NODEVICE, "copy stream");
  HIPCHK(hipEventRecord(ctx->S().ev[E_CALL], cs), BV_E_LAUNCH, "event");
  // arrays in bv_host_alloc memory are DMA'd from where they are (no
  // staging copy: what a cgo caller gets by building the wire batch there)
  std::vector<char> direct(segs.size());
  for (size_t i = 0; i < segs.size(); i++) direct[i] = segs[i].src && bv_is_pinned(segs[i].src, segs[i].n);
  auto stage = [&](size_t a0, size_t a1) -> int {
    for (size_t a = a0; a < a1; a += kChunk) {
      const size_t z = std::min(a1, a + kChunk);
      std::vector<CopyPool::Piece> pieces;
      bool any_direct = false;
      for (size_t i = 0; i < segs.size(); i++) {
        const Seg &g = segs[i];
        const size_t lo = std::max(a, g.off), hi = std::min(z, g.off + g.n);
        if (g.kind != ALL || !g.src || lo >= hi) continue;
        if (direct[i]) {
          any_direct = true;
          HIPCHK(hipMemcpyAsync(dev + lo, (const uint8_t *)g.src + (lo - g.off), hi - lo, hipMemcpyHostToDevice, cs),
                 BV_E_LAUNCH, "h2d (pinned caller buffer)");
        } else {
          pieces.push_back({pin + lo, (const uint8_t *)g.src + (lo - g.off), hi - lo});
        }
      }
      ctx->pool->copy_many(pieces);
      if (!any_direct) {
        HIPCHK(hipMemcpyAsync(dev + a, pin + a, z - a, hipMemcpyHostToDevice, cs), BV_E_LAUNCH, "h2d");
      } else {  // the staged pieces only: the range also holds direct segments
        for (const CopyPool::Piece &q : pieces) {
          const size_t o = (uint8_t *)q.dst - pin;
          HIPCHK(hipMemcpyAsync(dev + o, q.dst, q.n, hipMemcpyHostToDevice, cs), BV_E_LAUNCH, "h2d");
        }
      }
    }
    return BV_OK;
  };
  rc = stage(0, keys_end);  // the keys: the key tables start once they land
  if (rc != BV_OK) return rc;
  HIPCHK(hipEventRecord(ctx->S().ev[E_KREADY], cs), BV_E_LAUNCH, "event");
  if (ctx->flags & BV_F_KEY_CACHE) {
    HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_KREADY], 0), BV_E_LAUNCH, "join");
    bv_kc_items items;
    items.n_items = eb->n_events;
    items.h_item_key = eb->creator;
    rc = bv_kc_prepare(ctx, eb->n_keys, eb->key_bytes, eb->key_off, d.key_bytes, d.key_off, st, &kc, false, &items);
    if (rc != BV_OK) return rc;
  }
  rc = stage(keys_end, s_end);  // s, pre (or the signature text): s^-1
  if (rc != BV_OK) return rc;
  HIPCHK(hipEventRecord(ctx->S().ev[E_SREADY], cs), BV_E_LAUNCH, "event");
  if (text) {  // r, s, pre from the text, ahead of s^-1; the verify stream reads them
    SigOut so;
    rc = sig_decode_on_device(ctx, n, (const uint64_t *)(dev + o_s), dev + o_pre, ctx->S().ev[E_SREADY], &so);
    if (rc != BV_OK) return rc;
    vb.r_be = d.r_be = so.r, vb.s_be = d.s_be = so.s, vb.pre = d.pre = so.pre;
    HIPCHK(hipStreamWaitEvent(vst, ctx->S().ev[E_SDEC], 0), BV_E_LAUNCH, "join decoded signatures");
  }
  pipe.kc = kc;
  rc = bv_run_keys(ctx, &vb, ctx->S().ev[E_KREADY], ctx->S().ev[E_SREADY], kc);
  if (rc != BV_OK) return rc;
  if (qf) {
    rc = stage(s_end, r_end);  // r, the creators: the key part
    if (rc != BV_OK) return rc;
    HIPCHK(hipEventRecord(ctx->S().ev[E_RREADY], cs), BV_E_LAUNCH, "event");
    rc = pipe.key_part(vst, ctx->S().ev[E_RREADY]);
    if (rc != BV_OK) return rc;
  }
  rc = stage(r_end, small_end);  // the parent hashes
  if (rc != BV_OK) return rc;
  HIPCHK(hipEventRecord(ctx->S().ev[E_SMALL], cs), BV_E_LAUNCH, "event");
  HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_SMALL], 0), BV_E_LAUNCH, "join");
  HIPCHK(bvk::iota(st, n, ctx->ev_iota.as<uint32_t>()), BV_E_LAUNCH, "k_iota");
  HIPCHK(hipEventRecord(ctx->S().ev[E_FORK], st), BV_E_LAUNCH, "event");

  // results: digests chunk by chunk (below), statuses and bits at the end
  const size_t o_st = align256(n * 32), o_bits = o_st + align256(n);
  HIPCHK(ctx->pin_out.ensure(o_bits + align256((n + 63) / 64 * 8) + 256), BV_E_OOM, "alloc pinned results");
  uint8_t *pout = (uint8_t *)ctx->pin_out.p;
  call.pout = pout;
  call.o_st = o_st;
  call.o_bits = o_bits;
  call.direct_hash = res && bv_is_pinned(res->msg_hash, n * 32);  // results straight into pinned caller buffers
  call.direct_status = res && bv_is_pinned(res->status, n);
  uint8_t *hout = call.direct_hash ? res->msg_hash : pout;
  const int d2h = ctx->ev_d2h;

  // per chunk: its fields cross PCIe on the copy stream; on the main stream
  // the chunk's bodies are hashed (k_ev_body_hash) and its digests go back
  // (the D2H direction is idle while the next chunk crosses); its items are
  // verified on `vst`
  for (size_t c = 0; c + 1 < cb.size(); c++) {
    const uint64_t e0 = cb[c], e1 = cb[c + 1];
    std::vector<CopyPool::Piece> pieces;
    for (size_t i = 0; i < segs.size(); i++) {
      const Seg &g = segs[i];
      if (g.kind == ALL || !g.src) continue;
      size_t lo, hi;
      seg_range(g, e0, e1, &lo, &hi);
      if (lo >= hi) continue;
      if (direct[i])
        HIPCHK(hipMemcpyAsync(dev + g.off + lo, (const uint8_t *)g.src + lo, hi - lo, hipMemcpyHostToDevice, cs),
               BV_E_LAUNCH, "h2d (pinned caller buffer)");
      else
        pieces.push_back({pin + g.off + lo, (const uint8_t *)g.src + lo, hi - lo});
    }
    ctx->pool->copy_many(pieces);  // the rest of the chunk into pinned memory, then its DMA
    for (const CopyPool::Piece &q : pieces) {
      const size_t o = (uint8_t *)q.dst - pin;
      HIPCHK(hipMemcpyAsync(dev + o, pin + o, q.n, hipMemcpyHostToDevice, cs), BV_E_LAUNCH, "h2d");
    }
    hipEvent_t landed = ctx->chunk_ev[c % ctx->chunk_ev.size()];
    HIPCHK(hipEventRecord(landed, cs), BV_E_LAUNCH, "event");
    HIPCHK(hipStreamWaitEvent(st, landed, 0), BV_E_LAUNCH, "join chunk");
    HIPCHK(bvk::ev_body_hash(st, d, e0, e1, dig), BV_E_LAUNCH, "k_ev_body_hash");
    HIPCHK(hipEventRecord(ctx->S().ev[E_HASHED], st), BV_E_LAUNCH, "event");  // the last chunk's record is used
    hipEvent_t hashed = ctx->chunk_ev[(c + 32) % ctx->chunk_ev.size()];  // waited on before chunk c+2's record
    HIPCHK(hipEventRecord(hashed, st), BV_E_LAUNCH, "event");
    if (split_verify) HIPCHK(hipStreamWaitEvent(vst, hashed, 0), BV_E_LAUNCH, "join chunk digests");
    if (d2h == 2 && c > 0) {  // the previous chunk's digests, on the copy stream behind this chunk's H2D
      const uint64_t p0 = cb[c - 1];
      HIPCHK(hipStreamWaitEvent(cs, ctx->chunk_ev[(c + 31) % ctx->chunk_ev.size()], 0), BV_E_LAUNCH, "join");
      HIPCHK(hipMemcpyAsync(hout + p0 * 32, dig + p0 * 8, (e0 - p0) * 32, hipMemcpyDeviceToHost, cs), BV_E_LAUNCH,
             "d2h digests");
    }
    rc = pipe.upto(e1);
    if (rc != BV_OK) return rc;
    if (d2h == 1)
      HIPCHK(hipMemcpyAsync(hout + e0 * 32, dig + e0 * 8, (e1 - e0) * 32, hipMemcpyDeviceToHost, st), BV_E_LAUNCH,
             "d2h digests");
  }
  if (d2h == 0) {  // one copy once the last chunk is hashed, on the copy stream
    HIPCHK(hipStreamWaitEvent(cs, ctx->S().ev[E_HASHED], 0), BV_E_LAUNCH, "join");
    HIPCHK(hipMemcpyAsync(hout, dig, n * 32, hipMemcpyDeviceToHost, cs), BV_E_LAUNCH, "d2h digests");
  } else if (d2h == 2) {  // the last chunk's digests
    const uint64_t p0 = cb[cb.size() - 2];
    HIPCHK(hipStreamWaitEvent(cs, ctx->S().ev[E_HASHED], 0), BV_E_LAUNCH, "join");
    HIPCHK(hipMemcpyAsync(hout + p0 * 32, dig + p0 * 8, (n - p0) * 32, hipMemcpyDeviceToHost, cs), BV_E_LAUNCH,
           "d2h digests");
  }
  HIPCHK(hipEventRecord(ctx->S().ev[E_STAGED], cs), BV_E_LAUNCH, "event");
  call.ms_prep = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - call.t0).count();

  HIPCHK(hipEventRecord(ctx->S().ev[E_SHA], st), BV_E_LAUNCH, "event");
  if (d2h != 2) HIPCHK(hipEventRecord(ctx->S().ev[E_CSDONE], d2h == 0 ? cs : st), BV_E_LAUNCH, "event");

  rc = pipe.finish();  // the last chunk's items
  if (rc != BV_OK) return rc;
  // statuses and bits: on the copy stream (SDMA) with the digests in mode 2,
  // else on the main stream
  hipStream_t os = d2h == 2 ? cs : st;
  if (split_verify || d2h == 2) HIPCHK(hipStreamWaitEvent(os, ctx->S().ev[E_END], 0), BV_E_LAUNCH, "join verify");
  HIPCHK(hipMemcpyAsync(call.direct_status ? res->status : pout + o_st, pipe.o.status, n, hipMemcpyDeviceToHost, os),
         BV_E_LAUNCH, "d2h status");
  HIPCHK(hipMemcpyAsync(pout + o_bits, pipe.o.bits, (n + 63) / 64 * 8, hipMemcpyDeviceToHost, os), BV_E_LAUNCH,
         "d2h bits");
  HIPCHK(hipEventRecord(ctx->S().ev[E_OUT], os), BV_E_LAUNCH, "event");
  if (d2h == 2) HIPCHK(hipEventRecord(ctx->S().ev[E_CSDONE], cs), BV_E_LAUNCH, "event");
  HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_CSDONE], 0), BV_E_LAUNCH, "join");  // digests out before ev_done
  HIPCHK(hipStreamWaitEvent(st, ctx->S().ev[E_STAGED], 0), BV_E_LAUNCH, "join");  // staging free after ev_done
  rc = bv_mark_done(ctx, st);
  if (rc != BV_OK) return rc;
  bv_batch sizes = {};
  sizes.n_msgs = n;
  sizes.n_items = n;
  return bv_host_finish(ctx, &sizes, res, &call, true);
}
