// bv_group.cpp — multi-GPU verifier behind the C ABI (include/babbleverify.h,
// bv_group_*): one process, one bv_ctx per device, items sharded by index,
// one RCCL all-gather of the accept bitmasks.
//
// The north star's multi-GPU step: VerifyBatch items are
// independent, so device g verifies a contiguous item range and no data
// crosses devices except the accept bits.  Shards never split the items of
// one message (bv_plan_shards): a BlockBody's 100 validator signatures
// (block.go:343, hashgraph.go:1599-1630) stay on one device, so the body is
// hashed once and a CheckBlock count is local.  Each device's bitmask
// (its shard's bits from bit 0, padded to the largest shard) is all-gathered
// with ONE ncclAllGather into device 0 and copied to the host once; the
// host merges the shard-local words into the global bitmask (bit shifts).
// RCCL is loaded with dlopen at bv_group_create (the PyTorch process may
// already hold it), so libbabbleverify.so has no link-time RCCL dependency
// and single-device users never load it.
//
// Logical shards: a device list that names ONE device several times makes
// that many shards (one ctx each) on it; the shard bitmasks are then copied
// into the gather buffer on the device instead of an RCCL all-gather (RCCL
// needs distinct devices per rank).  Everything else — the shard plan, the
// concurrent per-shard staging threads, the shifted merge — is the
// multi-device code path, so it runs on hardware with one GPU
// (tests/test_gpu_cache_group.py::test_group_logical_shards).
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <thread>
#include <tuple>

#include "bv_internal.h"
#include "hostplan.h"

namespace {

// the RCCL entry points used (rccl.h; ncclUint64 = 5, ncclSuccess = 0)
typedef void *nccl_comm;
typedef int (*fn_init_all)(nccl_comm *, int, const int *);
typedef int (*fn_destroy)(nccl_comm);
typedef int (*fn_all_gather)(const void *, void *, size_t, int, nccl_comm, hipStream_t);
typedef int (*fn_group)(void);
typedef const char *(*fn_errstr)(int);
constexpr int kNcclUint64 = 5;

struct Rccl {
  void *h = nullptr;
  fn_init_all init_all = nullptr;
  fn_destroy destroy = nullptr;
  fn_all_gather all_gather = nullptr;
  fn_group group_start = nullptr, group_end = nullptr;
  fn_errstr errstr = nullptr;
  bool load(std::string &err) {
    if (h) return true;
    const char *names[] = {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
    for (const char *n : names) {  // prefer a copy already in the process (PyTorch's)
      h = dlopen(n, RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
      if (h) break;
    }
    for (const char *n : names) {
      if (h) break;
      h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
    }
    if (!h) {
      err = "RCCL (librccl.so) not found";
      return false;
    }
    init_all = (fn_init_all)dlsym(h, "ncclCommInitAll");
    destroy = (fn_destroy)dlsym(h, "ncclCommDestroy");
    all_gather = (fn_all_gather)dlsym(h, "ncclAllGather");
    group_start = (fn_group)dlsym(h, "ncclGroupStart");
    group_end = (fn_group)dlsym(h, "ncclGroupEnd");
    errstr = (fn_errstr)dlsym(h, "ncclGetErrorString");
    if (!init_all || !destroy || !all_gather || !group_start || !group_end || !errstr) {
      err = "RCCL symbols missing";
      return false;
    }
    return true;
  }
};
Rccl g_rccl;
std::mutex g_rccl_mu;

}  // namespace

struct bv_group {
  std::vector<int> devices;
  std::vector<bv_ctx *> ctx;
  std::vector<nccl_comm> comms;
  bool logical = false;  // every entry of `devices` is the same device: no RCCL
  std::vector<DevBuf> send, recv;  // per device: shard bits, gathered bits
  std::vector<hipEvent_t> sent;    // per device: its send buffer is written (recorded on its ctx's stream)
  // per device: its shard's re-based message offsets and item -> message
  // indices, in bv_host_alloc memory so the shard's staging DMAs them in
  // place (grown on demand, reused across calls)
  std::vector<void *> sub_off, sub_msg;
  std::vector<size_t> sub_off_cap, sub_msg_cap;
  std::string err;
  std::mutex mu;
};

static int gfail(bv_group *g, int code, const std::string &what) {
  if (g) g->err = what;
  return code;
}

extern "C" const char *bv_group_last_error(const bv_group *g) { return g ? g->err.c_str() : "null group"; }

extern "C" void bv_group_destroy(bv_group *g) {
  if (!g) return;
  for (size_t i = 0; i < g->ctx.size(); i++) {
    if (i < g->comms.size() && g->comms[i]) {
      (void)hipSetDevice(g->devices[i]);
      g_rccl.destroy(g->comms[i]);
    }
    (void)hipSetDevice(g->devices[i]);
    if (i < g->sent.size() && g->sent[i]) (void)hipEventDestroy(g->sent[i]);
    if (i < g->send.size()) g->send[i].release();
    if (i < g->recv.size()) g->recv[i].release();
    bv_destroy(g->ctx[i]);
  }
  for (void *p : g->sub_off) bv_host_free(p);
  for (void *p : g->sub_msg) bv_host_free(p);
  delete g;
}

extern "C" int bv_group_create(bv_group **out, const int *devices, int n_devices, uint32_t flags) {
  if (!out || !devices || n_devices <= 0 || n_devices > 64) return BV_E_ARGS;
  *out = nullptr;
  bool same = true;
  for (int i = 1; i < n_devices; i++) same = same && devices[i] == devices[0];
  for (int i = 0; i < n_devices && !same; i++)
    for (int j = 0; j < i; j++)
      if (devices[i] == devices[j]) return BV_E_ARGS;  // repeats only as logical shards of one device
  bv_group *g = new bv_group();
  g->devices.assign(devices, devices + n_devices);
  g->logical = same && n_devices > 1;
  for (int i = 0; i < n_devices; i++) {
    bv_ctx *c = nullptr;
    int rc = bv_create(&c, devices[i], flags);
    if (rc != BV_OK) {
      bv_group_destroy(g);
      return rc;
    }
    if (g->logical) c->kc_budget /= (uint64_t)n_devices;  // the shards share the device's HBM
    g->ctx.push_back(c);
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      bv_group_destroy(g);
      return BV_E_NODEVICE;
    }
    g->sent.push_back(e);
  }
  g->send.resize(n_devices);
  g->recv.resize(n_devices);
  g->sub_off.assign(n_devices, nullptr);
  g->sub_msg.assign(n_devices, nullptr);
  g->sub_off_cap.assign(n_devices, 0);
  g->sub_msg_cap.assign(n_devices, 0);
  if (g->logical) {
    *out = g;
    return BV_OK;
  }
  {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    std::string e;
    if (!g_rccl.load(e)) {
      bv_group_destroy(g);
      return BV_E_COMM;
    }
  }
  g->comms.assign(n_devices, nullptr);
  const int r = g_rccl.init_all(g->comms.data(), n_devices, devices);
  if (r != 0) {
    g->comms.assign(n_devices, nullptr);
    bv_group_destroy(g);
    return BV_E_COMM;
  }
  *out = g;
  return BV_OK;
}

extern "C" int bv_group_get_timing(const bv_group *g, int i, bv_timing *out) {
  if (!g || i < 0 || i >= (int)g->ctx.size()) return BV_E_ARGS;
  return bv_get_timing(g->ctx[i], out);
}

static int group_verify(bv_group *g, const bv_batch *b, bv_result *res, GroupPlan &p);

extern "C" int bv_group_verify_batch(bv_group *g, const bv_batch *b, bv_result *res) {
  if (!g || !b || !res) return BV_E_ARGS;
  std::lock_guard<std::mutex> lk(g->mu);
  GroupPlan p;
  const int rc = group_verify(g, b, res, p);
  if (rc != BV_OK)
    for (bv_ctx *c : g->ctx) {  // nothing of the failed call stays in flight
      std::lock_guard<std::mutex> clk(c->mu);
      (void)hipSetDevice(c->device);
      (void)bv_drain(c, c->stream, rc);
    }
  return rc;
}

static int group_verify(bv_group *g, const bv_batch *b, bv_result *res, GroupPlan &p) {
  const int D = (int)g->ctx.size();
  if (b->n_items > UINT32_MAX || b->n_msgs > UINT32_MAX)  // the group plan indexes items and messages with u32
    return gfail(g, BV_E_ARGS, "more than 2^32 items or messages in one group call");
  bv_ctx *c0 = g->ctx[0];
  int rc = bv_validate_host_batch(c0, b);
  if (rc != BV_OK) return gfail(g, rc, c0->err);
  // (the O(n) order check on the copy pool: 8M items ~1 ms instead of ~8)
  const bool in_order = c0->pool->parallel_for(b->n_items > 0 ? b->n_items - 1 : 0, 1 << 17,
                                                [b](uint64_t lo, uint64_t hi) {
                                                  for (uint64_t i = lo; i < hi; i++)
                                                    if (b->item_msg[i] > b->item_msg[i + 1]) return false;
                                                  return true;
                                                });
  bv_batch sorted;
  plan_group(b, D, p, sorted, in_order ? 1 : 0);
  const std::vector<uint64_t> &bounds = p.bounds;
  // per-device pinned buffers for the shards' re-based arrays (allocated
  // here, on the calling thread: bv_host_alloc is process-wide)
  for (int d = 0; d < D; d++) {
    const size_t noff = (p.mhi[d] - p.mlo[d] + 1) * 8, nim = std::max<uint64_t>(bounds[d + 1] - bounds[d], 1) * 4;
    for (auto [buf, cap, need] : {std::make_tuple(&g->sub_off[d], &g->sub_off_cap[d], noff),
                                  std::make_tuple(&g->sub_msg[d], &g->sub_msg_cap[d], nim)})
      if (*cap < need) {
        bv_host_free(*buf);
        *buf = nullptr;
        *cap = 0;
        if (bv_host_alloc(need + need / 4, buf) != BV_OK) return gfail(g, BV_E_OOM, "pinned shard arrays");
        *cap = need + need / 4;
      }
  }
  uint64_t words = 1;
  for (int d = 0; d < D; d++) words = std::max<uint64_t>(words, (bounds[d + 1] - bounds[d] + 63) / 64);

  if (p.permuted && res->status) p.s_status.resize(b->n_items);
  uint8_t *st_out = p.permuted ? (res->status ? p.s_status.data() : nullptr) : res->status;
  // build, stage and launch every shard concurrently (one host thread per
  // device): the shard's items and its message range with re-based offsets
  // and indices; keys are replicated (small)
  std::vector<bv_batch> sb(D);
  std::vector<bv_host_call> calls(D);
  std::vector<int> rcs(D, BV_OK);
  std::vector<std::thread> th;
  for (int d = 0; d < D; d++)
    th.emplace_back([&, d]() {
      {
        const uint64_t a = bounds[d], z = bounds[d + 1], lo = p.mlo[d], hi = p.mhi[d];
        uint64_t *off = (uint64_t *)g->sub_off[d];
        const uint64_t base = b->msg_off ? b->msg_off[lo] : 0;  // (null only with no messages)
        for (uint64_t m = lo; m <= hi; m++) off[m - lo] = b->msg_off ? b->msg_off[m] - base : 0;
        uint32_t *im = (uint32_t *)g->sub_msg[d];
        for (uint64_t i = a; i < z; i++) im[i - a] = (uint32_t)(sorted.item_msg[i] - lo);
        bv_batch &s = sb[d];
        s = sorted;
        s.n_msgs = hi - lo;
        s.msg_bytes = b->msg_bytes ? b->msg_bytes + (hi > lo ? base : 0) : nullptr;
        s.msg_off = off;
        s.n_items = z - a;
        s.item_msg = im;
        s.item_key = sorted.item_key ? sorted.item_key + a : nullptr;
        s.r_be = sorted.r_be ? sorted.r_be + 32 * a : nullptr;
        s.s_be = sorted.s_be ? sorted.s_be + 32 * a : nullptr;
        s.pre = sorted.pre ? sorted.pre + a : nullptr;
      }
      bv_ctx *c = g->ctx[d];
      std::lock_guard<std::mutex> clk(c->mu);
      if (hipSetDevice(c->device) != hipSuccess) {
        rcs[d] = BV_E_NODEVICE;
        return;
      }
      bv_result sr = {};
      sr.msg_hash = res->msg_hash ? res->msg_hash + 32 * p.mlo[d] : nullptr;
      sr.status = st_out ? st_out + bounds[d] : nullptr;
      rcs[d] = bv_host_launch(c, &sb[d], &calls[d], &sr);
      if (rcs[d] != BV_OK) return;
      // the shard's bits, zero-padded to `words`, as the all-gather send buffer
      if (g->send[d].ensure(words * 8) != hipSuccess || g->recv[d].ensure(words * 8 * D) != hipSuccess) {
        rcs[d] = BV_E_OOM;
        return;
      }
      const uint64_t sw = (sb[d].n_items + 63) / 64;
      if (hipMemsetAsync(g->send[d].p, 0, words * 8, c->stream) != hipSuccess ||
          (sw && hipMemcpyAsync(g->send[d].p, c->S().bits.p, sw * 8, hipMemcpyDeviceToDevice, c->stream) != hipSuccess) ||
          hipEventRecord(g->sent[d], c->stream) != hipSuccess)
        rcs[d] = BV_E_LAUNCH;
    });
  for (auto &t : th) t.join();
  for (int d = 0; d < D; d++)
    if (rcs[d] != BV_OK) return gfail(g, rcs[d], "device " + std::to_string(g->devices[d]) + ": " + g->ctx[d]->err);

  if (g->logical) {
    // logical shards of one device: the gather is D copies into shard 0's
    // buffer on shard 0's stream, each ordered after that shard's send
    // buffer by its event (whatever stream the shard ran on)
    (void)hipSetDevice(g->devices[0]);
    for (int d = 0; d < D; d++)
      if (hipStreamWaitEvent(g->ctx[0]->stream, g->sent[d], 0) != hipSuccess ||
          hipMemcpyAsync((uint8_t *)g->recv[0].p + (size_t)d * words * 8, g->send[d].p, words * 8,
                         hipMemcpyDeviceToDevice, g->ctx[0]->stream) != hipSuccess)
        return gfail(g, BV_E_LAUNCH, "gather shard bits");
  } else {
    // ONE all-gather of the accept bitmasks over RCCL (xGMI)
    int r = g_rccl.group_start();
    for (int d = 0; d < D && r == 0; d++) {
      (void)hipSetDevice(g->devices[d]);
      r = g_rccl.all_gather(g->send[d].p, g->recv[d].p, words, kNcclUint64, g->comms[d], g->ctx[d]->stream);
    }
    const int r2 = g_rccl.group_end();
    if (r != 0 || r2 != 0) return gfail(g, BV_E_COMM, std::string("ncclAllGather: ") + g_rccl.errstr(r ? r : r2));
  }
  std::vector<uint64_t> gathered(words * D);
  (void)hipSetDevice(g->devices[0]);
  if (hipMemcpyAsync(gathered.data(), g->recv[0].p, words * 8 * D, hipMemcpyDeviceToHost, g->ctx[0]->stream) !=
      hipSuccess)
    return gfail(g, BV_E_LAUNCH, "d2h gathered bits");

  // per-device results (digests of its message range, statuses of its shard)
  for (int d = 0; d < D; d++) {
    bv_ctx *c = g->ctx[d];
    std::lock_guard<std::mutex> clk(c->mu);
    (void)hipSetDevice(c->device);
    if (bv_mark_done(c, c->stream) != BV_OK) return gfail(g, BV_E_LAUNCH, "event");
    bv_result sr = {};
    sr.msg_hash = res->msg_hash ? res->msg_hash + 32 * p.mlo[d] : nullptr;
    sr.status = st_out ? st_out + bounds[d] : nullptr;
    rc = bv_host_finish(c, &sb[d], &sr, &calls[d], false);
    if (rc != BV_OK) return gfail(g, rc, c->err);
  }
  if (!res->accept_bits && !p.permuted) return BV_OK;
  // merge the shard-local words into the bitmask (message order), then back
  // to the caller's item order when the items were permuted
  const uint64_t n = b->n_items, W = (n + 63) / 64;
  uint64_t *merged = res->accept_bits;
  if (p.permuted) {
    p.s_bits.assign(std::max<uint64_t>(W, 1), 0);
    merged = p.s_bits.data();
  }
  if (merged && bv_merge_shard_bits(gathered.data(), words, D, bounds.data(), merged) != BV_OK)
    return gfail(g, BV_E_ARGS, "merge shard bits");
  if (p.permuted) {
    if (res->status)
      for (uint64_t j = 0; j < n; j++) res->status[p.perm[j]] = p.s_status[j];
    if (res->accept_bits) {
      memset(res->accept_bits, 0, W * 8);
      for (uint64_t j = 0; j < n; j++)
        if (merged[j >> 6] >> (j & 63) & 1) res->accept_bits[p.perm[j] >> 6] |= 1ull << (p.perm[j] & 63);
    }
  }
  return BV_OK;
}
