// hostplan.cpp — host helpers of the multi-device group (no device, no HIP):
//
//   bv_plan_shards       contiguous item ranges balanced by count, cut only
//                        where the message changes (a BlockBody's validator
//                        signatures, block.go:343 / hashgraph.go:1599-1630,
//                        stay on one device);
//   bv_plan_group        the whole plan of bv_group_verify_batch: item order,
//                        item shards, message partition;
//   bv_merge_shard_bits  the accept bitmask from the all-gathered shard words.
//
// Pure C++ so the same source links into the ASan/UBSan fuzz harness
// (tests/hostfuzz) and into libbabbleverify.so.
#include "hostplan.h"

#include <algorithm>
#include <cstring>

// Contiguous item ranges balanced by count, cut only where the next item
// names a different message than the previous one (message-aligned), so the
// items of one message are never split.  Empty shards are allowed.
extern "C" int bv_plan_shards(const bv_batch *b, int n_shards, uint64_t *bounds) {
  if (!b || n_shards <= 0 || !bounds) return BV_E_ARGS;
  const uint64_t n = b->n_items;
  if (n && !b->item_msg) return BV_E_ARGS;
  bounds[0] = 0;
  for (int g = 1; g < n_shards; g++) {
    uint64_t c = std::max<uint64_t>(bounds[g - 1], (uint64_t)((__uint128_t)n * g / n_shards));
    while (c > 0 && c < n && b->item_msg[c] == b->item_msg[c - 1]) c++;
    bounds[g] = std::min(c, n);
  }
  bounds[n_shards] = n;
  return BV_OK;
}

// The global accept bitmask from the all-gathered shard bitmasks: shard d's
// words start at gathered[d * words_per_shard], its bit 0 is item bounds[d].
// Bits past a shard's item count are ignored (the device pads with zeros, but
// the merge does not rely on it).  Host only.
extern "C" int bv_merge_shard_bits(const uint64_t *gathered, uint64_t words_per_shard, int n_shards,
                                   const uint64_t *bounds, uint64_t *out) {
  if (!bounds || n_shards <= 0 || bounds[0] != 0) return BV_E_ARGS;
  const uint64_t n_items = bounds[n_shards];
  for (int d = 0; d < n_shards; d++)
    if (bounds[d] > bounds[d + 1] || (bounds[d + 1] - bounds[d] + 63) / 64 > words_per_shard) return BV_E_ARGS;
  if (n_items == 0) return BV_OK;
  if (!gathered || !out) return BV_E_ARGS;
  const uint64_t W = (n_items + 63) / 64;
  memset(out, 0, W * 8);
  for (int d = 0; d < n_shards; d++) {
    const uint64_t a = bounds[d], n = bounds[d + 1] - a;
    const uint64_t *src = gathered + (uint64_t)d * words_per_shard;
    const uint64_t q0 = a / 64, s = a % 64;
    for (uint64_t w = 0; w < (n + 63) / 64; w++) {
      uint64_t v = src[w];
      const uint64_t valid = std::min<uint64_t>(64, n - 64 * w);
      if (valid < 64) v &= (1ull << valid) - 1;
      out[q0 + w] |= v << s;
      if (s && q0 + w + 1 < W) out[q0 + w + 1] |= v >> (64 - s);
    }
  }
  return BV_OK;
}

static bool items_in_message_order(const bv_batch *b) {
  for (uint64_t i = 1; i < b->n_items; i++)
    if (b->item_msg[i] < b->item_msg[i - 1]) return false;
  return true;
}

// One group call's host-side plan: items in message order (a stable counting
// sort when the caller's item_msg is not non-decreasing), message-aligned item
// shards, and a PARTITION of the messages [0, n_msgs) into contiguous device
// ranges — every message is hashed exactly once, including messages no item
// references (bv_verify_batch writes every digest too).
void plan_group(const bv_batch *b, int D, GroupPlan &p, bv_batch &sorted, int in_order) {
  sorted = *b;
  p.permuted = in_order < 0 ? !items_in_message_order(b) : in_order == 0;
  if (p.permuted) {
    const uint64_t n = b->n_items, M = b->n_msgs;
    std::vector<uint64_t> cnt(M + 1, 0);
    for (uint64_t i = 0; i < n; i++) cnt[b->item_msg[i] + 1]++;
    for (uint64_t m = 0; m < M; m++) cnt[m + 1] += cnt[m];
    p.perm.resize(n);
    for (uint64_t i = 0; i < n; i++) p.perm[cnt[b->item_msg[i]]++] = (uint32_t)i;
    p.s_msg.resize(n);
    p.s_key.resize(n);
    p.s_r.resize(32 * n);
    p.s_s.resize(32 * n);
    if (b->pre) p.s_pre.resize(n);
    for (uint64_t j = 0; j < n; j++) {
      const uint64_t i = p.perm[j];
      p.s_msg[j] = b->item_msg[i];
      p.s_key[j] = b->item_key[i];
      memcpy(&p.s_r[32 * j], b->r_be + 32 * i, 32);
      memcpy(&p.s_s[32 * j], b->s_be + 32 * i, 32);
      if (b->pre) p.s_pre[j] = b->pre[i];
    }
    sorted.item_msg = p.s_msg.data();
    sorted.item_key = p.s_key.data();
    sorted.r_be = p.s_r.data();
    sorted.s_be = p.s_s.data();
    sorted.pre = b->pre ? p.s_pre.data() : nullptr;
  }
  p.bounds.assign(D + 1, 0);
  bv_plan_shards(&sorted, D, p.bounds.data());
  // message cut d = the first message of item shard d (shards never split a
  // message, so shard d's items name messages in [cut d, cut d+1)); messages
  // before the first referenced one go to device 0, after the last to the
  // last device, between shards to the earlier shard
  p.mlo.assign(D, 0);
  p.mhi.assign(D, 0);
  uint64_t prev = 0;
  for (int d = 0; d < D; d++) {
    const uint64_t cut = d == 0 ? 0 : p.bounds[d] < b->n_items ? sorted.item_msg[p.bounds[d]] : b->n_msgs;
    p.mlo[d] = std::max(prev, cut);
    prev = p.mlo[d];
  }
  for (int d = 0; d < D; d++) p.mhi[d] = d + 1 < D ? p.mlo[d + 1] : b->n_msgs;
}

extern "C" int bv_plan_group(const bv_batch *b, int n_shards, uint64_t *item_bounds, uint64_t *msg_bounds,
                             uint32_t *perm) {
  if (!b || n_shards <= 0 || !item_bounds || !msg_bounds) return BV_E_ARGS;
  // the plan's permutation and sorted indices are u32 (item_msg is u32 too)
  if (b->n_items > UINT32_MAX || b->n_msgs > UINT32_MAX) return BV_E_ARGS;
  if (b->n_items && (!b->item_msg || !b->item_key || !b->r_be || !b->s_be)) return BV_E_ARGS;
  for (uint64_t i = 0; i < b->n_items; i++)
    if (b->item_msg[i] >= b->n_msgs) return BV_E_ARGS;
  GroupPlan p;
  bv_batch sorted;
  plan_group(b, n_shards, p, sorted);
  for (int d = 0; d <= n_shards; d++) item_bounds[d] = p.bounds[d];
  for (int d = 0; d < n_shards; d++) msg_bounds[d] = p.mlo[d];
  msg_bounds[n_shards] = b->n_msgs;
  if (perm)
    for (uint64_t j = 0; j < b->n_items; j++) perm[j] = p.permuted ? p.perm[j] : (uint32_t)j;
  return p.permuted ? 1 : 0;
}

