// hostplan.h — host-only planning of a multi-device group call (no HIP):
// item order, message-aligned item shards and the message partition
// (hostplan.cpp; used by bv_group.cpp, sanitized by tests/hostfuzz).
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/babbleverify.h"

struct GroupPlan {
  std::vector<uint64_t> bounds, mlo, mhi;
  bool permuted = false;
  std::vector<uint32_t> perm;  // sorted position j -> caller's item index
  std::vector<uint32_t> s_msg, s_key;
  std::vector<uint8_t> s_r, s_s, s_pre, s_status;
  std::vector<uint64_t> s_bits;
};

// Fills `p` for `b` over D shards; `sorted` = b with its item arrays in the
// plan's order (p's own copies when permuted).  b's item_msg must be < n_msgs.
// `in_order`: whether item_msg is non-decreasing, when the caller already
// knows (-1: checked here).
void plan_group(const bv_batch *b, int D, GroupPlan &p, bv_batch &sorted, int in_order = -1);
