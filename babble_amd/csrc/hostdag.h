// hostdag.h — the in-batch DAG of bv_verify_events on the host: every
// canonical EventBody built from its wire fields (evjson.h, the same code the
// device runs for bulk batches) and hashed in topological order, each child
// getting its in-batch parents' "0X"+hex spliced in once their digests exist
// (Hashgraph.ReadWireInfo resolving parents inside one SyncResponse,
// src/hashgraph/hashgraph.go:1540-1595, src/node/core.go:214-245).  The
// device verifies the signatures meanwhile (bv_events.cpp).  Host-only code.
#pragma once
#include <stdint.h>

#include <functional>
#include <vector>

#include "../../include/babbleverify.h"

// fn(lo, hi) over [0, n) in `grain`-sized ranges, possibly on several threads
using HostParFor = std::function<void(uint64_t n, uint64_t grain, const std::function<void(uint64_t, uint64_t)> &fn)>;

struct HostDagScratch {
  std::vector<uint64_t> off;   // n + 1 body offsets
  std::vector<uint32_t> ppos;  // 2 per event: byte offset of an in-batch parent's hex, or EVJ_NOPOS
  std::vector<uint32_t> mid;   // 8 per event: SHA-256 state after the parent-independent blocks
  std::vector<uint8_t> bodies;
};

// Levels (level_off, n_levels + 1 entries) and `order` (events sorted by
// level) as bv_events.cpp computes them; writes the n 32-byte digests.
void bv_host_dag_hash(const bv_event_batch &b, const uint32_t *order, const uint32_t *level_off, uint32_t n_levels,
                      const HostParFor &pf, HostDagScratch &w, uint8_t *digests);
