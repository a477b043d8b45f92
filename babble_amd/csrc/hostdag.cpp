// hostdag.cpp — bv_host_dag_hash (hostdag.h).
//
// Work per event (T=1 body, 8 SHA-256 blocks): the body written from its
// wire fields, then — all events in parallel — either its whole digest (level
// 0: no in-batch parent) or the midstate of the blocks wholly before its
// first in-batch parent's hex (2 of 8 blocks); then, level by level, the
// parents' hex spliced in and the remaining blocks (6 of 8) hashed from the
// midstate.  Only that last step is serial along the DAG: ~6 blocks per
// event at ~40 ns a block with the SHA extensions (a 1000-event SyncResponse
// of 333 levels: ~0.25 ms on one core, against ~14 us per level for one GPU
// wave, profiles/r03_chain_ab.log).  Wide levels are spread over the pool.
#include "hostdag.h"

#include <string.h>

#include "evjson.h"
#include "hostsha.h"

void bv_host_dag_hash(const bv_event_batch &b, const uint32_t *order, const uint32_t *level_off, uint32_t n_levels,
                      const HostParFor &pf, HostDagScratch &w, uint8_t *digests) {
  const uint64_t n = b.n_events;
  if (n == 0) return;
  w.off.assign(n + 1, 0);
  w.ppos.assign(2 * n, EVJ_NOPOS);
  w.mid.assign(8 * n, 0);
  uint64_t *off = w.off.data();
  uint32_t *ppos = w.ppos.data();
  pf(n, 512, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t e = lo; e < hi; e++) off[e + 1] = evj_len(b, e, ppos + 2 * e);
  });
  for (uint64_t e = 0; e < n; e++) off[e + 1] += off[e];
  w.bodies.resize(off[n] + 64);
  uint8_t *bodies = w.bodies.data();
  pf(n, 256, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t e = lo; e < hi; e++) evj_write(b, e, bodies + off[e]);
  });
  // level 0: whole digests; above: midstates of the parent-independent blocks
  const uint64_t n0 = level_off[1];
  uint32_t *mid = w.mid.data();
  pf(n, 64, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; i++) {
      const uint32_t e = order[i];
      const uint8_t *body = bodies + off[e];
      if (i < n0) {
        hsha::digest(body, off[e + 1] - off[e], digests + 32ull * e);
      } else {
        hsha::init(mid + 8ull * e);
        hsha::compress(mid + 8ull * e, body, ev_mid_blocks(ppos + 2 * e));
      }
    }
  });
  // the chain: level L's events need only levels < L; a level's events are
  // finished in pairs whose compressions interleave (hsha::finish2)
  auto splice = [&](uint32_t e) {
    uint8_t *body = bodies + off[e];
    for (int p = 0; p < 2; p++)
      if (ppos[2 * e + p] != EVJ_NOPOS) evj_hex32(body + ppos[2 * e + p], digests + 32ull * b.parent_ref[2 * e + p]);
  };
  auto finish = [&](uint64_t lo, uint64_t hi) {
    uint64_t i = lo;
    for (; i + 1 < hi; i += 2) {
      const uint32_t e = order[i], f = order[i + 1];
      splice(e);
      splice(f);
      uint32_t he[8], hf[8];
      memcpy(he, mid + 8ull * e, sizeof he);
      memcpy(hf, mid + 8ull * f, sizeof hf);
      hsha::finish2(he, bodies + off[e], 64ull * ev_mid_blocks(ppos + 2 * e), off[e + 1] - off[e],
                    digests + 32ull * e, hf, bodies + off[f], 64ull * ev_mid_blocks(ppos + 2 * f),
                    off[f + 1] - off[f], digests + 32ull * f);
    }
    if (i < hi) {
      const uint32_t e = order[i];
      splice(e);
      uint32_t h[8];
      memcpy(h, mid + 8ull * e, sizeof h);
      hsha::finish(h, bodies + off[e], 64ull * ev_mid_blocks(ppos + 2 * e), off[e + 1] - off[e], digests + 32ull * e);
    }
  };
  for (uint32_t L = 1; L < n_levels; L++) {
    const uint64_t a = level_off[L], z = level_off[L + 1];
    if (z - a >= 128)
      pf(z - a, 32, [&](uint64_t lo, uint64_t hi) { finish(a + lo, a + hi); });
    else
      finish(a, z);
  }
}
