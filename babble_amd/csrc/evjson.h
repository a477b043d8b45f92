// evjson.h — canonical EventBody JSON built on the device from WireEvent
// fields, as __host__ __device__ functions so the host
// emulator (tests/emu) runs the same code against Go-semantics fixtures.
//
// EventBody.Marshal (src/hashgraph/event.go:38-45) is Go 1.13 encoding/json
// of the exported fields in declaration order, then '\n' (json.Encoder):
//   {"Transactions":T,"InternalTransactions":I,"Parents":["p0","p1"],
//    "Creator":"<b64>","Index":<dec>,"BlockSignatures":B,"Timestamp":<dec>}\n
//   T  nil -> null, else [x,...] with x = null (nil []byte) or "<b64>"
//      (padded StdEncoding; empty -> "")
//   I, B  verbatim JSON from the host (encoding/json of the slices; rare in
//      gossip); an empty fragment means nil -> null
//   p  "" (no parent, ReadWireInfo index < 0, hashgraph.go:1541-1573) or
//      "0X" + 64 UPPERCASE hex (Event.Hex, common/hex.go:10-12) of a known
//      hash or of an EARLIER event of the batch (spliced in when that
//      event's digest is known: the in-batch DAG dependency of core.sync)
//   Creator  the creator key's raw bytes (ReadWireInfo: DecodeFromString of
//      the repertoire peer's PubKeyHex), base64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/babbleverify.h"
#include "sha256.h"

#ifndef DEV
#define DEV __host__ __device__ __forceinline__
#endif

#define EVJ_NOPOS 0xFFFFFFFFu

DEV uint32_t evj_b64_len(uint64_t n) { return (uint32_t)(4 * ((n + 2) / 3)); }

DEV uint32_t evj_dec_len(int64_t v) {
  uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  uint32_t n = v < 0 ? 2 : 1;
  while (m >= 10) {
    m /= 10;
    n++;
  }
  return n;
}

DEV uint8_t *evj_lit(uint8_t *o, const char *s) {
  while (*s) *o++ = (uint8_t)*s++;
  return o;
}

DEV uint8_t *evj_dec(uint8_t *o, int64_t v) {
  const uint32_t n = evj_dec_len(v);
  uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  if (v < 0) o[0] = '-';
  for (uint32_t i = n; i > (v < 0 ? 1u : 0u); i--) {
    o[i - 1] = (uint8_t)('0' + m % 10);
    m /= 10;
  }
  return o + n;
}

DEV uint8_t evj_b64c(uint32_t x) {
  return (uint8_t)(x < 26 ? 'A' + x : x < 52 ? 'a' + (x - 26) : x < 62 ? '0' + (x - 52) : x == 62 ? '+' : '/');
}

DEV uint8_t *evj_b64(uint8_t *o, const uint8_t *src, uint64_t n) {
  uint64_t i = 0;
  for (; i + 3 <= n; i += 3) {
    const uint32_t v = ((uint32_t)src[i] << 16) | ((uint32_t)src[i + 1] << 8) | src[i + 2];
    o[0] = evj_b64c(v >> 18);
    o[1] = evj_b64c((v >> 12) & 63);
    o[2] = evj_b64c((v >> 6) & 63);
    o[3] = evj_b64c(v & 63);
    o += 4;
  }
  if (n - i == 1) {
    const uint32_t v = (uint32_t)src[i] << 16;
    o[0] = evj_b64c(v >> 18);
    o[1] = evj_b64c((v >> 12) & 63);
    o[2] = '=';
    o[3] = '=';
    o += 4;
  } else if (n - i == 2) {
    const uint32_t v = ((uint32_t)src[i] << 16) | ((uint32_t)src[i + 1] << 8);
    o[0] = evj_b64c(v >> 18);
    o[1] = evj_b64c((v >> 12) & 63);
    o[2] = evj_b64c((v >> 6) & 63);
    o[3] = '=';
    o += 4;
  }
  return o;
}

// 32 digest bytes -> 64 uppercase hex chars
DEV void evj_hex32(uint8_t *o, const uint8_t *d) {
  for (int i = 0; i < 32; i++) {
    const uint32_t hi = d[i] >> 4, lo = d[i] & 15;
    o[2 * i] = (uint8_t)(hi < 10 ? '0' + hi : 'A' + hi - 10);
    o[2 * i + 1] = (uint8_t)(lo < 10 ? '0' + lo : 'A' + lo - 10);
  }
}

// literal pieces of the template (lengths derived from the strings)
#define EVJ_L0 "{\"Transactions\":"
#define EVJ_L1 ",\"InternalTransactions\":"
#define EVJ_L2 ",\"Parents\":["
#define EVJ_L3 ",\"Creator\":\""
#define EVJ_L4 "\",\"Index\":"
#define EVJ_L5 ",\"BlockSignatures\":"
#define EVJ_L6 ",\"Timestamp\":"
#define EVJ_LEN(s) ((uint32_t)(sizeof(s) - 1))

DEV uint64_t evj_frag_len(const uint64_t *off, uint64_t e) {
  if (!off) return 0;
  return off[e + 1] - off[e];
}

// Body length of event e and the offsets of its in-batch parents' 64 hex
// characters within the body (EVJ_NOPOS when that parent is not an event
// of the batch).
DEV uint64_t evj_len(const bv_event_batch &b, uint64_t e, uint32_t ppos[2]) {
  uint64_t n = EVJ_LEN(EVJ_L0);
  if (b.tx_list_nil && b.tx_list_nil[e]) {
    n += 4;
  } else {
    const uint64_t t0 = b.tx_start[e], t1 = b.tx_start[e + 1];
    n += 2 + (t1 > t0 ? t1 - t0 - 1 : 0);
    for (uint64_t t = t0; t < t1; t++)
      n += (b.tx_nil && b.tx_nil[t]) ? 4 : 2 + evj_b64_len(b.tx_off[t + 1] - b.tx_off[t]);
  }
  n += EVJ_LEN(EVJ_L1);
  const uint64_t il = evj_frag_len(b.itx_off, e);
  n += il ? il : 4;
  n += EVJ_LEN(EVJ_L2);
  for (int p = 0; p < 2; p++) {
    const uint8_t k = b.parent_kind[2 * e + p];
    ppos[p] = (k == BV_PARENT_EVENT) ? (uint32_t)(n + 3) : EVJ_NOPOS;
    n += k == BV_PARENT_NONE ? 2 : 68;
    if (p == 0) n += 1;  // ','
  }
  n += 1;  // ']'
  const uint32_t c = b.creator[e];
  n += EVJ_LEN(EVJ_L3) + evj_b64_len(b.key_off[c + 1] - b.key_off[c]);
  n += EVJ_LEN(EVJ_L4) + evj_dec_len(b.index[e]);
  const uint64_t bl = evj_frag_len(b.bsig_off, e);
  n += EVJ_LEN(EVJ_L5) + (bl ? bl : 4);
  n += EVJ_LEN(EVJ_L6) + evj_dec_len(b.timestamp[e]) + 2;  // "}\n"
  return n;
}

// Write event e's body at `o` (evj_len bytes).  In-batch parents get 64 '0'
// placeholders, overwritten by evj_hex32 once the parent's digest exists.
DEV void evj_write(const bv_event_batch &b, uint64_t e, uint8_t *o) {
  o = evj_lit(o, EVJ_L0);
  if (b.tx_list_nil && b.tx_list_nil[e]) {
    o = evj_lit(o, "null");
  } else {
    const uint64_t t0 = b.tx_start[e], t1 = b.tx_start[e + 1];
    *o++ = '[';
    for (uint64_t t = t0; t < t1; t++) {
      if (t > t0) *o++ = ',';
      if (b.tx_nil && b.tx_nil[t]) {
        o = evj_lit(o, "null");
      } else {
        *o++ = '"';
        o = evj_b64(o, b.tx_bytes + b.tx_off[t], b.tx_off[t + 1] - b.tx_off[t]);
        *o++ = '"';
      }
    }
    *o++ = ']';
  }
  o = evj_lit(o, EVJ_L1);
  const uint64_t il = evj_frag_len(b.itx_off, e);
  if (il) {
    for (uint64_t i = 0; i < il; i++) o[i] = b.itx_json[b.itx_off[e] + i];
    o += il;
  } else {
    o = evj_lit(o, "null");
  }
  o = evj_lit(o, EVJ_L2);
  for (int p = 0; p < 2; p++) {
    const uint8_t k = b.parent_kind[2 * e + p];
    if (p == 1) *o++ = ',';
    if (k == BV_PARENT_NONE) {
      o = evj_lit(o, "\"\"");
      continue;
    }
    o = evj_lit(o, "\"0X");
    if (k == BV_PARENT_HASH)
      evj_hex32(o, b.parent_hashes + 32 * b.parent_ref[2 * e + p]);
    else
      for (int i = 0; i < 64; i++) o[i] = '0';
    o += 64;
    *o++ = '"';
  }
  *o++ = ']';
  o = evj_lit(o, EVJ_L3);
  const uint32_t c = b.creator[e];
  o = evj_b64(o, b.key_bytes + b.key_off[c], b.key_off[c + 1] - b.key_off[c]);
  o = evj_lit(o, EVJ_L4);
  o = evj_dec(o, b.index[e]);
  o = evj_lit(o, EVJ_L5);
  const uint64_t bl = evj_frag_len(b.bsig_off, e);
  if (bl) {
    for (uint64_t i = 0; i < bl; i++) o[i] = b.bsig_json[b.bsig_off[e] + i];
    o += bl;
  } else {
    o = evj_lit(o, "null");
  }
  o = evj_lit(o, EVJ_L6);
  o = evj_dec(o, b.timestamp[e]);
  o[0] = '}';
  o[1] = '\n';
}

// ---------------------------------------------------------------------------
// Hashing along the in-batch DAG (hostdag.cpp).  A body's blocks that lie
// wholly before its first in-batch parent's hex do not depend on any other
// event: they are compressed once, all events in parallel, into a midstate;
// only the remaining blocks sit on the serial chain (T=1 bodies: 6 of 8
// blocks).
// ---------------------------------------------------------------------------
DEV uint32_t ev_mid_blocks(const uint32_t pp[2]) {
  uint32_t m = EVJ_NOPOS;
  for (int p = 0; p < 2; p++)
    if (pp[p] != EVJ_NOPOS && pp[p] < m) m = pp[p];
  return m == EVJ_NOPOS ? 0u : m / 64u;
}
