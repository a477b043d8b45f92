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

// Output sinks: anything with put(uint8_t), bytes in order.  EvjMem writes
// them to memory (the host DAG path and the emulator); the device's bulk
// path feeds them straight into SHA-256 (kernels.hip EvjShaSink).
struct EvjMem {
  uint8_t *p;
  DEV void put(uint8_t c) { *p++ = c; }
};

template <class O>
DEV void evj_lit(O &o, const char *s) {
  while (*s) o.put((uint8_t)*s++);
}

// decimal, most significant digit first: the digits (<= 20) are collected
// least significant first as nibbles of lo (16) and hi (4), then emitted
template <class O>
DEV void evj_dec(O &o, int64_t v) {
  uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  if (v < 0) o.put('-');
  uint64_t lo = 0, hi = 0;
  int n = 0;
  do {
    const uint64_t d = m % 10;
    m /= 10;
    if (n < 16) lo |= d << (4 * n);
    else hi |= d << (4 * (n - 16));
    n++;
  } while (m);
  for (int i = n - 1; i >= 0; i--) o.put((uint8_t)('0' + ((i < 16 ? lo >> (4 * i) : hi >> (4 * (i - 16))) & 15)));
}

DEV uint8_t evj_b64c(uint32_t x) {
  return (uint8_t)(x < 26 ? 'A' + x : x < 52 ? 'a' + (x - 26) : x < 62 ? '0' + (x - 52) : x == 62 ? '+' : '/');
}

template <class O>
DEV void evj_b64(O &o, const uint8_t *src, uint64_t n) {
  uint64_t i = 0;
  for (; i + 3 <= n; i += 3) {
    const uint32_t v = ((uint32_t)src[i] << 16) | ((uint32_t)src[i + 1] << 8) | src[i + 2];
    o.put(evj_b64c(v >> 18));
    o.put(evj_b64c((v >> 12) & 63));
    o.put(evj_b64c((v >> 6) & 63));
    o.put(evj_b64c(v & 63));
  }
  if (n - i == 1) {
    const uint32_t v = (uint32_t)src[i] << 16;
    o.put(evj_b64c(v >> 18));
    o.put(evj_b64c((v >> 12) & 63));
    o.put('=');
    o.put('=');
  } else if (n - i == 2) {
    const uint32_t v = ((uint32_t)src[i] << 16) | ((uint32_t)src[i + 1] << 8);
    o.put(evj_b64c(v >> 18));
    o.put(evj_b64c((v >> 12) & 63));
    o.put(evj_b64c((v >> 6) & 63));
    o.put('=');
  }
}

DEV uint8_t evj_hexc(uint32_t x) { return (uint8_t)(x < 10 ? '0' + x : 'A' + x - 10); }

// 32 digest bytes -> 64 uppercase hex chars (in place: the host DAG splice)
DEV void evj_hex32(uint8_t *o, const uint8_t *d) {
  for (int i = 0; i < 32; i++) {
    o[2 * i] = evj_hexc(d[i] >> 4);
    o[2 * i + 1] = evj_hexc(d[i] & 15);
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

// Event e's body into sink `o` (evj_len bytes).  In-batch parents get 64 '0'
// placeholders, overwritten by evj_hex32 once the parent's digest exists.
template <class O>
DEV void evj_emit(const bv_event_batch &b, uint64_t e, O &o) {
  evj_lit(o, EVJ_L0);
  if (b.tx_list_nil && b.tx_list_nil[e]) {
    evj_lit(o, "null");
  } else {
    const uint64_t t0 = b.tx_start[e], t1 = b.tx_start[e + 1];
    o.put('[');
    for (uint64_t t = t0; t < t1; t++) {
      if (t > t0) o.put(',');
      if (b.tx_nil && b.tx_nil[t]) {
        evj_lit(o, "null");
      } else {
        o.put('"');
        evj_b64(o, b.tx_bytes + b.tx_off[t], b.tx_off[t + 1] - b.tx_off[t]);
        o.put('"');
      }
    }
    o.put(']');
  }
  evj_lit(o, EVJ_L1);
  const uint64_t il = evj_frag_len(b.itx_off, e);
  if (il) {
    for (uint64_t i = 0; i < il; i++) o.put(b.itx_json[b.itx_off[e] + i]);
  } else {
    evj_lit(o, "null");
  }
  evj_lit(o, EVJ_L2);
  for (int p = 0; p < 2; p++) {
    const uint8_t k = b.parent_kind[2 * e + p];
    if (p == 1) o.put(',');
    if (k == BV_PARENT_NONE) {
      evj_lit(o, "\"\"");
      continue;
    }
    evj_lit(o, "\"0X");
    if (k == BV_PARENT_HASH) {
      const uint8_t *d = b.parent_hashes + 32 * b.parent_ref[2 * e + p];
      for (int i = 0; i < 32; i++) {
        o.put(evj_hexc(d[i] >> 4));
        o.put(evj_hexc(d[i] & 15));
      }
    } else {
      for (int i = 0; i < 64; i++) o.put('0');
    }
    o.put('"');
  }
  o.put(']');
  evj_lit(o, EVJ_L3);
  const uint32_t c = b.creator[e];
  evj_b64(o, b.key_bytes + b.key_off[c], b.key_off[c + 1] - b.key_off[c]);
  evj_lit(o, EVJ_L4);
  evj_dec(o, b.index[e]);
  evj_lit(o, EVJ_L5);
  const uint64_t bl = evj_frag_len(b.bsig_off, e);
  if (bl) {
    for (uint64_t i = 0; i < bl; i++) o.put(b.bsig_json[b.bsig_off[e] + i]);
  } else {
    evj_lit(o, "null");
  }
  evj_lit(o, EVJ_L6);
  evj_dec(o, b.timestamp[e]);
  o.put('}');
  o.put('\n');
}

// Streaming SHA-256 sink (k_ev_body_hash: the body is never stored).
// `row` holds the chaining value (8 words) and the current block (16 words,
// big-endian); bytes are packed into `w` and stored a word at a time.  The
// compression is out of line: one copy of the rounds, not one per put()
// call site of evj_emit.
__host__ __device__ __attribute__((noinline)) inline void evj_sha_block(uint32_t *row) {
  uint32_t h[8], w[16];
  for (int i = 0; i < 8; i++) h[i] = row[i];
  for (int i = 0; i < 16; i++) w[i] = row[8 + i];
  sha256_compress(h, w);
  for (int i = 0; i < 8; i++) row[i] = h[i];
}

struct EvjSha {
  uint32_t *row;
  uint32_t w, n, nblk;  // pending word, bytes in the current block, full blocks
  DEV void put(uint8_t c) {
    w = (w << 8) | c;
    if ((++n & 3) == 0) {
      row[8 + (n >> 2) - 1] = w;
      if (n == 64) {
        evj_sha_block(row);
        n = 0;
        nblk++;
      }
    }
  }
};

DEV EvjSha evj_sha_begin(uint32_t *row) {
  uint32_t h[8];
  sha256_init(h);
  for (int i = 0; i < 8; i++) row[i] = h[i];
  return EvjSha{row, 0, 0, 0};
}

// FIPS 180-4 padding, then the digest as big-endian bytes packed in words
// (the layout of sha256_one's digest words)
DEV void evj_sha_finish(EvjSha &o, uint32_t be[8]) {
  const uint64_t bits = ((uint64_t)o.nblk * 64 + o.n) * 8;
  o.put(0x80);
  while (o.n != 56) o.put(0);
  for (int i = 7; i >= 0; i--) o.put((uint8_t)(bits >> (8 * i)));
  for (int i = 0; i < 8; i++) be[i] = bswap32(o.row[i]);
}

// Event e's body written at `o` (evj_len bytes).
DEV void evj_write(const bv_event_batch &b, uint64_t e, uint8_t *o) {
  EvjMem m{o};
  evj_emit(b, e, m);
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
