// hostsha.h — SHA-256 on the host CPU (FIPS 180-4), for the one place the
// verifier hashes on the host: the in-batch DAG of a SyncResponse
// (bv_verify_events, hostdag.cpp), whose digests form a dependency chain that
// one CPU core walks ~50x faster than one GPU wave (SURVEY §8f-1's first
// option).  x86 SHA extensions when the CPU has them, else portable C++;
// chosen once per process.  Not a fallback for the device path.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace hsha {
void init(uint32_t h[8]);
// h <- compress(h, blocks) over `nblocks` 64-byte blocks
void compress(uint32_t h[8], const uint8_t *blocks, size_t nblocks);
// The digest of msg[0, len) given h = the state after its first `from`
// bytes (from a multiple of 64): the remaining whole blocks, the FIPS
// padding, and the 32 big-endian digest bytes into `out`.
void finish(uint32_t h[8], const uint8_t *msg, size_t from, size_t len, uint8_t out[32]);
// finish() of two independent messages, their compressions interleaved
// (SHA extensions; the portable code runs them one after the other)
void finish2(uint32_t ha[8], const uint8_t *ma, size_t from_a, size_t len_a, uint8_t out_a[32], uint32_t hb[8],
             const uint8_t *mb, size_t from_b, size_t len_b, uint8_t out_b[32]);
void digest(const uint8_t *msg, size_t len, uint8_t out[32]);
// 1 when the SHA extensions are used; force_portable(true) selects the
// portable code (tests exercise both)
int accelerated();
void force_portable(bool on);
}  // namespace hsha
