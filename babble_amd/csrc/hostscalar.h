// hostscalar.h — the item record of a latency batch (k_small with at most
// BV_HOST_SCALARS items): everything workgroup b reads, in ONE
// 256-byte record of the mapped host buffer (one wave-wide load over PCIe
// instead of chains of dependent reads), with the scalar half of
// ecdsa.Verify (crypto/ecdsa verify, steps 4-5: w = s^-1, u1 = e w, u2 = r w
// mod N, and u2's GLV split) already done on the host.
//
// Why on the host: that part is one serial chain — Bernstein–Yang divsteps
// plus a few Montgomery products — of ~80k shader clocks (~35 us) on one GPU
// lane (profiles/r06_ubench_sinv.txt) against ~3.4 us on one host core for
// one item (~1.3 us an item more in a batch), and for a single event
// nothing runs beside it.  The point half (the table
// leaves and the XYZZ sums, the Q doubling chain of the cold path) stays on
// the device; batches past the threshold invert on the device as before.
// The host runs the SAME functions (field.h / modinv.h compiled for the
// host: sc_mont's portable body, modinv_var, glv_split), so u1, k1, k2 are
// the values the device path computes.  Host-only code.
#pragma once
#include <stdint.h>

namespace hrec {
constexpr uint32_t kWords = 64;  // dwords per record (256 bytes)
// dword offsets
constexpr uint32_t kKey = 0;      // the public key bytes (<= 65 used, 72 readable)
constexpr uint32_t kKeyLen = 18;  // min(length, 66): 0 empty, 65 the only decodable one
constexpr uint32_t kPre = 19;     // the item's pre-class byte (bv_batch.pre)
constexpr uint32_t kR = 20;       // r, s: 32 big-endian bytes each, as given
constexpr uint32_t kS = 28;
constexpr uint32_t kU1 = 36;      // u1 = e s^-1 mod N, 8 little-endian limbs
constexpr uint32_t kK = 44;       // |k1| (4 limbs), |k2| (4 limbs): u2 = k1 + k2 lambda
constexpr uint32_t kSigns = 52;   // bit 0: k1 < 0, bit 1: k2 < 0
constexpr uint32_t kTab = 54;     // the key cache's table address (u64; 0: none)
}  // namespace hrec

// One item's inputs: the SHA-256 digest of its message, r and s (32
// big-endian bytes each), the pre-class byte (0 when the signature text
// parsed cleanly), its key's bytes and key-cache table address.
struct HostRecItem {
  const uint8_t *digest, *r, *s, *key;
  uint64_t key_len, table;
  uint8_t pre;
};

// The records of n items (recs: n * hrec::kWords dwords): the fields, and
// for every item whose s is usable (pre == 0, 0 < s < N) u1, k1, k2, signs
// — one inversion per 64 items (Montgomery's trick, as k_sinv does), so a
// batch costs ~2.2 us + ~1.3 us per item on one core.  Unusable items keep
// zero scalars (the kernel's decision table rejects them first).
void bv_host_item_records(uint32_t *recs, const HostRecItem *items, uint64_t n);
