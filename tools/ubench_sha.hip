// Latency of one SHA-256 compression on ONE wave (the k_ev_hash_chain
// regime: a few lanes active, nothing else on the SIMD): cycles per block for
// the plain compress (message schedule inline) and for rounds-only with a
// precomputed W+K schedule read from LDS.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../babble_amd/csrc/sha256.h"

DEV void rounds_wk_unrolled(uint32_t h[8], const uint32_t *wk) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25)) + ((e & f) ^ (~e & g)) + wk[i];
    uint32_t t2 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22)) + maj3(a, b, c);
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// rounds with h + K + W formed one round early (off the e -> e' path):
// e' = d + (hkw + S1(e) + Ch), a' = T1 + S0(a) + Maj, fully unrolled
DEV void rounds_wk_hkw(uint32_t h[8], const uint32_t *wk) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  uint32_t hkw = hh + wk[0];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    const uint32_t s1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hkw + s1 + ch;
    const uint32_t nhkw = i < 63 ? g + wk[i + 1] : 0;  // next round's h is this round's g
    const uint32_t t2 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22)) + maj3(a, b, c);
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
    hkw = nhkw;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// ... and d + (h + K + W) formed one round early too (d of round i+1 is c of
// round i), so e' = add3(dhkw, S1(e), Ch(e, f, g)): one dependent add fewer
// on the e -> e' chain per round (one more instruction per round)
DEV void rounds_wk_dhkw(uint32_t h[8], const uint32_t *wk) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  uint32_t hkw = hh + wk[0];
  uint32_t dhkw = d + hkw;
#pragma unroll
  for (int i = 0; i < 64; i++) {
    const uint32_t s1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t ne = dhkw + s1 + ch;
    const uint32_t t1 = hkw + s1 + ch;
    const uint32_t nhkw = i < 63 ? g + wk[i + 1] : 0;
    const uint32_t t2 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22)) + maj3(a, b, c);
    hh = g;
    g = f;
    f = e;
    e = ne;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
    hkw = nhkw;
    dhkw = d + hkw;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

template <int MODE>
__global__ void k(uint64_t *out, int nblk) {
  __shared__ uint32_t sW[64 * 64];
  const uint32_t t = threadIdx.x;
  for (int i = t; i < 64 * 64; i += blockDim.x) sW[i] = i * 2654435761u;
  __syncthreads();
  uint32_t h[8];
  sha256_init(h);
  h[0] ^= t;
  const uint64_t t0 = __builtin_readcyclecounter();
  if (t < 4) {
    for (int b = 0; b < nblk; b++) {
      if (MODE == 0) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = sW[(b & 63) * 64 + i] ^ h[i & 7];
        sha256_compress(h, w);
      } else if (MODE == 1) {
        rounds_wk_unrolled(h, sW + (b & 63) * 64);
      } else if (MODE == 3) {
        sha256_rounds_wk(h, sW + (b & 63) * 64);  // sha256.h: 8-trip loop of 8 rounds
      } else if (MODE == 4) {
        rounds_wk_hkw(h, sW + (b & 63) * 64);
      } else if (MODE == 5) {
        rounds_wk_dhkw(h, sW + (b & 63) * 64);
      } else {
        // the k_ev_hash_chain tail: a 446-byte T=1 body from block 2 (6
        // blocks, the last two partial) out of an LDS slot, byte shift 2
        sW[(b & 63)] ^= h[0];
        sha256_blocks(h, sW + (b & 15) * 128, 2, 446, 2, sha256_nblocks(446));
      }
    }
  }
  const uint64_t t1 = __builtin_readcyclecounter();
  if (t == 0) out[0] = t1 - t0;
  if (h[0] == 42) out[1] = h[1];
}

template <int MODE>
void run(const char *name) {
  uint64_t *d;
  hipMalloc(&d, 64);
  const int nblk = 2000;
  hipLaunchKernelGGL(k<MODE>, dim3(1), dim3(64), 0, 0, d, 10);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(1), dim3(64), 0, 0, d, nblk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  uint64_t cyc;
  hipMemcpy(&cyc, d, 8, hipMemcpyDeviceToHost);
  printf("%-40s %8.3f us/block (wall)   %8.1f counter ticks/block\n", name, ms * 1e3 / nblk, (double)cyc / nblk);
  hipFree(d);
}

int main() {
  run<0>("compress (schedule inline)");
  run<1>("rounds only (W+K from LDS)");
  run<2>("sha256_blocks tail (6 blocks/iter)");
  run<3>("rounds only, 8x8 loop (sha256.h)");
  run<4>("rounds only, hkw early, unrolled");
  run<5>("rounds only, d+hkw early, unrolled");
  return 0;
}
