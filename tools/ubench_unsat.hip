// A/B prototype: the shipped saturated 8 x 32-bit field
// multiply (field_asm.h, v_mad_u64_u32 with carry-out + addc chains) against
// an UNSATURATED 9 x 29-bit multiply whose column sums fit the 64-bit mad
// addend (81 carry-free mads, then normalisation and the fold
// 2^261 = 2^37 + 31264 mod p).  Both run as dependent chains in every lane
// at full occupancy; the results are cross-checked (canonical values equal).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_unsat tools/ubench_unsat.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../babble_amd/csrc/field.h"

#define M29 0x1FFFFFFFu

__device__ __forceinline__ void fe9_mul(uint32_t r[9], const uint32_t a[9], const uint32_t b[9]) {
  uint64_t c[17];
#pragma unroll
  for (int k = 0; k < 17; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++)
#pragma unroll
    for (int j = 0; j < 9; j++) c[i + j] += (uint64_t)a[i] * b[j];  // v_mad_u64_u32, no carries
  uint32_t l[17];
  uint64_t cy = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    const uint64_t v = c[k] + cy;
    l[k] = (uint32_t)v & M29;
    cy = v >> 29;
  }
  // fold limbs 9..16 and the top carry (weight 2^(29 k) = 2^(29 (k-9)) 2^261)
  uint64_t t[10];
#pragma unroll
  for (int k = 0; k < 9; k++) t[k] = l[k];
  t[9] = 0;
#pragma unroll
  for (int k = 9; k < 17; k++) {
    t[k - 9] += (uint64_t)l[k] * 31264u;
    t[k - 8] += (uint64_t)l[k] << 8;
  }
  t[8] += cy * 31264u;  // cy has weight 2^(29*17) = 2^(29*8) 2^261
  t[9] += cy << 8;
  cy = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const uint64_t v = t[k] + cy;
    r[k] = (uint32_t)v & M29;
    cy = v >> 29;
  }
  const uint64_t top = t[9] + cy;  // weight 2^261, small
  uint64_t v0 = (uint64_t)r[0] + top * 31264u, v1 = (uint64_t)r[1] + (top << 8) + (v0 >> 29);
  r[0] = (uint32_t)v0 & M29;
  r[1] = (uint32_t)v1 & M29;
  r[2] += (uint32_t)(v1 >> 29);  // limbs may exceed 29 bits by a little: inputs < 2^30 are fine
}

__device__ void to9(uint32_t o[9], const fe &a) {
  for (int k = 0; k < 9; k++) {
    const int bit = 29 * k, w = bit / 32, s = bit % 32;
    uint64_t x = a.v[w];
    if (w + 1 < 8) x |= (uint64_t)a.v[w + 1] << 32;
    o[k] = (uint32_t)(x >> s) & M29;
  }
}
__device__ void from9(fe &o, const uint32_t a[9]) {  // value < 2^262 -> weak mod p via 8-limb add
  uint32_t w[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < 9; k++) {
    const int bit = 29 * k, wi = bit / 32, s = bit % 32;
    const uint64_t x = (uint64_t)a[k] << s;
    uint64_t acc = (uint64_t)w[wi] + (uint32_t)x;
    w[wi] = (uint32_t)acc;
    uint64_t carry = (acc >> 32) + (x >> 32);
    for (int q = wi + 1; q < 9 && carry; q++) {
      acc = (uint64_t)w[q] + carry;
      w[q] = (uint32_t)acc;
      carry = acc >> 32;
    }
  }
  // w[8] * 2^256 = w[8] (2^32 + 977)
  fe lo, hi;
  for (int k = 0; k < 8; k++) lo.v[k] = w[k];
  for (int k = 0; k < 8; k++) hi.v[k] = 0;
  uint64_t m = (uint64_t)w[8] * 977u;
  hi.v[0] = (uint32_t)m;
  hi.v[1] = (uint32_t)(m >> 32) + w[8];
  fe_add(o, lo, hi);
}

template <int MODE>
__global__ void __launch_bounds__(256) k(uint32_t seed, int iters, uint32_t *out, uint32_t *bad) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fe x, y;
  for (int i = 0; i < 8; i++) {
    x.v[i] = (seed + t) * 2654435761u ^ (i * 40503u);
    y.v[i] = (t * 97u + i) * 2246822519u;
  }
  x.v[7] &= 0x7FFFFFFFu;
  y.v[7] &= 0x7FFFFFFFu;
  if (MODE == 0) {
    for (int it = 0; it < iters; it++) fe_mul(x, x, y);
    fe_canon(x);
    for (int i = 0; i < 8; i++) out[8 * t + i] = x.v[i];
  } else if (MODE == 2) {  // variable-time inversion (modinv.h), the batched-affine cost model's unknown
    for (int it = 0; it < iters / 16; it++) {
      fe_inv_var(x, x);
      x.v[0] ^= it;
    }
    for (int i = 0; i < 8; i++) out[8 * t + i] ^= x.v[i];
  } else if (MODE == 1) {
    uint32_t a[9], b[9];
    to9(a, x);
    to9(b, y);
    for (int it = 0; it < iters; it++) fe9_mul(a, a, b);
    fe r;
    from9(r, a);
    fe_canon(r);
    for (int i = 0; i < 8; i++)
      if (out[8 * t + i] != r.v[i]) atomicAdd(bad, 1u);
  }
}

int main() {
  const int blocks = 256 * 16, threads = 256, iters = 256;
  uint32_t *out, *bad;
  hipMalloc(&out, (size_t)blocks * threads * 32);
  hipMalloc(&bad, 4);
  hipMemset(bad, 0, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms[2];
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, 1u, iters, out, bad);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, 1u, iters, out, bad);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms[0], e0, e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, 1u, iters, out, bad);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms[1], e0, e1);
  }
  float msi;
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(threads), 0, 0, 1u, iters, out, bad);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&msi, e0, e1);
  uint32_t nb = 0;
  hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost);
  const double ops = (double)blocks * threads * iters;
  printf("saturated 8x32 fe_mul (field_asm.h)   %7.3f ms  %7.1f G mul/s\n", ms[0], ops / ms[0] / 1e6);
  printf("unsaturated 9x29 fe9_mul (prototype)  %7.3f ms  %7.1f G mul/s  (%.2fx)\n", ms[1], ops / ms[1] / 1e6,
         ms[1] / ms[0]);
  printf("cross-check: %u mismatching words (unsaturated vs saturated results)\n", nb);
  printf("fe_inv_var (divsteps)                 %7.3f ms  %7.1f G inv/s  = %.1f fe_mul-equivalents\n", msi,
         ops / 16 / msi / 1e6, (msi / (ops / 16)) / (ms[0] / ops));
  return nb != 0;
}
