// VERDICT r4 #2a: could the 256-bit field multiply run on the FP64 FMA
// pipe?  A 5 x 52-bit-limb product needs 25 partial products, each split
// exactly into two 52-bit halves with FP64 FMAs (round toward zero: hi =
// fma(a, b, 2^104) holds floor(ab / 2^52) in its mantissa, t = (2^104 +
// 2^52) - hi, lo = fma(a, b, t) = ab mod 2^52 + 2^52 exactly; both read as
// integers from their bit patterns), the halves summed per column in 64-bit
// integers.  This prototype times that PRODUCT PHASE ALONE — no carry
// normalisation, no reduction mod p (the next iteration's operands are the
// low 52 bits of five column sums) — against the shipped 8 x 32-bit fe_mul
// (field_asm.h: product, reduction and all).  If the partial product phase
// alone is not faster than the whole shipped multiply, the FP64 limb layout
// cannot win.  Correctness of the split is checked on the host for every
// lane's first products (exact 104-bit products against __int128).
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_fp64 tools/ubench_fp64.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../babble_amd/csrc/field.h"

#define M52 ((1ull << 52) - 1)

__device__ __forceinline__ double u2d(uint64_t x) { return __longlong_as_double((long long)x); }
__device__ __forceinline__ uint64_t d2u(double x) { return (uint64_t)__double_as_longlong(x); }

// FP64 round toward zero for the whole wave: MODE.FP_ROUND[3:2] = 3 (the
// compiler resets the mode around its own u64 -> f64 conversions, so this
// is set again right before the products; the asm is a scheduling barrier)
__device__ __forceinline__ void fp64_round_toward_zero(double a[5], double b[5]) {
  // (the operands pass through the asm: no product can be scheduled above it)
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 3"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]),
                 "+v"(b[3]), "+v"(b[4])
               :
               : "memory");
}

// 25 exact partial products of a[5] x b[5] (52-bit limbs as doubles) summed
// per column (10 columns, 64-bit integers)
__device__ __forceinline__ void prod52(uint64_t c[10], double a[5], double b[5]) {
  fp64_round_toward_zero(a, b);
  const double C104 = 20282409603651670423947251286016.0;  // 2^104
  const double C104p52 = C104 + 4503599627370496.0;      // 2^104 + 2^52 (exact)
  const uint64_t B104 = d2u(C104), B52 = d2u(4503599627370496.0);
#pragma unroll
  for (int k = 0; k < 10; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 5; i++)
#pragma unroll
    for (int j = 0; j < 5; j++) {
      const double hi = fma(a[i], b[j], C104);  // (the MODE register rounds toward zero)
      const double t = C104p52 - hi;
      const double lo = fma(a[i], b[j], t);
      c[i + j] += d2u(lo) - B52;      // ab mod 2^52
      c[i + j + 1] += d2u(hi) - B104;  // floor(ab / 2^52)
    }
}

template <int MODE>
__global__ void __launch_bounds__(256) k(uint32_t seed, int iters, uint64_t *out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (MODE == 0) {
    fe x, y;
    for (int i = 0; i < 8; i++) {
      x.v[i] = (seed + t) * 2654435761u ^ (i * 40503u);
      y.v[i] = (t * 97u + i) * 2246822519u;
    }
    for (int it = 0; it < iters; it++) fe_mul(x, x, y);
    uint64_t s = 0;
    for (int i = 0; i < 8; i++) s ^= x.v[i];
    out[t] = s;
  } else {
    double a[5], b[5];
    for (int i = 0; i < 5; i++) {
      a[i] = (double)((((uint64_t)((seed + t) * 2654435761u) << 20) ^ (i * 0x9E3779B97ull)) & M52);
      b[i] = (double)((((uint64_t)(t * 97u + i) * 2246822519ull) << 9) & M52);
    }
    uint64_t c[10];
    for (int it = 0; it < iters; it++) {
      prod52(c, a, b);
#pragma unroll
      for (int i = 0; i < 5; i++) a[i] = u2d((c[i] & M52) | d2u(4503599627370496.0)) - 4503599627370496.0;
    }
    uint64_t s = 0;
    for (int k = 0; k < 10; k++) s ^= c[k];
    out[t] = s;
  }
}

// the split on known operands: c[] of one prod52 against exact products
__global__ void k_check(const uint64_t *ops, uint64_t *c_out) {
  double a[5], b[5];
  for (int i = 0; i < 5; i++) a[i] = (double)ops[i], b[i] = (double)ops[5 + i];
  uint64_t c[10];
  prod52(c, a, b);
  for (int k = 0; k < 10; k++) c_out[k] = c[k];
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int blocks = 256 * 16, threads = 256, iters = 256;
  uint64_t *out;
  if (hipMalloc(&out, sizeof(uint64_t) * blocks * threads) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms[2] = {0, 0};
  for (int rep = 0; rep < 2; rep++) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, 1u, iters, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms[0], e0, e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, 1u, iters, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms[1], e0, e1);
  }
  // exactness of the split (host __int128 reference), edge and random limbs
  uint64_t hops[10], hc[10], *dops, *dc;
  (void)hipMalloc(&dops, 80);
  (void)hipMalloc(&dc, 80);
  int bad = 0;
  uint64_t st = 88172645463325252ull;
  for (int trial = 0; trial < 64; trial++) {
    for (int i = 0; i < 10; i++) {
      st ^= st << 13, st ^= st >> 7, st ^= st << 17;
      hops[i] = trial == 0 ? M52 : (trial == 1 ? 0 : st & M52);
    }
    (void)hipMemcpy(dops, hops, 80, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(1), dim3(1), 0, 0, dops, dc);
    (void)hipMemcpy(hc, dc, 80, hipMemcpyDeviceToHost);
    // the full check: sum_k c[k] 2^(52 k) == sum_{i,j} a_i b_j 2^(52 (i + j)), compared limb by limb
    // through a 52-bit carry walk on both sides
    uint64_t ref[11] = {0};
    for (int i = 0; i < 5; i++)
      for (int j = 0; j < 5; j++) {
        unsigned __int128 p = (unsigned __int128)hops[i] * hops[5 + j];
        int k2 = i + j;
        while (p) {
          unsigned __int128 s = (unsigned __int128)ref[k2] + (uint64_t)(p & M52);
          ref[k2] = (uint64_t)(s & M52);
          p = (p >> 52) + (s >> 52);
          k2++;
        }
      }
    uint64_t norm[11] = {0};
    unsigned __int128 cy = 0;
    for (int k2 = 0; k2 < 11; k2++) {
      const unsigned __int128 s = cy + (k2 < 10 ? hc[k2] : 0);
      norm[k2] = (uint64_t)(s & M52);
      cy = s >> 52;
    }
    for (int k2 = 0; k2 < 11; k2++) bad += norm[k2] != ref[k2];
  }
  const double ops = (double)blocks * threads * iters;
  printf("shipped 8x32 fe_mul (product + reduction, field_asm.h)  %7.3f ms  %7.1f G mul/s\n", ms[0],
         ops / ms[0] / 1e6);
  printf("FP64 5x52 partial products ONLY (25 FMA splits + column sums, no reduction)  %7.3f ms  %7.1f G/s  "
         "(%.2fx the whole shipped multiply's time)\n",
         ms[1], ops / ms[1] / 1e6, ms[1] / ms[0]);
  printf("split exactness: %d mismatching 52-bit limbs over 64 operand sets (0 = exact)\n", bad);
  return bad != 0;
}
