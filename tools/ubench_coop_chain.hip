// Latency of coop.h's cooperative products on one wave (the cold path's
// situation: one dependent chain, nothing beside it): a chain of coop::mul,
// a chain of coop::dbl_xyzz (the Q doubling chain of k_small's cold path),
// and a chain of coop::add_xyzz.  Built twice for a same-box A/B:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCOOP_HEADER='"/tmp/coop_old.h"' ...
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 ...   (the tree's coop.h)
// and checks that the chains' results agree with a per-lane fe_mul chain.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#ifndef COOP_HEADER
#define COOP_HEADER "../babble_amd/csrc/coop.h"
#endif
#include COOP_HEADER

#define CHK(x)                                                    \
  do {                                                            \
    hipError_t e_ = (x);                                          \
    if (e_ != hipSuccess) {                                       \
      printf("%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                   \
    }                                                             \
  } while (0)

__global__ void __launch_bounds__(64) k_mul_chain(uint32_t *out, int chain) {
  const uint32_t k = coop::pos();
  uint32_t r = k < 8 ? 0x9E3779B9u * (k + 3) + coop::row() : 0u, b = k < 8 ? 0x85EBCA6Bu * (k + 1) : 0u;
  for (int c = 0; c < chain; c++) r = coop::mul(r, b);
  if (threadIdx.x < 64) out[threadIdx.x] = r;
}
// the same chain per lane (fe_mul), lanes 0..3 one row's value each
__global__ void __launch_bounds__(64) k_mul_ref(uint32_t *out, int chain) {
  const uint32_t row = threadIdx.x;
  if (row >= 4) return;
  fe r, b;
  for (int k = 0; k < 8; k++) r.v[k] = 0x9E3779B9u * (k + 3) + row, b.v[k] = 0x85EBCA6Bu * (k + 1);
  for (int c = 0; c < chain; c++) fe_mul(r, r, b);
  fe_canon(r);
  for (int k = 0; k < 8; k++) out[64 + 8 * row + k] = r.v[k];
}
__global__ void __launch_bounds__(64) k_dbl_chain(uint32_t *out, int chain) {
  const uint32_t k = coop::pos();
  // G in XYZZ (ZZ = ZZZ = 1)
  const uint32_t gx[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                          0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
  const uint32_t gy[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                          0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
  uint32_t X = k < 8 ? gx[k] : 0u, Y = k < 8 ? gy[k] : 0u, ZZ = k == 0 ? 1u : 0u, ZZZ = ZZ, BX;
  for (int c = 0; c < chain; c++) coop::dbl_xyzz(X, Y, ZZ, ZZZ, BX);
  if (threadIdx.x < 16) out[128 + threadIdx.x] = X ^ Y ^ ZZ ^ ZZZ ^ BX;
}
__global__ void __launch_bounds__(64) k_add_chain(uint32_t *out, int chain) {
  const uint32_t k = coop::pos();
  const uint32_t gx[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                          0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
  const uint32_t gy[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                          0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
  uint32_t X = k < 8 ? gx[k] : 0u, Y = k < 8 ? gy[k] : 0u, ZZ = k == 0 ? 1u : 0u, ZZZ = ZZ, BX;
  coop::dbl_xyzz(X, Y, ZZ, ZZZ, BX);  // 2G, then += G repeatedly
  const uint32_t one = k == 0 ? 1u : 0u;
  bool inf = false;
  for (int c = 0; c < chain; c++)
    coop::add_xyzz(X, Y, ZZ, ZZZ, inf, k < 8 ? gx[k] : 0u, k < 8 ? gy[k] : 0u, one, one);
  if (threadIdx.x < 16) out[144 + threadIdx.x] = X ^ Y ^ ZZ ^ ZZZ;
}

int main() {
  uint32_t *d;
  CHK(hipMalloc(&d, 4096));
  CHK(hipMemset(d, 0, 4096));
  const int chain = 4096;
  hipLaunchKernelGGL(k_mul_chain, dim3(1), dim3(64), 0, 0, d, chain);
  hipLaunchKernelGGL(k_mul_ref, dim3(1), dim3(64), 0, 0, d, chain);
  CHK(hipDeviceSynchronize());
  uint32_t h[160];
  CHK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int row = 0; row < 4; row++) {
    // canonicalise the coop result (< 2^256, weakly reduced) for the compare
    uint32_t c[8];
    uint64_t br = 0;
    bool ge = true;
    static const uint32_t P[8] = {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                  0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    for (int i = 7; i >= 0; i--)
      if (h[16 * row + i] != P[i]) {
        ge = h[16 * row + i] > P[i];
        break;
      }
    for (int i = 0; i < 8; i++) {
      const uint64_t x = (uint64_t)h[16 * row + i] - (ge ? P[i] : 0u) - br;
      c[i] = (uint32_t)x;
      br = (x >> 63) & 1;
    }
    for (int i = 0; i < 8; i++) bad += c[i] != h[64 + 8 * row + i];
  }
  printf("%s: coop mul chain of %d vs per-lane fe_mul: %d limbs differ\n", COOP_HEADER, chain, bad);
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto timeit = [&](auto kern, int n) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, d, 8);
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, d, n);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    return (double)best * 1e6 / n;
  };
  printf("  mul       %.1f ns\n", timeit(k_mul_chain, 4096));
  printf("  dbl_xyzz  %.1f ns\n", timeit(k_dbl_chain, 1024));
  printf("  add_xyzz  %.1f ns\n", timeit(k_add_chain, 1024));
  return bad != 0;
}
