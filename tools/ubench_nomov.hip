// VERDICT r4 #2b: what could a column layout that removes fe_mul's 25
// v_mov_b32 gain?  Times the shipped fe_mul_asm against the same program with
// every move deleted (tools/strip_movs.py; wrong results, same mads, carry
// counts, rare-block branches and wait states), in a dependent chain per lane
// at the verify kernels' occupancy (4 waves per SIMD) and at full occupancy.
// The gap is the ceiling for any move-free layout; a real one must spend
// instructions (carry adds at ~4.7 cycles) where the moves spend 2.4.
//   python tools/strip_movs.py > tools/_fe_mul_nomov.h
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_nomov tools/ubench_nomov.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../babble_amd/csrc/field.h"
#if defined(__HIP_DEVICE_COMPILE__)
#include "_fe_mul_nomov.h"
#endif

template <int MODE>
__global__ void __launch_bounds__(256) k(uint32_t seed, int iters, uint32_t *out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fe x, y;
  for (int i = 0; i < 8; i++) {
    x.v[i] = (seed + t) * 2654435761u ^ (i * 40503u);
    y.v[i] = (t * 97u + i) * 2246822519u;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  for (int it = 0; it < iters; it++) {
    if (MODE == 0)
      fe_mul_asm(x, x, y);
    else
      fe_mul_nomov_asm(x, x, y);
  }
#endif
  uint32_t s = 0;
  for (int i = 0; i < 8; i++) s ^= x.v[i];
  out[t] = s;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int threads = 256, iters = 512;
  uint32_t *out;
  if (hipMalloc(&out, sizeof(uint32_t) * 256 * 32 * threads) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // 1024 blocks = 4 waves per SIMD (the verify kernels), 8192 = as many as fit
  for (int blocks : {1024, 8192}) {
    float best[2] = {1e30f, 1e30f};
    for (int rep = 0; rep < 3; rep++)
      for (int mode = 0; mode < 2; mode++) {
        float ms;
        (void)hipEventRecord(e0);
        if (mode == 0)
          hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, 1u, iters, out);
        else
          hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, 1u, iters, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best[mode]) best[mode] = ms;
      }
    const double muls = (double)blocks * threads * iters;
    printf("%5d blocks (%2d waves/SIMD requested): shipped fe_mul %.3f ms %6.1f G mul/s | without its 25 v_mov "
           "%.3f ms %6.1f G mul/s | move-free ceiling %.1f%%\n",
           blocks, blocks * 4 / 1024, best[0], muls / best[0] / 1e6, best[1], muls / best[1] / 1e6,
           100.0 * (best[0] - best[1]) / best[0]);
  }
  return 0;
}
