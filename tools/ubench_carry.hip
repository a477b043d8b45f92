// Microbenchmark: cost of VCC carry chains (__builtin_addc, which hipcc pads
// with s_nop between links on gfx950) against carry-free 32-bit adds and
// against the field multiply, at full occupancy.  Informs the choice of
// limb radix in babble_amd/csrc/field.h.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../babble_amd/csrc/field.h"

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) {                                                                 \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

// 4 independent 8-limb carry chains per iteration (32 addc)
__global__ void __launch_bounds__(256) k_chain(uint32_t *out, uint32_t seed, int iters) {
  uint32_t a[4][8], b[8];
  for (int i = 0; i < 8; i++) {
    b[i] = seed * (i + 3);
    for (int c = 0; c < 4; c++) a[c][i] = threadIdx.x + 31 * i + c;
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      uint32_t cy = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) a[c][i] = addc32(a[c][i], b[i], cy);
      b[0] ^= cy;
    }
  }
  uint32_t s = 0;
  for (int c = 0; c < 4; c++)
    for (int i = 0; i < 8; i++) s ^= a[c][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// same count of carry-free adds (32 per iteration)
__global__ void __launch_bounds__(256) k_plain(uint32_t *out, uint32_t seed, int iters) {
  uint32_t a[4][8], b[8];
  for (int i = 0; i < 8; i++) {
    b[i] = seed * (i + 3);
    for (int c = 0; c < 4; c++) a[c][i] = threadIdx.x + 31 * i + c;
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
#pragma unroll
      for (int i = 0; i < 8; i++) a[c][i] += b[i];
      b[0] ^= a[c][7];
    }
  }
  uint32_t s = 0;
  for (int c = 0; c < 4; c++)
    for (int i = 0; i < 8; i++) s ^= a[c][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// field multiply throughput (2 independent chains per thread)
__global__ void __launch_bounds__(256) k_femul(uint32_t *out, uint32_t seed, int iters) {
  fe a, b, c;
  for (int i = 0; i < 8; i++) {
    a.v[i] = seed + threadIdx.x * 7 + i;
    b.v[i] = seed * 3 + i;
    c.v[i] = seed ^ i;
  }
  for (int it = 0; it < iters; it++) {
    fe_mul(a, a, b);
    fe_mul(c, c, b);
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; i++) s ^= a.v[i] ^ c.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_fesqr(uint32_t *out, uint32_t seed, int iters) {
  fe a, c;
  for (int i = 0; i < 8; i++) {
    a.v[i] = seed + threadIdx.x * 7 + i;
    c.v[i] = seed ^ i;
  }
  for (int it = 0; it < iters; it++) {
    fe_sqr(a, a);
    fe_sqr(c, c);
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; i++) s ^= a.v[i] ^ c.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_feadd(uint32_t *out, uint32_t seed, int iters) {
  fe a, b, c;
  for (int i = 0; i < 8; i++) {
    a.v[i] = seed + threadIdx.x * 7 + i;
    b.v[i] = seed * 3 + i;
    c.v[i] = seed ^ i;
  }
  for (int it = 0; it < iters; it++) {
    fe_add(a, a, b);
    fe_sub(c, c, b);
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; i++) s ^= a.v[i] ^ c.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint32_t *, uint32_t, int);

static int run(const char *name, kfn k, uint32_t *out, int blocks, int iters, double ops_per_iter) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 2u, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double n = (double)blocks * 256 * iters * ops_per_iter;
  printf("%-34s %8.3f ms  %9.3f G ops/s  %8.2f ns per 1M lane-ops\n", name, ms, n / (ms * 1e-3) / 1e9,
         ms * 1e6 / (n / 1e6) / 1e3);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int blocks = p.multiProcessorCount * 8;
  uint32_t *out;
  CHECK(hipMalloc(&out, sizeof(uint32_t) * 256 * blocks));
  run("addc chain (32 addc/iter)", k_chain, out, blocks, 4096, 32);
  run("plain add (32 add/iter)", k_plain, out, blocks, 4096, 32);
  run("fe_mul (2/iter)", k_femul, out, blocks, 512, 2);
  run("fe_sqr (2/iter)", k_fesqr, out, blocks, 512, 2);
  run("fe_add+fe_sub (2/iter)", k_feadd, out, blocks, 2048, 2);
  return 0;
}
