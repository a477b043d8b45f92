// Throughput of the batch SHA-256 (k_sha256's per-lane sha256_msg) on 1M
// C2-sized messages (446 B, 8 blocks) packed back to back in HBM, against the
// same compression work with the message words generated in registers (no
// loads): shows whether the kernel is bound by its gathers or by VALU.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../babble_amd/csrc/sha256.h"

__global__ void __launch_bounds__(256) k_mem(uint64_t n, const uint8_t *bytes, uint64_t len, uint32_t *out) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  uint32_t h[8];
  sha256_msg(h, bytes, m * len, len);
  out[m] = h[0] ^ h[7];
}
__global__ void __launch_bounds__(256) k_reg(uint64_t n, uint64_t len, uint32_t *out) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  uint32_t h[8];
  sha256_init(h);
  const uint64_t nb = sha256_nblocks(len);
  for (uint64_t b = 0; b < nb; b++) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)m * 2654435761u + i * 40503u + (uint32_t)b;
    sha256_compress(h, w);
  }
  out[m] = h[0] ^ h[7];
}

int main() {
  const uint64_t n = 1000000, len = 446;
  uint8_t *bytes;
  uint32_t *out;
  hipMalloc(&bytes, n * len + 64);
  hipMemset(bytes, 0x5A, n * len + 64);
  hipMalloc(&out, n * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float a = 0, b = 0, t;
  for (int rep = 0; rep < 3; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mem, dim3((n + 255) / 256), dim3(256), 0, 0, n, bytes, len, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&t, e0, e1);
    a = rep ? (t < a ? t : a) : t;
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_reg, dim3((n + 255) / 256), dim3(256), 0, 0, n, len, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&t, e0, e1);
    b = rep ? (t < b ? t : b) : t;
  }
  printf("sha256 1M x 446 B from HBM (k_sha256 path)  %.3f ms  (%.0f GB/s)\n", a, n * len / a / 1e6);
  printf("same compressions, words in registers       %.3f ms\n", b);
  return 0;
}
