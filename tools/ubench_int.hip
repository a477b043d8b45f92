// Microbenchmark: VALU integer multiply throughput on gfx950.
// Measures independent-chain throughput of v_mad_u64_u32 (32x32+64 -> 64),
// v_mul_lo_u32 + v_mul_hi_u32, v_mul_u32_u24 and f64 FMA, to price the
// 256-bit modular multiplication used by the verifier.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int CH = 8;  // independent chains per lane

__global__ void k_mad64(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;
  uint64_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      // d = a*b + acc  (v_mad_u64_u32); feed back low half to keep a chain
      acc[c] = (uint64_t)(a + c) * (uint64_t)b + acc[c];
    }
    b += 1;
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullohi(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;
  uint32_t lo[CH], hi[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) { lo[c] = c; hi[c] = threadIdx.x; }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      lo[c] ^= (a + c) * (b ^ lo[c]);
      hi[c] ^= __umulhi(a + c, b ^ hi[c]);
    }
    b += 1;
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= ((uint64_t)hi[c] << 32) | lo[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_u24(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = (seed ^ threadIdx.x) & 0xffffff, b = (seed * 2654435761u + blockIdx.x) & 0xffffff;
  uint32_t lo[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) lo[c] = c + threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) lo[c] = __mul24(a + c, lo[c]) + b;
    b += 1;
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= lo[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_f64(uint64_t* out, uint32_t seed, int iters) {
  double a = 1.0 + 1e-9 * threadIdx.x, b = 0.999999 + 1e-12 * seed;
  double acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_fma(acc[c], b, a);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_addc(uint64_t* out, uint32_t seed, int iters) {
  // 8-limb add-with-carry chain (v_add_co_u32 / v_addc_co_u32)
  uint32_t x[8], y[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) { x[c] = seed + c * 77 + threadIdx.x; y[c] = seed ^ (c * 1234567u); }
  for (int i = 0; i < iters; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) { uint64_t t = (uint64_t)x[c] + y[c] + carry; x[c] = (uint32_t)t; carry = t >> 32; }
    y[0] += (uint32_t)carry;
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int dev = 0; CHECK(hipSetDevice(dev));
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, dev));
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  const int threads = 256, blocks = p.multiProcessorCount * 8, iters = 1 << 14;
  uint64_t* out; CHECK(hipMalloc(&out, sizeof(uint64_t) * threads * blocks));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  struct K { const char* name; void (*f)(uint64_t*, uint32_t, int); double ops_per_iter; };
  K ks[] = {{"v_mad_u64_u32", k_mad64, CH}, {"mul_lo+mul_hi (pairs)", k_mullohi, CH},
            {"v_mul_u32_u24", k_u24, CH}, {"v_fma_f64", k_f64, CH}, {"addc 8-limb chain (adds)", k_addc, 8}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 12345u + rep, iters);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 777u + rep, iters);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      double ops = (double)threads * blocks * iters * k.ops_per_iter;
      if (rep == 2) printf("%-28s %8.3f ms  %8.2f T lane-ops/s\n", k.name, ms, ops / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
