// FETCH_SIZE calibration for the verify kernels' access pattern (VERDICT r4
// #3).  The guide calibrates rocprofv3's FETCH_SIZE only for 16-B-per-lane
// streaming reads (it reports half the bytes: 128-B requests tallied at
// 64 B).  k_verify_g / k_verify_q instead gather one random 64-B table entry
// per lane per window (fe_load4 x 2: four dwordx4 loads of one 64-B-aligned
// entry, verify_core.h g_table_add / key_table_add).  Three kernels over a
// 4 GiB table (far past the 256 MiB Infinity Cache), each moving a known
// number of algorithmic bytes:
//   stream   16 B per lane, coalesced (the guide's reference pattern)
//   gather64 random 64-B entries, 64-B aligned (the verify kernels)
//   gather128 random 128-B lines (two adjacent entries per lane)
// The host prints each kernel's algorithmic bytes and HIP-event time; the
// PMC passes (tools/gpu_gather_pmc.sh) read FETCH_SIZE / TCC_EA0_RDREQ per
// dispatch, and tools/gather_calib.py divides.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x)                                               \
  do {                                                       \
    hipError_t e_ = (x);                                     \
    if (e_ != hipSuccess) {                                  \
      printf("%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                              \
    }                                                        \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  return x ^ (x >> 16);
}

__global__ void k_fill(uint4 *t, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = make_uint4((uint32_t)i, mix((uint32_t)i), (uint32_t)(i >> 32), 7u);
}

// every lane reads 16 B per step, consecutive lanes consecutive 16 B
__global__ void __launch_bounds__(256) k_stream(const uint4 *__restrict__ t, uint64_t n16, uint32_t *__restrict__ out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = t[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// L random entries of ENT_U4 x 16 B per lane (ENT_U4 = 4: 64 B; 8: 128 B)
template <int ENT_U4>
__global__ void __launch_bounds__(256) k_gather(const uint4 *__restrict__ t, uint64_t n_ent, int L,
                                                 uint32_t *__restrict__ out) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0, h = mix(tid * 0x9E3779B9u + 1u);
  for (int j = 0; j < L; j++) {
    h = mix(h + (uint32_t)j);
    const uint64_t e = ((uint64_t)h * n_ent) >> 32;
    const uint4 *p = t + e * ENT_U4;
#pragma unroll
    for (int k = 0; k < ENT_U4; k++) {
      const uint4 v = p[k];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  out[tid] = acc;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const uint64_t bytes = 4ull << 30;  // 4 GiB table
  const uint64_t n16 = bytes / 16;
  uint4 *t;
  uint32_t *out;
  const int blocks = prop.multiProcessorCount * 16, nt = 256, L = 32;
  CHK(hipMalloc(&t, bytes));
  CHK(hipMalloc(&out, sizeof(uint32_t) * (uint64_t)blocks * nt));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, t, n16);
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const uint64_t lanes = (uint64_t)blocks * nt;
  for (int rep = 0; rep < 2; rep++) {  // rep 0 warms up; the PMC passes see both
    float ms;
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(nt), 0, 0, t, n16, out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("stream    rep %d bytes %llu ms %.4f GB/s %.1f\n", rep, (unsigned long long)bytes, ms, bytes / (ms * 1e6));
    const uint64_t g64 = lanes * L * 64;
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_gather<4>, dim3(blocks), dim3(nt), 0, 0, t, bytes / 64, L, out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("gather64  rep %d bytes %llu ms %.4f GB/s %.1f\n", rep, (unsigned long long)g64, ms, g64 / (ms * 1e6));
    const uint64_t g128 = lanes * L * 128;
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_gather<8>, dim3(blocks), dim3(nt), 0, 0, t, bytes / 128, L, out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("gather128 rep %d bytes %llu ms %.4f GB/s %.1f\n", rep, (unsigned long long)g128, ms, g128 / (ms * 1e6));
  }
  return 0;
}
