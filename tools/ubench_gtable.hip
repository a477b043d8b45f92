// u1 G from an LDS-staged small-window generator table vs the 26-bit-window
// HBM table the verifier uses (k_verify_g; csrc/geometry.h) — the north
// star's "LDS-staged precomputed base-point tables", settled by measurement
// (DESIGN.md §4).  Timing only: the tables hold arbitrary
// field elements (the XYZZ mixed addition costs the same for any operands
// off its exceptional branches), so no table build is needed.
//
//   hbm26: 10 signed 26-bit windows (T[10][2^25] x 64 B = 21.5 GB in HBM),
//          9 mixed additions per item, one 64-B gather per window;
//   lds6:  43 signed 6-bit windows (T[43][32] x 64 B = 88 KB, staged into
//          LDS per workgroup), 42 mixed additions per item, LDS gathers;
//   lds7:  37 signed 7-bit windows (148 KB: one workgroup per CU).
// Same digit recoding and point addition (point.h gexz_add_ge) in all three.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../babble_amd/csrc/point.h"

#define CHK(x)                                               \
  do {                                                       \
    hipError_t e_ = (x);                                     \
    if (e_ != hipSuccess) {                                  \
      printf("%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                              \
    }                                                        \
  } while (0)

__device__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  return x ^ (x >> 16);
}

__global__ void k_fill(uint32_t *t, uint64_t n_u32) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_u32; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = mix((uint32_t)i ^ (uint32_t)(i >> 32) * 0x9E3779B9u);
}

// u = 256 random bits per item; W-bit signed windows; table rows of 16 words
template <int W, int NWIN, bool LDS, int NT>
__global__ void __launch_bounds__(NT) k_ug(const uint32_t *__restrict__ gtab, uint64_t n_items,
                                            uint32_t *__restrict__ out) {
  constexpr uint32_t ENT = 1u << (W - 1);
  extern __shared__ uint32_t sTab[];
  const uint32_t *tab = gtab;
  if (LDS) {
    for (uint32_t x = threadIdx.x; x < NWIN * ENT * 16; x += blockDim.x) sTab[x] = gtab[x];
    __syncthreads();
    tab = sTab;
  }
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_items; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t u[8];
    for (int k = 0; k < 8; k++) u[k] = mix((uint32_t)i * 8 + k);
    u[7] &= 0x7FFFFFFFu;
    gexz R;
    bool inf = true;
    uint32_t carry = 0;
    for (int j = 0; j < NWIN; j++) {
      uint32_t d = (u[0] & ((1u << W) - 1u)) + carry;
#pragma unroll
      for (int c = 0; c < 7; c++) u[c] = (u[c] >> W) | (u[c + 1] << (32 - W));
      u[7] >>= W;
      carry = d > ENT ? 1u : 0u;
      const bool dneg = carry != 0;
      if (dneg) d = (1u << W) - d;
      if (d) {
        const uint32_t *e = tab + ((uint64_t)j * ENT + (d - 1)) * 16;
        fe x, y;
        for (int k = 0; k < 8; k++) x.v[k] = e[k], y.v[k] = e[8 + k];
        if (dneg) fe_neg(y, y);
        gexz_add_ge(R, inf, x, y);
      }
    }
    uint32_t h = 0;
    for (int k = 0; k < 8; k++) h ^= R.X.v[k] ^ R.ZZ.v[k];
    if (h == 0x12345678u) out[0] = (uint32_t)i;
  }
}

template <int W, int NWIN, bool LDS, int NT>
double run(const uint32_t *tab, uint64_t n_items, uint32_t *out, int blocks) {
  const size_t lds = LDS ? (size_t)NWIN * (1u << (W - 1)) * 64 : 0;
  if (LDS) hipFuncSetAttribute((const void *)k_ug<W, NWIN, LDS, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((k_ug<W, NWIN, LDS, NT>), dim3(blocks), dim3(NT), lds, 0, tab, n_items / 16, out);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_ug<W, NWIN, LDS, NT>), dim3(blocks), dim3(NT), lds, 0, tab, n_items, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  if (hipGetLastError() != hipSuccess) return -1;
  return n_items / (ms * 1e-3);
}

int main() {
  const uint64_t n_items = 1u << 20;
  uint32_t *big, *out;
  const uint64_t big_u32 = 10ull * (1ull << 25) * 16;  // 21.5 GB
  CHK(hipMalloc(&big, big_u32 * 4));
  CHK(hipMalloc(&out, 64));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, big, big_u32);
  CHK(hipDeviceSynchronize());
  // LDS tables: one 1024-thread workgroup per CU (4 waves per SIMD share
  // the CU's copy), grid-stride over the items
  const double hbm = run<26, 10, false, 256>(big, n_items, out, 4096);
  const double l6 = run<6, 43, true, 1024>(big, n_items, out, 256);
  const double l7 = run<7, 37, true, 1024>(big, n_items, out, 256);
  printf("u1 G, 1M items (XYZZ madd, signed windows):\n");
  printf("  hbm26 (10 windows,  9 adds, 21.5 GB HBM table): %8.1f M items/s\n", hbm / 1e6);
  printf("  lds6  (43 windows, 42 adds, 88 KB LDS table):   %8.1f M items/s  (%.2fx slower)\n", l6 / 1e6, hbm / l6);
  printf("  lds7  (37 windows, 36 adds, 148 KB LDS table):  %8.1f M items/s  (%.2fx slower)\n", l7 / 1e6, hbm / l7);
  return 0;
}
