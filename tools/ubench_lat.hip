// Latency / throughput of the VALU integer ops used by field_asm.h, at one
// wave per SIMD and at full occupancy: dependent chains vs interleaved
// independent chains.  Informs the list scheduler in tools/gen_field_asm.py.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP8(x) x x x x x x x x
template <int MODE>
__global__ void k(uint64_t *out, uint32_t a, uint32_t b, int iters) {
  uint64_t p0 = threadIdx.x, p1 = p0 + 1, p2 = p0 + 2, p3 = p0 + 3;
  uint32_t c = 0;
  uint64_t s = 0, sc;
  const uint64_t t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) {  // 1 dependent mad chain
      REP8(asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(p0), "=s"(sc) : "v"(a), "v"(b));)
    } else if (MODE == 1) {  // 2 interleaved chains
      REP8(asm volatile("v_mad_u64_u32 %0, %2, %3, %4, %0\n v_mad_u64_u32 %1, %2, %3, %4, %1" : "+v"(p0), "+v"(p1), "=s"(sc) : "v"(a), "v"(b));)
    } else if (MODE == 2) {  // 4 interleaved chains
      REP8(asm volatile("v_mad_u64_u32 %0, %4, %5, %6, %0\n v_mad_u64_u32 %1, %4, %5, %6, %1\n v_mad_u64_u32 %2, %4, %5, %6, %2\n v_mad_u64_u32 %3, %4, %5, %6, %3" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "=s"(sc) : "v"(a), "v"(b));)
    } else if (MODE == 3) {  // dependent addc chain through the carry SGPR, s_nop 1 between links
      REP8(asm volatile("v_add_co_u32_e64 %0, %1, %0, %2\n s_nop 1\n v_addc_co_u32_e64 %0, %1, %0, %2, %1\n s_nop 1" : "+v"(c), "=s"(sc) : "v"(a));)
    } else if (MODE == 4) {  // mad then 2 indep movs then dependent mad (latency 3 slots)
      REP8(asm volatile("v_mad_u64_u32 %0, %2, %3, %4, %0\n v_mov_b32 %1, %3\n v_mov_b32 %1, %4" : "+v"(p0), "=v"(c), "=s"(sc) : "v"(a), "v"(b));)
    } else if (MODE == 5) {  // plain v_add_u32 dependent chain
      REP8(asm volatile("v_add_u32 %0, %0, %1" : "+v"(c) : "v"(a));)
    } else if (MODE == 6) {  // mad + addc pairs (Comba step) with carry use 2 slots later, 3 rotating carries
      REP8(asm volatile(
          "v_mad_u64_u32 %0, %3, %5, %6, %0\n v_mad_u64_u32 %0, %4, %5, %6, %0\n v_addc_co_u32_e64 %1, %3, %1, 0, %3\n v_addc_co_u32_e64 %1, %4, %1, 0, %4"
          : "+v"(p0), "+v"(c), "+v"(p1), "=s"(sc), "=s"(s) : "v"(a), "v"(b));)
    } else if (MODE == 7) {  // v_lshl_add_u64 dependent chain
      REP8(asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(p0) : "v"(p1));)
    }
  }
  const uint64_t t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (p0 + p1 + p2 + p3 + c == 42) out[1 << 20] = 1;
}

template <int MODE>
static void run(const char *name, int per_iter, uint64_t *d, int blocks, int threads) {
  const int iters = 2048;
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, d, 3u, 5u, 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, d, 3u, 5u, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  uint64_t cyc;
  hipMemcpy(&cyc, d, 8, hipMemcpyDeviceToHost);
  const double ninst = (double)iters * 8 * per_iter;
  const double waves = (double)blocks * threads / 64;
  printf("%-48s blocks=%5d cyc/inst(wave0)=%6.2f  chip lane-ops/s=%7.2f T\n", name, blocks, cyc / ninst,
         waves * 64 * ninst / (ms * 1e-3) / 1e12);
}

int main() {
  uint64_t *d;
  hipMalloc(&d, (8 << 20) + 64);
  for (int occ : {1, 4}) {
    const int blocks = 256 * 4 * occ / 4;  // 256-thread blocks = 4 waves -> 1 wave/SIMD per block/CU
    printf("--- %d wave(s) per SIMD ---\n", occ);
    run<0>("mad dependent chain", 1, d, blocks, 256);
    run<1>("mad 2 interleaved chains", 2, d, blocks, 256);
    run<2>("mad 4 interleaved chains", 4, d, blocks, 256);
    run<3>("add_co/addc dependent via SGPR + s_nop 1 (x2)", 4, d, blocks, 256);
    run<4>("mad, 2 movs, dependent mad", 3, d, blocks, 256);
    run<5>("v_add_u32 dependent", 1, d, blocks, 256);
    run<6>("comba step: 2 mad (dep) + 2 addc", 4, d, blocks, 256);
    run<7>("v_lshl_add_u64 dependent", 1, d, blocks, 256);
  }
  return 0;
}
