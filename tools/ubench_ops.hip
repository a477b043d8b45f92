// Microbenchmark: per-instruction VALU throughput on gfx950 for the integer
// ops the field arithmetic can be built from.  Each kernel runs a loop of
// 16 independent instances of one instruction (inline asm, so the exact
// opcode is issued), full occupancy; reports wave-instructions per cycle per
// SIMD relative to the measured clock-free rate (T lane-ops/s).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) {                                                                 \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__global__ void __launch_bounds__(256) kop(uint32_t *out, uint32_t seed, int iters) {
  uint32_t a[16];
  uint64_t w[16];
#pragma unroll
  for (int c = 0; c < 16; c++) {
    a[c] = seed + c * 77u + threadIdx.x;
    w[c] = ((uint64_t)a[c] << 7) ^ c;
  }
  const uint32_t b = seed * 2654435761u;
  uint64_t cy[16];
#pragma unroll
  for (int c = 0; c < 16; c++) cy[c] = (uint64_t)(seed >> c) & 0x5555555555555555ull;
  const uint64_t m = 0xF0F0F0F0F0F0F0F0ull ^ seed;
  for (int i = 0; i < iters; i++) {
#define BODY(c)                                                                                      \
  if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));                 \
  if constexpr (OP == 1) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[c]) : "v"(a[c]), "v"(b) : "vcc"); \
  if constexpr (OP == 2) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[c]) : "v"(b));         \
  if constexpr (OP == 3) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(b));          \
  if constexpr (OP == 4) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w[c]) : "v"(w[(c + 1) & 15])); \
  if constexpr (OP == 5) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));              \
  if constexpr (OP == 6) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));              \
  if constexpr (OP == 7) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(w[c]) : "v"(w[(c + 3) & 15]));   \
  if constexpr (OP == 8) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a[c]));                  \
  if constexpr (OP == 9) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[c]) : "v"(b), "v"(a[(c + 1) & 15])); \
  if constexpr (OP == 10) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b), "v"(a[(c + 1) & 15])); \
  if constexpr (OP == 11) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[c]) : "v"(b));                 \
  if constexpr (OP == 12) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[c]));                       \
  if constexpr (OP == 13) asm volatile("v_addc_co_u32_e64 %0, %1, %0, %2, %1" : "+v"(a[c]), "+s"(cy[c]) : "v"(b)); \
  if constexpr (OP == 14) asm volatile("v_mov_b32 %0, %1" : "=v"(a[c]) : "v"(a[(c + 1) & 15]));       \
  if constexpr (OP == 15) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b), "s"(m)); \
  if constexpr (OP == 16) asm volatile("v_sub_co_u32_e64 %0, %1, %0, %2" : "+v"(a[c]), "=s"(cy[c]) : "v"(b)); \
  if constexpr (OP == 17) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(a[c]) : "v"(b) : "vcc"); \
  if constexpr (OP == 18) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b), "v"(a[(c + 1) & 15])); \
  if constexpr (OP >= 19 && OP <= 22) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[c]) : "v"(a[c]), "v"(b) : "vcc"); \
  if constexpr (OP >= 20 && OP <= 22) asm volatile("s_xor_b64 %0, %0, %1" : "+s"(cy[c]) : "s"(m) : "scc");     \
  if constexpr (OP >= 21 && OP <= 22) asm volatile("s_and_b64 %0, %0, %1" : "+s"(cy[(c + 5) & 15]) : "s"(m) : "scc"); \
  if constexpr (OP == 22) asm volatile("s_or_b64 %0, %0, %1\n s_xor_b64 %0, %0, %1" : "+s"(cy[(c + 9) & 15]) : "s"(m) : "scc"); \
  if constexpr (OP == 23) asm volatile("v_addc_co_u32_e64 %0, %1, %0, %2, %1" : "+v"(a[c]), "+s"(cy[c]) : "v"(b)); \
  if constexpr (OP == 23) asm volatile("s_xor_b64 %0, %0, %1\n s_and_b64 %0, %0, %1" : "+s"(cy[(c + 5) & 15]) : "s"(m) : "scc");
    REP16(BODY)
#undef BODY
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) s ^= a[c] ^ (uint32_t)w[c] ^ (uint32_t)(w[c] >> 32) ^ (uint32_t)cy[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
static int run(const char *name, uint32_t *out, int blocks) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int iters = 4096;
  hipLaunchKernelGGL(kop<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kop<OP>, dim3(blocks), dim3(256), 0, 0, out, 2u, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = (double)blocks * 256 * iters * 16;
  // wave-instructions per SIMD per ns, then cycles at 2.4 GHz
  const double wave_instr = ops / 64.0;
  const double per_simd_per_s = wave_instr / 1024.0 / (ms * 1e-3);
  printf("%-20s %8.3f ms  %7.2f T lane-ops/s  %5.2f cycles/wave-instr @2.4GHz\n", name, ms, ops / (ms * 1e-3) / 1e12,
         2.4e9 / per_simd_per_s);
  return 0;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  uint32_t *out;
  const int blocks = p.multiProcessorCount * 8;
  CHECK(hipMalloc(&out, sizeof(uint32_t) * 256 * blocks));
  run<0>("v_add_u32", out, blocks);
  run<1>("v_mad_u64_u32", out, blocks);
  run<2>("v_mad_u32_u24", out, blocks);
  run<3>("v_mul_hi_u32_u24", out, blocks);
  run<4>("v_lshl_add_u64", out, blocks);
  run<5>("v_mul_lo_u32", out, blocks);
  run<6>("v_mul_hi_u32", out, blocks);
  run<7>("v_fma_f64", out, blocks);
  run<8>("v_alignbit_b32", out, blocks);
  run<9>("v_bitop3_b32", out, blocks);
  run<10>("v_add3_u32", out, blocks);
  run<11>("v_xor_b32", out, blocks);
  run<12>("v_lshrrev_b32", out, blocks);
  run<13>("v_addc_co_u32_e64", out, blocks);
  run<14>("v_mov_b32", out, blocks);
  run<15>("v_cndmask_b32_e64", out, blocks);
  run<16>("v_sub_co_u32_e64", out, blocks);
  run<17>("v_add_co_u32_e32", out, blocks);
  run<18>("v_perm_b32", out, blocks);
  // SALU beside VALU (per 16 mads: 0 / 16 / 32 / 64 independent 64-bit SALU
  // ops; per 16 addc: 32): whether the scalar ops cost VALU issue slots
  run<19>("mad + 0 salu", out, blocks);
  run<20>("mad + 1 salu", out, blocks);
  run<21>("mad + 2 salu", out, blocks);
  run<22>("mad + 4 salu", out, blocks);
  run<23>("addc + 2 salu", out, blocks);
  return 0;
}
