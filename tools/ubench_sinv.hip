// Where k_small's s^-1 goes (modinv.h, the Bernstein-Yang inversion of one
// item; its values are wave-uniform in k_small, so the compiler runs it on
// the scalar unit).  One workgroup, wave 0 lane 0 inverts `reps` scalars
// back to back with s_memtime around each part: the divsteps batches, the
// (d, e) updates, the (f, g) updates, the normalisation.  Prints shader
// clocks per inversion (average over reps; the inner stamps add their own
// latency, so k_sinv_one times the inversion whole as well).  Correctness is
// tests/test_gpu_field.py's.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_sinv tools/ubench_sinv.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../babble_amd/csrc/field.h"

// divsteps_30_var with the eta < 0 swap as selects instead of a branch
// (candidate; same results)
__device__ __forceinline__ int32_t divsteps_30_sel(int32_t eta, uint32_t f0, uint32_t g0, int32_t t[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1, f = f0, g = g0;
  int i = 30;
  for (;;) {
    const int zeros = ctz32(g | (0xFFFFFFFFu << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    const bool sw = eta < 0;
    const uint32_t nf = sw ? g : f, ng = sw ? 0u - f : g;
    const uint32_t nu = sw ? q : u, nq = sw ? 0u - u : q;
    const uint32_t nv = sw ? r : v, nr = sw ? 0u - v : r;
    eta = sw ? -eta : eta;
    f = nf, g = ng, u = nu, q = nq, v = nv, r = nr;
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xFFFFFFFFu >> (32 - limit)) & 63u;
    const uint32_t w = (f * g * (f * f - 2u)) & m;
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t[0] = (int32_t)u;
  t[1] = (int32_t)v;
  t[2] = (int32_t)q;
  t[3] = (int32_t)r;
  return eta;
}

// the inversion with the divsteps variant D (0: modinv.h, 1: selects)
template <int D>
__device__ __forceinline__ void modinv_variant(uint32_t r[8], const uint32_t x[8], const modinfo30 &mi) {
  s30 d, e, f, g;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    d.v[i] = 0;
    e.v[i] = 0;
    f.v[i] = mi.m[i];
  }
  e.v[0] = 1;
  s30_from_u256(g, x);
  int32_t eta = -1;
  for (;;) {
    int32_t t[4];
    eta = D ? divsteps_30_sel(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t)
            : divsteps_30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de_30(d, e, t, mi);
    update_fg_30(f, g, t);
    int32_t z = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) z |= g.v[i];
    if (z == 0) break;
  }
  normalize_30(d, f.v[8] >> 31, mi);
  s30_to_u256(r, d);
}

template <int D>
__global__ void __launch_bounds__(64) k_variant(const uint32_t *__restrict__ xs, int reps, uint32_t *__restrict__ out,
                                                uint64_t *__restrict__ clk) {
  if (threadIdx.x != 0) return;
  modinfo30 mi;
  modinfo_n(mi);
  uint64_t c_all = 0;
  for (int k = 0; k < reps; k++) {
    uint32_t x[8], r[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = __builtin_amdgcn_readfirstlane(xs[8 * k + i]);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    modinv_variant<D>(r, x, mi);
    c_all += __builtin_amdgcn_s_memtime() - t0;
#pragma unroll
    for (int i = 0; i < 8; i++) out[8 * k + i] = r[i];
  }
  clk[D] = c_all;
}

__global__ void __launch_bounds__(64) k_sinv_parts(const uint32_t *__restrict__ xs, int reps,
                                                    uint32_t *__restrict__ out, uint64_t *__restrict__ clk) {
  if (threadIdx.x != 0) return;
  uint64_t c_div = 0, c_de = 0, c_fg = 0, c_norm = 0, c_all = 0, iters = 0;
  modinfo30 mi;
  modinfo_n(mi);
  for (int k = 0; k < reps; k++) {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = __builtin_amdgcn_readfirstlane(xs[8 * k + i]);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    s30 d, e, f, g;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      d.v[i] = 0;
      e.v[i] = 0;
      f.v[i] = mi.m[i];
    }
    e.v[0] = 1;
    s30_from_u256(g, x);
    int32_t eta = -1;
    for (;;) {
      int32_t t[4];
      const uint64_t a = __builtin_amdgcn_s_memtime();
      eta = divsteps_30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
      const uint64_t b = __builtin_amdgcn_s_memtime();
      update_de_30(d, e, t, mi);
      const uint64_t c = __builtin_amdgcn_s_memtime();
      update_fg_30(f, g, t);
      const uint64_t dd = __builtin_amdgcn_s_memtime();
      c_div += b - a;
      c_de += c - b;
      c_fg += dd - c;
      iters++;
      int32_t z = 0;
#pragma unroll
      for (int i = 0; i < 9; i++) z |= g.v[i];
      if (z == 0) break;
    }
    const uint64_t n0 = __builtin_amdgcn_s_memtime();
    normalize_30(d, f.v[8] >> 31, mi);
    uint32_t r[8];
    s30_to_u256(r, d);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    c_norm += t1 - n0;
    c_all += t1 - t0;
#pragma unroll
    for (int i = 0; i < 8; i++) out[8 * k + i] = r[i];
  }
  clk[0] = c_all;
  clk[1] = c_div;
  clk[2] = c_de;
  clk[3] = c_fg;
  clk[4] = c_norm;
  clk[5] = iters;
}

// the same inversion as k_small calls it (sinv_one: sc_inverse_var + one
// Montgomery product), timed whole
__global__ void __launch_bounds__(64) k_sinv_one(const uint32_t *__restrict__ xs, int reps, uint32_t *__restrict__ out,
                                                  uint64_t *__restrict__ clk) {
  if (threadIdx.x != 0) return;
  uint64_t c_all = 0;
  for (int k = 0; k < reps; k++) {
    sc s, w, t, one;
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = __builtin_amdgcn_readfirstlane(xs[8 * k + i]), one.v[i] = i == 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    sc_inverse_var(t, s);
    sc_mont(w, t, one);
    c_all += __builtin_amdgcn_s_memtime() - t0;
#pragma unroll
    for (int i = 0; i < 8; i++) out[8 * k + i] ^= w.v[i];
  }
  clk[6] = c_all;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int reps = 64;
  uint32_t hx[8 * reps];
  uint64_t st = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < 8 * reps; i++) {
    st ^= st << 13, st ^= st >> 7, st ^= st << 17;
    hx[i] = (uint32_t)st;
  }
  for (int k = 0; k < reps; k++) hx[8 * k + 7] &= 0x7FFFFFFFu;  // < N
  uint32_t *dx, *dout;
  uint64_t *dclk;
  hipMalloc(&dx, sizeof hx);
  hipMalloc(&dout, sizeof hx);
  hipMalloc(&dclk, 8 * 8);
  hipMemcpy(dx, hx, sizeof hx, hipMemcpyHostToDevice);
  hipMemset(dclk, 0, 64);
  hipLaunchKernelGGL(k_sinv_parts, dim3(1), dim3(64), 0, 0, dx, reps, dout, dclk);
  hipLaunchKernelGGL(k_sinv_parts, dim3(1), dim3(64), 0, 0, dx, reps, dout, dclk);
  hipLaunchKernelGGL(k_sinv_one, dim3(1), dim3(64), 0, 0, dx, reps, dout, dclk);
  uint64_t c[8];
  uint32_t ho[8 * reps];
  hipMemcpy(c, dclk, 64, hipMemcpyDeviceToHost);
  hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
  uint64_t *dclk2;
  uint32_t *dout2;
  hipMalloc(&dclk2, 64);
  hipMalloc(&dout2, sizeof hx);
  uint64_t c2[8];
  uint32_t r0[8 * reps], r1[8 * reps];
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_variant<0>, dim3(1), dim3(64), 0, 0, dx, reps, dout2, dclk2);
    hipMemcpy(r0, dout2, sizeof r0, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k_variant<1>, dim3(1), dim3(64), 0, 0, dx, reps, dout2, dclk2);
    hipMemcpy(r1, dout2, sizeof r1, hipMemcpyDeviceToHost);
  }
  hipMemcpy(c2, dclk2, 64, hipMemcpyDeviceToHost);
  int diff = 0;
  for (int i = 0; i < 8 * reps; i++) diff += r0[i] != r1[i];
  printf("modinv_var per inversion: divsteps_30_var %.0f clocks, divsteps with select swap %.0f clocks "
         "(%d differing words)\n", (double)c2[0] / reps, (double)c2[1] / reps, diff);
  printf("modinv_var per inversion (shader clocks): total %.0f  divsteps %.0f  update_de %.0f  update_fg %.0f  "
         "normalize+convert %.0f  outer iterations %.2f\n",
         (double)c[0] / reps, (double)c[1] / reps, (double)c[2] / reps, (double)c[3] / reps, (double)c[4] / reps,
         (double)c[5] / reps);
  printf("sinv_one (sc_inverse_var + Montgomery product, as k_small) per inversion: %.0f clocks\n",
         (double)c[6] / reps);
  return 0;
}
