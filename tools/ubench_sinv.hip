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

// Jump divsteps: a table of every 5-divstep transition, indexed by eta
// (clamped to [-5, 5]: beyond it the next 5 steps take the same decisions),
// f mod 32 (odd) and g mod 32; entry = int8 (u, v, q, r) with
// (f5, g5) 2^5 = (u f + v g, q f + r g), and eta5 = s eta + c (s = +-1).
// 11 x 16 x 32 entries of 8 bytes = 45 KB of LDS, built by the workgroup.
constexpr int kJumpK = 5;
constexpr int kJumpEntries = (2 * kJumpK + 1) * 16 * 32;
__device__ __forceinline__ uint2 jump_entry(int idx) {
  int eta = idx / 512 - kJumpK;
  uint32_t f = (((idx >> 5) & 15u) << 1) | 1u, g = idx & 31u;
  int u = 1, v = 0, q = 0, r = 1, sgn = 1, c = 0;
  int32_t fi = (int32_t)f, gi = (int32_t)g;
  for (int i = 0; i < kJumpK; i++) {
    if (gi & 1) {
      if (eta < 0) {
        int t;
        eta = -eta, sgn = -sgn, c = -c;
        t = fi, fi = gi, gi = -t;
        t = u, u = q, q = -t;
        t = v, v = r, r = -t;
      }
      gi += fi, q += u, r += v;
    }
    gi >>= 1, u *= 2, v *= 2, eta -= 1, c -= 1;
  }
  const uint32_t lo = (uint32_t)(uint8_t)u | ((uint32_t)(uint8_t)v << 8) | ((uint32_t)(uint8_t)q << 16) |
                      ((uint32_t)(uint8_t)r << 24);
  const uint32_t hi = (uint32_t)(uint8_t)c | ((sgn < 0 ? 1u : 0u) << 8);
  return make_uint2(lo, hi);
}

__device__ __forceinline__ int32_t divsteps_30_jump(int32_t eta, uint32_t f0, uint32_t g0, int32_t t[4],
                                                    const uint2 *tab) {
  int32_t U = 1, V = 0, Q = 0, R = 1;
  int32_t f = (int32_t)f0, g = (int32_t)g0;
#pragma unroll
  for (int j = 0; j < 30 / kJumpK; j++) {
    const int ec = eta < -kJumpK ? -kJumpK : (eta > kJumpK ? kJumpK : eta);
    const int idx = ((ec + kJumpK) << 9) | ((((uint32_t)f >> 1) & 15u) << 5) | ((uint32_t)g & 31u);
    const uint2 e = tab[idx];
    const uint32_t lo = __builtin_amdgcn_readfirstlane(e.x), hi = __builtin_amdgcn_readfirstlane(e.y);
    const int32_t u = (int8_t)lo, v = (int8_t)(lo >> 8), q = (int8_t)(lo >> 16), r = (int8_t)(lo >> 24);
    const int32_t c = (int8_t)hi;
    eta = ((hi >> 8) & 1u ? -eta : eta) + c;
    const int32_t nf = (int32_t)((uint32_t)u * (uint32_t)f + (uint32_t)v * (uint32_t)g) >> kJumpK;
    const int32_t ng = (int32_t)((uint32_t)q * (uint32_t)f + (uint32_t)r * (uint32_t)g) >> kJumpK;
    f = nf, g = ng;
    const int32_t nU = u * U + v * Q, nV = u * V + v * R, nQ = q * U + r * Q, nR = q * V + r * R;
    U = nU, V = nV, Q = nQ, R = nR;
  }
  t[0] = U;
  t[1] = V;
  t[2] = Q;
  t[3] = R;
  return eta;
}

// the inversion with the divsteps variant D (0: modinv.h, 1: selects, 2: jump
// table, 3: selects on the VECTOR unit: the input is moved to VGPRs first, so
// every value derived from it (f, g, eta, the matrices, d, e) is VALU work —
// 64-bit products are single v_mad_i64_i32 — and the loop exit is an EXEC
// test instead of a scalar branch on SALU results)
template <int D>
__device__ __forceinline__ void modinv_variant(uint32_t r[8], const uint32_t x_in[8], const modinfo30 &mi,
                                               const uint2 *tab) {
  uint32_t x[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x[i] = x_in[i];
    if (D == 3) asm volatile("v_mov_b32 %0, %1" : "=v"(x[i]) : "v"(x_in[i]));
  }
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
    eta = D == 2   ? divsteps_30_jump(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t, tab)
          : D >= 1 ? divsteps_30_sel(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t)
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
__global__ void __launch_bounds__(256) k_variant(const uint32_t *__restrict__ xs, int reps, uint32_t *__restrict__ out,
                                                 uint64_t *__restrict__ clk) {
  __shared__ uint2 tab[kJumpEntries];
  const uint64_t b0 = __builtin_amdgcn_s_memtime();
  if (D == 2) {
    for (int i = threadIdx.x; i < kJumpEntries; i += blockDim.x) tab[i] = jump_entry(i);
    __syncthreads();
  }
  if (threadIdx.x == 0) clk[4] = __builtin_amdgcn_s_memtime() - b0;
  if (threadIdx.x != 0) return;
  modinfo30 mi;
  modinfo_n(mi);
  uint64_t c_all = 0;
  for (int k = 0; k < reps; k++) {
    uint32_t x[8], r[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = __builtin_amdgcn_readfirstlane(xs[8 * k + i]);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    modinv_variant<D>(r, x, mi, tab);
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
    hipLaunchKernelGGL(k_variant<0>, dim3(1), dim3(256), 0, 0, dx, reps, dout2, dclk2);
    hipMemcpy(r0, dout2, sizeof r0, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k_variant<1>, dim3(1), dim3(256), 0, 0, dx, reps, dout2, dclk2);
    hipMemcpy(r1, dout2, sizeof r1, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k_variant<2>, dim3(1), dim3(256), 0, 0, dx, reps, dout2, dclk2);
  }
  uint32_t r2[8 * reps];
  hipMemcpy(r2, dout2, sizeof r2, hipMemcpyDeviceToHost);
  uint32_t r3[8 * reps];
  for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k_variant<3>, dim3(1), dim3(256), 0, 0, dx, reps, dout2, dclk2);
  hipMemcpy(r3, dout2, sizeof r3, hipMemcpyDeviceToHost);
  hipMemcpy(c2, dclk2, 64, hipMemcpyDeviceToHost);
  int diff = 0, diff2 = 0, diff3 = 0;
  for (int i = 0; i < 8 * reps; i++) diff += r0[i] != r1[i], diff2 += r0[i] != r2[i], diff3 += r0[i] != r3[i];
  printf("modinv_var per inversion, selects on the VECTOR unit: %.0f clocks (%d differing words)\n",
         (double)c2[3] / reps, diff3);
  printf("modinv_var per inversion: divsteps_30_var %.0f clocks, divsteps with select swap %.0f clocks "
         "(%d differing words), jump table %.0f clocks (%d differing words; table build %.0f clocks)\n",
         (double)c2[0] / reps, (double)c2[1] / reps, diff, (double)c2[2] / reps, diff2, (double)c2[4]);
  printf("modinv_var per inversion (shader clocks): total %.0f  divsteps %.0f  update_de %.0f  update_fg %.0f  "
         "normalize+convert %.0f  outer iterations %.2f\n",
         (double)c[0] / reps, (double)c[1] / reps, (double)c[2] / reps, (double)c[3] / reps, (double)c[4] / reps,
         (double)c[5] / reps);
  printf("sinv_one (sc_inverse_var + Montgomery product, as k_small) per inversion: %.0f clocks\n",
         (double)c[6] / reps);
  return 0;
}
