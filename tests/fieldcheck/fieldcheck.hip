// fieldcheck.hip — TEST INFRASTRUCTURE: runs the device field / scalar
// primitives of babble_amd/csrc/field.h (the generated gfx950 inline asm of
// field_asm.h on the device) over operand arrays supplied by the test, so
// tests/test_gpu_field.py can compare every result with Python integers
// (mod p and Montgomery mod N).  This checks the real ISA semantics of the
// hand-scheduled programs (carry-outs, hazards, rare blocks), which the
// generator's own interpreter (tests/test_field_asm.py) cannot.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../babble_amd/csrc/field.h"
#include "../../babble_amd/csrc/point.h"
#include "../../babble_amd/csrc/verify_core.h"
#include "../../babble_amd/csrc/coop.h"

// OP_ZSSM + k: component k of the zipped (x^2, y^2, x y) program;
// OP_ZSSS + k: component k of the zipped (x^2, y^2, (x ^ y)^2) program
// (field_asm.h gen_zip, used by the key-table doubling chain).
// OP_CNEG: fe_cneg_canon(x, y.v[0] & 1) (branch-free conditional negate of
// a canonical element, the verify kernels' signed-digit lookup).
enum { OP_MUL = 0, OP_SQR = 1, OP_ADD = 2, OP_SUB = 3, OP_MONT = 4, OP_INV = 5, OP_ZSSM = 6, OP_ZSSS = 9,
       OP_CNEG = 12, OP_LAST = 12 };

__global__ void __launch_bounds__(256) k_field(int op, uint32_t n, const uint32_t *__restrict__ a,
                                               const uint32_t *__restrict__ b, uint32_t *__restrict__ r) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe x, y, z;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    x.v[k] = a[8 * (uint64_t)i + k];
    y.v[k] = b[8 * (uint64_t)i + k];
  }
  switch (op) {
    case OP_MUL: fe_mul(z, x, y); break;
    case OP_SQR: fe_sqr(z, x); break;
    case OP_ADD: fe_add(z, x, y); break;
    case OP_SUB: fe_sub(z, x, y); break;
    case OP_MONT: {
      sc p, q, s;
#pragma unroll
      for (int k = 0; k < 8; k++) { p.v[k] = x.v[k]; q.v[k] = y.v[k]; }
      sc_mont(s, p, q);
#pragma unroll
      for (int k = 0; k < 8; k++) z.v[k] = s.v[k];
      break;
    }
    case OP_INV: fe_inv_var(z, x); break;
    case OP_CNEG: z = x; fe_cneg_canon(z, (y.v[0] & 1u) != 0); break;
    default: {
      fe w, o[3];
#pragma unroll
      for (int k = 0; k < 8; k++) w.v[k] = x.v[k] ^ y.v[k];
#if defined(__HIP_DEVICE_COMPILE__)
      if (op < OP_ZSSS) fe_sqr_sqr_mul_zip_asm(o[0], x, o[1], y, o[2], x, y);
      else fe_sqr_sqr_sqr_zip_asm(o[0], x, o[1], y, o[2], w);
#endif
      z = o[(op - OP_ZSSM) % 3];
      break;
    }
  }
#pragma unroll
  for (int k = 0; k < 8; k++) r[8 * (uint64_t)i + k] = z.v[k];
}

// Host entry: n operand pairs (8 little-endian u32 limbs each).  Returns 0,
// or a negative HIP error code.  Synchronous.
extern "C" int fc_run(int op, uint32_t n, const uint32_t *a, const uint32_t *b, uint32_t *r) {
  if (op < OP_MUL || op > OP_LAST) return -1000;
  uint32_t *da = nullptr, *db = nullptr, *dr = nullptr;
  const size_t bytes = (size_t)n * 32;
  hipError_t e = hipMalloc(&da, bytes ? bytes : 32);
  if (e == hipSuccess) e = hipMalloc(&db, bytes ? bytes : 32);
  if (e == hipSuccess) e = hipMalloc(&dr, bytes ? bytes : 32);
  if (e == hipSuccess && n) e = hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) e = hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) {
    hipLaunchKernelGGL(k_field, dim3((n + 255) / 256), dim3(256), 0, 0, op, n, da, db, dr);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess && n) e = hipMemcpy(r, dr, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dr);
  return e == hipSuccess ? 0 : -(int)e;
}

// XYZZ mixed additions of the verify kernels (point.h gexz_add_ge and the
// zipped gexz_add_ge_lat), exceptional cases included: acc = 33 words per
// lane (X, Y, ZZ, ZZZ, inf flag), pts = 16 words (affine x2, y2); out = the
// accumulator after acc += pt (P == Q doubles, P == -Q gives the
// identity, the identity takes the point).
__global__ void __launch_bounds__(256) k_xyzz(int lat, uint32_t n, const uint32_t *__restrict__ acc,
                                              const uint32_t *__restrict__ pts, uint32_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  gexz R;
  fe x, y;
  const uint32_t *a = acc + 33 * (uint64_t)i, *q = pts + 16 * (uint64_t)i;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    R.X.v[k] = a[k], R.Y.v[k] = a[8 + k], R.ZZ.v[k] = a[16 + k], R.ZZZ.v[k] = a[24 + k];
    x.v[k] = q[k], y.v[k] = q[8 + k];
  }
  bool inf = a[32] != 0;
  if (lat) gexz_add_ge_lat(R, inf, x, y);
  else gexz_add_ge(R, inf, x, y);
  uint32_t *o = out + 33 * (uint64_t)i;
#pragma unroll
  for (int k = 0; k < 8; k++) o[k] = R.X.v[k], o[8 + k] = R.Y.v[k], o[16 + k] = R.ZZ.v[k], o[24 + k] = R.ZZZ.v[k];
  o[32] = inf ? 1u : 0u;
}

extern "C" int fc_xyzz(int lat, uint32_t n, const uint32_t *acc, const uint32_t *pts, uint32_t *out) {
  uint32_t *da = nullptr, *dp = nullptr, *dr = nullptr;
  const size_t ab = (size_t)(n ? n : 1) * 33 * 4, pb = (size_t)(n ? n : 1) * 16 * 4;
  hipError_t e = hipMalloc(&da, ab);
  if (e == hipSuccess) e = hipMalloc(&dp, pb);
  if (e == hipSuccess) e = hipMalloc(&dr, ab);
  if (e == hipSuccess && n) e = hipMemcpy(da, acc, ab, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) e = hipMemcpy(dp, pts, pb, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) {
    hipLaunchKernelGGL(k_xyzz, dim3((n + 255) / 256), dim3(256), 0, 0, lat, n, da, dp, dr);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess && n) e = hipMemcpy(out, dr, ab, hipMemcpyDeviceToHost);
  (void)hipFree(da);
  (void)hipFree(dp);
  (void)hipFree(dr);
  return e == hipSuccess ? 0 : -(int)e;
}

// The wave-cooperative XYZZ point ops of k_small's cold path (coop.h), one
// wave per case: out[74 i ..] = acc + pt (33 words: X, Y, ZZ, ZZZ, identity
// flag; add_xyzz), 2 pt (33 words; dbl_xyzz) and the doubling's beta X (8
// words).  acc and pt are XYZZ (33 words each), pt finite.
__global__ void __launch_bounds__(64) k_coop_xyzz(uint32_t n, const uint32_t *acc, const uint32_t *pts, uint32_t *out) {
  const uint32_t b = blockIdx.x;
  if (b >= n) return;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t c = coop::pos(), lane = __lane_id();
  const uint32_t *a = acc + 33 * (uint64_t)b, *q = pts + 33 * (uint64_t)b;
  const auto ld = [&](const uint32_t *p, int o) { return c < 8 ? p[o + c] : 0u; };
  uint32_t X1 = ld(a, 0), Y1 = ld(a, 8), ZZ1 = ld(a, 16), ZZZ1 = ld(a, 24);
  bool inf = a[32] != 0;
  const uint32_t X2 = ld(q, 0), Y2 = ld(q, 8), ZZ2 = ld(q, 16), ZZZ2 = ld(q, 24);
  coop::add_xyzz(X1, Y1, ZZ1, ZZZ1, inf, X2, Y2, ZZ2, ZZZ2);
  uint32_t DX = X2, DY = Y2, DZZ = ZZ2, DZZZ = ZZZ2, BX;
  coop::dbl_xyzz(DX, DY, DZZ, DZZZ, BX);
  uint32_t *o = out + 74 * (uint64_t)b;
  if (lane < 8) {
    o[lane] = X1, o[8 + lane] = Y1, o[16 + lane] = ZZ1, o[24 + lane] = ZZZ1;
    o[33 + lane] = DX, o[41 + lane] = DY, o[49 + lane] = DZZ, o[57 + lane] = DZZZ;
    o[66 + lane] = BX;
  }
  if (lane == 0) o[32] = inf ? 1u : 0u, o[65] = 0u;
#endif
}

extern "C" int fc_coop_xyzz(uint32_t n, const uint32_t *acc, const uint32_t *pts, uint32_t *out) {
  uint32_t *da = nullptr, *dp = nullptr, *dr = nullptr;
  const size_t ab = (size_t)(n ? n : 1) * 33 * 4, ob = (size_t)(n ? n : 1) * 74 * 4;
  hipError_t e = hipMalloc(&da, ab);
  if (e == hipSuccess) e = hipMalloc(&dp, ab);
  if (e == hipSuccess) e = hipMalloc(&dr, ob);
  if (e == hipSuccess && n) e = hipMemcpy(da, acc, ab, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) e = hipMemcpy(dp, pts, ab, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) {
    hipLaunchKernelGGL(k_coop_xyzz, dim3(n), dim3(64), 0, 0, n, da, dp, dr);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess && n) e = hipMemcpy(out, dr, ob, hipMemcpyDeviceToHost);
  (void)hipFree(da);
  (void)hipFree(dp);
  (void)hipFree(dr);
  return e == hipSuccess ? 0 : -(int)e;
}

// coop.h's products and reductions on hardware, four cases a wave (one a
// DPP row): op 0 mul(a, b), 1 norm(a + (M4 - b)), 2 norm(a + 8 (M4 - b)),
// 3 norm(3 a); a, b: n x 8 words, out: n x 8 words (NORMAL, < 2^256).
__global__ void __launch_bounds__(64) k_coop_ops(int op, uint32_t n, const uint32_t *a, const uint32_t *b,
                                                 uint32_t *out) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t c = coop::pos(), i = 4 * blockIdx.x + coop::row();
  const bool live = i < n;  // (every lane runs the row code: the DPP reads and ballots are wave-wide)
  const uint32_t x = live && c < 8 ? a[8 * (uint64_t)i + c] : 0u, y = live && c < 8 ? b[8 * (uint64_t)i + c] : 0u;
  uint32_t r;
  if (op == 0) r = coop::mul(x, y);
  else if (op == 1) r = coop::norm((uint64_t)x + coop::negw(y));
  else if (op == 2) r = coop::norm((uint64_t)x + 8ull * coop::negw(y));
  else r = coop::norm(3ull * x);
  if (live && c < 8) out[8 * (uint64_t)i + c] = r;
#endif
}

extern "C" int fc_coop_ops(int op, uint32_t n, const uint32_t *a, const uint32_t *b, uint32_t *out) {
  uint32_t *da = nullptr, *db = nullptr, *dr = nullptr;
  const size_t bytes = (size_t)(n ? n : 1) * 32;
  hipError_t e = hipMalloc(&da, bytes);
  if (e == hipSuccess) e = hipMalloc(&db, bytes);
  if (e == hipSuccess) e = hipMalloc(&dr, bytes);
  if (e == hipSuccess && n) e = hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) e = hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) {
    hipLaunchKernelGGL(k_coop_ops, dim3((n + 3) / 4), dim3(64), 0, 0, op, n, da, db, dr);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess && n) e = hipMemcpy(out, dr, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dr);
  return e == hipSuccess ? 0 : -(int)e;
}

// Key-table base chains B_j = 2^(w j) Q (j < nwin) of n affine points
// (16 words each: x, y limbs), per lane (verify_core.h table_bases_one, the
// zipped doubling) or wave-cooperative (coop.h: one wave per point, the
// doubling's products spread over the DPP rows); out: n x nwin x 24 words
// (X, Y, Z).  Both must agree mod p (same formulas).
__global__ void __launch_bounds__(64) k_bases_lane(uint32_t n, const uint32_t *xy, uint32_t *out, int w, int nwin) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < n) table_bases_one<true>(b, xy, out, w, nwin);
}
__global__ void __launch_bounds__(64) k_bases_coop(uint32_t n, const uint32_t *xy, uint32_t *out, int w, int nwin) {
  const uint32_t b = blockIdx.x;
  if (b >= n) return;
#if defined(__HIP_DEVICE_COMPILE__)
  coop_bases_one(b, xy, out, w, nwin);
#endif
}

extern "C" int fc_bases(int coop, uint32_t n, const uint32_t *xy, uint32_t *out, int w, int nwin, float *ms) {
  uint32_t *dxy = nullptr, *dout = nullptr;
  const size_t ob = (size_t)n * nwin * 24 * 4;
  hipError_t e = hipMalloc(&dxy, (size_t)n * 64 + 64);
  if (e == hipSuccess) e = hipMalloc(&dout, ob + 64);
  if (e == hipSuccess) e = hipMemcpy(dxy, xy, (size_t)n * 64, hipMemcpyHostToDevice);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  for (int rep = 0; rep < 2 && e == hipSuccess; rep++) {  // the second run is timed
    (void)hipEventRecord(e0, 0);
    if (coop)
      hipLaunchKernelGGL(k_bases_coop, dim3(n), dim3(64), 0, 0, n, dxy, dout, w, nwin);
    else
      hipLaunchKernelGGL(k_bases_lane, dim3((n + 63) / 64), dim3(64), 0, 0, n, dxy, dout, w, nwin);
    e = hipGetLastError();
    (void)hipEventRecord(e1, 0);
    if (e == hipSuccess) e = hipDeviceSynchronize();
  }
  if (e == hipSuccess && ms) e = hipEventElapsedTime(ms, e0, e1);
  if (e == hipSuccess) e = hipMemcpy(out, dout, ob, hipMemcpyDeviceToHost);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipFree(dxy);
  (void)hipFree(dout);
  return e == hipSuccess ? 0 : -(int)e;
}
