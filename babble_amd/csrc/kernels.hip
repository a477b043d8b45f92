// kernels.hip — gfx950 kernels of the batch verifier (per-unit work lives in
// verify_core.h).
//
// Pipeline for one batch (bv_api.cpp drives it; two streams):
//   main stream                               keys stream
//   k_key_decode  (Unmarshal, public_key.go:14)
//        |--------- fork ------------------>  k_table_bases  B_j = 2^(8j) Q
//   k_sha256      (crypto.SHA256, hash.go:8)  k_table_fill<8> d * B_j, affine
//   k_scalar_prep (batched s^-1; u1, u2)            |
//   k_verify_g    (R_G = u1 G, 16 adds from         |
//                  the 64 MiB G table)              |
//        |<-------- join ------------------------- -+
//   k_verify_q    (R = R_G + u2 Q, 32 adds from the key's table; decision
//                  table; x(R) mod N == r; status + __ballot accept bits)
// k_verify_generic replaces g/q when keys carry too few items for a table.
// The G table (k_table_bases + k_table_fill<16>) is built once per context.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "verify_core.h"

__global__ void __launch_bounds__(256) k_sha256(uint64_t n_msgs, const uint8_t *__restrict__ bytes,
                                                const uint64_t *__restrict__ off,
                                                uint32_t *__restrict__ digest_words) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m < n_msgs) sha256_one(m, bytes, off, digest_words);
}

__global__ void __launch_bounds__(64) k_key_decode(uint32_t n_keys, const uint8_t *__restrict__ kbytes,
                                                   const uint64_t *__restrict__ koff, uint8_t *__restrict__ kstatus,
                                                   uint32_t *__restrict__ kxy) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n_keys) key_decode_one(k, kbytes, koff, kstatus, kxy);
}

__global__ void __launch_bounds__(64) k_table_bases(uint32_t n_bases, const uint32_t *__restrict__ bxy,
                                                    const uint8_t *__restrict__ bstatus,
                                                    uint32_t *__restrict__ bases_jac, int w, int nwin) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_bases) return;
  if (bstatus && bstatus[b] != KS_OK) return;
  table_bases_one(b, bxy, bases_jac, w, nwin);
}

// blockDim = 256, grid (NWIN * 2^W/256, n_bases).  Block (j, c) computes
// entries d = 256c + t of window j and normalises them to affine with one
// field inversion (prefix/suffix products in LDS).  PHI: also write the
// phi(T) half of a GLV key table.
template <int W, int NWIN, bool PHI>
__global__ void __launch_bounds__(256) k_table_fill(const uint32_t *__restrict__ bases_jac,
                                                    const uint8_t *__restrict__ bstatus,
                                                    uint32_t *__restrict__ table) {
  constexpr uint32_t chunks = (1u << W) / 256u;
  constexpr uint64_t half_u32 = (uint64_t)NWIN * (1ull << W) * BV_ENTRY_U32;
  const uint32_t b = blockIdx.y;
  const uint32_t j = blockIdx.x / chunks;
  const uint32_t d = (blockIdx.x % chunks) * 256u + threadIdx.x;
  const uint32_t t = threadIdx.x;
  if (bstatus && bstatus[b] != KS_OK) return;  // uniform per block
  __shared__ fe sPre[256];
  __shared__ fe sSuf[256];
  __shared__ fe sBx, sBy, sInvTotal;
  if (t == 0) {
    fe x, y;
    jac_to_affine(x, y, bases_jac + ((uint64_t)b * NWIN + j) * 24);
    sBx = x;
    sBy = y;
  }
  __syncthreads();
  const fe bx = sBx, by = sBy;
  gej R;
  bool inf;
  fe Z;
  table_point(R, inf, Z, bx, by, d, W);
  sPre[t] = Z;
  sSuf[t] = Z;
  __syncthreads();
  for (uint32_t s = 1; s < 256; s <<= 1) {
    fe p = sPre[t], q = sSuf[t];
    if (t >= s) fe_mul(p, p, sPre[t - s]);
    if (t + s < 256) fe_mul(q, q, sSuf[t + s]);
    __syncthreads();
    sPre[t] = p;
    sSuf[t] = q;
    __syncthreads();
  }
  if (t == 0) {
    fe x;
    fe_inv(x, sPre[255]);
    sInvTotal = x;
  }
  __syncthreads();
  fe zi = sInvTotal;  // Z_t^-1 = prefix(t-1) * suffix(t+1) * (prod Z)^-1
  if (t > 0) fe_mul(zi, zi, sPre[t - 1]);
  if (t < 255) fe_mul(zi, zi, sSuf[t + 1]);
  uint32_t *entry = table + (uint64_t)b * (PHI ? 2 : 1) * half_u32 + (((uint64_t)j << W) + d) * BV_ENTRY_U32;
  table_store(entry, PHI ? entry + half_u32 : nullptr, d, R, inf, zi);
}

__global__ void __launch_bounds__(256) k_scalar_prep(uint64_t n_items, uint32_t M, const uint32_t *__restrict__ r_be,
                                                     const uint32_t *__restrict__ s_be, const uint8_t *__restrict__ pre,
                                                     const uint32_t *__restrict__ item_msg,
                                                     const uint32_t *__restrict__ digest_words,
                                                     uint32_t *__restrict__ scratch, uint32_t *__restrict__ u12) {
  const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  scalar_prep_thread(t, T, n_items, M, r_be, s_be, pre, item_msg, digest_words, scratch, u12);
}

__device__ __forceinline__ void write_status(uint64_t i, uint64_t n_items, uint8_t st, uint8_t *status,
                                             uint64_t *bits) {
  if (i < n_items) status[i] = st;
  const uint64_t mask = __ballot(i < n_items && st == BV_ACCEPT);
  if ((threadIdx.x & 63) == 0 && i < n_items) bits[i >> 6] = mask;
}

__global__ void __launch_bounds__(256) k_verify_g(uint64_t n_items, const uint32_t *__restrict__ item_key,
                                                  const uint32_t *__restrict__ r_be, const uint32_t *__restrict__ s_be,
                                                  const uint8_t *__restrict__ pre, const uint8_t *__restrict__ kstatus,
                                                  const uint32_t *__restrict__ u12,
                                                  const uint32_t *__restrict__ g_table, uint32_t *__restrict__ rg) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_items) verify_item_g(i, n_items, item_key, r_be, s_be, pre, kstatus, u12, g_table, rg);
}

__global__ void __launch_bounds__(256) k_verify_q(uint64_t n_items, const uint32_t *__restrict__ item_key,
                                                  const uint32_t *__restrict__ r_be, const uint32_t *__restrict__ s_be,
                                                  const uint8_t *__restrict__ pre, const uint8_t *__restrict__ kstatus,
                                                  const uint32_t *__restrict__ u12,
                                                  const uint32_t *__restrict__ key_table,
                                                  const uint32_t *__restrict__ rg, uint8_t *__restrict__ status,
                                                  uint64_t *__restrict__ bits) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t st = BV_REJECT;
  if (i < n_items) st = verify_item_q(i, n_items, item_key, r_be, s_be, pre, kstatus, u12, key_table, rg);
  write_status(i, n_items, st, status, bits);
}

__global__ void __launch_bounds__(256) k_verify_generic(uint64_t n_items, const uint32_t *__restrict__ item_key,
                                                        const uint32_t *__restrict__ r_be,
                                                        const uint32_t *__restrict__ s_be,
                                                        const uint8_t *__restrict__ pre,
                                                        const uint8_t *__restrict__ kstatus,
                                                        const uint32_t *__restrict__ kxy,
                                                        const uint32_t *__restrict__ u12,
                                                        const uint32_t *__restrict__ g_table,
                                                        uint8_t *__restrict__ status, uint64_t *__restrict__ bits) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t st = BV_REJECT;
  if (i < n_items) st = verify_item_generic(i, item_key, r_be, s_be, pre, kstatus, kxy, u12, g_table);
  write_status(i, n_items, st, status, bits);
}

// ---------------------------------------------------------------------------
// Launch wrappers (called from bv_api.cpp)
// ---------------------------------------------------------------------------
namespace bvk {

static inline dim3 grid1(uint64_t n, uint32_t block) { return dim3((uint32_t)((n + block - 1) / block)); }

hipError_t sha256(hipStream_t st, uint64_t n, const uint8_t *bytes, const uint64_t *off, uint32_t *dig) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sha256, grid1(n, 256), dim3(256), 0, st, n, bytes, off, dig);
  return hipGetLastError();
}

hipError_t key_decode(hipStream_t st, uint32_t n, const uint8_t *kb, const uint64_t *ko, uint8_t *kst, uint32_t *kxy) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_key_decode, grid1(n, 64), dim3(64), 0, st, n, kb, ko, kst, kxy);
  return hipGetLastError();
}

// key = false: the generator table (16-bit windows over 256 bits, built once
// per ctx); key = true: GLV key tables (8-bit windows over 128 bits + phi).
hipError_t build_tables(hipStream_t st, bool key, uint32_t n_bases, const uint32_t *bxy, const uint8_t *bstatus,
                        uint32_t *bases_jac, uint32_t *table) {
  if (n_bases == 0) return hipSuccess;
  const int w = key ? BV_KW : BV_GW, nwin = key ? BV_KNWIN : BV_GNWIN;
  hipLaunchKernelGGL(k_table_bases, grid1(n_bases, 64), dim3(64), 0, st, n_bases, bxy, bstatus, bases_jac, w, nwin);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (key)
    hipLaunchKernelGGL((k_table_fill<BV_KW, BV_KNWIN, true>), dim3(BV_KNWIN * ((1u << BV_KW) / 256u), n_bases),
                       dim3(256), 0, st, bases_jac, bstatus, table);
  else
    hipLaunchKernelGGL((k_table_fill<BV_GW, BV_GNWIN, false>), dim3(BV_GNWIN * ((1u << BV_GW) / 256u), n_bases),
                       dim3(256), 0, st, bases_jac, bstatus, table);
  return hipGetLastError();
}

hipError_t scalar_prep(hipStream_t st, uint64_t n, uint32_t M, const uint32_t *r_be, const uint32_t *s_be,
                       const uint8_t *pre, const uint32_t *item_msg, const uint32_t *dig, uint32_t *scratch,
                       uint32_t *u12) {
  if (n == 0) return hipSuccess;
  const uint64_t threads = (n + M - 1) / M;
  hipLaunchKernelGGL(k_scalar_prep, grid1(threads, 256), dim3(256), 0, st, n, M, r_be, s_be, pre, item_msg, dig,
                     scratch, u12);
  return hipGetLastError();
}

hipError_t verify_g(hipStream_t st, uint64_t n, const uint32_t *item_key, const uint32_t *r_be, const uint32_t *s_be,
                    const uint8_t *pre, const uint8_t *kst, const uint32_t *u12, const uint32_t *g_table,
                    uint32_t *rg) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verify_g, grid1(n, 256), dim3(256), 0, st, n, item_key, r_be, s_be, pre, kst, u12, g_table, rg);
  return hipGetLastError();
}

hipError_t verify_q(hipStream_t st, uint64_t n, const uint32_t *item_key, const uint32_t *r_be, const uint32_t *s_be,
                    const uint8_t *pre, const uint8_t *kst, const uint32_t *u12, const uint32_t *key_table,
                    const uint32_t *rg, uint8_t *status, uint64_t *bits) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verify_q, grid1(n, 256), dim3(256), 0, st, n, item_key, r_be, s_be, pre, kst, u12, key_table,
                     rg, status, bits);
  return hipGetLastError();
}

hipError_t verify_generic(hipStream_t st, uint64_t n, const uint32_t *item_key, const uint32_t *r_be,
                          const uint32_t *s_be, const uint8_t *pre, const uint8_t *kst, const uint32_t *kxy,
                          const uint32_t *u12, const uint32_t *g_table, uint8_t *status, uint64_t *bits) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verify_generic, grid1(n, 256), dim3(256), 0, st, n, item_key, r_be, s_be, pre, kst, kxy, u12,
                     g_table, status, bits);
  return hipGetLastError();
}

}  // namespace bvk
