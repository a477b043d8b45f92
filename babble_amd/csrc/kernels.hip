// kernels.hip — gfx950 kernels of the batch verifier (per-unit work lives in
// verify_core.h).
//
// Pipeline for one batch (bv_api.cpp drives it on the ctx stream):
//   k_sha256       one lane per message: digest of the canonical JSON body
//                  (crypto.SHA256, src/crypto/hash.go:8)
//   k_key_decode   one lane per key: elliptic.Unmarshal(btcec.S256(), b)
//                  (src/crypto/keys/public_key.go:14-20)
//   k_table_bases  one lane per base point: B_j = 2^(8j) P, j = 0..31
//   k_table_fill   one workgroup per (base, window): d * B_j for d = 1..255,
//                  batch-normalised to affine with one field inversion
//                  (prefix/suffix products in LDS)
//   k_scalar_prep  Montgomery-trick batch inversion of s mod N, then
//                  u1 = e/s, u2 = r/s (ecdsa.Verify steps 4-6)
//   k_verify       one lane per signature item: the SURVEY §8a-9 decision
//                  table, R = u1 G + u2 Q as 64 affine table additions
//                  (fixed-base 8-bit windows for G and for every key), the
//                  projective x(R) mod N == r check, status byte and
//                  __ballot accept bits (one u64 word per wave)
//   k_verify_generic  same item semantics for keys without a table
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
                                                    uint32_t *__restrict__ bases_jac) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_bases) return;
  if (bstatus && bstatus[b] != KS_OK) return;
  table_bases_one(b, bxy, bases_jac);
}

// blockDim = 256, grid (32 windows, n_bases).  Thread d computes d * B_j;
// the block normalises its 256 points with one inversion.
__global__ void __launch_bounds__(256) k_table_fill(const uint32_t *__restrict__ bases_jac,
                                                    const uint8_t *__restrict__ bstatus,
                                                    uint32_t *__restrict__ table) {
  const uint32_t b = blockIdx.y;
  const uint32_t j = blockIdx.x;
  const uint32_t d = threadIdx.x;
  if (bstatus && bstatus[b] != KS_OK) return;  // uniform per block
  __shared__ fe sPre[256];
  __shared__ fe sSuf[256];
  __shared__ fe sBx, sBy, sInvTotal;
  if (d == 0) {
    fe x, y;
    jac_to_affine(x, y, bases_jac + ((uint64_t)b * BV_NWIN + j) * 24);
    sBx = x;
    sBy = y;
  }
  __syncthreads();
  const fe bx = sBx, by = sBy;
  gej R;
  bool inf;
  fe Z;
  table_point(R, inf, Z, bx, by, d);
  sPre[d] = Z;
  sSuf[d] = Z;
  __syncthreads();
  // Hillis-Steele inclusive prefix (sPre) and suffix (sSuf) products
  for (uint32_t s = 1; s < 256; s <<= 1) {
    fe p = sPre[d], q = sSuf[d];
    if (d >= s) fe_mul(p, p, sPre[d - s]);
    if (d + s < 256) fe_mul(q, q, sSuf[d + s]);
    __syncthreads();
    sPre[d] = p;
    sSuf[d] = q;
    __syncthreads();
  }
  if (d == 0) {
    fe t;
    fe_inv(t, sPre[255]);
    sInvTotal = t;
  }
  __syncthreads();
  // Z_d^-1 = prefix(d-1) * suffix(d+1) * (prod Z)^-1
  fe zi = sInvTotal;
  if (d > 0) fe_mul(zi, zi, sPre[d - 1]);
  if (d < 255) fe_mul(zi, zi, sSuf[d + 1]);
  table_store(table, b, j, d, R, inf, zi);
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

__global__ void __launch_bounds__(256) k_verify(uint64_t n_items, const uint32_t *__restrict__ item_key,
                                                const uint32_t *__restrict__ r_be, const uint32_t *__restrict__ s_be,
                                                const uint8_t *__restrict__ pre, const uint8_t *__restrict__ kstatus,
                                                const uint32_t *__restrict__ u12,
                                                const uint32_t *__restrict__ g_table,
                                                const uint32_t *__restrict__ key_table, uint8_t *__restrict__ status,
                                                uint64_t *__restrict__ bits) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t st = BV_REJECT;
  if (i < n_items) st = verify_item_tables(i, item_key, r_be, s_be, pre, kstatus, u12, g_table, key_table);
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

hipError_t sha256(hipStream_t st, uint64_t n, const uint8_t *bytes, const uint64_t *off, uint32_t *dig) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sha256, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, n, bytes, off, dig);
  return hipGetLastError();
}

hipError_t key_decode(hipStream_t st, uint32_t n, const uint8_t *kb, const uint64_t *ko, uint8_t *kst, uint32_t *kxy) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_key_decode, dim3((n + 63) / 64), dim3(64), 0, st, n, kb, ko, kst, kxy);
  return hipGetLastError();
}

hipError_t build_tables(hipStream_t st, uint32_t n_bases, const uint32_t *bxy, const uint8_t *bstatus,
                        uint32_t *bases_jac, uint32_t *table) {
  if (n_bases == 0) return hipSuccess;
  hipLaunchKernelGGL(k_table_bases, dim3((n_bases + 63) / 64), dim3(64), 0, st, n_bases, bxy, bstatus, bases_jac);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_table_fill, dim3(BV_NWIN, n_bases), dim3(256), 0, st, bases_jac, bstatus, table);
  return hipGetLastError();
}

hipError_t scalar_prep(hipStream_t st, uint64_t n, uint32_t M, const uint32_t *r_be, const uint32_t *s_be,
                       const uint8_t *pre, const uint32_t *item_msg, const uint32_t *dig, uint32_t *scratch,
                       uint32_t *u12) {
  if (n == 0) return hipSuccess;
  const uint64_t threads = (n + M - 1) / M;
  hipLaunchKernelGGL(k_scalar_prep, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, st, n, M, r_be, s_be, pre,
                     item_msg, dig, scratch, u12);
  return hipGetLastError();
}

hipError_t verify(hipStream_t st, uint64_t n, const uint32_t *item_key, const uint32_t *r_be, const uint32_t *s_be,
                  const uint8_t *pre, const uint8_t *kst, const uint32_t *u12, const uint32_t *g_table,
                  const uint32_t *key_table, uint8_t *status, uint64_t *bits) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verify, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, n, item_key, r_be, s_be, pre, kst,
                     u12, g_table, key_table, status, bits);
  return hipGetLastError();
}

hipError_t verify_generic(hipStream_t st, uint64_t n, const uint32_t *item_key, const uint32_t *r_be,
                          const uint32_t *s_be, const uint8_t *pre, const uint8_t *kst, const uint32_t *kxy,
                          const uint32_t *u12, const uint32_t *g_table, uint8_t *status, uint64_t *bits) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verify_generic, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, n, item_key, r_be, s_be,
                     pre, kst, kxy, u12, g_table, status, bits);
  return hipGetLastError();
}

}  // namespace bvk
