// H2D copy rate from pinned host memory (hipHostMalloc) into HBM, as the host
// entries use it: 512 MB moved in 64 MB chunks issued on 1, 2 or 4 streams
// (round robin), timed from before the first issue to after the last
// completion.  Does a second copy stream (a second SDMA engine) raise the
// PCIe rate?  Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/ubench_h2d tools/ubench_h2d.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

#define CHK(x)                                                          \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      return 1;                                                         \
    }                                                                   \
  } while (0)

int main() {
  const size_t total = 512ull << 20, chunk = 64ull << 20;
  void *h = nullptr, *d = nullptr;
  CHK(hipHostMalloc(&h, total, hipHostMallocDefault));
  CHK(hipMalloc(&d, total));
  memset(h, 1, total);
  hipStream_t s[4];
  for (auto &x : s) CHK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  for (int ns : {1, 2, 4, 1, 2, 4}) {
    double best = 1e30;
    for (int rep = 0; rep < 5; rep++) {
      CHK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      for (size_t o = 0, k = 0; o < total; o += chunk, k++)
        CHK(hipMemcpyAsync((char *)d + o, (char *)h + o, chunk, hipMemcpyHostToDevice, s[k % ns]));
      for (int i = 0; i < ns; i++) CHK(hipStreamSynchronize(s[i]));
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms < best) best = ms;
    }
    printf("h2d 512 MB in 64 MB chunks over %d stream(s): best %.3f ms = %.1f GB/s\n", ns, best, total / best / 1e6);
  }
  return 0;
}
