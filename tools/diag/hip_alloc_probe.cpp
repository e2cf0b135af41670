// Times hipMalloc / hipMemsetAsync / hipFree of large buffers with the HIP
// runtime this binary links (the system ROCm), to explain slow allocation-heavy
// phases outside a torch process.  usage: hip_alloc_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

int main() {
  using clk = std::chrono::steady_clock;
  hipSetDevice(0);
  hipFree(nullptr);
  size_t fr = 0, tot = 0;
  hipMemGetInfo(&fr, &tot);
  printf("free %.1f GB of %.1f GB\n", fr / 1e9, tot / 1e9);
  const double gbs[] = {0.25, 1, 4, 16, 64};
  for (double gb : gbs) {
    void *p = nullptr;
    const size_t n = (size_t)(gb * 1e9);
    auto t0 = clk::now();
    hipError_t e = hipMalloc(&p, n);
    auto t1 = clk::now();
    if (e) { printf("%.2f GB: hipMalloc failed %d\n", gb, (int)e); continue; }
    hipMemsetAsync(p, 0, 1 << 20, 0);
    hipStreamSynchronize(0);
    auto t2 = clk::now();
    hipFree(p);
    auto t3 = clk::now();
    printf("%6.2f GB: malloc %.1f ms, first small memset %.1f ms, free %.1f ms\n", gb,
           std::chrono::duration<double, std::milli>(t1 - t0).count(),
           std::chrono::duration<double, std::milli>(t2 - t1).count(),
           std::chrono::duration<double, std::milli>(t3 - t2).count());
    fflush(stdout);
  }
  return 0;
}
