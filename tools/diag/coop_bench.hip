// coop_bench.hip — microbenchmark of the value pass's segmented selection
// (coop_select.hpp, never the product): every wave runs chains of adds on
// 2S-lane segments like phase B of estep_values — S new likelihoods (few
// distinct values, so ties occur) behind the segment's S kept ones, then
// std::nth_element(.., S-1, ..) — and a checksum of the kept lists.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I hmc_amd/csrc tools/diag/coop_bench.hip -o coop_bench
//   ./coop_bench [waves_per_cu] [adds]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "coop_select.hpp"

using namespace hmc;

__device__ inline uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(64) void bench(int S, int adds, double *out) {
  extern __shared__ unsigned char sm[];
  const int lane = threadIdx.x;
  SegScratch ss{(int *)sm, (int *)sm + 64, (int *)sm + 128, (double *)(sm + 1024), (uint32_t *)(sm + 1024 + 512)};
  const Seg sg = make_seg(2 * S);
  const int G = 64 / (2 * S);
  const bool in = sg.g < G;
  uint32_t h = mix(blockIdx.x * 64 + lane);
  if (in && sg.k < S) {
    ss.slik[lane] = (double)(mix(h) % 64);
    ss.smeta[lane] = sg.k;
  }
  wave_lds_sync();
  for (int r = 0; r < adds; ++r) {
    h = mix(h + r);
    if (in && sg.k >= S) {
      ss.slik[lane] = (double)(h % 64);
      ss.smeta[lane] = 1000u * r + sg.k;
    }
    wave_lds_sync();
    seg_nth_slots(in ? 2 * S : 0, S - 1, sg, ss);
  }
  double acc = 0.0;
  if (in && sg.k < S) acc = ss.slik[lane] * (double)(ss.smeta[lane] % 97);
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) out[blockIdx.x] = acc;
}

int main(int argc, char **argv) {
  const int wpc = argc > 1 ? atoi(argv[1]) : 16, adds = argc > 2 ? atoi(argv[2]) : 2000, S = 10;
  int cu = 256;
  hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = cu * wpc;
  double *out;
  hipMalloc(&out, grid * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(bench, dim3(grid), dim3(64), 2048, 0, S, 10, out);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(bench, dim3(grid), dim3(64), 2048, 0, S, adds, out);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  double *h = (double *)malloc(grid * sizeof(double)), cs = 0;
  hipMemcpy(h, out, grid * sizeof(double), hipMemcpyDeviceToHost);
  for (int i = 0; i < grid; ++i) cs += h[i];
  const double segs = (double)grid * (64 / (2 * S));
  printf("waves/CU %d adds %d: %.2f ms, %.1f ns per add per segment (wall), %.0f cycles per add per wave at 2.4 GHz, checksum %.17g\n",
         wpc, adds, ms, ms * 1e6 / (segs * adds), ms * 1e-3 * 2.4e9 / adds, cs);
  return 0;
}
