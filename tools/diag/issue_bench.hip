// Issue cost of wave64 VALU instruction classes on gfx950 (MI355X), measured
// at 1..8 resident waves per SIMD — the calibration of the VALU-issue roof that
// tools/sq_summary.py prices estep_values' instruction mix against.
//
//   hipcc --offload-arch=gfx950 -O3 tools/diag/issue_bench.hip -o tools/diag/issue_bench
//   ./tools/diag/issue_bench [iters] > issue_cpi.json
//
// Each wavefront runs `iters` x 32 instructions of ONE class on 8 independent
// registers (inline asm, so the compiler neither merges nor reorders them), and
// stamps s_memtime (shader clock) and s_memrealtime (100 MHz) before and after.
// Every CU holds 4 x W waves (one block of 256 threads per wave per SIMD), all
// resident at once, so a SIMD runs W waves side by side:
//   cpi_wave = shader cycles of a wave / its instructions
//   cpi_simd = cpi_wave / W  = SIMD cycles per wave64 instruction (issue cost)
// The guide (MI355X_MICROARCH.md: SIMD-32, a wave64 VALU instruction over 2
// cycles; one wave alone sustains 4) gives the expectation for 32-bit ops.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

enum Op { ADD_U32, CNDMASK, ADD_F64, MUL_F64, CMP_F64, LSHL_B64, MOV_B32, FMA_F32, N_OPS };
static const char *kName[N_OPS] = {"v_add_u32",    "v_cndmask_b32", "v_add_f64",  "v_mul_f64",
                                   "v_cmp_gt_f64", "v_lshlrev_b64", "v_mov_b32", "v_fma_f32"};
static const char *kClass[N_OPS] = {"INT32", "other32", "ADD_F64", "MUL_F64", "cmp_f64", "INT64", "other32", "FMA_F32"};

template <int OP>
__device__ __forceinline__ void body(unsigned (&u)[8], double (&d)[8], float (&f)[8], unsigned long long (&m)[8],
                                     unsigned ub, double db, float fb, unsigned long long mk) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (OP == ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[j]) : "v"(ub));
      if constexpr (OP == CNDMASK) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[j]) : "v"(ub), "s"(mk));
      if constexpr (OP == ADD_F64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[j]) : "v"(db));
      if constexpr (OP == MUL_F64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[j]) : "v"(db));
      if constexpr (OP == CMP_F64) asm volatile("v_cmp_gt_f64_e64 %0, %1, %2" : "+s"(m[j]) : "v"(d[j]), "v"(db));
      if constexpr (OP == LSHL_B64) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(d[j]));
      if constexpr (OP == MOV_B32) asm volatile("v_mov_b32 %0, %1" : "=v"(u[j]) : "v"(ub));
      if constexpr (OP == FMA_F32) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[j]) : "v"(fb));
    }
  }
}

template <int OP>
__global__ void __launch_bounds__(256) issue_kernel(int iters, unsigned long long *stamps, unsigned *sink) {
  unsigned u[8];
  double d[8];
  float f[8];
  unsigned long long m[8] = {};
  const unsigned ub = threadIdx.x | 1u;
  const double db = 1.0 + threadIdx.x * 1e-9;
  const float fb = 0.999f;
  const unsigned long long mk = 0x5555555555555555ull;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    u[j] = threadIdx.x + j;
    d[j] = 1.0 + j * 1e-3;
    f[j] = 1.0f + j;
  }
  __syncthreads();
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) body<OP>(u, d, f, m, ub, db, fb, mk);
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  unsigned acc = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc ^= u[j] ^ (unsigned)__double_as_longlong(d[j]) ^ __float_as_uint(f[j]) ^ (unsigned)m[j];
  if (acc == 0x12345678u) sink[0] = acc;  // keeps the registers live; never true in practice
  if ((threadIdx.x & 63) == 0) {
    const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    stamps[4 * w + 0] = c1 - c0;
    stamps[4 * w + 1] = r1 - r0;
    stamps[4 * w + 2] = r0;
    stamps[4 * w + 3] = r1;
  }
}

using KFn = void (*)(int, unsigned long long *, unsigned *);
static KFn kern(int op) {
  switch (op) {
    case ADD_U32: return issue_kernel<ADD_U32>;
    case CNDMASK: return issue_kernel<CNDMASK>;
    case ADD_F64: return issue_kernel<ADD_F64>;
    case MUL_F64: return issue_kernel<MUL_F64>;
    case CMP_F64: return issue_kernel<CMP_F64>;
    case LSHL_B64: return issue_kernel<LSHL_B64>;
    case MOV_B32: return issue_kernel<MOV_B32>;
    default: return issue_kernel<FMA_F32>;
  }
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4096;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cu = p.multiProcessorCount;
  int wall_khz = 100000;
  CHECK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
  unsigned long long *d_st;
  unsigned *d_sink;
  const int WMAX = 8;
  CHECK(hipMalloc(&d_st, (size_t)cu * WMAX * 4 * 4 * sizeof(unsigned long long)));
  CHECK(hipMalloc(&d_sink, 64));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("{\"device\": \"%s\", \"cus\": %d, \"wall_clock_khz\": %d, \"iters\": %d, \"insts_per_wave\": %lld, "
         "\"rows\": [\n", p.gcnArchName, cu, wall_khz, iters, (long long)iters * 32);
  bool first = true;
  for (int op = 0; op < N_OPS; ++op)
    for (int W : {1, 2, 4, 8}) {
      const int grid = cu * W, nw = grid * 4;
      for (int rep = 0; rep < 2; ++rep) {  // the first launch warms the clocks
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern(op), dim3(grid), dim3(256), 0, 0, iters, d_st, d_sink);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
      }
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<unsigned long long> h((size_t)nw * 4);
      CHECK(hipMemcpy(h.data(), d_st, h.size() * 8, hipMemcpyDeviceToHost));
      double cyc = 0, rt = 0;
      unsigned long long rmin = ~0ull, rmax = 0;
      for (int w = 0; w < nw; ++w) {
        cyc += (double)h[4 * w];
        rt += (double)h[4 * w + 1];
        rmin = h[4 * w + 2] < rmin ? h[4 * w + 2] : rmin;
        rmax = h[4 * w + 3] > rmax ? h[4 * w + 3] : rmax;
      }
      cyc /= nw;
      rt /= nw;
      const double n_inst = (double)iters * 32;
      const double clk_ghz = cyc / (rt * 1e6 / wall_khz);  // s_memrealtime ticks at the wall-clock rate
      // overlap: the waves' spans over the whole launch span (1 = all resident together)
      const double overlap = rt / (double)(rmax - rmin);
      printf("%s {\"op\": \"%s\", \"class\": \"%s\", \"waves_per_simd\": %d, \"cpi_wave\": %.3f, \"cpi_simd\": %.3f, "
             "\"clock_ghz\": %.3f, \"overlap\": %.3f, \"kernel_ms\": %.3f}",
             first ? "" : ",\n", kName[op], kClass[op], W, cyc / n_inst, cyc / n_inst / W, clk_ghz, overlap, ms);
      first = false;
    }
  printf("\n]}\n");
  return 0;
}
