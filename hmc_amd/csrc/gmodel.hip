// gmodel.hip — the pattern table in end-locus order, for the structure pass.
//
// The structure pass looks up, per contribution, the successors of the two
// patterns of a pair (m_successor, HaploPattern.h; HaploBuilder.cpp:230-245)
// and, per state, their transition probabilities and last alleles.  In the
// table's own order (DFS pre-order of the start-locus tries) the patterns that
// end at one locus are spread over the whole table, so every lookup is a
// random line from HBM: cfg 3's E2 structure pass fetched ~16 KB per
// individual-locus (profiles/r04/pmc_fetch_estep_structure_cfg3.csv), near
// the HBM roofline for 4-byte reads.  Here the same table is re-indexed by g =
// (end locus, id) order — a stable radix sort of the ids by end locus — so the
// lookups of one locus fall in one block of the table (cfg 3's E2 model: ~3 300
// patterns per locus, 40 KB).  Within one end locus g order equals id order,
// and every comparison of the structure pass is between patterns that end at
// the same locus (the two successors of a pair; the two patterns of a head
// pair), so keys, reversed flags and creation order are unchanged.
#include <hipcub/hipcub.hpp>

#include "hmc_internal.hpp"

namespace hmc {

namespace {

__global__ void g_keys(const int32_t *start, const int32_t *len, int P, uint32_t *key, uint32_t *ids) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P) {
    key[i] = (uint32_t)(start[i] + len[i] - 1);
    ids[i] = (uint32_t)i;
  }
}

__global__ void g_inverse(const uint32_t *gid, int P, uint32_t *inv) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < P) inv[gid[g]] = (uint32_t)g;
}

__global__ void g_gather(const uint32_t *gid, const uint32_t *inv, const uint32_t *succ, const double *tp,
                         const uint8_t *last, int P, int A, uint32_t *gsucc, double *gtp, uint8_t *glast) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= P) return;
  const uint32_t id = gid[g];
  gtp[g] = tp[id];
  glast[g] = last[id];
  for (int x = 0; x < A; ++x) {
    const uint32_t s = succ[(size_t)id * A + x];
    gsucc[(size_t)g * A + x] = s == NONE ? NONE : inv[s];
  }
}

int end_bits(int L) {
  int b = 1;
  while ((1 << b) < L) ++b;
  return b;
}

}  // namespace

size_t gmodel_sort_bytes(int P, int L) {
  size_t bytes = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                     (const uint32_t *)nullptr, (uint32_t *)nullptr, P, 0, end_bits(L));
  return bytes;
}

hipError_t build_gmodel(const GModelArgs &g, hipStream_t st) {
  const int P = g.P;
  if (P <= 0) return hipSuccess;
  const int B = 256, grid = (P + B - 1) / B;
  hipLaunchKernelGGL(g_keys, dim3(grid), dim3(B), 0, st, g.start, g.len, P, g.key_in, g.id_in);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t bytes = g.temp_bytes;
  // LSD radix sort: stable, so ids stay in order within one end locus
  if ((e = hipcub::DeviceRadixSort::SortPairs(g.temp, bytes, g.key_in, g.key_out, g.id_in, g.gid, P, 0, end_bits(g.L),
                                              st)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(g_inverse, dim3(grid), dim3(B), 0, st, g.gid, P, g.inv);
  hipLaunchKernelGGL(g_gather, dim3(grid), dim3(B), 0, st, g.gid, g.inv, g.succ, g.tp, g.last, P, g.A, g.gsucc, g.gtp,
                     g.glast);
  return hipGetLastError();
}

}  // namespace hmc
