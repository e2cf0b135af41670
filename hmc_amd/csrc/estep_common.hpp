// estep_common.hpp — helpers shared by the E-step kernels: the fused
// single-pass kernel (estep.hip) and the split structure/value pass
// (estep_split.hip).  Device-only, no state.
#pragma once
#include "hmc_internal.hpp"

namespace hmc {

constexpr unsigned long long KEY_EMPTY = ~0ull;
constexpr unsigned long long TRACE_CHUNK = 1ull << 16;  // words per bump allocation
constexpr int NP_MAX = A_MAX * (A_MAX + 1) / 2;          // allele pairs at a fully missing locus
constexpr int PROBE_LDS = 16;                            // LDS probes before a key goes to the HBM table

__host__ __device__ inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

__device__ inline int lane_id() { return (int)(threadIdx.x & (WAVE - 1)); }
__device__ inline uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Key (id_a, id_b) of m_best_pair (HaploBuilder.cpp:251-259) -> table slot hash.
__device__ inline uint32_t key_hash(uint32_t lo, uint32_t hi) {
  uint32_t h = lo * 0x9E3779B1u ^ (hi + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 13;
  return h;
}

// Trace record of one locus at word `off`: [Fn][Fn headers][pad to an even
// word][Fn x S link words]; this is the word index of the link block.
__host__ __device__ inline unsigned long long trace_links(unsigned long long off, uint32_t F) {
  return (off + 1 + F + 1) & ~1ull;
}

// Copy the first ns links of predecessor state s into a successor list at
// position k0, transformed as by the extension constructor / add
// (HaploPair.cpp:35-61, 63-80): likelihood x tp, link = s, index = position in
// s's list, reversed flag, and the homozygous rule (a homozygous link entering
// a pair with different last alleles loses the flag and, when reversed, its
// likelihood).  Groups of GRP links: the loads of a group issue together.
// tl != nullptr: the link words also go to tl[k0 + k] (the trace record of
// the locus, written while the list is built).
template <int GRP = 8>
__device__ inline void copy_extended(const double *xl, const uint32_t *xm, double *yl, uint32_t *ym, int k0, int ns,
                                     uint32_t s, double tpv, bool rev, bool differ, uint32_t *tl = nullptr) {
  for (int k = 0; k < ns; k += GRP) {
    double v[GRP];
    uint32_t m[GRP];
#pragma unroll
    for (int u = 0; u < GRP; ++u)
      if (k + u < ns) {
        v[u] = xl[k + u];
        m[u] = xm[k + u];
      }
#pragma unroll
    for (int u = 0; u < GRP; ++u)
      if (k + u < ns) {
        double lk = v[u] * tpv;
        bool homo = meta_homo(m[u]);
        if (differ && homo) {
          if (rev) lk = 0.0;
          homo = false;
        }
        const uint32_t mw = meta_pack(s, (uint32_t)(k + u), rev, homo, false);
        yl[k0 + k + u] = lk;
        ym[k0 + k + u] = mw;
        if (tl) tl[k0 + k + u] = mw;
      }
  }
}

// copy_extended on the compact frontier (value_front.hpp): the predecessor's
// homozygous flags as a bit mask xhm, the new flags into *yhm; the link words
// go to the trace record tl only.
template <int GRP = 4>
__device__ inline void copy_extended_hm(const double *xl, unsigned long long xhm, double *yl, unsigned long long &yhm,
                                        int k0, int ns, uint32_t s, double tpv, bool rev, bool differ, uint32_t *tl) {
  for (int k = 0; k < ns; k += GRP) {
    double v[GRP];
#pragma unroll
    for (int u = 0; u < GRP; ++u)
      if (k + u < ns) v[u] = xl[k + u];
#pragma unroll
    for (int u = 0; u < GRP; ++u)
      if (k + u < ns) {
        double lk = v[u] * tpv;
        bool homo = (xhm >> (k + u)) & 1ull;
        if (differ && homo) {
          if (rev) lk = 0.0;
          homo = false;
        }
        yl[k0 + k + u] = lk;
        yhm |= (unsigned long long)homo << (k0 + k + u);
        tl[k0 + k + u] = meta_pack(s, (uint32_t)(k + u), rev, homo, false);
      }
  }
}

}  // namespace hmc
