// value_front.hpp — the value pass's frontier view (one frontier of k-best
// lists with an LDS tier and an HBM tier), shared by the locus-synchronous
// value pass (estep_split.hip) and the dataflow one (estep_df.hip).
#pragma once
#include "hmc_internal.hpp"
#include "estep_common.hpp"

namespace hmc {

// Value frontier: forward likelihood, list length, first overflowing add,
// the homozygous flags of the list's links (bit k = position k) and the S
// likelihoods of every state.  One region per tier, arrays at fixed offsets
// (8-byte aligned): fwd[n] nl[n] r0[n] hm[n] lik[n][S], n = fc (LDS) or fcap
// (HBM): 24 + 8 S bytes per state.  The link words themselves live only in
// the locus's trace record (written as the lists are built; a chain's
// partial list is read back from it): the next locus needs of a predecessor's
// link only its likelihood and homozygous flag.
struct VFront {
  unsigned char *l, *g;
  int fc, fcap, S;
  __device__ double *fwd(int t) const {
    return t < fc ? (double *)l + t : (double *)g + (t - fc);
  }
  __device__ uint32_t *nl(int t) const {
    return t < fc ? (uint32_t *)(l + (size_t)fc * 8) + t : (uint32_t *)(g + (size_t)fcap * 8) + (t - fc);
  }
  __device__ uint32_t *r0(int t) const {
    return t < fc ? (uint32_t *)(l + (size_t)fc * 12) + t : (uint32_t *)(g + (size_t)fcap * 12) + (t - fc);
  }
  __device__ unsigned long long *hm(int t) const {
    return t < fc ? (unsigned long long *)(l + (size_t)fc * 16) + t
                  : (unsigned long long *)(g + (size_t)fcap * 16) + (t - fc);
  }
  __device__ double *lik(int t) const {
    return t < fc ? (double *)(l + (size_t)fc * 24) + t * S : (double *)(g + (size_t)fcap * 24) + (size_t)(t - fc) * S;
  }
  // Link k's likelihood and state t's homozygous flags with address-space-
  // specific loads (ds_read for the LDS tier, global_load for the HBM tier): a
  // flat load would count against lgkmcnt and make every later LDS wait also
  // wait on HBM.
  __device__ void ld_link(int t, int k, double &lk, unsigned long long &hmw) const {
    if (t < fc) {
      typedef __attribute__((address_space(3))) const double lds_f64;
      typedef __attribute__((address_space(3))) const unsigned long long lds_u64;
      lk = *((lds_f64 *)(l + (size_t)fc * 24) + t * S + k);
      hmw = *((lds_u64 *)(l + (size_t)fc * 16) + t);
    } else {
      typedef __attribute__((address_space(1))) const double glb_f64;
      typedef __attribute__((address_space(1))) const unsigned long long glb_u64;
      lk = *((glb_f64 *)(g + (size_t)fcap * 24) + (size_t)(t - fc) * S + k);
      hmw = *((glb_u64 *)(g + (size_t)fcap * 16) + (t - fc));
    }
  }
};

__host__ __device__ inline size_t k2_front_bytes(int fcap, int S) { return al256((size_t)fcap * (24 + 8 * S)); }

}  // namespace hmc
