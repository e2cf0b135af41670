// value_front.hpp — the value pass's frontier view (one frontier of k-best
// lists with an LDS tier and an HBM tier), shared by the locus-synchronous
// value pass (estep_split.hip) and the dataflow one (estep_df.hip).
#pragma once
#include "hmc_internal.hpp"
#include "estep_common.hpp"

namespace hmc {

// Value frontier: forward likelihood, list length, first overflowing add,
// and the k-best list (S likelihoods + S link words) of every state.  One
// region per tier, arrays at fixed offsets (8-byte aligned): fwd[n] nl[n]
// r0[n] lik[n][S] meta[n][S], n = fc (LDS) or fcap (HBM).
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
  __device__ double *lik(int t) const {
    return t < fc ? (double *)(l + (size_t)fc * 16) + t * S : (double *)(g + (size_t)fcap * 16) + (size_t)(t - fc) * S;
  }
  __device__ uint32_t *meta(int t) const {
    return t < fc ? (uint32_t *)(l + (size_t)fc * (16 + 8 * S)) + t * S
                  : (uint32_t *)(g + (size_t)fcap * (16 + 8 * S)) + (size_t)(t - fc) * S;
  }
  // Link k of state t with address-space-specific loads (ds_read for the LDS
  // tier, global_load for the HBM tier): a flat load would count against
  // lgkmcnt and make every later LDS wait also wait on HBM.
  __device__ void ld_link(int t, int k, double &lk, uint32_t &mt) const {
    if (t < fc) {
      typedef __attribute__((address_space(3))) const double lds_f64;
      typedef __attribute__((address_space(3))) const uint32_t lds_u32;
      lk = *((lds_f64 *)(l + (size_t)fc * 16) + t * S + k);
      mt = *((lds_u32 *)(l + (size_t)fc * (16 + 8 * S)) + t * S + k);
    } else {
      typedef __attribute__((address_space(1))) const double glb_f64;
      typedef __attribute__((address_space(1))) const uint32_t glb_u32;
      lk = *((glb_f64 *)(g + (size_t)fcap * 16) + (size_t)(t - fc) * S + k);
      mt = *((glb_u32 *)(g + (size_t)fcap * (16 + 8 * S)) + (size_t)(t - fc) * S + k);
    }
  }
};

__host__ __device__ inline size_t k2_front_bytes(int fcap, int S) { return al256((size_t)fcap * (16 + 12 * S)); }

}  // namespace hmc
