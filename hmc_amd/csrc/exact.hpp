// exact.hpp — device arguments of the exact M-step kernels (exact.hip).
#pragma once
#include "hmc_internal.hpp"

namespace hmc {

// Fixed-point scale of the frequency accumulators: 2^-44 resolution, totals
// up to 2^19 individuals fit in 63 bits.
constexpr double EXACT_FIXED_SCALE = 17592186044416.0;  // 2^44

struct ExactArgs {
  int L, head_len, width;          // loci, head length, alleles per trie node (max alleles per locus)
  const int32_t *order;            // individuals of this group (batch indices)
  int n_order;
  const uint32_t *rec;             // structure records (exact mode)
  const unsigned long long *rec_off;  // [batch][L+1]
  int32_t *status;                 // [batch]: EST_OK, or EST_NEEDS_EXACT when a forward likelihood underflows
  const double *gprob;             // [batch] P(genotype) of the last E-step
  // fwd/bwd store: per individual a region at x_base, per locus fwd[F] bwd[F]
  uint32_t *x;
  const unsigned long long *x_base;   // [batch]
  unsigned long long *x_off;          // [batch][L+1] (written by exact_fb)
  // ForwardPatternTree of the round's candidates (host-built)
  const int32_t *tr_child;         // [nodes][width], -1 = none
  const int32_t *tr_data;          // [nodes] candidate index or -1
  const int32_t *tr_root;          // [L] root node of each start locus, -1 = empty
  int max_depth;                   // longest candidate
  const uint8_t *head_al;          // [P][head_len] head patterns' alleles (head_len > 1)
  // per-wave scratch (exact_walk_scratch_doubles): lists [max_depth+1][width][3][fmax],
  // children's frequencies [max_depth+2][width] (doubles), touched states
  // [max_depth+1][fmax] (u32); zero before the launch
  double *scratch;
  size_t scratch_stride;           // doubles
  int fmax;                        // most states of any locus of the group
  long long span = 0;              // the walk's per-item list span: most states over max_depth + 2 consecutive depths
  unsigned *span_max = nullptr;    // exact_span: atomicMax of each individual's largest span (zeroed by the host)
  unsigned long long *acc_freq, *acc_prefix;  // [candidates] fixed point
  long long item0 = 0, item1 = -1;  // walk items [item0, item1) of n_order x L (individual-major); -1 = all
};

// Breadth-first trie walk (exact_walk_units): one lane per work unit — a trie
// node of one item (individual q of the group, start locus) at depth `depth`
// with the non-zero entries of its three lists (state ascending; weights w0
// both haplotypes match the node's pattern, w1 only the a side, w2 only the b
// side).  A lane scatters the entries along the forward links into its
// private accumulators, adds every child's frequency and prefix term, and
// emits the children that have non-zero lists and children of their own as the
// next level's units.  Roots (depth 0) carry no entries: every state after
// max(start, head_len) loci with its forward likelihood.
struct XUnits {
  int32_t *q = nullptr, *start = nullptr, *node = nullptr;  // node < 0: a hole (skipped)
  double *freq = nullptr;                                   // the node's frequency: its children's prefix term
  unsigned long long *e0 = nullptr;                         // first entry in the pool
  uint32_t *ne = nullptr;                                   // entries
};
struct XWalkArgs {
  XUnits u;                       // the unit pool
  uint32_t *e_t = nullptr;        // entry pool: state
  double *e_w = nullptr;          // [3][e_cap] weights
  unsigned long long e_cap = 0, u_cap = 0;
  unsigned long long in_base = 0; // this level's units: [in_base, in_base + n_in), or idx[0, n_in) when idx
  const int32_t *idx = nullptr;
  int n_in = 0, depth = 0;
  bool roots = false;
  unsigned long long *cursor = nullptr;  // [2] next free unit, next free entry (outputs)
  int32_t *defer = nullptr;       // input units whose outputs did not fit (re-run later)
  int *n_defer = nullptr;
  double *lacc = nullptr;         // per thread [2][3][fmax]: the a-allele and b-allele child of each state
  uint32_t *lbits = nullptr;      // per thread reached-state bitmap [fmax / 32 + 1]
  size_t lacc_stride = 0, lbits_stride = 0;  // doubles, words
};
hipError_t launch_exact_walk_units(const ExactArgs &a, const XWalkArgs &x, int grid, hipStream_t st);

hipError_t launch_exact_fb(const ExactArgs &a, int grid, hipStream_t st);
// ExactArgs::span_max (atomicMax, zeroed by the caller) over the group
hipError_t launch_exact_span(const ExactArgs &a, int grid, hipStream_t st);
// items_per_wave 1 (64 lanes per item) or 4 (16 lanes each); scratch: grid x items x stride
hipError_t launch_exact_walk(const ExactArgs &a, int grid, hipStream_t st, int items_per_wave = 1);
size_t exact_walk_scratch_doubles(int max_depth, long long span, int width);
// Tries of at most this many alleles per node keep, per depth and slot, the
// child ids and the non-zero masks of the walk in LDS (wider ones read them)
constexpr int XWALK_CACHE_W = 8;
__host__ __device__ inline int exact_walk_cache_w(int width) { return width <= XWALK_CACHE_W ? width : 0; }
// LDS of one walked item: per depth two masks, two record offsets, eleven ints
// and 64 cached touched states (u16), per depth and cached slot a non-zero mask
// and a child id, the reached-state bitmap (8-byte multiple)
__host__ __device__ inline size_t exact_walk_lds_bytes(int max_depth, int fmax, int width) {
  const size_t D = (size_t)max_depth + 2, wc = (size_t)exact_walk_cache_w(width);
  return (D * 32 + D * wc * 8 + D * 44 + D * wc * 4 + D * 128 + (size_t)((fmax + 31) / 32 + 1) * 4 + 7) & ~(size_t)7;
}
constexpr size_t EXACT_WALK_LDS_MAX = 160 * 1024;  // gfx950 LDS per workgroup

}  // namespace hmc
