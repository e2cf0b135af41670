// mstep.hpp — device layout of the level-synchronous pattern miner (mstep.hip).
#pragma once
#include "hmc_internal.hpp"

namespace hmc {

constexpr uint8_t NODE_ACC = 1;  // accepted into m_patterns (PatternManager.cpp:130-133)
constexpr uint8_t NODE_EXT = 2;  // extended by one allele   (PatternManager.cpp:110-111)

// Candidate nodes of all levels live in flat arrays; roots (the empty pattern
// at each start) are virtual and encoded as -(start + 2); -1 = none.  Node
// indices are global over the whole search; when the search runs in blocks
// of start loci, the arrays hold a window of them and the MineArgs node
// pointers are offset so that kernels index them globally.
constexpr int RM_SLOTS = 64;  // R_M counters, 16 words (128 B) apart

struct MineArgs {
  int L = 0, amax = 0, n_items = 0;     // items scanned by the root lists (this rank)
  int item_base = 0, item_stride = 0;   // first root item; row stride of geno_lm / samp_lm
  bool genotype = true;                 // genotype branch (M0) or sample branch
  const uchar2 *geno_lm = nullptr;      // [L][N]
  const uint8_t *samp_lm = nullptr;     // [L][H]
  const double *w = nullptr;            // [H]
  unsigned long long *stamps = nullptr; // diagnostic build: shader cycles per mine_count phase [8]
  const double *afreq = nullptr;        // [L][amax]
  const uint8_t *anum = nullptr;        // [L+1]
  const uint8_t *npos = nullptr;        // [L+1] alleles with frequency > 0
  const uint8_t *pos_allele = nullptr;  // [L][amax] those alleles, ascending
  const uint8_t *rank_of = nullptr;     // [L][amax] rank among them, 0xFF if none
  double denom = 1.0, min_freq = 0.0;
  int min_len = 1, max_len = 30;
  // nodes
  int32_t *parent = nullptr, *start = nullptr;
  uint8_t *allele = nullptr, *flags = nullptr;
  double *freq = nullptr, *prefix = nullptr, *tp = nullptr, *sum = nullptr;
  uint32_t *cnt = nullptr, *size = nullptr, *pos = nullptr;
  int32_t *child_base = nullptr, *link = nullptr;
  unsigned long long *list_off = nullptr;  // node -> its matching list in the level's list buffer
  unsigned long long *region = nullptr;    // extended node -> its children's lists in the next buffer (nc x cnt)
  const unsigned long long *r_region = nullptr;  // [L] the same for the roots
  const int32_t *r_child_base = nullptr;  // [L+1]
  // matching lists of the parent level (in) and the child level (out)
  const uint32_t *lin_idx = nullptr;
  const double *lin_val = nullptr;
  uint32_t *lout_idx = nullptr;
  double *lout_val = nullptr;
  unsigned long long *rm = nullptr;      // R_M counter
  // Ordered reduction over ranks: every child's sum starts from sum[c] (the
  // running sum of the ranks before this one, whose items precede this
  // rank's in the reference's order) instead of 0.
  bool seeded = false;
};

// Pattern table in id (= DFS pre-order) order.
struct PatternTable {
  int32_t *start = nullptr, *len = nullptr, *node = nullptr;
  // prefix pattern (the pattern without its last allele): its id, -1 for
  // length-1 patterns, -2 when the prefix is no pattern (below min_len, or a
  // table installed from outside); spells allele strings without the tree
  int32_t *ppat = nullptr;
  double *freq = nullptr, *prefix = nullptr, *tp = nullptr;
  uint8_t *last = nullptr;
  uint32_t *succ = nullptr;  // [P][amax]
};

// checkFrequency of n candidates of length `level` (start[n], allele indices
// [n][level], 0xFD = a symbol the locus does not have) over this rank's items:
// sum[c] = ordered sum of the matching items' values (continued when seeded).
hipError_t launch_mine_scan(const MineArgs &a, int level, int n, const int32_t *cstart, const uint8_t *cal,
                            double *sum, hipStream_t st);
// Ordered reduction: child sums of [cb, ce) continued over this rank's lists
// (the ones the level's mine_count wrote to lout_idx / lout_val).
hipError_t launch_mine_sum(const MineArgs &a, int cb, int ce, hipStream_t st);
hipError_t launch_mine_count(const MineArgs &a, int level, int pbeg, int pend, hipStream_t st);
hipError_t launch_mine_finalize(const MineArgs &a, int level, int b, int e, unsigned long long *ext_list,
                                int32_t *next_children, hipStream_t st);
hipError_t launch_mine_offsets(const MineArgs &a, int b, int e, unsigned long long *ext_list, int32_t *next_children,
                               int next_base, void *tmp, size_t tmp_bytes, unsigned long long *totals,
                               hipStream_t st);
size_t mine_scan_tmp_bytes(int n);
hipError_t launch_mine_size(const MineArgs &a, int level, int b, int e, hipStream_t st);
// roots [lo, hi) (a block of start loci, see Ctx::mine_impl)
hipError_t launch_mine_root_size(const MineArgs &a, uint32_t *rsize, int lo, int hi, hipStream_t st);
hipError_t launch_mine_pos(const MineArgs &a, int level, int pbeg, int pend, const uint32_t *rpos, hipStream_t st);
hipError_t launch_mine_emit(const MineArgs &a, const int *lev_begin, int maxlev, int n, const PatternTable &t,
                            hipStream_t st);
// successors of the patterns [id0, id0 + n)
// Successors of the patterns of one level (nodes [cb, ce) of length `level`),
// levels in increasing length; *err |= 1 if a walk needed a node below node_lo.
hipError_t launch_mine_succ_level(const MineArgs &a, const PatternTable &t, int level, int cb, int ce, int32_t node_lo,
                                  int *err, hipStream_t st);

}  // namespace hmc
