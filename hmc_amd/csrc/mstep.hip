// mstep.hip — pattern mining (M-step) of the HaploModel EM on CDNA4 (gfx950).
//
// Restates PatternManager::findPatternByFreq (PatternManager.cpp:27-42), its
// DFS candidate search searchPattern (:100-144), the frequency scans
// checkFrequency / checkFrequencyWithExtension / getMatchingFrequency
// (:146-291) and initialize (:293-318: ids, head list, successors through the
// BackwardPatternTree, PatternTree.cpp:50-72,98-134).
//
// The reference grows the candidate tree depth-first with an explicit stack.
// Here the same tree is grown breadth-first, one pattern length per step, so
// that every candidate of a level is scanned in parallel:
//   mine_count    one wavefront per extendable parent streams the parent's
//                 matching list (sample or individual indices, in ascending
//                 order, exactly the MatchingState the reference passes down)
//                 and produces every child's weighted sum.  The sum of each
//                 child is accumulated strictly in list order (a single
//                 dependent add chain per child, lane k owns child k) so the
//                 frequencies are bit-identical to the reference's sequential
//                 `total_freq += ...` loops.
//   mine_finalize frequency, prefix frequency, transition probability and the
//                 accept / extend rules of searchPattern.
//                 The same pass writes the stable partition of the parent
//                 list into the children's lists (child k of a parent with n
//                 entries owns n slots at region + k*n of the next buffer).
// After the last level the DFS pre-order of the reference (start L-1 first,
// then descending allele index; PatternManager.cpp:94-97,112-113) is rebuilt
// from subtree sizes (bottom-up) and positions (top-down): position = pattern
// id.  Successors are found by walking suffix links (link(v) = v without its
// first allele) from the longest suffix down, which visits exactly the
// candidates the backward trie walk of findLongestMatchPattern would test.
#include <hipcub/hipcub.hpp>

#include "hmc_internal.hpp"
#include "mstep.hpp"

namespace hmc {

namespace {

__device__ inline int32_t root_code(int k) { return -(k + 2); }

// LDS hand-off between the lanes of a one-wavefront block: the LDS executes a
// wave's accesses in order, so only the compiler must keep program order (a
// __syncthreads would also wait for every outstanding HBM store).
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ inline double rl_f64(double x, int lane) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ inline bool is_root(int32_t u) { return u <= -2; }
__device__ inline int root_start(int32_t u) { return -u - 2; }

// One matching-list entry's contribution to child allele `al` at locus e.
struct EntryView {
  bool in;
  uint32_t item;
  double v;    // genotype branch: product carried from the parent
  uchar2 g;    // genotype branch: both alleles at e
  uint8_t h;   // sample branch: allele at e
  double w;    // sample branch: weight
};

template <bool WANT_W = true>  // the scatter only needs the allele, not the weight
__device__ inline EntryView load_entry(const MineArgs &a, bool root, const uint32_t *lidx, const double *lval,
                                       int i, int n, int e) {
  EntryView x;
  x.in = i < n;
  x.item = x.in ? (root ? (uint32_t)(a.item_base + i) : lidx[i]) : 0u;
  x.v = 1.0;
  x.w = 0.0;
  x.h = 0xFE;
  x.g = make_uchar2(0xFE, 0xFE);
  if (x.in) {
    if (a.genotype) {
      if (!root) x.v = lval[i];
      x.g = a.geno_lm[(size_t)e * a.item_stride + x.item];
    } else {
      x.h = a.samp_lm[(size_t)e * a.item_stride + x.item];
      if (WANT_W) x.w = a.w[x.item];
    }
  }
  return x;
}

// getMatchingFrequency (PatternManager.cpp:267-291) for one allele, times the
// carried product (checkFrequencyWithExtension :243-248); sample branch
// (:252-263) contributes the haplotype weight.
__device__ inline bool contribution(const MineArgs &a, const EntryView &x, int e, uint8_t al, double &c) {
  if (!x.in) { c = 0.0; return false; }
  if (a.genotype) {
    const bool m0 = x.g.x == MISSING, m1 = x.g.y == MISSING;
    if (!(m0 || m1 || x.g.x == al || x.g.y == al)) { c = 0.0; return false; }
    const double af = a.afreq[(size_t)e * a.amax + al];
    const double x0 = m0 ? af : (x.g.x == al ? 1.0 : 0.0);
    const double x1 = m1 ? af : (x.g.y == al ? 1.0 : 0.0);
    const double f = (0.0 + x0) + x1;
    const double t = 1.0 * (0.5 * f);
    c = x.v * t;
    return true;
  }
  if (x.h != al) { c = 0.0; return false; }
  c = x.w;
  return true;
}

struct ParentView {
  bool ok;
  int start, e, n, cb, nc;
  double pfreq;
  const uint32_t *lidx;
  const double *lval;
};

__device__ inline ParentView parent_view(const MineArgs &a, int level, int pidx) {
  ParentView p;
  p.ok = true;
  p.lidx = nullptr;
  p.lval = nullptr;
  if (level == 1) {
    p.start = pidx;
    p.e = pidx;
    p.n = a.n_items;
    p.cb = a.r_child_base[pidx];
    p.pfreq = 1.0;  // HaploPattern ctor: empty pattern has frequency 1 (HaploPattern.h:86)
  } else {
    if (!(a.flags[pidx] & NODE_EXT)) { p.ok = false; return p; }
    p.start = a.start[pidx];
    p.e = p.start + level - 1;
    p.n = (int)a.cnt[pidx];
    p.cb = a.child_base[pidx];
    p.pfreq = a.freq[pidx];
    p.lidx = a.lin_idx + a.list_off[pidx];
    if (a.genotype) p.lval = a.lin_val + a.list_off[pidx];
  }
  p.nc = a.npos[p.e];
  return p;
}

}  // namespace

// ---------------------------------------------------------------------------
constexpr int CROW = WAVE + 18;  // LDS row stride (doubles): one chunk's contributions + batch padding
#ifndef MC_U_DEF
#define MC_U_DEF 4
#endif
constexpr int MC_U = MC_U_DEF;    // chunks of 64 list entries per load group of mine_count
// one LDS buffer per chunk only while the block stays small (occupancy of the
// one-wave blocks matters more than the deferred stores for many alleles)
__host__ __device__ inline int mine_count_bufs(int amax) { return amax <= 2 ? MC_U : 1; }

// Child k's matching entries of one chunk (compacted in LDS) to its list:
// child k of a parent with n entries owns n slots at region + k*n; `mine` and
// `run` are lane k's entry count in this chunk and before it.
__device__ inline void store_child_lists(const MineArgs &a, const uint32_t *ibuf, const double *cbuf, int nc, int n,
                                         unsigned long long region, int mine, int run, int lane) {
  for (int k = 0; k < nc; ++k) {
    const int mk = __builtin_amdgcn_readlane(mine, k);
    const uint32_t rk = (uint32_t)__builtin_amdgcn_readlane(run, k);
    if (lane < mk) {
      const unsigned long long at = region + (unsigned long long)k * (unsigned long long)n + rk + lane;
      a.lout_idx[at] = ibuf[k * WAVE + lane];
      if (a.genotype) a.lout_val[at] = cbuf[k * CROW + lane];
    }
  }
}

#ifdef HMC_STAMPS
#define MSTAMP(k)                                                \
  do {                                                           \
    __builtin_amdgcn_s_waitcnt(0);                               \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();  \
    ms_acc[k] += t1 - ms_t0;                                     \
    ms_t0 = t1;                                                  \
  } while (0)
#else
#define MSTAMP(k) do { } while (0)
#endif

// Counting and the matching-list partition in one pass: child k of a parent
// with n entries owns n slots at region + k*n of the next list buffer, so the
// children's lists are written while the parent list streams through, before
// any child is known to be extended (lists of children that are not extended
// are simply never read).
__global__ __launch_bounds__(64) void mine_count(MineArgs a, int level, int pbeg, int pend) {
  // [ub][amax][CROW] contributions, then [ub][amax][WAVE] items: one buffer
  // per chunk of a load group (ub = U when amax <= 8, else 1)
  extern __shared__ __align__(16) double cbuf0[];
  const int tid = threadIdx.x, lane = tid;
  const int pidx = pbeg + blockIdx.x;
  if (pidx >= pend) return;
#ifdef HMC_STAMPS
  unsigned long long ms_t0 = __builtin_amdgcn_s_memtime(), ms_acc[8] = {};
#endif
  const ParentView p = parent_view(a, level, pidx);
  MSTAMP(0);
  if (!p.ok) return;
  const int ub = mine_count_bufs(a.amax);
  uint32_t *ibuf0 = (uint32_t *)(cbuf0 + (size_t)ub * a.amax * CROW);
  const uint8_t *ca = a.pos_allele + (size_t)p.e * a.amax;
  const uint64_t lt = (1ull << lane) - 1ull;
  const unsigned long long region = level == 1 ? a.r_region[pidx] : a.region[pidx];
  const bool write_lists = a.lout_idx != nullptr;
  // lane k: child k's allele (and, genotype branch, its population frequency),
  // read once; the child loop takes them with readlane
  const int my_al = lane < p.nc ? (int)ca[lane] : 0;
  const double my_af = (a.genotype && lane < p.nc) ? a.afreq[(size_t)p.e * a.amax + my_al] : 0.0;
  // lane k: child k's ordered sum, continued from the previous ranks' running
  // sum in ordered-reduction mode (the adds below extend the same chain)
  double sum = (a.seeded && lane < p.nc) ? a.sum[p.cb + lane] : 0.0;
  uint32_t cnt = 0, run = 0;  // lane k: child k's entries so far
  constexpr int U = MC_U;     // chunks whose loads are in flight together
  const size_t erow = (size_t)p.e * a.item_stride;
  for (int base = 0; base < p.n; base += U * WAVE) {
    // loads in two batches over all U chunks: list entries, then the gathers
    // that depend on them (one exposed latency each per U*64 entries).
    // Branch-free (lanes past the end load entry n-1 and are masked by `in`),
    // so each batch is one run of loads and one wait.
    EntryView xs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * WAVE + lane;
      const int ic = i < p.n ? i : p.n - 1;
      xs[u].in = i < p.n;
      xs[u].item = level == 1 ? (uint32_t)(a.item_base + ic) : p.lidx[ic];
      xs[u].v = (a.genotype && level != 1) ? p.lval[ic] : 1.0;
      xs[u].w = 0.0;
      xs[u].h = 0xFE;
      xs[u].g = make_uchar2(0xFE, 0xFE);
    }
    if (a.genotype) {
#pragma unroll
      for (int u = 0; u < U; ++u) xs[u].g = a.geno_lm[erow + xs[u].item];
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        xs[u].h = a.samp_lm[erow + xs[u].item];
        xs[u].w = a.w[xs[u].item];
      }
    }
    MSTAMP(1);
    int mine_u[U], run_u[U];  // lane k: child k's entries in chunk u, and before it
#pragma unroll
    for (int u = 0; u < U; ++u) {
      mine_u[u] = 0;
      run_u[u] = 0;
      if (base + u * WAVE >= p.n) break;
      const EntryView &x = xs[u];
      double *cbuf = cbuf0 + (size_t)(ub == U ? u : 0) * a.amax * CROW;
      uint32_t *ibuf = ibuf0 + (size_t)(ub == U ? u : 0) * a.amax * WAVE;
      // Each child's matching entries, compacted in list order.  Non-matching
      // entries would add +0.0, an exact no-op on a sum >= +0, so skipping them
      // leaves every child's add chain — and its rounding — unchanged.  Rows
      // are pre-filled with +0.0 so the summation below can run whole
      // 16-value batches without predication (x + 0.0 == x exactly).
      int mine = 0;
      for (int k = 0; k < p.nc; ++k) {
        const uint8_t al = (uint8_t)__builtin_amdgcn_readlane(my_al, k);
        double c;
        bool m;
        if (a.genotype) {
          // getMatchingFrequency (PatternManager.cpp:267-291) x carried product (:243-248)
          const bool m0 = x.g.x == MISSING, m1 = x.g.y == MISSING;
          m = x.in && (m0 || m1 || x.g.x == al || x.g.y == al);
          const double af = rl_f64(my_af, k);
          const double x0 = m0 ? af : (x.g.x == al ? 1.0 : 0.0);
          const double x1 = m1 ? af : (x.g.y == al ? 1.0 : 0.0);
          const double f = (0.0 + x0) + x1;
          const double t = 1.0 * (0.5 * f);
          c = m ? x.v * t : 0.0;
        } else {  // sample branch (:252-263): the haplotype weight
          m = x.in && x.h == al;
          c = m ? x.w : 0.0;
        }
        const uint64_t b = __ballot(m);
        cbuf[k * CROW + lane] = 0.0;
        if (lane < 16) cbuf[k * CROW + WAVE + lane] = 0.0;
        if (m) {
          cbuf[k * CROW + __popcll(b & lt)] = c;
          ibuf[k * WAVE + __popcll(b & lt)] = x.item;
        }
        if (lane == k) mine = __popcll(b);
      }
      wave_sync();  // one wavefront per block: LDS order suffices, no wait on the list stores
      MSTAMP(2);
      mine_u[u] = mine;
      run_u[u] = (int)run;
      if (write_lists && ub == 1) store_child_lists(a, ibuf, cbuf, p.nc, p.n, region, mine, (int)run, lane);
      if (lane < p.nc) {
        cnt += (uint32_t)mine;
        run += (uint32_t)mine;
        double s = sum;
        const double2 *row = (const double2 *)(cbuf + lane * CROW);
        // 16 values per batch: the reads issue together, the adds stay one
        // ordered chain (the +0.0 padding past `mine` changes nothing)
        for (int j = 0; j < mine; j += 16) {
          double2 q[8];
#pragma unroll
          for (int v = 0; v < 8; ++v) q[v] = row[(j >> 1) + v];
#pragma unroll
          for (int v = 0; v < 8; ++v) {
            s = s + q[v].x;
            s = s + q[v].y;
          }
        }
        sum = s;
      }
      wave_sync();
      MSTAMP(3);
    }
    // the group's child lists: all stores after the last chunk, so no chunk
    // waits on the previous chunk's stores
    if (write_lists && ub == U)
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (base + u * WAVE < p.n)
          store_child_lists(a, ibuf0 + (size_t)u * a.amax * WAVE, cbuf0 + (size_t)u * a.amax * CROW, p.nc, p.n,
                            region, mine_u[u], run_u[u], lane);
  }
  const int lane_c = tid;  // child lanes: threads 0..nc-1
  if (lane_c < p.nc) {
    const int c = p.cb + lane_c;
    const uint8_t al = ca[lane_c];
    a.sum[c] = sum;
    a.cnt[c] = cnt;
    a.list_off[c] = region + (unsigned long long)lane_c * (unsigned long long)p.n;
    a.start[c] = p.start;
    a.allele[c] = al;
    a.prefix[c] = p.pfreq;
    a.parent[c] = level == 1 ? root_code(p.start) : pidx;
    // suffix link: node for this pattern without its first allele
    int32_t lk;
    if (level == 1) {
      lk = root_code(p.start + 1);
    } else {
      const int32_t lp = a.link[pidx];
      const uint8_t rk = a.rank_of[(size_t)p.e * a.amax + al];
      if (lp == -1 || rk == 0xFF) lk = -1;
      else if (is_root(lp)) lk = a.r_child_base[root_start(lp)] + rk;
      else lk = (a.flags[lp] & NODE_EXT) ? a.child_base[lp] + rk : -1;
    }
    a.link[c] = lk;
  }
  // R_M: spread over RM_SLOTS counters a cache line apart (one shared counter
  // serialises every wave of the level in a single L2 channel)
  // A parent with an empty matching list sends every child through
  // checkFrequency's full scan (checkFrequencyWithExtension, PatternManager.cpp:
  // 197-199); no item matches a child of an unmatched parent, so only the count
  // changes.  (Zero-frequency parents are extended under MC, or below min_len.)
  const unsigned long long scanned = (p.n == 0 && level > 1) ? (unsigned long long)a.n_items : (unsigned long long)p.n;
  if (tid == 0) atomicAdd(&a.rm[(blockIdx.x % RM_SLOTS) * 16], scanned * (unsigned long long)p.nc);
#ifdef HMC_STAMPS
  MSTAMP(4);
  if (tid == 0 && a.stamps) {  // one private slot per block: no contended atomics
    unsigned long long *o = a.stamps + (size_t)blockIdx.x * 8;
    for (int k = 0; k < 5; ++k) o[k] = ms_acc[k];
    o[5] = 1ull;
    o[6] = (unsigned long long)p.n;
  }
#endif
}

// searchPattern's rules (PatternManager.cpp:110-133) for the nodes [b, e) of one level.
__global__ void mine_finalize(MineArgs a, int level, int b, int e, unsigned long long *ext_list,
                              int32_t *next_children) {
  const int c = b + blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= e) return;
  const double freq = a.sum[c] / a.denom;
  const double pre = a.prefix[c];
  double tp = pre > 0 ? freq / pre : freq;
  tp = tp < 1.0 ? tp : 1.0;  // HaploPattern::setTransitionProb (HaploPattern.h:47)
  a.freq[c] = freq;
  a.tp[c] = tp;
  const int st = a.start[c];
  const bool acc = (freq >= a.min_freq || level <= a.min_len) && level > 0 && level >= a.min_len;
  const bool ext = (freq >= a.min_freq || level < a.min_len) && (st + level < a.L) && (level < a.max_len);
  a.flags[c] = (acc ? NODE_ACC : 0) | (ext ? NODE_EXT : 0);
  // the node's children will need nc x cnt list slots (mine_count)
  ext_list[c - b] = ext ? (unsigned long long)a.npos[st + level] * a.cnt[c] : 0ull;
  next_children[c - b] = ext ? (int32_t)a.npos[st + level] : 0;
}

// Both per-node counts of a level scanned together (one device scan instead of two).
struct LevelOffsets {
  unsigned long long list;  // list slots before this node
  long long child;          // children before this node
};
struct LevelOffsetsSum {
  __host__ __device__ LevelOffsets operator()(const LevelOffsets &x, const LevelOffsets &y) const {
    return {x.list + y.list, x.child + y.child};
  }
};
struct LevelCounts {
  const unsigned long long *ext_list;
  const int32_t *next_children;
  __host__ __device__ LevelOffsets operator()(int i) const { return {ext_list[i], (long long)next_children[i]}; }
};
// Offsets applied to the level's nodes; the last node's thread also writes the level
// totals (list slots and nodes of the next level) for the host readback.
__global__ void mine_apply_offsets(MineArgs a, int b, int e, const LevelOffsets *scan,
                                   const unsigned long long *ext_list, const int32_t *next_children, int next_base,
                                   unsigned long long *totals) {
  const int c = b + blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= e) return;
  const LevelOffsets o = scan[c - b];
  const bool ext = a.flags[c] & NODE_EXT;
  a.region[c] = ext ? o.list : 0ull;
  a.child_base[c] = ext ? next_base + (int)o.child : -1;
  if (c == e - 1) {
    totals[0] = o.list + ext_list[c - b];
    totals[1] = (unsigned long long)(o.child + next_children[c - b]);
  }
}

// ---- DFS order ------------------------------------------------------------
__global__ void mine_size(MineArgs a, int level, int b, int e) {
  const int c = b + blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= e) return;
  uint32_t s = (a.flags[c] & NODE_ACC) ? 1u : 0u;
  if (a.flags[c] & NODE_EXT) {
    const int cb = a.child_base[c];
    const int nc = a.npos[a.start[c] + level];
    for (int k = 0; k < nc; ++k) s += a.size[cb + k];
  }
  a.size[c] = s;
}

__global__ void mine_root_size(MineArgs a, uint32_t *rsize, int lo, int hi) {
  const int s = lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= hi) return;
  uint32_t t = 0;
  const int cb = a.r_child_base[s];
  for (int k = 0; k < a.npos[s]; ++k) t += a.size[cb + k];
  rsize[s] = t;
}

// Pre-order positions: parent first, then children in descending allele order.
__global__ void mine_pos(MineArgs a, int level, int pbeg, int pend, const uint32_t *rpos) {
  const int pidx = pbeg + blockIdx.x * blockDim.x + threadIdx.x;
  if (pidx >= pend) return;
  uint32_t running;
  int cb, nc;
  if (level == 1) {
    running = rpos[pidx];
    cb = a.r_child_base[pidx];
    nc = a.npos[pidx];
  } else {
    if (!(a.flags[pidx] & NODE_EXT)) return;
    running = a.pos[pidx] + ((a.flags[pidx] & NODE_ACC) ? 1u : 0u);
    cb = a.child_base[pidx];
    nc = a.npos[a.start[pidx] + level - 1];
  }
  for (int k = nc - 1; k >= 0; --k) {
    a.pos[cb + k] = running;
    running += a.size[cb + k];
  }
}

// All levels in one launch: node c's level (= pattern length) is found by binary
// search over the level start offsets lev_begin[1..maxlev+1].
__global__ void mine_emit(MineArgs a, const int *lev_begin, int maxlev, PatternTable t) {
  const int c = lev_begin[1] + blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= lev_begin[maxlev + 1]) return;
  if (!(a.flags[c] & NODE_ACC)) return;
  int lo = 1, hi = maxlev;  // largest level whose begin <= c
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (lev_begin[mid] <= c) lo = mid;
    else hi = mid - 1;
  }
  const uint32_t id = a.pos[c];
  const int32_t par = a.parent[c];
  t.ppat[id] = is_root(par) ? -1 : ((a.flags[par] & NODE_ACC) ? (int32_t)a.pos[par] : -2);
  t.start[id] = a.start[c];
  t.len[id] = lo;
  t.freq[id] = a.freq[c];
  t.prefix[id] = a.prefix[c];
  t.tp[id] = a.tp[c];
  t.last[id] = a.allele[c];
  t.node[id] = c;
}

// successor[j] = longest stored suffix of (pattern + allele j)
// (PatternManager.cpp:308-317), for the patterns of one level (length
// `level`, nodes [cb, ce)).  The walk goes down the suffix links; the first
// suffix that is itself a pattern is shorter, so its successor for the same
// extension locus is already in the table (an earlier level, or a block of
// higher start loci), and the rest of the walk would be exactly its walk: the
// answer is taken from there.  Frequent patterns' suffixes are frequent, so
// this is normally one step, and it never leaves the node window (a suffix
// link reaches at most one block up).  Nodes below `node_lo` (slid out of the
// window) are never read: a walk that would need one sets *err.
__global__ void mine_succ_level(MineArgs a, PatternTable t, int level, int cb, int ce, int32_t node_lo, int *err) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)(ce - cb) * a.amax) return;
  const int c = cb + (int)(gid / a.amax), j = (int)(gid % a.amax);
  if (!(a.flags[c] & NODE_ACC)) return;
  const uint32_t id = a.pos[c];
  const int e = a.start[c] + level;
  uint32_t res = NONE;
  bool lost = false;
  if (e < a.L && j < a.anum[e]) {
    const uint8_t rk = a.rank_of[(size_t)e * a.amax + j];
    int32_t u = c;
    int depth = 0;  // leading alleles dropped so far
    while (true) {
      if (is_root(u)) {
        if (rk != 0xFF) {
          const int ch = a.r_child_base[root_start(u)] + rk;
          if (ch < node_lo) { lost = true; break; }
          if (a.flags[ch] & NODE_ACC) res = a.pos[ch];
        }
        break;
      }
      if (u == -1) {
        // Chain broken: the suffix dropped so far is no candidate (models
        // whose patterns are not suffix-closed: min_len > 1, findPatternByNum
        // — searched in one block).  Navigate the shorter suffixes from their
        // roots.  The pattern's alleles are read through a window of AW
        // positions, refilled by walking the parent chain.
        constexpr int AW = 128;
        const int vs = a.start[c];
        const int L0 = level;
        uint8_t al[AW];
        int w0 = -1;  // first position held in the window (-1: empty)
        auto allele_at = [&](int q) -> uint8_t {
          if (w0 < 0 || q < w0 || q >= w0 + AW) {
            w0 = q;
            const int hi = min(q + AW, L0) - 1;
            int32_t w = c;
            for (int r = L0 - 1; r > hi; --r) w = a.parent[w];
            for (int r = hi; r >= q; --r) {
              al[r - q] = a.allele[w];
              w = a.parent[w];
            }
          }
          return al[q - w0];
        };
        for (int d = depth + 1; d <= L0 && res == NONE && !lost; ++d) {
          const int ks = vs + d;  // suffix start
          int32_t nd = root_code(ks);
          bool ok = true;
          for (int q = d; q < L0 && ok; ++q) {
            const int loc = vs + q;
            const uint8_t r = a.rank_of[(size_t)loc * a.amax + allele_at(q)];
            if (r == 0xFF) { ok = false; break; }
            if (is_root(nd)) nd = a.r_child_base[root_start(nd)] + r;
            else if (a.flags[nd] & NODE_EXT) nd = a.child_base[nd] + r;
            else ok = false;
            if (ok && nd < node_lo) lost = true;
            ok = ok && !lost;
          }
          if (!ok || rk == 0xFF) continue;
          int ch;
          if (is_root(nd)) ch = a.r_child_base[root_start(nd)] + rk;
          else if (a.flags[nd] & NODE_EXT) ch = a.child_base[nd] + rk;
          else continue;
          if (ch < node_lo) { lost = true; break; }
          if (a.flags[ch] & NODE_ACC) res = a.pos[ch];
        }
        break;
      }
      if (u < node_lo) { lost = true; break; }
      if (depth > 0 && (a.flags[u] & NODE_ACC)) {  // a shorter pattern: its successor is known
        res = t.succ[(size_t)a.pos[u] * a.amax + j];
        break;
      }
      if ((a.flags[u] & NODE_EXT) && rk != 0xFF) {
        const int ch = a.child_base[u] + rk;
        if (a.flags[ch] & NODE_ACC) { res = a.pos[ch]; break; }
      }
      u = a.link[u];
      ++depth;
    }
  }
  if (lost) atomicOr(err, 1);
  t.succ[(size_t)id * a.amax + j] = res;
}

// ---- host-side launch helpers -----------------------------------------------
// PatternManager::checkFrequency (PatternManager.cpp:146-193) for arbitrary
// candidates of one length: one wavefront per candidate scans every item of
// this rank in order.  Genotype branch: getMatchingFrequency (:267-291), the
// product taken locus by locus as `total_freq *= 0.5 * freq`; sample branch:
// the haplotype weight.  Lane 0 adds the matching items' values in item order
// (non-matching items add nothing), continuing sum[c] when seeded.
__global__ __launch_bounds__(64) void mine_scan(MineArgs a, int level, int n, const int32_t *cstart,
                                                const uint8_t *cal, double *sum) {
  __shared__ double vals[WAVE];
  const int lane = threadIdx.x;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int c = blockIdx.x; c < n; c += gridDim.x) {
    const int st = cstart[c];
    const uint8_t *al = cal + (size_t)c * level;
    double s = a.seeded ? sum[c] : 0.0;
    for (int base = 0; base < a.n_items; base += WAVE) {
      const int i = base + lane;
      const uint32_t item = (uint32_t)(a.item_base + (i < a.n_items ? i : a.n_items - 1));
      bool m = i < a.n_items;
      double v = 1.0;
      for (int j = 0; j < level; ++j) {
        const int e = st + j;
        const uint8_t pa = al[j];
        if (a.genotype) {
          const uchar2 g = a.geno_lm[(size_t)e * a.item_stride + item];
          const bool m0 = g.x == MISSING, m1 = g.y == MISSING;
          m = m && (m0 || m1 || g.x == pa || g.y == pa);
          const double af = pa < a.amax ? a.afreq[(size_t)e * a.amax + pa] : 0.0;
          const double x0 = m0 ? af : (g.x == pa ? 1.0 : 0.0);
          const double x1 = m1 ? af : (g.y == pa ? 1.0 : 0.0);
          v = v * (0.5 * ((0.0 + x0) + x1));
        } else {
          m = m && a.samp_lm[(size_t)e * a.item_stride + item] == pa;
        }
        if (!__ballot(m)) break;
      }
      const uint64_t b = __ballot(m);
      if (m) vals[__popcll(b & lt)] = a.genotype ? v : a.w[item];
      wave_sync();
      if (lane == 0) {
        const int k = __popcll(b);
        for (int q = 0; q < k; ++q) s = s + vals[q];
      }
      wave_sync();
    }
    if (lane == 0) sum[c] = s;
  }
}

hipError_t launch_mine_scan(const MineArgs &a, int level, int n, const int32_t *cstart, const uint8_t *cal,
                            double *sum, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (level < 1 || a.n_items < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mine_scan, dim3(n < 65536 ? n : 65536), dim3(WAVE), 0, st, a, level, n, cstart, cal, sum);
  return hipGetLastError();
}

// Ordered cross-rank reduction, the add chain alone: child c's sum continues
// from sum[c] (the running sum of the ranks before this one) over the values
// of its matching list that mine_count just wrote on this rank (genotype
// branch: the carried products; sample branch: the haplotype weights), in
// list order.  mine_count itself runs on all ranks at once, so only this
// cheap pass is sequential across ranks.
__global__ __launch_bounds__(64) void mine_sum(MineArgs a, int cb, int ce) {
  __shared__ double vals[WAVE];
  const int lane = threadIdx.x;
  for (int c = cb + blockIdx.x; c < ce; c += gridDim.x) {
    const uint32_t n = a.cnt[c];
    const unsigned long long off = a.list_off[c];
    double s = a.sum[c];
    for (uint32_t base = 0; base < n; base += WAVE) {
      const uint32_t i = base + lane;
      double v = 0.0;
      if (i < n) v = a.genotype ? a.lout_val[off + i] : a.w[a.lout_idx[off + i]];
      vals[lane] = v;
      wave_sync();
      if (lane == 0) {
        const uint32_t k = n - base < (uint32_t)WAVE ? n - base : (uint32_t)WAVE;
        for (uint32_t q = 0; q < k; ++q) s = s + vals[q];
      }
      wave_sync();
    }
    if (lane == 0) a.sum[c] = s;
  }
}

hipError_t launch_mine_sum(const MineArgs &a, int cb, int ce, hipStream_t st) {
  if (ce <= cb) return hipSuccess;
  if (!a.lout_idx || (a.genotype && !a.lout_val)) return hipErrorInvalidValue;
  const int n = ce - cb;
  hipLaunchKernelGGL(mine_sum, dim3(n < 65536 ? n : 65536), dim3(WAVE), 0, st, a, cb, ce);
  return hipGetLastError();
}

hipError_t launch_mine_count(const MineArgs &a, int level, int pbeg, int pend, hipStream_t st) {
  if (pend <= pbeg) return hipSuccess;
  const size_t lds = (size_t)mine_count_bufs(a.amax) * ((size_t)a.amax * CROW * 8 + (size_t)a.amax * WAVE * 4);
  if (lds > 65536 - 1024) {  // many alleles: opt in to the CU's full LDS (per device: set on every launch)
    hipError_t e = hipFuncSetAttribute((const void *)mine_count, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds + 1024);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(mine_count, dim3(pend - pbeg), dim3(WAVE), lds, st, a, level, pbeg, pend);
  return hipGetLastError();
}
hipError_t launch_mine_finalize(const MineArgs &a, int level, int b, int e, unsigned long long *ext_list,
                                int32_t *next_children, hipStream_t st) {
  if (e <= b) return hipSuccess;
  hipLaunchKernelGGL(mine_finalize, dim3((e - b + 255) / 256), dim3(256), 0, st, a, level, b, e, ext_list, next_children);
  return hipGetLastError();
}
static size_t scan_storage_bytes(int n) {
  size_t need = 0;
  hipcub::TransformInputIterator<LevelOffsets, LevelCounts, hipcub::CountingInputIterator<int>> in(
      hipcub::CountingInputIterator<int>(0), LevelCounts{nullptr, nullptr});
  hipcub::DeviceScan::ExclusiveScan(nullptr, need, in, (LevelOffsets *)nullptr, LevelOffsetsSum(), LevelOffsets{0, 0},
                                    n);
  return (need + 255) & ~(size_t)255;
}
hipError_t launch_mine_offsets(const MineArgs &a, int b, int e, unsigned long long *ext_list, int32_t *next_children,
                               int next_base, void *tmp, size_t tmp_bytes, unsigned long long *totals, hipStream_t st) {
  const int n = e - b;
  if (n <= 0) return hipSuccess;
  size_t need = scan_storage_bytes(n);
  if (need + (size_t)n * sizeof(LevelOffsets) > tmp_bytes) return hipErrorInvalidValue;
  LevelOffsets *scan = (LevelOffsets *)((char *)tmp + need);
  hipcub::TransformInputIterator<LevelOffsets, LevelCounts, hipcub::CountingInputIterator<int>> in(
      hipcub::CountingInputIterator<int>(0), LevelCounts{ext_list, next_children});
  hipError_t err =
      hipcub::DeviceScan::ExclusiveScan(tmp, need, in, scan, LevelOffsetsSum(), LevelOffsets{0, 0}, n, st);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(mine_apply_offsets, dim3((n + 255) / 256), dim3(256), 0, st, a, b, e, scan, ext_list,
                     next_children, next_base, totals);
  return hipGetLastError();
}
size_t mine_scan_tmp_bytes(int n) { return scan_storage_bytes(n) + (size_t)n * sizeof(LevelOffsets); }
hipError_t launch_mine_size(const MineArgs &a, int level, int b, int e, hipStream_t st) {
  if (e <= b) return hipSuccess;
  hipLaunchKernelGGL(mine_size, dim3((e - b + 255) / 256), dim3(256), 0, st, a, level, b, e);
  return hipGetLastError();
}
hipError_t launch_mine_root_size(const MineArgs &a, uint32_t *rsize, int lo, int hi, hipStream_t st) {
  if (hi <= lo) return hipSuccess;
  hipLaunchKernelGGL(mine_root_size, dim3((hi - lo + 255) / 256), dim3(256), 0, st, a, rsize, lo, hi);
  return hipGetLastError();
}
hipError_t launch_mine_pos(const MineArgs &a, int level, int pbeg, int pend, const uint32_t *rpos, hipStream_t st) {
  if (pend <= pbeg) return hipSuccess;
  hipLaunchKernelGGL(mine_pos, dim3((pend - pbeg + 255) / 256), dim3(256), 0, st, a, level, pbeg, pend, rpos);
  return hipGetLastError();
}
hipError_t launch_mine_emit(const MineArgs &a, const int *lev_begin, int maxlev, int n, const PatternTable &t,
                            hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mine_emit, dim3((n + 255) / 256), dim3(256), 0, st, a, lev_begin, maxlev, t);
  return hipGetLastError();
}
hipError_t launch_mine_succ_level(const MineArgs &a, const PatternTable &t, int level, int cb, int ce, int32_t node_lo,
                                  int *err, hipStream_t st) {
  const long long n = (long long)(ce - cb) * a.amax;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mine_succ_level, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, t, level, cb, ce, node_lo,
                     err);
  return hipGetLastError();
}

// Test hook of the bounded collective wait (hmc_debug_stall): one wavefront
// that keeps the context stream busy for `ticks` of the device's
// constant-rate wall clock, then exits — every launch ends on its own.
__global__ void __launch_bounds__(64) stall_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

hipError_t launch_stall(double ms, hipStream_t st) {
  if (!(ms > 0) || ms > 60000) return hipErrorInvalidValue;
  int dev = 0, khz = 0;
  hipError_t e;
  if ((e = hipGetDevice(&dev)) || (e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev))) return e;
  if (khz <= 0) khz = 100000;
  hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, st, (long long)(ms * khz));
  return hipGetLastError();
}

}  // namespace hmc
