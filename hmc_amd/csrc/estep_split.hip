// estep_split.hip — the E-step of the HaploModel EM as two passes on CDNA4.
//
// HaploBuilder::resolve (HaploBuilder.cpp:35-126) mixes two kinds of work per
// locus: the *structure* — which HaploPair states exist, created in which
// order, and which predecessor contributes to which state in which order
// (extendAll/extend/addHaploPair, :226-261, keyed by m_best_pair) — and the
// *values* — forward likelihoods and the k-best link lists (HaploPair.cpp:35-89).
// The structure only depends on pattern ids and on `forward_likelihood() > 0`
// (extend, :237), which holds unless a likelihood underflows to zero.  So:
//
//   pass 1, estep_structure — one wavefront per individual walks the loci with
//     the integer work only: successor gathers, the (id_a, id_b) key table in
//     LDS, creation-order state numbering, per-state contribution lists in add
//     order, list lengths min(S, sum of predecessor lengths), and the states
//     whose adds overflow S ("chains", sorted longest first).  It writes one
//     structure record per locus.
//   pass 2, estep_values — W wavefronts per individual replay the records:
//     a thread per state runs the constructor, the in-place appends and the
//     ordered forward sum; the adds that overflow S run as chains on 2S-lane
//     segments with the libstdc++-exact segmented nth_element (coop_select.hpp),
//     each segment pulling the next chain from a block queue.  No hashing, no
//     gathers of the pattern table, two barriers per locus.
//
// If pass 2 meets a forward likelihood of 0 before the last locus (the
// reference would skip that pair) the individual is flagged EST_NEEDS_EXACT
// and the host re-runs only it through pass 1 in prune mode (each new state's
// forward sum in add order, extend()'s test `forward_likelihood() > 0`,
// HaploBuilder.cpp:237) and then pass 2 again, in the same store regions.
// The fused kernel (estep.hip) is a variants-library option only.
#include "hmc_internal.hpp"
#include "select.hpp"
#include "coop_select.hpp"
#include "estep_common.hpp"
#include "value_front.hpp"

namespace hmc {

namespace {

constexpr unsigned long long REC_CHUNK = 1ull << 16;  // record words per bump allocation
constexpr int NBUCKET = 32;                           // chain-length buckets (longest first)

// An array whose entries [0, fc) live in LDS and [fc, ..) in HBM scratch.
template <class T>
struct Tier {
  T *l, *g;
  int fc;
  __device__ T *at(int t) const { return t < fc ? l + t : g + (t - fc); }
};

// Visibility of LDS and global (HBM-tier) writes between the lanes of the
// wave that forms the whole workgroup of pass 1.
__device__ inline void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ inline int wave_incl_scan(int x) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x;
}

// ============================================================ pass 1 ======

// Frontier of pass 1 (m_haplopairs[i] as pattern-id pairs): per state the
// pattern ids, list length nl, key slot, running sum of predecessor list
// lengths, and the first contribution's position in the record.  Six u32
// arrays; entries [0, fc) in LDS, the rest in HBM scratch.
enum { F_LO, F_HI, F_NL, F_SLOT, F_NS, F_CB, F_NARR };
struct IdFront {
  uint32_t *l, *g;
  int fc, gs;  // LDS entries per array, HBM words per array
  __device__ uint32_t *at(int k, int t) const { return t < fc ? l + k * fc + t : g + (size_t)k * gs + (t - fc); }
};

// The frontiers of estep_structure: LO, HI and NL alternate between the two
// (the previous frontier's are read, the new one's written); SLOT, NS and CB
// belong to the new frontier only while its locus is built (key slots,
// predecessor-length sums, first contributions), so one set serves both and
// a state takes 36 bytes of LDS instead of 48 — at two 4-wave blocks per CU
// the LDS tier holds 528 states instead of 432 (cfg 3's E1: 468 on average).
struct IdFront1 {
  uint32_t *l, *g, *ls, *gsh;
  int fc, gs;
  __device__ uint32_t *at(int k, int t) const {
    if (k < F_SLOT) return t < fc ? l + k * fc + t : g + (size_t)k * gs + (t - fc);
    return t < fc ? ls + (k - F_SLOT) * fc + t : gsh + (size_t)(k - F_SLOT) * gs + (t - fc);
  }
};

// m_best_pair: slots < hc in LDS, the rest in the HBM table.  Per slot the
// key, one 64-bit lane mask per wavefront of the block (the contributions of
// the current chunk that carry the key), the count of contributions so far
// and the state the key created.
__host__ __device__ inline int k1_slot_bytes(int nw) { return 16 + 8 * nw; }
// estep_structure with up to 4 waves per block keeps no lane masks in the
// slots: the first contribution of a chunk to claim a slot writes
// (chunk tag << 10 | its thread index) into the slot's tag word, and the chunk's
// lane masks for that key go to an LDS array indexed by that thread index
// ([NT][NW] words, zeroed again by the key's first contribution).  A slot is
// then 20 bytes instead of 16 + 8 NW (48 at 4 waves): at two 4-wave blocks
// per CU the LDS table holds 2 048 keys instead of 1 024 for the same LDS, so
// the probe sequences stay short and few keys reach the HBM tier (cfg 3's E1:
// 20 of 700 contributions per locus did, and a wave with one such lane waits
// for two global round trips per chunk).  16-wave blocks (cfg 4's small E1
// groups) keep the masks in the slots: their [NT][NW] array would be 128 KB.
__host__ __device__ inline bool k1_lid(int nw) { return nw <= 4; }
__host__ __device__ inline int k1v_slot_bytes(int nw) { return k1_lid(nw) ? 20 : k1_slot_bytes(nw); }
constexpr int LID_BITS = 10;  // thread index (NT <= 1024) in a tag word; the chunk tag above it
struct K1Keys {
  unsigned char *l, *g;
  int hc, hcap, nw;
  __device__ unsigned long long *key(uint32_t s) const {
    return s < (uint32_t)hc ? (unsigned long long *)l + s : (unsigned long long *)g + (s - hc);
  }
  __device__ unsigned long long *lanes(uint32_t s) const {  // [nw] words
    return s < (uint32_t)hc ? (unsigned long long *)(l + (size_t)hc * 8) + (size_t)s * nw
                            : (unsigned long long *)(g + (size_t)hcap * 8) + (size_t)(s - hc) * nw;
  }
  __device__ uint32_t *cnt(uint32_t s) const {
    return s < (uint32_t)hc ? (uint32_t *)(l + (size_t)hc * (8 + 8 * nw)) + s
                            : (uint32_t *)(g + (size_t)hcap * (8 + 8 * nw)) + (s - hc);
  }
  __device__ uint32_t *state(uint32_t s) const {
    return s < (uint32_t)hc ? (uint32_t *)(l + (size_t)hc * (12 + 8 * nw)) + s
                            : (uint32_t *)(g + (size_t)hcap * (12 + 8 * nw)) + (s - hc);
  }
  __device__ uint32_t *tag(uint32_t s) const {  // estep_structure's local-id layout (nw = 0) only
    return s < (uint32_t)hc ? (uint32_t *)(l + (size_t)hc * (16 + 8 * nw)) + s
                            : (uint32_t *)(g + (size_t)hcap * (16 + 8 * nw)) + (s - hc);
  }
};

// The locus's contributions in extendAll order: (pred | reversed), state, rank.
enum { C_SR, C_ST, C_RK };
struct CTier {
  uint32_t *l, *g;
  int cc, ccap;
  __device__ uint32_t *at(int k, int c) const {
    return c < cc ? l + k * cc + c : g + (size_t)k * ccap + (c - cc);
  }
};

struct K1Plan {
  int o_pairs, o_bucket, o_red, o_front[2], o_fsh, o_keys, o_lanes, o_contrib, bytes;
};

// npm: allele pairs of a fully missing locus, amax (amax + 1) / 2
__host__ __device__ inline K1Plan k1_plan(int fc, int hc, int cc, int npm, int nw) {
  K1Plan p;
  int o = 0;
  auto take = [&](int bytes) { int r = o; o += (bytes + 15) & ~15; return r; };
  p.o_pairs = take((npm + 2) * 4 + 3 * npm);
  p.o_bucket = take(NBUCKET * 4);
  p.o_red = take((2 * nw + 4) * 8);
  p.o_front[0] = take(F_SLOT * fc * 4);  // LO, HI, NL of one frontier
  p.o_front[1] = take(F_SLOT * fc * 4);
  p.o_fsh = take((F_NARR - F_SLOT) * fc * 4);  // SLOT, NS, CB of the one being built
  p.o_keys = take(hc * k1v_slot_bytes(nw));
  p.o_lanes = take(k1_lid(nw) ? 64 * nw * nw * 8 : 0);
  p.o_contrib = take(3 * cc * 4);
  p.bytes = o;
  return p;
}

// Insert-or-find of the successor key: the first free or matching slot of its
// LDS probe sequence, else the HBM table.  Slots never empty during a locus.
__device__ inline uint32_t k1_key_slot(const K1Keys &K, unsigned long long key, uint32_t h0, int probes = PROBE_LDS) {
  unsigned long long *lk = (unsigned long long *)K.l, *gk = (unsigned long long *)K.g;
  uint32_t h = h0 & (uint32_t)(K.hc - 1);
  for (int p = 0; p < probes; ++p) {
    const unsigned long long prev = atomicCAS(&lk[h], KEY_EMPTY, key);
    if (prev == KEY_EMPTY || prev == key) return h;
    h = (h + (uint32_t)p + 1u) & (uint32_t)(K.hc - 1);  // triangular steps: no primary clusters
  }
  const uint32_t gmask = (uint32_t)K.hcap - 1u;
  uint32_t g = (h0 * 0x9E3779B1u) & gmask;
  while (true) {
    const unsigned long long prev = atomicCAS(&gk[g], KEY_EMPTY, key);
    if (prev == KEY_EMPTY || prev == key) return (uint32_t)K.hc + g;
    g = (g + 1) & gmask;
  }
}

// As k1_key_slot, but NONE when the HBM table is full (estep_structure2
// inserts a whole locus's keys before it counts the new states, so a locus
// with more distinct successor pairs than hcap slots must not probe forever).
__device__ inline uint32_t k2_key_slot(const K1Keys &K, unsigned long long key, uint32_t h0) {
  unsigned long long *lk = (unsigned long long *)K.l, *gk = (unsigned long long *)K.g;
  uint32_t h = h0 & (uint32_t)(K.hc - 1);
  for (int p = 0; p < PROBE_LDS; ++p) {
    const unsigned long long prev = atomicCAS(&lk[h], KEY_EMPTY, key);
    if (prev == KEY_EMPTY || prev == key) return h;
    h = (h + 1) & (uint32_t)(K.hc - 1);
  }
  const uint32_t gmask = (uint32_t)K.hcap - 1u;
  uint32_t g = (h0 * 0x9E3779B1u) & gmask;
  for (int p = 0; p < K.hcap; ++p) {
    const unsigned long long prev = atomicCAS(&gk[g], KEY_EMPTY, key);
    if (prev == KEY_EMPTY || prev == key) return (uint32_t)K.hc + g;
    g = (g + 1) & gmask;
  }
  return 0xFFFFFFFFu;
}

__device__ inline unsigned long long ld_acq(unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline uint32_t ld_acq(uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr unsigned long long REC_NONE = ~0ull;

// Block-wide helpers of pass 1 (NW wavefronts per individual; NW == 1 keeps
// the single-wave hand-offs: LDS order within a wave, lane shuffles).
template <int NW>
struct Blk {
  int *red;  // LDS: [NW] wave totals, [NW] second, [8] broadcast words
  int tid, lane, wv;
  __device__ void sync() const {
    if (NW == 1) wsync();
    else __syncthreads();
  }
  // exclusive scan of x over the block in thread order; *total = the sum
  __device__ int scan(int x, int *total) const {
    const int incl = wave_incl_scan(x);
    if (NW == 1) {
      *total = __shfl(incl, 63);
      return incl - x;
    }
    if (lane == 63) red[wv] = incl;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int v = red[w];
      off += w < wv ? v : 0;
      tot += v;
    }
    __syncthreads();
    *total = tot;
    return off + incl - x;
  }
  __device__ unsigned long long reduce_u64(unsigned long long x) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (NW == 1) return x;
    unsigned long long *r = (unsigned long long *)(red + 2 * NW + 8);
    if (lane == 0) r[wv] = x;
    __syncthreads();
    unsigned long long t = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += r[w];
    __syncthreads();
    return t;
  }
  // thread 0's value, to every thread
  __device__ int bcast(int v) const {
    if (NW == 1) return __shfl(v, 0);
    if (tid == 0) red[2 * NW] = v;
    __syncthreads();
    const int r = red[2 * NW];
    __syncthreads();
    return r;
  }
  __device__ unsigned long long bcast64(unsigned long long v) const {
    const unsigned lo = (unsigned)bcast((int)(uint32_t)v), hi = (unsigned)bcast((int)(uint32_t)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
  }
};

// Next record of `words` words, or REC_NONE when it does not fit: the store
// (bump allocator) or the individual's own region (rec_base / rec_size).
// Block-uniform call.
template <int NW>
__device__ inline unsigned long long rec_alloc(const StructArgs &a, const Blk<NW> &B, unsigned long long &cur,
                                               unsigned long long &end, unsigned long long words) {
  words = (words + 1) & ~1ull;  // records start on even words (8-byte aligned tpv)
  if (cur + words > end) {
    if (a.rec_base) return REC_NONE;  // past this individual's region
    const unsigned long long take = words > REC_CHUNK ? words : REC_CHUNK;
    unsigned long long base = 0;
    if (B.tid == 0) base = atomicAdd(a.rec_cursor, take);
    base = B.bcast64(base);
    cur = base;
    end = base + take;
  }
  const unsigned long long off = cur;
  if (off + words > a.rec_cap) return REC_NONE;
  cur += words;
  return off;
}

}  // namespace

__host__ __device__ inline size_t k1_front_words(int fcap) { return al256((size_t)fcap * 4) / 4; }

size_t estep_s1_scratch_bytes(int fcap, int hcap, int ccap, int nw, bool prune) {
  return 2 * al256(F_NARR * k1_front_words(fcap) * 4) + al256((size_t)hcap * k1v_slot_bytes(nw)) +
         al256((size_t)ccap * 12) + (prune ? 2 * al256((size_t)fcap * 8) : 0);
}
size_t estep_s1_lds_bytes(int fc, int hc, int cc, int amax, int nw) {
  return (size_t)k1_plan(fc, hc, cc, amax * (amax + 1) / 2, nw).bytes;
}

// Diagnostic build only (-DHMC_STAMPS): thread 0's shader cycles per phase of
// the structure pass (each stamp drains the wave's memory counters), plus
// counters; summed over individuals into a.stamps[16].
#ifdef HMC_STAMPS
#define S1_T0 unsigned long long s1t = __builtin_amdgcn_s_memtime(), s1acc[20] = {};
#define S1_ST(k)                                                   \
  do {                                                             \
    __builtin_amdgcn_s_waitcnt(0);                                 \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();    \
    s1acc[k] += t1 - s1t;                                          \
    s1t = t1;                                                      \
  } while (0)
#define S1_CNT(k, v) s1acc[k] += (unsigned long long)(v)
#define S1_FLUSH                                                   \
  if (a.stamps && tid == 0)                                        \
    for (int k = 0; k < 20; ++k) atomicAdd(&a.stamps[k], s1acc[k]);
#else
#define S1_T0
#define S1_ST(k) do { } while (0)
#define S1_CNT(k, v) do { } while (0)
#define S1_FLUSH
#endif

// NW wavefronts per individual: one wave (many individuals per CU) or four
// (the first E-step's large frontiers: 4x the LDS tier and 4x the
// contributions per step of the extendAll scan).
template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(3))) void estep_structure(StructArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr int NT = 64 * NW;
  S1_T0
  const int npm = a.pan.amax * (a.pan.amax + 1) / 2;
  const K1Plan plan = k1_plan(a.lds_fc, a.lds_hc, a.lds_cc, npm, NW);
  const int tid = threadIdx.x, lane = lane_id(), wv = tid / WAVE;
  const uint64_t lt = lanemask_lt();
  const Blk<NW> B{(int *)(smem + plan.o_red), tid, lane, wv};
  const int S = a.S, L = a.pan.L, amax = a.pan.amax, hl = a.mod.head_len;
  // locus window of record indices [wlo, whi) (classic: the head to L)
  const int wlo = a.w.hi > 0 ? a.w.lo : hl, whi = a.w.hi > 0 ? a.w.hi : L + 1;
  const bool from_ck = wlo > hl;
  // the pattern table in end-locus order when the host built it (gmodel.hip):
  // frontier states carry g instead of pattern ids, and one locus's lookups
  // fall in one block of the table
  const bool gsp = a.mod.gsucc != nullptr;
  const uint32_t *SUCC = gsp ? a.mod.gsucc : a.mod.succ;
  const double *TP = gsp ? a.mod.gtp : a.mod.tp;
  const uint8_t *LAST = gsp ? a.mod.glast : a.mod.last;
  auto to_g = [&](uint32_t id) -> uint32_t { return gsp ? a.mod.ginv[id] : id; };
  auto to_id = [&](uint32_t gv) -> uint32_t { return gsp ? a.mod.gid[gv] : gv; };
  int *pr_off = (int *)(smem + plan.o_pairs);  // [npm+2]; [npm+1] = npairs
  uint8_t *pr_x = (uint8_t *)(pr_off + npm + 2);
  uint8_t *pr_y = pr_x + npm;
  uint8_t *pr_o = pr_y + npm;
  int *bucket = (int *)(smem + plan.o_bucket);

  char *sp = a.scratch + (size_t)blockIdx.x * a.scratch_stride;
  const int gs = (int)k1_front_words(a.fcap);
  // HBM tiers: the first region's arrays 0-2 (LO, HI, NL) and 3-5 (the shared
  // SLOT, NS, CB), the second region's arrays 0-2
  uint32_t *const gsh = (uint32_t *)sp + (size_t)F_SLOT * gs;
  uint32_t *const lsh = (uint32_t *)(smem + plan.o_fsh);
  const IdFront1 FA{(uint32_t *)(smem + plan.o_front[0]), (uint32_t *)sp, lsh, gsh, a.lds_fc, gs};
  sp += al256(F_NARR * (size_t)gs * 4);
  const IdFront1 FB{(uint32_t *)(smem + plan.o_front[1]), (uint32_t *)sp, lsh, gsh, a.lds_fc, gs};
  sp += al256(F_NARR * (size_t)gs * 4);
  constexpr bool LID = NW <= 4;  // k1_lid: lane masks by local id, not per slot
  const K1Keys K{smem + plan.o_keys, (unsigned char *)sp, a.lds_hc, a.hcap, LID ? 0 : NW};
  sp += al256((size_t)a.hcap * k1v_slot_bytes(NW));
  unsigned long long *const lanes = (unsigned long long *)(smem + plan.o_lanes);  // LID: [NT][NW]
  const CTier CT{(uint32_t *)(smem + plan.o_contrib), (uint32_t *)sp, a.lds_cc, a.ccap};
  sp += al256((size_t)a.ccap * 12);
  // prune: forward likelihoods of the previous and the current frontier (HBM)
  double *fwx = a.prune ? (double *)sp : nullptr, *fwy = a.prune ? (double *)sp + al256((size_t)a.fcap * 8) / 8 : nullptr;
  // the key table's plainly stored fields; with several waves the HBM tier is
  // read past the vector L1 (another wave of the block may have written it)
  auto kcnt = [&](uint32_t sl) -> uint32_t {
    return (NW == 1 || sl < (uint32_t)K.hc) ? *K.cnt(sl) : ld_acq(K.cnt(sl));
  };
  auto kstate = [&](uint32_t sl) -> uint32_t {
    return (NW == 1 || sl < (uint32_t)K.hc) ? *K.state(sl) : ld_acq(K.state(sl));
  };

  auto reset_tables = [&]() {
    for (int h = tid; h < K.hc + a.hcap; h += NT) {
      *K.key(h) = KEY_EMPTY;
      if constexpr (LID) *K.tag(h) = 0u;
      else
        for (int w = 0; w < NW; ++w) K.lanes(h)[w] = 0ull;
      *K.cnt(h) = 0;
    }
    if constexpr (LID)
      for (int w = tid; w < NT * NW; w += NT) lanes[w] = 0ull;
    __threadfence();
    B.sync();
  };
  reset_tables();

  // individuals are taken from the heaviest-first order list one at a time as
  // blocks finish (longest-processing-time-first), not round-robin
  auto next_q = [&]() -> int {
    int t = 0;
    if (tid == 0) t = atomicAdd(a.next_q, 1);
    return B.bcast(t) + (int)gridDim.x;
  };
  for (int q = blockIdx.x; q < a.n_order; q = next_q()) {
    const int bi = a.order[q];
    const int gi = a.indiv_begin + bi;
    const uchar2 *g = a.pan.geno_im + (size_t)gi * L;
    unsigned long long *roff = a.rec_off + (size_t)bi * (L + 1);
    int status = EST_OK;
    unsigned long long re = 0;  // per thread; summed at the end
    // records: this individual's reserved region, else the bump allocator; once
    // a record does not fit, `counting` keeps the walk going without writes
    unsigned long long rcur = a.rec_base ? a.rec_base[bi] : 0;
    unsigned long long rend = a.rec_base ? (a.rec_size ? rcur + a.rec_size[bi] : ~0ull) : 0;
    bool counting = false;
    unsigned long long rneed = 0, tneed = 0;  // exact record / trace words (block-uniform)
    IdFront1 X = FA, Y = FB;

    // ---- initHeadList (HaploBuilder.cpp:153-224) ----------------------------
    // head_len == 1 on the device; longer heads from the host's list.  A locus
    // window after the first starts from its checkpoint (the frontier after
    // record index wlo - 1) instead.
    int Fp0 = 0, st0 = EST_OK;
    if (from_ck) {
      const uint32_t *ck = a.w.ck_in + a.w.ck_off[(size_t)bi * (a.w.nwin + 1) + a.w.win];
      Fp0 = (int)ck[0];
      if (Fp0 > a.fcap) {
        st0 = EST_OVERFLOW_FRONTIER;
      } else {
        for (int t = tid; t < Fp0; t += NT) {
          *X.at(F_LO, t) = ck[2 + t];
          *X.at(F_HI, t) = ck[2 + Fp0 + t];
          *X.at(F_NL, t) = ck[2 + 2 * Fp0 + t];
        }
      }
    }
    if (!from_ck && tid == 0 && hl > 1) {
      const int li = gi - a.mod.hf_base;
      st0 = a.mod.hf_status[li];
      for (uint32_t t = a.mod.hf_off[li]; t < a.mod.hf_off[li + 1] && st0 == EST_OK; ++t) {
        if (Fp0 >= a.fcap) { st0 = EST_OVERFLOW_FRONTIER; break; }
        *X.at(F_LO, Fp0) = to_g(a.mod.hf_pairs[2 * t]);
        *X.at(F_HI, Fp0) = to_g(a.mod.hf_pairs[2 * t + 1]);
        *X.at(F_NL, Fp0) = 1;
        ++Fp0;
      }
    }
    if (!from_ck && tid == 0 && hl == 1) {
      const uchar2 g0 = g[0];
      const bool m0 = g0.x == MISSING, m1 = g0.y == MISSING;
      for (int hix = 0; hix < a.mod.n_head; ++hix) {
        const uint32_t head = a.mod.head_ids[hix];
        const uint8_t ah = a.mod.last[head];
        if (!(m0 || m1 || g0.x == ah || g0.y == ah)) continue;  // head->isMatch(genotype)
        // the complementary alleles in order (no private array: it would take
        // registers from the whole kernel)
        const bool hasAllele = g0.x == ah || g0.y == ah;
        const bool expand = (m0 && m1) || ((m0 || m1) && hasAllele);
        const int nx = expand ? (int)a.pan.anum[0] : 1;
        for (int k = 0; k < nx; ++k) {
          uint32_t xk;
          if (expand) {
            if (!(a.pan.afreq[k] > 0)) continue;
            xk = (uint32_t)k;
          } else {
            xk = (!m0 && !m1 && g0.x != g0.y) ? ((ah == g0.x) ? g0.y : g0.x)
                                              : g0.x;  // may be missing: resolved like findLongestMatchPattern
          }
          const uint32_t hq = xk == MISSING ? a.mod.head_pat0[amax] : a.mod.head_pat0[xk];
          if (hq == NONE) { st0 = EST_NO_HEAD_PATTERN; break; }
          if (hq < head) continue;  // hp->id() >= head->id()
          if (Fp0 >= a.fcap) { st0 = EST_OVERFLOW_FRONTIER; break; }
          *X.at(F_LO, Fp0) = to_g(head);  // (head <= hq by id, so by g: both end at locus 0)
          *X.at(F_HI, Fp0) = to_g(hq);
          *X.at(F_NL, Fp0) = 1;
          ++Fp0;
        }
        if (st0 != EST_OK) break;
      }
    }
    int Fp = B.bcast(Fp0);
    status = B.bcast(st0);
    int fbig = Fp;  // the head frontier counts too: the value pass sizes its HBM tier by this
    B.sync();
    if (status == EST_OK && !from_ck) {
      const unsigned long long words = 4 + 4ull * Fp + 1 + (a.exact ? 2ull * Fp : 0ull);
      rneed += (words + 1) & ~1ull;
      tneed += a.exact ? 4ull * Fp + 2 : trace_locus_words((unsigned long long)Fp, S);
      const unsigned long long o = rec_alloc<NW>(a, B, rcur, rend, words);
      if (o == REC_NONE) {
        counting = true;
        if (tid == 0) re += (unsigned long long)Fp;
      } else {
        uint32_t *R = a.rec + o;
        double *Rtp = (double *)(R + 4);
        uint32_t *Rhd = R + 4 + 2 * Fp, *Rcb = Rhd + Fp;
        for (int t = tid; t < Fp; t += NT) {
          const uint32_t lo = *X.at(F_LO, t), hi = *X.at(F_HI, t);
          Rtp[t] = a.mod.freq[to_id(lo)] * a.mod.freq[to_id(hi)];  // HaploPair.cpp:27
          Rhd[t] = (uint32_t)LAST[lo] | (uint32_t)LAST[hi] << 8 | 1u << 16 | (lo == hi ? 1u << 24 : 0u);
          Rcb[t] = 0;
          if (a.exact) {  // head pairs' pattern ids (their alleles before head_len)
            Rcb[Fp + 1 + t] = to_id(lo);
            Rcb[2 * Fp + 1 + t] = to_id(hi);
          }
        }
        if (tid == 0) {
          Rcb[Fp] = 0;
          R[0] = (uint32_t)Fp;
          R[1] = 0;
          R[2] = 0;
          R[3] = 0;
          roff[hl] = o;
          re += (unsigned long long)Fp;
        }
      }
    }

    if (a.prune && status == EST_OK) {  // head pairs' forward likelihoods (HaploPair.cpp:27-32)
      for (int t = tid; t < Fp; t += NT) {
        const uint32_t lo = *X.at(F_LO, t), hi = *X.at(F_HI, t);
        const double tpv = a.mod.freq[to_id(lo)] * a.mod.freq[to_id(hi)];
        fwx[t] = lo == hi ? tpv : tpv * 2.0;
      }
      B.sync();
    }
    // ---- structure of the forward over loci (HaploBuilder.cpp:47-82) -------
    S1_ST(5);
    for (int i = from_ck ? wlo - 1 : hl; i < whi - 1 && status == EST_OK; ++i) {
      if (Fp == 0) { status = EST_UNRESOLVED; break; }
      const uchar2 gg = g[i];
      if (tid == 0) {  // allele-pair list in extendAll call order
        const double *af = a.pan.afreq + (size_t)i * amax;
        const int an = a.pan.anum[i];
        int np = 0;
        auto push = [&](int x, int y) { pr_x[np] = (uint8_t)x; pr_y[np] = (uint8_t)y; pr_o[np] = x == y ? 1 : 2; ++np; };
        if (gg.x == MISSING && gg.y == MISSING) {
          for (int j = 0; j < an; ++j)
            if (af[j] > 0)
              for (int k = j; k < an; ++k)
                if (af[k] > 0) push(j, k);
        } else if (gg.x == MISSING) {
          for (int j = 0; j < an; ++j)
            if (af[j] > 0) push(j, gg.y);
        } else if (gg.y == MISSING) {
          for (int j = 0; j < an; ++j)
            if (af[j] > 0) push(j, gg.x);
        } else {
          push(gg.x, gg.y);
        }
        int off = 0;
        for (int p = 0; p < np; ++p) { pr_off[p] = off; off += Fp * pr_o[p]; }
        pr_off[np] = off;
        pr_off[npm + 1] = np;
      }
      B.sync();
      const int npairs = pr_off[npm + 1];
      const int C = pr_off[npairs];
      if (C > a.ccap) { status = EST_OVERFLOW_CONTRIB; break; }
      // (LID: chunk tags must stay below 2^(32 - LID_BITS); the host then fails loudly)
      if (NW <= 4 && (long long)C >= ((1ll << (32 - LID_BITS)) - 1) * NT) { status = EST_OVERFLOW_CONTRIB; break; }
      S1_ST(0);
      S1_CNT(8, C);
      S1_CNT(9, Fp);
      S1_CNT(13, 1);
      int Fn = 0;
      // successor gathers of up to GB chunks issued together (one exposed
      // latency per GB*NT contributions), then the chunks' keys in order
      constexpr int GB = 4;
      uint32_t g_sa[GB], g_sb[GB], g_s[GB];
      for (int c0 = 0; c0 < C; c0 += NT) {
        const int c = c0 + tid;
        const int gq = (c0 / NT) % GB;
        if (gq == 0) {
#pragma unroll
          for (int q = 0; q < GB; ++q) {
            const int cq = c + q * NT;
            g_sa[q] = g_sb[q] = NONE;
            g_s[q] = 0;
            if (cq < C) {
              int p = 0;
              while (p + 1 < npairs && cq >= pr_off[p + 1]) ++p;
              const int local = cq - pr_off[p];
              const int o = pr_o[p] == 2 ? (local & 1) : 0;
              g_s[q] = pr_o[p] == 2 ? (uint32_t)(local >> 1) : (uint32_t)local;
              const uint32_t x = o ? pr_y[p] : pr_x[p];
              const uint32_t y = o ? pr_x[p] : pr_y[p];
              g_sa[q] = SUCC[(size_t)*X.at(F_LO, (int)g_s[q]) * amax + x];
              g_sb[q] = SUCC[(size_t)*X.at(F_HI, (int)g_s[q]) * amax + y];
            }
          }
        }
        S1_ST(14);
        uint32_t sa = g_sa[0], sb = g_sb[0], s = g_s[0];
#pragma unroll
        for (int q = 1; q < GB; ++q)
          if (gq == q) {
            sa = g_sa[q];
            sb = g_sb[q];
            s = g_s[q];
          }
        bool valid = c < C;
        uint32_t lo = 0, hi = 0, slot = 0;
        bool rev = false;
        if (valid) {
          // extend(): a pair whose forward likelihood is 0 is not extended
          // (HaploBuilder.cpp:237), then both successors must exist (:239-243)
          valid = sa != NONE && sb != NONE && (!a.prune || fwx[s] > 0.0);
          rev = sa > sb;  // addHaploPair: id_a > id_b -> swap, reversed
          lo = rev ? sb : sa;
          hi = rev ? sa : sb;
        }
        // this key's lane masks for the chunk: in the slot, or (LID) in the
        // lanes row of the slot's first claimant in this chunk
        unsigned long long *lw = nullptr;
        bool lw_lds = true;
        if (valid) {
          slot = k1_key_slot(K, ((unsigned long long)lo << 32) | hi, key_hash(lo, hi), a.probe_lds);
          if constexpr (LID) {
            const uint32_t ctag = (uint32_t)(c0 / NT) + 1u;  // < 2^22: C <= ccap (EST_OVERFLOW_CONTRIB above)
            uint32_t *tg = K.tag(slot);
            uint32_t w = slot < (uint32_t)K.hc ? *tg : ld_acq(tg);
            while ((w >> LID_BITS) != ctag) {
              const uint32_t mine = ctag << LID_BITS | (uint32_t)tid;
              const uint32_t prev = atomicCAS(tg, w, mine);
              w = prev == w ? mine : prev;
            }
            lw = lanes + (size_t)(w & ((1u << LID_BITS) - 1u)) * NW;
          } else {
            lw = K.lanes(slot);
            lw_lds = slot < (uint32_t)K.hc;
          }
          atomicOr(lw + wv, 1ull << lane);
        }
        S1_CNT(10, 1);
        S1_CNT(11, __popcll(__ballot(valid && slot >= (uint32_t)K.hc)));
        S1_ST(15);
        B.sync();
        // this contribution's rank among the chunk's ones with the same key
        // (waves before it, then lanes below it) and the chunk's count
        int li = 0, gsz = 0;
        uint32_t cnt0 = 0;
        if (valid) {
#pragma unroll 4
          for (int w = 0; w < NW; ++w) {
            const uint64_t m = lw_lds ? lw[w] : ld_acq(lw + w);
            li += w < wv ? __popcll(m) : (w == wv ? __popcll(m & lt) : 0);
            gsz += __popcll(m);
          }
          cnt0 = kcnt(slot);
        }
        B.sync();
        S1_ST(16);
        if (valid && li == 0) {
          *K.cnt(slot) = cnt0 + (uint32_t)gsz;
#pragma unroll 4
          for (int w = 0; w < NW; ++w) lw[w] = 0ull;
        }
        const bool is_new = valid && cnt0 == 0 && li == 0;
        int nnew = 0;
        const int rk_new = B.scan(is_new ? 1 : 0, &nnew);
        S1_ST(17);
        if (Fn + nnew > a.fcap) { status = EST_OVERFLOW_FRONTIER; break; }
        uint32_t st = 0;
        if (is_new) {
          st = (uint32_t)(Fn + rk_new);
          *K.state(slot) = st;
          *Y.at(F_LO, (int)st) = lo;
          *Y.at(F_HI, (int)st) = hi;
          *Y.at(F_SLOT, (int)st) = slot;
          *Y.at(F_NS, (int)st) = 0;
        }
        Fn += nnew;
        B.sync();
        if (valid && !is_new) st = kstate(slot);
        if (valid) atomicAdd(Y.at(F_NS, (int)st), *X.at(F_NL, (int)s));
        if (c < C) {
          *CT.at(C_SR, c) = cw_pack(s, rev);
          *CT.at(C_ST, c) = valid ? st : NONE;
          *CT.at(C_RK, c) = cnt0 + (uint32_t)li;
        }
        S1_ST(7);
      }
      if (status != EST_OK) break;
      if (Fn == 0) { status = EST_UNRESOLVED; break; }
      fbig = Fn > fbig ? Fn : fbig;
      B.sync();
      S1_ST(1);
      S1_CNT(12, Fn > X.fc ? Fn - X.fc : 0);

      // contributions per state -> first position (exclusive scan, creation order)
      int Cv = 0;
      for (int t0 = 0; t0 < Fn; t0 += NT) {
        const int t = t0 + tid;
        const int m = t < Fn ? (int)kcnt(*Y.at(F_SLOT, t)) : 0;
        int tot = 0;
        const int ex = B.scan(m, &tot);
        if (t < Fn) *Y.at(F_CB, t) = (uint32_t)(Cv + ex);
        Cv += tot;
      }
      S1_ST(18);
      const unsigned long long words =
          4 + 4ull * Fn + 1 + (unsigned long long)Cv + Fn + (a.exact ? (unsigned long long)C + npairs : 0ull);
      rneed += (words + 1) & ~1ull;
      tneed += a.exact ? 4ull * Fn + 2 : trace_locus_words((unsigned long long)Fn, S);
      const unsigned long long o = counting ? 0 : rec_alloc<NW>(a, B, rcur, rend, words);
      if (o == REC_NONE) counting = true;
      uint32_t *R = a.rec + (counting ? 0 : o);  // not dereferenced while counting
      double *Rtp = (double *)(R + 4);
      uint32_t *Rhd = R + 4 + 2 * Fn, *Rcb = Rhd + Fn, *Rct = Rcb + Fn + 1, *Rch = Rct + Cv;
      if (tid < NBUCKET) bucket[tid] = 0;
      B.sync();
      S1_ST(19);
      // per state: k-best list length min(S, sum of predecessor lengths) (the
      // adds keep S once they overflow, HaploPair.cpp:85-88), tp product, last
      // alleles; states whose lists overflow get a chain entry
      for (int t0 = 0; t0 < Fn; t0 += NT) {
        const int t = t0 + tid;
        if (t < Fn) {
          const uint32_t lo = *Y.at(F_LO, t), hi = *Y.at(F_HI, t);
          const uint32_t nsum = t < Y.fc ? *Y.at(F_NS, t) : ld_acq(Y.at(F_NS, t));
          const uint32_t nl = nsum < (uint32_t)S ? nsum : (uint32_t)S;
          *Y.at(F_NL, t) = nl;
          re += nl;
          if (!counting) {
            Rtp[t] = TP[lo] * TP[hi];  // m_transition_prob, HaploPair.cpp:42
            // bit 27: the state's adds overflow S (a chain; the dataflow value pass
            // takes the chains first, estep_df.hip)
            Rhd[t] = (uint32_t)LAST[lo] | (uint32_t)LAST[hi] << 8 | nl << 16 | (nsum > (uint32_t)S ? HDR_CHAIN : 0u);
            Rcb[t] = *Y.at(F_CB, t);
          }
          if (!counting && nsum > (uint32_t)S) {  // bucket 0 = most contributions
            const int m = (int)kcnt(*Y.at(F_SLOT, t));
            atomicAdd(&bucket[NBUCKET - 1 - (m - 1 < NBUCKET - 1 ? m - 1 : NBUCKET - 1)], 1);
          }
        }
      }
      B.sync();
      S1_ST(2);
      int nch = 0;
      {  // every wave scans the 32 bucket counts; wave 0 writes the offsets
        const int b = lane < NBUCKET ? bucket[lane] : 0;
        const int incl = wave_incl_scan(b);
        nch = __shfl(incl, 63);
        B.sync();
        if (wv == 0 && lane < NBUCKET) bucket[lane] = incl - b;
      }
      B.sync();
      for (int t0 = 0; t0 < Fn && !counting; t0 += NT) {
        const int t = t0 + tid;
        if (t < Fn) {
          const uint32_t nsum = t < Y.fc ? *Y.at(F_NS, t) : ld_acq(Y.at(F_NS, t));
          if (nsum > (uint32_t)S) {
            const int m = (int)kcnt(*Y.at(F_SLOT, t));
            const int pos = atomicAdd(&bucket[NBUCKET - 1 - (m - 1 < NBUCKET - 1 ? m - 1 : NBUCKET - 1)], 1);
            Rch[pos] = (uint32_t)t;
          }
        }
      }
      // contributions of each state in add order
      uint32_t *Rout = Rct + Cv + nch;  // exact: contributions in extendAll order, then pair orientations
      for (int c0 = 0; c0 < C && !counting; c0 += NT) {
        const int c = c0 + tid;
        if (c < C) {
          const uint32_t st = *CT.at(C_ST, c);
          const uint32_t w = *CT.at(C_SR, c);
          if (st != NONE) {
            const uint32_t ns = *X.at(F_NL, (int)cw_state(w));
            Rct[*Y.at(F_CB, (int)st) + *CT.at(C_RK, c)] = w | ns << 24;
          }
          if (a.exact)
            Rout[c] = st == NONE ? NONE
                                 : (st | (w & CW_REV) |
                                    xpair_index(LAST[*Y.at(F_LO, (int)st)], LAST[*Y.at(F_HI, (int)st)]) << XPAIR_SHIFT);
        }
      }
      if (a.exact && !counting)
        for (int p = tid; p < npairs; p += NT) Rout[C + p] = pr_o[p];
      if (tid == 0 && !counting) {
        Rcb[Fn] = (uint32_t)Cv;
        R[0] = (uint32_t)Fn;
        R[1] = (uint32_t)Cv;
        R[2] = (uint32_t)nch;
        // C <= EXACT_C_MAX (the host caps ccap in exact mode), npairs < 2^10 (amax <= 44 in exact mode)
        R[3] = a.exact ? (uint32_t)C << 10 | (uint32_t)npairs : 0u;
        roff[i + 1] = o;
      }
      S1_ST(3);
      if (a.prune) {  // the new states' forward likelihoods, in add order (HaploPair.cpp:42, :66)
        B.sync();
        for (int t = tid; t < Fn; t += NT) {
          double f = 1.0;  // counting (no records): sizes only, nothing pruned
          if (!counting) {
            const double tpv = Rtp[t];
            for (uint32_t r = Rcb[t]; r < Rcb[t + 1]; ++r) {
              const double v = fwx[cw_state(Rct[r])] * tpv;
              f = r == Rcb[t] ? v : f + v;
            }
          }
          fwy[t] = f;
        }
      }
      // m_best_pair.clear() for the next locus
      for (int t0 = 0; t0 < Fn; t0 += NT) {
        const int t = t0 + tid;
        if (t < Fn) {
          const uint32_t sl = *Y.at(F_SLOT, t);
          *K.key(sl) = KEY_EMPTY;
          *K.cnt(sl) = 0;
          if constexpr (LID) *K.tag(sl) = 0u;
        }
      }
      B.sync();
      const IdFront1 T = X;
      X = Y;
      Y = T;
      double *const ft = fwx;
      fwx = fwy;
      fwy = ft;
      Fp = Fn;
      S1_ST(4);
    }
    if (status == EST_OK && Fp == 0) status = EST_UNRESOLVED;
    // the window's last frontier is the next window's checkpoint (also while
    // counting: the frontier is exact, only the records were not stored)
    if (status == EST_OK && whi <= L && a.w.ck_write) {
      const unsigned long long words = ck_words((unsigned long long)Fp, S);
      unsigned long long o = 0;
      if (tid == 0) {
        o = atomicAdd(a.w.ck_cursor, words);
        if (o + words > a.w.ck_cap) o = REC_NONE;
        a.w.ck_off[(size_t)bi * (a.w.nwin + 1) + a.w.win + 1] = o;
      }
      o = B.bcast64(o);
      if (o == REC_NONE) {
        status = EST_OVERFLOW_CKPT;
      } else {
        uint32_t *ck = a.w.ck_out + o;
        if (tid == 0) {
          ck[0] = (uint32_t)Fp;
          ck[1] = 0;
        }
        for (int t = tid; t < Fp; t += NT) {
          ck[2 + t] = *X.at(F_LO, t);
          ck[2 + Fp + t] = *X.at(F_HI, t);
          ck[2 + 2 * Fp + t] = *X.at(F_NL, t);
        }
      }
    }
    if (counting && status != EST_OVERFLOW_FRONTIER && status != EST_OVERFLOW_CONTRIB && status != EST_NO_HEAD_PATTERN &&
        status != EST_OVERFLOW_CKPT)
      status = EST_OVERFLOW_REC;
    fbig = Fp > fbig ? Fp : fbig;
    if (status < 0) reset_tables();  // aborted mid-locus: keys may be left
    if (status == EST_OK && a.prune) status = EST_OK_PRUNED;
    re = B.reduce_u64(re);
    if (tid == 0) {
      a.rec_need[bi] = rneed;
      a.trace_need[bi] = tneed;
      a.status[bi] = status;
      if (a.re_mode == 0) a.re_count[bi] = re;
      else if (a.re_mode == 1) a.re_count[bi] += re;
      a.fmax[bi] = fbig;
      atomicMax(a.max_states, (unsigned)fbig);
    }
    S1_ST(6);
  }
  S1_FLUSH
}

#ifdef HMC_VARIANTS  // (estep_structure2: measured slower, the variants library only)
// ======================================================= pass 1, v2 ======
//
// The same structure records with fewer block-wide hand-offs per locus
// (estep_structure: ~26 barriers per locus, five per chunk of NT
// contributions, which the cfg 3 E1 stamps show as the pass's cost).  Each
// thread owns a contiguous run of the locus's contributions in extendAll
// order and a contiguous run of the new states, so creation order and each
// state's contribution order come from three block scans instead of a
// per-chunk ranking:
//   1. every contribution: successor key, insert-or-find its slot, and per
//      slot atomically: the first contribution (min), the count, the sum of
//      predecessor list lengths;
//   2. a contribution that is its slot's first creates a state: numbered by
//      an exclusive scan of those flags in contribution order (= the order in
//      which addHaploPair creates pairs, HaploBuilder.cpp:246-261);
//   3. states: first positions by an exclusive scan of their counts; a slot
//      with one contribution places it directly, the others append to their
//      state's segment and take as rank the number of members before them.
// Slot fields (K1Keys with nw = 2: the lane-mask words hold firstc, ns, fill).
__host__ __device__ inline K1Plan k2s_plan(int fc, int hc, int cc, int npm, int nw) {
  K1Plan p;
  int o = 0;
  auto take = [&](int bytes) { int r = o; o += (bytes + 15) & ~15; return r; };
  p.o_pairs = take((npm + 2) * 4 + 3 * npm);
  p.o_bucket = take(NBUCKET * 4);
  p.o_red = take((2 * nw + 8) * 4 + nw * 8 + 16);
  p.o_front[0] = take(F_NARR * fc * 4);
  p.o_front[1] = take(F_NARR * fc * 4);
  p.o_keys = take(hc * k1_slot_bytes(2));
  p.o_contrib = take(3 * cc * 4);
  p.bytes = o;
  return p;
}
size_t estep_s1v2_lds_bytes(int fc, int hc, int cc, int amax, int nw) {
  return (size_t)k2s_plan(fc, hc, cc, amax * (amax + 1) / 2, nw).bytes;
}

enum { C2_SR, C2_SL, C2_AUX };  // contribution: (pred | reversed), slot (NONE: no pair), segment scratch
constexpr uint32_t FIRST_NONE = 0xFFFFFFFFu;

template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(3))) void estep_structure2(StructArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr int NT = 64 * NW;
  const int npm = a.pan.amax * (a.pan.amax + 1) / 2;
  const K1Plan plan = k2s_plan(a.lds_fc, a.lds_hc, a.lds_cc, npm, NW);
  const int tid = threadIdx.x, lane = lane_id(), wv = tid / WAVE;
  const Blk<NW> B{(int *)(smem + plan.o_red), tid, lane, wv};
  const int S = a.S, L = a.pan.L, amax = a.pan.amax, hl = a.mod.head_len;
  int *pr_off = (int *)(smem + plan.o_pairs);  // [npm+2]; [npm+1] = npairs
  uint8_t *pr_x = (uint8_t *)(pr_off + npm + 2);
  uint8_t *pr_y = pr_x + npm;
  uint8_t *pr_o = pr_y + npm;
  int *bucket = (int *)(smem + plan.o_bucket);

  char *sp = a.scratch + (size_t)blockIdx.x * a.scratch_stride;
  const int gs = (int)k1_front_words(a.fcap);
  const IdFront FA{(uint32_t *)(smem + plan.o_front[0]), (uint32_t *)sp, a.lds_fc, gs};
  sp += al256(F_NARR * (size_t)gs * 4);
  const IdFront FB{(uint32_t *)(smem + plan.o_front[1]), (uint32_t *)sp, a.lds_fc, gs};
  sp += al256(F_NARR * (size_t)gs * 4);
  const K1Keys K{smem + plan.o_keys, (unsigned char *)sp, a.lds_hc, a.hcap, 2};
  sp += al256((size_t)a.hcap * k1_slot_bytes(2));
  const CTier CT{(uint32_t *)(smem + plan.o_contrib), (uint32_t *)sp, a.lds_cc, a.ccap};
  sp += al256((size_t)a.ccap * 12);
  double *fwx = a.prune ? (double *)sp : nullptr, *fwy = a.prune ? (double *)sp + al256((size_t)a.fcap * 8) / 8 : nullptr;
  // slot fields: atomically updated ones are read past the vector L1 in the HBM tier
  auto f_first = [&](uint32_t sl) { return (uint32_t *)K.lanes(sl); };
  auto f_ns = [&](uint32_t sl) { return (uint32_t *)K.lanes(sl) + 1; };
  auto f_fill = [&](uint32_t sl) { return (uint32_t *)K.lanes(sl) + 2; };
  auto rd = [&](uint32_t *p, uint32_t sl) -> uint32_t { return sl < (uint32_t)K.hc ? *p : ld_acq(p); };

  auto reset_tables = [&]() {
    for (int h = tid; h < K.hc + a.hcap; h += NT) {
      *K.key(h) = KEY_EMPTY;
      *f_first(h) = FIRST_NONE;
      *f_ns(h) = 0;
      *f_fill(h) = 0;
      *K.cnt(h) = 0;
    }
    __threadfence();
    B.sync();
  };
  reset_tables();

  auto next_q = [&]() -> int {
    int t = 0;
    if (tid == 0) t = atomicAdd(a.next_q, 1);
    return B.bcast(t) + (int)gridDim.x;
  };
  for (int q = blockIdx.x; q < a.n_order; q = next_q()) {
    const int bi = a.order[q];
    const int gi = a.indiv_begin + bi;
    const uchar2 *g = a.pan.geno_im + (size_t)gi * L;
    unsigned long long *roff = a.rec_off + (size_t)bi * (L + 1);
    int status = EST_OK;
    unsigned long long re = 0;
    unsigned long long rcur = a.rec_base ? a.rec_base[bi] : 0;
    unsigned long long rend = a.rec_base ? (a.rec_size ? rcur + a.rec_size[bi] : ~0ull) : 0;
    bool counting = false;
    unsigned long long rneed = 0, tneed = 0;
    IdFront X = FA, Y = FB;

    // ---- initHeadList (HaploBuilder.cpp:153-224), as in estep_structure ----
    int Fp0 = 0, st0 = EST_OK;
    if (tid == 0 && hl > 1) {
      const int li = gi - a.mod.hf_base;
      st0 = a.mod.hf_status[li];
      for (uint32_t t = a.mod.hf_off[li]; t < a.mod.hf_off[li + 1] && st0 == EST_OK; ++t) {
        if (Fp0 >= a.fcap) { st0 = EST_OVERFLOW_FRONTIER; break; }
        *X.at(F_LO, Fp0) = a.mod.hf_pairs[2 * t];
        *X.at(F_HI, Fp0) = a.mod.hf_pairs[2 * t + 1];
        *X.at(F_NL, Fp0) = 1;
        ++Fp0;
      }
    }
    if (tid == 0 && hl == 1) {
      const uchar2 g0 = g[0];
      const bool m0 = g0.x == MISSING, m1 = g0.y == MISSING;
      for (int hix = 0; hix < a.mod.n_head; ++hix) {
        const uint32_t head = a.mod.head_ids[hix];
        const uint8_t ah = a.mod.last[head];
        if (!(m0 || m1 || g0.x == ah || g0.y == ah)) continue;
        const bool hasAllele = g0.x == ah || g0.y == ah;
        const bool expand = (m0 && m1) || ((m0 || m1) && hasAllele);
        const int nx = expand ? (int)a.pan.anum[0] : 1;
        for (int k = 0; k < nx; ++k) {
          uint32_t xk;
          if (expand) {
            if (!(a.pan.afreq[k] > 0)) continue;
            xk = (uint32_t)k;
          } else {
            xk = (!m0 && !m1 && g0.x != g0.y) ? ((ah == g0.x) ? g0.y : g0.x) : g0.x;
          }
          const uint32_t hq = xk == MISSING ? a.mod.head_pat0[amax] : a.mod.head_pat0[xk];
          if (hq == NONE) { st0 = EST_NO_HEAD_PATTERN; break; }
          if (hq < head) continue;
          if (Fp0 >= a.fcap) { st0 = EST_OVERFLOW_FRONTIER; break; }
          *X.at(F_LO, Fp0) = head;
          *X.at(F_HI, Fp0) = hq;
          *X.at(F_NL, Fp0) = 1;
          ++Fp0;
        }
        if (st0 != EST_OK) break;
      }
    }
    int Fp = B.bcast(Fp0);
    status = B.bcast(st0);
    int fbig = Fp;
    B.sync();
    if (status == EST_OK) {
      const unsigned long long words = 4 + 4ull * Fp + 1 + (a.exact ? 2ull * Fp : 0ull);
      rneed += (words + 1) & ~1ull;
      tneed += a.exact ? 4ull * Fp + 2 : trace_locus_words((unsigned long long)Fp, S);
      const unsigned long long o = rec_alloc<NW>(a, B, rcur, rend, words);
      if (o == REC_NONE) {
        counting = true;
        if (tid == 0) re += (unsigned long long)Fp;
      } else {
        uint32_t *R = a.rec + o;
        double *Rtp = (double *)(R + 4);
        uint32_t *Rhd = R + 4 + 2 * Fp, *Rcb = Rhd + Fp;
        for (int t = tid; t < Fp; t += NT) {
          const uint32_t lo = *X.at(F_LO, t), hi = *X.at(F_HI, t);
          Rtp[t] = a.mod.freq[lo] * a.mod.freq[hi];
          Rhd[t] = (uint32_t)a.mod.last[lo] | (uint32_t)a.mod.last[hi] << 8 | 1u << 16 | (lo == hi ? 1u << 24 : 0u);
          Rcb[t] = 0;
          if (a.exact) {
            Rcb[Fp + 1 + t] = lo;
            Rcb[2 * Fp + 1 + t] = hi;
          }
        }
        if (tid == 0) {
          Rcb[Fp] = 0;
          R[0] = (uint32_t)Fp;
          R[1] = 0;
          R[2] = 0;
          R[3] = 0;
          roff[hl] = o;
          re += (unsigned long long)Fp;
        }
      }
    }
    if (a.prune && status == EST_OK) {
      for (int t = tid; t < Fp; t += NT) {
        const uint32_t lo = *X.at(F_LO, t), hi = *X.at(F_HI, t);
        const double tpv = a.mod.freq[lo] * a.mod.freq[hi];
        fwx[t] = lo == hi ? tpv : tpv * 2.0;
      }
      B.sync();
    }

    // ---- structure of the forward over loci (HaploBuilder.cpp:47-82) -------
    for (int i = hl; i < L && status == EST_OK; ++i) {
      if (Fp == 0) { status = EST_UNRESOLVED; break; }
      const uchar2 gg = g[i];
      // allele pairs in extendAll call order; a locus without missing alleles
      // has one pair, which every thread derives itself (no hand-off)
      const bool simple = gg.x != MISSING && gg.y != MISSING;
      if (!simple) {
        if (tid == 0) {
          const double *af = a.pan.afreq + (size_t)i * amax;
          const int an = a.pan.anum[i];
          int np = 0;
          auto push = [&](int x, int y) { pr_x[np] = (uint8_t)x; pr_y[np] = (uint8_t)y; pr_o[np] = x == y ? 1 : 2; ++np; };
          if (gg.x == MISSING && gg.y == MISSING) {
            for (int j = 0; j < an; ++j)
              if (af[j] > 0)
                for (int k = j; k < an; ++k)
                  if (af[k] > 0) push(j, k);
          } else if (gg.x == MISSING) {
            for (int j = 0; j < an; ++j)
              if (af[j] > 0) push(j, gg.y);
          } else {
            for (int j = 0; j < an; ++j)
              if (af[j] > 0) push(j, gg.x);
          }
          int off = 0;
          for (int p = 0; p < np; ++p) { pr_off[p] = off; off += Fp * pr_o[p]; }
          pr_off[np] = off;
          pr_off[npm + 1] = np;
        }
        B.sync();
      }
      const int npairs = simple ? 1 : pr_off[npm + 1];
      const int o1 = simple ? (gg.x == gg.y ? 1 : 2) : 0;
      const int C = simple ? Fp * o1 : pr_off[npairs];
      if (C > a.ccap) { status = EST_OVERFLOW_CONTRIB; break; }
      // contribution c -> (predecessor state, orientation, alleles)
      auto decode = [&](int c, uint32_t &s, uint32_t &x, uint32_t &y) {
        int oo, local;
        uint32_t px, py;
        if (simple) {
          oo = o1;
          local = c;
          px = gg.x;
          py = gg.y;
        } else {
          int p = 0;
          while (p + 1 < npairs && c >= pr_off[p + 1]) ++p;
          oo = pr_o[p];
          local = c - pr_off[p];
          px = pr_x[p];
          py = pr_y[p];
        }
        const int o = oo == 2 ? (local & 1) : 0;
        s = oo == 2 ? (uint32_t)(local >> 1) : (uint32_t)local;
        x = o ? py : px;
        y = o ? px : py;
      };
      const int Q = (C + NT - 1) / NT;  // this thread's contributions: [c0, c1)
      const int c0 = min(C, tid * Q), c1 = min(C, c0 + Q);
      // ---- 1. keys, slots; per slot: first contribution, count, predecessor lengths
      bool full = false;  // the key table is full: more new states than fcap
      for (int cb = c0; cb < c1; cb += 4) {
        uint32_t sa[4], sb[4], ss[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          sa[u] = sb[u] = NONE;
          ss[u] = 0;
          if (cb + u < c1) {
            uint32_t x, y;
            decode(cb + u, ss[u], x, y);
            const bool live = !a.prune || fwx[ss[u]] > 0.0;  // extend(): fwd <= 0 is not extended (HaploBuilder.cpp:237)
            if (live) {
              sa[u] = a.mod.succ[(size_t)*X.at(F_LO, (int)ss[u]) * amax + x];
              sb[u] = a.mod.succ[(size_t)*X.at(F_HI, (int)ss[u]) * amax + y];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (cb + u >= c1) continue;
          const int c = cb + u;
          const bool valid = sa[u] != NONE && sb[u] != NONE;
          const bool rev = sa[u] > sb[u];  // addHaploPair: id_a > id_b -> swap, reversed
          uint32_t slot = NONE;
          if (valid) {
            const uint32_t lo = rev ? sb[u] : sa[u], hi = rev ? sa[u] : sb[u];
            slot = k2_key_slot(K, ((unsigned long long)lo << 32) | hi, key_hash(lo, hi));
            if (slot == NONE) {
              full = true;
            } else {
              atomicMin(f_first(slot), (uint32_t)c);
              atomicAdd(K.cnt(slot), 1u);
              atomicAdd(f_ns(slot), *X.at(F_NL, (int)ss[u]));
            }
          }
          *CT.at(C2_SR, c) = cw_pack(ss[u], rev);
          *CT.at(C2_SL, c) = slot;
        }
      }
      __threadfence_block();
      B.sync();
      // ---- 2. new states in creation order
      int mynew = 0;
      for (int c = c0; c < c1; ++c) {
        const uint32_t sl = *CT.at(C2_SL, c);
        if (sl != NONE && rd(f_first(sl), sl) == (uint32_t)c) ++mynew;
      }
      int Fn = 0;  // (a full table: past fcap without a hand-off of its own; < 0 on wrap-around)
      int st = B.scan(full ? a.fcap + 1 : mynew, &Fn);
      if (Fn > a.fcap || Fn < 0) { status = EST_OVERFLOW_FRONTIER; break; }
      if (Fn == 0) { status = EST_UNRESOLVED; break; }
      for (int c = c0; c < c1; ++c) {
        const uint32_t sl = *CT.at(C2_SL, c);
        if (sl != NONE && rd(f_first(sl), sl) == (uint32_t)c) {
          const unsigned long long key = sl < (uint32_t)K.hc ? *K.key(sl) : ld_acq(K.key(sl));
          *K.state(sl) = (uint32_t)st;
          *Y.at(F_LO, st) = (uint32_t)(key >> 32);
          *Y.at(F_HI, st) = (uint32_t)key;
          *Y.at(F_SLOT, st) = sl;
          ++st;
        }
      }
      fbig = Fn > fbig ? Fn : fbig;
      if (tid < NBUCKET) bucket[tid] = 0;
      __threadfence_block();
      B.sync();
      // ---- 3. states: first positions (scan of counts), list lengths, chains
      const int QS = (Fn + NT - 1) / NT;
      const int t0 = min(Fn, tid * QS), t1 = min(Fn, t0 + QS);
      int mycnt = 0;
      for (int t = t0; t < t1; ++t) mycnt += (int)rd(K.cnt(*Y.at(F_SLOT, t)), *Y.at(F_SLOT, t));
      int Cv = 0;
      int cpos = B.scan(mycnt, &Cv);
      for (int t = t0; t < t1; ++t) {
        const uint32_t sl = *Y.at(F_SLOT, t);
        const int m = (int)rd(K.cnt(sl), sl);
        *Y.at(F_CB, t) = (uint32_t)cpos;
        cpos += m;
        const uint32_t nsum = rd(f_ns(sl), sl);
        const uint32_t nl = nsum < (uint32_t)S ? nsum : (uint32_t)S;
        *Y.at(F_NL, t) = nl;
        re += nl;
        if (nsum > (uint32_t)S)  // bucket 0 = most contributions
          atomicAdd(&bucket[NBUCKET - 1 - (m - 1 < NBUCKET - 1 ? m - 1 : NBUCKET - 1)], 1);
      }
      const unsigned long long words =
          4 + 4ull * Fn + 1 + (unsigned long long)Cv + Fn + (a.exact ? (unsigned long long)C + npairs : 0ull);
      rneed += (words + 1) & ~1ull;
      tneed += a.exact ? 4ull * Fn + 2 : trace_locus_words((unsigned long long)Fn, S);
      __threadfence_block();
      B.sync();
      const unsigned long long o = counting ? 0 : rec_alloc<NW>(a, B, rcur, rend, words);
      if (o == REC_NONE) counting = true;
      uint32_t *R = a.rec + (counting ? 0 : o);  // not dereferenced while counting
      double *Rtp = (double *)(R + 4);
      uint32_t *Rhd = R + 4 + 2 * Fn, *Rcb = Rhd + Fn, *Rct = Rcb + Fn + 1, *Rch = Rct + Cv;
      int nch = 0;
      {  // every wave scans the 32 bucket counts; wave 0 writes the offsets
        const int b = lane < NBUCKET ? bucket[lane] : 0;
        const int incl = wave_incl_scan(b);
        nch = __shfl(incl, 63);
        B.sync();
        if (wv == 0 && lane < NBUCKET) bucket[lane] = incl - b;
      }
      // contributions of slots with more than one: into their state's segment
      for (int c = c0; c < c1; ++c) {
        const uint32_t sl = *CT.at(C2_SL, c);
        if (sl != NONE && rd(K.cnt(sl), sl) > 1u) {
          const uint32_t stt = rd(K.state(sl), sl);
          const uint32_t pos = atomicAdd(f_fill(sl), 1u);
          *CT.at(C2_AUX, (int)(*Y.at(F_CB, (int)stt) + pos)) = (uint32_t)c;
        }
      }
      __threadfence_block();
      B.sync();
      // the records: per state (creation order) and per contribution (add order)
      if (!counting) {
        for (int t = t0; t < t1; ++t) {
          const uint32_t lo = *Y.at(F_LO, t), hi = *Y.at(F_HI, t), sl = *Y.at(F_SLOT, t);
          const uint32_t nl = *Y.at(F_NL, t);
          const uint32_t nsum = rd(f_ns(sl), sl);
          Rtp[t] = a.mod.tp[lo] * a.mod.tp[hi];  // m_transition_prob, HaploPair.cpp:42
          Rhd[t] = (uint32_t)a.mod.last[lo] | (uint32_t)a.mod.last[hi] << 8 | nl << 16 | (nsum > (uint32_t)S ? HDR_CHAIN : 0u);
          Rcb[t] = *Y.at(F_CB, t);
          if (nsum > (uint32_t)S) {
            const int m = (int)rd(K.cnt(sl), sl);
            const int pos = atomicAdd(&bucket[NBUCKET - 1 - (m - 1 < NBUCKET - 1 ? m - 1 : NBUCKET - 1)], 1);
            Rch[pos] = (uint32_t)t;
          }
        }
        uint32_t *Rout = Rct + Cv + nch;  // exact: contributions in extendAll order, then pair orientations
        for (int c = c0; c < c1; ++c) {
          const uint32_t sl = *CT.at(C2_SL, c);
          const uint32_t w = *CT.at(C2_SR, c);
          uint32_t stt = NONE;
          if (sl != NONE) {
            stt = rd(K.state(sl), sl);
            const uint32_t m = rd(K.cnt(sl), sl), cb = *Y.at(F_CB, (int)stt);
            uint32_t rank = 0;
            if (m > 1u)  // members of the state before this one, in contribution order
              for (uint32_t k = 0; k < m; ++k) rank += *CT.at(C2_AUX, (int)(cb + k)) < (uint32_t)c ? 1u : 0u;
            const uint32_t ns = *X.at(F_NL, (int)cw_state(w));
            Rct[cb + rank] = w | ns << 24;
          }
          if (a.exact)
            Rout[c] = stt == NONE ? NONE
                                  : (stt | (w & CW_REV) |
                                     xpair_index(a.mod.last[*Y.at(F_LO, (int)stt)], a.mod.last[*Y.at(F_HI, (int)stt)])
                                         << XPAIR_SHIFT);
        }
        if (a.exact)
          for (int p = tid; p < npairs; p += NT) Rout[C + p] = simple ? (uint32_t)o1 : pr_o[p];
        if (tid == 0) {
          Rcb[Fn] = (uint32_t)Cv;
          R[0] = (uint32_t)Fn;
          R[1] = (uint32_t)Cv;
          R[2] = (uint32_t)nch;
          // C <= EXACT_C_MAX (the host caps ccap in exact mode), npairs < 2^10 (amax <= 44 in exact mode)
          R[3] = a.exact ? (uint32_t)C << 10 | (uint32_t)npairs : 0u;
          roff[i + 1] = o;
        }
      }
      if (a.prune) {  // the new states' forward likelihoods, in add order (HaploPair.cpp:42, :66)
        B.sync();
        for (int t = t0; t < t1; ++t) {
          double f = 1.0;  // counting (no records): sizes only, nothing pruned
          if (!counting) {
            const double tpv = Rtp[t];
            for (uint32_t r = Rcb[t]; r < Rcb[t + 1]; ++r) {
              const double v = fwx[cw_state(Rct[r])] * tpv;
              f = r == Rcb[t] ? v : f + v;
            }
          }
          fwy[t] = f;
        }
      } else {
        B.sync();  // every contribution's slot fields read (state, count) before they are cleared
      }
      // m_best_pair.clear() for the next locus
      for (int t = t0; t < t1; ++t) {
        const uint32_t sl = *Y.at(F_SLOT, t);
        *K.key(sl) = KEY_EMPTY;
        *f_first(sl) = FIRST_NONE;
        *f_ns(sl) = 0;
        *f_fill(sl) = 0;
        *K.cnt(sl) = 0;
      }
      __threadfence_block();
      B.sync();
      const IdFront T = X;
      X = Y;
      Y = T;
      double *const ft = fwx;
      fwx = fwy;
      fwy = ft;
      Fp = Fn;
    }
    if (status == EST_OK && Fp == 0) status = EST_UNRESOLVED;
    if (counting && status != EST_OVERFLOW_FRONTIER && status != EST_OVERFLOW_CONTRIB && status != EST_NO_HEAD_PATTERN)
      status = EST_OVERFLOW_REC;
    fbig = Fp > fbig ? Fp : fbig;
    if (status < 0) reset_tables();  // aborted mid-locus: keys may be left
    if (status == EST_OK && a.prune) status = EST_OK_PRUNED;
    re = B.reduce_u64(re);
    if (tid == 0) {
      a.rec_need[bi] = rneed;
      a.trace_need[bi] = tneed;
      a.status[bi] = status;
      a.re_count[bi] = re;
      a.fmax[bi] = fbig;
      atomicMax(a.max_states, (unsigned)fbig);
    }
  }
}

#endif  // HMC_VARIANTS

// ============================================================ pass 2 ======

namespace {

struct K2Shared {
  unsigned long long u[2];
  int next;  // chain queue head
  int flag;  // a forward likelihood hit 0 before the last locus
  int iters; // diagnostic build: most chain-loop iterations of any wave this locus
  int tie;   // FAST: a non-zero likelihood straddles some list's S-cut
  int q;     // next individual of the order list
};

struct K2Plan {
  int o_lpos, o_rpos, o_junk, o_slik, o_smeta, o_bs, o_front[2], bytes;
};

// Selection slots per wave: one wavefront of lists of 2S links (S <= 32), or
// one list of 2S links (S > 32); with two links per lane (PAIR builds,
// S <= 16) 64 / S lists of 2S plus a dead segment for the lanes past the last.
__host__ __device__ inline int k2_slots(int S, bool pair = false) {
  return pair ? (WAVE / S + 1) * 2 * S : (2 * S > WAVE ? 2 * S : WAVE);
}

__host__ __device__ inline K2Plan k2_plan(int S, int fc, int nw, bool pair = false) {
  K2Plan p;
  int o = 0;
  auto take = [&](int bytes) { int r = o; o += (bytes + 15) & ~15; return r; };
  const int sl = k2_slots(S, pair), pos = pair ? sl : WAVE;
  p.o_lpos = take(nw * pos * 4);
  p.o_rpos = take(nw * pos * 4);
  p.o_junk = take(nw * (pair ? 4 : 2) * WAVE * 4);
  p.o_slik = take(nw * sl * 8);
  p.o_smeta = take(nw * sl * 4);
  p.o_bs = take((int)sizeof(K2Shared));
  p.o_front[0] = take(fc * (24 + 8 * S));  // value_front.hpp: 24 + 8 S bytes per state
  p.o_front[1] = take(fc * (24 + 8 * S));
  p.bytes = o;
  return p;
}


// Bump-allocate `words` trace words for this block (block-uniform call).
__device__ inline unsigned long long k2_trace_alloc(const ValueArgs &a, K2Shared *bs, unsigned long long &cur,
                                                    unsigned long long &end, unsigned long long words) {
  if (cur + words > end) {
    const unsigned long long take = words > TRACE_CHUNK ? words : TRACE_CHUNK;
    if (threadIdx.x == 0) bs->u[0] = atomicAdd(a.trace_cursor, take);
    __syncthreads();
    const unsigned long long base = bs->u[0];
    __syncthreads();
    cur = base;
    end = base + take;
  }
  const unsigned long long off = cur;
  cur += words;
  return off;
}

// Trace record of locus j allocated before its lists are built: phase A
// writes every state's header and link words as it builds the list, the end
// of a chain of adds overwrites its state's (no second pass over the
// frontier).  Returns false when the trace store is full.
struct TraceRec {
  uint32_t *hdr, *lnk;
  unsigned long long off;
};
__device__ inline bool k2_trace_begin(const ValueArgs &a, K2Shared *bs, int F, unsigned long long &cur,
                                      unsigned long long &end, TraceRec &tr) {
  const unsigned long long words = trace_locus_words((unsigned long long)F, a.S);
  tr.off = k2_trace_alloc(a, bs, cur, end, words);
  if (tr.off + words > a.trace_cap) return false;
  tr.hdr = a.trace + tr.off + 1;
  tr.lnk = a.trace + trace_links(tr.off, (uint32_t)F);
  return true;
}
__device__ inline void k2_trace_end(const ValueArgs &a, const TraceRec &tr, int F, int j, int bi) {
  if (threadIdx.x == 0) {
    a.trace[tr.off] = (uint32_t)F;
    a.loc_off[(size_t)bi * (a.L + 1) + j] = tr.off;
  }
}

}  // namespace

// Diagnostic build only (-DHMC_STAMPS): thread 0 accumulates shader cycles of
// the block's critical path per phase of the value pass.
#ifdef HMC_STAMPS
#define K2_T0 unsigned long long k2t = __builtin_amdgcn_s_memtime(); unsigned long long k2acc[16] = {};
#define K2_ST(k)                                                   \
  do {                                                             \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();    \
    k2acc[k] += t1 - k2t;                                          \
    k2t = t1;                                                      \
  } while (0)
#define K2_CNT(k, v) k2acc[k] += (v)
#define K2_FLUSH                                                   \
  if (a.stamps && tid == 0)                                        \
    for (int k = 0; k < 16; ++k) atomicAdd(&a.stamps[k], k2acc[k]);
#else
#define K2_T0
#define K2_ST(k) do { } while (0)
#define K2_CNT(k, v) do { } while (0)
#define K2_FLUSH
#endif

#ifndef HMC_PA_UNROLL  // 4: measured equal to 8 at 4 waves per SIMD, and lets 5 fit in 96 VGPRs
#define HMC_PA_UNROLL 4
#endif
size_t estep_s2_scratch_bytes(int fcap, int S) { return 2 * k2_front_bytes(fcap, S); }
size_t estep_s2_lds_bytes(int S, int fc, int nw, bool pair) { return (size_t)k2_plan(S, fc, nw, pair).bytes; }

// WPE: resident waves per SIMD the register allocation targets — 4 (127
// VGPRs: shapes of up to 16 waves per CU) or 5 (96 VGPRs, a few spills in
// the per-individual epilogue: the 1 x 20 shape of full groups, 5-6 % faster
// than 1 x 16 at cfg 3, profiles/r02/values_ab/).
// FAST: the k-best lists are kept by value only (seg_rank_select): a list's
// arrangement differs from the reference's, which changes no result while no
// non-zero likelihood ties across a list's S-cut and the final candidates are
// tie-free and non-zero; otherwise the individual reports EST_NEEDS_ORDER and
// is re-run by the exact instantiation (FAST = false, libstdc++ permutations).
// WIDE: sample sizes 33..64 — lists of up to 2S = 128 links, one per wave,
// each lane holding positions k and k + 64, selection by the sequential
// libstdc++ code on the wave's first lane (the sw > 32 path of seg_nth_slots).
// PAIR: two links per lane in phase B (seg2_nth_slots: S lanes and 64 / S
// lists of up to 2S links per wavefront, S <= 16) — heavy groups, whose loci
// have many chains of adds (cfg 3's E1: ~130), get 2x the lists per wave.
template <bool FAST, int WPE, bool WIDE = false, bool PAIR = false>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(WPE))) void estep_values(ValueArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int S = a.S, L = a.L, hl = a.head_len;
  // locus window of trace indices [wlo, whi) (classic: the head to L)
  const int wlo = a.w.hi > 0 ? a.w.lo : hl, whi = a.w.hi > 0 ? a.w.hi : L + 1;
  const bool from_ck = wlo > hl, last_win = whi == L + 1;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid / WAVE;
  const int NT = blockDim.x, NW = NT / WAVE;
  const K2Plan plan = k2_plan(S, a.lds_fc, NW, PAIR);
  K2Shared *bs = (K2Shared *)(smem + plan.o_bs);
  const int sws = k2_slots(S, PAIR);  // selection slots per wave
  const int sps = PAIR ? sws : WAVE;  // stop-position slots per wave
  const SegScratch ss{(int *)(smem + plan.o_lpos) + wv * sps, (int *)(smem + plan.o_rpos) + wv * sps,
                      (int *)(smem + plan.o_junk) + wv * (PAIR ? 4 : 2) * WAVE, (double *)(smem + plan.o_slik) + wv * sws,
                      (uint32_t *)(smem + plan.o_smeta) + wv * sws};
  const Seg sg = make_seg(WIDE ? WAVE : (PAIR ? S : 2 * S));
  const int G = WIDE ? 1 : (PAIR ? WAVE / S : WAVE / (2 * S));
  // PAIR: this lane's two positions are slots sb + k and sb + k + S
  const int sb = sg.g * 2 * S;
  const LinkList W{(double *)(smem + plan.o_slik), (uint32_t *)(smem + plan.o_smeta), 1};  // final selection

  char *sp = a.scratch + (size_t)blockIdx.x * a.scratch_stride;
  const VFront FA{smem + plan.o_front[0], (unsigned char *)sp, a.lds_fc, a.fcap, S};
  const VFront FB{smem + plan.o_front[1], (unsigned char *)sp + k2_front_bytes(a.fcap, S), a.lds_fc, a.fcap, S};

  K2_T0
  // individuals are taken from the heaviest-first order list one at a time as
  // blocks finish (longest-processing-time-first), not round-robin
  auto next_q = [&]() -> int {
    __syncthreads();
    if (tid == 0) bs->q = atomicAdd(a.next_q, 1) + (int)gridDim.x;
    __syncthreads();
    return bs->q;
  };
  for (int q = blockIdx.x; q < a.n_order; q = next_q()) {
    const int bi = a.order[q];
    const unsigned long long t_indiv = __builtin_amdgcn_s_memtime();
    int status = a.status[bi];
    if (status == EST_NEEDS_ORDER) status = EST_OK;  // the re-run of a value-only pass
    const bool pruned = status == EST_OK_PRUNED;     // records built with extend()'s forward test
    if (pruned) status = EST_OK;
    if (status != EST_OK) {  // pass 1 found no resolution (dead frontier)
      if (tid == 0) {
        a.total[bi] = 0.0;
        a.ncand[bi] = 0;
        a.cost[bi] = 0;
      }
      continue;
    }
    const unsigned long long *roff = a.rec_off + (size_t)bi * (L + 1);
    // the individual's reserved trace region, else the bump allocator
    unsigned long long tcur = a.trace_base ? a.trace_base[bi] : 0, tend = a.trace_base ? ~0ull : 0;
    VFront X = FA, Y = FB;

    // ---- head list (HaploPair.cpp:14-33) -----------------------------------
    // (a locus window after the first: the frontier its checkpoint holds)
    const uint32_t *R = from_ck ? a.rec : a.rec + roff[hl];
    int Fp = 0;
    if (from_ck) {
      const uint32_t *ck = a.w.ck_in + a.w.ck_off[(size_t)bi * (a.w.nwin + 1) + a.w.win];
      Fp = (int)ck[0];
      const double *cf = (const double *)(ck + ck_value_off((unsigned long long)Fp));
      const unsigned long long *ch = (const unsigned long long *)(cf + Fp);
      const double *cl = (const double *)(ch + Fp);
      for (int t = tid; t < Fp; t += NT) {
        const uint32_t n = ck[2 + 2 * Fp + t];
        *X.fwd(t) = cf[t];
        *X.hm(t) = ch[t];
        *X.nl(t) = n;
        double *xl = X.lik(t);
        for (uint32_t k = 0; k < n; ++k) xl[k] = cl[(size_t)t * S + k];
      }
      __syncthreads();
    } else {
      Fp = (int)R[0];
      const double *Rtp = (const double *)(R + 4);
      const uint32_t *Rhd = R + 4 + 2 * Fp;
      TraceRec tr;
      if (!k2_trace_begin(a, bs, Fp, tcur, tend, tr)) {
        status = EST_OVERFLOW_TRACE;
      } else {
        for (int t = tid; t < Fp; t += NT) {
          const bool homo = (Rhd[t] >> 24) & 1u;
          const double tpv = Rtp[t];
          *X.fwd(t) = homo ? tpv : tpv * 2.0;
          X.lik(t)[0] = tpv;
          *X.hm(t) = homo ? 1ull : 0ull;
          *X.nl(t) = 1;
          tr.hdr[t] = (Rhd[t] & 0xFFFFu) | 1u << 16;
          uint32_t *tl = tr.lnk + (size_t)t * S;
          tl[0] = meta_pack(0, 0, false, homo, true);
          for (int k = 1; k < S; ++k) tl[k] = 0u;
        }
        k2_trace_end(a, tr, Fp, hl, bi);
      }
      __syncthreads();
    }

    // ---- forward over loci ----------------------------------------------------
    for (int j = from_ck ? wlo : hl + 1; j < whi && status == EST_OK; ++j) {
      R = a.rec + roff[j];
      const int F = (int)R[0], C = (int)R[1], NCH = (int)R[2];
      const double *Rtp = (const double *)(R + 4);
      const uint32_t *Rhd = R + 4 + 2 * F, *Rcb = Rhd + F, *Rct = Rcb + F + 1, *Rch = Rct + C;
      K2_ST(0);
      if (tid == 0) {
        bs->next = 0;
        bs->flag = 0;
        bs->iters = 0;
        bs->tie = 0;

      }
      TraceRec tr;
      if (!k2_trace_begin(a, bs, F, tcur, tend, tr)) {
        status = EST_OVERFLOW_TRACE;
        break;
      }
      // A: one thread per state — extension constructor (HaploPair.cpp:35-61),
      // the appends that still fit (HaploPair::add without selection,
      // :63-84) and the whole ordered forward sum (:42, :66)
      for (int t = tid; t < F; t += NT) {
        const double tpv = Rtp[t];
        const uint32_t hd = Rhd[t];
        const bool differ = (hd & 0xFFu) != ((hd >> 8) & 0xFFu);
        const int cb = (int)Rcb[t], ce = (int)Rcb[t + 1];
        // ordered forward sum (HaploPair.cpp:42, :66): words and predecessor
        // likelihoods of HMC_PA_UNROLL contributions loaded together, the adds in order
        double fwd = 0.0;
        for (int rb = cb; rb < ce; rb += HMC_PA_UNROLL) {
          uint32_t ws[HMC_PA_UNROLL];
          double fs[HMC_PA_UNROLL];
#pragma unroll
          for (int u = 0; u < HMC_PA_UNROLL; ++u) ws[u] = rb + u < ce ? Rct[rb + u] : Rct[cb];
#pragma unroll
          for (int u = 0; u < HMC_PA_UNROLL; ++u) fs[u] = *X.fwd((int)cw_state(ws[u]));
#pragma unroll
          for (int u = 0; u < HMC_PA_UNROLL; ++u)
            if (rb + u < ce) {
              const double v = fs[u] * tpv;
              fwd = rb + u == cb ? v : fwd + v;
            }
        }
        // extension constructor + the appends that still fit; the link words
        // also go to the trace record (a state with a chain of adds gets its
        // final words at the chain's end)
        uint32_t w = Rct[cb];
        uint32_t s = cw_state(w), ns = cw_ns(w);
        double *yl = Y.lik(t);
        unsigned long long yhm = 0ull;
        uint32_t *tl = tr.lnk + (size_t)t * S;
        copy_extended_hm<HMC_PA_UNROLL>(X.lik((int)s), *X.hm((int)s), yl, yhm, 0, (int)ns, s, tpv, cw_rev(w), differ, tl);
        int k = (int)ns, r0 = ce;
        for (int r = cb + 1; r < ce; ++r) {
          w = Rct[r];
          s = cw_state(w);
          ns = cw_ns(w);
          if (k + (int)ns <= S) {
            copy_extended_hm<HMC_PA_UNROLL>(X.lik((int)s), *X.hm((int)s), yl, yhm, k, (int)ns, s, tpv, cw_rev(w), differ,
                                            tl);
            k += (int)ns;
          } else {
            r0 = r;
            break;
          }
        }
        if (r0 == ce) {  // the list is final: zero the unused link words
          for (int q = k; q < S; ++q) tl[q] = 0u;
        }
        tr.hdr[t] = (hd & 0xFFFFu) | (uint32_t)k << 16;
        *Y.fwd(t) = fwd;
        *Y.hm(t) = yhm;  // (a chain's state: the flags of its partial list; the chain's end rewrites them)
        *Y.nl(t) = (uint32_t)k;
        *Y.r0(t) = (uint32_t)r0;
        if (!(fwd > 0.0) && j < L && !pruned) bs->flag = 1;

      }
      __syncthreads();
      K2_ST(1);
      K2_CNT(8, NCH);
      K2_CNT(9, F);
      K2_CNT(7, F > Y.fc ? F - Y.fc : 0);  // states written to the frontier's HBM tier
      if (bs->flag) {
        status = EST_NEEDS_EXACT;
        break;
      }
      // B: the adds that overflow S, one chain of adds per state, run by 2S-lane
      // segments that pull chains (longest first) from the block queue.  The
      // list lives in the segment's LDS selection slots for the whole chain;
      // each add writes its transformed links behind it and selects in place.
      // The contribution word of add r+1 is loaded one add ahead.
      if (NCH > 0) {
        int ci = -1, r = 0, re_ = 0, st = 0, k0 = 0;
        [[maybe_unused]] int nit = 0;
#ifdef HMC_STAMPS
        unsigned long long tstep = __builtin_amdgcn_s_memtime();
#endif
        double tpv = 0.0, tie_v = 0.0;
        uint32_t wc = 0, wn = 0;
        bool differ = false, done = sg.g >= G;
        // this lane's first slot (position k; PAIR: also k + S, one segment of
        // slots further than the 2S-lane layout's)
        double *slot_l = ss.slik + sb + sg.k;
        uint32_t *slot_m = ss.smeta + sb + sg.k;
        while (true) {
          const bool idle = !done && ci < 0;
          if (wave_ballot(idle)) {
            int got = 0;
            if (idle && sg.k == 0) got = atomicAdd(&bs->next, 1);
            got = __shfl(got, sg.base);
            if (idle) {
              if (got < NCH) {
                ci = got;
                st = (int)Rch[ci];
                r = (int)*Y.r0(st);
                re_ = (int)Rcb[st + 1];
                tpv = Rtp[st];
                const uint32_t hd = Rhd[st];
                differ = (hd & 0xFFu) != ((hd >> 8) & 0xFFu);
                k0 = (int)*Y.nl(st);
                wc = Rct[r];
                wn = r + 1 < re_ ? Rct[r + 1] : 0u;
                // the partial list: likelihoods in the frontier, link words in the trace record
                const uint32_t *pl = tr.lnk + (size_t)st * S;
                if constexpr (WIDE) {
                  for (int kk = sg.k; kk < k0; kk += WAVE) {
                    slot_l[kk - sg.k] = Y.lik(st)[kk];
                    slot_m[kk - sg.k] = pl[kk];
                  }
                } else if (sg.k < k0) {
                  *slot_l = Y.lik(st)[sg.k];
                  *slot_m = pl[sg.k];
                }
              } else {
                done = true;
              }
            }
          }
          const bool act = ci >= 0;
          if (!wave_ballot(act)) break;
          int n = 0;
          if (act) {
            const uint32_t s = cw_state(wc), ns = cw_ns(wc);
            const bool rev = cw_rev(wc);
            n = k0 + (int)ns;
            // HaploPair::add transformation (HaploPair.cpp:63-80)
            auto extend = [&](int kk) {
              const int qk = kk - k0;
              double lk;
              unsigned long long xhm;
              X.ld_link((int)s, qk, lk, xhm);
              lk *= tpv;
              bool homo = (xhm >> qk) & 1ull;
              if (differ && homo) {
                if (rev) lk = 0.0;
                homo = false;
              }
              slot_l[kk - sg.k] = lk;
              slot_m[kk - sg.k] = meta_pack(s, (uint32_t)qk, rev, homo, false);
            };
            if constexpr (WIDE) {
              for (int kk = sg.k; kk < n; kk += WAVE)
                if (kk >= k0) extend(kk);
            } else {
              if (sg.k >= k0 && sg.k < n) extend(sg.k);
              if (PAIR && sg.k + S >= k0 && sg.k + S < n) extend(sg.k + S);
            }
            wc = wn;
            wn = r + 2 < re_ ? Rct[r + 2] : 0u;
          }
          wave_lds_sync();
          K2_CNT(10, 1);
          ++nit;
#ifdef HMC_STAMPS
          const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
          K2_CNT(14, ts0 - tstep);
#endif
          if (FAST) {
            const double tv = seg_rank_select(n, S, sg, ss);
            tie_v = tv > tie_v ? tv : tie_v;
          } else if (PAIR) {
            seg2_nth_slots(n, S - 1, sg, ss);
          } else {
            seg_nth_slots(n, S - 1, sg, ss);
          }
#ifdef HMC_STAMPS
          tstep = __builtin_amdgcn_s_memtime();
          K2_CNT(13, tstep - ts0);
#endif
          if (act) {
            k0 = S;
            if (++r == re_) {
              // FAST: a tie recorded on the way that is still at the final cut
              if (FAST && tie_v != 0.0 && tie_v == ss.slik[sg.base + S - 1]) bs->tie = 1;
              tie_v = 0.0;
              uint32_t *tl = tr.lnk + (size_t)st * S;
              // (every lane of the segment is here: its positions < S are k, and for
              // WIDE k + 64 >= S) the final list's homozygous flags, bit k = position k
              const uint32_t fm = sg.k < S ? slot_m[0] : 0u;
              const unsigned long long hb = (wave_ballot(sg.k < S && meta_homo(fm)) >> sg.base) &
                                            (S >= 64 ? ~0ull : ((1ull << S) - 1ull));
              if constexpr (WIDE) {
                for (int kk = sg.k; kk < S; kk += WAVE) {
                  Y.lik(st)[kk] = slot_l[kk - sg.k];
                  tl[kk] = slot_m[kk - sg.k];
                }
              } else if (sg.k < S) {
                Y.lik(st)[sg.k] = *slot_l;
                tl[sg.k] = *slot_m;
              }
              if (sg.k == 0) {
                *Y.nl(st) = (uint32_t)S;
                *Y.hm(st) = hb;
                tr.hdr[st] = (Rhd[st] & 0xFFFFu) | (uint32_t)S << 16;
              }
              ci = -1;
            }
          }
        }
#ifdef HMC_STAMPS
        if (lane == 0) atomicMax(&bs->iters, nit);
#endif
      }
      __syncthreads();
      K2_ST(2);
      K2_CNT(12, bs->iters);
      if (FAST && bs->tie) {
        status = EST_NEEDS_ORDER;
        break;
      }
      k2_trace_end(a, tr, F, j, bi);
      K2_ST(3);
      K2_CNT(11, 1);
      const VFront T = X;
      X = Y;
      Y = T;
      Fp = F;
    }

    // ---- a window before the last: its last frontier (values) goes to the
    // next window's checkpoint, which the structure pass allocated ----------
    __syncthreads();
    if (!last_win) {
      if (status == EST_OK && a.w.ck_write) {
        uint32_t *ck = a.w.ck_out + a.w.ck_off[(size_t)bi * (a.w.nwin + 1) + a.w.win + 1];
        double *cf = (double *)(ck + ck_value_off((unsigned long long)Fp));
        unsigned long long *ch = (unsigned long long *)(cf + Fp);
        double *cl = (double *)(ch + Fp);
        for (int t = tid; t < Fp; t += NT) {
          const uint32_t n = *X.nl(t);
          cf[t] = *X.fwd(t);
          ch[t] = *X.hm(t);
          const double *xl = X.lik(t);
          for (uint32_t k = 0; k < n; ++k) cl[(size_t)t * S + k] = xl[k];
        }
      }
      if (tid == 0) {
        if (a.w.ck_write) a.cost[bi] += (int32_t)((__builtin_amdgcn_s_memtime() - t_indiv) >> 10);
        a.status[bi] = status;
      }
      __syncthreads();
      continue;
    }
    // ---- final selection (HaploBuilder.cpp:87-116) ------------------------
    K2_ST(4);
    if (tid == 0) {
      const int32_t spent = (int32_t)((__builtin_amdgcn_s_memtime() - t_indiv) >> 10);
      a.cost[bi] = a.w.windowed() ? a.cost[bi] + spent : spent;
      int cnt = 0;
      double total = 0.0;
      if (status == EST_OK) {
        double out_max = 0.0;  // FAST: best likelihood the selection dropped
        bool out_any = false;
        for (int t = 0; t < Fp; ++t) {
          total += *X.fwd(t);
          const uint32_t n = *X.nl(t);
          for (uint32_t k = 0; k < n; ++k) {
            double lk = X.lik(t)[k];
            const bool homo = (*X.hm(t) >> k) & 1ull;
            if (!homo) lk *= 2.0;
            W.set(cnt++, lk, meta_pack((uint32_t)t, k, false, homo, false));
          }
          if (cnt > S) {
            if (cnt <= 32) nth_element_greater_masks(W, cnt, S - 1, cnt);
            else nth_element_greater(W, cnt, S - 1);
            if (FAST)
              for (int q = S; q < cnt; ++q) {
                out_max = out_any && out_max > W.l(q) ? out_max : W.l(q);
                out_any = true;
              }
            cnt = S;
          }
        }
        sort_greater(W, cnt, ss.lpos);  // the selection scratch is free here
        if (FAST) {  // the candidates and their order must not depend on list order
          bool tie = out_any && cnt > 0 && out_max == W.l(cnt - 1);
          for (int c = 0; c < cnt; ++c) tie = tie || W.l(c) == 0.0 || (c > 0 && W.l(c) == W.l(c - 1));
          if (tie) status = EST_NEEDS_ORDER;
        }
      }
      a.status[bi] = status;
      if (status == EST_OK) {
        double coverage = 0.0;
        for (int c = 0; c < cnt; ++c) {
          const uint32_t mm = W.m(c);
          const uint32_t t = meta_pred(mm), k = meta_idx(mm);
          const double own = X.lik((int)t)[k];
          const double prior = meta_homo(mm) ? own : own * 2.0;  // HaploPair.cpp:97-102
          const double post = prior / total;
          coverage += post;
          a.cand_state[(size_t)bi * S_MAX + c] = t;
          a.cand_idx[(size_t)bi * S_MAX + c] = k;
          a.prior[(size_t)bi * S_MAX + c] = prior;
          a.posterior[(size_t)bi * S_MAX + c] = post;
        }
        for (int c = 0; c < cnt; ++c)  // HaploModel.cpp:97-98
          a.weight[(size_t)bi * S_MAX + c] = a.posterior[(size_t)bi * S_MAX + c] / coverage;
      } else {
        cnt = 0;
      }
      a.total[bi] = total;
      a.ncand[bi] = cnt;
    }
    __syncthreads();
    K2_ST(5);
  }
  K2_FLUSH
}

#ifdef HMC_VARIANTS
hipError_t launch_estep_structure2(const StructArgs &a, int grid, int nw, hipStream_t st) {
  if (a.S < 1 || a.S > S_MAX || a.pan.amax > A_MAX || a.fcap > F_MAX || (a.hcap & (a.hcap - 1)) || a.lds_hc < 1 ||
      (a.lds_hc & (a.lds_hc - 1)) || a.lds_fc < 0 || a.lds_cc < 0 || a.ccap < 1 || a.mod.head_len < 1 ||
      (a.exact && a.ccap > EXACT_C_MAX) ||
      (a.mod.head_len > 1 && (!a.mod.hf_off || !a.mod.hf_pairs || !a.mod.hf_status)) ||
      (nw != 1 && nw != 4 && nw != 8 && nw != 16))
    return hipErrorInvalidValue;
  const size_t lds = estep_s1v2_lds_bytes(a.lds_fc, a.lds_hc, a.lds_cc, a.pan.amax, nw);
  const void *f = nw == 16 ? (const void *)estep_structure2<16>
                           : (nw == 8 ? (const void *)estep_structure2<8>
                                      : (nw == 4 ? (const void *)estep_structure2<4> : (const void *)estep_structure2<1>));
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (nw == 16) hipLaunchKernelGGL(estep_structure2<16>, dim3(grid), dim3(16 * WAVE), lds, st, a);
  else if (nw == 8) hipLaunchKernelGGL(estep_structure2<8>, dim3(grid), dim3(8 * WAVE), lds, st, a);
  else if (nw == 4) hipLaunchKernelGGL(estep_structure2<4>, dim3(grid), dim3(4 * WAVE), lds, st, a);
  else hipLaunchKernelGGL(estep_structure2<1>, dim3(grid), dim3(WAVE), lds, st, a);
  return hipGetLastError();
}

#else
// the product library: estep_structure2 is built into libhmc_amd_variants.so only
size_t estep_s1v2_lds_bytes(int, int, int, int, int) { return 0; }
hipError_t launch_estep_structure2(const StructArgs &, int, int, hipStream_t) { return hipErrorNotSupported; }
#endif


// ---- trace garbage collection (windowed E-step, TraceGcArgs) ----------------
// HaploPair::getGenotype (HaploPair.cpp:91-124) only ever follows links from
// the final candidates, and the k-best lists' links coalesce fast: on cfg 2's
// E1 the ~1 000-2 300 list entries of the last locus reach ~10 entries 50 loci
// back.  A block per individual marks, in one bitmap per locus (F x S bits),
// the entries of [lo0, hi1) reachable from every entry at hi1 - 1, then writes
// the marked entries of [lo0, mid) as nodes (ascending key per locus; the
// predecessor's node by a prefix popcount of the locus below, or by a binary
// search of the boundary list of the window before).
constexpr uint32_t GC_LDS_WORDS = 1024;  // marks of loci up to 32 768 list entries in LDS (8 KB per block)
template <int NW>
__global__ __launch_bounds__(64 * NW) void estep_trace_gc(TraceGcArgs a) {
  constexpr int NT = 64 * NW;
  __shared__ unsigned long long red64[16];  // Blk<NW <= 4>: 2 NW + 8 ints, then NW u64 (8-byte aligned)
  __shared__ int sq;
  __shared__ uint32_t lmk[2][GC_LDS_WORDS];  // two loci's marks
  const int tid = threadIdx.x, lane = lane_id(), wv = tid / WAVE;
  const Blk<NW> B{(int *)red64, tid, lane, wv};
  const int S = a.S, L = a.L, hl = a.head_len;
  const int nloc = a.hi1 - a.lo0;
  uint32_t *moff = a.scratch + (size_t)blockIdx.x * a.scratch_stride;  // [nloc + 1]
  uint32_t *preA = moff + nloc + 1, *preB = preA + a.max_words + 1;
  uint32_t *M = preB + a.max_words + 1;
  for (int q = blockIdx.x; q < a.n_order;) {
    const int bi = a.order[q];
    const unsigned long long *lo = a.loc_off + (size_t)bi * (L + 1);
    auto words_at = [&](int j) -> uint32_t { return (a.trace[lo[j]] * (uint32_t)S + 31u) >> 5; };
    // ---- bitmap offsets per locus
    uint32_t acc = 0;
    for (int c0 = 0; c0 < nloc; c0 += NT) {
      const int c = c0 + tid;
      const int w = c < nloc ? (int)words_at(a.lo0 + c) : 0;
      int tot = 0;
      const int ex = B.scan(w, &tot);
      if (c < nloc) moff[c] = acc + (uint32_t)ex;
      acc += (uint32_t)tot;
    }
    B.sync();
    for (uint32_t w = tid; w < acc; w += NT) M[w] = 0u;
    B.sync();
    // ---- every list entry of the last locus, then backward along the links.
    // A locus's marks live in one of two LDS buffers when they fit (LDS
    // atomics instead of L2 atomics: the first loci back mark nearly every
    // entry), else in its bitmap in M; marks of [lo0, mid) end up in M for
    // the compaction below.
    int cb = 0;  // the LDS buffer holding locus j's marks
    {
      const int j = a.hi1 - 1;
      const uint32_t F = a.trace[lo[j]];
      const uint32_t *hdr = a.trace + lo[j] + 1;
      const uint32_t nw = (F * (uint32_t)S + 31u) >> 5;
      uint32_t *C = nw <= GC_LDS_WORDS ? lmk[cb] : M + moff[j - a.lo0];
      for (uint32_t w = tid; w < nw; w += NT) {  // word by word: entries (t, k < nl(t))
        uint32_t word = 0u;
        uint32_t t = w * 32u / (uint32_t)S, k = w * 32u - t * (uint32_t)S;
        uint32_t n = t < F ? (hdr[t] >> 16) & 0xFFu : 0u;
        for (uint32_t i = 0; i < 32u; ++i) {
          if (t < F && k < n) word |= 1u << i;
          if (++k == (uint32_t)S) {
            k = 0;
            ++t;
            n = t < F ? (hdr[t] >> 16) & 0xFFu : 0u;
          }
        }
        C[w] = word;
      }
    }
    B.sync();
    for (int j = a.hi1 - 1; j > a.lo0; --j) {
      const uint32_t F = a.trace[lo[j]];
      const uint32_t *links = a.trace + trace_links(lo[j], F);
      const uint32_t nw = (F * (uint32_t)S + 31u) >> 5;
      const uint32_t nwp = (a.trace[lo[j - 1]] * (uint32_t)S + 31u) >> 5;
      const uint32_t *Cj = nw <= GC_LDS_WORDS ? lmk[cb] : M + moff[j - a.lo0];
      const bool pl = nwp <= GC_LDS_WORDS;
      uint32_t *P = pl ? lmk[cb ^ 1] : M + moff[j - 1 - a.lo0];  // (M starts zeroed)
      if (pl) {
        for (uint32_t w = tid; w < nwp; w += NT) P[w] = 0u;
        B.sync();
      }
      for (uint32_t w = tid; w < nw; w += NT)
        for (uint32_t b = Cj[w]; b; b &= b - 1u) {
          const uint32_t bit = w * 32u + (uint32_t)__builtin_ctz(b);
          const uint32_t m = links[bit];
          if (meta_head(m)) continue;
          const uint32_t pb = meta_pred(m) * (uint32_t)S + meta_idx(m);
          atomicOr(P + (pb >> 5), 1u << (pb & 31u));
        }
      B.sync();
      if (pl && j - 1 < a.mid) {  // the older window's marks, for the compaction
        uint32_t *Mp = M + moff[j - 1 - a.lo0];
        for (uint32_t w = tid; w < nwp; w += NT) Mp[w] = P[w];
      }
      cb ^= 1;
    }
    B.sync();
    // ---- the survivors of [lo0, mid) as nodes
    unsigned long long cnt = 0;
    for (uint32_t w = tid; w < moff[a.mid - a.lo0]; w += NT) cnt += (unsigned long long)__popc(M[w]);
    const unsigned long long total = B.reduce_u64(cnt);
    unsigned long long base = 0;
    if (tid == 0) {
      base = atomicAdd(a.node_cursor, total);
      if (base + total > a.node_cap) base = ~0ull;
    }
    base = B.bcast64(base);
    if (base == ~0ull) {
      if (tid == 0) a.status[bi] = EST_OVERFLOW_NODES;
    } else {
      const unsigned long long ob = a.bnd_off[bi];
      const uint32_t on = a.lo0 > hl ? a.bnd_n[bi] : 0u;
      unsigned long long nb = base, nb_prev = base;
      uint32_t cnt_last = 0;
      int miss = 0;
      uint32_t *Pc = preA, *Pp = preB;
      for (int j = a.lo0; j < a.mid; ++j) {
        const uint32_t F = a.trace[lo[j]];
        const uint32_t *hdr = a.trace + lo[j] + 1;
        const uint32_t *links = a.trace + trace_links(lo[j], F);
        const uint32_t *Mj = M + moff[j - a.lo0];
        const uint32_t nw = (F * (uint32_t)S + 31u) >> 5;
        uint32_t acc2 = 0;
        for (uint32_t c0 = 0; c0 < nw; c0 += NT) {
          const uint32_t w = c0 + tid;
          const int v = w < nw ? __popc(Mj[w]) : 0;
          int tot = 0;
          const int ex = B.scan(v, &tot);
          if (w < nw) Pc[w] = acc2 + (uint32_t)ex;
          acc2 += (uint32_t)tot;
        }
        B.sync();
        const uint32_t *Mp = j > a.lo0 ? M + moff[j - 1 - a.lo0] : nullptr;
        for (uint32_t w = tid; w < nw; w += NT) {
          unsigned long long r = nb + Pc[w];
          for (uint32_t b = Mj[w]; b; b &= b - 1u) {
            const uint32_t bit = w * 32u + (uint32_t)__builtin_ctz(b);
            const uint32_t t = bit / (uint32_t)S, k = bit - t * (uint32_t)S;
            const uint32_t m = links[bit];
            uint32_t pred = NONE;
            if (!meta_head(m) && j > hl) {
              const uint32_t pt = meta_pred(m), pk = meta_idx(m);
              if (j > a.lo0) {
                const uint32_t pb = pt * (uint32_t)S + pk;
                pred = (uint32_t)(nb_prev + Pp[pb >> 5] + (uint32_t)__popc(Mp[pb >> 5] & ((1u << (pb & 31u)) - 1u)));
              } else {  // the window before: its boundary list, ascending keys
                const uint32_t key = pt << 8 | pk;
                uint32_t l0 = 0, l1 = on;
                while (l0 < l1) {
                  const uint32_t md = (l0 + l1) >> 1;
                  if (a.nodes[3 * (ob + md)] < key) l0 = md + 1;
                  else l1 = md;
                }
                if (l0 < on && a.nodes[3 * (ob + l0)] == key) pred = (uint32_t)(ob + l0);
                else miss = 1;
              }
            }
            uint32_t *nd = a.nodes + 3 * r;
            nd[0] = t << 8 | k;
            nd[1] = (hdr[t] & 0xFFFFu) | (meta_rev(m) ? 1u << 16 : 0u);
            nd[2] = pred;
            ++r;
          }
        }
        nb_prev = nb;
        nb += acc2;
        cnt_last = acc2;
        uint32_t *const tp_ = Pc;
        Pc = Pp;
        Pp = tp_;
        B.sync();
      }
      miss = B.reduce_u64((unsigned long long)miss) != 0;
      if (tid == 0) {
        a.bnd_off[bi] = nb_prev;
        a.bnd_n[bi] = cnt_last;
        if (miss) a.status[bi] = EST_GC_MISS;
      }
    }
    B.sync();
    if (tid == 0) sq = atomicAdd(a.next_q, 1) + (int)gridDim.x;
    B.sync();
    q = sq;
  }
}

hipError_t launch_estep_trace_gc(const TraceGcArgs &a, int grid, hipStream_t st, int nw) {
  if (a.n_order <= 0) return hipSuccess;
  if (a.S < 1 || a.S > S_MAX || a.lo0 < a.head_len || a.mid <= a.lo0 || a.hi1 <= a.mid || a.hi1 > a.L + 1 || grid < 1 ||
      (nw != 1 && nw != 4))
    return hipErrorInvalidValue;
  // nw = 1: a wavefront per individual — the marking walks the loci one after
  // another, so more individuals in flight hide its latency
  if (nw == 4) hipLaunchKernelGGL(estep_trace_gc<4>, dim3(grid), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(estep_trace_gc<1>, dim3(grid), dim3(64), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_estep_structure(const StructArgs &a, int grid, int nw, hipStream_t st) {
  if (a.S < 1 || a.S > S_MAX || a.pan.amax > A_MAX || a.fcap > F_MAX || (a.hcap & (a.hcap - 1)) || a.lds_hc < 1 ||
      (a.lds_hc & (a.lds_hc - 1)) || a.lds_fc < 0 || a.lds_cc < 0 || a.ccap < 1 || a.mod.head_len < 1 ||
      (a.exact && a.ccap > EXACT_C_MAX) ||
      (a.mod.head_len > 1 && (!a.mod.hf_off || !a.mod.hf_pairs || !a.mod.hf_status)) ||
      (nw != 1 && nw != 4 && nw != 8 && nw != 16))
    return hipErrorInvalidValue;
  const size_t lds = estep_s1_lds_bytes(a.lds_fc, a.lds_hc, a.lds_cc, a.pan.amax, nw);
  const void *f = nw == 16 ? (const void *)estep_structure<16>
                           : (nw == 8 ? (const void *)estep_structure<8>
                                      : (nw == 4 ? (const void *)estep_structure<4> : (const void *)estep_structure<1>));
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (nw == 16) hipLaunchKernelGGL(estep_structure<16>, dim3(grid), dim3(16 * WAVE), lds, st, a);
  else if (nw == 8) hipLaunchKernelGGL(estep_structure<8>, dim3(grid), dim3(8 * WAVE), lds, st, a);
  else if (nw == 4) hipLaunchKernelGGL(estep_structure<4>, dim3(grid), dim3(4 * WAVE), lds, st, a);
  else hipLaunchKernelGGL(estep_structure<1>, dim3(grid), dim3(WAVE), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_estep_values(const ValueArgs &a, int grid, int nw, bool fast, int wpe, hipStream_t st, bool pair) {
  if (a.S < 1 || a.S > S_MAX || a.fcap > F_MAX || a.lds_fc < 0 || nw < 1 || nw > 16 || (wpe != 4 && wpe != 5) ||
      (a.S > 32 && fast) || (pair && (fast || a.S > 16)))
    return hipErrorInvalidValue;
  const size_t lds = estep_s2_lds_bytes(a.S, a.lds_fc, nw, pair);
  void (*k)(ValueArgs);
  if (a.S > 32) k = estep_values<false, 4, true>;  // lists of more than one wavefront: exact order only
  else if (pair) k = wpe == 5 ? estep_values<false, 5, false, true> : estep_values<false, 4, false, true>;
  else if (wpe == 5) k = fast ? estep_values<true, 5> : estep_values<false, 5>;
  else k = fast ? estep_values<true, 4> : estep_values<false, 4>;
  if (lds > 65536) {  // (per device: set on every launch that needs it)
    hipError_t e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(WAVE * nw), lds, st, a);
  return hipGetLastError();
}

}  // namespace hmc
