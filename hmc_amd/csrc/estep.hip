// estep.hip — E-step of the HaploModel EM on CDNA4 (gfx950).
//
// Restates HaploBuilder::resolve (HaploBuilder.cpp:35-126) with its helpers
// initHeadList (:153-224), extendAll/extend/addHaploPair (:226-261) and the
// HaploPair constructors/add (HaploPair.cpp:14-89), then the final k-best
// selection (HaploBuilder.cpp:87-116) and getGenotype traceback
// (HaploPair.cpp:91-124).
//
// Mapping: one 64-lane wavefront owns one individual and walks its loci left
// to right.  Per locus the wave
//   1. enumerates the (allele pair, state, orientation) contributions of
//      extendAll in the reference's order, 64 per chunk, one per lane;
//   2. inserts each successor key (id_a, id_b) into a per-wave open-address
//      table (atomicCAS) that replaces the per-pattern std::map m_best_pair;
//   3. groups lanes that hit the same key with a ballot loop, so every lane
//      knows its rank among contributions to that key in reference order;
//      new keys get state numbers in order of first occurrence (ballot prefix);
//   4. applies contributions round by round (round r = rank r inside the
//      chunk), so same-key merges stay in reference order while distinct keys
//      merge in parallel — create copies the predecessor's k-best list, add
//      appends and runs the libstdc++-exact nth_element of select.hpp on the
//      lane's private LDS column.
// Frontiers (fwd, pattern ids, k-best likelihoods/links) live in a per-wave
// HBM scratch region that stays L2-resident; the finished k-best link lists of
// every locus are streamed once into the trace store (4 B per link), which the
// traceback kernel reads to rebuild the sampled haplotypes.
//
// Arithmetic order follows the reference exactly; the file is compiled with
// -ffp-contract=off so `fwd += fwd_pred * tp` is not fused into an FMA.
#include "hmc_internal.hpp"
#include "select.hpp"
#include "coop_select.hpp"
#include "estep_common.hpp"

namespace hmc {

namespace {



// HBM-tier arrays of one frontier (states fc .. fcap-1 of the wave).
struct FrontG {
  double *fwd, *lik;
  uint32_t *lo, *hi, *nl, *slot, *meta;
};

__host__ __device__ inline size_t front_bytes(int fcap, int S) {
  return al256((size_t)fcap * 8) + 4 * al256((size_t)fcap * 4) + al256((size_t)fcap * S * 8) +
         al256((size_t)fcap * S * 4);
}

__device__ inline FrontG carve_front(char *&p, int fcap, int S) {
  FrontG f;
  f.fwd = (double *)p; p += al256((size_t)fcap * 8);
  f.lo = (uint32_t *)p; p += al256((size_t)fcap * 4);
  f.hi = (uint32_t *)p; p += al256((size_t)fcap * 4);
  f.nl = (uint32_t *)p; p += al256((size_t)fcap * 4);
  f.slot = (uint32_t *)p; p += al256((size_t)fcap * 4);
  f.lik = (double *)p; p += al256((size_t)fcap * S * 8);
  f.meta = (uint32_t *)p; p += al256((size_t)fcap * S * 4);
  return f;
}

// A frontier (m_haplopairs[i]): states [0, fc) live in LDS, states >= fc in
// the wave's HBM scratch.  Every accessor branches on the tier so both sides
// compile to native ds_* / global_* instructions.
struct Front {
  int fc, S;
  int o_fwd, o_lo, o_hi, o_nl, o_slot, o_lik, o_meta;  // LDS byte offsets
  FrontG g;
};

struct Lds {
  unsigned char *base;
  __device__ double *d(int off) const { return (double *)(base + off); }
  __device__ uint32_t *u(int off) const { return (uint32_t *)(base + off); }
};

// Accessors select a flat pointer into the state's tier instead of branching,
// so lanes whose states sit in different tiers stay converged and a list's S
// loads issue back to back.
#define FR_SCALAR(NAME, T, ARR, OFF)                                                  \
  __device__ inline T *NAME##_ptr(const Lds &l, const Front &F, int t) {              \
    return t < F.fc ? (T *)(l.base + F.OFF) + t : F.g.ARR + (t - F.fc);               \
  }                                                                                   \
  __device__ inline T get_##NAME(const Lds &l, const Front &F, int t) { return *NAME##_ptr(l, F, t); } \
  __device__ inline void set_##NAME(const Lds &l, const Front &F, int t, T v) { *NAME##_ptr(l, F, t) = v; }
FR_SCALAR(fwd, double, fwd, o_fwd)
FR_SCALAR(lo, uint32_t, lo, o_lo)
FR_SCALAR(hi, uint32_t, hi, o_hi)
FR_SCALAR(nl, uint32_t, nl, o_nl)
FR_SCALAR(slot, uint32_t, slot, o_slot)
#undef FR_SCALAR

__device__ inline double *lik_ptr(const Lds &l, const Front &F, int t) {
  return t < F.fc ? (double *)(l.base + F.o_lik) + t * F.S : F.g.lik + (size_t)(t - F.fc) * F.S;
}
__device__ inline uint32_t *meta_ptr(const Lds &l, const Front &F, int t) {
  return t < F.fc ? (uint32_t *)(l.base + F.o_meta) + t * F.S : F.g.meta + (size_t)(t - F.fc) * F.S;
}
__device__ inline double get_lik(const Lds &l, const Front &F, int t, int k) { return lik_ptr(l, F, t)[k]; }
__device__ inline uint32_t get_meta(const Lds &l, const Front &F, int t, int k) { return meta_ptr(l, F, t)[k]; }
__device__ inline void set_link(const Lds &l, const Front &F, int t, int k, double x, uint32_t m) {
  lik_ptr(l, F, t)[k] = x;
  meta_ptr(l, F, t)[k] = m;
}

// Key table replacing m_best_pair: slot ids < hc are LDS slots, >= hc HBM slots.
struct Keys {
  int hc, nw, o_key, o_cnt, o_state, o_lanes;  // LDS tier (nw lane-mask words per slot)
  unsigned long long *gkey, *glanes;        // HBM tier
  uint32_t *gcnt, *gstate;
  uint32_t gmask;
};

// Insert-or-find: a key lands in the first free or matching slot of its LDS
// probe sequence (at most PROBE_LDS slots), else in the HBM table.  Slots never
// empty during a locus, so every lane holding the same key ends in one slot.
__device__ inline uint32_t key_slot(const Lds &l, const Keys &K, unsigned long long key, uint32_t h0) {
  unsigned long long *lk = (unsigned long long *)(l.base + K.o_key);
  uint32_t h = h0 & (uint32_t)(K.hc - 1);
  for (int p = 0; p < PROBE_LDS; ++p) {
    const unsigned long long prev = atomicCAS(&lk[h], KEY_EMPTY, key);
    if (prev == KEY_EMPTY || prev == key) return h;
    h = (h + 1) & (uint32_t)(K.hc - 1);
  }
  uint32_t g = (h0 * 0x9E3779B1u) & K.gmask;
  while (true) {
    const unsigned long long prev = atomicCAS(&K.gkey[g], KEY_EMPTY, key);
    if (prev == KEY_EMPTY || prev == key) return (uint32_t)K.hc + g;
    g = (g + 1) & K.gmask;
  }
}
__device__ inline uint32_t slot_cnt(const Lds &l, const Keys &K, uint32_t s) {
  return s < (uint32_t)K.hc ? ((uint32_t *)(l.base + K.o_cnt))[s] : K.gcnt[s - K.hc];
}
__device__ inline void set_slot_cnt(const Lds &l, const Keys &K, uint32_t s, uint32_t v) {
  if (s < (uint32_t)K.hc) ((uint32_t *)(l.base + K.o_cnt))[s] = v;
  else K.gcnt[s - K.hc] = v;
}
__device__ inline uint32_t slot_state(const Lds &l, const Keys &K, uint32_t s) {
  return s < (uint32_t)K.hc ? ((uint32_t *)(l.base + K.o_state))[s] : K.gstate[s - K.hc];
}
__device__ inline void set_slot_state(const Lds &l, const Keys &K, uint32_t s, uint32_t v) {
  if (s < (uint32_t)K.hc) ((uint32_t *)(l.base + K.o_state))[s] = v;
  else K.gstate[s - K.hc] = v;
}
// Threads of the current chunk holding each key: one 64-bit lane mask per
// wave (OR is order-free, so the grouping needs no serial ballot loop).
__device__ inline void slot_or_lanes(const Lds &l, const Keys &K, uint32_t s, int w, unsigned long long bit) {
  if (s < (uint32_t)K.hc) atomicOr(&((unsigned long long *)(l.base + K.o_lanes))[s * K.nw + w], bit);
  else atomicOr(&K.glanes[(size_t)(s - K.hc) * K.nw + w], bit);
}
__device__ inline unsigned long long slot_lanes(const Lds &l, const Keys &K, uint32_t s, int w) {
  return s < (uint32_t)K.hc ? ((unsigned long long *)(l.base + K.o_lanes))[s * K.nw + w]
                            : __hip_atomic_load(&K.glanes[(size_t)(s - K.hc) * K.nw + w], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void clear_slot_lanes(const Lds &l, const Keys &K, uint32_t s) {
  for (int w = 0; w < K.nw; ++w) {
    if (s < (uint32_t)K.hc) ((unsigned long long *)(l.base + K.o_lanes))[s * K.nw + w] = 0ull;
    else atomicExch(&K.glanes[(size_t)(s - K.hc) * K.nw + w], 0ull);
  }
}
__device__ inline void clear_slot(const Lds &l, const Keys &K, uint32_t s) {
  if (s < (uint32_t)K.hc) {
    ((unsigned long long *)(l.base + K.o_key))[s] = KEY_EMPTY;
    ((uint32_t *)(l.base + K.o_cnt))[s] = 0;
  } else {
    K.gkey[s - K.hc] = KEY_EMPTY;
    K.gcnt[s - K.hc] = 0;
  }
}

// Block-wide scalars exchanged through LDS (a block = one individual, NW waves).
struct BlockShared {
  unsigned long long u[2];
  int i[4];
  int wcnt[4];   // per-wave counts (new states / selection adds)
  int wmax[4];   // per-wave maxima
};

// Bump-allocate `words` contiguous trace words for this block (block-uniform call).
__device__ inline unsigned long long trace_alloc(const EstepArgs &a, BlockShared *bs, unsigned long long &cur,
                                                 unsigned long long &end, unsigned long long words) {
  if (cur + words > end) {
    unsigned long long take = words > TRACE_CHUNK ? words : TRACE_CHUNK;
    if (threadIdx.x == 0) bs->u[0] = atomicAdd(a.trace_cursor, take);
    __syncthreads();
    const unsigned long long base = bs->u[0];
    __syncthreads();
    cur = base;
    end = base + take;
  }
  unsigned long long off = cur;
  cur += words;
  return off;
}

// Stream the finished k-best lists of one locus into the trace store.
__device__ inline bool write_trace(const EstepArgs &a, const Lds &l, BlockShared *bs, const Front &F, int Fn,
                                   int locus, int bi, unsigned long long &cur, unsigned long long &end) {
  const int S = a.S, NT = (int)blockDim.x;
  // +1: the link block starts on an even word (8-byte aligned), see trace_links()
  const unsigned long long words = 2ull + (unsigned long long)Fn * (1 + S);
  const unsigned long long off = trace_alloc(a, bs, cur, end, words);
  if (off + words > a.trace_cap) return false;
  uint32_t *hdr = a.trace + off + 1;
  uint32_t *lnk = a.trace + trace_links(off, (uint32_t)Fn);
  for (int t = threadIdx.x; t < Fn; t += NT)
    hdr[t] = hdr_pack(a.mod.last[get_lo(l, F, t)], a.mod.last[get_hi(l, F, t)], get_nl(l, F, t));
  // one thread per state: its S link words (zero past nl), the loads of each
  // 16-word chunk issued before its stores (the source may be LDS or HBM)
  for (int t = threadIdx.x; t < Fn; t += NT) {
    const uint32_t n = get_nl(l, F, t);
    const uint32_t *pm = meta_ptr(l, F, t);
    uint32_t *dst = lnk + (size_t)t * S;
    for (int k0 = 0; k0 < S; k0 += 16) {
      uint32_t v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k0 + k < S) v[k] = pm[k0 + k];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k0 + k < S) dst[k0 + k] = (uint32_t)(k0 + k) < n ? v[k] : 0u;
    }
  }
  if (threadIdx.x == 0) {
    a.trace[off] = (uint32_t)Fn;
    a.loc_off[(size_t)bi * (a.pan.L + 1) + locus] = off;
  }
  return true;
}

}  // namespace

size_t estep_scratch_bytes(int fcap, int hcap, int S, int nw) {
  return al256(2 * front_bytes(fcap, S) + al256((size_t)hcap * 8) + al256((size_t)hcap * 8 * nw) +
               al256((size_t)hcap * 4) + al256((size_t)hcap * 4));
}

// One add handed to a selection segment.
struct AddPar {
  double tpv;
  uint32_t st, s;
  uint32_t k0ns;   // k0 | ns << 8 | rev << 16 | differ << 17
  uint32_t pad;
};

// LDS carve of one block (nw waves, one individual): [per-wave selection
// scratch] [add parameters] [block scalars] [allele pairs] [key table hc x
// (key, cnt, state, nw lane masks)] [frontier A] [frontier B], each frontier
// fc x (fwd, lo, hi, nl, slot, lik[S], meta[S]).
struct LdsPlan {
  int o_lpos, o_rpos, o_junk, o_slik, o_smeta, o_par, o_bs, o_pairs, o_key, o_cnt, o_state, o_lanes, o_front[2][7],
      bytes;
};

__host__ __device__ inline LdsPlan lds_plan(int S, int fc, int hc, int nw, int npm) {
  LdsPlan p;
  int o = 0;
  auto take = [&](int bytes) { int r = o; o += (bytes + 15) & ~15; return r; };
  p.o_lpos = take(nw * WAVE * 4);
  p.o_rpos = take(nw * WAVE * 4);
  p.o_junk = take(nw * 2 * WAVE * 4);
  p.o_slik = take(nw * WAVE * 8);
  p.o_smeta = take(nw * WAVE * 4);
  p.o_par = take(nw * WAVE * (int)sizeof(AddPar));
  p.o_bs = take((int)sizeof(BlockShared));
  p.o_pairs = take((npm + 2) * 4 + 3 * npm);
  p.o_key = take(hc * 8);
  p.o_cnt = take(hc * 4);
  p.o_state = take(hc * 4);
  p.o_lanes = take(hc * 8 * nw);
  for (int f = 0; f < 2; ++f) {
    p.o_front[f][0] = take(fc * 8);       // fwd
    p.o_front[f][1] = take(fc * 4);       // lo
    p.o_front[f][2] = take(fc * 4);       // hi
    p.o_front[f][3] = take(fc * 4);       // nl
    p.o_front[f][4] = take(fc * 4);       // slot
    p.o_front[f][5] = take(fc * S * 8);   // lik
    p.o_front[f][6] = take(fc * S * 4);   // meta
  }
  p.bytes = o;
  return p;
}

size_t estep_lds_bytes(int S, int fc, int hc, int nw, int amax) {
  return (size_t)lds_plan(S, fc, hc, nw, amax * (amax + 1) / 2).bytes;
}

// Diagnostic build only (-DHMC_STAMPS): per-phase shader-clock shares.  Each
// stamp drains the wave's memory counters so a phase is charged with the
// latency of the loads it issued.  The product build compiles these out.
#ifdef HMC_STAMPS
#define STAMP_DECL unsigned long long st_t0 = __builtin_amdgcn_s_memtime(), st_acc[20] = {};
#define STAMP(k)                                              \
  do {                                                        \
    __builtin_amdgcn_s_waitcnt(0);                            \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t1 - st_t0;                                  \
    st_t0 = t1;                                               \
  } while (0)
// Per-lane shares inside divergent code (summed over lanes): 14, 15, 17-19.
#define DIAG_T0 \
  __builtin_amdgcn_s_waitcnt(0);                     \
  unsigned long long dg0 = __builtin_amdgcn_s_memtime();
#define DIAG(k)                                               \
  do {                                                        \
    __builtin_amdgcn_s_waitcnt(0);                            \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t1 - dg0;                                    \
    dg0 = t1;                                                 \
  } while (0)
#define STAMP_FLUSH                                                                       \
  if (a.stamps && (a.diag_indiv < 0 || a.diag_indiv == (int)blockIdx.x))                  \
    for (int k = 0; k < 20; ++k) {                                                        \
      const bool per_lane = k == 14 || k == 17;                                \
      if (per_lane || threadIdx.x == 0) atomicAdd(&a.stamps[k], st_acc[k]);               \
    }
#else
#define DIAG_T0
#define DIAG(k) do { } while (0)
#define STAMP_DECL
#define STAMP(k) do { } while (0)
#define STAMP_FLUSH
#endif

#ifdef HMC_VARIANTS  // (the fused single-pass kernel: tests of the variants library only)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void estep_forward(EstepArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  STAMP_DECL
  const int S = a.S, L = a.pan.L, amax = a.pan.amax;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid / WAVE;
  const int NT = blockDim.x, NW = NT / WAVE;
  const int npm = a.pan.amax * (a.pan.amax + 1) / 2;  // allele pairs of a fully missing locus
  const LdsPlan plan = lds_plan(S, a.lds_fc, a.lds_hc, NW, npm);
  const Lds l{smem};
  int *pr_off = (int *)(smem + plan.o_pairs);  // [npm+2]; [npm+1] = npairs
  uint8_t *pr_x = (uint8_t *)(pr_off + npm + 2);
  uint8_t *pr_y = pr_x + npm;
  uint8_t *pr_o = pr_y + npm;
  BlockShared *bs = (BlockShared *)(smem + plan.o_bs);
  // this wave's selection scratch
  const SegScratch ss{(int *)(smem + plan.o_lpos) + wv * WAVE, (int *)(smem + plan.o_rpos) + wv * WAVE,
                      (int *)(smem + plan.o_junk) + wv * 2 * WAVE, (double *)(smem + plan.o_slik) + wv * WAVE,
                      (uint32_t *)(smem + plan.o_smeta) + wv * WAVE};
  AddPar *par = (AddPar *)(smem + plan.o_par);
  const Seg sg = make_seg(2 * S);
  const int G = WAVE / (2 * S);
  const LinkList W{(double *)(smem + plan.o_slik), (uint32_t *)(smem + plan.o_smeta), 1};  // final selection

  char *sp = a.scratch + (size_t)blockIdx.x * a.scratch_stride;
  Front FA, FB;
  FA.g = carve_front(sp, a.fcap, S);
  FB.g = carve_front(sp, a.fcap, S);
  Keys K;
  K.gkey = (unsigned long long *)sp; sp += al256((size_t)a.hcap * 8);
  K.glanes = (unsigned long long *)sp; sp += al256((size_t)a.hcap * 8 * NW);
  K.gcnt = (uint32_t *)sp; sp += al256((size_t)a.hcap * 4);
  K.gstate = (uint32_t *)sp;
  K.gmask = (uint32_t)a.hcap - 1u;
  K.hc = a.lds_hc;
  K.nw = NW;
  K.o_key = plan.o_key;
  K.o_cnt = plan.o_cnt;
  K.o_state = plan.o_state;
  K.o_lanes = plan.o_lanes;
  Front *FF[2] = {&FA, &FB};
  for (int f = 0; f < 2; ++f) {
    FF[f]->fc = a.lds_fc;
    FF[f]->S = S;
    FF[f]->o_fwd = plan.o_front[f][0];
    FF[f]->o_lo = plan.o_front[f][1];
    FF[f]->o_hi = plan.o_front[f][2];
    FF[f]->o_nl = plan.o_front[f][3];
    FF[f]->o_slot = plan.o_front[f][4];
    FF[f]->o_lik = plan.o_front[f][5];
    FF[f]->o_meta = plan.o_front[f][6];
  }
  auto reset_tables = [&]() {
    for (int h = tid; h < a.hcap; h += NT) {
      K.gkey[h] = KEY_EMPTY;
      K.gcnt[h] = 0;
    }
    for (int h = tid; h < a.hcap * NW; h += NT) K.glanes[h] = 0ull;
    for (int h = tid; h < K.hc; h += NT) {
      ((unsigned long long *)(smem + K.o_key))[h] = KEY_EMPTY;
      ((uint32_t *)(smem + K.o_cnt))[h] = 0;
    }
    for (int h = tid; h < K.hc * NW; h += NT) ((unsigned long long *)(smem + K.o_lanes))[h] = 0ull;
  };
  reset_tables();
  unsigned long long tcur = 0, tend = 0;
  __syncthreads();

  // Individuals in the host's visit order (heaviest first: blocks b, b+256,
  // ... share a CU, so the heaviest ones land on distinct CUs).
  const int nvisit = a.order ? a.n_order : a.indiv_end - a.indiv_begin;
  for (int q = blockIdx.x; q < nvisit; q += gridDim.x) {
    const int bi = a.order ? a.order[q] : q;
    const int gi = a.indiv_begin + bi;
    const uchar2 *g = a.pan.geno_im + (size_t)gi * L;
    const int hl = a.mod.head_len;
    const unsigned long long t_indiv = __builtin_amdgcn_s_memtime();
    if (a.trace_base) {  // this individual's reserved trace region (exact sizes from the structure pass)
      tcur = a.trace_base[bi];
      tend = ~0ull;
    }
    int status = EST_OK;
    unsigned long long re = 0;
    int fbig = 0;
    Front X = FA, Y = FB;

    // ---- initHeadList (HaploBuilder.cpp:153-224) --------------------------
    // head_len == 1 on the device; longer heads from the host's list
    if (tid == 0 && hl > 1) {
      int Fp0 = 0;
      const int li = gi - a.mod.hf_base;
      int st0 = a.mod.hf_status[li];
      for (uint32_t t = a.mod.hf_off[li]; t < a.mod.hf_off[li + 1] && st0 == EST_OK; ++t) {
        if (Fp0 >= a.fcap) { st0 = EST_OVERFLOW_FRONTIER; break; }
        const uint32_t head = a.mod.hf_pairs[2 * t], q = a.mod.hf_pairs[2 * t + 1];
        const double tpv = a.mod.freq[head] * a.mod.freq[q];  // HaploPair.cpp:27-32
        const bool homo = (q == head);
        set_fwd(l, X, Fp0, homo ? tpv : tpv * 2.0);
        set_lo(l, X, Fp0, head);
        set_hi(l, X, Fp0, q);
        set_nl(l, X, Fp0, 1);
        set_link(l, X, Fp0, 0, tpv, meta_pack(0, 0, false, homo, true));
        ++Fp0;
      }
      bs->i[0] = Fp0;
      bs->i[1] = st0;
    }
    if (tid == 0 && hl == 1) {
      int Fp0 = 0, st0 = EST_OK;
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
          const uint32_t q = xk == MISSING ? a.mod.head_pat0[amax] : a.mod.head_pat0[xk];
          if (q == NONE) { st0 = EST_NO_HEAD_PATTERN; break; }
          if (q < head) continue;  // hp->id() >= head->id()
          if (Fp0 >= a.fcap) { st0 = EST_OVERFLOW_FRONTIER; break; }
          const double tpv = a.mod.freq[head] * a.mod.freq[q];  // HaploPair.cpp:27-32
          const bool homo = (q == head);
          set_fwd(l, X, Fp0, homo ? tpv : tpv * 2.0);
          set_lo(l, X, Fp0, head);
          set_hi(l, X, Fp0, q);
          set_nl(l, X, Fp0, 1);
          set_link(l, X, Fp0, 0, tpv, meta_pack(0, 0, false, homo, true));
          ++Fp0;
        }
        if (st0 != EST_OK) break;
      }
      bs->i[0] = Fp0;
      bs->i[1] = st0;
    }
    __syncthreads();
    int Fp = bs->i[0];
    status = bs->i[1];
    __syncthreads();
    if (status == EST_OK) {
      if (!write_trace(a, l, bs, X, Fp, hl, bi, tcur, tend)) status = EST_OVERFLOW_TRACE;
      for (int t = tid; t < Fp; t += NT) re += get_nl(l, X, t);
    }

    // ---- forward over loci (HaploBuilder.cpp:47-82) -----------------------
    for (int i = hl; i < L && status == EST_OK; ++i) {
      if (Fp == 0) { status = EST_UNRESOLVED; break; }
      STAMP(0);
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
      __syncthreads();
      const int npairs = pr_off[npm + 1];
      const int C = pr_off[npairs];
      int Fn = 0;

      for (int c0 = 0; c0 < C && status == EST_OK; c0 += NT) {
        const int c = c0 + tid;
        bool valid = c < C;
        uint32_t s = 0, lo = 0, hi = 0, slot = 0;
        bool rev = false;
        double fwd_s = 0.0, tpv = 0.0;
        bool differ = false;
        if (valid) {
          int p = 0;
          while (p + 1 < npairs && c >= pr_off[p + 1]) ++p;
          const int local = c - pr_off[p];
          const int o = pr_o[p] == 2 ? (local & 1) : 0;
          s = pr_o[p] == 2 ? (uint32_t)(local >> 1) : (uint32_t)local;
          const uint32_t x = o ? pr_y[p] : pr_x[p];
          const uint32_t y = o ? pr_x[p] : pr_y[p];
          fwd_s = get_fwd(l, X, s);
          valid = fwd_s > 0.0;  // extend(): forward_likelihood() <= 0 -> skip
          STAMP(1);
          if (valid) {
            const uint32_t sa = a.mod.succ[(size_t)get_lo(l, X, s) * amax + x];
            const uint32_t sb = a.mod.succ[(size_t)get_hi(l, X, s) * amax + y];
            STAMP(2);
            valid = sa != NONE && sb != NONE;
            rev = sa > sb;  // addHaploPair: id_a > id_b -> swap, reversed
            lo = rev ? sb : sa;
            hi = rev ? sa : sb;
            if (valid) {  // issue the pattern gathers early; consumed after the key work
              tpv = a.mod.tp[lo] * a.mod.tp[hi];
              differ = a.mod.last[lo] != a.mod.last[hi];
            }
          }
        }
        STAMP(3);
        if (valid) slot = key_slot(l, K, ((unsigned long long)lo << 32) | hi, key_hash(lo, hi));
        STAMP(4);
        // group threads by key: rank of each contribution among the chunk's with its key
        if (valid) slot_or_lanes(l, K, slot, wv, 1ull << lane);
        __syncthreads();
        int li = 0, gsz = 0;
        if (valid)
          for (int w = 0; w < NW; ++w) {
            const uint64_t gm = slot_lanes(l, K, slot, w);
            gsz += __popcll(gm);
            if (w < wv) li += __popcll(gm);
            else if (w == wv) li += __popcll(gm & lanemask_lt());
          }
        __syncthreads();
        if (valid && li == 0) clear_slot_lanes(l, K, slot);
        STAMP(5);
        const uint32_t cnt0 = valid ? slot_cnt(l, K, slot) : 0u;
        const bool is_new = valid && cnt0 == 0 && li == 0;
        const uint64_t nm = __ballot(is_new);
        if (lane == 0) bs->wcnt[wv] = __popcll(nm);
        __syncthreads();
        int pre = 0, tot = 0;
        for (int w = 0; w < NW; ++w) {
          const int cw = bs->wcnt[w];
          pre += w < wv ? cw : 0;
          tot += cw;
        }
        if (Fn + tot > a.fcap) { status = EST_OVERFLOW_FRONTIER; break; }
        uint32_t st = 0;
        if (is_new) {
          st = (uint32_t)(Fn + pre + __popcll(nm & lanemask_lt()));
          set_slot_state(l, K, slot, st);
          set_slot(l, Y, (int)st, slot);
        }
        Fn += tot;
        if (valid && li == 0) set_slot_cnt(l, K, slot, cnt0 + (uint32_t)gsz);
        __syncthreads();
        if (valid && !is_new) st = slot_state(l, K, slot);
        const uint32_t rank = cnt0 + (uint32_t)li;
        STAMP(6);

        // first contribution of a key: extension constructor (HaploPair.cpp:35-61), thread-parallel
        if (valid && rank == 0) {
          const uint32_t ns = get_nl(l, X, s);
          set_fwd(l, Y, st, fwd_s * tpv);
          set_lo(l, Y, st, lo);
          set_hi(l, Y, st, hi);
          set_nl(l, Y, st, ns);
          copy_extended(lik_ptr(l, X, s), meta_ptr(l, X, s), lik_ptr(l, Y, st), meta_ptr(l, Y, st), 0, (int)ns, s, tpv,
                        rev, differ);
        }
        // later contributions: HaploPair::add (HaploPair.cpp:63-89).  Round r
        // applies every contribution whose key rank inside the chunk is r, so
        // distinct keys merge in parallel and each key sees its adds in
        // reference order.  An add that still fits appends in place; adds that
        // overflow S are packed 64/(2S) per selection step, the steps dealt to
        // the block's waves, and keep the S best with the libstdc++-exact
        // segmented nth_element (coop_select.hpp).
        int rounds = (valid && rank != 0) ? li + 1 : 0;
        for (int o = 32; o > 0; o >>= 1) { const int t = __shfl_xor(rounds, o); rounds = t > rounds ? t : rounds; }
        if (lane == 0) bs->wmax[wv] = rounds;
        __syncthreads();
        for (int w = 0; w < NW; ++w) rounds = bs->wmax[w] > rounds ? bs->wmax[w] : rounds;
#ifdef HMC_STAMPS
        st_acc[10] += __popcll(__ballot(valid && rank != 0));
        st_acc[11] += rounds;
#endif
        for (int r = 0; r < rounds; ++r) {
          STAMP(7);
          bool sel = false;
          uint32_t k0 = 0, ns = 0;
          if (valid && rank != 0 && li == r) {
            DIAG_T0
            k0 = get_nl(l, Y, st);
            ns = get_nl(l, X, s);
            set_fwd(l, Y, st, get_fwd(l, Y, st) + fwd_s * tpv);
            if (k0 + ns <= (uint32_t)S) {  // room left: append, no selection
              copy_extended(lik_ptr(l, X, s), meta_ptr(l, X, s), lik_ptr(l, Y, st), meta_ptr(l, Y, st), (int)k0, (int)ns,
                            s, tpv, rev, differ);
              set_nl(l, Y, st, k0 + ns);
            } else {
              sel = true;
            }
            DIAG(14);
#ifdef HMC_STAMPS
            st_acc[17] += st < (uint32_t)a.lds_fc ? 1 : 0;
#endif
          }
          // number the overflowing adds across the block (chunk order)
          const uint64_t selm = __ballot(sel);
          if (lane == 0) bs->wcnt[wv] = __popcll(selm);
          __syncthreads();
          int spre = 0, nsel = 0;
          for (int w = 0; w < NW; ++w) {
            const int cw = bs->wcnt[w];
            spre += w < wv ? cw : 0;
            nsel += cw;
          }
          if (sel) {
            AddPar &P = par[spre + __popcll(selm & lanemask_lt())];
            P.tpv = tpv;
            P.st = st;
            P.s = s;
            P.k0ns = k0 | ns << 8 | (rev ? 1u << 16 : 0u) | (differ ? 1u << 17 : 0u);
          }
          __syncthreads();
          STAMP(13);
          const int nbatch = (nsel + G - 1) / G;
          for (int bt = wv; bt < nbatch; bt += NW) {
            const int nseg = nsel - bt * G < G ? nsel - bt * G : G;
            int n = 0;
            double v = 0.0;
            uint32_t m = 0, pst = 0;
            if (sg.g < nseg) {
              const AddPar P = par[bt * G + sg.g];
              const int pk0 = (int)(P.k0ns & 0xFF), pns = (int)((P.k0ns >> 8) & 0xFF);
              pst = P.st;
              n = pk0 + pns;
              if (sg.k < n) {
                const bool fromY = sg.k < pk0;
                const int q = fromY ? sg.k : sg.k - pk0;
                const double *pl = fromY ? lik_ptr(l, Y, (int)P.st) : lik_ptr(l, X, (int)P.s);
                const uint32_t *pm = fromY ? meta_ptr(l, Y, (int)P.st) : meta_ptr(l, X, (int)P.s);
                v = pl[q];
                m = pm[q];
                if (!fromY) {  // HaploPair::add transformation (HaploPair.cpp:63-80)
                  bool homo = meta_homo(m);
                  const bool prev = (P.k0ns >> 16) & 1u, pdiff = (P.k0ns >> 17) & 1u;
                  v = v * P.tpv;
                  if (pdiff && homo) {
                    if (prev) v = 0.0;
                    homo = false;
                  }
                  m = meta_pack(P.s, (uint32_t)q, prev, homo, false);
                }
              }
            }
            STAMP(15);
            seg_nth_element(v, m, n, S - 1, sg, ss);
            STAMP(19);
#ifdef HMC_STAMPS
            st_acc[18] += 1;
#endif
            if (sg.g < nseg && sg.k < S) {
              set_link(l, Y, (int)pst, sg.k, v, m);
              if (sg.k == 0) set_nl(l, Y, (int)pst, (uint32_t)S);
            }
            STAMP(12);
          }
          __syncthreads();
          STAMP(16);
        }
        STAMP(7);
      }
      if (status != EST_OK) break;
      if (Fn == 0) { status = EST_UNRESOLVED; break; }
      if (!write_trace(a, l, bs, Y, Fn, i + 1, bi, tcur, tend)) { status = EST_OVERFLOW_TRACE; break; }
      for (int t = tid; t < Fn; t += NT) {
        re += get_nl(l, Y, t);
        clear_slot(l, K, get_slot(l, Y, t));
      }
      fbig = Fn > fbig ? Fn : fbig;
      __syncthreads();
      Front T = X; X = Y; Y = T;
      Fp = Fn;
      STAMP(8);
    }
    if (status == EST_OK && Fp == 0) status = EST_UNRESOLVED;

    // ---- final selection (HaploBuilder.cpp:87-116) ------------------------
    if (status < 0) {  // aborted mid-locus: keys may be left in the tables
      __syncthreads();
      reset_tables();
    }
    for (int o = 32; o > 0; o >>= 1) re += __shfl_xor(re, o);
    if (tid == 0) bs->u[1] = 0ull;
    __syncthreads();
    if (lane == 0) atomicAdd(&bs->u[1], re);
    __syncthreads();
    if (tid == 0) {
      if (a.cost) a.cost[bi] = (int32_t)((__builtin_amdgcn_s_memtime() - t_indiv) >> 10);
      if (a.max_states) atomicMax(a.max_states, (unsigned)(fbig > Fp ? fbig : Fp));
      a.re_count[bi] = bs->u[1];
      a.status[bi] = status;
      if (a.fmax) a.fmax[bi] = fbig > Fp ? fbig : Fp;
#ifdef HMC_STAMPS  // diagnostic build: the slot carries the individual's shader time (kcycles)
      if (a.fmax) a.fmax[bi] = (int32_t)((__builtin_amdgcn_s_memtime() - t_indiv) >> 10);
#endif
      int cnt = 0;
      double total = 0.0;
      if (status == EST_OK) {
        for (int t = 0; t < Fp; ++t) {
          total += get_fwd(l, X, t);
          const uint32_t n = get_nl(l, X, t);
          for (uint32_t k = 0; k < n; ++k) {
            double lk = get_lik(l, X, t, k);
            const bool homo = meta_homo(get_meta(l, X, t, k));
            if (!homo) lk *= 2.0;
            W.set(cnt++, lk, meta_pack((uint32_t)t, k, false, homo, false));
          }
          if (cnt > S) {
            if (cnt <= 32) nth_element_greater_masks(W, cnt, S - 1, cnt);
            else nth_element_greater(W, cnt, S - 1);
            cnt = S;
          }
        }
        sort_greater(W, cnt, ss.lpos);  // the selection scratch is free here
        double coverage = 0.0;
        for (int c = 0; c < cnt; ++c) {
          const uint32_t m = W.m(c);
          const uint32_t t = meta_pred(m), k = meta_idx(m);
          const double own = get_lik(l, X, (int)t, (int)k);
          const double prior = meta_homo(m) ? own : own * 2.0;  // HaploPair.cpp:97-102
          const double post = prior / total;
          coverage += post;
          a.cand_state[(size_t)bi * S_MAX + c] = t;
          a.cand_idx[(size_t)bi * S_MAX + c] = k;
          a.prior[(size_t)bi * S_MAX + c] = prior;
          a.posterior[(size_t)bi * S_MAX + c] = post;
        }
        for (int c = 0; c < cnt; ++c)  // HaploModel.cpp:97-98
          a.weight[(size_t)bi * S_MAX + c] = a.posterior[(size_t)bi * S_MAX + c] / coverage;
      }
      a.total[bi] = total;
      a.ncand[bi] = cnt;
    }
    __syncthreads();
    STAMP(9);
  }
  STAMP_FLUSH
}

#endif  // HMC_VARIANTS

// Traceback (HaploPair::getGenotype, HaploPair.cpp:91-124): 16, 32 or 64
// lanes per individual, one per candidate; walks the trace store from locus L back to
// the head locus and writes both haplotypes as sample rows.
__global__ __launch_bounds__(256) void estep_traceback(TracebackArgs a) {
  // one lane per candidate, cw (16, 32 or 64) lanes per individual
  const int cw = a.S > 32 ? 64 : (a.S > 16 ? 32 : 16);
  const int q = blockIdx.x * (256 / cw) + threadIdx.x / cw;
  const int c = threadIdx.x % cw;
  if (q >= a.nbatch) return;
  const int bi = a.order ? a.order[q] : q;
  if (c >= a.ncand[bi]) return;
  const int L = a.L, S = a.S;
  const size_t h0 = (size_t)a.sample_base[bi] + 2 * c;
  uint8_t *row[2] = {a.rows + h0 * L, a.rows + (h0 + 1) * L};
  const unsigned long long *lo = a.loc_off + (size_t)bi * (L + 1);
  uint32_t st = a.cand_state[(size_t)bi * S_MAX + c];
  uint32_t idx = a.cand_idx[(size_t)bi * S_MAX + c];
  int ra = 0, rb = 1;
  // trace indices still in the store: from L down to full_lo (windowed E-step), else to the head
  const int jstop = a.full_lo > a.head_len ? a.full_lo : a.head_len + 1;
  for (int j = L; j >= jstop; --j) {
    const uint32_t *r = a.trace + lo[j];
    const uint32_t F = r[0];
    const uint32_t hdr = r[1 + st];
    const uint32_t m = a.trace[trace_links(lo[j], F) + (size_t)st * S + idx];
    row[ra][j - 1] = (uint8_t)(hdr & 0xFF);
    row[rb][j - 1] = (uint8_t)((hdr >> 8) & 0xFF);
    if (meta_rev(m)) { int t = ra; ra = rb; rb = t; }
    st = meta_pred(m);
    idx = meta_idx(m);
  }
  uint32_t hdr;  // the head pair's alleles at locus head_len - 1
  if (a.full_lo > a.head_len) {  // the survivor nodes below full_lo: the boundary list, then the chain
    const unsigned long long ob = a.bnd_off[bi];
    const uint32_t on = a.bnd_n[bi], key = st << 8 | idx;
    uint32_t l0 = 0, l1 = on;
    while (l0 < l1) {
      const uint32_t md = (l0 + l1) >> 1;
      if (a.nodes[3 * (ob + md)] < key) l0 = md + 1;
      else l1 = md;
    }
    unsigned long long nd = ob + l0;  // (present: the collection kept every entry reachable from the candidates' locus)
    for (int j = a.full_lo - 1; j > a.head_len; --j) {
      const uint32_t *x = a.nodes + 3 * nd;
      row[ra][j - 1] = (uint8_t)(x[1] & 0xFF);
      row[rb][j - 1] = (uint8_t)((x[1] >> 8) & 0xFF);
      if ((x[1] >> 16) & 1u) { int t = ra; ra = rb; rb = t; }
      nd = x[2];
    }
    st = a.nodes[3 * nd] >> 8;  // the head pair (HaploPair.cpp:112-120)
    hdr = a.nodes[3 * nd + 1];
  } else {
    hdr = a.trace[lo[a.head_len] + 1 + st];
  }
  row[ra][a.head_len - 1] = (uint8_t)(hdr & 0xFF);
  row[rb][a.head_len - 1] = (uint8_t)((hdr >> 8) & 0xFF);
  if (a.head_len > 1) {  // the head pair's patterns cover loci 0..head_len-1 (HaploPair.cpp:112-120)
    const int li = a.indiv_begin + bi - a.mod.hf_base;
    const uint32_t t = a.mod.hf_off[li] + st;
    const uint8_t *pa = a.mod.head_al + (size_t)a.mod.hf_pairs[2 * t] * a.head_len;
    const uint8_t *pb = a.mod.head_al + (size_t)a.mod.hf_pairs[2 * t + 1] * a.head_len;
    for (int k = 0; k < a.head_len - 1; ++k) {
      row[ra][k] = pa[k];
      row[rb][k] = pb[k];
    }
  }
  const double w = a.weight[(size_t)bi * S_MAX + c];
  a.w_out[h0] = w;
  a.w_out[h0 + 1] = w;
}

// Sample rows in slot layout -> locus-major dense samples: out[l][r] =
// in[rowmap[r]][l] (64x64 LDS tiles; rowmap lists the dense sample order,
// individuals in order, candidates in order, h0 then h1: HaploModel.cpp:105-106).
__global__ __launch_bounds__(256) void transpose_rows_u8(const uint8_t *in, const int32_t *rowmap, uint8_t *out,
                                                         int rows, int cols) {
  __shared__ uint8_t tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int k = threadIdx.x; k < 64 * 64; k += 256) {
    const int r = k / 64, c = k % 64;
    if (r0 + r < rows && c0 + c < cols) tile[r][c] = in[(size_t)rowmap[r0 + r] * cols + c0 + c];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 64 * 64; k += 256) {
    const int c = k / 64, r = k % 64;
    if (r0 + r < rows && c0 + c < cols) out[(size_t)(c0 + c) * rows + r0 + r] = tile[r][c];
  }
}

// [rows][cols] -> out[c][col0 + r] with leading dimension ld_out, 64x64 LDS tiles.
__global__ __launch_bounds__(256) void transpose_u8(const uint8_t *in, uint8_t *out, int rows, int cols,
                                                    int ld_out, int col0) {
  __shared__ uint8_t tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int k = threadIdx.x; k < 64 * 64; k += 256) {
    const int r = k / 64, c = k % 64;
    if (r0 + r < rows && c0 + c < cols) tile[r][c] = in[(size_t)(r0 + r) * cols + c0 + c];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 64 * 64; k += 256) {
    const int c = k / 64, r = k % 64;
    if (r0 + r < rows && c0 + c < cols) out[(size_t)(c0 + c) * ld_out + col0 + r0 + r] = tile[r][c];
  }
}

// Exclusive scan of in[i]*mul (one workgroup; n is at most a few 1e5).
__global__ __launch_bounds__(1024) void scan_i32(const int32_t *in, int32_t *out, int n, int mul, int32_t *total) {
  __shared__ int32_t part[1024];
  __shared__ int32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 1024) {
    const int i = base + threadIdx.x;
    const int32_t v = i < n ? in[i] * mul : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      int32_t t = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < n) out[i] = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

// Selected pair per individual (res_list.front(), HaploBuilder.cpp:115) or the
// input genotype when unresolved (HaploBuilder.cpp:117-124): out[n][2][L].
__global__ void gather_resolutions(const uint8_t *rows, int L, const int32_t *sbase, const int32_t *ncand,
                                   const uchar2 *geno_im, int i0, int n, uint8_t *out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)n * L) return;
  const int i = (int)(t / L), l = (int)(t % L);
  uint8_t a, b;
  if (ncand[i] > 0) {
    a = rows[(size_t)sbase[i] * L + l];
    b = rows[(size_t)(sbase[i] + 1) * L + l];
  } else {
    const uchar2 g = geno_im[(size_t)(i0 + i) * L + l];
    a = g.x;
    b = g.y;
  }
  out[((size_t)i * 2) * L + l] = a;
  out[((size_t)i * 2 + 1) * L + l] = b;
}

// HaploComp counters of one individual (HaploComp.cpp:29-76, Genotype.cpp:
// 44-55, 97-116, 160-175, 224-266): the input genotypes (phase as given)
// against the accepted resolution, one thread per individual.  cnt[i][6] =
// switch distance, heterozygous loci, (unused), -, min mismatches, non-missing
// loci; bad[i] = first locus where the two are inconsistent, else -1.
__global__ void haplocomp_counts(const uchar2 *geno_im, int i0, int n, int L, const uint8_t *res, int32_t *cnt,
                                 int32_t *bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uchar2 *g = geno_im + (size_t)(i0 + i) * L;
  const uint8_t *f0 = res + (size_t)i * 2 * L, *f1 = f0 + L;
  auto am = [](uint8_t x, uint8_t y) { return x == MISSING || y == MISSING || x == y; };  // Allele::isMatch
  auto match = [&](int k, bool rev) {
    const uchar2 r = g[k];
    return rev ? (am(r.x, f1[k]) && am(r.y, f0[k])) : (am(r.x, f0[k]) && am(r.y, f1[k]));
  };
  int het = 0, miss = 0, d1 = 0, d2 = 0, sd = 0, start = -1, bad_at = -1;
  bool rev = false;
  for (int k = 0; k < L; ++k) {
    const uchar2 r = g[k];
    const bool hm = r.x == MISSING || r.y == MISSING;
    het += am(r.x, r.y) ? 0 : 1;
    miss += hm ? 1 : 0;
    if (hm) continue;
    const bool mt = match(k, true), mf = match(k, false);
    d1 += mt ? 0 : 1;
    d2 += mf ? 0 : 1;
    if (bad_at >= 0) continue;
    if (start < 0) {  // getSwitchDistanceIgnoreMissing: the first locus not matching both ways
      if (mt && mf) continue;
      start = k;
      if (mt) rev = true;
      else if (mf) rev = false;
      else bad_at = k;
      continue;
    }
    if (rev ? mt : mf) continue;
    if (!(rev ? mf : mt)) {
      bad_at = k;
      continue;
    }
    rev = !rev;
    ++sd;
  }
  int32_t *c = cnt + (size_t)i * 6;
  c[0] = sd;
  c[1] = het;
  c[2] = 0;
  c[3] = 0;
  c[4] = d1 < d2 ? d1 : d2;
  c[5] = L - miss;
  bad[i] = bad_at;
}

hipError_t launch_haplocomp_counts(const uchar2 *geno_im, int i0, int n, int L, const uint8_t *res, int32_t *cnt,
                                   int32_t *bad, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(haplocomp_counts, dim3((n + 127) / 128), dim3(128), 0, st, geno_im, i0, n, L, res, cnt, bad);
  return hipGetLastError();
}

hipError_t launch_gather_resolutions(const uint8_t *rows, int L, const int32_t *sbase, const int32_t *ncand,
                                     const uchar2 *geno_im, int i0, int n, uint8_t *out, hipStream_t st) {
  const long long tot = (long long)n * L;
  if (tot <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_resolutions, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, rows, L, sbase, ncand,
                     geno_im, i0, n, out);
  return hipGetLastError();
}

// Test kernel: segmented selection, 64/sw lists per wave; list j (offset
// off[j], length n[j] <= sw) -> nth_element(nth[j]).
__global__ __launch_bounds__(64) void test_seg_nth(double *lik, uint32_t *tag, const int *off, const int *n,
                                                   const int *nth, int count, int sw) {
  __shared__ int lpos[64], rpos[64], junk[128];
  __shared__ double slik[64];
  __shared__ uint32_t smeta[64];
  const Seg sg = make_seg(sw);
  const int G = 64 / sw;
  const int j = blockIdx.x * G + sg.g;
  const bool mine = sg.mask != 0ull && j < count;
  const int nj = mine ? n[j] : 0;
  double v = 0.0;
  uint32_t m = 0;
  if (mine && sg.k < nj) {
    v = lik[off[j] + sg.k];
    m = tag[off[j] + sg.k];
  }
  const SegScratch ss{lpos, rpos, junk, slik, smeta};
  seg_nth_element(v, m, nj, mine ? nth[j] : 0, sg, ss);
  if (mine && sg.k < nj) {
    lik[off[j] + sg.k] = v;
    tag[off[j] + sg.k] = m;
  }
}

hipError_t launch_test_coop_nth(double *lik, uint32_t *tag, const int *off, const int *n, const int *nth, int count,
                                int sw, hipStream_t st) {
  if (sw < 2 || sw > 32) return hipErrorInvalidValue;
  const int G = 64 / sw;
  hipLaunchKernelGGL(test_seg_nth, dim3((count + G - 1) / G), dim3(WAVE), 0, st, lik, tag, off, n, nth, count, sw);
  return hipGetLastError();
}

#ifdef HMC_VARIANTS
hipError_t launch_estep(const EstepArgs &a, int grid, int nw, hipStream_t st) {
  if (a.S < 1 || a.S > 32 || a.pan.amax > A_MAX || a.fcap > F_MAX || (a.hcap & (a.hcap - 1)) ||
      a.lds_hc < 1 || (a.lds_hc & (a.lds_hc - 1)) || a.lds_fc < 0 || nw < 1 || nw > 4)
    return hipErrorInvalidValue;
  const size_t lds = estep_lds_bytes(a.S, a.lds_fc, a.lds_hc, nw, a.pan.amax);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void *)estep_forward, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(estep_forward, dim3(grid), dim3(WAVE * nw), lds, st, a);
  return hipGetLastError();
}

#else
hipError_t launch_estep(const EstepArgs &, int, int, hipStream_t) { return hipErrorNotSupported; }
#endif

hipError_t launch_traceback(const TracebackArgs &a, int, hipStream_t st) {
  if (a.nbatch <= 0) return hipSuccess;
  if (a.S < 1 || a.S > S_MAX) return hipErrorInvalidValue;
  const int per = 256 / (a.S > 32 ? 64 : (a.S > 16 ? 32 : 16));  // individuals per block
  hipLaunchKernelGGL(estep_traceback, dim3((a.nbatch + per - 1) / per), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_transpose_u8(const uint8_t *in, uint8_t *out, int rows, int cols, int ld_out, int col0,
                               hipStream_t st) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  hipLaunchKernelGGL(transpose_u8, dim3((cols + 63) / 64, (rows + 63) / 64), dim3(256), 0, st, in, out, rows, cols,
                     ld_out, col0);
  return hipGetLastError();
}

hipError_t launch_transpose_rows_u8(const uint8_t *in, const int32_t *rowmap, uint8_t *out, int rows, int cols,
                                    hipStream_t st) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  hipLaunchKernelGGL(transpose_rows_u8, dim3((cols + 63) / 64, (rows + 63) / 64), dim3(256), 0, st, in, rowmap, out,
                     rows, cols);
  return hipGetLastError();
}

hipError_t launch_scan_i32(const int32_t *in, int32_t *out_excl, int n, int mul, int32_t *total, hipStream_t st) {
  hipLaunchKernelGGL(scan_i32, dim3(1), dim3(1024), 0, st, in, out_excl, n, mul, total);
  return hipGetLastError();
}

}  // namespace hmc
