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

namespace hmc {

namespace {

constexpr unsigned long long KEY_EMPTY = ~0ull;
constexpr unsigned long long TRACE_CHUNK = 1ull << 16;  // words per bump allocation
constexpr int NP_MAX = A_MAX * (A_MAX + 1) / 2;          // allele pairs at a fully missing locus

struct Front {
  double *fwd;
  uint32_t *lo, *hi, *nl, *slot_of;
  double *lik;     // [fcap][S]
  uint32_t *meta;  // [fcap][S]
};

struct WaveScratch {
  Front f[2];
  unsigned long long *hkey;
  uint32_t *hcnt, *hstate;
};

__host__ __device__ inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

__host__ __device__ inline size_t front_bytes(int fcap, int S) {
  return al256((size_t)fcap * 8) + 4 * al256((size_t)fcap * 4) + al256((size_t)fcap * S * 8) +
         al256((size_t)fcap * S * 4);
}

__device__ inline Front carve_front(char *&p, int fcap, int S) {
  Front f;
  f.fwd = (double *)p; p += al256((size_t)fcap * 8);
  f.lo = (uint32_t *)p; p += al256((size_t)fcap * 4);
  f.hi = (uint32_t *)p; p += al256((size_t)fcap * 4);
  f.nl = (uint32_t *)p; p += al256((size_t)fcap * 4);
  f.slot_of = (uint32_t *)p; p += al256((size_t)fcap * 4);
  f.lik = (double *)p; p += al256((size_t)fcap * S * 8);
  f.meta = (uint32_t *)p; p += al256((size_t)fcap * S * 4);
  return f;
}

__device__ inline WaveScratch carve(char *base, int fcap, int hcap, int S) {
  WaveScratch w;
  char *p = base;
  w.f[0] = carve_front(p, fcap, S);
  w.f[1] = carve_front(p, fcap, S);
  w.hkey = (unsigned long long *)p; p += al256((size_t)hcap * 8);
  w.hcnt = (uint32_t *)p; p += al256((size_t)hcap * 4);
  w.hstate = (uint32_t *)p;
  return w;
}

__device__ inline uint32_t key_hash(uint32_t lo, uint32_t hi) {
  uint32_t h = lo * 0x9E3779B1u ^ (hi + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 13;
  return h;
}

__device__ inline uint64_t lanemask_lt() { return (1ull << threadIdx.x) - 1ull; }

// Bump-allocate `words` contiguous trace words for this wave (lane-uniform).
__device__ inline unsigned long long trace_alloc(const EstepArgs &a, unsigned long long &cur,
                                                 unsigned long long &end, unsigned long long words) {
  if (cur + words > end) {
    unsigned long long take = words > TRACE_CHUNK ? words : TRACE_CHUNK;
    unsigned long long base = 0;
    if (threadIdx.x == 0) base = atomicAdd(a.trace_cursor, take);
    base = __shfl(base, 0);
    cur = base;
    end = base + take;
  }
  unsigned long long off = cur;
  cur += words;
  return off;
}

// Stream the finished k-best lists of one locus into the trace store.
__device__ inline bool write_trace(const EstepArgs &a, const Front &F, int Fn, int locus, int bi,
                                   unsigned long long &cur, unsigned long long &end) {
  const int S = a.S, rec = 1 + S;
  unsigned long long words = (unsigned long long)Fn * rec;
  unsigned long long off = trace_alloc(a, cur, end, words);
  if (off + words > a.trace_cap) return false;
  for (unsigned long long w = threadIdx.x; w < words; w += WAVE) {
    uint32_t t = (uint32_t)(w / rec), k = (uint32_t)(w % rec);
    uint32_t v;
    if (k == 0) v = hdr_pack(a.mod.last[F.lo[t]], a.mod.last[F.hi[t]], F.nl[t]);
    else v = (k - 1 < F.nl[t]) ? F.meta[(size_t)t * S + k - 1] : 0u;
    a.trace[off + w] = v;
  }
  if (threadIdx.x == 0) a.loc_off[(size_t)bi * (a.pan.L + 1) + locus] = off;
  return true;
}

}  // namespace

size_t estep_scratch_bytes(int fcap, int hcap, int S) {
  return al256(2 * front_bytes(fcap, S) + al256((size_t)hcap * 8) + al256((size_t)hcap * 4) +
               al256((size_t)hcap * 4));
}

__global__ __launch_bounds__(64) void estep_forward(EstepArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int S = a.S, L = a.pan.L, amax = a.pan.amax;
  const int lane = threadIdx.x;
  double *wl = (double *)smem;                               // [2S][64]
  uint32_t *wm = (uint32_t *)(smem + (size_t)2 * S * WAVE * 8);  // [2S][64]
  int *pr_off = (int *)(smem + (size_t)2 * S * WAVE * 12);   // [NP_MAX+2]; [NP_MAX+1] = npairs
  uint8_t *pr_x = (uint8_t *)(pr_off + NP_MAX + 2);
  uint8_t *pr_y = pr_x + NP_MAX;
  uint8_t *pr_o = pr_y + NP_MAX;
  const LinkList W{wl + lane, wm + lane, WAVE};

  WaveScratch ws = carve(a.scratch + (size_t)blockIdx.x * a.scratch_stride, a.fcap, a.hcap, S);
  const uint32_t hmask = (uint32_t)a.hcap - 1u;
  for (int h = lane; h < a.hcap; h += WAVE) {
    ws.hkey[h] = KEY_EMPTY;
    ws.hcnt[h] = 0;
  }
  unsigned long long tcur = 0, tend = 0;
  __syncthreads();

  for (int gi = a.indiv_begin + blockIdx.x; gi < a.indiv_end; gi += gridDim.x) {
    const int bi = gi - a.indiv_begin;
    const uchar2 *g = a.pan.geno_im + (size_t)gi * L;
    const int hl = a.mod.head_len;
    int status = EST_OK;
    unsigned long long re = 0;
    Front X = ws.f[0], Y = ws.f[1];

    // ---- initHeadList (HaploBuilder.cpp:153-224), head_len == 1 ---------
    int Fp = 0;
    if (lane == 0) {
      const uchar2 g0 = g[0];
      const bool m0 = g0.x == MISSING, m1 = g0.y == MISSING;
      for (int hix = 0; hix < a.mod.n_head; ++hix) {
        const uint32_t head = a.mod.head_ids[hix];
        const uint8_t ah = a.mod.last[head];
        if (!(m0 || m1 || g0.x == ah || g0.y == ah)) continue;  // head->isMatch(genotype)
        uint8_t xs[A_MAX];
        int nx = 0;
        const bool hasAllele = g0.x == ah || g0.y == ah;
        if ((m0 && m1) || ((m0 || m1) && hasAllele)) {
          for (int x = 0; x < a.pan.anum[0]; ++x)
            if (a.pan.afreq[x] > 0) xs[nx++] = (uint8_t)x;
        } else if (!m0 && !m1 && g0.x != g0.y) {
          xs[nx++] = (ah == g0.x) ? g0.y : g0.x;
        } else {
          xs[nx++] = g0.x;  // may be missing: resolved below like findLongestMatchPattern
        }
        for (int k = 0; k < nx; ++k) {
          uint32_t q = xs[k] == MISSING ? a.mod.head_pat0[amax] : a.mod.head_pat0[xs[k]];
          if (q == NONE) { status = EST_NO_HEAD_PATTERN; break; }
          if (q < head) continue;  // hp->id() >= head->id()
          if (Fp >= a.fcap) { status = EST_OVERFLOW_FRONTIER; break; }
          const double tpv = a.mod.freq[head] * a.mod.freq[q];  // HaploPair.cpp:27-32
          const bool homo = (q == head);
          X.fwd[Fp] = homo ? tpv : tpv * 2.0;
          X.lo[Fp] = head;
          X.hi[Fp] = q;
          X.nl[Fp] = 1;
          X.lik[(size_t)Fp * S] = tpv;
          X.meta[(size_t)Fp * S] = meta_pack(0, 0, false, homo, true);
          ++Fp;
        }
        if (status != EST_OK) break;
      }
    }
    Fp = __shfl(Fp, 0);
    status = __shfl(status, 0);
    __syncthreads();
    if (status == EST_OK) {
      if (!write_trace(a, X, Fp, hl, bi, tcur, tend)) status = EST_OVERFLOW_TRACE;
      for (int t = lane; t < Fp; t += WAVE) re += X.nl[t];
    }

    // ---- forward over loci (HaploBuilder.cpp:47-82) -----------------------
    for (int i = hl; i < L && status == EST_OK; ++i) {
      if (Fp == 0) { status = EST_UNRESOLVED; break; }
      const uchar2 gg = g[i];
      if (lane == 0) {  // allele-pair list in extendAll call order
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
        pr_off[NP_MAX + 1] = np;
      }
      __syncthreads();
      const int npairs = pr_off[NP_MAX + 1];
      const int C = pr_off[npairs];
      int Fn = 0;

      for (int c0 = 0; c0 < C && status == EST_OK; c0 += WAVE) {
        const int c = c0 + lane;
        bool valid = c < C;
        uint32_t s = 0, lo = 0, hi = 0, slot = 0;
        bool rev = false;
        double fwd_s = 0.0;
        if (valid) {
          int p = 0;
          while (p + 1 < npairs && c >= pr_off[p + 1]) ++p;
          const int local = c - pr_off[p];
          const int o = pr_o[p] == 2 ? (local & 1) : 0;
          s = pr_o[p] == 2 ? (uint32_t)(local >> 1) : (uint32_t)local;
          const uint32_t x = o ? pr_y[p] : pr_x[p];
          const uint32_t y = o ? pr_x[p] : pr_y[p];
          fwd_s = X.fwd[s];
          valid = fwd_s > 0.0;  // extend(): forward_likelihood() <= 0 -> skip
          if (valid) {
            const uint32_t sa = a.mod.succ[(size_t)X.lo[s] * amax + x];
            const uint32_t sb = a.mod.succ[(size_t)X.hi[s] * amax + y];
            valid = sa != NONE && sb != NONE;
            rev = sa > sb;  // addHaploPair: id_a > id_b -> swap, reversed
            lo = rev ? sb : sa;
            hi = rev ? sa : sb;
          }
        }
        if (valid) {
          const unsigned long long key = ((unsigned long long)lo << 32) | hi;
          uint32_t h = key_hash(lo, hi) & hmask;
          while (true) {
            unsigned long long prev = atomicCAS(&ws.hkey[h], KEY_EMPTY, key);
            if (prev == KEY_EMPTY || prev == key) break;
            h = (h + 1) & hmask;
          }
          slot = h;
        }
        // group lanes by key, in lane (= reference) order
        int li = 0, gsz = 0;
        uint64_t rem = __ballot(valid);
        while (rem) {
          const int leader = __ffsll((long long)rem) - 1;
          const uint32_t lslot = (uint32_t)__builtin_amdgcn_readlane((int)slot, leader);
          const bool mine = valid && slot == lslot;
          const uint64_t grp = __ballot(mine);
          if (mine) {
            li = __popcll(grp & lanemask_lt());
            gsz = __popcll(grp);
          }
          rem &= ~grp;
        }
        const uint32_t cnt0 = valid ? ws.hcnt[slot] : 0u;
        const bool is_new = valid && cnt0 == 0 && li == 0;
        const uint64_t nm = __ballot(is_new);
        if (Fn + __popcll(nm) > a.fcap) { status = EST_OVERFLOW_FRONTIER; break; }
        uint32_t st = 0;
        if (is_new) {
          st = (uint32_t)(Fn + __popcll(nm & lanemask_lt()));
          ws.hstate[slot] = st;
          Y.slot_of[st] = slot;
        }
        Fn += __popcll(nm);
        if (valid && li == 0) ws.hcnt[slot] = cnt0 + (uint32_t)gsz;
        __syncthreads();
        if (valid && !is_new) st = ws.hstate[slot];
        const uint32_t rank = cnt0 + (uint32_t)li;

        for (int r = 0; __ballot(valid && li == r) != 0; ++r) {
          if (valid && li == r) {
            const double tpv = a.mod.tp[lo] * a.mod.tp[hi];
            const bool differ = a.mod.last[lo] != a.mod.last[hi];
            const uint32_t ns = X.nl[s];
            const double *pl = X.lik + (size_t)s * S;
            const uint32_t *pm = X.meta + (size_t)s * S;
            double *yl = Y.lik + (size_t)st * S;
            uint32_t *ym = Y.meta + (size_t)st * S;
            if (rank == 0) {  // extension constructor, HaploPair.cpp:35-61
              Y.fwd[st] = fwd_s * tpv;
              Y.lo[st] = lo;
              Y.hi[st] = hi;
              Y.nl[st] = ns;
              for (uint32_t k = 0; k < ns; ++k) {
                double lk = pl[k] * tpv;
                bool homo = meta_homo(pm[k]);
                if (differ && homo) {
                  if (rev) lk = 0.0;
                  homo = false;
                }
                yl[k] = lk;
                ym[k] = meta_pack(s, k, rev, homo, false);
              }
            } else {  // HaploPair::add, HaploPair.cpp:63-89
              const double inc = fwd_s * tpv;
              Y.fwd[st] = Y.fwd[st] + inc;
              const int k0 = (int)Y.nl[st];
              for (int k = 0; k < k0; ++k) W.set(k, yl[k], ym[k]);
              for (uint32_t k = 0; k < ns; ++k) {
                double lk = pl[k] * tpv;
                bool homo = meta_homo(pm[k]);
                if (differ && homo) {
                  if (rev) lk = 0.0;
                  homo = false;
                }
                W.set(k0 + (int)k, lk, meta_pack(s, k, rev, homo, false));
              }
              int n = k0 + (int)ns;
              if (n > S) {
                nth_element_greater(W, n, S - 1);
                n = S;
              }
              for (int k = 0; k < n; ++k) {
                yl[k] = W.l(k);
                ym[k] = W.m(k);
              }
              Y.nl[st] = (uint32_t)n;
            }
          }
          __syncthreads();
        }
      }
      if (status != EST_OK) break;
      if (Fn == 0) { status = EST_UNRESOLVED; break; }
      if (!write_trace(a, Y, Fn, i + 1, bi, tcur, tend)) { status = EST_OVERFLOW_TRACE; break; }
      for (int t = lane; t < Fn; t += WAVE) {
        re += Y.nl[t];
        const uint32_t sl = Y.slot_of[t];
        ws.hkey[sl] = KEY_EMPTY;
        ws.hcnt[sl] = 0;
      }
      if (lane == 0 && a.max_states) atomicMax(a.max_states, (unsigned)Fn);
      __syncthreads();
      Front T = X; X = Y; Y = T;
      Fp = Fn;
    }
    if (status == EST_OK && Fp == 0) status = EST_UNRESOLVED;

    // ---- final selection (HaploBuilder.cpp:87-116) ------------------------
    if (status < 0) {  // aborted mid-locus: keys may be left in the table
      for (int h = lane; h < a.hcap; h += WAVE) {
        ws.hkey[h] = KEY_EMPTY;
        ws.hcnt[h] = 0;
      }
    }
    for (int o = 32; o > 0; o >>= 1) re += __shfl_xor(re, o);
    if (lane == 0) {
      a.re_count[bi] = re;
      a.status[bi] = status;
      int cnt = 0;
      double total = 0.0;
      if (status == EST_OK) {
        for (int t = 0; t < Fp; ++t) {
          total += X.fwd[t];
          const uint32_t n = X.nl[t];
          for (uint32_t k = 0; k < n; ++k) {
            double lk = X.lik[(size_t)t * S + k];
            const bool homo = meta_homo(X.meta[(size_t)t * S + k]);
            if (!homo) lk *= 2.0;
            W.set(cnt++, lk, meta_pack((uint32_t)t, k, false, homo, false));
          }
          if (cnt > S) {
            nth_element_greater(W, cnt, S - 1);
            cnt = S;
          }
        }
        sort_greater_small(W, cnt);
        double coverage = 0.0;
        for (int c = 0; c < cnt; ++c) {
          const uint32_t m = W.m(c);
          const uint32_t t = meta_pred(m), k = meta_idx(m);
          const double own = X.lik[(size_t)t * S + k];
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
  }
}

// Traceback (HaploPair::getGenotype, HaploPair.cpp:91-124): 16 lanes per
// individual, one per candidate; walks the trace store from locus L back to
// the head locus and writes both haplotypes as sample rows.
__global__ __launch_bounds__(256) void estep_traceback(TracebackArgs a) {
  const int bi = blockIdx.x * 16 + threadIdx.x / 16;
  const int c = threadIdx.x % 16;
  if (bi >= a.nbatch || c >= a.ncand[bi]) return;
  const int L = a.L, S = a.S, rec = 1 + S;
  const size_t h0 = (size_t)a.sample_base[bi] + 2 * c;
  uint8_t *row[2] = {a.rows + h0 * L, a.rows + (h0 + 1) * L};
  const unsigned long long *lo = a.loc_off + (size_t)bi * (L + 1);
  uint32_t st = a.cand_state[(size_t)bi * S_MAX + c];
  uint32_t idx = a.cand_idx[(size_t)bi * S_MAX + c];
  int ra = 0, rb = 1;
  for (int j = L; j > a.head_len; --j) {
    const uint32_t *r = a.trace + lo[j] + (size_t)st * rec;
    const uint32_t hdr = r[0];
    const uint32_t m = r[1 + idx];
    row[ra][j - 1] = (uint8_t)(hdr & 0xFF);
    row[rb][j - 1] = (uint8_t)((hdr >> 8) & 0xFF);
    if (meta_rev(m)) { int t = ra; ra = rb; rb = t; }
    st = meta_pred(m);
    idx = meta_idx(m);
  }
  const uint32_t hdr = a.trace[lo[a.head_len] + (size_t)st * rec];
  row[ra][a.head_len - 1] = (uint8_t)(hdr & 0xFF);
  row[rb][a.head_len - 1] = (uint8_t)((hdr >> 8) & 0xFF);
  const double w = a.weight[(size_t)bi * S_MAX + c];
  a.w_out[h0] = w;
  a.w_out[h0 + 1] = w;
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

hipError_t launch_gather_resolutions(const uint8_t *rows, int L, const int32_t *sbase, const int32_t *ncand,
                                     const uchar2 *geno_im, int i0, int n, uint8_t *out, hipStream_t st) {
  const long long tot = (long long)n * L;
  if (tot <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_resolutions, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, rows, L, sbase, ncand,
                     geno_im, i0, n, out);
  return hipGetLastError();
}

hipError_t launch_estep(const EstepArgs &a, int grid, hipStream_t st) {
  if (a.S < 1 || a.S > S_MAX || a.pan.amax > A_MAX || a.fcap > 65535 || (a.hcap & (a.hcap - 1)))
    return hipErrorInvalidValue;
  const size_t lds = (size_t)2 * a.S * WAVE * 12 + (NP_MAX + 2) * 4 + 3 * NP_MAX;
  hipLaunchKernelGGL(estep_forward, dim3(grid), dim3(WAVE), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_traceback(const TracebackArgs &a, int, hipStream_t st) {
  if (a.nbatch <= 0) return hipSuccess;
  hipLaunchKernelGGL(estep_traceback, dim3((a.nbatch + 15) / 16), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_transpose_u8(const uint8_t *in, uint8_t *out, int rows, int cols, int ld_out, int col0,
                               hipStream_t st) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  hipLaunchKernelGGL(transpose_u8, dim3((cols + 63) / 64, (rows + 63) / 64), dim3(256), 0, st, in, out, rows, cols,
                     ld_out, col0);
  return hipGetLastError();
}

hipError_t launch_scan_i32(const int32_t *in, int32_t *out_excl, int n, int mul, int32_t *total, hipStream_t st) {
  hipLaunchKernelGGL(scan_i32, dim3(1), dim3(1024), 0, st, in, out_excl, n, mul, total);
  return hipGetLastError();
}

}  // namespace hmc
