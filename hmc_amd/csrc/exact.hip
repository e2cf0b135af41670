// exact.hip — the exact M-step (--exact-estimate) of the HaploModel EM on CDNA4.
//
// PatternManager::estimatePatterns (PatternManager.cpp:364-410) re-estimates
// pattern frequencies as expected counts under the current model instead of
// re-mining the sampled haplotypes.  Per individual, HaploBuilder::
// estimateFrequency (HaploBuilder.cpp:274-332) resolves the genotype, runs the
// backward pass over the forward links (calcBackwardLikelihood, :263-272,
// HaploPair.cpp:126-136) and, for every start locus, walks the candidates'
// ForwardPatternTree (PatternTree.cpp:179-212) carrying three state -> weight
// lists: both haplotypes of the pair match the pattern so far / only the a-side
// / only the b-side (:334-450).  A node's frequency is sum(weight * backward) /
// P(genotype); its pattern gains that frequency and, as prefix frequency, the
// parent node's.
//
// Here the structure pass (estep_split.hip) supplies the states, their
// incoming contributions in add order and, in exact mode, every locus's
// contributions in extendAll order (the forward links in push order):
//   exact_fb    one block per individual: forward likelihoods (the ordered sums
//               of HaploPair.cpp:42,66) and backward likelihoods (links[0]
//               then links[1], each in push order), stored per locus;
//   exact_walk  one wavefront per (individual, start locus): the trie walk,
//               depth first, with the three lists held densely per state of
//               the node's locus and gathered from each state's incoming
//               contributions (the reference scatters along forward links;
//               same terms).  Subtrees whose lists are all zero are skipped:
//               their nodes would add 0 to every frequency and prefix.
// Frequencies accumulate across individuals in 2^-44 fixed point with 64-bit
// integer atomics: the totals do not depend on the order in which waves or
// ranks add, so the result is deterministic and identical for any sharding.
// The reference sums its lists in std::map<HaploPair*, double> pointer order,
// which no restatement reproduces: the bar is 1e-6 relative (north star).
#include "hmc_internal.hpp"
#include "estep_common.hpp"
#include "exact.hpp"

namespace hmc {

namespace {

// The sum of a wavefront's 64 virtual lanes in one fixed butterfly order
// (xor 32, 16, ..., 1), for groups of GL lanes that each carry WAVE / GL
// virtual lanes (virtual lane gl + GL k in p[k]): the in-lane steps first,
// then the shuffles within the group.  Every GL gives the same double, so a
// walk of four items per wavefront sums exactly as the one-item walk.
template <int GL>
__device__ inline double group_sum_fixed(double (&p)[WAVE / GL]) {
  constexpr int NV = WAVE / GL;
#pragma unroll
  for (int s = NV / 2; s > 0; s >>= 1) {
    double q[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) q[k] = p[k] + p[k ^ s];
#pragma unroll
    for (int k = 0; k < NV; ++k) p[k] = q[k];
  }
  double x = p[0];
#pragma unroll
  for (int o = GL / 2; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

struct RecView {  // one locus record of the structure pass
  int F, C, NCH, CF, NP;  // states, stored contributions, chains, contributions in extendAll order, allele pairs
  const double *tpv;
  const uint32_t *hdr, *cb, *ct, *out, *npo;
  __device__ RecView(const uint32_t *R, bool head) { set(R, (int)R[0], (int)R[1], (int)R[2], R[3], head); }
  // from header words the caller already holds (exact_walk's per-depth cache)
  __device__ RecView(const uint32_t *R, int f, int c, int nch, uint32_t cfnp, bool head) { set(R, f, c, nch, cfnp, head); }
  __device__ void set(const uint32_t *R, int f, int c, int nch, uint32_t cfnp, bool head) {
    F = f;
    C = c;
    NCH = nch;
    CF = (int)(cfnp >> 10);
    NP = (int)(cfnp & 1023u);
    tpv = (const double *)(R + 4);
    hdr = R + 4 + 2 * F;
    cb = hdr + F;
    ct = cb + F + 1;
    out = head ? nullptr : ct + C + NCH;
    npo = head ? nullptr : out + CF;
  }
};

}  // namespace

// Forward and backward likelihoods of every state of every locus (block per individual).
__global__ __launch_bounds__(256) void exact_fb(ExactArgs a) {
  const int tid = threadIdx.x, NT = blockDim.x;
  const int L = a.L, hl = a.head_len;
  __shared__ int flag;
  for (int q = blockIdx.x; q < a.n_order; q += gridDim.x) {
    const int bi = a.order[q];
    const int st0 = a.status[bi];
    if (st0 != EST_OK && st0 != EST_OK_PRUNED) continue;
    const bool pruned = st0 == EST_OK_PRUNED;  // zero forward likelihoods are expected (not extended)
    const unsigned long long *roff = a.rec_off + (size_t)bi * (L + 1);
    unsigned long long *xo = a.x_off + (size_t)bi * (L + 1);
    // x-store layout per locus: fwd[F] then bwd[F] (doubles), even word offsets
    unsigned long long cur = a.x_base[bi];
    for (int j = hl; j <= L; ++j) {
      const RecView R(a.rec + roff[j], j == hl);
      if (tid == 0) xo[j] = cur;
      cur += 4ull * R.F + 2;
    }
    if (tid == 0) flag = 0;
    __syncthreads();
    // forward (HaploPair.cpp:27-32 head, :42 / :66 extension and add)
    {
      const RecView R(a.rec + roff[hl], true);
      double *fw = (double *)(a.x + xo[hl]);
      for (int t = tid; t < R.F; t += NT) {
        const bool homo = (R.hdr[t] >> 24) & 1u;
        fw[t] = homo ? R.tpv[t] : R.tpv[t] * 2.0;
      }
    }
    __syncthreads();
    for (int j = hl + 1; j <= L; ++j) {
      const RecView R(a.rec + roff[j], false);
      const double *fp = (const double *)(a.x + xo[j - 1]);
      double *fw = (double *)(a.x + xo[j]);
      for (int t = tid; t < R.F; t += NT) {
        const double tpv = R.tpv[t];
        double f = 0.0;
        for (uint32_t r = R.cb[t]; r < R.cb[t + 1]; ++r) {
          const double v = fp[cw_state(R.ct[r])] * tpv;
          f = r == R.cb[t] ? v : f + v;
        }
        fw[t] = f;
        if (!(f > 0.0) && j < L && !pruned) flag = 1;  // extend() would skip this pair (HaploBuilder.cpp:237)
      }
      __syncthreads();
    }
    // every thread reads the flag before any thread can reset it for the next
    // individual (the reset sits before the barrier at the top of the loop)
    const bool underflow = flag != 0;
    __syncthreads();
    if (underflow) {
      if (tid == 0) a.status[bi] = EST_NEEDS_EXACT;
      continue;
    }
    // backward: states of m_haplopairs[L] keep m_backward_likelihood = 1.0
    {
      const RecView R(a.rec + roff[L], L == hl);
      double *bw = (double *)(a.x + xo[L]) + R.F;
      for (int t = tid; t < R.F; t += NT) bw[t] = 1.0;
    }
    __syncthreads();
    for (int j = L - 1; j >= hl; --j) {
      const RecView R(a.rec + roff[j], j == hl);       // states s at locus j
      const RecView N(a.rec + roff[j + 1], false);     // their forward links
      const double *bn = (const double *)(a.x + xo[j + 1]) + N.F;
      double *bw = (double *)(a.x + xo[j]) + R.F;
      for (int s = tid; s < R.F; s += NT) {
        double b = 0.0;
        for (int pass = 0; pass < 2; ++pass) {  // m_forward_links[0], then [1], each in push order
          uint32_t off = 0;
          for (int p = 0; p < N.NP; ++p) {
            const uint32_t no = N.npo[p];
            for (uint32_t o = 0; o < no; ++o) {
              const uint32_t w = N.out[off + (uint32_t)s * no + o];
              if (w != NONE && (uint32_t)cw_rev(w) == (uint32_t)pass) {
                const uint32_t t = cw_state(w);
                b += bn[t] * N.tpv[t];
              }
            }
            off += (uint32_t)R.F * no;
          }
        }
        bw[s] = b;
      }
      __syncthreads();
    }
  }
}

// The walk's largest per-item span (exact_walk's scratch layout): the states
// of records max(s + d, head_len), d = 0..max_depth + 1, over every start
// locus s of every individual of the group (block per individual).
__global__ __launch_bounds__(256) void exact_span(ExactArgs a) {
  const int tid = threadIdx.x, NT = blockDim.x;
  const int L = a.L, hl = a.head_len;
  for (int q = blockIdx.x; q < a.n_order; q += gridDim.x) {
    const int bi = a.order[q];
    const int st0 = a.status[bi];
    if (st0 != EST_OK && st0 != EST_OK_PRUNED) continue;
    const unsigned long long *roff = a.rec_off + (size_t)bi * (L + 1);
    unsigned sp = 0;
    for (int s0 = tid; s0 < L; s0 += NT) {
      unsigned long long sum = 0;
      for (int d = 0; d <= a.max_depth + 1; ++d) {
        const int r = s0 + d > hl ? s0 + d : hl;
        if (r > L) break;
        sum += a.rec[roff[r]];
      }
      const unsigned v = (unsigned)(sum < 0xFFFFFFFFull ? sum : 0xFFFFFFFFull);
      sp = v > sp ? v : sp;
    }
    atomicMax(a.span_max, sp);
  }
}

// One contribution's terms into a child list set (HaploBuilder.cpp:375-427):
// ma / mb = the child's allele is the pair's a / b allele at this locus.
__device__ inline void walk_terms(bool ma, bool mb, bool rev, double w0, double w1, double w2, double tp, double &n0,
                                  double &n1, double &n2) {
  if (ma && mb) n0 += w0 * tp;
  else if (ma) n1 += w0 * tp * 0.5;
  else n2 += w0 * tp * 0.5;
  // a-side list follows the a haplotype: links[0] keep it on a, links[1] move it to b
  if (!rev ? ma : mb) (!rev ? n1 : n2) += w1 * tp;
  if (!rev ? mb : ma) (!rev ? n2 : n1) += w2 * tp;
}

// The ForwardPatternTree walk of HaploBuilder::estimateFrequency (:296-308,
// :334-450), one wavefront per (individual, start locus), sparse like the
// reference's maps.  A node's children are computed together: the states
// its non-zero states link to (forward links of the record, marked in an
// LDS bitmap and compacted in state order) gather, over their incoming
// contributions in record order, the three lists of every child whose allele
// their pair carries — a heterozygous state feeds two children from one pass
// over its contributions.  The children's lists are kept per depth, one slot
// per allele, so the walk descends into them in allele order without
// recomputing.  Each child's frequency is sum(weight * backward) over the
// union of reached states in state order (zero entries add +0.0).  Scratch
// invariant: every dense entry not in a touched list is 0.0 (the host zeroes
// the scratch before the launch and every item clears what it wrote).
#ifndef HMC_XWALK_WPE
#define HMC_XWALK_WPE 4  // resident waves per SIMD the walk's registers allow (tuning builds vary it)
#endif
template <int GL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HMC_XWALK_WPE))) void exact_walk(ExactArgs a) {
  extern __shared__ unsigned long long lds64[];  // per group: exact_walk_lds_bytes
  constexpr int NG = WAVE / GL;  // items walked at once by the wavefront, GL lanes each
  const int lane = threadIdx.x, g = lane / GL, gl = lane % GL;
  // this group's lanes of a wave ballot
  auto gballot = [&](bool p) -> unsigned long long {
    const unsigned long long b = __ballot(p);
    return GL == WAVE ? b : (b >> (g * GL)) & ((1ull << GL) - 1ull);
  };
  const int L = a.L, hl = a.head_len, W = a.width, maxd = a.max_depth;
  const int D = maxd + 2;
  unsigned long long *stk64 = lds64 + (size_t)g * (exact_walk_lds_bytes(maxd, a.fmax, a.width) / 8);
  unsigned long long *sdesc = stk64, *smask = stk64 + D;
  // per depth, read once per item: the record's offset, the x-store offset of its locus
  unsigned long long *droff = stk64 + 2 * D, *dxo = stk64 + 3 * D;
  // narrow tries (width <= XWALK_CACHE_W): per depth and slot, the non-zero
  // entries of the slot's lists among the first GL touched states (bit j), and the child ids
  const int wc = exact_walk_cache_w(W);
  unsigned long long *nzm = stk64 + 4 * D;
  int *snode = (int *)(nzm + (size_t)D * wc), *snext = snode + D, *sslot = snext + D, *tcnt = sslot + D;
  int *sF = tcnt + D, *soff = sF + D;        // per depth: the states of its locus, their first entry in the item's layout
  int *dC = soff + D, *dNCH = dC + D;        // per depth: the record's header words (RecView)
  uint32_t *dCFNP = (uint32_t *)(dNCH + D), *dnpo0 = dCFNP + D;  // ... and its first allele pair's out-degree
  int *dnzv = (int *)(dnpo0 + D);            // per depth: nzm holds its slots' masks
  int *schild = dnzv + D;                    // [D][wc]: the children of the node at depth d
  // per depth: the first GL entries of the touched list (u16 states; the rest,
  // and every entry when a locus has more than 65 536 states, in the scratch)
  uint16_t *tl16 = (uint16_t *)(schild + (size_t)D * wc);
  uint32_t *marks = (uint32_t *)(tl16 + (size_t)D * WAVE);  // [fmax/32 + 1] reached-state bitmap
  const int nwords = (a.fmax + 31) >> 5;
  const int tlc = a.fmax <= 65536 ? GL : 0;
  // one item per wave and at most 64 unordered allele pairs (width <= 10):
  // lane p holds pair p's alleles, and a node's pairs that carry an allele of
  // one of its children form one ballot, tested against the links' pair bits
  const bool pmk = GL == WAVE && W * (W + 1) / 2 <= WAVE;
  int px = 0;
  while ((px + 1) * (px + 2) / 2 <= lane) ++px;
  const int py = lane - px * (px + 1) / 2;
  const bool pin = lane < W * (W + 1) / 2;
  // The item's lists: per depth d, W slots of three lists over the F_d states
  // of d's locus (slot i of depth d at 3 (W soff[d] + i F_d)); the wave's
  // region holds the largest such span of any item (ExactArgs::span)
  double *lists = a.scratch + ((size_t)blockIdx.x * NG + g) * a.scratch_stride;  // [3 W span]
  double *cfreq = lists + (size_t)3 * W * a.span;                          // [maxd+2][W]
  uint32_t *touched = (uint32_t *)(cfreq + (size_t)(maxd + 2) * W);       // [span]: per depth at soff[d]
  auto slot = [&](int d, int i) { return lists + (size_t)3 * ((size_t)W * soff[d] + (size_t)i * sF[d]); };
  // entry j of depth d's touched list
  auto tget = [&](int d, int j) -> uint32_t { return j < tlc ? (uint32_t)tl16[d * WAVE + j] : touched[soff[d] + j]; };
  auto tput = [&](int d, int j, uint32_t t) {
    if (j < tlc) tl16[d * WAVE + j] = (uint16_t)t;
    else touched[soff[d] + j] = t;
  };
  for (int d = gl; d < D; d += GL) {
    tcnt[d] = 0;
    smask[d] = 0ull;
  }
  for (int w = gl; w < nwords; w += GL) marks[w] = 0u;
  __builtin_amdgcn_wave_barrier();
  __threadfence_block();
  const long long n_items = a.item1 < 0 ? (long long)a.n_order * L : a.item1;
  for (long long it = a.item0 + (long long)blockIdx.x * NG + g; it < n_items; it += (long long)gridDim.x * NG) {
    const int q = (int)(it / L), start = (int)(it % L);
    const int bi = a.order[q];
    const int root = a.tr_root[start];
    if (root < 0 || (a.status[bi] != EST_OK && a.status[bi] != EST_OK_PRUNED)) continue;
    const double pg = a.gprob[bi];  // P(genotype) of the last E-step (HaploModel.cpp:109, HaploBuilder.cpp:294)
    if (!(pg > 0.0)) continue;
    const unsigned long long *roff = a.rec_off + (size_t)bi * (L + 1);
    const unsigned long long *xo = a.x_off + (size_t)bi * (L + 1);
    const uint32_t *Rh = a.rec + roff[hl];
    const int Fh = (int)Rh[0];
    {  // the item's layout: depth d's states are those of record max(start + d, head_len);
       // each depth's record header and offsets are read here once
      int carry = 0;
      for (int d0 = 0; d0 < D; d0 += GL) {
        const int dd = d0 + gl;
        const int r = start + dd > hl ? start + dd : hl;
        const bool has = dd < D && r <= L;
        int f = 0;
        if (has) {
          const unsigned long long ro = roff[r];
          const uint32_t *R = a.rec + ro;
          const uint32_t hx = R[0], hy = R[1], hz = R[2], hw = R[3];  // F, C, NCH, CF << 10 | NP
          f = (int)hx;
          droff[dd] = ro;
          dxo[dd] = xo[r];
          dC[dd] = (int)hy;
          dNCH[dd] = (int)hz;
          dCFNP[dd] = hw;
          // out-degree of the first allele pair (npo[0]) of a non-head record
          dnpo0[dd] = r > hl && (hw & 1023u) > 0u ? R[4 + 4 * (size_t)f + 1 + hy + hz + (hw >> 10)] : 0u;
        }
        int incl = f;
#pragma unroll
        for (int o = 1; o < GL; o <<= 1) {
          const int y = __shfl_up(incl, o, GL);
          if (gl >= o) incl += y;
        }
        if (dd < D) {
          sF[dd] = f;
          soff[dd] = carry + incl - f;
        }
        carry += __shfl(incl, GL - 1, GL);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    // depth 0: every state after max(start, head_len) loci, weight = forward likelihood
    {
      const int F0 = sF[0];
      const double *fw = (const double *)(a.x + dxo[0]);
      double *S0 = slot(0, 0);
      for (int t = gl; t < F0; t += GL) {
        S0[3 * t] = fw[t];
        tput(0, t, (uint32_t)t);
      }
      if (gl == 0) {
        tcnt[0] = F0;
        smask[0] = 1ull;
        snode[0] = root;
        snext[0] = -1;  // children not computed yet
        sslot[0] = 0;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    int d = 0;
    while (d >= 0) {
      __builtin_amdgcn_wave_barrier();
      __threadfence_block();
      const int node = snode[d];
      if (snext[d] < 0) {  // ---- all children of this node, into depth d+1 ----
        unsigned long long cm = 0ull;  // alleles with a child
        // (one item per wave: lane i holds child i and its pattern, read here once)
        int chv = -1, patv = -1;
        if (d < maxd) {
          if constexpr (GL == WAVE) {
            chv = gl < W ? a.tr_child[(size_t)node * W + gl] : -1;
            cm = gballot(chv >= 0);
            patv = chv >= 0 ? a.tr_data[chv] : -1;
            if (gl < wc) schild[d * wc + gl] = chv;
          } else {
            for (int i0 = 0; i0 < W; i0 += GL) {
              const int i = i0 + gl;
              cm |= gballot(i < W && a.tr_child[(size_t)node * W + i] >= 0) << i0;
            }
          }
        }
        if (cm == 0ull) {  // node done
          --d;
          continue;
        }
        const int locus = start + d;  // the children's allele is at this locus
        const double last_freq = d == 0 ? 1.0 : cfreq[(size_t)d * W + sslot[d]];  // prefix freq (HaploBuilder.cpp:305)
        const double *P0 = slot(d, sslot[d]), *P1 = P0 + 1, *P2 = P0 + 2;  // [F][3]: n0 n1 n2 of a state together
        {  // the previous sibling's children at depth d+1 back to zero
          const int nc = tcnt[d + 1];
          const unsigned long long wm = smask[d + 1];
          for (int j = gl; j < nc; j += GL) {
            const uint32_t t = tget(d + 1, j);
            for (unsigned long long m = wm; m; m &= m - 1) {
              double *C0 = slot(d + 1, __builtin_ctzll(m));
              C0[3 * t] = 0.0;
              C0[3 * t + 1] = 0.0;
              C0[3 * t + 2] = 0.0;
            }
          }
        }
        int ntc = 0;
        const double *bw;
        // one reached state per lane (ntc <= GL, not the head): its children's
        // three weights stay in registers for the frequencies (4)
        bool regs = false;
        uint32_t rxa = 0, rxb = 0;
        bool rca = false, rcb = false;
        double ra0 = 0.0, ra1 = 0.0, ra2 = 0.0, rb0 = 0.0, rb1 = 0.0, rb2 = 0.0, rbw = 0.0;
        if (locus < hl) {  // head pairs: their patterns' alleles (HaploBuilder.cpp:340-367), same states
          const RecView R(Rh, true);
          const uint32_t *plo = R.cb + Fh + 1, *phi = plo + Fh;
          bw = (const double *)(a.x + xo[hl]) + Fh;
          for (int t = gl; t < Fh; t += GL) {
            uint32_t xa, xb;
            if (hl == 1) {
              xa = R.hdr[t] & 0xFFu;
              xb = (R.hdr[t] >> 8) & 0xFFu;
            } else {
              xa = a.head_al[(size_t)plo[t] * hl + locus];
              xb = a.head_al[(size_t)phi[t] * hl + locus];
            }
            const double w0 = P0[3 * t], w1 = P1[3 * t], w2 = P2[3 * t];
            for (unsigned long long m = cm; m; m &= m - 1) {
              const uint32_t i = (uint32_t)__builtin_ctzll(m);
              const bool ma = xa == i, mb = xb == i;
              double n0 = 0.0, n1 = 0.0, n2 = 0.0;
              if (ma) {
                if (mb) n0 = w0;
                else n1 = w0 * 0.5;
              } else if (mb) {
                n2 = w0 * 0.5;
              }
              if (ma) n1 += w1;
              if (mb) n2 += w2;
              double *C0 = slot(d + 1, (int)i);
              C0[3 * t] = n0;
              C0[3 * t + 1] = n1;
              C0[3 * t + 2] = n2;
            }
            tput(d + 1, t, (uint32_t)t);
          }
          ntc = Fh;
        } else {  // along the forward links into the states after `locus` (:369-427)
          // depth d's record is `locus`, depth d+1's `locus + 1` (both >= head_len)
          const RecView R(a.rec + droff[d + 1], sF[d + 1], dC[d + 1], dNCH[d + 1], dCFNP[d + 1], false);
          const uint32_t npo0 = dnpo0[d + 1];
          bw = (const double *)(a.x + dxo[d + 1]) + R.F;
          // (1) mark the states the parent's non-zero states link to and whose
          //     pair carries the allele of some child on either side
          const int np = tcnt[d];
          const int Fp = sF[d];  // states the links leave from
          const unsigned long long pm = pmk ? __ballot(pin && (((cm >> px) & 1ull) || ((cm >> py) & 1ull))) : 0ull;
          // the parent's non-zero entries among its first GL states, when its
          // parent computed them in registers (otherwise the lists are read)
          const bool nzk = wc > 0 && d > 0 && dnzv[d] != 0;
          const unsigned long long nzb = nzk ? nzm[d * wc + sslot[d]] : ~0ull;
          for (int j = gl; j < np; j += GL) {
            const uint32_t s = tget(d, j);
            if (nzk && j < GL) {
              if (!((nzb >> j) & 1ull)) continue;
            } else if (P0[3 * s] == 0.0 && P1[3 * s] == 0.0 && P2[3 * s] == 0.0) {
              continue;
            }
            uint32_t off = 0;
            for (int p = 0; p < R.NP; ++p) {
              const uint32_t no = p == 0 ? npo0 : R.npo[p];
              // four links at a time: their words, then their pairs' alleles, then the marks
              for (uint32_t o = 0; o < no; o += 4) {
                uint32_t wv[4], hv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) wv[u] = o + u < no ? R.out[off + s * no + o + u] : NONE;
#pragma unroll
                for (int u = 0; u < 4; ++u) hv[u] = !pmk && wv[u] != NONE ? R.hdr[cw_state(wv[u])] : 0u;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                  if (wv[u] != NONE && (pmk ? ((pm >> cw_xpair(wv[u])) & 1ull) != 0ull
                                            : (((cm >> (hv[u] & 0xFFu)) & 1ull) || ((cm >> ((hv[u] >> 8) & 0xFFu)) & 1ull)))) {
                    const uint32_t t = cw_state(wv[u]);
                    atomicOr(&marks[t >> 5], 1u << (t & 31u));
                  }
              }
              off += (uint32_t)Fp * no;
            }
          }
          __builtin_amdgcn_wave_barrier();
          __threadfence_block();
          // (2) the marked states in ascending order; the bitmap back to zero
          const int nw = (R.F + 31) >> 5;
          for (int w0 = 0; w0 < nw; w0 += GL) {
            const int w = w0 + gl;
            uint32_t bits = w < nw ? marks[w] : 0u;
            const int c = __popc(bits);
            int incl = c;
#pragma unroll
            for (int dd = 1; dd < GL; dd <<= 1) {
              const int y = __shfl_up(incl, dd);
              if (gl >= dd) incl += y;
            }
            int at = ntc + incl - c;
            while (bits) {
              const int b = __builtin_ctz(bits);
              bits &= bits - 1u;
              tput(d + 1, at++, (uint32_t)(w * 32 + b));
            }
            if (w < nw) marks[w] = 0u;
            ntc += __shfl(incl, g * GL + GL - 1);
          }
          __builtin_amdgcn_wave_barrier();
          __threadfence_block();
          regs = GL == WAVE && ntc <= GL;
          // (3) each reached state gathers over its incoming contributions, for
          //     the children of its a allele and of its b allele in one pass
          //     (contributions two at a time: both words, then both weight sets,
          //     then the terms in record order)
          for (int j = gl; j < ntc; j += GL) {
            const uint32_t t = tget(d + 1, j);
            const uint32_t hd = R.hdr[t];
            const uint32_t xa = hd & 0xFFu, xb = (hd >> 8) & 0xFFu;
            const bool ca = (cm >> xa) & 1ull, cb = xb != xa && ((cm >> xb) & 1ull);
            double a0 = 0.0, a1 = 0.0, a2 = 0.0, b0 = 0.0, b1 = 0.0, b2 = 0.0;
            const double tp = R.tpv[t];
            const uint32_t r0 = R.cb[t], r1 = R.cb[t + 1];
            if (regs) rbw = bw[t];
            for (uint32_t r = r0; r < r1; r += 2) {
              const bool two = r + 1 < r1;
              const uint32_t wA = R.ct[r], wB = two ? R.ct[r + 1] : 0u;
              const uint32_t sA = cw_state(wA), sB = cw_state(wB);
              const double u0 = P0[3 * sA], u1 = P1[3 * sA], u2 = P2[3 * sA];
              double v0 = 0.0, v1 = 0.0, v2 = 0.0;
              if (two) {
                v0 = P0[3 * sB];
                v1 = P1[3 * sB];
                v2 = P2[3 * sB];
              }
              if (ca) walk_terms(true, xb == xa, cw_rev(wA), u0, u1, u2, tp, a0, a1, a2);
              if (cb) walk_terms(false, true, cw_rev(wA), u0, u1, u2, tp, b0, b1, b2);
              if (two) {
                if (ca) walk_terms(true, xb == xa, cw_rev(wB), v0, v1, v2, tp, a0, a1, a2);
                if (cb) walk_terms(false, true, cw_rev(wB), v0, v1, v2, tp, b0, b1, b2);
              }
            }
            if (ca) {
              double *C0 = slot(d + 1, (int)xa);
              C0[3 * t] = a0;
              C0[3 * t + 1] = a1;
              C0[3 * t + 2] = a2;
            }
            if (cb) {
              double *C0 = slot(d + 1, (int)xb);
              C0[3 * t] = b0;
              C0[3 * t + 1] = b1;
              C0[3 * t + 2] = b2;
            }
            rxa = xa;
            rxb = xb;
            rca = ca;
            rcb = cb;
            ra0 = a0;
            ra1 = a1;
            ra2 = a2;
            rb0 = b0;
            rb1 = b1;
            rb2 = b2;
          }
        }
        __builtin_amdgcn_wave_barrier();
        __threadfence_block();
        // (4) every child's frequency: hp->setFrequency(+freq), setPrefixFreq(+last_freq) (:437-441)
        unsigned long long desc = 0ull;
        for (unsigned long long m = cm; m; m &= m - 1) {
          const int i = __builtin_ctzll(m);
          double part[NG];  // virtual lane gl + GL k of a 64-lane sum (group_sum_fixed)
#pragma unroll
          for (int k = 0; k < NG; ++k) part[k] = 0.0;
          bool any = false;
          if (regs) {  // this lane's state (if any) from (3): the same terms the scratch holds
            if (gl < ntc) {
              const bool isa = rca && rxa == (uint32_t)i, isb = rcb && rxb == (uint32_t)i;
              const double n0 = isa ? ra0 : (isb ? rb0 : 0.0), n1 = isa ? ra1 : (isb ? rb1 : 0.0),
                           n2 = isa ? ra2 : (isb ? rb2 : 0.0);
              part[0] += ((n0 + n1) + n2) * rbw;
              any = (n0 != 0.0) | (n1 != 0.0) | (n2 != 0.0);
            }
          } else {
            const double *C0 = slot(d + 1, i);
            for (int j = gl; j < ntc; j += GL) {
              const uint32_t t = tget(d + 1, j);
              const double n0 = C0[3 * t], n1 = C0[3 * t + 1], n2 = C0[3 * t + 2];
              const double v = ((n0 + n1) + n2) * bw[t];
              if constexpr (NG == 1) {
                part[0] += v;
              } else {
                const int k = (j / GL) & (NG - 1);
#pragma unroll
                for (int u = 0; u < NG; ++u)
                  if (u == k) part[u] += v;
              }
              any |= (n0 != 0.0) | (n1 != 0.0) | (n2 != 0.0);
            }
          }
          const double freq = group_sum_fixed<GL>(part) / pg;
          int pat;
          if constexpr (GL == WAVE) {
            pat = __shfl(patv, i);
          } else {
            const int child = a.tr_child[(size_t)node * W + i];
            pat = a.tr_data[child];
          }
          if (gl == 0) {
            cfreq[(size_t)(d + 1) * W + i] = freq;
            if (pat >= 0) {
              atomicAdd(&a.acc_freq[pat], (unsigned long long)__double2ll_rn(freq * EXACT_FIXED_SCALE));
              atomicAdd(&a.acc_prefix[pat], (unsigned long long)__double2ll_rn(last_freq * EXACT_FIXED_SCALE));
            }
          }
          const unsigned long long anym = gballot(any);
          if (anym != 0ull && d + 1 <= maxd) desc |= 1ull << i;
          if (gl == 0 && i < wc) nzm[(d + 1) * wc + i] = anym;  // (bit j = touched entry j when regs)
        }
        if (gl == 0) {
          if (wc > 0) dnzv[d + 1] = regs ? 1 : 0;
          tcnt[d + 1] = ntc;
          smask[d + 1] = cm;
          sdesc[d] = desc;
          snext[d] = 0;
        }
        __builtin_amdgcn_wave_barrier();
        __threadfence_block();
      }
      // ---- descend into the next child whose lists are not all zero ----
      const unsigned long long left = sdesc[d] & ~((1ull << snext[d]) - 1ull);
      if (left == 0ull) {  // node done
        --d;
        continue;
      }
      const int i = __builtin_ctzll(left);
      const int child = GL == WAVE && wc > 0 ? schild[d * wc + i] : a.tr_child[(size_t)node * W + i];
      __builtin_amdgcn_wave_barrier();
      if (gl == 0) {
        snext[d] = i + 1;
        snode[d + 1] = child;
        snext[d + 1] = -1;
        sslot[d + 1] = i;
      }
      ++d;
    }
    // the item's entries back to zero (scratch invariant)
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    for (int dd = 0; dd <= maxd; ++dd) {
      const int nc = tcnt[dd];
      const unsigned long long wm = smask[dd];
      for (int j = gl; j < nc; j += GL) {
        const uint32_t t = tget(dd, j);
        for (unsigned long long m = wm; m; m &= m - 1) {
          double *D0 = slot(dd, __builtin_ctzll(m));
          D0[3 * t] = 0.0;
          D0[3 * t + 1] = 0.0;
          D0[3 * t + 2] = 0.0;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    for (int dd = gl; dd < D; dd += GL) {
      tcnt[dd] = 0;
      smask[dd] = 0ull;
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
  }
}


#ifdef HMC_VARIANTS  // (the breadth-first walk: measured slower, the variants library only)
// ---- breadth-first walk ----------------------------------------------------
// The depth-first walk above spends a wavefront and a dozen dependent,
// barriered steps on every trie node, while a node's lists hold a handful of
// non-zero states (300 x 200 panel, restatement counts: 14.9 M live nodes, 5.0
// non-zero entries each).  Here a lane takes a whole node (a work unit,
// XWalkArgs): it scatters the node's entries along their forward links
// (HaploBuilder.cpp:369-427 scatters the same way) into private accumulators —
// per reached state the lists of its a-allele child and of its b-allele child —
// then adds every child's frequency (states ascending) and prefix term
// (:437-441) and emits the children with non-zero lists that have children of
// their own.  The host runs the levels depth by depth over batches of items;
// a wave reserves its outputs with one atomic pair, and units whose outputs do
// not fit are deferred and re-run once the deeper levels are done.
__device__ inline unsigned long long wave_excl_u64(unsigned long long v, unsigned long long &total) {
  const int lane = (int)(threadIdx.x & 63);
  unsigned long long incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  total = __shfl(incl, 63);
  return incl - v;
}

__global__ __launch_bounds__(256) void exact_walk_units(ExactArgs a, XWalkArgs x) {
  const int gtid = blockIdx.x * blockDim.x + threadIdx.x, nthr = gridDim.x * blockDim.x;
  const int lane = (int)(threadIdx.x & 63);
  const int L = a.L, hl = a.head_len, W = a.width, fmax = a.fmax;
  double *acc = x.lacc + (size_t)gtid * x.lacc_stride;  // [a side | b side][3][fmax]
  uint32_t *bits = x.lbits + (size_t)gtid * x.lbits_stride;
  const double *ew0 = x.e_w, *ew1 = x.e_w + x.e_cap, *ew2 = x.e_w + 2 * x.e_cap;
  double *ow0 = x.e_w, *ow1 = x.e_w + x.e_cap, *ow2 = x.e_w + 2 * x.e_cap;
  const int rounds = (x.n_in + nthr - 1) / nthr;  // wave-uniform: every lane joins its wave's reservation
  for (int it = 0; it < rounds; ++it) {
    const int j = it * nthr + gtid;
    bool live = j < x.n_in;
    unsigned long long u = 0;
    int q = 0, start = 0, node = -1, bi = 0;
    double pg = 0.0, pfreq = 1.0;
    if (live) {
      if (x.roots) {  // item j of the batch: its start locus's trie root, every state with its forward likelihood
        const long long item = (long long)x.in_base + (x.idx ? x.idx[j] : j);
        q = (int)(item / L);
        start = (int)(item % L);
        node = a.tr_root[start];
      } else {
        u = x.idx ? (unsigned long long)x.idx[j] : x.in_base + (unsigned long long)j;
        node = x.u.node[u];
        if (node >= 0) {
          q = x.u.q[u];
          start = x.u.start[u];
          pfreq = x.u.freq[u];
        }
      }
      live = node >= 0;
    }
    if (live) {
      bi = a.order[q];
      const int s0 = a.status[bi];
      pg = a.gprob[bi];  // P(genotype) of the last E-step (HaploModel.cpp:109, HaploBuilder.cpp:294)
      live = (s0 == EST_OK || s0 == EST_OK_PRUNED) && pg > 0.0;
    }
    unsigned long long cm = 0ull;  // alleles with a child
    if (live)
      for (int i = 0; i < W; ++i) cm |= (a.tr_child[(size_t)node * W + i] >= 0 ? 1ull : 0ull) << i;
    live = live && cm != 0ull;
    const int locus = start + x.depth;  // the children's allele is at this locus
    const bool head = locus < hl;       // head pairs: their patterns' alleles, same states (HaploBuilder.cpp:340-367)
    int FT = 0;
    const double *bw = nullptr;
    const uint32_t *thdr = nullptr, *plo = nullptr, *phi = nullptr;
    // the children's two alleles of state t (a side, b side)
    auto alleles = [&](uint32_t t, uint32_t &xa, uint32_t &xb) {
      if (!head || hl == 1) {
        xa = thdr[t] & 0xFFu;
        xb = (thdr[t] >> 8) & 0xFFu;
      } else {
        xa = a.head_al[(size_t)plo[t] * hl + locus];
        xb = a.head_al[(size_t)phi[t] * hl + locus];
      }
    };
    if (live) {
      const unsigned long long *roff = a.rec_off + (size_t)bi * (L + 1);
      const unsigned long long *xo = a.x_off + (size_t)bi * (L + 1);
      const int tix = head ? hl : locus + 1, pix = head ? hl : locus;  // the children's / the node's states
      const RecView R(a.rec + roff[tix], head);
      FT = R.F;
      thdr = R.hdr;
      if (head) {
        plo = R.cb + FT + 1;
        phi = plo + FT;
      }
      bw = (const double *)(a.x + xo[tix]) + FT;
      const int FP = (int)a.rec[roff[pix]];
      const double *fwp = (const double *)(a.x + xo[pix]);
      const unsigned long long e0 = x.roots ? 0ull : x.u.e0[u];
      const int ne = x.roots ? FP : (int)x.u.ne[u];
      for (int k = 0; k < ne; ++k) {
        const uint32_t s = x.roots ? (uint32_t)k : x.e_t[e0 + k];
        const double w0 = x.roots ? fwp[s] : ew0[e0 + k];
        const double w1 = x.roots ? 0.0 : ew1[e0 + k], w2 = x.roots ? 0.0 : ew2[e0 + k];
        if (w0 == 0.0 && w1 == 0.0 && w2 == 0.0) continue;
        if (head) {
          uint32_t xa, xb;
          alleles(s, xa, xb);
          const bool ca = (cm >> xa) & 1ull, cb = xb != xa && ((cm >> xb) & 1ull);
          if (!ca && !cb) continue;
          bits[s >> 5] |= 1u << (s & 31u);
          if (ca) {  // child xa: both sides when xb == xa, else the a side
            double *A = acc + s;
            if (xb == xa) {
              A[0] = w0;
              A[fmax] = w1;
              A[2 * fmax] = w2;
            } else {
              A[fmax] = w0 * 0.5 + w1;
            }
          }
          if (cb) acc[3 * (size_t)fmax + 2 * (size_t)fmax + s] = w0 * 0.5 + w2;  // child xb: the b side
          continue;
        }
        uint32_t off = 0;
        for (int p = 0; p < R.NP; ++p) {  // m_forward_links of the pair, in push order
          const uint32_t no = R.npo[p];
          for (uint32_t o = 0; o < no; ++o) {
            const uint32_t w = R.out[off + s * no + o];
            if (w == NONE) continue;
            const uint32_t t = cw_state(w);
            const bool rev = cw_rev(w);
            uint32_t xa, xb;
            alleles(t, xa, xb);
            const bool ca = (cm >> xa) & 1ull, cb = xb != xa && ((cm >> xb) & 1ull);
            if (!ca && !cb) continue;
            bits[t >> 5] |= 1u << (t & 31u);
            const double tp = R.tpv[t];
            if (ca) {
              double *A = acc + t;
              walk_terms(true, xb == xa, rev, w0, w1, w2, tp, A[0], A[fmax], A[2 * fmax]);
            }
            if (cb) {
              double *B = acc + 3 * (size_t)fmax + t;
              walk_terms(false, true, rev, w0, w1, w2, tp, B[0], B[fmax], B[2 * fmax]);
            }
          }
          off += (uint32_t)FP * no;
        }
      }
    }
    const int nwT = (FT + 31) >> 5;
    // child i's lists at state t: the a-side accumulators when t's a allele is i, else the b side's
    auto side = [&](uint32_t t, uint32_t i) -> const double * {
      uint32_t xa, xb;
      alleles(t, xa, xb);
      return xa == i ? acc + t : (xb == i ? acc + 3 * (size_t)fmax + t : nullptr);
    };
    auto has_children = [&](int c) {
      bool g = false;
      for (int i = 0; i < W; ++i) g = g || a.tr_child[(size_t)c * W + i] >= 0;
      return g;
    };
    // pass 1: the children this node emits and their entries
    unsigned long long nu = 0, nent = 0;
    if (live)
      for (unsigned long long m = cm; m; m &= m - 1) {
        const uint32_t i = (uint32_t)__builtin_ctzll(m);
        const int child = a.tr_child[(size_t)node * W + i];
        if (!has_children(child)) continue;
        unsigned long long cnt = 0;
        for (int w = 0; w < nwT; ++w)
          for (uint32_t b = bits[w]; b; b &= b - 1u) {
            const uint32_t t = (uint32_t)w * 32u + (uint32_t)__builtin_ctz(b);
            const double *n = side(t, i);
            if (n && (n[0] != 0.0 || n[fmax] != 0.0 || n[2 * fmax] != 0.0)) ++cnt;
          }
        if (cnt) {
          ++nu;
          nent += cnt;
        }
      }
    // one reservation per wave
    unsigned long long tu = 0, te = 0;
    const unsigned long long xu = wave_excl_u64(nu, tu), xe = wave_excl_u64(nent, te);
    unsigned long long bu = 0, be = 0;
    if (lane == 0 && (tu | te)) {
      bu = atomicAdd(x.cursor, tu);
      be = atomicAdd(x.cursor + 1, te);
    }
    bu = __shfl(bu, 0) + xu;
    be = __shfl(be, 0) + xe;
    const bool ok = live && bu + nu <= x.u_cap && be + nent <= x.e_cap;
    if (live && !ok) {  // re-run later: nothing of this node is added now
      const int d = atomicAdd(x.n_defer, 1);
      x.defer[d] = x.roots ? (x.idx ? x.idx[j] : (int32_t)j) : (int32_t)u;
      for (unsigned long long k = bu; k < bu + nu && k < x.u_cap; ++k) x.u.node[k] = -1;  // holes
    }
    // pass 2: frequencies (hp->setFrequency, setPrefixFreq, HaploBuilder.cpp:437-441) and the emitted children
    if (ok)
      for (unsigned long long m = cm; m; m &= m - 1) {
        const uint32_t i = (uint32_t)__builtin_ctzll(m);
        const int child = a.tr_child[(size_t)node * W + i];
        const bool gk = has_children(child);
        double f = 0.0;
        unsigned long long cnt = 0;
        for (int w = 0; w < nwT; ++w)
          for (uint32_t b = bits[w]; b; b &= b - 1u) {
            const uint32_t t = (uint32_t)w * 32u + (uint32_t)__builtin_ctz(b);
            const double *n = side(t, i);
            if (!n) continue;
            const double n0 = n[0], n1 = n[fmax], n2 = n[2 * fmax];
            if (n0 == 0.0 && n1 == 0.0 && n2 == 0.0) continue;
            f += ((n0 + n1) + n2) * bw[t];
            if (gk) {
              x.e_t[be + cnt] = t;
              ow0[be + cnt] = n0;
              ow1[be + cnt] = n1;
              ow2[be + cnt] = n2;
            }
            ++cnt;
          }
        const double freq = f / pg;
        const int pat = a.tr_data[child];
        if (pat >= 0) {
          atomicAdd(&a.acc_freq[pat], (unsigned long long)__double2ll_rn(freq * EXACT_FIXED_SCALE));
          atomicAdd(&a.acc_prefix[pat], (unsigned long long)__double2ll_rn(pfreq * EXACT_FIXED_SCALE));
        }
        if (gk && cnt) {
          x.u.q[bu] = q;
          x.u.start[bu] = start;
          x.u.node[bu] = child;
          x.u.freq[bu] = freq;
          x.u.e0[bu] = be;
          x.u.ne[bu] = (uint32_t)cnt;
          ++bu;
          be += cnt;
        }
      }
    // the accumulators and the bitmap back to zero
    if (live)
      for (int w = 0; w < nwT; ++w) {
        for (uint32_t b = bits[w]; b; b &= b - 1u) {
          const uint32_t t = (uint32_t)w * 32u + (uint32_t)__builtin_ctz(b);
          for (int c = 0; c < 6; ++c) acc[(size_t)c * fmax + t] = 0.0;
        }
        bits[w] = 0u;
      }
  }
}

hipError_t launch_exact_walk_units(const ExactArgs &a, const XWalkArgs &x, int grid, hipStream_t st) {
  if (x.n_in <= 0) return hipSuccess;
  if (a.width < 1 || a.width > 64 || grid < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(exact_walk_units, dim3(grid), dim3(256), 0, st, a, x);
  return hipGetLastError();
}
#else
hipError_t launch_exact_walk_units(const ExactArgs &, const XWalkArgs &, int, hipStream_t) { return hipErrorNotSupported; }
#endif

size_t exact_walk_scratch_doubles(int max_depth, long long span, int width) {
  return (size_t)3 * width * (size_t)span + (size_t)(max_depth + 2) * width + ((size_t)span + 1) / 2;
}


hipError_t launch_exact_fb(const ExactArgs &a, int grid, hipStream_t st) {
  if (a.n_order <= 0) return hipSuccess;
  hipLaunchKernelGGL(exact_fb, dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_exact_span(const ExactArgs &a, int grid, hipStream_t st) {
  if (a.n_order <= 0) return hipSuccess;
  if (!a.span_max) return hipErrorInvalidValue;
  hipLaunchKernelGGL(exact_span, dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_exact_walk(const ExactArgs &a, int grid, hipStream_t st, int items_per_wave) {
  if (a.n_order <= 0) return hipSuccess;
  if (a.width < 1 || a.width > 64 || (items_per_wave != 1 && items_per_wave != 4)) return hipErrorInvalidValue;
  const size_t lds = exact_walk_lds_bytes(a.max_depth, a.fmax, a.width) * (size_t)items_per_wave;
  if (lds > EXACT_WALK_LDS_MAX) return hipErrorInvalidValue;  // the host reports it (exact_walk_group)
#ifdef HMC_VARIANTS
  void (*k)(ExactArgs) = items_per_wave == 4 ? exact_walk<16> : exact_walk<WAVE>;
#else
  if (items_per_wave != 1) return hipErrorNotSupported;  // (four items per wave: the variants library only)
  void (*k)(ExactArgs) = exact_walk<WAVE>;
#endif
  if (lds > 65536) {  // wide frontiers: a larger reached-state bitmap, fewer waves per CU (set per launch: per device)
    hipError_t e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(WAVE), lds, st, a);
  return hipGetLastError();
}

}  // namespace hmc
