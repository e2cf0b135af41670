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

__device__ inline double wave_sum_fixed(double x) {  // fixed butterfly: same result on every run
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

struct RecView {  // one locus record of the structure pass
  int F, C, NCH, CF, NP;  // states, stored contributions, chains, contributions in extendAll order, allele pairs
  const double *tpv;
  const uint32_t *hdr, *cb, *ct, *out, *npo;
  __device__ RecView(const uint32_t *R, bool head) {
    F = (int)R[0];
    C = (int)R[1];
    NCH = (int)R[2];
    CF = (int)(R[3] >> 10);
    NP = (int)(R[3] & 1023u);
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
    if (a.status[bi] != EST_OK) continue;
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
        if (!(f > 0.0) && j < L) flag = 1;  // extend() would skip this pair (HaploBuilder.cpp:237)
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

// The ForwardPatternTree walk of HaploBuilder::estimateFrequency (:296-308,
// :334-450), one wavefront per (individual, start locus), sparse like the
// reference's maps: a node's three lists are held densely per state (zero
// where absent) but only the states listed in the depth's `touched` list are
// ever written, and a child's states are found by following the forward
// links (the extendAll contributions of the record) of its parent's non-zero
// states, as the reference pushes along forward_links (:369-427).  Each
// reached state then gathers over its incoming contributions in record order
// (the same terms; zero sources add +0.0), so the sums do not depend on the
// order the states were reached in.  Scratch invariant: every dense entry not
// in a touched list is 0.0 (the host zeroes the scratch before the launch and
// every item clears what it wrote).
__global__ __launch_bounds__(64) void exact_walk(ExactArgs a) {
  extern __shared__ int stk[];  // [maxd+1] node, [maxd+1] next child, [maxd+1] touched count, marks
  const int lane = threadIdx.x;
  const int L = a.L, hl = a.head_len, W = a.width, maxd = a.max_depth;
  int *snode = stk, *snext = stk + maxd + 1, *tcnt = stk + 2 * (maxd + 1);
  uint32_t *marks = (uint32_t *)(stk + 3 * (maxd + 1));  // [fmax/32 + 1] reached-state bitmap
  const int nwords = (a.fmax + 31) >> 5;
  double *lists = a.scratch + (size_t)blockIdx.x * a.scratch_stride;  // [maxd+1][3][fmax]
  double *nf = lists + (size_t)(maxd + 1) * 3 * a.fmax;                // [maxd+2]
  uint32_t *touched = (uint32_t *)(nf + maxd + 2);                      // [maxd+1][fmax]
  for (int d = lane; d <= maxd; d += WAVE) tcnt[d] = 0;
  for (int w = lane; w < nwords; w += WAVE) marks[w] = 0u;
  __builtin_amdgcn_wave_barrier();
  __threadfence_block();
  const long long n_items = a.item1 < 0 ? (long long)a.n_order * L : a.item1;
  for (long long it = a.item0 + blockIdx.x; it < n_items; it += gridDim.x) {
    const int q = (int)(it / L), start = (int)(it % L);
    const int bi = a.order[q];
    const int root = a.tr_root[start];
    if (root < 0 || a.status[bi] != EST_OK) continue;
    const double pg = a.gprob[bi];  // P(genotype) of the last E-step (HaploModel.cpp:109, HaploBuilder.cpp:294)
    if (!(pg > 0.0)) continue;
    const unsigned long long *roff = a.rec_off + (size_t)bi * (L + 1);
    const unsigned long long *xo = a.x_off + (size_t)bi * (L + 1);
    const uint32_t *Rh = a.rec + roff[hl];
    const int Fh = (int)Rh[0];
    // depth 0: every state after max(start, head_len) loci, weight = forward likelihood
    {
      const int e0 = start > hl ? start : hl;
      const int F0 = (int)a.rec[roff[e0]];
      const double *fw = (const double *)(a.x + xo[e0]);
      for (int t = lane; t < F0; t += WAVE) {
        lists[t] = fw[t];
        touched[t] = (uint32_t)t;
      }
      if (lane == 0) {
        tcnt[0] = F0;
        snode[0] = root;
        snext[0] = 0;
        nf[0] = 1.0;  // the root's children get prefix frequency 1.0 (HaploBuilder.cpp:305)
      }
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    int d = 0;
    while (d >= 0) {
      __builtin_amdgcn_wave_barrier();
      __threadfence_block();
      const int node = snode[d];
      int i = snext[d];
      int child = -1;
      while (i < W && child < 0) {
        child = a.tr_child[(size_t)node * W + i];
        if (child < 0) ++i;
      }
      if (child < 0 || d >= maxd) {  // node done
        --d;
        continue;
      }
      if (lane == 0) snext[d] = i + 1;
      const int locus = start + d;       // the child's allele is at this locus
      const double last_freq = nf[d];
      const double *P0 = lists + (size_t)d * 3 * a.fmax, *P1 = P0 + a.fmax, *P2 = P1 + a.fmax;
      double *C0 = lists + (size_t)(d + 1) * 3 * a.fmax, *C1 = C0 + a.fmax, *C2 = C1 + a.fmax;
      const uint32_t *Tp = touched + (size_t)d * a.fmax;
      uint32_t *Tc = touched + (size_t)(d + 1) * a.fmax;
      // the previous sibling's entries at depth d+1 back to zero
      {
        const int nc = tcnt[d + 1];
        for (int j = lane; j < nc; j += WAVE) {
          const uint32_t t = Tc[j];
          C0[t] = 0.0;
          C1[t] = 0.0;
          C2[t] = 0.0;
        }
      }
      double part = 0.0;
      bool any = false;
      int ntc = 0;
      if (locus < hl) {  // head pairs: their patterns' alleles (HaploBuilder.cpp:340-367), same states
        const RecView R(Rh, true);
        const uint32_t *plo = R.cb + Fh + 1, *phi = plo + Fh;
        const double *bw = (const double *)(a.x + xo[hl]) + Fh;
        for (int t = lane; t < Fh; t += WAVE) {
          uint32_t xa, xb;
          if (hl == 1) {
            xa = R.hdr[t] & 0xFFu;
            xb = (R.hdr[t] >> 8) & 0xFFu;
          } else {
            xa = a.head_al[(size_t)plo[t] * hl + locus];
            xb = a.head_al[(size_t)phi[t] * hl + locus];
          }
          const bool ma = xa == (uint32_t)i, mb = xb == (uint32_t)i;
          const double w0 = P0[t], w1 = P1[t], w2 = P2[t];
          double n0 = 0.0, n1 = 0.0, n2 = 0.0;
          if (ma) {
            if (mb) n0 = w0;
            else n1 = w0 * 0.5;
          } else if (mb) {
            n2 = w0 * 0.5;
          }
          if (ma) n1 += w1;
          if (mb) n2 += w2;
          C0[t] = n0;
          C1[t] = n1;
          C2[t] = n2;
          Tc[t] = (uint32_t)t;
          part += ((n0 + n1) + n2) * bw[t];
          any |= (n0 != 0.0) | (n1 != 0.0) | (n2 != 0.0);
        }
        ntc = Fh;
      } else {  // along the forward links into the states after `locus` (:369-427)
        const RecView R(a.rec + roff[locus + 1], false);
        const double *bw = (const double *)(a.x + xo[locus + 1]) + R.F;
        // (1) mark the states the parent's non-zero states link to and whose
        //     pair carries the child's allele on either side
        const int np = tcnt[d];
        const int Fp = (int)a.rec[roff[locus]];  // states the links leave from
        for (int j = lane; j < np; j += WAVE) {
          const uint32_t s = Tp[j];
          if (P0[s] == 0.0 && P1[s] == 0.0 && P2[s] == 0.0) continue;
          uint32_t off = 0;
          for (int p = 0; p < R.NP; ++p) {
            const uint32_t no = R.npo[p];
            for (uint32_t o = 0; o < no; ++o) {
              const uint32_t w = R.out[off + s * no + o];
              if (w != NONE) {
                const uint32_t t = cw_state(w);
                const uint32_t hd = R.hdr[t];
                if ((hd & 0xFFu) == (uint32_t)i || ((hd >> 8) & 0xFFu) == (uint32_t)i)
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
        for (int w0 = 0; w0 < nw; w0 += WAVE) {
          const int w = w0 + lane;
          uint32_t bits = w < nw ? marks[w] : 0u;
          const int c = __popc(bits);
          int incl = c;
#pragma unroll
          for (int dd = 1; dd < 64; dd <<= 1) {
            const int y = __shfl_up(incl, dd);
            if (lane >= dd) incl += y;
          }
          int at = ntc + incl - c;
          while (bits) {
            const int b = __builtin_ctz(bits);
            bits &= bits - 1u;
            Tc[at++] = (uint32_t)(w * 32 + b);
          }
          if (w < nw) marks[w] = 0u;
          ntc += __shfl(incl, 63);
        }
        __builtin_amdgcn_wave_barrier();
        __threadfence_block();
        // (3) each reached state gathers over its incoming contributions
        for (int j = lane; j < ntc; j += WAVE) {
          const uint32_t t = Tc[j];
          const uint32_t hd = R.hdr[t];
          const bool ma = (hd & 0xFFu) == (uint32_t)i, mb = ((hd >> 8) & 0xFFu) == (uint32_t)i;
          double n0 = 0.0, n1 = 0.0, n2 = 0.0;
          const double tp = R.tpv[t];
          for (uint32_t r = R.cb[t]; r < R.cb[t + 1]; ++r) {
            const uint32_t w = R.ct[r];
            const uint32_t s = cw_state(w);
            const bool rev = cw_rev(w);
            const double w0 = P0[s], w1 = P1[s], w2 = P2[s];
            if (ma && mb) n0 += w0 * tp;
            else if (ma) n1 += w0 * tp * 0.5;
            else n2 += w0 * tp * 0.5;
            // a-side list follows the a haplotype: links[0] keep it on a, links[1] move it to b
            if (!rev ? ma : mb) (!rev ? n1 : n2) += w1 * tp;
            if (!rev ? mb : ma) (!rev ? n2 : n1) += w2 * tp;
          }
          C0[t] = n0;
          C1[t] = n1;
          C2[t] = n2;
          part += ((n0 + n1) + n2) * bw[t];
          any |= (n0 != 0.0) | (n1 != 0.0) | (n2 != 0.0);
        }
      }
      if (lane == 0) tcnt[d + 1] = ntc;
      const double freq = wave_sum_fixed(part) / pg;
      const int pat = a.tr_data[child];
      if (lane == 0 && pat >= 0) {  // hp->setFrequency(+freq), setPrefixFreq(+last_freq) (:437-441)
        atomicAdd(&a.acc_freq[pat], (unsigned long long)__double2ll_rn(freq * EXACT_FIXED_SCALE));
        atomicAdd(&a.acc_prefix[pat], (unsigned long long)__double2ll_rn(last_freq * EXACT_FIXED_SCALE));
      }
      const bool descend = __ballot(any) != 0ull && d + 1 <= maxd;
      __builtin_amdgcn_wave_barrier();
      __threadfence_block();
      if (descend) {
        if (lane == 0) {
          snode[d + 1] = child;
          snext[d + 1] = 0;
          nf[d + 1] = freq;
        }
        ++d;
      }
    }
    // the item's entries back to zero (scratch invariant)
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    for (int dd = 0; dd <= maxd; ++dd) {
      const int nc = tcnt[dd];
      double *D0 = lists + (size_t)dd * 3 * a.fmax;
      const uint32_t *T = touched + (size_t)dd * a.fmax;
      for (int j = lane; j < nc; j += WAVE) {
        const uint32_t t = T[j];
        D0[t] = 0.0;
        D0[a.fmax + t] = 0.0;
        D0[2 * a.fmax + t] = 0.0;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    for (int dd = lane; dd <= maxd; dd += WAVE) tcnt[dd] = 0;
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
  }
}

size_t exact_walk_scratch_doubles(int max_depth, int fmax) {
  return (size_t)(max_depth + 1) * 3 * fmax + max_depth + 2 + ((size_t)(max_depth + 1) * fmax + 1) / 2;
}

hipError_t launch_exact_fb(const ExactArgs &a, int grid, hipStream_t st) {
  if (a.n_order <= 0) return hipSuccess;
  hipLaunchKernelGGL(exact_fb, dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_exact_walk(const ExactArgs &a, int grid, hipStream_t st) {
  if (a.n_order <= 0) return hipSuccess;
  const size_t lds = (size_t)3 * (a.max_depth + 1) * sizeof(int) + (size_t)((a.fmax + 31) / 32 + 1) * 4;
  if (lds > 65536) return hipErrorInvalidValue;
  hipLaunchKernelGGL(exact_walk, dim3(grid), dim3(WAVE), lds, st, a);
  return hipGetLastError();
}

}  // namespace hmc
