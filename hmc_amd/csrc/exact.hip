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
          const double v = fp[R.ct[r] & 0xFFFFu] * tpv;
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
              if (w != NONE && ((w >> 16) & 1u) == (uint32_t)pass) {
                const uint32_t t = w & 0xFFFFu;
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
// :334-450), one wavefront per (individual, start locus).
__global__ __launch_bounds__(64) void exact_walk(ExactArgs a) {
  extern __shared__ int stk[];  // [maxd+1] node, [maxd+1] next child
  const int lane = threadIdx.x;
  const int L = a.L, hl = a.head_len, W = a.width, maxd = a.max_depth;
  int *snode = stk, *snext = stk + maxd + 1;
  double *lists = a.scratch + (size_t)blockIdx.x * a.scratch_stride;  // [maxd+1][3][fmax]
  const long long n_items = (long long)a.n_order * L;
  for (long long it = blockIdx.x; it < n_items; it += gridDim.x) {
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
        lists[a.fmax + t] = 0.0;
        lists[2 * a.fmax + t] = 0.0;
      }
    }
    // per-depth node frequencies: a child's prefix frequency is its parent's
    // (the root's children get 1.0, HaploBuilder.cpp:305)
    double *nf = lists + (size_t)(maxd + 1) * 3 * a.fmax;
    if (lane == 0) {
      snode[0] = root;
      snext[0] = 0;
      nf[0] = 1.0;
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
      double part = 0.0;
      bool any = false;
      if (locus < hl) {  // head pairs: their patterns' alleles (HaploBuilder.cpp:340-367)
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
          part += ((n0 + n1) + n2) * bw[t];
          any |= (n0 != 0.0) | (n1 != 0.0) | (n2 != 0.0);
        }
      } else {  // along the forward links into the states after `locus` (:369-427)
        const RecView R(a.rec + roff[locus + 1], false);
        const double *bw = (const double *)(a.x + xo[locus + 1]) + R.F;
        for (int t = lane; t < R.F; t += WAVE) {
          const uint32_t hd = R.hdr[t];
          const bool ma = (hd & 0xFFu) == (uint32_t)i, mb = ((hd >> 8) & 0xFFu) == (uint32_t)i;
          double n0 = 0.0, n1 = 0.0, n2 = 0.0;
          if (ma || mb) {
            const double tp = R.tpv[t];
            for (uint32_t r = R.cb[t]; r < R.cb[t + 1]; ++r) {
              const uint32_t w = R.ct[r];
              const uint32_t s = w & 0xFFFFu;
              const bool rev = (w >> 16) & 1u;
              const double w0 = P0[s], w1 = P1[s], w2 = P2[s];
              if (ma && mb) n0 += w0 * tp;
              else if (ma) n1 += w0 * tp * 0.5;
              else n2 += w0 * tp * 0.5;
              // a-side list follows the a haplotype: links[0] keep it on a, links[1] move it to b
              if (!rev ? ma : mb) (!rev ? n1 : n2) += w1 * tp;
              if (!rev ? mb : ma) (!rev ? n2 : n1) += w2 * tp;
            }
          }
          C0[t] = n0;
          C1[t] = n1;
          C2[t] = n2;
          part += ((n0 + n1) + n2) * bw[t];
          any |= (n0 != 0.0) | (n1 != 0.0) | (n2 != 0.0);
        }
      }
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
  }
}

hipError_t launch_exact_fb(const ExactArgs &a, int grid, hipStream_t st) {
  if (a.n_order <= 0) return hipSuccess;
  hipLaunchKernelGGL(exact_fb, dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_exact_walk(const ExactArgs &a, int grid, hipStream_t st) {
  if (a.n_order <= 0) return hipSuccess;
  const size_t lds = (size_t)2 * (a.max_depth + 1) * sizeof(int);
  hipLaunchKernelGGL(exact_walk, dim3(grid), dim3(WAVE), lds, st, a);
  return hipGetLastError();
}

}  // namespace hmc
