// coop_bench.hip — microbenchmark of k-best list selections (never the
// product): chains of adds like phase B of estep_values — S new likelihoods
// (few distinct values, so ties occur) behind a list's S kept ones, then
// std::nth_element(.., S-1, ..).  Every mode processes the same lists (list
// g's values depend only on g, the add and the position) and prints a
// checksum of the kept lists, which must agree between modes.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I hmc_amd/csrc tools/diag/coop_bench.hip -o coop_bench
//   ./coop_bench [waves_per_cu] [adds] [mode] [S]
//   mode 0: 2S-lane segments, 64/2S lists per wave (seg_nth_slots, LDS slots)
//   (mode 1, one list per wave in registers with wave-uniform scalar control,
//   was measured at 6 200 cycles per add alone and 1.0 ns per add at 24 waves
//   per CU — slower than mode 0 — and removed; profiles/r03/coop/)
//   mode 2: one list per lane, sequential libstdc++ code on an LDS column
//   mode 3: one list per lane, mask partition (nth_element_greater_masks)
//   mode 4: as mode 0 with two sets of segments per wave, interleaved
//   mode 5: two elements per lane, S lanes per list (seg2_nth_slots)
//   mode 6: four elements per lane, ceil(S / 2) lanes per list (segE_nth_slots<4>)
//   mode 7: as mode 5 with lane-major slots (seg2m_nth_slots)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "coop_select.hpp"

using namespace hmc;

__device__ inline uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ inline double val(uint32_t g, int r, int k) { return (double)(mix(g * 1000003u + (uint32_t)r * 64u + (uint32_t)k) % 64u); }

// ---- selection layouts measured here only (not in the product) ----------

// seg_nth_slots on K independent sets of segments at once (set u: lists in
// the slots of ss[u], n[u] / nth[u] per lane as above; SW <= 32).  The
// partitions of the K sets are interleaved phase by phase — K sets of reads,
// median, stop masks and pairing writes, one LDS sync, K sets of partner reads
// and moves, one sync — so the dependent instruction chains of one set fill
// the latencies of the others.  Every set ends with the same permutation as
// seg_nth_slots.
template <int K>
__device__ inline void seg_nth_slots_multi(const int (&n)[K], const int (&nth)[K], const Seg &sg,
                                           const SegScratch (&ss)[K]) {
  const int lane = (int)(threadIdx.x & 63);
  const int k = sg.k;
  const int kmax = sg.sw - 1;
  int first[K], last[K], depth[K];
  bool act[K];
  double *sl[K];
  uint32_t *sm[K];
  int *lp[K], *rp[K], *jl[K], *jr[K];
#pragma unroll
  for (int u = 0; u < K; ++u) {
    first[u] = 0;
    last[u] = n[u];
    depth[u] = n[u] > 0 ? lg2_floor(n[u]) * 2 : 0;
    act[u] = n[u] > 0 && nth[u] != n[u] && sg.mask != 0ull;
    sl[u] = ss[u].slik + sg.base;
    sm[u] = ss[u].smeta + sg.base;
    lp[u] = ss[u].lpos + sg.base;
    rp[u] = ss[u].rpos + sg.base;
    jl[u] = ss[u].junk + lane;
    jr[u] = ss[u].junk + 64 + lane;
  }
  while (true) {
    bool part[K];
    uint64_t any = 0;
#pragma unroll
    for (int u = 0; u < K; ++u) {
      part[u] = act[u] && last[u] - first[u] > 3 && depth[u] > 0;
      any |= wave_ballot(part[u]);
    }
    if (!any) break;
    double v[K];
    uint32_t m[K];
    int r[K], x[K], kL[K], kR[K], nL[K], nR[K];
    bool isL[K], isR[K];
#pragma unroll
    for (int u = 0; u < K; ++u) {
      depth[u] -= part[u] ? 1 : 0;
      const int f = first[u], l = last[u];
      const int a = f + 1, b = f + ((l - f) >> 1), c = l > 0 ? l - 1 : 0;
      const double va = sl[u][a], vb = sl[u][b], vc = sl[u][c], vf = sl[u][f];
      v[u] = sl[u][k];
      m[u] = sm[u][k];
      const int idx = (va > vb ? 4 : 0) | (vb > vc ? 2 : 0) | (va > vc ? 1 : 0);
      const int w = (22561 >> (2 * idx)) & 3;
      r[u] = w == 0 ? a : (w == 1 ? b : c);
      const double pivot = w == 0 ? va : (w == 1 ? vb : vc);
      const double pv = k == f ? pivot : (k == r[u] ? vf : v[u]);
      const uint64_t b_part = wave_ballot(part[u]), b_in = wave_ballot(k > f) & wave_ballot(k < l);
      const uint64_t b_first = wave_ballot(k == f);
      const uint64_t b_le = wave_ballot(!(pv > pivot)), b_ge = wave_ballot(!(pivot > pv));
      const uint32_t Lw = seg_bits(b_part & b_in & b_le, sg);
      const uint32_t Rw = seg_bits(b_part & (b_in | b_first) & b_ge, sg);
      nL[u] = __popc(Lw);
      nR[u] = __popc(Rw);
      x[u] = !part[u] ? k : (k == f ? r[u] : (k == r[u] ? f : k));
      const uint32_t xb = (1u << x[u]) - 1u;
      isL[u] = part[u] && ((Lw >> x[u]) & 1u);
      isR[u] = part[u] && ((Rw >> x[u]) & 1u);
      kL[u] = __popc(Lw & xb);
      kR[u] = nR[u] - 1 - __popc(Rw & xb);
      *(isL[u] ? lp[u] + kL[u] : jl[u]) = x[u];
      *(isR[u] ? rp[u] + kR[u] : jr[u]) = x[u];
    }
    wave_lds_sync();
    int cut[K];
#pragma unroll
    for (int u = 0; u < K; ++u) {
      const int qR = rp[u][kL[u] < kmax ? kL[u] : kmax];
      const int qL = lp[u][kR[u] < 0 ? 0 : (kR[u] < kmax ? kR[u] : kmax)];
      const bool lsw = isL[u] && kL[u] < nR[u] && x[u] < qR;
      const bool rsw = isR[u] && kR[u] < nL[u] && qL < x[u];
      const int dest = lsw ? qR : (rsw ? qL : x[u]);
      sl[u][dest] = v[u];
      sm[u][dest] = m[u];
      const uint32_t bl = seg_bits(wave_ballot(isL[u] && !lsw), sg), br = seg_bits(wave_ballot(rsw), sg);
      const uint32_t keep = ~((1u << first[u]) | (1u << r[u]));
      const uint32_t ml = (bl & keep) | (((bl >> first[u]) & 1u) << r[u]);
      const uint32_t mr = (br & keep) | (((br >> first[u]) & 1u) << r[u]);
      const int lK = seg_lowest(ml), rK = seg_lowest(mr);
      cut[u] = lK < rK ? lK : rK;
    }
    wave_lds_sync();
#pragma unroll
    for (int u = 0; u < K; ++u) {
      const bool p = part[u];
      const int c = cut[u];
      first[u] = p && c <= nth[u] ? c : first[u];
      last[u] = p && c > nth[u] ? c : last[u];
    }
  }
#pragma unroll
  for (int u = 0; u < K; ++u) {
    // depth limit (std::__heap_select + iter_swap) and the final insertion
    // sort, as in seg_nth_slots
    const bool heap = act[u] && last[u] - first[u] > 3;
    if (wave_ballot(heap)) {
      if (heap && k == 0) {
        const LinkList wl{sl[u], sm[u], 1};
        heap_select(wl, first[u], nth[u] + 1, last[u]);
        wl.swap(first[u], nth[u]);
      }
      wave_lds_sync();
    }
    const bool ins = act[u] && !heap && last[u] - first[u] > 1;
    if (wave_ballot(ins)) {
      const int f = first[u], len = last[u] - f;
      const int f0 = f < kmax ? f : kmax;
      const int f1 = f + 1 < kmax ? f + 1 : kmax, f2 = f + 2 < kmax ? f + 2 : kmax;
      double x0 = sl[u][f0], x1 = sl[u][f1], x2 = sl[u][f2];
      uint32_t y0 = sm[u][f0], y1 = sm[u][f1], y2 = sm[u][f2];
      if (x1 > x0) {
        const double t = x1; x1 = x0; x0 = t;
        const uint32_t q = y1; y1 = y0; y0 = q;
      }
      if (len > 2) {
        if (x2 > x0) {
          const double t = x2; const uint32_t q = y2;
          x2 = x1; y2 = y1; x1 = x0; y1 = y0; x0 = t; y0 = q;
        } else if (x2 > x1) {
          const double t = x2; const uint32_t q = y2;
          x2 = x1; y2 = y1; x1 = t; y1 = q;
        }
      }
      const int j = k - f;
      const bool mine = ins && (j == 0 || j == 1 || (j == 2 && len > 2));
      const double xv = j == 0 ? x0 : (j == 1 ? x1 : x2);
      const uint32_t yv = j == 0 ? y0 : (j == 1 ? y1 : y2);
      wave_lds_sync();
      if (mine) {
        ss[u].slik[lane] = xv;
        ss[u].smeta[lane] = yv;
      }
      wave_lds_sync();
    }
  }
}

__device__ inline double fold(double acc) {
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  return acc;
}

// E links per lane (E = 2 is seg2_nth_slots): segment of W = ceil(2S / E)
// lanes, lane k carries positions k + j W (j < E); sg = make_seg(W); slots
// (64 / W + 1) x E W per wave.  Measured here only.
template <int E>
__device__ inline void segE_nth_slots(int n, int nth, const Seg &sg, const SegScratch &ss) {
  const int lane = (int)(threadIdx.x & 63);
  const int W = sg.sw, k = sg.k;
  int first = 0, last = n, depth = n > 0 ? lg2_floor(n) * 2 : 0;
  const bool act = n > 0 && nth != n && sg.mask != 0ull;
  const int sb = sg.g * E * W;
  double *sl = ss.slik + sb;
  uint32_t *sm = ss.smeta + sb;
  int *lp = ss.lpos + sb, *rp = ss.rpos + sb;
  const int kmax = E * W - 1;
  while (true) {
    const bool part = act && last - first > 3 && depth > 0;
    if (!wave_ballot(part)) break;
    depth -= part ? 1 : 0;
    const int a = first + 1, b = first + ((last - first) >> 1), c = last > 0 ? last - 1 : 0;
    const double va = sl[a], vb = sl[b], vc = sl[c], vf = sl[first];
    const int idx = (va > vb ? 4 : 0) | (vb > vc ? 2 : 0) | (va > vc ? 1 : 0);
    const int w = (22561 >> (2 * idx)) & 3;
    const int r = w == 0 ? a : (w == 1 ? b : c);
    const double pivot = w == 0 ? va : (w == 1 ? vb : vc);
    double v[E];
    uint32_t m[E];
    int x[E], kL[E], kR[E];
    bool isL[E], isR[E];
    uint32_t le = 0, ge = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int p = k + j * W;
      v[j] = sl[p];
      m[j] = sm[p];
      const double pv = p == first ? pivot : (p == r ? vf : v[j]);
      le |= seg_bits(wave_ballot(!(pv > pivot)), sg) << (j * W);
      ge |= seg_bits(wave_ballot(!(pivot > pv)), sg) << (j * W);
      x[j] = !part ? p : (p == first ? r : (p == r ? first : p));
    }
    const uint32_t below_last = last >= 32 ? ~0u : ((1u << last) - 1u);
    const uint32_t inR = part ? below_last & ~((1u << first) - 1u) : 0u;
    const uint32_t inL = inR & ~(1u << first);
    const uint32_t Lw = le & inL, Rw = ge & inR;
    const int nL = __popc(Lw), nR = __popc(Rw);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      isL[j] = part && ((Lw >> x[j]) & 1u);
      isR[j] = part && ((Rw >> x[j]) & 1u);
      const uint32_t xb = (1u << x[j]) - 1u;
      kL[j] = __popc(Lw & xb);
      kR[j] = nR - 1 - __popc(Rw & xb);
      *(isL[j] ? lp + kL[j] : ss.junk + j * 64 + lane) = x[j];
      *(isR[j] ? rp + kR[j] : ss.junk + (E + j) * 64 + lane) = x[j];
    }
    wave_lds_sync();
    uint32_t bl = 0, br = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int qR = rp[kL[j] < kmax ? kL[j] : kmax];
      const int qL = lp[kR[j] < 0 ? 0 : (kR[j] < kmax ? kR[j] : kmax)];
      const bool lsw = isL[j] && kL[j] < nR && x[j] < qR;
      const bool rsw = isR[j] && kR[j] < nL && qL < x[j];
      const int d = lsw ? qR : (rsw ? qL : x[j]);
      sl[d] = v[j];
      sm[d] = m[j];
      bl |= seg_bits(wave_ballot(isL[j] && !lsw), sg) << (j * W);
      br |= seg_bits(wave_ballot(rsw), sg) << (j * W);
    }
    const uint32_t keep = ~((1u << first) | (1u << r));
    const uint32_t ml = (bl & keep) | (((bl >> first) & 1u) << r);
    const uint32_t mr = (br & keep) | (((br >> first) & 1u) << r);
    const int lK = seg_lowest(ml), rK = seg_lowest(mr);
    const int cut = lK < rK ? lK : rK;
    wave_lds_sync();
    first = part && cut <= nth ? cut : first;
    last = part && cut > nth ? cut : last;
  }
  const bool heap = act && last - first > 3;
  if (wave_ballot(heap)) {
    if (heap && k == 0) {
      const LinkList wl{sl, sm, 1};
      heap_select(wl, first, nth + 1, last);
      wl.swap(first, nth);
    }
    wave_lds_sync();
  }
  const bool ins = act && !heap && last - first > 1;
  if (wave_ballot(ins)) {
    const int len = last - first;
    const int f0 = first < kmax ? first : kmax;
    const int f1 = first + 1 < kmax ? first + 1 : kmax, f2 = first + 2 < kmax ? first + 2 : kmax;
    double y0 = sl[f0], y1 = sl[f1], y2 = sl[f2];
    uint32_t t0 = sm[f0], t1 = sm[f1], t2 = sm[f2];
    if (y1 > y0) {
      const double t = y1; y1 = y0; y0 = t;
      const uint32_t u = t1; t1 = t0; t0 = u;
    }
    if (len > 2) {
      if (y2 > y0) {
        const double t = y2; const uint32_t u = t2;
        y2 = y1; t2 = t1; y1 = y0; t1 = t0; y0 = t; t0 = u;
      } else if (y2 > y1) {
        const double t = y2; const uint32_t u = t2;
        y2 = y1; t2 = t1; y1 = t; t1 = u;
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int p = k + j * W, q = p - first;
      if (ins && (q == 0 || q == 1 || (q == 2 && len > 2))) {
        sl[p] = q == 0 ? y0 : (q == 1 ? y1 : y2);
        sm[p] = q == 0 ? t0 : (q == 1 ? t1 : t2);
      }
    }
    wave_lds_sync();
  }
}

// Two links per lane with lane-major slots: position p of segment g lives
// in slot g W + p (p < W) or 64 + g W + p - W (p >= W), so the lanes' own
// reads and writes of both links are consecutive (bank-conflict free).
struct PairSlots {
  double *l;      // [128]
  uint32_t *m;    // [128]
  int gw, W;
  __device__ int at(int p) const { return gw + p + (p >= W ? 64 - W : 0); }
  __device__ double lv(int p) const { return l[at(p)]; }
  // LinkList-like view for the sequential heap select
  __device__ double l_(int p) const { return l[at(p)]; }
};
struct PairView {
  double *lk;
  uint32_t *mt;
  int gw, W;
  __device__ int at(int p) const { return gw + p + (p >= W ? 64 - W : 0); }
  __device__ double l(int k) const { return lk[at(k)]; }
  __device__ uint32_t m(int k) const { return mt[at(k)]; }
  __device__ void set(int k, double x, uint32_t y) const {
    lk[at(k)] = x;
    mt[at(k)] = y;
  }
  __device__ void copy(int dst, int src) const { set(dst, l(src), m(src)); }
  __device__ void swap(int a, int b) const {
    const double x = l(a);
    const uint32_t y = m(a);
    copy(a, b);
    set(b, x, y);
  }
  __device__ bool gt(int a, int b) const { return l(a) > l(b); }
};

__device__ inline void seg2m_nth_slots(int n, int nth, const Seg &sg, double *slik, uint32_t *smeta, int *lpos,
                                       int *rpos, int *junk) {
  const int lane = (int)(threadIdx.x & 63);
  const int W = sg.sw, k = sg.k;
  int first = 0, last = n, depth = n > 0 ? lg2_floor(n) * 2 : 0;
  const bool act = n > 0 && nth != n && sg.mask != 0ull;
  const PairView V{slik, smeta, sg.g * W, W};
  const int sb = sg.g * 2 * W;
  int *lp = lpos + sb, *rp = rpos + sb;
  int *jl0 = junk + lane, *jl1 = junk + 64 + lane, *jr0 = junk + 128 + lane, *jr1 = junk + 192 + lane;
  const int kmax = 2 * W - 1;
  const int p0 = k, p1 = k + W;
  double *s0 = slik + lane, *s1 = slik + 64 + lane;  // this lane's own slots
  uint32_t *t0s = smeta + lane, *t1s = smeta + 64 + lane;
  while (true) {
    const bool part = act && last - first > 3 && depth > 0;
    if (!wave_ballot(part)) break;
    depth -= part ? 1 : 0;
    const int a = first + 1, b = first + ((last - first) >> 1), c = last > 0 ? last - 1 : 0;
    const double va = V.l(a), vb = V.l(b), vc = V.l(c), vf = V.l(first);
    const double v0 = *s0, v1 = *s1;
    const uint32_t m0 = *t0s, m1 = *t1s;
    const int idx = (va > vb ? 4 : 0) | (vb > vc ? 2 : 0) | (va > vc ? 1 : 0);
    const int w = (22561 >> (2 * idx)) & 3;
    const int r = w == 0 ? a : (w == 1 ? b : c);
    const double pivot = w == 0 ? va : (w == 1 ? vb : vc);
    const double pv0 = p0 == first ? pivot : (p0 == r ? vf : v0);
    const double pv1 = p1 == first ? pivot : (p1 == r ? vf : v1);
    const uint32_t le = seg_bits(wave_ballot(!(pv0 > pivot)), sg) | seg_bits(wave_ballot(!(pv1 > pivot)), sg) << W;
    const uint32_t ge = seg_bits(wave_ballot(!(pivot > pv0)), sg) | seg_bits(wave_ballot(!(pivot > pv1)), sg) << W;
    const uint32_t below_last = last >= 32 ? ~0u : ((1u << last) - 1u);
    const uint32_t inR = part ? below_last & ~((1u << first) - 1u) : 0u;
    const uint32_t inL = inR & ~(1u << first);
    const uint32_t Lw = le & inL, Rw = ge & inR;
    const int nL = __popc(Lw), nR = __popc(Rw);
    const int x0 = !part ? p0 : (p0 == first ? r : (p0 == r ? first : p0));
    const int x1 = !part ? p1 : (p1 == first ? r : (p1 == r ? first : p1));
    const bool isL0 = part && ((Lw >> x0) & 1u), isR0 = part && ((Rw >> x0) & 1u);
    const bool isL1 = part && ((Lw >> x1) & 1u), isR1 = part && ((Rw >> x1) & 1u);
    const uint32_t xb0 = (1u << x0) - 1u, xb1 = (1u << x1) - 1u;
    const int kL0 = __popc(Lw & xb0), kL1 = __popc(Lw & xb1);
    const int kR0 = nR - 1 - __popc(Rw & xb0), kR1 = nR - 1 - __popc(Rw & xb1);
    *(isL0 ? lp + kL0 : jl0) = x0;
    *(isL1 ? lp + kL1 : jl1) = x1;
    *(isR0 ? rp + kR0 : jr0) = x0;
    *(isR1 ? rp + kR1 : jr1) = x1;
    wave_lds_sync();
    const int qR0 = rp[kL0 < kmax ? kL0 : kmax], qR1 = rp[kL1 < kmax ? kL1 : kmax];
    const int qL0 = lp[kR0 < 0 ? 0 : (kR0 < kmax ? kR0 : kmax)];
    const int qL1 = lp[kR1 < 0 ? 0 : (kR1 < kmax ? kR1 : kmax)];
    const bool lsw0 = isL0 && kL0 < nR && x0 < qR0, lsw1 = isL1 && kL1 < nR && x1 < qR1;
    const bool rsw0 = isR0 && kR0 < nL && qL0 < x0, rsw1 = isR1 && kR1 < nL && qL1 < x1;
    const int d0 = lsw0 ? qR0 : (rsw0 ? qL0 : x0), d1 = lsw1 ? qR1 : (rsw1 ? qL1 : x1);
    V.set(d0, v0, m0);
    V.set(d1, v1, m1);
    const uint32_t bl = seg_bits(wave_ballot(isL0 && !lsw0), sg) | seg_bits(wave_ballot(isL1 && !lsw1), sg) << W;
    const uint32_t br = seg_bits(wave_ballot(rsw0), sg) | seg_bits(wave_ballot(rsw1), sg) << W;
    const uint32_t keep = ~((1u << first) | (1u << r));
    const uint32_t ml = (bl & keep) | (((bl >> first) & 1u) << r);
    const uint32_t mr = (br & keep) | (((br >> first) & 1u) << r);
    const int lK = seg_lowest(ml), rK = seg_lowest(mr);
    const int cut = lK < rK ? lK : rK;
    wave_lds_sync();
    first = part && cut <= nth ? cut : first;
    last = part && cut > nth ? cut : last;
  }
  const bool heap = act && last - first > 3;
  if (wave_ballot(heap)) {
    if (heap && k == 0) {
      heap_select(V, first, nth + 1, last);
      V.swap(first, nth);
    }
    wave_lds_sync();
  }
  const bool ins = act && !heap && last - first > 1;
  if (wave_ballot(ins)) {
    const int len = last - first;
    const int f0 = first < kmax ? first : kmax;
    const int f1 = first + 1 < kmax ? first + 1 : kmax, f2 = first + 2 < kmax ? first + 2 : kmax;
    double y0 = V.l(f0), y1 = V.l(f1), y2 = V.l(f2);
    uint32_t t0 = V.m(f0), t1 = V.m(f1), t2 = V.m(f2);
    if (y1 > y0) {
      const double t = y1; y1 = y0; y0 = t;
      const uint32_t u = t1; t1 = t0; t0 = u;
    }
    if (len > 2) {
      if (y2 > y0) {
        const double t = y2; const uint32_t u = t2;
        y2 = y1; t2 = t1; y1 = y0; t1 = t0; y0 = t; t0 = u;
      } else if (y2 > y1) {
        const double t = y2; const uint32_t u = t2;
        y2 = y1; t2 = t1; y1 = t; t1 = u;
      }
    }
    const int j0 = p0 - first, j1 = p1 - first;
    const bool mine0 = ins && (j0 == 0 || j0 == 1 || (j0 == 2 && len > 2));
    const bool mine1 = ins && (j1 == 0 || j1 == 1 || (j1 == 2 && len > 2));
    const double z0 = j0 == 0 ? y0 : (j0 == 1 ? y1 : y2), z1 = j1 == 0 ? y0 : (j1 == 1 ? y1 : y2);
    const uint32_t u0 = j0 == 0 ? t0 : (j0 == 1 ? t1 : t2), u1 = j1 == 0 ? t0 : (j1 == 1 ? t1 : t2);
    wave_lds_sync();
    if (mine0) {
      *s0 = z0;
      *t0s = u0;
    }
    if (mine1) {
      *s1 = z1;
      *t1s = u1;
    }
    wave_lds_sync();
  }
}

// mode 7: two links per lane, lane-major slots (seg2m_nth_slots)
__global__ __launch_bounds__(64) void bench_seg2m(int S, int adds, double *out) {
  extern __shared__ unsigned char sm[];
  const int lane = threadIdx.x;
  int *lpos = (int *)sm, *rpos = (int *)(sm + 640), *junk = (int *)(sm + 1280);
  double *slik = (double *)(sm + 2304);          // 128 doubles
  uint32_t *smeta = (uint32_t *)(sm + 2304 + 1024);  // 128
  const Seg sg = make_seg(S);
  const int G = 64 / S;
  const bool in = sg.g < G;
  const uint32_t g = blockIdx.x * G + sg.g;
  if (in) {
    slik[lane] = val(g, 0, sg.k);
    smeta[lane] = sg.k;
  }
  wave_lds_sync();
  for (int r = 1; r <= adds; ++r) {
    if (in) {
      slik[64 + lane] = val(g, r, sg.k);
      smeta[64 + lane] = 64u * r + sg.k;
    }
    wave_lds_sync();
    seg2m_nth_slots(in ? 2 * S : 0, S - 1, sg, slik, smeta, lpos, rpos, junk);
  }
  double acc = 0.0;
  if (in) acc = slik[lane] * (double)(smeta[lane] % 97);
  acc = fold(acc);
  if (lane == 0) out[blockIdx.x] = acc;
}

// mode 6: four links per lane (segE_nth_slots<4>)
__global__ __launch_bounds__(64) void bench_seg4e(int S, int adds, double *out) {
  extern __shared__ unsigned char sm[];
  const int lane = threadIdx.x;
  const int W = (2 * S + 3) / 4;
  // slots (64 / W + 1) x 4W <= 16 x 20 = 320 per wave
  SegScratch ss{(int *)sm, (int *)(sm + 1280), (int *)(sm + 2560), (double *)(sm + 4608), (uint32_t *)(sm + 7168)};
  const Seg sg = make_seg(W);
  const int G = 64 / W;
  const bool in = sg.g < G;
  const uint32_t g = blockIdx.x * G + sg.g;
  const int sb = sg.g * 4 * W;
  for (int j = 0; j < 4; ++j) {
    const int p = sg.k + j * W;
    if (in && p < S) {
      ss.slik[sb + p] = val(g, 0, p);
      ss.smeta[sb + p] = p;
    }
  }
  wave_lds_sync();
  for (int r = 1; r <= adds; ++r) {
    for (int j = 0; j < 4; ++j) {
      const int p = sg.k + j * W;
      if (in && p >= S && p < 2 * S) {
        ss.slik[sb + p] = val(g, r, p - S);
        ss.smeta[sb + p] = 64u * r + p - S;
      }
    }
    wave_lds_sync();
    segE_nth_slots<4>(in ? 2 * S : 0, S - 1, sg, ss);
  }
  double acc = 0.0;
  for (int j = 0; j < 4; ++j) {
    const int p = sg.k + j * W;
    if (in && p < S) acc += ss.slik[sb + p] * (double)(ss.smeta[sb + p] % 97);
  }
  acc = fold(acc);
  if (lane == 0) out[blockIdx.x] = acc;
}


__global__ __launch_bounds__(64) void bench_seg(int S, int adds, double *out) {
  extern __shared__ unsigned char sm[];
  const int lane = threadIdx.x;
  SegScratch ss{(int *)sm, (int *)sm + 64, (int *)sm + 128, (double *)(sm + 1024), (uint32_t *)(sm + 1024 + 512)};
  const Seg sg = make_seg(2 * S);
  const int G = 64 / (2 * S);
  const bool in = sg.g < G;
  const uint32_t g = blockIdx.x * G + sg.g;
  if (in && sg.k < S) {
    ss.slik[lane] = val(g, 0, sg.k);
    ss.smeta[lane] = sg.k;
  }
  wave_lds_sync();
  for (int r = 1; r <= adds; ++r) {
    if (in && sg.k >= S) {
      ss.slik[lane] = val(g, r, sg.k - S);
      ss.smeta[lane] = 64u * r + sg.k - S;
    }
    wave_lds_sync();
    seg_nth_slots(in ? 2 * S : 0, S - 1, sg, ss);
  }
  double acc = 0.0;
  if (in && sg.k < S) acc = ss.slik[lane] * (double)(ss.smeta[lane] % 97);
  acc = fold(acc);
  if (lane == 0) out[blockIdx.x] = acc;
}

// mode 4: two sets of 64 / 2S lists per wave, selections interleaved
// (seg_nth_slots_multi<2>)
__global__ __launch_bounds__(64) void bench_seg2(int S, int adds, double *out) {
  extern __shared__ unsigned char sm[];
  const int lane = threadIdx.x;
  SegScratch ss[2] = {
      {(int *)sm, (int *)sm + 64, (int *)sm + 128, (double *)(sm + 1024), (uint32_t *)(sm + 1024 + 512)},
      {(int *)(sm + 2048), (int *)(sm + 2048) + 64, (int *)(sm + 2048) + 128, (double *)(sm + 2048 + 1024),
       (uint32_t *)(sm + 2048 + 1024 + 512)}};
  const Seg sg = make_seg(2 * S);
  const int G = 64 / (2 * S);
  const bool in = sg.g < G;
  uint32_t g[2];
  for (int u = 0; u < 2; ++u) {
    g[u] = (blockIdx.x * 2 + u) * G + sg.g;
    if (in && sg.k < S) {
      ss[u].slik[lane] = val(g[u], 0, sg.k);
      ss[u].smeta[lane] = sg.k;
    }
  }
  wave_lds_sync();
  for (int r = 1; r <= adds; ++r) {
    for (int u = 0; u < 2; ++u)
      if (in && sg.k >= S) {
        ss[u].slik[lane] = val(g[u], r, sg.k - S);
        ss[u].smeta[lane] = 64u * r + sg.k - S;
      }
    wave_lds_sync();
    const int n[2] = {in ? 2 * S : 0, in ? 2 * S : 0}, nth[2] = {S - 1, S - 1};
    seg_nth_slots_multi<2>(n, nth, sg, ss);
  }
  double acc = 0.0;
  for (int u = 0; u < 2; ++u)
    if (in && sg.k < S) acc += ss[u].slik[lane] * (double)(ss[u].smeta[lane] % 97);
  acc = fold(acc);
  if (lane == 0) out[blockIdx.x] = acc;
}

// mode 5: two elements per lane, S lanes per list (seg2_nth_slots); mode 8:
// the same (the round-4 A/B of the cut from the swap count, now the only one)
template <bool KCUT>
__global__ __launch_bounds__(64) void bench_seg2e(int S, int adds, double *out) {
  extern __shared__ unsigned char sm[];
  const int lane = threadIdx.x;
  // slots: (64 / S + 1) x 2S <= 160 per wave (lanes past the last segment
  // address a dead segment of their own)
  SegScratch ss{(int *)sm, (int *)(sm + 640), (int *)(sm + 1280), (double *)(sm + 2304), (uint32_t *)(sm + 3584)};
  const Seg sg = make_seg(S);
  const int G = 64 / S;
  const bool in = sg.g < G;
  const uint32_t g = blockIdx.x * G + sg.g;
  const int sb = sg.g * 2 * S;
  if (in) {
    ss.slik[sb + sg.k] = val(g, 0, sg.k);
    ss.smeta[sb + sg.k] = sg.k;
  }
  wave_lds_sync();
  for (int r = 1; r <= adds; ++r) {
    if (in) {
      ss.slik[sb + S + sg.k] = val(g, r, sg.k);
      ss.smeta[sb + S + sg.k] = 64u * r + sg.k;
    }
    wave_lds_sync();
    (void)KCUT;
    seg2_nth_slots(in ? 2 * S : 0, S - 1, sg, ss);
  }
  double acc = 0.0;
  if (in) acc = ss.slik[sb + sg.k] * (double)(ss.smeta[sb + sg.k] % 97);
  acc = fold(acc);
  if (lane == 0) out[blockIdx.x] = acc;
}

template <bool MASKS>
__global__ __launch_bounds__(64) void bench_lane(int S, int adds, double *out) {
  extern __shared__ unsigned char sm[];
  const int lane = threadIdx.x;
  const uint32_t g = blockIdx.x * 64 + lane;
  // column `lane` of a [2S][64] image: element k at row k
  double *col = (double *)sm + lane;
  uint32_t *mcol = (uint32_t *)(sm + (size_t)2 * S * 64 * 8) + lane;
  const LinkList L{col, mcol, 64};
  for (int k = 0; k < S; ++k) L.set(k, val(g, 0, k), (uint32_t)k);
  for (int r = 1; r <= adds; ++r) {
    for (int k = 0; k < S; ++k) L.set(S + k, val(g, r, k), 64u * r + k);
    if (MASKS) nth_element_greater_masks(L, 2 * S, S - 1, 2 * S);
    else nth_element_greater(L, 2 * S, S - 1);
  }
  double acc = 0.0;
  for (int k = 0; k < S; ++k) acc += L.l(k) * (double)(L.m(k) % 97);
  acc = fold(acc);
  if (lane == 0) out[blockIdx.x] = acc;
}

int main(int argc, char **argv) {
  const int wpc = argc > 1 ? atoi(argv[1]) : 16, adds = argc > 2 ? atoi(argv[2]) : 2000;
  const int mode = argc > 3 ? atoi(argv[3]) : 0, S = argc > 4 ? atoi(argv[4]) : 10;
  int cu = 256;
  (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  // mode 0: lists = cu * wpc * (64 / 2S);
  // modes 2/3: wpc waves of 64 lists per CU.  Mode 0 with the same wpc and
  // mode 2/3 with wpc / (32 / S) process the same lists.
  const int G = 64 / (2 * S);
  const int lists = mode == 2 || mode == 3 ? cu * wpc * 64 : cu * wpc * G;
  if (mode < 0 || mode == 1 || mode > 8) return 1;
  const int G5 = 64 / S, G6 = 64 / ((2 * S + 3) / 4);
  int grid = mode == 0 ? cu * wpc
                       : (mode == 4 ? cu * wpc / 2
                                    : (mode == 5 || mode == 7 || mode == 8 ? (lists + G5 - 1) / G5
                                                              : (mode == 6 ? (lists + G6 - 1) / G6 : (lists + 63) / 64)));
  size_t lds = mode == 2 || mode == 3 ? (size_t)2 * S * 64 * 12 : (mode == 4 ? 4096 : (mode == 5 || mode == 7 || mode == 8 ? 4608 : (mode == 6 ? 8448 : 2048)));
  void (*kern)(int, int, double *) =
      mode == 0 ? bench_seg
                : (mode == 2 ? bench_lane<false>
                             : (mode == 3 ? bench_lane<true>
                                          : (mode == 4 ? bench_seg2
                                                       : (mode == 5 ? bench_seg2e<false> : (mode == 8 ? bench_seg2e<true> : (mode == 6 ? bench_seg4e : bench_seg2m))))));
  if (lds > 65536) (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  double *out;
  (void)hipMalloc(&out, grid * sizeof(double));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, 0, S, 10, out);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, 0, S, adds, out);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  double *h = (double *)malloc(grid * sizeof(double)), cs = 0;
  (void)hipMemcpy(h, out, grid * sizeof(double), hipMemcpyDeviceToHost);
  for (int i = 0; i < grid; ++i) cs += h[i];
  printf("mode %d S %d lists %d (%d waves, %.1f per CU) adds %d: %.2f ms, %.2f ns per add (throughput), "
         "%.0f cycles per add per list at 2.4 GHz (latency), checksum %.17g\n",
         mode, S, lists, grid, (double)grid / cu, adds, ms, ms * 1e6 / ((double)lists * adds), ms * 1e-3 * 2.4e9 / adds, cs);
  return 0;
}
