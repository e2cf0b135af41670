// coop_select.hpp — the libstdc++ (GCC 11) std::nth_element of select.hpp,
// run by a wavefront on several lists at once.  The wave is cut into
// segments of SW = 2S lanes; segment g holds one list, element k in lane
// g*SW + k.  Every step is evaluated for all segments together with ballots,
// lane shuffles and small LDS exchanges, and produces exactly the element
// permutation of the sequential algorithm (select.hpp).
//
// Partition (std::__unguarded_partition, stl_algo.h:1878-1896; comp =
// greater, pivot at `first`): the left scan stops at positions p in
// [first+1,last) with !(v[p] > pivot) ("left stops"), the right scan at p in
// [first,last) with !(pivot > v[p]) ("right stops"; `first` itself is one).
// Let l_k be the k-th left stop from the left and r_k the k-th right stop
// from the right, on the values the partition starts from.  A swapped value
// is only met again where the scans cross, and there it stops the scan at once
// (a value moved right came from a left stop and vice versa), so the loop
// swaps l_k <-> r_k exactly for the k with l_k < r_k — a prefix k < K, both
// sequences being monotone — and returns cut = min(l_K, r_{K-1}) (r_{-1} =
// infinity).  No position takes part in two swaps.  Each segment therefore
// numbers its stops (ballot + popcount), the stops publish their positions in
// two small LDS arrays, and every stop reads its partner: one shuffle then
// moves all swapped elements.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "select.hpp"

namespace hmc {

__device__ inline double rl_f64(double x, int lane) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ inline uint32_t rl_u32(uint32_t x, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)x, lane); }

// Lane gather over the whole wave (ds_bpermute); src is taken modulo 64.
__device__ inline uint32_t gat_u32(uint32_t x, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)x);
}
__device__ inline double gat_f64(double x, int src) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const uint32_t lo = gat_u32((uint32_t)b, src), hi = gat_u32((uint32_t)(b >> 32), src);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Cross-lane LDS exchange inside one wavefront: the LDS executes a wave's
// instructions in order, so only the compiler must keep the accesses in
// program order (no s_barrier, no wait on outstanding HBM stores).
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// This lane's place in the segmentation (SW lanes per segment, G segments).
struct Seg {
  int g;          // segment index (>= G: lane outside every segment)
  int base;       // first lane of the segment
  int k;          // element index inside the segment
  int sw;         // segment width
  uint64_t mask;  // lanes of the segment
  uint64_t lt;    // lanes of the segment below this lane
  uint32_t wm;    // segment-relative: all SW bits (0 outside every segment)
  uint32_t ltk;   // segment-relative: bits below k
};

// Lane mask of a predicate; unlike __ballot(int) the predicate stays a mask
// (no 0/1 materialisation and re-compare).
__device__ inline uint64_t wave_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// A wave ballot seen from this lane's segment (bit k = element k).
__device__ inline uint32_t seg_bits(uint64_t ballot, const Seg &sg) { return (uint32_t)(ballot >> sg.base) & sg.wm; }

__device__ inline Seg make_seg(int SW) {
  Seg s;
  const int lane = (int)(threadIdx.x & 63);
  const int G = 64 / SW;
  s.g = lane / SW;
  s.base = s.g * SW;
  s.k = lane - s.base;
  s.sw = SW;
  const uint64_t w = SW >= 64 ? ~0ull : ((1ull << SW) - 1ull);
  s.mask = s.g < G ? (w << s.base) : 0ull;
  s.lt = s.mask & ((1ull << lane) - 1ull);
  s.wm = s.g < G ? (SW >= 32 ? ~0u : ((1u << SW) - 1u)) : 0u;
  s.ltk = s.k < 32 ? (1u << s.k) - 1u : ~0u;
  return s;
}

// Lowest set element of a segment-relative mask (64 if none).
__device__ inline int seg_lowest(uint32_t bits) {
  return bits ? __builtin_ctz(bits) : 64;
}

// LDS scratch of the segmented selection, one entry per lane (segment g uses
// [base, base+SW)): left-stop and right-stop positions, a per-lane junk slot
// pair that absorbs the writes of lanes that are not stops, and a spill list
// for the heap-select path.
struct SegScratch {
  int *lpos;      // [64]
  int *rpos;      // [64]
  int *junk;      // [128]
  double *slik;   // [64]
  uint32_t *smeta;
};

// std::nth_element(v, v+nth, v+n, greater) on every segment's list, in
// place in the LDS slots slik/smeta (segment g's element k in slot
// g*SW + k; n, nth uniform inside a segment, n <= SW <= 64; n == 0 marks an
// idle segment).  Whole-wave call, branch-free per lane for SW <= 32.
//
// One partition costs two LDS round trips: one batch that reads the median
// candidates, the value at `first` and every lane's own element, and the stop
// pairing; each lane then writes its element straight into its destination
// slot (the LDS executes a wave's accesses in order, so no wait).  The median
// swap (std::__move_median_to_first) is not executed as a data move: the
// ballots are taken over *positions* (lane p evaluates the value position p
// holds after the swap: the pivot at `first`, first's value at r), and each
// lane's element enters the partition at x = tau(lane), tau = (first r).
__device__ inline void seg_nth_slots(int n, int nth, const Seg &sg, const SegScratch &ss) {
  const int lane = (int)(threadIdx.x & 63);
  const int k = sg.k;
  if (sg.sw > 32) {  // lists of up to 64 (S > 16): one per wave, the sequential algorithm on its first lane
    if (n > 0 && nth != n && sg.mask != 0ull && k == 0) {
      const LinkList wl{ss.slik + sg.base, ss.smeta + sg.base, 1};
      nth_element_greater(wl, n, nth);
    }
    wave_lds_sync();
    return;
  }
  int first = 0, last = n, depth = n > 0 ? lg2_floor(n) * 2 : 0;
  const bool act = n > 0 && nth != n && sg.mask != 0ull;
  double *sl = ss.slik + sg.base;
  uint32_t *sm = ss.smeta + sg.base;
  int *lp = ss.lpos + sg.base, *rp = ss.rpos + sg.base;
  int *jl = ss.junk + lane, *jr = ss.junk + 64 + lane;
  const int kmax = sg.sw - 1;
  while (true) {
    // a segment whose depth budget is spent stops here with > 3 elements left
    // and finishes with the heap select below (its range no longer changes)
    const bool part = act && last - first > 3 && depth > 0;
    if (!wave_ballot(part)) break;
    depth -= part ? 1 : 0;
    // std::__move_median_to_first(first, first+1, mid, last-1) (stl_algo.h:79-102)
    const int a = first + 1, b = first + ((last - first) >> 1), c = last > 0 ? last - 1 : 0;
    const double va = sl[a], vb = sl[b], vc = sl[c], vf = sl[first];
    const double v = sl[k];
    const uint32_t m = sm[k];
    // which of a (0), b (1), c (2) is the median, as a table over the three
    // comparisons (index ab*4 + bc*2 + ac) so it compiles to selects
    const int idx = (va > vb ? 4 : 0) | (vb > vc ? 2 : 0) | (va > vc ? 1 : 0);
    const int w = (22561 >> (2 * idx)) & 3;
    const int r = w == 0 ? a : (w == 1 ? b : c);
    const double pivot = w == 0 ? va : (w == 1 ? vb : vc);
    // stops by position (std::__unguarded_partition, stl_algo.h:1878-1896):
    // left scan over [first+1, last) stops at !(x > pivot), right scan over
    // [first, last) at !(pivot > x)
    const double pv = k == first ? pivot : (k == r ? vf : v);
    // each ballot of a single comparison stays a lane mask; the conjunctions
    // are scalar ANDs (a ballot of a && b would be materialised and re-compared)
    const uint64_t b_part = wave_ballot(part), b_in = wave_ballot(k > first) & wave_ballot(k < last);
    const uint64_t b_first = wave_ballot(k == first);
    const uint64_t b_le = wave_ballot(!(pv > pivot)), b_ge = wave_ballot(!(pivot > pv));
    const uint32_t Lw = seg_bits(b_part & b_in & b_le, sg);
    const uint32_t Rw = seg_bits(b_part & (b_in | b_first) & b_ge, sg);
    const int nL = __popc(Lw), nR = __popc(Rw);
    // this lane's element is at position x once the median is at first
    const int x = !part ? k : (k == first ? r : (k == r ? first : k));
    const uint32_t xb = (1u << x) - 1u;
    const bool isL = part && ((Lw >> x) & 1u), isR = part && ((Rw >> x) & 1u);
    const int kL = __popc(Lw & xb);
    const int kR = nR - 1 - __popc(Rw & xb);
    *(isL ? lp + kL : jl) = x;
    *(isR ? rp + kR : jr) = x;
    wave_lds_sync();
    const int qR = rp[kL < kmax ? kL : kmax];
    const int qL = lp[kR < 0 ? 0 : (kR < kmax ? kR : kmax)];
    // pair k swaps iff l_k < r_k; both roles are checked, a position swaps at most once
    const bool lsw = isL && kL < nR && x < qR;
    const bool rsw = isR && kR < nL && qL < x;
    const int dest = lsw ? qR : (rsw ? qL : x);
    sl[dest] = v;
    sm[dest] = m;
    // cut = min(l_K, r_{K-1}): the first left stop that does not swap and the
    // lowest right stop that does.  The swaps are a prefix of the stop pairs,
    // so with K = the number of swapping pairs both come from the stop
    // positions still in lp / rp.
    const int K = __popcll(wave_ballot(lsw) & sg.mask);
    const int lK = K < nL ? lp[K < kmax ? K : kmax] : 64;
    const int rK = K > 0 ? rp[K - 1 < kmax ? K - 1 : kmax] : 64;
    const int cut = lK < rK ? lK : rK;
    wave_lds_sync();
    first = part && cut <= nth ? cut : first;
    last = part && cut > nth ? cut : last;
  }
  // Depth limit reached (std::__heap_select + iter_swap, stl_algo.h:1973-1979):
  // rare; the segment's first lane runs the sequential code on the slots.
  const bool heap = act && last - first > 3;
  if (wave_ballot(heap)) {
    if (heap && k == 0) {
      const LinkList wl{sl, sm, 1};
      heap_select(wl, first, nth + 1, last);
      wl.swap(first, nth);
    }
    wave_lds_sync();
  }
  // std::__insertion_sort of the <= 3 remaining elements (stl_algo.h:1819-1849)
  const bool ins = act && !heap && last - first > 1;
  if (wave_ballot(ins)) {
    const int len = last - first;
    const int f0 = first < kmax ? first : kmax;
    const int f1 = first + 1 < kmax ? first + 1 : kmax, f2 = first + 2 < kmax ? first + 2 : kmax;
    double x0 = sl[f0], x1 = sl[f1], x2 = sl[f2];
    uint32_t y0 = sm[f0], y1 = sm[f1], y2 = sm[f2];
    if (x1 > x0) {
      const double t = x1; x1 = x0; x0 = t;
      const uint32_t u = y1; y1 = y0; y0 = u;
    }
    if (len > 2) {
      if (x2 > x0) {
        const double t = x2; const uint32_t u = y2;
        x2 = x1; y2 = y1; x1 = x0; y1 = y0; x0 = t; y0 = u;
      } else if (x2 > x1) {
        const double t = x2; const uint32_t u = y2;
        x2 = x1; y2 = y1; x1 = t; y1 = u;
      }
    }
    const int j = k - first;
    const bool mine = ins && (j == 0 || j == 1 || (j == 2 && len > 2));
    const double xv = j == 0 ? x0 : (j == 1 ? x1 : x2);
    const uint32_t yv = j == 0 ? y0 : (j == 1 ? y1 : y2);
    wave_lds_sync();
    if (mine) {
      ss.slik[lane] = xv;
      ss.smeta[lane] = yv;
    }
    wave_lds_sync();
  }
}

// The same selection with two elements per lane: segment g of W = S lanes
// holds a list of up to 2S <= 32 links in its slots [g*2W, g*2W + 2W); lane k
// of the segment carries positions k (element 0) and k + W (element 1), so a
// wavefront works on 64 / W lists (S = 10: 6) instead of 64 / 2W.  The
// per-segment work of a partition (median, stop masks, cut) is shared by the
// two elements; only the per-element compares, ranks and moves double.  The
// permutation is the one of seg_nth_slots (the stop masks are assembled from
// the two elements' ballots, bit p = position p).  sg = make_seg(W); the
// scratch arrays hold (64 / W + 1) x 2W slots: lanes past the last segment
// address a dead segment of their own.
__device__ inline void seg2_nth_slots(int n, int nth, const Seg &sg, const SegScratch &ss) {
  const int lane = (int)(threadIdx.x & 63);
  const int W = sg.sw, k = sg.k;
  int first = 0, last = n, depth = n > 0 ? lg2_floor(n) * 2 : 0;
  const bool act = n > 0 && nth != n && sg.mask != 0ull;
  const int sb = sg.g * 2 * W;  // the segment's first slot
  double *sl = ss.slik + sb;
  uint32_t *sm = ss.smeta + sb;
  int *lp = ss.lpos + sb, *rp = ss.rpos + sb;
  int *jl0 = ss.junk + lane, *jl1 = ss.junk + 64 + lane, *jr0 = ss.junk + 128 + lane, *jr1 = ss.junk + 192 + lane;
  const int kmax = 2 * W - 1;
  const int p0 = k, p1 = k + W;  // this lane's positions
  while (true) {
    const bool part = act && last - first > 3 && depth > 0;
    if (!wave_ballot(part)) break;
    depth -= part ? 1 : 0;
    // std::__move_median_to_first(first, first+1, mid, last-1) (stl_algo.h:79-102)
    const int a = first + 1, b = first + ((last - first) >> 1), c = last > 0 ? last - 1 : 0;
    const double va = sl[a], vb = sl[b], vc = sl[c], vf = sl[first];
    const double v0 = sl[p0], v1 = sl[p1];
    const uint32_t m0 = sm[p0], m1 = sm[p1];
    const int idx = (va > vb ? 4 : 0) | (vb > vc ? 2 : 0) | (va > vc ? 1 : 0);
    const int w = (22561 >> (2 * idx)) & 3;
    const int r = w == 0 ? a : (w == 1 ? b : c);
    const double pivot = w == 0 ? va : (w == 1 ? vb : vc);
    // the value each position holds once the median is at first
    const double pv0 = p0 == first ? pivot : (p0 == r ? vf : v0);
    const double pv1 = p1 == first ? pivot : (p1 == r ? vf : v1);
    // stop masks over positions: ballot bits of element 0 at [0, W), element 1 at [W, 2W)
    const uint32_t le = seg_bits(wave_ballot(!(pv0 > pivot)), sg) | seg_bits(wave_ballot(!(pv1 > pivot)), sg) << W;
    const uint32_t ge = seg_bits(wave_ballot(!(pivot > pv0)), sg) | seg_bits(wave_ballot(!(pivot > pv1)), sg) << W;
    const uint32_t below_last = last >= 32 ? ~0u : ((1u << last) - 1u);
    const uint32_t inR = part ? below_last & ~((1u << first) - 1u) : 0u;  // [first, last)
    const uint32_t inL = inR & ~(1u << first);                             // (first, last)
    const uint32_t Lw = le & inL, Rw = ge & inR;
    const int nL = __popc(Lw), nR = __popc(Rw);
    // each element's position once the median is at first
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
    sl[d0] = v0;
    sm[d0] = m0;
    sl[d1] = v1;
    sm[d1] = m1;
    // cut = min(l_K, r_{K-1}) (see seg_nth_slots), K = the number of swapping
    // pairs: the swaps are a prefix of the stop pairs, and the stops' positions
    // are still in lp / rp (one popcount and two LDS reads instead of four
    // stop ballots re-based to positions: 3.7-4.5 % less time per add,
    // coop_bench mode 8 vs 5, profiles/r04/coop/)
    const int K = __popcll(wave_ballot(lsw0) & sg.mask) + __popcll(wave_ballot(lsw1) & sg.mask);
    const int lK = K < nL ? lp[K < kmax ? K : kmax] : 64;
    const int rK = K > 0 ? rp[K - 1 < kmax ? K - 1 : kmax] : 64;
    const int cut = lK < rK ? lK : rK;
    wave_lds_sync();
    first = part && cut <= nth ? cut : first;
    last = part && cut > nth ? cut : last;
  }
  // depth limit: std::__heap_select + iter_swap on the segment's first lane
  const bool heap = act && last - first > 3;
  if (wave_ballot(heap)) {
    if (heap && k == 0) {
      const LinkList wl{sl, sm, 1};
      heap_select(wl, first, nth + 1, last);
      wl.swap(first, nth);
    }
    wave_lds_sync();
  }
  // std::__insertion_sort of the <= 3 remaining elements (stl_algo.h:1819-1849)
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
    const int j0 = p0 - first, j1 = p1 - first;
    const bool mine0 = ins && (j0 == 0 || j0 == 1 || (j0 == 2 && len > 2));
    const bool mine1 = ins && (j1 == 0 || j1 == 1 || (j1 == 2 && len > 2));
    const double z0 = j0 == 0 ? y0 : (j0 == 1 ? y1 : y2), z1 = j1 == 0 ? y0 : (j1 == 1 ? y1 : y2);
    const uint32_t u0 = j0 == 0 ? t0 : (j0 == 1 ? t1 : t2), u1 = j1 == 0 ? t0 : (j1 == 1 ? t1 : t2);
    wave_lds_sync();
    if (mine0) {
      sl[p0] = z0;
      sm[p0] = u0;
    }
    if (mine1) {
      sl[p1] = z1;
      sm[p1] = u1;
    }
    wave_lds_sync();
  }
}

// Value-only top-S of every segment's list (slots [0, n), n <= SW): each
// element's rank is the number of elements greater than it plus the equal ones
// in lower slots, and the S best are written to slots [0, S) in rank order.
// Returns, on the lane that finds one, the non-zero value straddling the
// S-cut (the element ranked S equals one ranked above it), else 0: only such
// a tie can make the retained set depend on the order libstdc++ would have
// left the list in — and only if it is still at the cut when the list is
// complete (a later, larger cut evicts both tied elements anyway).  Segments
// with n <= S are left untouched.  Whole-wave call.
__device__ inline double seg_rank_select(int n, int S, const Seg &sg, const SegScratch &ss) {
  const int k = sg.k;
  const double *sl = ss.slik + (sg.mask != 0ull ? sg.base : 0);
  const bool mine = sg.mask != 0ull && n > S && k < n;
  const double v = mine ? sl[k] : 0.0;
  const uint32_t m = mine ? ss.smeta[sg.base + k] : 0u;
  int gt = 0, eq = 0;
  for (int q = 0; q < sg.sw; q += 2) {  // two slots per read; segment lanes read the same address
    const double2 y = *(const double2 *)(sl + q);
    gt += (q < n && y.x > v) ? 1 : 0;
    eq += (q < k && y.x == v) ? 1 : 0;
    gt += (q + 1 < n && y.y > v) ? 1 : 0;
    eq += (q + 1 < k && y.y == v) ? 1 : 0;
  }
  const int rank = gt + eq;
  wave_lds_sync();
  if (mine && rank < S) {
    ss.slik[sg.base + rank] = v;
    ss.smeta[sg.base + rank] = m;
  }
  wave_lds_sync();
  return mine && rank == S && eq > 0 ? v : 0.0;
}

// Register interface: lane g*SW+k holds element k of segment g's list.
__device__ inline void seg_nth_element(double &v, uint32_t &m, int n, int nth, const Seg &sg,
                                       const SegScratch &ss) {
  const int lane = (int)(threadIdx.x & 63);
  ss.slik[lane] = v;
  ss.smeta[lane] = m;
  wave_lds_sync();
  seg_nth_slots(n, nth, sg, ss);
  v = ss.slik[lane];
  m = ss.smeta[lane];
}

}  // namespace hmc
