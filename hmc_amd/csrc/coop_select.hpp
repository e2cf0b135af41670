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
  uint64_t mask;  // lanes of the segment
  uint64_t lt;    // lanes of the segment below this lane
};

__device__ inline Seg make_seg(int SW) {
  Seg s;
  const int lane = threadIdx.x;
  const int G = 64 / SW;
  s.g = lane / SW;
  s.base = s.g * SW;
  s.k = lane - s.base;
  const uint64_t w = SW >= 64 ? ~0ull : ((1ull << SW) - 1ull);
  s.mask = s.g < G ? (w << s.base) : 0ull;
  s.lt = s.mask & ((1ull << lane) - 1ull);
  return s;
}

// LDS scratch of the segmented selection, one entry per lane (segment g uses
// [base, base+SW)): left-stop and right-stop positions, and a spill list for
// the heap-select path.
struct SegScratch {
  int *lpos;      // [64]
  int *rpos;      // [64]
  double *slik;   // [64]
  uint32_t *smeta;
};

// std::nth_element(v, v+nth, v+n, greater) on every segment's list (lane
// g*SW+k holds element k; n, nth uniform inside a segment, n <= SW <= 32;
// n == 0 marks an idle segment).  Whole-wave call.
__device__ inline void seg_nth_element(double &v, uint32_t &m, int n, int nth, const Seg &sg,
                                       const SegScratch &ss) {
  const int lane = threadIdx.x;
  int first = 0, last = n, depth = n > 0 ? lg2_floor(n) * 2 : 0;
  bool act = n > 0 && nth != n && sg.mask != 0ull;
  bool heap = false;
  int *lp = ss.lpos + sg.base, *rp = ss.rpos + sg.base;
  while (true) {
    if (act && last - first > 3 && depth == 0) heap = true;
    const bool part = act && !heap && last - first > 3;
    if (!__any(part)) break;
    if (part) --depth;
    // std::__move_median_to_first(first, first+1, mid, last-1) (stl_algo.h:79-102)
    const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
    const double va = gat_f64(v, sg.base + a), vb = gat_f64(v, sg.base + b), vc = gat_f64(v, sg.base + c);
    const double vf = gat_f64(v, sg.base + first);
    const int r = va > vb ? (vb > vc ? b : (va > vc ? c : a)) : (va > vc ? a : (vb > vc ? c : b));
    const double vr = r == a ? va : (r == b ? vb : vc);
    const uint32_t mr = gat_u32(m, sg.base + r), mf = gat_u32(m, sg.base + first);
    if (part) {
      if (sg.k == first) { v = vr; m = mr; }
      else if (sg.k == r) { v = vf; m = mf; }
    }
    const double pivot = vr;
    const bool inr = part && sg.k >= first && sg.k < last;
    const bool isL = inr && sg.k != first && !(v > pivot);
    const bool isR = inr && !(pivot > v);
    const uint64_t Lw = __ballot(isL) & sg.mask, Rw = __ballot(isR) & sg.mask;
    const int nL = __popcll(Lw), nR = __popcll(Rw);
    const int kL = __popcll(Lw & sg.lt);
    const int kR = nR - 1 - __popcll(Rw & sg.lt);
    if (isL) lp[kL] = sg.k;
    if (isR) rp[kR] = sg.k;
    wave_lds_sync();
    int partner = lane;
    bool lswap = false;  // swapped in the left-stop role (a tie can be both stops)
    if (isL && kL < nR) {
      const int q = rp[kL];
      if (sg.k < q) {
        partner = sg.base + q;
        lswap = true;
      }
    }
    if (isR && kR < nL) {
      const int q = lp[kR];
      if (q < sg.k) partner = sg.base + q;
    }
    const int K = __popcll(__ballot(lswap) & sg.mask);
    const int lK = K < nL ? lp[K] : 64;
    const int rK = K >= 1 ? rp[K - 1] : 64;
    wave_lds_sync();
    const double nv = gat_f64(v, partner);
    const uint32_t nm = gat_u32(m, partner);
    if (part) {
      v = nv;
      m = nm;
      const int cut = lK < rK ? lK : rK;
      if (cut <= nth) first = cut;
      else last = cut;
    }
  }
  // Depth limit reached (std::__heap_select + iter_swap, stl_algo.h:1973-1979):
  // rare, so the segment spills to LDS and its first lane runs the sequential code.
  if (__any(heap)) {
    double *sl = ss.slik + sg.base;
    uint32_t *sm = ss.smeta + sg.base;
    if (heap && sg.k < n) { sl[sg.k] = v; sm[sg.k] = m; }
    wave_lds_sync();
    if (heap && sg.k == 0) {
      const LinkList w{sl, sm, 1};
      heap_select(w, first, nth + 1, last);
      w.swap(first, nth);
    }
    wave_lds_sync();
    if (heap && sg.k < n) { v = sl[sg.k]; m = sm[sg.k]; }
    wave_lds_sync();
  }
  // std::__insertion_sort of the <= 3 remaining elements (stl_algo.h:1819-1849)
  const bool ins = act && !heap && last - first > 1;
  if (__any(ins)) {
    const int len = last - first;
    double x0 = gat_f64(v, sg.base + first), x1 = gat_f64(v, sg.base + first + 1), x2 = gat_f64(v, sg.base + first + 2);
    uint32_t y0 = gat_u32(m, sg.base + first), y1 = gat_u32(m, sg.base + first + 1), y2 = gat_u32(m, sg.base + first + 2);
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
    if (ins) {
      const int j = sg.k - first;
      if (j == 0) { v = x0; m = y0; }
      else if (j == 1) { v = x1; m = y1; }
      else if (j == 2 && len > 2) { v = x2; m = y2; }
    }
  }
}

}  // namespace hmc
