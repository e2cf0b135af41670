// select.hpp — k-best selection with libstdc++ (GCC 11) tie semantics.
//
// The reference keeps the k best HaploPairLinks with
//   std::nth_element(v.begin(), v.begin()+k-1, v.end(), greater<HaploPairLink>())
// (HaploPair.cpp:86, HaploBuilder.cpp:101) and orders the final list with
//   std::sort(..., greater<HaploPairLink>())            (HaploBuilder.cpp:105).
// The comparator looks at the likelihood only (HaploPair.h:44-52), so WHICH of
// several equal-likelihood links survive is decided by the element permutation
// the library algorithm performs.  Bit-exact parity of the selected haplotype
// pair therefore needs the same algorithm, step for step: introselect with a
// median-of-three pivot and an unguarded Hoare partition, heap-select fallback
// at depth 2*lg(n), and a final insertion sort (for n <= 16 std::sort is just
// the insertion sort).  This header restates that algorithm over an abstract
// "list" so one body serves device code (lists striped across a wavefront in
// LDS) and host code (plain arrays, used by the CPU-side tests).
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define HMC_HD __host__ __device__ __forceinline__
#else
#define HMC_HD inline
#endif

namespace hmc {

// A list view: element k lives at lik[k*stride], meta[k*stride].  The
// algorithms below take any view with the same members (l, m, set, copy,
// swap, gt), e.g. one typed for LDS in the value pass.
struct LinkList {
  double *lik;
  uint32_t *meta;
  int stride;
  HMC_HD double l(int k) const { return lik[k * stride]; }
  HMC_HD uint32_t m(int k) const { return meta[k * stride]; }
  HMC_HD void set(int k, double x, uint32_t y) const {
    lik[k * stride] = x;
    meta[k * stride] = y;
  }
  HMC_HD void copy(int dst, int src) const { set(dst, l(src), m(src)); }
  HMC_HD void swap(int a, int b) const {
    double x = l(a);
    uint32_t y = m(a);
    copy(a, b);
    set(b, x, y);
  }
  // comp(a, b) == greater<HaploPairLink>()(v[a], v[b])
  HMC_HD bool gt(int a, int b) const { return l(a) > l(b); }
};

HMC_HD int lg2_floor(int n) { return 31 - __builtin_clz((unsigned)n); }

// std::__move_median_to_first (stl_algo.h:79-102)
template <class V>
HMC_HD void move_median_to_first(const V &v, int result, int a, int b, int c) {
  if (v.gt(a, b)) {
    if (v.gt(b, c)) v.swap(result, b);
    else if (v.gt(a, c)) v.swap(result, c);
    else v.swap(result, a);
  } else if (v.gt(a, c)) v.swap(result, a);
  else if (v.gt(b, c)) v.swap(result, c);
  else v.swap(result, b);
}

// std::__unguarded_partition (stl_algo.h:1878-1896); pivot value stays at `pivot`.
template <class V>
HMC_HD int unguarded_partition(const V &v, int first, int last, int pivot) {
  while (true) {
    while (v.gt(first, pivot)) ++first;
    --last;
    while (v.gt(pivot, last)) --last;
    if (!(first < last)) return first;
    v.swap(first, last);
    ++first;
  }
}

// std::__unguarded_partition_pivot (stl_algo.h:1900-1907)
template <class V>
HMC_HD int unguarded_partition_pivot(const V &v, int first, int last) {
  int mid = first + (last - first) / 2;
  move_median_to_first(v, first, first + 1, mid, last - 1);
  return unguarded_partition(v, first + 1, last, first);
}

// std::__insertion_sort + __unguarded_linear_insert (stl_algo.h:1799-1849)
template <class V>
HMC_HD void insertion_sort(const V &v, int first, int last) {
  if (first == last) return;
  for (int i = first + 1; i != last; ++i) {
    double x = v.l(i);
    uint32_t y = v.m(i);
    if (x > v.l(first)) {
      for (int k = i; k > first; --k) v.copy(k, k - 1);
      v.set(first, x, y);
    } else {
      int hole = i, next = i - 1;
      while (x > v.l(next)) {
        v.copy(hole, next);
        hole = next;
        --next;
      }
      v.set(hole, x, y);
    }
  }
}

// std::__push_heap with a value comparator (stl_heap.h:134-149)
template <class V>
HMC_HD void push_heap(const V &v, int first, int hole, int top, double x, uint32_t y) {
  int parent = (hole - 1) / 2;
  while (hole > top && v.l(first + parent) > x) {
    v.copy(first + hole, first + parent);
    hole = parent;
    parent = (hole - 1) / 2;
  }
  v.set(first + hole, x, y);
}

// std::__adjust_heap (stl_heap.h:223-250)
template <class V>
HMC_HD void adjust_heap(const V &v, int first, int hole, int len, double x, uint32_t y) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (v.gt(first + second, first + (second - 1))) second--;
    v.copy(first + hole, first + second);
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    v.copy(first + hole, first + (second - 1));
    hole = second - 1;
  }
  push_heap(v, first, hole, top, x, y);
}

// std::__make_heap (stl_heap.h:339-360)
template <class V>
HMC_HD void make_heap(const V &v, int first, int last) {
  int len = last - first;
  if (len < 2) return;
  int parent = (len - 2) / 2;
  while (true) {
    double x = v.l(first + parent);
    uint32_t y = v.m(first + parent);
    adjust_heap(v, first, parent, len, x, y);
    if (parent == 0) return;
    parent--;
  }
}

// std::__heap_select with std::__pop_heap (stl_algo.h:1642-1651, stl_heap.h:253-266)
template <class V>
HMC_HD void heap_select(const V &v, int first, int middle, int last) {
  make_heap(v, first, middle);
  for (int i = middle; i < last; ++i) {
    if (v.gt(i, first)) {
      double x = v.l(i);
      uint32_t y = v.m(i);
      v.copy(i, first);
      adjust_heap(v, first, 0, middle - first, x, y);
    }
  }
}

// std::nth_element(first, first+nth, first+n, greater) (stl_algo.h:1964-1986, 4794-4812)
template <class V>
HMC_HD void nth_element_greater(const V &v, int n, int nth) {
  if (n == 0 || nth == n) return;
  int first = 0, last = n, depth = lg2_floor(n) * 2;
  while (last - first > 3) {
    if (depth == 0) {
      heap_select(v, first, nth + 1, last);
      v.swap(first, nth);
      return;
    }
    --depth;
    int cut = unguarded_partition_pivot(v, first, last);
    if (cut <= nth) first = cut;
    else last = cut;
  }
  insertion_sort(v, first, last);
}

// ---------------------------------------------------------------------------
// Same algorithm, partition evaluated with stop masks (lists of <= 32).
// std::__unguarded_partition with comp = greater and the pivot at `first`
// stops its left scan at p in [first+1,last) with !(v[p] > pivot) and its
// right scan at p in [first,last) with !(pivot > v[p]).  Pairing the k-th
// left stop l_k with the k-th right stop r_k (counted from the right) on the
// values the scans start from, the loop swaps l_k <-> r_k while l_k < r_k and
// returns min(l_{K+1}, r_K) after K swaps: an element moved to the right half
// came from a left stop (and vice versa), so a scan that runs into the
// already-swapped region stops at once (see coop_select.hpp).  Reading the
// range once and scanning masks replaces the pointer walk's dependent loads.
HMC_HD uint32_t bit_lo(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
HMC_HD uint32_t bit_hi(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }

// `span` >= last is the scan bound; on the device it is the same for every
// lane (2S), so the reads of one partition issue back to back.
template <class V>
HMC_HD int partition_pivot_masks(const V &v, int first, int last, int span) {
  const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
  const double va = v.l(a), vb = v.l(b), vc = v.l(c);
  // the branch tree of move_median_to_first as selects
  const int r = va > vb ? (vb > vc ? b : (va > vc ? c : a)) : (va > vc ? a : (vb > vc ? c : b));
  v.swap(first, r);
  const double pivot = v.l(first);
  uint32_t Lm = 0, Rm = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 4
#endif
  for (int k = 0; k < span; ++k) {
    const double x = v.l(k);
    const bool inr = k >= first && k < last;
    Lm |= (uint32_t)(inr && k != first && !(x > pivot)) << k;
    Rm |= (uint32_t)(inr && !(pivot > x)) << k;
  }
  int rlast = 64;
  while (true) {
    const int l = Lm ? (int)bit_lo(Lm) : 64;
    const int rr = Rm ? (int)bit_hi(Rm) : -1;
    if (!(l < rr)) return l < rlast ? l : rlast;
    v.swap(l, rr);
    Lm &= Lm - 1u;
    Rm &= ~(1u << rr);
    rlast = rr;
  }
}

// nth_element_greater with the mask partition (n <= span <= 32).
template <class V>
HMC_HD void nth_element_greater_masks(const V &v, int n, int nth, int span) {
  if (n == 0 || nth == n) return;
  int first = 0, last = n, depth = lg2_floor(n) * 2;
  while (last - first > 3) {
    if (depth == 0) {
      heap_select(v, first, nth + 1, last);
      v.swap(first, nth);
      return;
    }
    --depth;
    const int cut = partition_pivot_masks(v, first, last, span);
    if (cut <= nth) first = cut;
    else last = cut;
  }
  insertion_sort(v, first, last);
}

// std::sort(first, first+n, greater) for n <= 16 (stl_algo.h:1925-1958):
// __introsort_loop is a no-op below _S_threshold, leaving __insertion_sort.
template <class V>
HMC_HD void sort_greater_small(const V &v, int n) { insertion_sort(v, 0, n); }

// std::__unguarded_linear_insert / __unguarded_insertion_sort (stl_algo.h:1799-1869)
template <class V>
HMC_HD void unguarded_insertion_sort(const V &v, int first, int last) {
  for (int i = first; i != last; ++i) {
    const double x = v.l(i);
    const uint32_t y = v.m(i);
    int hole = i, next = i - 1;
    while (x > v.l(next)) {
      v.copy(hole, next);
      hole = next;
      --next;
    }
    v.set(hole, x, y);
  }
}

// std::sort(first, first+n, greater) for any n (stl_algo.h:1896-1958, 1925-1948):
// __introsort_loop with _S_threshold 16 (right part first, then the loop
// continues on the left part), __partial_sort = heap sort at depth 0, then
// __final_insertion_sort.  The recursion runs on an explicit stack.
// stk: 48 ints of scratch for the explicit stack (depth <= 2 lg n <= 16 pushes).
template <class V>
HMC_HD void sort_greater(const V &v, int n, int *stk) {
  if (n <= 16) {
    insertion_sort(v, 0, n);
    return;
  }
  int *sf = stk, *sl = stk + 16, *sd = stk + 32, top = 0;
  sf[0] = 0;
  sl[0] = n;
  sd[0] = lg2_floor(n) * 2;
  top = 1;
  while (top > 0) {
    --top;
    int first = sf[top], last = sl[top], depth = sd[top];
    while (last - first > 16) {
      if (depth == 0) {  // std::__partial_sort(first, last, last): heap select + sort_heap
        make_heap(v, first, last);
        for (int e = last; e - first > 1;) {  // std::__sort_heap / __pop_heap (stl_heap.h:253-266, 423-432)
          --e;
          const double x = v.l(e);
          const uint32_t y = v.m(e);
          v.copy(e, first);
          adjust_heap(v, first, 0, e - first, x, y);
        }
        break;
      }
      --depth;
      const int cut = unguarded_partition_pivot(v, first, last);
      sf[top] = first;  // the loop's continuation on [first, cut) after the recursive call
      sl[top] = cut;
      sd[top] = depth;
      ++top;
      first = cut;  // std::__introsort_loop(cut, last, depth)
    }
  }
  insertion_sort(v, 0, 16);  // std::__final_insertion_sort
  unguarded_insertion_sort(v, 16, n);
}
template <class V>
HMC_HD void sort_greater(const V &v, int n) {
  int stk[48];
  sort_greater(v, n, stk);
}

}  // namespace hmc
