// plan.hpp — the E-step's store planning as pure host functions (no HIP):
// which individuals form the next structure-pass group and where each one's
// record region lies (Ctx::estep_split), and which of them form a value-pass
// sub-group whose traces fit the trace store.  Kept free of device state so
// that host unit tests (tests/test_sanitize.py, under ASan / UBSan) can check
// the arithmetic.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

namespace hmc {

struct RegionPlanIn {
  bool have_est = false;  // estimates exist (a pass measured some individuals, or the previous E-step)
  bool light = false;     // the model is smaller than the panel: every individual gets an even share
  int dev_cu = 256;
  int L = 1;
  uint64_t rec_budget = 0;  // words
  uint64_t trace_budget = 0;
  uint64_t rec_alloc = 0;   // words of the record store as allocated now
};

// Record regions of the next structure pass over `pending` (heaviest first).
// Before any estimate: the first min(np, 4 CUs) individuals spread over the
// cost order (every np/k-th, moved to the front of `pending`) — or all of them
// on a light model — each get an even share, at most 8 192 words per locus or
// the allocated store's share.  With estimates: the prefix whose regions (and
// measured traces) fit the budgets; the store left over goes to the estimated
// regions (up to 3x, within the allocation or 1.25x the estimates).  Returns
// the number of individuals k planned (pending[0, k)); base / rsz of those
// individuals are set (indexed by individual), *words = the region total.
inline int plan_record_regions(const RegionPlanIn &in, std::vector<int32_t> &pending, const std::vector<char> &exact_need,
                               const std::vector<unsigned long long> &rneed, const std::vector<unsigned long long> &tneed,
                               const std::vector<unsigned long long> &est, std::vector<unsigned long long> &base,
                               std::vector<unsigned long long> &rsz, uint64_t *words) {
  const int np = (int)pending.size();
  uint64_t r = 0, t = 0;
  int k = 0;
  if (!in.have_est) {
    k = in.light ? np : std::min(np, 4 * in.dev_cu);
    if (np > k) {  // every np/k-th of the heaviest-first list
      std::vector<int32_t> pick, other;
      pick.reserve(k);
      other.reserve(np - k);
      for (int q = 0; q < np; ++q)
        ((int64_t)q * k / np != (int64_t)(q - 1) * k / np || q == 0 ? pick : other).push_back(pending[q]);
      pending = pick;
      pending.insert(pending.end(), other.begin(), other.end());
      k = (int)pick.size();
    }
    if (k == 0) {
      *words = 0;
      return 0;
    }
    const uint64_t cap = std::max<uint64_t>(in.rec_alloc / (uint64_t)k, std::max<uint64_t>(1ull << 22, 8192ull * (uint64_t)in.L));
    const uint64_t share = std::min<uint64_t>(in.rec_budget / (uint64_t)k, cap);
    for (int q = 0; q < k; ++q) {
      base[pending[q]] = (uint64_t)q * share;
      rsz[pending[q]] = share;
    }
    *words = share * (uint64_t)k;
    return k;
  }
  uint64_t r_est = 0;
  while (k < np) {
    const int bi = pending[k];
    const uint64_t need = exact_need[bi] ? rneed[bi] : std::min<uint64_t>(est[bi], in.rec_budget);
    // (estimated traces are not counted: groups cut by records and then split
    // by exact traces measured faster at cfg 3's E1)
    const uint64_t tn = exact_need[bi] ? tneed[bi] : 0;
    if (k > 0 && (r + need > in.rec_budget || t + tn > in.trace_budget)) break;
    rsz[bi] = need;
    r += need;
    t += tn;
    r_est += exact_need[bi] ? 0 : need;
    ++k;
  }
  const uint64_t room = std::min<uint64_t>(in.rec_budget, std::max<uint64_t>(in.rec_alloc, r + r / 4));
  const double grow = r_est > 0 && r < room ? std::min(3.0, 1.0 + (double)(room - r) / (double)r_est) : 1.0;
  r = 0;
  for (int q = 0; q < k; ++q) {
    const int bi = pending[q];
    if (!exact_need[bi]) rsz[bi] = std::min<uint64_t>((uint64_t)((double)rsz[bi] * grow), in.rec_budget);
    if (r + rsz[bi] > in.rec_budget) rsz[bi] = in.rec_budget - r;
    base[bi] = r;
    r += rsz[bi];
  }
  *words = r;
  return k;
}

// The value-pass sub-group starting at ids[pos]: the longest run whose exact
// trace words fit `budget` (at least one individual); trace bases are set.
inline size_t plan_trace_group(const std::vector<int32_t> &ids, size_t pos, const std::vector<unsigned long long> &tneed,
                               uint64_t budget, std::vector<unsigned long long> &base, uint64_t *words) {
  uint64_t t = 0;
  size_t k = 0;
  while (pos + k < ids.size() && (k == 0 || t + tneed[ids[pos + k]] <= budget)) {
    base[ids[pos + k]] = t;
    t += tneed[ids[pos + k]];
    ++k;
  }
  *words = t;
  return k;
}

}  // namespace hmc
