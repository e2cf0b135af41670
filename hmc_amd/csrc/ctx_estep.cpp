// ctx_estep.cpp — Ctx members: the E-step: HaploModel::resolveAll through the structure and value passes.
#include "ctx.hpp"
#include "plan.hpp"

namespace hmc {

int Ctx::build_head_frontier() {
  const int n = nloc(), hl = head_len;
  const int nh = (int)h_head_ids.size();
  if (nh == 0 && !h_head_al.empty()) return fail(HMC_EARG, "head alleles without heads");
  // the start-0 length-hl pattern matching `as` (MISSING = wildcard): the
  // trie walk of PatternTree.cpp:98-134 goes from locus hl-1 down and keeps
  // the first full-length hit, i.e. the smallest allele index at the
  // highest missing locus first
  auto lookup = [&](const std::vector<uint8_t> &as) -> uint32_t {
    int best = -1;
    for (int h = 0; h < nh; ++h) {
      const uint8_t *al = h_head_al.data() + (size_t)h * hl;
      bool ok = true;
      for (int k = 0; k < hl && ok; ++k) ok = as[k] == MISSING || as[k] == al[k];
      if (!ok) continue;
      if (best < 0) { best = h; continue; }
      const uint8_t *bl = h_head_al.data() + (size_t)best * hl;
      for (int k = hl - 1; k >= 0; --k)
        if (al[k] != bl[k]) {
          if (al[k] < bl[k]) best = h;
          break;
        }
    }
    return best < 0 ? NONE : h_head_ids[best];
  };
  std::vector<uint32_t> off(n + 1, 0), pairs;
  std::vector<int32_t> status(n, EST_OK);
  for (int i = 0; i < n; ++i) {
    off[i] = (uint32_t)(pairs.size() / 2);
    const uint8_t *g0 = pan.idx.data() + ((size_t)(i0 + i) * 2) * pan.L, *g1 = g0 + pan.L;
    for (int h = 0; h < nh && status[i] == EST_OK; ++h) {
      const uint8_t *H = h_head_al.data() + (size_t)h * hl;
      bool match = true;  // HaploPattern::isMatch(genotype): every locus matches one allele
      for (int j = 0; j < hl && match; ++j)
        match = g0[j] == MISSING || g1[j] == MISSING || g0[j] == H[j] || g1[j] == H[j];
      if (!match) continue;
      std::vector<std::vector<uint8_t>> last(1), next;
      for (int j = 0; j < hl; ++j) {
        next.clear();
        const bool miss0 = g0[j] == MISSING, miss1 = g1[j] == MISSING;
        const bool isMissing = miss0 && miss1, hasMissing = miss0 || miss1;
        const bool hasAllele = g0[j] == H[j] || g1[j] == H[j];  // Allele == (missing == missing)
        const bool het = !(hasMissing || g0[j] == g1[j]);
        if (isMissing || (hasMissing && hasAllele)) {
          for (auto &as : last)
            for (int k = 0; k < (int)pan.sym[j].size(); ++k)
              if (pan.sym[j][k].second > 0) {
                next.push_back(as);
                next.back().push_back((uint8_t)k);
              }
        } else if (het) {
          for (auto &as : last) {
            next.push_back(as);
            next.back().push_back(H[j] == g0[j] ? g1[j] : g0[j]);
          }
        } else {
          for (auto &as : last) {
            next.push_back(as);
            next.back().push_back(g0[j]);
          }
        }
        last.swap(next);
      }
      for (auto &as : last) {
        const uint32_t q = lookup(as);
        if (q == NONE) { status[i] = EST_NO_HEAD_PATTERN; break; }
        if (q >= h_head_ids[h]) {
          pairs.push_back(h_head_ids[h]);
          pairs.push_back(q);
        }
      }
    }
  }
  off[n] = (uint32_t)(pairs.size() / 2);
  hipError_t e;
  if ((e = d_hf_off.ensure(n + 1)) || (e = d_hf_pairs.ensure(std::max<size_t>(pairs.size(), 2))) ||
      (e = d_hf_status.ensure(std::max(n, 1))) ||
      (e = hipMemcpyAsync(d_hf_off.p, off.data(), (size_t)(n + 1) * 4, hipMemcpyHostToDevice, st)) ||
      (!pairs.empty() && (e = hipMemcpyAsync(d_hf_pairs.p, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice, st))) ||
      (n && (e = hipMemcpyAsync(d_hf_status.p, status.data(), (size_t)n * 4, hipMemcpyHostToDevice, st))) ||
      (e = sync_st()))
    return hipfail(e, "head frontier");
  hf_valid = true;
  return HMC_OK;
}

int Ctx::estep(double *ll_out, int *H_out, uint64_t *re_out) {
  if (!have_model) return fail(HMC_EARG, "no pattern model");
  auto hp_t0 = std::chrono::steady_clock::now();
  if (head_len > 1) {
    if (h_head_al.size() != h_head_ids.size() * (size_t)head_len || (h_head_ids.empty() && n_head > 0))
      return fail(HMC_EUNSUPPORTED, "head_len > 1 needs the head patterns' alleles (mined tables only)");
    int rc = build_head_frontier();
    if (rc) return rc;
  }
  const int L = pan.L, S = this->S(), n = nloc();
  if (S > S_MAX) return fail(HMC_EUNSUPPORTED, "sample_size > %d", S_MAX);
  if (S > 32 && estep_mode != ESTEP_SPLIT)
    return fail(HMC_EUNSUPPORTED, "sample_size > 32 needs the split E-step (hmc_set_estep_mode 0)");
  hipError_t e;
  if ((e = d_total.ensure(n)) || (e = d_ncand.ensure(n)) || (e = d_status.ensure(n)) || (e = d_re.ensure(n)) ||
      (e = d_sbase.ensure(n)) || (e = d_prior.ensure((size_t)n * S_MAX)) || (e = d_post.ensure((size_t)n * S_MAX)) ||
      (e = d_weight.ensure((size_t)n * S_MAX)) || (e = d_cstate.ensure((size_t)n * S_MAX)) ||
      (e = d_cidx.ensure((size_t)n * S_MAX)) || (e = d_rows.ensure((size_t)2 * S * n * L)) ||
      (e = d_wslot.ensure((size_t)2 * S * n)) || (e = d_trace_cursor.ensure(1)) || (e = d_maxst.ensure(1)) ||
      (e = d_fmax.ensure(n)) || (e = d_loc_off.ensure((size_t)n * (L + 1))) || (e = d_order.ensure(n)) ||
      (e = d_order2.ensure(n)) || (e = d_cost.ensure(n)) || (e = d_tbase.ensure(n)) || (e = d_rbase.ensure(n)) ||
      (e = d_rneed.ensure(n)) || (e = d_tneed.ensure(n)) || (e = d_recsz.ensure(n)))
    return hipfail(e, "estep alloc");
  // store budgets: trace store and record store grow (never shrink) up to these
  size_t freeb = 0, totb = 0;
  hipMemGetInfo(&freeb, &totb);
  const double avail = (double)freeb + (double)d_trace.n * 4 + (double)d_rec.n * 4;
  // Frontier capacity of the structure pass: a frontier past it restarts the
  // E-step with twice the capacity (cfg 3's E1 on the M0 model needs 2^14:
  // three restarts from 2^11, ~0.6 s).  With HBM to spare, start there: the
  // pass's per-block scratch is ~190 B per state (3 GB per 1 000 blocks).
  if (!fcap_user_set && fcap < FCAP_BIG && avail > 96e9) fcap = FCAP_BIG;
  // (cfg 3's E1 with the M0 model needs ~2x HBM in records + traces; larger
  // stores (fewer groups) measured no faster and crowd out the next M0.  The
  // trace cap keeps cfg 3's E2.. (~90 GB of traces) in one value pass.)
  // (round 4, compact value frontier: 130 / 88 GiB gives cfg 3's E1 five
  // groups instead of five or six, E1 3.47 -> 3.36 s; 145 / 98 and 110 / 74
  // measured slower, profiles/r04/shapes/store_ab_cfg3.log)
  trace_budget = std::max<uint64_t>(trace_bytes ? trace_bytes : std::min<uint64_t>((uint64_t)(avail * 0.46), 130ull << 30),
                                    1ull << 16) / 4;
  rec_budget = std::max<uint64_t>(rec_bytes ? rec_bytes : trace_bytes ? trace_bytes
                                  : std::min<uint64_t>((uint64_t)(avail * 0.31), 88ull << 30),
                                  1ull << 16) / 4;
  if (debug_mem)
    fprintf(stderr, "[hmc] E-step: free %.1f GB, stores %.1f + %.1f GB, budgets trace %.1f rec %.1f GB\n",
            freeb / 1e9, d_trace.n * 4 / 1e9, d_rec.n * 4 / 1e9, trace_budget * 4 / 1e9, rec_budget * 4 / 1e9);
  // Stores sized by an earlier E-step when more HBM was free (E1, before an
  // exact M-step's tables) shrink to this E-step's budgets: the pass
  // scratch is allocated from what they leave free.  (Past the budget by more
  // than 1/8 only: the budgets move by a few GB with the M-step's buffers,
  // and re-mapping a store of ~100 GB costs seconds.)
  {
    HpTimer hpt(hp_ms[HP_STORES]);
    if (d_trace.n > trace_budget + trace_budget / 8) d_trace.release();
    if (d_rec.n > rec_budget + rec_budget / 8) d_rec.release();
  }
  // A store up to 10 % below its new budget stays as it is and becomes the
  // budget: growing it re-maps the whole store (cfg 4's per-rank E2: 79.3 ->
  // 80.0 GB of traces cost 2.2 s of a 5.5 s iteration, profiles/r06/cfg4/),
  // while a few GB less only moves the group cut.
  if (d_trace.p && d_trace.n < trace_budget && d_trace.n * 10 >= trace_budget * 9) trace_budget = d_trace.n;
  if (d_rec.p && d_rec.n < rec_budget && d_rec.n * 10 >= rec_budget * 9) rec_budget = d_rec.n;
  h_total.assign(n, 0.0);
  h_ncand.assign(n, 0);
  h_status.assign(n, 0);
  h_re.assign(n, 0);
  h_sbase.assign(n, 0);
  for (int i = 0; i < n; ++i) h_sbase[i] = 2 * S * i;  // sample slots of individual i
  if ((e = hipMemcpyAsync(d_sbase.p, h_sbase.data(), (size_t)n * 4, hipMemcpyHostToDevice, st)) ||
      (e = hipMemsetAsync(d_maxst.p, 0, 4, st)) || (e = hipMemsetAsync(d_ncand.p, 0, (size_t)n * 4, st)))
    return hipfail(e, "estep");
  if ((e = d_stamps.ensure(40)) || (e = hipMemsetAsync(d_stamps.p, 0, 40 * 8, st))) return hipfail(e, "stamps");
  // heaviest individuals first (cost of the previous E-step; before the
  // first one, the number of heterozygous or missing loci)
  if ((int)h_cost.size() != n) {
    h_cost.assign(n, 0);
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < L; ++k) {
        const uint8_t x = pan.idx[((size_t)(i0 + i) * 2) * L + k], y = pan.idx[((size_t)(i0 + i) * 2 + 1) * L + k];
        h_cost[i] += (x != y || x == MISSING) ? 1 : 0;
      }
  }
  std::vector<int32_t> order(n);
  for (int q = 0; q < n; ++q) order[q] = q;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return h_cost[x] > h_cost[y]; });
  hp_ms[HP_SETUP] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - hp_t0).count();
  if ((e = hipMemcpyAsync(d_cost.p, h_cost.data(), (size_t)n * 4, hipMemcpyHostToDevice, st)))
    return hipfail(e, "estep");
  ms_fwd = ms_tb = 0;
  ms_s1 = ms_s2 = ms_fb = ms_order = ms_ck = 0;
  last_windows = last_window_loci = last_window_groups = 0;
  n_fallback = n_order_redo = 0;
  n_struct_passes = n_value_passes = 0;
  int rc = 0;
  n_restarts = 0;
  while (true) {  // a frontier overflow (fcap grows) restarts the E-step
    rc = estep_mode == ESTEP_SPLIT ? estep_split(order) : estep_fused(order);
    if (rc != ESTEP_RESTART) break;
    ++n_restarts;
  }
  if (rc) return rc;
  if (estep_mode == ESTEP_SPLIT) ms_fwd = ms_s1 + ms_s2 + ms_fb;
  if (last_fast && value_mode == VM_AUTO && (double)n_order_redo > 0.35 * (double)n) fast_off = true;
  // samples in the reference's order: individuals in order, candidates in
  // order, h0 then h1 (HaploModel.cpp:105-106)
  HpTimer hpt_samples(hp_ms[HP_SAMPLES]);
  std::vector<int32_t> rowmap;
  rowmap.reserve((size_t)2 * S * n);
  for (int i = 0; i < n; ++i)
    for (int c = 0; c < 2 * h_ncand[i]; ++c) rowmap.push_back(h_sbase[i] + c);
  H = (int)rowmap.size();
  std::vector<double> wslot((size_t)2 * S * n), w(H);
  if ((e = d_samp_lm.ensure((size_t)std::max(H, 1) * L)) || (e = d_rowmap.ensure(std::max(H, 1))) ||
      (e = d_w.ensure(std::max(H, 1))))
    return hipfail(e, "samples");
  if ((H && (e = hipMemcpyAsync(d_rowmap.p, rowmap.data(), (size_t)H * 4, hipMemcpyHostToDevice, st))) ||
      (e = launch_transpose_rows_u8(d_rows.p, d_rowmap.p, d_samp_lm.p, H, L, st)) ||
      (e = hipMemcpyAsync(wslot.data(), d_wslot.p, wslot.size() * 8, hipMemcpyDeviceToHost, st)) ||
      (e = hipMemcpyAsync(h_total.data(), d_total.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
      (e = hipMemcpyAsync(h_re.data(), d_re.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
      (e = hipMemcpyAsync(h_cost.data(), d_cost.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
      (e = sync_st()))
    return hipfail(e, "estep");
  for (int h = 0; h < H; ++h) w[h] = wslot[rowmap[h]];
  if (H && ((e = hipMemcpyAsync(d_w.p, w.data(), (size_t)H * 8, hipMemcpyHostToDevice, st)) ||
            (e = sync_st())))
    return hipfail(e, "estep");
  h_rowmap.swap(rowmap);
  // ll += log(genotype probability) in individual order (HaploModel.cpp:110);
  // HaploData::checkTotalWeight (HaploData.cpp:120-126) in sample order
  double red[2] = {0.0, 0.0};
  auto local_sums = [&](double *acc) {
    double ll = acc[0], tw = acc[1];
    for (int i = 0; i < n; ++i) ll += log(h_total[i]);
    for (int h = 0; h < H; ++h) tw += w[h];
    acc[0] = ll;
    acc[1] = tw;
  };
  if (multi() && reduction == RED_ORDERED) {  // the chain continues rank by rank
    if ((rc = ordered_chain_host(red, 2, local_sums))) return rc;
  } else {
    local_sums(red);
    if ((rc = allreduce_host(red, 2))) return rc;
  }
  const double ll = red[0];
  total_weight = red[1];
  uint64_t re = 0;
  for (int i = 0; i < n; ++i) re += h_re[i];
  have_samples = true;
  have_estep = true;
  if (ll_out) *ll_out = ll;
  if (H_out) *H_out = H;
  if (re_out) *re_out = re;
  return HMC_OK;
}

int Ctx::ensure_store(DevBuf<uint32_t> &b, uint64_t words, uint64_t budget, const char *what) {
  if (b.n >= words && b.p) return HMC_OK;
  HpTimer hpt(hp_ms[HP_STORES]);
  if (words > budget) return fail(HMC_ENOMEM, "%s: one individual needs %llu words (budget %llu)", what,
                                  (unsigned long long)words, (unsigned long long)budget);
  b.release();  // 1.25x headroom: a store of tens of GB is mapped eagerly, re-allocations are slow
  const uint64_t want = std::min<uint64_t>(budget, words + words / 4);
  hipError_t e = b.ensure(want);
  if (e == hipErrorOutOfMemory && want > words) {  // the device is shared: no headroom
    (void)hipGetLastError();
    e = b.ensure(words);
  }
  if (e) return hipfail(e, what);
  return HMC_OK;
}

EstepArgs Ctx::estep_args(int S) {
  EstepArgs a;
  a.pan = dev_panel();
  a.mod = dev_model();
  a.S = S;
  a.indiv_begin = i0;
  a.indiv_end = i1;
  a.scratch = d_scratch.p;
  a.fcap = fcap;
  a.hcap = next_pow2(2 * fcap);
  a.scratch_stride = estep_scratch_bytes(fcap, a.hcap, S, estep_nw);
  lds_tier(S, a.lds_fc, a.lds_hc);
  a.trace = d_trace.p;
  a.trace_cap = d_trace.n;
  a.trace_cursor = d_trace_cursor.p;
  a.trace_base = nullptr;
  a.loc_off = d_loc_off.p;
  a.total = d_total.p;
  a.ncand = d_ncand.p;
  a.status = d_status.p;
  a.cand_state = d_cstate.p;
  a.cand_idx = d_cidx.p;
  a.prior = d_prior.p;
  a.posterior = d_post.p;
  a.weight = d_weight.p;
  a.re_count = d_re.p;
  a.max_states = d_maxst.p;
  a.fmax = d_fmax.p;
  a.order = nullptr;
  a.n_order = 0;
  a.cost = d_cost.p;
  a.stamps = d_stamps.p;
  a.diag_indiv = -1;  // diagnostic build: stamps of every individual
  return a;
}

int Ctx::traceback_group(int k) {
  TracebackArgs t;
  t.L = pan.L;
  t.S = S();
  t.head_len = head_len;
  t.nbatch = k;
  t.order = d_order2.p;
  t.indiv_begin = i0;
  t.mod = dev_model();
  t.trace = d_trace.p;
  t.loc_off = d_loc_off.p;
  t.ncand = d_ncand.p;
  t.cand_state = d_cstate.p;
  t.cand_idx = d_cidx.p;
  t.weight = d_weight.p;
  t.sample_base = d_sbase.p;
  t.rows = d_rows.p;
  t.w_out = d_wslot.p;
  hipError_t e;
  hipEventRecord(ev[2], st);
  if ((e = launch_traceback(t, 0, st))) return hipfail(e, "traceback");
  hipEventRecord(ev[3], st);
  if ((e = sync_st())) return hipfail(e, "traceback");
  float ms = 0;
  hipEventElapsedTime(&ms, ev[2], ev[3]);
  ms_tb += ms;
  return HMC_OK;
}

int Ctx::estep_fused(const std::vector<int32_t> &order) {
  const int S = this->S(), n = nloc();
  int dev_cu = 256;
  hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, device);
  const int G = std::max(1, std::min(waves > 0 ? waves : dev_cu * std::max(8, lds_waves_per_cu), n));
  hipError_t e;
  size_t pos = 0;
  int batch = n;
  if (d_trace.n == 0) {
    int rc = ensure_store(d_trace, std::min<uint64_t>(trace_budget, std::max<uint64_t>((uint64_t)n * pan.L * (1 + S) * 96, 16ull << 20)),
                          trace_budget, "trace store");
    if (rc) return rc;
  }
  while (pos < order.size()) {
    const int k = (int)std::min<size_t>(batch, order.size() - pos);
    EstepArgs a = estep_args(S);
    const int grid = std::min(G, k);
    if ((e = d_scratch.ensure(a.scratch_stride * grid))) return hipfail(e, "estep scratch");
    a.scratch = d_scratch.p;
    int rc = upload_order(d_order2, order.data() + pos, k);
    if (rc) return rc;
    a.order = d_order2.p;
    a.n_order = k;
    if ((e = hipMemsetAsync(d_trace_cursor.p, 0, 8, st))) return hipfail(e, "estep");
    hipEventRecord(ev[0], st);
    if ((e = launch_estep(a, grid, estep_nw, st))) return hipfail(e, "estep_forward launch");
    hipEventRecord(ev[1], st);
    if ((rc = read_status(order, k, true))) return rc;
    float ms = 0;
    hipEventElapsedTime(&ms, ev[0], ev[1]);
    ms_fwd += ms;
    bool ovf_trace = false;
    for (int q = 0; q < k; ++q) {
      const int s = h_status[order[pos + q]];
      if (s == EST_NO_HEAD_PATTERN) return fail(HMC_ENOPATTERN, "Can not find matching pattern!");
      if (s == EST_OVERFLOW_FRONTIER) {
        if (fcap >= F_MAX) return fail(HMC_EUNSUPPORTED, "frontier exceeds %d states", F_MAX);
        fcap = (int)std::min<int64_t>(F_MAX, (int64_t)fcap * 4);  // x4: each overflow costs a whole pass
        return ESTEP_RESTART;
      }
      if (s == EST_OVERFLOW_TRACE) ovf_trace = true;
    }
    if (ovf_trace) {
      if (d_trace.n < trace_budget) {  // grow the store before splitting the group
        if ((rc = ensure_store(d_trace, std::min<uint64_t>(trace_budget, d_trace.n * 4), trace_budget, "trace store")))
          return rc;
        continue;
      }
      if (k == 1) return fail(HMC_ENOMEM, "trace store too small for one individual");
      batch = std::max(1, k / 2);
      continue;
    }
    if ((rc = traceback_group(k))) return rc;
    pos += k;
  }
  return HMC_OK;
}

int Ctx::estep_split(const std::vector<int32_t> &order, bool exact) {
  const int S = this->S(), n = nloc(), L = pan.L;
  {
    const int rc0 = ensure_gmodel();
    if (rc0) return rc0;
  }
  int32_t *dstatus = exact ? d_xstatus.p : d_status.p;
  // value-only lists first (hmc_set_value_mode; lists longer than a wavefront:
  // exact order only)
  const bool light_model = (double)P <= (double)pan.N * (double)pan.L;
  const bool vfast = !exact && S <= 32 &&
                     (value_mode == VM_FAST || (value_mode == VM_AUTO && pan.amax > 2 && light_model && !fast_off));
  if (!exact) last_fast = vfast;
  int dev_cu = 256;
  hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, device);
  const int G = std::max(1, std::min(waves > 0 ? waves : dev_cu * std::max(8, lds_waves_per_cu), n));
  hipError_t e;
  float ms = 0;
  // Loci in windows with checkpoints (ctx_window.cpp) when the first E-step
  // on a model larger than the panel would otherwise run in groups too small
  // to fill the GPU (cfg 4's per-rank E1) or in three or more groups (cfg 3's
  // E1); a probe of the first loci decides.
  if (!exact && windows_allowed() &&
      (window_mode == WIN_ALWAYS || ((double)P > (double)pan.N * (double)pan.L && n > 2 * dev_cu))) {
    const int rw_ = estep_windowed(order);
    if (rw_ != WIN_DECLINED) return rw_;
  }
  std::vector<int32_t> pending(order), sset, rest;
  std::vector<unsigned long long> rneed(n, 0), tneed(n, 0), base(n, 0), rsz(n, 0);
  std::vector<int32_t> fbig(n, 0);  // largest frontier of each individual (structure pass)
  // Every individual gets its own record region: its exact size once a pass
  // has measured it (`exact_need`), else an estimate — the previous E-step's
  // size when the model is of the same scale, or the records-per-cost ratio
  // of the individuals measured so far.  A region that turns out too small
  // only defers that individual (it keeps walking without writing and
  // reports its exact size), so no pass is ever repeated in full.
  std::vector<char> exact_need(n, 0);
  std::vector<unsigned long long> est(n, 0);
  const bool prev_ok = !exact && (int)prev_rneed.size() == n && prev_P > 0 && P < 2 * (int64_t)prev_P &&
                       2 * (int64_t)P > prev_P;
  if (prev_ok)
    for (int i = 0; i < n; ++i) est[i] = prev_rneed[i] + prev_rneed[i] / 10 + 64;
  bool have_est = prev_ok;
  int rc;
  while (!pending.empty()) {
    // ---- pass 1: structure records --------------------------------------
    int np = (int)pending.size();
    {
      // (the first pass spans the whole cost range and later estimates use the
      // measured individuals nearest in cost (cfg 3 E1 after E5: 7.1 -> 5.9 s,
      // deferred 1 713 -> 12 per group, profiles/r02/e1_groups/); a model
      // smaller than the panel — cfg 3's E2 after the M0-based E1 — gives every
      // individual a share: its records fit, and the E-step runs in one group;
      // the first pass caps a share at 8 192 words per locus or the store
      // already allocated: mapping the whole budget, tens of GB, costs seconds
      // per E-step on a fresh context; a region too small only defers its
      // individual; the store left over goes to the estimated regions (A/B on
      // one box, cfg 3: E1 value passes 3.88 -> 3.60 s, E2 structure 218 -> 177 ms))
      RegionPlanIn pin;
      pin.have_est = have_est;
      pin.light = exact ? false : (double)P <= (double)pan.N * (double)pan.L;
      pin.dev_cu = dev_cu;
      pin.L = L;
      pin.rec_budget = rec_budget;
      pin.trace_budget = trace_budget;
      pin.rec_alloc = d_rec.n;
      uint64_t r = 0;
      const int k = plan_record_regions(pin, pending, exact_need, rneed, tneed, est, base, rsz, &r);
      np = k;
      rec_words = r;
      std::vector<unsigned long long> rb(n, 0), rs(n, 0);
      for (int q = 0; q < np; ++q) {
        rb[pending[q]] = base[pending[q]];
        rs[pending[q]] = rsz[pending[q]];
      }
      if ((e = hipMemcpyAsync(d_rbase.p, rb.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)) ||
          (e = hipMemcpyAsync(d_recsz.p, rs.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)))
        return hipfail(e, "estep");
    }
    const int hcap1 = next_pow2(2 * fcap);
    // (exact records pack a locus's contribution count in 22 bits, R[3] = C << 10 | npairs)
    const int ccap1 = (int)std::min<int64_t>(exact ? EXACT_C_MAX : INT32_MAX / 2, (int64_t)ccap_mult * fcap);
    // Structure pass over ids[0, np_) in the record regions set above (d_rbase /
    // d_recsz).  prune_: with extend()'s forward test (HaploBuilder.cpp:237),
    // for the individuals the value pass found underflowing.
    auto structure_pass = [&](const int32_t *ids, int np_, bool prune_) -> int {
      int rc;
      hipError_t e;
      float ms = 0;
      // structure pass: one wave per individual; 12 per CU (3 per SIMD at 145
      // VGPRs) above 8 per CU, so cfg 3's E1 groups of 2 200-2 700 run in one
      // round (profiles/r02/e1_groups/: 603-658 -> 484-586 ms per group).  On a
      // model larger than the panel (the genotype-mined M0: 2.5 patterns per
      // individual-locus at cfg 3, 0.3 later) frontiers are large (cfg 3 E1:
      // 470 states per locus, 80 % of them past a one-wave block's LDS tier):
      // four waves per individual, two per CU (each block's LDS tier holds
      // more of the frontier: cfg 3 E1 structure 1.65 -> 1.32 s against three
      // per CU, profiles/r03/e1/e1_s1shapes.log)
      const bool heavy_model = (double)P > (double)pan.N * (double)pan.L;
      // (a heavy group of at most one individual per CU — cfg 4's per-rank E1,
      // records of ~250 MB per individual — takes the whole CU: 16 waves)
      const int nw1 = s1_nw > 0 ? s1_nw : (heavy_model ? (np_ <= dev_cu ? 16 : 4) : 1);
      const int bpc1 = s1_ipc > 0 ? s1_ipc
                                  : (nw1 == 16 ? 1 : (nw1 == 4 ? 2 : (np_ > 8 * dev_cu ? 12 : (np_ > 4 * dev_cu ? 8 : 4))));
      const bool v2 = structure_pass_version == 2;
      const size_t per1 = estep_s1_scratch_bytes(fcap, hcap1, ccap1, v2 ? 2 : nw1, prune_);
      // (huge frontiers: fewer resident individuals rather than scratch past SCRATCH_MAX)
      const int grid1 = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::min(np_, dev_cu * bpc1), SCRATCH_MAX / per1));
      // the scratch first: both stores are dead here (the groups before have
      // been traced back), so they give way to it when HBM is short
      // (a prune re-run runs between a value pass and its traceback: both stores are live)
      if ((e = scratch_ensure(d_scr1, per1 * grid1, !prune_, !prune_)) || (e = d_rec_off.ensure((size_t)n * (L + 1))) ||
          (e = d_rec_cursor.ensure(1)) || (e = hipMemsetAsync(d_rec_cursor.p, 0, 8, st)))
        return hipfail(e, "estep pass-1 alloc");
      if ((rc = ensure_store(d_rec, rec_words, rec_budget, "record store"))) return rc;
      if ((rc = upload_order(d_order, ids, np_))) return rc;
      StructArgs s1;
      s1.pan = dev_panel();
      s1.mod = dev_model();
      s1.S = S;
      s1.indiv_begin = i0;
      s1.order = d_order.p;
      s1.n_order = np_;
      s1.scratch = d_scr1.p;
      s1.scratch_stride = per1;
      s1.fcap = fcap;
      s1.hcap = hcap1;
      s1.ccap = ccap1;
      s1_tier(160 * 1024 / bpc1 - 256, pan.amax, nw1, s1.lds_fc, s1.lds_hc, s1.lds_cc, v2);
    s1.probe_lds = key_probes;
      s1.rec = d_rec.p;
      s1.rec_cap = d_rec.n;
      s1.rec_cursor = d_rec_cursor.p;
      s1.rec_base = d_rbase.p;
      s1.rec_size = d_recsz.p;
      s1.rec_off = d_rec_off.p;
      s1.rec_need = d_rneed.p;
      s1.trace_need = d_tneed.p;
      s1.status = dstatus;
      s1.re_count = exact ? d_xre.p : d_re.p;
      s1.fmax = exact ? d_xfmax.p : d_fmax.p;
      s1.max_states = d_maxst.p;
      s1.stamps = d_stamps.p + 20;
      s1.exact = exact;
      s1.prune = prune_;
      if ((e = d_nextq.ensure(2)) || (e = hipMemsetAsync(d_nextq.p, 0, 8, st))) return hipfail(e, "estep");
      s1.next_q = d_nextq.p;
      if (debug_mem)
        fprintf(stderr, "[hmc] structure pass v%d: %d individuals, %d waves x %d per CU, grid %d, LDS tier %d states%s\n",
                v2 ? 2 : 1, np_, nw1, bpc1, grid1, s1.lds_fc, prune_ ? " (prune)" : "");
      hipEventRecord(ev[0], st);
      if ((e = v2 ? launch_estep_structure2(s1, grid1, nw1, st) : launch_estep_structure(s1, grid1, nw1, st)))
        return hipfail(e, "estep_structure launch");
      hipEventRecord(ev[1], st);
      if ((e = hipMemcpyAsync(rneed.data(), d_rneed.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
          (e = hipMemcpyAsync(tneed.data(), d_tneed.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
          (e = hipMemcpyAsync(fbig.data(), s1.fmax, (size_t)n * 4, hipMemcpyDeviceToHost, st)))
        return hipfail(e, "estep_structure");
      if ((rc = read_status(pending, np_, false, dstatus))) return rc;
      if (check_records && (rc = validate_records(ids, np_, i0))) return rc;
      hipEventElapsedTime(&ms, ev[0], ev[1]);
      if (prune_) {
        ms_fb += ms;
      } else {
        ms_s1 += ms;
        ++n_struct_passes;
      }
      return HMC_OK;
    };
    if ((rc = structure_pass(pending.data(), np, false))) return rc;
    if (debug_mem) {
      int ndef = 0;
      uint64_t rsum = 0, rmax = 0, tsum = 0, rres = 0;
      for (int q = 0; q < np; ++q) {
        const int bi = pending[q];
        ndef += h_status[bi] == EST_OVERFLOW_REC ? 1 : 0;
        rsum += rneed[bi];
        rmax = std::max<uint64_t>(rmax, rneed[bi]);
        tsum += tneed[bi];
        rres += rsz[bi];
      }
      fprintf(stderr, "[hmc] structure pass %d: %d individuals, %.1f ms; deferred %d, records need %.2f GB (max %.1f MB, "
              "reserved %.2f GB), traces %.2f GB\n", n_struct_passes, np, ms, ndef, rsum * 4e-9, rmax * 4e-6, rres * 4e-9,
              tsum * 4e-9);
    }
    sset.clear();
    rest.clear();
    for (int q = 0; q < np; ++q) {
      const int bi = pending[q], s = h_status[bi];
      if (s == EST_NO_HEAD_PATTERN) return fail(HMC_ENOPATTERN, "Can not find matching pattern!");
      if (s == EST_OVERFLOW_CONTRIB) {  // missing genotypes: up to amax^2 contributions per state
        if ((int64_t)ccap_mult * fcap >= INT32_MAX / 2) return fail(HMC_EUNSUPPORTED, "too many contributions at a locus");
        if (exact && ccap1 >= EXACT_C_MAX)
          return fail(HMC_EUNSUPPORTED, "exact M-step: more than %d contributions at a locus", EXACT_C_MAX);
        ccap_mult *= 2;
        return ESTEP_RESTART;
      }
      if (s == EST_OVERFLOW_FRONTIER) {  // (deferring only these individuals measured slower)
        if (fcap >= F_MAX) return fail(HMC_EUNSUPPORTED, "frontier exceeds %d states", F_MAX);
        if (debug_mem) fprintf(stderr, "[hmc] frontier over %d states: capacity x4, E-step restarts\n", fcap);
        fcap = (int)std::min<int64_t>(F_MAX, (int64_t)fcap * 4);  // x4: each overflow costs a whole pass
        return ESTEP_RESTART;
      }
      if (s == EST_OVERFLOW_REC) {
        if (exact_need[bi]) return fail(HMC_EHIP, "record store overflow with exact sizes");
        rest.push_back(bi);
      } else {
        sset.push_back(bi);
      }
      exact_need[bi] = 1;
    }
    for (int q = np; q < (int)pending.size(); ++q) rest.push_back(pending[q]);
    // estimates for the individuals not measured yet: records per unit of
    // cost of those measured (after a pass where estimates fell short, or
    // when there were none)
    {
      int deferred = 0;
      double rs_ = 0, cs = 0;
      for (int i = 0; i < n; ++i)
        if (exact_need[i]) {
          rs_ += (double)rneed[i];
          cs += (double)std::max(1, h_cost[i]);
        }
      for (int q = 0; q < np; ++q) deferred += h_status[pending[q]] == EST_OVERFLOW_REC ? 1 : 0;
      if (!have_est || deferred * 10 > np) {
        const double ratio = cs > 0 ? rs_ / cs : 0.0;
        std::vector<std::pair<int, double>> cr;  // (cost, records per cost) of the measured
        for (int i = 0; i < n; ++i)
          if (exact_need[i]) cr.emplace_back(std::max(1, h_cost[i]), (double)rneed[i] / std::max(1, h_cost[i]));
        std::sort(cr.begin(), cr.end());
        for (int bi : rest) {
          if (exact_need[bi]) continue;
          const int c = std::max(1, h_cost[bi]);
          if (cr.empty()) {
            est[bi] = (uint64_t)(1.25 * ratio * c) + 64;
            continue;
          }
          // the largest ratio among the 4 measured nearest in cost on each side
          const int at = (int)(std::lower_bound(cr.begin(), cr.end(), std::make_pair(c, -1.0)) - cr.begin());
          double q = 0.0;
          for (int u = std::max(0, at - 4); u < std::min((int)cr.size(), at + 4); ++u) q = std::max(q, cr[u].second);
          est[bi] = (uint64_t)(1.1 * q * c) + 64;
        }
        have_est = true;
      }
    }
    // ---- pass 2: values, in groups whose traces fit the store -------------
    size_t pos = 0;
    while (pos < sset.size()) {
      uint64_t t = 0;
      size_t k = plan_trace_group(sset, pos, tneed, trace_budget, base, &t);
      // traces over the budget by a few individuals while structure groups
      // still follow: those join the next group (re-walked there, exact sizes
      // known) instead of a value pass of their own, which would cost one
      // heavy individual's whole latency (cfg 3 E1: 61-78 individuals,
      // 230-270 ms each, profiles/r02/e1_groups/)
      if (pos == 0 && !exact && !rest.empty() && k < sset.size() && 4 * (sset.size() - k) <= sset.size()) {
        rest.insert(rest.begin(), sset.begin() + (std::ptrdiff_t)k, sset.end());
        sset.resize(k);
      }
      if ((rc = ensure_store(d_trace, std::max<uint64_t>(t, 1), trace_budget, "trace store"))) return rc;
      // the value pass heaviest first by the records the structure pass just
      // measured (the group's end waits on its slowest individual; the
      // genotype cost order only approximates the work)
      if (!exact)
        std::stable_sort(sset.begin() + (std::ptrdiff_t)pos, sset.begin() + (std::ptrdiff_t)(pos + k),
                         [&](int32_t x, int32_t y) { return rneed[x] > rneed[y]; });
      std::vector<unsigned long long> tb(n, 0);
      for (size_t q = 0; q < k; ++q) tb[sset[pos + q]] = base[sset[pos + q]];
      if ((e = hipMemcpyAsync(d_tbase.p, tb.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)))
        return hipfail(e, "estep");
      if ((rc = upload_order(d_order2, sset.data() + pos, (int)k))) return rc;
      if (exact) {
        // individuals whose forward likelihood underflows: records rebuilt with
        // extend()'s forward test (HaploBuilder.cpp:237, 291-314) before the walk
        auto rerun = [&](std::vector<int32_t> &ids) { return structure_pass(ids.data(), (int)ids.size(), true); };
        if ((rc = exact_group(sset.data() + pos, (int)k, rerun))) return rc;
        pos += k;
        continue;
      }
      // by individuals per CU (cfg 3 and its rank shards, tools/shard_shapes.py,
      // profiles/r02/shard_shapes/): 1:16 from 32 per CU (10 000: 557 vs 615 ms
      // at 2:8), 2:8 from 8 (4 994: 290 vs 333 ms at 1:16), else 3:8 (1 239:
      // 101 vs 112 ms at 2:8)
      // (1:20 runs the 5-waves-per-SIMD build: 505-514 vs 535-558 ms at
      // 1:16 for cfg 3's E3, profiles/r02/values_ab/)
      // Heavy individuals (the first E-step on the genotype-mined model: cfg 3's
      // E1 averages ~3 000 record words per locus against ~650 later) take 4
      // waves each, 4 per CU: more selection segments per individual and a
      // 4x larger LDS frontier tier (cfg 3 E1 value passes 3.84 -> 2.99 s,
      // profiles/r03/e1_shapes/).
      double rw = 0;
      for (size_t q = 0; q < k; ++q) rw += (double)rneed[sset[pos + q]];
      const bool heavy = rw / ((double)k * L) > 1500.0;
      // Heavy groups too small to give every CU four individuals (records and
      // traces of hundreds of MB each: cfg 4's per-rank E1 on the 720 M-pattern
      // M0 runs in groups of ~200) spread the CU's 16 waves over fewer
      // individuals: more selection segments and LDS per individual.
      const int per_cu = (int)((k + dev_cu - 1) / dev_cu);
      const bool small_heavy = heavy && per_cu < 4;
      // (heavy groups filling the GPU: 4 waves x 4 per CU since the compact
      // frontier, cfg 3 E1 values 2 192 -> 2 134 ms against 8 x 2,
      // profiles/r04/shapes/value_shapes_cfg3.log; with the round-3 frontier
      // 8 x 2 had won, 2.95 -> 2.68 s, profiles/r03/e1/e1_wide.log)
      // (five per CU: 4 waves x 5 on the 5-waves-per-SIMD build, one round
      // instead of 1.2 — cfg 3's E1 on rank 0 of 8, 1 239 individuals: values
      // 296 -> 262 ms; 3 x 5 and 2 x 8 383-386 ms; at ten per CU 4 x 4 stays:
      // 481 ms against 583-869, profiles/r05/shards/)
      const bool five_heavy = heavy && per_cu == 5;
      int vnw = vp_nw > 0 ? vp_nw
                          : (small_heavy ? 16 / per_cu
                                         : (heavy ? 4 : ((int)k >= 32 * dev_cu ? 1 : ((int)k >= 8 * dev_cu ? 2 : 3))));
      int vipc = vp_ipc > 0 ? vp_ipc
                            : (small_heavy ? per_cu
                                           : (five_heavy && vnw == 4 ? 5
                                                                     : (vnw == 1 ? 16 : (vnw >= 8 ? 2 : (vnw >= 4 ? 4 : 8)))));  // a half-given shape completes by the same rule
      // (one wave per individual: 16 per CU on the 4-wave build since the
      // swap-count cut, cfg 3 E3 values 507 -> 479 ms, E2 equal; 20 on the
      // 5-wave build before, profiles/r04/shapes/one_wave_16_vs_20_cfg3.log)
      // the HBM tier of the value frontiers holds the group's largest
      // frontier (pass 1 measured it), not the structure pass's capacity
      int fgrp = 1;
      for (size_t q = 0; q < k; ++q) fgrp = std::max(fgrp, (int)fbig[sset[pos + q]]);
      fgrp = std::min(fcap, (fgrp + 63) & ~63);
      // two links per lane (cfg 3: E1 values 2.68 -> 2.34 s, E2 ~3 % less)
      const bool pair = !vfast && S <= 16 && (value_pair == 2 || (value_pair == 1 && heavy));
      // Dataflow value pass (estep_df.hip): one wave walks the loci and
      // builds the lists, the others run the chains of adds of any open locus.
      DfShape df;
      const bool use_df = !vfast && S <= 32 && (value_pass == VP_DATAFLOW || (value_pass == VP_AUTO && df_auto(heavy))) &&
                          df_shape(S, pair, heavy, small_heavy, per_cu, fgrp, df);
      if (use_df) {
        vnw = df.nw;
        vipc = df.ipc;
      }
      const int G2 = std::max(1, std::min(waves > 0 ? waves : dev_cu * vipc, n));
      // register budget: 5 waves per SIMD once the shape asks for more than 16 per CU
      const int vwpe = vnw * vipc > 16 && vnw * vipc <= 20 ? 5 : 4;
      const size_t per2 = use_df ? estep_df_scratch_bytes(fgrp, S, df.R) : estep_s2_scratch_bytes(fgrp, S);
      const int grid2 = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::min<int>(G2, (int)k), SCRATCH_MAX / per2));
      if ((e = scratch_ensure(d_scr2, per2 * grid2, false, true))) return hipfail(e, "estep pass-2 scratch");
      if ((rc = ensure_store(d_trace, std::max<uint64_t>(t, 1), trace_budget, "trace store"))) return rc;
      ValueArgs v;
      v.S = S;
      v.L = L;
      v.head_len = head_len;
      v.order = d_order2.p;
      v.n_order = (int)k;
      v.rec = d_rec.p;
      v.rec_off = d_rec_off.p;
      v.scratch = d_scr2.p;
      v.scratch_stride = per2;
      v.fcap = fgrp;
      v.lds_fc = use_df ? df.fc : s2_tier(S, vnw, vipc, pair);
      v.trace = d_trace.p;
      v.trace_cap = d_trace.n;
      v.trace_cursor = d_trace_cursor.p;
      v.trace_base = d_tbase.p;
      v.loc_off = d_loc_off.p;
      v.status = d_status.p;
      v.total = d_total.p;
      v.ncand = d_ncand.p;
      v.cand_state = d_cstate.p;
      v.cand_idx = d_cidx.p;
      v.prior = d_prior.p;
      v.posterior = d_post.p;
      v.weight = d_weight.p;
      v.cost = d_cost.p;
      v.stamps = d_stamps.p;
      v.next_q = d_nextq.p + 1;
      if ((e = hipMemsetAsync(d_nextq.p + 1, 0, 4, st))) return hipfail(e, "estep");
      const bool fast = vfast;
      hipEventRecord(ev[0], st);
      if (use_df) {
        if ((e = launch_estep_values_df(v, grid2, vnw, df.na, vwpe, pair, df.R, df.qcap, st)))
          return hipfail(e, "estep_values_df launch");
      } else if ((e = launch_estep_values(v, grid2, vnw, fast, vwpe, st, pair))) {
        return hipfail(e, "estep_values launch");
      }
      last_value_df = use_df;
      hipEventRecord(ev[1], st);
      if ((rc = read_status(sset, (int)k, true))) return rc;
      hipEventElapsedTime(&ms, ev[0], ev[1]);
      ms_s2 += ms;
      ++n_value_passes;
      if (debug_mem)
        fprintf(stderr, "[hmc] value pass %d: %zu individuals, %d x %d per CU (%.0f record words per individual-locus), %.1f ms\n",
                n_value_passes, k, vnw, vipc, rw / ((double)k * L), ms);
      // ---- ties: individuals whose result would depend on the libstdc++ list
      // order re-run on the exact value pass, in their own trace regions
      std::vector<int> h_order;
      for (size_t q = 0; q < k; ++q)
        if (h_status[sset[pos + q]] == EST_NEEDS_ORDER) h_order.push_back(sset[pos + q]);
      n_order_redo += (int)h_order.size();
      if (!h_order.empty()) {
        const int nr = (int)h_order.size();
        if ((e = d_redo.ensure(nr))) return hipfail(e, "estep order re-run");
        if ((rc = upload_order(d_redo, h_order.data(), nr))) return rc;
        ValueArgs v2 = v;
        v2.order = d_redo.p;
        v2.n_order = nr;
        if ((e = hipMemsetAsync(d_nextq.p + 1, 0, 4, st))) return hipfail(e, "estep");
        hipEventRecord(ev[0], st);
        if ((e = launch_estep_values(v2, std::max(1, std::min(G2, nr)), vnw, false, vwpe, st)))
          return hipfail(e, "estep_values launch");
        hipEventRecord(ev[1], st);
        if ((rc = read_status(sset, (int)k, true))) return rc;
        hipEventElapsedTime(&ms, ev[0], ev[1]);
        ms_s2 += ms;
        ms_order += ms;
        ++n_value_passes;  // (every value-kernel launch counts: the PMC pairing in tools/pmc_traffic.py)
      }
      h_redo.clear();
      for (size_t q = 0; q < k; ++q) {
        const int bi = sset[pos + q];
        if (h_status[bi] == EST_OVERFLOW_TRACE) return fail(HMC_EHIP, "trace store overflow with exact sizes");
        if (h_status[bi] == EST_NEEDS_ORDER) return fail(HMC_EHIP, "exact value pass reported a tie");
        if (h_status[bi] == EST_DF_STALL) {  // the kernel leaves the watchdog's site in cost / total
          int32_t at = 0;
          double val = 0;
          (void)hipMemcpy(&at, d_cost.p + bi, 4, hipMemcpyDeviceToHost);
          (void)hipMemcpy(&val, d_total.p + bi, 8, hipMemcpyDeviceToHost);
          return fail(HMC_EHIP, "dataflow value pass stalled (individual %d; site %d, wave %d, locus %d, value %.0f)", i0 + bi,
                      at >> 24, (at >> 16) & 0xFF, at & 0xFFFF, val);
        }
        if (h_status[bi] == EST_NEEDS_EXACT) h_redo.push_back(bi);
      }
      // ---- individuals whose forward likelihood underflowed: the reference
      // skips a pair with fwd <= 0 (extend(), HaploBuilder.cpp:237), which
      // changes their structure.  Their records are rebuilt with that test
      // (structure pass, prune) in their own regions — a subset of the
      // frontiers just walked, so they fit — and their lists re-built.
      n_fallback += (int)h_redo.size();
      if (!h_redo.empty()) {
        const int nr = (int)h_redo.size();
        if ((rc = structure_pass(h_redo.data(), nr, true))) return rc;
        for (int r : h_redo) {
          const int s = h_status[r];
          if (s != EST_OK_PRUNED && s != EST_UNRESOLVED)
            return fail(HMC_EHIP, "underflow re-run: structure status %d (individual %d)", s, i0 + r);
        }
        if ((e = d_redo.ensure(nr))) return hipfail(e, "estep underflow re-run");
        if ((rc = upload_order(d_redo, h_redo.data(), nr))) return rc;
        ValueArgs v2 = v;
        v2.order = d_redo.p;
        v2.n_order = nr;
        if ((e = hipMemsetAsync(d_nextq.p + 1, 0, 4, st))) return hipfail(e, "estep");
        hipEventRecord(ev[0], st);
        if (use_df) {
          if ((e = launch_estep_values_df(v2, std::max(1, std::min(G2, nr)), vnw, df.na, vwpe, pair, df.R, df.qcap, st)))
            return hipfail(e, "estep_values_df launch");
        } else if ((e = launch_estep_values(v2, std::max(1, std::min(G2, nr)), vnw, false, vwpe, st, pair))) {
          return hipfail(e, "estep_values launch");
        }
        hipEventRecord(ev[1], st);
        if ((rc = read_status(sset, (int)k, true))) return rc;
        hipEventElapsedTime(&ms, ev[0], ev[1]);
        ms_fb += ms;
        ++n_value_passes;
        for (int r : h_redo)
          if (h_status[r] != EST_OK && h_status[r] != EST_UNRESOLVED)
            return fail(HMC_EHIP, "underflow re-run: value status %d (individual %d)", h_status[r], i0 + r);
      }
      if ((rc = traceback_group((int)k))) return rc;
      pos += k;
    }
    pending.swap(rest);
  }
  if (!exact) {
    prev_rneed = rneed;
    prev_P = P;
  }
  return HMC_OK;
}

bool Ctx::df_shape(int S, bool pair, bool heavy, bool small_heavy, int per_cu, int fgrp, DfShape &d) const {
  d.nw = vp_nw > 0 ? std::max(2, vp_nw) : (small_heavy ? std::max(2, 16 / per_cu) : (heavy ? 8 : 2));
  d.ipc = vp_ipc > 0 ? vp_ipc : (small_heavy ? per_cu : (heavy ? 2 : 8));
  if (d.nw * d.ipc > 20) d.ipc = std::max(1, 20 / d.nw);
  // A waves: a fixed share of every locus's states each (cfg 3's E1: 468
  // states per locus, ~8 rounds of 64 for a lone A wave)
  d.na = df_na > 0 ? std::min(df_na, d.nw - 1) : std::max(1, d.nw / 4);
  d.R = df_ring;
  const int G = pair ? WAVE / S : WAVE / (2 * S);
  const int nseg = (d.nw - d.na) * G;
  d.qcap = 64;
  // (queue slots carry a 32-byte chain descriptor: cfg 3's E1 has ~130 chains
  // per locus, about two loci in flight)
  while (d.qcap < std::max(4 * nseg, heavy ? 256 : 64)) d.qcap *= 2;
  const int budget = 160 * 1024 / std::max(1, d.ipc) - 256;
  if ((int)estep_df_lds_bytes(S, 0, d.nw, d.na, pair, d.R, d.qcap, fgrp) > budget) return false;
  int lo = 0, hi = fgrp;  // largest LDS tier that fits
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    if ((int)estep_df_lds_bytes(S, mid, d.nw, d.na, pair, d.R, d.qcap, fgrp) <= budget) lo = mid;
    else hi = mid - 1;
  }
  d.fc = lo;
  return true;
}

DevModel Ctx::dev_model() const {
  DevModel m;
  m.P = P;
  m.succ = t_succ.p;
  m.tp = t_tp.p;
  m.freq = t_freq.p;
  m.last = t_last.p;
  m.n_head = n_head;
  m.head_len = head_len;
  m.head_ids = d_head_ids.p;
  m.head_pat0 = d_head_pat0.p;
  if (head_len > 1) {
    m.hf_base = i0;
    m.hf_off = d_hf_off.p;
    m.hf_pairs = d_hf_pairs.p;
    m.hf_status = d_hf_status.p;
    m.head_al = d_head_al.p;
  }
  if (end_order && gmodel_gen == model_gen && P > 0) {
    m.gsucc = g_succ.p;
    m.gtp = g_tp.p;
    m.glast = g_last.p;
    m.gid = g_gid.p;
    m.ginv = g_inv.p;
  }
  return m;
}

// The end-locus-ordered table of the current model (gmodel.hip): sorted ids,
// their inverse, successors / tp / last alleles by g.  Without the HBM for it
// the structure pass keeps the id-ordered table (same records).
int Ctx::ensure_gmodel() {
  if (!end_order || gmodel_gen == model_gen || P <= 0) return HMC_OK;
  HpTimer hpt(hp_ms[HP_GMODEL]);
  const int A = pan.amax;
  const size_t tb = gmodel_sort_bytes(P, pan.L);
  hipError_t e;
  if ((e = g_gid.ensure(P)) || (e = g_inv.ensure(P)) || (e = g_succ.ensure((size_t)P * A)) || (e = g_keys.ensure(3 * (size_t)P)) ||
      (e = g_tp.ensure(P)) || (e = g_last.ensure(P)) || (e = g_temp.ensure(std::max<size_t>(tb, 1)))) {
    if (e != hipErrorOutOfMemory) return hipfail(e, "end-order table");
    (void)hipGetLastError();
    g_gid.release(), g_inv.release(), g_succ.release(), g_keys.release(), g_tp.release(), g_last.release(), g_temp.release();
    return HMC_OK;  // gmodel_gen stays stale: the id-ordered table
  }
  GModelArgs g;
  g.P = P;
  g.A = A;
  g.L = pan.L;
  g.start = t_start.p;
  g.len = t_len.p;
  g.succ = t_succ.p;
  g.tp = t_tp.p;
  g.last = t_last.p;
  g.key_in = g_keys.p;
  g.key_out = g_keys.p + P;
  g.id_in = g_keys.p + 2 * (size_t)P;
  g.temp = g_temp.p;
  g.temp_bytes = g_temp.n;
  g.gid = g_gid.p;
  g.inv = g_inv.p;
  g.gsucc = g_succ.p;
  g.gtp = g_tp.p;
  g.glast = g_last.p;
  if ((e = build_gmodel(g, st)) || (e = sync_st())) return hipfail(e, "end-order table");
  if (g_keys.n * 4 + g_temp.n > (2ull << 30)) {  // only the build needs them: give large ones back (cfg 4's
    g_keys.release();                              // 720 M patterns: ~10 GB); small ones stay mapped (re-mapping
    g_temp.release();                              // costs more than the next model's build)
  }
  gmodel_gen = model_gen;
  return HMC_OK;
}

int Ctx::resolutions_idx(std::vector<uint8_t> &out) {
  if (!have_estep) return fail(HMC_EARG, "no E-step has run");
  const int n = nloc(), L = pan.L;
  hipError_t e;
  if ((e = d_res.ensure((size_t)n * 2 * L))) return hipfail(e, "resolutions");
  if ((e = launch_gather_resolutions(d_rows.p, L, d_sbase.p, d_ncand.p, d_geno_im.p, i0, n, d_res.p, st)))
    return hipfail(e, "resolutions");
  out.resize((size_t)n * 2 * L);
  if ((e = hipMemcpyAsync(out.data(), d_res.p, out.size(), hipMemcpyDeviceToHost, st)) ||
      (e = sync_st()))
    return hipfail(e, "resolutions");
  return HMC_OK;
}
// Diagnostic (HMC_CHECK_RECORDS): the structure records of individuals
// ids[0, np_) against the invariants the value passes rely on — per locus,
// contribution offsets ascending to Cv; every contribution's predecessor below
// the previous frontier with that state's list length; a state's list length
// min(S, sum of its contributions'); the chain flag and list exactly the states
// whose sum exceeds S.  The first violation fails the E-step (HMC_EHIP) with
// its individual and locus instead of letting a value pass walk bad records.
int Ctx::validate_records(const int32_t *ids, int np_, int i0) {
  hipError_t e;
  if ((e = sync_st())) return hipfail(e, "validate_records");
  const int L = pan.L, hl = head_len;
  std::vector<unsigned long long> off(d_rec_off.n);
  std::vector<uint32_t> rec(d_rec.n);
  if ((e = hipMemcpy(off.data(), d_rec_off.p, off.size() * 8, hipMemcpyDeviceToHost)) ||
      (e = hipMemcpy(rec.data(), d_rec.p, rec.size() * 4, hipMemcpyDeviceToHost)))
    return hipfail(e, "validate_records");
  int bad = 0;
  for (int q = 0; q < np_ && !bad; ++q) {
    const int bi = ids[q];
    const int stt = h_status[bi];
    if (stt != EST_OK && stt != EST_OK_PRUNED) continue;
    const unsigned long long *ro = off.data() + (size_t)bi * (L + 1);
    std::vector<uint32_t> nl_prev;
    for (int i = hl - 1; i < L && !bad; ++i) {
      const unsigned long long o = ro[i + 1];
      if (o + 4 > rec.size()) { fprintf(stderr, "[hmc] records: indiv %d locus %d offset %llu past the store\n", i0 + bi, i, o); bad = 1; break; }
      const uint32_t *R = rec.data() + o;
      const uint32_t Fn = R[0], Cv = R[1], nch = R[2];
      const uint32_t *Rhd = R + 4 + 2 * Fn, *Rcb = Rhd + Fn, *Rct = Rcb + Fn + 1, *Rch = Rct + Cv;
      if (o + 4 + 4ull * Fn + 1 + Cv + nch > rec.size()) { fprintf(stderr, "[hmc] records: indiv %d locus %d past the store\n", i0 + bi, i); bad = 1; break; }
      std::vector<uint32_t> nl(Fn);
      uint32_t flagged = 0;
      for (uint32_t t = 0; t < Fn && !bad; ++t) {
        nl[t] = (Rhd[t] >> 16) & 0xFFu;  // (bit 24: the head's homozygous flag, bit 27: chain)
        if (i == hl - 1) continue;  // head locus: lists of one, no contributions
        if (Rcb[t] > Rcb[t + 1] || Rcb[t + 1] > Cv) {
          fprintf(stderr, "[hmc] records: indiv %d locus %d state %u: offsets %u %u (Cv %u)\n", i0 + bi, i, t, Rcb[t], Rcb[t + 1], Cv);
          bad = 1;
          break;
        }
        uint32_t sum = 0;
        for (uint32_t r = Rcb[t]; r < Rcb[t + 1]; ++r) {
          const uint32_t ps = cw_state(Rct[r]), ns = cw_ns(Rct[r]);
          if (ps >= nl_prev.size() || ns != nl_prev[ps]) {
            fprintf(stderr, "[hmc] records: indiv %d locus %d state %u add %u: predecessor %u (of %zu) ns %u\n", i0 + bi, i, t,
                    r - Rcb[t], ps, nl_prev.size(), ns);
            bad = 1;
            break;
          }
          sum += ns;
        }
        const bool chain = (Rhd[t] & HDR_CHAIN) != 0;
        if (!bad && (nl[t] != std::min<uint32_t>(sum, (uint32_t)S()) || chain != (sum > (uint32_t)S()) || Rcb[t] == Rcb[t + 1])) {
          fprintf(stderr, "[hmc] records: indiv %d locus %d state %u: list %u, sum %u, chain %d, adds %u\n", i0 + bi, i, t, nl[t], sum,
                  (int)chain, Rcb[t + 1] - Rcb[t]);
          bad = 1;
        }
        flagged += chain ? 1u : 0u;
      }
      if (!bad && i >= hl) {
        if (Rcb[Fn] != Cv || flagged != nch) {
          fprintf(stderr, "[hmc] records: indiv %d locus %d: Rcb[F] %u Cv %u, chains %u listed %u\n", i0 + bi, i, Rcb[Fn], Cv, flagged, nch);
          bad = 1;
        }
        std::vector<char> seen(Fn, 0);
        for (uint32_t k = 0; k < nch && !bad; ++k)
          if (Rch[k] >= Fn || seen[Rch[k]] || !(Rhd[Rch[k]] & HDR_CHAIN)) {
            fprintf(stderr, "[hmc] records: indiv %d locus %d: chain entry %u = %u\n", i0 + bi, i, k, Rch[k]);
            bad = 1;
          } else {
            seen[Rch[k]] = 1;
          }
      }
      nl_prev.swap(nl);
    }
  }
  return bad ? fail(HMC_EHIP, "structure records failed validation (HMC_CHECK_RECORDS)") : HMC_OK;
}

}  // namespace hmc
