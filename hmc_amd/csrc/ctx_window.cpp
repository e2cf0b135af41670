// ctx_window.cpp — Ctx members: the checkpoint-and-recompute E-step (locus
// windows, SURVEY §7 hard part 4) for panels whose per-individual records and
// traces leave the stores room for only a few hundred individuals at a time.
//
// HaploBuilder::resolve (HaploBuilder.cpp:35-126) walks the loci once forward
// and the traceback (HaploPair::getGenotype, HaploPair.cpp:91-124) once
// backward; the forward state at a locus is the frontier alone (pattern pairs,
// list lengths, forward likelihoods, k-best lists).  So the record indices
// hl..L are cut into windows: the forward saves each window's last frontier
// (a checkpoint of ~(7 + 2S) words per state) and keeps no records or traces
// past the window; the backward recomputes each window from its checkpoint —
// the same passes over the same records, so the same traces — and continues
// the traceback through it.  Records and traces then take one window's worth
// per individual, and the whole shard runs as one group that fills the GPU.
#include "ctx.hpp"

namespace hmc {

bool Ctx::windows_allowed() const {
  return window_mode != WIN_NEVER && estep_mode == ESTEP_SPLIT && structure_pass_version != 2 &&
         value_pass != VP_DATAFLOW;
}

int Ctx::estep_windowed(const std::vector<int32_t> &order) {
  const int S = this->S(), n = nloc(), L = pan.L, hl = head_len;
  const int NR = L + 1 - hl;  // record / trace indices hl..L
  int dev_cu = 256;
  hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, device);
  hipError_t e;
  int rc;
  size_t freeb = 0, totb = 0;
  hipMemGetInfo(&freeb, &totb);
  const double pool = (double)freeb + 4.0 * ((double)d_trace.n + (double)d_rec.n + (double)d_ck.n);
  const uint64_t rbud = (uint64_t)std::min(0.27 * pool, (double)(88ull << 30)) / 4;
  const uint64_t tbud = (uint64_t)std::min(0.40 * pool, (double)(130ull << 30)) / 4;
  const uint64_t cbud = (uint64_t)std::min(0.12 * pool, (double)(40ull << 30)) / 4;
  if ((e = d_nextq.ensure(2)) || (e = d_rec_off.ensure((size_t)n * (L + 1))) || (e = d_rec_cursor.ensure(1)))
    return hipfail(e, "windowed E-step alloc");
  std::vector<unsigned long long> hr(n), ht(n), rb(n, 0), rs(n, 0), tbv(n, 0);
  std::vector<int32_t> hf(n);
  const bool heavy_model = (double)P > (double)pan.N * (double)pan.L;
  float ms = 0;
  int nwin = 1;
  std::vector<int> bound{hl, L + 1};
  std::vector<unsigned long long> rw, tw;  // exact needs per individual and window
  std::vector<int32_t> fw;                 // largest frontier per individual and window

  // Structure pass of the record indices [bound[w], bound[w + 1]) over
  // ids[0, np_) in the regions rb / rs.
  auto structure = [&](int w, const int32_t *ids, int np_, bool ck_write, int re_mode, bool fwd) -> int {
    const int nw1 = s1_nw > 0 ? s1_nw : (heavy_model ? (np_ <= dev_cu ? 16 : 4) : 1);
    const int bpc1 = s1_ipc > 0 ? s1_ipc
                                : (nw1 == 16 ? 1 : (nw1 == 4 ? 2 : (np_ > 8 * dev_cu ? 12 : (np_ > 4 * dev_cu ? 8 : 4))));
    const int hcap1 = next_pow2(2 * fcap);
    const int ccap1 = (int)std::min<int64_t>(INT32_MAX / 2, (int64_t)ccap_mult * fcap);
    const size_t per1 = estep_s1_scratch_bytes(fcap, hcap1, ccap1, nw1, false);
    const int grid1 = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::min(np_, dev_cu * bpc1), SCRATCH_MAX / per1));
    hipError_t e2;
    int rc2;
    if ((e2 = d_scr1.ensure(per1 * grid1)) || (e2 = hipMemcpyAsync(d_rbase.p, rb.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)) ||
        (e2 = hipMemcpyAsync(d_recsz.p, rs.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)) ||
        (e2 = hipMemsetAsync(d_nextq.p, 0, 8, st)))
      return hipfail(e2, "windowed structure pass");
    if ((rc2 = upload_order(d_order, ids, np_))) return rc2;
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
    s1_tier(160 * 1024 / bpc1 - 256, pan.amax, nw1, s1.lds_fc, s1.lds_hc, s1.lds_cc);
    s1.rec = d_rec.p;
    s1.rec_cap = d_rec.n;
    s1.rec_cursor = d_rec_cursor.p;
    s1.rec_base = d_rbase.p;
    s1.rec_size = d_recsz.p;
    s1.rec_off = d_rec_off.p;
    s1.rec_need = d_rneed.p;
    s1.trace_need = d_tneed.p;
    s1.status = d_status.p;
    s1.re_count = d_re.p;
    s1.re_mode = re_mode;
    s1.fmax = d_fmax.p;
    s1.max_states = d_maxst.p;
    s1.stamps = d_stamps.p + 20;
    s1.exact = false;
    s1.prune = false;
    s1.next_q = d_nextq.p;
    s1.w.lo = bound[w];
    s1.w.hi = bound[w + 1];
    s1.w.win = w;
    s1.w.nwin = nwin;
    s1.w.ck_store = d_ck.p;
    s1.w.ck_cap = d_ck.n;
    s1.w.ck_cursor = d_ck_cursor.p;
    s1.w.ck_off = d_ck_off.p;
    s1.w.ck_write = ck_write;
    hipEventRecord(ev[0], st);
    if ((e2 = launch_estep_structure(s1, grid1, nw1, st))) return hipfail(e2, "estep_structure launch");
    hipEventRecord(ev[1], st);
    if ((e2 = hipMemcpyAsync(hr.data(), d_rneed.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
        (e2 = hipMemcpyAsync(ht.data(), d_tneed.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
        (e2 = hipMemcpyAsync(hf.data(), d_fmax.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)))
      return hipfail(e2, "windowed structure pass");
    if ((rc2 = read_status({}, 0, false))) return rc2;
    hipEventElapsedTime(&ms, ev[0], ev[1]);
    ms_s1 += ms;
    if (!fwd) ms_ck += ms;
    ++n_struct_passes;
    if (debug_mem)
      fprintf(stderr, "[hmc] window %d/%d %s: structure pass %d individuals, %d x %d per CU, %.1f ms\n", w + 1, nwin,
              fwd ? "forward" : "recompute", np_, nw1, bpc1, ms);
    return HMC_OK;
  };
  auto restart_status = [&](int s) -> int {  // statuses that end the E-step (or restart it)
    if (s == EST_NO_HEAD_PATTERN) return fail(HMC_ENOPATTERN, "Can not find matching pattern!");
    if (s == EST_OVERFLOW_CONTRIB) {
      if ((int64_t)ccap_mult * fcap >= INT32_MAX / 2) return fail(HMC_EUNSUPPORTED, "too many contributions at a locus");
      ccap_mult *= 2;
      return ESTEP_RESTART;
    }
    if (s == EST_OVERFLOW_FRONTIER) {
      if (fcap >= F_MAX) return fail(HMC_EUNSUPPORTED, "frontier exceeds %d states", F_MAX);
      fcap = (int)std::min<int64_t>(F_MAX, (int64_t)fcap * 4);
      return ESTEP_RESTART;
    }
    return HMC_OK;
  };

  // ---- probe: the first loci of a sample spread over the cost order --------
  // (counting only: no records are stored) give each individual's record and
  // trace words per locus; the classic passes run unless their groups would
  // be too small to fill the GPU (more than one group of fewer than two
  // individuals per CU)
  const int LP = std::min(NR, window_loci > 0 ? std::max(window_loci, 64) : std::max(64, NR / 8));
  bound = {hl, hl + LP};
  const int kp = std::min(n, 4 * dev_cu);
  std::vector<int32_t> pick;
  for (int q = 0; q < n; ++q)
    if ((int64_t)q * kp / n != (int64_t)(q - 1) * kp / n || q == 0) pick.push_back(order[q]);
  std::fill(rs.begin(), rs.end(), 0ull);  // regions of size 0: counting only
  if ((rc = structure(0, pick.data(), (int)pick.size(), false, 2, true))) return rc;
  double rl = 0, tl = 0, rmean = 0, tmean = 0;
  for (int bi : pick) {
    if ((rc = restart_status(h_status[bi]))) return rc;
    rl = std::max(rl, (double)hr[bi] / LP);
    tl = std::max(tl, (double)ht[bi] / LP);
    rmean += (double)hr[bi] / LP / pick.size();
    tmean += (double)ht[bi] / LP / pick.size();
  }
  const double k_classic = std::min((double)rec_budget / std::max(1.0, rmean * NR), (double)trace_budget / std::max(1.0, tmean * NR));
  if (debug_mem)
    fprintf(stderr, "[hmc] window probe: %zu individuals x %d loci; per locus records %.0f (max %.0f), traces %.0f (max %.0f) "
            "words: classic groups of ~%.0f\n", pick.size(), LP, rmean, rl, tmean, tl, k_classic);
  if (window_mode != WIN_ALWAYS && !(k_classic < 2.0 * dev_cu && (double)n > k_classic)) return WIN_DECLINED;
  if (rl <= 0) return fail(HMC_EHIP, "windowed E-step without a measured individual");

  // ---- plan: window length and group size --------------------------------
  // Every individual of a group gets an even share of each store per window,
  // sized for the heaviest probed one with 25 % headroom; one whose window
  // needs more runs that window again with its exact size.
  const double fmax_est = std::max(1.0, (tl - 2.0) / (1.0 + S));  // states per locus of the heaviest
  const double ckw = (double)ck_words((unsigned long long)fmax_est, S) + 2.0;
  int k = n, WL = 0;
  for (int div = 1;; ++div) {
    k = (n + div - 1) / div;
    const double wl_r = (double)rbud / ((double)k * rl * 1.25), wl_t = (double)tbud / ((double)k * tl * 1.25);
    WL = window_loci > 0 ? window_loci : (int)std::max(1.0, std::min(wl_r, wl_t));
    WL = std::min(WL, NR);
    nwin = (NR + WL - 1) / WL;
    if ((double)k * (nwin - 1) * ckw <= (double)cbud || k == 1) break;
  }
  WL = (NR + nwin - 1) / nwin;  // even windows
  bound.assign(nwin + 1, 0);
  for (int w = 0; w <= nwin; ++w) bound[w] = hl + std::min(NR, w * WL);
  const int ngroups = (n + k - 1) / k;
  last_windows = nwin;
  last_window_loci = WL;
  last_window_groups = ngroups;
  if (debug_mem)
    fprintf(stderr, "[hmc] windowed E-step: %d individuals in %d group(s) of <= %d, %d windows of %d loci; "
            "per locus %.0f record / %.0f trace words (heaviest), budgets rec %.1f trace %.1f ckpt %.1f GB\n",
            n, ngroups, k, nwin, WL, rl, tl, rbud * 4e-9, tbud * 4e-9, cbud * 4e-9);
  // ---- buffers ------------------------------------------------------------
  const uint64_t ck_need = nwin > 1 ? (uint64_t)((double)k * (nwin - 1) * ckw * 1.25) + 1024 : 1024;
  if (d_ck.n < ck_need) {
    d_ck.release();
    e = d_ck.ensure(std::min<uint64_t>(ck_need, std::max<uint64_t>(cbud, 1024)));
    if (e == hipErrorOutOfMemory) {  // the stores are dead here: they give way
      (void)hipGetLastError();
      d_trace.release();
      d_rec.release();
      e = d_ck.ensure(std::min<uint64_t>(ck_need, std::max<uint64_t>(cbud, 1024)));
    }
    if (e) return hipfail(e, "checkpoint store");
  }
  if ((e = d_ck_off.ensure((size_t)n * (nwin + 1))) || (e = d_ck_cursor.ensure(1)) ||
      (e = d_cur_state.ensure((size_t)n * S_MAX)) || (e = d_cur_idx.ensure((size_t)n * S_MAX)) ||
      (e = d_cur_swap.ensure((size_t)n * S_MAX)) || (e = hipMemsetAsync(d_re.p, 0, (size_t)n * 8, st)) ||
      (e = hipMemsetAsync(d_cost.p, 0, (size_t)n * 4, st)))
    return hipfail(e, "windowed E-step alloc");
  rw.assign((size_t)n * nwin, 0);
  tw.assign((size_t)n * nwin, 0);
  fw.assign((size_t)n * nwin, 0);
  std::vector<int32_t> underflow;  // individuals whose likelihoods underflow: the classic passes (prune mode)

  // Value pass of window w over ids[0, k_) (trace regions in tbv), then the
  // traceback through the window when `tb`.
  auto values = [&](int w, const int32_t *ids, int k_, bool ck_write, bool tb, bool fwd) -> int {
    hipError_t e2;
    int rc2;
    double rsum = 0;
    int fgrp = 1;
    for (int q = 0; q < k_; ++q) {
      rsum += (double)rw[(size_t)ids[q] * nwin + w];
      fgrp = std::max(fgrp, (int)fw[(size_t)ids[q] * nwin + w]);
    }
    fgrp = std::min(fcap, (fgrp + 63) & ~63);
    const int wl = bound[w + 1] - bound[w];
    const bool heavy = rsum / ((double)k_ * wl) > 1500.0;
    const int per_cu = (k_ + dev_cu - 1) / dev_cu;
    const bool small_heavy = heavy && per_cu < 4;
    const int vnw = vp_nw > 0 ? vp_nw : (small_heavy ? 16 / per_cu : (heavy ? 4 : (k_ >= 32 * dev_cu ? 1 : (k_ >= 8 * dev_cu ? 2 : 3))));
    const int vipc = vp_ipc > 0 ? vp_ipc : (small_heavy ? per_cu : (vnw == 1 ? 16 : (vnw >= 8 ? 2 : (vnw >= 4 ? 4 : 8))));
    const bool pair = S <= 16 && (value_pair == 2 || (value_pair == 1 && heavy));
    const int G2 = std::max(1, std::min(waves > 0 ? waves : dev_cu * vipc, n));
    const int vwpe = vnw * vipc > 16 && vnw * vipc <= 20 ? 5 : 4;
    const size_t per2 = estep_s2_scratch_bytes(fgrp, S);
    const int grid2 = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::min(G2, k_), SCRATCH_MAX / per2));
    if ((e2 = d_scr2.ensure(per2 * grid2)) || (e2 = hipMemcpyAsync(d_tbase.p, tbv.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)) ||
        (e2 = hipMemsetAsync(d_nextq.p + 1, 0, 4, st)))
      return hipfail(e2, "windowed value pass");
    if ((rc2 = upload_order(d_order2, ids, k_))) return rc2;
    ValueArgs v;
    v.S = S;
    v.L = L;
    v.head_len = hl;
    v.order = d_order2.p;
    v.n_order = k_;
    v.rec = d_rec.p;
    v.rec_off = d_rec_off.p;
    v.scratch = d_scr2.p;
    v.scratch_stride = per2;
    v.fcap = fgrp;
    v.lds_fc = s2_tier(S, vnw, vipc, pair);
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
    v.w.lo = bound[w];
    v.w.hi = bound[w + 1];
    v.w.win = w;
    v.w.nwin = nwin;
    v.w.ck_store = d_ck.p;
    v.w.ck_cap = d_ck.n;
    v.w.ck_cursor = d_ck_cursor.p;
    v.w.ck_off = d_ck_off.p;
    v.w.ck_write = ck_write;
    hipEventRecord(ev[0], st);
    if ((e2 = launch_estep_values(v, grid2, vnw, false, vwpe, st, pair))) return hipfail(e2, "estep_values launch");
    hipEventRecord(ev[1], st);
    if ((rc2 = read_status({}, 0, true))) return rc2;
    hipEventElapsedTime(&ms, ev[0], ev[1]);
    ms_s2 += ms;
    if (!fwd) ms_ck += ms;
    ++n_value_passes;
    if (debug_mem)
      fprintf(stderr, "[hmc] window %d/%d %s: value pass %d individuals, %d x %d per CU, %.1f ms\n", w + 1, nwin,
              fwd ? "forward" : "recompute", k_, vnw, vipc, ms);
    for (int q = 0; q < k_; ++q) {
      const int s = h_status[ids[q]];
      if (s == EST_OVERFLOW_TRACE) return fail(HMC_EHIP, "trace store overflow with exact sizes (window %d)", w);
      if (s != EST_OK && s != EST_UNRESOLVED && s != EST_NEEDS_EXACT)
        return fail(HMC_EHIP, "windowed value pass: status %d (individual %d, window %d)", s, i0 + ids[q], w);
    }
    if (tb) {
      TracebackArgs t;
      t.L = L;
      t.S = S;
      t.head_len = hl;
      t.nbatch = k_;
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
      t.win_lo = bound[w];
      t.win_hi = bound[w + 1];
      t.cur_state = d_cur_state.p;
      t.cur_idx = d_cur_idx.p;
      t.cur_swap = d_cur_swap.p;
      hipEventRecord(ev[2], st);
      if ((e2 = launch_traceback(t, 0, st))) return hipfail(e2, "traceback");
      hipEventRecord(ev[3], st);
      if ((e2 = hipStreamSynchronize(st))) return hipfail(e2, "traceback");
      hipEventElapsedTime(&ms, ev[2], ev[3]);
      ms_tb += ms;
    }
    return HMC_OK;
  };

  // One window over the group `grp` (forward or recompute): structure pass,
  // then value passes (and tracebacks) in sub-groups whose traces fit; an
  // individual whose window records overflowed its share runs again with its
  // exact size.  Individuals that die (no resolution) or underflow leave `grp`.
  auto window = [&](int w, std::vector<int32_t> &grp, bool fwd, bool tb) -> int {
    std::vector<int32_t> todo(grp), dead;
    bool first = true;
    while (!todo.empty()) {
      std::fill(rb.begin(), rb.end(), 0ull);
      std::fill(rs.begin(), rs.end(), 0ull);
      int np = 0;
      uint64_t r = 0;
      if (fwd && first) {  // an even share each
        const uint64_t share = std::max<uint64_t>(2, (rbud / (uint64_t)todo.size()) & ~1ull);
        for (int bi : todo) {
          rb[bi] = r;
          rs[bi] = share;
          r += share;
        }
        np = (int)todo.size();
      } else {  // exact sizes: the prefix that fits
        for (int bi : todo) {
          const uint64_t need = std::max<uint64_t>(rw[(size_t)bi * nwin + w], 2);
          if (np > 0 && r + need > rbud) break;
          rb[bi] = r;
          rs[bi] = need;
          r += need;
          ++np;
        }
      }
      if ((rc = ensure_store(d_rec, r, std::max<uint64_t>(rbud, r), "record store"))) return rc;
      if ((rc = structure(w, todo.data(), np, fwd && first, fwd && first ? 1 : 2, fwd))) return rc;
      std::vector<int32_t> ok, deferred;
      for (int q = 0; q < np; ++q) {
        const int bi = todo[q], s = h_status[bi];
        if ((rc = restart_status(s))) return rc;
        if (s == EST_OVERFLOW_CKPT) return fail(HMC_ENOMEM, "checkpoint store too small (window %d)", w);
        if (!fwd && s == EST_OVERFLOW_REC) return fail(HMC_EHIP, "record store overflow with exact sizes (window %d)", w);
        if (fwd && first) {
          rw[(size_t)bi * nwin + w] = hr[bi];
          tw[(size_t)bi * nwin + w] = ht[bi];
          fw[(size_t)bi * nwin + w] = hf[bi];
        }
        (s == EST_OVERFLOW_REC ? deferred : ok).push_back(bi);
      }
      for (int q = np; q < (int)todo.size(); ++q) deferred.push_back(todo[q]);
      // value passes in sub-groups whose traces fit the budget
      size_t pos = 0;
      while (pos < ok.size()) {
        uint64_t t = 0;
        size_t kk = 0;
        std::fill(tbv.begin(), tbv.end(), 0ull);
        while (pos + kk < ok.size()) {
          const int bi = ok[pos + kk];
          const uint64_t need = tw[(size_t)bi * nwin + w];
          if (kk > 0 && t + need > tbud) break;
          tbv[bi] = t;
          t += need;
          ++kk;
        }
        if ((rc = ensure_store(d_trace, std::max<uint64_t>(t, 1), std::max<uint64_t>(tbud, t), "trace store"))) return rc;
        if ((rc = values(w, ok.data() + pos, (int)kk, fwd, tb, fwd))) return rc;
        for (size_t q = 0; q < kk; ++q) {
          const int bi = ok[pos + q], s = h_status[bi];
          if (s == EST_NEEDS_EXACT) underflow.push_back(bi);
          if (s != EST_OK) dead.push_back(bi);
        }
        pos += kk;
      }
      todo.swap(deferred);
      first = false;
    }
    if (!dead.empty()) {  // out of the later windows and the recompute
      std::vector<char> gone(n, 0);
      for (int bi : dead) gone[bi] = 1;
      std::vector<int32_t> keep;
      for (int bi : grp)
        if (!gone[bi]) keep.push_back(bi);
      grp.swap(keep);
    }
    return HMC_OK;
  };

  std::vector<unsigned long long> rec_all(n, 0);
  for (int g = 0; g < ngroups; ++g) {
    std::vector<int32_t> grp(order.begin() + (std::ptrdiff_t)g * k, order.begin() + std::min<size_t>(order.size(), (size_t)(g + 1) * k));
    if ((e = hipMemsetAsync(d_ck_cursor.p, 0, 8, st))) return hipfail(e, "windowed E-step");
    for (int w = 0; w < nwin; ++w)  // forward; the last window traces back through itself
      if ((rc = window(w, grp, true, w == nwin - 1))) return rc;
    for (int w = nwin - 2; w >= 0; --w)  // backward: recompute and trace back
      if ((rc = window(w, grp, false, true))) return rc;
    for (int q = g * k; q < std::min(n, (g + 1) * k); ++q) {
      const int bi = order[q];
      for (int w = 0; w < nwin; ++w) rec_all[bi] += rw[(size_t)bi * nwin + w];
    }
  }
  prev_rneed.swap(rec_all);  // record words per individual (the next E-step's estimates at this scale)
  prev_P = P;
  // individuals whose forward likelihoods underflow: the classic passes, which
  // rebuild their structure with extend()'s forward test (prune mode)
  if (!underflow.empty()) {
    std::sort(underflow.begin(), underflow.end(), [&](int x, int y) { return h_cost[x] > h_cost[y]; });
    const int saved = window_mode;
    window_mode = WIN_NEVER;
    rc = estep_split(underflow);
    window_mode = saved;
    if (rc) return rc;
  }
  return HMC_OK;
}

}  // namespace hmc
