// ctx_window.cpp — Ctx members: the windowed E-step (locus windows with
// frontier checkpoints and trace garbage collection, SURVEY §7 hard part 4) for
// panels whose per-individual records and traces leave the stores room for
// only a few hundred individuals at a time (cfg 4's per-rank E1: ~250 MB of
// records and ~390 MB of traces per individual).
//
// HaploBuilder::resolve (HaploBuilder.cpp:35-126) walks the loci once forward
// and the traceback (HaploPair::getGenotype, HaploPair.cpp:91-124) once
// backward from the final candidates.  The forward state at a window boundary
// is the frontier alone (pattern pairs and list lengths; forward likelihoods
// and k-best lists): each window's passes start from the checkpoint the
// window before left, so records are kept for one window only.  The traces
// needed later are only those reachable backward from the final candidates,
// and the k-best links coalesce within a few dozen loci (cfg 2's E1: the
// ~1 000-2 300 list entries of a locus reach ~10 entries 50 loci back): after
// each window, the window before it is collected — its entries reachable from
// any entry at the current window's end become survivor nodes
// (estep_trace_gc) — so full traces are kept for two windows only.  The
// traceback walks the two full windows and then the survivors' chains.  Every
// pass runs the same arithmetic on the same inputs in the same order as the
// classic passes, so the results are bit-identical.
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
  const double pool = (double)freeb + 4.0 * ((double)d_trace.n + (double)d_rec.n + (double)d_ck[0].n + (double)d_ck[1].n);
  // budgets (words) from the free HBM, within the caller's store caps when set
  // (ranks sharing one GPU: hmc_set_store_budgets / hmc_set_tuning)
  const bool capped = trace_bytes || rec_bytes;
  // (pooling the two budgets and splitting them by need gave cfg 3's E1 8
  // windows instead of 10 and 1 % — but stores past the classic E-step's
  // budgets are re-mapped by the next E2, seconds per chain step: not kept)
  const uint64_t rbud = std::min<uint64_t>((uint64_t)std::min(0.27 * pool, (double)(88ull << 30)) / 4, capped ? rec_budget : ~0ull);
  const uint64_t tbud = std::min<uint64_t>((uint64_t)std::min(0.40 * pool, (double)(130ull << 30)) / 4, capped ? trace_budget : ~0ull);
  const uint64_t cbud = std::min<uint64_t>((uint64_t)std::min(0.12 * pool, (double)(40ull << 30)) / 4, capped ? trace_budget / 3 : ~0ull);
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

  bool bump = false;            // records from the store's bump allocator (the windows), else the regions rb / rs (the probe)
  // the structure pass's state capacity for the current window: twice the
  // largest frontier of the window before (its key table, HBM tier included,
  // stays small enough for the caches; cfg 4's E1 reaches 65 923 states at one
  // locus, which sized every window's tables for 2^18 states)
  int wfcap = fcap;
  // Structure pass of the record indices [bound[w], bound[w + 1]) over
  // ids[0, np_).
  auto structure = [&](int w, const int32_t *ids, int np_, bool ck_write, int re_mode, bool fwd) -> int {
    const int nw1 = s1_nw > 0 ? s1_nw : (heavy_model ? (np_ <= dev_cu ? 16 : 4) : 1);
    const int bpc1 = s1_ipc > 0 ? s1_ipc
                                : (nw1 == 16 ? 1 : (nw1 == 4 ? 2 : (np_ > 8 * dev_cu ? 12 : (np_ > 4 * dev_cu ? 8 : 4))));
    const int hcap1 = next_pow2(2 * wfcap);
    const int ccap1 = (int)std::min<int64_t>(INT32_MAX / 2, (int64_t)ccap_mult * wfcap);
    const size_t per1 = estep_s1_scratch_bytes(wfcap, hcap1, ccap1, nw1, false);
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
    s1.fcap = wfcap;
    s1.hcap = hcap1;
    s1.ccap = ccap1;
    s1_tier(160 * 1024 / bpc1 - 256, pan.amax, nw1, s1.lds_fc, s1.lds_hc, s1.lds_cc);
    s1.probe_lds = key_probes;
    s1.rec = d_rec.p;
    s1.rec_cap = d_rec.n;
    s1.rec_cursor = d_rec_cursor.p;
    s1.rec_base = bump ? nullptr : d_rbase.p;
    s1.rec_size = bump ? nullptr : d_recsz.p;
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
    s1.w.ck_in = d_ck[w & 1].p;
    s1.w.ck_out = d_ck[(w + 1) & 1].p;
    s1.w.ck_cap = d_ck[(w + 1) & 1].n;
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
  // trace words per locus; the classic passes run unless they would need
  // several groups (see below)
  // (at most 160 loci over two individuals per CU: one round of the pass, not
  // a tail — cfg 4's probe of 625 loci over 1 024 took as long as a window)
  const int LP = std::min(NR, window_loci > 0 ? std::max(window_loci, 64) : std::max(64, std::min(NR / 8, 160)));
  bound = {hl, hl + LP};
  const int kp = std::min(n, 2 * dev_cu);
  std::vector<int32_t> pick;
  for (int q = 0; q < n; ++q)
    if ((int64_t)q * kp / n != (int64_t)(q - 1) * kp / n || q == 0) pick.push_back(order[q]);
  std::fill(rs.begin(), rs.end(), 0ull);  // regions of size 0: counting only
  if ((rc = structure(0, pick.data(), (int)pick.size(), false, 2, true))) return rc;
  double rl = 0, tl = 0, rmean = 0, tmean = 0;
  int probe_fmax = 1;
  for (int bi : pick) {
    probe_fmax = std::max(probe_fmax, hf[bi]);
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
  // windows when the classic groups would hold fewer than two individuals per
  // CU, or when they would be three or more (cfg 3's E1: five groups, 3.41 s;
  // windows 3.23 s — fewer pass tails; two groups: the same time either way)
  if (window_mode != WIN_ALWAYS && !((double)n > k_classic && (k_classic < 2.0 * dev_cu || (double)n > 2.0 * k_classic)))
    return WIN_DECLINED;
  if (rl <= 0) return fail(HMC_EHIP, "windowed E-step without a measured individual");

  // ---- plan: window length and group size --------------------------------
  // The group's records (one window, bump-allocated) and traces (two windows)
  // are sized by the probe's mean per-locus needs with 25 % headroom; an
  // individual whose window records do not fit runs that window again.
  const double fmean = std::max(1.0, (tmean - 2.0) / (1.0 + S));  // states per locus, mean
  const double ckw = (double)ck_words((unsigned long long)fmean, S) + 4.0;
  // a checkpoint slot holds every individual's frontier at the heaviest probed size
  // (a slot that fills up grows and the window's structure pass runs again)
  const double ckw_max = (double)ck_words((unsigned long long)std::max(1.0, (tl - 2.0) / (1.0 + S) * 1.25), S) + 4.0;
  (void)rl;
  (void)tl;
  int k = n, WL = 0;
  for (int div = 1;; ++div) {
    k = (n + div - 1) / div;
    const double wl_r = (double)rbud / ((double)k * rmean * 1.25), wl_t = (double)tbud / (2.0 * (double)k * tmean * 1.25);
    WL = window_loci > 0 ? window_loci : (int)std::max(1.0, std::min(wl_r, wl_t) * win_scale);
    WL = std::min(WL, NR);
    // a fixed window length takes smaller groups until its records and traces fit
    const bool fits = window_loci > 0 ? std::min(wl_r, wl_t) * win_scale >= (double)WL : WL >= 16;
    if (fits && 2.0 * (double)k * ckw * 1.5 <= (double)cbud) break;
    if (k == 1) break;
  }
  nwin = (NR + WL - 1) / WL;
  WL = (NR + nwin - 1) / nwin;  // even windows
  bound.assign(nwin + 1, 0);
  for (int w = 0; w <= nwin; ++w) bound[w] = hl + std::min(NR, w * WL);
  const int ngroups = (n + k - 1) / k;
  last_windows = nwin;
  last_window_loci = WL;
  last_window_groups = ngroups;
  if (debug_mem)
    fprintf(stderr, "[hmc] windowed E-step: %d individuals in %d group(s) of <= %d, %d windows of %d loci; per locus "
            "%.0f record / %.0f trace words (mean), budgets rec %.1f trace %.1f ckpt %.1f GB\n",
            n, ngroups, k, nwin, WL, rmean, tmean, rbud * 4e-9, tbud * 4e-9, cbud * 4e-9);
  // ---- buffers: checkpoints in two slots (the window's input and output)
  const uint64_t ck_slot = std::max<uint64_t>(1024, (uint64_t)((double)k * ckw_max));
  for (int sl = 0; sl < 2; ++sl)
    if (d_ck[sl].n < ck_slot) {
      d_ck[sl].release();
      e = d_ck[sl].ensure(ck_slot);
      if (e == hipErrorOutOfMemory) {  // the stores are dead here: they give way
        (void)hipGetLastError();
        d_trace.release();
        d_rec.release();
        e = d_ck[sl].ensure(ck_slot);
      }
      if (e) return hipfail(e, "checkpoint store");
    }
  bump = true;
  const unsigned long long zero64 = 0;
  std::vector<unsigned long long> h_re_w(n), re_tot(n, 0);  // R_E per window (host sums: a pass can run twice)
  if ((e = d_ck_off.ensure((size_t)n * (nwin + 1))) || (e = d_ck_cursor.ensure(1)) || (e = d_bnd_off.ensure(n)) ||
      (e = d_bnd_n.ensure(n)) || (e = d_node_cursor.ensure(1)) || (e = hipMemsetAsync(d_cost.p, 0, (size_t)n * 4, st)))
    return hipfail(e, "windowed E-step alloc");
  rw.assign((size_t)n * nwin, 0);
  tw.assign((size_t)n * nwin, 0);
  fw.assign((size_t)n * nwin, 0);
  std::vector<int32_t> underflow;  // individuals whose likelihoods underflow: the classic passes (prune mode)
  // trace store: even windows fill it from the bottom, odd windows from the top
  uint64_t tr_lo = 0, tr_hi = 0;

  bool gc_pending = false;
  std::vector<int32_t> gc_ids;  // the collection's individuals

  // Value pass of window w over ids[0, k_) (trace regions in tbv).
  auto values = [&](int w, const int32_t *ids, int k_) -> int {
    hipError_t e2;
    int rc2;
    double rsum = 0, tsum = 0;
    int fgrp = 1;
    for (int q = 0; q < k_; ++q) {
      rsum += (double)rw[(size_t)ids[q] * nwin + w];
      tsum += (double)tw[(size_t)ids[q] * nwin + w];
      fgrp = std::max(fgrp, (int)fw[(size_t)ids[q] * nwin + w]);
    }
    fgrp = std::min(fcap, (fgrp + 63) & ~63);
    const int wl = bound[w + 1] - bound[w];
    const bool heavy = rsum / ((double)k_ * wl) > 1500.0;
    const int per_cu = (k_ + dev_cu - 1) / dev_cu;
    // heavy groups whose mean frontier passes 1 000 states take half a CU per
    // individual, 8 x 2 (cfg 4's E1, ~1 600 states per locus: 4 x 4 -> 16 x 1,
    // values 14.3 -> 13.4-13.7 s in round 5; 16 x 1 -> 8 x 2 in round 6, 12.48
    // -> 11.96 s at the same 80-loci windows,
    // profiles/r06/cfg4/cfg4_rank0_value_shapes_fixed80.log; cfg 3's E1, ~430:
    // 4 x 4 stays — 16 x 1 there: 270-300 instead of ~215 ms per window, E1
    // values 2.10 -> 2.75 s)
    const double fmean = (tsum / std::max(1.0, (double)k_ * wl) - 2.0) / (1.0 + S);
    const bool small_heavy = heavy && (per_cu < 4 || (vp_nw == 0 && fmean > 1000.0));
    const int sh_ipc = per_cu < 4 ? per_cu : 2;
    const int vnw = vp_nw > 0 ? vp_nw : (small_heavy ? 16 / sh_ipc : (heavy ? 4 : (k_ >= 32 * dev_cu ? 1 : (k_ >= 8 * dev_cu ? 2 : 3))));
    // (heavy groups of five or more per CU: 4 x 5 on the 5-wave build — cfg 3's
    // E1 windows 1 917-1 921 -> 1 891 ms, profiles/r06/ab/value_shapes_e1_cfg3.log)
    const int vipc = vp_ipc > 0 ? vp_ipc
                                : (small_heavy ? sh_ipc
                                               : (vnw == 1 ? 16 : (vnw >= 8 ? 2 : (vnw >= 4 ? (per_cu >= 5 ? 5 : 4) : 8))));
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
    v.w.ck_in = d_ck[w & 1].p;
    v.w.ck_out = d_ck[(w + 1) & 1].p;
    v.w.ck_cap = d_ck[(w + 1) & 1].n;
    v.w.ck_cursor = d_ck_cursor.p;
    v.w.ck_off = d_ck_off.p;
    v.w.ck_write = true;
    hipEventRecord(ev[0], st);
    if ((e2 = launch_estep_values(v, grid2, vnw, false, vwpe, st, pair))) return hipfail(e2, "estep_values launch");
    hipEventRecord(ev[1], st);
    if ((rc2 = read_status({}, 0, true))) return rc2;
    hipEventElapsedTime(&ms, ev[0], ev[1]);
    ms_s2 += ms;
    ++n_value_passes;
    if (debug_mem)
      fprintf(stderr, "[hmc] window %d/%d: value pass %d individuals, %d x %d per CU, %.1f ms\n", w + 1, nwin, k_, vnw, vipc, ms);
    for (int q = 0; q < k_; ++q) {
      const int s2 = h_status[ids[q]];
      if (s2 == EST_OVERFLOW_TRACE) return fail(HMC_EHIP, "trace store overflow with exact sizes (window %d)", w);
      if (s2 != EST_OK && s2 != EST_UNRESOLVED && s2 != EST_NEEDS_EXACT)
        return fail(HMC_EHIP, "windowed value pass: status %d (individual %d, window %d)", s2, i0 + ids[q], w);
    }
    return HMC_OK;
  };

  // One window over the group `grp`: the structure pass (records bump-allocated
  // from the record store), then the value passes; an individual whose window
  // records did not fit runs the window again once the others' records are
  // dead.  Traces go to the window's half of the trace store.  Individuals
  // that die (no resolution) or underflow leave `grp`.
  auto window = [&](int w, std::vector<int32_t> &grp) -> int {
    std::vector<int32_t> todo(grp), dead;
    bool first = true;
    // heaviest first within the window (each pass ends on its slowest
    // individual): by the traces of the window before, a proxy for this one
    if (w > 0)
      std::stable_sort(todo.begin(), todo.end(), [&](int32_t x, int32_t y) {
        return tw[(size_t)x * nwin + w - 1] > tw[(size_t)y * nwin + w - 1];
      });
    {
      int fprev = probe_fmax;
      if (w > 0)
        for (int bi : grp) fprev = std::max(fprev, fw[(size_t)bi * nwin + w - 1]);
      wfcap = std::max(std::min(4096, fcap), std::min(fcap, next_pow2(2 * std::max(fprev, 1))));
    }
    if ((e = hipMemcpyAsync(d_ck_cursor.p, &zero64, 8, hipMemcpyHostToDevice, st))) return hipfail(e, "windowed E-step");
    if (w % 2 == 0) tr_lo = 0;
    else tr_hi = d_trace.n;
    while (!todo.empty()) {
      if ((e = hipMemsetAsync(d_rec_cursor.p, 0, 8, st))) return hipfail(e, "windowed E-step");
      if ((rc = structure(w, todo.data(), (int)todo.size(), first, 0, true))) return rc;
      if (first) {  // a checkpoint slot that filled up: twice the size, the pass again
        bool ckf = false;
        for (int bi : todo) ckf = ckf || h_status[bi] == EST_OVERFLOW_CKPT;
        if (ckf) {
          DevBuf<uint32_t> &o = d_ck[(w + 1) & 1];
          const size_t want = o.n * 2;
          o.release();
          if ((e = o.ensure(want)) || (e = hipMemcpyAsync(d_ck_cursor.p, &zero64, 8, hipMemcpyHostToDevice, st)))
            return hipfail(e, "checkpoint store");
          if (debug_mem) fprintf(stderr, "[hmc] window %d/%d: checkpoint slot full, %.2f GB\n", w + 1, nwin, want * 4e-9);
          continue;
        }
        // a frontier or contribution list past the pass's capacities: larger
        // capacities and the window again (its checkpoints are intact)
        bool grow = false;
        for (int bi : todo) {
          const int s = h_status[bi];
          if (s == EST_NO_HEAD_PATTERN) return fail(HMC_ENOPATTERN, "Can not find matching pattern!");
          if (s == EST_OVERFLOW_FRONTIER || s == EST_OVERFLOW_CONTRIB) grow = true;
        }
        if (grow) {
          // as restart_status: fail only when the capacity that overflowed was
          // already the largest (F_MAX itself is tried), contributions bounded
          // like ccap1 (INT32_MAX / 2)
          bool f_over = false, c_over = false;
          for (int bi : todo) {
            f_over = f_over || h_status[bi] == EST_OVERFLOW_FRONTIER;
            c_over = c_over || h_status[bi] == EST_OVERFLOW_CONTRIB;
          }
          if (f_over && wfcap >= F_MAX) return fail(HMC_EUNSUPPORTED, "frontier exceeds %d states", F_MAX);
          if (c_over && (int64_t)ccap_mult * wfcap >= INT32_MAX / 2)
            return fail(HMC_EUNSUPPORTED, "contributions of one locus exceed %d", INT32_MAX / 2);
          if (f_over) {
            wfcap = (int)std::min<int64_t>(F_MAX, (int64_t)wfcap * 4);
            fcap = std::max(fcap, wfcap);
          }
          if (c_over) ccap_mult *= 2;
          if (debug_mem) fprintf(stderr, "[hmc] window %d/%d: capacities %d states x %d, the window again\n", w + 1, nwin, wfcap, ccap_mult);
          if ((e = hipMemcpyAsync(d_ck_cursor.p, &zero64, 8, hipMemcpyHostToDevice, st))) return hipfail(e, "windowed E-step");
          continue;
        }
        if ((e = hipMemcpyAsync(h_re_w.data(), d_re.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
            (e = sync_st()))
          return hipfail(e, "windowed E-step");
        for (int bi : todo) re_tot[bi] += h_re_w[bi];
      }
      std::vector<int32_t> ok, deferred;
      for (int bi : todo) {
        const int s = h_status[bi];
        if ((rc = restart_status(s))) return rc;
        if (s == EST_OVERFLOW_CKPT) return fail(HMC_EHIP, "checkpoint slot overflow after growth (window %d)", w);
        if (first) {
          rw[(size_t)bi * nwin + w] = hr[bi];
          tw[(size_t)bi * nwin + w] = ht[bi];
          fw[(size_t)bi * nwin + w] = hf[bi];
        }
        (s == EST_OVERFLOW_REC ? deferred : ok).push_back(bi);
      }
      // traces of this window: exact sizes, bottom-up (even windows) or
      // top-down (odd) in the store, clear of the window before
      uint64_t t = 0;
      for (int bi : ok) t += tw[(size_t)bi * nwin + w];
      if (tr_lo + t > tr_hi) {  // two windows of traces do not fit: smaller windows, the E-step again
        win_scale *= 0.6;
        if (win_scale < 1e-3)
          return fail(HMC_ENOMEM, "windowed E-step: the traces of one window of %d loci exceed the trace store", WL);
        if (debug_mem) fprintf(stderr, "[hmc] windowed E-step: traces of two windows exceed the store; windows x0.6, restart\n");
        return ESTEP_RESTART;
      }
      std::fill(tbv.begin(), tbv.end(), 0ull);
      for (int bi : ok) {
        const uint64_t need = tw[(size_t)bi * nwin + w];
        if (w % 2 == 0) {
          tbv[bi] = tr_lo;
          tr_lo += need;
        } else {
          tr_hi -= need;
          tbv[bi] = tr_hi;
        }
      }
      // the value pass by this window's own record words, heaviest first
      std::stable_sort(ok.begin(), ok.end(), [&](int32_t x, int32_t y) {
        return rw[(size_t)x * nwin + w] > rw[(size_t)y * nwin + w];
      });
      if (!ok.empty() && (rc = values(w, ok.data(), (int)ok.size()))) return rc;
      for (int bi : ok) {
        const int s2 = h_status[bi];
        if (s2 == EST_NEEDS_EXACT) underflow.push_back(bi);
        if (s2 != EST_OK) dead.push_back(bi);
      }
      if (!first && deferred.size() == todo.size())
        return fail(HMC_ENOMEM, "windowed E-step: one individual's records of window %d exceed the record store", w);
      todo.swap(deferred);
      first = false;
    }
    if (!dead.empty()) {  // out of the later windows and the collections
      std::vector<char> gone(n, 0);
      for (int bi : dead) gone[bi] = 1;
      std::vector<int32_t> keep;
      for (int bi : grp)
        if (!gone[bi]) keep.push_back(bi);
      grp.swap(keep);
    }
    return HMC_OK;
  };

  // Collection of window w - 1 (the survivors of every list entry at the end
  // of window w) over `grp`, after window w's value pass, a wavefront per
  // individual.  (Run beside window w + 1's structure pass on a stream of its
  // own it made that pass 50-60 % slower, more than the collection's own time:
  // both are latency-bound on the same CUs.)  A node store that fills up is
  // grown (contents kept) and the individuals that did not fit run again.
  int gc_w = 0;
  auto collect_launch = [&](int w, const std::vector<int32_t> &grp) -> int {
    gc_w = w;
    const int lo0 = bound[w - 1], mid = bound[w], hi1 = bound[w + 1];
    uint64_t mwords = 0;
    int fb = 1;
    for (int bi : grp) {
      mwords = std::max<uint64_t>(mwords, (tw[(size_t)bi * nwin + w - 1] + tw[(size_t)bi * nwin + w]) / 32);
      fb = std::max(fb, std::max(fw[(size_t)bi * nwin + w - 1], fw[(size_t)bi * nwin + w]));
    }
    if (grp.empty()) return HMC_OK;
    const int max_words = (int)(((uint64_t)fb * S + 31) / 32) + 1;
    const size_t stride = (size_t)(hi1 - lo0 + 1) + 2 * (size_t)(max_words + 1) + mwords + (size_t)(hi1 - lo0) + 64;
    const int grid = std::max(1, std::min((int)grp.size(), dev_cu * 16));  // a wavefront per individual
    gc_ids = grp;  // heaviest collections first: the traces of the two windows
    std::stable_sort(gc_ids.begin(), gc_ids.end(), [&](int32_t x, int32_t y) {
      return tw[(size_t)x * nwin + w - 1] + tw[(size_t)x * nwin + w] > tw[(size_t)y * nwin + w - 1] + tw[(size_t)y * nwin + w];
    });
    hipError_t e2;
    if ((e2 = d_gc_scr.ensure(stride * grid)) || (e2 = d_gc_order.ensure(n)) || (e2 = d_gc_status.ensure(n)) ||
        (e2 = d_gc_nextq.ensure(1)) ||
        (e2 = hipMemcpyAsync(d_gc_order.p, gc_ids.data(), gc_ids.size() * 4, hipMemcpyHostToDevice, st)) ||
        (e2 = hipMemsetAsync(d_gc_status.p, 0, (size_t)n * 4, st)) || (e2 = hipMemsetAsync(d_gc_nextq.p, 0, 4, st)))
      return hipfail(e2, "trace collection");
    TraceGcArgs g;
    g.L = L;
    g.S = S;
    g.head_len = hl;
    g.order = d_gc_order.p;
    g.n_order = (int)gc_ids.size();
    g.next_q = d_gc_nextq.p;
    g.trace = d_trace.p;
    g.loc_off = d_loc_off.p;
    g.lo0 = lo0;
    g.mid = mid;
    g.hi1 = hi1;
    g.scratch = d_gc_scr.p;
    g.scratch_stride = stride;
    g.max_words = max_words;
    g.nodes = d_nodes.p;
    g.node_cap = d_nodes.n / 3;
    g.node_cursor = d_node_cursor.p;
    g.bnd_off = d_bnd_off.p;
    g.bnd_n = d_bnd_n.p;
    g.status = d_gc_status.p;
    hipEventRecord(ev[4], st);
    if ((e2 = launch_estep_trace_gc(g, grid, st, 1))) return hipfail(e2, "estep_trace_gc launch");
    hipEventRecord(ev[5], st);
    gc_pending = true;
    if (debug_mem)
      fprintf(stderr, "[hmc] window %d/%d: collection of window %d for %zu individuals\n", w + 1, nwin, w, gc_ids.size());
    return HMC_OK;
  };
  std::function<int()> collect_finish;
  collect_finish = [&]() -> int {
    if (!gc_pending) return HMC_OK;
    gc_pending = false;
    hipError_t e2;
    std::vector<int32_t> gs(n);
    if ((e2 = hipMemcpyAsync(gs.data(), d_gc_status.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
        (e2 = sync_st()))
      return hipfail(e2, "trace collection");
    hipEventElapsedTime(&ms, ev[4], ev[5]);
    ms_ck += ms;
    ms_s2 += ms;
    std::vector<int32_t> again;  // node store full: grown (contents kept), those individuals again
    for (int bi : gc_ids) {
      if (gs[bi] == EST_GC_MISS) return fail(HMC_EHIP, "trace collection: a survivor's predecessor is missing (individual %d)", i0 + bi);
      if (gs[bi] == EST_OVERFLOW_NODES) again.push_back(bi);
    }
    if (debug_mem)
      fprintf(stderr, "[hmc] collection for %zu individuals: %.1f ms%s\n", gc_ids.size(), ms, again.empty() ? "" : " (node store full: grows)");
    if (!again.empty()) {
      unsigned long long used = 0;
      if ((e2 = hipMemcpyAsync(&used, d_node_cursor.p, 8, hipMemcpyDeviceToHost, st)) || (e2 = sync_st()))
        return hipfail(e2, "trace collection");
      used = std::min<unsigned long long>(used, d_nodes.n / 3);
      if ((e2 = hipMemcpyAsync(d_node_cursor.p, &used, 8, hipMemcpyHostToDevice, st)) ||
          (e2 = d_nodes.grow_keep(d_nodes.n * 2, used * 3, st)))
        return hipfail(e2, "trace survivor nodes");
      int rc2;
      if ((rc2 = collect_launch(gc_w, again))) return rc2;
      return collect_finish();
    }
    return HMC_OK;
  };

  std::vector<unsigned long long> rec_all(n, 0);
  for (int g = 0; g < ngroups; ++g) {
    std::vector<int32_t> grp(order.begin() + (std::ptrdiff_t)g * k, order.begin() + std::min<size_t>(order.size(), (size_t)(g + 1) * k));
    const unsigned long long node0 = 0;
    if ((e = hipMemcpyAsync(d_node_cursor.p, &node0, 8, hipMemcpyHostToDevice, st))) return hipfail(e, "windowed E-step");
    if (nwin >= 3 && d_nodes.n == 0 && (e = d_nodes.ensure(std::max<size_t>(3 << 20, (size_t)3 * grp.size() * NR * 16))))
      return hipfail(e, "trace survivor nodes");
    {  // the record store (one window, bump-allocated) and the trace store (two windows)
      double tsum = 0;
      for (int bi : grp) (void)bi;
      tsum = 2.0 * (double)grp.size() * WL * tmean * 1.35 + 4.0 * (1 << 20);
      if ((rc = ensure_store(d_rec, (uint64_t)std::min<double>((double)rbud, (double)grp.size() * WL * rmean * 1.3 + (1 << 22)), rbud,
                             "record store")) ||
          (rc = ensure_store(d_trace, (uint64_t)std::min<double>((double)tbud, tsum), tbud, "trace store")))
        return rc;
    }
    tr_lo = 0;
    tr_hi = d_trace.n;
    for (int w = 0; w < nwin; ++w) {
      if ((rc = window(w, grp))) return rc;
      if (w >= 1 && w < nwin - 1 && ((rc = collect_launch(w, grp)) || (rc = collect_finish()))) return rc;
    }
    // the traceback: the last two windows' traces, then the survivors' chains
    if (!grp.empty()) {
      TracebackArgs t;
      t.L = L;
      t.S = S;
      t.head_len = hl;
      t.nbatch = (int)grp.size();
      if ((rc = upload_order(d_order2, grp.data(), (int)grp.size()))) return rc;
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
      t.full_lo = nwin >= 3 ? bound[nwin - 2] : 0;
      t.nodes = d_nodes.p;
      t.bnd_off = d_bnd_off.p;
      t.bnd_n = d_bnd_n.p;
      hipEventRecord(ev[2], st);
      if ((e = launch_traceback(t, 0, st))) return hipfail(e, "traceback");
      hipEventRecord(ev[3], st);
      if ((e = sync_st())) return hipfail(e, "traceback");
      hipEventElapsedTime(&ms, ev[2], ev[3]);
      ms_tb += ms;
    }
    for (int q = g * k; q < std::min(n, (g + 1) * k); ++q) {
      const int bi = order[q];
      for (int w = 0; w < nwin; ++w) rec_all[bi] += rw[(size_t)bi * nwin + w];
    }
  }
  if ((e = hipMemcpyAsync(d_re.p, re_tot.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)) || (e = sync_st()))
    return hipfail(e, "windowed E-step");
  // individuals whose forward likelihoods underflow: the classic passes, which
  // rebuild their structure with extend()'s forward test (prune mode)
  if (!underflow.empty()) {
    std::sort(underflow.begin(), underflow.end(), [&](int x, int y) { return h_cost[x] > h_cost[y]; });
    const int saved = window_mode;
    window_mode = WIN_NEVER;
    rc = estep_split(underflow);
    window_mode = saved;
    if (rc) return rc;
    // estep_split left prev_rneed = its own needs (non-zero only for the
    // underflow individuals): keep every other individual's windowed record
    // words, or the next E-step would estimate 64 words for them and re-run
    // nearly everyone's structure pass
    if (prev_rneed.size() == rec_all.size())
      for (int bi : underflow) rec_all[bi] = prev_rneed[bi];
  }
  prev_rneed.swap(rec_all);  // record words per individual (the next E-step's estimates at this scale)
  prev_P = P;
  return HMC_OK;
}

}  // namespace hmc
