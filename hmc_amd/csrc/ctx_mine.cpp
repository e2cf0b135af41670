// ctx_mine.cpp — Ctx members: the sampling M-step: PatternManager::findPatternByFreq / ByNum / Block on the device.
#include "ctx.hpp"

namespace hmc {

int Ctx::grow_nodes(size_t need_global, size_t used_global) {
  const size_t need = need_global - (size_t)wbase, used = used_global - (size_t)wbase;
  if (need <= node_cap) return HMC_OK;
  // doubling (each growth re-maps and copies 15 arrays)
  size_t cap = std::max<size_t>(need, 2 * node_cap);
  hipError_t e;
#define G(b)                                                                 \
if ((e = b.grow_keep(cap, used, st)) == hipErrorOutOfMemory && (d_trace.p || d_rec.p)) { \
  (void)hipGetLastError();                                                   \
  d_trace.release();                                                         \
  d_rec.release();                                                           \
  e = b.grow_keep(cap, used, st);                                            \
}                                                                            \
if (e) { nodes_oom = e == hipErrorOutOfMemory; return hipfail(e, "grow_nodes"); }
  G(n_parent) G(n_start) G(n_child_base) G(n_link) G(n_allele) G(n_flags) G(n_freq) G(n_prefix) G(n_tp) G(n_sum)
  G(n_cnt) G(n_size) G(n_pos) G(n_list_off) G(n_region)
#undef G
  node_cap = cap;
  return HMC_OK;
}

MineArgs Ctx::mine_args(bool genotype) const {
  MineArgs a;
  a.L = pan.L;
  a.amax = pan.amax;
  a.genotype = genotype;
  if (genotype) {
    a.n_items = nloc();
    a.item_base = i0;
    a.item_stride = pan.N;
  } else {
    a.n_items = H;
    a.item_base = 0;
    a.item_stride = H;
  }
  a.geno_lm = d_geno_lm.p;
  a.samp_lm = d_samp_lm.p;
  a.w = d_w.p;
  a.afreq = d_afreq.p;
  a.anum = d_anum.p;
  a.npos = d_npos.p;
  a.pos_allele = d_pos_allele.p;
  a.rank_of = d_rank_of.p;
  const long long w = wbase;  // global node index g lives at [g - wbase]
  a.parent = n_parent.p - w;
  a.start = n_start.p - w;
  a.allele = n_allele.p - w;
  a.flags = n_flags.p - w;
  a.freq = n_freq.p - w;
  a.prefix = n_prefix.p - w;
  a.tp = n_tp.p - w;
  a.sum = n_sum.p - w;
  a.cnt = n_cnt.p - w;
  a.size = n_size.p - w;
  a.pos = n_pos.p - w;
  a.child_base = n_child_base.p - w;
  a.link = n_link.p - w;
  a.list_off = n_list_off.p - w;
  a.region = n_region.p - w;
  a.r_region = d_r_region.p;
  a.r_child_base = d_r_child_base.p;
  a.rm = d_rm.p;
  return a;
}

int Ctx::mine(int *P_out, uint64_t *rm_out) {
  // HaploModel.cpp:140-144: after an E-step, --exact-estimate re-estimates
  // (estimatePatterns) instead of re-mining the samples
  if (exact_estimate && have_samples && have_model) return estimate_patterns(P_out, rm_out);
  table_on_host = false;
  if (!(num_patterns > 0 && model != 1)) return mine_impl(P_out, rm_out, 0);
  int k = 8;
  while (true) {
    const int rc = mine_impl(P_out, rm_out, k);
    if (rc != MINE_RETRY) return rc;
    k = std::max(bynum_need, 2 * k);
  }
}

int Ctx::mine_impl_body(int *P_out, uint64_t *rm_out, int bynum_rounds) {
  if (!have_panel) return fail(HMC_EARG, "no panel loaded");
  const int L = pan.L;
  hipError_t e;
  hipEventRecord(ev[4], st);
  ms_red = 0;
  n_red_levels = 0;
  // PatternManager::findPatternByFreq argument normalisation (PatternManager.cpp:29-32)
  int mxl = max_len <= 0 ? L : max_len;
  int mnl = std::max(min_len, 1);
  mxl = std::max(mxl, mnl);
  double mf = current_min_freq();
  if (model == 1) {  // MC: findPatternBlock(mc_order+1) (PatternManager.cpp:72-88)
    mnl = mxl = std::max(1, mc_order + 1);
    mf = -1.0;
  }
  if (bynum_rounds > 0) mf = bynum_theta(bynum_rounds);
  if ((e = d_rm.ensure(RM_SLOTS * 16)) || (e = d_totals.ensure(2)) || (e = h_totals.ensure(2)) ||
      (e = d_rsize.ensure(L)) || (e = d_rpos.ensure(L)) || (e = d_r_region.ensure(L)) ||
      (e = hipMemsetAsync(d_rm.p, 0, RM_SLOTS * 16 * 8, st)))
    return hipfail(e, "mine");
  int W = block_width(L, mxl, mnl, bynum_rounds);
  if ((e = d_mine_err.ensure(1)) || (e = hipMemsetAsync(d_mine_err.p, 0, 4, st))) return hipfail(e, "mine");
  wbase = 0;
  long long next_node = 0;  // global index of the next node
  long long id_base = 0;    // patterns of the blocks above
  uint64_t rm_bynum = 0;
  int rc, nblocks = 0;
  mine_touched = true;
  for (int hi = L; hi > 0;) {
    const int lo = std::max(0, hi - W);
    MineBlock mb;
    if ((e = d_rm_save.ensure(RM_SLOTS * 16)) ||
        (e = hipMemcpyAsync(d_rm_save.p, d_rm.p, RM_SLOTS * 16 * 8, hipMemcpyDeviceToDevice, st)))
      return hipfail(e, "mine");
    rc = mine_block(lo, hi, mxl, mnl, mf, bynum_rounds, next_node, id_base, mb, rm_bynum);
    if (rc == MINE_SPLIT) {  // nothing of the block is kept: its R_M counts go, its nodes are overwritten
      if (bynum_rounds > 0 || mnl > 1 || hi - lo <= 1)
        return fail(HMC_ENOMEM, "pattern search: out of device memory (blocks of %d start loci)", hi - lo);
      if ((e = hipMemcpyAsync(d_rm.p, d_rm_save.p, RM_SLOTS * 16 * 8, hipMemcpyDeviceToDevice, st)))
        return hipfail(e, "mine");
      W = std::max(1, (hi - lo + 1) / 2);
      if (debug_mem) fprintf(stderr, "[hmc] mine block [%d, %d): out of memory, %d start loci per block from here\n", lo, hi, W);
      continue;
    }
    if (rc) return rc;
    // the block above this one is no longer needed
    if ((rc = slide_window(mb.first_node, mb.end_node))) return rc;
    next_node = mb.end_node;
    id_base += mb.patterns;
    ++nblocks;
    if (debug_mem && W < L)
      fprintf(stderr, "[hmc] mine block %d: start loci [%d, %d), %lld patterns so far, node window %lld..%lld\n",
              nblocks, lo, hi, id_base, (long long)mb.first_node, (long long)mb.end_node);
    hi = lo;
  }
  {  // before anything is committed: a failed successor walk leaves no table
    int merr = 0;
    if ((e = hipMemcpyAsync(&merr, d_mine_err.p, 4, hipMemcpyDeviceToHost, st)) || (e = sync_st()))
      return hipfail(e, "mine");
    if (merr) return fail(HMC_EUNSUPPORTED, "successor walk left the node window (blocks of %d start loci)", W);
  }
  tree_complete = nblocks == 1;
  P = (int)id_base;
  if (!tree_complete) {  // a partial tree is of no further use (strings come from ppat): give its memory back
    n_parent.release(); n_start.release(); n_child_base.release(); n_link.release(); n_allele.release();
    n_flags.release(); n_freq.release(); n_prefix.release(); n_tp.release(); n_sum.release(); n_cnt.release();
    n_size.release(); n_pos.release(); n_list_off.release(); n_region.release();
    last_mine_window_gb = (double)node_cap * 70.0 / 1e9;
    node_cap = 0;
    wbase = 0;
  } else {
    last_mine_window_gb = (double)node_cap * 70.0 / 1e9;
  }
  std::vector<unsigned long long> rm_slots((size_t)RM_SLOTS * 16);
  if ((e = hipMemcpyAsync(rm_slots.data(), d_rm.p, rm_slots.size() * 8, hipMemcpyDeviceToHost, st)))
    return hipfail(e, "mine");
  hipEventRecord(ev[5], st);
  if ((e = sync_st())) return hipfail(e, "mine");
  // The matching lists of the genotype branch (M0) reach tens of GB at
  // cfg 3 (R_M ~ 10^11 entries); give them back to the E-step's stores.
  for (int k = 0; k < 2; ++k) {
    if (l_idx[k].n * 4 > (4ull << 30)) l_idx[k].release();
    if (l_val[k].n * 8 > (4ull << 30)) l_val[k].release();
  }
  if (debug_mem) {
    size_t fb = 0, tb = 0;
    hipMemGetInfo(&fb, &tb);
    fprintf(stderr, "[hmc] after mining: %d patterns in %d block(s) of %d start loci, %lld nodes; free %.1f GB of %.1f; "
            "node window %.1f GB\n", P, nblocks, W, next_node, fb / 1e9, tb / 1e9, last_mine_window_gb);
  }
  unsigned long long rm = 0;
  for (int k = 0; k < RM_SLOTS; ++k) rm += rm_slots[(size_t)k * 16];
  if (bynum_rounds > 0) rm = rm_bynum;  // the scans of the candidates the rounds generated
  float ms = 0;
  hipEventElapsedTime(&ms, ev[4], ev[5]);
  ms_m = ms;
  have_model = true;
  new_table(true);
  last_mine_blocks = nblocks;
  last_mine_nodes = next_node;
  if (P_out) *P_out = P;
  if (rm_out) *rm_out = rm;
  return HMC_OK;
}

int Ctx::mine_block(int lo, int hi, int mxl, int mnl, double mf, int bynum_rounds, long long node0, long long id_base,
               MineBlock &mb, uint64_t &rm_bynum) {
  const bool genotype = !have_samples;
  const int L = pan.L;
  hipError_t e;
  int rc;
  std::vector<long long> lbeg{0, 0}, lend{0, 0};  // per level node ranges (index = level), global
  long long n1 = 0;
  for (int k = lo; k < hi; ++k) n1 += h_npos[k];
  // Out of device memory for the block's nodes or lists: the block is
  // re-run with half the width (mine_impl).  Ranks agree on it (one flag
  // all-reduced per level), so that all of them split the same block.
  auto oom_split = [&](int rc_in, bool oom) -> int {
    if (multi()) {
      double f = oom ? 1.0 : 0.0;
      hipError_t e2;
      if ((e2 = d_flag.ensure(1)) || (e2 = hipMemcpyAsync(d_flag.p, &f, 8, hipMemcpyHostToDevice, st)))
        return hipfail(e2, "mine");
      if (int r2 = allreduce_sum(d_flag.p, 1)) return r2;
      if ((e2 = hipMemcpyAsync(&f, d_flag.p, 8, hipMemcpyDeviceToHost, st)) || (e2 = sync_st()))
        return hipfail(e2, "mine");
      oom = f > 0.0;
    }
    if (oom) {
      (void)hipGetLastError();
      return MINE_SPLIT;
    }
    return rc_in;
  };
  nodes_oom = false;
  rc = grow_nodes((size_t)std::max<long long>(node0 + n1, 1), (size_t)node0);
  if ((rc = oom_split(rc, rc && nodes_oom))) return rc;
  if (node0 + n1 > (long long)INT32_MAX) return fail(HMC_EUNSUPPORTED, "candidate tree exceeds 2^31 nodes");
  // level-1 nodes of the block's roots (r_child_base of root k) and the
  // roots' child lists: root r owns npos[r] x n_items slots of the next buffer
  unsigned long long next_total = 0;
  {
    const unsigned long long ni = (unsigned long long)mine_args(genotype).n_items;
    std::vector<unsigned long long> rr(hi - lo);
    std::vector<int32_t> rcb(hi - lo);
    long long c = node0;
    for (int k = lo; k < hi; ++k) {
      rr[k - lo] = next_total;
      next_total += (unsigned long long)h_npos[k] * ni;
      rcb[k - lo] = (int32_t)c;
      c += h_npos[k];
    }
    if ((e = hipMemcpyAsync(d_r_region.p + lo, rr.data(), rr.size() * 8, hipMemcpyHostToDevice, st)) ||
        (e = hipMemcpyAsync(d_r_child_base.p + lo, rcb.data(), rcb.size() * 4, hipMemcpyHostToDevice, st)))
      return hipfail(e, "mine");
  }
  lbeg[1] = node0;
  lend[1] = node0 + n1;
  int level = 1;
  long long pbeg = lo, pend = hi;  // level-1 parents are the block's roots
  int cur = 0;                     // list buffer holding the parents' lists
  while (true) {
    const long long cb = lbeg[level], ce = lend[level];
    const int nlev = (int)(ce - cb);
    const int nxt = cur ^ 1;  // children's lists are written here during the count
    const unsigned long long list_bytes = next_total * (genotype ? 12ull : 4ull);
    if (mine_list_cap && list_bytes > mine_list_cap) {
      if ((rc = oom_split(HMC_OK, true))) return rc;
    }
    e = ensure_or_release(l_idx[nxt], std::max<unsigned long long>(next_total, 1));
    if (!e && genotype) e = ensure_or_release(l_val[nxt], std::max<unsigned long long>(next_total, 1));
    if ((rc = oom_split(e ? hipfail(e, "mine lists") : HMC_OK, e == hipErrorOutOfMemory))) return rc;
    MineArgs a = mine_args(genotype);
    a.lout_idx = l_idx[nxt].p;
    a.lout_val = genotype ? l_val[nxt].p : nullptr;
    a.denom = genotype ? (double)pan.N : total_weight;
    a.min_freq = mf;
    a.min_len = mnl;
    a.max_len = mxl;
    a.lin_idx = level == 1 ? nullptr : l_idx[cur].p;
    a.lin_val = level == 1 ? nullptr : l_val[cur].p;
    hipEvent_t dm0 = nullptr, dm1 = nullptr;
    if (diag_mine) {
      hipEventCreate(&dm0);
      hipEventCreate(&dm1);
      hipEventRecord(dm0, st);
    }
#ifdef HMC_STAMPS
    if (diag_mine) {
      d_mstamps.ensure((size_t)(pend - pbeg) * 8);
      hipMemsetAsync(d_mstamps.p, 0, (size_t)(pend - pbeg) * 64, st);
      a.stamps = d_mstamps.p;
    }
#endif
    if (multi() && reduction == RED_ORDERED) {
      // every rank scans its items and writes the children's lists at once;
      // then rank r continues every child's sum from ranks 0..r-1 (items in
      // order) over its lists and passes it on
      if ((e = launch_mine_count(a, level, (int)pbeg, (int)pend, st))) return hipfail(e, "mine_count");
      hipEventRecord(ev[6], st);
      if ((rc = ordered_chain(n_sum.p + (cb - wbase), nlev, [&]() -> int {
             hipError_t e2 = launch_mine_sum(a, (int)cb, (int)ce, st);
             return e2 ? hipfail(e2, "mine_sum") : HMC_OK;
           })))
        return rc;
      hipEventRecord(ev[7], st);
      red_timed = true;
    } else if ((e = launch_mine_count(a, level, (int)pbeg, (int)pend, st))) {
      return hipfail(e, "mine_count");
    }
    if (diag_mine) {  // per-level list statistics of the parents (diagnostic)
      hipEventRecord(dm1, st);
      sync_st();
      float ms = 0;
      hipEventElapsedTime(&ms, dm0, dm1);
      size_t tot_n = 0, max_n = 0, npar = 0;
      if (level == 1) {
        npar = (size_t)(hi - lo);
        tot_n = npar * (size_t)a.n_items;
        max_n = (size_t)a.n_items;
      } else {
        std::vector<uint32_t> hc((size_t)(pend - pbeg));
        std::vector<uint8_t> hf((size_t)(pend - pbeg));
        hipMemcpy(hc.data(), n_cnt.p + (pbeg - wbase), hc.size() * 4, hipMemcpyDeviceToHost);
        hipMemcpy(hf.data(), n_flags.p + (pbeg - wbase), hf.size(), hipMemcpyDeviceToHost);
        for (size_t q = 0; q < hc.size(); ++q)
          if (hf[q] & 2) {
            ++npar;
            tot_n += hc[q];
            max_n = std::max<size_t>(max_n, hc[q]);
          }
      }
      fprintf(stderr, "mine block [%d,%d) level %2d: %7zu ext parents of %7lld, entries %9zu, max list %7zu, "
              "mine_count %.3f ms\n", lo, hi, level, npar, pend - pbeg, tot_n, max_n, ms);
#ifdef HMC_STAMPS
      unsigned long long hs[8] = {};
      std::vector<unsigned long long> hv((size_t)(pend - pbeg) * 8);
      hipMemcpy(hv.data(), d_mstamps.p, hv.size() * 8, hipMemcpyDeviceToHost);
      for (size_t q = 0; q < hv.size(); ++q) hs[q % 8] += hv[q];
      const double nwv = hs[5] ? (double)hs[5] : 1.0;
      fprintf(stderr, "   per wave (cycles): view %.0f  loads %.0f  compact %.0f  sum %.0f  epilogue %.0f; waves %llu\n",
              hs[0] / nwv, hs[1] / nwv, hs[2] / nwv, hs[3] / nwv, hs[4] / nwv, hs[5]);
#endif
      hipEventDestroy(dm0);
      hipEventDestroy(dm1);
    }
    if (!(multi() && reduction == RED_ORDERED) && multi()) {
      hipEventRecord(ev[6], st);
      if ((rc = allreduce_sum(n_sum.p + (cb - wbase), nlev))) return rc;
      hipEventRecord(ev[7], st);
      red_timed = true;
    }
    if ((e = s_ext.ensure(nlev)) || (e = s_child.ensure(nlev))) return hipfail(e, "mine");
    const size_t tmpb = mine_scan_tmp_bytes(nlev);
    if ((e = s_tmp.ensure(tmpb))) return hipfail(e, "mine");
    if ((e = launch_mine_finalize(a, level, (int)cb, (int)ce, s_ext.p, s_child.p, st))) return hipfail(e, "mine_finalize");
    if ((e = launch_mine_offsets(a, (int)cb, (int)ce, s_ext.p, s_child.p, (int)ce, s_tmp.p, s_tmp.n, d_totals.p, st)))
      return hipfail(e, "mine_offsets");
    const unsigned long long *tot = h_totals.p;
    if ((e = hipMemcpyAsync(h_totals.p, d_totals.p, 16, hipMemcpyDeviceToHost, st)) || (e = sync_st()))
      return hipfail(e, "mine");
    if (red_timed) {  // this level's cross-rank reduction (the stream has drained)
      float ms = 0;
      hipEventElapsedTime(&ms, ev[6], ev[7]);
      ms_red += ms;
      ++n_red_levels;
      red_timed = false;
    }
    next_total = tot[0];  // list slots the next level's children need
    if (tot[1] > (unsigned long long)INT32_MAX - (unsigned long long)ce)
      return fail(HMC_EUNSUPPORTED, "candidate tree exceeds 2^31 nodes at length %d", level + 1);
    const long long nnext = (long long)tot[1];
    cur = nxt;
    if (nnext == 0) break;
    pbeg = cb;
    pend = ce;
    ++level;
    lbeg.push_back(ce);
    lend.push_back(ce + nnext);
    nodes_oom = false;
    rc = grow_nodes((size_t)(ce + nnext), (size_t)ce);
    if ((rc = oom_split(rc, rc && nodes_oom))) return rc;
  }
  const int maxlev = level;
  MineArgs a = mine_args(genotype);
  long long Pb = 0;
  if (bynum_rounds > 0) {  // one block: the node window starts at 0
    rc = bynum_replay(a, (int)lend[maxlev], mnl, mxl, bynum_rounds, rm_bynum);
    if (rc) return rc;
    Pb = P;
  } else {
    // DFS pre-order ids from subtree sizes
    for (int lv = maxlev; lv >= 1; --lv)
      if ((e = launch_mine_size(a, lv, (int)lbeg[lv], (int)lend[lv], st))) return hipfail(e, "mine_size");
    if ((e = launch_mine_root_size(a, d_rsize.p, lo, hi, st))) return hipfail(e, "mine_root_size");
    std::vector<uint32_t> rsize(hi - lo), rpos(hi - lo);
    if ((e = hipMemcpyAsync(rsize.data(), d_rsize.p + lo, rsize.size() * 4, hipMemcpyDeviceToHost, st)) ||
        (e = sync_st()))
      return hipfail(e, "mine");
    uint64_t acc = (uint64_t)id_base;
    for (int s = hi - 1; s >= lo; --s) {  // roots popped from the back: start L-1 first
      rpos[s - lo] = (uint32_t)acc;
      acc += rsize[s - lo];
    }
    if (acc > (uint64_t)INT32_MAX) return fail(HMC_EUNSUPPORTED, "too many patterns (%llu)", (unsigned long long)acc);
    Pb = (long long)acc - id_base;
    if ((e = hipMemcpyAsync(d_rpos.p + lo, rpos.data(), rpos.size() * 4, hipMemcpyHostToDevice, st)))
      return hipfail(e, "mine");
    if ((e = launch_mine_pos(a, 1, lo, hi, d_rpos.p, st))) return hipfail(e, "mine_pos");
    for (int lv = 2; lv <= maxlev; ++lv)
      if ((e = launch_mine_pos(a, lv, (int)lbeg[lv - 1], (int)lend[lv - 1], d_rpos.p, st))) return hipfail(e, "mine_pos");
  }
  if ((rc = grow_table((size_t)(id_base + Pb), (size_t)id_base))) return rc;
  PatternTable t = table();
  std::vector<int> lb(maxlev + 2);  // the block's level ranges (global node indices < 2^31)
  for (int lv = 1; lv <= maxlev; ++lv) lb[lv] = (int)lbeg[lv];
  lb[maxlev + 1] = (int)lend[maxlev];
  if ((e = d_lev_begin.ensure(lb.size())) ||
      (e = hipMemcpyAsync(d_lev_begin.p, lb.data(), lb.size() * 4, hipMemcpyHostToDevice, st)) ||
      (e = launch_mine_emit(a, d_lev_begin.p, maxlev, lb[maxlev + 1] - lb[1], t, st)))
    return hipfail(e, "mine_emit");
  for (int lv = 1; lv <= maxlev; ++lv)
    if ((e = launch_mine_succ_level(a, t, lv, (int)lbeg[lv], (int)lend[lv], (int32_t)wbase, d_mine_err.p, st)))
      return hipfail(e, "mine_succ");
  if (lo == 0) {
    head_len = mnl;
    P = (int)(id_base + Pb);  // the head pairs' lookups see the whole table
    if ((rc = build_heads_from_nodes(a, mnl <= maxlev ? (int)lbeg[mnl] : 0, mnl <= maxlev ? (int)lend[mnl] : 0))) return rc;
  }
  mb.first_node = node0;
  mb.end_node = lend[maxlev];
  mb.patterns = Pb;
  return HMC_OK;
}

int Ctx::grow_table(size_t n, size_t used) {
  hipError_t e;
  n = std::max<size_t>(n, 1);
  const size_t A = (size_t)pan.amax;
  auto grow = [&]() -> hipError_t {
    hipError_t r;
    if ((r = t_start.grow_keep(n, used, st)) || (r = t_len.grow_keep(n, used, st)) ||
        (r = t_node.grow_keep(n, used, st)) || (r = t_freq.grow_keep(n, used, st)) ||
        (r = t_prefix.grow_keep(n, used, st)) || (r = t_tp.grow_keep(n, used, st)) ||
        (r = t_last.grow_keep(n, used, st)) || (r = t_ppat.grow_keep(n, used, st)) ||
        (r = t_succ.grow_keep(n * A, used * A, st)))
      return r;
    return hipSuccess;
  };
  if ((e = grow()) == hipErrorOutOfMemory) {
    // the table grows after a block's search: its matching lists (sized by
    // the block's largest level) and the E-step stores can go
    (void)hipGetLastError();
    for (int k = 0; k < 2; ++k) {
      l_idx[k].release();
      l_val[k].release();
    }
    d_trace.release();
    d_rec.release();
    e = grow();
  }
  if (e) return hipfail(e, "grow_table");
  return HMC_OK;
}

PatternTable Ctx::table() const {
  PatternTable t;
  t.start = t_start.p;
  t.len = t_len.p;
  t.node = t_node.p;
  t.ppat = t_ppat.p;
  t.freq = t_freq.p;
  t.prefix = t_prefix.p;
  t.tp = t_tp.p;
  t.last = t_last.p;
  t.succ = t_succ.p;
  return t;
}

int Ctx::set_heads(const std::vector<std::pair<uint32_t, uint8_t>> &heads /* (id, allele at 0) */) {
  std::vector<uint32_t> ids, pat0(pan.amax + 1, NONE);
  for (auto &h : heads) {
    ids.push_back(h.first);
    pat0[h.second] = h.first;
  }
  std::sort(ids.begin(), ids.end());
  for (int x = 0; x < pan.amax; ++x)
    if (pat0[x] != NONE) { pat0[pan.amax] = pat0[x]; break; }
  n_head = (int)ids.size();
  hipError_t e;
  if ((e = d_head_ids.ensure(std::max<size_t>(ids.size(), 1))) || (e = d_head_pat0.ensure(pat0.size())))
    return hipfail(e, "set_heads");
  if (!ids.empty() &&
      (e = hipMemcpyAsync(d_head_ids.p, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, st)))
    return hipfail(e, "set_heads");
  if ((e = hipMemcpyAsync(d_head_pat0.p, pat0.data(), pat0.size() * 4, hipMemcpyHostToDevice, st)) ||
      (e = sync_st()))
    return hipfail(e, "set_heads");
  return HMC_OK;
}

int Ctx::bynum_replay(const MineArgs &, int ntot, int mnl, int mxl, int, uint64_t &rm_out) {
  const int L = pan.L;
  hipError_t e;
  std::vector<uint8_t> fl(ntot);
  std::vector<int32_t> cb(ntot), stt(ntot);
  std::vector<double> fr(ntot);
  std::vector<uint32_t> cnt(ntot);
  if (ntot > 0 &&
      ((e = hipMemcpyAsync(fl.data(), n_flags.p, (size_t)ntot, hipMemcpyDeviceToHost, st)) ||
       (e = hipMemcpyAsync(cb.data(), n_child_base.p, (size_t)ntot * 4, hipMemcpyDeviceToHost, st)) ||
       (e = hipMemcpyAsync(stt.data(), n_start.p, (size_t)ntot * 4, hipMemcpyDeviceToHost, st)) ||
       (e = hipMemcpyAsync(fr.data(), n_freq.p, (size_t)ntot * 8, hipMemcpyDeviceToHost, st)) ||
       (e = hipMemcpyAsync(cnt.data(), n_cnt.p, (size_t)ntot * 4, hipMemcpyDeviceToHost, st)) ||
       (e = sync_st())))
    return hipfail(e, "bynum");
  const unsigned long long n_items = (unsigned long long)mine_args(!have_samples).n_items;
  struct C { int32_t v; int len; };  // v < 0: root of start -v-1 (the empty pattern)
  std::vector<C> stack, kept;
  std::vector<int32_t> out;
  for (int s0 = 0; s0 < L; ++s0) stack.push_back({-(s0 + 1), 0});  // generateCandidates
  uint64_t rm = 0;
  double theta = 1.0;
  int max_num = num_patterns, last_size = 0;
  // searchPattern(true) at threshold theta (PatternManager.cpp:100-144)
  auto search = [&](int round) -> int {
    kept.clear();
    while (!stack.empty()) {
      const C c = stack.back();
      stack.pop_back();
      const bool root = c.v < 0;
      const int start = root ? -c.v - 1 : stt[c.v];
      const double f = root ? 1.0 : fr[c.v];  // the empty pattern has frequency 1
      const int end = start + c.len;
      if (f >= theta || c.len < mnl) {
        if (end < L && c.len < mxl) {
          if (!root && !(fl[c.v] & NODE_EXT)) return round;  // the mined tree is too shallow
          const int base = root ? [&] { int b = 0; for (int k = 0; k < start; ++k) b += h_npos[k]; return b; }()
                                : cb[c.v];
          const unsigned long long scan = root ? n_items : (cnt[c.v] > 0 ? cnt[c.v] : n_items);
          for (int j = 0; j < h_npos[end]; ++j) {
            stack.push_back({base + j, c.len + 1});
            rm += scan;  // checkFrequencyWithExtension of the new candidate
          }
        }
      }
      if (f >= theta || c.len <= mnl) {
        if (c.len > 0 && c.len >= mnl) out.push_back(c.v);
      } else {
        kept.push_back(c);
      }
    }
    stack.swap(kept);
    return 0;
  };
  int round = 1;
  if (int need = search(round)) { bynum_need = need; return MINE_RETRY; }
  max_num = std::max(max_num, (int)out.size());
  while ((int)out.size() < max_num && theta > 1e-38) {
    if (stack.empty()) break;  // nothing left to accept: later rounds change nothing
    last_size = (int)out.size();
    theta *= 0.9;
    ++round;
    if (int need = search(round)) { bynum_need = need; return MINE_RETRY; }
  }
  if ((int)out.size() > max_num) {
    std::sort(out.begin() + last_size, out.end(), [&](int32_t x, int32_t y) { return fr[x] > fr[y]; });
    out.resize(max_num);
  }
  std::vector<uint32_t> pos(ntot, 0);
  for (int32_t v = 0; v < ntot; ++v) fl[v] &= (uint8_t)~NODE_ACC;
  for (size_t i = 0; i < out.size(); ++i) {
    fl[out[i]] |= NODE_ACC;
    pos[out[i]] = (uint32_t)i;
  }
  if (ntot > 0 &&
      ((e = hipMemcpyAsync(n_flags.p, fl.data(), (size_t)ntot, hipMemcpyHostToDevice, st)) ||
       (e = hipMemcpyAsync(n_pos.p, pos.data(), (size_t)ntot * 4, hipMemcpyHostToDevice, st)) ||
       (e = sync_st())))
    return hipfail(e, "bynum");
  P = (int)out.size();
  rm_out = rm;
  bynum_theta_last = theta;  // m_min_freq after the search (estimatePatterns filters by it)
  return HMC_OK;
}

int Ctx::build_heads_from_nodes(const MineArgs &, int hb, int he) {
  std::vector<std::pair<uint32_t, uint8_t>> heads;
  hf_valid = false;
  h_head_ids.clear();
  h_head_al.clear();
  if (head_len == 1 && pan.L > 0) {
    const int n0 = h_npos[0];
    std::vector<int32_t> rcb(1);
    hipError_t e;
    std::vector<uint8_t> fl(n0), alle(n0);
    std::vector<uint32_t> pos(n0);
    if ((e = hipMemcpyAsync(rcb.data(), d_r_child_base.p, 4, hipMemcpyDeviceToHost, st)) ||
        (e = sync_st()))
      return hipfail(e, "heads");
    if (n0 > 0) {
      const long long r0 = (long long)rcb[0] - wbase;  // physical index of root 0's first child
      if ((e = hipMemcpyAsync(fl.data(), n_flags.p + r0, n0, hipMemcpyDeviceToHost, st)) ||
          (e = hipMemcpyAsync(alle.data(), n_allele.p + r0, n0, hipMemcpyDeviceToHost, st)) ||
          (e = hipMemcpyAsync(pos.data(), n_pos.p + r0, (size_t)n0 * 4, hipMemcpyDeviceToHost, st)) ||
          (e = sync_st()))
        return hipfail(e, "heads");
    }
    for (int k = 0; k < n0; ++k)
      if (fl[k] & NODE_ACC) heads.push_back({pos[k], alle[k]});
  } else if (head_len > 1 && he > hb) {
    // head list = accepted start-0 nodes of level head_len; their alleles by
    // walking parent links (levels 1..head_len are nodes [0, he))
    hipError_t e;
    std::vector<int32_t> par(he), stt(he);
    std::vector<uint8_t> fl(he), alle(he);
    std::vector<uint32_t> pos(he);
    if ((e = hipMemcpyAsync(par.data(), n_parent.p, (size_t)he * 4, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(stt.data(), n_start.p, (size_t)he * 4, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(fl.data(), n_flags.p, (size_t)he, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(alle.data(), n_allele.p, (size_t)he, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(pos.data(), n_pos.p, (size_t)he * 4, hipMemcpyDeviceToHost, st)) ||
        (e = sync_st()))
      return hipfail(e, "heads");
    std::vector<std::pair<uint32_t, std::vector<uint8_t>>> hs;
    for (int v = hb; v < he; ++v) {
      if (stt[v] != 0 || !(fl[v] & NODE_ACC)) continue;
      std::vector<uint8_t> al(head_len);
      int32_t w = v;
      for (int q = head_len - 1; q >= 0; --q) {
        al[q] = alle[w];
        w = par[w];
      }
      hs.push_back({pos[v], al});
    }
    std::sort(hs.begin(), hs.end());
    std::vector<uint8_t> tab((size_t)std::max(P, 1) * head_len, 0);
    for (auto &h : hs) {
      heads.push_back({h.first, h.second[head_len - 1]});
      h_head_ids.push_back(h.first);
      h_head_al.insert(h_head_al.end(), h.second.begin(), h.second.end());
      std::copy(h.second.begin(), h.second.end(), tab.begin() + (size_t)h.first * head_len);
    }
    if ((e = d_head_al.ensure(tab.size())) ||
        (e = hipMemcpyAsync(d_head_al.p, tab.data(), tab.size(), hipMemcpyHostToDevice, st)) ||
        (e = sync_st()))
      return hipfail(e, "heads");
  }
  return set_heads(heads);
}

int Ctx::mine_level(int level, int n, const int32_t *start, const int32_t *alleles, double *freq, uint64_t *scanned) {
  if (!have_panel) return fail(HMC_EARG, "no genotypes loaded");
  if (level < 0 || n < 0 || (n > 0 && (!start || !freq || (level > 0 && !alleles))))
    return fail(HMC_EARG, "mine_level arguments");
  const int L = pan.L;
  if (scanned) *scanned = 0;
  if (n == 0) return HMC_OK;
  if (level == 0) {  // HaploPattern of length 0: frequency 1 (checkFrequency :149-150)
    for (int c = 0; c < n; ++c) freq[c] = 1.0;
    return HMC_OK;
  }
  std::vector<uint8_t> al((size_t)n * level);
  for (int c = 0; c < n; ++c) {
    if (start[c] < 0 || start[c] + level > L) return fail(HMC_EARG, "candidate %d outside the loci", c);
    for (int j = 0; j < level; ++j) {
      const auto &sy = pan.sym[start[c] + j];
      const int32_t a = alleles[(size_t)c * level + j];
      uint8_t ix = 0xFD;  // a symbol the locus does not have: matches only missing alleles
      for (size_t q = 0; q < sy.size(); ++q)
        if (sy[q].first == a) ix = (uint8_t)q;
      al[(size_t)c * level + j] = ix;
    }
  }
  hipError_t e;
  if ((e = d_lv_start.ensure(n)) || (e = d_lv_al.ensure(al.size())) || (e = d_lv_sum.ensure(n)) ||
      (e = hipMemcpyAsync(d_lv_start.p, start, (size_t)n * 4, hipMemcpyHostToDevice, st)) ||
      (e = hipMemcpyAsync(d_lv_al.p, al.data(), al.size(), hipMemcpyHostToDevice, st)))
    return hipfail(e, "mine_level");
  const bool genotype = !have_samples;
  MineArgs a = mine_args(genotype);
  int rc;
  if (multi() && reduction == RED_ORDERED) {
    a.seeded = false;
    if (rank == 0 && (e = launch_mine_scan(a, level, n, d_lv_start.p, d_lv_al.p, d_lv_sum.p, st)))
      return hipfail(e, "mine_scan");
    if ((rc = ordered_chain(d_lv_sum.p, n, [&]() -> int {
           a.seeded = true;
           hipError_t e2 = launch_mine_scan(a, level, n, d_lv_start.p, d_lv_al.p, d_lv_sum.p, st);
           return e2 ? hipfail(e2, "mine_scan") : HMC_OK;
         })))
      return rc;
  } else {
    if ((e = launch_mine_scan(a, level, n, d_lv_start.p, d_lv_al.p, d_lv_sum.p, st))) return hipfail(e, "mine_scan");
    if ((rc = allreduce_sum(d_lv_sum.p, n))) return rc;
  }
  if ((e = hipMemcpyAsync(freq, d_lv_sum.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) || (e = sync_st()))
    return hipfail(e, "mine_level");
  const double denom = genotype ? (double)pan.N : total_weight;  // :178, :190
  for (int c = 0; c < n; ++c) freq[c] = freq[c] / denom;
  if (scanned) *scanned = (uint64_t)n * (uint64_t)a.n_items;
  return HMC_OK;
}
}  // namespace hmc
