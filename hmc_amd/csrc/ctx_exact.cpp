// ctx_exact.cpp — Ctx members: the exact M-step (--exact-estimate): PatternManager::estimatePatterns.
#include "ctx.hpp"

namespace hmc {

int Ctx::spell_table(const std::vector<int32_t> &ln, std::vector<int64_t> &off, std::vector<uint8_t> &al) {
  const int P = this->P;
  std::vector<int32_t> pp(P), node;
  std::vector<uint8_t> last(P);
  hipError_t e;
  if ((e = hipMemcpyAsync(pp.data(), t_ppat.p, (size_t)P * 4, hipMemcpyDeviceToHost, st)) ||
      (e = hipMemcpyAsync(last.data(), t_last.p, (size_t)P, hipMemcpyDeviceToHost, st)) ||
      (e = sync_st()))
    return hipfail(e, "table strings");
  off.assign((size_t)P + 1, 0);
  for (int i = 0; i < P; ++i) off[i + 1] = off[i] + ln[i];
  al.assign((size_t)off[P], 0);
  std::vector<int32_t> par;
  std::vector<uint8_t> alc;
  bool tree_loaded = false;
  for (int i = 0; i < P; ++i) {
    uint8_t *o = al.data() + off[i];
    o[ln[i] - 1] = last[i];
    const int32_t q = pp[i];
    if (ln[i] == 1) continue;
    if (q >= 0 && q < i && ln[q] == ln[i] - 1) {
      std::copy(al.data() + off[q], al.data() + off[q] + ln[q], o);
      continue;
    }
    if (!tree_ok()) return fail(HMC_EUNSUPPORTED, "allele strings of this table are unknown (a table set from outside)");
    if (!tree_loaded) {
      node.resize(P);
      if ((e = hipMemcpyAsync(node.data(), t_node.p, (size_t)P * 4, hipMemcpyDeviceToHost, st)) ||
          (e = sync_st()))
        return hipfail(e, "table strings");
      int nmax = 0;
      for (int k = 0; k < P; ++k) nmax = std::max(nmax, node[k] + 1);
      par.resize(nmax);
      alc.resize(nmax);
      if (nmax && ((e = hipMemcpyAsync(par.data(), n_parent.p, (size_t)nmax * 4, hipMemcpyDeviceToHost, st)) ||
                   (e = hipMemcpyAsync(alc.data(), n_allele.p, (size_t)nmax, hipMemcpyDeviceToHost, st)) ||
                   (e = sync_st())))
        return hipfail(e, "table strings");
      tree_loaded = true;
    }
    int32_t v = node[i];
    for (int k = ln[i] - 1; k >= 0; --k) {
      o[k] = alc[v];
      v = par[v];
    }
  }
  return HMC_OK;
}

int Ctx::table_to_host(Cands &c, std::vector<int32_t> &succ) {
  if (table_on_host) {
    c = ht;
    succ = ht_succ;
    return HMC_OK;
  }
  const int P = this->P, A = pan.amax;
  std::vector<int32_t> st(P), ln(P);
  std::vector<double> fr(P), pre(P), tp(P);
  std::vector<uint32_t> su((size_t)P * A);
  hipError_t e;
  if ((e = hipMemcpyAsync(st.data(), t_start.p, (size_t)P * 4, hipMemcpyDeviceToHost, this->st)) ||
      (e = hipMemcpyAsync(ln.data(), t_len.p, (size_t)P * 4, hipMemcpyDeviceToHost, this->st)) ||
      (e = hipMemcpyAsync(fr.data(), t_freq.p, (size_t)P * 8, hipMemcpyDeviceToHost, this->st)) ||
      (e = hipMemcpyAsync(pre.data(), t_prefix.p, (size_t)P * 8, hipMemcpyDeviceToHost, this->st)) ||
      (e = hipMemcpyAsync(tp.data(), t_tp.p, (size_t)P * 8, hipMemcpyDeviceToHost, this->st)) ||
      (e = hipMemcpyAsync(su.data(), t_succ.p, su.size() * 4, hipMemcpyDeviceToHost, this->st)) ||
      (e = this->sync_st()))
    return hipfail(e, "exact: table");
  std::vector<int64_t> off;
  std::vector<uint8_t> al;
  int rc = spell_table(ln, off, al);
  if (rc) return rc;
  c = Cands();
  for (int i = 0; i < P; ++i) c.push(st[i], ln[i], al.data() + off[i], 0, false, fr[i], pre[i], tp[i]);
  succ.resize((size_t)P * A);
  for (size_t i = 0; i < su.size(); ++i) succ[i] = su[i] == NONE ? -1 : (int32_t)su[i];
  return HMC_OK;
}

int Ctx::estimate_round(Cands &c, size_t b, size_t e) {
  const int L = pan.L, A = pan.amax, N = pan.N;
  const auto t_round = std::chrono::steady_clock::now();
  const double walk0 = ms_walk;
  const bool reused = xc_reuse;
  std::vector<int32_t> child, data, root(L, -1);
  int maxd = 0;
  auto new_node = [&]() {
    child.insert(child.end(), A, -1);
    data.push_back(-1);
    return (int32_t)data.size() - 1;
  };
  for (size_t k = b; k < e; ++k) {  // ForwardPatternTree::addPattern (PatternTree.cpp:188-212)
    const int s = c.start[k];
    if (root[s] < 0) root[s] = new_node();
    int32_t u = root[s];
    const uint8_t *al = c.alleles(k);
    for (int q = 0; q < c.len[k]; ++q) {
      if (al[q] >= A) return fail(HMC_EUNSUPPORTED, "exact M-step: pattern with a missing allele");
      int32_t v = child[(size_t)u * A + al[q]];
      if (v < 0) {
        v = new_node();
        child[(size_t)u * A + al[q]] = v;
      }
      u = v;
    }
    data[u] = (int32_t)(k - b);
    maxd = std::max(maxd, (int)c.len[k]);
  }
  const size_t nc = e - b;
  hipError_t er;
  if ((er = d_tr_child.ensure(std::max<size_t>(child.size(), 1))) || (er = d_tr_data.ensure(std::max<size_t>(data.size(), 1))) ||
      (er = d_tr_root.ensure(L)) || (er = d_xacc.ensure(2 * std::max<size_t>(nc, 1))) ||
      (!child.empty() && (er = hipMemcpyAsync(d_tr_child.p, child.data(), child.size() * 4, hipMemcpyHostToDevice, st))) ||
      (!data.empty() && (er = hipMemcpyAsync(d_tr_data.p, data.data(), data.size() * 4, hipMemcpyHostToDevice, st))) ||
      (er = hipMemcpyAsync(d_tr_root.p, root.data(), (size_t)L * 4, hipMemcpyHostToDevice, st)) ||
      (er = hipMemsetAsync(d_xacc.p, 0, 2 * nc * 8, st)))
    return hipfail(er, "exact: trie");
  tr_maxd = maxd;
  // the individuals of the shard, heaviest first, through the split machinery
  const int n = nloc();
  if ((er = d_xstatus.ensure(n)) || (er = d_xre.ensure(n)) || (er = d_xfmax.ensure(n))) return hipfail(er, "exact");
  std::vector<int32_t> order(n);
  for (int q = 0; q < n; ++q) order[q] = q;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return h_cost[x] > h_cost[y]; });
  xacc_nc = nc;
  int rc;
  if (xc_reuse) {
    if ((rc = exact_group(nullptr, xc_k))) return rc;
  } else {
    const int passes0 = n_struct_passes;
    while (true) {
      xc_groups = 0;
      rc = estep_split(order, true);
      if (rc != ESTEP_RESTART) break;
      if ((er = hipMemsetAsync(d_xacc.p, 0, 2 * nc * 8, st))) return hipfail(er, "exact");
    }
    if (rc) return rc;
    // one structure pass and one walk group: the stores hold every individual
    xc_reuse = n_struct_passes == passes0 + 1 && xc_groups == 1;
  }
  std::vector<unsigned long long> acc(2 * nc);
  if ((er = hipMemcpyAsync(acc.data(), d_xacc.p, acc.size() * 8, hipMemcpyDeviceToHost, st)) ||
      (er = sync_st()))
    return hipfail(er, "exact");
  if (multi()) {  // integer sums over ranks, exactly: 32-bit halves through the double collective
    std::vector<double> h(4 * nc);
    for (size_t i = 0; i < 2 * nc; ++i) {
      h[2 * i] = (double)(acc[i] & 0xFFFFFFFFull);
      h[2 * i + 1] = (double)(acc[i] >> 32);
    }
    if ((rc = allreduce_host(h.data(), h.size()))) return rc;
    for (size_t i = 0; i < 2 * nc; ++i) acc[i] = ((unsigned long long)h[2 * i + 1] << 32) + (unsigned long long)h[2 * i];
  }
  for (size_t k = 0; k < nc; ++k) {  // HaploBuilder.cpp:317-331
    double freq = std::min((double)acc[k] / EXACT_FIXED_SCALE, (double)N);
    const double pre = std::min((double)acc[nc + k] / EXACT_FIXED_SCALE, (double)N);
    freq = std::min(freq, pre);
    c.freq[b + k] = freq / N;
    c.prefix[b + k] = pre / N;
    const double t = pre > 0 ? freq / pre : freq / N;
    c.tp[b + k] = t < 1.0 ? t : 1.0;  // HaploPattern::setTransitionProb (HaploPattern.h:47)
  }
  ++exact_rounds;
  exact_candidates += nc;
  if (debug_mem)
    fprintf(stderr, "[hmc] exact round %d: %zu candidates, trie depth %d, walk %.1f ms, round %.1f ms%s\n", exact_rounds,
            nc, maxd, ms_walk - walk0,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_round).count(),
            reused ? " (E-step data reused)" : "");
  return HMC_OK;
}

int Ctx::exact_group(const int32_t *ids, int k, const std::function<int(std::vector<int32_t> &)> &rerun) {
  const int L = pan.L;
  int dev_cu = 256;
  hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, device);
  hipError_t e;
  ExactArgs x;
  x.L = L;
  x.head_len = head_len;
  x.width = pan.amax;
  x.order = d_order2.p;
  x.n_order = k;
  x.rec = d_rec.p;
  x.rec_off = d_rec_off.p;
  x.status = d_xstatus.p;
  x.gprob = d_total.p;
  x.x = d_trace.p;
  x.x_base = d_tbase.p;
  x.x_off = d_loc_off.p;
  x.tr_child = d_tr_child.p;
  x.tr_data = d_tr_data.p;
  x.tr_root = d_tr_root.p;
  x.max_depth = tr_maxd;
  x.head_al = d_head_al.p;
  x.acc_freq = d_xacc.p;
  x.acc_prefix = d_xacc.p + xacc_nc;
  if (xc_reuse) {  // a later round over the same group: records and fwd/bwd sums are still in place
    x.fmax = xc_fmax;
    return exact_walk_group(x, k, dev_cu);
  }
  if ((e = launch_exact_fb(x, std::max(1, std::min(k, dev_cu * 8)), st))) return hipfail(e, "exact_fb");
  const int n = nloc();
  std::vector<int32_t> xs(n), fm(n);
  if ((e = hipMemcpyAsync(xs.data(), d_xstatus.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
      (e = hipMemcpyAsync(fm.data(), d_xfmax.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
      (e = sync_st()))
    return hipfail(e, "exact_fb");
  std::vector<int32_t> redo;
  for (int q = 0; q < k; ++q)
    if (xs[ids[q]] == EST_NEEDS_EXACT) redo.push_back(ids[q]);
  if (!redo.empty()) {  // their records again, pruned, then their fwd/bwd sums
    if (!rerun) return fail(HMC_EHIP, "exact M-step: a forward likelihood underflows (individual %d)", i0 + redo[0]);
    exact_pruned += (int)redo.size();
    int rc;
    if ((rc = rerun(redo))) return rc;
    const int nr = (int)redo.size();
    if ((e = d_redo.ensure(nr))) return hipfail(e, "exact underflow re-run");
    if ((rc = upload_order(d_redo, redo.data(), nr))) return rc;
    ExactArgs x2 = x;
    x2.order = d_redo.p;
    x2.n_order = nr;
    if ((e = launch_exact_fb(x2, std::max(1, std::min(nr, dev_cu * 8)), st))) return hipfail(e, "exact_fb");
    if ((e = hipMemcpyAsync(xs.data(), d_xstatus.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(fm.data(), d_xfmax.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
        (e = sync_st()))
      return hipfail(e, "exact_fb");
    for (int r : redo)
      if (xs[r] == EST_NEEDS_EXACT) return fail(HMC_EHIP, "exact M-step: pruned records still underflow (individual %d)", i0 + r);
  }
  int fmax = 1;
  for (int q = 0; q < k; ++q) fmax = std::max(fmax, fm[ids[q]]);
  x.fmax = fmax;
  xc_fmax = fmax;
  xc_k = k;
  ++xc_groups;
  return exact_walk_group(x, k, dev_cu);
}

int Ctx::exact_walk_group(ExactArgs &x, int k, int dev_cu) {
  if (exact_ipw == 2) return exact_walk_bfs(x, k, dev_cu);  // (variants)
  const int L = pan.L;
  hipError_t e;
  if (exact_walk_lds_bytes(tr_maxd, x.fmax, x.width) > EXACT_WALK_LDS_MAX)
    return fail(HMC_EUNSUPPORTED, "exact M-step: a frontier of %d states (trie depth %d) exceeds the walk's LDS bitmap",
                x.fmax, tr_maxd);
  // (variants) items per wavefront: 4 (16 lanes each) when their LDS fits, else 1
  const int ipw = exact_ipw == 4 && exact_walk_lds_bytes(tr_maxd, x.fmax, x.width) * 4 <= EXACT_WALK_LDS_MAX ? 4 : 1;
  {  // the largest list span of any item of the group (the per-wave scratch)
    unsigned span = 0;
    if ((e = d_xspan.ensure(1))) return hipfail(e, "exact_span");
    x.span_max = d_xspan.p;
    if ((e = hipMemsetAsync(d_xspan.p, 0, 4, st)) || (e = launch_exact_span(x, std::max(1, std::min(k, dev_cu * 8)), st)) ||
        (e = hipMemcpyAsync(&span, d_xspan.p, 4, hipMemcpyDeviceToHost, st)) || (e = sync_st()))
      return hipfail(e, "exact_span");
    x.span = std::max<long long>(span, 1);
  }
  x.scratch_stride = exact_walk_scratch_doubles(tr_maxd, x.span, x.width);
  const long long items = (long long)k * L;
  // 28 waves per CU, fewer when the per-item lists would pass SCRATCH_MAX
  const long long by_mem = std::max<long long>(1, (long long)(SCRATCH_MAX / (x.scratch_stride * 8 * ipw)));
  const int grid = (int)std::max<long long>(1, std::min<long long>(std::min<long long>(items, (long long)dev_cu * 28), by_mem));
  // the walk's zero invariant (its lists; the child frequencies and touched
  // lists are left behind by each item and would land inside the lists of
  // a group whose depth or frontier differs): zeroed for every group
  const size_t need = x.scratch_stride * grid * ipw;
  if ((e = d_xscr.ensure(need)) || (e = hipMemsetAsync(d_xscr.p, 0, need * 8, st)))
    return hipfail(e, "exact scratch");
  x.scratch = d_xscr.p;
  // long walks (over 4 M items) in 16 slices, so that they report progress
  // (the lists return to zero between slices: every item clears its entries)
  const long long slice = items > (4ll << 20) ? std::max<long long>(grid, (items + 15) / 16) : items;
  for (long long i0 = 0; i0 < items; i0 += slice) {
    x.item0 = i0;
    x.item1 = std::min(items, i0 + slice);
    hipEventRecord(ev[0], st);
    if ((e = launch_exact_walk(x, grid, st, ipw))) return hipfail(e, "exact_walk");
    hipEventRecord(ev[1], st);
    if ((e = sync_st())) return hipfail(e, "exact_walk");
    float ms = 0;
    hipEventElapsedTime(&ms, ev[0], ev[1]);
    ms_walk += ms;
    if (debug_mem)
      fprintf(stderr, "[hmc] exact walk: items %lld..%lld of %lld (%d individuals), %.1f ms; grid %d (%.1f waves per CU), "
              "fmax %d, depth %d, %.1f MB per wave\n", i0, x.item1, items, k, ms, grid, (double)grid / dev_cu, x.fmax, tr_maxd,
              x.scratch_stride * 8e-6);
  }
  return HMC_OK;
}

int Ctx::exact_walk_bfs(ExactArgs &x, int k, int dev_cu) {
  const int L = pan.L, fmax = std::max(x.fmax, 1);
  const long long items = (long long)k * L;
  hipError_t e;
  // lanes: 8 waves per CU; each owns [a side | b side][3][fmax] accumulators and a state bitmap
  const int grid = dev_cu * 2, nthr = grid * 256;
  const size_t lacc = 6 * (size_t)fmax, lbits = (size_t)fmax / 32 + 2;
  // unit and entry pools: a third of what is free (entries 28 B, units 32 B)
  size_t freeb = 0, totb = 0;
  hipMemGetInfo(&freeb, &totb);
  const double scratch_b = (double)nthr * (lacc * 8 + lbits * 4);
  const double pool_b = std::max(256e6, std::min(24e9, ((double)freeb - scratch_b) / 3.0));
  const unsigned long long ecap = (unsigned long long)(pool_b * 0.8 / 28.0), ucap = (unsigned long long)(pool_b * 0.2 / 32.0);
  const long long batch = std::max<long long>(1, std::min<long long>({items, (long long)(ecap / (2ull * (unsigned long long)fmax)),
                                                                        (long long)ucap / 2, 1ll << 30}));
  if ((e = d_xu_q.ensure(ucap)) || (e = d_xu_start.ensure(ucap)) || (e = d_xu_node.ensure(ucap)) || (e = d_xu_freq.ensure(ucap)) ||
      (e = d_xu_e0.ensure(ucap)) || (e = d_xu_ne.ensure(ucap)) || (e = d_xe_t.ensure(ecap)) || (e = d_xe_w.ensure(3 * ecap)) ||
      (e = d_xcur.ensure(2)) || (e = d_xndef.ensure(1)) || (e = d_xdef.ensure(std::max<size_t>((size_t)batch, ucap))) ||
      (e = d_xidx.ensure(std::max<size_t>((size_t)batch, ucap))) || (e = d_xlacc.ensure((size_t)nthr * lacc)) ||
      (e = d_xlbits.ensure((size_t)nthr * lbits)) || (e = hipMemsetAsync(d_xlacc.p, 0, (size_t)nthr * lacc * 8, st)) ||
      (e = hipMemsetAsync(d_xlbits.p, 0, (size_t)nthr * lbits * 4, st)))
    return hipfail(e, "exact walk pools");
  XWalkArgs w;
  w.u.q = d_xu_q.p;
  w.u.start = d_xu_start.p;
  w.u.node = d_xu_node.p;
  w.u.freq = d_xu_freq.p;
  w.u.e0 = d_xu_e0.p;
  w.u.ne = d_xu_ne.p;
  w.e_t = d_xe_t.p;
  w.e_w = d_xe_w.p;
  w.e_cap = ecap;
  w.u_cap = ucap;
  w.cursor = d_xcur.p;
  w.defer = d_xdef.p;
  w.n_defer = d_xndef.p;
  w.lacc = d_xlacc.p;
  w.lbits = d_xlbits.p;
  w.lacc_stride = lacc;
  w.lbits_stride = lbits;
  x.scratch = nullptr;
  hipEventRecord(ev[0], st);
  // One level: the units [in_base, in_base + n) (or the listed ones) at
  // `depth`, outputs from (u_top, e_top); then the next level over those
  // outputs, then — with the pools above free again — the deferred units (a
  // loop at the same depth: the recursion is as deep as the trie only).
  std::function<int(int, bool, unsigned long long, std::vector<int32_t> *, int, unsigned long long, unsigned long long)> level;
  level = [&](int depth, bool roots, unsigned long long in_base, std::vector<int32_t> *idx0, int n,
              unsigned long long u_top, unsigned long long e_top) -> int {
    std::vector<int32_t> idx_v;
    if (idx0) idx_v.swap(*idx0);
    bool listed = idx0 != nullptr;
    while (n > 0) {
      hipError_t e2;
      const unsigned long long cur0[2] = {u_top, e_top};
      const int zero = 0;
      if ((e2 = hipMemcpyAsync(d_xcur.p, cur0, 16, hipMemcpyHostToDevice, st)) ||
          (e2 = hipMemcpyAsync(d_xndef.p, &zero, 4, hipMemcpyHostToDevice, st)) ||
          (listed && (e2 = hipMemcpyAsync(d_xidx.p, idx_v.data(), idx_v.size() * 4, hipMemcpyHostToDevice, st))) ||
          (listed && (e2 = sync_st())))
        return hipfail(e2, "exact walk");
      XWalkArgs w2 = w;
      w2.in_base = in_base;
      w2.idx = listed ? d_xidx.p : nullptr;
      w2.n_in = n;
      w2.depth = depth;
      w2.roots = roots;
      if ((e2 = launch_exact_walk_units(x, w2, std::max(1, std::min(grid, (n + 255) / 256)), st)))
        return hipfail(e2, "exact_walk_units");
      unsigned long long cur[2];
      int nd = 0;
      if ((e2 = hipMemcpyAsync(cur, d_xcur.p, 16, hipMemcpyDeviceToHost, st)) ||
          (e2 = hipMemcpyAsync(&nd, d_xndef.p, 4, hipMemcpyDeviceToHost, st)) || (e2 = sync_st()))
        return hipfail(e2, "exact walk");
      ++xw_launches;
      xw_units += n;
      std::vector<int32_t> def((size_t)nd);
      if (nd && ((e2 = hipMemcpyAsync(def.data(), d_xdef.p, (size_t)nd * 4, hipMemcpyDeviceToHost, st)) ||
                 (e2 = sync_st())))
        return hipfail(e2, "exact walk");
      const unsigned long long u_end = std::min(cur[0], ucap), e_end = std::min(cur[1], ecap);
      if (nd == n && u_end == u_top)
        return fail(HMC_ENOMEM, "exact M-step: one trie node's children exceed the walk's pools (%llu units, %llu entries)",
                    ucap, ecap);
      int rc2;
      if (u_end > u_top && (rc2 = level(depth + 1, false, u_top, nullptr, (int)(u_end - u_top), u_end, e_end))) return rc2;
      xw_defers += nd;
      std::sort(def.begin(), def.end());  // (any order gives the same sums: fixed-point adds)
      idx_v.swap(def);
      listed = true;
      n = nd;
    }
    return HMC_OK;
  };
  for (long long b = 0; b < items; b += batch) {
    const int nb = (int)std::min<long long>(batch, items - b);
    int rc = level(0, true, (unsigned long long)b, nullptr, nb, 0, 0);
    if (rc) return rc;
  }
  hipEventRecord(ev[1], st);
  if ((e = sync_st())) return hipfail(e, "exact walk");
  float ms = 0;
  hipEventElapsedTime(&ms, ev[0], ev[1]);
  ms_walk += ms;
  if (debug_mem)
    fprintf(stderr, "[hmc] exact walk (breadth-first): %lld items, %d individuals, %.1f ms; %lld units in %lld launches, "
            "%lld deferred; pools %llu units / %llu entries\n", items, k, ms, xw_units, xw_launches, xw_defers, ucap, ecap);
  return HMC_OK;
}

void Ctx::host_successors(const Cands &c, std::vector<int32_t> &succ) {
  const int L = pan.L, A = pan.amax;
  const size_t P = c.size();
  std::vector<int32_t> child, data, root(L, -1);
  auto new_node = [&]() {
    child.insert(child.end(), A, -1);
    data.push_back(-1);
    return (int32_t)data.size() - 1;
  };
  for (size_t k = 0; k < P; ++k) {
    const int s = c.start[k];
    if (root[s] < 0) root[s] = new_node();
    int32_t u = root[s];
    const uint8_t *al = c.alleles(k);
    for (int q = 0; q < c.len[k]; ++q) {
      int32_t v = child[(size_t)u * A + al[q]];
      if (v < 0) {
        v = new_node();
        child[(size_t)u * A + al[q]] = v;
      }
      u = v;
    }
    data[u] = (int32_t)k;
  }
  succ.assign(P * A, -1);
  for (size_t k = 0; k < P; ++k) {
    const int s = c.start[k], ln = c.len[k], e = s + ln;
    if (e >= L) continue;
    const uint8_t *al = c.alleles(k);
    for (int j = 0; j < h_anum[e]; ++j) {
      int32_t res = -1;
      for (int s2 = s; s2 <= e && res < 0; ++s2) {  // longest first
        int32_t u = root[s2];
        for (int q = s2 - s; q < ln && u >= 0; ++q) u = child[(size_t)u * A + al[q]];
        if (u >= 0) u = child[(size_t)u * A + j];
        if (u >= 0) res = data[u];
      }
      succ[k * A + j] = res;
    }
  }
}

int Ctx::install_host_table(Cands &c, std::vector<int32_t> &succ) {
  const int P = (int)c.size(), A = pan.amax;
  if ((int64_t)P > INT32_MAX) return fail(HMC_EUNSUPPORTED, "too many patterns");
  int rc = alloc_table(std::max(P, 1));
  if (rc) return rc;
  std::vector<uint8_t> last(P);
  std::vector<int32_t> node(P, -1);
  std::vector<uint32_t> su((size_t)P * A);
  for (int i = 0; i < P; ++i) last[i] = c.alleles(i)[c.len[i] - 1];
  for (size_t i = 0; i < su.size(); ++i) su[i] = succ[i] < 0 ? NONE : (uint32_t)succ[i];
  hipError_t e;
  if (P && ((e = hipMemcpyAsync(t_start.p, c.start.data(), (size_t)P * 4, hipMemcpyHostToDevice, st)) ||
            (e = hipMemcpyAsync(t_len.p, c.len.data(), (size_t)P * 4, hipMemcpyHostToDevice, st)) ||
            (e = hipMemcpyAsync(t_node.p, node.data(), (size_t)P * 4, hipMemcpyHostToDevice, st)) ||
            (e = hipMemcpyAsync(t_freq.p, c.freq.data(), (size_t)P * 8, hipMemcpyHostToDevice, st)) ||
            (e = hipMemcpyAsync(t_prefix.p, c.prefix.data(), (size_t)P * 8, hipMemcpyHostToDevice, st)) ||
            (e = hipMemcpyAsync(t_tp.p, c.tp.data(), (size_t)P * 8, hipMemcpyHostToDevice, st)) ||
            (e = hipMemcpyAsync(t_last.p, last.data(), (size_t)P, hipMemcpyHostToDevice, st)) ||
            (e = hipMemcpyAsync(t_succ.p, su.data(), su.size() * 4, hipMemcpyHostToDevice, st)) ||
            (e = hipMemsetAsync(t_ppat.p, 0xFE, (size_t)P * 4, st)) ||  // alleles are kept on the host (ht)
            (e = sync_st())))
    return hipfail(e, "exact: install table");
  this->P = P;
  // head list: start 0, length head_len, id order (PatternManager.cpp:304-306)
  std::vector<std::pair<uint32_t, uint8_t>> heads;
  h_head_ids.clear();
  h_head_al.clear();
  std::vector<uint8_t> tab;
  if (head_len > 1) tab.assign((size_t)std::max(P, 1) * head_len, 0);
  for (int i = 0; i < P; ++i)
    if (c.start[i] == 0 && c.len[i] == head_len) {
      heads.push_back({(uint32_t)i, c.alleles(i)[head_len - 1]});
      if (head_len > 1) {
        h_head_ids.push_back((uint32_t)i);
        h_head_al.insert(h_head_al.end(), c.alleles(i), c.alleles(i) + head_len);
        std::copy(c.alleles(i), c.alleles(i) + head_len, tab.begin() + (size_t)i * head_len);
      }
    }
  if (head_len > 1 && ((e = d_head_al.ensure(tab.size())) ||
                       (e = hipMemcpyAsync(d_head_al.p, tab.data(), tab.size(), hipMemcpyHostToDevice, st)) ||
                       (e = sync_st())))
    return hipfail(e, "exact: heads");
  if ((rc = set_heads(heads))) return rc;
  ht = c;
  ht_succ = succ;
  table_on_host = true;
  have_model = true;
  new_table(false);
  return HMC_OK;
}

int Ctx::estimate_patterns(int *P_out, uint64_t *rm_out) {
  if (!have_estep) return fail(HMC_EARG, "exact M-step needs an E-step first");
  // after findPatternByNum the reference estimates at that search's last
  // threshold (m_min_freq, PatternManager.cpp:53-60, 364-408)
  const bool bynum = num_patterns > 0 && model != 1;
  if (bynum && !(bynum_theta_last > 0))
    return fail(HMC_EARG, "exact M-step after findPatternByNum needs the search's threshold (mine first)");
  if (pan.amax > 44)  // the records pack a locus's allele pairs (amax (amax + 1) / 2) in 10 bits
    return fail(HMC_EUNSUPPORTED, "exact M-step with more than 44 alleles per locus");
  hipEventRecord(ev[4], st);
  const int L = pan.L;
  int mxl = max_len <= 0 ? L : max_len;  // m_max_len / m_min_len of the last findPatternByFreq
  int mnl = std::max(min_len, 1);
  mxl = std::max(mxl, mnl);
  double mf = bynum ? bynum_theta_last : current_min_freq();
  if (model == 1) {  // findPatternBlock: m_min_freq = -1 (PatternManager.cpp:75-88)
    mnl = mxl = std::max(1, mc_order + 1);
    mf = -1.0;
  }
  exact_rounds = 0;
  exact_candidates = 0;
  ms_walk = 0;
  xw_units = xw_launches = xw_defers = 0;
  exact_pruned = 0;
  xc_reuse = false;
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  auto t0 = clk::now();
  Cands cur;
  std::vector<int32_t> succ;
  int rc = table_to_host(cur, succ);
  if (rc) return rc;
  const double ms_to_host = ms_since(t0);
  t0 = clk::now();
  const int A = pan.amax;
  if (mf < 0) {  // estimateFrequency() (:347-362): re-estimate in place, ids and successors unchanged
    if ((rc = estimate_round(cur, 0, cur.size()))) return rc;
    if ((rc = install_host_table(cur, succ))) return rc;
  } else {
    Cands all;
    std::vector<size_t> seeds;
    for (size_t i = 0; i < cur.size(); ++i) {
      all.push(cur.start[i], cur.len[i], cur.alleles(i), 0, false, cur.freq[i], cur.prefix[i], cur.tp[i]);
      const int s = cur.start[i], e = s + cur.len[i];
      if (e < L && cur.len[i] < mxl)
        for (int j = 0; j < h_anum[e]; ++j) {
          const int32_t sj = succ[i * A + j];
          if (sj < 0 || cur.start[sj] != s) {  // the extension is not stored: a seed
            all.push(s, cur.len[i] + 1, cur.alleles(i), (uint8_t)j, true, cur.freq[i]);
            seeds.push_back(all.size() - 1);
          }
        }
    }
    size_t rb = 0, re = all.size();
    std::vector<uint8_t> buf;
    while (rb < re) {
      if ((rc = estimate_round(all, rb, re))) return rc;
      const size_t nb = all.size();
      for (int level = 0; level < 4; ++level) {  // extendPatterns (:412-438)
        std::vector<size_t> ns;
        for (size_t si : seeds) {
          const int s = all.start[si], ln = all.len[si], e = s + ln;
          if (e < L && ln < mxl && all.freq[si] >= mf) {
            buf.assign(all.alleles(si), all.alleles(si) + ln);
            const double f = all.freq[si];
            for (int j = 0; j < h_anum[e]; ++j) {
              all.push(s, ln + 1, buf.data(), (uint8_t)j, true, f);
              ns.push_back(all.size() - 1);
            }
          }
        }
        seeds.swap(ns);
      }
      rb = nb;
      re = all.size();
    }
    const double ms_rounds = ms_since(t0);
    t0 = clk::now();
    Cands kept;  // (:396-408)
    for (size_t i = 0; i < all.size(); ++i)
      if (all.freq[i] >= mf || all.len[i] <= mnl)
        kept.push(all.start[i], all.len[i], all.alleles(i), 0, false, all.freq[i], all.prefix[i], all.tp[i]);
    std::vector<int32_t> ksucc;
    host_successors(kept, ksucc);
    const double ms_succ = ms_since(t0);
    t0 = clk::now();
    if ((rc = install_host_table(kept, ksucc))) return rc;
    if (debug_mem)
      fprintf(stderr, "[hmc] exact M-step: table to host %.1f ms, rounds %.1f ms (walks %.1f), kept + successors %.1f ms, "
              "install %.1f ms\n", ms_to_host, ms_rounds, ms_walk, ms_succ, ms_since(t0));
  }
  xc_reuse = false;
  hipEventRecord(ev[5], st);
  hipError_t e;
  if ((e = sync_st())) return hipfail(e, "exact");
  // the walk's scratch (up to SCRATCH_MAX) and the tries go back to the E-step
  d_xscr.release();
  d_tr_child.release();
  d_tr_data.release();
  float ms = 0;
  hipEventElapsedTime(&ms, ev[4], ev[5]);
  ms_m = ms;
  if (P_out) *P_out = P;
  if (rm_out) *rm_out = 0;  // no candidate x item scans: the cost is in the trie walks
  return HMC_OK;
}
}  // namespace hmc
