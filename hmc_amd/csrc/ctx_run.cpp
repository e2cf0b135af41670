// ctx_run.cpp — Ctx members: HaploComp, the EM driver (HaploModel::run) and the model snapshot.
#include "ctx.hpp"

namespace hmc {

int Ctx::haplocomp(double out[3]) {
  const int n = nloc(), L = pan.L;
  const int ncmp = std::max(0, std::min(n, pan.unphased - i0));  // m_genotype_num = unphased_num() (HaploComp.cpp:40)
  hipError_t e;
  std::vector<int32_t> hc((size_t)ncmp * 6), bad(ncmp);
  if (ncmp > 0) {
    if ((e = d_hc_cnt.ensure((size_t)ncmp * 6)) || (e = d_hc_bad.ensure(ncmp)) ||
        (e = launch_haplocomp_counts(d_geno_im.p, i0, ncmp, L, d_best.p, d_hc_cnt.p, d_hc_bad.p, st)) ||
        (e = hipMemcpyAsync(hc.data(), d_hc_cnt.p, hc.size() * 4, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(bad.data(), d_hc_bad.p, bad.size() * 4, hipMemcpyDeviceToHost, st)) ||
        (e = sync_st()))
      return hipfail(e, "haplocomp");
  }
  double cnt[6] = {0, 0, 0, 0, 0, 0};  // se_num, se_den, ihp_num, ihp_den, igp_num, igp_den
  for (int i = 0; i < ncmp; ++i) {
    if (bad[i] >= 0) return fail(HMC_EARG, "Inconsistent genotypes at locus %d!", bad[i]);
    const int32_t *c = hc.data() + (size_t)i * 6;
    const int sd = c[0], het = c[1];
    cnt[0] += sd;
    cnt[1] += het - 1;
    cnt[2] += sd > 0 ? 1 : 0;
    cnt[3] += het > 1 ? 1 : 0;
    cnt[4] += c[4];
    cnt[5] += c[5];
  }
  int rc = allreduce_host(cnt, 6);  // integers < 2^53: exact in any order
  if (rc) return rc;
  out[0] = cnt[0] / cnt[1];
  out[1] = cnt[2] / cnt[3];
  out[2] = cnt[4] / cnt[5];
  return HMC_OK;
}

int Ctx::init_best() {
  const int n = nloc(), L = pan.L;
  best_res.assign((size_t)n * 2 * L, 0);
  for (int i = 0; i < n; ++i)
    for (int h = 0; h < 2; ++h)
      for (int k = 0; k < L; ++k)
        best_res[((size_t)i * 2 + h) * L + k] = pan.idx[((size_t)(i0 + i) * 2 + h) * L + k];
  hipError_t e;
  if ((e = d_best.ensure(best_res.size())) ||
      (e = hipMemcpyAsync(d_best.p, best_res.data(), best_res.size(), hipMemcpyHostToDevice, st)) ||
      (e = sync_st()))
    return hipfail(e, "resolutions");
  have_best = best_on_host = true;
  return HMC_OK;
}

int Ctx::em_iteration(int it, int max_iter, bool force_m, double &old_ll, hmc_iter_log &rec, bool &go) {
  using clk = std::chrono::steady_clock;
  int rc;
  if (!have_best && (rc = init_best())) return rc;
  for (double &x : hp_ms) x = 0.0;
  auto t1 = clk::now();
  double ll = 0;
  int Hs = 0;
  uint64_t re = 0;
  if ((rc = estep(&ll, &Hs, &re))) return rc;
  const double te = std::chrono::duration<double>(clk::now() - t1).count();
  hp_ms[HP_ESTEP] = te * 1e3;
  if (ll >= old_ll && (rc = accept_resolutions())) return rc;
  rec = hmc_iter_log{};
  double hc[3];
  {
    HpTimer hpt(hp_ms[HP_HAPLOCOMP]);
    if ((rc = haplocomp(hc))) return rc;  // HaploModel.cpp:134-136
  }
  rec.switch_error = hc[0];
  rec.ihp = hc[1];
  rec.igp = hc[2];
  rec.log_likelihood = ll;
  rec.t_estep_s = te;
  rec.r_e = re;
  rec.n_samples = Hs;
  rec.n_patterns = P;
  go = it < max_iter && ll >= old_ll && (old_ll - ll) / old_ll > 0.0001;  // HaploModel.cpp:139
  if (go || force_m) {
    auto t2 = clk::now();
    int np = 0;
    uint64_t rm = 0;
    if ((rc = mine(&np, &rm))) return rc;
    rec.t_mstep_s = std::chrono::duration<double>(clk::now() - t2).count();
    hp_ms[HP_MSTEP] = rec.t_mstep_s * 1e3;
    rec.r_m = rm;
    rec.n_patterns = np;
    old_ll = ll;
  }
  return HMC_OK;
}

int Ctx::model_save() {
  if (!have_model) return fail(HMC_EARG, "no pattern model to save");
  const size_t p = (size_t)std::max(P, 1), A = (size_t)pan.amax;
  // a table over 8 GB (cfg 4's M0: 720 M patterns, 35 GB) is kept in pinned
  // host memory: HBM is the E-step stores'; a rewind then reads it over PCIe
  const bool on_host = (double)p * (41.0 + 4.0 * (double)A) > 8e9;
  snap.start.set_host(on_host);
  snap.len.set_host(on_host);
  snap.node.set_host(on_host);
  snap.ppat.set_host(on_host);
  snap.freq.set_host(on_host);
  snap.prefix.set_host(on_host);
  snap.tp.set_host(on_host);
  snap.last.set_host(on_host);
  snap.succ.set_host(on_host);
  hipError_t e;
  if ((e = dcopy(snap.start, t_start, p)) || (e = dcopy(snap.len, t_len, p)) || (e = dcopy(snap.node, t_node, p)) ||
      (e = dcopy(snap.ppat, t_ppat, p)) ||
      (e = dcopy(snap.freq, t_freq, p)) || (e = dcopy(snap.prefix, t_prefix, p)) || (e = dcopy(snap.tp, t_tp, p)) ||
      (e = dcopy(snap.last, t_last, p)) || (e = dcopy(snap.succ, t_succ, p * A)) ||
      (e = dcopy(snap.head_ids, d_head_ids, std::max<size_t>(n_head, 1))) ||
      (e = dcopy(snap.head_pat0, d_head_pat0, A + 1)) ||
      (head_len > 1 && (e = dcopy(snap.head_al, d_head_al, p * head_len))) || (e = sync_st()))
    return hipfail(e, "model_save");
  snap.P = P;
  snap.L = pan.L;
  snap.amax = pan.amax;
  snap.head_len = head_len;
  snap.n_head = n_head;
  snap.gen = model_gen;
  snap.h_head_ids = h_head_ids;
  snap.h_head_al = h_head_al;
  snap.table_on_host = table_on_host;
  if (table_on_host) {
    snap.ht = ht;
    snap.ht_succ = ht_succ;
  }
  snap.valid = true;
  return HMC_OK;
}

int Ctx::em_rewind() {
  if (!snap.valid) return fail(HMC_EARG, "no saved model (hmc_model_save)");
  if (!have_panel || snap.L != pan.L || snap.amax != pan.amax)
    return fail(HMC_EARG, "the saved model belongs to another panel");
  const size_t p = (size_t)std::max(snap.P, 1), A = (size_t)pan.amax;
  hipError_t e;
  if ((e = dcopy(t_start, snap.start, p)) || (e = dcopy(t_len, snap.len, p)) || (e = dcopy(t_node, snap.node, p)) ||
      (e = dcopy(t_ppat, snap.ppat, p)) ||
      (e = dcopy(t_freq, snap.freq, p)) || (e = dcopy(t_prefix, snap.prefix, p)) || (e = dcopy(t_tp, snap.tp, p)) ||
      (e = dcopy(t_last, snap.last, p)) || (e = dcopy(t_succ, snap.succ, p * A)) ||
      (e = dcopy(d_head_ids, snap.head_ids, std::max<size_t>(snap.n_head, 1))) ||
      (e = dcopy(d_head_pat0, snap.head_pat0, A + 1)) ||
      (snap.head_len > 1 && (e = dcopy(d_head_al, snap.head_al, p * snap.head_len))) ||
      (e = sync_st()))
    return hipfail(e, "em_rewind");
  P = snap.P;
  head_len = snap.head_len;
  n_head = snap.n_head;
  model_gen = snap.gen;  // the candidate tree is valid again only if nothing was mined since
  h_head_ids = snap.h_head_ids;
  h_head_al = snap.h_head_al;
  table_on_host = snap.table_on_host;
  if (table_on_host) {
    ht = snap.ht;
    ht_succ = snap.ht_succ;
  }
  have_model = true;
  hf_valid = false;
  // the EM state of a fresh HaploModel::run after this M-step
  have_samples = have_estep = have_best = best_on_host = false;
  H = 0;
  total_weight = 0.0;
  h_cost.clear();
  prev_rneed.clear();
  prev_P = 0;
  win_scale = 1.0;
  fcap = fcap_user;
  return HMC_OK;
}

int Ctx::run(int max_iter, hmc_iter_log *log, int cap, int *iters, double *t_m0, uint64_t *rm0, int *np0) {
  using clk = std::chrono::steady_clock;
  have_samples = false;  // HaploModel::build -> setGenoData clears samples (HaploBuilder.cpp:19-23)
  auto t0 = clk::now();
  int np = 0;
  uint64_t rm = 0;
  int rc = mine(&np, &rm);
  if (rc) return rc;
  if (t_m0) *t_m0 = std::chrono::duration<double>(clk::now() - t0).count();
  if (rm0) *rm0 = rm;
  if (np0) *np0 = np;
  if ((rc = init_best())) return rc;
  double old_ll = -DBL_MAX;
  int it = 0;
  for (it = 1; it <= max_iter; ++it) {
    hmc_iter_log rec{};
    bool go = false;
    if ((rc = em_iteration(it, max_iter, false, old_ll, rec, go))) return rc;
    if (log && it - 1 < cap) log[it - 1] = rec;
    if (!go) break;
  }
  if (iters) *iters = std::min(it, max_iter);
  return HMC_OK;
}
}  // namespace hmc
