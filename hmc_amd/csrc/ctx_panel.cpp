// ctx_panel.cpp — Ctx members: collectives across ranks and the panel upload.
#include "ctx.hpp"

namespace hmc {

void Ctx::shard(int N, int L) {
  if (world == 1) { i0 = 0; i1 = N; return; }
  std::vector<double> pre((size_t)N + 1, 0.0);
  for (int i = 0; i < N; ++i) {
    int h = 0;
    for (int k = 0; k < L; ++k) {
      const uint8_t x = pan.idx[((size_t)i * 2) * L + k], y = pan.idx[((size_t)i * 2 + 1) * L + k];
      h += (x != y || x == MISSING) ? 1 : 0;
    }
    pre[i + 1] = pre[i] + L / 8.0 + h;
  }
  auto cut = [&](int r) {
    if (r <= 0) return 0;
    if (r >= world) return N;
    const double target = pre[N] * r / world;
    return (int)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
  };
  i0 = cut(rank);
  i1 = cut(rank + 1);
}

int Ctx::upload_panel() {
  const int N = pan.N, L = pan.L, A = pan.amax;
  shard(N, L);
  fast_off = false;
  std::vector<uchar2> im((size_t)N * L), lm((size_t)L * N);
  for (int i = 0; i < N; ++i)
    for (int k = 0; k < L; ++k) {
      uchar2 g = make_uchar2(pan.idx[((size_t)i * 2) * L + k], pan.idx[((size_t)i * 2 + 1) * L + k]);
      im[(size_t)i * L + k] = g;
      lm[(size_t)k * N + i] = g;
    }
  h_anum.assign(L + 1, 0);
  h_npos.assign(L + 1, 0);
  std::vector<double> af((size_t)L * A, 0.0);
  std::vector<uint8_t> pa((size_t)L * A, 0xFF), rk((size_t)L * A, 0xFF);
  std::vector<int32_t> rcb(L + 1, 0);
  int tot = 0;
  for (int k = 0; k < L; ++k) {
    h_anum[k] = (uint8_t)pan.sym[k].size();
    for (size_t j = 0; j < pan.sym[k].size(); ++j) {
      af[(size_t)k * A + j] = pan.sym[k][j].second;
      if (pan.sym[k][j].second > 0) {
        pa[(size_t)k * A + h_npos[k]] = (uint8_t)j;
        rk[(size_t)k * A + j] = h_npos[k];
        h_npos[k]++;
      }
    }
    rcb[k] = tot;
    tot += h_npos[k];
  }
  rcb[L] = tot;
  hipError_t e;
#define UP(buf, vec)                                                                              \
if ((e = buf.ensure(vec.size())) ||                                                             \
    (e = hipMemcpyAsync(buf.p, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice, st))) \
  return hipfail(e, "upload_panel");
  UP(d_geno_im, im);
  UP(d_geno_lm, lm);
  UP(d_anum, h_anum);
  UP(d_npos, h_npos);
  UP(d_afreq, af);
  UP(d_pos_allele, pa);
  UP(d_rank_of, rk);
  UP(d_r_child_base, rcb);
#undef UP
  if ((e = sync_st())) return hipfail(e, "upload_panel");
  have_panel = true;
  have_model = have_samples = have_estep = have_best = false;
  snap.valid = false;  // a saved table belongs to the panel it was built on
  win_scale = 1.0;     // window shrinking learnt on another panel does not carry over
  P = 0;
  H = 0;
  return HMC_OK;
}
}  // namespace hmc
