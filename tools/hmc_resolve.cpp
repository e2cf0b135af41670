// hmc_resolve — C++ drop-in for HMC's resolve mode (HMC.cpp:179-233) built on
// the C-ABI of libhmc_amd.so.  Reads the input files in the given format
// (HaploFile::getHaploFile + readGenoData), runs HaploModel::run on the GPU
// and writes <first file>.reconstructed in the same format
// (HaploFile::writeGenoData; BENCH2/3 also rewrite the position file, as
// HaploFileBench::writeGenoData does), and with --output-patterns the
// .patterns dump (HMC.cpp:229-232).  Options use the reference's names and
// defaults (HMC.cpp:17-47).
//
//   hmc_resolve [-f PHASE|HPM|HPM2|BENCH2|BENCH3] [-a 1.5] [-r min_freq] [-n num]
//               [-m MV|MC|MA] [-o mc_order] [--exact-estimate] [-i 1]
//               [--sample-size 10] [--min-pattern-len 1] [--max-pattern-len 30]
//               [--output-patterns x] [--device 0] datafile ...
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/hmc_amd.h"
#include "hmc_options.hpp"

int main(int argc, char **argv) {
  hmc_cli::Options o;
  std::string perr;
  if (hmc_cli::parse_options(argc, argv, o, perr)) {
    fprintf(stderr, "%s\n", perr.c_str());
    return 1;
  }
  const double min_freq_abs = o.min_freq_abs, min_freq = o.min_freq;
  const int max_iteration = o.max_iteration, sample_size = o.sample_size, min_len = o.min_len, max_len = o.max_len,
            device = o.device, mc_order = o.mc_order, num_patterns = o.num_patterns;
  const std::vector<std::string> &files = o.files;
  const std::string &model = o.model, &format = o.format;
  const bool exact = o.exact, output_patterns = o.output_patterns;
  hmc_ctx *ctx = nullptr;
  int rc = hmc_ctx_create(device, &ctx);
  auto die = [&](const char *what) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, hmc_ctx_error(ctx));
    hmc_ctx_destroy(ctx);
    exit(1);
  };
  if (rc) die("hmc_ctx_create");
  if ((rc = hmc_set_params(ctx, min_freq_abs, min_freq, min_len, max_len, sample_size))) die("hmc_set_params");
  if ((rc = hmc_set_model(ctx, model.c_str(), mc_order))) die("hmc_set_model");
  if ((rc = hmc_set_num_patterns(ctx, num_patterns))) die("hmc_set_num_patterns");
  if ((rc = hmc_set_exact_estimate(ctx, exact ? 1 : 0))) die("hmc_set_exact_estimate");
  printf("Reading genotype file ...\n");
  std::vector<const char *> names;
  for (auto &f : files) names.push_back(f.c_str());
  if ((rc = hmc_load_files(ctx, format.c_str(), names.data(), (int)names.size()))) die("hmc_load_files");
  int N = 0, L = 0, A = 0;
  hmc_panel_info(ctx, &N, &L, &A);
  printf("Succesfully read Haplotype file with %d markers and %d genotypes.\n", L, N);
  hmc_iter_log log[256];
  int iters = 0, np0 = 0;
  double t_m0 = 0;
  uint64_t rm0 = 0;
  if ((rc = hmc_run(ctx, max_iteration, log, 256, &iters, &t_m0, &rm0, &np0))) die("hmc_run");
  printf("Found haplotype patterns: %d (%.3f s)\n", np0, t_m0);
  double solve = t_m0;
  for (int k = 0; k < iters && k < 256; ++k) {
    printf("  Switch Error = %f, IHP = %f, IGP = %f, LL = %f\n", log[k].switch_error, log[k].ihp, log[k].igp,
           log[k].log_likelihood);  // HaploModel.cpp:135-136
    printf("  iteration %d: LL = %f, patterns = %d, E %.3f s, M %.3f s\n", k + 1, log[k].log_likelihood,
           log[k].n_patterns, log[k].t_estep_s, log[k].t_mstep_s);
    solve += log[k].t_estep_s + log[k].t_mstep_s;
  }
  printf("Solving Time = %f\n", solve);
  // HaploFile::writeGenoData(resolutions, ".reconstructed") on the first file
  std::vector<std::string> outs{files[0] + ".reconstructed"};
  if (format == "BENCH2" || format == "BENCH3") outs.push_back(files.size() > 1 ? files[1] : "");
  std::vector<const char *> onames;
  for (auto &f : outs) onames.push_back(f.c_str());
  if ((rc = hmc_write_files(ctx, format.c_str(), onames.data(), (int)onames.size()))) die("hmc_write_files");
  if (output_patterns) {
    const std::string pf = files[0] + ".patterns";
    if ((rc = hmc_write_patterns(ctx, pf.c_str()))) die("hmc_write_patterns");
  }
  hmc_ctx_destroy(ctx);
  return 0;
}
