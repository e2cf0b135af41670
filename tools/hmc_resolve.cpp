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

int main(int argc, char **argv) {
  double min_freq_abs = 1.5, min_freq = -1.0;
  int max_iteration = 1, sample_size = 10, min_len = 1, max_len = 30, device = 0;
  std::vector<std::string> files;
  std::string model = "MV", format = "PHASE";
  int mc_order = 1, num_patterns = -1;
  bool exact = false, output_patterns = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char * {
      if (i + 1 >= argc) { fprintf(stderr, "missing value for %s\n", a.c_str()); exit(1); }
      return argv[++i];
    };
    if (a == "-a" || a == "--min-freq-abs") min_freq_abs = atof(next());
    else if (a == "-r" || a == "--min-freq-rel") { min_freq = atof(next()); min_freq_abs = 0; }
    else if (a == "-i" || a == "--max-iteration") max_iteration = atoi(next());
    else if (a == "--sample-size") sample_size = atoi(next());
    else if (a == "--min-pattern-len") min_len = atoi(next());
    else if (a == "--max-pattern-len") max_len = atoi(next());
    else if (a == "--device") device = atoi(next());
    else if (a == "-d" || a == "--debug") (void)next();                 // Logger level (HMC.cpp:28)
    else if (a == "-f" || a == "--input-format") format = next();      // HMC.cpp:29
    else if (a == "--exact-estimate") exact = true;                      // HMC.cpp:42
    else if (a == "--output-patterns") { (void)next(); output_patterns = true; }  // HMC.cpp:30, 229-232
    else if (a == "-m" || a == "--model") model = next();             // HMC.cpp:35
    else if (a == "-o" || a == "--mc-order") mc_order = atoi(next());  // HMC.cpp:41
    else if (a == "-n" || a == "--num-patterns") num_patterns = atoi(next());  // HMC.cpp:38
    else if (a[0] == '-') { fprintf(stderr, "unknown option %s\n", a.c_str()); return 1; }
    else files.push_back(argv[i]);
  }
  if (files.empty()) {
    fprintf(stderr, "Usage: hmc_resolve [option ...] datafiles\n");
    return 1;
  }
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
