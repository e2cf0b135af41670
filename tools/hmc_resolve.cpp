// hmc_resolve — C++ drop-in for HMC's resolve mode (HMC.cpp:179-233) built on
// the C-ABI of libhmc_amd.so.  Reads a PHASE file (HaploFile::readGenoData),
// runs HaploModel::run on the GPU and writes <input>.reconstructed
// (HaploFile::writeGenoData).  Options use the reference's names and defaults
// (HMC.cpp:35-47).
//
//   hmc_resolve [-a 1.5] [-i 1] [--sample-size 10] [--min-pattern-len 1]
//               [--max-pattern-len 30] [-r min_freq] [-d device] input.phase
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../include/hmc_amd.h"

int main(int argc, char **argv) {
  double min_freq_abs = 1.5, min_freq = -1.0;
  int max_iteration = 1, sample_size = 10, min_len = 1, max_len = 30, device = 0;
  const char *input = nullptr;
  std::string model = "MV";
  int mc_order = 1, num_patterns = -1;
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
    else if (a == "-d" || a == "--device") device = atoi(next());
    else if (a == "-m" || a == "--model") model = next();             // HMC.cpp:35
    else if (a == "-o" || a == "--mc-order") mc_order = atoi(next());  // HMC.cpp:41
    else if (a == "-n" || a == "--num-patterns") num_patterns = atoi(next());  // HMC.cpp:38
    else if (a[0] == '-') { fprintf(stderr, "unknown option %s\n", a.c_str()); return 1; }
    else input = argv[i];
  }
  if (!input) {
    fprintf(stderr, "Usage: hmc_resolve [option ...] datafile\n");
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
  printf("Reading genotype file ...\n");
  if ((rc = hmc_load_phase(ctx, input))) die("hmc_load_phase");
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
  std::string out = std::string(input) + ".reconstructed";
  if ((rc = hmc_write_phase(ctx, out.c_str()))) die("hmc_write_phase");
  hmc_ctx_destroy(ctx);
  return 0;
}
