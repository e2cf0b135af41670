// hmc_options.hpp — hmc_resolve's command line: the reference's option names
// and defaults (HMC.cpp:17-47).  Header-only and free of the C-ABI so that the
// host sanitizer test (tests/test_sanitize.py) can drive it.
#pragma once
#include <cstdlib>
#include <string>
#include <vector>

namespace hmc_cli {

struct Options {
  double min_freq_abs = 1.5, min_freq = -1.0;
  int max_iteration = 1, sample_size = 10, min_len = 1, max_len = 30, device = 0;
  std::vector<std::string> files;
  std::string model = "MV", format = "PHASE";
  int mc_order = 1, num_patterns = -1;
  bool exact = false, output_patterns = false;
};

// 0 on success; otherwise `err` says what is wrong (a missing value, an
// unknown option, no data file).
inline int parse_options(int argc, const char *const *argv, Options &o, std::string &err) {
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    const char *v = nullptr;
    auto next = [&]() -> bool {
      if (i + 1 >= argc) {
        err = "missing value for " + a;
        return false;
      }
      v = argv[++i];
      return true;
    };
    if (a == "-a" || a == "--min-freq-abs") { if (!next()) return 1; o.min_freq_abs = atof(v); }
    else if (a == "-r" || a == "--min-freq-rel") { if (!next()) return 1; o.min_freq = atof(v); o.min_freq_abs = 0; }
    else if (a == "-i" || a == "--max-iteration") { if (!next()) return 1; o.max_iteration = atoi(v); }
    else if (a == "--sample-size") { if (!next()) return 1; o.sample_size = atoi(v); }
    else if (a == "--min-pattern-len") { if (!next()) return 1; o.min_len = atoi(v); }
    else if (a == "--max-pattern-len") { if (!next()) return 1; o.max_len = atoi(v); }
    else if (a == "--device") { if (!next()) return 1; o.device = atoi(v); }
    else if (a == "-d" || a == "--debug") { if (!next()) return 1; }                      // Logger level (HMC.cpp:28)
    else if (a == "-f" || a == "--input-format") { if (!next()) return 1; o.format = v; }  // HMC.cpp:29
    else if (a == "--exact-estimate") o.exact = true;                                      // HMC.cpp:42
    else if (a == "--output-patterns") { if (!next()) return 1; o.output_patterns = true; }  // HMC.cpp:30, 229-232
    else if (a == "-m" || a == "--model") { if (!next()) return 1; o.model = v; }          // HMC.cpp:35
    else if (a == "-o" || a == "--mc-order") { if (!next()) return 1; o.mc_order = atoi(v); }      // HMC.cpp:41
    else if (a == "-n" || a == "--num-patterns") { if (!next()) return 1; o.num_patterns = atoi(v); }  // HMC.cpp:38
    else if (!a.empty() && a[0] == '-') { err = "unknown option " + a; return 1; }
    else o.files.push_back(a);
  }
  if (o.files.empty()) {
    err = "Usage: hmc_resolve [option ...] datafiles";
    return 1;
  }
  return 0;
}

}  // namespace hmc_cli
