// Host sanitizer job: the host code that runs without a GPU —
// the E-step store planning (hmc_amd/csrc/plan.hpp), the HaploFile readers and
// writers (hmc_amd/csrc/haplofile.cpp), hmc_resolve's option parser
// (tools/hmc_options.hpp) and the CPU restatement (oracle/hmc_oracle.cpp,
// test infrastructure) — built with -fsanitize=address,undefined and driven
// over small seeded inputs, including malformed files.  tests/test_sanitize.py
// builds and runs it; any sanitizer report fails the run (halt_on_error).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../hmc_amd/csrc/haplofile.hpp"
#include "../../hmc_amd/csrc/plan.hpp"
#include "../../tools/hmc_options.hpp"

extern "C" {
void *ora_create(int N, int L, const int *alleles, const char *types);
void *ora_create_from_phase(const char *path);
void ora_destroy(void *h);
void ora_set_threads(int n);
void ora_set_params(void *h, double min_freq_abs, int min_len, int max_len, int sample_size, int max_iter);
void ora_set_model(void *h, int model, int mc_order);
void ora_set_exact(void *h, int on);
void ora_set_num_patterns(void *h, int n);
int ora_run(void *h);
int ora_find_patterns(void *h);
double ora_resolve_all(void *h);
int ora_sample_count(void *h);
void ora_best_resolutions(void *h, int *out);
void ora_std_nth_element(double *lik, int *tag, int n, int nth);
}

static int failures = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                         \
    }                                                                     \
  } while (0)

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {  // SplitMix64
  uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// ---- store planning ----------------------------------------------------------
static void test_plan() {
  for (int trial = 0; trial < 400; ++trial) {
    const int n = 1 + (int)(rnd() % 3000);
    hmc::RegionPlanIn in;
    in.have_est = rnd() % 2;
    in.light = rnd() % 4 == 0;
    in.dev_cu = 1 + (int)(rnd() % 300);
    in.L = 1 + (int)(rnd() % 6000);
    in.rec_budget = 1 + rnd() % (1ull << 34);
    in.trace_budget = 1 + rnd() % (1ull << 35);
    in.rec_alloc = rnd() % 3 == 0 ? 0 : rnd() % (1ull << 34);
    std::vector<int32_t> pending(n);
    for (int i = 0; i < n; ++i) pending[i] = i;
    for (int i = n - 1; i > 0; --i) std::swap(pending[i], pending[rnd() % (i + 1)]);
    const std::vector<int32_t> before = pending;
    std::vector<char> exact(n);
    std::vector<unsigned long long> rneed(n), tneed(n), est(n), base(n, ~0ull), rsz(n, 0);
    for (int i = 0; i < n; ++i) {
      exact[i] = rnd() % 2;
      rneed[i] = rnd() % (1ull << 28);
      tneed[i] = rnd() % (1ull << 29);
      est[i] = rnd() % (1ull << 29);
    }
    uint64_t words = 0;
    const int k = hmc::plan_record_regions(in, pending, exact, rneed, tneed, est, base, rsz, &words);
    CHECK(k >= 1 && k <= n);
    // pending stays a permutation of the individuals
    std::vector<int32_t> a = pending, b = before;
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    CHECK(a == b);
    // the planned regions tile [0, words) in order and stay within the budget
    uint64_t at = 0;
    for (int q = 0; q < k; ++q) {
      const int bi = pending[q];
      CHECK(base[bi] == at);
      at += rsz[bi];
    }
    CHECK(at == words);
    if (in.have_est) {
      CHECK(words <= in.rec_budget);
      for (int q = 0; q < k; ++q)
        if (exact[pending[q]]) CHECK(rsz[pending[q]] == rneed[pending[q]] || words == in.rec_budget);
    } else {
      CHECK(k == (in.light ? n : std::min(n, 4 * in.dev_cu)));
      CHECK(words <= in.rec_budget);
    }
    // trace sub-groups cover the list, each within the budget unless alone
    std::vector<unsigned long long> tb(n, 0);
    size_t pos = 0, groups = 0;
    while (pos < pending.size()) {
      uint64_t t = 0;
      const size_t kk = hmc::plan_trace_group(pending, pos, tneed, in.trace_budget, tb, &t);
      CHECK(kk >= 1);
      CHECK(kk == 1 || t <= in.trace_budget);
      uint64_t s = 0;
      for (size_t q = 0; q < kk; ++q) {
        CHECK(tb[pending[pos + q]] == s);
        s += tneed[pending[pos + q]];
      }
      CHECK(s == t);
      pos += kk;
      ++groups;
    }
    CHECK(groups >= 1);
  }
}

// ---- HaploFile readers / writers ---------------------------------------------
static std::string dir;
static std::string put(const char *name, const std::string &text) {
  const std::string p = dir + "/" + name;
  FILE *f = fopen(p.c_str(), "w");
  fputs(text.c_str(), f);
  fclose(f);
  return p;
}

static void test_haplofile() {
  hmc::FileData d;
  std::string err;
  CHECK(hmc::read_geno_file("HPM", {put("a.hpm", "Id\tStatus\tM1 M2 M3\nind1\t0\t1 2 3\nind1\t0\t2 2 1\n"
                                                 "ind2\t1\t0 1 12\nind2\t1\t1 2 12\n")}, d, err));
  CHECK(d.N == 2 && d.L == 3 && d.types == "SSM");
  CHECK(hmc::read_geno_file("HPM2", {put("a.hpm2", "Id M1 M2 M3\nx\t1 A 1\nx\t2 0 3\ny\t2 A 4\ny\t1 A 2\n")}, d, err));
  CHECK(d.N == 2 && d.L == 3);
  const std::string g = put("g.txt", "1290   0 0 fam1\n2190   1 0 fam1\n1111   2 0 fam2\n2221   3 0 fam2\n");
  const std::string p = put("p.txt", " 0   rs1   100\n 1   rs2   250\n 2   rs3   400\n 3   rs4   900\n");
  CHECK(hmc::read_geno_file("BENCH2", {g, p}, d, err));
  CHECK(d.N == 2 && d.L == 4);
  const std::string c = put("c.txt", "1290   4 0 c1\n2190   5 0 c1\n");
  CHECK(hmc::read_geno_file("BENCH3", {g, p, c}, d, err));
  CHECK(d.N == 3 && d.unphased == 2);
  // writers: every format, the panel's own alleles as the resolutions
  for (const char *fmt : {"HPM", "HPM2", "BENCH2"}) {
    hmc::FileData e;
    std::vector<std::string> in = std::string(fmt) == "BENCH2" ? std::vector<std::string>{g, p}
                                                               : std::vector<std::string>{dir + "/a." + (std::string(fmt) == "HPM" ? "hpm" : "hpm2")};
    CHECK(hmc::read_geno_file(fmt, in, e, err));
    const std::string out = dir + "/out_" + fmt, out2 = dir + "/out2_" + fmt;
    CHECK(hmc::write_geno_file(fmt, out.c_str(), out2.c_str(), e, e.al, err));
    hmc::FileData back;
    std::vector<std::string> again = std::string(fmt) == "BENCH2" ? std::vector<std::string>{out, out2} : std::vector<std::string>{out};
    CHECK(hmc::read_geno_file(fmt, again, back, err));
    CHECK(back.al == e.al);
  }
  // malformed inputs: every reader must fail cleanly, never read past a line
  const char *bad_hpm[] = {"", "Id M1\n", "Id M1\nx\t1\ny\t2\nz\t1\n", "Name M1\nx\t1\nx\t2\n", "Id M1 M2\nx\t1\nx\t2 2 2 2 2\n",
                           "Id\nx\t\nx\t\n", "Id M1 M2 M3\nx\t1 2\nx\t1 2 3 4 5 6 7 8 9\n"};
  for (const char *t : bad_hpm) {
    hmc::FileData e;
    (void)hmc::read_geno_file("HPM", {put("bad.hpm", t)}, e, err);
    (void)hmc::read_geno_file("HPM2", {put("bad.hpm2", t)}, e, err);
  }
  const char *bad_bench[] = {"", "12\n", "129 0 0 a\n", "12345678901234567890 0 0 a\n1 1 0 a\n", "99 x y\n99 x y\n", "\n\n\n"};
  for (const char *t : bad_bench) {
    hmc::FileData e;
    (void)hmc::read_geno_file("BENCH2", {put("bad_g.txt", t), p}, e, err);
    (void)hmc::read_geno_file("BENCH3", {g, p, put("bad_c.txt", t)}, e, err);
    (void)hmc::read_geno_file("BENCH2", {g, put("bad_p.txt", t)}, e, err);
  }
  CHECK(!hmc::read_geno_file("HPM", {dir + "/missing.hpm"}, d, err));
  CHECK(!hmc::read_geno_file("BENCH9", {g}, d, err));
  CHECK(hmc::geno_file_count("BENCH3") == 3 && hmc::geno_file_count("PHASE") == 1 && hmc::geno_file_count("X") == 0);
}

// ---- hmc_resolve's options ---------------------------------------------------
static void test_options() {
  {
    const char *argv[] = {"hmc_resolve", "-f", "HPM", "-a", "2.5", "-m", "MC", "-o", "2", "--exact-estimate",
                          "--sample-size", "16", "-i", "7", "--output-patterns", "x", "a.hpm"};
    hmc_cli::Options o;
    std::string err;
    CHECK(hmc_cli::parse_options(17, argv, o, err) == 0);
    CHECK(o.format == "HPM" && o.min_freq_abs == 2.5 && o.model == "MC" && o.mc_order == 2 && o.exact &&
          o.sample_size == 16 && o.max_iteration == 7 && o.output_patterns && o.files.size() == 1);
  }
  {
    const char *argv[] = {"hmc_resolve", "-r", "0.01", "f1", "f2"};
    hmc_cli::Options o;
    std::string err;
    CHECK(hmc_cli::parse_options(5, argv, o, err) == 0 && o.min_freq_abs == 0 && o.min_freq == 0.01 && o.files.size() == 2);
  }
  for (int argc : {2, 3}) {
    const char *argv[] = {"hmc_resolve", "-a", "--bogus"};
    hmc_cli::Options o;
    std::string err;
    CHECK(hmc_cli::parse_options(argc, argv, o, err) != 0 && !err.empty());
  }
  {
    const char *argv[] = {"hmc_resolve"};
    hmc_cli::Options o;
    std::string err;
    CHECK(hmc_cli::parse_options(1, argv, o, err) != 0);
  }
}

// ---- the CPU restatement -----------------------------------------------------
static std::vector<int> mosaic(int N, int L, int A, double miss) {
  std::vector<int> f(8 * (size_t)L), al((size_t)N * 2 * L);
  for (auto &x : f) x = '1' + (int)(rnd() % A);
  for (int i = 0; i < N; ++i)
    for (int h = 0; h < 2; ++h) {
      int src = (int)(rnd() % 8);
      for (int k = 0; k < L; ++k) {
        if (rnd() % 1000 < 20) src = (int)(rnd() % 8);
        al[((size_t)i * 2 + h) * L + k] = (double)(rnd() % 10000) / 10000.0 < miss ? -1 : f[(size_t)src * L + k];
      }
    }
  return al;
}

static void test_oracle() {
  struct Case {
    int N, L, A;
    double miss;
    int model, order, S, threads, num;
    bool exact;
  } cases[] = {{30, 40, 2, 0.0, 0, 1, 10, 1, -1, false}, {40, 30, 3, 0.05, 0, 1, 5, 2, -1, false},
               {25, 30, 4, 0.02, 1, 2, 10, 2, -1, false}, {30, 25, 2, 0.0, 2, 1, 3, 1, -1, false},
               {20, 20, 2, 0.0, 0, 1, 10, 1, 60, false}, {20, 24, 3, 0.0, 0, 1, 10, 2, -1, true}};
  for (const Case &c : cases) {
    std::vector<int> al = mosaic(c.N, c.L, c.A, c.miss);
    ora_set_threads(c.threads);
    void *h = ora_create(c.N, c.L, al.data(), nullptr);
    ora_set_params(h, 1.5, 1, 30, c.S, 6);
    ora_set_model(h, c.model, c.order);
    if (c.num > 0) ora_set_num_patterns(h, c.num);
    ora_set_exact(h, c.exact ? 1 : 0);
    const int it = ora_run(h);
    CHECK(it >= 1);
    std::vector<int> res((size_t)c.N * 2 * c.L);
    ora_best_resolutions(h, res.data());
    for (int i = 0; i < c.N; ++i)  // the accepted pair phases the genotype
      for (int k = 0; k < c.L; ++k) {
        const int g0 = al[((size_t)i * 2) * c.L + k], g1 = al[((size_t)i * 2 + 1) * c.L + k];
        const int r0 = res[((size_t)i * 2) * c.L + k], r1 = res[((size_t)i * 2 + 1) * c.L + k];
        if (g0 >= 0 && g1 >= 0) CHECK((r0 == g0 && r1 == g1) || (r0 == g1 && r1 == g0));
      }
    ora_destroy(h);
  }
  ora_set_threads(1);
  // PHASE reader of the restatement, and a malformed file
  const std::string ph = put("a.inp", "2\n3\nP 100 250 400\nSSM\nfam1\n1 2 12\n2 2 3\n#7\n? 1 -\n1 1 4\n");
  void *h = ora_create_from_phase(ph.c_str());
  CHECK(h != nullptr);
  if (h) ora_destroy(h);
  void *bad = ora_create_from_phase(put("b.inp", "2\n3\nSSM\nfam1\n1 2\n").c_str());
  if (bad) ora_destroy(bad);
  // the libstdc++ selection the product's replica is checked against
  std::vector<double> lik(40);
  std::vector<int> tag(40);
  for (int i = 0; i < 40; ++i) { lik[i] = (double)(rnd() % 7); tag[i] = i; }
  ora_std_nth_element(lik.data(), tag.data(), 40, 9);
}

int main(int argc, char **argv) {
  dir = argc > 1 ? argv[1] : "/tmp";
  test_plan();
  test_options();
  test_haplofile();
  test_oracle();
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("sanitized host checks ok\n");
  return 0;
}
