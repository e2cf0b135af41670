// ============================================================================
// hmc_oracle.cpp — TEST INFRASTRUCTURE ONLY (never shipped, never measured as
// the product).  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load liboracle.so.
//
// A single-threaded CPU restatement of Wu-Lab/HMC's HaploModel EM loop (model
// "MV", sampling EM), written from a reading of /root/reference.  Each routine
// cites the reference file:line it restates.
//
// PARITY UNPINNED: the reference cannot be built in this image without
// stand-ins for Boost (boost/pool, tr1::shared_ptr, program_options are absent),
// which the build rules forbid, and the reference ships no tests, fixtures or
// golden vectors.  This restatement is therefore pinned only by hand-derived
// known-answer tests (tests/test_oracle.py) and by its own frozen regression
// vectors (tests/golden/).  See DESIGN.md §Oracle.
//
// Tie semantics: the reference selects k-best links with std::nth_element and
// std::sort (HaploPair.cpp:86, HaploBuilder.cpp:101,105).  This file calls the
// same libstdc++ (GCC 11.4) algorithms on the same element sequences, so its
// tie order is the one a g++-11 build of the reference would produce.
// ============================================================================
#include <algorithm>
#include <array>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <atomic>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace ora {

// Worker threads for the digest generators (tests/golden/make_*_digest.py):
// mining splits the start loci (each root's DFS subtree is independent,
// PatternManager.cpp:94-97,106-108), initialize() the successor lookups and
// resolveAll() the individuals (HaploModel.cpp:86 is independent per
// individual).  Every result is assembled in the reference's order, so the
// outputs are identical to the single-threaded run (default 1).
static int g_threads = 1;
template <class F>
static void parallel_for(int n, int chunk, F f) {  // f(begin, end), dynamic chunks
  const int nt = std::max(1, std::min(g_threads, (n + chunk - 1) / std::max(chunk, 1)));
  if (nt <= 1) { if (n > 0) f(0, n); return; }
  std::atomic<int> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (int b; (b = next.fetch_add(chunk)) < n;) f(b, std::min(n, b + chunk));
    });
  for (auto &x : th) x.join();
}

// ---------------------------------------------------------------- alleles --
// Allele.h:11-36 — an int, negative = missing; isMatch treats missing as a
// wildcard, operator== treats two missings as equal.
static inline bool missing(int a) { return a < 0; }
static inline bool amatch(int a, int b) { return a < 0 || b < 0 || a == b; }
static inline bool aeq(int a, int b) { return a == b || (a < 0 && b < 0); }

// --------------------------------------------------------------- genodata --
struct Geno {
  int N = 0, L = 0;
  std::vector<int> al;  // [N][2][L] allele symbols
  std::string types;    // per-locus type char ('S' SNP, 'M' microsatellite)
  std::vector<std::vector<std::pair<int, double>>> sym;  // per locus (symbol, freq)

  int at(int i, int h, int k) const { return al[((size_t)i * 2 + h) * L + k]; }
  int num(int k) const { return (int)sym[k].size(); }
  int symbol(int k, int j) const { return sym[k][j].first; }
  double afreq(int k, int j) const { return sym[k][j].second; }
  int maxnum() const {
    int m = 0;
    for (int k = 0; k < L; ++k) m = std::max(m, num(k));
    return m;
  }
  // GenoData.cpp:27-44 — linear search with Allele operator==.
  int index(int k, int a) const {
    for (int j = 0; j < num(k); ++j)
      if (aeq(a, sym[k][j].first)) return j;
    return -1;
  }
  // Genotype.h:115-133
  bool isMissing(int i, int k) const { return missing(at(i, 0, k)) && missing(at(i, 1, k)); }
  bool hasMissing(int i, int k) const { return missing(at(i, 0, k)) || missing(at(i, 1, k)); }
  bool hasAllele(int i, int k, int a) const { return aeq(at(i, 0, k), a) || aeq(at(i, 1, k), a); }
  bool isHet(int i, int k) const { return !amatch(at(i, 0, k), at(i, 1, k)); }
  bool gmatch(int i, int k, int a) const { return amatch(at(i, 0, k), a) || amatch(at(i, 1, k), a); }

  // GenoData.cpp:78-118 — distinct non-missing symbols in first-seen order,
  // sorted by value, frequency = count / non-missing count (weights are 1.0).
  void checkAlleleSymbol() {
    sym.assign(L, {});
    for (int i = 0; i < N; ++i)
      for (int h = 0; h < 2; ++h)
        for (int k = 0; k < L; ++k) {
          int a = at(i, h, k);
          if (!missing(a) && index(k, a) < 0) sym[k].push_back({a, 0.0});
        }
    for (int k = 0; k < L; ++k) std::sort(sym[k].begin(), sym[k].end());
    std::vector<double> tot(L, 0.0);
    for (int i = 0; i < N; ++i)
      for (int h = 0; h < 2; ++h)
        for (int k = 0; k < L; ++k) {
          int a = at(i, h, k);
          if (!missing(a)) {
            sym[k][index(k, a)].second += 1.0;
            tot[k] += 1.0;
          }
        }
    for (int k = 0; k < L; ++k)
      for (auto &p : sym[k]) p.second /= tot[k];
  }
};

// ------------------------------------------------------------ PHASE input --
// HaploFile.cpp:54-118 (m_has_id = true, HaploFile.h:44-53) and
// Allele.cpp:55-153 (readAllele / AlleleSequence::read with types).
static const char *DELIM = " \t\r\n";
static char *read_allele(char type, char *buf, int &a) {
  buf += strspn(buf, DELIM);
  if (type == 'S') {
    a = (buf[0] == '-' || buf[0] == '?') ? -1 : (int)(unsigned char)buf[0];
    if (buf[0]) buf++;
  } else {
    if (buf[0] == '-' || buf[0] == '?') a = -1;
    else {
      int v = atoi(buf);
      a = v > 0 ? v : -1;
    }
    buf += strcspn(buf, DELIM);
  }
  return buf;
}

static bool read_phase(const char *path, Geno &g, std::string &err) {
  FILE *fp = fopen(path, "r");
  if (!fp) { err = "Can not open file"; return false; }
  int n = 0, l = 0;
  if (fscanf(fp, "%d\n", &n) != 1 || fscanf(fp, "%d\n", &l) != 1 || n <= 0 || l <= 0) {
    fclose(fp);
    err = "Invalid file type!";
    return false;
  }
  g.N = n;
  g.L = l;
  g.al.assign((size_t)n * 2 * l, -1);
  std::vector<char> line(std::max<size_t>(409600, (size_t)l * 64 + 1024));
  if (!fgets(line.data(), (int)line.size(), fp)) { fclose(fp); err = "truncated"; return false; }
  char *s = line.data() + strspn(line.data(), DELIM);
  if (s[0] == 'P') {
    if (!fgets(line.data(), (int)line.size(), fp)) { fclose(fp); err = "truncated"; return false; }
    s = line.data() + strspn(line.data(), DELIM);
  }
  g.types.assign(l, 'M');
  for (int k = 0; k < l; ++k) {
    g.types[k] = s[0];
    if (s[0]) s++;
    s += strspn(s, DELIM);
  }
  for (int i = 0; i < n; ++i) {
    for (int r = 0; r < 3; ++r) {
      if (!fgets(line.data(), (int)line.size(), fp)) { fclose(fp); err = "truncated"; return false; }
      if (r == 0) continue;  // id line
      char *b = line.data();
      for (int k = 0; k < l; ++k) {
        int a;
        b = read_allele(g.types[k], b, a);
        g.al[((size_t)i * 2 + (r - 1)) * l + k] = a;
      }
    }
  }
  fclose(fp);
  g.checkAlleleSymbol();
  return true;
}

// ---------------------------------------------------------------- pattern --
// HaploPattern.h:16-98.  Alleles are symbols; end is exclusive.
struct Pat {
  int start = 0, end = 0;
  std::vector<int> al;
  unsigned id = 0;
  double freq = 1.0, prefix = 1.0, tp = 1.0;  // HaploPattern.h:86-88 defaults
  std::vector<int> succ;                     // successor pattern index or -1
  int len() const { return (int)al.size(); }
  void setTp(double p) { tp = p < 1.0 ? p : 1.0; }  // HaploPattern.h:47
};

// ----------------------------------------------------- BackwardPatternTree --
// PatternTree.cpp:15-72,98-134, Tree.h:12-99: one trie per end locus, walked
// from the last allele backwards.  Node data = pattern index (or -1).
struct BTree {
  struct Node { std::vector<int> ch; int data = -1; };
  const Geno *g = nullptr;
  std::vector<Node> nodes;
  std::vector<int> root;  // per end locus 0..L
  int width = 0;

  int newNode() { nodes.push_back(Node{std::vector<int>(width, -1), -1}); return (int)nodes.size() - 1; }
  void init(const Geno &gd) {
    g = &gd;
    width = gd.maxnum();
    nodes.clear();
    root.assign(gd.L + 1, -1);
    for (int e = 0; e <= gd.L; ++e) root[e] = newNode();
  }
  int addChild(int n, int i) {
    if (nodes[n].ch[i] < 0) { int c = newNode(); nodes[n].ch[i] = c; }
    return nodes[n].ch[i];
  }
  // PatternTree.cpp:24-48
  void add(const std::vector<Pat> &P, int pi) { addRec(root[P[pi].end], P, pi, P[pi].len()); }
  void addRec(int n, const std::vector<Pat> &P, int pi, int len) {
    const Pat &p = P[pi];
    int locus = p.start + len - 1;
    int a = p.al[len - 1];
    int i = missing(a) ? -1 : g->index(locus, a);
    if (i < 0) {
      for (int j = 0; j < g->num(locus); ++j) {
        if (len == 1) nodes[addChild(n, j)].data = pi;
        else addRec(addChild(n, j), P, pi, len - 1);
      }
    } else {
      if (len == 1) nodes[addChild(n, i)].data = pi;
      else addRec(addChild(n, i), P, pi, len - 1);
    }
  }
  // PatternTree.cpp:62-72 (AlleleSequence overload)
  int longest(const std::vector<Pat> &P, int end, const std::vector<int> &as, int as_start) const {
    int aslen = (int)as.size();
    if (end <= as_start || end > as_start + aslen) return -1;
    int maxl = end - as_start;
    return walk(P, root[end], as, end - 1, maxl - 1, maxl);
  }
  // PatternTree.cpp:98-134
  int walk(const std::vector<Pat> &P, int n, const std::vector<int> &as, int lg, int ll, int len) const {
    int result = nodes[n].data;
    auto consider = [&](int c) {
      int tmp = len > 1 ? walk(P, c, as, lg - 1, ll - 1, len - 1) : nodes[c].data;
      if (result < 0 || (tmp >= 0 && P[tmp].len() > P[result].len())) result = tmp;
    };
    if (missing(as[ll])) {
      for (int i = 0; i < g->num(lg); ++i)
        if (nodes[n].ch[i] >= 0) consider(nodes[n].ch[i]);
    } else {
      int i = g->index(lg, as[ll]);
      if (i >= 0 && nodes[n].ch[i] >= 0) consider(nodes[n].ch[i]);
    }
    return result;
  }
};

// --------------------------------------------------------------- E-step --
// HaploPair.h:14-52 — a k-best link.  pred = -1 marks a head pair.
struct Link {
  int pred;
  int index;
  bool rev;
  bool homo;
  double lik;
};
struct GreaterLik {  // std::greater<HaploPairLink> via HaploPair.h:49-52
  bool operator()(const Link &a, const Link &b) const { return a.lik > b.lik; }
};

// HaploPair.h:55-100 — an unordered pattern pair (canonical: id_a <= id_b).
struct Pair {
  int pa, pb;
  int alA, alB;  // last alleles of the two patterns
  double tp, fwd;
  std::vector<Link> links;
  // exact M-step only: m_forward_links[reversed] (HaploPair.cpp:44,67) as
  // indices into the next locus, and m_backward_likelihood (default 1.0)
  std::vector<int> fl[2];
  double bwd = 1.0;
  // exact M-step only: the pair's contributions in add order (predecessor,
  // reversed) — the order HaploPair.cpp:42 / :66 sums its forward likelihood
  std::vector<std::pair<int, bool>> in;
};

struct Sample {  // one weighted haplotype of HaploData (HaploData.h:57-65)
  std::vector<int> al;
  double w;
};

struct Candidate {  // one entry of res_list (HaploBuilder.cpp:105-114)
  std::vector<int> h0, h1;
  double prior, posterior, gp;
};

struct Params {
  double min_freq_abs = 1.5;  // HMC.cpp:37
  double min_freq = -1;       // HaploModel.cpp:10
  int min_len = 1;            // HMC.cpp:39
  int max_len = 30;           // HMC.cpp:40
  int sample_size = 10;       // HMC.cpp:43
  int max_iter = 1;           // HMC.cpp:46
  int model = 0;              // HaploModel::setModel (HaploModel.cpp:26-36): 0 MV, 1 MC, 2 MA
  int num_patterns = -1;      // HMC.cpp:38 (findPatternByNum when > 0)
  int mc_order = 1;           // HMC.cpp:41
  bool exact = false;         // --exact-estimate (HMC.cpp:42, HaploModel.h:26)
  // exact M-step summation: 0 = the device walk's order (xwalk, bit-exact
  // with exact.hip); 1 = the reference's grouping in double (rwalk: list 0,
  // then 1, then 2, predecessors in creation order for std::map's pointer
  // order, every frequency and prefix added in double) — the independent
  // check at the north star's 1e-6 bar
  int exact_order = 0;
};

struct Timing { double m0 = 0, e = 0, m = 0; };

struct Model {
  Geno g;       // the input panel (true phase kept for HaploComp)
  Params prm;
  std::vector<Pat> P;
  BTree tree;
  std::vector<int> head_list;
  std::vector<int> minlen, maxlen;
  double min_freq = 0;
  // samples (HaploData)
  std::vector<Sample> samples;
  double total_weight = 0;
  // last E-step results
  std::vector<std::vector<Candidate>> res;  // per individual
  std::vector<double> gp;                   // genotype probability per individual
  std::vector<std::vector<int>> resolution; // per individual: [2][L]
  std::vector<std::vector<int>> best_res;   // accepted resolutions (HaploModel.cpp:132)
  // counters
  uint64_t R_E = 0, R_M = 0;
  // Tie diagnostics of the last E-step, per individual (bit 0: some key's
  // union of contributions has a non-zero tie across its S-cut, bit 1: the
  // same at likelihood 0, bit 2: the final union has a tie across the S-cut,
  // bit 3: two of the final candidates have equal non-zero priors, bit 4: the
  // final union has a tie across the S-cut at 0, bit 5: a final candidate has
  // prior 0).  With none set,
  // every k-best set is decided by likelihood values alone.
  std::vector<int> tie_flags;
  static thread_local std::vector<std::vector<double>> uni;  // per state of the next locus
  static thread_local int tie_cur;
  static thread_local uint64_t tl_rm;  // R_M of this thread's scans, folded into R_M per search
  void uni_add(int st, const Link *l, int n) {
    if ((int)uni.size() <= st) uni.resize(st + 1);
    for (int i = 0; i < n; ++i) uni[st].push_back(l[i].lik);
  }
  void uni_check(int nst) {
    for (int s = 0; s < nst && s < (int)uni.size(); ++s) {
      std::vector<double> &u = uni[s];
      if ((int)u.size() > S) {
        std::sort(u.begin(), u.end(), std::greater<double>());
        if (u[S - 1] == u[S]) tie_cur |= u[S] == 0.0 ? 2 : 1;
      }
      u.clear();
    }
  }
  // EM log
  std::vector<double> ll_log;
  std::vector<uint64_t> re_log, rm_log;
  std::vector<int> npat_log;
  std::vector<double> t_e_log, t_m_log;
  double t_m0 = 0;
  int iterations = 0;

  // ------------------------------------------------------------ mining ----
  struct Cand {
    Pat p;
    std::vector<std::pair<int, double>> st;  // MatchingState (PatternManager.h:19)
  };

  int head_len() const { return minlen[0]; }

  // PatternManager.cpp:349-373
  double matchFreq(int i, const int *pa, int start, int len) const {
    double tot = 1.0;
    for (int k = 0; k < len; ++k) {
      if (missing(pa[k])) continue;
      double f = 0;
      for (int h = 0; h < 2; ++h) {
        int b = g.at(i, h, start + k);
        if (missing(b)) f += g.afreq(start + k, g.index(start + k, pa[k]));
        else if (aeq(b, pa[k])) f += 1.0;
      }
      tot *= 0.5 * f;
    }
    return tot;
  }
  bool genoMatch(int i, const Pat &p, int start, int len) const {  // Genotype.cpp:79-96
    int s2 = start - p.start;
    if (start + len > g.L || s2 + len > p.len()) return false;
    for (int k = 0; k < len; ++k)
      if (!g.gmatch(i, start + k, p.al[s2 + k])) return false;
    return true;
  }
  bool hapMatch(const Sample &h, const Pat &p, int start, int len) const {  // Allele.cpp:11-28
    int s2 = start - p.start;
    if (start + len > (int)h.al.size() || s2 + len > p.len()) return false;
    for (int k = 0; k < len; ++k)
      if (!amatch(h.al[start + k], p.al[s2 + k])) return false;
    return true;
  }

  // PatternManager.cpp:146-193 (phased branches are dead: Genotype.cpp:40)
  void checkFrequency(Pat &p, std::vector<std::pair<int, double>> &ms) {
    ms.clear();
    if (p.len() == 0) { p.freq = 1.0; return; }
    double tot = 0;
    if (samples.empty()) {
      for (int i = 0; i < g.N; ++i) {
        ++tl_rm;
        if (genoMatch(i, p, p.start, p.len())) {
          double f = matchFreq(i, p.al.data(), p.start, p.len());
          tot += f;
          ms.push_back({i, f});
        }
      }
      p.freq = tot / g.N;
    } else {
      for (int i = 0; i < (int)samples.size(); ++i) {
        ++tl_rm;
        if (hapMatch(samples[i], p, p.start, p.len())) {
          tot += samples[i].w;
          ms.push_back({i, 0.0});
        }
      }
      p.freq = tot / total_weight;
    }
  }
  // PatternManager.cpp:195-265
  void checkFreqExt(Pat &p, std::vector<std::pair<int, double>> &ms,
                    const std::vector<std::pair<int, double>> &oms, int start) {
    if (p.len() == 0 || oms.empty()) { checkFrequency(p, ms); return; }
    ms.clear();
    double tot = 0;
    if (samples.empty()) {
      for (auto &e : oms) {
        ++tl_rm;
        if (genoMatch(e.first, p, start, 1)) {
          double f = e.second * matchFreq(e.first, &p.al[start - p.start], start, 1);
          tot += f;
          ms.push_back({e.first, f});
        }
      }
      p.freq = tot / g.N;
    } else {
      for (auto &e : oms) {
        ++tl_rm;
        if (hapMatch(samples[e.first], p, start, 1)) {
          tot += samples[e.first].w;
          ms.push_back({e.first, 0.0});
        }
      }
      p.freq = tot / total_weight;
    }
  }

  // PatternManager::searchPattern (:100-144) on an explicit candidate stack;
  // with `reserve`, candidates that fail the threshold are kept (in pop order)
  // for the next round instead of deleted.
  std::vector<Cand *> searchPattern(std::vector<Cand *> &stack, bool reserve) { return searchPattern(stack, reserve, P); }
  std::vector<Cand *> searchPattern(std::vector<Cand *> &stack, bool reserve, std::vector<Pat> &out) {
    const int L = g.L;
    std::vector<Cand *> kept;
    while (!stack.empty()) {
      Cand *pc = stack.back();
      stack.pop_back();
      const Pat &hp = pc->p;
      if (hp.freq >= min_freq || hp.len() < minlen[hp.start]) {
        if (hp.end < L && hp.len() < maxlen[hp.start]) {
          for (int i = 0; i < g.num(hp.end); ++i) {
            if (g.afreq(hp.end, i) > 0) {
              Cand *nc = new Cand;
              nc->p.start = hp.start;
              nc->p.end = hp.end + 1;
              nc->p.al = hp.al;
              nc->p.al.push_back(g.symbol(hp.end, i));
              nc->p.freq = hp.freq;
              checkFreqExt(nc->p, nc->st, pc->st, hp.end);
              nc->p.prefix = hp.freq;
              if (nc->p.prefix > 0) nc->p.setTp(nc->p.freq / nc->p.prefix);
              else nc->p.setTp(nc->p.freq);
              stack.push_back(nc);
            }
          }
        }
      }
      if (hp.freq >= min_freq || hp.len() <= minlen[hp.start]) {
        if (hp.len() > 0 && hp.len() >= minlen[hp.start]) out.push_back(pc->p);
        delete pc;
      } else if (reserve) {
        kept.push_back(pc);
      } else {
        delete pc;
      }
    }
    __atomic_fetch_add(&R_M, tl_rm, __ATOMIC_RELAXED);
    tl_rm = 0;
    return kept;
  }

  // generateCandidates (:90-98): one empty pattern per start locus
  std::vector<Cand *> generateCandidates() {
    std::vector<Cand *> stack;
    for (int s = 0; s < g.L; ++s) {
      Cand *c = new Cand;
      c->p.start = c->p.end = s;
      stack.push_back(c);
    }
    return stack;
  }

  // PatternManager.cpp:27-42 — DFS mining; output order = DFS pre-order.
  void findPatternByFreq(double mf, int mnl, int mxl) {
    int L = g.L;
    mxl = mxl <= 0 ? L : mxl;
    mnl = std::max(mnl, 1);
    mxl = std::max(mxl, mnl);
    minlen.resize(L, mnl);  // vector::resize keeps old values (PatternManager.cpp:33-34)
    maxlen.resize(L, mxl);
    P.clear();
    min_freq = mf;
    if (g_threads <= 1) {
      std::vector<Cand *> stack = generateCandidates();
      searchPattern(stack, false);
    } else {
      // roots are popped from the back (start L-1 first): chunk c of start
      // loci [c*K, c*K+K) yields the DFS blocks of its roots in descending
      // start order, and the chunks concatenate in descending order
      const int K = 4, nch = (L + K - 1) / K;
      std::vector<std::vector<Pat>> part(nch);
      parallel_for(nch, 1, [&](int b, int e) {
        for (int c = b; c < e; ++c) {
          std::vector<Cand *> stack;
          for (int s = c * K; s < std::min(L, c * K + K); ++s) {
            Cand *x = new Cand;
            x->p.start = x->p.end = s;
            stack.push_back(x);
          }
          searchPattern(stack, false, part[c]);
        }
      });
      size_t tot = 0;
      for (auto &v : part) tot += v.size();
      P.reserve(tot);
      for (int c = nch - 1; c >= 0; --c) {
        for (auto &p : part[c]) P.push_back(std::move(p));
        std::vector<Pat>().swap(part[c]);
      }
    }
    initialize();
  }

  // PatternManager::findPatternByNum (:44-70): thresholds 1.0, 0.9, 0.81, ...
  // over rounds of searchPattern(true) until max_num patterns; the last
  // round's patterns sorted by frequency (std::sort, greater_frequency) and cut.
  void findPatternByNum(int max_num, int mnl, int mxl) {
    int L = g.L;
    mxl = mxl <= 0 ? L : mxl;
    mnl = std::max(mnl, 1);
    mxl = std::max(mxl, mnl);
    minlen.resize(L, mnl);
    maxlen.resize(L, mxl);
    P.clear();
    std::vector<Cand *> stack = generateCandidates();
    min_freq = 1.0;
    stack = searchPattern(stack, true);
    max_num = std::max(max_num, (int)P.size());
    int last_size = 0;
    while ((int)P.size() < max_num && min_freq > 1e-38) {
      last_size = (int)P.size();
      min_freq *= 0.9;
      stack = searchPattern(stack, true);
    }
    if ((int)P.size() > max_num) {
      std::sort(P.begin() + last_size, P.end(), [](const Pat &a, const Pat &b) { return a.freq > b.freq; });
      P.resize(max_num);
    }
    for (Cand *c : stack) delete c;
    initialize();
  }

  // PatternManager.cpp:293-318
  void initialize() {
    tree.init(g);
    head_list.clear();
    int n = (int)P.size();
    for (int i = 0; i < n; ++i) {
      P[i].id = i;
      tree.add(P, i);
      if (P[i].start == 0 && P[i].len() == head_len()) head_list.push_back(i);
    }
    parallel_for(n, 4096, [&](int b, int e) {
      std::vector<int> tmp;
      for (int i = b; i < e; ++i) {
        Pat &p = P[i];
        p.succ.clear();
        if (p.end < g.L) {
          tmp = p.al;
          tmp.push_back(-1);
          for (int j = 0; j < g.num(p.end); ++j) {
            tmp.back() = g.symbol(p.end, j);
            int s = tree.longest(P, p.end + 1, tmp, p.start);
            p.succ.resize(j + 1);
            p.succ[j] = s;
          }
        }
      }
    });
  }

  // HaploModel.cpp:52-63
  void findPatterns() {
    if (prm.min_freq_abs > 0) prm.min_freq = prm.min_freq_abs / (2.0 * g.N);
    if (prm.model == 1) {
      // MC: findPatternBlock(mc_order+1) (PatternManager.cpp:72-88): every
      // candidate of length mc_order+1 (m_min_freq = -1 accepts all)
      const int len = std::max(1, prm.mc_order + 1);
      findPatternByFreq(-1.0, len, len);
    } else if (prm.num_patterns > 0) {  // HaploModel.cpp:58-60, 70-72
      findPatternByNum(prm.num_patterns, prm.min_len, prm.max_len);
    } else {
      // MV, and MA whose adjustFrequency (PatternManager.cpp:320-345) only
      // range-checks the table
      findPatternByFreq(prm.min_freq, prm.min_len, prm.max_len);
    }
  }

  // ------------------------------------------------------------ E-step ----
  static thread_local std::vector<std::vector<Pair>> hp;  // m_haplopairs
  static thread_local int S;
  static thread_local bool track_links;  // record forward links (exact M-step)

  int succOf(int pi, int a, int locus) const {  // HaploPattern.h:36-37
    int j = g.index(locus, a);
    const Pat &p = P[pi];
    return (j >= 0 && j < (int)p.succ.size()) ? p.succ[j] : -1;
  }

  // HaploPair.cpp:14-33 — head constructor.
  Pair headPair(int a, int b) {
    Pair x;
    x.pa = a; x.pb = b;
    x.alA = P[a].al.back(); x.alB = P[b].al.back();
    x.fwd = x.tp = P[a].freq * P[b].freq;
    bool homo = (P[a].id == P[b].id);
    if (!homo) x.fwd *= 2.0;
    x.links.push_back(Link{-1, 0, false, homo, x.tp});
    return x;
  }

  // HaploBuilder.cpp:153-224 (head_len general).
  void initHeadList(int gi, std::unordered_map<uint64_t, int> &best) {
    int hl = head_len();
    for (int head : head_list) {
      const Pat &H = P[head];
      if (!genoMatch(gi, H, H.start, H.len())) continue;
      std::vector<std::vector<int>> last(1), next;
      for (int j = 0; j < hl; ++j) {
        next.clear();
        if (g.isMissing(gi, j) || (g.hasMissing(gi, j) && g.hasAllele(gi, j, H.al[j]))) {
          for (auto &as : last)
            for (int k = 0; k < g.num(j); ++k)
              if (g.afreq(j, k) > 0) { next.push_back(as); next.back().push_back(g.symbol(j, k)); }
        } else if (g.isHet(gi, j)) {
          for (auto &as : last) {
            next.push_back(as);
            next.back().push_back(aeq(H.al[j], g.at(gi, 0, j)) ? g.at(gi, 1, j) : g.at(gi, 0, j));
          }
        } else {
          for (auto &as : last) { next.push_back(as); next.back().push_back(g.at(gi, 0, j)); }
        }
        last.swap(next);
      }
      for (auto &as : last) {
        int q = tree.longest(P, hl, as, 0);
        if (q >= 0 && P[q].start == 0) {
          if (P[q].id >= H.id) {
            hp[hl].push_back(headPair(head, q));
            best[((uint64_t)P[head].id << 32) | P[q].id] = (int)hp[hl].size();
          }
        } else {
          fprintf(stderr, "Can not find matching pattern!\n");
          exit(1);
        }
      }
    }
  }

  // HaploBuilder.cpp:246-261 + HaploPair.cpp:35-89
  void addPair(int locus, int predIdx, int a, int b, std::unordered_map<uint64_t, int> &best) {
    const Pair &pred = hp[locus][predIdx];
    bool rev = false;
    if (P[a].id > P[b].id) { rev = true; std::swap(a, b); }
    uint64_t key = ((uint64_t)P[a].id << 32) | P[b].id;
    auto it = best.find(key);
    std::vector<Pair> &nxt = hp[locus + 1];
    if (track_links)  // hp->m_forward_links[reversed].push_back(this) (HaploPair.cpp:44, 67)
      hp[locus][predIdx].fl[rev ? 1 : 0].push_back(it == best.end() ? (int)nxt.size() : it->second - 1);
    if (it == best.end()) {
      Pair x;  // extension constructor HaploPair.cpp:35-61
      x.pa = a; x.pb = b;
      x.alA = P[a].al.back(); x.alB = P[b].al.back();
      x.tp = P[a].tp * P[b].tp;
      x.fwd = pred.fwd * x.tp;
      x.links = pred.links;
      for (int i = 0; i < (int)x.links.size(); ++i) {
        x.links[i].pred = predIdx;
        x.links[i].index = i;
        x.links[i].rev = rev;
        x.links[i].lik *= x.tp;
      }
      if (!aeq(x.alA, x.alB))
        for (auto &l : x.links)
          if (l.homo) { if (rev) l.lik = 0; l.homo = false; }
      if (track_links) x.in.emplace_back(predIdx, rev);
      nxt.push_back(std::move(x));
      best[key] = (int)nxt.size();
      uni_add((int)nxt.size() - 1, nxt.back().links.data(), (int)nxt.back().links.size());
    } else {
      Pair &x = nxt[it->second - 1];  // HaploPair::add, HaploPair.cpp:63-89
      if (track_links) x.in.emplace_back(predIdx, rev);
      x.fwd += pred.fwd * x.tp;
      int k = (int)x.links.size();
      int n = (int)pred.links.size();
      x.links.insert(x.links.end(), pred.links.begin(), pred.links.end());
      for (int i = k; i < k + n; ++i) {
        x.links[i].pred = predIdx;
        x.links[i].index = i - k;
        x.links[i].rev = rev;
        x.links[i].lik *= x.tp;
      }
      if (!aeq(x.alA, x.alB))
        for (int i = k; i < k + n; ++i)
          if (x.links[i].homo) { if (rev) x.links[i].lik = 0; x.links[i].homo = false; }
      uni_add(it->second - 1, x.links.data() + k, n);
      if ((int)x.links.size() > S) {
        std::nth_element(x.links.begin(), x.links.begin() + S - 1, x.links.end(), GreaterLik());
        x.links.resize(S);
      }
    }
  }

  // HaploBuilder.cpp:226-244
  void extendAll(int locus, int a1, int a2, std::unordered_map<uint64_t, int> &best) {
    int n = (int)hp[locus].size();
    for (int s = 0; s < n; ++s) {
      for (int o = 0; o < (aeq(a1, a2) ? 1 : 2); ++o) {
        int x = o ? a2 : a1, y = o ? a1 : a2;
        const Pair &q = hp[locus][s];
        if (q.fwd <= 0) {  // extend(): not extended (HaploBuilder.cpp:237); counted for the tests' panel search
          ++n_skip;
          continue;
        }
        int sa = succOf(q.pa, x, P[q.pa].end);
        int sb = succOf(q.pb, y, P[q.pb].end);
        if (sa >= 0 && sb >= 0) addPair(locus, s, sa, sb, best);
      }
    }
  }

  // HaploPair.cpp:91-124
  void traceback(int locus, int state, int index, std::vector<int> &h0, std::vector<int> &h1) const {
    std::vector<int> *gh[2] = {&h0, &h1};
    h0.assign(g.L, -1);
    h1.assign(g.L, -1);
    int a = 0, b = 1;
    int i = g.L - 1;
    int lc = locus, st = state;
    while (true) {
      const Pair &x = hp[lc][st];
      if (index < (int)x.links.size() && x.links[index].pred >= 0) {
        (*gh[a])[i] = P[x.pa].al[i - P[x.pa].start];
        (*gh[b])[i] = P[x.pb].al[i - P[x.pb].start];
        if (x.links[index].rev) std::swap(a, b);
        int nst = x.links[index].pred;
        index = x.links[index].index;
        st = nst;
        --lc;
        --i;
      } else {
        const Pat &pa = P[x.pa], &pb = P[x.pb];
        for (int k = 0; k < i + 1 - pa.start; ++k) (*gh[a])[pa.start + k] = pa.al[k];
        for (int k = 0; k < i + 1 - pb.start; ++k) (*gh[b])[pb.start + k] = pb.al[k];
        break;
      }
    }
  }

  // HaploBuilder.cpp:35-126 — returns coverage.
  double resolve(int gi, std::vector<Candidate> &out, std::vector<int> &resol, double &gprob, int sample_size = 0) {
    int L = g.L, hl = head_len();
    const int ss = sample_size > 0 ? sample_size : prm.sample_size;
    S = ss > 1 ? ss : 1;
    hp.assign(L + 1, {});
    tie_cur = 0;
    std::vector<std::unordered_map<uint64_t, int>> best(L + 1);
    initHeadList(gi, best[hl]);
    for (int i = hl; i < L; ++i) {
      std::unordered_map<uint64_t, int> &bm = best[i + 1];
      if (g.isMissing(gi, i)) {
        for (int j = 0; j < g.num(i); ++j)
          if (g.afreq(i, j) > 0)
            for (int k = j; k < g.num(i); ++k)
              if (g.afreq(i, k) > 0) extendAll(i, g.symbol(i, j), g.symbol(i, k), bm);
      } else if (missing(g.at(gi, 0, i))) {
        for (int j = 0; j < g.num(i); ++j)
          if (g.afreq(i, j) > 0) extendAll(i, g.symbol(i, j), g.at(gi, 1, i), bm);
      } else if (missing(g.at(gi, 1, i))) {
        for (int j = 0; j < g.num(i); ++j)
          if (g.afreq(i, j) > 0) extendAll(i, g.symbol(i, j), g.at(gi, 0, i), bm);
      } else {
        extendAll(i, g.at(gi, 0, i), g.at(gi, 1, i), bm);
      }
      uni_check((int)hp[i + 1].size());
      if (hp[i + 1].empty()) break;
    }
    uint64_t re = 0;
    for (int i = hl; i <= L; ++i)
      for (auto &x : hp[i]) re += x.links.size();
    __atomic_fetch_add(&R_E, re, __ATOMIC_RELAXED);
    out.clear();
    double coverage = 0;
    if (!hp[L].empty()) {
      double total = 0;
      std::vector<Link> rl;
      std::vector<double> fu;
      for (int s = 0; s < (int)hp[L].size(); ++s) {
        const Pair &x = hp[L][s];
        total += x.fwd;
        int k = (int)rl.size(), n = (int)x.links.size();
        rl.insert(rl.end(), x.links.begin(), x.links.end());
        for (int i = k; i < k + n; ++i) {
          rl[i].pred = s;
          rl[i].index = i - k;
          if (!rl[i].homo) rl[i].lik *= 2.0;
          fu.push_back(rl[i].lik);
        }
        if ((int)rl.size() > S) {
          std::nth_element(rl.begin(), rl.begin() + S - 1, rl.end(), GreaterLik());
          rl.resize(S);
        }
      }
      std::sort(rl.begin(), rl.end(), GreaterLik());
      std::sort(fu.begin(), fu.end(), std::greater<double>());
      if ((int)fu.size() > S && fu[S - 1] == fu[S]) tie_cur |= fu[S] == 0.0 ? 16 : 4;
      for (int i = 1; i < (int)rl.size(); ++i)
        if (rl[i].lik == rl[i - 1].lik && rl[i].lik != 0.0) tie_cur |= 8;
      for (auto &l : rl)
        if (l.lik == 0.0) tie_cur |= 32;
      for (auto &l : rl) {
        Candidate c;
        traceback(L, l.pred, l.index, c.h0, c.h1);
        const Link &own = hp[L][l.pred].links[l.index];
        c.prior = own.homo ? own.lik : own.lik * 2.0;  // HaploPair.cpp:97-102
        c.posterior = c.prior / total;
        c.gp = total;
        coverage += c.posterior;
        out.push_back(std::move(c));
      }
      resol.assign(2 * L, 0);
      std::copy(out[0].h0.begin(), out[0].h0.end(), resol.begin());
      std::copy(out[0].h1.begin(), out[0].h1.end(), resol.begin() + L);
      gprob = total;
    } else {  // HaploBuilder.cpp:117-124
      resol.assign(2 * L, 0);
      for (int k = 0; k < L; ++k) { resol[k] = g.at(gi, 0, k); resol[L + k] = g.at(gi, 1, k); }
      gprob = 0;
    }
    return coverage;
  }

  // HaploModel.cpp:79-115
  double resolveAll() {
    samples.clear();
    res.assign(g.N, {});
    gp.assign(g.N, 0.0);
    resolution.assign(g.N, {});
    tie_flags.assign(g.N, 0);
    std::vector<double> cov(g.N, 0.0);
    parallel_for(g.N, 1, [&](int b, int e) {
      for (int i = b; i < e; ++i) {
        cov[i] = resolve(i, res[i], resolution[i], gp[i]);
        tie_flags[i] = tie_cur;
      }
      hp.clear();
    });
    double ll = 0;
    for (int i = 0; i < g.N; ++i) {
      for (auto &c : res[i]) {
        double w = c.posterior / cov[i];
        samples.push_back(Sample{c.h0, w});
        samples.push_back(Sample{c.h1, w});
      }
      ll += log(gp[i]);
    }
    total_weight = 0;  // HaploData.cpp:120-126
    for (auto &s : samples) total_weight += s.w;
    hp.clear();
    return ll;
  }

  // ------------------------------------------------- exact M-step --------
  // --exact-estimate: PatternManager::estimatePatterns / extendPatterns
  // (PatternManager.cpp:347-438) over HaploBuilder::estimateFrequency
  // (HaploBuilder.cpp:263-450) and the ForwardPatternTree (PatternTree.cpp:179-212).
  // The reference sums the match lists over std::map<HaploPair*, double> in
  // pointer (allocation) order, which nothing reproduces; here the walk runs
  // in the device walk's order (xwalk below), so the two agree bit for bit.
  struct FNode { std::vector<int> ch; int data = -1; };
  std::vector<FNode> fnodes;
  std::vector<int> froot;
  std::vector<Pat> *fpats = nullptr;
  double cur_gp = 1.0;
  uint64_t R_X = 0;  // trie-walk match-list entries visited (counter)
  static thread_local uint64_t n_skip;  // pairs extend() skipped (forward likelihood 0) in this thread's resolves

  int fnew(int width) { fnodes.push_back(FNode{std::vector<int>(width, -1), -1}); return (int)fnodes.size() - 1; }
  // ForwardPatternTree::addPattern (PatternTree.cpp:188-212); a missing allele
  // fans out to every allele of its locus
  void faddRec(int node, int k, int q, int width) {
    const Pat &p = (*fpats)[k];
    const int locus = p.start + q, a = p.al[q];
    const int i = missing(a) ? -1 : g.index(locus, a);
    const int lo = i < 0 ? 0 : i, hi = i < 0 ? g.num(locus) : i + 1;
    for (int j = lo; j < hi; ++j) {
      if (fnodes[node].ch[j] < 0) { const int c = fnew(width); fnodes[node].ch[j] = c; }
      const int c = fnodes[node].ch[j];
      if (q == p.len() - 1) fnodes[c].data = k;
      else faddRec(c, k, q + 1, width);
    }
  }
  // HaploBuilder::calcBackwardLikelihood (:263-272, HaploPair.cpp:126-136)
  void calcBackward() {
    const int L = g.L, hl = head_len();
    for (int i = L - 1; i >= hl; --i)
      for (auto &x : hp[i]) {
        x.bwd = 0;
        for (int r = 0; r < 2; ++r)
          for (int t : x.fl[r]) x.bwd += hp[i + 1][t].bwd * hp[i + 1][t].tp;
      }
  }
  // The same walk (HaploBuilder.cpp:334-450) in the order of the device walk
  // (hmc_amd/csrc/exact.hip, exact_walk), so that the two agree bit for bit:
  // the reference sums its match lists in std::map<HaploPair*, double>
  // pointer order, which no restatement reproduces, so any order is the
  // reference's up to its allocator; this one is the device's.  All children
  // of a trie node come from one pass: the states reached from the node's
  // non-zero states along the forward links whose pair carries some child's
  // allele, ascending; each gathers its contributions in add order (the
  // terms of :375-427); a child's frequency is sum(((n0 + n1) + n2) * bwd)
  // over those states, state j into partial j % 64, the 64 partials reduced
  // by the butterfly x += x[lane ^ o], o = 32 .. 1; frequencies and prefix
  // terms accumulate in 2^-44 fixed point (order-free).
  static constexpr double XFIX = 17592186044416.0;  // 2^44
  std::vector<uint64_t> xacc_f, xacc_p;
  struct XLev {
    std::vector<std::vector<double>> slot;  // [child allele][3 F]
    std::vector<int> touched;
  };
  std::vector<XLev> xlev;
  static void xterms(bool ma, bool mb, bool rev, double w0, double w1, double w2, double tp, double &n0, double &n1,
                     double &n2) {
    if (ma && mb) n0 += w0 * tp;
    else if (ma) n1 += w0 * tp * 0.5;
    else n2 += w0 * tp * 0.5;
    if (!rev ? ma : mb) (!rev ? n1 : n2) += w1 * tp;
    if (!rev ? mb : ma) (!rev ? n2 : n1) += w2 * tp;
  }
  // node at depth d of start locus `start`; its lists over the F states of
  // record max(start + d, head_len): P[0..3F)
  void xwalk(int node, int start, int d, int F, const double *P, double last_freq) {
    const int hl = head_len(), W = g.maxnum();
    const FNode &nd = fnodes[node];
    uint64_t cm = 0;
    for (int i = 0; i < (int)nd.ch.size(); ++i)
      if (nd.ch[i] >= 0) cm |= 1ull << i;
    if (!cm) return;
    const int locus = start + d;
    if ((int)xlev.size() < d + 2) xlev.resize(d + 2);
    XLev &C = xlev[d + 1];
    const bool head = locus < hl;
    const std::vector<Pair> &Z = hp[head ? hl : locus + 1];
    const int Fc = (int)Z.size();
    C.slot.assign(W, std::vector<double>());
    for (int i = 0; i < W; ++i)
      if ((cm >> i) & 1ull) C.slot[i].assign(3 * (size_t)Fc, 0.0);
    C.touched.clear();
    auto alleles = [&](int t, int &xa, int &xb) {
      if (head) {
        xa = g.index(locus, P_al(Z[t].pa, locus));
        xb = g.index(locus, P_al(Z[t].pb, locus));
      } else {
        xa = g.index(locus, Z[t].alA);
        xb = g.index(locus, Z[t].alB);
      }
    };
    if (head) {  // head pairs: their patterns' alleles, same states (:340-367)
      for (int t = 0; t < Fc; ++t) {
        int xa, xb;
        alleles(t, xa, xb);
        const double w0 = P[t], w1 = P[F + t], w2 = P[2 * F + t];
        for (int i = 0; i < W; ++i) {
          if (!((cm >> i) & 1ull)) continue;
          const bool ma = xa == i, mb = xb == i;
          double n0 = 0.0, n1 = 0.0, n2 = 0.0;
          if (ma) {
            if (mb) n0 = w0;
            else n1 = w0 * 0.5;
          } else if (mb) {
            n2 = w0 * 0.5;
          }
          if (ma) n1 += w1;
          if (mb) n2 += w2;
          std::vector<double> &c = C.slot[i];
          c[t] = n0;
          c[Fc + t] = n1;
          c[2 * (size_t)Fc + t] = n2;
        }
        C.touched.push_back(t);
      }
    } else {  // along the forward links into the states after `locus`
      const std::vector<Pair> &X = hp[locus];
      std::vector<char> mark(Fc, 0);
      for (int s2 = 0; s2 < F; ++s2) {
        if (P[s2] == 0.0 && P[F + s2] == 0.0 && P[2 * F + s2] == 0.0) continue;
        for (int r = 0; r < 2; ++r)
          for (int t : X[s2].fl[r]) {
            int xa, xb;
            alleles(t, xa, xb);
            if (((cm >> xa) & 1ull) || ((cm >> xb) & 1ull)) mark[t] = 1;
          }
      }
      for (int t = 0; t < Fc; ++t) {
        if (!mark[t]) continue;
        C.touched.push_back(t);
        int xa, xb;
        alleles(t, xa, xb);
        const bool ca = (cm >> xa) & 1ull, cb = xb != xa && ((cm >> xb) & 1ull);
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, b0 = 0.0, b1 = 0.0, b2 = 0.0;
        const double tp = Z[t].tp;
        for (const auto &c : Z[t].in) {
          const int s2 = c.first;
          const double w0 = P[s2], w1 = P[F + s2], w2 = P[2 * F + s2];
          if (ca) xterms(true, xb == xa, c.second, w0, w1, w2, tp, a0, a1, a2);
          if (cb) xterms(false, true, c.second, w0, w1, w2, tp, b0, b1, b2);
        }
        if (ca) {
          std::vector<double> &v = C.slot[xa];
          v[t] = a0;
          v[Fc + t] = a1;
          v[2 * (size_t)Fc + t] = a2;
        }
        if (cb) {
          std::vector<double> &v = C.slot[xb];
          v[t] = b0;
          v[Fc + t] = b1;
          v[2 * (size_t)Fc + t] = b2;
        }
      }
    }
    // every child's frequency: hp->setFrequency(+freq), setPrefixFreq(+last_freq) (:437-441)
    std::vector<double> cf(W, 0.0);
    std::vector<char> desc(W, 0);
    for (int i = 0; i < W; ++i) {
      if (!((cm >> i) & 1ull)) continue;
      const std::vector<double> &c = C.slot[i];
      double part[64] = {0.0};
      bool any = false;
      for (size_t j = 0; j < C.touched.size(); ++j) {
        const int t = C.touched[j];
        const double n0 = c[t], n1 = c[Fc + t], n2 = c[2 * (size_t)Fc + t];
        part[j % 64] += ((n0 + n1) + n2) * Z[t].bwd;
        any = any || n0 != 0.0 || n1 != 0.0 || n2 != 0.0;
      }
      for (int o = 32; o > 0; o >>= 1) {
        double q[64];
        for (int l = 0; l < 64; ++l) q[l] = part[l] + part[l ^ o];
        for (int l = 0; l < 64; ++l) part[l] = q[l];
      }
      const double freq = part[0] / cur_gp;
      cf[i] = freq;
      desc[i] = any;
      const int pat = fnodes[nd.ch[i]].data;
      if (pat >= 0) {
        xacc_f[pat] += (uint64_t)llrint(freq * XFIX);
        xacc_p[pat] += (uint64_t)llrint(last_freq * XFIX);
      }
    }
    // descend into the children with non-zero lists, allele order
    std::vector<std::vector<double>> lists(W);
    for (int i = 0; i < W; ++i)
      if (desc[i]) lists[i] = C.slot[i];  // (the level's buffers are reused below)
    for (int i = 0; i < W; ++i)
      if (desc[i]) xwalk(nd.ch[i], start, d + 1, Fc, lists[i].data(), cf[i]);
  }
  int P_al(int pat, int locus) const { return P[pat].al[locus - P[pat].start]; }

  // HaploBuilder::estimateFrequency(node, locus, a, last_freq, last_match)
  // (HaploBuilder.cpp:334-450) as the reference writes it, in double: the
  // three std::map<HaploPair*, double> lists become dense arrays over the
  // locus's states, iterated in creation order (the pool allocator's pointer
  // order, the closest reproducible stand-in); list 0's terms first, then
  // list 1's, then list 2's (:369-427); the child's frequency one running
  // sum over list 0, 1, 2 (:429-434); hp->setFrequency / setPrefixFreq in
  // double in visiting order (:437-441); every child of every node visited
  // (the reference does not skip zero lists; their terms are +0.0).
  std::vector<double> racc_f, racc_p;
  void rwalk(int node, int locus, int ai, double last_freq, int F, const double *L0, const double *L1,
             const double *L2) {
    const int hl = head_len();
    const bool head = locus < hl;
    const std::vector<Pair> &Z = hp[head ? hl : locus + 1];
    const int Fc = head ? F : (int)Z.size();
    std::vector<double> M0(Fc, 0.0), M1(Fc, 0.0), M2(Fc, 0.0);
    auto alA = [&](int t) { return head ? g.index(locus, P_al(Z[t].pa, locus)) : g.index(locus, Z[t].alA); };
    auto alB = [&](int t) { return head ? g.index(locus, P_al(Z[t].pb, locus)) : g.index(locus, Z[t].alB); };
    if (head) {  // :340-367
      for (int t = 0; t < F; ++t) {
        const double w = L0[t];
        if (alA(t) == ai) {
          if (alB(t) == ai) M0[t] += w;
          else M1[t] += w * 0.5;
        } else if (alB(t) == ai) {
          M2[t] += w * 0.5;
        }
      }
      for (int t = 0; t < F; ++t)
        if (alA(t) == ai) M1[t] += L1[t];
      for (int t = 0; t < F; ++t)
        if (alB(t) == ai) M2[t] += L2[t];
    } else {  // :369-427
      const std::vector<Pair> &X = hp[locus];
      for (int s2 = 0; s2 < F; ++s2) {
        const double w = L0[s2];
        if (w == 0.0) continue;  // (its terms are +0.0)
        for (int r = 0; r < 2; ++r)
          for (int t : X[s2].fl[r]) {
            const double tp = Z[t].tp;
            if (alA(t) == ai) {
              if (alB(t) == ai) M0[t] += w * tp;
              else M1[t] += w * tp * 0.5;
            } else if (alB(t) == ai) {
              M2[t] += w * tp * 0.5;
            }
          }
      }
      for (int s2 = 0; s2 < F; ++s2) {
        const double w = L1[s2];
        if (w == 0.0) continue;
        for (int t : X[s2].fl[0])
          if (alA(t) == ai) M1[t] += w * Z[t].tp;
        for (int t : X[s2].fl[1])
          if (alB(t) == ai) M2[t] += w * Z[t].tp;
      }
      for (int s2 = 0; s2 < F; ++s2) {
        const double w = L2[s2];
        if (w == 0.0) continue;
        for (int t : X[s2].fl[0])
          if (alB(t) == ai) M2[t] += w * Z[t].tp;
        for (int t : X[s2].fl[1])
          if (alA(t) == ai) M1[t] += w * Z[t].tp;
      }
    }
    double freq = 0;
    bool any = false;
    for (const std::vector<double> *M : {&M0, &M1, &M2})
      for (int t = 0; t < Fc; ++t) {
        freq += (*M)[t] * Z[t].bwd;
        any = any || (*M)[t] != 0.0;
      }
    freq /= cur_gp;
    const FNode &nd = fnodes[node];
    if (nd.data >= 0) {
      racc_f[nd.data] += freq;
      racc_p[nd.data] += last_freq;
    }
    if (!any) {  // every descendant adds +0.0 (its lists stay zero), prefixes +0.0
      return;
    }
    for (int i = 0; i < (int)nd.ch.size(); ++i)
      if (nd.ch[i] >= 0) rwalk(nd.ch[i], locus + 1, i, freq, Fc, M0.data(), M1.data(), M2.data());
  }

  // HaploBuilder::estimateFrequency(patterns) (:274-332) for pats[b, e)
  void estimateFreqs(std::vector<Pat> &pats, size_t b, size_t e) {
    const int L = g.L, N = g.N, hl = head_len(), width = g.maxnum();
    fnodes.clear();
    froot.assign(L + 1, -1);
    for (int s = 0; s <= L; ++s) froot[s] = fnew(width);
    fpats = &pats;
    for (size_t k = b; k < e; ++k) {
      faddRec(froot[pats[k].start], (int)k, 0, width);
      pats[k].freq = 0;
      pats[k].prefix = 0;
    }
    xacc_f.assign(pats.size(), 0);
    xacc_p.assign(pats.size(), 0);
    racc_f.assign(pats.size(), 0.0);
    racc_p.assign(pats.size(), 0.0);
    const bool ref_order = prm.exact_order == 1;
    std::vector<Candidate> out;
    std::vector<int> resol;
    for (int gi = 0; gi < N; ++gi) {
      double gprob;
      track_links = true;
      resolve(gi, out, resol, gprob, 1);  // HaploBuilder::resolve default sample_size 1 (HaploBuilder.h:49)
      track_links = false;
      calcBackward();
      cur_gp = gp[gi];  // (*m_genos)[geno].genotype_probability(): set by the last resolveAll (HaploModel.cpp:109)
      if (!(cur_gp > 0.0)) continue;
      for (int start = 0; start < L; ++start) {
        // depth 0: every state after max(start, head_len) loci, weight = forward likelihood (:296-305)
        const int end = std::max(start, hl);
        const int F0 = (int)hp[end].size();
        std::vector<double> l0(3 * (size_t)F0, 0.0);
        for (int i = 0; i < F0; ++i) l0[i] = hp[end][i].fwd;
        if (ref_order) {  // :296-308: match_list[0] = forward likelihoods, lists 1 and 2 empty
          const FNode &rt = fnodes[froot[start]];
          for (int i = 0; i < (int)rt.ch.size(); ++i)
            if (rt.ch[i] >= 0) rwalk(rt.ch[i], start, i, 1.0, F0, l0.data(), l0.data() + F0, l0.data() + 2 * F0);
        } else {
          xwalk(froot[start], start, 0, F0, l0.data(), 1.0);
        }
      }
    }
    hp.clear();
    for (size_t k = b; k < e; ++k) {
      Pat &p = pats[k];
      double freq = std::min(ref_order ? racc_f[k] : (double)xacc_f[k] / XFIX, (double)N);
      double pre = std::min(ref_order ? racc_p[k] : (double)xacc_p[k] / XFIX, (double)N);
      freq = std::min(freq, pre);
      p.freq = freq / N;
      p.prefix = pre / N;
      p.setTp(pre > 0 ? freq / pre : freq / N);
    }
  }
  // PatternManager::estimatePatterns (:364-410) + extendPatterns (:412-438)
  void estimatePatterns() {
    const int L = g.L;
    if (min_freq < 0) {  // estimateFrequency() (:347-362): the same patterns re-estimated
      std::vector<Pat> pats = P;
      estimateFreqs(pats, 0, pats.size());
      for (size_t i = 0; i < P.size(); ++i) {
        P[i].freq = pats[i].freq;
        P[i].prefix = pats[i].prefix;
        P[i].tp = pats[i].tp;
      }
      return;
    }
    std::vector<Pat> all;
    std::vector<int> seeds;
    auto extend = [&](const Pat &hp0, int j) {
      Pat n;
      n.start = hp0.start;
      n.end = hp0.end + 1;
      n.al = hp0.al;
      n.al.push_back(g.symbol(hp0.end, j));
      n.freq = hp0.freq;
      return n;
    };
    for (size_t i = 0; i < P.size(); ++i) {
      all.push_back(P[i]);
      const Pat &hp0 = P[i];
      if (hp0.end < L && hp0.len() < maxlen[hp0.start])
        for (int j = 0; j < g.num(hp0.end); ++j) {
          const int s = j < (int)hp0.succ.size() ? hp0.succ[j] : -1;
          if (s < 0 || P[s].start != hp0.start) {
            all.push_back(extend(hp0, j));
            seeds.push_back((int)all.size() - 1);
          }
        }
    }
    size_t rb = 0, re = all.size();
    while (rb < re) {
      estimateFreqs(all, rb, re);
      const size_t nb = all.size();
      for (int level = 0; level < 4; ++level) {
        std::vector<int> ns;
        for (int si : seeds) {
          const Pat hp0 = all[si];
          if (hp0.end < L && hp0.len() < maxlen[hp0.start] && hp0.freq >= min_freq)
            for (int j = 0; j < g.num(hp0.end); ++j) {
              all.push_back(extend(hp0, j));
              ns.push_back((int)all.size() - 1);
            }
        }
        seeds.swap(ns);
      }
      rb = nb;
      re = all.size();
    }
    P.clear();
    for (auto &c : all)
      if (c.freq >= min_freq || c.len() <= minlen[c.start]) P.push_back(c);
    initialize();
  }

  // HaploComp (HaploComp.cpp:29-76, 144-155) of the input panel (the "real"
  // phase, as given) against inferred haplotypes infer[i] = [2][L] symbols;
  // m_genos_input == m_genos_real, so no missing error.  out = {switch error,
  // IHP, IGP}; returns false where the reference would stop with
  // "Inconsistent genotypes" (Genotype.cpp:246-263).
  bool haploComp(const std::vector<std::vector<int>> &infer, double out[3]) const {
    const int L = g.L;
    long long se_n = 0, se_d = 0, ig_n = 0, ig_d = 0, ih_n = 0, ih_d = 0;
    const int nc = unphased >= 0 ? std::min(unphased, g.N) : g.N;  // HaploComp.cpp:40
    for (int i = 0; i < nc; ++i) {
      const int *f = infer[i].data();
      auto hasMissing = [&](int k) { return missing(g.at(i, 0, k)) || missing(g.at(i, 1, k)); };
      // Genotype::isMatch(g, i, reversed) (Genotype.cpp:97-116)
      auto match = [&](int k, bool rev) {
        return rev ? (amatch(g.at(i, 0, k), f[L + k]) && amatch(g.at(i, 1, k), f[k]))
                   : (amatch(g.at(i, 0, k), f[k]) && amatch(g.at(i, 1, k), f[L + k]));
      };
      int het = 0, miss = 0;  // Genotype::checkGenotype (Genotype.cpp:44-55)
      for (int k = 0; k < L; ++k) {
        if (!amatch(g.at(i, 0, k), g.at(i, 1, k))) ++het;
        if (hasMissing(k)) ++miss;
      }
      // getSwitchDistanceIgnoreMissing (Genotype.cpp:224-266)
      int start = L;
      for (int k = 0; k < L; ++k)
        if (!(hasMissing(k) || (match(k, true) && match(k, false)))) { start = k; break; }
      int sd = 0;
      if (start < L) {
        bool rev;
        if (match(start, true)) rev = true;
        else if (match(start, false)) rev = false;
        else return false;
        for (int k = start + 1; k < L; ++k) {
          if (hasMissing(k) || match(k, rev)) continue;
          if (match(k, !rev)) { rev = !rev; ++sd; }
          else return false;
        }
      }
      // getDiffNumIgnoreMissing (Genotype.cpp:160-175)
      int d1 = 0, d2 = 0;
      for (int k = 0; k < L; ++k)
        if (!hasMissing(k)) {
          if (!match(k, true)) ++d1;
          if (!match(k, false)) ++d2;
        }
      se_n += sd;
      se_d += het - 1;
      ig_n += d1 < d2 ? d1 : d2;
      ig_d += L - miss;
      if (sd > 0) ++ih_n;
      if (het > 1) ++ih_d;
    }
    out[0] = (double)se_n / se_d;
    out[1] = (double)ih_n / ih_d;
    out[2] = (double)ig_n / ig_d;
    return true;
  }
  std::vector<std::array<double, 3>> comp_log;
  int unphased = -1;  // GenoData::unphased_num (BENCH3: the parents); -1 = all

  // HaploModel.cpp:117-155 (MV, sampling EM).
  void run() {
    using clk = std::chrono::steady_clock;
    samples.clear();
    auto t0 = clk::now();
    findPatterns();  // M0 on genotypes
    t_m0 = std::chrono::duration<double>(clk::now() - t0).count();
    npat_log.assign(1, (int)P.size());
    rm_log.assign(1, R_M);
    best_res.assign(g.N, {});
    for (int i = 0; i < g.N; ++i) {
      best_res[i].assign(2 * g.L, 0);
      for (int k = 0; k < g.L; ++k) { best_res[i][k] = g.at(i, 0, k); best_res[i][g.L + k] = g.at(i, 1, k); }
    }
    ll_log.clear(); re_log.clear(); t_e_log.clear(); t_m_log.clear(); comp_log.clear();
    double old_ll = -DBL_MAX;
    iterations = 0;
    for (int it = 1; it <= prm.max_iter; ++it) {
      uint64_t re0 = R_E;
      auto t1 = clk::now();
      double ll = resolveAll();
      t_e_log.push_back(std::chrono::duration<double>(clk::now() - t1).count());
      re_log.push_back(R_E - re0);
      ll_log.push_back(ll);
      iterations = it;
      if (ll >= old_ll) best_res = resolution;
      std::array<double, 3> hc{};  // HaploComp compare(&genos, &resolutions) (HaploModel.cpp:134)
      if (!haploComp(best_res, hc.data())) hc.fill(std::nan(""));
      comp_log.push_back(hc);
      if (it < prm.max_iter && ll >= old_ll && (old_ll - ll) / old_ll > 0.0001) {
        uint64_t rm0 = R_M;
        auto t2 = clk::now();
        if (prm.exact) estimatePatterns();  // HaploModel.cpp:140-141
        else findPatterns();
        t_m_log.push_back(std::chrono::duration<double>(clk::now() - t2).count());
        rm_log.push_back(R_M - rm0);
        npat_log.push_back((int)P.size());
        old_ll = ll;
      } else {
        break;
      }
    }
  }
};

thread_local int Model::tie_cur = 0;
thread_local uint64_t Model::tl_rm = 0;
thread_local std::vector<std::vector<double>> Model::uni;
thread_local std::vector<std::vector<Pair>> Model::hp;
thread_local int Model::S = 1;
thread_local bool Model::track_links = false;
thread_local uint64_t Model::n_skip = 0;

}  // namespace ora

// ============================================================== C API ======
using ora::Model;
extern "C" {

void *ora_create(int N, int L, const int *alleles, const char *types) {
  Model *m = new Model;
  m->g.N = N;
  m->g.L = L;
  m->g.al.assign(alleles, alleles + (size_t)N * 2 * L);
  m->g.types = types ? std::string(types) : std::string(L, 'S');
  m->g.checkAlleleSymbol();
  return m;
}

void *ora_create_from_phase(const char *path) {
  Model *m = new Model;
  std::string err;
  if (!ora::read_phase(path, m->g, err)) {
    fprintf(stderr, "oracle: %s (%s)\n", err.c_str(), path);
    delete m;
    return nullptr;
  }
  return m;
}

void ora_destroy(void *h) { delete (Model *)h; }
// worker threads for mining, successors and resolveAll (results unchanged)
void ora_set_threads(int n) { ora::g_threads = n > 1 ? n : 1; }

void ora_set_params(void *h, double min_freq_abs, int min_len, int max_len, int sample_size, int max_iter) {
  Model *m = (Model *)h;
  m->prm.min_freq_abs = min_freq_abs;
  m->prm.min_len = min_len;
  m->prm.max_len = max_len;
  m->prm.sample_size = sample_size;
  m->prm.max_iter = max_iter;
}

void ora_dims(void *h, int *N, int *L, int *amax) {
  Model *m = (Model *)h;
  *N = m->g.N;
  *L = m->g.L;
  *amax = m->g.maxnum();
}
// allele tables: num[L], sym[L][amax], freq[L][amax]
void ora_allele_table(void *h, int amax, int *num, int *sym, double *freq) {
  Model *m = (Model *)h;
  for (int k = 0; k < m->g.L; ++k) {
    num[k] = m->g.num(k);
    for (int j = 0; j < amax; ++j) {
      sym[k * amax + j] = j < m->g.num(k) ? m->g.symbol(k, j) : -1;
      freq[k * amax + j] = j < m->g.num(k) ? m->g.afreq(k, j) : 0.0;
    }
  }
}
void ora_genotypes(void *h, int *out) {
  Model *m = (Model *)h;
  std::copy(m->g.al.begin(), m->g.al.end(), out);
}

// M-step: findPatterns() (genotype branch while no samples exist).
int ora_find_patterns(void *h) {
  Model *m = (Model *)h;
  m->findPatterns();
  return (int)m->P.size();
}
int ora_pattern_count(void *h) { return (int)((Model *)h)->P.size(); }
int ora_head_len(void *h) { return ((Model *)h)->head_len(); }
// pattern table in id order; succ is [P][amax] pattern ids, -1 = none;
// alleles is [P][maxlen] symbols padded with -1.
void ora_patterns(void *h, int amax, int maxlen, int *start, int *len, double *freq, double *prefix,
                  double *tp, int *succ, int *alleles) {
  Model *m = (Model *)h;
  for (size_t i = 0; i < m->P.size(); ++i) {
    const ora::Pat &p = m->P[i];
    start[i] = p.start;
    len[i] = p.len();
    freq[i] = p.freq;
    prefix[i] = p.prefix;
    tp[i] = p.tp;
    for (int j = 0; j < amax; ++j) succ[i * amax + j] = j < (int)p.succ.size() ? p.succ[j] : -1;
    if (alleles)
      for (int k = 0; k < maxlen; ++k) alleles[i * maxlen + k] = k < p.len() ? p.al[k] : -1;
  }
}

// E-step: resolveAll(); returns the log-likelihood.
double ora_resolve_all(void *h) { return ((Model *)h)->resolveAll(); }
int ora_sample_count(void *h) { return (int)((Model *)h)->samples.size(); }
double ora_total_weight(void *h) { return ((Model *)h)->total_weight; }
void ora_samples(void *h, int *al /*[H][L]*/, double *w) {
  Model *m = (Model *)h;
  int L = m->g.L;
  for (size_t s = 0; s < m->samples.size(); ++s) {
    std::copy(m->samples[s].al.begin(), m->samples[s].al.end(), al + s * L);
    w[s] = m->samples[s].w;
  }
}
// per individual: number of candidates, genotype probability (total)
void ora_estep_summary(void *h, int *ncand, double *gprob) {
  Model *m = (Model *)h;
  for (int i = 0; i < m->g.N; ++i) {
    ncand[i] = (int)m->res[i].size();
    gprob[i] = m->gp[i];
  }
}
// candidate c of individual i: haplotypes [2][L], prior, posterior
int ora_candidate(void *h, int i, int c, int *hap, double *prior, double *posterior) {
  Model *m = (Model *)h;
  if (i < 0 || i >= m->g.N || c < 0 || c >= (int)m->res[i].size()) return -1;
  const ora::Candidate &x = m->res[i][c];
  std::copy(x.h0.begin(), x.h0.end(), hap);
  std::copy(x.h1.begin(), x.h1.end(), hap + m->g.L);
  *prior = x.prior;
  *posterior = x.posterior;
  return 0;
}
// resolution (selected pair) per individual from the last E-step: [N][2][L]
void ora_resolutions(void *h, int *out) {
  Model *m = (Model *)h;
  for (int i = 0; i < m->g.N; ++i) std::copy(m->resolution[i].begin(), m->resolution[i].end(), out + (size_t)i * 2 * m->g.L);
}
void ora_counters(void *h, uint64_t *re, uint64_t *rm) {
  *re = ((Model *)h)->R_E;
  *rm = ((Model *)h)->R_M;
}
void ora_reset_counters(void *h) { ((Model *)h)->R_E = ((Model *)h)->R_M = 0; }

// Whole EM (HaploModel::run).  Returns iterations run.
int ora_run(void *h) {
  Model *m = (Model *)h;
  m->R_E = m->R_M = 0;
  m->run();
  return m->iterations;
}
// per-iteration logs; arrays sized >= iterations (npat, rm: iterations + 1 entries: M0 first)
void ora_run_log(void *h, double *ll, uint64_t *re, uint64_t *rm, int *npat, double *t_e, double *t_m,
                 double *t_m0) {
  Model *m = (Model *)h;
  for (size_t i = 0; i < m->ll_log.size(); ++i) { ll[i] = m->ll_log[i]; re[i] = m->re_log[i]; t_e[i] = m->t_e_log[i]; }
  for (size_t i = 0; i < m->rm_log.size(); ++i) rm[i] = m->rm_log[i];
  for (size_t i = 0; i < m->npat_log.size(); ++i) npat[i] = m->npat_log[i];
  for (size_t i = 0; i < m->t_m_log.size(); ++i) t_m[i] = m->t_m_log[i];
  *t_m0 = m->t_m0;
}
// HaploComp triple {switch error, IHP, IGP} of every iteration of run(): [iters][3]
void ora_run_comp_log(void *h, double *out) {
  Model *m = (Model *)h;
  for (size_t i = 0; i < m->comp_log.size(); ++i)
    for (int j = 0; j < 3; ++j) out[i * 3 + j] = m->comp_log[i][j];
}
// HaploComp of the panel against infer[N][2][L] symbols; 0 ok, -1 inconsistent
int ora_haplocomp(void *h, const int *infer, double *out3) {
  Model *m = (Model *)h;
  std::vector<std::vector<int>> f(m->g.N);
  for (int i = 0; i < m->g.N; ++i) f[i].assign(infer + (size_t)i * 2 * m->g.L, infer + (size_t)(i + 1) * 2 * m->g.L);
  return m->haploComp(f, out3) ? 0 : -1;
}
// accepted resolutions after run(): [N][2][L]
void ora_best_resolutions(void *h, int *out) {
  Model *m = (Model *)h;
  for (int i = 0; i < m->g.N; ++i) std::copy(m->best_res[i].begin(), m->best_res[i].end(), out + (size_t)i * 2 * m->g.L);
}

// Exposes std::nth_element / std::sort on (lik, tag) records so that tests can
// check the product's libstdc++-exact selection replica against the real thing.
void ora_std_nth_element(double *lik, int *tag, int n, int nth) {
  std::vector<ora::Link> v(n);
  for (int i = 0; i < n; ++i) v[i] = ora::Link{tag[i], 0, false, false, lik[i]};
  std::nth_element(v.begin(), v.begin() + nth, v.end(), ora::GreaterLik());
  for (int i = 0; i < n; ++i) { lik[i] = v[i].lik; tag[i] = v[i].pred; }
}
void ora_std_sort(double *lik, int *tag, int n) {
  std::vector<ora::Link> v(n);
  for (int i = 0; i < n; ++i) v[i] = ora::Link{tag[i], 0, false, false, lik[i]};
  std::sort(v.begin(), v.end(), ora::GreaterLik());
  for (int i = 0; i < n; ++i) { lik[i] = v[i].lik; tag[i] = v[i].pred; }
}

// ---- seams used by bench.py's cpu_baseline leg ------------------------------
// Install a pattern table (id order) and run initialize()'s tree build; the
// given successors are kept (they come from a parity-checked M-step).
int ora_set_patterns(void *h, int P, const int *start, const int *len, const int *alleles, int maxlen,
                     const double *freq, const double *prefix, const double *tp, const int *succ, int amax) {
  Model *m = (Model *)h;
  m->P.assign(P, ora::Pat{});
  for (int i = 0; i < P; ++i) {
    ora::Pat &p = m->P[i];
    p.start = start[i];
    p.end = start[i] + len[i];
    p.al.assign(alleles + (size_t)i * maxlen, alleles + (size_t)i * maxlen + len[i]);
    p.freq = freq[i];
    p.prefix = prefix[i];
    p.tp = tp[i];
    p.id = i;
    if (p.end < m->g.L) {
      p.succ.assign(succ + (size_t)i * amax, succ + (size_t)i * amax + m->g.num(p.end));
    }
  }
  if (m->minlen.empty()) {
    m->minlen.assign(m->g.L, std::max(m->prm.min_len, 1));
    m->maxlen.assign(m->g.L, m->prm.max_len <= 0 ? m->g.L : m->prm.max_len);
  }
  m->tree.init(m->g);
  m->head_list.clear();
  for (int i = 0; i < P; ++i) {
    m->tree.add(m->P, i);
    if (m->P[i].start == 0 && m->P[i].len() == m->head_len()) m->head_list.push_back(i);
  }
  return 0;
}
// Time HaploBuilder::resolve over individuals [i0, i1) (results discarded).
double ora_time_resolve_range(void *h, int i0, int i1) {
  Model *m = (Model *)h;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<ora::Candidate> out;
  std::vector<int> resol;
  double gp;
  for (int i = i0; i < i1; ++i) m->resolve(i, out, resol, gp);
  m->hp.clear();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
// Install HaploData samples ([H][L] symbols, weights) and total_weight.
void ora_set_samples(void *h, int H, const int *al, const double *w) {
  Model *m = (Model *)h;
  int L = m->g.L;
  m->samples.assign(H, ora::Sample{});
  m->total_weight = 0;
  for (int s = 0; s < H; ++s) {
    m->samples[s].al.assign(al + (size_t)s * L, al + (size_t)s * L + L);
    m->samples[s].w = w[s];
    m->total_weight += w[s];
  }
}
// Time findPatterns() (sample branch when samples are installed).
double ora_time_find_patterns(void *h) {
  Model *m = (Model *)h;
  auto t0 = std::chrono::steady_clock::now();
  m->findPatterns();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// Time the sampling M-step (searchPattern + initialize) restricted to the
// start loci [s0, s1): each root's DFS subtree is independent
// (PatternManager.cpp:94-97,106-108), so a subset of roots is a bounded
// sample of findPatternByFreq.  Leaves the subset's table installed.
double ora_time_find_patterns_roots(void *h, int s0, int s1) {
  Model *m = (Model *)h;
  ora::Params &pr = m->prm;
  if (pr.min_freq_abs > 0) pr.min_freq = pr.min_freq_abs / (2.0 * m->g.N);
  const int L = m->g.L;
  int mxl = pr.max_len <= 0 ? L : pr.max_len, mnl = std::max(pr.min_len, 1);
  mxl = std::max(mxl, mnl);
  m->minlen.resize(L, mnl);
  m->maxlen.resize(L, mxl);
  auto t0 = std::chrono::steady_clock::now();
  m->P.clear();
  m->min_freq = pr.min_freq;
  std::vector<ora::Model::Cand *> stack;
  for (int s = std::max(0, s0); s < std::min(L, s1); ++s) {
    auto *c = new ora::Model::Cand;
    c->p.start = c->p.end = s;
    stack.push_back(c);
  }
  m->searchPattern(stack, false);
  m->initialize();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// The same two samples over explicit lists (stratified samples for the bench's
// CPU baseline): HaploBuilder::resolve of individuals ids[0, n), and the
// sampling M-step over the start loci roots[0, n) (ascending; each root's DFS
// subtree is independent, PatternManager.cpp:94-97,106-108).
double ora_time_resolve_list(void *h, const int *ids, int n) {
  Model *m = (Model *)h;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<ora::Candidate> out;
  std::vector<int> resol;
  double gp;
  for (int q = 0; q < n; ++q) m->resolve(ids[q], out, resol, gp);
  m->hp.clear();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
// HaploBuilder::initialize (HaploBuilder.cpp:25-33) clears one std::map per
// pattern (m_best_pair, vector<map<int, int> >, HaploBuilder.h:29) before every
// individual — O(P) work the restatement's resolve skips (its key table is
// per-locus).  The bench's CPU baseline adds it back: seconds of one such
// pass over P empty maps, the best of `reps` passes.
double ora_time_best_pair_reset(long long P, int reps) {
  if (P <= 0 || reps <= 0) return 0.0;
  std::vector<std::map<int, int>> best((size_t)P);
  double best_s = 1e300;
  for (int r = 0; r < reps; ++r) {
    best[(size_t)(r * 7919) % (size_t)P][r] = r;  // one live entry, as after an individual
    auto t0 = std::chrono::steady_clock::now();
    for (auto &x : best) x.clear();
    best_s = std::min(best_s, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  }
  return best_s;
}
double ora_time_find_patterns_root_list(void *h, const int *roots, int n) {
  Model *m = (Model *)h;
  ora::Params &pr = m->prm;
  if (pr.min_freq_abs > 0) pr.min_freq = pr.min_freq_abs / (2.0 * m->g.N);
  const int L = m->g.L;
  int mxl = pr.max_len <= 0 ? L : pr.max_len, mnl = std::max(pr.min_len, 1);
  mxl = std::max(mxl, mnl);
  m->minlen.resize(L, mnl);
  m->maxlen.resize(L, mxl);
  auto t0 = std::chrono::steady_clock::now();
  m->P.clear();
  m->min_freq = pr.min_freq;
  std::vector<ora::Model::Cand *> stack;
  for (int q = 0; q < n; ++q) {
    if (roots[q] < 0 || roots[q] >= L) continue;
    auto *c = new ora::Model::Cand;
    c->p.start = c->p.end = roots[q];
    stack.push_back(c);
  }
  m->searchPattern(stack, false);
  m->initialize();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// HaploModel::resolveAll restricted to individuals [i0, i1) (the shard one
// rank of the sharded E-step owns); samples/results cover only that range.
double ora_resolve_range(void *h, int i0, int i1) {
  Model *m = (Model *)h;
  m->samples.clear();
  m->res.assign(m->g.N, {});
  m->gp.assign(m->g.N, 0.0);
  m->resolution.assign(m->g.N, {});
  double ll = 0;
  for (int i = i0; i < i1; ++i) {
    double cov = m->resolve(i, m->res[i], m->resolution[i], m->gp[i]);
    for (auto &c : m->res[i]) {
      double w = c.posterior / cov;
      m->samples.push_back(ora::Sample{c.h0, w});
      m->samples.push_back(ora::Sample{c.h1, w});
    }
    ll += log(m->gp[i]);
  }
  m->total_weight = 0;
  for (auto &x : m->samples) m->total_weight += x.w;
  m->hp.clear();
  return ll;
}

// HaploModel::setModel / mc_order (HaploModel.cpp:26-36, HMC.cpp:41): 0 MV, 1 MC, 2 MA
void ora_set_model(void *h, int model, int mc_order) {
  Model *m = (Model *)h;
  m->prm.model = model;
  m->prm.mc_order = mc_order;
}
// HaploModel::exact_estimate (HMC.cpp:42): M-steps by estimatePatterns
void ora_set_exact(void *h, int on) { ((Model *)h)->prm.exact = on != 0; }
// 0: the device walk's summation order (bit-exact check); 1: the reference's
// grouping in double (rwalk, the independent 1e-6 check)
void ora_set_exact_order(void *h, int mode) { ((Model *)h)->prm.exact_order = mode; }
// One exact M-step (PatternManager::estimatePatterns) after an E-step; returns
// the pattern count; *rx = match-list entries visited by the trie walks.
int ora_estimate_patterns(void *h, uint64_t *rx) {
  Model *m = (Model *)h;
  m->R_X = 0;
  m->estimatePatterns();
  if (rx) *rx = m->R_X;
  return (int)m->P.size();
}
// GenoData::unphased_num (HaploFile.cpp:475): HaploComp covers [0, n)
void ora_set_unphased(void *h, int n) { ((Model *)h)->unphased = n; }
// HaploModel::num_patterns (HMC.cpp:38): > 0 selects findPatternByNum
void ora_set_num_patterns(void *h, int n) { ((Model *)h)->prm.num_patterns = n; }
// Pairs extend() skipped because their forward likelihood is 0 (HaploBuilder.cpp:237)
// while resolving individuals [i0, i1) on this thread (diagnostic of the tests'
// underflow panels).
uint64_t ora_skip_count_range(void *h, int i0, int i1) {
  Model *m = (Model *)h;
  Model::n_skip = 0;
  for (int i = i0; i < i1; ++i) {
    std::vector<ora::Candidate> out;
    std::vector<int> resol;
    double gprob = 0.0;
    m->resolve(i, out, resol, gprob, m->prm.sample_size);
  }
  return Model::n_skip;
}
// Tie diagnostics of the last resolveAll (see Model::tie_flags), [N].
void ora_tie_flags(void *h, int *out) {
  Model *m = (Model *)h;
  for (int i = 0; i < (int)m->tie_flags.size(); ++i) out[i] = m->tie_flags[i];
}
}  // extern "C"
